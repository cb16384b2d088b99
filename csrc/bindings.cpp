// Python bindings of the native runtime: rocmdash._native.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <memory>
#include <stdexcept>

#include "device_window.h"
#include "frame_render.h"
#include "long_window.h"
#include "node_window.h"
#include "publish.h"
#include "rccl_comm.h"

namespace rocmdash {
int launch_spin(uint32_t workgroups, double us, void* stream);  // calib.hip
int launch_gather32(const void* src, uint64_t src_bytes, void* out, uint64_t out_bytes, uint32_t threads,
                    uint32_t seed, void* stream);
int launch_store64(void* dst, uint64_t dst_bytes, uint32_t threads, void* stream);
int launch_store32(void* dst, uint64_t dst_bytes, uint32_t threads, void* stream);
}  // namespace rocmdash
#include "ring.h"
#include "node_counters.h"
#include "sampler.h"
#include "sources.h"
#include "window_stats.h"

namespace py = pybind11;
using namespace rocmdash;

namespace {

py::dict info_dict(const GpuInfo& g) {
  py::dict d;
  d["index"] = g.index;
  d["bdf"] = g.bdf;
  d["model_number"] = g.model_number;
  d["product_name"] = g.product_name;
  d["market_name"] = g.market_name;
  d["power_limit_w"] = g.power_limit_w;
  d["vram_total_mb"] = g.vram_total_mb;
  d["edge_is_hotspot"] = g.edge_is_hotspot;
  d["metrics_path"] = g.metrics_path;
  d["metrics_table"] = g.metrics_table;
  d["metrics_calibration"] = g.metrics_calibration;
  return d;
}

py::list names(const char* const* n) {
  py::list l;
  for (; *n; ++n) l.append(*n);
  return l;
}

}  // namespace

PYBIND11_MODULE(_native, m) {
  m.doc() = "rocmdash native runtime: rings, samplers (amd-smi, rocprofiler-sdk), HIP window stats";

  m.attr("SMI_FIELDS") = names(smi_field_names());
  m.attr("CTR_FIELDS") = names(ctr_field_names());
  m.attr("STAT_NAMES") = py::make_tuple("min", "max", "mean", "p0", "p1", "p2", "last", "count");
  m.attr("MAX_SERIES_PER_LAUNCH") = int(kMaxSeriesPerLaunch);

  py::class_<SeriesRing, std::shared_ptr<SeriesRing>>(m, "SeriesRing")
      .def(py::init<uint32_t, uint64_t>(), py::arg("width"), py::arg("capacity"))
      .def_property_readonly("width", &SeriesRing::width)
      .def_property_readonly("capacity", &SeriesRing::capacity)
      .def_property_readonly("pinned", &SeriesRing::pinned)
      .def_property_readonly("head", &SeriesRing::head)
      .def_property_readonly("last_timestamp", &SeriesRing::last_timestamp)
      .def_property_readonly("rows_ptr", [](const SeriesRing& r) { return reinterpret_cast<uintptr_t>(r.rows()); })
      .def(
          "push",
          [](SeriesRing& r, py::array_t<float, py::array::c_style | py::array::forcecast> row, uint64_t t_ns) {
            if (row.size() != r.width()) throw std::invalid_argument("row size != ring width");
            r.push(row.data(), t_ns);
          },
          py::arg("row"), py::arg("t_ns"))
      .def(
          "push_many",
          [](SeriesRing& r, py::array_t<float, py::array::c_style | py::array::forcecast> rows,
             py::array_t<uint64_t, py::array::c_style | py::array::forcecast> ts) {
            if (rows.ndim() != 2 || rows.shape(1) != r.width() || ts.size() != rows.shape(0))
              throw std::invalid_argument("rows must be [n, width] with n timestamps");
            for (py::ssize_t i = 0; i < rows.shape(0); ++i) r.push(rows.data(i, 0), ts.data()[i]);
          },
          py::arg("rows"), py::arg("ts"))
      .def(
          "window",
          [](const SeriesRing& r, uint64_t n) {
            py::array_t<float> rows({py::ssize_t(n), py::ssize_t(r.width())});
            py::array_t<uint64_t> ts{py::ssize_t(n)};
            uint64_t got;
            {
              py::gil_scoped_release nogil;
              got = r.read_window(n, rows.mutable_data(), ts.mutable_data());
            }
            rows.resize({py::ssize_t(got), py::ssize_t(r.width())});
            ts.resize({py::ssize_t(got)});
            return py::make_tuple(rows, ts);
          },
          py::arg("n"), "Newest <= n rows (oldest first) and their timestamps; torn rows dropped.");

  py::class_<Source, std::shared_ptr<Source>>(m, "Source")
      .def_property_readonly("width", &Source::width)
      .def_property_readonly("kind", &Source::kind)
      .def_property_readonly("backend", &Source::backend)
      .def("info", [](const Source& s) { return info_dict(s.info()); })
      .def("counts", [](const Source& s) {
        py::dict d;
        for (const auto& kv : s.counts()) d[py::str(kv.first)] = kv.second;
        return d;
      })
      .def("xcd_detail", [](const Source& s) -> py::object {
        const std::vector<float> v = s.xcd_detail();
        if (v.empty()) return py::none();
        const py::ssize_t n = py::ssize_t(v.size() / 2);
        py::array_t<float> busy{n}, clk{n};
        std::memcpy(busy.mutable_data(), v.data(), sizeof(float) * size_t(n));
        std::memcpy(clk.mutable_data(), v.data() + n, sizeof(float) * size_t(n));
        py::dict d;
        d["busy"] = busy;
        d["clock_mhz"] = clk;
        return d;
      }, "Per-XCD busy (%) and gfx clock (MHz) of the last sample, or None")
      .def("sample", [](Source& s) -> py::object {
        py::array_t<float> row{py::ssize_t(s.width())};
        bool ok;
        {
          py::gil_scoped_release nogil;
          ok = s.sample(row.mutable_data());
        }
        if (!ok) return py::none();
        return row;
      });

  m.def("make_synthetic_source", &make_synthetic_source, py::arg("kind"), py::arg("seed"),
        py::arg("total_vram_mb") = 294896.0);
  m.def("make_smi_source", &make_smi_source, py::arg("bdf") = 0, py::arg("index") = 0);
  m.def("make_counter_source", &make_counter_source, py::arg("bdf") = 0, py::arg("index") = 0);
  m.def("make_counter_source_all", &make_counter_source_all, py::arg("bdf") = 0, py::arg("index") = 0,
        "Counters of the whole physical GPU at this PCI address (every compute partition combined).");
  m.def("amdsmi_gpu_count", &amdsmi_gpu_count);
  m.def("amdsmi_enumerate", []() {
    py::list l;
    for (auto& g : amdsmi_enumerate()) l.append(info_dict(g));
    return l;
  });
  m.def("counters_preinit", &counters_preinit, py::arg("counter_names"), py::arg("only_ordinal") = -1,
        py::arg("only_bdf") = 0);
  m.def("make_null_source", &make_null_source, py::arg("kind"));
  m.def(
      "make_shm_source",
      [](const std::string& path, double hz, const std::string& kind) -> std::shared_ptr<Source> {
        return std::make_shared<ShmSource>(path, hz, kind);
      },
      py::arg("path"), py::arg("hz"), py::arg("kind") = "counter",
      "A rank's view of its GPU's rows published by the node's counter process (shm_ring.h).");
  py::class_<ShmPublisher, std::shared_ptr<ShmPublisher>>(
      m, "ShmPublisher", "The node counter process's publisher: one lane (thread) per GPU source -> its shm ring.")
      .def(py::init<const std::vector<std::string>&, std::vector<std::shared_ptr<Source>>, double, uint64_t>(),
           py::arg("paths"), py::arg("sources"), py::arg("hz"), py::arg("capacity") = 4096)
      .def("start", &ShmPublisher::start)
      .def("stop", &ShmPublisher::stop, py::arg("grace_s") = 2.0, py::call_guard<py::gil_scoped_release>())
      .def("replace", &ShmPublisher::replace, py::arg("lane"), py::arg("source"),
           "Abandon lane i and start a fresh one with `source` and a new ring file; returns its generation.")
      .def("stats", &ShmPublisher::stats,
           "per ring: [samples, failures, mean read us, last read us, beat age s, lane generation, in-read s]");
  m.def("make_hanging_source", &make_hanging_source, py::arg("inner"), py::arg("after_s"),
        "Fault injection: a source whose reads block forever `after_s` seconds after its first read.");
  m.def(
      "make_replay_source",
      [](const std::string& kind, py::array_t<float, py::array::c_style | py::array::forcecast> rows, py::dict info) {
        if (rows.ndim() != 2) throw std::invalid_argument("rows must be [n, width]");
        std::vector<float> v(rows.data(), rows.data() + rows.size());
        GpuInfo g;
        if (info.contains("index")) g.index = info["index"].cast<int>();
        if (info.contains("bdf")) g.bdf = info["bdf"].cast<uint64_t>();
        if (info.contains("model_number")) g.model_number = info["model_number"].cast<std::string>();
        if (info.contains("product_name")) g.product_name = info["product_name"].cast<std::string>();
        if (info.contains("market_name")) g.market_name = info["market_name"].cast<std::string>();
        if (info.contains("power_limit_w")) g.power_limit_w = info["power_limit_w"].cast<double>();
        if (info.contains("vram_total_mb")) g.vram_total_mb = info["vram_total_mb"].cast<double>();
        return make_replay_source(kind, v, uint32_t(rows.shape(1)), g);
      },
      py::arg("kind"), py::arg("rows"), py::arg("info") = py::dict());
  py::class_<RawCalibrationPolicy>(m, "RawCalibrationPolicy",
                                    "The SMI source's raw SMU-table calibration / retry policy (CPU-testable).")
      .def(py::init<double, int, int>(), py::arg("retry_s") = 60.0, py::arg("need") = 6, py::arg("trials") = 8)
      .def("due", &RawCalibrationPolicy::due, py::arg("now_ns"))
      .def("record", &RawCalibrationPolicy::record, py::arg("matched"), py::arg("now_ns"), py::arg("final") = false)
      .def_property_readonly("raw", &RawCalibrationPolicy::raw)
      .def_property_readonly("final_refusal", &RawCalibrationPolicy::final_refusal)
      .def_property_readonly("attempts", &RawCalibrationPolicy::attempts)
      .def_property_readonly("promotions", &RawCalibrationPolicy::promotions)
      .def_property_readonly("last_matched", &RawCalibrationPolicy::last_matched);
  m.def("counters_ready", &counters_ready);
  m.def("counters_status", &counters_status);

  py::class_<Sampler, std::shared_ptr<Sampler>>(m, "Sampler")
      .def(py::init<std::shared_ptr<Source>, std::shared_ptr<SeriesRing>, double>(), py::arg("source"),
           py::arg("ring"), py::arg("hz"))
      .def("start", &Sampler::start)
      .def("start_free", &Sampler::start_free, py::arg("max_hz") = 50000.0)
      .def("calls", &Sampler::calls)
      .def("last_start_ns", &Sampler::last_start_ns)
      .def("wait_calls", &Sampler::wait_calls, py::arg("target"), py::arg("timeout_s"),
           py::call_guard<py::gil_scoped_release>())
      .def("stop", &Sampler::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("running", &Sampler::running)
      .def_property_readonly("hz", &Sampler::hz)
      .def_property_readonly("ring", &Sampler::ring)
      .def_property_readonly("source", &Sampler::source)
      .def("sample_once", &Sampler::sample_once, py::call_guard<py::gil_scoped_release>())
      .def("request", &Sampler::request, py::call_guard<py::gil_scoped_release>())
      .def("wait", &Sampler::wait, py::call_guard<py::gil_scoped_release>())
      .def("stats", [](const Sampler& s) {
        auto st = s.stats();
        py::dict d;
        d["samples"] = st.samples;
        d["failures"] = st.failures;
        d["overruns"] = st.overruns;
        d["last_us"] = st.last_us;
        d["max_us"] = st.max_us;
        d["mean_us"] = st.mean_us;
        d["p50_us"] = st.p50_us;
        d["p99_us"] = st.p99_us;
        return d;
      })
      .def("recent_us", &Sampler::recent_us)
      .def("counts", [](const Sampler& s) {
        const auto st = s.counts();
        return py::make_tuple(st.samples, st.failures, st.overruns);
      })
      .def("set_affinity", &Sampler::set_affinity, py::arg("cpus"))
      .def("set_spin_us", &Sampler::set_spin_us, py::arg("us"));

  m.def("long_window_chunk_plan", &long_window_chunk_plan, py::arg("window"), py::arg("widths"), py::arg("cus") = 256,
        py::arg("chunk_rows") = 0, py::arg("rounds") = 1,
        "per ring (rows per workgroup, workgroups per segment) of the long-window passes");
  m.def("long_window_node_cap", &long_window_node_cap, py::arg("maxmid"), py::arg("nranks"),
        "node bracket records: the next refresh's key cap from the node's most kept keys");
  py::class_<LongWindowSet, std::shared_ptr<LongWindowSet>>(m, "LongWindowSet")
      .def(py::init<uint32_t, int, bool, uint32_t>(), py::arg("window"), py::arg("device"), py::arg("use_graph") = false,
           py::arg("chunk_rows") = 0)
      .def_property_readonly("chunk_rows", &LongWindowSet::chunk_rows)
      .def_property_readonly("chunk_plan", &LongWindowSet::chunk_plan)
      .def_property("brackets", &LongWindowSet::brackets, &LongWindowSet::set_brackets)
      .def_property("incremental", &LongWindowSet::incremental, &LongWindowSet::set_incremental,
                    "incremental bracket mode: pass B streams only the chunks new rows landed in (A/B switch)")
      .def_property("fused_passb", &LongWindowSet::fused_passb, &LongWindowSet::set_fused_passb,
                    "a short incremental work list: scan B streams the changed chunks itself, one kernel (A/B switch)")
      .def("bracket_stats", &LongWindowSet::bracket_stats, py::arg("mode") = 0,
           "Per series [refreshes, hits, last refresh hit] of the local (0) or node (1) brackets")
      .def(
          "bracket_state",
          [](const LongWindowSet& w, int mode) {
            py::list out;
            for (const auto& r : w.bracket_state(mode)) {
              py::dict d;
              py::list lo, hi, delta, cin;
              for (int q = 0; q < 3; ++q) {
                lo.append(r[q]);
                hi.append(r[3 + q]);
                float f;
                std::memcpy(&f, &r[6 + q], 4);
                delta.append(f);
                cin.append(r[9 + q]);
              }
              d["lo"] = lo;
              d["hi"] = hi;
              d["delta"] = delta;
              d["cin"] = cin;
              d["valid"] = r[12];
              d["nounion"] = r[13];
              d["hit"] = r[15];
              d["refreshes"] = r[16];
              d["hits"] = r[17];
              out.append(d);
            }
            return out;
          },
          py::arg("mode") = 0, "Every series' bracket record (keys as uint32 order keys, delta in value units)")
      .def_property("wave_private_level", &LongWindowSet::wave_private_level,
                    &LongWindowSet::set_wave_private_level)
      .def_property("wave_private", &LongWindowSet::wave_private, &LongWindowSet::set_wave_private,
                    "pass 0: per-wave LDS histogram copies for 8-bit digits (A/B switch)")
      .def_property("prefetch", &LongWindowSet::prefetch, &LongWindowSet::set_prefetch,
                    "load the next iteration's rows while counting this one's (A/B switch)")
      .def_property("brk_target", &LongWindowSet::brk_target, &LongWindowSet::set_brk_target,
                    "samples a local bracket aims to hold (256..2048)")
      .def("set_phase_clocks", &LongWindowSet::set_phase_clocks, py::arg("on"))
      .def("phase_clocks", &LongWindowSet::phase_clocks)
      .def_property("plan_rounds", &LongWindowSet::plan_rounds, &LongWindowSet::set_plan_rounds,
                    "rounds of the chip's workgroup slots a planned full pass takes (before the first refresh)")
      .def_property("compact", &LongWindowSet::compact, &LongWindowSet::set_compact,
                    "pass 2 keeps the keys it counts and pass 3 reads only those (A/B switch)")
      .def("add_ring", &LongWindowSet::add_ring, py::arg("ring"))
      .def_property_readonly("num_series", &LongWindowSet::num_series)
      .def_property_readonly("window", &LongWindowSet::window)
      .def(
          "refresh",
          [](LongWindowSet& w, uintptr_t out, uintptr_t stream, float p0, float p1, float p2) {
            py::gil_scoped_release nogil;
            w.refresh(reinterpret_cast<float*>(out), reinterpret_cast<void*>(stream), p0, p1, p2);
          },
          py::arg("out_ptr"), py::arg("stream"), py::arg("p0") = 50.0f, py::arg("p1") = 90.0f, py::arg("p2") = 99.0f)
      .def(
          "refresh_node",
          [](LongWindowSet& w, uintptr_t out, uintptr_t stream, float p0, float p1, float p2,
             std::shared_ptr<RcclComm> comm, bool timing, double timeout_s, py::object abandon) {
            std::function<bool()> ab;
            if (!abandon.is_none()) {
              // polled from the host wait with the GIL released: take it for each call
              ab = [abandon]() {
                py::gil_scoped_acquire gil;
                return abandon().cast<bool>();
              };
            }
            py::gil_scoped_release nogil;
            w.refresh_node(reinterpret_cast<float*>(out), reinterpret_cast<void*>(stream), p0, p1, p2, comm.get(),
                           timing, timeout_s, ab);
          },
          py::arg("out_ptr"), py::arg("stream"), py::arg("p0") = 50.0f, py::arg("p1") = 90.0f, py::arg("p2") = 99.0f,
          py::arg("comm") = py::none(), py::arg("timing") = false, py::arg("timeout_s") = 60.0,
          py::arg("abandon") = py::none(),
          "Collective: node-wide statistics over every rank's window (radix select with the digit histograms "
          "all-reduced over `comm` between the passes; None = a one-rank node). out [S][8], last = NaN.")
      .def("set_node_brackets", &LongWindowSet::set_node_brackets, py::arg("series"), py::arg("lo"), py::arg("hi"),
           py::call_guard<py::gil_scoped_release>(),
           "Test hook: the node brackets of one series (3 lo / 3 hi order-preserving keys) for the next node refresh.")
      .def_property_readonly("node_cap", &LongWindowSet::node_cap)
      .def_property_readonly("node_last_maxmid", &LongWindowSet::node_last_maxmid)
      .def("reset_node", &LongWindowSet::reset_node, py::call_guard<py::gil_scoped_release>(),
           "Forget the node's bracket state (every member, at the start of a membership epoch).")
      .def("node_collective_us", &LongWindowSet::node_collective_us,
           "µs of the last timed node refresh's 5 collective steps (synchronises their events).")
      .def("stats", [](const LongWindowSet& w) {
        const auto s = w.stats();
        py::dict d;
        d["refreshes"] = s.refreshes;
        d["node_refreshes"] = s.node_refreshes;
        d["node_resets"] = s.node_resets;
        d["bracket_refreshes"] = s.bracket_refreshes;
        d["passb_chunks"] = s.passb_chunks;
        d["chain_refreshes"] = s.chain_refreshes;
        d["rows_copied"] = s.rows_copied;
        d["bytes_copied"] = s.bytes_copied;
        d["memcpy_calls"] = s.memcpy_calls;
        d["rows_lost"] = s.rows_lost;
        d["graph_launches"] = s.graph_launches;
        d["kernel_launches"] = s.kernel_launches;
        d["ingest_launches"] = s.ingest_launches;  // staging kernels (in place of DMA copies)
        d["fused_refreshes"] = s.fused_refreshes;  // bracket refreshes whose scan B streamed chunks
        d["single_kernel_refreshes"] = s.single_kernel_refreshes;  // ... with no pass B kernel
        d["fused_segments"] = s.fused_segments;
        d["node_record_bytes"] = s.node_record_bytes;  // node bracket records all-gathered (this rank's, summed)
        d["host_stage_ns"] = s.host_stage_ns;  // refresh()'s host time: staging,
        d["host_enqueue_ns"] = s.host_enqueue_ns;  // a bracket refresh's work list + launches,
        d["host_wait_ns"] = s.host_wait_ns;  // and its wait for the report
        return d;
      });

  m.def("set_pinned_host_rings", &set_pinned_host_rings, py::arg("on"));
  m.def("set_pull_mode", &set_pull_mode, py::arg("on"));
  m.def("hip_device_count", &hip_device_count);
  m.def("hip_device_bdf", &hip_device_bdf, py::arg("device"));

  py::class_<DeviceWindowSet, std::shared_ptr<DeviceWindowSet>>(m, "DeviceWindowSet")
      .def(py::init<uint32_t, int>(), py::arg("window"), py::arg("device"))
      .def("add_ring", &DeviceWindowSet::add_ring, py::arg("ring"))
      .def_property_readonly("num_series", &DeviceWindowSet::num_series)
      .def_property_readonly("window", &DeviceWindowSet::window)
      .def_property_readonly("device", &DeviceWindowSet::device)
      .def(
          "refresh",
          [](DeviceWindowSet& w, uintptr_t out, uintptr_t stream, float p0, float p1, float p2, int signal) {
            if (signal < DeviceWindowSet::kSignalNone || signal > DeviceWindowSet::kSignalTagged)
              throw std::invalid_argument("signal: 0 (none), 1 (flag) or 2 (tagged host output)");
            py::gil_scoped_release nogil;
            return w.refresh(reinterpret_cast<float*>(out), reinterpret_cast<void*>(stream), p0, p1, p2, signal);
          },
          py::arg("out_ptr"), py::arg("stream"), py::arg("p0") = 50.f, py::arg("p1") = 90.f, py::arg("p2") = 99.f,
          py::arg("signal") = int(DeviceWindowSet::kSignalFlag),
          "Enqueue the refresh; returns its completion sequence number (0: no completion signal). signal: "
          "0 = none (synchronise the stream), 1 = completion flag, 2 = tagged outputs (out_ptr is host memory, "
          "filled by wait_done()).")
      .def(
          "wait_done",
          [](const DeviceWindowSet& w, uint32_t seq, double timeout_s) {
            py::gil_scoped_release nogil;
            return w.wait_done(seq, timeout_s * 1e6);
          },
          py::arg("seq"), py::arg("timeout_s") = 1.0,
          "Spin until refresh `seq` has written its outputs (flag in mapped host memory); False on timeout, for "
          "an older tagged refresh, or when a newer refresh superseded it (never a mixed copy).")
      .def_property_readonly("superseded", &DeviceWindowSet::superseded)
      .def("invalidate", &DeviceWindowSet::invalidate)
      .def(
          "export_sorted",
          [](const DeviceWindowSet& w, uintptr_t dst, uintptr_t stream) {
            py::gil_scoped_release nogil;
            w.export_sorted(reinterpret_cast<float*>(dst), reinterpret_cast<void*>(stream));
          },
          py::arg("dst_ptr"), py::arg("stream"),
          "Enqueue every series' resident sorted window as [S][1 + W] floats (count, samples, +inf).")
      .def("stats", [](const DeviceWindowSet& w) {
        auto st = w.stats();
        py::dict d;
        d["refreshes"] = st.refreshes;
        d["rows_copied"] = st.rows_copied;
        d["bytes_copied"] = st.bytes_copied;
        d["memcpy_calls"] = st.memcpy_calls;
        d["launches"] = st.launches;
        d["incremental_launches"] = st.incremental_launches;
        d["pulled_series"] = st.pulled_series;
        d["inline_rows"] = st.inline_rows;
        return d;
      });

  // Direct, stateless kernel entry for tests/benchmarks: one device ring
  // [mask + 1][stride] float32 (time-major), window rows head - n .. head - 1, one
  // output row of 8 statistics per listed column.
  m.def(
      "window_stats_raw",
      [](uintptr_t base, uint64_t head, uint32_t stride, uint32_t mask, uint32_t n, const std::vector<uint32_t>& cols,
         uintptr_t out, uintptr_t stream, float p0, float p1, float p2) {
        if (cols.empty()) return;
        if (cols.size() > size_t(kMaxSeriesPerLaunch)) throw std::invalid_argument("too many series for one launch");
        if (n > mask + 1 || n > head) throw std::invalid_argument("n must be <= capacity and <= head");
        if (((mask + 1) & mask) != 0) throw std::invalid_argument("capacity must be a power of two");
        if (n > 32768) throw std::invalid_argument("window must be <= 32768");
        StatsArgs args{};
        args.pct[0] = p0;
        args.pct[1] = p1;
        args.pct[2] = p2;
        args.num_rings = 1;
        RingDesc& r = args.rings[0];
        for (size_t j = 0; j < cols.size(); ++j) {
          if (cols[j] >= stride) throw std::invalid_argument("column must be < stride");
          if (cols[j] != cols[0] + j) throw std::invalid_argument("columns must be one ascending run");
        }
        // the run of columns c0 .. c0 + count - 1 as a ring that starts at column c0
        r.base = reinterpret_cast<float*>(base) + cols[0];  // read only: no state, nothing entering
        r.head = head;
        r.pred_head0 = ~0ull;
        r.stride = stride;
        r.cols = uint32_t(cols.size());
        r.mask = mask;
        r.n = n;
        args.num_series = uint32_t(cols.size());
        int e;
        {
          py::gil_scoped_release nogil;
          e = launch_window_stats(args, sort_width_for(std::max<uint32_t>(n, 1)), reinterpret_cast<float*>(out),
                                  reinterpret_cast<void*>(stream));
        }
        if (e != 0) throw std::runtime_error("window_stats launch failed: " + std::to_string(e));
      },
      py::arg("base_ptr"), py::arg("head"), py::arg("stride"), py::arg("mask"), py::arg("n"), py::arg("cols"),
      py::arg("out_ptr"), py::arg("stream"), py::arg("p0") = 50.f, py::arg("p1") = 90.f, py::arg("p2") = 99.f);
  m.def("sort_width_for", &sort_width_for, py::arg("n"));
  m.def("rccl_load", &rccl_load, py::arg("lib_path") = "",
        "Load RCCL without creating anything; returns its version code (every rank, before the init).");
  m.def(
      "rccl_unique_id", [](const std::string& lib) { return py::bytes(rccl_unique_id(lib)); }, py::arg("lib_path") = "",
      "A new RCCL communicator's 128-byte unique id (rank 0; share it with every rank).");
  py::class_<RcclComm, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def(py::init([](int device, int nranks, int rank, py::bytes uid, const std::string& lib, double timeout_s) {
             std::string id = uid;
             py::gil_scoped_release nogil;  // collective: waits (at most timeout_s) until every rank joins
             return std::make_shared<RcclComm>(device, nranks, rank, id, lib, timeout_s);
           }),
           py::arg("device"), py::arg("nranks"), py::arg("rank"), py::arg("unique_id"), py::arg("lib_path") = "",
           py::arg("timeout_s") = 120.0)
      .def(
          "all_gather",
          [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t count, uintptr_t stream) {
            c.all_gather(reinterpret_cast<const float*>(send), reinterpret_cast<float*>(recv), count,
                         reinterpret_cast<void*>(stream));
          },
          py::arg("send_ptr"), py::arg("recv_ptr"), py::arg("count"), py::arg("stream"),
          "Enqueue ncclAllGather of `count` float32 per rank on `stream`.")
      .def(
          "all_gather_bytes",
          [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t bytes, uintptr_t stream) {
            c.all_gather_bytes(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), bytes,
                               reinterpret_cast<void*>(stream));
          },
          py::arg("send_ptr"), py::arg("recv_ptr"), py::arg("bytes"), py::arg("stream"),
          "Enqueue ncclAllGather of `bytes` per rank on `stream` (moved bit for bit).")
      .def(
          "all_reduce_sum_u32",
          [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t count, uintptr_t stream) {
            c.all_reduce_sum_u32(reinterpret_cast<const uint32_t*>(send), reinterpret_cast<uint32_t*>(recv), count,
                                 reinterpret_cast<void*>(stream));
          },
          py::arg("send_ptr"), py::arg("recv_ptr"), py::arg("count"), py::arg("stream"),
          "Enqueue ncclAllReduce(sum) of `count` uint32 on `stream`.")
      .def(
          "view",
          [](const RcclComm& c) {
            const RcclView v = c.view();
            py::dict d;
            d["nranks"] = v.nranks;
            d["rank"] = v.rank;
            d["device"] = v.device;
            return d;
          },
          "RCCL's own view: ncclCommCount, ncclCommUserRank, ncclCommCuDevice (-1 where refused).")
      .def("async_error", &RcclComm::async_error, "0 while healthy, else the communicator's ncclResult_t")
      .def("abort", &RcclComm::abort, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("init_seconds", &RcclComm::init_seconds)
      .def_property_readonly("nranks", &RcclComm::nranks)
      .def_property_readonly("rank", &RcclComm::rank);
  py::class_<HostPublisher, std::shared_ptr<HostPublisher>>(m, "HostPublisher")
      .def(py::init<int, bool>(), py::arg("device"), py::arg("tagged") = true)
      .def(
          "publish",
          [](HostPublisher& p, uintptr_t src, uintptr_t dst, uint32_t n, uintptr_t stream) {
            return p.publish(reinterpret_cast<const float*>(src), reinterpret_cast<float*>(dst), n,
                             reinterpret_cast<void*>(stream));
          },
          py::arg("src_ptr"), py::arg("dst_ptr"), py::arg("n"), py::arg("stream"),
          "Enqueue: copy n floats device -> pinned host, then publish; returns the sequence number.")
      .def(
          "wait",
          [](const HostPublisher& p, uint32_t seq, double timeout_s) {
            py::gil_scoped_release nogil;
            return p.wait(seq, timeout_s * 1e6);
          },
          py::arg("seq"), py::arg("timeout_s") = 1.0)
      .def_property_readonly("superseded", &HostPublisher::superseded,
                             "Tagged waits that found a newer publication in the words (no mixed copy returned).");
  m.def(
      "spin",
      [](uint32_t workgroups, double us, uintptr_t stream) {
        const int e = launch_spin(workgroups, us, reinterpret_cast<void*>(stream));
        if (e != 0) throw std::runtime_error("spin launch failed: " + std::to_string(e));
      },
      py::arg("workgroups"), py::arg("us"), py::arg("stream"),
      "Calibration load: `workgroups` one-wave workgroups, each busy for `us` microseconds.");
  m.def(
      "calib_gather32",
      [](uintptr_t src, uint64_t src_bytes, uintptr_t out, uint64_t out_bytes, uint32_t threads, uint32_t seed,
         uintptr_t stream) {
        const int e = launch_gather32(reinterpret_cast<const void*>(src), src_bytes, reinterpret_cast<void*>(out),
                                      out_bytes, threads, seed, reinterpret_cast<void*>(stream));
        if (e != 0) throw std::runtime_error("gather32 launch failed: " + std::to_string(e));
      },
      py::arg("src"), py::arg("src_bytes"), py::arg("out"), py::arg("out_bytes"), py::arg("threads"),
      py::arg("seed"), py::arg("stream"), "Calibration load: one 32 B read per thread at a random 32 B slot.");
  m.def(
      "calib_store64",
      [](uintptr_t dst, uint64_t dst_bytes, uint32_t threads, uintptr_t stream) {
        const int e = launch_store64(reinterpret_cast<void*>(dst), dst_bytes, threads, reinterpret_cast<void*>(stream));
        if (e != 0) throw std::runtime_error("store64 launch failed: " + std::to_string(e));
      },
      py::arg("dst"), py::arg("dst_bytes"), py::arg("threads"), py::arg("stream"),
      "Calibration load: one 64 B store per thread, 256 B apart.");
  m.def(
      "calib_store32",
      [](uintptr_t dst, uint64_t dst_bytes, uint32_t threads, uintptr_t stream) {
        const int e = launch_store32(reinterpret_cast<void*>(dst), dst_bytes, threads, reinterpret_cast<void*>(stream));
        if (e != 0) throw std::runtime_error("store32 launch failed: " + std::to_string(e));
      },
      py::arg("dst"), py::arg("dst_bytes"), py::arg("threads"), py::arg("stream"),
      "Calibration load: one 32 B store per thread, 256 B apart.");
  m.def(
      "node_select",
      [](uintptr_t node, uint32_t N, uint32_t S, uint32_t W, uintptr_t out, uintptr_t stream, float p0, float p1,
         float p2) {
        int e;
        {
          py::gil_scoped_release nogil;
          e = launch_node_select(reinterpret_cast<const float*>(node), N, S, W, p0, p1, p2, reinterpret_cast<float*>(out),
                                 reinterpret_cast<void*>(stream));
        }
        if (e != 0) throw std::runtime_error("node_select launch failed: " + std::to_string(e));
      },
      py::arg("node_ptr"), py::arg("n_ranks"), py::arg("num_series"), py::arg("window"), py::arg("out_ptr"),
      py::arg("stream"), py::arg("p0") = 50.f, py::arg("p1") = 90.f, py::arg("p2") = 99.f,
      "Order statistics over the union of N ranks' exported sorted windows: node [N][S][1 + W] -> out [S][8].");

  // ---- native frame renderer (csrc/frame_render.h) ---------------------------------
  py::class_<FramePlan, std::shared_ptr<FramePlan>>(m, "FramePlan")
      .def(py::init([](py::list panels, std::vector<int> sel_rows, int power_col, std::string headers_json,
                       std::string stats_columns_json, int num_columns, bool window, std::string window_gpus_json,
                       std::string window_series_json, std::string window_stats_json, std::vector<int> window_stat_idx,
                       int window_series) {
             auto p = std::make_shared<FramePlan>();
             for (auto item : panels) {
               auto t = item.cast<py::tuple>();
               if (t.size() != 8) throw std::invalid_argument("panel = (key_prefix, head, mid, tail, max_val, src, row, col)");
               PanelPlan pp;
               pp.key_prefix = t[0].cast<std::string>();
               pp.head = t[1].cast<std::string>();
               pp.mid = t[2].cast<std::string>();
               pp.tail = t[3].cast<std::string>();
               pp.max_val = t[4].cast<double>();
               pp.src = t[5].cast<int>();
               pp.row = t[6].cast<int>();
               pp.col = t[7].cast<int>();
               if (pp.src < 0 || pp.src > 2 || pp.col < 0 || (pp.src != 2 && pp.col >= num_columns))
                 throw std::invalid_argument("panel column out of range");
               p->panels.push_back(std::move(pp));
             }
             p->sel_rows = std::move(sel_rows);
             p->power_col = power_col;
             p->headers_json = std::move(headers_json);
             p->stats_columns_json = std::move(stats_columns_json);
             p->num_columns = num_columns;
             p->window = window;
             p->window_gpus_json = std::move(window_gpus_json);
             p->window_series_json = std::move(window_series_json);
             p->window_stats_json = std::move(window_stats_json);
             p->window_stat_idx = std::move(window_stat_idx);
             p->window_series = window_series;
             return p;
           }),
           py::arg("panels"), py::arg("sel_rows"), py::arg("power_col"), py::arg("headers_json"),
           py::arg("stats_columns_json"), py::arg("num_columns"), py::arg("window"), py::arg("window_gpus_json"),
           py::arg("window_series_json"), py::arg("window_stats_json"), py::arg("window_stat_idx"),
           py::arg("window_series"));
  m.def(
      "render_frame",
      [](const FramePlan& plan, py::array_t<double, py::array::c_style | py::array::forcecast> values, py::object window,
         const std::string& ts_key, const std::string& updated_json, bool as_bytes) -> py::object {
        if (values.ndim() != 2 || values.shape(1) != plan.num_columns) throw std::invalid_argument("values must be [G, C]");
        const int G = int(values.shape(0));
        for (const auto& p : plan.panels)
          if (p.src == 0 && p.row >= G) throw std::invalid_argument("panel row out of range");
        for (int r : plan.sel_rows)
          if (r < 0 || r >= G) throw std::invalid_argument("selected row out of range");
        py::array_t<float, py::array::c_style | py::array::forcecast> w;
        const float* wp = nullptr;
        if (plan.window && !window.is_none()) {
          w = window.cast<py::array_t<float, py::array::c_style | py::array::forcecast>>();
          if (w.ndim() != 3 || w.shape(0) != G || w.shape(1) != plan.window_series || w.shape(2) != 8)
            throw std::invalid_argument("window must be [G, S, 8]");
          wp = w.data();
        }
        thread_local std::string s;  // capacity kept across refreshes: no page faults per frame
        {
          py::gil_scoped_release nogil;  // renders beside Python threads
          render_frame_into(s, plan, values.data(), G, wp, ts_key, updated_json);
        }
        if (as_bytes) return py::bytes(s.data(), s.size());  // what a socket / file writer takes
        if (plan.all_ascii() && is_ascii(ts_key) && is_ascii(updated_json)) {
          // every byte is 7-bit (templates checked once, numbers are ASCII): build the
          // str by copy instead of a UTF-8 decode of the whole payload
          PyObject* o = PyUnicode_New(py::ssize_t(s.size()), 127);
          if (!o) throw py::error_already_set();
          std::memcpy(PyUnicode_1BYTE_DATA(o), s.data(), s.size());
          return py::reinterpret_steal<py::str>(o);
        }
        return py::str(s);
      },
      py::arg("plan"), py::arg("values"), py::arg("window"), py::arg("ts_key"), py::arg("updated_json"),
      py::arg("as_bytes") = false);
  m.def("py_round2_repr", [](double x) {
    std::string s;
    append_round2(s, x);
    return s;
  });
  m.def("py_float_repr", [](double x) {
    std::string s;
    append_py_float(s, x);
    return s;
  });
}
