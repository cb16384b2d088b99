// GPU-box probe: the synchronous device-counter read of the 5-counter set (~72 us) is
// the throughput floor of the refresh (profiles/r01/counter_cost_sets.jsonl: the cost
// grows with the number of counter instances read). Can the set be split over several
// device-counting contexts on the same agent, running at the same time, and read from
// one thread per context so the reads overlap?
//
//   combined   one context, all 5 counters                        (today's layout)
//   split2     {GRBM x2, MFMA} | {RDREQ, WRREQ}
//   split3     {GRBM x2, MFMA} | {RDREQ} | {WRREQ}
//
// For each layout: whether all of its contexts start together, us per read with the
// contexts read back to back on one thread and in parallel (one thread each), bad reads
// (status != success or a short record count), non-monotonic counter totals, and the
// HBM read/write rates and GRBM busy % seen under the same device-to-device copy load,
// so a split layout can be checked against the combined one.
//
// Build + run (gpurun): hipcc -O2 --offload-arch=gfx950 probe_counter_split.cpp -lrocprofiler-sdk
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {
using clk = std::chrono::steady_clock;
double us_since(clk::time_point t0) { return std::chrono::duration<double, std::micro>(clk::now() - t0).count(); }

struct Ctx {
  std::vector<std::string> names;
  rocprofiler_counter_config_id_t cfg{};
  rocprofiler_context_id_t ctx{};
  std::unordered_map<uint64_t, int> slot;
  size_t nrec = 0;
  bool ok = false;
};

const std::vector<std::vector<std::vector<std::string>>> kLayouts = {
    {{"GRBM_COUNT", "GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES", "TCC_EA0_RDREQ_sum", "TCC_EA0_WRREQ_sum"}},
    {{"GRBM_COUNT", "GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES"}, {"TCC_EA0_RDREQ_sum", "TCC_EA0_WRREQ_sum"}},
    {{"GRBM_COUNT", "GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES"}, {"TCC_EA0_RDREQ_sum"}, {"TCC_EA0_WRREQ_sum"}},
};
const char* kLayoutNames[] = {"combined", "split2", "split3"};
std::vector<std::vector<Ctx>> g_layouts;

int tool_init(rocprofiler_client_finalize_t, void*) {
  std::vector<rocprofiler_agent_v0_t> agents;
  rocprofiler_query_available_agents(
      ROCPROFILER_AGENT_INFO_VERSION_0,
      [](rocprofiler_agent_version_t, const void** arr, size_t n, void* ud) {
        auto* v = static_cast<std::vector<rocprofiler_agent_v0_t>*>(ud);
        for (size_t i = 0; i < n; ++i) {
          auto* a = static_cast<const rocprofiler_agent_v0_t*>(arr[i]);
          if (a->type == ROCPROFILER_AGENT_TYPE_GPU) v->push_back(*a);
        }
        return ROCPROFILER_STATUS_SUCCESS;
      },
      sizeof(rocprofiler_agent_v0_t), &agents);
  if (agents.empty()) return -1;
  const auto agent = agents[0].id;
  std::vector<rocprofiler_counter_id_t> all;
  rocprofiler_iterate_agent_supported_counters(
      agent,
      [](rocprofiler_agent_id_t, rocprofiler_counter_id_t* c, size_t n, void* ud) {
        auto* v = static_cast<std::vector<rocprofiler_counter_id_t>*>(ud);
        for (size_t i = 0; i < n; ++i) v->push_back(c[i]);
        return ROCPROFILER_STATUS_SUCCESS;
      },
      &all);
  std::unordered_map<std::string, std::pair<rocprofiler_counter_id_t, size_t>> byname;
  for (auto& c : all) {
    rocprofiler_counter_info_v1_t info{};
    if (rocprofiler_query_counter_info(c, ROCPROFILER_COUNTER_INFO_VERSION_1, &info) == ROCPROFILER_STATUS_SUCCESS)
      byname[info.name] = {c, size_t(info.dimensions_instances_count)};
  }
  g_layouts.reserve(kLayouts.size());
  for (auto& layout : kLayouts) {
    g_layouts.emplace_back();
    g_layouts.back().reserve(layout.size());  // the configure callbacks keep Ctx pointers
    for (auto& names : layout) {
      g_layouts.back().emplace_back();
      Ctx& c = g_layouts.back().back();
      c.names = names;
      std::vector<rocprofiler_counter_id_t> ids;
      for (auto& n : names) {
        auto it = byname.find(n);
        if (it == byname.end()) continue;
        c.slot[it->second.first.handle] = int(ids.size());
        ids.push_back(it->second.first);
        c.nrec += it->second.second;
      }
      if (rocprofiler_create_counter_config(agent, ids.data(), ids.size(), &c.cfg) != ROCPROFILER_STATUS_SUCCESS) continue;
      if (rocprofiler_create_context(&c.ctx) != ROCPROFILER_STATUS_SUCCESS) continue;
      c.ok = rocprofiler_configure_device_counting_service(
                 c.ctx, rocprofiler_buffer_id_t{0}, agent,
                 [](rocprofiler_context_id_t ctx, rocprofiler_agent_id_t, rocprofiler_device_counting_agent_cb_t set,
                    void* ud) { set(ctx, static_cast<Ctx*>(ud)->cfg); },
                 &c) == ROCPROFILER_STATUS_SUCCESS;
    }
  }
  return 0;
}

void tool_fini(void*) {}

// counter name -> summed (or maxed, GRBM) value of one read
bool read_ctx(Ctx& c, std::vector<rocprofiler_counter_record_t>& recs, std::unordered_map<std::string, double>& out) {
  size_t n = recs.size();
  if (rocprofiler_sample_device_counting_service(c.ctx, {}, ROCPROFILER_COUNTER_FLAG_NONE, recs.data(), &n) !=
          ROCPROFILER_STATUS_SUCCESS ||
      n != c.nrec)
    return false;
  std::vector<double> v(c.names.size(), 0.0);
  for (size_t i = 0; i < n; ++i) {
    rocprofiler_counter_id_t cid{};
    if (rocprofiler_query_record_counter_id(recs[i].id, &cid) != ROCPROFILER_STATUS_SUCCESS) continue;
    auto it = c.slot.find(cid.handle);
    if (it == c.slot.end()) continue;
    const bool mx = c.names[it->second].rfind("GRBM_", 0) == 0;
    v[it->second] = mx ? std::max(v[it->second], recs[i].counter_value) : v[it->second] + recs[i].counter_value;
  }
  for (size_t i = 0; i < v.size(); ++i) out[c.names[i]] = v[i];
  return true;
}

}  // namespace

extern "C" rocprofiler_tool_configure_result_t* probe_configure(uint32_t, const char*, uint32_t,
                                                                rocprofiler_client_id_t* id) {
  id->name = "rocmdash-probe-split";
  static rocprofiler_tool_configure_result_t cfg{sizeof(rocprofiler_tool_configure_result_t), &tool_init, &tool_fini,
                                                 nullptr};
  return &cfg;
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? std::atoi(argv[1]) : 300;
  rocprofiler_force_configure(&probe_configure);
  if (hipSetDevice(0) != hipSuccess) return 1;

  // background HBM load: D2D copies of 1 GiB on their own stream until told to stop
  const size_t bytes = size_t(1) << 30;
  void *a = nullptr, *b = nullptr;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
  (void)hipMemset(a, 1, bytes);
  (void)hipDeviceSynchronize();
  std::atomic<bool> stop{false};
  std::thread load([&]() {
    (void)hipSetDevice(0);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    while (!stop.load()) {
      (void)hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, s);
      (void)hipStreamSynchronize(s);
    }
    (void)hipStreamDestroy(s);
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(200));

  for (size_t L = 0; L < g_layouts.size(); ++L) {
    auto& ctxs = g_layouts[L];
    bool cfg_ok = true;
    for (auto& c : ctxs) cfg_ok = cfg_ok && c.ok;
    std::vector<int> started;
    std::string start_err;
    for (auto& c : ctxs) {
      auto st = cfg_ok ? rocprofiler_start_context(c.ctx) : ROCPROFILER_STATUS_ERROR;
      started.push_back(st == ROCPROFILER_STATUS_SUCCESS);
      if (st != ROCPROFILER_STATUS_SUCCESS && start_err.empty()) start_err = rocprofiler_get_status_string(st);
    }
    const bool all_started = std::all_of(started.begin(), started.end(), [](int s) { return s; });
    std::printf("{\"layout\": \"%s\", \"contexts\": %zu, \"configured\": %s, \"started\": %s, \"start_error\": \"%s\"",
                kLayoutNames[L], ctxs.size(), cfg_ok ? "true" : "false", all_started ? "true" : "false",
                start_err.c_str());
    if (all_started) {
      std::vector<std::vector<rocprofiler_counter_record_t>> recs(ctxs.size());
      for (size_t i = 0; i < ctxs.size(); ++i) recs[i].resize(ctxs[i].nrec + 256);
      std::unordered_map<std::string, double> v0, v1;
      int bad = 0;
      for (int w = 0; w < 20; ++w)
        for (size_t i = 0; i < ctxs.size(); ++i) bad += !read_ctx(ctxs[i], recs[i], v0);
      // back to back on one thread
      std::vector<double> lat;
      for (int k = 0; k < K; ++k) {
        auto t = clk::now();
        for (size_t i = 0; i < ctxs.size(); ++i) bad += !read_ctx(ctxs[i], recs[i], v1);
        lat.push_back(us_since(t));
      }
      std::sort(lat.begin(), lat.end());
      // in parallel, one thread per context, released together per round
      std::unordered_map<std::string, double> p0;
      for (size_t i = 0; i < ctxs.size(); ++i) read_ctx(ctxs[i], recs[i], p0);
      std::atomic<int> round{-1}, done{0}, pbad{0}, nonmono{0};
      std::vector<std::thread> th;
      for (size_t i = 0; i < ctxs.size(); ++i) {
        th.emplace_back([&, i]() {
          std::unordered_map<std::string, double> cur, prev;
          for (int k = 0; k < K; ++k) {
            while (round.load(std::memory_order_acquire) < k) {
            }
            if (!read_ctx(ctxs[i], recs[i], cur)) pbad.fetch_add(1);
            for (auto& kv : cur)
              if (prev.count(kv.first) && kv.second < prev[kv.first]) nonmono.fetch_add(1);
            prev = cur;
            done.fetch_add(1, std::memory_order_acq_rel);
          }
        });
      }
      std::vector<double> plat;
      auto tp0 = clk::now();
      for (int k = 0; k < K; ++k) {
        auto t = clk::now();
        round.store(k, std::memory_order_release);
        while (done.load(std::memory_order_acquire) < int(ctxs.size()) * (k + 1)) {
        }
        plat.push_back(us_since(t));
      }
      for (auto& x : th) x.join();
      const double dt_s = us_since(tp0) * 1e-6;
      std::unordered_map<std::string, double> p1;
      for (size_t i = 0; i < ctxs.size(); ++i) read_ctx(ctxs[i], recs[i], p1);
      std::sort(plat.begin(), plat.end());
      auto delta = [&](const char* n) { return p1.count(n) && p0.count(n) ? (p1[n] - p0[n]) : -1.0; };
      const double busy = delta("GRBM_COUNT") > 0 ? 100.0 * delta("GRBM_GUI_ACTIVE") / delta("GRBM_COUNT") : -1.0;
      std::printf(
          ", \"serial_p50_us\": %.2f, \"serial_p90_us\": %.2f, \"parallel_p50_us\": %.2f, \"parallel_p90_us\": %.2f, "
          "\"bad_serial\": %d, \"bad_parallel\": %d, \"non_monotonic\": %d, \"hbm_read_GBps\": %.1f, "
          "\"hbm_write_GBps\": %.1f, \"gfx_busy_pct\": %.1f, \"mfma_cycles_per_s\": %.3g",
          lat[K / 2], lat[9 * K / 10], plat[K / 2], plat[9 * K / 10], bad, pbad.load(), nonmono.load(),
          delta("TCC_EA0_RDREQ_sum") * 128.0 / dt_s / 1e9, delta("TCC_EA0_WRREQ_sum") * 64.0 / dt_s / 1e9, busy,
          delta("SQ_VALU_MFMA_BUSY_CYCLES") / dt_s);
    }
    std::printf("}\n");
    std::fflush(stdout);
    for (size_t i = 0; i < ctxs.size(); ++i)
      if (started[i]) rocprofiler_stop_context(ctxs[i].ctx);
  }
  stop = true;
  load.join();
  (void)hipFree(a);
  (void)hipFree(b);
  return 0;
}
