// GPU-box probe: the device-counter read (rocprofiler-sdk device counting service) is the
// throughput floor of the refresh (~72 us per synchronous read of the 5-counter set,
// BASELINE.md). Does the ASYNC form overlap reads, i.e. is the floor the wait for one
// read's completion rather than the hardware / driver work per read?
//
//   sync      K synchronous reads back to back                  -> us per read
//   async     K ASYNC reads issued back to back, then wait for  -> us per read (issue and
//             all K x records in the buffer (flush + poll)          completion)
//   async-1   one ASYNC read, wait for its records               -> latency of one read
//   threadsT  T threads, synchronous reads on one context         -> us per read (serialised?)
//   pread     the same for the SMU metrics table (sysfs gpu_metrics)
//
// Build + run (gpurun): hipcc -O2 --offload-arch=gfx950 probe_counter_async.cpp -lrocprofiler-sdk
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#define RC(x)                                                                                         \
  do {                                                                                                \
    auto s_ = (x);                                                                                    \
    if (s_ != ROCPROFILER_STATUS_SUCCESS)                                                             \
      std::printf("%s -> %d %s\n", #x, (int)s_, rocprofiler_get_status_string(s_));                 \
  } while (0)

namespace {
using clk = std::chrono::steady_clock;
double us_since(clk::time_point t0) { return std::chrono::duration<double, std::micro>(clk::now() - t0).count(); }

const std::vector<std::string> kNames = {"GRBM_COUNT", "GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES",
                                         "TCC_EA0_RDREQ_sum", "TCC_EA0_WRREQ_sum"};
rocprofiler_agent_id_t g_agent{};
rocprofiler_counter_config_id_t g_cfg{};
rocprofiler_context_id_t g_ctx_sync{}, g_ctx_async{};
rocprofiler_buffer_id_t g_buf{};
size_t g_nrec = 0;
bool g_ok_sync = false, g_ok_async = false;
std::atomic<uint64_t> g_buffered{0};

void buffer_cb(rocprofiler_context_id_t, rocprofiler_buffer_id_t, rocprofiler_record_header_t** headers, size_t n,
               void*, uint64_t) {
  uint64_t c = 0;
  for (size_t i = 0; i < n; ++i)
    if (headers[i]->category == ROCPROFILER_BUFFER_CATEGORY_COUNTERS && headers[i]->kind == ROCPROFILER_COUNTER_RECORD_VALUE)
      ++c;
  g_buffered.fetch_add(c);
}

int tool_init(rocprofiler_client_finalize_t, void*) {
  std::vector<rocprofiler_agent_v0_t> agents;
  RC(rocprofiler_query_available_agents(
      ROCPROFILER_AGENT_INFO_VERSION_0,
      [](rocprofiler_agent_version_t, const void** arr, size_t n, void* ud) {
        auto* v = static_cast<std::vector<rocprofiler_agent_v0_t>*>(ud);
        for (size_t i = 0; i < n; ++i) {
          auto* a = static_cast<const rocprofiler_agent_v0_t*>(arr[i]);
          if (a->type == ROCPROFILER_AGENT_TYPE_GPU) v->push_back(*a);
        }
        return ROCPROFILER_STATUS_SUCCESS;
      },
      sizeof(rocprofiler_agent_v0_t), &agents));
  if (agents.empty()) return -1;
  g_agent = agents[0].id;
  std::vector<rocprofiler_counter_id_t> all;
  RC(rocprofiler_iterate_agent_supported_counters(
      g_agent,
      [](rocprofiler_agent_id_t, rocprofiler_counter_id_t* c, size_t n, void* ud) {
        auto* v = static_cast<std::vector<rocprofiler_counter_id_t>*>(ud);
        for (size_t i = 0; i < n; ++i) v->push_back(c[i]);
        return ROCPROFILER_STATUS_SUCCESS;
      },
      &all));
  std::unordered_map<std::string, std::pair<rocprofiler_counter_id_t, size_t>> byname;
  for (auto& c : all) {
    rocprofiler_counter_info_v1_t info{};
    if (rocprofiler_query_counter_info(c, ROCPROFILER_COUNTER_INFO_VERSION_1, &info) == ROCPROFILER_STATUS_SUCCESS)
      byname[info.name] = {c, size_t(info.dimensions_instances_count)};
  }
  std::vector<rocprofiler_counter_id_t> ids;
  for (auto& n : kNames) {
    auto it = byname.find(n);
    if (it == byname.end()) {
      std::printf("missing counter %s\n", n.c_str());
      continue;
    }
    ids.push_back(it->second.first);
    g_nrec += it->second.second;
  }
  RC(rocprofiler_create_counter_config(g_agent, ids.data(), ids.size(), &g_cfg));
  auto set_cfg = [](rocprofiler_context_id_t ctx, rocprofiler_agent_id_t, rocprofiler_device_counting_agent_cb_t set,
                    void*) { set(ctx, g_cfg); };
  RC(rocprofiler_create_context(&g_ctx_sync));
  g_ok_sync = rocprofiler_configure_device_counting_service(g_ctx_sync, rocprofiler_buffer_id_t{0}, g_agent, set_cfg,
                                                            nullptr) == ROCPROFILER_STATUS_SUCCESS;
  RC(rocprofiler_create_context(&g_ctx_async));
  RC(rocprofiler_create_buffer(g_ctx_async, 1 << 22, 1 << 21, ROCPROFILER_BUFFER_POLICY_LOSSLESS, buffer_cb, nullptr,
                               &g_buf));
  g_ok_async = rocprofiler_configure_device_counting_service(g_ctx_async, g_buf, g_agent, set_cfg, nullptr) ==
               ROCPROFILER_STATUS_SUCCESS;
  std::printf("configured: sync %d async %d, %zu records per read\n", g_ok_sync, g_ok_async, g_nrec);
  return 0;
}

void tool_fini(void*) {}

}  // namespace

extern "C" rocprofiler_tool_configure_result_t* probe_configure(uint32_t, const char*, uint32_t,
                                                                rocprofiler_client_id_t* id) {
  id->name = "rocmdash-probe-async";
  static rocprofiler_tool_configure_result_t cfg{sizeof(rocprofiler_tool_configure_result_t), &tool_init, &tool_fini,
                                                 nullptr};
  return &cfg;
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? std::atoi(argv[1]) : 200;
  RC(rocprofiler_force_configure(&probe_configure));
  int ndev = 0;
  (void)hipGetDeviceCount(&ndev);
  std::printf("hip devices %d, K = %d\n", ndev, K);
  if (!g_ok_sync) return 1;
  std::vector<rocprofiler_counter_record_t> recs(g_nrec + 256);

  // --- sync
  RC(rocprofiler_start_context(g_ctx_sync));
  for (int i = 0; i < 20; ++i) {
    size_t n = recs.size();
    rocprofiler_sample_device_counting_service(g_ctx_sync, {}, ROCPROFILER_COUNTER_FLAG_NONE, recs.data(), &n);
  }
  std::vector<double> lat;
  auto t0 = clk::now();
  for (int i = 0; i < K; ++i) {
    size_t n = recs.size();
    auto t = clk::now();
    rocprofiler_sample_device_counting_service(g_ctx_sync, {}, ROCPROFILER_COUNTER_FLAG_NONE, recs.data(), &n);
    lat.push_back(us_since(t));
  }
  const double sync_total = us_since(t0);
  std::sort(lat.begin(), lat.end());
  std::printf("{\"mode\": \"sync\", \"us_per_read\": %.2f, \"p50_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f}\n",
              sync_total / K, lat[K / 2], lat[K / 10], lat[9 * K / 10]);

  // --- T threads, synchronous reads on the one context: do reads overlap?
  for (int T = 2; T <= 4; ++T) {
    std::atomic<int> go{0};
    std::atomic<int> bad{0};
    auto worker = [&]() {
      std::vector<rocprofiler_counter_record_t> r(g_nrec + 256);
      while (!go.load()) {
      }
      for (int i = 0; i < K / T; ++i) {
        size_t n = r.size();
        if (rocprofiler_sample_device_counting_service(g_ctx_sync, {}, ROCPROFILER_COUNTER_FLAG_NONE, r.data(), &n) !=
                ROCPROFILER_STATUS_SUCCESS ||
            n != g_nrec)
          bad.fetch_add(1);
      }
    };
    std::vector<std::thread> th;
    for (int i = 0; i < T; ++i) th.emplace_back(worker);
    auto t1 = clk::now();
    go = 1;
    for (auto& x : th) x.join();
    std::printf("{\"mode\": \"threads%d_sync\", \"us_per_read\": %.2f, \"bad_reads\": %d}\n", T,
                us_since(t1) / (T * (K / T)), bad.load());
  }
  // counters stay monotonic when reads overlap: per counter, sum over instances
  {
    std::vector<rocprofiler_counter_record_t> r(g_nrec + 256);
    double prev = -1;
    int nonmono = 0;
    for (int i = 0; i < 50; ++i) {
      size_t n = r.size();
      rocprofiler_sample_device_counting_service(g_ctx_sync, {}, ROCPROFILER_COUNTER_FLAG_NONE, r.data(), &n);
      double tot = 0;
      for (size_t j = 0; j < n; ++j) tot += r[j].counter_value;
      if (tot < prev) ++nonmono;
      prev = tot;
    }
    std::printf("{\"mode\": \"monotonic_check\", \"non_monotonic\": %d}\n", nonmono);
  }
  RC(rocprofiler_stop_context(g_ctx_sync));

  // --- SMU metrics table: concurrent preads of the sysfs blob
  {
    int fd = -1;
    for (int c = 0; c < 64 && fd < 0; ++c) {
      const std::string path = "/sys/class/drm/card" + std::to_string(c) + "/device/gpu_metrics";
      fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    }
    if (fd >= 0) {
      for (int T = 1; T <= 3; ++T) {
        std::atomic<int> go{0};
        auto worker = [&]() {
          std::vector<char> buf(8192);
          while (!go.load()) {
          }
          for (int i = 0; i < K / T; ++i) (void)::pread(fd, buf.data(), buf.size(), 0);
        };
        std::vector<std::thread> th;
        for (int i = 0; i < T; ++i) th.emplace_back(worker);
        auto t1 = clk::now();
        go = 1;
        for (auto& x : th) x.join();
        std::printf("{\"mode\": \"gpu_metrics_pread_threads%d\", \"us_per_read\": %.2f}\n", T,
                    us_since(t1) / (T * (K / T)));
      }
      ::close(fd);
    }
  }

  // --- async
  if (g_ok_async) {
    RC(rocprofiler_start_context(g_ctx_async));
    auto wait_records = [&](uint64_t want, double limit_us) {
      auto t = clk::now();
      while (g_buffered.load() < want && us_since(t) < limit_us) {
        rocprofiler_flush_buffer(g_buf);
      }
      return g_buffered.load() >= want;
    };
    // one read at a time: latency through the async path
    std::vector<double> one;
    for (int i = 0; i < 50; ++i) {
      const uint64_t before = g_buffered.load();
      auto t = clk::now();
      auto st = rocprofiler_sample_device_counting_service(g_ctx_async, {}, ROCPROFILER_COUNTER_FLAG_ASYNC, nullptr, nullptr);
      if (st != ROCPROFILER_STATUS_SUCCESS) {
        std::printf("async sample -> %d %s\n", int(st), rocprofiler_get_status_string(st));
        break;
      }
      const bool ok = wait_records(before + g_nrec, 2e6);
      one.push_back(ok ? us_since(t) : -1.0);
    }
    if (!one.empty()) {
      std::sort(one.begin(), one.end());
      std::printf("{\"mode\": \"async_one\", \"p50_us\": %.2f, \"min_us\": %.2f}\n", one[one.size() / 2], one[0]);
    }
    // K reads issued back to back
    const uint64_t before = g_buffered.load();
    auto t2 = clk::now();
    int issued = 0;
    for (int i = 0; i < K; ++i)
      issued += rocprofiler_sample_device_counting_service(g_ctx_async, {}, ROCPROFILER_COUNTER_FLAG_ASYNC, nullptr,
                                                           nullptr) == ROCPROFILER_STATUS_SUCCESS;
    const double issue_us = us_since(t2);
    const bool ok = wait_records(before + uint64_t(issued) * g_nrec, 5e6);
    const double total_us = us_since(t2);
    std::printf(
        "{\"mode\": \"async_burst\", \"issued\": %d, \"complete\": %s, \"issue_us_per_read\": %.2f, "
        "\"us_per_read\": %.2f, \"records\": %llu}\n",
        issued, ok ? "true" : "false", issue_us / std::max(issued, 1), total_us / std::max(issued, 1),
        (unsigned long long)(g_buffered.load() - before));
    RC(rocprofiler_stop_context(g_ctx_async));
  }
  return 0;
}
