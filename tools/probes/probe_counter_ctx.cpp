// GPU-box probe: the device-counter read costs 72-140 us depending on the PROCESS
// (profiles/r01/probe_overlap.txt, interrupt_ab.txt). Is the cost a property of the
// counting context (its internal queue), so that a process could configure several
// contexts at start-up and keep the fastest? Configures kCtx sync contexts on one agent
// and times reads through each in turn (start, K reads, stop), twice round.
//
// Build + run (gpurun): hipcc -O2 --offload-arch=gfx950 probe_counter_ctx.cpp -lrocprofiler-sdk
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <string>
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
constexpr int kCtx = 4;
rocprofiler_agent_id_t g_agent{};
rocprofiler_counter_config_id_t g_cfg{};
rocprofiler_context_id_t g_ctx[kCtx]{};
bool g_ok[kCtx]{};
size_t g_nrec = 0;

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
  for (int i = 0; i < kCtx; ++i) {
    RC(rocprofiler_create_context(&g_ctx[i]));
    g_ok[i] = rocprofiler_configure_device_counting_service(g_ctx[i], rocprofiler_buffer_id_t{0}, g_agent, set_cfg,
                                                            nullptr) == ROCPROFILER_STATUS_SUCCESS;
  }
  std::printf("configured %d contexts, %zu records per read\n", kCtx, g_nrec);
  return 0;
}

void tool_fini(void*) {}

}  // namespace

extern "C" rocprofiler_tool_configure_result_t* probe_configure(uint32_t, const char*, uint32_t,
                                                                rocprofiler_client_id_t* id) {
  id->name = "rocmdash-probe-ctx";
  static rocprofiler_tool_configure_result_t cfg{sizeof(rocprofiler_tool_configure_result_t), &tool_init, &tool_fini,
                                                 nullptr};
  return &cfg;
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? std::atoi(argv[1]) : 400;
  RC(rocprofiler_force_configure(&probe_configure));
  int ndev = 0;
  (void)hipGetDeviceCount(&ndev);
  std::vector<rocprofiler_counter_record_t> recs(g_nrec + 256);
  std::printf("{");
  for (int round = 0; round < 2; ++round) {
    for (int c = 0; c < kCtx; ++c) {
      if (!g_ok[c]) {
        std::printf("\"r%d_ctx%d\": null, ", round, c);
        continue;
      }
      RC(rocprofiler_start_context(g_ctx[c]));
      for (int i = 0; i < 20; ++i) {
        size_t n = recs.size();
        rocprofiler_sample_device_counting_service(g_ctx[c], {}, ROCPROFILER_COUNTER_FLAG_NONE, recs.data(), &n);
      }
      std::vector<double> lat;
      for (int i = 0; i < K; ++i) {
        size_t n = recs.size();
        auto t = clk::now();
        rocprofiler_sample_device_counting_service(g_ctx[c], {}, ROCPROFILER_COUNTER_FLAG_NONE, recs.data(), &n);
        lat.push_back(us_since(t));
      }
      RC(rocprofiler_stop_context(g_ctx[c]));
      std::sort(lat.begin(), lat.end());
      std::printf("\"r%d_ctx%d\": %.1f, ", round, c, lat[K / 2]);
    }
  }
  std::printf("\"K\": %d}\n", K);
  return 0;
}
