// GPU-box probe: does rocprofiler-sdk device counting work unprivileged, and at what rate?
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#define RC(x) do { auto s_ = (x); if (s_ != ROCPROFILER_STATUS_SUCCESS) { std::printf("%s -> %d %s\n", #x, (int)s_, rocprofiler_get_status_string(s_)); } } while (0)


struct CSet { std::vector<std::string> names; rocprofiler_counter_config_id_t cfg{}; rocprofiler_context_id_t ctx{}; bool ok = false; size_t nrec = 0; };
static std::vector<CSet> g_sets = [](){ std::vector<CSet> v; v.reserve(64); return v; }();
static rocprofiler_agent_id_t g_agent{};
static std::unordered_map<uint64_t, std::string> g_names;

static int tool_init(rocprofiler_client_finalize_t, void*) {
  std::vector<rocprofiler_agent_v0_t> agents;
  RC(rocprofiler_query_available_agents(ROCPROFILER_AGENT_INFO_VERSION_0,
     [](rocprofiler_agent_version_t, const void** arr, size_t n, void* ud) {
       auto* v = static_cast<std::vector<rocprofiler_agent_v0_t>*>(ud);
       for (size_t i = 0; i < n; ++i) { auto* a = static_cast<const rocprofiler_agent_v0_t*>(arr[i]); if (a->type == ROCPROFILER_AGENT_TYPE_GPU) v->push_back(*a); }
       return ROCPROFILER_STATUS_SUCCESS; }, sizeof(rocprofiler_agent_v0_t), &agents));
  if (agents.empty()) return -1;
  g_agent = agents[0].id;
  std::vector<rocprofiler_counter_id_t> all;
  RC(rocprofiler_iterate_agent_supported_counters(g_agent,
     [](rocprofiler_agent_id_t, rocprofiler_counter_id_t* c, size_t n, void* ud) {
       auto* v = static_cast<std::vector<rocprofiler_counter_id_t>*>(ud); for (size_t i = 0; i < n; ++i) v->push_back(c[i]); return ROCPROFILER_STATUS_SUCCESS; }, &all));
  std::unordered_map<std::string, rocprofiler_counter_id_t> byname; std::unordered_map<std::string, size_t> inst;
  for (auto& c : all) { rocprofiler_counter_info_v1_t info{}; rocprofiler_query_counter_info(c, ROCPROFILER_COUNTER_INFO_VERSION_1, &info); g_names[c.handle] = info.name; byname[info.name] = c; inst[info.name] = info.dimensions_instances_count; }
  std::vector<std::vector<std::string>> cand = {
    {"GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES"},
    {"GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAVES"},
    {"TCC_EA0_RDREQ_sum", "TCC_EA0_WRREQ_sum"},
    {"TCC_EA0_RDREQ_sum"},
    {"GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES", "TCC_EA0_RDREQ_sum", "TCC_EA0_WRREQ_sum"},
    {"GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES", "TCC_EA0_RDREQ_sum", "TCC_EA0_WRREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_WRREQ_64B_sum"},
    {"GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES", "TCC_EA0_RDREQ", "TCC_EA0_WRREQ"},
    {"TCC_EA0_RDREQ", "TCC_EA0_WRREQ", "TCC_EA0_RDREQ_32B", "TCC_EA0_WRREQ_64B", "TCC_BUBBLE"},
    {"FETCH_SIZE"}, {"WRITE_SIZE"}, {"MfmaUtil"},
    {"GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU_MFMA_MOPS_BF16", "SQ_INSTS_VALU_MFMA_MOPS_F16"},
  };
  for (auto& names : cand) {
    CSet s; s.names = names; std::vector<rocprofiler_counter_id_t> ids; bool all_found = true;
    for (auto& n : names) { auto it = byname.find(n); if (it == byname.end()) { std::printf("  missing counter %s\n", n.c_str()); all_found = false; break; } ids.push_back(it->second); s.nrec += inst[n]; }
    if (!all_found) { g_sets.push_back(s); continue; }
    auto st = rocprofiler_create_counter_config(g_agent, ids.data(), ids.size(), &s.cfg);
    std::printf("set[%zu] {", g_sets.size()); for (auto& n : names) std::printf("%s,", n.c_str()); std::printf("} config -> %d %s (nrec %zu)\n", (int)st, rocprofiler_get_status_string(st), s.nrec);
    if (st == ROCPROFILER_STATUS_SUCCESS) {
      RC(rocprofiler_create_context(&s.ctx));
      g_sets.push_back(s);
      auto* ps = &g_sets.back();
      auto st2 = rocprofiler_configure_device_counting_service(ps->ctx, rocprofiler_buffer_id_t{0}, g_agent,
        [](rocprofiler_context_id_t ctx, rocprofiler_agent_id_t, rocprofiler_device_counting_agent_cb_t set, void* ud) { set(ctx, static_cast<CSet*>(ud)->cfg); }, ps);
      (void)st2;
      ps->ok = (st2 == ROCPROFILER_STATUS_SUCCESS);
      std::printf("   configure_device_counting -> %d\n", (int)st2);
    } else g_sets.push_back(s);
  }
  return 0;
}
static void tool_fini(void*) {}

extern "C" rocprofiler_tool_configure_result_t* probe_configure(uint32_t, const char*, uint32_t, rocprofiler_client_id_t* id) {
  id->name = "rocmdash-probe";
  static rocprofiler_tool_configure_result_t cfg{sizeof(rocprofiler_tool_configure_result_t), &tool_init, &tool_fini, nullptr};
  return &cfg;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
__global__ void mfma_burn(float* out, int iters) {
  f32x4 acc = {0, 0, 0, 0};
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (short)(threadIdx.x + i); b[i] = (short)(threadIdx.x * 3 + i); }
  for (int i = 0; i < iters; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}
__global__ void stream_copy(const float4* __restrict__ in, float4* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) out[i] = in[i];
}

int main() {
  RC(rocprofiler_force_configure(&probe_configure));
  int ndev = 0; (void)hipGetDeviceCount(&ndev);
  std::printf("hip devices %d\n", ndev);
  float* out; (void)hipMalloc(&out, 1 << 24);
  size_t nbytes = 1ull << 30; float4 *a, *b; (void)hipMalloc(&a, nbytes); (void)hipMalloc(&b, nbytes); (void)hipMemset(a, 1, nbytes);
  (void)hipDeviceSynchronize();
  for (auto& s : g_sets) {
    if (!s.ok) continue;
    std::printf("=== set {"); for (auto& n : s.names) std::printf("%s,", n.c_str()); std::printf("}\n");
    auto st = rocprofiler_start_context(s.ctx); std::printf("start -> %d\n", (int)st);
    std::vector<rocprofiler_counter_record_t> recs(s.nrec + 256);
    auto sample = [&](const char* tag) {
      size_t n = recs.size();
      auto t0 = std::chrono::steady_clock::now();
      auto r = rocprofiler_sample_device_counting_service(s.ctx, {}, ROCPROFILER_COUNTER_FLAG_NONE, recs.data(), &n);
      double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      std::unordered_map<std::string, double> agg;
      for (size_t i = 0; i < n; ++i) { rocprofiler_counter_id_t cid{}; rocprofiler_query_record_counter_id(recs[i].id, &cid); agg[g_names[cid.handle]] += recs[i].counter_value; }
      std::printf("  [%s] status=%d recs=%zu sample_us=%.1f :", tag, (int)r, n, us);
      for (auto& kv : agg) std::printf(" %s=%.6g", kv.first.c_str(), kv.second);
      std::printf("\n");
    };
    sample("idle0");
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
    sample("idle+10ms");
    hipLaunchKernelGGL(mfma_burn, dim3(2048), dim3(256), 0, 0, out, 20000);
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
    sample("during_mfma");
    (void)hipDeviceSynchronize();
    sample("after_mfma");
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(stream_copy, dim3(4096), dim3(256), 0, 0, a, b, nbytes / 16);
    (void)hipDeviceSynchronize();
    double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    sample("after_copy_20GiB");
    std::printf("  copy: %.2f ms\n", ms);
    auto t1 = std::chrono::steady_clock::now(); int ok = 0;
    for (int i = 0; i < 100; ++i) { size_t n = recs.size(); if (rocprofiler_sample_device_counting_service(s.ctx, {}, ROCPROFILER_COUNTER_FLAG_NONE, recs.data(), &n) == ROCPROFILER_STATUS_SUCCESS) ok++; }
    std::printf("  100 samples in %.2f ms (%d ok)\n", std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count(), ok);
    sample("final");
    RC(rocprofiler_stop_context(s.ctx));
  }
  return 0;
}
