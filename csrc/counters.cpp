// rocprofiler-sdk device-counting source (agent-wide hardware counters, no kernel
// serialisation). Reference counterpart: none - the reference has no HW counters.
//
// The SDK is dlopen()ed only when counters are enabled, so processes that never ask
// for counters (tests, rocprofv3 --pmc runs of other code) never load it. The tool
// registers through rocprofiler_force_configure(), which must run before the HSA
// runtime initialises: counters_preinit() is called by rocmdash.runtime before any
// HIP call (see rocmdash/runtime/native.py).
//
// Counters (verified on the MI355X box, profiles/probe_devcount2.txt):
//   GRBM_COUNT, GRBM_GUI_ACTIVE   8 instances (per XCD) -> max
//   SQ_VALU_MFMA_BUSY_CYCLES      32 instances (per SE) -> sum; = 16 x #16x16x32 MFMAs
//   TCC_EA0_RDREQ_DRAM_32B_sum    memory-side read traffic in 32 B units (a 64 B request
//                                 counts 2, a 128 B one 4): read bytes = 32 x delta for
//                                 every request size (TCC_EA0_RDREQ_sum x 128 B only when
//                                 the agent lacks it)
//   TCC_EA0_WRREQ_WRITE_DRAM_32B_sum  memory-side write traffic in 32 B units (gfx950;
//                                 a 64 B request counts 2): write bytes = 32 x delta from ONE
//                                 counter. It replaces the pair below, which costs one more
//                                 128-instance TCC counter on every read (+~27 us per read,
//                                 profiles/r06/counter_ab/)
//   TCC_EA0_WRREQ_sum, _WRREQ_64B_sum  write requests, and the 64 B ones among them:
//                                 write bytes = 64 x WR64 + 32 x (WR - WR64) (rocprofiler's
//                                 WRITE_SIZE for gfx950), used only where the agent lacks
//                                 the 32 B-unit counter
//   SQ_BUSY_CU_CYCLES             per-SE sums of per-CU busy quad-cycles -> sum; CU active
//                                 = sum / (GRBM_COUNT delta x CUs) x kCuBusyScale, the
//                                 scale calibrated with one-wave spin kernels on a known
//                                 number of CUs (tests/test_gpu.py)
// Known-traffic kernels under rocprofv3 --pmc on gfx950 (profiles/r05/hbm_bytes/): a 1 GiB
// copy -> RDREQ_DRAM_32B = 1 GiB / 32 and WRREQ = WRREQ_64B = 1 GiB / 64 exactly; random
// 32 B reads -> one 128 B line fill each (RDREQ_128B = reads, RDREQ_DRAM_32B = 4 x reads:
// the memory side moves whole L2 lines); 64 B stores at a 256 B stride -> WRREQ_64B = stores.
// TCC_BUBBLE (rocprofiler's FETCH_SIZE term for 128 B reads) stays 0 on gfx950, which is
// why FETCH_SIZE under-reports wide streams (MI355X_MICROARCH.md). The EA requests include
// Infinity Cache (MALL) hits: a 64 MiB copy loop counts every byte, so the series are
// memory-side (fabric) traffic, an upper bound of what the HBM stacks moved. All counters
// are cumulative since context start; rates are deltas over the host's steady-clock
// interval.
#include <dlfcn.h>

#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "sources.h"

namespace rocmdash {
namespace {

struct Api {
  void* lib = nullptr;
  decltype(&rocprofiler_force_configure) force_configure = nullptr;
  decltype(&rocprofiler_query_available_agents) query_agents = nullptr;
  decltype(&rocprofiler_iterate_agent_supported_counters) iterate_counters = nullptr;
  decltype(&rocprofiler_query_counter_info) counter_info = nullptr;
  decltype(&rocprofiler_create_counter_config) create_config = nullptr;
  decltype(&rocprofiler_create_context) create_context = nullptr;
  decltype(&rocprofiler_configure_device_counting_service) configure_devcount = nullptr;
  decltype(&rocprofiler_start_context) start_context = nullptr;
  decltype(&rocprofiler_stop_context) stop_context = nullptr;
  decltype(&rocprofiler_sample_device_counting_service) sample = nullptr;
  decltype(&rocprofiler_query_record_counter_id) record_counter_id = nullptr;
  decltype(&rocprofiler_get_status_string) status_string = nullptr;

  bool load() {
    if (lib) return true;
    lib = dlopen("librocprofiler-sdk.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!lib) lib = dlopen("/opt/rocm/lib/librocprofiler-sdk.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!lib) return false;
#define RD_SYM(field, name) field = reinterpret_cast<decltype(field)>(dlsym(lib, #name)); if (!field) return false;
    RD_SYM(force_configure, rocprofiler_force_configure)
    RD_SYM(query_agents, rocprofiler_query_available_agents)
    RD_SYM(iterate_counters, rocprofiler_iterate_agent_supported_counters)
    RD_SYM(counter_info, rocprofiler_query_counter_info)
    RD_SYM(create_config, rocprofiler_create_counter_config)
    RD_SYM(create_context, rocprofiler_create_context)
    RD_SYM(configure_devcount, rocprofiler_configure_device_counting_service)
    RD_SYM(start_context, rocprofiler_start_context)
    RD_SYM(stop_context, rocprofiler_stop_context)
    RD_SYM(sample, rocprofiler_sample_device_counting_service)
    RD_SYM(record_counter_id, rocprofiler_query_record_counter_id)
    RD_SYM(status_string, rocprofiler_get_status_string)
#undef RD_SYM
    return true;
  }
};

Api g_api;

enum Agg { AGG_SUM, AGG_MAX };

struct AgentCtx {
  rocprofiler_agent_id_t agent{};
  uint64_t bdf = 0;  // domain<<32 | location_id, comparable with amd-smi bdf ids
  int ordinal = 0;   // order among GPU agents
  uint32_t simds = 0;
  uint32_t cus = 0;
  rocprofiler_context_id_t ctx{};
  rocprofiler_counter_config_id_t cfg{};
  std::vector<std::string> names;                    // selected counters
  std::unordered_map<uint64_t, int> slot_of_counter;  // counter handle -> slot in names
  std::vector<Agg> agg;
  size_t nrec = 0;
  bool ok = false;
  bool started = false;
  // one sampler at a time per agent; timed: a read that never returned (a hung lane,
  // rocmdash/runtime/lanes.py) must not block a fresh lane's construction forever
  std::timed_mutex mu;
};

std::mutex g_mu;
std::vector<std::string> g_requested;
int g_only_ordinal = -1;  // >= 0: configure only this GPU agent (rank-per-GPU processes)
uint64_t g_only_bdf = 0;  // != 0: configure only the GPU agent at this PCI address (preferred)
std::vector<AgentCtx*> g_agents;  // owned, never freed (tool lifetime = process)
std::atomic<int> g_state{0};      // 0 none, 1 configured, -1 failed
std::string g_status = "not initialised";

bool counter_optional(const std::string& n) {
  return n == "GRBM_COUNT" || n == "SQ_BUSY_CU_CYCLES" || n == "TCC_EA0_WRREQ_64B_sum";
}

// A requested counter that stands in for a better one: skipped when the agent has that
// one and it was requested too (traffic in 32 B units replaces request counts x a size).
const char* counter_preferred_over(const std::string& n) {
  if (n == "TCC_EA0_RDREQ_sum") return "TCC_EA0_RDREQ_DRAM_32B_sum";
  if (n == "TCC_EA0_WRREQ_sum" || n == "TCC_EA0_WRREQ_64B_sum") return "TCC_EA0_WRREQ_WRITE_DRAM_32B_sum";
  return nullptr;
}

// SQ_BUSY_CU_CYCLES counts quad-cycles (4 clocks) per busy CU: 4 x sum / (cycles x CUs)
// is the busy share of CU-cycles
constexpr double kCuBusyScale = 4.0;

int tool_init(rocprofiler_client_finalize_t, void*) {
  std::vector<rocprofiler_agent_v0_t> agents;
  auto st = g_api.query_agents(
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
  if (st != ROCPROFILER_STATUS_SUCCESS) {
    g_status = std::string("query agents: ") + g_api.status_string(st);
    return 0;
  }
  int ordinal = 0;
  for (auto& a : agents) {
    const int this_ordinal = ordinal++;
    // A rank-per-GPU process touches only its own GPU's counter hardware, so that
    // N processes on one node never configure the same agent twice.
    const uint64_t bdf = (uint64_t(a.domain) << 32) | uint64_t(a.location_id);
    if (g_only_bdf != 0 ? bdf != g_only_bdf : (g_only_ordinal >= 0 && this_ordinal != g_only_ordinal)) continue;
    auto* ac = new AgentCtx;
    ac->agent = a.id;
    ac->bdf = bdf;
    ac->ordinal = this_ordinal;
    ac->simds = a.cu_count * a.simd_per_cu;
    ac->cus = a.cu_count;
    std::vector<rocprofiler_counter_id_t> all;
    g_api.iterate_counters(
        a.id,
        [](rocprofiler_agent_id_t, rocprofiler_counter_id_t* c, size_t n, void* ud) {
          auto* v = static_cast<std::vector<rocprofiler_counter_id_t>*>(ud);
          for (size_t i = 0; i < n; ++i) v->push_back(c[i]);
          return ROCPROFILER_STATUS_SUCCESS;
        },
        &all);
    std::unordered_map<std::string, std::pair<rocprofiler_counter_id_t, size_t>> byname;
    for (auto& c : all) {
      rocprofiler_counter_info_v1_t info{};
      if (g_api.counter_info(c, ROCPROFILER_COUNTER_INFO_VERSION_1, &info) == ROCPROFILER_STATUS_SUCCESS)
        byname[info.name] = {c, size_t(info.dimensions_instances_count)};
    }
    // Try the full request, then without optional counters (PMC slot limits).
    for (int attempt = 0; attempt < 2 && !ac->ok; ++attempt) {
      std::vector<rocprofiler_counter_id_t> ids;
      ac->names.clear();
      ac->slot_of_counter.clear();
      ac->agg.clear();
      ac->nrec = 0;
      for (auto& n : g_requested) {
        if (attempt == 1 && counter_optional(n)) continue;
        auto it = byname.find(n);
        if (it == byname.end()) continue;
        if (const char* better = counter_preferred_over(n)) {
          if (byname.count(better) && std::find(g_requested.begin(), g_requested.end(), better) != g_requested.end())
            continue;
        }
        ac->slot_of_counter[it->second.first.handle] = int(ac->names.size());
        ac->names.push_back(n);
        ac->agg.push_back(n.rfind("GRBM_", 0) == 0 ? AGG_MAX : AGG_SUM);
        ids.push_back(it->second.first);
        ac->nrec += it->second.second;
      }
      if (ids.empty()) break;
      if (g_api.create_config(a.id, ids.data(), ids.size(), &ac->cfg) != ROCPROFILER_STATUS_SUCCESS) continue;
      if (g_api.create_context(&ac->ctx) != ROCPROFILER_STATUS_SUCCESS) break;
      auto cs = g_api.configure_devcount(
          ac->ctx, rocprofiler_buffer_id_t{0}, a.id,
          [](rocprofiler_context_id_t ctx, rocprofiler_agent_id_t, rocprofiler_device_counting_agent_cb_t set,
             void* ud) { set(ctx, static_cast<AgentCtx*>(ud)->cfg); },
          ac);
      ac->ok = cs == ROCPROFILER_STATUS_SUCCESS;
    }
    g_agents.push_back(ac);
  }
  g_status = "configured " + std::to_string(g_agents.size()) + " GPU agent(s)";
  return 0;
}

void tool_fini(void*) {}

rocprofiler_tool_configure_result_t* configure(uint32_t, const char*, uint32_t, rocprofiler_client_id_t* id) {
  id->name = "rocmdash-device-counters";
  static rocprofiler_tool_configure_result_t cfg{sizeof(rocprofiler_tool_configure_result_t), &tool_init,
                                                 &tool_fini, nullptr};
  return &cfg;
}

class CounterSource final : public Source {
 public:
  explicit CounterSource(AgentCtx* ac) : ac_(ac) {
    std::unique_lock<std::timed_mutex> lk(ac_->mu, std::defer_lock);
    if (!lk.try_lock_for(std::chrono::seconds(2)))
      throw std::runtime_error("device counters: the agent's counting context is busy (a read did not return)");
    if (!ac_->started) {
      auto st = g_api.start_context(ac_->ctx);
      if (st != ROCPROFILER_STATUS_SUCCESS)
        throw std::runtime_error(std::string("rocprofiler_start_context: ") + g_api.status_string(st));
      ac_->started = true;
    }
    if (const char* v = std::getenv("ROCMDASH_COUNTER_DUTY_US")) duty_us_ = std::atoi(v);
    if (duty_us_ > 0 && ac_->started && g_api.stop_context(ac_->ctx) == ROCPROFILER_STATUS_SUCCESS)
      ac_->started = false;  // duty mode: the context runs only around reads
    recs_.resize(ac_->nrec + 64);
    cur_.assign(ac_->names.size(), 0.0);
    prev_.assign(ac_->names.size(), 0.0);
    for (size_t i = 0; i < ac_->names.size(); ++i) {
      const auto& n = ac_->names[i];
      if (n == "GRBM_COUNT") i_count_ = int(i);
      else if (n == "GRBM_GUI_ACTIVE") i_active_ = int(i);
      else if (n == "SQ_VALU_MFMA_BUSY_CYCLES") i_mfma_ = int(i);
      else if (n == "TCC_EA0_RDREQ_sum") i_rd_ = int(i);
      else if (n == "TCC_EA0_RDREQ_DRAM_32B_sum") i_rd32_ = int(i);
      else if (n == "TCC_EA0_WRREQ_sum") i_wr_ = int(i);
      else if (n == "TCC_EA0_WRREQ_64B_sum") i_wr64_ = int(i);
      else if (n == "TCC_EA0_WRREQ_WRITE_DRAM_32B_sum") i_wr32_ = int(i);
      else if (n == "SQ_BUSY_CU_CYCLES") i_cu_ = int(i);
    }
  }
  uint32_t width() const override { return CTR_NUM_FIELDS; }
  std::string kind() const override { return "counter"; }
  std::string backend() const override { return "rocprofiler"; }
  uint32_t simds() const { return ac_->simds; }
  uint32_t cus() const { return ac_->cus; }
  // the configured set's size: a read's cost grows with the instance records it returns
  std::vector<std::pair<std::string, double>> counts() const override {
    return {{"counters", double(ac_->names.size())}, {"records", double(ac_->nrec)}};
  }

  // One read of every counter into `into` (instances aggregated), and when it was taken.
  bool read(std::vector<double>& into, std::chrono::steady_clock::time_point& when) {
    size_t n = recs_.size();
    rocprofiler_status_t st;
    {
      std::lock_guard<std::timed_mutex> lk(ac_->mu);
      st = g_api.sample(ac_->ctx, rocprofiler_user_data_t{}, ROCPROFILER_COUNTER_FLAG_NONE, recs_.data(), &n);
      when = std::chrono::steady_clock::now();
    }
    if (st != ROCPROFILER_STATUS_SUCCESS) return false;
    std::fill(into.begin(), into.end(), 0.0);
    for (size_t i = 0; i < n; ++i) {
      rocprofiler_counter_id_t cid{};
      if (g_api.record_counter_id(recs_[i].id, &cid) != ROCPROFILER_STATUS_SUCCESS) continue;
      auto it = ac_->slot_of_counter.find(cid.handle);
      if (it == ac_->slot_of_counter.end()) continue;
      const int s = it->second;
      if (ac_->agg[s] == AGG_MAX) into[s] = std::max(into[s], recs_[i].counter_value);
      else into[s] += recs_[i].counter_value;
    }
    return true;
  }

  bool sample(float* row) override {
    constexpr float nan = std::numeric_limits<float>::quiet_NaN();
    for (int i = 0; i < CTR_NUM_FIELDS; ++i) row[i] = nan;
    if (duty_us_ > 0) return sample_duty(row);
    std::chrono::steady_clock::time_point now;
    if (!read(cur_, now)) return false;
    const bool have_prev = have_prev_;
    const double dt = std::chrono::duration<double>(now - t_prev_).count();
    t_prev_ = now;
    prev_.swap(cur_);  // prev_ now holds this sample, cur_ the previous one
    have_prev_ = true;
    if (!have_prev || dt <= 0) return false;
    rates(row, dt);
    return true;
  }

 private:
  // Experiment (ROCMDASH_COUNTER_DUTY_US > 0): the counting context runs only around a
  // read - start, read, wait duty_us, read, stop - so the runtime's completion poller has
  // nothing to poll between reads; the rates cover that window, not the whole period.
  bool sample_duty(float* row) {
    {
      std::lock_guard<std::timed_mutex> lk(ac_->mu);
      if (!ac_->started && g_api.start_context(ac_->ctx) != ROCPROFILER_STATUS_SUCCESS) return false;
      ac_->started = true;
    }
    std::chrono::steady_clock::time_point t0, t1;
    const bool ok = read(cur_, t0) && (std::this_thread::sleep_for(std::chrono::microseconds(duty_us_)), true) &&
                    read(prev_, t1);
    {
      std::lock_guard<std::timed_mutex> lk(ac_->mu);
      if (g_api.stop_context(ac_->ctx) == ROCPROFILER_STATUS_SUCCESS) ac_->started = false;
    }
    const double dt = std::chrono::duration<double>(t1 - t0).count();
    if (!ok || dt <= 0) return false;
    rates(row, dt);
    return true;
  }

  // rates from prev_ (newer) - cur_ (older) over dt seconds
  void rates(float* row, double dt) {
    auto d = [&](int i) { return i < 0 ? -1.0 : prev_[i] - cur_[i]; };
    const double cyc = i_count_ >= 0 ? d(i_count_) : d(i_active_);
    if (i_mfma_ >= 0 && cyc > 0 && ac_->simds) row[CTR_MFMA_UTIL] = float(std::min(100.0, 100.0 * d(i_mfma_) / (cyc * ac_->simds)));
    if (i_rd32_ >= 0) row[CTR_HBM_READ_GBPS] = float(d(i_rd32_) * 32.0 / dt / 1e9);
    else if (i_rd_ >= 0) row[CTR_HBM_READ_GBPS] = float(d(i_rd_) * 128.0 / dt / 1e9);
    if (i_wr32_ >= 0) {
      row[CTR_HBM_WRITE_GBPS] = float(d(i_wr32_) * 32.0 / dt / 1e9);
    } else if (i_wr_ >= 0 && i_wr64_ >= 0) {
      const double w64 = std::min(d(i_wr64_), d(i_wr_));
      row[CTR_HBM_WRITE_GBPS] = float((64.0 * w64 + 32.0 * (d(i_wr_) - w64)) / dt / 1e9);
    } else if (i_wr_ >= 0) {
      row[CTR_HBM_WRITE_GBPS] = float(d(i_wr_) * 64.0 / dt / 1e9);
    }
    if (i_count_ >= 0 && i_active_ >= 0 && d(i_count_) > 0)
      row[CTR_GFX_BUSY] = float(std::min(100.0, 100.0 * d(i_active_) / d(i_count_)));
    if (i_cu_ >= 0 && cyc > 0 && ac_->cus)
      row[CTR_CU_ACTIVE] = float(std::min(100.0, 100.0 * kCuBusyScale * d(i_cu_) / (cyc * ac_->cus)));
  }

  AgentCtx* ac_;
  std::vector<rocprofiler_counter_record_t> recs_;
  std::vector<double> cur_, prev_;
  std::chrono::steady_clock::time_point t_prev_{};
  bool have_prev_ = false;
  int i_count_ = -1, i_active_ = -1, i_mfma_ = -1, i_rd_ = -1, i_rd32_ = -1, i_wr_ = -1, i_wr64_ = -1, i_wr32_ = -1, i_cu_ = -1;
  int duty_us_ = 0;
};

// One physical GPU in a compute-partition mode (DPX / QPX / CPX): its partitions are
// separate agents with the GPU's PCI address, each counting only its own XCDs and L2
// slices. The GPU's row: MFMA busy and CU active over all its SIMDs / CUs (weighted by
// each partition's share), HBM traffic summed, gfx busy averaged. A row is produced only
// when every partition was read (a missing partition would understate the sums).
class GroupCounterSource final : public Source {
 public:
  explicit GroupCounterSource(std::vector<std::shared_ptr<CounterSource>> parts) : parts_(std::move(parts)) {}
  uint32_t width() const override { return CTR_NUM_FIELDS; }
  std::string kind() const override { return "counter"; }
  std::string backend() const override { return "rocprofiler"; }
  std::vector<std::pair<std::string, double>> counts() const override {
    return {{"partitions", double(parts_.size())}};
  }

  bool sample(float* row) override {
    constexpr float nan = std::numeric_limits<float>::quiet_NaN();
    double mfma = 0, simds = 0, rd = 0, wr = 0, gfx = 0, cu = 0, cus = 0;
    int ok = 0, n_gfx = 0;
    bool have_mfma = false, have_rd = false, have_wr = false, have_cu = false;
    float r[CTR_NUM_FIELDS];
    for (auto& p : parts_) {
      if (!p->sample(r)) continue;
      ++ok;
      if (std::isfinite(r[CTR_MFMA_UTIL])) mfma += double(r[CTR_MFMA_UTIL]) * p->simds(), simds += p->simds(), have_mfma = true;
      if (std::isfinite(r[CTR_HBM_READ_GBPS])) rd += r[CTR_HBM_READ_GBPS], have_rd = true;
      if (std::isfinite(r[CTR_HBM_WRITE_GBPS])) wr += r[CTR_HBM_WRITE_GBPS], have_wr = true;
      if (std::isfinite(r[CTR_GFX_BUSY])) gfx += r[CTR_GFX_BUSY], ++n_gfx;
      if (std::isfinite(r[CTR_CU_ACTIVE])) cu += double(r[CTR_CU_ACTIVE]) * p->cus(), cus += p->cus(), have_cu = true;
    }
    for (int i = 0; i < CTR_NUM_FIELDS; ++i) row[i] = nan;
    if (ok != int(parts_.size())) return false;
    if (have_mfma && simds > 0) row[CTR_MFMA_UTIL] = float(mfma / simds);
    if (have_rd) row[CTR_HBM_READ_GBPS] = float(rd);
    if (have_wr) row[CTR_HBM_WRITE_GBPS] = float(wr);
    if (n_gfx) row[CTR_GFX_BUSY] = float(gfx / n_gfx);
    if (have_cu && cus > 0) row[CTR_CU_ACTIVE] = float(cu / cus);
    return true;
  }

 private:
  std::vector<std::shared_ptr<CounterSource>> parts_;
};

}  // namespace

int counters_preinit(const std::vector<std::string>& counter_names, int only_ordinal, uint64_t only_bdf) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_state.load() != 0) return g_state.load() > 0 ? 0 : -1;
  if (!g_api.load()) {
    g_state = -1;
    g_status = "librocprofiler-sdk.so.1 not loadable";
    return -1;
  }
  g_requested = counter_names;
  g_only_ordinal = only_ordinal;
  g_only_bdf = only_bdf;
  auto st = g_api.force_configure(&configure);
  if (st != ROCPROFILER_STATUS_SUCCESS) {
    g_state = -1;
    g_status = std::string("rocprofiler_force_configure: ") + g_api.status_string(st);
    return int(st);
  }
  g_state = 1;
  return 0;
}

bool counters_ready() {
  if (g_state.load() <= 0) return false;
  for (auto* a : g_agents)
    if (a->ok) return true;
  return false;
}

std::string counters_status() { return g_status; }

std::shared_ptr<Source> make_counter_source(uint64_t bdf, int index) {
  if (!counters_ready()) throw std::runtime_error("device counters unavailable: " + g_status);
  for (auto* a : g_agents) {
    if (!a->ok) continue;
    if ((bdf != 0 && a->bdf == bdf) || (bdf == 0 && a->ordinal == index)) return std::make_shared<CounterSource>(a);
  }
  throw std::runtime_error("device counters: no configured GPU agent for the requested bdf/index");
}

std::shared_ptr<Source> make_counter_source_all(uint64_t bdf, int index) {
  if (!counters_ready()) throw std::runtime_error("device counters unavailable: " + g_status);
  std::vector<std::shared_ptr<CounterSource>> parts;
  if (bdf != 0)
    for (auto* a : g_agents)
      if (a->ok && a->bdf == bdf) parts.push_back(std::make_shared<CounterSource>(a));
  if (parts.size() > 1) return std::make_shared<GroupCounterSource>(std::move(parts));
  if (parts.size() == 1) return parts[0];
  return make_counter_source(bdf, index);
}

}  // namespace rocmdash
