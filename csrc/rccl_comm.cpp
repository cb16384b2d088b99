// The node tensor's all-gather without torch.distributed on the hot path.
//
// torch's ProcessGroupNCCL spends ~14 us of host time per all_gather_into_tensor
// (work objects, events that hand the data between the caller's stream and its own
// NCCL stream; tools/probes/probe_step_overhead.py --rccl). Here the refresh's gather is
// one ncclAllGather on the CALLER's stream, right behind the stats kernel, on a
// communicator of our own - the ONLY RCCL communicator of the process: torch's process
// group stays on gloo (start-up agreement, validation, fallback). RCCL is dlopen()ed: the
// library torch already loaded (same SONAME librccl.so.1) is reused, so there is one RCCL
// in the process. The unique id travels through torch's store at start-up
// (rocmdash/parallel/node.py).
//
// The communicator is created non-blocking (ncclConfig_t.blocking = 0) and polled with a
// deadline, so a peer that failed before or inside its init turns into an error on every
// other rank (and the ranks fall back together) instead of a node that hangs at start-up.
#include "rccl_comm.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types and constants only: every function comes from dlsym

#include <chrono>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <thread>

namespace rocmdash {
namespace {

static_assert(sizeof(ncclUniqueId) == NCCL_UNIQUE_ID_BYTES, "unique id size");

struct Api {
  void* lib = nullptr;
  int version = 0;
  ncclResult_t (*get_version)(int*) = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank_config)(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*) = nullptr;
  ncclResult_t (*comm_get_async_error)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*comm_count)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*comm_user_rank)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*comm_device)(const ncclComm_t, int*) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

Api g_api;
std::mutex g_mu;

template <typename F>
void sym(void* lib, const char* name, F& f) {
  f = reinterpret_cast<F>(dlsym(lib, name));
  if (!f) throw std::runtime_error(std::string("RCCL: missing symbol ") + name);
}

const Api& api(const std::string& path) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_api.lib) return g_api;
  void* lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // the copy torch loaded
  if (!lib && !path.empty()) lib = dlopen(path.c_str(), RTLD_NOW | RTLD_GLOBAL);
  if (!lib) lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!lib) throw std::runtime_error("RCCL not loadable (librccl.so.1)");
  Api a;
  a.lib = lib;
  sym(lib, "ncclGetVersion", a.get_version);
  sym(lib, "ncclGetUniqueId", a.get_unique_id);
  sym(lib, "ncclCommInitRankConfig", a.comm_init_rank_config);
  sym(lib, "ncclCommGetAsyncError", a.comm_get_async_error);
  sym(lib, "ncclCommAbort", a.comm_abort);
  sym(lib, "ncclCommDestroy", a.comm_destroy);
  sym(lib, "ncclAllGather", a.all_gather);
  sym(lib, "ncclAllReduce", a.all_reduce);
  sym(lib, "ncclCommCount", a.comm_count);
  sym(lib, "ncclCommUserRank", a.comm_user_rank);
  sym(lib, "ncclCommCuDevice", a.comm_device);
  sym(lib, "ncclGetErrorString", a.error_string);
  if (a.get_version(&a.version) != ncclSuccess) throw std::runtime_error("RCCL: ncclGetVersion failed");
  g_api = a;
  return g_api;
}

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess && r != ncclInProgress) throw std::runtime_error(std::string(what) + ": " + g_api.error_string(r));
}

// Poll a non-blocking communicator until its pending operation settles; returns the final
// state (ncclInProgress on timeout).
ncclResult_t settle(ncclComm_t c, double timeout_s) {
  const auto end = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  ncclResult_t st = ncclInProgress;
  for (int i = 0;; ++i) {
    if (g_api.comm_get_async_error(c, &st) != ncclSuccess) return ncclInternalError;
    if (st != ncclInProgress) return st;
    if (std::chrono::steady_clock::now() >= end) return ncclInProgress;
    if (i > 64) std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}

}  // namespace

int rccl_load(const std::string& lib_path) { return api(lib_path).version; }

std::string rccl_unique_id(const std::string& lib_path) {
  const Api& a = api(lib_path);
  ncclUniqueId id{};
  check(a.get_unique_id(&id), "ncclGetUniqueId");
  return std::string(id.internal, NCCL_UNIQUE_ID_BYTES);
}

RcclComm::RcclComm(int device, int nranks, int rank, const std::string& unique_id, const std::string& lib_path,
                   double timeout_s)
    : device_(device), nranks_(nranks), rank_(rank) {
  if (unique_id.size() != size_t(NCCL_UNIQUE_ID_BYTES)) throw std::invalid_argument("RCCL unique id must be 128 bytes");
  if (nranks < 1 || rank < 0 || rank >= nranks) throw std::invalid_argument("RCCL: bad rank / nranks");
  const Api& a = api(lib_path);
  ncclUniqueId id;
  std::memcpy(id.internal, unique_id.data(), NCCL_UNIQUE_ID_BYTES);
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) throw std::runtime_error("hipGetDevice");
  if (hipSetDevice(device_) != hipSuccess) throw std::runtime_error("hipSetDevice");
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclComm_t c = nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  ncclResult_t r = a.comm_init_rank_config(&c, nranks, id, rank, &cfg);  // collective: every rank
  if ((r == ncclSuccess || r == ncclInProgress) && c != nullptr) r = settle(c, timeout_s);
  init_s_ = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  (void)hipSetDevice(prev);
  if (r != ncclSuccess) {
    if (c != nullptr) (void)a.comm_abort(c);
    if (r == ncclInProgress)
      throw std::runtime_error("ncclCommInitRank: not every rank joined within " + std::to_string(timeout_s) + " s");
    throw std::runtime_error(std::string("ncclCommInitRank: ") + a.error_string(r));
  }
  comm_ = c;
}

RcclComm::~RcclComm() {
  if (!comm_) return;
  // a communicator with an error (a peer is gone) or an operation still pending cannot be
  // destroyed collectively: ncclCommDestroy would wait for it (at process exit)
  ncclResult_t st = ncclSuccess;
  const bool ok = g_api.comm_get_async_error(static_cast<ncclComm_t>(comm_), &st) == ncclSuccess && st == ncclSuccess;
  if (ok) (void)g_api.comm_destroy(static_cast<ncclComm_t>(comm_));
  else (void)g_api.comm_abort(static_cast<ncclComm_t>(comm_));
}

void RcclComm::abort() {
  if (comm_) (void)g_api.comm_abort(static_cast<ncclComm_t>(comm_));
  comm_ = nullptr;
}

int RcclComm::async_error() const {
  if (!comm_) return int(ncclInvalidUsage);
  ncclResult_t st = ncclSuccess;
  if (g_api.comm_get_async_error(static_cast<ncclComm_t>(comm_), &st) != ncclSuccess) return int(ncclInternalError);
  return st == ncclInProgress ? 0 : int(st);
}

// non-blocking communicator: an enqueue that connects lazily may report in-progress; the
// next call must wait until it has settled (the enqueue itself, not the transfer). An
// enqueue that never settles leaves the communicator unusable: abort it here (its
// destructor would otherwise wait on the pending operation at process exit).
void RcclComm::finish_enqueue(int result, const char* what) {
  auto r = static_cast<ncclResult_t>(result);
  if (r == ncclInProgress) r = settle(static_cast<ncclComm_t>(comm_), 30.0);
  if (r == ncclSuccess) return;
  if (r == ncclInProgress) {
    abort();
    throw std::runtime_error(std::string(what) + ": enqueue did not settle within 30 s (communicator aborted)");
  }
  throw std::runtime_error(std::string(what) + ": " + g_api.error_string(r));
}

void RcclComm::all_gather(const float* send, float* recv, size_t count, void* stream) {
  all_gather_bytes(send, recv, count * sizeof(float), stream);
}

void RcclComm::all_gather_bytes(const void* send, void* recv, size_t bytes, void* stream) {
  if (!comm_) throw std::runtime_error("ncclAllGather: communicator aborted");
  // whole 4-byte words go as float32 (bit-exact: RCCL moves them, never computes)
  const bool words = bytes % 4 == 0;
  const ncclResult_t r = g_api.all_gather(send, recv, words ? bytes / 4 : bytes, words ? ncclFloat32 : ncclUint8,
                                          static_cast<ncclComm_t>(comm_), static_cast<hipStream_t>(stream));
  finish_enqueue(int(r), "ncclAllGather");
}

void RcclComm::all_reduce_sum_u32(const uint32_t* send, uint32_t* recv, size_t count, void* stream) {
  if (!comm_) throw std::runtime_error("ncclAllReduce: communicator aborted");
  const ncclResult_t r = g_api.all_reduce(send, recv, count, ncclUint32, ncclSum, static_cast<ncclComm_t>(comm_),
                                          static_cast<hipStream_t>(stream));
  finish_enqueue(int(r), "ncclAllReduce");
}

RcclView RcclComm::view() const {
  RcclView v;
  if (!comm_) return v;
  auto c = static_cast<ncclComm_t>(comm_);
  if (g_api.comm_count(c, &v.nranks) != ncclSuccess) v.nranks = -1;
  if (g_api.comm_user_rank(c, &v.rank) != ncclSuccess) v.rank = -1;
  if (g_api.comm_device(c, &v.device) != ncclSuccess) v.device = -1;
  return v;
}

}  // namespace rocmdash
