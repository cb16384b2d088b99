// The node tensor's all-gather without torch.distributed on the hot path.
//
// torch's ProcessGroupNCCL spends ~14 us of host time per all_gather_into_tensor
// (work objects, events that hand the data between the caller's stream and its own
// NCCL stream; tools/probes/probe_step_overhead.py --rccl). Here the refresh's gather is
// one ncclAllGather on the CALLER's stream, right behind the stats kernel, on a
// communicator of our own. RCCL is dlopen()ed: the library torch already loaded (same
// SONAME librccl.so.1) is reused, so there is one RCCL in the process. The unique id
// travels through torch's store at start-up (rocmdash/parallel/node.py).
#include "rccl_comm.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>
#include <stdexcept>

namespace rocmdash {
namespace {

constexpr int kIdBytes = 128;  // NCCL_UNIQUE_ID_BYTES
struct UniqueId {
  char internal[kIdBytes];
};
using Comm = void*;
enum { kSuccess = 0, kFloat32 = 7 };  // ncclSuccess, ncclFloat32 (rccl.h)

struct Api {
  void* lib = nullptr;
  int (*get_unique_id)(UniqueId*) = nullptr;
  int (*comm_init_rank)(Comm*, int, UniqueId, int) = nullptr;
  int (*comm_destroy)(Comm) = nullptr;
  int (*all_gather)(const void*, void*, size_t, int, Comm, hipStream_t) = nullptr;
  const char* (*error_string)(int) = nullptr;
};

Api g_api;
std::mutex g_mu;

const Api& api(const std::string& path) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_api.lib) return g_api;
  void* lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // the copy torch loaded
  if (!lib && !path.empty()) lib = dlopen(path.c_str(), RTLD_NOW | RTLD_GLOBAL);
  if (!lib) lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!lib) throw std::runtime_error("RCCL not loadable (librccl.so.1)");
  Api a;
  a.lib = lib;
  a.get_unique_id = reinterpret_cast<decltype(a.get_unique_id)>(dlsym(lib, "ncclGetUniqueId"));
  a.comm_init_rank = reinterpret_cast<decltype(a.comm_init_rank)>(dlsym(lib, "ncclCommInitRank"));
  a.comm_destroy = reinterpret_cast<decltype(a.comm_destroy)>(dlsym(lib, "ncclCommDestroy"));
  a.all_gather = reinterpret_cast<decltype(a.all_gather)>(dlsym(lib, "ncclAllGather"));
  a.error_string = reinterpret_cast<decltype(a.error_string)>(dlsym(lib, "ncclGetErrorString"));
  if (!a.get_unique_id || !a.comm_init_rank || !a.comm_destroy || !a.all_gather || !a.error_string)
    throw std::runtime_error("RCCL: missing symbols");
  g_api = a;
  return g_api;
}

void check(int r, const char* what) {
  if (r != kSuccess) throw std::runtime_error(std::string(what) + ": " + g_api.error_string(r));
}

}  // namespace

std::string rccl_unique_id(const std::string& lib_path) {
  const Api& a = api(lib_path);
  UniqueId id{};
  check(a.get_unique_id(&id), "ncclGetUniqueId");
  return std::string(id.internal, kIdBytes);
}

RcclComm::RcclComm(int device, int nranks, int rank, const std::string& unique_id, const std::string& lib_path)
    : device_(device), nranks_(nranks), rank_(rank) {
  if (unique_id.size() != size_t(kIdBytes)) throw std::invalid_argument("RCCL unique id must be 128 bytes");
  if (nranks < 1 || rank < 0 || rank >= nranks) throw std::invalid_argument("RCCL: bad rank / nranks");
  const Api& a = api(lib_path);
  UniqueId id;
  std::memcpy(id.internal, unique_id.data(), kIdBytes);
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) throw std::runtime_error("hipGetDevice");
  if (hipSetDevice(device_) != hipSuccess) throw std::runtime_error("hipSetDevice");
  Comm c = nullptr;
  const int r = a.comm_init_rank(&c, nranks, id, rank);  // collective: every rank of the node
  (void)hipSetDevice(prev);
  check(r, "ncclCommInitRank");
  comm_ = c;
}

RcclComm::~RcclComm() {
  if (comm_) (void)g_api.comm_destroy(comm_);
}

void RcclComm::all_gather(const float* send, float* recv, size_t count, void* stream) {
  check(g_api.all_gather(send, recv, count, kFloat32, comm_, static_cast<hipStream_t>(stream)), "ncclAllGather");
}

}  // namespace rocmdash
