// A persistent RCCL communicator driven from C++ on the caller's stream (rccl_comm.cpp).
#pragma once

#include <cstdint>
#include <string>

namespace rocmdash {

// Load RCCL (the copy torch loaded, else `lib_path`) without creating anything; returns
// its version code (e.g. 22606). Every rank calls this and shares the outcome BEFORE any
// rank enters the collective communicator init, so a rank that cannot load RCCL never
// leaves its peers blocked inside ncclCommInitRank.
int rccl_load(const std::string& lib_path);

// 128-byte ncclUniqueId of a new communicator (rank 0 creates it, every rank gets a copy).
std::string rccl_unique_id(const std::string& lib_path);

// The communicator as RCCL itself reports it (ncclCommCount / ncclCommUserRank /
// ncclCommCuDevice): -1 where RCCL refused the query.
struct RcclView {
  int nranks = -1, rank = -1, device = -1;
};

class RcclComm {
 public:
  // Non-blocking init (ncclConfig_t.blocking = 0) polled for at most timeout_s: a peer
  // that never joins makes this throw (after ncclCommAbort) instead of hanging.
  RcclComm(int device, int nranks, int rank, const std::string& unique_id, const std::string& lib_path,
           double timeout_s = 120.0);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  // Enqueue ncclAllGather of `count` floats per rank on `stream` (recv holds nranks * count).
  void all_gather(const float* send, float* recv, size_t count, void* stream);
  // The same for any `bytes` per rank (moved bit for bit: structs of partial results).
  void all_gather_bytes(const void* send, void* recv, size_t bytes, void* stream);
  // Enqueue ncclAllReduce(sum) of `count` uint32 on `stream` (exact: histogram counts).
  void all_reduce_sum_u32(const uint32_t* send, uint32_t* recv, size_t count, void* stream);
  // RCCL's own view of the communicator (rank count, this rank, its device).
  RcclView view() const;
  // ncclCommGetAsyncError: 0 = healthy; anything else = the communicator is broken.
  int async_error() const;
  // Tear the communicator down without waiting for peers (a rank lost mid-collective).
  void abort();
  int nranks() const { return nranks_; }
  int rank() const { return rank_; }
  double init_seconds() const { return init_s_; }

 private:
  void finish_enqueue(int result, const char* what);
  int device_, nranks_, rank_;
  void* comm_ = nullptr;
  double init_s_ = 0.0;
};

}  // namespace rocmdash
