// A persistent RCCL communicator driven from C++ on the caller's stream (rccl_comm.cpp).
#pragma once

#include <cstdint>
#include <string>

namespace rocmdash {

// 128-byte ncclUniqueId of a new communicator (rank 0 creates it, every rank gets a copy).
std::string rccl_unique_id(const std::string& lib_path);

class RcclComm {
 public:
  RcclComm(int device, int nranks, int rank, const std::string& unique_id, const std::string& lib_path);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  // Enqueue ncclAllGather of `count` floats per rank on `stream` (recv holds nranks * count).
  void all_gather(const float* send, float* recv, size_t count, void* stream);
  int nranks() const { return nranks_; }
  int rank() const { return rank_; }

 private:
  int device_, nranks_, rank_;
  void* comm_ = nullptr;
};

}  // namespace rocmdash
