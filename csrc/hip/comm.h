// RCCL communicator (one process per GPU; xGMI on an MI355X node).
//
// Replaces the reference's Spark treeAggregate/broadcast traffic (SURVEY §2.5
// CS1-CS10) with device-side collectives issued on the engine's compute
// stream: the packed [gradient | loss] buffer is all-reduced in place every
// GD iteration, the batch statistics once per batch.  The communicator is
// bootstrapped from an ncclUniqueId that rank 0 creates and torch.distributed
// broadcasts (parallel/dist.py).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <memory>
#include <string>

namespace twtml {

class Comm {
 public:
  Comm(const std::string& unique_id, int rank, int world, int device);
  ~Comm();
  Comm(const Comm&) = delete;
  Comm& operator=(const Comm&) = delete;

  void allreduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t s);
  void broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t s);
  void check_async() const;
  void abort();

  int rank() const { return rank_; }
  int world() const { return world_; }

 private:
  ncclComm_t comm_ = nullptr;
  int rank_ = 0, world_ = 1;
};

std::string rccl_unique_id();
std::string rccl_version();

}  // namespace twtml
