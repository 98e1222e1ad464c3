// Collective communicators for the engines (one process per GPU).
//
// RcclComm replaces the reference's Spark treeAggregate/broadcast traffic
//  with device-side RCCL collectives issued on the
// engine's compute stream: the packed [gradient | loss] buffer is all-reduced
// in place every GD iteration, the batch statistics once per batch.  It is
// bootstrapped from an ncclUniqueId that rank 0 creates and torch.distributed
// broadcasts (parallel/dist.py).
//
// LoopbackComm is a test double: N engines in ONE process (threads), possibly
// on the same GPU, reduce through host memory.  RCCL refuses two ranks on one
// device, so this is how the data-parallel engine path is exercised on a
// single-GPU machine (tests/test_gpu_dp_loopback.py).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace twtml {

class Comm {
 public:
  virtual ~Comm() = default;
  virtual void allreduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t s) = 0;
  virtual void broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t s) = 0;
  // recv[r * count .. (r + 1) * count) = rank r's send[0 .. count)
  virtual void allgather(const void* send, void* recv, size_t count, ncclDataType_t dt, hipStream_t s) = 0;
  virtual void check_async() const {}
  virtual void abort() {}
  virtual std::string kind() const = 0;
  int rank() const { return rank_; }
  int world() const { return world_; }
  // collectives issued through this communicator: {all-reduce, all-gather,
  // broadcast} x {calls, bytes} (tests and the bench check that the engine's
  // DP traffic really went through it)
  std::vector<uint64_t> counters() const {
    std::vector<uint64_t> v(6);
    for (int i = 0; i < 6; ++i) v[size_t(i)] = ctr_[i].load(std::memory_order_relaxed);
    return v;
  }

 protected:
  void tally(int kind, size_t bytes) {
    ctr_[2 * kind].fetch_add(1, std::memory_order_relaxed);
    ctr_[2 * kind + 1].fetch_add(bytes, std::memory_order_relaxed);
  }
  int rank_ = 0, world_ = 1;
  std::atomic<uint64_t> ctr_[6] = {};
};

class RcclComm final : public Comm {
 public:
  RcclComm(const std::string& unique_id, int rank, int world, int device);
  ~RcclComm() override;
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;
  void allreduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t s) override;
  void broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t s) override;
  void allgather(const void* send, void* recv, size_t count, ncclDataType_t dt, hipStream_t s) override;
  void check_async() const override;
  void abort() override;
  std::string kind() const override { return "rccl"; }

 private:
  ncclComm_t comm_ = nullptr;
};

class LoopbackHub {
 public:
  explicit LoopbackHub(int world) : world_(world), bufs_(size_t(world), nullptr) {}
  // Blocking collective: every rank calls it with its device buffer.
  void allreduce(int rank, void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op);
  void broadcast(int rank, void* buf, size_t count, ncclDataType_t dt, int root);
  void allgather(int rank, const void* send, void* recv, size_t count, ncclDataType_t dt);
  int world() const { return world_; }

 private:
  void arrive_and_wait(int rank, void* buf, const std::function<void()>& leader_work);
  int world_;
  std::mutex m_;
  std::condition_variable cv_;
  int arrived_ = 0;
  unsigned long long generation_ = 0;
  std::vector<void*> bufs_;
  std::vector<const void*> sends_;
};

class LoopbackComm final : public Comm {
 public:
  LoopbackComm(std::shared_ptr<LoopbackHub> hub, int rank);
  void allreduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t s) override;
  void broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t s) override;
  void allgather(const void* send, void* recv, size_t count, ncclDataType_t dt, hipStream_t s) override;
  std::string kind() const override { return "loopback"; }

 private:
  std::shared_ptr<LoopbackHub> hub_;
};

// Host-staged communicator over a callback -- in practice torch.distributed
// gloo (parallel/dist.py make_comm(kind="gloo")): the engine's stream is
// synchronised, the buffer staged through pinned host memory, the callback
// runs the collective in place on it, and the result goes back to the
// device.  This is how the multi-PROCESS engine path (torchrun, one engine per
// process, real process group) runs with several ranks on ONE GPU, which RCCL
// refuses; slow by design, not a production data plane.
class HostComm final : public Comm {
 public:
  // fn(host, count, dtype, op, root): op 0 sum, 1 max, 2 min, -1 broadcast
  // from root, -2 all-gather (host holds world * count elements, rank r's at r * count)
  using Fn = std::function<void(void* host, size_t count, ncclDataType_t dt, int op, int root)>;
  HostComm(int rank, int world, Fn fn);
  ~HostComm() override;
  void allreduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t s) override;
  void broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t s) override;
  void allgather(const void* send, void* recv, size_t count, ncclDataType_t dt, hipStream_t s) override;
  std::string kind() const override { return "host"; }

 private:
  void* stage(size_t bytes);
  Fn fn_;
  void* host_ = nullptr;
  size_t cap_ = 0;
};

size_t comm_dtype_size(ncclDataType_t dt);

std::string rccl_unique_id();
std::string rccl_version();

}  // namespace twtml
