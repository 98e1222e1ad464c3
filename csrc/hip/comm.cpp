#include "comm.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

#include "common.h"
#include "trace.h"

#define TWTML_NCCL_CHECK(expr)                                                                \
  do {                                                                                        \
    ncclResult_t _r = (expr);                                                                 \
    if (_r != ncclSuccess)                                                                    \
      throw std::runtime_error(std::string("RCCL error ") + ncclGetErrorString(_r) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__) + ": " #expr);         \
  } while (0)

namespace twtml {

std::string rccl_unique_id() {
  ncclUniqueId id;
  TWTML_NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(id.internal, NCCL_UNIQUE_ID_BYTES);
}

std::string rccl_version() {
  int v = 0;
  TWTML_NCCL_CHECK(ncclGetVersion(&v));
  return std::to_string(v);
}

// ---------------------------------------------------------------------------
RcclComm::RcclComm(const std::string& unique_id, int rank, int world, int device) {
  rank_ = rank;
  world_ = world;
  if (unique_id.size() != NCCL_UNIQUE_ID_BYTES)
    throw std::invalid_argument("ncclUniqueId must be 128 bytes");
  if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("bad rank/world");
  ncclUniqueId id;
  std::memcpy(id.internal, unique_id.data(), NCCL_UNIQUE_ID_BYTES);
  TWTML_HIP_CHECK(hipSetDevice(device));
  TWTML_NCCL_CHECK(ncclCommInitRank(&comm_, world, id, rank));
}

RcclComm::~RcclComm() {
  if (comm_) ncclCommDestroy(comm_);
}

void RcclComm::allreduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t s) {
  // world 1 still goes through RCCL (the engines skip their collectives at
  // world 1; the direct binding uses this to check a communicator on one GPU)
  if (count == 0) return;
  TraceRange tr("twtml.rccl.allreduce");
  tally(0, count * comm_dtype_size(dt));
  TWTML_NCCL_CHECK(ncclAllReduce(buf, buf, count, dt, op, comm_, s));
}

void RcclComm::broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t s) {
  if (world_ == 1 || count == 0) return;
  tally(2, count * comm_dtype_size(dt));
  TWTML_NCCL_CHECK(ncclBroadcast(buf, buf, count, dt, root, comm_, s));
}

void RcclComm::allgather(const void* send, void* recv, size_t count, ncclDataType_t dt, hipStream_t s) {
  if (count == 0) return;
  TraceRange tr("twtml.rccl.allgather");
  tally(1, count * comm_dtype_size(dt) * size_t(world_));
  TWTML_NCCL_CHECK(ncclAllGather(send, recv, count, dt, comm_, s));
}

void RcclComm::check_async() const {
  ncclResult_t r = ncclSuccess;
  TWTML_NCCL_CHECK(ncclCommGetAsyncError(comm_, &r));
  if (r != ncclSuccess && r != ncclInProgress)
    throw std::runtime_error(std::string("RCCL async error: ") + ncclGetErrorString(r));
}

void RcclComm::abort() {
  if (comm_) {
    ncclCommAbort(comm_);
    comm_ = nullptr;
  }
}

// ---------------------------------------------------------------------------
size_t comm_dtype_size(ncclDataType_t dt) {
  switch (dt) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: throw std::invalid_argument("loopback: unsupported dtype");
  }
}

template <typename T>
static void reduce_into(T* acc, const T* x, size_t n, ncclRedOp_t op) {
  for (size_t i = 0; i < n; ++i) {
    switch (op) {
      case ncclSum: acc[i] = T(acc[i] + x[i]); break;
      case ncclMax: acc[i] = acc[i] > x[i] ? acc[i] : x[i]; break;
      case ncclMin: acc[i] = acc[i] < x[i] ? acc[i] : x[i]; break;
      default: throw std::invalid_argument("loopback: unsupported op");
    }
  }
}

void LoopbackHub::arrive_and_wait(int rank, void* buf, const std::function<void()>& leader_work) {
  std::unique_lock<std::mutex> lk(m_);
  const unsigned long long gen = generation_;
  bufs_[size_t(rank)] = buf;
  if (++arrived_ == world_) {
    leader_work();
    // the leader's pageable H2D copies may return before their DMA lands and
    // are unordered against the ranks' non-blocking streams: complete them
    TWTML_HIP_CHECK(hipDeviceSynchronize());
    arrived_ = 0;
    ++generation_;
    cv_.notify_all();
  } else {
    cv_.wait(lk, [&] { return generation_ != gen; });
  }
}

void LoopbackHub::allreduce(int rank, void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op) {
  const size_t bytes = count * comm_dtype_size(dt);
  arrive_and_wait(rank, buf, [&] {
    std::vector<unsigned char> acc(bytes), tmp(bytes);
    TWTML_HIP_CHECK(hipMemcpy(acc.data(), bufs_[0], bytes, hipMemcpyDeviceToHost));
    for (int r = 1; r < world_; ++r) {
      TWTML_HIP_CHECK(hipMemcpy(tmp.data(), bufs_[size_t(r)], bytes, hipMemcpyDeviceToHost));
      switch (dt) {
        case ncclUint8: reduce_into(acc.data(), tmp.data(), count, op); break;
        case ncclInt32: reduce_into(reinterpret_cast<int32_t*>(acc.data()), reinterpret_cast<int32_t*>(tmp.data()), count, op); break;
        case ncclInt64: reduce_into(reinterpret_cast<int64_t*>(acc.data()), reinterpret_cast<int64_t*>(tmp.data()), count, op); break;
        case ncclUint32: reduce_into(reinterpret_cast<uint32_t*>(acc.data()), reinterpret_cast<uint32_t*>(tmp.data()), count, op); break;
        case ncclUint64: reduce_into(reinterpret_cast<uint64_t*>(acc.data()), reinterpret_cast<uint64_t*>(tmp.data()), count, op); break;
        case ncclFloat32: reduce_into(reinterpret_cast<float*>(acc.data()), reinterpret_cast<float*>(tmp.data()), count, op); break;
        case ncclFloat64: reduce_into(reinterpret_cast<double*>(acc.data()), reinterpret_cast<double*>(tmp.data()), count, op); break;
        default: throw std::invalid_argument("loopback: unsupported dtype");
      }
    }
    for (int r = 0; r < world_; ++r)
      TWTML_HIP_CHECK(hipMemcpy(bufs_[size_t(r)], acc.data(), bytes, hipMemcpyHostToDevice));
  });
}

void LoopbackHub::broadcast(int rank, void* buf, size_t count, ncclDataType_t dt, int root) {
  const size_t bytes = count * comm_dtype_size(dt);
  arrive_and_wait(rank, buf, [&] {
    std::vector<unsigned char> acc(bytes);
    TWTML_HIP_CHECK(hipMemcpy(acc.data(), bufs_[size_t(root)], bytes, hipMemcpyDeviceToHost));
    for (int r = 0; r < world_; ++r)
      TWTML_HIP_CHECK(hipMemcpy(bufs_[size_t(r)], acc.data(), bytes, hipMemcpyHostToDevice));
  });
}

void LoopbackHub::allgather(int rank, const void* send, void* recv, size_t count, ncclDataType_t dt) {
  const size_t bytes = count * comm_dtype_size(dt);
  {
    std::lock_guard<std::mutex> lk(m_);
    if (sends_.size() != size_t(world_)) sends_.assign(size_t(world_), nullptr);
    sends_[size_t(rank)] = send;
  }
  arrive_and_wait(rank, recv, [&] {
    std::vector<unsigned char> all(bytes * size_t(world_));
    for (int r = 0; r < world_; ++r)
      TWTML_HIP_CHECK(hipMemcpy(all.data() + bytes * size_t(r), sends_[size_t(r)], bytes, hipMemcpyDeviceToHost));
    for (int r = 0; r < world_; ++r)
      TWTML_HIP_CHECK(hipMemcpy(bufs_[size_t(r)], all.data(), all.size(), hipMemcpyHostToDevice));
  });
}

LoopbackComm::LoopbackComm(std::shared_ptr<LoopbackHub> hub, int rank) : hub_(std::move(hub)) {
  rank_ = rank;
  world_ = hub_->world();
}

void LoopbackComm::allreduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t s) {
  if (world_ == 1 || count == 0) return;
  tally(0, count * comm_dtype_size(dt));
  TWTML_HIP_CHECK(hipStreamSynchronize(s));
  hub_->allreduce(rank_, buf, count, dt, op);
}

void LoopbackComm::broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t s) {
  if (world_ == 1 || count == 0) return;
  TWTML_HIP_CHECK(hipStreamSynchronize(s));
  hub_->broadcast(rank_, buf, count, dt, root);
}

void LoopbackComm::allgather(const void* send, void* recv, size_t count, ncclDataType_t dt, hipStream_t s) {
  if (count == 0) return;
  tally(1, count * comm_dtype_size(dt) * size_t(world_));
  TWTML_HIP_CHECK(hipStreamSynchronize(s));
  if (world_ == 1) {
    TWTML_HIP_CHECK(hipMemcpyAsync(recv, send, count * comm_dtype_size(dt), hipMemcpyDeviceToDevice, s));
    return;
  }
  hub_->allgather(rank_, send, recv, count, dt);
}

// ---------------------------------------------------------------------------
HostComm::HostComm(int rank, int world, Fn fn) : fn_(std::move(fn)) {
  if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("bad rank/world");
  rank_ = rank;
  world_ = world;
}

HostComm::~HostComm() {
  if (host_) (void)hipHostFree(host_);
}

void* HostComm::stage(size_t bytes) {
  if (bytes > cap_) {
    if (host_) TWTML_HIP_CHECK(hipHostFree(host_));
    cap_ = std::max(bytes, cap_ * 2);
    TWTML_HIP_CHECK(hipHostMalloc(&host_, cap_, hipHostMallocDefault));
  }
  return host_;
}

static int op_code(ncclRedOp_t op) {
  switch (op) {
    case ncclSum: return 0;
    case ncclMax: return 1;
    case ncclMin: return 2;
    default: throw std::invalid_argument("HostComm: unsupported reduction");
  }
}

// Floating-point sums over > 2 ranks depend on the summation order, and
// gloo's order differs between ranks: the parts are all-gathered and every
// rank adds them in rank order, so all replicas get the same bits.
// TWTML_HOSTCOMM_ORDER=rotate (tests): rank r adds them starting at part r
// instead, i.e. every rank in a different order -- the engines' collectives
// are int64 sums (or fp64 sums of exact zeros), so their results must not
// change (tests/test_gpu_dp_procs.py).
template <typename T>
static void sum_parts_in_order(T* parts, size_t count, int world, int first) {
  std::vector<T> acc(parts + size_t(first) * count, parts + size_t(first + 1) * count);
  for (int k = 1; k < world; ++k) {
    const T* p = parts + size_t((first + k) % world) * count;
    for (size_t i = 0; i < count; ++i) acc[i] += p[i];
  }
  std::copy(acc.begin(), acc.end(), parts);
}

static bool rotate_order() {
  static const bool v = [] {
    const char* e = std::getenv("TWTML_HOSTCOMM_ORDER");
    return e && std::string(e) == "rotate";
  }();
  return v;
}

void HostComm::allreduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t s) {
  if (count == 0) return;
  tally(0, count * comm_dtype_size(dt));
  TraceRange tr("twtml.hostcomm.allreduce");
  const size_t bytes = count * comm_dtype_size(dt);
  if (op == ncclSum && world_ > 2 && (dt == ncclFloat64 || dt == ncclFloat32)) {
    uint8_t* h = static_cast<uint8_t*>(stage(bytes * size_t(world_)));
    TWTML_HIP_CHECK(hipMemcpyAsync(h + bytes * size_t(rank_), buf, bytes, hipMemcpyDeviceToHost, s));
    TWTML_HIP_CHECK(hipStreamSynchronize(s));
    fn_(h, count, dt, -2, 0);
    const int first = rotate_order() ? rank_ : 0;
    if (dt == ncclFloat64) sum_parts_in_order(reinterpret_cast<double*>(h), count, world_, first);
    else sum_parts_in_order(reinterpret_cast<float*>(h), count, world_, first);
    TWTML_HIP_CHECK(hipMemcpyAsync(buf, h, bytes, hipMemcpyHostToDevice, s));
    TWTML_HIP_CHECK(hipStreamSynchronize(s));
    return;
  }
  void* h = stage(bytes);
  TWTML_HIP_CHECK(hipMemcpyAsync(h, buf, bytes, hipMemcpyDeviceToHost, s));
  TWTML_HIP_CHECK(hipStreamSynchronize(s));
  fn_(h, count, dt, op_code(op), 0);
  TWTML_HIP_CHECK(hipMemcpyAsync(buf, h, bytes, hipMemcpyHostToDevice, s));
  TWTML_HIP_CHECK(hipStreamSynchronize(s));   // the staging buffer is reused by the next call
}

void HostComm::broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t s) {
  if (count == 0 || world_ == 1) return;
  const size_t bytes = count * comm_dtype_size(dt);
  void* h = stage(bytes);
  TWTML_HIP_CHECK(hipMemcpyAsync(h, buf, bytes, hipMemcpyDeviceToHost, s));
  TWTML_HIP_CHECK(hipStreamSynchronize(s));
  fn_(h, count, dt, -1, root);
  TWTML_HIP_CHECK(hipMemcpyAsync(buf, h, bytes, hipMemcpyHostToDevice, s));
  TWTML_HIP_CHECK(hipStreamSynchronize(s));
}

void HostComm::allgather(const void* send, void* recv, size_t count, ncclDataType_t dt, hipStream_t s) {
  if (count == 0) return;
  tally(1, count * comm_dtype_size(dt) * size_t(world_));
  const size_t bytes = count * comm_dtype_size(dt);
  uint8_t* h = static_cast<uint8_t*>(stage(bytes * size_t(world_)));
  TWTML_HIP_CHECK(hipMemcpyAsync(h + bytes * size_t(rank_), send, bytes, hipMemcpyDeviceToHost, s));
  TWTML_HIP_CHECK(hipStreamSynchronize(s));
  fn_(h, count, dt, -2, 0);
  TWTML_HIP_CHECK(hipMemcpyAsync(recv, h, bytes * size_t(world_), hipMemcpyHostToDevice, s));
  TWTML_HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace twtml
