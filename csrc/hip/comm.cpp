#include "comm.h"

#include <cstring>
#include <stdexcept>

#include "common.h"

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

Comm::Comm(const std::string& unique_id, int rank, int world, int device)
    : rank_(rank), world_(world) {
  if (unique_id.size() != NCCL_UNIQUE_ID_BYTES)
    throw std::invalid_argument("ncclUniqueId must be 128 bytes");
  if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("bad rank/world");
  ncclUniqueId id;
  std::memcpy(id.internal, unique_id.data(), NCCL_UNIQUE_ID_BYTES);
  TWTML_HIP_CHECK(hipSetDevice(device));
  TWTML_NCCL_CHECK(ncclCommInitRank(&comm_, world, id, rank));
}

Comm::~Comm() {
  if (comm_) ncclCommDestroy(comm_);
}

void Comm::allreduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t s) {
  if (world_ == 1 || count == 0) return;
  TWTML_NCCL_CHECK(ncclAllReduce(buf, buf, count, dt, op, comm_, s));
}

void Comm::broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t s) {
  if (world_ == 1 || count == 0) return;
  TWTML_NCCL_CHECK(ncclBroadcast(buf, buf, count, dt, root, comm_, s));
}

void Comm::check_async() const {
  ncclResult_t r = ncclSuccess;
  TWTML_NCCL_CHECK(ncclCommGetAsyncError(comm_, &r));
  if (r != ncclSuccess && r != ncclInProgress)
    throw std::runtime_error(std::string("RCCL async error: ") + ncclGetErrorString(r));
}

void Comm::abort() {
  if (comm_) {
    ncclCommAbort(comm_);
    comm_ = nullptr;
  }
}

}  // namespace twtml
