// C-ABI collectives over RCCL (xGMI within a node) for callers without torch.distributed: the
// candidate sweep's one exchange (every rank's pair scores all-gathered, then the
// same arg-max on every rank) and a scalar all-reduce for timing / agreement checks.
//
// One communicator per process and device, ordered on the library's stream (aqc::mps_stream), so
// a device-output sweep (aqc_pair_grads_batch, out_is_device) followed by aqc_allgather_f64 needs
// no host wait between them.  The unique id travels between the ranks by the caller's own channel
// (a file, a socket, an environment variable): 128 opaque bytes.
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>

#include "mps_internal.h"

struct aqc_comm_s {
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1, device = 0;
  // staging for the host-pointer variant (device send + recv, pinned host mirror)
  double* dbuf = nullptr;
  double* hbuf = nullptr;
  size_t cap = 0;  // doubles (send + recv)
  std::mutex mu;
};

namespace {

int nccl_check(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return AQC_OK;
  aqc::set_error(std::string(what) + ": " + ncclGetErrorString(r));
  return AQC_ERR_HIP;
}

#define AQC_NCCL_CHECK(expr)                          \
  do {                                                \
    const int _rc = nccl_check((expr), #expr);        \
    if (_rc != AQC_OK) return _rc;                    \
  } while (0)

}  // namespace

extern "C" {

int aqc_comm_unique_id(char* out) {
  AQC_REQUIRE(out, "aqc_comm_unique_id: null argument");
  ncclUniqueId id;
  AQC_NCCL_CHECK(ncclGetUniqueId(&id));
  std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return AQC_OK;
}

int aqc_comm_init(const char* unique_id, int rank, int world, aqc_comm_t* out) {
  AQC_REQUIRE(unique_id && out && world >= 1 && rank >= 0 && rank < world, "aqc_comm_init: bad arguments");
  ncclUniqueId id;
  std::memcpy(id.internal, unique_id, NCCL_UNIQUE_ID_BYTES);
  aqc_comm_s* c = new aqc_comm_s();
  c->rank = rank;
  c->world = world;
  hipGetDevice(&c->device);
  const ncclResult_t r = ncclCommInitRank(&c->comm, world, id, rank);
  if (r != ncclSuccess) {
    delete c;
    return nccl_check(r, "ncclCommInitRank");
  }
  *out = c;
  return AQC_OK;
}

int aqc_comm_destroy(aqc_comm_t c) {
  if (!c) return AQC_OK;
  if (c->comm) ncclCommDestroy(c->comm);
  if (c->dbuf) hipFree(c->dbuf);
  if (c->hbuf) hipHostFree(c->hbuf);
  delete c;
  return AQC_OK;
}

int aqc_comm_rank(aqc_comm_t c, int* rank, int* world) {
  AQC_REQUIRE(c && rank && world, "aqc_comm_rank: null argument");
  *rank = c->rank;
  *world = c->world;
  return AQC_OK;
}

int aqc_allgather_f64(aqc_comm_t c, const double* send, double* recv, size_t count) {
  AQC_REQUIRE(c && send && recv, "aqc_allgather_f64: null argument");
  if (count == 0) return AQC_OK;
  AQC_NCCL_CHECK(ncclAllGather(send, recv, count, ncclDouble, c->comm, aqc::mps_stream()));
  return AQC_OK;
}

int aqc_allgather_f64_host(aqc_comm_t c, const double* send, double* recv, size_t count) {
  AQC_REQUIRE(c && send && recv, "aqc_allgather_f64_host: null argument");
  if (count == 0) return AQC_OK;
  std::lock_guard<std::mutex> lk(c->mu);
  const size_t need = count * (1 + (size_t)c->world);
  hipStream_t st = aqc::mps_stream();
  if (need > c->cap) {
    AQC_HIP_CHECK(hipStreamSynchronize(st));
    if (c->dbuf) hipFree(c->dbuf);
    if (c->hbuf) hipHostFree(c->hbuf);
    c->dbuf = nullptr, c->hbuf = nullptr, c->cap = 0;
    AQC_HIP_CHECK(hipMalloc(&c->dbuf, need * sizeof(double)));
    AQC_HIP_CHECK(hipHostMalloc((void**)&c->hbuf, need * sizeof(double), hipHostMallocDefault));
    c->cap = need;
  }
  std::memcpy(c->hbuf, send, count * sizeof(double));
  AQC_HIP_CHECK(hipMemcpyAsync(c->dbuf, c->hbuf, count * sizeof(double), hipMemcpyHostToDevice, st));
  AQC_NCCL_CHECK(ncclAllGather(c->dbuf, c->dbuf + count, count, ncclDouble, c->comm, st));
  AQC_HIP_CHECK(hipMemcpyAsync(c->hbuf + count, c->dbuf + count, count * c->world * sizeof(double),
                               hipMemcpyDeviceToHost, st));
  AQC_HIP_CHECK(hipStreamSynchronize(st));
  std::memcpy(recv, c->hbuf + count, count * c->world * sizeof(double));
  return AQC_OK;
}

int aqc_allreduce_max_f64(aqc_comm_t c, double* value) {
  AQC_REQUIRE(c && value, "aqc_allreduce_max_f64: null argument");
  std::lock_guard<std::mutex> lk(c->mu);
  hipStream_t st = aqc::mps_stream();
  if (c->cap < 2) {
    AQC_HIP_CHECK(hipStreamSynchronize(st));
    if (c->dbuf) hipFree(c->dbuf);
    if (c->hbuf) hipHostFree(c->hbuf);
    c->dbuf = nullptr, c->hbuf = nullptr, c->cap = 0;
    AQC_HIP_CHECK(hipMalloc(&c->dbuf, 64 * sizeof(double)));
    AQC_HIP_CHECK(hipHostMalloc((void**)&c->hbuf, 64 * sizeof(double), hipHostMallocDefault));
    c->cap = 64;
  }
  c->hbuf[0] = *value;
  AQC_HIP_CHECK(hipMemcpyAsync(c->dbuf, c->hbuf, sizeof(double), hipMemcpyHostToDevice, st));
  AQC_NCCL_CHECK(ncclAllReduce(c->dbuf, c->dbuf + 1, 1, ncclDouble, ncclMax, c->comm, st));
  AQC_HIP_CHECK(hipMemcpyAsync(c->hbuf + 1, c->dbuf + 1, sizeof(double), hipMemcpyDeviceToHost, st));
  AQC_HIP_CHECK(hipStreamSynchronize(st));
  *value = c->hbuf[1];
  return AQC_OK;
}

}  // extern "C"
