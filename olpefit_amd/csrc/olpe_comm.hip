// olpe_comm.hip -- end-of-run collectives over RCCL/xGMI.
//
// Walkers are sharded across GPUs with no communication while sampling (the
// reference's per-iteration comm.barrier() at apf_step2.py:338 carries no data).
// The only exchange is at the end of a run:
//   * all-gather of the final walker states      (ncclAllGather, rank-major)
//   * all-reduce of per-parameter moment sums    (ncclAllReduce, sum)
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <string.h>

#include "../../include/olpe.h"
#include "olpe_internal.h"

using olpe::set_err;

namespace {

// sums[k] / sumsq[k] over `rows` samples of a [rows][ps] array (one block per k)
__global__ __launch_bounds__(256) void moments_kernel(const double *x, long long rows, int ps,
                                                      double *out) {
  __shared__ double s1[256], s2[256];
  const int k = blockIdx.x;
  double a = 0.0, b = 0.0;
  for (long long r = threadIdx.x; r < rows; r += blockDim.x) {
    const double v = x[r * ps + k];
    a += v;
    b += v * v;
  }
  s1[threadIdx.x] = a;
  s2[threadIdx.x] = b;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      s1[threadIdx.x] += s1[threadIdx.x + o];
      s2[threadIdx.x] += s2[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[1 + k] = s1[0];
    out[1 + ps + k] = s2[0];
    if (k == 0) out[0] = (double)rows;
  }
}

#define NCCLCHK(expr)                                                                   \
  do {                                                                                  \
    ncclResult_t r_ = (expr);                                                           \
    if (r_ != ncclSuccess)                                                              \
      return set_err(OLPE_ECOMM, "%s failed: %s", #expr, ncclGetErrorString(r_));      \
  } while (0)
#define HIPCHK(expr)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return set_err(OLPE_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_));         \
  } while (0)

}  // namespace

void olpe_comm_release(olpe_ctx *c) {
  if (c && c->comm) {
    (void)ncclCommDestroy((ncclComm_t)c->comm);
    c->comm = nullptr;
  }
}

extern "C" {

int olpe_comm_unique_id(uint8_t *id128) {
  if (!id128) return set_err(OLPE_EINVAL, "NULL id buffer");
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId must be 128 bytes");
  ncclUniqueId id;
  NCCLCHK(ncclGetUniqueId(&id));
  memcpy(id128, &id, sizeof(id));
  return OLPE_OK;
}

int olpe_comm_init(olpe_ctx *c, const uint8_t *id128, int nranks, int rank) {
  if (!c || !id128) return set_err(OLPE_EINVAL, "NULL argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return set_err(OLPE_EINVAL, "bad rank/nranks");
  HIPCHK(hipSetDevice(c->device));
  olpe_comm_release(c);
  ncclUniqueId id;
  memcpy(&id, id128, sizeof(id));
  ncclComm_t comm;
  NCCLCHK(ncclCommInitRank(&comm, nranks, id, rank));
  c->comm = comm;
  c->nranks = nranks;
  c->rank = rank;
  return OLPE_OK;
}

int olpe_comm_allgather_state(olpe_ctx *c, double *out) {
  if (!c || !out) return set_err(OLPE_EINVAL, "NULL argument");
  if (!c->comm) return set_err(OLPE_ESTATE, "call olpe_comm_init first");
  if (!c->d_state) return set_err(OLPE_ESTATE, "no ensemble");
  HIPCHK(hipSetDevice(c->device));
  const size_t per = (size_t)c->W * c->ps;
  double *d = nullptr;
  HIPCHK(hipMalloc(&d, per * c->nranks * sizeof(double)));
  ncclResult_t r = ncclAllGather(c->d_state, d, per, ncclDouble, (ncclComm_t)c->comm, c->stream);
  hipError_t e = hipSuccess;
  if (r == ncclSuccess)
    e = hipMemcpyAsync(out, d, per * c->nranks * sizeof(double), hipMemcpyDeviceToHost,
                       c->stream);
  if (r == ncclSuccess && e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(d);
  if (r != ncclSuccess) return set_err(OLPE_ECOMM, "ncclAllGather: %s", ncclGetErrorString(r));
  if (e != hipSuccess) return set_err(OLPE_EHIP, "allgather copy: %s", hipGetErrorString(e));
  return OLPE_OK;
}

int olpe_comm_allreduce_moments(olpe_ctx *c, double *out) {
  if (!c || !out) return set_err(OLPE_EINVAL, "NULL argument");
  if (!c->d_state) return set_err(OLPE_ESTATE, "no ensemble");
  HIPCHK(hipSetDevice(c->device));
  const int m = 1 + 2 * c->ps;
  double *d = nullptr;
  HIPCHK(hipMalloc(&d, m * sizeof(double)));
  const bool chain = c->chain_rows > 0;
  const double *src = chain ? c->d_chain : c->d_state;
  const long long rows = chain ? (long long)c->W * c->chain_rows : (long long)c->W;
  hipLaunchKernelGGL(moments_kernel, dim3(c->ps), dim3(256), 0, c->stream, src, rows, c->ps, d);
  hipError_t e = hipGetLastError();
  ncclResult_t r = ncclSuccess;
  if (e == hipSuccess && c->comm)
    r = ncclAllReduce(d, d, m, ncclDouble, ncclSum, (ncclComm_t)c->comm, c->stream);
  if (e == hipSuccess && r == ncclSuccess)
    e = hipMemcpyAsync(out, d, m * sizeof(double), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess && r == ncclSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(d);
  if (r != ncclSuccess) return set_err(OLPE_ECOMM, "ncclAllReduce: %s", ncclGetErrorString(r));
  if (e != hipSuccess) return set_err(OLPE_EHIP, "moments: %s", hipGetErrorString(e));
  return OLPE_OK;
}

}  // extern "C"
