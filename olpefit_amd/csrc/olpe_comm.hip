// olpe_comm.hip -- end-of-run collectives over RCCL/xGMI.
//
// Walkers are sharded across GPUs with no communication while sampling (the
// reference's per-iteration comm.barrier() at apf_step2.py:338 carries no data).
// The only exchange is at the end of a run:
//   * all-gather of the final walker states      (ncclAllGather, rank-major)
//   * all-gather of the chains (concatenation)   (ncclAllGather per walker range, so the
//                                                 receive buffer is bounded by the range)
//   * all-reduce of per-parameter moment sums    (ncclAllReduce, sum)
// The reference's equivalent is one chain file per MPI rank behind the lockstep
// barrier (apf_step2.py:338, :355-360).  RCCL gathers need equal counts on every rank:
// each gather first all-reduces {W, -W, rows, -rows} (max) and returns OLPE_EINVAL on
// every rank when the shards differ, instead of hanging or mixing rows.
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

// every rank has the same W and (if rows >= 0) the same chain rows; the verdict is
// the same on every rank, so a mismatch is an error everywhere and nothing hangs
static int check_uniform(olpe_ctx *c, long long rows) {
  long long h[4] = {c->W, -(long long)c->W, rows, -rows};
  long long *d = nullptr;
  HIPCHK(hipMalloc(&d, sizeof(h)));
  hipError_t e = hipMemcpyAsync(d, h, sizeof(h), hipMemcpyHostToDevice, c->stream);
  ncclResult_t r = ncclSuccess;
  if (e == hipSuccess) r = ncclAllReduce(d, d, 4, ncclInt64, ncclMax, (ncclComm_t)c->comm, c->stream);
  if (e == hipSuccess && r == ncclSuccess)
    e = hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess && r == ncclSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(d);
  if (r != ncclSuccess) return set_err(OLPE_ECOMM, "ncclAllReduce: %s", ncclGetErrorString(r));
  if (e != hipSuccess) return set_err(OLPE_EHIP, "uniformity check: %s", hipGetErrorString(e));
  if (h[0] != -h[1])
    return set_err(OLPE_EINVAL, "walkers per rank differ (%lld..%lld): RCCL gathers need equal "
                   "shards", -h[1], h[0]);
  if (h[2] != -h[3])
    return set_err(OLPE_EINVAL, "chain rows per rank differ (%lld..%lld)", -h[3], h[2]);
  return OLPE_OK;
}

int olpe_comm_allgather_state(olpe_ctx *c, double *out) {
  if (!c || !out) return set_err(OLPE_EINVAL, "NULL argument");
  if (!c->comm) return set_err(OLPE_ESTATE, "call olpe_comm_init first");
  if (!c->d_state) return set_err(OLPE_ESTATE, "no ensemble");
  HIPCHK(hipSetDevice(c->device));
  int rc;
  if ((rc = check_uniform(c, 0))) return rc;
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

int olpe_comm_allgather_chain(olpe_ctx *c, long long w0, long long wn, double *out,
                              long long *nrec_out) {
  if (!c) return set_err(OLPE_EINVAL, "NULL ctx");
  if (!c->comm) return set_err(OLPE_ESTATE, "call olpe_comm_init first");
  if (!c->d_state) return set_err(OLPE_ESTATE, "no ensemble");
  HIPCHK(hipSetDevice(c->device));
  int rc;
  if ((rc = check_uniform(c, c->chain_rows))) return rc;
  if (nrec_out) *nrec_out = c->chain_rows;
  if (w0 < 0 || wn < 0 || w0 + wn > c->W)
    return set_err(OLPE_EINVAL, "walker range [%lld, %lld) outside [0, %d)", w0, w0 + wn, c->W);
  const size_t row = (size_t)c->chain_rows * c->ps;     // doubles per walker
  const size_t per = (size_t)wn * row;                  // doubles per rank in this range
  if (per == 0) return OLPE_OK;
  const size_t need = per * c->nranks;
  if (need > c->gather_cap) {
    if (c->d_gather) (void)hipFree(c->d_gather);
    c->d_gather = nullptr;
    c->gather_cap = 0;
    hipError_t e = hipMalloc(&c->d_gather, need * sizeof(double));
    if (e != hipSuccess)
      return set_err(OLPE_ENOMEM, "hipMalloc(%zu bytes) for the chain gather: %s (gather a "
                     "smaller walker range)", need * sizeof(double), hipGetErrorString(e));
    c->gather_cap = need;
  }
  NCCLCHK(ncclAllGather(c->d_chain + (size_t)w0 * row, c->d_gather, per, ncclDouble,
                        (ncclComm_t)c->comm, c->stream));
  if (out)
    HIPCHK(hipMemcpyAsync(out, c->d_gather, need * sizeof(double), hipMemcpyDeviceToHost,
                          c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
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
