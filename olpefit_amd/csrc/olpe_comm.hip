// olpe_comm.hip -- end-of-run collectives over RCCL/xGMI.
//
// Walkers are sharded across GPUs with no communication while sampling (the
// reference's per-iteration comm.barrier() at apf_step2.py:338 carries no data).
// The only exchange is at the end of a run:
//   * all-gather of the final walker states      (ncclAllGather, rank-major)
//   * all-gather of the chains (concatenation)   (ncclAllGather per walker range, so the
//                                                 receive buffer is bounded by the range)
//   * the posterior summary from the whole-run moments (olpe_moments.hip): two
//     all-reduces (sum) -- the pooled mean, then the walkers' deviations about it
// The reference's equivalent is one chain file per MPI rank behind the lockstep
// barrier (apf_step2.py:338, :355-360).  RCCL gathers need equal counts on every rank:
// each collective first all-reduces {W, -W, rows, -rows, range, -range, bad, alloc}
// (max) and returns OLPE_EINVAL / OLPE_ENOMEM on every rank when the shards or the
// requested ranges differ, a range is invalid or an allocation failed on some rank,
// instead of hanging or mixing rows.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <string.h>

#include <vector>

#include "../../include/olpe.h"
#include "olpe_internal.h"

using olpe::set_err;

namespace {

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
  // the uniformity check's word buffer, before the communicator: a failure here is
  // reported before this rank joins the collective initialisation
  if (!c->d_check) {
    hipError_t e = hipMalloc(&c->d_check, 16 * sizeof(long long));
    if (e != hipSuccess) {
      c->d_check = nullptr;
      return set_err(OLPE_ENOMEM, "hipMalloc(128 bytes) for the communicator: %s",
                     hipGetErrorString(e));
    }
  }
  ncclUniqueId id;
  memcpy(&id, id128, sizeof(id));
  ncclComm_t comm;
  NCCLCHK(ncclCommInitRank(&comm, nranks, id, rank));
  c->comm = comm;
  c->nranks = nranks;
  c->rank = rank;
  return OLPE_OK;
}

// The verdict of one max all-reduce, the same on every rank, so that an error on one
// rank is an error everywhere and nothing is left waiting in a collective: every rank
// has the same chain / moment rows, the same W (when `equal_w`: the gathers need equal
// shards; a sum all-reduce does not), the same gather range, the range is valid
// everywhere, and every rank allocated what the collective needs (`alloc_failed`).  Its
// device word buffer is allocated in olpe_comm_init, so the check itself allocates
// nothing.
static int check_uniform(olpe_ctx *c, long long rows, bool equal_w, long long w0 = 0,
                         long long wn = 0, bool bad_range = false, bool alloc_failed = false) {
  const long long w = equal_w ? c->W : 0;
  long long h[10] = {w, -w, rows, -rows, w0, -w0, wn, -wn, bad_range ? 1 : 0,
                     alloc_failed ? 1 : 0};
  long long *d = c->d_check;
  hipError_t e = hipMemcpyAsync(d, h, sizeof(h), hipMemcpyHostToDevice, c->stream);
  ncclResult_t r = ncclSuccess;
  if (e == hipSuccess) r = ncclAllReduce(d, d, 10, ncclInt64, ncclMax, (ncclComm_t)c->comm, c->stream);
  if (e == hipSuccess && r == ncclSuccess)
    e = hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess && r == ncclSuccess) e = hipStreamSynchronize(c->stream);
  if (r != ncclSuccess) return set_err(OLPE_ECOMM, "ncclAllReduce: %s", ncclGetErrorString(r));
  if (e != hipSuccess) return set_err(OLPE_EHIP, "uniformity check: %s", hipGetErrorString(e));
  if (h[9])
    return set_err(OLPE_ENOMEM, "a device allocation for the collective failed on %s rank",
                   alloc_failed ? "this" : "another");
  if (h[0] != -h[1])
    return set_err(OLPE_EINVAL, "walkers per rank differ (%lld..%lld): RCCL gathers need equal "
                   "shards", -h[1], h[0]);
  if (h[2] != -h[3])
    return set_err(OLPE_EINVAL, "rows per rank differ (%lld..%lld)", -h[3], h[2]);
  if (h[8])
    return set_err(OLPE_EINVAL, "walker range outside [0, %d) on some rank", c->W);
  if (h[4] != -h[5] || h[6] != -h[7])
    return set_err(OLPE_EINVAL, "ranks asked for different walker ranges");
  return OLPE_OK;
}

int olpe_comm_allgather_state(olpe_ctx *c, double *out) {
  if (!c || !out) return set_err(OLPE_EINVAL, "NULL argument");
  if (!c->comm) return set_err(OLPE_ESTATE, "call olpe_comm_init first");
  if (!c->d_state) return set_err(OLPE_ESTATE, "no ensemble");
  HIPCHK(hipSetDevice(c->device));
  const size_t per = (size_t)c->W * c->ps;
  double *d = nullptr;
  // allocate first; the outcome travels in the uniformity check
  if (hipMalloc(&d, per * c->nranks * sizeof(double)) != hipSuccess) {
    d = nullptr;
    (void)hipGetLastError();     // so that a later launch check does not report it
  }
  int rc;
  if ((rc = check_uniform(c, 0, true, 0, 0, false, d == nullptr))) {
    if (d) (void)hipFree(d);
    return rc;
  }
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
  // the range is validated and the receive buffer allocated locally, and both verdicts
  // travel in the uniformity check, so a rank with a bad range or a failed allocation
  // cannot leave the others waiting in the gather
  const bool bad = w0 < 0 || wn < 0 || w0 + wn > c->W;
  const size_t row = (size_t)c->chain_rows * c->ps;     // doubles per walker
  const size_t per = bad ? 0 : (size_t)wn * row;        // doubles per rank in this range
  const size_t need = per * c->nranks;
  bool alloc_failed = false;
  hipError_t ae = hipSuccess;
  if (c->gather_limit && need * sizeof(double) > c->gather_limit) {
    alloc_failed = true;                                // olpe_comm_gather_limit
  } else if (need > c->gather_cap) {
    if (c->d_gather) (void)hipFree(c->d_gather);
    c->d_gather = nullptr;
    c->gather_cap = 0;
    if ((ae = hipMalloc(&c->d_gather, need * sizeof(double))) != hipSuccess) {
      c->d_gather = nullptr;
      alloc_failed = true;
      (void)hipGetLastError();
    } else {
      c->gather_cap = need;
    }
  }
  int rc;
  if ((rc = check_uniform(c, c->chain_rows, true, w0, wn, bad, alloc_failed))) {
    if (bad)
      return set_err(OLPE_EINVAL, "walker range [%lld, %lld) outside [0, %d)", w0, w0 + wn, c->W);
    if (alloc_failed)
      return set_err(OLPE_ENOMEM, "%zu bytes for the chain gather's receive buffer: %s (gather "
                     "a smaller walker range)", need * sizeof(double),
                     ae != hipSuccess ? hipGetErrorString(ae) : "over olpe_comm_gather_limit");
    return rc;
  }
  if (nrec_out) *nrec_out = c->chain_rows;
  if (per == 0) return OLPE_OK;
  NCCLCHK(ncclAllGather(c->d_chain + (size_t)w0 * row, c->d_gather, per, ncclDouble,
                        (ncclComm_t)c->comm, c->stream));
  if (out)
    HIPCHK(hipMemcpyAsync(out, c->d_gather, need * sizeof(double), hipMemcpyDeviceToHost,
                          c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return OLPE_OK;
}

int olpe_comm_gather_limit(olpe_ctx *c, long long bytes) {
  if (!c || bytes < 0) return set_err(OLPE_EINVAL, "bad argument");
  c->gather_limit = (size_t)bytes;
  return OLPE_OK;
}

int olpe_comm_allreduce_moments(olpe_ctx *c, double *out) {
  if (!c || !out) return set_err(OLPE_EINVAL, "NULL argument");
  if (!c->d_state) return set_err(OLPE_ESTATE, "no ensemble");
  HIPCHK(hipSetDevice(c->device));
  const int ps = c->ps;
  const size_t len = (size_t)OLPE_MOMENTS_LEN(ps, c->np);
  double *d = nullptr;
  if (hipMalloc(&d, (len + ps) * sizeof(double)) != hipSuccess) {
    d = nullptr;
    (void)hipGetLastError();
  }
  // a sum needs equal row counts (step 3's N), not equal shards
  int rc = c->comm ? check_uniform(c, c->mom_n, false, 0, 0, false, d == nullptr)
                   : d ? OLPE_OK : set_err(OLPE_ENOMEM, "hipMalloc for the moments summary");
  if (rc) {
    if (d) (void)hipFree(d);
    return rc;
  }
  double *dcen = d + len;
  // round 1: every column's sums over all ranks; slot 1 sums to the walker total
  // (slot 0 stays 0: n is the same on every rank, checked above)
  double h01[2] = {0.0, (double)c->W};
  std::vector<double> cen(ps);
  hipError_t e = hipMemcpyAsync(d, h01, sizeof(h01), hipMemcpyHostToDevice, c->stream);
  ncclResult_t r = ncclSuccess;
  rc = e == hipSuccess ? olpe_moments_local(c, nullptr, d) : OLPE_OK;
  if (e == hipSuccess && !rc && c->comm)
    r = ncclAllReduce(d, d, len, ncclDouble, ncclSum, (ncclComm_t)c->comm, c->stream);
  if (e == hipSuccess && !rc && r == ncclSuccess)
    e = hipMemcpyAsync(out, d, len * sizeof(double), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess && !rc && r == ncclSuccess) e = hipStreamSynchronize(c->stream);
  // round 2: the deviations of the walkers' means about the pooled mean
  if (e == hipSuccess && !rc && r == ncclSuccess) {
    for (int k = 0; k < ps; ++k) cen[k] = out[1] > 0 ? out[2 + k] / out[1] : 0.0;
    e = hipMemcpyAsync(dcen, cen.data(), ps * sizeof(double), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) rc = olpe_moments_local(c, dcen, d);
    double *dev = d + 2 + 2 * ps;
    if (e == hipSuccess && !rc && c->comm)
      r = ncclAllReduce(dev, dev, ps, ncclDouble, ncclSum, (ncclComm_t)c->comm, c->stream);
    if (e == hipSuccess && !rc && r == ncclSuccess)
      e = hipMemcpyAsync(out + 2 + 2 * ps, dev, ps * sizeof(double), hipMemcpyDeviceToHost,
                         c->stream);
    if (e == hipSuccess && !rc && r == ncclSuccess) e = hipStreamSynchronize(c->stream);
  }
  (void)hipStreamSynchronize(c->stream);
  (void)hipFree(d);
  if (rc) return rc;
  if (r != ncclSuccess) return set_err(OLPE_ECOMM, "ncclAllReduce: %s", ncclGetErrorString(r));
  if (e != hipSuccess) return set_err(OLPE_EHIP, "moments all-reduce: %s", hipGetErrorString(e));
  out[0] = (double)c->mom_n;
  return OLPE_OK;
}

}  // extern "C"
