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

#include <stdio.h>
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
  // nothing here can fail on one rank alone once the arguments are valid: the device
  // was set by olpe_create, and the uniformity check's word buffer was allocated there
  // too, so no rank returns early while its peers wait in ncclCommInitRank
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

// The verdict of one max all-reduce, the same on every rank, so that an error on one
// rank is an error everywhere and nothing is left waiting in a collective: every rank
// has the same chain / moment rows, the same W (when `equal_w`: the gathers need equal
// shards; a sum all-reduce does not), the same gather range, the range is valid
// everywhere, and every rank allocated what the collective needs (`alloc_failed`).  Its
// device word buffer is allocated with the context (olpe_create), so the check itself
// allocates nothing.
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

// One sum round of the moments all-reduce over d[0, cnt): the local summary
// (olpe_moments_local, centre dcen or NULL), then slot 0 = this rank's status (0 = fine,
// 1 = its summary failed) and slot 1 = its walker count, then the all-reduce, then
// d[0, cnt) to host h.  Past the uniformity check every rank calls the all-reduce
// whatever its local summary did: a failure is summed into slot 0, so every rank sees
// how many ranks failed and all of them leave the same way, instead of the failing rank
// skipping a collective its peers wait in (verdict r04 item 1).  pre_rc != OLPE_OK: this
// rank already failed (its error is set) and enters with status 1 without a summary.
// Returns this rank's own error, or OLPE_OK; *failed_ranks = the summed status (-1 if
// this rank could not read it back).
static int moments_round(olpe_ctx *c, double *d, const double *dcen, size_t cnt, double *h,
                         double *failed_ranks, int pre_rc = OLPE_OK) {
  *failed_ranks = -1.0;
  const int lrc = pre_rc ? pre_rc : olpe_moments_local(c, dcen, d);
  const double h01[2] = {lrc ? 1.0 : 0.0, (double)c->W};
  hipError_t e = hipMemcpyAsync(d, h01, sizeof(h01), hipMemcpyHostToDevice, c->stream);
  ncclResult_t r = ncclSuccess;
  if (c->comm)   // entered even after a local failure (the status word carries it)
    r = ncclAllReduce(d, d, cnt, ncclDouble, ncclSum, (ncclComm_t)c->comm, c->stream);
  hipError_t e2 = hipMemcpyAsync(h, d, cnt * sizeof(double), hipMemcpyDeviceToHost, c->stream);
  const hipError_t es = hipStreamSynchronize(c->stream);   // (h01 is read by then)
  if (e2 == hipSuccess) e2 = es;
  if (e2 == hipSuccess && e == hipSuccess && r == ncclSuccess) *failed_ranks = h[0];
  if (lrc) return lrc;
  if (e != hipSuccess) return set_err(OLPE_EHIP, "moments status word: %s", hipGetErrorString(e));
  if (r != ncclSuccess) return set_err(OLPE_ECOMM, "ncclAllReduce: %s", ncclGetErrorString(r));
  if (e2 != hipSuccess) return set_err(OLPE_EHIP, "moments all-reduce: %s", hipGetErrorString(e2));
  return OLPE_OK;
}

int olpe_comm_allreduce_moments(olpe_ctx *c, double *out) {
  if (!c || !out) return set_err(OLPE_EINVAL, "NULL argument");
  if (!c->d_state) return set_err(OLPE_ESTATE, "no ensemble");
  HIPCHK(hipSetDevice(c->device));
  const int ps = c->ps;
  const size_t len = (size_t)OLPE_MOMENTS_LEN(ps, c->np);
  // every local preparation before the uniformity check -- the summary buffer, the
  // partials, the moments and their zeroing (olpe_moments_prepare) -- and its outcome in
  // the check, so a rank that cannot prepare fails the call on every rank
  double *d = nullptr;
  if (hipMalloc(&d, (len + ps) * sizeof(double)) != hipSuccess) {
    d = nullptr;
    (void)hipGetLastError();
  }
  int prc = d ? olpe_moments_prepare(c)
              : set_err(OLPE_ENOMEM, "hipMalloc(%zu bytes) for the moments summary",
                        (len + ps) * sizeof(double));
  char pmsg[512] = "";
  if (prc) snprintf(pmsg, sizeof(pmsg), "%s", olpe_last_error());
  // a sum needs equal row counts (step 3's N), not equal shards
  int rc = c->comm ? check_uniform(c, c->mom_n, false, 0, 0, false, prc != OLPE_OK) : OLPE_OK;
  if (rc || prc) {
    if (d) (void)hipFree(d);
    return prc ? set_err(prc, "%s", pmsg) : rc;
  }
  double *dcen = d + len;
  std::vector<double> h(len), cen(ps);
  double failed = 0.0;
  // round 1: every column's sums over all ranks; slot 1 sums to the walker total
  rc = moments_round(c, d, nullptr, len, h.data(), &failed);
  // round 2 (the deviations of the walkers' means about the pooled mean) only if every
  // rank's round 1 succeeded -- a verdict every rank read from the same all-reduced word
  // (a rank that could not read it back leaves too: its stream is broken, and its peers'
  // round 2 is then left to the callers' watchdogs, bench.py --comm-timeout)
  if (failed == 0.0) {
    for (int k = 0; k < ps; ++k) cen[k] = h[1] > 0 ? h[2 + k] / h[1] : 0.0;
    hipError_t e = hipMemcpyAsync(dcen, cen.data(), ps * sizeof(double), hipMemcpyHostToDevice,
                                  c->stream);
    // a failed centre copy still enters the round, as a failed summary (status 1)
    const int crc = e == hipSuccess
                        ? OLPE_OK
                        : set_err(OLPE_EHIP, "moments centre: %s", hipGetErrorString(e));
    std::vector<double> h2(2 + 3 * (size_t)ps);
    const int rc2 = moments_round(c, d, dcen, h2.size(), h2.data(), &failed, crc);
    if (!rc2 && failed == 0.0)
      for (int k = 0; k < ps; ++k) h[2 + 2 * ps + k] = h2[2 + 2 * ps + k];
    rc = rc2;
  }
  (void)hipStreamSynchronize(c->stream);
  (void)hipFree(d);
  if (rc) return rc;
  if (failed != 0.0)
    return set_err(OLPE_ECOMM, "the moments summary failed on %.0f other rank(s)", failed);
  memcpy(out, h.data(), len * sizeof(double));
  out[0] = (double)c->mom_n;
  return OLPE_OK;
}

}  // extern "C"
