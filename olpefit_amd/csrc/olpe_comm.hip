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
// barrier (apf_step2.py:338, :355-360).
//
// Which rank enters which collective is decided by the protocol in olpe_comm_proto.h
// (shared with the CPU tests' N-thread world); this file is its RCCL backend:
//   * the communicator is non-blocking (ncclConfig_t::blocking = 0), so that every wait
//     on it is bounded: a rank that waits longer than olpe_comm_timeout (default 600 s)
//     for its peers -- a collective a dead peer never enters -- aborts its communicator
//     (ncclCommAbort) and returns OLPE_ECOMM instead of hanging (joining it is RCCL's
//     set-up and waits for every rank: olpe_comm_init);
//   * the uniformity check's words and the poisoned defaults a rank sends when its own
//     words cannot reach the device live in one buffer allocated with the context.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <thread>
#include <vector>

#include "../../include/olpe.h"
#include "../../include/olpe_test.h"
#include "olpe_comm_proto.h"
#include "olpe_internal.h"

using olpe::set_err;
namespace proto = olpe::proto;

namespace {

#define HIPCHK(expr)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return set_err(OLPE_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_));         \
  } while (0)

// the context's comm buffer (olpe_comm_setup): check words | i64 poison | f64 poison
constexpr size_t kPoisonI64Off = 16, kPoisonF64Off = 32;
static_assert(proto::kCheckWords <= 16, "check words fit their slot");

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// OLPE_COMM_DEBUG=1: the communicator's steps on stderr (set-up, waits, aborts)
void dbg(const char *fmt, ...) {
  static const bool on = getenv("OLPE_COMM_DEBUG") != nullptr;
  if (!on) return;
  va_list ap;
  va_start(ap, fmt);
  fprintf(stderr, "[olpe comm %.3f] ", now_s());
  vfprintf(stderr, fmt, ap);
  fprintf(stderr, "\n");
  va_end(ap);
}

// Abort the communicator (every later collective of this context is OLPE_ESTATE until a
// new olpe_comm_init), drain the stream the aborted collective ran on, return OLPE_ECOMM.
int abort_comm(olpe_ctx *c, const char *fmt, ...) {
  char msg[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(msg, sizeof(msg), fmt, ap);
  va_end(ap);
  dbg("abort: %s", msg);
  if (c->comm) (void)ncclCommAbort((ncclComm_t)c->comm);
  dbg("abort returned");
  c->comm = nullptr;
  c->comm_aborted = true;
  // the aborted kernels see RCCL's abort flag and exit; bounded all the same
  const double t0 = now_s();
  while (hipStreamQuery(c->stream) == hipErrorNotReady && now_s() - t0 < 10.0)
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  (void)hipGetLastError();
  return set_err(OLPE_ECOMM, "%s", msg);
}

// pause between polls: spin briefly (a collective of the end-of-run exchange usually
// completes in microseconds to milliseconds), then sleep
void poll_pause(int &spins) {
  if (++spins < 2000)
    std::this_thread::yield();
  else
    std::this_thread::sleep_for(std::chrono::microseconds(100));
}

// An RCCL call on the non-blocking communicator: ncclInProgress means it completes in
// the background -- poll the communicator's state, bounded by the timeout.
int settle(olpe_ctx *c, ncclResult_t r, const char *what) {
  if (r == ncclSuccess) return OLPE_OK;
  if (r != ncclInProgress) {
    if (c->comm) return abort_comm(c, "%s: %s", what, ncclGetErrorString(r));
    return set_err(OLPE_ECOMM, "%s: %s", what, ncclGetErrorString(r));
  }
  const double t0 = now_s();
  int spins = 0;
  dbg("settle %s: in progress", what);
  for (;;) {
    ncclResult_t a = ncclInProgress;
    const ncclResult_t q = ncclCommGetAsyncError((ncclComm_t)c->comm, &a);
    if (spins == 0 || spins % 20000 == 0) dbg("settle %s: async state %d (%d)", what, (int)a, (int)q);
    if (q != ncclSuccess) return abort_comm(c, "%s: ncclCommGetAsyncError: %s", what,
                                            ncclGetErrorString(q));
    if (a == ncclSuccess) return OLPE_OK;
    if (a != ncclInProgress) return abort_comm(c, "%s: %s", what, ncclGetErrorString(a));
    if (c->comm_timeout_s > 0 && now_s() - t0 > c->comm_timeout_s)
      return abort_comm(c, "%s: the other ranks did not answer within %g s (olpe_comm_timeout): "
                        "communicator aborted", what, c->comm_timeout_s);
    poll_pause(spins);
  }
}

// Wait for the context's stream.  With a communicator the wait is bounded by the timeout
// and watches RCCL's asynchronous errors: a collective whose peers never come (a rank
// that died or left) ends in an abort here, not in a hang.
int comm_wait(olpe_ctx *c, const char *what) {
  if (!c->comm) {
    const hipError_t e = hipStreamSynchronize(c->stream);
    return e == hipSuccess ? OLPE_OK : set_err(OLPE_EHIP, "%s: %s", what, hipGetErrorString(e));
  }
  const double t0 = now_s();
  int spins = 0;
  for (;;) {
    const hipError_t e = hipStreamQuery(c->stream);
    if (e == hipSuccess) return OLPE_OK;
    if (e != hipErrorNotReady) return set_err(OLPE_EHIP, "%s: %s", what, hipGetErrorString(e));
    ncclResult_t a = ncclSuccess;
    if (ncclCommGetAsyncError((ncclComm_t)c->comm, &a) == ncclSuccess && a != ncclSuccess &&
        a != ncclInProgress)
      return abort_comm(c, "%s: RCCL reported %s", what, ncclGetErrorString(a));
    if (c->comm_timeout_s > 0 && now_s() - t0 > c->comm_timeout_s)
      return abort_comm(c, "%s: still waiting for the other ranks after %g s "
                        "(olpe_comm_timeout): communicator aborted", what, c->comm_timeout_s);
    poll_pause(spins);
  }
}

// The RCCL backend of olpe_comm_proto.h.  Without a communicator (the moments summary
// of one context) the collectives are copies.
struct Rccl {
  olpe_ctx *c;
  // (an aborted communicator is still a communicator: its collectives fail, they do not
  // turn into local copies)
  bool has_comm() const { return c->comm != nullptr || c->comm_aborted; }
  int aborted(proto::Site s) const {
    return set_err(OLPE_ECOMM, "%s: the communicator was aborted earlier in this call",
                   proto::site_name(s));
  }
  // test hook (olpe_moments_fault 3 / 4): a copy fails as a HIP error would
  bool forced(proto::Site s) const {
    return (c->mom_fault == 3 && s == proto::kCheckSend) ||
           (c->mom_fault == 4 && s == proto::kR1Back);
  }
  int fail(proto::Site s) const {
    return set_err(OLPE_EHIP, "%s: failure forced (olpe_moments_fault)", proto::site_name(s));
  }
  int copy(void *dst, const void *src, size_t n, hipMemcpyKind kind, proto::Site s) {
    if (forced(s)) return fail(s);
    const hipError_t e = hipMemcpyAsync(dst, src, n, kind, c->stream);
    return e == hipSuccess ? OLPE_OK
                           : set_err(OLPE_EHIP, "%s: %s", proto::site_name(s), hipGetErrorString(e));
  }
  int h2d(void *d, const void *h, size_t n, proto::Site s) {
    return copy(d, h, n, hipMemcpyHostToDevice, s);
  }
  int d2h(void *h, const void *d, size_t n, proto::Site s) {
    return copy(h, d, n, hipMemcpyDeviceToHost, s);
  }
  template <class T>
  int reduce(const T *send, T *recv, size_t n, ncclDataType_t t, ncclRedOp_t op, proto::Site s) {
    if (c->comm_aborted) return aborted(s);
    if (!c->comm) return send == recv ? OLPE_OK : copy(recv, send, n * sizeof(T),
                                                       hipMemcpyDeviceToDevice, s);
    return settle(c, ncclAllReduce(send, recv, n, t, op, (ncclComm_t)c->comm, c->stream),
                  proto::site_name(s));
  }
  int allreduce_max_i64(const long long *s, long long *r, size_t n, proto::Site site) {
    return reduce(s, r, n, ncclInt64, ncclMax, site);
  }
  int allreduce_sum_f64(const double *s, double *r, size_t n, proto::Site site) {
    return reduce(s, r, n, ncclDouble, ncclSum, site);
  }
  int allgather_f64(const double *s, double *r, size_t n, proto::Site site) {
    if (c->comm_aborted) return aborted(site);
    if (!c->comm) return copy(r, s, n * sizeof(double), hipMemcpyDeviceToDevice, site);
    return settle(c, ncclAllGather(s, r, n, ncclDouble, (ncclComm_t)c->comm, c->stream),
                  proto::site_name(site));
  }
  int wait(proto::Site s) { return comm_wait(c, proto::site_name(s)); }
  int local_summary(const double *dcen, double *d, proto::Site) {
    return olpe_moments_local(c, dcen, d);
  }
  long long *check_words() { return c->d_check; }
  const long long *poison_i64() { return c->d_check + kPoisonI64Off; }
  const double *poison_f64() { return reinterpret_cast<const double *>(c->d_check + kPoisonF64Off); }
};

}  // namespace

// The context's comm buffer, allocated and filled by olpe_create (so that joining a
// communicator allocates nothing that could fail on one rank while the others wait in
// ncclCommInitRank): the check words, then the poisoned defaults -- i64: zeros with kLost
// = 1; f64: status 1.0, then zeros.
int olpe_comm_setup(olpe_ctx *c) {
  constexpr size_t words = kPoisonF64Off + proto::kPoisonF64;
  if (hipMalloc((void **)&c->d_check, words * sizeof(long long)) != hipSuccess) {
    c->d_check = nullptr;
    (void)hipGetLastError();
    return set_err(OLPE_ENOMEM, "hipMalloc(%zu bytes) for the collectives' words", words * 8);
  }
  std::vector<long long> h(words, 0);
  h[kPoisonI64Off + proto::kLost] = 1;
  const double one = 1.0;
  memcpy(&h[kPoisonF64Off], &one, sizeof(one));
  HIPCHK(hipMemcpy(c->d_check, h.data(), words * sizeof(long long), hipMemcpyHostToDevice));
  return OLPE_OK;
}

void olpe_comm_release(olpe_ctx *c) {
  if (!c || !c->comm) return;
  // finalize (bounded on the non-blocking communicator), then destroy; abort if it stalls
  ncclComm_t comm = (ncclComm_t)c->comm;
  const ncclResult_t r = ncclCommFinalize(comm);
  if (r == ncclSuccess || r == ncclInProgress) {
    const double t0 = now_s();
    ncclResult_t a = ncclInProgress;
    while (ncclCommGetAsyncError(comm, &a) == ncclSuccess && a == ncclInProgress &&
           now_s() - t0 < 30.0)
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    if (a == ncclSuccess) {
      (void)ncclCommDestroy(comm);
      c->comm = nullptr;
      return;
    }
  }
  (void)ncclCommAbort(comm);
  c->comm = nullptr;
}

extern "C" {

int olpe_comm_unique_id(uint8_t *id128) {
  if (!id128) return set_err(OLPE_EINVAL, "NULL id buffer");
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId must be 128 bytes");
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return set_err(OLPE_ECOMM, "ncclGetUniqueId: %s", ncclGetErrorString(r));
  memcpy(id128, &id, sizeof(id));
  return OLPE_OK;
}

int olpe_comm_timeout(olpe_ctx *c, double seconds) {
  if (!c || !(seconds >= 0)) return set_err(OLPE_EINVAL, "bad argument");
  c->comm_timeout_s = seconds;
  return OLPE_OK;
}

// Joining a communicator.  The communicator is non-blocking (ncclConfig_t::blocking = 0)
// so that every later wait on it is bounded (settle, comm_wait).  The set-up itself is
// not: RCCL 2.27's ncclCommInitRankConfig returns only once every rank has arrived, even
// with blocking = 0, bare or inside ncclGroupStart/End (measured: profiles/r06/join/), and
// aborting the half-made communicator from another thread frees it under the set-up
// thread.  So a rank that never comes is caught before this call, where the ranks meet
// on their host group to share the unique id with a timeout of its own (bench.py,
// olpefit_amd/dist.py), not here.
int olpe_comm_init(olpe_ctx *c, const uint8_t *id128, int nranks, int rank) {
  if (!c || !id128) return set_err(OLPE_EINVAL, "NULL argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return set_err(OLPE_EINVAL, "bad rank/nranks");
  // nothing here can fail on one rank alone once the arguments are valid: the device
  // was set by olpe_create, and the collectives' word buffer was allocated there too,
  // so no rank returns early while its peers wait in the communicator's set-up
  HIPCHK(hipSetDevice(c->device));
  olpe_comm_release(c);
  c->comm_aborted = false;
  ncclUniqueId id;
  memcpy(&id, id128, sizeof(id));
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclComm_t comm = nullptr;
  dbg("ncclCommInitRankConfig %d/%d", rank, nranks);
  const ncclResult_t r = ncclCommInitRankConfig(&comm, nranks, id, rank, &cfg);
  dbg("ncclCommInitRankConfig returned %d", (int)r);
  if (r != ncclSuccess && r != ncclInProgress) {
    if (comm) (void)ncclCommAbort(comm);
    return set_err(OLPE_ECOMM, "ncclCommInitRankConfig: %s", ncclGetErrorString(r));
  }
  c->comm = comm;
  int rc;
  if ((rc = settle(c, r, "ncclCommInitRankConfig"))) return rc;
  // RCCL's own view of the communicator must be the one asked for
  int cnt = -1, me = -1;
  if (ncclCommCount(comm, &cnt) != ncclSuccess || ncclCommUserRank(comm, &me) != ncclSuccess ||
      cnt != nranks || me != rank)
    return abort_comm(c, "the communicator has %d ranks and this is rank %d, not %d / %d", cnt,
                      me, nranks, rank);
  c->nranks = nranks;
  c->rank = rank;
  return OLPE_OK;
}

int olpe_comm_info(olpe_ctx *c, int *nranks, int *rank) {
  if (!c || !nranks || !rank) return set_err(OLPE_EINVAL, "NULL argument");
  if (!c->comm)
    return set_err(OLPE_ESTATE, c->comm_aborted ? "the communicator was aborted"
                                                : "call olpe_comm_init first");
  ncclResult_t r = ncclCommCount((ncclComm_t)c->comm, nranks);
  if (r == ncclSuccess) r = ncclCommUserRank((ncclComm_t)c->comm, rank);
  if (r != ncclSuccess) return set_err(OLPE_ECOMM, "ncclCommCount / ncclCommUserRank: %s",
                                       ncclGetErrorString(r));
  return OLPE_OK;
}

static int need_comm(olpe_ctx *c) {
  if (!c->comm)
    return set_err(OLPE_ESTATE, c->comm_aborted
                                    ? "the communicator was aborted (olpe_comm_timeout); call "
                                      "olpe_comm_init again"
                                    : "call olpe_comm_init first");
  return OLPE_OK;
}

int olpe_comm_allgather_state(olpe_ctx *c, double *out) {
  if (!c || !out) return set_err(OLPE_EINVAL, "NULL argument");
  int rc;
  if ((rc = need_comm(c))) return rc;
  if (!c->d_state) return set_err(OLPE_ESTATE, "no ensemble");
  HIPCHK(hipSetDevice(c->device));
  const size_t per = (size_t)c->W * c->ps;
  double *d = nullptr;
  proto::First f;
  // allocate first; the outcome travels in the uniformity check
  if (hipMalloc(&d, per * c->nranks * sizeof(double)) != hipSuccess) {
    d = nullptr;
    (void)hipGetLastError();     // so that a later launch check does not report it
    f.add(set_err(OLPE_ENOMEM, "hipMalloc(%zu bytes) for the state all-gather",
                  per * c->nranks * sizeof(double)));
  }
  Rccl b{c};
  rc = proto::allgather(b, c->d_state, d, per, c->nranks, c->W, 0, 0, 0, false, c->W, out, f);
  if (d) (void)hipFree(d);
  return rc;
}

int olpe_comm_allgather_chain(olpe_ctx *c, long long w0, long long wn, double *out,
                              long long *nrec_out) {
  if (!c) return set_err(OLPE_EINVAL, "NULL ctx");
  int rc;
  if ((rc = need_comm(c))) return rc;
  if (!c->d_state) return set_err(OLPE_ESTATE, "no ensemble");
  HIPCHK(hipSetDevice(c->device));
  // the range is validated and the receive buffer allocated locally, and both verdicts
  // travel in the uniformity check, so a rank with a bad range or a failed allocation
  // cannot leave the others waiting in the gather
  proto::First f;
  const bool bad = w0 < 0 || wn < 0 || w0 + wn > c->W;
  if (bad) f.add(set_err(OLPE_EINVAL, "walker range [%lld, %lld) outside [0, %d)", w0, w0 + wn, c->W));
  const size_t row = (size_t)c->chain_rows * c->ps;     // doubles per walker
  const size_t per = bad ? 0 : (size_t)wn * row;        // doubles per rank in this range
  const size_t need = per * c->nranks;
  bool alloc_failed = false;
  if (c->gather_limit && need * sizeof(double) > c->gather_limit) {
    alloc_failed = true;                                // olpe_comm_gather_limit
    f.add(set_err(OLPE_ENOMEM, "%zu bytes for the chain gather's receive buffer: over "
                  "olpe_comm_gather_limit (gather a smaller walker range)", need * sizeof(double)));
  } else if (need > c->gather_cap) {
    if (c->d_gather) (void)hipFree(c->d_gather);
    c->d_gather = nullptr;
    c->gather_cap = 0;
    const hipError_t ae = hipMalloc(&c->d_gather, need * sizeof(double));
    if (ae != hipSuccess) {
      c->d_gather = nullptr;
      alloc_failed = true;
      (void)hipGetLastError();
      f.add(set_err(OLPE_ENOMEM, "%zu bytes for the chain gather's receive buffer: %s (gather "
                    "a smaller walker range)", need * sizeof(double), hipGetErrorString(ae)));
    } else {
      c->gather_cap = need;
    }
  }
  Rccl b{c};
  double *recv = alloc_failed ? nullptr : (c->d_gather ? c->d_gather : nullptr);
  // (an empty range needs no buffer: any non-null pointer passes the check)
  if (!alloc_failed && !recv) recv = reinterpret_cast<double *>(c->d_check);
  rc = proto::allgather(b, c->d_chain + (bad ? 0 : (size_t)w0 * row), recv, per, c->nranks,
                        c->W, c->chain_rows, w0, wn, bad, c->W, out, f);
  if (rc == OLPE_OK && nrec_out) *nrec_out = c->chain_rows;
  return rc;
}

int olpe_comm_gather_limit(olpe_ctx *c, long long bytes) {
  if (!c || bytes < 0) return set_err(OLPE_EINVAL, "bad argument");
  c->gather_limit = (size_t)bytes;
  return OLPE_OK;
}

int olpe_comm_allreduce_moments(olpe_ctx *c, double *out) {
  if (!c || !out) return set_err(OLPE_EINVAL, "NULL argument");
  if (!c->d_state) return set_err(OLPE_ESTATE, "no ensemble");
  if (c->comm_aborted && !c->comm) return need_comm(c);
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
  const int prc = d ? olpe_moments_prepare(c)
                    : set_err(OLPE_ENOMEM, "hipMalloc(%zu bytes) for the moments summary",
                              (len + ps) * sizeof(double));
  Rccl b{c};
  // (a rank that could not allocate d still takes part: the protocol sends no data from
  // it then -- prc fails the check on every rank -- so the scratch words stand in)
  const int rc = proto::allreduce_moments(b, d ? d : reinterpret_cast<double *>(c->d_check),
                                          len, ps, c->W, c->mom_n, prc, out);
  if (d) (void)hipFree(d);
  if (rc) return rc;
  out[0] = (double)c->mom_n;
  return OLPE_OK;
}

}  // extern "C"
