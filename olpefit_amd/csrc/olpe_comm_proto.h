// olpe_comm_proto.h -- the agreement protocol of the end-of-run collectives (SURVEY.md
// §8(e)), written once against a backend B so that the same code runs over RCCL in the
// library (olpe_comm.hip) and over an in-process world of N threads in the CPU tests
// (tests/c/comm_proto_test.cpp, which injects a failure at every step on every rank).
//
// The reference's ranks meet at one comm.barrier() per iteration (apf_step2.py:338) and
// each writes its own chain file; the build's ranks meet only at the end, in RCCL
// collectives, and a rank that leaves a collective its peers entered leaves them waiting
// for ever.  The rule every function below keeps: a rank decides whether to enter a
// collective only from values every rank holds (an all-reduced word), never from a
// local outcome alone.
//   * Every collective call starts with the uniformity check: a max all-reduce of
//     kCheckWords words (shard sizes, ranges, and local failures: a bad range, a failed
//     allocation).  A rank whose words cannot reach the device still enters it, sending
//     a device-resident poisoned default (kLost = 1), so all ranks fail it together.
//   * A rank that cannot read the verdict back does what its peers do when only its own
//     words count: enter the data collective if its words were clean, else leave.
//   * The moments all-reduce runs both rounds on every rank past the check, whatever
//     happened locally; slot 0 of each round is a status word (1 = the round failed
//     here, the poisoned default when even the status cannot be sent) summed with the
//     data, and success is decided from the summed words.
// What remains is a failure inside a collective itself (an RCCL error on one rank, a
// device that dies mid-collective): the backend's bounded wait (olpe_comm_timeout)
// aborts the communicator on every rank that waits longer, so no rank waits for ever.
#pragma once
#include <stddef.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "../../include/olpe.h"

namespace olpe {
int set_err(int code, const char *fmt, ...);

namespace proto {

// the uniformity check's words (max all-reduce): v and -v give min and max over ranks
enum CheckSlot {
  kW, kNegW, kRows, kNegRows, kW0, kNegW0, kWn, kNegWn, kBadRange, kAllocFailed, kLost,
  kCheckWords
};
// the f64 poisoned default (status 1, then zeros): at least OLPE_MOMENTS_LEN(20, 19)
constexpr int kPoisonF64 = 128;
static_assert(OLPE_MOMENTS_LEN(20, 19) <= kPoisonF64, "poison covers a moments summary");

// every step a backend performs, tagged with where in the protocol it happens (the
// fault hooks and the CPU test's trace name them)
enum Site {
  kCheckSend, kCheckReduce, kCheckBack, kCheckWait,
  kR1Local, kR1Send, kR1Reduce, kR1Back, kR1Wait,
  kCentreSend,
  kR2Local, kR2Send, kR2Reduce, kR2Back, kR2Wait,
  kGather, kGatherBack, kGatherWait,
  kSites
};
inline const char *site_name(int s) {
  static const char *const n[kSites] = {
      "check.send", "check.reduce", "check.back", "check.wait",
      "r1.local", "r1.send", "r1.reduce", "r1.back", "r1.wait",
      "centre.send",
      "r2.local", "r2.send", "r2.reduce", "r2.back", "r2.wait",
      "gather", "gather.back", "gather.wait"};
  return s >= 0 && s < kSites ? n[s] : "?";
}

// The first error of a call, with its message (later steps may overwrite the
// thread-local message; the call returns the first).
struct First {
  int rc = OLPE_OK;
  char msg[512] = "";
  int add(int r) {
    if (r != OLPE_OK && rc == OLPE_OK) {
      rc = r;
      snprintf(msg, sizeof(msg), "%s", olpe_last_error());
    }
    return r;
  }
  int get() const { return rc == OLPE_OK ? OLPE_OK : set_err(rc, "%s", msg); }
};

// Backend B (all steps return OLPE_OK or an OLPE_E* code with the message set; the
// transfer and collective steps are asynchronous on one stream, wait() drains it):
//   bool has_comm();
//   int h2d(void *dev, const void *host, size_t bytes, Site);
//   int d2h(void *host, const void *dev, size_t bytes, Site);
//   int allreduce_max_i64(const long long *send, long long *recv, size_t n, Site);
//   int allreduce_sum_f64(const double *send, double *recv, size_t n, Site);
//   int allgather_f64(const double *send, double *recv, size_t n_per_rank, Site);
//   int wait(Site);                       // bounded when there is a communicator
//   int local_summary(const double *dcen, double *d, Site);
//   long long *check_words();             // device, kCheckWords
//   const long long *poison_i64();        // device, kCheckWords: 0 ... 0, kLost = 1
//   const double *poison_f64();           // device, kPoisonF64: 1, 0, ..., 0

struct Verdict {
  bool enter;   // whether this rank enters the collectives that follow the check
};

// The uniformity check (h: this rank's words in, the max over ranks out).
template <class B> Verdict check_uniform(B &b, First &f, long long h[kCheckWords], int W) {
  const bool own_flag = h[kBadRange] || h[kAllocFailed];
  long long *d = b.check_words();
  const int rs = f.add(b.h2d(d, h, sizeof(long long) * kCheckWords, kCheckSend));
  // a rank whose words did not reach the device sends the poisoned default instead
  const int rr = f.add(b.allreduce_max_i64(rs ? b.poison_i64() : d, d, kCheckWords,
                                           kCheckReduce));
  const int rb = rr ? OLPE_OK : f.add(b.d2h(h, d, sizeof(long long) * kCheckWords, kCheckBack));
  const int rw = f.add(b.wait(kCheckWait));
  if (rs || rr) return {false};        // peers read kLost / the collective failed here
  if (rb || rw) return {!own_flag};    // verdict unknown: what peers do if only ours counts
  if (h[kLost])
    return {(f.add(set_err(OLPE_ECOMM, "the uniformity words could not be sent on another "
                           "rank")), false)};
  if (h[kAllocFailed])
    return {(f.add(set_err(OLPE_ENOMEM, "a device allocation for the collective failed on "
                           "another rank")), false)};
  if (h[kW] != -h[kNegW])
    return {(f.add(set_err(OLPE_EINVAL, "walkers per rank differ (%lld..%lld): RCCL gathers "
                           "need equal shards", -h[kNegW], h[kW])), false)};
  if (h[kRows] != -h[kNegRows])
    return {(f.add(set_err(OLPE_EINVAL, "rows per rank differ (%lld..%lld)", -h[kNegRows],
                           h[kRows])), false)};
  if (h[kBadRange])
    return {(f.add(set_err(OLPE_EINVAL, "walker range outside [0, %d) on some rank", W)), false)};
  if (h[kW0] != -h[kNegW0] || h[kWn] != -h[kNegWn])
    return {(f.add(set_err(OLPE_EINVAL, "ranks asked for different walker ranges")), false)};
  return {true};
}

inline void fill_check_words(long long h[kCheckWords], long long w, long long rows,
                             long long w0, long long wn, bool bad_range, bool alloc_failed) {
  const long long v[kCheckWords] = {w,  -w,  rows, -rows, w0, -w0, wn, -wn, bad_range ? 1 : 0,
                                    alloc_failed ? 1 : 0, 0};
  memcpy(h, v, sizeof(v));
}

// All-gather of n_per_rank doubles from every rank (d_recv: the receive buffer, NULL when
// its allocation failed here; that travels in the check).  out: host copy or NULL.
template <class B>
int allgather(B &b, const double *d_send, double *d_recv, size_t n_per_rank, int nranks,
              long long equal_w, long long rows, long long w0, long long wn, bool bad_range,
              int W, double *out, First &f) {
  long long h[kCheckWords];
  fill_check_words(h, equal_w, rows, w0, wn, bad_range, d_recv == nullptr);
  if (!check_uniform(b, f, h, W).enter) return f.get();
  if (n_per_rank == 0) return f.get();
  const int rr = f.add(b.allgather_f64(d_send, d_recv, n_per_rank, kGather));
  if (!rr && out)
    f.add(b.d2h(out, d_recv, n_per_rank * (size_t)nranks * sizeof(double), kGatherBack));
  f.add(b.wait(kGatherWait));
  return f.get();
}

// One sum round over d[0, cnt): the local summary (centre dcen or NULL), slot 0 = this
// rank's status (1 = failed here: `failed_here`, or the summary), slot 1 = its walkers,
// the all-reduce, then d to h.  Returns whether the summed words were read back.
template <class B>
bool moments_round(B &b, First &f, bool r2, double *d, const double *dcen, size_t cnt,
                   double *h, double walkers, bool failed_here, double *status_sum) {
  const int lrc = failed_here ? OLPE_OK : f.add(b.local_summary(dcen, d, r2 ? kR2Local : kR1Local));
  const double st[2] = {failed_here || lrc ? 1.0 : 0.0, walkers};
  const int rs = f.add(b.h2d(d, st, sizeof(st), r2 ? kR2Send : kR1Send));
  const int rr = f.add(b.allreduce_sum_f64(rs ? b.poison_f64() : d, d, cnt,
                                           r2 ? kR2Reduce : kR1Reduce));
  const int rb = rr ? OLPE_OK : f.add(b.d2h(h, d, cnt * sizeof(double), r2 ? kR2Back : kR1Back));
  const int rw = f.add(b.wait(r2 ? kR2Wait : kR1Wait));     // (st is read by then)
  if (rr || rb || rw) return false;
  *status_sum = h[0];
  return true;
}

// The posterior moments over every rank (olpe_comm_allreduce_moments): d holds len + ps
// device doubles (the summary, then the centre); prc = the local preparation's outcome
// (its message set), which travels in the check.  out[len] on success.
template <class B>
int allreduce_moments(B &b, double *d, size_t len, int ps, int W, long long rows, int prc,
                      double *out) {
  First f;
  f.add(prc);
  if (b.has_comm()) {
    long long h[kCheckWords];
    fill_check_words(h, 0, rows, 0, 0, false, prc != OLPE_OK);
    if (!check_uniform(b, f, h, W).enter) return f.get();
  } else if (prc) {
    return f.get();
  }
  double *dcen = d + len;
  std::vector<double> h1(len), h2(2 + 3 * (size_t)ps), cen(ps, 0.0);
  double s1 = -1.0, s2 = -1.0;
  // round 1: every column's sums over all ranks; slot 1 sums to the walker total
  const bool k1 = moments_round(b, f, false, d, nullptr, len, h1.data(), (double)W,
                                f.rc != OLPE_OK, &s1);
  // round 2 (the deviations of the walkers' means about the pooled mean) is entered by
  // every rank whatever round 1 did; a rank where round 1 failed, or that could not read
  // its sums, enters it as failed (status 1), so all ranks leave with an error
  bool bad = f.rc != OLPE_OK || !k1 || s1 != 0.0;
  if (!bad) {
    for (int k = 0; k < ps; ++k) cen[k] = h1[1] > 0 ? h1[2 + k] / h1[1] : 0.0;
    bad = f.add(b.h2d(dcen, cen.data(), ps * sizeof(double), kCentreSend)) != OLPE_OK;
  }
  const bool k2 = moments_round(b, f, true, d, dcen, h2.size(), h2.data(), (double)W, bad, &s2);
  if (f.rc) return f.get();
  if (!k1 || !k2) return set_err(OLPE_EHIP, "moments all-reduce: summed words not read back");
  if (s1 != 0.0 || s2 != 0.0)
    return set_err(OLPE_ECOMM, "the moments summary failed on %.0f other rank(s)",
                   s1 != 0.0 ? s1 : s2);
  memcpy(out, h1.data(), len * sizeof(double));
  for (int k = 0; k < ps; ++k) out[2 + 2 * ps + k] = h2[2 + 2 * ps + k];
  return OLPE_OK;
}

}  // namespace proto
}  // namespace olpe
