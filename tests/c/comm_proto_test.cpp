// comm_proto_test.cpp -- the collectives' agreement protocol (olpefit_amd/csrc/
// olpe_comm_proto.h, the code libolpe.so runs over RCCL) over an in-process world of N
// ranks, one thread each, with a failure injected at every step of every rank.
//
// The world's collectives match calls by sequence number, as RCCL does, and a rank that
// waits longer than the world's timeout in one records itself as stuck (the library's
// bounded wait, olpe_comm_timeout, would abort its communicator there).  The property
// checked for every single failure that is not inside a collective itself (a copy, a
// stream wait, the local summary, an allocation, a bad range): NO rank is ever stuck --
// the protocol alone keeps every rank entering the same collectives -- every rank
// returns, the failing rank returns an error, the ranks agree on the outcome (except a
// rank that fails only to read back the last round's sums), and the next clean call
// succeeds everywhere with the exact sums.  A failure inside a collective (its enqueue
// fails on one rank) is bounded instead: its peers time out and every rank returns an
// error.  A negative control (a rank that skips one collective) must be caught as stuck.
//
// usage: comm_proto_test [timeout_ms]; prints one line per case family and
// "ALL OK cases=<n>", exit 0; failures are printed and the exit status is 1.
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../olpefit_amd/csrc/olpe_comm_proto.h"

thread_local char g_err[512];
namespace olpe {
int set_err(int code, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}
}  // namespace olpe
extern "C" const char *olpe_last_error(void) { return g_err; }

using namespace olpe::proto;
using olpe::set_err;

static int g_fail = 0;
static int g_cases = 0;
#define EXPECT(cond, ...)                                    \
  do {                                                       \
    if (!(cond)) {                                           \
      ++g_fail;                                              \
      printf("FAIL %s:%d: %s -- ", __FILE__, __LINE__, #cond); \
      printf(__VA_ARGS__);                                   \
      printf("\n");                                          \
    }                                                        \
  } while (0)

// ---------------------------------------------------------------------------------------
struct World {
  int n;
  std::chrono::milliseconds timeout;
  std::mutex m;
  std::condition_variable cv;
  struct Slot {
    int arrived = 0, taken = 0, kind = -1;
    size_t bytes = 0;
    bool mismatch = false;
    std::vector<std::vector<char>> data;
    std::vector<char> result;
  };
  std::map<long, Slot> slots;
  std::vector<std::string> stuck;
  int mismatches = 0;
  World(int n_, int timeout_ms) : n(n_), timeout(timeout_ms) {}

  // kind 0: max i64, 1: sum f64, 2: all-gather (rank-major)
  int collective(int rank, long id, int kind, const void *send, void *recv, size_t bytes,
                 const char *site) {
    std::unique_lock<std::mutex> lk(m);
    Slot &s = slots[id];
    if (s.data.empty()) s.data.resize(n);
    if (s.kind < 0) {
      s.kind = kind;
      s.bytes = bytes;
    } else if (s.kind != kind || s.bytes != bytes) {
      s.mismatch = true;
    }
    s.data[rank].assign((const char *)send, (const char *)send + bytes);
    if (++s.arrived == n) {
      if (kind == 2) {
        for (auto &d : s.data) s.result.insert(s.result.end(), d.begin(), d.end());
      } else {
        s.result = s.data[0];
        for (int r = 1; r < n; ++r) {
          if (s.data[r].size() != s.result.size()) continue;
          if (kind == 0) {
            auto *o = (long long *)s.result.data();
            auto *v = (const long long *)s.data[r].data();
            for (size_t i = 0; i < bytes / 8; ++i) o[i] = o[i] > v[i] ? o[i] : v[i];
          } else {
            auto *o = (double *)s.result.data();
            auto *v = (const double *)s.data[r].data();
            for (size_t i = 0; i < bytes / 8; ++i) o[i] += v[i];
          }
        }
      }
      cv.notify_all();
    } else if (!cv.wait_until(lk, std::chrono::system_clock::now() + timeout,
                              [&] { return s.arrived == n; })) {
      // (system_clock: libstdc++ waits on it with pthread_cond_timedwait, which
      // ThreadSanitizer intercepts; steady_clock's pthread_cond_clockwait it does not)
      char b[160];
      snprintf(b, sizeof b, "rank %d stuck in collective #%ld (%s)", rank, id, site);
      stuck.push_back(b);
      return set_err(OLPE_ECOMM, "%s: timed out waiting for the other ranks", site);
    }
    if (s.mismatch) ++mismatches;
    const size_t want = kind == 2 ? bytes * n : bytes;
    memcpy(recv, s.result.data(), s.result.size() < want ? s.result.size() : want);
    if (++s.taken == n) slots.erase(id);
    return OLPE_OK;
  }
};

// per-rank walkers and moments of the fake local summary
static int walkers_of(int r) { return 3 + r; }
static double mean_of(int r, int k) { return 1.0 + r + 0.1 * k; }

struct Fake {
  World *w;
  int rank;
  bool comm = true;
  int ps = 17, np = 16;
  long seq = 0;
  bool aborted = false;
  int fault_site = -1, fault_occ = -1;   // fail this step ...
  bool skip = false;                     // ... or (negative control) skip the collective
  std::map<int, int> occ;
  std::vector<int> trace;
  long long words[kCheckWords] = {};
  long long pois_i[kCheckWords] = {};
  double pois_f[kPoisonF64] = {};
  Fake(World *w_, int r) : w(w_), rank(r) {
    pois_i[kLost] = 1;
    pois_f[0] = 1.0;
  }
  bool hit(Site s) {
    const int k = occ[s]++;
    trace.push_back(s);
    return s == fault_site && k == fault_occ;
  }
  bool has_comm() const { return comm; }
  int fail(Site s, int code = OLPE_EHIP) {
    return set_err(code, "%s: failure injected on rank %d", site_name(s), rank);
  }
  int h2d(void *d, const void *h, size_t n, Site s) {
    if (hit(s)) return fail(s);
    memcpy(d, h, n);
    return OLPE_OK;
  }
  int d2h(void *h, const void *d, size_t n, Site s) {
    if (hit(s)) return fail(s);
    memcpy(h, d, n);
    return OLPE_OK;
  }
  int coll(int kind, const void *send, void *recv, size_t bytes, Site s) {
    const bool f = hit(s);
    if (f && skip) return OLPE_OK;                      // negative control: left out
    if (f) {
      aborted = true;                                   // the enqueue failed: RCCL error
      return fail(s, OLPE_ECOMM);
    }
    if (aborted) return set_err(OLPE_ECOMM, "%s: aborted", site_name(s));
    if (!comm) {
      if (send != recv) memmove(recv, send, bytes);
      return OLPE_OK;
    }
    const int rc = w->collective(rank, seq++, kind, send, recv, bytes, site_name(s));
    if (rc) aborted = true;                             // timed out: bounded wait aborts
    return rc;
  }
  int allreduce_max_i64(const long long *s, long long *r, size_t n, Site site) {
    return coll(0, s, r, n * 8, site);
  }
  int allreduce_sum_f64(const double *s, double *r, size_t n, Site site) {
    return coll(1, s, r, n * 8, site);
  }
  int allgather_f64(const double *s, double *r, size_t n, Site site) {
    return coll(2, s, r, n * 8, site);
  }
  int wait(Site s) { return hit(s) ? fail(s) : OLPE_OK; }
  int local_summary(const double *dcen, double *d, Site s) {
    if (hit(s)) return fail(s);
    const int W = walkers_of(rank);
    for (int k = 0; k < ps; ++k) {
      d[2 + k] = W * mean_of(rank, k);
      d[2 + ps + k] = 0.5 * W * (k + 1);
      const double dv = dcen ? mean_of(rank, k) - dcen[k] : 0.0;
      d[2 + 2 * ps + k] = dcen ? W * dv * dv : 0.0;
    }
    for (int j = 0; j < np; ++j) {
      d[2 + 3 * ps + j] = 10.0 * W;
      d[2 + 3 * ps + np + j] = 4.0 * W;
    }
    return OLPE_OK;
  }
  long long *check_words() { return words; }
  const long long *poison_i64() { return pois_i; }
  const double *poison_f64() { return pois_f; }
};

// ---------------------------------------------------------------------------------------
struct Out {
  int rc = OLPE_OK;
  std::string msg;
  std::vector<double> v;
  std::vector<int> trace;
};

static bool moments_exact(int n, const std::vector<double> &o, int ps, int np) {
  double W = 0;
  for (int r = 0; r < n; ++r) W += walkers_of(r);
  if (o[1] != W) return false;
  for (int k = 0; k < ps; ++k) {
    double s = 0, m2 = 0;
    for (int r = 0; r < n; ++r) {
      s += walkers_of(r) * mean_of(r, k);
      m2 += 0.5 * walkers_of(r) * (k + 1);
    }
    const double c = s / W;
    double dev = 0;
    for (int r = 0; r < n; ++r) {
      const double d = mean_of(r, k) - c;
      dev += walkers_of(r) * d * d;
    }
    auto close = [](double a, double b) { return fabs(a - b) <= 1e-12 * (fabs(b) + 1e-300); };
    if (!close(o[2 + k], s) || !close(o[2 + ps + k], m2) || !close(o[2 + 2 * ps + k], dev))
      return false;
  }
  for (int j = 0; j < np; ++j)
    if (o[2 + 3 * ps + j] != 10.0 * W || o[2 + 3 * ps + np + j] != 4.0 * W) return false;
  return true;
}

// What one rank does in one case: `call` with its fault, then (follow_up) a clean call.
using Call = std::function<int(Fake &, std::vector<double> &)>;

static std::vector<Out> run_world(int n, int timeout_ms, const Call &call, int frank,
                                  int fsite, int focc, bool skip, bool follow_up,
                                  std::vector<Out> *second, World **wout = nullptr,
                                  std::vector<std::string> *stuck = nullptr, int *mism = nullptr,
                                  bool comm = true) {
  auto wp = std::make_unique<World>(n, timeout_ms);   // (heap: no mutex address reuse)
  World &w = *wp;
  std::vector<Out> out(n), out2(n);
  std::vector<std::thread> th;
  for (int r = 0; r < n; ++r)
    th.emplace_back([&, r] {
      Fake f(&w, r);
      f.comm = comm;
      if (r == frank) {
        f.fault_site = fsite;
        f.fault_occ = focc;
        f.skip = skip;
      }
      out[r].rc = call(f, out[r].v);
      out[r].msg = olpe_last_error();
      out[r].trace = f.trace;
      if (follow_up) {
        f.fault_site = -1;
        out2[r].rc = call(f, out2[r].v);
        out2[r].msg = olpe_last_error();
      }
    });
  for (auto &t : th) t.join();
  if (second) *second = out2;
  if (stuck) *stuck = w.stuck;
  if (mism) *mism = w.mismatches;
  (void)wout;
  return out;
}

static bool is_collective(int s) {
  return s == kCheckReduce || s == kR1Reduce || s == kR2Reduce || s == kGather;
}

// ---------------------------------------------------------------------------------------
static void moments_cases(int n, int timeout_ms) {
  const int ps = 17, np = 16;
  const size_t len = OLPE_MOMENTS_LEN(ps, np);
  auto call_prc = [&](int prc_rank) -> Call {
    return [=](Fake &f, std::vector<double> &o) {
      std::vector<double> d(len + ps, 0.0);
      o.assign(len, 0.0);
      int prc = OLPE_OK;
      if (f.rank == prc_rank && f.fault_site >= 0)
        prc = set_err(OLPE_ENOMEM, "preparation failure injected on rank %d", f.rank);
      return allreduce_moments(f, d.data(), len, ps, walkers_of(f.rank), 50, prc, o.data());
    };
  };
  const Call call = call_prc(-1);
  // clean
  std::vector<std::string> stuck;
  auto o = run_world(n, timeout_ms, call, -1, -1, -1, false, false, nullptr, nullptr, &stuck);
  ++g_cases;
  for (int r = 0; r < n; ++r) {
    EXPECT(o[r].rc == OLPE_OK, "clean moments rank %d: %s", r, o[r].msg.c_str());
    EXPECT(o[r].rc || moments_exact(n, o[r].v, ps, np), "clean moments rank %d sums", r);
  }
  EXPECT(stuck.empty(), "clean moments stuck");
  // every step of every rank
  for (int fr = 0; fr < n; ++fr) {
    std::map<int, int> seen;
    for (int s : o[fr].trace) {
      const int occ = seen[s]++;
      std::vector<Out> o2;
      int mism = 0;
      auto a = run_world(n, timeout_ms, call, fr, s, occ, false, !is_collective(s), &o2,
                         nullptr, &stuck, &mism);
      ++g_cases;
      const char *sn = site_name(s);
      EXPECT(a[fr].rc != OLPE_OK, "moments fault %s#%d on rank %d: no error", sn, occ, fr);
      EXPECT(mism == 0, "moments fault %s#%d on rank %d: mismatched collectives", sn, occ, fr);
      if (is_collective(s)) {
        // bounded, not hang-free: the peers time out, and nobody reports success
        for (int r = 0; r < n; ++r)
          EXPECT(a[r].rc != OLPE_OK, "collective fault %s on rank %d: rank %d succeeded", sn, fr, r);
        continue;
      }
      EXPECT(stuck.empty(), "moments fault %s#%d on rank %d: %s", sn, occ, fr,
             stuck.empty() ? "" : stuck[0].c_str());
      const bool last_read = s == kR2Back || s == kR2Wait;
      for (int r = 0; r < n; ++r) {
        if (r == fr) continue;
        if (last_read)
          EXPECT(a[r].rc == OLPE_OK && moments_exact(n, a[r].v, ps, np),
                 "fault %s on rank %d: peer %d rc %d %s", sn, fr, r, a[r].rc, a[r].msg.c_str());
        else
          EXPECT(a[r].rc != OLPE_OK, "fault %s#%d on rank %d: peer %d succeeded", sn, occ, fr, r);
      }
      for (int r = 0; r < n; ++r)
        EXPECT(o2[r].rc == OLPE_OK && moments_exact(n, o2[r].v, ps, np),
               "after fault %s#%d on rank %d: rank %d follow-up rc %d %s", sn, occ, fr, r,
               o2[r].rc, o2[r].msg.c_str());
    }
    // the preparation failing on this rank (its outcome travels in the check)
    std::vector<Out> o2;
    auto a = run_world(n, timeout_ms, call_prc(fr), fr, kSites, 0, false, true, &o2, nullptr,
                       &stuck);
    ++g_cases;
    EXPECT(stuck.empty(), "prepare fault on rank %d stuck", fr);
    for (int r = 0; r < n; ++r) {
      EXPECT(a[r].rc == (r == fr ? OLPE_ENOMEM : OLPE_ENOMEM), "prepare fault rank %d: rc %d",
             r, a[r].rc);
      EXPECT(o2[r].rc == OLPE_OK, "after prepare fault: rank %d follow-up %s", r,
             o2[r].msg.c_str());
    }
  }
  printf("moments n=%d: every step of every rank\n", n);
}

static void gather_cases(int n, int timeout_ms) {
  const size_t per = 6;
  auto mk = [&](int bad_rank, int alloc_rank, int range_rank) -> Call {
    return [=](Fake &f, std::vector<double> &o) {
      std::vector<double> send(per), recv(per * n, -1.0);
      for (size_t i = 0; i < per; ++i) send[i] = 100.0 * f.rank + (double)i;
      o.assign(per * n, 0.0);
      const bool faulted = f.fault_site >= 0;
      const bool bad = faulted && f.rank == bad_rank;
      const bool nomem = faulted && f.rank == alloc_rank;
      const long long w0 = faulted && f.rank == range_rank ? 1 : 0;
      First fe;
      if (bad) fe.add(set_err(OLPE_EINVAL, "bad range injected"));
      if (nomem) fe.add(set_err(OLPE_ENOMEM, "allocation failure injected"));
      return allgather(f, send.data(), nomem ? nullptr : recv.data(), bad ? 0 : per, n, 4, 10,
                       w0, 2, bad, 4, o.data(), fe);
    };
  };
  auto exact = [&](const std::vector<double> &o) {
    for (int r = 0; r < n; ++r)
      for (size_t i = 0; i < per; ++i)
        if (o[r * per + i] != 100.0 * r + (double)i) return false;
    return true;
  };
  const Call clean = mk(-1, -1, -1);
  std::vector<std::string> stuck;
  auto o = run_world(n, timeout_ms, clean, -1, -1, -1, false, false, nullptr, nullptr, &stuck);
  ++g_cases;
  for (int r = 0; r < n; ++r) EXPECT(o[r].rc == OLPE_OK && exact(o[r].v), "clean gather %d", r);
  for (int fr = 0; fr < n; ++fr) {
    std::map<int, int> seen;
    for (int s : o[fr].trace) {
      const int occ = seen[s]++;
      std::vector<Out> o2;
      auto a = run_world(n, timeout_ms, clean, fr, s, occ, false, !is_collective(s), &o2,
                         nullptr, &stuck);
      ++g_cases;
      const char *sn = site_name(s);
      EXPECT(a[fr].rc != OLPE_OK, "gather fault %s on rank %d: no error", sn, fr);
      if (is_collective(s)) {
        for (int r = 0; r < n; ++r)
          EXPECT(a[r].rc != OLPE_OK, "gather collective fault %s rank %d: %d ok", sn, fr, r);
        continue;
      }
      EXPECT(stuck.empty(), "gather fault %s#%d on rank %d: %s", sn, occ, fr,
             stuck.empty() ? "" : stuck[0].c_str());
      const bool after_check = s == kGatherBack || s == kGatherWait || s == kCheckBack ||
                               s == kCheckWait;
      for (int r = 0; r < n; ++r) {
        if (r != fr && !after_check)
          EXPECT(a[r].rc != OLPE_OK, "gather fault %s on rank %d: peer %d ok", sn, fr, r);
        if (r != fr && after_check)
          EXPECT(a[r].rc == OLPE_OK && exact(a[r].v), "gather fault %s on rank %d: peer %d %s",
                 sn, fr, r, a[r].msg.c_str());
        EXPECT(o2[r].rc == OLPE_OK && exact(o2[r].v), "after gather fault %s: rank %d", sn, r);
      }
    }
    // local failures that travel in the check: a bad range, a failed allocation, a
    // different range -- every rank returns the error, nobody enters the gather
    const struct { int bad, alloc, range, code; } loc[3] = {
        {fr, -1, -1, OLPE_EINVAL}, {-1, fr, -1, OLPE_ENOMEM}, {-1, -1, fr, OLPE_EINVAL}};
    for (auto &L : loc) {
      std::vector<Out> o2;
      auto a = run_world(n, timeout_ms, mk(L.bad, L.alloc, L.range), fr, kSites, 0, false, true,
                         &o2, nullptr, &stuck);
      ++g_cases;
      EXPECT(stuck.empty(), "local gather failure on rank %d stuck", fr);
      for (int r = 0; r < n; ++r) {
        EXPECT(n == 1 && L.range >= 0 ? a[r].rc == OLPE_OK : a[r].rc == L.code,
               "local gather failure on rank %d: rank %d rc %d (%s)", fr, r, a[r].rc,
               a[r].msg.c_str());
        EXPECT(o2[r].rc == OLPE_OK, "after local gather failure: rank %d", r);
      }
    }
  }
  printf("gather n=%d: every step of every rank\n", n);
}

// the negative control: a rank that skips a collective (what the round-5 moments code did
// when round 1's read-back failed) leaves its peers stuck -- the harness must see it
static void negative_control(int n, int timeout_ms) {
  const int ps = 17, np = 16;
  const size_t len = OLPE_MOMENTS_LEN(ps, np);
  const Call call = [=](Fake &f, std::vector<double> &o) {
    std::vector<double> d(len + ps, 0.0);
    o.assign(len, 0.0);
    return allreduce_moments(f, d.data(), len, ps, walkers_of(f.rank), 50, OLPE_OK, o.data());
  };
  std::vector<std::string> stuck;
  run_world(n, timeout_ms, call, n - 1, kR2Reduce, 0, true, false, nullptr, nullptr, &stuck);
  ++g_cases;
  EXPECT(!stuck.empty(), "a skipped collective was not detected");
  printf("negative control n=%d: skipped collective detected (%zu stuck)\n", n, stuck.size());
}

// one context without a communicator: the collectives are local copies
static void no_comm_case() {
  const int ps = 17, np = 16;
  const size_t len = OLPE_MOMENTS_LEN(ps, np);
  const Call call = [=](Fake &f, std::vector<double> &o) {
    std::vector<double> d(len + ps, 0.0);
    o.assign(len, 0.0);
    return allreduce_moments(f, d.data(), len, ps, walkers_of(f.rank), 50, OLPE_OK, o.data());
  };
  auto o = run_world(1, 100, call, -1, -1, -1, false, false, nullptr, nullptr, nullptr, nullptr,
                     false);
  ++g_cases;
  EXPECT(o[0].rc == OLPE_OK && moments_exact(1, o[0].v, ps, np), "no-comm moments");
  printf("no communicator: local summary\n");
}

int main(int argc, char **argv) {
  const int tmo = argc > 1 ? atoi(argv[1]) : 200;
  no_comm_case();
  for (int n : {1, 2, 3, 4}) {
    moments_cases(n, tmo);
    gather_cases(n, tmo);
  }
  negative_control(2, tmo);
  negative_control(4, tmo);
  if (g_fail) {
    printf("FAILED %d checks over %d cases\n", g_fail, g_cases);
    return 1;
  }
  printf("ALL OK cases=%d\n", g_cases);
  return 0;
}
