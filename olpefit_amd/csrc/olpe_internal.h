// olpe_internal.h -- the context object behind the opaque olpe_ctx handle.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

struct olpe_ctx {
  int device = 0;
  int n = 0;           // square cutout side
  int nsrc = 2;
  int bkgd_mode = 0;
  int np = 16, ps = 17;
  int eval_mode = 1;   // OLPE_EVAL_FAST (default) / OLPE_EVAL_EXACT
  bool lds_img = true; // cutout + 1/err staged in LDS by the sampler
  int wpb = 0;         // waves per workgroup of the 64x64 LDS sampler (0 = 12)
  hipStream_t stream = nullptr;
  // start/stop events of the last kRing sampler launches (olpe_kernel_times)
  static constexpr int kRing = 64;
  hipEvent_t ev[kRing][2] = {};
  long long launches = 0;
  double2 *d_DE = nullptr;   // [n*n] {data as f64, 1/err}, {0,0} where masked (EXACT)
  double2 *d_DW = nullptr;   // [n*n] {data/err, 1/err}, {0,0} where masked (FAST)
  // walker ensemble
  int W = 0;
  bool seeded = false;
  long long count = 0;
  double *d_state = nullptr;     // [W][ps]
  uint32_t *d_tries = nullptr;   // [W][np]
  uint32_t *d_acc = nullptr;     // [W][np]
  uint32_t *d_mt = nullptr;      // [W][624]
  int *d_mtpos = nullptr;        // [W]
  double *d_gauss = nullptr;     // [W]
  int *d_hasg = nullptr;         // [W]
  long long *d_done = nullptr;   // [W]
  // last launch's chain / trace
  double *d_chain = nullptr;
  size_t chain_cap = 0;
  long long chain_rows = 0;
  double *d_trace = nullptr;
  size_t trace_cap = 0;
  int trace_on = 0;
  long long trace_iters = 0;
  // scratch for olpe_model / olpe_chi2_batch
  double *d_scratch = nullptr, *d_scratch2 = nullptr;
  size_t scratch_cap = 0, scratch2_cap = 0;
  // walker queue of the sampler (one 64-bit counter; each launch takes W + its waves
  // from it, so no reset between launches): qbase = the counter's value at launch
  unsigned long long *d_queue = nullptr;
  unsigned long long qbase = 0;
  bool queue_on = true;
  int n_cu = 0;
  // work units (choose_units): walkers cut into chunks handed between waves through
  // uflag[W]; utag = the last launch's tag base (+16 per launch)
  unsigned *d_uflag = nullptr;
  unsigned utag = 0;
  int units_override = 0;   // OLPE_UNITS
  bool hold_handoff = false; // test hook (olpe_test_hold_handoff)
  int last_units = 1;       // chunks per walker of the last launch (olpe_last_units)
  bool units_used = false;  // some launch handed chunks between waves (check_units)
  double wait_limit_s = 30; // hand-off wait limit of the last launch (unit_wait)
  double wait_ticks_override = 0;  // OLPE_WAIT_TICKS (tests of the time-out path)
  int balance = -1;         // progress balancing (-1: launch_gibbs_t picks)
  int ring_wpb = 12;        // 128x128 FAST: the lockstep LDS-ring sampler's waves per
                            // workgroup, 0 = the L2-resident sampler (OLPE_RING)
  int stagger = 0;          // wave start offsets (always 0; see GibbsArgs)
  // whole-run moments of the recorded rows (olpe_moments.hip): running mean / M2 per
  // walker and column, [ps][W]; mom_n rows folded per walker; mom_folded = the launch
  // whose rows were folded last (a launch is folded at most once)
  double *d_mmean = nullptr, *d_mm2 = nullptr;
  size_t mom_cap = 0;
  long long mom_n = 0;
  long long mom_folded = 0;
  double *d_mpart = nullptr;    // partial sums of olpe_moments_local
  size_t mpart_cap = 0;
  int mom_fault = 0;            // test hook (olpe_moments_fault, include/olpe_test.h): 1 =
                                // the preparation's allocation fails, 2 = the summary launch
                                // fails, 3 = the check words' send fails, 4 = round 1's
                                // read-back fails
  // RCCL communicator (olpe_comm.hip)
  void *comm = nullptr;
  int nranks = 1, rank = 0;
  double *d_gather = nullptr;   // receive buffer of olpe_comm_allgather_chain
  size_t gather_cap = 0;
  size_t gather_limit = 0;      // its byte limit (olpe_comm_gather_limit; 0 = none)
  long long *d_check = nullptr; // the collectives' words: the uniformity check's, then the
                                // poisoned defaults (olpe_comm_setup, called by olpe_create,
                                // so that joining a communicator allocates nothing)
  double comm_timeout_s = 600;  // bound on every wait for the other ranks (olpe_comm_timeout)
  bool comm_aborted = false;    // the communicator was aborted after a timeout / RCCL error
};

namespace olpe {
int set_err(int code, const char *fmt, ...);
}
void olpe_comm_release(olpe_ctx *c);
// the collectives' word buffer with its poisoned defaults (olpe_comm.hip; olpe_create)
int olpe_comm_setup(olpe_ctx *c);
// the buffers (and zeroing) of the per-column sums (olpe_moments.hip); then the sums over
// this context's walkers into d_out[2 ..], launches only
int olpe_moments_prepare(olpe_ctx *c);
int olpe_moments_local(olpe_ctx *c, const double *d_centre, double *d_out);
