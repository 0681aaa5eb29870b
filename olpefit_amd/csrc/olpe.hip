// olpe.hip -- gfx950 kernels and the C-ABI (include/olpe.h) of libolpe.so.
//
// Kernels
//   olpe_gibbs_kernel  fused sampler: W walkers, one per wavefront at a time (a
//                      persistent grid whose waves take walkers from a device queue),
//                      n_iters Gibbs iterations each (apf_step2.py:300-351) with the
//                      cutout and inverse-sigma map staged once per workgroup into LDS
//                      (64x64 and smaller; L2-resident above).
//   olpe_eval_kernel   build_analytical_model / chi_squared of explicit parameter
//                      vectors (olpe_model test hook, olpe_chi2_batch)
//   olpe_seed_kernel   np.random.seed per walker
//   olpe_stream_kernel RNG stream dump (test hook)
#include <hip/hip_runtime.h>

#include <limits.h>
#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <atomic>
#include <vector>

#include "../../include/olpe.h"
#include "../../include/olpe_test.h"
#include "olpe_device.h"
#include "olpe_internal.h"

using namespace olpe;

namespace {

// ---------------------------------------------------------------------------------
// Jump widths (apf_step2.py:234; 3body/apf_step2_3body.py:220-238)
// ---------------------------------------------------------------------------------
__constant__ double c_widths2[16] = {0.01, 0.01, 0.3,   0.3,    0.08,  0.09,
                                     0.0025, 0.02, 0.001, 0.0008, 0.002, 0.002,
                                     0.001, 0.001, 0.008, 0.01};
__constant__ double c_widths3[19] = {0.01,  0.01,  0.3,   0.3,  0.3,   0.3,   0.08,
                                     0.09,  0.0025, 0.02, 0.02, 0.001, 0.0008, 0.002,
                                     0.002, 0.001, 0.001, 0.008, 0.01};

template <int NSRC> __device__ __forceinline__ double width_of(int r) {
  return NSRC == 2 ? c_widths2[r] : c_widths3[r];
}

struct GibbsArgs {
  const double2 *DE;   // [n*n] {data, 1/err} (EXACT) or {data/err, 1/err} (FAST); {0,0} masked
  int n;
  int bkgd_mode;
  long long W;
  double *state;       // [W][PS]
  uint32_t *tries;     // [W][NP]
  uint32_t *accepts;   // [W][NP]
  uint32_t *mt;        // [W][624]
  int *mt_pos;         // [W]
  double *gauss;       // [W]
  int *has_gauss;      // [W]
  long long *done_at;  // [W]
  long long n_iters;
  long long count0;
  long long burn_in;
  long long stride;    // 0 = no chain
  long long row0;      // global row index of the first row of this launch
  long long nrows;     // rows per walker in `chain`
  double *chain;       // [W][nrows][PS]
  long long accept_min;
  double *trace;       // [W][n_iters][6] or null
  // walker queue: null = one walker per wave at blockIdx*WPB + wave; otherwise each
  // wave takes work units qbase.. from the counter until it passes W * units
  // (persistent grid)
  unsigned long long *queue;
  unsigned long long qbase;
  // work units: each walker's n_iters iterations are cut into `units` consecutive
  // chunks, unit u = chunk u / W of walker u % W (chunk-major, so a chunk's predecessor
  // was handed out W units earlier).  Chunk k > 0 waits until uflag[w] == utag + k;
  // the wave that ran chunk k publishes utag + k + 1 (launch_gibbs_t)
  int units;
  unsigned *uflag;     // [W]
  unsigned utag;       // this launch's tag base (a multiple of 16)
  unsigned *uerr;      // set to 1 when a hand-off wait times out (olpe_sync reports it)
  unsigned long long wait_ticks;   // a hand-off wait gives up after this many 100 MHz ticks
  int balance;         // progress balancing of the LDS sampler (launch_gibbs_t picks)
  int stagger;         // start offset per wave rank within a SIMD, in ~0.5 us: always 0
                       // (round 2's OLPE_STAGGER changed nothing; the host knob is gone,
                       // the argument kept so that the sampler's code is unchanged)
  unsigned *hold;      // test hook (olpe_test_hold_handoff), null otherwise: a wave that
                       // ends a walker's first chunk waits, before it hands the walker on,
                       // until a wave waiting for some walker's next chunk sets the word --
                       // so every launch with chunks has a hand-off that waits, whatever
                       // the dispatch order (verdict r05 item 5)
};

constexpr int kTraceF = 6;
// sampler LDS header: the exp table, then 64 B of progress-balancing words
constexpr int kSampHdr = kEtabBytes + 64;


// ---------------------------------------------------------------------------------
// The fused sampler
// ---------------------------------------------------------------------------------
// Per-wave LDS slice: tries[NP] | accepts[NP] | state doubles (below) | per-step model
// descriptor | the proposal's column terms of the Gaussians it moves (E, rho per lane,
// NSRC slots) | (after BYTES) the shape tables / V table.  The MT key stays in HBM.
template <int NP> struct WaveSlice {
  static constexpr int U32 = 2 * NP;                         // 8-byte multiple for NP 16/19
  static constexpr int PS = NP + 1;
  static constexpr int NSRC = NP == 16 ? 2 : 3;
  // doubles: params[PS] | T1[5] T2[5] | C1[3] C2[3] | pending T[5] C[3] | proposal[PS];
  // a shape set's T holds cos^2, sin^2, sin 2theta and (FAST) 1/sigma_x^2, 1/sigma_y^2
  static constexpr int OT1 = PS, OT2 = PS + 5, OC1 = PS + 10, OC2 = PS + 13;
  static constexpr int OPT = PS + 16, OPC = PS + 21;
  static constexpr int OPR = PS + 24;
  static constexpr int F64 = 2 * PS + 24;
  static constexpr int OMD = ((U32 * 4 + F64 * 8 + 15) & ~15);             // ModelDesc
  // col_coef [G][3], then (128 x 128) the pass-step factors exp(-64 b) [G]
  static constexpr int OCC = (OMD + (int)sizeof(ModelDesc<NSRC>) + 15) & ~15;
  static constexpr int OPE = (OCC + 2 * NSRC * 4 * 8 + 15) & ~15;
  static constexpr int BYTES = OPE + NSRC * 2 * 64 * 8;
};
// MTWave draw tables (kDrawTab doubles per wave).  Kernels with the FAST3 column-term
// cache (NT = 32, 64) keep them after the slice; the others in the parking area of
// the proposal's column terms, which only that cache uses.
// EXACT samplers keep no accept thresholds (MTWave::thr): kThr doubles
constexpr int kDrawTabBytes = (kDrawTab * 8 + 15) & ~15;
constexpr int kDrawTabExactBytes = (kThr * 8 + 15) & ~15;
__host__ __device__ constexpr int drawtab_extra(int nt, bool fast = true) {
  return (nt != 0 && nt <= 64) ? (fast ? kDrawTabBytes : kDrawTabExactBytes) : 0;
}
// bytes of the per-wave V table of sweep_fast: n rows x 2*nsrc doubles
__host__ __device__ inline int vtab_bytes(int n, int nsrc) { return (n * 2 * nsrc * 8 + 15) & ~15; }
// per-wave table area of the sampler: the V table (or the two FAST3 shape-table slots,
// 2 x rows x 16 B, which fit in it); the 3-source 64x64 sampler keeps only the shape
// tables (its V-table fallback runs the exact sweep instead) so that its LDS layout
// fits 12 waves beside the cutout
// The 16-wave 2-source 64x64 FAST sampler keeps ONE shape-table slot (HCache::single:
// a shape proposal rebuilds its set in place, and after a reject the current state's
// set is rebuilt at the next step) and has no V-table fallback (its lvl-1 steps take
// the exact sweep), so that 16 wave slices fit the LDS beside the 64 KiB cutout.
__host__ __device__ constexpr bool single_h(int nsrc, int nt, int wpb, bool fast) {
  return nsrc == 2 && nt == 64 && wpb == 16 && fast;
}
__host__ __device__ constexpr int sampler_vtab_bytes(int n, int nsrc, int nt, int wpb = 12,
                                                     bool fast = false) {
  return single_h(nsrc, nt, wpb, fast) ? 64 * 16
       : (nsrc == 3 && nt == 64) ? 2 * 64 * 16 : ((n * 2 * nsrc * 8 + 15) & ~15);
}
// the ring sampler's per-wave slice: the WaveSlice fields up to the parking area, the
// draw tables there (its sweeps park nothing) and the two FAST3 shape-table slots (no
// V-table fallback)
template <int NP> __host__ __device__ constexpr int ring_wave_bytes(int n) {
  return WaveSlice<NP>::OPE + kDrawTabBytes + 2 * n * 16;
}
// (8 waves: the diagnostic 8-wave ring of tools/diag/diag_hooks.patch only -- the same sweep at 2 waves per
// SIMD, the bound on the 4-wave layout's gain)
__host__ __device__ constexpr bool ring_wpb(int nt, int wpb) {
  return nt == 128 && (wpb == 12 || wpb == 8);
}
static_assert((WaveSlice<16>::U32 * 4) % 8 == 0 && (WaveSlice<19>::U32 * 4) % 8 == 0, "align");
// the EXACT samplers' row tables (sweep_exact_rows, [n][G] doubles each): 64x64 2-source
// dy in the parking area and c*dy^2 in the V-table area; 64x64 3-source c*dy^2 in the
// parking area; 32x32 both in the parking area; 128x128 c*dy^2 in the V-table area
// (the parking area holds the draw tables there)
template <int NP> constexpr int parking_bytes() { return WaveSlice<NP>::BYTES - WaveSlice<NP>::OPE; }
static_assert(parking_bytes<16>() >= 64 * 4 * 8 && sampler_vtab_bytes(64, 2, 64) >= 64 * 4 * 8 &&
              parking_bytes<19>() >= 64 * 6 * 8 && parking_bytes<16>() >= 2 * 32 * 4 * 8 &&
              parking_bytes<19>() >= 2 * 32 * 6 * 8 && sampler_vtab_bytes(128, 2, 128) >= 128 * 4 * 8 &&
              sampler_vtab_bytes(128, 3, 128) >= 128 * 6 * 8 && drawtab_extra(32) && drawtab_extra(64),
              "sweep_exact_rows tables");

__device__ __forceinline__ Trig ld_trig(const double *s) { return Trig{s[0], s[1], s[2]}; }
__device__ __forceinline__ Coef ld_coef(const double *s) { return Coef{s[0], s[1], s[2]}; }
__device__ __forceinline__ void st_trig(double *s, const Trig &t) {
  s[0] = t.cost2; s[1] = t.sint2; s[2] = t.sin2t;
}
// a shape set's cached terms: trig + the reciprocal variances (FAST coefficients)
__device__ __forceinline__ void st_shape(double *s, const Trig &t, double ix, double iy) {
  st_trig(s, t);
  s[3] = ix; s[4] = iy;
}
__device__ __forceinline__ void st_coef(double *s, const Coef &k) {
  s[0] = k.a; s[1] = k.b; s[2] = k.c;
}

// Work-unit hand-off between waves of one launch (possibly on different XCDs), the
// publish/consume protocol of cdna_hip_programming.md Guideline 16 (R1): the producing
// wave stores the walker's words write-through (sc1: state, counters, RNG position and
// cached deviate, done_at; the MT key words are agent-scope stores too), drains them
// (s_waitcnt vmcnt(0)) and sets the flag with a relaxed agent store; the consumer polls
// the flag with relaxed agent loads and takes one agent acquire before its loads.  The
// poll ends after wait_ticks of real time (100 MHz s_memrealtime; the host sizes it to
// the chunk: at least 30 s, launch_gibbs_t) whatever happens, so the grid always drains.
// Write-through (sc1) stores of the handed-off words through global-address-space
// pointers (never flat), so the hand-off needs no L2 write-back (release fence): the
// guide's R1 form.  The same stores run at the end of every unit.
typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;
__device__ __forceinline__ void st_wt(double *p, double v) {
  __hip_atomic_store((gu64 *)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(long long *p, long long v) {
  __hip_atomic_store((gu64 *)p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T> __device__ __forceinline__ void st_wt(T *p, T v) {
  static_assert(sizeof(T) == 4, "32-bit word");
  unsigned u;
  __builtin_memcpy(&u, &v, 4);
  __hip_atomic_store((gu32 *)p, u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one handed-off 32-bit word read by a vector load (never the scalar cache), uniform
template <class T> __device__ __forceinline__ T ld_uniform(const T *p) {
  static_assert(sizeof(T) == 4, "32-bit word");
  const unsigned u = (unsigned)__builtin_amdgcn_readfirstlane(
      (int)__hip_atomic_load((gu32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  T v;
  __builtin_memcpy(&v, &u, 4);
  return v;
}
__device__ __forceinline__ void unit_publish(unsigned *flag, unsigned v, int lane) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the wave's sc1 stores have landed
  if (lane == 0) __hip_atomic_store((gu32 *)flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void unit_wait(unsigned *flag, unsigned want, unsigned *err,
                                          unsigned long long *stats, int lane,
                                          unsigned long long limit, unsigned *hold) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  bool waited = false;
  for (;;) {
    const unsigned v = (unsigned)__builtin_amdgcn_readfirstlane(
        (int)__hip_atomic_load((gu32 *)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (v == want) break;
    // (test hook: this wait releases the first chunks held at their hand-off)
    if (!waited && hold && lane == 0)
      __hip_atomic_store((gu32 *)hold, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    waited = true;
    if (__builtin_amdgcn_s_memrealtime() - t0 > limit) {
      __hip_atomic_store((gu32 *)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(4);
  }
  // hand-off statistics (olpe_unit_stats): waits and their 100 MHz ticks
  if (waited && lane == 0) {
    atomicAdd(stats, 1ull);
    atomicAdd(stats + 1, __builtin_amdgcn_s_memrealtime() - t0);
  }
  // ONE acquire after the match: this CU's L1 may hold lines of the walker from an
  // earlier chunk
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// test hook (olpe_test_hold_handoff): hold a first chunk's hand-off until some wave is
// waiting for a hand-off (bounded like unit_wait: the grid always drains)
__device__ __forceinline__ void hold_handoff(unsigned *hold, unsigned *err, unsigned long long limit) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_readfirstlane((int)__hip_atomic_load((gu32 *)hold, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT)) == 0) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > limit) {
      __hip_atomic_store((gu32 *)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(4);
  }
}

// wave priority of the step's control chain (the sweep runs at 0, or 0/1 with balancing)
constexpr int kCtrlPrio = 2;
// the global-memory sampler's minimum waves per SIMD (its launch bound, below)
constexpr int kGlobalWavesPerEU = 3;
template <int NSRC, int NT, bool LDS_IMG, int WPB, bool FAST>
// The global-memory (large cutout) variant runs 4-wave workgroups and waits on L2: it
// is asked to fit 3 of them per CU (168 VGPRs, no spills; 3-source 128x128 +0.9 % over
// 4 per CU at 128 VGPRs, +4.5 % over 2 per CU)
// (hipcc passes the second bound on as the minimum waves per SIMD; the ring sampler,
// NT = 128 with one 12-wave workgroup per CU, keeps 3 per SIMD with 168 VGPRs)
// (the diagnostic 8-wave ring keeps the 12-wave one's register budget -- at least 3 waves
// per SIMD, 168 VGPRs -- so that it runs the same code at 2 waves per SIMD)
__global__ __launch_bounds__(WPB * 64, (LDS_IMG || (NT == 128 && WPB == 12)) ? 1 : kGlobalWavesPerEU)
void olpe_gibbs_kernel(GibbsArgs A) {
  using L = Layout<NSRC>;
  using WS = WaveSlice<L::NP>;
  constexpr int NP = L::NP, PS = L::PS;
  // the 128x128 lockstep sampler: 12 waves share an LDS ring of the cutout (LdsRing,
  // olpe_device.h); they take work units as batches of 12 and run their steps together
  constexpr bool RING = !LDS_IMG && FAST && ring_wpb(NT, WPB);
  using Ring = LdsRing<WPB>;
  extern __shared__ __align__(16) unsigned char smem[];
  const int n = NT ? NT : A.n;
  const int npix = n * n;
  const int lane = threadIdx.x & 63;
  // wave index as a provably uniform (SGPR) value: LDS slice addresses stay scalar
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  // ---- LDS carve: exp table, [DE] (if staged), then one {WaveSlice, V table} per wave
  double *etab = reinterpret_cast<double *>(smem);
  unsigned *s_prog = reinterpret_cast<unsigned *>(smem + kEtabBytes);  // progress balancing
  double2 *sDE = reinterpret_cast<double2 *>(smem + kSampHdr);
  constexpr int TABX = drawtab_extra(NT, FAST);
  const int wstride = RING ? ring_wave_bytes<NP>(n)
                           : WS::BYTES + TABX + sampler_vtab_bytes(n, NSRC, NT, WPB, FAST);
  unsigned char *wb = reinterpret_cast<unsigned char *>(sDE + (LDS_IMG ? npix : 0)) +
                      (RING ? Ring::BYTES : 0) + (size_t)wave * wstride;
  uint32_t *s_tries = reinterpret_cast<uint32_t *>(wb);
  uint32_t *s_acc = s_tries + NP;
  double *st = reinterpret_cast<double *>(wb + WS::U32 * 4);
  double *vtab = reinterpret_cast<double *>(wb + (RING ? WS::OPE + kDrawTabBytes : WS::BYTES + TABX));
  double *drawtab = reinterpret_cast<double *>(wb + (TABX ? WS::BYTES : WS::OPE));
  ModelDesc<NSRC> *mdl = reinterpret_cast<ModelDesc<NSRC> *>(wb + WS::OMD);
  double *colc = reinterpret_cast<double *>(wb + WS::OCC);

  if constexpr (LDS_IMG) {
    // one coalesced 16-B-per-lane staging pass of {data, 1/err}
    for (int k = threadIdx.x; k < npix; k += blockDim.x) sDE[k] = A.DE[k];
  }
  if (threadIdx.x < 64) etab[threadIdx.x] = c_exp2_64[threadIdx.x];
  if (threadIdx.x == 0) s_prog[0] = 0u;
  __syncthreads();
  const double2 *DE = LDS_IMG ? sDE : A.DE;
  [[maybe_unused]] Ring ring;
  if constexpr (RING) ring.prologue(smem + kSampHdr, A.DE, wave, lane);
  unsigned my_steps = 0;   // iterations this wave has started in this launch
  // start offset: the waves of a SIMD (wave, wave + 4, wave + 8) start a fraction of a
  // step apart so that their latency-bound control phases do not coincide
  for (int i = 0, n = (wave >> 2) * A.stagger; i < n; ++i) __builtin_amdgcn_s_sleep(8);

  // Arguments used once per walker are read where they are used, through a kernarg
  // pointer the compiler cannot see through, so that they do not hold SGPRs across
  // the sampler loop (SGPR pressure spills into VGPR lanes).
  auto K = []() {
    const __attribute__((address_space(4))) GibbsArgs *p =
        (const __attribute__((address_space(4))) GibbsArgs *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return p;
  };

  // walker of this wave: static, or the next one off the queue -- a wave that
  // finishes its walker takes another at once, instead of idling until the slowest
  // wave of its workgroup is done (waves of one SIMD run at different speeds: VALU
  // issue goes by age)
  // (the host keeps W < 2^31, so the walker index is a 32-bit value)
  auto take = [&]() -> int {
    unsigned long long v = 0;
    if (lane == 0) v = atomicAdd(K()->queue, 1ull) - K()->qbase;
    const unsigned d = v > 0x7fffffffull ? 0x7fffffffu : (unsigned)v;
    return __builtin_amdgcn_readfirstlane((int)d);
  };

  // chain rows: the iteration (0-based, this launch) of the next record -- count =
  // count0 + it + 1 >= burn_in and (count - burn_in) % stride == 0 -- and its row,
  // advanced by 32-bit addition (host: n_iters < 2^31); the same for every walker
  const int niter = (int)A.n_iters;
  const int rstride = (int)A.stride;
  const int nrows = (int)A.nrows;
  int rec_it0 = -1, rec_row0 = 0;
  if (A.stride > 0) {
    const long long c1 = A.count0 + 1;
    const long long k = c1 > A.burn_in ? (c1 - A.burn_in + A.stride - 1) / A.stride : 0;
    const long long first = A.burn_in + k * A.stride - c1;
    rec_it0 = first < niter ? (int)first : -1;
    rec_row0 = (int)(k - A.row0);
  }
  // ring sampler: the workgroup takes its units as batches of WPB (wave 0 draws the batch,
  // an LDS word hands it to the others); s_prog[1] holds the batch, s_prog[2 + wave] the
  // waves' iteration counts
  auto take_batch = [&]() -> int {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (wave == 0 && lane == 0) {
      const unsigned long long v = atomicAdd(K()->queue, 1ull) - K()->qbase;
      s_prog[1] = v > 0x7fffffffull ? 0x7fffffffu : (unsigned)v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    return __builtin_amdgcn_readfirstlane((int)s_prog[1]);
  };
  const int total = (int)K()->W * K()->units;      // (host: W * units < 2^31)
  int u = RING ? 0 : A.queue ? take() : (int)blockIdx.x * WPB + wave;
  for (;;) {
    bool active = true;
    if constexpr (RING) {
      const int bt = take_batch();
      if (bt >= (total + WPB - 1) / WPB) break;    // uniform over the workgroup
      u = bt * WPB + wave;
      active = u < total;
      if (!active) u = 0;       // an idle wave of the last batch: walker 0, read only
    } else {
      if (u >= total) break;
    }
    // ---- the unit: chunk k of walker w, iterations [it_s, it_e) of this launch
    const int units = K()->units;
    const int Wn = (int)K()->W;
    int w = u, k = 0, it_s = 0, it_e = niter;
    if (units > 1) {
      k = u / Wn;
      w = u - k * Wn;
      // floor(niter * k / units) in 32 bits: niter = q units + r, r k < 15 * 15
      const int q = niter / units, r = niter - q * units;
      it_s = q * k + (r * k) / units;
      it_e = q * (k + 1) + (r * (k + 1)) / units;
      // the walker's previous chunk ran on another wave: wait for its hand-off
      if (k > 0 && active)
        unit_wait(K()->uflag + w, K()->utag + (unsigned)k, K()->uerr, K()->queue + 2, lane,
                  K()->wait_ticks, K()->hold);
    }
    // ring sampler: the batch's waves run max(it_e - it_s) lockstep steps; a wave past
    // its own iterations (or without a unit) keeps the phase barriers (idle steps)
    int it_end = it_e;
    if constexpr (RING) {
      if (lane == 0) s_prog[2 + wave] = active ? (unsigned)(it_e - it_s) : 0u;
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      unsigned mx = 0;
      for (int j = 0; j < WPB; ++j) mx = max(mx, s_prog[2 + j]);
      it_end = it_s + (int)__builtin_amdgcn_readfirstlane((int)mx);
      if (!active) it_e = it_s;
    }
    // ---- walker state -> LDS slice
    if (lane < NP) {
      s_tries[lane] = K()->tries[(size_t)w * NP + lane];
      s_acc[lane] = K()->accepts[(size_t)w * NP + lane];
    }
    if (lane < PS) st[lane] = K()->state[(size_t)w * PS + lane];
    wave_sync();
    if (lane == 0) {
      const Trig t1 = make_trig<FAST>(st[L::T1]), t2 = make_trig<FAST>(st[L::T2]);
      st_shape(st + WS::OT1, t1, inv_var(st[L::S1X]), inv_var(st[L::S1Y]));
      st_shape(st + WS::OT2, t2, inv_var(st[L::S2X]), inv_var(st[L::S2Y]));
      st_coef(st + WS::OC1, make_coef<FAST>(st[L::S1X], st[L::S1Y], t1));
      st_coef(st + WS::OC2, make_coef<FAST>(st[L::S2X], st[L::S2Y], t2));
    }
    wave_sync();

    MTWave mt;
    mt.key = K()->mt + (size_t)w * MT_N;
    mt.pos = ld_uniform(K()->mt_pos + w);
    mt.bstart = mt.pos;
    mt.bsize = 0;
    mt.batch = 0;
    mt.has_gauss = ld_uniform(K()->has_gauss + w);
    mt.gauss = uniform_f64(K()->gauss[w]);
    mt.tab = drawtab;
    mt.thr = FAST;

    // accept_min stop (apf_step2.py:300): done_at = the first count at which every
    // parameter has been tried accept_min times.  Touched only when ndone changes (a
    // draw whose tries reach accept_min, once per parameter), so that the step carries
    // no per-iteration VALU work for it and no wait on done_at's load: a per-iteration
    // test kept done_at in VGPRs and made every iteration wait vmcnt(0) -- also on the
    // chain-row stores of the iteration before
    int ndone = 0;
    long long done_at = K()->done_at[w];
    if (A.accept_min > 0) {
      for (int k = 0; k < NP; ++k) ndone += (s_tries[k] >= (uint32_t)A.accept_min);
      ndone = __builtin_amdgcn_readfirstlane(ndone);
      // every parameter tried accept_min times before this unit (a launch with
      // accept_min after one without): done at the end of the unit's first iteration
      if (ndone == NP && done_at < 0 && it_s < it_e) done_at = A.count0 + it_s + 1;
    }

    int rec_it = rec_it0, rec_row = rec_row0;
    if (rec_it0 >= 0 && it_s > rec_it0) {      // the chunk's first record
      const int j = (it_s - rec_it0 + rstride - 1) / rstride;
      rec_it += j * rstride;
      rec_row += j;
    }
    double *chain_w = K()->chain + (size_t)w * nrows * PS;

    HCache hcache;
    hcache.single = single_h(NSRC, NT, WPB, FAST);
    GuardCache gcache;
    ColCache<2 * NSRC> ccache;     // FAST3 column terms of the current state
    ccache.pbuf = reinterpret_cast<double *>(wb + WS::OPE);
    ccache.colc = colc;
    __builtin_amdgcn_s_setprio(kCtrlPrio);
    for (int it = it_s; it < it_end; ++it) {
      if constexpr (RING) {
        if (it >= it_e) {
          ring.idle_step();
          continue;
        }
      }
      // the iteration's draws: randint(0, NP) (apf_step2.py:302), the proposal's gauss()
      // (:63-70) and accept_reject's rand() (:144), left in drawtab[dice_idx]
      int r0 = 0, dice_idx = 0;
      double g = 0.0;
      mt.template draw<NP>(lane, 0, 2, r0, g, dice_idx);
      const int r = __builtin_amdgcn_readfirstlane(r0);
      // total_tries[rand] += 1  (:304)
      const uint32_t tr = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_tries[r]) + 1u;
      wave_sync();
      if (lane == 0) s_tries[r] = tr;
      if (A.accept_min > 0 && tr == (uint32_t)A.accept_min) {
        if (++ndone == NP && done_at < 0) done_at = A.count0 + it + 1;
      }

      // proposal / logproposal (:63-70, :306-309): loc + scale*gauss
      // (read by every lane: nv is made uniform below, cur needs no readfirstlane)
      const double cur = st[r];
      const double wr = width_of<NSRC>(r);
      double nv;
      if ((L::LOGMASK >> r) & 1u) {
        if constexpr (FAST) {
          // 10**(log10(cur) + w g) = cur * e^(w g ln10): no log10, and the exponent is
          // small (|w g ln10| < 0.06 for |g| < 10) -- a degree-9 Taylor polynomial, the
          // table exp beyond; cur < 0 keeps the reference's NaN (log10 of a negative)
          const double x = (wr * g) * 2.302585092994046;
          double e;
          if (fabs(x) < 0.0625) {
            // (constants as SGPR addends: fma_sc, olpe_device.h)
            double p = fma_sc(x, 1.0 / 362880, 1.0 / 40320);
            p = fma_sc(x, p, 1.0 / 5040);
            p = fma_sc(x, p, 1.0 / 720);
            p = fma_sc(x, p, 1.0 / 120);
            p = fma_sc(x, p, 1.0 / 24);
            p = fma_sc(x, p, 1.0 / 6);
            p = fma(x, p, 0.5);
            p = fma(x, p, 1.0);
            e = fma(x, p, 1.0);
          } else {
            e = ExpTab{etab}(x);
          }
          nv = cur < 0.0 ? __builtin_nan("") : cur * e;
        } else {
          const double lv = log10(cur);
          nv = exp10(lv + wr * g);   // 10**lognew (apf_step2.py:69)
        }
      } else {
        nv = cur + wr * g;
      }
      nv = uniform_f64(nv);

      // coefficient sets of the proposal: only the set that r touches is rebuilt
      auto q = [&](int k) -> double { return (k == r) ? nv : st[k]; };
      const int grp = (r == L::S1X || r == L::S1Y || r == L::T1) ? 1
                    : (r == L::S2X || r == L::S2Y || r == L::T2) ? 2 : 0;
      // (FAST: from the set's cached reciprocal variances -- a sigma draw forms one
      // reciprocal, a theta draw none; the same values as make_coef's)
      auto set_coef = [&](int ot, int isx, int isy, int ith) -> Coef {
        const Trig t = (r == ith) ? make_trig<FAST>(nv) : ld_trig(st + ot);
        Coef C;
        if constexpr (FAST) {
          double ix = st[ot + 3], iy = st[ot + 4];
          if (r == isx || r == isy) {
            const double iv = inv_var(nv);
            ix = r == isx ? iv : ix;
            iy = r == isy ? iv : iy;
          }
          C = coef_inv(t, ix, iy);
          if (lane == 0) st_shape(st + WS::OPT, t, ix, iy);
        } else {
          C = make_coef<FAST>(q(isx), q(isy), t);
          if (lane == 0) st_trig(st + WS::OPT, t);
        }
        if (lane == 0) st_coef(st + WS::OPC, C);
        return C;
      };
      Coef C1p, C2p;
      if (grp == 1) C1p = set_coef(WS::OT1, L::S1X, L::S1Y, L::T1);
      else C1p = ld_coef(st + WS::OC1);
      if (grp == 2) C2p = set_coef(WS::OT2, L::S2X, L::S2Y, L::T2);
      else C2p = ld_coef(st + WS::OC2);
      // the step's model descriptor goes to LDS (the sweep loads each field where it is
      // used instead of holding 6*G doubles in registers across it), built lane-parallel:
      // lane g < G writes Gaussian g with make_model's operations, lane G the background
      // the proposal vector, lane-parallel, so that the descriptor lanes read their
      // fields without a per-field select against the drawn index
      if (lane < PS) st[WS::OPR + lane] = (lane == r) ? nv : st[lane];
      wave_sync();
      if (lane < 2 * NSRC) {
        const int s = lane >> 1;
        const bool narrow = lane & 1;
        auto ql = [&](int k) -> double { return st[WS::OPR + k]; };
        const double tot = ql(L::sa(s)) - ql(L::OFF);
        const double wide = tot * ql(L::RATIO);
        const double xc = ql(L::sx(s)), yc = ql(L::sy(s));
        // component-wise selects (a select of whole structs goes through scratch)
        const Coef C{narrow ? C1p.a : C2p.a, narrow ? C1p.b : C2p.b, narrow ? C1p.c : C2p.c};
        const double dx = narrow ? 0.0 : ql(L::DX), dy = narrow ? 0.0 : ql(L::DY);
        const Gauss gq{narrow ? tot - wide : wide, narrow ? xc : xc + dx,
                       narrow ? yc : yc + dy, C};
        mdl->g[lane] = gq;
        // FAST sweeps of n = 64 / 128: the column-term coefficients of this Gaussian
        // (col_term64, row group 0 and S = 1 in both)
        if constexpr (FAST && NT >= 64) col_coef(gq, (double)(NT / 2), colc + 3 * lane);
        // (two column passes: rho of pass 1 = rho of pass 0 x exp(-64 b), pass_rho)
        if constexpr (FAST && NT == 128) colc[6 * NSRC + lane] = ExpTab{etab}(-64.0 * gq.k.b);
      } else if (lane == 2 * NSRC) {
        mdl->bg = q(A.bkgd_mode == 0 ? L::BG_QUIRK : L::BG_FIXED);
      }
      wave_sync();

      // build_analytical_model + chi_squared (:314-316)
      // the step's scalar control is a latency-bound chain: it runs at raised wave
      // priority so that it is not queued behind the other waves' sweeps
      if (LDS_IMG && K()->balance) {
        // progress balancing: VALU issue among a SIMD's waves goes by age, so left alone
        // the waves of a workgroup run at different speeds (per-wave step times spread
        // +-25 %) and a launch ends on its slowest wave, with the SIMDs under-occupied
        // meanwhile (one full round of walkers took 1.4x the steady-state time).  A wave
        // that has started fewer iterations than its workgroup's mean sweeps at
        // priority 1, the others at 0 (the control chain runs at kCtrlPrio above
        // both).
        const unsigned tot = (unsigned)__builtin_amdgcn_readfirstlane((int)s_prog[0]);
        const bool behind = my_steps * (unsigned)WPB < tot;
        if (lane == 0) atomicAdd(s_prog, 1u);
        ++my_steps;
        if (behind) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      } else {
        __builtin_amdgcn_s_setprio(0);
      }
      hcache.grp = grp;
      const unsigned gmask = gauss_mask<NSRC>(r);
      gcache.same = gmask == 0 && grp == 0;
      // (per-column guard cache: the Gaussians this draw moves or reshapes -- a shape
      // set is the narrow Gaussians, odd g, or the wide ones, even g)
      gcache.changed = gmask | ((grp == 1 ? 0xAAAu : grp == 2 ? 0x555u : 0u) & ((1u << (2 * NSRC)) - 1u));
      // A NaN proposal (logproposal of a value <= 0, apf_step2.py:66-69: a background
      // guessed below 0 proposes NaN at every draw of it) makes the reference's model NaN
      // at every pixel, its masked chi^2 NaN and the step a reject (:134-148): no sweep
      // (the guards would send it to the exact sweep, and in the ring sampler hold up
      // the workgroup), the caches left as they are.
      const bool nan_prop = !(nv == nv);
      double part;
      if (nan_prop) {
        gcache.same = false;
        if constexpr (RING) ring.idle_step();
        part = __builtin_nan("");
      } else {
        part = sweep<NSRC, NT, false, FAST, (WPB <= 12), Ring>(*mdl, DE, vtab, nullptr, n, lane, etab,
                                                     &hcache, &ccache, gmask, &gcache,
                                                     RING ? &ring : nullptr);
      }
      __builtin_amdgcn_s_setprio(kCtrlPrio);
      // (the total is valid in lane 63: the accept ballots that lane's test, and lane 63
      // stores an accepted chi^2, so the step needs no readlanes of the sum)
      const double chi = wave_sum_v(part);

      // accept_reject (:139-148): EXACT dice < exp(-(chi - cur)/2); FAST the same test
      // as chi - cur < -2 log(dice) against the batch's threshold table (a NaN chi^2
      // rejects in both)
      const double dchi = chi - st[PS - 1];
      const double la = -dchi / 2.;
      const double dice = drawtab[dice_idx];
      bool acc;
      uint32_t acc_bit;
      if constexpr (FAST) {
        const double thr = drawtab[kThr + (dice_idx == 128 ? 64 : dice_idx)];
        acc_bit = (uint32_t)(__builtin_amdgcn_ballot_w64(dchi < thr) >> 32) >> 31;
      } else {
        acc_bit = (uint32_t)(__builtin_amdgcn_ballot_w64(dice < exp(la)) >> 32) >> 31;
      }
      asm volatile("" : "+s"(acc_bit));     // (kept a scalar: no VALU compare of the ballot)
      acc = acc_bit != 0;
      if (acc && lane == 63) st[PS - 1] = chi;
      // (the trace's uniform copies, taken here so that the sum's VGPRs die at the store)
      double chi_u = 0.0, la_u = 0.0;
      if (A.trace) {
        chi_u = lane63_f64(chi);
        la_u = lane63_f64(la);
      }
      hcache.after(acc);
      gcache.after(acc);
      if constexpr (FAST && NT != 0 && NT <= 64) {
        if (acc && gmask) colcache_accept<NSRC, NT>(ccache, *mdl, gmask, lane, etab);
        ccache.pend = 0;              // parked terms belong to this step only
      }
      wave_sync();
      if (acc && lane == 0) {
        s_acc[r] = s_acc[r] + 1u;
        st[r] = nv;
        if (grp) {
          double *dt = st + (grp == 1 ? WS::OT1 : WS::OT2);
          double *dc = st + (grp == 1 ? WS::OC1 : WS::OC2);
          for (int k = 0; k < 5; ++k) dt[k] = st[WS::OPT + k];
          for (int k = 0; k < 3; ++k) dc[k] = st[WS::OPC + k];
        }
      }
      wave_sync();

      if (A.trace) {
       if (lane == 0) {
        double *t = A.trace + ((size_t)w * A.n_iters + it) * kTraceF;
        t[0] = (double)r;
        t[1] = nv;
        t[2] = chi_u;
        t[3] = dice;
        t[4] = FAST ? (la_u == la_u ? ExpTab{etab}(la_u) : la_u) : exp(la_u);   // p_accept
        t[5] = acc ? 1.0 : 0.0;
       }
      }
      // chain record (:342-351, generalised to a stride)
      if (it == rec_it) {
        if (rec_row >= 0 && rec_row < nrows && lane < PS) chain_w[rec_row * PS + lane] = st[lane];
        rec_it += rstride;
        ++rec_row;
      }
    }

    // ---- write back (the walker index laundered: its per-lane addresses are
    // recomputed here, not kept live across the sampler loop from the loads above)
    wave_sync();
    if (RING && !active) continue;     // (no walker of its own in this batch)
    // (k and w recomputed from u: one SGPR live across the loop instead of three)
    asm volatile("" : "+s"(u));
    k = K()->units > 1 ? u / (int)K()->W : 0;
    w = u - k * (int)K()->W;
    if (lane < PS) st_wt(K()->state + (size_t)w * PS + lane, st[lane]);
    if (lane < NP) {
      st_wt(K()->tries + (size_t)w * NP + lane, s_tries[lane]);
      st_wt(K()->accepts + (size_t)w * NP + lane, s_acc[lane]);
    }
    if (lane == 0) {
      st_wt(K()->mt_pos + w, mt.pos);
      st_wt(K()->has_gauss + w, mt.has_gauss);
      st_wt(K()->gauss + w, mt.gauss);
      st_wt(K()->done_at + w, done_at);
    }
    // hand the walker to the wave that takes its next chunk
    if (k < K()->units - 1) {
      if (k == 0 && K()->hold) hold_handoff(K()->hold, K()->uerr, K()->wait_ticks);
      unit_publish(K()->uflag + w, K()->utag + (unsigned)(k + 1), lane);
    }
    wave_sync();      // the slice is reused by the wave's next walker
    if constexpr (!RING) u = K()->queue ? take() : INT_MAX;
  }
  // ring sampler: the DMAs of the phases after the last one land before the workgroup's
  // LDS is released
  if constexpr (RING) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ---------------------------------------------------------------------------------
// Model / chi^2 of explicit parameter vectors (one wave per vector; image in global)
// ---------------------------------------------------------------------------------
template <int NSRC, bool WRITE>
__global__ __launch_bounds__(256) void olpe_eval_kernel(const double2 *DE, int n, int bkgd_mode,
                                                        int fast, const double *params, int W,
                                                        double *out) {
  using L = Layout<NSRC>;
  constexpr int PS = L::PS;
  extern __shared__ __align__(16) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  double *etab = reinterpret_cast<double *>(smem);
  double *vtab =
      reinterpret_cast<double *>(smem + kEtabBytes + (size_t)wave * vtab_bytes(n, NSRC));
  if (threadIdx.x < 64) etab[threadIdx.x] = c_exp2_64[threadIdx.x];
  __syncthreads();
  const long long w = (long long)blockIdx.x * (blockDim.x / 64) + wave;
  if (w >= W) return;
  double p[PS];
#pragma unroll
  for (int k = 0; k < PS; ++k) p[k] = uniform_f64(params[w * PS + k]);
  auto q = [&](int k) -> double { return p[k]; };
  double *o = WRITE ? out + (size_t)w * n * n : nullptr;
  double part;
  if (fast) {
    const Trig T1 = make_trig<true>(p[L::T1]), T2 = make_trig<true>(p[L::T2]);
    const ModelDesc<NSRC> md = make_model<NSRC>(
        q, make_coef<true>(p[L::S1X], p[L::S1Y], T1), make_coef<true>(p[L::S2X], p[L::S2Y], T2),
        bkgd_mode);
    part = sweep<NSRC, 0, WRITE, true>(md, DE, vtab, o, n, lane, etab);
  } else {
    const Trig T1 = make_trig<false>(p[L::T1]), T2 = make_trig<false>(p[L::T2]);
    const ModelDesc<NSRC> md = make_model<NSRC>(
        q, make_coef<false>(p[L::S1X], p[L::S1Y], T1),
        make_coef<false>(p[L::S2X], p[L::S2Y], T2), bkgd_mode);
    part = sweep<NSRC, 0, WRITE, false>(md, DE, vtab, o, n, lane, etab);
  }
  if constexpr (!WRITE) {
    const double chi = wave_sum(part);
    if (lane == 0) out[w] = chi;
  }
}

__global__ void olpe_seed_kernel(const uint32_t *seeds, int W, uint32_t *mt, int *pos,
                                 int *has_gauss, double *gauss) {
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= W) return;
  mt_seed_serial(mt + (size_t)w * MT_N, seeds[w]);
  pos[w] = MT_N;
  has_gauss[w] = 0;
  gauss[w] = 0.0;
}

// RNG stream dump: one wave per walker, same draw path as the sampler.
template <int NP>
__global__ __launch_bounds__(64) void olpe_stream_kernel(uint32_t *mtg, int *posg,
                                                         int *hasg, double *gg, int W,
                                                         int kind, int nd, void *out) {
  const int lane = threadIdx.x;
  const int w = blockIdx.x;
  if (w >= W) return;
  __shared__ double drawtab[kDrawTab];
  MTWave mt;
  mt.tab = drawtab;
  mt.key = mtg + (size_t)w * MT_N;
  mt.pos = __builtin_amdgcn_readfirstlane(posg[w]);
  mt.bstart = mt.pos;
  mt.bsize = 0;
  mt.batch = 0;
  mt.has_gauss = __builtin_amdgcn_readfirstlane(hasg[w]);
  mt.gauss = uniform_f64(gg[w]);
  for (int i = 0; i < nd; ++i) {
    if (kind == 0) {
      const uint32_t v = mt.next(lane);
      if (lane == 0) reinterpret_cast<uint32_t *>(out)[(size_t)w * nd + i] = v;
    } else {
      // the sampler's draw path, one stage at a time
      int r = 0, di = 0;
      double v = 0.0;
      const int stage = kind == 1 ? 2 : kind == 2 ? 1 : 0;
      mt.template draw<NP>(lane, stage, stage, r, v, di);
      if (kind == 1) v = drawtab[di];
      else if (kind == 3) v = (double)r;
      if (lane == 0) reinterpret_cast<double *>(out)[(size_t)w * nd + i] = v;
    }
  }
  if (lane == 0) {
    posg[w] = mt.pos;
    hasg[w] = mt.has_gauss;
    gg[w] = mt.gauss;
  }
}

}  // namespace

// =================================================================================
// Host side
// =================================================================================
namespace olpe {

thread_local char g_err[512] = "";

int set_err(int code, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

}  // namespace olpe

#define HIPCHK(expr)                                                                \
  do {                                                                              \
    hipError_t e_ = (expr);                                                         \
    if (e_ != hipSuccess)                                                           \
      return set_err(OLPE_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_));     \
  } while (0)

namespace {

template <class T> int dev_alloc(T **p, size_t count) {
  if (*p) {
    (void)hipFree(*p);
    *p = nullptr;
  }
  if (count == 0) return OLPE_OK;
  hipError_t e = hipMalloc((void **)p, count * sizeof(T));
  if (e != hipSuccess) {
    *p = nullptr;
    return set_err(OLPE_ENOMEM, "hipMalloc(%zu bytes): %s", count * sizeof(T),
                   hipGetErrorString(e));
  }
  return OLPE_OK;
}

// per-wave LDS of the kernel launch_gibbs_m picks: NT = n for LDS images of 32 and 64
// pixels, otherwise NT = 0 / 128 (no extra draw-table bytes)
size_t wave_lds(int n, int np, bool lds_img, bool ring = false, int wpb = 12,
                bool fast = false) {
  if (ring) return (size_t)(np == 16 ? ring_wave_bytes<16>(n) : ring_wave_bytes<19>(n));
  const int nt = lds_img && (n == 32 || n == 64) ? n : 0;
  return (size_t)(np == 16 ? WaveSlice<16>::BYTES : WaveSlice<19>::BYTES) +
         drawtab_extra(nt, fast) + sampler_vtab_bytes(n, np == 16 ? 2 : 3, nt, wpb, fast);
}

// Chunks per walker of one launch.  A launch runs W walker chains of n_iters
// iterations on `slots` resident waves.  With whole walkers as the queue's units, W
// just above a multiple of the slots leaves most slots idle for the last walker's
// whole launch (configs[1]: 4,096 walkers on 3,072 slots take two walker-times instead
// of 1 1/3).  Cutting every chain into P consecutive chunks (chunk-major queue order,
// a chunk handed between waves through HBM, unit_wait/unit_publish) lets the queue fill
// the slots; a chain still runs its chunks in order, so a launch takes at least one
// chain's time.  Modelled time, in iterations, with s0 iterations' worth of per-chunk
// setup (state and counter loads, cache setup, the hand-off):
//   T(P) = max(ceil(W P / slots) (n_iters / P + s0), n_iters + P s0)
// P > 1 is taken only when it beats P = 1 by more than 3 %.  override > 0 forces P
// (OLPE_UNITS, tests and A/B).
int choose_units(long long W, long long slots, long long n_iters, int override_p) {
  const int pmax = 15;                 // the chunk index lives in 4 bits of the tag
  auto ok = [&](int p) { return p <= pmax && p <= n_iters && W * p < 0x7fffffffLL; };
  if (override_p > 0) {
    int p = override_p;
    while (p > 1 && !ok(p)) --p;
    return p;
  }
  if (n_iters < 16 || slots <= 0 || W <= 0) return 1;
  const double s0 = 2.0;
  auto T = [&](int p) {
    const double rounds = (double)((W * p + slots - 1) / slots);
    return std::max(rounds * ((double)n_iters / p + s0), (double)n_iters + p * s0);
  };
  int best = 1;
  double tb = T(1);
  for (int p = 2; p <= 8; ++p) {
    if (!ok(p) || n_iters / p < 8) break;
    const double t = T(p);
    if (t < tb) {
      tb = t;
      best = p;
    }
  }
  return tb < 0.97 * T(1) ? best : 1;
}

size_t lds_bytes(const olpe_ctx *c, int wpb, bool ring = false) {
  size_t b = (size_t)wpb * wave_lds(c->n, c->np, c->lds_img, ring, wpb,
                                    c->eval_mode == OLPE_EVAL_FAST) + kSampHdr;
  if (c->lds_img) b += (size_t)c->n * c->n * sizeof(double2);
  if (ring) b += wpb >= 12 ? LdsRing<12>::BYTES : LdsRing<8>::BYTES;
  return b;
}


template <int NSRC, int NT, bool LDS, int WPB, bool FAST>
int launch_gibbs_t(olpe_ctx *c, const GibbsArgs &a) {
  constexpr bool RING = !LDS && FAST && ring_wpb(NT, WPB);    // (olpe_gibbs_kernel)
  const size_t shm = lds_bytes(c, WPB, RING);
  auto k = olpe_gibbs_kernel<NSRC, NT, LDS, WPB, FAST>;
  // the dynamic-LDS limit is a per-device function attribute: set once per device
  // (contexts on several GPUs may launch from different host threads)
  static std::atomic<uint64_t> attr_set{0};
  const uint64_t bit = 1ull << (c->device & 63);
  if (!(attr_set.load(std::memory_order_acquire) & bit)) {
    HIPCHK(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                               160 * 1024));
    attr_set.fetch_or(bit, std::memory_order_release);
  }
  unsigned blocks = (unsigned)((a.W + WPB - 1) / WPB);
  GibbsArgs q = a;
  q.queue = nullptr;
  q.qbase = 0;
  q.units = 1;
  q.uflag = c->d_uflag;
  q.utag = 0;
  q.uerr = reinterpret_cast<unsigned *>(c->d_queue + 1);
  q.stagger = c->stagger;
  q.hold = nullptr;
  int per_cu = 0;
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, WPB * 64, shm));
  const unsigned resident = (unsigned)std::max(1, per_cu) * (unsigned)c->n_cu;
  // (ring sampler: a batch's 12 units run in lockstep, so a chunk must never wait on its
  // predecessor inside its own batch -- the predecessor of unit u is u - W, in an earlier
  // batch whenever W >= 12; fewer walkers run whole)
  const int units = c->queue_on && c->d_queue && c->d_uflag && !(RING && a.W < WPB)
                        ? choose_units(a.W, (long long)resident * WPB, a.n_iters, c->units_override)
                        : 1;
  // the LDS sampler always runs persistent; the L2-resident one only when it cuts the
  // walkers into chunks (with whole walkers the hardware's workgroup dispatch is as good);
  // the ring sampler always (launch_gibbs_m picks it only with the queue on)
  if (c->queue_on && c->d_queue && (LDS || RING || units > 1)) {
    // persistent grid: as many workgroups as fit on the device at once, the work
    // units handed out by the queue
    if (blocks > resident) blocks = resident;
    q.queue = c->d_queue;
    q.qbase = c->qbase;
    q.units = units;
    c->utag += 16;
    q.utag = c->utag;
    if (c->hold_handoff && units > 1) {
      // test hook: one workgroup more than the first chunks need, so that some wave's
      // first unit is a later chunk whose predecessor is held -- it must wait, and its
      // wait releases the hold.  Every workgroup must be resident for that.
      const unsigned need = (unsigned)((a.W + WPB - 1) / WPB) + 1;
      if (need > resident)
        return set_err(OLPE_EINVAL, "olpe_test_hold_handoff: %lld walkers need %u resident "
                       "workgroups, the device holds %u", a.W, need, resident);
      blocks = need;
      HIPCHK(hipMemsetAsync(c->d_queue + 4, 0, sizeof(unsigned long long), c->stream));
      q.hold = reinterpret_cast<unsigned *>(c->d_queue + 4);
    }
  }
  // progress balancing (olpe_gibbs_kernel): on by default for a 16-wave 2-source FAST
  // launch that runs its walkers whole in one round, which ends on its slowest wave
  // (configs[1]: +2 % over the 12-wave sampler; profiles/r02/ab_w16.log)
  q.balance = c->balance >= 0 ? c->balance
            : (LDS && FAST && NSRC == 2 && WPB == 16 && q.units == 1 &&
               a.W <= (long long)resident * WPB) ? 1 : 0;
  c->last_units = q.units;
  if (q.units > 1) c->units_used = true;
  // a hand-off waits at most for one chunk of the same walker (its predecessor) to run:
  // bound a chunk's time generously -- 8 ns per pixel-Gaussian per iteration, ~30x the
  // slowest sampler (EXACT, 3 sources, 128x128) -- and never below 30 s
  {
    const double chunk = (double)((a.n_iters + q.units - 1) / q.units);
    const double ticks = chunk * (double)a.n * (double)a.n * (2.0 * NSRC) * 0.8;
    q.wait_ticks = c->wait_ticks_override > 0
                       ? (unsigned long long)c->wait_ticks_override
                       : (unsigned long long)std::min(std::max(ticks, 3e9), 1e15);
    c->wait_limit_s = (double)q.wait_ticks * 1e-8;
  }
  hipLaunchKernelGGL(k, dim3(blocks), dim3(WPB * 64), shm, c->stream, q);
  HIPCHK(hipGetLastError());
  // the launch takes W * units + (its waves) values off the counter (the ring sampler:
  // one per batch of WPB units + one per workgroup): the next launch's base (advanced
  // only once the launch is in the stream)
  if (q.queue) {
    const unsigned long long tot = (unsigned long long)a.W * (unsigned long long)q.units;
    c->qbase += RING ? (tot + WPB - 1) / WPB + blocks : tot + (unsigned long long)blocks * WPB;
  }
  return OLPE_OK;
}

template <int NSRC, bool FAST> int launch_gibbs_m(olpe_ctx *c, const GibbsArgs &a) {
  if (c->lds_img) {
    switch (c->n) {
      // 12 waves at 32x32 as well (168 VGPRs: no spills; 3-source +77 %, 2-source +1 %
      // over 16)
      case 32: return launch_gibbs_t<NSRC, 32, true, 12, FAST>(c, a);
      case 64: {
        // 12 waves per workgroup (168 VGPRs: four-row update and shape-table prefetch
        // without spills, 3 waves per SIMD with the walker queue keeping them busy);
        // 16 waves (4 per SIMD: the FP64 issue rate of 4 waves, 4.80 against 5.11
        // cycles per op) for 2 sources: FAST when the launch has walkers for >= 8 rounds
        // of its slots (configs[2]: +1.0-1.4 %) or for one round that the 12-wave
        // sampler cannot hold, run whole with progress balancing (configs[1]'s 4,096:
        // +2 %; one 12-wave round runs on more CUs: 2,048 walkers -12 % at 16 waves; in
        // between the 12-wave sampler's chunked rounds balance better), EXACT
        // always (configs[1]: +19 %, its 4,096 walkers one round of 16-wave slots;
        // configs[2] level; profiles/r02/ab_w16.log).  The FAST layout needs the single
        // shape-table slot (single_h), the EXACT one draw tables without the accept
        // thresholds; 3 sources stay at 12 (their slices do not fit 16)
        const long long r16 = 16LL * c->n_cu, r12 = 12LL * c->n_cu;   // one round
        int wpb = c->wpb ? c->wpb
                : (NSRC == 2 && (!FAST || a.W >= 8 * r16 || (a.W > r12 && a.W <= r16)))
                      ? 16 : 12;
        if (wpb == 16 && lds_bytes(c, 16) > 160 * 1024) wpb = 12;
        if (wpb == 8) return launch_gibbs_t<NSRC, 64, true, 8, FAST>(c, a);
        if (wpb == 12) return launch_gibbs_t<NSRC, 64, true, 12, FAST>(c, a);
        return launch_gibbs_t<NSRC, 64, true, 16, FAST>(c, a);
      }
      default: return launch_gibbs_t<NSRC, 0, true, 16, FAST>(c, a);
    }
  }
  if (c->n == 128) {
    // FAST: the lockstep ring sampler (the cutout streamed through LDS, one 12-wave
    // workgroup per CU); OLPE_RING=0 or no walker queue: the L2-resident one
    if constexpr (FAST) {
      // (two 6-wave workgroups per CU with rings of their own -- their control phases
      // apart -- ran at 0.65x: the dispatcher does not pack two of them on a CU)
      if (c->ring_wpb && c->queue_on && c->d_queue && c->d_uflag) {
        return launch_gibbs_t<NSRC, 128, false, 12, FAST>(c, a);
      }
    }
    return launch_gibbs_t<NSRC, 128, false, 4, FAST>(c, a);
  }
  // large cutouts (a full 1024 x 1024 NIRC2 frame): one wave per workgroup once four
  // waves' row tables (n x 2 NSRC doubles each) no longer fit the LDS; olpe_create
  // rejects sides where even one does not
  if (lds_bytes(c, 4) > 160 * 1024) return launch_gibbs_t<NSRC, 0, false, 1, FAST>(c, a);
  return launch_gibbs_t<NSRC, 0, false, 4, FAST>(c, a);
}

int launch_gibbs(olpe_ctx *c, const GibbsArgs &a) {
  const bool fast = c->eval_mode == OLPE_EVAL_FAST;
  if (c->nsrc == 2) return fast ? launch_gibbs_m<2, true>(c, a) : launch_gibbs_m<2, false>(c, a);
  return fast ? launch_gibbs_m<3, true>(c, a) : launch_gibbs_m<3, false>(c, a);
}

int ensure_ensemble(olpe_ctx *c, int W) {
  if (W <= 0) return set_err(OLPE_EINVAL, "W must be > 0 (got %d)", W);
  if (c->W == W && c->d_state) return OLPE_OK;
  int rc;
  if ((rc = dev_alloc(&c->d_state, (size_t)W * c->ps))) return rc;
  if ((rc = dev_alloc(&c->d_tries, (size_t)W * c->np))) return rc;
  if ((rc = dev_alloc(&c->d_acc, (size_t)W * c->np))) return rc;
  if ((rc = dev_alloc(&c->d_mt, (size_t)W * MT_N))) return rc;
  if ((rc = dev_alloc(&c->d_mtpos, (size_t)W))) return rc;
  if ((rc = dev_alloc(&c->d_gauss, (size_t)W))) return rc;
  if ((rc = dev_alloc(&c->d_hasg, (size_t)W))) return rc;
  if ((rc = dev_alloc(&c->d_done, (size_t)W))) return rc;
  if ((rc = dev_alloc(&c->d_uflag, (size_t)W))) return rc;
  HIPCHK(hipMemsetAsync(c->d_uflag, 0, (size_t)W * sizeof(unsigned), c->stream));
  HIPCHK(hipMemsetAsync(c->d_state, 0, (size_t)W * c->ps * sizeof(double), c->stream));
  HIPCHK(hipMemsetAsync(c->d_tries, 0, (size_t)W * c->np * sizeof(uint32_t), c->stream));
  HIPCHK(hipMemsetAsync(c->d_acc, 0, (size_t)W * c->np * sizeof(uint32_t), c->stream));
  HIPCHK(hipMemsetAsync(c->d_done, 0xff, (size_t)W * sizeof(long long), c->stream));
  c->W = W;
  c->seeded = false;
  c->count = 0;
  c->chain_rows = 0;
  c->mom_n = 0;
  return OLPE_OK;
}

}  // namespace

extern "C" {

int olpe_version(void) { return 101; }


const char *olpe_last_error(void) { return g_err; }

int olpe_device_count(int *count) {
  if (!count) return set_err(OLPE_EINVAL, "count is NULL");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  *count = (e == hipSuccess) ? n : 0;
  return OLPE_OK;
}

int olpe_device_pci_id(int device, char *buf, int len) {
  if (!buf || len < 16) return set_err(OLPE_EINVAL, "buffer of at least 16 bytes needed");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return set_err(OLPE_EHIP, "no HIP device visible");
  if (device < 0 || device >= ndev) return set_err(OLPE_EINVAL, "bad device %d", device);
  HIPCHK(hipDeviceGetPCIBusId(buf, len, device));
  return OLPE_OK;
}

int olpe_device_mem(int device, long long *free_bytes, long long *total_bytes) {
  if (!free_bytes || !total_bytes) return set_err(OLPE_EINVAL, "NULL argument");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return set_err(OLPE_EHIP, "no HIP device visible");
  if (device < 0 || device >= ndev) return set_err(OLPE_EINVAL, "bad device %d", device);
  HIPCHK(hipSetDevice(device));
  size_t f = 0, t = 0;
  HIPCHK(hipMemGetInfo(&f, &t));
  *free_bytes = (long long)f;
  *total_bytes = (long long)t;
  return OLPE_OK;
}

int olpe_create(const void *image, int image_dtype, const void *pois2, double readnoise2,
                const uint8_t *mask, int ny, int nx, int nsrc, int bkgd_mode, int device,
                olpe_ctx **out) {
  if (!out) return set_err(OLPE_EINVAL, "out is NULL");
  *out = nullptr;
  if (!image || !pois2) return set_err(OLPE_EINVAL, "image/pois2 is NULL");
  if (ny <= 0 || nx <= 0) return set_err(OLPE_EINVAL, "bad shape %dx%d", ny, nx);
  if (ny != nx)
    return set_err(OLPE_EINVAL,
                   "non-square image %dx%d: the reference model is square-only "
                   "(apf_step2.py:237, :119-123)", ny, nx);
  if (nx > 4096) return set_err(OLPE_EINVAL, "image too large (%d)", nx);
  if (nsrc != 2 && nsrc != 3) return set_err(OLPE_EINVAL, "nsrc must be 2 or 3");
  {
    // the largest sampler workgroup is one wave with its row tables (n x 2 nsrc doubles)
    // and wave slice in the 160 KiB of LDS: sides up to ~5,000 with 2 sources (the 4,096
    // cap comes first) and ~3,380 with 3
    const size_t one = wave_lds(nx, nsrc == 2 ? 16 : 19, false) + kSampHdr;
    if (one > 160 * 1024)
      return set_err(OLPE_EINVAL, "%dx%d cutout: its row tables need %zu bytes of LDS per "
                     "wave, more than the 163840 a workgroup has (cut the frame to the stars)",
                     nx, nx, one);
  }
  if (image_dtype != OLPE_DTYPE_F32 && image_dtype != OLPE_DTYPE_F64)
    return set_err(OLPE_EINVAL, "image_dtype must be OLPE_DTYPE_F32/F64");
  if (bkgd_mode != 0 && bkgd_mode != 1) return set_err(OLPE_EINVAL, "bkgd_mode must be 0/1");
  if (device < 0) return set_err(OLPE_EINVAL, "device must be a HIP ordinal (no CPU path)");
  // stage image + 1/err in LDS when it fits beside a workgroup's wave slices (12 waves
  // at 32x32 and 64x64, 16 for other sides; launch_gibbs_m)
  const int np_ = nsrc == 2 ? 16 : 19;
  const size_t npix_ = (size_t)nx * nx;
  const bool lds_img = npix_ * sizeof(double2) +
                           ((nx == 64 || nx == 32) ? 12 : 16) * wave_lds(nx, np_, true) +
                           kSampHdr <= 160 * 1024;
  int wpb = 0;
  if (const char *e = getenv("OLPE_WPB")) {                  // tuning experiments
    // only the 64x64 LDS sampler has a choice (8 / 12 / 16 waves); its layout must fit
    // the 160 KiB of LDS beside the cutout, or the launch would fail
    wpb = atoi(e);
    if (wpb != 8 && wpb != 12 && wpb != 16)
      return set_err(OLPE_EINVAL, "OLPE_WPB=%s: must be 8, 12 or 16", e);
    const size_t b = (size_t)wpb * wave_lds(nx, np_, true, false, wpb, true) + kSampHdr +
                     npix_ * sizeof(double2);
    if (lds_img && nx == 64 && b > 160 * 1024)
      return set_err(OLPE_EINVAL, "OLPE_WPB=%d needs %zu bytes of LDS at %dx%d (%d sources) > 163840",
                     wpb, b, nx, nx, nsrc);
    if (!(lds_img && nx == 64)) wpb = 0;     // no choice at other sides
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return set_err(OLPE_EHIP, "no HIP device visible");
  if (device >= ndev) return set_err(OLPE_EINVAL, "device %d >= device count %d", device, ndev);
  HIPCHK(hipSetDevice(device));

  olpe_ctx *c = new olpe_ctx();
  c->device = device;
  c->n = nx;
  c->nsrc = nsrc;
  c->bkgd_mode = bkgd_mode;
  c->np = nsrc == 2 ? 16 : 19;
  c->ps = c->np + 1;
  const size_t npix = (size_t)nx * nx;
  // stage image + 1/err in LDS when it fits beside a workgroup's wave slices (12 waves
  // at 32x32 and 64x64, 16 for other sides; launch_gibbs_m)
  c->lds_img = lds_img;
  c->wpb = wpb;
  std::vector<double2> hDE(npix), hDW(npix);
  for (size_t i = 0; i < npix; ++i) {
    const double d = image_dtype == OLPE_DTYPE_F32 ? (double)((const float *)image)[i]
                                                   : ((const double *)image)[i];
    const double p2 = image_dtype == OLPE_DTYPE_F32 ? (double)((const float *)pois2)[i]
                                                    : ((const double *)pois2)[i];
    const double e = sqrt(readnoise2 + p2);   // apf_step2.py:210
    // the reference's np.ma chi_squared (:134-137) drops a pixel whose quotient
    // (D - M) / err is non-finite or whose err is 0 (np.ma.divide's domain): a NaN or
    // -inf data pixel, or an err that is NaN or 0 (+inf data is above the saturation
    // mask of :188 already).  Staged {0, 0}, such a pixel adds nothing to chi^2.
    if ((mask && mask[i]) || !std::isfinite(d) || !(e > 0.0)) {
      hDE[i] = make_double2(0.0, 0.0);
      hDW[i] = make_double2(0.0, 0.0);
    } else {
      hDE[i] = make_double2(d, 1.0 / e);
      hDW[i] = make_double2(d * (1.0 / e), 1.0 / e);
    }
  }
  // an all-masked cutout: the reference's masked sum is np.ma.masked, which :289 stores
  // as NaN and :144 never accepts (bool(masked) is False); one NaN pixel gives every chi^2
  // that NaN (an empty sum here would be 0 and accept every proposal)
  bool any_pixel = false;
  for (size_t i = 0; i < npix && !any_pixel; ++i) any_pixel = hDE[i].y != 0.0;
  if (!any_pixel) {
    hDE[0] = make_double2(NAN, NAN);
    hDW[0] = make_double2(NAN, NAN);
  }
  int rc;
  hipError_t e1 = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e1 != hipSuccess) {
    delete c;
    return set_err(OLPE_EHIP, "hipStreamCreate: %s", hipGetErrorString(e1));
  }
  for (auto &pair : c->ev)
    for (auto &ev : pair)
      if (hipEventCreate(&ev) != hipSuccess) ev = nullptr;
  // the collectives' words (olpe_comm_setup), allocated here so that olpe_comm_init has
  // nothing to allocate that could fail on one rank while the others wait for it
  if ((rc = dev_alloc(&c->d_DE, npix)) || (rc = dev_alloc(&c->d_DW, npix)) ||
      (rc = dev_alloc(&c->d_queue, 5)) || (rc = olpe_comm_setup(c))) {
    olpe_destroy(c);
    return rc;
  }
  // [0] the queue counter, [1] the hand-off error word, [2..3] hand-off statistics
  // (unit_wait), [4] the hand-off hold word (olpe_test_hold_handoff)
  if (hipMemset(c->d_queue, 0, 5 * sizeof(unsigned long long)) != hipSuccess ||
      hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device) !=
          hipSuccess || c->n_cu <= 0) {
    olpe_destroy(c);
    return set_err(OLPE_EHIP, "walker queue setup failed");
  }
  if (const char *e = getenv("OLPE_NO_QUEUE")) c->queue_on = atoi(e) == 0;  // A/B only
  if (const char *e = getenv("OLPE_UNITS")) {                                // tests, A/B
    const int p = atoi(e);
    if (p < 0 || p > 15) {
      olpe_destroy(c);
      return set_err(OLPE_EINVAL, "OLPE_UNITS=%s: must be 0 (automatic) .. 15", e);
    }
    c->units_override = p;
  }
  if (const char *e = getenv("OLPE_RING")) {                                // A/B, tests
    const int v = atoi(e);
    if (v != 0 && v != 12) {
      olpe_destroy(c);
      return set_err(OLPE_EINVAL, "OLPE_RING=%s: must be 0 (off) or 12 (waves per workgroup)", e);
    }
    c->ring_wpb = v;
  }
  // tests only: the hand-off wait limit in 100 MHz ticks instead of the launch's bound
  if (const char *e = getenv("OLPE_WAIT_TICKS")) c->wait_ticks_override = std::max(0.0, atof(e));
  hipError_t e2 = hipMemcpy(c->d_DE, hDE.data(), npix * sizeof(double2), hipMemcpyHostToDevice);
  if (e2 == hipSuccess)
    e2 = hipMemcpy(c->d_DW, hDW.data(), npix * sizeof(double2), hipMemcpyHostToDevice);
  if (e2 != hipSuccess) {
    olpe_destroy(c);
    return set_err(OLPE_EHIP, "hipMemcpy image: %s", hipGetErrorString(e2));
  }
  *out = c;
  return OLPE_OK;
}

void olpe_destroy(olpe_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  olpe_comm_release(c);
  void *ptrs[] = {c->d_DE, c->d_DW, c->d_state, c->d_tries, c->d_acc,
                  c->d_mt, c->d_mtpos, c->d_gauss, c->d_hasg,  c->d_done,
                  c->d_chain, c->d_trace, c->d_scratch, c->d_scratch2, c->d_queue,
                  c->d_gather, c->d_uflag, c->d_mmean, c->d_mm2, c->d_mpart, c->d_check};
  for (void *p : ptrs)
    if (p) (void)hipFree(p);
  for (auto &pair : c->ev)
    for (auto &ev : pair)
      if (ev) (void)hipEventDestroy(ev);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int olpe_set_eval_mode(olpe_ctx *c, int mode) {
  if (!c) return set_err(OLPE_EINVAL, "ctx is NULL");
  if (mode != OLPE_EVAL_EXACT && mode != OLPE_EVAL_FAST)
    return set_err(OLPE_EINVAL, "unknown eval mode %d", mode);
  c->eval_mode = mode;
  return OLPE_OK;
}

static int eval_batch(olpe_ctx *c, const double *params, int W, double *out, bool write) {
  if (!c || !params || !out) return set_err(OLPE_EINVAL, "NULL argument");
  if (W <= 0) return set_err(OLPE_EINVAL, "W must be > 0");
  HIPCHK(hipSetDevice(c->device));
  const size_t pin = (size_t)W * c->ps;
  const size_t pout = write ? (size_t)W * c->n * c->n : (size_t)W;
  int rc;
  if (c->scratch_cap < pin && (rc = dev_alloc(&c->d_scratch, pin))) return rc;
  if (c->scratch_cap < pin) c->scratch_cap = pin;
  if (c->scratch2_cap < pout && (rc = dev_alloc(&c->d_scratch2, pout))) return rc;
  if (c->scratch2_cap < pout) c->scratch2_cap = pout;
  HIPCHK(hipMemcpyAsync(c->d_scratch, params, pin * 8, hipMemcpyHostToDevice, c->stream));
  // four vectors per workgroup, fewer where their row tables would not fit the LDS
  int wpb = 4;
  while (wpb > 1 && (size_t)wpb * vtab_bytes(c->n, c->nsrc) + kEtabBytes > 160 * 1024) wpb /= 2;
  dim3 grid((W + wpb - 1) / wpb), block(wpb * 64);
  const size_t shm = (size_t)wpb * vtab_bytes(c->n, c->nsrc) + kEtabBytes;
  const int fast = c->eval_mode == OLPE_EVAL_FAST;
  if (shm > 160 * 1024) return set_err(OLPE_EINVAL, "image too large for the eval kernel");
  if (shm > 65536) {
    // per device, like the sampler's (launch_gibbs_t): the device's bit is set only
    // after every kernel's attribute is, with this context's device current, so a
    // failed set is retried and no caller launches before it took effect
    static std::atomic<uint64_t> eval_attr{0};
    const uint64_t bit = 1ull << (c->device & 63);
    if (!(eval_attr.load(std::memory_order_acquire) & bit)) {
      const void *ks[4] = {(const void *)olpe_eval_kernel<2, true>,
                           (const void *)olpe_eval_kernel<2, false>,
                           (const void *)olpe_eval_kernel<3, true>,
                           (const void *)olpe_eval_kernel<3, false>};
      for (const void *k : ks)
        HIPCHK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      eval_attr.fetch_or(bit, std::memory_order_release);
    }
  }
  if (c->nsrc == 2) {
    if (write)
      hipLaunchKernelGGL((olpe_eval_kernel<2, true>), grid, block, shm, c->stream, fast ? c->d_DW : c->d_DE,
                         c->n, c->bkgd_mode, fast, c->d_scratch, W, c->d_scratch2);
    else
      hipLaunchKernelGGL((olpe_eval_kernel<2, false>), grid, block, shm, c->stream, fast ? c->d_DW : c->d_DE,
                         c->n, c->bkgd_mode, fast, c->d_scratch, W, c->d_scratch2);
  } else {
    if (write)
      hipLaunchKernelGGL((olpe_eval_kernel<3, true>), grid, block, shm, c->stream, fast ? c->d_DW : c->d_DE,
                         c->n, c->bkgd_mode, fast, c->d_scratch, W, c->d_scratch2);
    else
      hipLaunchKernelGGL((olpe_eval_kernel<3, false>), grid, block, shm, c->stream, fast ? c->d_DW : c->d_DE,
                         c->n, c->bkgd_mode, fast, c->d_scratch, W, c->d_scratch2);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, c->d_scratch2, pout * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return OLPE_OK;
}

int olpe_model(olpe_ctx *c, const double *params, double *model_out) {
  return eval_batch(c, params, 1, model_out, true);
}

int olpe_chi2_batch(olpe_ctx *c, const double *params, int W, double *chi2_out) {
  return eval_batch(c, params, W, chi2_out, false);
}

int olpe_seed(olpe_ctx *c, const uint32_t *seeds, int W) {
  if (!c || !seeds) return set_err(OLPE_EINVAL, "NULL argument");
  HIPCHK(hipSetDevice(c->device));
  int rc;
  if ((rc = ensure_ensemble(c, W))) return rc;
  uint32_t *ds = nullptr;
  if ((rc = dev_alloc(&ds, (size_t)W))) return rc;
  HIPCHK(hipMemcpyAsync(ds, seeds, (size_t)W * 4, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(olpe_seed_kernel, dim3((W + 255) / 256), dim3(256), 0, c->stream, ds, W,
                     c->d_mt, c->d_mtpos, c->d_hasg, c->d_gauss);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  (void)hipFree(ds);
  c->seeded = true;
  c->mom_n = 0;                  // a new run: no rows folded into the moments yet
  c->mom_folded = c->launches;
  return OLPE_OK;
}

// the hand-off error word of the work-unit queue (unit_wait): a wait that timed out
// means a chunk may have run from a stale state -- reported, never silently used
static int check_units(olpe_ctx *c) {
  if (!c->d_queue || !c->units_used) return OLPE_OK;   // (the word is sticky)
  unsigned long long e = 0;
  HIPCHK(hipMemcpy(&e, c->d_queue + 1, sizeof(e), hipMemcpyDeviceToHost));
  if (e)
    return set_err(OLPE_EHIP, "sampler chunk hand-off timed out (%.0f s): results invalid",
                   c->wait_limit_s);
  return OLPE_OK;
}

static int counters_to_dev(olpe_ctx *c, const double *h, uint32_t *d) {
  const size_t m = (size_t)c->W * c->np;
  std::vector<uint32_t> t(m, 0u);
  if (h)
    for (size_t i = 0; i < m; ++i) {
      if (!(h[i] >= 0.0) || h[i] > 4294967295.0)
        return set_err(OLPE_EINVAL, "counter %zu out of range (%g)", i, h[i]);
      t[i] = (uint32_t)h[i];
    }
  HIPCHK(hipMemcpyAsync(d, t.data(), m * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return OLPE_OK;
}

static int counters_to_host(olpe_ctx *c, const uint32_t *d, double *h) {
  const size_t m = (size_t)c->W * c->np;
  std::vector<uint32_t> t(m);
  HIPCHK(hipMemcpy(t.data(), d, m * 4, hipMemcpyDeviceToHost));
  for (size_t i = 0; i < m; ++i) h[i] = (double)t[i];
  return OLPE_OK;
}

int olpe_state_set(olpe_ctx *c, const double *state, const double *tries,
                   const double *accepts) {
  if (!c || !state) return set_err(OLPE_EINVAL, "NULL argument");
  if (!c->d_state) return set_err(OLPE_ESTATE, "call olpe_seed first");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipMemcpyAsync(c->d_state, state, (size_t)c->W * c->ps * 8, hipMemcpyHostToDevice,
                        c->stream));
  int rc;
  if ((rc = counters_to_dev(c, tries, c->d_tries))) return rc;
  if ((rc = counters_to_dev(c, accepts, c->d_acc))) return rc;
  HIPCHK(hipMemsetAsync(c->d_done, 0xff, (size_t)c->W * sizeof(long long), c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return OLPE_OK;
}

int olpe_state_get(olpe_ctx *c, double *state, double *tries, double *accepts) {
  if (!c) return set_err(OLPE_EINVAL, "NULL ctx");
  if (!c->d_state) return set_err(OLPE_ESTATE, "no ensemble");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (state)
    HIPCHK(hipMemcpy(state, c->d_state, (size_t)c->W * c->ps * 8, hipMemcpyDeviceToHost));
  int rc;
  if (tries && (rc = counters_to_host(c, c->d_tries, tries))) return rc;
  if (accepts && (rc = counters_to_host(c, c->d_acc, accepts))) return rc;
  return check_units(c);
}

int olpe_run(olpe_ctx *c, long long n_iters, long long burn_in, int record_stride,
             long long accept_min, long long *nrec_out) {
  if (!c) return set_err(OLPE_EINVAL, "NULL ctx");
  if (!c->d_state || !c->seeded) return set_err(OLPE_ESTATE, "call olpe_seed first");
  if (n_iters < 0 || burn_in < 0 || record_stride < 0 || accept_min < 0)
    return set_err(OLPE_EINVAL, "negative argument");
  if (n_iters > 0x7fffffffLL)
    return set_err(OLPE_EINVAL, "n_iters per launch must be < 2^31 (split the run)");
  HIPCHK(hipSetDevice(c->device));
  // rows recorded in (count0, count0 + n_iters]
  long long row0 = 0, nrows = 0;
  const long long c0 = c->count, c1 = c->count + n_iters;
  if (record_stride > 0 && c1 >= burn_in) {
    const long long s = record_stride;
    const long long lo = std::max(c0 + 1, burn_in);
    const long long first = (lo - burn_in + s - 1) / s;   // first row index >= lo
    const long long last = (c1 - burn_in) / s;            // last row index <= c1
    if (last >= first) {
      row0 = first;
      nrows = last - first + 1;
    }
  }
  int rc;
  const size_t chain_need = (size_t)c->W * nrows * c->ps;
  if (chain_need > c->chain_cap) {
    if ((rc = dev_alloc(&c->d_chain, chain_need))) return rc;
    c->chain_cap = chain_need;
  }
  c->chain_rows = nrows;
  const size_t trace_need = c->trace_on ? (size_t)c->W * n_iters * kTraceF : 0;
  if (trace_need > c->trace_cap) {
    if ((rc = dev_alloc(&c->d_trace, trace_need))) return rc;
    c->trace_cap = trace_need;
  }
  c->trace_iters = c->trace_on ? n_iters : 0;

  GibbsArgs a;
  a.DE = c->eval_mode == OLPE_EVAL_FAST ? c->d_DW : c->d_DE;
  a.n = c->n;
  a.bkgd_mode = c->bkgd_mode;
  a.W = c->W;
  a.state = c->d_state;
  a.tries = c->d_tries;
  a.accepts = c->d_acc;
  a.mt = c->d_mt;
  a.mt_pos = c->d_mtpos;
  a.gauss = c->d_gauss;
  a.has_gauss = c->d_hasg;
  a.done_at = c->d_done;
  a.n_iters = n_iters;
  a.count0 = c0;
  a.burn_in = burn_in;
  a.stride = nrows > 0 ? record_stride : 0;
  a.row0 = row0;
  a.nrows = nrows;
  a.chain = c->d_chain;
  a.accept_min = accept_min;
  a.trace = c->trace_on ? c->d_trace : nullptr;
  hipEvent_t *ev = c->ev[c->launches % olpe_ctx::kRing];
  if (!ev[0] || !ev[1]) return set_err(OLPE_EHIP, "launch events were not created");
  HIPCHK(hipEventRecord(ev[0], c->stream));
  if ((rc = launch_gibbs(c, a))) return rc;
  HIPCHK(hipEventRecord(ev[1], c->stream));
  ++c->launches;
  c->count = c1;
  if (nrec_out) *nrec_out = nrows;
  return OLPE_OK;
}

int olpe_chain_read(olpe_ctx *c, double *chain_out) {
  if (!c || !chain_out) return set_err(OLPE_EINVAL, "NULL argument");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  const size_t m = (size_t)c->W * c->chain_rows * c->ps;
  if (m) HIPCHK(hipMemcpy(chain_out, c->d_chain, m * 8, hipMemcpyDeviceToHost));
  return check_units(c);
}

int olpe_count(olpe_ctx *c, long long *count) {
  if (!c || !count) return set_err(OLPE_EINVAL, "NULL argument");
  *count = c->count;
  return OLPE_OK;
}

int olpe_count_reset(olpe_ctx *c, long long count) {
  if (!c || count < 0) return set_err(OLPE_EINVAL, "bad argument");
  c->count = count;
  return OLPE_OK;
}

int olpe_done_at(olpe_ctx *c, long long *done_at) {
  if (!c || !done_at) return set_err(OLPE_EINVAL, "NULL argument");
  if (!c->d_done) return set_err(OLPE_ESTATE, "no ensemble");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipMemcpy(done_at, c->d_done, (size_t)c->W * 8, hipMemcpyDeviceToHost));
  return check_units(c);
}

int olpe_run_gibbs(olpe_ctx *c, double *state, double *tries, double *accepts, int W,
                   long long n_iters, long long burn_in, int record_stride,
                   double *chain_out) {
  if (!c || !state) return set_err(OLPE_EINVAL, "NULL argument");
  if (!c->seeded || c->W != W)
    return set_err(OLPE_ESTATE, "seed %d walkers with olpe_seed first", W);
  int rc;
  if ((rc = olpe_state_set(c, state, tries, accepts))) return rc;
  c->count = 0;
  if ((rc = olpe_run(c, n_iters, burn_in, record_stride, 0, nullptr))) return rc;
  if ((rc = olpe_state_get(c, state, tries, accepts))) return rc;
  if (chain_out && (rc = olpe_chain_read(c, chain_out))) return rc;
  return OLPE_OK;
}

int olpe_rng_get(olpe_ctx *c, uint32_t *mt_state, double *gauss_cache) {
  if (!c) return set_err(OLPE_EINVAL, "NULL ctx");
  if (!c->d_mt) return set_err(OLPE_ESTATE, "no ensemble");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  const int W = c->W;
  if (mt_state) {
    std::vector<uint32_t> key((size_t)W * MT_N);
    std::vector<int> pos(W);
    HIPCHK(hipMemcpy(key.data(), c->d_mt, key.size() * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(pos.data(), c->d_mtpos, (size_t)W * 4, hipMemcpyDeviceToHost));
    for (int w = 0; w < W; ++w) {
      memcpy(mt_state + (size_t)w * (MT_N + 1), key.data() + (size_t)w * MT_N, MT_N * 4);
      mt_state[(size_t)w * (MT_N + 1) + MT_N] = (uint32_t)pos[w];
    }
  }
  if (gauss_cache) {
    std::vector<int> h(W);
    std::vector<double> g(W);
    HIPCHK(hipMemcpy(h.data(), c->d_hasg, (size_t)W * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(g.data(), c->d_gauss, (size_t)W * 8, hipMemcpyDeviceToHost));
    for (int w = 0; w < W; ++w) {
      gauss_cache[2 * w] = h[w];
      gauss_cache[2 * w + 1] = g[w];
    }
  }
  return OLPE_OK;
}

int olpe_rng_set(olpe_ctx *c, const uint32_t *mt_state, const double *gauss_cache) {
  if (!c || !mt_state || !gauss_cache) return set_err(OLPE_EINVAL, "NULL argument");
  if (!c->d_mt) return set_err(OLPE_ESTATE, "no ensemble (call olpe_seed)");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  const int W = c->W;
  std::vector<uint32_t> key((size_t)W * MT_N);
  std::vector<int> pos(W), h(W);
  std::vector<double> g(W);
  for (int w = 0; w < W; ++w) {
    memcpy(key.data() + (size_t)w * MT_N, mt_state + (size_t)w * (MT_N + 1), MT_N * 4);
    pos[w] = (int)mt_state[(size_t)w * (MT_N + 1) + MT_N];
    if (pos[w] < 0 || pos[w] > MT_N) return set_err(OLPE_EINVAL, "bad MT position");
    h[w] = gauss_cache[2 * w] != 0.0;
    g[w] = gauss_cache[2 * w + 1];
  }
  HIPCHK(hipMemcpy(c->d_mt, key.data(), key.size() * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(c->d_mtpos, pos.data(), (size_t)W * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(c->d_hasg, h.data(), (size_t)W * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(c->d_gauss, g.data(), (size_t)W * 8, hipMemcpyHostToDevice));
  c->seeded = true;
  return OLPE_OK;
}

int olpe_rng_stream(olpe_ctx *c, int kind, int n, void *out) {
  if (!c || !out) return set_err(OLPE_EINVAL, "NULL argument");
  if (kind < 0 || kind > 3 || n <= 0) return set_err(OLPE_EINVAL, "bad kind/n");
  if (!c->seeded) return set_err(OLPE_ESTATE, "call olpe_seed first");
  HIPCHK(hipSetDevice(c->device));
  const size_t esz = kind == 0 ? 4 : 8;
  const size_t bytes = (size_t)c->W * n * esz;
  void *d = nullptr;
  HIPCHK(hipMalloc(&d, bytes));
  if (c->np == 16)
    hipLaunchKernelGGL(olpe_stream_kernel<16>, dim3(c->W), dim3(64), 0, c->stream, c->d_mt,
                       c->d_mtpos, c->d_hasg, c->d_gauss, c->W, kind, n, d);
  else
    hipLaunchKernelGGL(olpe_stream_kernel<19>, dim3(c->W), dim3(64), 0, c->stream, c->d_mt,
                       c->d_mtpos, c->d_hasg, c->d_gauss, c->W, kind, n, d);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(out, d, bytes, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return set_err(OLPE_EHIP, "rng stream: %s", hipGetErrorString(e));
  return OLPE_OK;
}

int olpe_test_hold_handoff(olpe_ctx *c, int on) {
  if (!c) return set_err(OLPE_EINVAL, "NULL ctx");
  c->hold_handoff = on != 0;
  return OLPE_OK;
}

int olpe_trace_enable(olpe_ctx *c, int on) {
  if (!c) return set_err(OLPE_EINVAL, "NULL ctx");
  c->trace_on = on != 0;
  return OLPE_OK;
}

int olpe_trace_read(olpe_ctx *c, double *out) {
  if (!c || !out) return set_err(OLPE_EINVAL, "NULL argument");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  const size_t m = (size_t)c->W * c->trace_iters * kTraceF;
  if (m) HIPCHK(hipMemcpy(out, c->d_trace, m * 8, hipMemcpyDeviceToHost));
  return OLPE_OK;
}

int olpe_sync(olpe_ctx *c) {
  if (!c) return set_err(OLPE_EINVAL, "NULL ctx");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  return check_units(c);
}

int olpe_unit_stats(olpe_ctx *c, long long *out) {
  if (!c || !out) return set_err(OLPE_EINVAL, "NULL argument");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  unsigned long long v[2] = {0, 0};
  HIPCHK(hipMemcpy(v, c->d_queue + 2, sizeof(v), hipMemcpyDeviceToHost));
  out[0] = (long long)v[0];
  out[1] = (long long)(v[1] * 10);       // 100 MHz ticks -> ns
  return OLPE_OK;
}

int olpe_last_units(olpe_ctx *c, int *units) {
  if (!c || !units) return set_err(OLPE_EINVAL, "NULL argument");
  *units = c->last_units;
  return OLPE_OK;
}

int olpe_kernel_times(olpe_ctx *c, int n, double *ms_out) {
  if (!c || !ms_out) return set_err(OLPE_EINVAL, "NULL argument");
  if (n < 1 || n > olpe_ctx::kRing || n > c->launches)
    return set_err(OLPE_EINVAL, "n = %d: 1..min(%d, launches so far = %lld)", n,
                   olpe_ctx::kRing, c->launches);
  HIPCHK(hipSetDevice(c->device));
  for (int i = 0; i < n; ++i) {
    hipEvent_t *ev = c->ev[(c->launches - n + i) % olpe_ctx::kRing];
    HIPCHK(hipEventSynchronize(ev[1]));
    float f = 0.f;
    HIPCHK(hipEventElapsedTime(&f, ev[0], ev[1]));
    ms_out[i] = f;
  }
  return OLPE_OK;
}

int olpe_last_kernel_ms(olpe_ctx *c, double *ms) {
  if (!c || !ms) return set_err(OLPE_EINVAL, "NULL argument");
  if (!c->launches) return set_err(OLPE_ESTATE, "no sampler launch yet");
  return olpe_kernel_times(c, 1, ms);
}

}  // extern "C"
