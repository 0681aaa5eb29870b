// olpe_device.h -- device building blocks of the gfx950 Gibbs sampler.
//
// One walker per 64-lane wavefront.  Everything a walker decides (parameter index,
// proposal, accept) is wave-uniform; the 64 lanes share the per-pixel work of the
// model + chi^2 sweep.  References are to the reference checkout.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "exp_table.h"

namespace olpe {

// ---------------------------------------------------------------------------------
// Parameter layouts (apf_step2.py:108, :215-234; 3body/apf_step2_3body.py:220-295)
// ---------------------------------------------------------------------------------
template <int NSRC> struct Layout;

template <> struct Layout<2> {
  static constexpr int NP = 16, PS = 17;
  static constexpr int DX = 4, DY = 5, RATIO = 8, OFF = 9;
  static constexpr int S1X = 10, S1Y = 11, S2X = 12, S2Y = 13, T1 = 14, T2 = 15;
  static constexpr int BG_QUIRK = 12, BG_FIXED = 9;   // apf_step2.py:120 vs :128
  // lognorm = [6,7,9,10,11,12,13] (apf_step2.py:217)
  static constexpr uint32_t LOGMASK = (1u << 6) | (1u << 7) | (1u << 9) | (1u << 10) |
                                      (1u << 11) | (1u << 12) | (1u << 13);
  __device__ static constexpr int sx(int s) { return s == 0 ? 0 : 2; }
  __device__ static constexpr int sy(int s) { return s == 0 ? 1 : 3; }
  __device__ static constexpr int sa(int s) { return s == 0 ? 6 : 7; }
};

template <> struct Layout<3> {
  static constexpr int NP = 19, PS = 20;
  static constexpr int DX = 6, DY = 7, RATIO = 11, OFF = 12;
  static constexpr int S1X = 13, S1Y = 14, S2X = 15, S2Y = 16, T1 = 17, T2 = 18;
  static constexpr int BG_QUIRK = 12, BG_FIXED = 12;  // 3body :121, p[12] is bkgd
  // lognorm = [8,9,10,12,13,14,15,16] (3body :295)
  static constexpr uint32_t LOGMASK = (1u << 8) | (1u << 9) | (1u << 10) | (1u << 12) |
                                      (1u << 13) | (1u << 14) | (1u << 15) | (1u << 16);
  __device__ static constexpr int sx(int s) { return 2 * s; }
  __device__ static constexpr int sy(int s) { return 2 * s + 1; }
  __device__ static constexpr int sa(int s) { return 8 + s; }
};

// ---------------------------------------------------------------------------------
// Wave helpers
// ---------------------------------------------------------------------------------
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ double uniform_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffffll));
  const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
  return __longlong_as_double(((long long)(unsigned)lo) | ((long long)hi << 32));
}

// one DPP move of a double (both halves); lanes outside row_mask read 0
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), CTRL, ROW_MASK, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROW_MASK, 0xf, false);
  return __longlong_as_double(((long long)(unsigned)lo) | ((long long)hi << 32));
}

// one DPP move of a double without an "old" operand: the lanes the row mask leaves
// out keep whatever the register held (no zeroing moves); only for reductions whose
// result is read from lanes every stage wrote
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_f64_any(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffffll), CTRL, ROW_MASK, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, ROW_MASK, 0xf, false);
  return __longlong_as_double(((long long)(unsigned)lo) | ((long long)hi << 32));
}

// Wave-wide sum with DPP (no LDS round trips): quad_perm [1,0,3,2] / [2,3,0,1],
// row_half_mirror, row_mirror (every lane of a row then holds the row's sum),
// row_bcast:15 (rows 1,3 add lane 15 / 47 of the row before), row_bcast:31 (rows 2,3
// add lane 31); lane 63 ends with the total, broadcast with readlane.  Only lanes
// 31 and 63 of the last two stages are read, and both lie in the rows those stages
// write, so the lanes the row masks leave out may hold anything: the moves need no
// zeroed "old" operand (2 VALU per stage fewer).
// The tree without the broadcast: the total is valid in lane 63 only (a caller that
// only tests it, e.g. the accept, ballots lane 63 and skips the two readlanes).
__device__ __forceinline__ double wave_sum_dpp_v(double v) {
  v += dpp_f64_any<0xB1, 0xf>(v);
  v += dpp_f64_any<0x4E, 0xf>(v);
  v += dpp_f64_any<0x141, 0xf>(v);
  v += dpp_f64_any<0x140, 0xf>(v);
  v += dpp_f64_any<0x142, 0xa>(v);
  v += dpp_f64_any<0x143, 0xc>(v);
  return v;
}
__device__ __forceinline__ double lane63_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), 63);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
  return __longlong_as_double(((long long)(unsigned)lo) | ((long long)hi << 32));
}
__device__ __forceinline__ double wave_sum_dpp(double v) { return lane63_f64(wave_sum_dpp_v(v)); }

// (The same sum on the matrix core -- two v_mfma_f64_16x16x4_f64 against a ones matrix,
// 8 VALU-port instructions where the DPP tree issues 20 -- ran 1.5 % slower on
// configs[2]: an FP64 MFMA holds the FP64 pipe; profiles/r02/ab_wavesum_mfma.log, removed
// in round 4.)
__device__ __forceinline__ double wave_sum(double v) {
  return wave_sum_dpp(v);
}
// the wave sum valid in lane 63
__device__ __forceinline__ double wave_sum_v(double v) {
  return wave_sum_dpp_v(v);
}

// ---------------------------------------------------------------------------------
// MT19937 + NumPy legacy distributions
// Draws are wave-uniform: a batch of 64 tempered outputs is held one-per-lane in a
// VGPR and read out with v_readlane, so a raw draw costs one VALU op plus scalar
// bookkeeping.  The floating-point draws are prepared lane-parallel once per batch
// (MTWave::prep): lane l computes rand() of words (l, l+1) and the whole polar
// attempt starting at word l (acceptance bit, factor sqrt(-2 log r2 / r2)), so a
// rand() or a gauss() whose words lie in the batch is a table read instead of ~100
// wave-uniform FP64 instructions; draws straddling the batch end take the scalar path.
// ---------------------------------------------------------------------------------
constexpr int MT_N = 624, MT_M = 397;
constexpr uint32_t MT_A = 0x9908b0dfu, MT_UP = 0x80000000u, MT_LO = 0x7fffffffu;

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

// The key stays in HBM (one 2,496-B row per walker); it is only touched by a refill
// of the 64-word batch (every 64 draws) and by the twist (every 624), through
// agent-scope atomics so that a load sees this wave's earlier stores.
// (global address space: sc1 global loads/stores, not flat -- the key is also handed
// between waves with a walker's chunks, olpe.hip unit_wait)
__device__ __forceinline__ uint32_t key_ld(const uint32_t *k, int i) {
  return __hip_atomic_load((__attribute__((address_space(1))) uint32_t *)(k + i), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void key_st(uint32_t *k, int i, uint32_t v) {
  __hip_atomic_store((__attribute__((address_space(1))) uint32_t *)(k + i), v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t lane_from(uint32_t v, int src_lane) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((src_lane & 63) << 2, (int)v);
}

// numpy mt19937_gen in registers: lane l holds key[64 p + l] in k[p] (p = 0..9).  Pass
// p writes key[i], i = 64p + l, from key[i], key[i+1] (old) and key[i+397] (old, i <
// 227: k[p+6] / k[p+7]) or key[i-227] (new, written by an EARLIER pass since 227 > 64:
// k[p-4] / k[p-3]); the cross-lane reads are ds_bpermute (no LDS storage).  10 ordered
// passes + the last word reproduce the sequential update exactly.  Returns the new
// words 0..63 (lane l: key[l]), the next batch.
__device__ inline uint32_t mt_twist(uint32_t *gkey, int lane) {
  uint32_t k[10];
#pragma unroll
  for (int p = 0; p < 10; ++p) k[p] = (64 * p + lane < MT_N) ? key_ld(gkey, 64 * p + lane) : 0u;
#pragma unroll
  for (int p = 0; p < 10; ++p) {
    const int i = 64 * p + lane;
    uint32_t ki1 = lane_from(k[p], lane + 1);                  // key[i+1], lanes 0..62
    if (p < 9) {
      const uint32_t nx = (uint32_t)__builtin_amdgcn_readlane((int)k[p + 1], 0);
      ki1 = lane == 63 ? nx : ki1;
    }
    // (every ds_bpermute runs with the whole wave active: it reads inactive lanes as 0)
    uint32_t src = 0;
    if (p + 6 <= 9) src = lane_from(k[p + 6], lane + 13);     // key[i+397], lanes 0..50
    if (p + 7 <= 9) {
      const uint32_t s7 = lane_from(k[p + 7], lane - 51);     // lanes 51..63
      src = lane > 50 ? s7 : src;
    }
    if (p >= 3) {                                             // key[i-227] (new)
      uint32_t nw = 0;
      if (p >= 4) nw = lane_from(k[p - 4], lane + 29);          // lanes 0..34
      const uint32_t nw2 = lane_from(k[p - 3], lane - 35);      // lanes 35..63
      nw = lane > 34 ? nw2 : nw;
      src = i >= MT_N - MT_M ? nw : src;
    }
    const uint32_t y = (k[p] & MT_UP) | (ki1 & MT_LO);
    const uint32_t nv = src ^ (y >> 1) ^ ((y & 1u) ? MT_A : 0u);
    k[p] = i < MT_N - 1 ? nv : k[p];
  }
  {  // the last word, key[623] = key[396] ^ twist(key[623], key[0]) with new key[0, 396]
    const uint32_t k623 = (uint32_t)__builtin_amdgcn_readlane((int)k[9], 47);
    const uint32_t k0 = (uint32_t)__builtin_amdgcn_readlane((int)k[0], 0);
    const uint32_t k396 = (uint32_t)__builtin_amdgcn_readlane((int)k[6], 12);
    const uint32_t y = (k623 & MT_UP) | (k0 & MT_LO);
    const uint32_t nv = k396 ^ (y >> 1) ^ ((y & 1u) ? MT_A : 0u);
    k[9] = lane == 47 ? nv : k[9];
  }
#pragma unroll
  for (int p = 0; p < 10; ++p)
    if (64 * p + lane < MT_N) key_st(gkey, 64 * p + lane, k[p]);
  return k[0];
}

// Accept test of FAST kernels: the reference accepts when dice < exp(-d/2), d = the
// chi^2 increase (apf_step2.py:139-148); for dice in [0, 1) that is d < -2 log(dice),
// so the threshold of every rand() of a batch is prepared lane-parallel with the draw
// tables (one log per 64 words) and the accept is one compare instead of an exp per
// step.  The two forms can only disagree where d and -2 log(dice) agree to rounding
// (the tests' flip criterion).  dice = 0 accepts below d = 1490.27, where exp(-d/2)
// underflows to 0 and the reference rejects.
__device__ __forceinline__ double accept_threshold(double u) {
  return u > 0.0 ? -2.0 * log(u) : 1490.2664382038824;
}
constexpr int kThr = 129;       // MTWave::tab offset of the accept thresholds


struct MTWave {
  uint32_t *key;  // HBM, MT_N words (this walker's row)
  int pos;        // numpy state->pos (uniform)
  int bstart;     // first key index held in `batch`
  int bsize;      // valid lanes in `batch`
  uint32_t batch; // tempered key[bstart + lane]
  int has_gauss;
  double gauss;
  // per-batch draw tables (LDS, kDrawTab doubles per wave): tab[l] = rand() of words
  // (l, l+1), tab[64 + l] = polar factor sqrt(-2 log r2 / r2) of the attempt at word
  // l, or -1 where that attempt is rejected (l + 3 < bsize), tab[128] = a rand()
  // assembled across the key end; tab[kThr + i] = accept threshold of the rand() at
  // tab[i] (i = 0..63, and 64 for tab[128]): -2 log(u), see accept_threshold
  double *tab;
  bool thr = true;   // write the accept thresholds (FAST samplers; EXACT has no room)

  // load the batch [pos, pos + 64) of the key (at most to its end; a used-up key is
  // twisted first) and prepare its draw tables
  __device__ void refill(int lane) {
    uint32_t v;
    if (pos >= MT_N) {
      v = mt_twist(key, lane);
      pos = 0;
    } else {
      const int n = (MT_N - pos) < 64 ? (MT_N - pos) : 64;
      v = (lane < n) ? key_ld(key, pos + lane) : 0u;
    }
    const int n = (MT_N - pos) < 64 ? (MT_N - pos) : 64;
    batch = mt_temper(v);
    bstart = pos;
    bsize = n;
    prep(lane);
  }
  // lane-parallel draw tables of the batch: lane l evaluates rand() at word l and the
  // polar attempt at word l with the operations of numpy's legacy_double /
  // legacy_gauss (x = 2 rand() - 1, r2 = x1*x1 + x2*x2, f = sqrt(-2 log(r2) / r2))
  __device__ void prep(int lane) {
    const uint32_t w1 = lane_from(batch, lane + 1);
    const double u = ((double)(batch >> 5) * 67108864.0 + (double)(w1 >> 6)) / 9007199254740992.0;
    const long long ub = __double_as_longlong(u);
    const uint32_t lo = lane_from((uint32_t)(ub & 0xffffffffll), lane + 2);
    const uint32_t hi = lane_from((uint32_t)(ub >> 32), lane + 2);
    const double u2 = __longlong_as_double((long long)lo | ((long long)hi << 32));
    const double x1 = 2.0 * u - 1.0;
    const double x2 = 2.0 * u2 - 1.0;
    const double r2 = x1 * x1 + x2 * x2;
    const double f = sqrt(-2.0 * log(r2) / r2);
    tab[lane] = u;
    tab[64 + lane] = ((r2 < 1.0) & (r2 != 0.0)) ? f : -1.0;   // bitwise &: no branches
    if (thr) tab[kThr + lane] = accept_threshold(u);
    wave_sync();
  }

  // The draws of Gibbs iterations in stream order, stages s0..s1:
  //   0  randint(0, NP)  apf_step2.py:302  buffered_bounded_masked_uint32 -> r
  //   1  gauss()         :307 (proposal)  legacy_gauss with the cached deviate -> g
  //   2  rand()          :144 (accept)    legacy_double -> tab[dice_idx]
  // One loop with ONE refill site, so the table preparation (log, sqrt, division) is
  // emitted once.  A draw whose words are in the batch is a table read; a batch with
  // fewer words left than the next draw needs is reloaded from pos, except at the key
  // end (pos + need > 624), where the draw is assembled word by word across the twist.
  template <int NP>
  __device__ void draw(int lane, int s0, int s1, int &r, double &g, int &dice_idx) {
    constexpr uint32_t rng = NP - 1;
    constexpr uint32_t m1 = rng | (rng >> 1);
    constexpr uint32_t m2 = m1 | (m1 >> 2);
    constexpr uint32_t m3 = m2 | (m2 >> 4);
    constexpr uint32_t mask = m3 | (m3 >> 8) | (m3 >> 16);
    if (s0 == 0 && s1 == 2) {
      // the common case first, without the loop: the whole iteration (randint word,
      // [attempt,] rand pair) lies in the batch and the first attempt is accepted
      const int p = pos - bstart;
      if (p + (has_gauss ? 3 : 7) <= bsize) {
        const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)batch, p) & mask;
        if (v <= rng) {
          r = (int)v;
          if (has_gauss) {
            has_gauss = 0;
            g = gauss;
            gauss = 0.0;
            dice_idx = p + 1;
            pos += 3;
            return;
          }
          const double f = uniform_f64(tab[64 + p + 1]);
          pos += 5;
          if (f >= 0.0) {
            const double x1 = 2.0 * tab[p + 1] - 1.0;
            const double x2 = 2.0 * tab[p + 3] - 1.0;
            gauss = uniform_f64(f * x1);
            has_gauss = 1;
            g = uniform_f64(f * x2);
            dice_idx = p + 5;
            pos += 2;
            return;
          }
          s0 = 1;                     // first attempt rejected: go on with the loop
        }
      }
    }
    int stage = s0;
    bool slow = false;
    int got = 0;
    uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;   // words gathered across the key end
    for (;;) {
      if (stage == 1 && has_gauss) {
        has_gauss = 0;
        g = gauss;
        gauss = 0.0;
        if (stage == s1) return;
        stage = 2;
        continue;
      }
      const int need = slow ? 1 : (stage == 0 ? 1 : stage == 1 ? 4 : 2);
      int p = pos - bstart;
      if (p + need > bsize) {
        if (!slow && pos < MT_N && pos + need > MT_N) {
          slow = true;
          continue;
        }
        refill(lane);
        p = 0;
      }
      if (!slow) {
        if (stage == 0) {
          const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)batch, p) & mask;
          ++pos;
          if (v > rng) continue;              // (NP = 19: masked rejection)
          r = (int)v;
        } else if (stage == 1) {
          pos += 4;
          const double f = uniform_f64(tab[64 + p]);
          if (f < 0.0) continue;               // rejected attempt
          const double x1 = 2.0 * tab[p] - 1.0;
          const double x2 = 2.0 * tab[p + 2] - 1.0;
          gauss = uniform_f64(f * x1);
          has_gauss = 1;
          g = uniform_f64(f * x2);
        } else {
          pos += 2;
          dice_idx = p;
        }
      } else {
        w0 = w1;
        w1 = w2;
        w2 = w3;
        w3 = (uint32_t)__builtin_amdgcn_readlane((int)batch, p);
        ++pos;
        if (++got < (stage == 1 ? 4 : 2)) continue;
        slow = false;
        got = 0;
        if (stage == 1) {
          const double x1 = 2.0 * (((double)(w0 >> 5) * 67108864.0 + (double)(w1 >> 6)) / 9007199254740992.0) - 1.0;
          const double x2 = 2.0 * (((double)(w2 >> 5) * 67108864.0 + (double)(w3 >> 6)) / 9007199254740992.0) - 1.0;
          const double r2 = uniform_f64(x1 * x1 + x2 * x2);
          if (!(r2 < 1.0 && r2 != 0.0)) continue;
          const double f = sqrt(-2.0 * log(r2) / r2);
          gauss = uniform_f64(f * x1);
          has_gauss = 1;
          g = uniform_f64(f * x2);
        } else {
          if (lane == 0) {
            const double u = ((double)(w2 >> 5) * 67108864.0 + (double)(w3 >> 6)) / 9007199254740992.0;
            tab[128] = u;
            if (thr) tab[kThr + 64] = accept_threshold(u);
          }
          wave_sync();
          dice_idx = 128;
        }
      }
      if (stage == s1) return;
      ++stage;
    }
  }

  // mt19937_next (raw stream test hook; the sampler draws through draw())
  __device__ uint32_t next(int lane) {
    if (pos - bstart >= bsize) refill(lane);
    const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)batch, pos - bstart);
    ++pos;
    return v;
  }
};
constexpr int kDrawTab = kThr + 65;   // doubles of MTWave::tab

// np.random.seed(s): init_genrand (mt19937_seed)
__device__ inline void mt_seed_serial(uint32_t *key, uint32_t s) {
  for (int i = 0; i < MT_N; ++i) {
    key[i] = s;
    s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(i + 1);
  }
}

// ---------------------------------------------------------------------------------
// Model pieces (astropy 4.3.1 Gaussian2D.evaluate, functional_models.py:366-381)
// ---------------------------------------------------------------------------------
// exp(x) for the FAST3 setup (guarded arguments): x = (64 k + j) ln2/64 + r with
// |r| <= ln2/128, exp(x) = 2^k * T[j] * (1 + q(r)), q of degree 5, T = 2^(j/64) from an
// LDS copy of c_exp2_64.  12 FP64 operations instead of ocml's 19 plus range selects;
// <= 1.13 ulp (tools/gen_exp_table.py --check).  Arguments are clamped to [-1000, 710]
// (underflow to 0, overflow to inf); NaN is not propagated (callers are guarded).
// (A {hi, lo}-table, degree-6 variant reaches 0.51 ulp but, with its LDS gather in the
// dependency chain, ran the EXACT sweep 13 % slower than ocml's exp: not used.)
constexpr int kEtabBytes = 64 * 8;
struct ExpTab {
  const double *T;
  __device__ __forceinline__ double operator()(double x) const {
    return raw(fmin(fmax(x, -1000.0), 710.0));
  }
  // without the clamp, for arguments whose use is guarded: the FAST3 column terms,
  // which are used only when fast3_ok / fast3_ok_cols has bounded every exponent over
  // the grid (|x| < ~750; a term computed ahead of a failing guard is discarded).  The
  // same value as operator() inside [-1000, 710]; 2 VALU fewer.
  __device__ __forceinline__ double raw(double x) const {
    const double kd = __builtin_rint(x * kExpInv);
    double r = fma(-kd, kExpHi, x);
    r = fma(-kd, kExpLo, r);
    double p = fma(r, 1.0 / 120, 1.0 / 24);
    p = fma(r, p, 1.0 / 6);
    p = fma(r, p, 0.5);
    p = fma(r, p, 1.0);
    const double q = r * p;
    const int k = (int)kd;
    const double t = T[k & 63];
    return ldexp(fma(t, q, t), k >> 6);
  }
};

// exp(-q) of the EXACT sweeps, q = the Gaussian's quadratic form (>= 0 up to rounding,
// or NaN, +inf).  The operations of ocml's exp, so the same bits: k = rint(-q log2 e),
// r = -q - k ln2 in two FMAs, 1 + r p(r) with p of degree 10, then 2^k by ldexp.  What is
// left out are ocml's range selects (two compares, three selects per call): an
// argument beyond the underflow point (q > 745.13) gives 0 through the ldexp (k <=
// -1075) as long as the reduction stays exact, so q > 1000 is clamped in its high word
// (one compare, one 32-bit select; the low word keeps q within [1000, 1000.0000001]),
// and NaN passes the compare and the reduction unchanged.  tools/micro/exp_check.hip
// compares it with ocml's exp bit for bit.  (A q far below 0 -- a quadratic form that
// rounding leaves negative by more than ~709 -- would give NaN where ocml gives inf;
// both make chi^2 reject the proposal.)
__device__ __forceinline__ double exp_neg(double q) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(q);
  const unsigned hi = q > 1000.0 ? 0x408F4000u : (unsigned)(b >> 32);
  q = __longlong_as_double((long long)(((unsigned long long)hi << 32) | (b & 0xffffffffull)));
  const double k = __builtin_rint(q * -0x1.71547652b82fep+0);
  double r = fma(k, -0x1.62e42fefa39efp-1, -q);
  r = fma(-0x1.abc9e3b39803fp-56, k, r);
  double p = fma(0x1.ade156a5dcb37p-26, r, 0x1.28af3fca7ab0cp-22);
  p = fma(r, p, 0x1.71dee623fde64p-19);
  p = fma(r, p, 0x1.a01997c89e6b0p-16);
  p = fma(r, p, 0x1.a01a014761f6ep-13);
  p = fma(r, p, 0x1.6c16c1852b7b0p-10);
  p = fma(r, p, 0x1.1111111122322p-7);
  p = fma(r, p, 0x1.55555555502a1p-5);
  p = fma(r, p, 0x1.5555555555511p-3);
  p = fma(r, p, 0x1.000000000000bp-1);
  p = fma(r, p, 1.0);
  p = fma(r, p, 1.0);
  return ldexp(p, (int)k);
}

struct Trig {
  double cost2, sint2, sin2t;
};
struct Coef {
  double a, b, c;
};
struct Gauss {
  double amp, x0, y0;
  Coef k;
};

// sin and cos of |th| <= pi/4 without range reduction: Taylor polynomials in t = th^2
// through th^17 (sin) and th^16 (cos), Horner form; the first omitted terms are below
// 1.3e-19 / 2.8e-18 relative at pi/4, so both are within ~1 ulp of the correctly rounded
// values (tools/check_sincos.py compares them with numpy over the range).  ~17 FP64
// operations against ~70 VALU instructions of ocml's sincos (range reduction, selects).
// The constants go in as SGPR operands (v_fma_f64 with an SGPR addend) instead of being
// materialised in VGPRs for v_fmac.
__device__ __forceinline__ double fma_sc(double a, double b, double c) {
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
  return r;
}
__device__ __forceinline__ void sincos_small(double th, double *s, double *c) {
  const double t = th * th;
  double p = fma_sc(t, 2.8114572543455207632e-15, -7.6471637318198164759e-13);  // 1/17!, -1/15!
  p = fma_sc(t, p, 1.6059043836821614599e-10);     // 1/13!
  p = fma_sc(t, p, -2.5052108385441718775e-8);     // -1/11!
  p = fma_sc(t, p, 2.7557319223985890653e-6);      // 1/9!
  p = fma_sc(t, p, -1.9841269841269841270e-4);     // -1/7!
  p = fma_sc(t, p, 8.3333333333333333333e-3);      // 1/5!
  p = fma_sc(t, p, -1.6666666666666666667e-1);     // -1/3!
  *s = fma(th * t, p, th);
  double q = fma_sc(t, 4.7794773323873852974e-14, -1.1470745597729724714e-11);  // 1/16!, -1/14!
  q = fma_sc(t, q, 2.0876756987868098979e-9);      // 1/12!
  q = fma_sc(t, q, -2.7557319223985890653e-7);     // -1/10!
  q = fma_sc(t, q, 2.4801587301587301587e-5);      // 1/8!
  q = fma_sc(t, q, -1.3888888888888888889e-3);     // -1/6!
  q = fma_sc(t, q, 4.1666666666666666667e-2);      // 1/4!
  q = fma(t, q, -0.5);
  *c = fma(t, q, 1.0);
}

// EXACT keeps astropy's operations (np.sin(2*theta), six divisions); FAST kernels use
// sin(2t) = 2 sin(t) cos(t), the polynomial sincos for |theta| <= pi/4 and two
// reciprocals (<= 2 ulp apart, within the fast tolerances of DESIGN.md §5).
template <bool FAST>
__device__ __forceinline__ Trig make_trig(double th) {
  double s, c;
  if (FAST && fabs(th) <= 0.78539816339744830962) {
    sincos_small(th, &s, &c);
  } else {
    sincos(th, &s, &c);        // np.sin(theta), np.cos(theta): one range reduction
  }
  return Trig{c * c, s * s, FAST ? 2.0 * (s * c) : sin(2. * th)};
}

// FAST coefficients from the shape's trig terms and the reciprocal variances
// ix = 1/sigma_x^2, iy = 1/sigma_y^2 (the sampler keeps those per shape set, so a draw
// of sigma_x recomputes one reciprocal and a draw of theta none)
__device__ __forceinline__ Coef coef_inv(const Trig &t, double ix, double iy) {
  Coef k;
  k.a = 0.5 * (t.cost2 * ix + t.sint2 * iy);
  k.b = 0.5 * (t.sin2t * (ix - iy));
  k.c = 0.5 * (t.sint2 * ix + t.cost2 * iy);
  return k;
}
__device__ __forceinline__ double inv_var(double s) { return 1.0 / (s * s); }

template <bool FAST>
__device__ __forceinline__ Coef make_coef(double sx, double sy, const Trig &t) {
  const double xstd2 = sx * sx, ystd2 = sy * sy;
  Coef k;
  if constexpr (FAST) {
    k = coef_inv(t, inv_var(sx), inv_var(sy));
  } else {
    k.a = 0.5 * ((t.cost2 / xstd2) + (t.sint2 / ystd2));
    k.b = 0.5 * ((t.sin2t / xstd2) - (t.sin2t / ystd2));
    k.c = 0.5 * ((t.sint2 / xstd2) + (t.cost2 / ystd2));
  }
  return k;
}

// Per-step model description: 2*NSRC Gaussians (wide, narrow per source; the order
// build_2d_gaussian adds them in, apf_step2.py:102) + constant background.
template <int NSRC> struct ModelDesc {
  Gauss g[2 * NSRC];
  double bg;
};

// Assemble the Gaussians for parameter vector q (accessor) and coefficient sets
// C1 (narrow: sigma_x, sigma_y, theta) and C2 (wide).  apf_step2.py:95-101, :115-120.
template <int NSRC, class Q>
__device__ __forceinline__ ModelDesc<NSRC> make_model(const Q &q, const Coef &C1,
                                                      const Coef &C2, int bkgd_mode) {
  using L = Layout<NSRC>;
  ModelDesc<NSRC> m;
#pragma unroll
  for (int s = 0; s < NSRC; ++s) {
    const double tot = q(L::sa(s)) - q(L::OFF);
    const double wide = tot * q(L::RATIO);
    const double narrow = tot - wide;
    const double xc = q(L::sx(s)), yc = q(L::sy(s));
    m.g[2 * s] = Gauss{wide, xc + q(L::DX), yc + q(L::DY), C2};
    m.g[2 * s + 1] = Gauss{narrow, xc, yc, C1};
  }
  m.bg = q(bkgd_mode == 0 ? L::BG_QUIRK : L::BG_FIXED);
  return m;
}

// ---------------------------------------------------------------------------------
// Pixel sweeps.  The cutout is stored interleaved, DE[pixel] = {D, 1/err} (one
// ds_read_b128 per pixel; masked pixels hold {0, 0}).  Lane L walks one column j
// (n >= 64: j = 64*pass + L; n < 64: the wave covers 64/n row groups, stride S), so
// per-column terms are computed once per step.
// ---------------------------------------------------------------------------------
__host__ __device__ constexpr int row_stride(int n) { return n >= 64 ? 1 : 64 / n; }

struct ColWalk {
  int S, nc, grp, jl;
  bool lane_ok;
  __device__ __forceinline__ ColWalk(int n, int lane) {
    S = n >= 64 ? 1 : 64 / n;      // row groups per wave
    nc = n >= 64 ? 64 : n;         // columns per pass
    grp = lane / nc;
    jl = lane - grp * nc;
    lane_ok = grp < S;
  }
};

// EXACT evaluation keeps the reference operation order per pixel:
//   q = ((a*dx^2) + ((b*dx)*dy)) + (c*dy^2);  v = A*exp(-q)
//   model = ((wide_0 + narrow_0) + (wide_1 + narrow_1) [+ ...]) + bg
//   t = (D - model) * invE;  acc += t*t
template <int NSRC, int NT, bool WRITE, int UNROLL = 2>
__device__ __forceinline__ double sweep_exact(const ModelDesc<NSRC> &m, const double2 *DE,
                                              double *out, int n_rt, int lane) {
  constexpr int G = 2 * NSRC;
  const int n = NT ? NT : n_rt;
  const ColWalk cw(n, lane);
  double acc = 0.0;
  for (int c0 = 0; c0 < n; c0 += 64) {
    const int j = c0 + cw.jl;
    const bool act = cw.lane_ok && j < n;
    const double xj = (double)j;
    double t1[G], t2[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const double xd = xj - m.g[g].x0;
      t1[g] = m.g[g].k.a * (xd * xd);
      t2[g] = m.g[g].k.b * xd;
    }
    const int jj = act ? j : 0;
#pragma unroll UNROLL
    for (int i = cw.grp; i < n; i += cw.S) {
      const double yi = (double)i;
      double v[G];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const double yd = yi - m.g[g].y0;
        const double qq = (t1[g] + t2[g] * yd) + m.g[g].k.c * (yd * yd);
        v[g] = m.g[g].amp * exp_neg(qq);
      }
      double mod = v[0] + v[1];
#pragma unroll
      for (int s = 1; s < NSRC; ++s) mod = mod + (v[2 * s] + v[2 * s + 1]);
      mod = mod + m.bg;
      if constexpr (WRITE) {
        if (act) out[i * n + j] = mod;
      } else {
        const double2 de = DE[i * n + jj];
        const double t = (de.x - mod) * de.y;
        acc = act ? fma(t, t, acc) : acc;
      }
    }
  }
  return acc;
}

// sweep_exact of the EXACT samplers (n = 32, 64, 128) with row terms from LDS:
// dy = i - y0 and c*(dy*dy) depend on the row and the Gaussian only, so the wave forms
// them once per step, lane-parallel over the rows, into qtab (c*dy^2) and, where there is
// room, ytab (dy) -- [n][G] doubles each, in LDS the EXACT sampler leaves unused -- and
// the row loop reads them as broadcasts: 3 operations per pixel and Gaussian for the
// quadratic form instead of 6 (4 without ytab).  The same operations on the same values
// as sweep_exact, so the same bits (test_exact_sampler_chi2_bitwise_equals_eval).
template <int NSRC, int NT, bool YT>
__device__ __forceinline__ double sweep_exact_rows(const ModelDesc<NSRC> &m, const double2 *DE,
                                                   int lane, double *ytab, double *qtab) {
  constexpr int G = 2 * NSRC;
  constexpr int S = NT >= 64 ? 1 : 64 / NT;      // row groups per wave
  constexpr int NC = NT >= 64 ? 64 : NT;         // columns per pass
#pragma unroll
  for (int r0 = 0; r0 < NT; r0 += 64) {
    const int r = r0 + lane;
    if (r < NT) {
      const double yi = (double)r;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const double yd = yi - m.g[g].y0;
        if constexpr (YT) ytab[r * G + g] = yd;
        qtab[r * G + g] = m.g[g].k.c * (yd * yd);
      }
    }
  }
  wave_sync();
  // the tables' LDS addresses in VGPRs, so that each row's reads are a VGPR base plus
  // immediate offsets (from SGPR bases the compiler copies every address to a VGPR)
  typedef __attribute__((address_space(3))) const double lds_f64;
  lds_f64 *yl = (lds_f64 *)(YT ? ytab : qtab);
  lds_f64 *ql = (lds_f64 *)qtab;
  asm volatile("" : "+v"(yl), "+v"(ql));
  const int grp = lane / NC, jl = lane - grp * NC;
  double acc = 0.0;
#pragma unroll 1
  for (int c0 = 0; c0 < NT; c0 += 64) {
    const int j = c0 + jl;
    const double xj = (double)j;
    double t1[G], t2[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const double xd = xj - m.g[g].x0;
      t1[g] = m.g[g].k.a * (xd * xd);
      t2[g] = m.g[g].k.b * xd;
    }
    // (two rows per trip; one for the 3-source 32x32 sampler, which spills with two)
    constexpr int kRowUnroll = NSRC == 3 && NT == 32 ? 1 : 2;
#pragma unroll kRowUnroll
    for (int i = grp; i < NT; i += S) {
      double v[G];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const double yd = YT ? yl[i * G + g] : (double)i - m.g[g].y0;
        const double qq = (t1[g] + t2[g] * yd) + ql[i * G + g];
        v[g] = m.g[g].amp * exp_neg(qq);
      }
      double mod = v[0] + v[1];
#pragma unroll
      for (int s = 1; s < NSRC; ++s) mod = mod + (v[2 * s] + v[2 * s + 1]);
      mod = mod + m.bg;
      const double2 de = DE[i * NT + j];
      const double t = (de.x - mod) * de.y;
      acc = fma(t, t, acc);
    }
  }
  wave_sync();   // the tables are rewritten by the next step
  return acc;
}

// Exact per-pixel model with the fast kernels' {D/err, 1/err} image: the fallback of
// FAST kernels for steps that fail both fast guards (residual in the fma form).
template <int NSRC, int NT, bool WRITE>
__device__ __forceinline__ double sweep_exact_dw(const ModelDesc<NSRC> &m, const double2 *DW,
                                                 double *out, int n_rt, int lane) {
  constexpr int G = 2 * NSRC;
  const int n = NT ? NT : n_rt;
  const ColWalk cw(n, lane);
  double acc = 0.0;
  for (int c0 = 0; c0 < n; c0 += 64) {
    const int j = c0 + cw.jl;
    const bool act = cw.lane_ok && j < n;
    const double xj = (double)j;
    const int jj = act ? j : 0;
#pragma unroll 1
    for (int i = cw.grp; i < n; i += cw.S) {
      const double yi = (double)i;
      double v[G];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const double xd = xj - m.g[g].x0;
        const double yd = yi - m.g[g].y0;
        const double qq = (m.g[g].k.a * (xd * xd) + (m.g[g].k.b * xd) * yd) +
                          m.g[g].k.c * (yd * yd);
        v[g] = m.g[g].amp * exp_neg(qq);
      }
      double mod = v[0] + v[1];
#pragma unroll
      for (int s = 1; s < NSRC; ++s) mod = mod + (v[2 * s] + v[2 * s + 1]);
      mod = mod + m.bg;
      if constexpr (WRITE) {
        if (act) out[i * n + j] = mod;
      } else {
        const double2 dw = DW[i * n + jj];
        const double t = fma(-mod, dw.y, dw.x);
        acc = act ? fma(t, t, acc) : acc;
      }
    }
  }
  return acc;
}

// FAST evaluation: with dx = j - x0, dy = i - y0,
//   A*exp(-(a dx^2 + b dx dy + c dy^2)) = V_i * W_ij
//   V_i  = exp(-c dy^2)                      one exp per lane (row), kept in LDS
//   W_ij = A*exp(-(a dx^2 + b dx dy))        one exp per lane (column) at the first row,
//          W_(i+S)j = W_ij * E_j,  E_j = exp(-b dx S)   one more exp per column
// so a pixel-Gaussian costs 2 multiplies instead of an exp.  The image is staged as
// DW[pixel] = {D/err, 1/err} so the residual is one fma: t = D/err - M*(1/err).
// Valid while the cross term stays bounded (|b dx dy| < kFastCross over the grid):
// then W can only underflow where the Gaussian is < e^-400.  Otherwise (or for
// non-finite parameters) the exact sweep runs -- a wave-uniform decision (fast_level).
constexpr double kFastCross = 300.0;
template <int NSRC, int NT, bool WRITE>
__device__ __forceinline__ double sweep_fast(const ModelDesc<NSRC> &m, const double2 *DW,
                                             double *vtab, double *out, int n_rt,
                                             int lane) {
  constexpr int G = 2 * NSRC;
  const int n = NT ? NT : n_rt;
  const ColWalk cw(n, lane);
  // row table V[i][g] = exp(-c_g dy^2), rows lane-parallel
  for (int i = lane; i < n; i += 64) {
    const double yi = (double)i;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const double yd = yi - m.g[g].y0;
      vtab[i * G + g] = exp(-(m.g[g].k.c * (yd * yd)));
    }
  }
  wave_sync();
  double acc = 0.0;
  const double S = (double)cw.S;
  const double y0r = (double)cw.grp;
  for (int c0 = 0; c0 < n; c0 += 64) {
    const int j = c0 + cw.jl;
    const bool act = cw.lane_ok && j < n;
    const double xj = (double)j;
    double E[G], Wc[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const double xd = xj - m.g[g].x0;
      const double bx = m.g[g].k.b * xd;
      Wc[g] = m.g[g].amp * exp(-(m.g[g].k.a * (xd * xd) + bx * (y0r - m.g[g].y0)));
      E[g] = exp(-(bx * S));
      // one Gaussian's exps at a time: caps the registers of this setup phase
      __builtin_amdgcn_sched_barrier(0);
    }
    const int jj = act ? j : 0;
    const double bg = m.bg;
    // software pipeline: the LDS rows (V table + pixel) of row i+S are read while
    // row i is computed, so the LDS latency hides behind the multiplies
    const double2 *vr = reinterpret_cast<const double2 *>(vtab) + cw.grp * (G / 2);
    const int vstep = cw.S * (G / 2);
    double2 vv[G / 2], dw;
#pragma unroll
    for (int h = 0; h < G / 2; ++h) vv[h] = vr[h];
    dw = WRITE ? make_double2(0.0, 0.0) : DW[cw.grp * n + jj];
#pragma unroll 2
    for (int i = cw.grp; i < n; i += cw.S) {
      const bool more = i + cw.S < n;
      double2 nv[G / 2], ndw;
      const double2 *nr = vr + (more ? vstep : 0);
#pragma unroll
      for (int h = 0; h < G / 2; ++h) nv[h] = nr[h];
      if constexpr (!WRITE) ndw = DW[(more ? i + cw.S : i) * n + jj];
      double v[G];
#pragma unroll
      for (int h = 0; h < G / 2; ++h) {
        v[2 * h] = vv[h].x * Wc[2 * h];
        v[2 * h + 1] = vv[h].y * Wc[2 * h + 1];
      }
#pragma unroll
      for (int g = 0; g < G; ++g) Wc[g] = Wc[g] * E[g];
      double mod = v[0] + v[1];
#pragma unroll
      for (int s = 1; s < NSRC; ++s) mod = mod + (v[2 * s] + v[2 * s + 1]);
      mod = mod + bg;
      if constexpr (WRITE) {
        if (act) out[i * n + j] = mod;
      } else {
        const double t = fma(-mod, dw.y, dw.x);
        acc = act ? fma(t, t, acc) : acc;
        dw = ndw;
      }
#pragma unroll
      for (int h = 0; h < G / 2; ++h) vv[h] = nv[h];
      vr = nr;
    }
  }
  wave_sync();   // vtab is rewritten by the next step
  return acc;
}

// FAST2 evaluation: second-order recurrence down each column, no row table.
// Q(i) = (a dx^2 + b dx dy_i) + c dy_i^2 is quadratic in the row i, so with stride S
//   G_(i+S) = G_i * R_i,   R_(i+S) = R_i * K,   K = exp(-2 c S^2)
// starting from G_i0 = A exp(-Q(i0)) and R_i0 = exp(-(Q(i0+S) - Q(i0))): two multiplies
// per pixel-Gaussian and no LDS traffic besides the pixel itself.  Rounding grows
// like m^2/2 ulp after m rows (<= 2048 ulp at 64 rows, typically ~300).  Guard
// (fast_level): Q stays below kFast2Q over the grid, so no G underflows and
// |Q(i+S) - Q(i)| < kFast2Q keeps R finite.
constexpr double kFast2Q = 690.0;

// Which sweep a FAST kernel may use for this model (wave-uniform): 2 = FAST2, 1 = the
// row-table FAST sweep, 0 = exact.  Per Gaussian, with mx = max|dx|, my = max|dy| over
// the grid: B = |b| mx my bounds the cross term and a mx^2 + B + c my^2 bounds Q.
template <int NSRC>
__device__ __forceinline__ int fast_level(const ModelDesc<NSRC> &m, int n) {
  const double hi = (double)(n - 1);
  bool ok1 = true, ok2 = true;
#pragma unroll
  for (int g = 0; g < 2 * NSRC; ++g) {
    const Gauss &q = m.g[g];
    const double mx = fmax(fabs(q.x0), fabs(hi - q.x0));
    const double my = fmax(fabs(q.y0), fabs(hi - q.y0));
    const double B = fabs(q.k.b) * mx * my;
    const double Qb = (q.k.a * (mx * mx) + B) + q.k.c * (my * my);
    const bool fin = isfinite(q.k.a) && isfinite(q.k.c) && isfinite(q.amp) &&
                     (q.k.a >= 0.0) && (q.k.c >= 0.0);
    ok1 = ok1 && fin && (B < kFastCross);
    ok2 = ok2 && fin && (Qb < kFast2Q);
  }
  return ok2 ? 2 : (ok1 ? 1 : 0);
}

template <int NSRC, int NT, bool WRITE>
__device__ __forceinline__ double sweep_fast2(const ModelDesc<NSRC> &m, const double2 *DW,
                                              double *out, int n_rt, int lane) {
  constexpr int G = 2 * NSRC;
  const int n = NT ? NT : n_rt;
  const ColWalk cw(n, lane);
  double acc = 0.0;
  const double S = (double)cw.S;
  const double yr = (double)cw.grp;
  for (int c0 = 0; c0 < n; c0 += 64) {
    const int j = c0 + cw.jl;
    const bool act = cw.lane_ok && j < n;
    const double xj = (double)j;
    double Gv[G], R[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const double xd = xj - m.g[g].x0;
      const double yd = yr - m.g[g].y0;
      const double bx = m.g[g].k.b * xd;
      const double q0 = (m.g[g].k.a * (xd * xd) + bx * yd) + m.g[g].k.c * (yd * yd);
      const double d1 = bx * S + (m.g[g].k.c * S) * (2.0 * yd + S);
      Gv[g] = m.g[g].amp * exp(-q0);
      R[g] = exp(-d1);
      __builtin_amdgcn_sched_barrier(0);
    }
    const int jj = act ? j : 0;
    const double bg = m.bg;
    double K[G];      // exp(-2 c S^2): the row step of the second-order recurrence
#pragma unroll
    for (int g = 0; g < G; ++g) K[g] = exp(-(2.0 * m.g[g].k.c * (S * S)));
    auto row = [&](int i, double2 dw) {
      double mod = Gv[0] + Gv[1];
#pragma unroll
      for (int s = 1; s < NSRC; ++s) mod = mod + (Gv[2 * s] + Gv[2 * s + 1]);
      mod = mod + bg;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        Gv[g] = Gv[g] * R[g];
        R[g] = R[g] * K[g];
      }
      if constexpr (WRITE) {
        if (act) out[i * n + j] = mod;
      } else {
        const double t = fma(-mod, dw.y, dw.x);
        acc = act ? fma(t, t, acc) : acc;
      }
    };
    constexpr int BLK = 4;
    const int rows = (n - cw.grp + cw.S - 1) / cw.S;       // rows of this lane
    if (!WRITE && NT != 0 && rows % BLK == 0) {
      // explicit software pipeline: the next block's pixels are loaded into their own
      // registers while this block computes, so one lgkmcnt wait per block is covered
      const int rstep = cw.S * n;
      const double2 *p = DW + cw.grp * n + jj;
      double2 cur[BLK], nxt[BLK];
#pragma unroll
      for (int k = 0; k < BLK; ++k) cur[k] = p[k * rstep];
      for (int b0 = 0; b0 < rows; b0 += BLK) {
        const double2 *pn = p + ((b0 + BLK < rows) ? BLK * rstep : 0);
#pragma unroll
        for (int k = 0; k < BLK; ++k) nxt[k] = pn[k * rstep];
#pragma unroll
        for (int k = 0; k < BLK; ++k) row(cw.grp + (b0 + k) * cw.S, cur[k]);
#pragma unroll
        for (int k = 0; k < BLK; ++k) cur[k] = nxt[k];
        p = pn;
      }
    } else {
#pragma unroll 4
      for (int i = cw.grp; i < n; i += cw.S)
        row(i, WRITE ? make_double2(0.0, 0.0) : DW[i * n + jj]);
    }
  }
  return acc;
}

// FAST3 evaluation (default path): the Gaussians of one shape set (all narrow ones
// share sigma_x, sigma_y, theta; all wide ones too) share c, so with k the lane's row
// step (row i = grp + k*S), a reference step kc and
//   H_k = exp(-c S^2 (k - kc)(k - kc - 1))            one table per set, k-uniform
//   a_k = A exp(-(Q_0 - c S^2 kc (kc+1))) * rho^k,   rho = exp(-(Q_1 - Q_0 + 2 c S^2 kc))
// G_k = a_k * H_k exactly (Q_k is quadratic in k).  a_k is geometric (1 multiply per
// pixel-Gaussian, <= k ulp), H comes from an LDS table read once per row for all
// Gaussians:  model = fma(sum_narrow a, H_n, fma(sum_wide a, H_w, bg)).
// 10 FP64 ops per pixel for 2 sources (FAST2: 14); 8.5 with the four-row update below.
// Guard (fast3_ok): c S^2 (kc+1)^2 < 600 keeps a_k from overflowing and H from
// underflowing, and the FAST2 bound on Q
// (relaxed by c S^2 kc (kc+1)) keeps a_0 from underflowing where G is significant.
// Lane-parallel: lane g < 2*NSRC tests Gaussian g (the descriptor is in LDS), one
// ballot combines them.
template <int NSRC>
__device__ __forceinline__ bool fast3_ok(const ModelDesc<NSRC> &m, int n, int rows, int kc,
                                         int lane) {
  const double hi = (double)(n - 1);
  const double S2 = (double)(row_stride(n) * row_stride(n));
  const double km = (double)(kc > rows - 1 - kc ? kc : rows - 1 - kc) + 1.0;
  const Gauss &q = m.g[lane < 2 * NSRC ? lane : 0];
  const double mx = fmax(fabs(q.x0), fabs(hi - q.x0));
  const double my = fmax(fabs(q.y0), fabs(hi - q.y0));
  const double Qb = (q.k.a * (mx * mx) + fabs(q.k.b) * mx * my) + q.k.c * (my * my);
  const double cs = q.k.c * S2;
  // bitwise &: no short-circuit branches (exec-mask juggling) in the lane-parallel test
  const bool ok = (int)(cs * km * km < 600.0) & (int)(Qb < 700.0 + cs * kc * (kc + 1.0)) &
                  (int)isfinite(Qb) & (int)isfinite(q.amp) & (int)(q.k.a >= 0.0) &
                  (int)(q.k.c >= 0.0);
  return __builtin_amdgcn_ballot_w64(!ok) == 0;
}
// The same test, returning the Gaussians that fail it (bit g), for the per-column
// guard to retest only those.
template <int NSRC>
__device__ __forceinline__ unsigned fast3_fails(const ModelDesc<NSRC> &m, int n, int rows,
                                                int kc, int lane) {
  const double hi = (double)(n - 1);
  const double S2 = (double)(row_stride(n) * row_stride(n));
  const double km = (double)(kc > rows - 1 - kc ? kc : rows - 1 - kc) + 1.0;
  const Gauss &q = m.g[lane < 2 * NSRC ? lane : 0];
  const double mx = fmax(fabs(q.x0), fabs(hi - q.x0));
  const double my = fmax(fabs(q.y0), fabs(hi - q.y0));
  const double Qb = (q.k.a * (mx * mx) + fabs(q.k.b) * mx * my) + q.k.c * (my * my);
  const double cs = q.k.c * S2;
  const bool ok = (int)(cs * km * km < 600.0) & (int)(Qb < 700.0 + cs * kc * (kc + 1.0)) &
                  (int)isfinite(Qb) & (int)isfinite(q.amp) & (int)(q.k.a >= 0.0) &
                  (int)(q.k.c >= 0.0);
  return (unsigned)__builtin_amdgcn_ballot_w64(!ok) & ((1u << (2 * NSRC)) - 1u);
}

// FAST3 guard, per column (when fast3_ok's whole-grid bound fails, e.g. a source far
// from the grid centre of a 128-pixel cutout, where Q over the whole grid exceeds the
// range the anchored a_0 can represent).  Per Gaussian: c S^2 km^2 < 600 as in
// fast3_ok (no a_k overflow, no H underflow) and, in every column j (lane-parallel,
// the quantities col_term evaluates):
//   |log rho| < 170                      (rho^4 of the four-row update finite), and
//   log(a_0 / A) > -700                  (a_0 normal: a_k = a_0 rho^k exact), or
//   (a - b^2 / 4c) dx^2 >= 100           (Q >= 100 on the whole column: the Gaussian is
//                                         below A e^-100 there, so an a_0 that underflows
//                                         only drops values below that).
// |A| < 1e20 keeps A e^-100 negligible beside any model value.
template <int NSRC>
__device__ __forceinline__ bool fast3_ok_cols(const ModelDesc<NSRC> &m, int n, int rows, int kc,
                                              int lane, unsigned which) {
  const ColWalk cw(n, lane);
  const double S = (double)cw.S;
  const double kcd = (double)kc;
  const double km = (double)(kc > rows - 1 - kc ? kc : rows - 1 - kc) + 1.0;
  const double yr = (double)cw.grp;
  int ok = 1;
  // not unrolled: the descriptor is in LDS, and the guard must not raise the sampler's
  // register pressure (an unrolled form spilled)
#pragma unroll 1
  for (unsigned f = which; f; f &= f - 1u) {
    const Gauss &q = m.g[__builtin_ctz(f)];
    const double cs = q.k.c * (S * S);
    const double K = cs * (kcd * (kcd + 1.0));
    const double amin = q.k.a - (q.k.b * q.k.b) / (4.0 * q.k.c);
    const double yd = yr - q.y0;
    ok &= (int)(cs * km * km < 600.0) & (int)(q.k.a >= 0.0) & (int)(q.k.c > 0.0) &
          (int)(fabs(q.amp) < 1e20) & (int)isfinite(amin);
#pragma unroll 1
    for (int c0 = 0; c0 < n; c0 += 64) {
      const int j = c0 + cw.jl;
      const bool act = cw.lane_ok && j < n;
      const double xd = (double)j - q.x0;
      const double bx = q.k.b * xd;
      const double q0 = (q.k.a * (xd * xd) + bx * yd) + q.k.c * (yd * yd);
      const double d0 = bx * S + (q.k.c * S) * (2.0 * yd + S);
      const double xe = K - q0;
      const double xr = d0 + 2.0 * cs * kcd;
      const int okc = (int)(fabs(xr) < 170.0) & ((int)(xe > -700.0) | (int)(amin * (xd * xd) >= 100.0));
      ok &= okc | (int)!act;
    }
  }
  return __builtin_amdgcn_ballot_w64(!ok) == 0;
}

// The per-column test of fast3_ok_cols for each Gaussian of `which`, without its
// amplitude bound: returns the Gaussians that pass.  Their result is a function of the
// Gaussian's centre and shape only, so the sampler keeps it per Gaussian across steps
// (GuardCache::colok) and retests only the Gaussians a draw moves or reshapes; the
// amplitude bound (|A| < 1e20) is checked every step (fast3_amp_ok).
template <int NSRC>
__device__ __forceinline__ unsigned fast3_cols_pass(const ModelDesc<NSRC> &m, int n, int rows, int kc,
                                                   int lane, unsigned which) {
  const ColWalk cw(n, lane);
  const double S = (double)cw.S;
  const double kcd = (double)kc;
  const double km = (double)(kc > rows - 1 - kc ? kc : rows - 1 - kc) + 1.0;
  const double yr = (double)cw.grp;
  unsigned passed = 0;
#pragma unroll 1
  for (unsigned f = which; f; f &= f - 1u) {
    const int g = __builtin_ctz(f);
    const Gauss &q = m.g[g];
    const double cs = q.k.c * (S * S);
    const double K = cs * (kcd * (kcd + 1.0));
    const double amin = q.k.a - (q.k.b * q.k.b) / (4.0 * q.k.c);
    const double yd = yr - q.y0;
    int ok = (int)(cs * km * km < 600.0) & (int)(q.k.a >= 0.0) & (int)(q.k.c > 0.0) &
             (int)isfinite(amin);
#pragma unroll 1
    for (int c0 = 0; c0 < n; c0 += 64) {
      const int j = c0 + cw.jl;
      const bool act = cw.lane_ok && j < n;
      const double xd = (double)j - q.x0;
      const double bx = q.k.b * xd;
      const double q0 = (q.k.a * (xd * xd) + bx * yd) + q.k.c * (yd * yd);
      const double d0 = bx * S + (q.k.c * S) * (2.0 * yd + S);
      const double xe = K - q0;
      const double xr = d0 + 2.0 * cs * kcd;
      const int okc = (int)(fabs(xr) < 170.0) & ((int)(xe > -700.0) | (int)(amin * (xd * xd) >= 100.0));
      ok &= okc | (int)!act;
    }
    if (__builtin_amdgcn_ballot_w64(!ok) == 0) passed |= 1u << g;
  }
  return passed;
}
// fast3_ok_cols's amplitude bound for the Gaussians of `which` (lane-parallel)
template <int NSRC>
__device__ __forceinline__ bool fast3_amp_ok(const ModelDesc<NSRC> &m, int lane, unsigned which) {
  const bool bad = lane < 2 * NSRC && ((which >> lane) & 1u) &&
                   !(fabs(m.g[lane < 2 * NSRC ? lane : 0].amp) < 1e20);
  return __builtin_amdgcn_ballot_w64(bad) == 0;
}

// FAST3's shape tables, tab[2k] = H_wide(k), tab[2k+1] = H_narrow(k), k lane-parallel.
// `which` selects the sets recomputed (bit 0 wide, bit 1 narrow); the others are copied
// from `from` (the table of the current state: a Gibbs step changes at most one set).
template <int NSRC>
__device__ __forceinline__ void build_htab(const ModelDesc<NSRC> &m, double *tab,
                                           const double *from, int which, int rows, int kc,
                                           double S, int lane, ExpTab ex) {
  const double cw2 = m.g[0].k.c * (S * S);        // wide set   (even g)
  const double cn2 = m.g[1].k.c * (S * S);        // narrow set (odd g)
  for (int k = lane; k < rows; k += 64) {
    const double dk = (double)(k - kc);
    const double e = dk * (dk - 1.0);
    double2 h;
    h.x = (which & 1) ? ex(-(cw2 * e)) : from[2 * k];
    h.y = (which & 2) ? ex(-(cn2 * e)) : from[2 * k + 1];
    reinterpret_cast<double2 *>(tab)[k] = h;
  }
  wave_sync();
}

// Per-walker cache of the FAST3 tables in the two halves of the wave's vtab area: slot
// `cur` holds the tables of the current state when `valid`; a shape proposal builds its
// tables in the other slot (`flip` = that slot holds the proposal's tables).
// FAST3 guard result of the current state (sampler kernels): a draw that moves no
// Gaussian and no shape (amplitudes, ratio, offset: gauss_mask 0, grp 0 -- 4 of the
// 16 draws of the 2-source model) leaves every guard input but the amplitudes
// unchanged, and the guard's only amplitude test (finite) cannot change the step's
// outcome: a non-finite amplitude makes chi^2 NaN, which rejects, in every sweep.
// So such a draw reuses the current state's result.
struct GuardCache {
  bool same = false;    // this step's draw leaves the guard inputs unchanged
  bool valid = false;   // cur holds the current state's guard
  bool cur = false, prop = false;
  // per-column guard (cutouts wider than 64): colok = the Gaussians known to pass
  // fast3_cols_pass in the current state; changed = the Gaussians this step's draw
  // moves or reshapes; colprop / coltest = the proposal's known passes / this step's
  // tested ones
  unsigned colok = 0, changed = 0, colprop = 0, coltest = 0;
  __device__ __forceinline__ void after(bool accepted) {
    if (same || accepted) {
      cur = prop;
      valid = true;
    }
    // an accept makes the proposal's results current; after a reject the results of
    // Gaussians the draw left unchanged still hold
    colok = accepted ? colprop : (colok & ~changed) | (coltest & ~changed);
    coltest = 0;
  }
};

struct HCache {
  int cur = 0;
  int valid = 0;        // (ints, not bools: a uniform bool carried across the sampler
                        // loop is kept as a lane mask, read back with v_cndmask +
                        // v_readfirstlane)
  int grp = 0;          // this step's proposal: 0 no shape change, 1 narrow set, 2 wide set
  int flip = 0;
  int single = 0;       // one slot (olpe.hip single_h): a shape proposal rebuilds its set
                        // in place, so the slot is current only if the proposal is taken
  int stale = 0;        // single slot: sets (bit 0 wide, bit 1 narrow) the slot holds
                        // for another state than the current one; rebuilt when next used
  __device__ __forceinline__ void after(bool accepted) {
    if (single) {
      // flip = this step rebuilt its set in place (FAST3 taken): stale unless accepted;
      // otherwise the slot still holds the state before the step: stale if accepted
      if (grp && (flip ? !accepted : accepted)) stale |= grp == 1 ? 2 : 1;
      flip = 0;
      return;
    }
    if (accepted && grp) {
      if (flip) cur ^= 1;
      else valid = false;
    }
    flip = false;
  }
};

// FAST3 per-column terms of Gaussian q at column xj, row-group offset yr:
// E = exp(-(Q_0 - c S^2 kc (kc+1))) (a_0 = amp E) and rho.
struct ColTerm {
  double E, R;
};
__device__ __forceinline__ ColTerm col_term(const Gauss &q, double xj, double yr, double S,
                                            double kcd, ExpTab ex) {
  const double xd = xj - q.x0;
  const double yd = yr - q.y0;
  const double c = q.k.c;
  const double cs = c * (S * S);
  const double bx = q.k.b * xd;
  const double q0 = (q.k.a * (xd * xd) + bx * yd) + c * (yd * yd);
  const double d0 = bx * S + (c * S) * (2.0 * yd + S);
  return ColTerm{ex.raw(-(q0 - cs * (kcd * (kcd + 1.0)))), ex.raw(-(d0 + 2.0 * cs * kcd))};
}

// The same terms for sweeps with S = 1 and row group 0 (n = 64 and 128), from
// per-step coefficients prepared lane-parallel with the descriptor (col_coef):
// q0 - K = (a xd + beta) xd + gamma and the rho exponent b xd + delta -- 3 fma per
// column-Gaussian instead of ~11 operations (the column terms' setup is on the step's
// critical path).  Every cached and refreshed term of such a sweep uses this form.
__device__ __forceinline__ void col_coef(const Gauss &q, double kcd, double *cc) {
  const double yd = -q.y0;
  cc[0] = q.k.b * yd;
  cc[1] = q.k.c * (yd * yd - kcd * (kcd + 1.0));
  cc[2] = q.k.c * ((2.0 * yd + 1.0) + 2.0 * kcd);
}
__device__ __forceinline__ ColTerm col_term64(const Gauss &q, const double *cc, double xj,
                                              ExpTab ex) {
  const double xd = xj - q.x0;
  return ColTerm{ex.raw(-fma(fma(q.k.a, xd, cc[0]), xd, cc[1])), ex.raw(-fma(q.k.b, xd, cc[2]))};
}
// 128 x 128 sweeps, second column pass (columns j + 64): E from its exponent, rho from
// the first pass's (held in the four-row update's powers) times the pass step
// exp(-64 b) the descriptor lanes prepare (colc[6 NSRC + g]): one exp per
// column-Gaussian instead of two.  Under the guards |64 b| < 340 (the per-column rho
// bound of both passes), so the step is finite; rho is within ~1 ulp of the direct exp.
__device__ __forceinline__ ColTerm col_term64_pass1(const Gauss &q, const double *cc, double xj,
                                                    double rho0, double step, ExpTab ex) {
  const double xd = xj - q.x0;
  return ColTerm{ex.raw(-fma(fma(q.k.a, xd, cc[0]), xd, cc[1])), rho0 * step};
}

// Gaussians whose column terms a proposal of parameter r changes (bit g): a source's
// position moves its two Gaussians, DX/DY the wide ones, a shape set its own; the
// amplitudes, ratio, offset and background change no E or rho.
template <int NSRC> __device__ __forceinline__ unsigned gauss_mask(int r) {
  using L = Layout<NSRC>;
  unsigned msk = 0;
#pragma unroll
  for (int s = 0; s < NSRC; ++s) {
    if (r == L::sx(s) || r == L::sy(s)) msk |= 3u << (2 * s);
    if (r == L::DX || r == L::DY || r == L::S2X || r == L::S2Y || r == L::T2) msk |= 1u << (2 * s);
    if (r == L::S1X || r == L::S1Y || r == L::T1) msk |= 2u << (2 * s);
  }
  return msk;
}

// Per-walker cache (registers) of the current state's FAST3 column terms, for
// single-pass sweeps (n <= 64): a step recomputes only the Gaussians its proposal
// changes, and an accepted step refreshes those from the new state.  Cached values are
// the same pure function of the Gaussian, so results do not depend on the cache.
template <int G> struct ColCache {
  double E[G], R[G];
  unsigned valid = 0;
  // LDS: the proposal's (E, rho) of the Gaussians it moves, [slot][2][64 lanes] with
  // slot = rank of g among the moved ones; an accept copies them instead of
  // recomputing (pend = the gmask they belong to)
  double *pbuf = nullptr;
  unsigned pend = 0;
  // the step's col_coef coefficients [G][3] (LDS), for n = 64 / 128 sweeps (col_term64)
  const double *colc = nullptr;
};

// The proposal's column terms of the Gaussians it moves (gauss_mask: 0, 2 or NSRC of
// them), lane = column of a single-pass sweep (n <= 64), in one straight-line block so
// that their independent exp chains interleave with each other and with the guard,
// which runs after it: the setup is latency-bound (a diagnostic build without column
// terms runs 25 % faster, for ~10 % of the VALU instructions).  One Gaussian per
// branch inside the sweep was 0.3-1.2 % slower; raised priority for the block
// gained nothing.
template <int NSRC> struct MovedTerms {
  double E[NSRC], R[NSRC];   // component-wise: struct selects go through scratch
  int gi[NSRC];              // Gaussian of slot k (-1: none)
  int nm;                    // moved Gaussians
};

template <int NSRC, int NT>
__device__ __forceinline__ void moved_terms(MovedTerms<NSRC> &mt, const ModelDesc<NSRC> &m,
                                            unsigned gmask, int n, int lane, int kc,
                                            ExpTab ex, const double *colc) {
  const ColWalk cw(n, lane);
  mt.nm = __builtin_popcount(gmask);
  unsigned rest = gmask;
#pragma unroll
  for (int k = 0; k < NSRC; ++k) {
    mt.gi[k] = rest ? __builtin_ctz(rest) : -1;
    rest &= rest - 1u;
  }
  if (mt.nm >= 2) {
    // (two moved with three sources: the third term repeats the first one)
#pragma unroll
    for (int k = 0; k < NSRC; ++k) {
      const int g = k < mt.nm ? mt.gi[k] : mt.gi[0];
      ColTerm t;
      if constexpr (NT == 64)
        t = col_term64(m.g[g], colc + 3 * g, (double)cw.jl, ex);
      else
        t = col_term(m.g[g], (double)cw.jl, (double)cw.grp, (double)cw.S, (double)kc, ex);
      mt.E[k] = t.E;
      mt.R[k] = t.R;
    }
  }
}

template <int NSRC, int NT, bool WRITE, bool CC = false, bool WIDE = false>
__device__ __forceinline__ double sweep_fast3(const ModelDesc<NSRC> &m, const double2 *DW,
                                              const double *htab, double *out, int n_rt,
                                              int lane, int rows, int kc, ExpTab ex,
                                              ColCache<2 * NSRC> *cc = nullptr,
                                              unsigned gmask = 0,
                                              const MovedTerms<NSRC> *pre = nullptr) {
  constexpr int G = 2 * NSRC;
  const int n = NT ? NT : n_rt;
  const ColWalk cw(n, lane);
  const double S = (double)cw.S;
  const double kcd = (double)kc;
  const double yr = (double)cw.grp;
  const double bg = m.bg;
  double acc = 0.0;
  [[maybe_unused]] double rho0[G];     // NT = 128: pass 0's rho (col_term64_pass1)
  for (int c0 = 0; c0 < n; c0 += 64) {
    const int j = c0 + cw.jl;
    const bool act = cw.lane_ok && j < n;
    const double xj = (double)j;
    double av[G], rho[G];
    // the moved Gaussians' terms come precomputed (moved_terms, before the guard)
    if constexpr (CC) {
      if (pre->nm >= 2) {
        if (cc->pbuf) {          // park the proposal's terms for an accept
#pragma unroll
          for (int k = 0; k < NSRC; ++k) {
            if (k < pre->nm) {
              cc->pbuf[(2 * k) * 64 + lane] = pre->E[k];
              cc->pbuf[(2 * k + 1) * 64 + lane] = pre->R[k];
            }
          }
        }
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      ColTerm t;
      if constexpr (CC) {
        const bool mine = (gmask >> g) & 1u;
        if (mine) {
          double e = pre->E[0], r = pre->R[0];
#pragma unroll
          for (int k = 1; k < NSRC; ++k) {
            e = (g == pre->gi[k]) ? pre->E[k] : e;
            r = (g == pre->gi[k]) ? pre->R[k] : r;
          }
          t = ColTerm{e, r};
        } else if ((cc->valid >> g) & 1u) {
          t = ColTerm{cc->E[g], cc->R[g]};
        } else {                 // (first step of a walker) a term of the current state
          if constexpr (NT == 64)
            t = col_term64(m.g[g], cc->colc + 3 * g, xj, ex);
          else
            t = col_term(m.g[g], xj, yr, S, kcd, ex);
          cc->E[g] = t.E;
          cc->R[g] = t.R;
          cc->valid |= 1u << g;
        }
      } else if constexpr (NT == 128) {     // sampler kernels (cc carries the coefficients)
        t = c0 == 0 ? col_term64(m.g[g], cc->colc + 3 * g, xj, ex)
                    : col_term64_pass1(m.g[g], cc->colc + 3 * g, xj, rho0[g],
                                       cc->colc[3 * G + g], ex);
        rho0[g] = t.R;
      } else if constexpr (NT >= 64) {
        t = col_term64(m.g[g], cc->colc + 3 * g, xj, ex);
      } else {
        t = col_term(m.g[g], xj, yr, S, kcd, ex);
      }
      av[g] = m.g[g].amp * t.E;
      rho[g] = t.R;
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (CC) cc->pend = gmask;
    const int jj = act ? j : 0;
    const double2 *hr = reinterpret_cast<const double2 *>(htab);
    auto row = [&](int i, double2 h, double2 dw) {
      double sw = av[0], sn = av[1];
#pragma unroll
      for (int s = 1; s < NSRC; ++s) {
        sw = sw + av[2 * s];
        sn = sn + av[2 * s + 1];
      }
      const double mod = fma(sn, h.y, fma(sw, h.x, bg));
#pragma unroll
      for (int g = 0; g < G; ++g) av[g] = av[g] * rho[g];
      if constexpr (WRITE) {
        if (act) out[i * n + j] = mod;
      } else {
        const double t = fma(-mod, dw.y, dw.x);
        acc = act ? fma(t, t, acc) : acc;
      }
    };
    // RU rows per update (the unrolled row loop): row k+r sums a_k rho^r (r < RU)
    // with fmas and a_(k+RU) = a_k rho^RU.  Per set of m Gaussians: RU = 4 costs 5m-1
    // operations per four rows (8.5 FP64 per pixel for two sources), RU = 2 3m-1 per
    // two rows (9), against 2m-1 per row without it (10).  RU = 2 only where registers
    // are short (LEAN below: with the walker queue it spilled less, 518 vs 502 M
    // walker-steps/s on one box); the 12-wave sampler runs RU = 4 with the prefetch
    // (510 vs 500 M against the 16-wave LEAN one; 3-source 128x128: 88.2 vs 85.7 M).
    // The powers are formed once per column; the recurrence rounds n/RU times down a
    // column.
    // LEAN: the 3-source 32x32 / 64x64 samplers: the two-row update (registers)
    // The 2-source 64x64 sampler at 16 waves per workgroup (128 VGPRs) runs the
    // four-row update with the shape-table prefetch too, at the cost of one 8-byte spill
    // (stored once per walker): +0.6-1.3 % over it without the prefetch (no spill), which
    // was +1.0-1.4 % over the 12-wave sampler; the two-row update ran level with 12
    // waves (profiles/r02/ab_w16.log)
    constexpr bool LEAN = NSRC == 3 && (NT == 64 || NT == 32);
    constexpr int RU = LEAN ? 2 : 4;
    constexpr bool HPF = !LEAN;
    double rp[RU][G];                  // rp[r] = rho^r, rp[0] = rho^RU
#pragma unroll
    for (int g = 0; g < G; ++g) {
      rp[1][g] = rho[g];
      if constexpr (RU == 4) {
        rp[2][g] = rho[g] * rho[g];
        rp[3][g] = rp[2][g] * rho[g];
        rp[0][g] = rp[2][g] * rp[2][g];
      } else {
        rp[0][g] = rho[g] * rho[g];
      }
    }
    auto row4 = [&](const double2 *h, const double2 *dw) {
      double sw[RU], sn[RU];
      sw[0] = av[0];
      sn[0] = av[1];
#pragma unroll
      for (int s = 1; s < NSRC; ++s) {
        sw[0] = sw[0] + av[2 * s];
        sn[0] = sn[0] + av[2 * s + 1];
      }
#pragma unroll
      for (int r = 1; r < RU; ++r) {
        sw[r] = av[2 * NSRC - 2] * rp[r][2 * NSRC - 2];
        sn[r] = av[2 * NSRC - 1] * rp[r][2 * NSRC - 1];
#pragma unroll
        for (int s = NSRC - 2; s >= 0; --s) {
          sw[r] = fma(av[2 * s], rp[r][2 * s], sw[r]);
          sn[r] = fma(av[2 * s + 1], rp[r][2 * s + 1], sn[r]);
        }
      }
#pragma unroll
      for (int g = 0; g < G; ++g) av[g] = av[g] * rp[0][g];
#pragma unroll
      for (int r = 0; r < RU; ++r) {
        const double mod = fma(sn[r], h[r].y, fma(sw[r], h[r].x, bg));
        const double t = fma(-mod, dw[r].y, dw[r].x);
        acc = act ? fma(t, t, acc) : acc;
      }
    };
    constexpr int BLK = 4;
    if (!WRITE && NT != 0 && rows % BLK == 0) {
      const int rstep = cw.S * n;
      const double2 *p = DW + cw.grp * n + jj;
      double2 cur[BLK], nxt[BLK];
      if constexpr (!HPF) {
        // the shape-table rows (wave-uniform broadcast reads) are read with their block;
        // only the cutout rows are prefetched a block ahead (16 VGPRs fewer)
        double2 hc[BLK];
#pragma unroll
        for (int k = 0; k < BLK; ++k) cur[k] = p[k * rstep];
        const int R = NT >= 64 ? NT : rows;
#pragma unroll 16
        for (int b0 = 0; b0 < R; b0 += BLK) {
          const bool more = b0 + BLK < R;
          const double2 *pn = p + (more ? BLK * rstep : 0);
#pragma unroll
          for (int k = 0; k < BLK; ++k) {
            hc[k] = hr[b0 + k];
            nxt[k] = pn[k * rstep];
          }
#pragma unroll
          for (int k = 0; k < BLK; k += RU) row4(hc + k, cur + k);
#pragma unroll
          for (int k = 0; k < BLK; ++k) cur[k] = nxt[k];
          p = pn;
        }
      } else {
        double2 hc[BLK], hn[BLK];
        // cutout row r of this lane's column.  The L2-resident cutout (n > 64) is read
        // through a buffer descriptor: the lane's column offset is a fixed VGPR and the
        // row offset a wave-uniform SGPR (SALU adds), where 64-bit flat addresses
        // took two VALU adds per row (~250 VALU per 128x128 walker-step)
        [[maybe_unused]] __amdgpu_buffer_rsrc_t rsrc;
        [[maybe_unused]] int voff = 0;
        if constexpr (NT > 64) {
          rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<double2 *>(DW), (short)0,
                                                   NT * NT * 16, 0x00020000);
          voff = (cw.grp * n + jj) * 16;
        }
        auto img = [&](int r) -> double2 {
          if constexpr (NT > 64) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, r * rstep * 16, 0);
            double2 d;
            __builtin_memcpy(&d, &v, 16);
            return d;
          } else {
            return p[r * rstep];
          }
        };
#pragma unroll
        for (int k = 0; k < BLK; ++k) {
          cur[k] = img(k);
          hc[k] = hr[k];
      }
      // n >= 64 (S = 1): rows = n is a compile-time count and the row loop is unrolled
      // (every LDS address an immediate offset, no loop counter): +3.6 %
      const int R = NT >= 64 ? NT : rows;
#pragma unroll 16
      for (int b0 = 0; b0 < R; b0 += BLK) {
        const bool more = b0 + BLK < R;
        const double2 *pn = p + (more ? BLK * rstep : 0);
        const int hb = more ? b0 + BLK : b0;
#pragma unroll
        for (int k = 0; k < BLK; ++k) {
          nxt[k] = NT > 64 ? img(hb + k) : pn[k * rstep];
          hn[k] = hr[hb + k];
        }
#pragma unroll
        for (int k = 0; k < BLK; k += RU) row4(hc + k, cur + k);
#pragma unroll
        for (int k = 0; k < BLK; ++k) {
          cur[k] = nxt[k];
          hc[k] = hn[k];
        }
        p = pn;
      }
      }
    } else {
      int k = 0;
#pragma unroll 2
      for (int i = cw.grp; i < n; i += cw.S, ++k)
        row(i, hr[k], WRITE ? make_double2(0.0, 0.0) : DW[i * n + jj]);
    }
  }
  wave_sync();   // the tables may be rewritten by the next step
  return acc;
}

// ---------------------------------------------------------------------------------
// Shared cutout ring of the 128x128 lockstep sampler (olpe_gibbs_kernel with RING).
// The 256 KiB {D/err, 1/err} cutout does not fit LDS, and read by every wave from L2
// it cost the sampler its latency.  So the WAVES waves of a workgroup
// sweep the cutout in lockstep and share one LDS ring of two phase slots (a phase is
// ROWS rows x 64 columns x 16 B; pass p covers columns 64p..64p+63), filled ahead by
// LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave-instruction, no VGPRs):
//   * a step's sweep is PHASES phases (2 column passes x 128/ROWS); the global phase
//     counter g advances identically in every wave, idle waves included;
//   * phase g lives in slot g % 2; at the start of phase g (begin_phase) every wave
//     drains its own DMAs and LDS reads (s_waitcnt vmcnt(0) lgkmcnt(0)), the workgroup
//     barriers, and then the DMA of phase g + 1 is issued into slot (g + 1) % 2 = the
//     slot of phase g - 1, whose rows every wave has in registers by then (a wave
//     reaches the barrier as it prefetches the first rows of phase g, while it computes
//     the last block of phase g - 1); rows r = wave (mod WAVES) are wave's share;
//   * so the DMA of phase g is issued at barrier g - 1 and drained before barrier g.
// The DMA is issued from inline asm: the compiler then inserts no vmcnt(0) before the
// issuing wave's next LDS reads (it cannot tell the ring slots apart), and its own
// counted waits stay correct because vector memory operations retire in order.

// (Windowed rings without barriers -- four and five slots of 16-row phases -- ran 6 %
// and 9 % slower; DESIGN_HISTORY.md §7.2, removed in round 4.)
template <int WAVES> struct LdsRing {
  static constexpr int ROWS = WAVES >= 8 ? 32 : 16;       // rows per phase
  static constexpr int SLOTS = 2, AHEAD = 1;              // ring slots; DMA lead in phases
  static constexpr int SLOT = ROWS * 64 * 16;
  static constexpr int BYTES = SLOTS * SLOT;
  static constexpr int PPP = 128 / ROWS;                  // phases per column pass
  static constexpr int PHASES = 2 * PPP;                  // phases per 128x128 sweep
  typedef __attribute__((address_space(3))) unsigned char lds_u8;

  const double2 *base;   // slot 0 (generic pointer into LDS, for the reads)
  unsigned lds;          // LDS byte address of slot 0 (M0 of the DMA)
  const double2 *DW;     // the cutout in global memory, [128][128]
  unsigned g;            // the phase begin_phase opens next (uniform)
  int wave;              // this wave's index in the workgroup (uniform)
  unsigned voff;         // lane * 16

  __device__ __forceinline__ void dma_row(int ph, int sl, int rr) const {
    // row rr of phase ph: cutout row ROWS (ph % PPP) + rr, columns 64 (ph / PPP) + lane
    const int row = (ph % PPP) * ROWS + rr;
    const double2 *src = DW + row * 128 + (ph / PPP) * 64;
    unsigned dst = lds + (unsigned)(sl * SLOT + rr * 1024);
    constexpr bool kFirstLane = WAVES != 12;
    if constexpr (kFirstLane) {
      // (the diagnostic 8-wave ring: the compiler loses the uniformity of the address
      // there; the 12-wave code is left exactly as it was)
      dst = (unsigned)__builtin_amdgcn_readfirstlane((int)dst);
      src = reinterpret_cast<const double2 *>(
          (((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane(
               (int)((unsigned long long)src >> 32)))
           << 32) |
          (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned long long)src));
    }
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %3\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(dst), "s"(src)
        : "memory");
  }
  // this wave's share of phase ph into slot sl
  __device__ __forceinline__ void dma_phase(int ph, int sl) const {
#pragma unroll
    for (int rr = 0; rr < ROWS; rr += WAVES)
      if (rr + wave < ROWS) dma_row(ph, sl, rr + wave);
  }
  // before the first phase: phase 0 into slot 0 (the workgroup barrier of the first
  // take_batch orders it before any wave's first phase)
  __device__ __forceinline__ void prologue(unsigned char *ring_lds, const double2 *dw, int w,
                                           int lane) {
    base = reinterpret_cast<const double2 *>(ring_lds);
    lds = (unsigned)(size_t)(lds_u8 *)ring_lds;
    DW = dw;
    wave = w;
    voff = (unsigned)lane * 16u;
    g = 0;
    dma_phase(0, 0);
  }
  // the barrier that opens phase g; returns phase g's slot
  __device__ __forceinline__ const double2 *begin_phase() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    dma_phase((int)((g + 1) % PHASES), (int)((g + 1) & 1));
    const double2 *p = base + (g & 1) * (SLOT / 16);
    ++g;
    return p;
  }
  // a step without a sweep of this wave's own (idle wave, or a fallback sweep that read
  // the cutout from global memory): the phases' barriers and DMA shares only
  __device__ __forceinline__ void idle_step() {
#pragma unroll 1
    for (int k = 0; k < PHASES; ++k) (void)begin_phase();
  }
};

// FAST3 sweep of a 128x128 cutout from the ring (sweep_fast3's NT > 64 form otherwise:
// column terms from the step's col_coef coefficients, four-row update, shape-table
// prefetch).  Two passes x 32 four-row blocks; a phase (four blocks) opens with
// begin_phase just before its first block is prefetched.
template <int NSRC, int WAVES>
__device__ __forceinline__ double sweep_fast3_ring(const ModelDesc<NSRC> &m, const double *htab,
                                                   int lane, ExpTab ex, const double *colc,
                                                   LdsRing<WAVES> &ring) {
  constexpr int G = 2 * NSRC;
  constexpr int BLK = 4, RU = 4, NB = 128 / BLK;    // 32 blocks per pass
  constexpr int BPP = LdsRing<WAVES>::ROWS / BLK;   // blocks per phase
  const double bg = m.bg;
  const double2 *hr = reinterpret_cast<const double2 *>(htab);
  double acc = 0.0;
  double rho0[G];                      // pass 0's rho (col_term64_pass1)
#pragma unroll 1
  for (int c0 = 0; c0 < 128; c0 += 64) {
    const double xj = (double)(c0 + lane);
    double av[G], rho[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const ColTerm t = c0 == 0 ? col_term64(m.g[g], colc + 3 * g, xj, ex)
                                : col_term64_pass1(m.g[g], colc + 3 * g, xj, rho0[g],
                                                   colc[3 * G + g], ex);
      av[g] = m.g[g].amp * t.E;
      rho[g] = t.R;
      rho0[g] = t.R;
      __builtin_amdgcn_sched_barrier(0);
    }
    double rp[RU][G];                  // rp[r] = rho^r, rp[0] = rho^4
#pragma unroll
    for (int g = 0; g < G; ++g) {
      rp[1][g] = rho[g];
      rp[2][g] = rho[g] * rho[g];
      rp[3][g] = rp[2][g] * rho[g];
      rp[0][g] = rp[2][g] * rp[2][g];
    }
    auto row4 = [&](const double2 *h, const double2 *dw) {
      double sw[RU], sn[RU];
      sw[0] = av[0];
      sn[0] = av[1];
#pragma unroll
      for (int s = 1; s < NSRC; ++s) {
        sw[0] = sw[0] + av[2 * s];
        sn[0] = sn[0] + av[2 * s + 1];
      }
#pragma unroll
      for (int r = 1; r < RU; ++r) {
        sw[r] = av[2 * NSRC - 2] * rp[r][2 * NSRC - 2];
        sn[r] = av[2 * NSRC - 1] * rp[r][2 * NSRC - 1];
#pragma unroll
        for (int s = NSRC - 2; s >= 0; --s) {
          sw[r] = fma(av[2 * s], rp[r][2 * s], sw[r]);
          sn[r] = fma(av[2 * s + 1], rp[r][2 * s + 1], sn[r]);
        }
      }
#pragma unroll
      for (int g = 0; g < G; ++g) av[g] = av[g] * rp[0][g];
#pragma unroll
      for (int r = 0; r < RU; ++r) {
        const double mod = fma(sn[r], h[r].y, fma(sw[r], h[r].x, bg));
        const double t = fma(-mod, dw[r].y, dw[r].x);
        acc = fma(t, t, acc);
      }
    };
    // rows of block b (0..31) of this pass: slot row (4b) % 16 of the phase's slot
    const double2 *sp = ring.begin_phase();
    double2 cur[BLK], nxt[BLK], hc[BLK];
#pragma unroll
    for (int k = 0; k < BLK; ++k) cur[k] = sp[k * 64 + lane];
#pragma unroll BPP
    for (int b = 0; b < NB; ++b) {
      // one block ahead only: without the fences the compiler gathers a whole phase's
      // ring reads (64 VGPRs) ahead of its arithmetic and spills
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      // the shape-table rows (wave-uniform broadcasts) are read with their block
#pragma unroll
      for (int k = 0; k < BLK; ++k) hc[k] = hr[b * BLK + k];
      if (b + 1 < NB) {
        const int nb = b + 1;
        if (nb % BPP == 0) sp = ring.begin_phase();   // the next phase opens
        const int r0 = (nb % BPP) * BLK;
#pragma unroll
        for (int k = 0; k < BLK; ++k) nxt[k] = sp[(r0 + k) * 64 + lane];
      }
      row4(hc, cur);
      // the block's arithmetic completes here (machine sinking would otherwise gather
      // a phase's four blocks behind its loads)
      asm volatile("" : "+v"(acc));
#pragma unroll
      for (int k = 0; k < BLK; ++k) cur[k] = nxt[k];
    }
  }
  return acc;
}

// FAST kernels keep the exact sweep only as the (rare) fallback, unrolled once so
// that it does not set the kernel's register budget.
// After an accepted step: refresh the cached column terms of the Gaussians the step
// changed from the new state's descriptor.
template <int NSRC, int NT>
__device__ __forceinline__ void colcache_accept(ColCache<2 * NSRC> &cc, const ModelDesc<NSRC> &m,
                                                unsigned gmask, int lane, const double *etab) {
  const ColWalk cw(NT, lane);
  const int rows0 = (NT + cw.S - 1) / cw.S;
  const double kcd = (double)(rows0 / 2);
  const bool parked = cc.pbuf && cc.pend == gmask;   // this step's FAST3 setup ran
#pragma unroll
  for (int g = 0; g < 2 * NSRC; ++g) {
    if ((gmask >> g) & 1u) {
      if (parked) {
        const int slot = __builtin_popcount(gmask & ((1u << g) - 1u));
        cc.E[g] = cc.pbuf[(2 * slot) * 64 + lane];
        cc.R[g] = cc.pbuf[(2 * slot + 1) * 64 + lane];
      } else {
        ColTerm t;
        if constexpr (NT == 64)
          t = col_term64(m.g[g], cc.colc + 3 * g, (double)cw.jl, ExpTab{etab});
        else
          t = col_term(m.g[g], (double)cw.jl, (double)cw.grp, (double)cw.S, kcd, ExpTab{etab});
        cc.E[g] = t.E;
        cc.R[g] = t.R;
      }
      cc.valid |= 1u << g;
    }
  }
  cc.pend = 0;
}

template <int NSRC, int NT, bool WRITE, bool FAST, bool WIDE = false, class RingT = LdsRing<12>>
__device__ __forceinline__ double sweep(const ModelDesc<NSRC> &m, const double2 *img,
                                        double *vtab, double *out, int n, int lane,
                                        const double *etab, HCache *hc = nullptr,
                                        ColCache<2 * NSRC> *cc = nullptr, unsigned gmask = 0,
                                        GuardCache *gc = nullptr, RingT *ring = nullptr) {
  // img is {D, 1/err} for EXACT kernels and {D/err, 1/err} for FAST kernels
  if constexpr (FAST) {
    const int nn = NT ? NT : n;
    const ColWalk cw(nn, lane);
    const int rows = (nn - cw.grp + cw.S - 1) / cw.S;    // uniform when S divides n
    const int rows0 = (nn + cw.S - 1) / cw.S;             // rows of row group 0 (most)
    const int kc = rows0 / 2;
    // the moved Gaussians' column terms first: their exp chains and the guard's form
    // one scheduling region (single-pass sampler kernels, which always pass cc)
    MovedTerms<NSRC> pre;
    if constexpr (NT != 0 && NT <= 64)
      moved_terms<NSRC, NT>(pre, m, gmask, nn, lane, kc, ExpTab{etab}, cc->colc);
    bool ok3;
    // the per-column guard only where the whole-grid one can fail on a well-placed
    // model (cutouts wider than 64 columns), and only for the Gaussians that failed
    // it (the 3-source 128x128 bench model: 2 of 6); at n <= 64 it would cost the
    // sampler registers for a branch the bench never takes
    if constexpr (NT == 0 || NT > 64) {
      const unsigned fails = fast3_fails<NSRC>(m, nn, rows0, kc, lane);
      ok3 = fails == 0;
      if (!ok3) {
        asm volatile("" ::: "memory");
        if (gc) {
          // per Gaussian: the column test's result for an unchanged Gaussian is reused
          const unsigned keep = gc->colok & ~gc->changed;
          const unsigned need = fails & ~keep;
          const unsigned passed = need ? fast3_cols_pass<NSRC>(m, nn, rows0, kc, lane, need) : 0u;
          gc->coltest = passed;
          gc->colprop = keep | passed;
          ok3 = (fails & ~(keep | passed)) == 0 && fast3_amp_ok<NSRC>(m, lane, fails);
        } else {
          ok3 = fast3_ok_cols<NSRC>(m, nn, rows0, kc, lane, fails);
        }
      } else if (gc) {
        gc->coltest = 0;
        gc->colprop = gc->colok & ~gc->changed;
      }
    } else {
      if (gc && gc->same && gc->valid) ok3 = gc->cur;
      else ok3 = fast3_ok<NSRC>(m, nn, rows0, kc, lane);
      if (gc) gc->prop = ok3;
    }
    asm volatile("" ::: "memory");
    if (ok3) {
      const int tw = 2 * rows0;                            // doubles per slot
      const double *h;
      if (!hc) {
        build_htab<NSRC>(m, vtab, vtab, 3, rows0, kc, (double)cw.S, lane, ExpTab{etab});
        h = vtab;
      } else if (hc->single) {
        // in place: this step's set (the proposal's) and the sets left stale by earlier
        // steps (a rejected proposal's, or the state's before an accepted step that took
        // another sweep); the other set stays
        const int need = (hc->valid ? hc->stale : 3) | (hc->grp ? (hc->grp == 1 ? 2 : 1) : 0);
        if (need)
          build_htab<NSRC>(m, vtab, vtab, need, rows0, kc, (double)cw.S, lane, ExpTab{etab});
        hc->valid = 1;
        hc->stale = 0;
        hc->flip = hc->grp != 0;
        h = vtab;
      } else if (hc->grp == 0) {
        if (!hc->valid) {
          build_htab<NSRC>(m, vtab + hc->cur * tw, vtab, 3, rows0, kc, (double)cw.S, lane, ExpTab{etab});
          hc->valid = true;
        }
        h = vtab + hc->cur * tw;
      } else {
        double *dst = vtab + (hc->cur ^ 1) * tw;
        build_htab<NSRC>(m, dst, vtab + hc->cur * tw, hc->valid ? (hc->grp == 1 ? 2 : 1) : 3,
                         rows0, kc, (double)cw.S, lane, ExpTab{etab});
        hc->flip = true;
        h = dst;
      }
      asm volatile("" ::: "memory");
      if constexpr (NT != 0 && NT <= 64) {
        if (cc)
          return sweep_fast3<NSRC, NT, WRITE, true, WIDE>(m, img, h, out, n, lane, rows, kc,
                                                          ExpTab{etab}, cc, gmask, &pre);
      }
      if constexpr (NT == 128 && !WRITE) {
        if (ring) return sweep_fast3_ring<NSRC>(m, h, lane, ExpTab{etab}, cc->colc, *ring);
      }
      return sweep_fast3<NSRC, NT, WRITE, false, WIDE>(m, img, h, out, n, lane, rows, kc,
                                                       ExpTab{etab}, cc);
    }
    const int lvl = fast_level<NSRC>(m, nn);
    // the descriptor lives in LDS: make the sweeps reload the fields they use instead
    // of keeping the guard's loads live (and spilled) across the row loop
    asm volatile("" ::: "memory");
    double part;
    if (lvl == 2) {
      part = sweep_fast2<NSRC, NT, WRITE>(m, img, out, n, lane);
    } else if (lvl == 1 && !(NSRC == 3 && NT == 64) && !ring && !(hc && hc->single)) {
      // (the 3-source 64x64 sampler and the ring sampler have no room for the V table:
      // sampler_vtab_bytes)
      if (hc) hc->valid = false;                           // the V table overwrites vtab
      part = sweep_fast<NSRC, NT, WRITE>(m, img, vtab, out, n, lane);
    } else {
      part = sweep_exact_dw<NSRC, NT, WRITE>(m, img, out, n, lane);
    }
    // the ring sampler's fallbacks read the cutout from global memory; the step still
    // keeps the workgroup's phase barriers and this wave's DMA shares
    if (ring) ring->idle_step();
    return part;
  } else {
    // the EXACT samplers' row tables (olpe.hip checks the sizes): the column-term
    // parking area (cc->pbuf, NSRC KiB; at n = 128 it holds the draw tables) and the V
    // table area (vtab), both otherwise unused in EXACT
    if constexpr (!WRITE && NT == 64 && NSRC == 2) {
      if (cc) return sweep_exact_rows<NSRC, 64, true>(m, img, lane, cc->pbuf, vtab);
    } else if constexpr (!WRITE && NT == 64) {
      if (cc) return sweep_exact_rows<NSRC, 64, false>(m, img, lane, nullptr, cc->pbuf);
    } else if constexpr (!WRITE && NT == 32) {
      if (cc) return sweep_exact_rows<NSRC, 32, true>(m, img, lane, cc->pbuf, cc->pbuf + 32 * 2 * NSRC);
    } else if constexpr (!WRITE && NT == 128) {
      if (cc) return sweep_exact_rows<NSRC, 128, false>(m, img, lane, nullptr, vtab);
    }
    return sweep_exact<NSRC, NT, WRITE, 2>(m, img, out, n, lane);
  }
}

}  // namespace olpe
