// olpe_moments.hip -- whole-run posterior moments of the recorded chains, on the device
// (the step-3 Gelman-Rubin / posterior summary without
// gathering the chains).
//
// Step 3 reads every walker's chain file (apf_step3.py:169-186) and reduces it to
// per-parameter means, sigmas and the Gelman-Rubin PSRF / RC (:258-278), which need,
// per walker w and column k, only the walker's mean and sum of squared deviations over
// its N rows (np.mean(p[:, i]), np.std(p[:, i])**2 * N) and the pooled mean.  So each
// context keeps, per walker and column, a running (mean, M2) of every row it recorded:
//   * olpe_moments_accumulate folds the last launch's chain rows in -- one thread per
//     (walker, column), one pass over the launch's rows in blocks of 8 (each block's
//     mean about its first row, then the squared deviations about that mean, in
//     registers), merged into the running pair with Chan et al.'s update (delta =
//     mean_b - mean_a; M2 += M2_b + delta^2 n_a n_b / n), so no sum of squares ever
//     cancels;
//   * olpe_moments_summary reduces the walkers of this context (two-stage, fixed order,
//     deterministic) to per-column sums of the means, of M2 and of the squared
//     deviations of the means about a given centre, plus the tries / accepts totals;
//   * olpe_comm_allreduce_moments (olpe_comm.hip) runs the summary twice over RCCL:
//     the pooled mean first, then the deviations about it.
// Device layout: mean / M2 as [PS][W] (the summary's reads are contiguous per column).
#include <hip/hip_runtime.h>

#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/olpe.h"
#include "olpe_internal.h"

using olpe::set_err;

namespace {

#define HIPCHK(expr)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return set_err(OLPE_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_));         \
  } while (0)

constexpr int kThreads = 256;
constexpr int kWalkersPerBlock = 256;    // summary stage 1: walkers per block

// fold the launch's rows chain[W][nrec][ps] into the running (mean, M2) [ps][W].
// One wave per walker: lane l = g * ps + k (g < G = 64 / ps row groups, 3 for 17 or 20
// columns) reads column k of rows g, g + G, g + 2G, ..., so each load instruction of the
// wave reads G consecutive rows -- G * ps * 8 contiguous bytes -- and a lane keeps
// kWaveRows loads in flight (one pass over HBM, each walker's rows streamed in order).
// (Round 3's kernel ran one thread per (walker, column): a wave's loads then touched
// four walkers 136 KB apart at stride 1, 3.4 TB/s on configs[1]'s 557 MB of rows.)  A
// lane's rows are taken in blocks of kWaveRows held in registers, each block's (mean,
// M2) formed by two passes over the registers (mean about its first value, then the
// squared deviations about that mean) and merged into the lane's running pair with
// Chan's update; the G row groups are then merged across lanes the same way, and the
// walker's pair merged into the running moments -- the two-pass arithmetic without a
// second read of the rows.
constexpr int kFoldRows = 8;
constexpr int kFoldWaves = 4;            // walkers (waves) per fold block
constexpr int kWaveRows = 16;            // loads in flight per lane (rows per block)
// launches of fewer rows per walker fold one thread per (walker, column) instead
// (fold_cols_kernel): a wave per walker has too little to read there (configs[2]'s 10
// rows: 48 us against 30 us per launch)
constexpr long long kFoldRowsMin = 64;

__device__ __forceinline__ void chan_merge(double &m, double &q, double &n, double mb,
                                           double qb, double nb) {
  if (nb == 0.0) return;
  if (n == 0.0) {
    m = mb;
    q = qb;
    n = nb;
    return;
  }
  const double nn = n + nb;
  const double delta = mb - m;
  m = m + delta * (nb / nn);
  q = q + qb + (delta * delta) * (n * nb / nn);
  n = nn;
}

__global__ __launch_bounds__(64 * kFoldWaves) void fold_rows_kernel(
    const double *__restrict__ chain, long long W, int ps, long long nrec, double n_a,
    double *__restrict__ mean, double *__restrict__ m2) {
  const int lane = threadIdx.x & 63;
  const long long w = (long long)blockIdx.x * kFoldWaves + (threadIdx.x >> 6);
  if (w >= W) return;                      // (whole waves: w is wave-uniform)
  const int G = 64 / ps;
  const int g = lane / ps;
  const int k = lane - g * ps;
  const bool act = g < G;
  const double *x = chain + (size_t)w * nrec * ps + (act ? g * ps + k : 0);
  const long long step = (long long)G * ps;           // doubles per row-group step
  double m = 0.0, q = 0.0, n = 0.0;
  for (long long r0 = 0; r0 < nrec; r0 += (long long)G * kWaveRows) {
    double v[kWaveRows];
    int nb = 0;
#pragma unroll
    for (int i = 0; i < kWaveRows; ++i) {
      const bool ok = act && r0 + g + (long long)i * G < nrec;
      v[i] = ok ? x[(size_t)(r0 / G) * step + (size_t)i * step] : 0.0;
      nb += ok ? 1 : 0;
    }
    if (nb == 0) continue;
    const double c = v[0];
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < kWaveRows; ++i) s += i < nb ? v[i] - c : 0.0;
    const double fb = (double)nb;
    const double mb = c + s / fb;
    double qb = 0.0;
#pragma unroll
    for (int i = 0; i < kWaveRows; ++i) {
      const double d = v[i] - mb;
      qb = i < nb ? fma(d, d, qb) : qb;
    }
    chan_merge(m, q, n, mb, qb, fb);
  }
  // the row groups of each column into group 0 (lane k), in group order
  for (int h = 1; h < G; ++h) {
    const int src = k + h * ps;
    const double mh = __shfl(m, src), qh = __shfl(q, src), nh = __shfl(n, src);
    if (g == 0) chan_merge(m, q, n, mh, qh, nh);
  }
  if (g != 0) return;
  const size_t o = (size_t)k * W + w;
  if (n_a == 0.0) {
    mean[o] = m;
    m2[o] = q;
    return;
  }
  double ma = mean[o], qa = m2[o], na = n_a;
  chan_merge(ma, qa, na, m, q, n);
  mean[o] = ma;
  m2[o] = qa;
}

// one thread t = w * ps + k per (walker, column), rows in blocks of kFoldRows (round 3's
// fold; kept for short launches)
__global__ __launch_bounds__(kThreads) void fold_cols_kernel(const double *__restrict__ chain,
                                                        long long W, int ps, long long nrec,
                                                        double n_a, double *__restrict__ mean,
                                                        double *__restrict__ m2) {
  const long long t = (long long)blockIdx.x * kThreads + threadIdx.x;
  if (t >= W * ps) return;
  const long long w = t / ps;
  const int k = (int)(t - w * ps);
  const double *x = chain + (size_t)w * nrec * ps + k;
  double m = 0.0, q = 0.0, n = 0.0;
  for (long long r0 = 0; r0 < nrec; r0 += kFoldRows) {
    const int nb = nrec - r0 < kFoldRows ? (int)(nrec - r0) : kFoldRows;
    double v[kFoldRows];
#pragma unroll
    for (int i = 0; i < kFoldRows; ++i) v[i] = i < nb ? x[(size_t)(r0 + i) * ps] : 0.0;
    const double c = v[0];
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < kFoldRows; ++i) s += i < nb ? v[i] - c : 0.0;
    const double fb = (double)nb;
    const double mb = c + s / fb;
    double qb = 0.0;
#pragma unroll
    for (int i = 0; i < kFoldRows; ++i) {
      const double d = v[i] - mb;
      qb = i < nb ? fma(d, d, qb) : qb;
    }
    chan_merge(m, q, n, mb, qb, fb);
  }
  const size_t o = (size_t)k * W + w;
  if (n_a == 0.0) {
    mean[o] = m;
    m2[o] = q;
    return;
  }
  double ma = mean[o], qa = m2[o], na = n_a;
  chan_merge(ma, qa, na, m, q, n);
  mean[o] = ma;
  m2[o] = qa;
}

__device__ double block_sum(double v, double *red) {
  red[threadIdx.x] = v;
  __syncthreads();
  for (int o = kThreads / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

// stage 1: block b reduces walkers [b*kWalkersPerBlock, ...) of every column into
// part[q][col][b], q = 0: sum of means, 1: sum of M2, 2: sum of (mean - centre)^2
// (centre may be NULL: block 2 is then 0), 3 / 4: tries / accepts (np columns)
__global__ __launch_bounds__(kThreads) void summary_stage1(
    const double *__restrict__ mean, const double *__restrict__ m2,
    const double *__restrict__ centre, const uint32_t *__restrict__ tries,
    const uint32_t *__restrict__ acc, long long W, int ps, int np, int nblk,
    double *__restrict__ part) {
  __shared__ double red[kThreads];
  __shared__ unsigned long long cnt[2 * 32];
  const int b = blockIdx.x;
  const long long w0 = (long long)b * kWalkersPerBlock;
  const long long w1 = w0 + kWalkersPerBlock < W ? w0 + kWalkersPerBlock : W;
  for (int k = 0; k < ps; ++k) {
    const double *mk = mean + (size_t)k * W, *qk = m2 + (size_t)k * W;
    const double ck = centre ? centre[k] : 0.0;
    double a = 0.0, q = 0.0, d2 = 0.0;
    for (long long w = w0 + threadIdx.x; w < w1; w += kThreads) {
      const double m = mk[w];
      a += m;
      q += qk[w];
      const double d = m - ck;
      d2 = fma(d, d, d2);
    }
    a = block_sum(a, red);
    q = block_sum(q, red);
    d2 = block_sum(d2, red);
    if (threadIdx.x == 0) {
      part[((size_t)0 * ps + k) * nblk + b] = a;
      part[((size_t)1 * ps + k) * nblk + b] = q;
      part[((size_t)2 * ps + k) * nblk + b] = centre ? d2 : 0.0;
    }
  }
  // tries / accepts [W][np] (integer sums: exact whatever the order)
  for (int i = threadIdx.x; i < 2 * np; i += kThreads) cnt[i] = 0;
  __syncthreads();
  const size_t e0 = (size_t)w0 * np, e1 = (size_t)w1 * np;
  for (size_t e = e0 + threadIdx.x; e < e1; e += kThreads) {
    const int k = (int)(e % (size_t)np);
    atomicAdd(&cnt[k], (unsigned long long)tries[e]);
    atomicAdd(&cnt[np + k], (unsigned long long)acc[e]);
  }
  __syncthreads();
  double *pc = part + (size_t)3 * ps * nblk;
  for (int i = threadIdx.x; i < 2 * np; i += kThreads) pc[(size_t)i * nblk + b] = (double)cnt[i];
}

// stage 2: one block per output column, the blocks' partials in a fixed order
__global__ __launch_bounds__(kThreads) void summary_stage2(const double *__restrict__ part,
                                                           int nblk, double *__restrict__ out) {
  __shared__ double red[kThreads];
  const double *p = part + (size_t)blockIdx.x * nblk;
  double a = 0.0;
  for (int b = threadIdx.x; b < nblk; b += kThreads) a += p[b];
  a = block_sum(a, red);
  if (threadIdx.x == 0) out[blockIdx.x] = a;
}

int ensure_moments(olpe_ctx *c) {
  const size_t need = (size_t)c->W * c->ps;
  if (c->d_mmean && c->mom_cap >= need) return OLPE_OK;
  if (c->d_mmean) (void)hipFree(c->d_mmean);
  if (c->d_mm2) (void)hipFree(c->d_mm2);
  c->d_mmean = c->d_mm2 = nullptr;
  c->mom_cap = 0;
  if (hipMalloc((void **)&c->d_mmean, need * sizeof(double)) != hipSuccess ||
      hipMalloc((void **)&c->d_mm2, need * sizeof(double)) != hipSuccess) {
    if (c->d_mmean) (void)hipFree(c->d_mmean);
    c->d_mmean = nullptr;
    return set_err(OLPE_ENOMEM, "hipMalloc(%zu bytes) for the walker moments", 2 * need * 8);
  }
  c->mom_cap = need;
  return OLPE_OK;
}

}  // namespace

// Everything olpe_moments_local needs besides its launches: the partials buffer, the
// moments themselves and (nothing folded yet) their zeroing.  The moments all-reduce
// calls it before its uniformity check, so that a rank that cannot prepare says so in
// that check instead of skipping the all-reduces its peers enter (olpe_comm.hip).
int olpe_moments_prepare(olpe_ctx *c) {
  if (c->mom_fault == 1)
    return set_err(OLPE_ENOMEM, "moment partials: allocation failure forced (olpe_moments_fault)");
  const int nblk = (int)((c->W + kWalkersPerBlock - 1) / kWalkersPerBlock);
  const size_t need = ((size_t)3 * c->ps + 2 * c->np) * nblk;
  if (need > c->mpart_cap) {
    if (c->d_mpart) (void)hipFree(c->d_mpart);
    c->d_mpart = nullptr;
    c->mpart_cap = 0;
    if (hipMalloc((void **)&c->d_mpart, need * sizeof(double)) != hipSuccess) {
      c->d_mpart = nullptr;
      (void)hipGetLastError();
      return set_err(OLPE_ENOMEM, "hipMalloc(%zu bytes) for the moment partials", need * 8);
    }
    c->mpart_cap = need;
  }
  int rc;
  if ((rc = ensure_moments(c))) return rc;
  if (c->mom_n == 0) {      // nothing folded yet: zero means / M2 (the sums are 0)
    HIPCHK(hipMemsetAsync(c->d_mmean, 0, (size_t)c->W * c->ps * 8, c->stream));
    HIPCHK(hipMemsetAsync(c->d_mm2, 0, (size_t)c->W * c->ps * 8, c->stream));
  }
  return OLPE_OK;
}

// the local summary into the device buffer d_out [OLPE_MOMENTS_LEN] (async on the
// context's stream; d_centre: device [ps] or NULL); n and W are filled in by the host.
// Launches only: olpe_moments_prepare must have succeeded.
int olpe_moments_local(olpe_ctx *c, const double *d_centre, double *d_out) {
  if (c->mom_fault == 2)
    return set_err(OLPE_EHIP, "moments summary launch: failure forced (olpe_moments_fault)");
  const int nblk = (int)((c->W + kWalkersPerBlock - 1) / kWalkersPerBlock);
  const size_t cols = (size_t)3 * c->ps + 2 * c->np;
  if (!c->d_mpart || c->mpart_cap < cols * nblk || !c->d_mmean)
    return set_err(OLPE_ESTATE, "moments summary before its buffers were prepared");
  hipLaunchKernelGGL(summary_stage1, dim3(nblk), dim3(kThreads), 0, c->stream, c->d_mmean,
                     c->d_mm2, d_centre, c->d_tries, c->d_acc, (long long)c->W, c->ps, c->np,
                     nblk, c->d_mpart);
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(summary_stage2, dim3((unsigned)cols), dim3(kThreads), 0, c->stream,
                     c->d_mpart, nblk, d_out + 2);
  HIPCHK(hipGetLastError());
  return OLPE_OK;
}

extern "C" {

int olpe_moments_fault(olpe_ctx *c, int where) {
  if (!c || where < 0 || where > 4) return set_err(OLPE_EINVAL, "bad argument");
  c->mom_fault = where;
  return OLPE_OK;
}

int olpe_moments_accumulate(olpe_ctx *c) {
  if (!c) return set_err(OLPE_EINVAL, "NULL ctx");
  if (!c->d_state || !c->launches) return set_err(OLPE_ESTATE, "no sampler launch yet");
  if (c->mom_folded == c->launches)
    return set_err(OLPE_ESTATE, "the last launch's rows are already in the moments");
  HIPCHK(hipSetDevice(c->device));
  int rc;
  if ((rc = ensure_moments(c))) return rc;
  c->mom_folded = c->launches;
  const long long nrec = c->chain_rows;
  if (nrec == 0) return OLPE_OK;
  if (nrec >= kFoldRowsMin && c->ps <= 64) {
    hipLaunchKernelGGL(fold_rows_kernel, dim3((unsigned)((c->W + kFoldWaves - 1) / kFoldWaves)),
                       dim3(64 * kFoldWaves), 0, c->stream, c->d_chain, (long long)c->W, c->ps,
                       nrec, (double)c->mom_n, c->d_mmean, c->d_mm2);
  } else {
    const long long total = (long long)c->W * c->ps;
    hipLaunchKernelGGL(fold_cols_kernel, dim3((unsigned)((total + kThreads - 1) / kThreads)),
                       dim3(kThreads), 0, c->stream, c->d_chain, (long long)c->W, c->ps, nrec,
                       (double)c->mom_n, c->d_mmean, c->d_mm2);
  }
  HIPCHK(hipGetLastError());
  c->mom_n += nrec;
  return OLPE_OK;
}

int olpe_moments_reset(olpe_ctx *c) {
  if (!c) return set_err(OLPE_EINVAL, "NULL ctx");
  c->mom_n = 0;
  c->mom_folded = c->launches;
  return OLPE_OK;
}

int olpe_moments_get(olpe_ctx *c, long long *n, double *mean, double *m2) {
  if (!c || !n) return set_err(OLPE_EINVAL, "NULL argument");
  if (!c->d_state) return set_err(OLPE_ESTATE, "no ensemble");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  *n = c->mom_n;
  const size_t m = (size_t)c->W * c->ps;
  std::vector<double> t(m, 0.0);
  double *outs[2] = {mean, m2};
  double *devs[2] = {c->d_mmean, c->d_mm2};
  for (int i = 0; i < 2; ++i) {
    if (!outs[i]) continue;
    if (c->mom_n && devs[i]) {
      HIPCHK(hipMemcpy(t.data(), devs[i], m * 8, hipMemcpyDeviceToHost));
    } else {
      std::fill(t.begin(), t.end(), 0.0);
    }
    for (int w = 0; w < c->W; ++w)             // [ps][W] -> [W][ps]
      for (int k = 0; k < c->ps; ++k) outs[i][(size_t)w * c->ps + k] = t[(size_t)k * c->W + w];
  }
  return OLPE_OK;
}

int olpe_moments_set(olpe_ctx *c, long long n, const double *mean, const double *m2) {
  if (!c || n < 0 || (n > 0 && (!mean || !m2))) return set_err(OLPE_EINVAL, "bad argument");
  if (!c->d_state) return set_err(OLPE_ESTATE, "call olpe_seed first");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  int rc;
  if ((rc = ensure_moments(c))) return rc;
  const size_t m = (size_t)c->W * c->ps;
  if (n > 0) {
    std::vector<double> t(m);
    const double *ins[2] = {mean, m2};
    double *devs[2] = {c->d_mmean, c->d_mm2};
    for (int i = 0; i < 2; ++i) {
      for (int w = 0; w < c->W; ++w)
        for (int k = 0; k < c->ps; ++k) t[(size_t)k * c->W + w] = ins[i][(size_t)w * c->ps + k];
      HIPCHK(hipMemcpy(devs[i], t.data(), m * 8, hipMemcpyHostToDevice));
    }
  }
  c->mom_n = n;
  c->mom_folded = c->launches;
  return OLPE_OK;
}

int olpe_moments_summary(olpe_ctx *c, const double *centre, double *out) {
  if (!c || !out) return set_err(OLPE_EINVAL, "NULL argument");
  if (!c->d_state) return set_err(OLPE_ESTATE, "no ensemble");
  HIPCHK(hipSetDevice(c->device));
  const size_t len = (size_t)OLPE_MOMENTS_LEN(c->ps, c->np);
  double *d = nullptr;
  HIPCHK(hipMalloc((void **)&d, (len + c->ps) * sizeof(double)));
  double *dc = nullptr;
  hipError_t e = hipSuccess;
  if (centre) {
    dc = d + len;
    e = hipMemcpyAsync(dc, centre, c->ps * sizeof(double), hipMemcpyHostToDevice, c->stream);
  }
  int rc = e == hipSuccess ? olpe_moments_prepare(c) : OLPE_OK;
  if (e == hipSuccess && rc == OLPE_OK) rc = olpe_moments_local(c, dc, d);
  if (e == hipSuccess && rc == OLPE_OK)
    e = hipMemcpyAsync(out, d, len * sizeof(double), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess && rc == OLPE_OK) e = hipStreamSynchronize(c->stream);
  (void)hipFree(d);
  if (rc) return rc;
  if (e != hipSuccess) return set_err(OLPE_EHIP, "moments summary: %s", hipGetErrorString(e));
  out[0] = (double)c->mom_n;
  out[1] = (double)c->W;
  return OLPE_OK;
}

}  // extern "C"
