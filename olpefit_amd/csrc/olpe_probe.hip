// olpe_probe.hip -- the core clock the chip holds behind a stream's work (olpe_clock_probe).
//
// MI355X runs its FP64 VALU stream below the 2.4 GHz spec clock (power-limited DVFS,
// MI355X_MICROARCH.md 'DVFS give-back'), by an amount that differs from box to box; the
// bench reports its roofline fraction against the spec peak and against the clock
// measured here.  One wave counts core cycles (s_memtime) over 2,000 ticks of the
// 100 MHz reference (s_memrealtime), 20 us: queued right behind sampler launches it
// reads the clock of their load, which the power controller changes only over
// milliseconds.  A kernel of its own in a source of its own, so that the sampler's code
// object carries no stamps and keeps its digest.
#include <hip/hip_runtime.h>

#include "../../include/olpe.h"
#include "olpe_internal.h"

using olpe::set_err;

#define HIPCHK(expr)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return set_err(OLPE_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_));         \
  } while (0)

namespace {

__global__ __launch_bounds__(64) void clock_probe_kernel(unsigned long long *out) {
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = r0, c1 = c0;
  while (r1 - r0 < 2000) {
    __builtin_amdgcn_s_sleep(1);
    r1 = __builtin_amdgcn_s_memrealtime();
    c1 = __builtin_amdgcn_s_memtime();
  }
  if (threadIdx.x == 0) {      // (vector stores of one lane)
    out[0] = r0;
    out[1] = c0;
    out[2] = r1;
    out[3] = c1;
  }
}

}  // namespace

extern "C" int olpe_clock_probe(olpe_ctx *c, double *ghz) {
  if (!c || !ghz) return set_err(OLPE_EINVAL, "NULL argument");
  if (!c->d_clk) return set_err(OLPE_ESTATE, "no device buffers");
  HIPCHK(hipSetDevice(c->device));
  hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, c->stream, c->d_clk);
  HIPCHK(hipGetLastError());
  unsigned long long v[4] = {0, 0, 0, 0};
  HIPCHK(hipMemcpyAsync(v, c->d_clk, sizeof(v), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  // core cycles per 100 MHz tick x 0.1 = GHz
  *ghz = v[2] > v[0] ? (double)(v[3] - v[1]) / (double)(v[2] - v[0]) * 0.1 : 0.0;
  return OLPE_OK;
}
