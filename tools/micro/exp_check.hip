// exp_neg (olpe_device.h, the EXACT sweeps' exp) against ocml's exp(-q), bit for bit.
// Arguments: a dense sweep of [0, 1100] (the sampler's range and past the underflow
// point), random bit patterns of positive doubles, the neighbourhoods of the range
// edges, and the specials (0, -0, +inf, NaN, tiny negatives).  Prints the mismatch count
// and the first few mismatches; exit status 1 on any.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I olpefit_amd/csrc \
//         -o tools/micro/exp_check tools/micro/exp_check.hip && tools/micro/exp_check
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>
#include "olpe_device.h"

__global__ void check(const double *q, unsigned long long *ref, unsigned long long *got,
                      long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double x = q[i];
  ref[i] = (unsigned long long)__double_as_longlong(exp(-x));
  got[i] = (unsigned long long)__double_as_longlong(olpe::exp_neg(x));
}

static double bits(unsigned long long u) {
  double d;
  std::memcpy(&d, &u, 8);
  return d;
}

int main() {
  std::vector<double> q;
  const long long dense = 1 << 22;
  for (long long i = 0; i < dense; ++i) q.push_back(1100.0 * (double)i / (double)dense);
  unsigned long long s = 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < (1 << 22); ++i) {          // random positive doubles, all exponents
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    q.push_back(bits(s & 0x7fffffffffffffffull));
  }
  for (int i = 0; i < (1 << 20); ++i) {          // random in [0, 800) at full precision
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    q.push_back(800.0 * (double)(s >> 11) * 0x1p-53);
  }
  const double edges[] = {708.3964185322641, 709.782712893384, 745.1332191019411,
                          745.1332191019412, 1000.0, 0.5 * 0.6931471805599453};
  for (double e : edges)
    for (int k = -2000; k <= 2000; ++k) q.push_back(std::nextafter(e, k < 0 ? 0.0 : 2e3) +
                                                    (double)k * 1e-13 * e);
  const double specials[] = {0.0, -0.0, INFINITY, NAN, -NAN, 1e-300, -1e-300, -1e-12,
                             -1e-6, -0.3, 4.9e-324, 1e300, 1e308};
  for (double e : specials) q.push_back(e);
  const long long n = (long long)q.size();

  double *dq;
  unsigned long long *dref, *dgot;
  if (hipMalloc(&dq, n * 8) || hipMalloc(&dref, n * 8) || hipMalloc(&dgot, n * 8)) return 2;
  if (hipMemcpy(dq, q.data(), n * 8, hipMemcpyHostToDevice)) return 2;
  hipLaunchKernelGGL(check, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, dq, dref, dgot, n);
  if (hipDeviceSynchronize()) return 2;
  std::vector<unsigned long long> ref(n), got(n);
  if (hipMemcpy(ref.data(), dref, n * 8, hipMemcpyDeviceToHost) ||
      hipMemcpy(got.data(), dgot, n * 8, hipMemcpyDeviceToHost)) return 2;
  long long bad = 0, bad_nan = 0;
  for (long long i = 0; i < n; ++i) {
    if (ref[i] == got[i]) continue;
    const bool both_nan = std::isnan(bits(ref[i])) && std::isnan(bits(got[i]));
    if (both_nan) { ++bad_nan; continue; }   // NaN payloads may differ; NaN stays NaN
    if (bad < 12)
      std::printf("q = %a (%.17g): ocml %a, exp_neg %a\n", q[i], q[i], bits(ref[i]),
                  bits(got[i]));
    ++bad;
  }
  std::printf("exp_check: %lld arguments, %lld mismatches (%lld NaN-payload only)\n", n,
              bad, bad_nan);
  return bad ? 1 : 0;
}
