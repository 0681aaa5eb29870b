// Microbenchmark: VALU issue rates per SIMD with 1..4 waves per SIMD and ILP 1..8,
// FP64 fma / add, FP32 fma, and FP64 fma interleaved with 32-bit integer ops; the
// shader clock from s_memtime against s_memrealtime (100 MHz).
// hipcc -O3 --offload-arch=gfx950 -o tools/micro/fp64_issue tools/micro/fp64_issue.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

enum Op { FMA64, ADD64, FMA32, FMA64_INT };

template <int ILP, int OP>
__global__ void chain(double *out, unsigned long long *clk, int iters, double a, double b) {
  double acc[ILP];
  float accf[ILP];
  unsigned iv[ILP];
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
#pragma unroll
  for (int k = 0; k < ILP; ++k) {
    acc[k] = threadIdx.x * 1e-3 + k;
    accf[k] = (float)acc[k];
    iv[k] = threadIdx.x + k;
  }
  const float af = (float)a, bf = (float)b;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < ILP; ++k) {
      if (OP == FMA64) acc[k] = fma(acc[k], a, b);
      if (OP == ADD64) acc[k] = acc[k] + b;
      if (OP == FMA32) accf[k] = fmaf(accf[k], af, bf);
      if (OP == FMA64_INT) {
        acc[k] = fma(acc[k], a, b);
        iv[k] = iv[k] * 3u + 1u;
      }
    }
  }
  double s = 0;
#pragma unroll
  for (int k = 0; k < ILP; ++k) s += acc[k] + accf[k] + iv[k];
  if (s == 12345.678) out[threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - t0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

template <int ILP, int OP>
void run(const char *name, int wps, int cus) {
  double *d;
  unsigned long long *clk, hc[2];
  (void)hipMalloc(&d, 8 * 1024);
  (void)hipMalloc(&clk, 16);
  const int iters = 20000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  chain<ILP, OP><<<cus, 256 * wps>>>(d, clk, 100, 0.999, 1e-3);
  (void)hipEventRecord(e0);
  chain<ILP, OP><<<cus, 256 * wps>>>(d, clk, iters, 0.999, 1e-3);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipMemcpy(hc, clk, 16, hipMemcpyDeviceToHost);
  const double ghz = (double)hc[0] / (double)hc[1] * 0.1;
  const double per_simd = (double)wps * iters * ILP;          // wave-ops per SIMD
  printf("%-9s waves/SIMD %d ILP %d: %.3f ms, clock %.2f GHz, %.2f cycles per wave-op\n", name,
         wps, ILP, ms, ghz, (ms * 1e-3 * ghz * 1e9) / per_simd);
  (void)hipFree(d);
  (void)hipFree(clk);
}

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (int wps = 1; wps <= 4; wps += 3) {
    run<1, FMA64>("fma64", wps, cus);
    run<4, FMA64>("fma64", wps, cus);
    run<8, FMA64>("fma64", wps, cus);
    run<8, ADD64>("add64", wps, cus);
    run<8, FMA32>("fma32", wps, cus);
    run<8, FMA64_INT>("fma64+int", wps, cus);
  }
  run<8, FMA64>("fma64", 2, cus);
  run<8, FMA64>("fma64", 3, cus);
  return 0;
}
