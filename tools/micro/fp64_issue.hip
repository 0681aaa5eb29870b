// Microbenchmark: FP64 VALU issue rate per SIMD with 1..4 waves per SIMD and ILP 1..8.
// hipcc -O3 --offload-arch=gfx950 -o /tmp/fp64_issue tools/micro/fp64_issue.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int ILP>
__global__ void fma_chain(double *out, int iters, double a, double b) {
  double acc[ILP];
#pragma unroll
  for (int k = 0; k < ILP; ++k) acc[k] = threadIdx.x * 1e-3 + k;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < ILP; ++k) acc[k] = fma(acc[k], a, b);
  }
  double s = 0;
#pragma unroll
  for (int k = 0; k < ILP; ++k) s += acc[k];
  if (s == 12345.678) out[threadIdx.x] = s;
}

template <int ILP>
void run(int wps, int cus) {
  double *d;
  hipMalloc(&d, 8 * 1024);
  const int iters = 20000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  fma_chain<ILP><<<cus, 256 * wps>>>(d, 100, 0.999, 1e-3);
  hipEventRecord(e0);
  fma_chain<ILP><<<cus, 256 * wps>>>(d, iters, 0.999, 1e-3);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double instr = (double)cus * 4 * wps * iters * ILP;   // wave-instructions
  // per SIMD: cus*4 SIMDs; cycles at ~2.4 GHz
  const double per_simd = instr / (cus * 4);
  printf("waves/SIMD %d ILP %d: %.3f ms, %.2f wave-FMA/us/SIMD, %.2f cycles per wave-FMA @2.4GHz\n",
         wps, ILP, ms, per_simd / (ms * 1e3), (ms * 1e-3 * 2.4e9) / per_simd);
  hipFree(d);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (int wps = 1; wps <= 4; ++wps) {
    run<1>(wps, cus);
    run<2>(wps, cus);
    run<4>(wps, cus);
    run<8>(wps, cus);
  }
  return 0;
}
