// Achievable HBM write bandwidth for the step kernel's history pattern: each
// lane stores 2 slots × 8 nontemporal 16-byte words per step (pair-interleaved
// SoA, slot stride 16·C bytes per word), 100 steps per launch, optional fp64
// VALU work per step (8 independent fma chains × WORK).  Grid: C chains at
// LPC = 2 ⇒ C/32 waves (C = 65,536: 2 waves per SIMD, as the step kernel).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)
typedef double d2 __attribute__((ext_vector_type(2)));

template <int WORK, int NT>
__global__ void __launch_bounds__(256) kw(d2 *hist, unsigned long long C, int steps) {
  const unsigned long long tid = blockIdx.x * 256ull + threadIdx.x, c = tid >> 1;
  const int sub = tid & 1;
  if (c >= C) return;
  double v[8];
  for (int i = 0; i < 8; ++i) v[i] = 1.0 + tid * 1e-9 + i;
  for (int s = 0; s < steps; ++s) {
#pragma unroll 1
    for (int w = 0; w < WORK; ++w)
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = fma(v[i], 0.9999999, 1e-9);
    d2 *slot = hist + (unsigned long long)s * 2 * 16 * C;  // two slots of 16 words-per-chain·C... (θ, θ°)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        d2 x = {v[j] + h, v[j] - s};
        d2 *p = slot + (unsigned long long)h * 16 * C + (unsigned long long)(sub * 8 + j) * C + c;
        if (NT) __builtin_nontemporal_store(x, p); else *p = x;
      }
  }
}

template <int WORK, int NT> void run(d2 *buf, unsigned long long C, int steps) {
  dim3 g((unsigned)((2 * C + 255) / 256));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  hipLaunchKernelGGL((kw<WORK, NT>), g, dim3(256), 0, 0, buf, C, steps);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((kw<WORK, NT>), g, dim3(256), 0, 0, buf, C, steps);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); if (ms < best) best = ms;
  }
  const double bytes = 512.0 * C * steps;
  printf("C=%7llu work=%3d nt=%d  %7.3f ms  %6.2f TB/s  %.3e chain-steps/s\n", C, WORK, NT, best, bytes / best / 1e9,
         C * (double)steps / (best * 1e-3));
}

int main() {
  const int steps = 100;
  const unsigned long long Cmax = 262144;
  d2 *buf; CK(hipMalloc(&buf, 512ull * Cmax * steps));
  for (unsigned long long C : {65536ull, 131072ull, 262144ull}) {
    run<0, 1>(buf, C, steps); run<0, 0>(buf, C, steps);
  }
  run<20, 1>(buf, 65536, steps); run<40, 1>(buf, 65536, steps); run<80, 1>(buf, 65536, steps);
  run<120, 1>(buf, 65536, steps); run<160, 1>(buf, 65536, steps);
  return 0;
}
