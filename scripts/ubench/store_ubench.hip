// Store-path microbenchmark for the history streams: SoA [step][D][C] fp64
// writes, one chain per lane, with optional fp64 work between steps.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

template <int MODE, int WORK>  // MODE 0 plain x2, 1 nt x2, 2 plain x4 (2 chains/lane), 3 nt x4
__global__ void __launch_bounds__(256) kstore(double *out, unsigned long long C, int D, int S, double seed) {
  unsigned long long t = blockIdx.x * 256ull + threadIdx.x;
  double v = seed + t;
  if (MODE < 2) {
    if (t >= C) return;
    for (int s = 0; s < S; ++s) {
      #pragma unroll 1
      for (int w = 0; w < WORK; ++w) v = fma(v, 0.999999, 1e-7);
      for (int d = 0; d < D; ++d) {
        double *p = out + ((unsigned long long)s * D + d) * C + t;
        if (MODE == 1) __builtin_nontemporal_store(v + d, p); else *p = v + d;
      }
    }
  } else {
    if (2 * t >= C) return;
    typedef double d2 __attribute__((ext_vector_type(2)));
    for (int s = 0; s < S; ++s) {
      #pragma unroll 1
      for (int w = 0; w < 2 * WORK; ++w) v = fma(v, 0.999999, 1e-7);
      for (int d = 0; d < D; ++d) {
        d2 x = {v + d, v - d};
        d2 *p = (d2 *)(out + ((unsigned long long)s * D + d) * C + 2 * t);
        if (MODE == 3) __builtin_nontemporal_store(x, p); else *p = x;
      }
    }
  }
}

template <int MODE, int WORK> void run(double *buf, unsigned long long C, int D, int S, const char *name) {
  unsigned long long threads = MODE < 2 ? C : C / 2;
  dim3 g((unsigned)((threads + 255) / 256));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  hipLaunchKernelGGL((kstore<MODE, WORK>), g, dim3(256), 0, 0, buf, C, D, S, 1.0);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((kstore<MODE, WORK>), g, dim3(256), 0, 0, buf, C, D, S, 1.0 + r);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); if (ms < best) best = ms;
  }
  double bytes = 8.0 * C * D * S;
  printf("%-28s work=%4d  %8.3f ms  %7.2f TB/s\n", name, WORK, best, bytes / best / 1e9);
}

int main() {
  const unsigned long long C = 65536; const int D = 64, S = 200;  // 6.7 GB per launch
  double *buf; CK(hipMalloc(&buf, 8ull * C * D * S));
  run<0, 0>(buf, C, D, S, "plain dwordx2");
  run<1, 0>(buf, C, D, S, "nt dwordx2");
  run<2, 0>(buf, C, D, S, "plain dwordx4");
  run<3, 0>(buf, C, D, S, "nt dwordx4");
  run<1, 64>(buf, C, D, S, "nt dwordx2");
  run<3, 64>(buf, C, D, S, "nt dwordx4");
  run<1, 256>(buf, C, D, S, "nt dwordx2");
  run<3, 256>(buf, C, D, S, "nt dwordx4");
  run<0, 256>(buf, C, D, S, "plain dwordx2");
  run<1, 1024>(buf, C, D, S, "nt dwordx2");
  run<0, 1024>(buf, C, D, S, "plain dwordx2");
  const unsigned long long C4 = 4 * 65536;  // more waves
  run<1, 0>(buf, C4, D, S / 4, "nt dwordx2 C=256k");
  run<1, 256>(buf, C4, D, S / 4, "nt dwordx2 C=256k");
  run<0, 256>(buf, C4, D, S / 4, "plain dwordx2 C=256k");
  return 0;
}
