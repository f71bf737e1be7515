// fp64 VALU throughput calibration on gfx950: independent fma / mul / add /
// div / sqrt streams at full occupancy; cycles per wave-instruction.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)
template <int OP>
__global__ void __launch_bounds__(256) kf(double *out, int n, double s) {
  double a[8];
  #pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = s + threadIdx.x + i;
  for (int it = 0; it < n; ++it) {
    #pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (OP == 0) a[i] = fma(a[i], 0.9999999, 1e-9);
      else if (OP == 1) a[i] = a[i] * 0.9999999;
      else if (OP == 2) a[i] = a[i] + 1e-9;
      else if (OP == 3) a[i] = 1.0001 / a[i];
      else if (OP == 4) a[i] = sqrt(a[i]) + 1.0;
      else if (OP == 5) { float f = (float)a[i]; f = fmaf(f, 0.999f, 1e-3f); a[i] = f; }
    }
  }
  double t = 0; for (int i = 0; i < 8; ++i) t += a[i];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}
template <int OP> void run(double *o, const char *nm, int per) {
  const int blocks = 8192, n = 2048;
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  hipLaunchKernelGGL(kf<OP>, dim3(blocks), dim3(256), 0, 0, o, 16, 1.0);
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(kf<OP>, dim3(blocks), dim3(256), 0, 0, o, n, 1.0);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  double winstr = (double)blocks * 4 * n * 8 * per;  // wave-instructions of the op class
  printf("%-10s %8.3f ms  %6.2f cycles/wave-instr @2.4GHz per SIMD\n", nm, ms, ms * 1e-3 * 2.4e9 * 1024 / winstr);
}
int main() {
  double *o; CK(hipMalloc(&o, 8192 * 256 * 8));
  run<0>(o, "fma_f64", 1); run<1>(o, "mul_f64", 1); run<2>(o, "add_f64", 1);
  run<3>(o, "div_f64", 1); run<4>(o, "sqrt_f64", 1); run<5>(o, "cvt+fmaf", 1);
  return 0;
}
