// Cycles per wave-instruction on gfx950 for the ops of the step kernel's hot
// loop: 8 independent register chains per lane, 2 or 8 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t *out, int n, uint32_t s) {
  uint32_t a[8]; uint64_t q[8]; double d[8];
  #pragma unroll
  for (int i = 0; i < 8; ++i) { a[i] = s + threadIdx.x * 7 + i; q[i] = a[i]; d[i] = 1.0 + a[i] * 1e-9; }
  const uint32_t M = 0xD2511F53u;
  for (int it = 0; it < n; ++it) {
    #pragma unroll
    for (int r = 0; r < 4; ++r)
    #pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (OP == 0) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(q[i]) : "v"(a[i]), "s"(M) : "s40", "s41");
      else if constexpr (OP == 1) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(a[(i+1)&7]), "s"(M));
      else if constexpr (OP == 2) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[i]) : "v"(d[(i+1)&7]));
      else if constexpr (OP == 3) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[i]) : "v"(d[(i+1)&7]));
      else if constexpr (OP == 4) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "s"(M));
      else if constexpr (OP == 5) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "s"(M));
      else if constexpr (OP == 6) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(a[(i+1)&7]));
      else if constexpr (OP == 7) asm volatile("v_alignbit_b32 %0, %0, %1, 12" : "+v"(a[i]) : "v"(a[(i+1)&7]));
      else if constexpr (OP == 8) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i+1)&7]));
      else if constexpr (OP == 9) asm volatile("v_cmp_gt_f64 vcc, %0, %1" : : "v"(d[i]), "v"(d[(i+1)&7]) : "vcc");
      else if constexpr (OP == 10) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(q[i]) : "v"(q[(i+1)&7]));
      else if constexpr (OP == 11) asm volatile("v_mov_b64 %0, %1" : "=v"(q[i]) : "v"(q[(i+1)&7]));
      else if constexpr (OP == 12) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(q[i]) : "v"(q[(i+1)&7]));
    }
  }
  uint32_t t = 0;
  #pragma unroll
  for (int i = 0; i < 8; ++i) t ^= a[i] ^ (uint32_t)q[i] ^ (uint32_t)(q[i] >> 32) ^ (uint32_t)__builtin_bit_cast(uint64_t, d[i]);
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

template <int OP> void run(uint32_t *o, const char *nm, int wps) {
  // wps waves per SIMD: 1024 SIMDs, 4 waves per block of 256 threads
  const int blocks = 256 * wps, n = 4096;
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, o, 16, 1u);
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, o, n, 1u);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  const double winstr_per_simd = (double)wps * n * 32;  // wave-instructions per SIMD
  printf("%-16s waves/SIMD=%d  %6.2f cycles/wave-instr (at 2.4 GHz)\n", nm, wps, ms * 1e-3 * 2.4e9 / winstr_per_simd);
}
int main() {
  uint32_t *o; CK(hipMalloc(&o, 256 * 8 * 256 * 4));
  for (int w : {1, 2, 4}) {
    run<0>(o, "v_mad_u64_u32", w); run<1>(o, "v_bitop3_b32", w); run<2>(o, "v_fma_f64", w);
    run<3>(o, "v_add_f64", w); run<4>(o, "v_mul_hi_u32", w); run<5>(o, "v_mul_lo_u32", w);
    run<6>(o, "v_cndmask_b32", w); run<7>(o, "v_alignbit_b32", w); run<8>(o, "v_add_u32", w);
    run<9>(o, "v_cmp_gt_f64", w); run<10>(o, "v_lshl_add_u64", w); run<11>(o, "v_mov_b64", w);
    run<12>(o, "v_pk_mul_f32", w);
  }
  return 0;
}
