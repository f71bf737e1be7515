// Do fp64 MFMA and fp64 VALU overlap on one SIMD?  Blocks of 1024 threads, one
// per CU (16 waves: 4 per SIMD).  MODE 1: waves 0–7 (2 per SIMD, enough to
// saturate the f64 MFMA pipe) run 8 v_mfma_f64_16x16x4f64 chains, the rest
// exit; MODE 2: waves 8–15 run 8 v_fma_f64 chains, the rest exit; MODE 3: both.  Overlap ⇔ t3 ≈ max(t1, t2); a shared fp64 datapath
// ⇔ t3 ≈ t1 + t2.  OP picks the VALU waves' operation: 0 v_fma_f64, 1 32-bit integer
// (v_add_u32 + v_xor_b32), 2 v_fma_f32, 3 v_cndmask_b32 — which of them share the f64 pipe.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)
typedef double d4 __attribute__((ext_vector_type(4)));

template <int MODE, int OP>
__global__ void __launch_bounds__(1024) k(double *out, int nm, int nv) {
  const int wave = threadIdx.x >> 6;
  const bool mf = wave < 8;  // 16 waves per CU: waves 0–7 (2 per SIMD) MFMA, 8–15 (2 per SIMD) VALU
  double acc = 0.0;
  if (mf && (MODE & 1)) {
    d4 c[8];
    for (int j = 0; j < 8; ++j) c[j] = d4{0, 0, 0, 0};
    double a = 1.0 + threadIdx.x * 1e-9, b = 0.5;
    for (int i = 0; i < nm; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) c[j] = __builtin_amdgcn_mfma_f64_16x16x4f64((j & 1) ? a : b, (j & 2) ? a : b, c[j], 0, 0, 0);
    for (int j = 0; j < 8; ++j) acc += c[j][j & 3];
  }
  if (!mf && (MODE & 2)) {
    if constexpr (OP == 0) {
      double v[8];
      for (int j = 0; j < 8; ++j) v[j] = 1.0 + threadIdx.x * 1e-9 + j;
      for (int i = 0; i < nv; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = fma(v[j], 0.9999999, 1e-9);
      for (int j = 0; j < 8; ++j) acc += v[j];
    } else if constexpr (OP == 1) {
      uint32_t v[8];
      for (int j = 0; j < 8; ++j) v[j] = threadIdx.x * 7u + j;
      for (int i = 0; i < nv; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[j] = v[j] + 0x9e3779b9u;
          asm volatile("" : "+v"(v[j]));
        }
      for (int j = 0; j < 8; ++j) acc += (double)v[j];
    } else if constexpr (OP == 2) {
      float v[8];
      for (int j = 0; j < 8; ++j) v[j] = 1.0f + threadIdx.x * 1e-6f + j;
      for (int i = 0; i < nv; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = fmaf(v[j], 0.9999f, 1e-6f);
      for (int j = 0; j < 8; ++j) acc += v[j];
    } else {
      uint32_t v[8];
      const bool c = (threadIdx.x & 1) != 0;
      for (int j = 0; j < 8; ++j) v[j] = threadIdx.x * 7u + j;
      for (int i = 0; i < nv; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          uint32_t w = v[j] ^ 0x5bd1e995u;
          asm volatile("" : "+v"(w));
          v[j] = c ? w : v[j];
          asm volatile("" : "+v"(v[j]));
        }
      for (int j = 0; j < 8; ++j) acc += (double)v[j];
    }
  }
  out[blockIdx.x * 1024 + threadIdx.x] = acc;
}

template <int MODE, int OP> float run(double *o, int nm, int nv) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  k<MODE, OP><<<dim3(256), dim3(1024), 0, 0>>>(o, nm, nv);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(a));
    k<MODE, OP><<<dim3(256), dim3(1024), 0, 0>>>(o, nm, nv);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); if (ms < best) best = ms;
  }
  return best;
}

template <int OP> void sweep(double *o, const char *name) {
  const int nm = 10000;
  for (int nv : {10000, 20000, 40000}) {
    const float t1 = run<1, OP>(o, nm, nv), t2 = run<2, OP>(o, nm, nv), t3 = run<3, OP>(o, nm, nv);
    printf("%s: mfma %d×8, valu %d×8 per wave: mfma-only %.3f ms, valu-only %.3f ms, both %.3f ms "
           "(max %.3f, sum %.3f)\n", name, nm, nv, t1, t2, t3, t1 > t2 ? t1 : t2, t1 + t2);
  }
}

int main() {
  double *o; CK(hipMalloc(&o, 256 * 1024 * 8));
  sweep<0>(o, "v_fma_f64");
  sweep<1>(o, "u32 add");
  sweep<2>(o, "v_fma_f32");
  sweep<3>(o, "xor+cndmask");
  return 0;
}
