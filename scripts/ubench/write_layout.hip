// History-store layouts at the cfg 2 shape: 65,536 chains, D = 32, LPC = 2
// (two lanes per chain, 16 coordinates each), θ and θ° histories (2 × 256 B per
// chain-step) + ll (8 B), no other work.  Compares the shipped slot layout
// (pair-interleaved SoA: word (pair k, chain c) at (k·C + c)·16 B, so a wave's
// 8 stores per history land 1 MiB apart) with wave-blocked tiles (the 32 chains
// of a wave keep their 16 pairs in one contiguous 8 KiB run), at 20 and 100
// steps per launch, nontemporal / plain / sc1 stores.
//   hipcc --offload-arch=gfx950 -O3 -o write_layout write_layout.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)
typedef double d2 __attribute__((ext_vector_type(2)));

template <int FL>
__device__ __forceinline__ void st(d2 x, d2 *p) {
  if constexpr (FL == 0) __builtin_nontemporal_store(x, p);
  else if constexpr (FL == 1) *p = x;
  else __hip_atomic_store(reinterpret_cast<unsigned long long *>(p), __double_as_longlong(x.x), __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT),
       __hip_atomic_store(reinterpret_cast<unsigned long long *>(p) + 1, __double_as_longlong(x.y), __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT);
}

// LAYOUT 0: shipped slot layout; 1: wave tile [C/32][16 pairs][32 chains];
// 2: wave tile with θ and θ° of a step interleaved per wave (16 KiB per wave-step)
template <int LAYOUT, int FL>
__global__ void __launch_bounds__(256) kw(d2 *hist, double *hll, unsigned long long C, int s0, int steps) {
  const unsigned long long tid = blockIdx.x * 256ull + threadIdx.x, c = tid >> 1;
  const int sub = tid & 1;
  if (c >= C) return;
  double v[8];
  for (int i = 0; i < 8; ++i) v[i] = 1.0 + tid * 1e-9 + i;
  const unsigned long long wc = c & 31, wb = c >> 5;  // chain within the wave, wave
  for (int s = s0; s < s0 + steps; ++s) {
    const unsigned long long slot = (unsigned long long)s * 2 * 16 * C;  // θ then θ° slot
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fma(v[j], 0.9999999, 1e-9);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        d2 x = {v[j] + h, v[j] - s};
        const unsigned long long k = sub * 8 + j;
        d2 *p;
        if constexpr (LAYOUT == 0) p = hist + slot + h * 16 * C + k * C + c;
        else if constexpr (LAYOUT == 1) p = hist + slot + h * 16 * C + wb * 512 + k * 32 + wc;
        else p = hist + slot + wb * 1024 + h * 512 + k * 32 + wc;
        st<FL>(x, p);
      }
    }
    if (sub == 0) __builtin_nontemporal_store(v[0], hll + (unsigned long long)s * C + c);
  }
}

template <int LAYOUT, int FL>
void run(d2 *buf, double *ll, unsigned long long C, int steps, int total, const char *name) {
  dim3 g((unsigned)((2 * C + 255) / 256));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  // warm: the whole buffer once
  for (int s0 = 0; s0 + steps <= total; s0 += steps) hipLaunchKernelGGL((kw<LAYOUT, FL>), g, dim3(256), 0, 0, buf, ll, C, s0, steps);
  CK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int r = 0; r < 3; ++r)
    for (int s0 = 0; s0 + steps <= total; s0 += steps) {
      CK(hipEventRecord(a));
      hipLaunchKernelGGL((kw<LAYOUT, FL>), g, dim3(256), 0, 0, buf, ll, C, s0, steps);
      CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b)); t.push_back(ms);
    }
  std::sort(t.begin(), t.end());
  const float med = t[t.size() / 2], best = t[0];
  const double bytes = 520.0 * C * steps;
  printf("%-22s steps=%3d  med %8.1f us  best %8.1f us  %5.2f TB/s (med)  %.3e chain-steps/s\n", name, steps,
         med * 1e3, best * 1e3, bytes / med / 1e9, C * (double)steps / (med * 1e-3));
}

int main() {
  const unsigned long long C = 65536;
  const int total = 200;
  d2 *buf; CK(hipMalloc(&buf, 512ull * C * total));
  double *ll; CK(hipMalloc(&ll, 8ull * C * total));
  CK(hipMemset(buf, 0, 512ull * C * total));
  for (int steps : {20, 100}) {
    run<0, 0>(buf, ll, C, steps, total, "slot nt");
    run<1, 0>(buf, ll, C, steps, total, "wavetile nt");
    run<2, 0>(buf, ll, C, steps, total, "wavetile-pair nt");
    run<0, 1>(buf, ll, C, steps, total, "slot plain");
    run<1, 1>(buf, ll, C, steps, total, "wavetile plain");
    run<2, 1>(buf, ll, C, steps, total, "wavetile-pair plain");
    run<0, 2>(buf, ll, C, steps, total, "slot sc1(8B)");
    run<1, 2>(buf, ll, C, steps, total, "wavetile sc1(8B)");
    run<0, 0>(buf, ll, C, steps, total, "slot nt (again)");
    run<1, 0>(buf, ll, C, steps, total, "wavetile nt (again)");
  }
  return 0;
}
