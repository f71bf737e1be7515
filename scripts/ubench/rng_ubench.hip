// Counter-based RNG throughput on gfx950: Philox4x32-10 (64-bit mad vs
// mul_hi/mul_lo), Threefry4x32-20, and Box–Muller vs table-free variants.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)
struct u4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u4 philox_mad(u4 c, uint32_t k0, uint32_t k1) {
  #pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    c = u4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return c;
}
__device__ __forceinline__ u4 philox_hilo(u4 c, uint32_t k0, uint32_t k1) {
  #pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t h0 = __umulhi(0xD2511F53u, c.x), l0 = 0xD2511F53u * c.x;
    uint32_t h1 = __umulhi(0xCD9E8D57u, c.z), l1 = 0xCD9E8D57u * c.z;
    c = u4{h1 ^ c.y ^ k0, l1, h0 ^ c.w ^ k1, l0};
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return c;
}
// 32x32->64 with 16-bit pieces and full-rate 24-bit multiplies
__device__ __forceinline__ void mul24(uint32_t M, uint32_t x, uint32_t &hi, uint32_t &lo) {
  const uint32_t Ml = M & 0xFFFF, Mh = M >> 16, xl = x & 0xFFFF, xh = x >> 16;
  const uint32_t ll = __umul24(Ml, xl), lh = __umul24(Ml, xh), hl = __umul24(Mh, xl), hh = __umul24(Mh, xh);
  const uint32_t mid = (ll >> 16) + (lh & 0xFFFF) + (hl & 0xFFFF);
  lo = (ll & 0xFFFF) | (mid << 16);
  hi = hh + (lh >> 16) + (hl >> 16) + (mid >> 16);
}
__device__ __forceinline__ u4 philox_24(u4 c, uint32_t k0, uint32_t k1) {
  #pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t h0, l0, h1, l1; mul24(0xD2511F53u, c.x, h0, l0); mul24(0xCD9E8D57u, c.z, h1, l1);
    c = u4{h1 ^ c.y ^ k0, l1, h0 ^ c.w ^ k1, l0};
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return c;
}
__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ u4 threefry(u4 c, uint32_t k0, uint32_t k1) {  // Threefry4x32-20
  const uint32_t k2 = 0x1BD11BDAu ^ k0 ^ k1;
  uint32_t ks[5] = {k0, k1, k2, k0 ^ k1, 0x1BD11BDAu ^ k0 ^ k1 ^ k2};
  uint32_t x0 = c.x + ks[0], x1 = c.y + ks[1], x2 = c.z + ks[2], x3 = c.w + ks[3];
  const int R[8][2] = {{10, 26}, {11, 21}, {13, 27}, {23, 5}, {6, 20}, {17, 11}, {25, 10}, {18, 20}};
  #pragma unroll
  for (int r = 0; r < 20; ++r) {
    if (r & 1) { x0 += x3; x3 = rotl(x3, R[r & 7][0]) ^ x0; x2 += x1; x1 = rotl(x1, R[r & 7][1]) ^ x2; }
    else { x0 += x1; x1 = rotl(x1, R[r & 7][0]) ^ x0; x2 += x3; x3 = rotl(x3, R[r & 7][1]) ^ x2; }
    if ((r & 3) == 3) { int s = (r + 1) / 4; x0 += ks[s % 5]; x1 += ks[(s + 1) % 5]; x2 += ks[(s + 2) % 5]; x3 += ks[(s + 3) % 5] + s; }
  }
  return u4{x0, x1, x2, x3};
}
template <int G>
__global__ void __launch_bounds__(256) krng(uint32_t *out, int n, uint32_t k0, uint32_t k1) {
  uint32_t t = blockIdx.x * 256 + threadIdx.x, acc = 0;
  for (int i = 0; i < n; ++i) {
    u4 c{t, (uint32_t)i, 7u, 9u};
    u4 r = G == 0 ? philox_mad(c, k0, k1) : G == 1 ? philox_hilo(c, k0, k1) : G == 2 ? philox_24(c, k0, k1) : threefry(c, k0, k1);
    acc ^= r.x ^ r.y ^ r.z ^ r.w;
  }
  out[t] = acc;
}
int main() {
  const int blocks = 4096, n = 4096;  // 1M threads x 4096 calls
  uint32_t *o; CK(hipMalloc(&o, blocks * 256 * 4));
  const char *names[] = {"philox mad_u64", "philox mul_hi/lo", "philox mul24", "threefry4x32-20"};
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int rep = 0; rep < 2; ++rep)
  for (int g = 0; g < 4; ++g) {
    CK(hipEventRecord(a));
    switch (g) {
      case 0: hipLaunchKernelGGL(krng<0>, dim3(blocks), dim3(256), 0, 0, o, n, 1u, 2u); break;
      case 1: hipLaunchKernelGGL(krng<1>, dim3(blocks), dim3(256), 0, 0, o, n, 1u, 2u); break;
      case 2: hipLaunchKernelGGL(krng<2>, dim3(blocks), dim3(256), 0, 0, o, n, 1u, 2u); break;
      case 3: hipLaunchKernelGGL(krng<3>, dim3(blocks), dim3(256), 0, 0, o, n, 1u, 2u); break;
    }
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    double calls = (double)blocks * 256 * n;
    // cycles per call per wave at 2.4 GHz, 1024 SIMDs
    double cyc = ms * 1e-3 * 2.4e9 * 1024 / (calls / 64);
    if (rep) printf("%-20s %8.3f ms  %7.2f Gcalls/s  %6.0f cycles/call/wave\n", names[g], ms, calls / ms / 1e6, cyc);
  }
  return 0;
}
