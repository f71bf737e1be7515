// Issue rate of v_mfma_f64_16x16x4f64 on dependent chains: K independent
// accumulators, each a chain of N/K MFMAs; cycles per MFMA from the shader clock
// (s_memtime), one or two waves per SIMD.  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int K>
__global__ void __launch_bounds__(256) chain(double *out, long long *cyc, int n) {
    d4 acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = d4{0.0, 0.0, 0.0, 0.0};
    const double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
    const long long t0 = clock64();
    for (int i = 0; i < n; i += K) {
#pragma unroll
        for (int k = 0; k < K; ++k) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
    }
    const long long t1 = clock64();
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < K; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int K>
void run(int blocks, int n, double *out, long long *cyc, long long *h) {
    hipLaunchKernelGGL(chain<K>, dim3(blocks), dim3(256), 0, 0, out, cyc, n);  // warm
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(chain<K>, dim3(blocks), dim3(256), 0, 0, out, cyc, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(h, cyc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < blocks; ++i) avg += (double)h[i];
    avg /= blocks;
    const double waves_per_simd = blocks * 4.0 / 1024.0;
    const double flop = 2048.0 * n * blocks * 4;
    printf("K=%d blocks=%d waves/SIMD=%.0f: %.1f clock64 ticks per MFMA per wave, %.3f ms, %.1f TFLOP/s\n", K, blocks,
           waves_per_simd, avg / n, ms, flop / ms / 1e9);
}

int main() {
    const int n = 1 << 14;
    double *out;
    long long *cyc, h[4096];
    hipMalloc(&out, 4096 * 256 * sizeof(double));
    hipMalloc(&cyc, 4096 * sizeof(long long));
    for (int blocks : {256, 512, 1024}) {
        run<1>(blocks, n, out, cyc, h);
        run<2>(blocks, n, out, cyc, h);
        run<4>(blocks, n, out, cyc, h);
        run<8>(blocks, n, out, cyc, h);
    }
    return 0;
}
