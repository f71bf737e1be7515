// Issue rate of v_fma_f64 (and v_mul_f64) with K independent chains per lane,
// 1, 2 and 4 waves per SIMD; TFLOP/s counting 2 per fma.  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>

template <int K>
__global__ void __launch_bounds__(256) fmas(double *out, int n) {
    double acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = threadIdx.x * 1e-3 + k;
    const double a = 0.999999 + threadIdx.x * 1e-12, b = 1e-7;
    for (int i = 0; i < n; i += K) {
#pragma unroll
        for (int k = 0; k < K; ++k) acc[k] = fma(acc[k], a, b);
    }
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < K; ++k) s += acc[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int K>
void run(int blocks, int n, double *out) {
    hipLaunchKernelGGL(fmas<K>, dim3(blocks), dim3(256), 0, 0, out, n);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(fmas<K>, dim3(blocks), dim3(256), 0, 0, out, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double flop = 2.0 * n * blocks * 256.0;
    printf("v_fma_f64 K=%d waves/SIMD=%.0f: %.3f ms, %.1f TFLOP/s\n", K, blocks * 4.0 / 1024.0, ms, flop / ms / 1e9);
}

int main() {
    const int n = 1 << 16;
    double *out;
    hipMalloc(&out, 4096 * 256 * sizeof(double));
    for (int blocks : {256, 512, 1024}) {
        run<1>(blocks, n, out);
        run<4>(blocks, n, out);
        run<8>(blocks, n, out);
    }
    return 0;
}
