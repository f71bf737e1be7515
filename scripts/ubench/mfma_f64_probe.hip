// Probe: arithmetic of v_mfma_f64_16x16x4f64 on gfx950.  For random A (16x4),
// B (4x16), C (16x16) with wide exponent spread, compare D against CPU
// candidates: (a) fma chain k = 0..3 starting from C; (b) fma chain k = 3..0;
// (c) exact dot + C rounded once (long double not exact; use two-sum check);
// (d) products rounded, summed left to right, then + C.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void probe(const double *A, const double *B, const double *C, double *D, int reps) {
    const int l = threadIdx.x;
    for (int r = 0; r < reps; ++r) {
        const double *a = A + r * 64, *b = B + r * 64, *c = C + r * 256;
        // lane l: A[row = l&15][k = l>>4], B[k = l>>4][col = l&15]
        double av = a[(l & 15) * 4 + (l >> 4)];
        double bv = b[(l >> 4) * 16 + (l & 15)];
        d4 acc;
        for (int i = 0; i < 4; ++i) acc[i] = c[((l >> 4) + 4 * i) * 16 + (l & 15)];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
        for (int i = 0; i < 4; ++i) D[r * 256 + ((l >> 4) + 4 * i) * 16 + (l & 15)] = acc[i];
    }
}

int main() {
    const int R = 2000;
    std::mt19937_64 g(1);
    std::uniform_real_distribution<double> u(-1, 1);
    std::uniform_int_distribution<int> e(-30, 30);
    double *A = new double[R * 64], *B = new double[R * 64], *C = new double[R * 256], *D = new double[R * 256];
    for (int i = 0; i < R * 64; ++i) { A[i] = std::ldexp(u(g), e(g)); B[i] = std::ldexp(u(g), e(g)); }
    for (int i = 0; i < R * 256; ++i) C[i] = std::ldexp(u(g), e(g));
    double *dA, *dB, *dC, *dD;
    hipMalloc(&dA, R * 64 * 8); hipMalloc(&dB, R * 64 * 8); hipMalloc(&dC, R * 256 * 8); hipMalloc(&dD, R * 256 * 8);
    hipMemcpy(dA, A, R * 64 * 8, hipMemcpyHostToDevice);
    hipMemcpy(dB, B, R * 64 * 8, hipMemcpyHostToDevice);
    hipMemcpy(dC, C, R * 256 * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD, R);
    hipMemcpy(D, dD, R * 256 * 8, hipMemcpyDeviceToHost);
    long n = 0, fwd = 0, rev = 0, prodsum = 0, prodsumC = 0, exact1 = 0;
    for (int r = 0; r < R; ++r)
        for (int i = 0; i < 16; ++i)
            for (int j = 0; j < 16; ++j) {
                const double *a = A + r * 64 + i * 4;
                double bk[4];
                for (int k = 0; k < 4; ++k) bk[k] = B[r * 64 + k * 16 + j];
                double c = C[r * 256 + i * 16 + j], d = D[r * 256 + i * 16 + j];
                double f = c; for (int k = 0; k < 4; ++k) f = std::fma(a[k], bk[k], f);
                double rv = c; for (int k = 3; k >= 0; --k) rv = std::fma(a[k], bk[k], rv);
                volatile double p0 = a[0] * bk[0], p1 = a[1] * bk[1], p2 = a[2] * bk[2], p3 = a[3] * bk[3];
                double ps = (((p0 + p1) + p2) + p3) + c;
                double pc = (((c + p0) + p1) + p2) + p3;
                __float128 q = (__float128)c;
                for (int k = 0; k < 4; ++k) q += (__float128)a[k] * (__float128)bk[k];
                double ex = (double)q;
                ++n; fwd += (f == d); rev += (rv == d); prodsum += (ps == d); prodsumC += (pc == d); exact1 += (ex == d);
            }
    printf("n=%ld fma_fwd=%ld fma_rev=%ld prod_sum_then_C=%ld C_then_prods=%ld exact_once=%ld\n", n, fwd, rev, prodsum,
           prodsumC, exact1);
    return 0;
}
