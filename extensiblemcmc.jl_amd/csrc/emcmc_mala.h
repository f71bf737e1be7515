// emcmc_mala.h — MALA on a logistic-regression target (row f2, BASELINE cfg 3):
// both contractions on the fp64 matrix cores (gfx950 v_mfma_f64_16x16x4f64).
//
// Semantics (the reference stubs MALAUpdate, updates.jl:216-218; see
// oracle/emcmc_oracle.c orc_run_mala for the full statement and evaluation
// order):  m = θ + h∇ℓ(θ), θ° = m + ϵz, h = ϵ²/2;  ℓ(θ) = Σ_n y_n η_n −
// softplus(η_n), η = Xθ, ∇ℓ = Xᵀ(y − σ(η));  llr and the accept test as the
// reference's accept_reject! (run.jl:268-281); ∇ℓ is carried with the state.
//
// One launch = one MCMC step of every chain.  A workgroup owns 64 chains, one
// wave 16 of them: lane l holds chain c0 + (l & 15) and the coordinates
// d ≡ (l >> 4) (mod 4).  Per 16-row block of X (staged through LDS, 64 rows
// per tile, shared by the 4 waves):
//   η   (16 rows × 16 chains) = Σ_j MFMA(X[rows][4j..4j+3], θ°[4j..4j+3][chains])
//   ℓ_n, r_n = y_n − σ(η_n)     elementwise on the MFMA output registers
//   ∇ℓ  (D × 16 chains)      += Σ_q MFMA(X[rows 4q..4q+3][d-block]ᵀ, r[rows 4q..4q+3])
// The η output layout (row = (l>>4) + 4q, col = l & 15) is exactly the B
// operand layout of the k-step over rows 4q..4q+3, so r never leaves registers.
// v_mfma_f64_16x16x4f64 is an fma chain over its k in order
// (scripts/ubench/mfma_f64_probe.hip), so η_n and ∇ℓ_d are fma chains over d and
// over n in increasing order — restated exactly by the oracle.
#pragma once

#include "emcmc_kernels.h"

namespace emcmc {

typedef double mala_d4 __attribute__((ext_vector_type(4)));

constexpr int kMalaTileRows = 64;     // rows of X per LDS tile (33.8 KB at D = 64)
constexpr int kMalaChainsPerWG = 64;  // 4 waves × 16 chains

struct MalaParams {
    double *theta;   // [D] state_pos layout
    double *grad;    // [D] state_pos layout: ∇ℓ(θ)
    double *ll;      // [C]
    double *ra;      // [C]
    uint64_t *ring;  // [C][2]
    uint32_t *nacc;  // [C]
    uint32_t *faults;
    uint32_t *fault_flag;
    double *ll_prop;  // [C] sub_ws°.ll
    double *hist_theta, *hist_prop, *hist_ll;
    uint8_t *hist_acc;
    const Ziggurat *zig;  // global memory (a few draws per lane per step)
    const double *X;      // [Npad][D] row-major, rows ≥ N zero
    const double *y;      // [Npad]
    uint64_t C;
    uint64_t row_bytes;
    uint64_t N0;     // GenericChainStats.N of this step
    uint64_t nrows;  // N
    uint32_t ntiles;
    uint32_t chain0, key0, key1, iter, W;
    double eps, h, ieps, c0;  // ϵ, ϵ²/2, 1/ϵ, −(D·log2π + logdet ϵ²I)/2
    double rcp_W;
};

// ℓ_n = y·η − softplus(η), r_n = y − σ(η), no division: t = e^{−|η|},
// u = 1 + t, log(u) and v ≈ 1/u from one reduction (log_rcp_1_2), log1p(t) =
// log(u) − ((u − 1) − t)·v (t if u == 1), σ = (η ≥ 0 ? 1 : t)·v.  exp and log
// are the table-driven forms (emcmc_math.h exp_le0 / log_rcp_1_2) with their
// tables in LDS.
struct MathLds {
    double exp2_64[64];
    double invc[128];
    double logc[128];
};
// exp_le0 without its NaN select: a NaN η still makes ℓ_n = y·η − … NaN, so the
// chain's ll° is NaN (fault bit, rejected) with the same bits everywhere else.
__device__ __forceinline__ void logistic_terms(double eta, double y, double &ell, double &r, const MathLds &mt) {
    const double t = exp_le0<false>(-fabs(eta), mt.exp2_64);
    const double u = 1.0 + t;
    double v;
    const double lu = log_rcp_1_2(u, mt.invc, mt.logc, v);
    const double lp1 = (u == 1.0) ? t : lu - ((u - 1.0) - t) * v;
    const double sp = (eta > 0.0 ? eta : 0.0) + lp1;
    const double sig = (eta >= 0.0 ? 1.0 : t) * v;
    ell = y * eta - sp;
    r = y - sig;
}

// (v_0 + v_1) + (v_2 + v_3) over the four lanes (l>>4 = 0..3) of a chain;
// every lane receives the total (fp add is commutative, so the order holds on
// all four)
__device__ __forceinline__ double quad_sum(double s) {
    const double a = s + __shfl_xor(s, 16);
    return a + __shfl_xor(a, 32);
}

// MODE 0: one MCMC step; MODE 1: ∇ℓ at the current θ only (initialisation)
template <int DB, bool FULL, int MODE>
__global__ void __launch_bounds__(256, 2) mala_logistic_kernel(const MalaParams a) {
    constexpr int D = 16 * DB;
    constexpr int J = 4 * DB;        // coordinates per lane
    constexpr int LD = D + 1;        // padded LDS row stride (doubles)
    __shared__ double xs[kMalaTileRows * LD];
    __shared__ double ys[kMalaTileRows];
    __shared__ MathLds mt;
    for (int i = threadIdx.x; i < 64; i += blockDim.x) mt.exp2_64[i] = EXP2_64[i];
    for (int i = threadIdx.x; i < 128; i += blockDim.x) {
        mt.invc[i] = LOG_INVC[i];
        mt.logc[i] = LOG_LOGC[i];
    }  // (the first tile's __syncthreads orders these before any use)

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, cl = lane & 15;
    const uint64_t C = a.C;
    const uint64_t chain = (uint64_t)blockIdx.x * kMalaChainsPerWG + wave * 16 + cl;
    const bool valid = chain < C;
    const uint32_t gid = a.chain0 + (uint32_t)chain;
    // element (d, chain) of a state_pos array; `ch` is made opaque per phase so
    // the J addresses are not kept live across the row loop
    auto pos = [&](int d, uint64_t ch) { return state_pos((uint64_t)d, ch, C, (uint32_t)D); };

    // ---- prologue: θ, ∇ℓ(θ) and the proposal (B operand fragments)
    double tp[J];
    uint32_t faults = valid ? a.faults[chain] : 0u;
    double ltd_fwd = 0.0;
    {
        uint64_t ch = chain;
        asm volatile("" : "+v"(ch));
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const double th = valid ? a.theta[pos(4 * j + g, ch)] : 0.0;
            if constexpr (MODE == 0) {
                const double gr = valid ? a.grad[pos(4 * j + g, ch)] : 0.0;
                const double z = normal_draw(zig_tabs(*a.zig), a.key0, a.key1, gid, a.iter, 0, (uint32_t)(4 * j + g), faults);
                const double m = th + a.h * gr;
                tp[j] = m + a.eps * z;
                const double v = (tp[j] - m) * a.ieps;
                s = (j == 0) ? v * v : fma(v, v, s);
            } else {
                tp[j] = th;
            }
        }
        if constexpr (MODE == 0) ltd_fwd = fma(-0.5, quad_sum(s), a.c0);
    }

    // ---- η = X θ°, ℓ, r, ∇ℓ over all rows
    mala_d4 G[DB];
#pragma unroll
    for (int e = 0; e < DB; ++e) G[e] = mala_d4{0.0, 0.0, 0.0, 0.0};
    double S = 0.0;
    for (uint32_t t = 0; t < a.ntiles; ++t) {
        const uint64_t n0 = (uint64_t)t * kMalaTileRows;
        __syncthreads();  // previous tile consumed
        {
            const double2 *src = reinterpret_cast<const double2 *>(a.X + n0 * D);
            constexpr int PAIRS = kMalaTileRows * D / 2;
#pragma unroll
            for (int i = threadIdx.x; i < PAIRS; i += 256) {
                const double2 v = src[i];
                const int row = i / (D / 2), col = 2 * (i % (D / 2));
                xs[row * LD + col] = v.x;
                xs[row * LD + col + 1] = v.y;
            }
            if (threadIdx.x < kMalaTileRows) ys[threadIdx.x] = a.y[n0 + threadIdx.x];
        }
        __syncthreads();
        // 16-row blocks, software-pipelined: the η MFMAs of block b+1 are issued
        // in the same scheduling region as the elementwise terms of block b, so
        // the matrix pipe works while the VALU evaluates exp/log/σ (they are
        // independent); a region holds one block's temporaries.
        constexpr int NB = kMalaTileRows / 16;
        // rows of this tile below N (all 64 but in the last tile)
        const uint32_t rem = (uint32_t)(a.nrows - n0 < (uint64_t)kMalaTileRows ? a.nrows - n0 : kMalaTileRows);
        mala_d4 en = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int j = 0; j < J; ++j)
            en = __builtin_amdgcn_mfma_f64_16x16x4f64(xs[cl * LD + 4 * j + g], tp[j], en, 0, 0, 0);
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            __builtin_amdgcn_sched_barrier(0);
            const mala_d4 eta = en;
            if (b + 1 < NB) {
                const double *xn = xs + (16 * (b + 1)) * LD;
                en = mala_d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int j = 0; j < J; ++j)
                    en = __builtin_amdgcn_mfma_f64_16x16x4f64(xn[cl * LD + 4 * j + g], tp[j], en, 0, 0, 0);
            }
            const int rb = 16 * b;
            const double *xb = xs + rb * LD;
            double r[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = 4 * q + g;
                double ell, rr;
                logistic_terms(eta[q], ys[rb + row], ell, rr, mt);
                // rows past N are zero rows of X, so their r only meets zeros in the
                // ∇ℓ MFMA (fma(0, r, G) = G for finite r); only ℓ is masked
                if ((uint32_t)(rb + row) < rem) S = S + ell;
                r[q] = rr;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int e = 0; e < DB; ++e)
                    G[e] = __builtin_amdgcn_mfma_f64_16x16x4f64(xb[(4 * q + g) * LD + 16 * e + cl], r[q], G[e], 0, 0,
                                                               0);
        }
    }
    // lane's ∇ℓ coordinates: G[e][i] ↔ d = 16e + g + 4i ↔ j = 4e + i
    double gp[J];
#pragma unroll
    for (int e = 0; e < DB; ++e)
#pragma unroll
        for (int i = 0; i < 4; ++i) gp[4 * e + i] = G[e][i];

    uint64_t ch = chain;
    asm volatile("" : "+v"(ch));
    if constexpr (MODE == 1) {
        if (valid)
#pragma unroll
            for (int j = 0; j < J; ++j) a.grad[pos(4 * j + g, ch)] = gp[j];
        return;
    }

    // ---- epilogue: reverse density, accept/reject, state, statistics, histories
    const double llp = quad_sum(S);
    double th[J];
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        th[j] = valid ? a.theta[pos(4 * j + g, ch)] : 0.0;
        const double v = (th[j] - (tp[j] + a.h * gp[j])) * a.ieps;
        s = (j == 0) ? v * v : fma(v, v, s);
    }
    const double ltd_rev = fma(-0.5, quad_sum(s), a.c0);
    const double ll = valid ? a.ll[chain] : 0.0;
    if (!(llp - llp == 0.0)) faults |= 1u;
    const double llr = ((((llp - ll) + ltd_rev) - ltd_fwd) + 0.0) - 0.0;
    const double E = exp_draw(zig_tabs(*a.zig), a.key0, a.key1, gid, a.iter, 0, faults);
    const bool acc = E > -llr;
    // the four lanes of a chain drew different normals: merge their fault bits
    faults |= (uint32_t)__shfl_xor((int)faults, 16);
    faults |= (uint32_t)__shfl_xor((int)faults, 32);
    const uint64_t slot = (uint64_t)(a.iter - 1);
    if (valid) {
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const uint64_t p = pos(4 * j + g, ch);
            if constexpr (FULL) {
                __builtin_nontemporal_store(tp[j], a.hist_prop + slot * D * C + p);
                __builtin_nontemporal_store(acc ? tp[j] : th[j], a.hist_theta + slot * D * C + p);
            }
            if (acc) {
                a.theta[p] = tp[j];
                a.grad[p] = gp[j];
            }
        }
    }
    {
        const uint64_t m = __ballot(acc && valid);
        if (lane == 0 && chain < C) {  // lanes 0..15 are the wave's 16 chains (g = 0)
            uint8_t *row = a.hist_acc + slot * a.row_bytes;
            *reinterpret_cast<uint16_t *>(row + (chain >> 3)) = (uint16_t)m;
        }
    }
    if (valid && g == 0) {
        const double lln = acc ? llp : ll;
        a.ll_prop[chain] = llp;
        a.ll[chain] = lln;
        if constexpr (FULL) __builtin_nontemporal_store(lln, a.hist_ll + slot * C + chain);
        uint64_t r0 = a.ring[2 * chain], r1 = a.ring[2 * chain + 1];
        a.ra[chain] = rolling_update(a.ra[chain], r0, r1, a.iter, a.W, a.N0, a.rcp_W, acc);
        a.ring[2 * chain] = r0;
        a.ring[2 * chain + 1] = r1;
        a.nacc[chain] += acc ? 1u : 0u;
        a.faults[chain] = faults;
        if (faults) *a.fault_flag = 1u;
    }
}

}  // namespace emcmc
