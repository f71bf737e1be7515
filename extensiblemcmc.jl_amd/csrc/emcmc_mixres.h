// emcmc_mixres.h — GaussianRandomWalkMix step with each chain's Haario factor
// L_B resident in registers for the whole K-step launch (BASELINE cfg 4, gfx950).
//
// Same semantics and the same bits as mix_gsn_kernel<D, FULL, LL, MIX=true,
// DIAG=true> (emcmc_mix.h; oracle/emcmc_oracle.c orc_run_mix), another layout:
// mix_gsn_kernel runs one lane per chain and streams the chain's 4.2 KB of
// L_B from HBM on every step (random_walk.jl:229-232 needs L_B⁻¹(θ° − θ) on
// every step whichever kernel was picked), which bounds it at the HBM roofline.
// Here a chain owns one 16-lane DPP row; lane r holds the folded row pair r and
// 31 − r of L_B (r + 1 and 32 − r nonzeros: 16 + 32 doubles in VGPRs with the
// zero padding, loaded once per launch), so every lane carries the same share of
// the triangle and columns j ≥ 16 touch one row per lane instead of two.
//
//   normals     lane r draws Philox block r: z_{2r}, z_{2r+1} (the pair layout of
//               normals<D>); lane 0 the mixture pick, lanes ≥ 1 the accept Exp(1)
//   θ° = θ + L z  column sweep: z_j broadcast from lane j/2 (row_newbcast), each
//               lane fma's it into its rows r (j < 16) and 31 − r — every row
//               still accumulates over j ascending from L_i0·z_0, the oracle's
//               order; columns past a row's diagonal add 0·z_j, which changes
//               nothing but the sign of an exact zero: a wave-uniform check redoes
//               that (never seen) case with masks
//   layouts     θ and θ° are kept per lane both as the pair (2r, 2r+1) — the HBM
//               layout of θ, the histories and the Σ_A / target terms — and as
//               the folded pair (r, 31 − r) of the L_B sweeps; θ° changes layout
//               through the chain's LDS row (which the per-observation ll reads)
//   y_B = L_B⁻¹(θ° − θ)  column sweep: at column j the owner of row j (lane j,
//               or lane 31 − j for j ≥ 16) forms y_j = acc_j / L_jj (as
//               acc·(1/L_jj)), broadcasts it, every row i > j subtracts L_ij·y_j —
//               the oracle's row order again; every lane sees every y_j, so
//               Σ y_j² is accumulated redundantly in the canonical order
//   Σ_A, Σ_t    diagonal: y_A,i and the target terms sit on the owner lane;
//               canonical blocks of 8 coordinates are exactly the row's quads
//               (serial quad scan, then the blocks' pairwise tree via row_shr)
//   per-observation ll  θ° goes through a per-wave LDS row; lane r evaluates
//               observation r (+16, +32, …) over all D coordinates, and the
//               sum over observations is folded k = 0, 1, … through broadcasts
// The accept bits of a block's 16 chains are two bytes per step: kept in LDS
// for the launch and written once at its end.
#pragma once

#include "emcmc_mix.h"

namespace emcmc {

constexpr int kResLanes = 16;        // lanes per chain: one DPP row
constexpr int kResChainsPerBlock = 16;  // 256-thread block
constexpr int kResWaves = 4;

// dynamic LDS of mix_res_kernel<D>: θ° rows [16 chains][D+2], observations
// [nobs][D+2] (per-observation mode; rows padded by 16 B so that 16 lanes
// reading 16 different rows hit 16 different bank groups), accept nibbles [nsteps][4]
__host__ __device__ constexpr size_t mixres_lds_bytes(int D, uint64_t nobs, uint64_t nsteps_max, bool perobs) {
    return (size_t)kResChainsPerBlock * (D + 2) * 8 + (perobs ? (size_t)nobs * (D + 2) * 8 : 0) +
           (((size_t)nsteps_max * kResWaves + 15) & ~(size_t)15);
}

// lane L of the 16-lane row, to every lane of the row (one v_mov_b64_dpp)
// (mov_dpp: every lane of the row has a source, so no "old" operand — update_dpp(0, …)
// materialised one with a v_mov_b64 + s_nop per broadcast, ≈ 100 per chain-step)
template <int L>
__device__ __forceinline__ double rbcast(double v) {
    const long b = __builtin_amdgcn_mov_dpp(__builtin_bit_cast(long, v), 0x150 + L, 0xF, 0xF, true);
    return __builtin_bit_cast(double, b);
}
template <int L>
__device__ __forceinline__ uint32_t rbcast_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x150 + L, 0xF, 0xF, true);
}

// acc = fma(v from lane L of the 16-lane row, m, acc) as ONE v_fmac_f64_dpp
// (row_newbcast): the broadcast rides on the fma's first source instead of a
// separate v_mov_b64_dpp (VOP3 fma has no DPP form; VOP2 fmac does).  NOP1: two wait
// states first, for a v written by the instruction just before (VALU write → DPP
// read); the callers pass it on the first read of each source.  fma is commutative
// in its products, so the bits are those of fma(m, bcast(v), acc).
template <int L, bool NOP1 = false>
__device__ __forceinline__ void fmac_bcast(double &acc, double v, double m) {
    if constexpr (NOP1)
        asm("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
            : "+v"(acc) : "v"(v), "v"(m), "n"(L));
    else
        asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(v), "v"(m), "n"(L));
}

// Σ y² over the chain's D = 32 coordinates in the canonical order (SumShape<32>:
// blocks of 8 as s = y0·y0, s = fma(y, y, s), then ((b0 + b1) + (b2 + b3))),
// lane r of the row holding coordinates 2r (y0) and 2r+1 (y1): block k is quad k
// of the row.  The result is on every lane of the row.
__device__ __forceinline__ double row_sumsq32(double y0, double y1, bool quad_lead) {
    double a = fma(y1, y1, y0 * y0);  // block start (quad lane 0): y0·y0, then fma
#pragma unroll
    for (int step = 1; step < 4; ++step) {
        // quad_perm [0,0,1,2]: lane q takes lane q−1's partial (lane 0 keeps its own)
        const double p = dpp_perm<0x90>(a);
        const double n = fma(y1, y1, fma(y0, y0, p));
        a = quad_lead ? a : n;
    }
    // block sums in quad lanes 3: lane 7 = b0 + b1, lane 15 = b2 + b3 (operands in order)
    const double s = dpp_perm<0x114>(a) + a;  // row_shr:4
    const double t = dpp_perm<0x118>(s) + s;  // row_shr:8: lane 15 = (b0 + b1) + (b2 + b3)
    return rbcast<15>(t);
}

constexpr int kMixResMinBlocks = 2;  // blocks per CU the register budget is sized for (256 VGPRs, 2 waves/SIMD)
template <int D, bool FULL, int LLMODE, bool UNIT_T>
__global__ void __launch_bounds__(256, kMixResMinBlocks) mix_res_kernel(const MixParams a) {
    static_assert(D == 2 * kResLanes, "two rows of L_B per lane");
    constexpr int DP = packed_n(D), DD = D * D, XS = D + 2;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const uint32_t nobs = a.nobs;
    const ZigTabs zt = stage_lds(lds, a.zig, a.consts, 0, a.obs, 0);  // tables only (static LDS)
    double *const ths = lds;                                           // [16 chains][XS]
    double *const X = lds + kResChainsPerBlock * XS;                   // [nobs][XS]
    uint8_t *const nib =
        reinterpret_cast<uint8_t *>(X + ((LLMODE == LL_PER_OBS) ? (size_t)nobs * XS : 0));  // [nsteps][4]
    if constexpr (LLMODE == LL_PER_OBS) {
        for (uint32_t e = threadIdx.x; e < nobs * D; e += blockDim.x) X[(e / D) * XS + e % D] = a.obs[e];
        __syncthreads();
    }

    const int lane = (int)(threadIdx.x & 63), w = (int)(threadIdx.x >> 6);
    const int g = lane >> 4, r = lane & 15;
    const int i0 = 2 * r, i1 = 2 * r + 1;  // the lane's rows / coordinates
    const bool qlead = (r & 3) == 0;
    const uint64_t C = a.C;
    const uint64_t chain = (uint64_t)blockIdx.x * kResChainsPerBlock + (uint64_t)(w * 4 + g);  // host: C % 16 == 0
    const uint32_t gid = a.chain0 + (uint32_t)chain;
    const uint32_t c32 = (uint32_t)chain;
    double *const tprow = ths + (w * 4 + g) * XS;

    // per-lane constants: Σ_A and Σ_t diagonal (consts = L_A | 1/L_A,ii | L_t | 1/L_t,ii | x̄)
    const double *cs = a.consts;
    const double LA0 = cs[i0 * D + i0], LA1 = cs[i1 * D + i1];
    const double iLA0 = cs[DD + i0], iLA1 = cs[DD + i1];
    const double iLt0 = cs[2 * DD + D + i0], iLt1 = cs[2 * DD + D + i1];
    const double xb0 = cs[2 * DD + 2 * D + i0], xb1 = cs[2 * DD + 2 * D + i1];
    const double *iLt = cs + 2 * DD + D;  // wave-uniform reads (per-observation, non-unit Σ_t)

    // folded rows fa = r (columns 0..15) and fb = 31 − r (columns 0..31) of L_B
    // (packed lower, state_pos layout), zero past the diagonal
    constexpr int H = D / 2;
    const int fa = r, fb = D - 1 - r;
    double La[H], Lb[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
        // lo_idx(i, j) ≤ lo_idx(31, 31) = DP − 1 for every j: the loads stay in bounds
        if (j < H) {
            const double v = a.LB[state_pos((uint64_t)lo_idx(fa, j), chain, C, DP)];
            La[j] = (j <= fa) ? v : 0.0;
        }
        const double v = a.LB[state_pos((uint64_t)lo_idx(fb, j), chain, C, DP)];
        Lb[j] = (j <= fb) ? v : 0.0;
    }
    const double iLBa = a.iLB[(uint64_t)fa * C + chain], iLBb = a.iLB[(uint64_t)fb * C + chain];
    const double c0B = a.c0B[chain];

    const uint64_t po = soa_row((uint64_t)r, chain, C, D / 2) * 16u;  // the lane's pair word in a slot (state_pos)
    double th0, th1;  // θ at coordinates 2r, 2r+1
    {
        const d2v t = *reinterpret_cast<const d2v *>(reinterpret_cast<const char *>(a.theta) + po);
        th0 = t.x;
        th1 = t.y;
    }
    double tfa = a.theta[state_pos((uint64_t)fa, chain, C, D)];  // θ at the folded rows
    double tfb = a.theta[state_pos((uint64_t)fb, chain, C, D)];
    double ll = a.ll[chain];
    double ra = a.ra[chain];
    uint64_t rg0 = a.ring[2 * chain], rg1 = a.ring[2 * chain + 1];
    uint32_t nacc = a.nacc[chain];
    uint32_t faults = a.faults[chain];

    for (uint32_t s = 0; s < a.nsteps; ++s) {
        const uint32_t iter = a.iter0 + s;  // consecutive (host splits gaps)
        const uint64_t N = a.N0 + s;
        const uint64_t slot = (uint64_t)(iter - 1);
        // ---- proposal!: normals (block r of normals<D>), the pick, the accept draw
        double z0, z1;
        {
            const u32x4 q = draw(a.key0, a.key1, gid, iter, (uint32_t)r, 0, 0);
            uint32_t pend = 0;
            if (!zig_normal_fast(zig_split_n(q.x, q.y), zt.n, z0)) pend |= 1u;
            if (!zig_normal_fast(zig_split_n(q.z, q.w), zt.n, z1)) pend |= 2u;
            while (__ballot(pend != 0) != 0) {
                const bool act = pend != 0;
                const uint32_t k = act ? (uint32_t)__builtin_ctz(pend) : 0u;
                pend &= pend - 1;
                double v = 0.0;
                if (act) v = normal_draw(zt, a.key0, a.key1, gid, iter, 0, (uint32_t)i0 + k, faults);
                z0 = (act && k == 0) ? v : z0;
                z1 = (act && k == 1) ? v : z1;
            }
        }
        double ue;
        {
            const bool pick = r == 0;
            const u32x4 q = draw(a.key0, a.key1, gid, pick ? iter : iter >> 1, pick ? kBlockMixPick : kBlockAccept, 0, 0);
            const double u = u01_closed0(q.x, q.y);
            const ZigDraw d = accept_split(q, iter);
            double e;
            const bool fast = zig_exp_fast(d, zt.e, e);
            if (!pick && !fast) e = zig_exp_slow(d, zt.e, zt.ef, a.key0, a.key1, gid, iter, kBlockAccept, 0, faults);
            ue = pick ? u : e;
        }
        const bool useB = rbcast<0>(ue) <= a.lam;
        const double E = rbcast<1>(ue);

        // ---- θ° = θ + L z (random_walk.jl:145-151), L = L_A (diagonal) or L_B
        double lza = 0.0, lzb = 0.0;  // folded rows fa, fb of L_B z
        static_for<0, D>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            if constexpr (j == 0) {
                const double zj = rbcast<0>(z0);
                lza = La[0] * zj;
                lzb = Lb[0] * zj;
            } else {
                // z0 / z1 were written long before the sweep; the first read of each
                // still waits its two states in case a copy was scheduled right before
                if constexpr (j < H) fmac_bcast<j / 2, j == 1 || j == 2>(lza, (j & 1) ? z1 : z0, La[j]);
                fmac_bcast<j / 2, (j == 1 || j == 2) && j >= H>(lzb, (j & 1) ? z1 : z0, Lb[j]);
            }
        });
        if (__ballot(useB && (lza == 0.0 || lzb == 0.0)) != 0) {
            // an exact zero may carry the wrong sign after the padding columns: redo with masks
            static_for<0, D>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                const double zj = rbcast<j / 2>((j & 1) ? z1 : z0);
                if constexpr (j == 0) {
                    lza = La[0] * zj;
                    lzb = Lb[0] * zj;
                } else {
                    if constexpr (j < H) {
                        const double n = fma(La[j], zj, lza);
                        lza = (j <= fa) ? n : lza;
                    }
                    const double n = fma(Lb[j], zj, lzb);
                    lzb = (j <= fb) ? n : lzb;
                }
            });
        }
        // θ° in the layout its kernel produced it in, then through the chain's LDS row
        // into the other one (every lane of the row writes before any reads)
        double thp0 = th0 + LA0 * z0, thp1 = th1 + LA1 * z1;  // pair layout (kernel A)
        double tpa = tfa + lza, tpb = tfb + lzb;              // folded layout (kernel B)
        if (useB) {
            tprow[fa] = tpa;
            tprow[fb] = tpb;
        } else {
            *reinterpret_cast<d2v *>(tprow + i0) = d2v{thp0, thp1};
        }
        wave_lds_sync();
        {
            const d2v t = *reinterpret_cast<const d2v *>(tprow + i0);
            thp0 = t.x;
            thp1 = t.y;
            tpa = tprow[fa];
            tpb = tprow[fb];
        }
        const double rr0 = thp0 - th0, rr1 = thp1 - th1;  // pair layout (Σ_A term)
        const double rra = tpa - tfa, rrb = tpb - tfb;    // folded layout (L_B solve)

        // ---- log_transition_density of the mixture (random_walk.jl:229-232)
        const double qa = row_sumsq32(rr0 * iLA0, rr1 * iLA1, qlead);
        double qbb[4];
        {
            // Column j: the owner's t_j = acc·(1/L_jj) is broadcast as y_B,j. Between the
            // product and its row broadcast (two wait states) go the column-(j−1) work t_j does
            // not need: the other folded row's update (j < 16) and y_{j−1}'s square — the same
            // operations, each accumulator's in its order.
            double acca = rra, accb = rrb, yl = 0.0;
            auto square = [&](auto JC, double y) {
                constexpr int j = decltype(JC)::value;
                if constexpr (j % 8 == 0) qbb[j / 8] = y * y;
                else qbb[j / 8] = fma(y, y, qbb[j / 8]);
            };
            static_for<0, D>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                if constexpr (j > 0) {  // the row t_j reads first
                    if constexpr (j < H) acca = fma(-La[j - 1], yl, acca);
                    else accb = fma(-Lb[j - 1], yl, accb);
                }
                // row j's owner: lane j (row fa) for j < 16, lane 31 − j (row fb) above
                const double t = (j < H) ? acca * iLBa : accb * iLBb;
                if constexpr (j > 0) {
                    if constexpr (j < H) accb = fma(-Lb[j - 1], yl, accb);
                    square(IntC<j - 1>{}, yl);
                }
                yl = rbcast<(j < H) ? j : D - 1 - j>(t);  // y_B,j
            });
            square(IntC<D - 1>{}, yl);
        }
        const double qb = tree_inplace(qbb);
        const double lpA = fma(-0.5, qa, a.c0A);
        const double lpB = fma(-0.5, qb, c0B);
        // both exponentials in one exp_any: lpA and lpB are on every lane of the chain's
        // row, so even lanes take e^{lpA}, odd lanes e^{lpB}, and a quad swap hands
        // each lane the other (one ≈ 35-instruction exp per step instead of two)
        double ltd;
        {
            const bool odd = (r & 1) != 0;
            const double ex = exp_any(odd ? lpB : lpA);
            const double exo = dpp_perm<0xB1>(ex);  // quad_perm [1,0,3,2]: the neighbour's
            const double eA = odd ? exo : ex, eB = odd ? ex : exo;
            ltd = log_any(a.oml * eA + a.lam * eB);
        }

        // ---- compute_ll! (gsn_target.jl:23-29)
        double llp;
        if constexpr (LLMODE == LL_PER_OBS) {
            llp = 0.0;  // θ° is in the chain's LDS row already
            for (uint32_t k0 = 0; k0 < nobs; k0 += kResLanes) {
                const uint32_t k = k0 + (uint32_t)r;
                const double *xr = X + (size_t)(k < nobs ? k : 0u) * XS;
                double b[4];
#pragma unroll
                for (int blk = 0; blk < 4; ++blk) {
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int i = 0; i < 8; i += 2) {
                        const d2v xv = *reinterpret_cast<const d2v *>(xr + 8 * blk + i);
                        const d2v tv = *reinterpret_cast<const d2v *>(tprow + 8 * blk + i);
                        double y0 = xv.x - tv.x, y1 = xv.y - tv.y;
                        if constexpr (!UNIT_T) {
                            y0 = y0 * iLt[8 * blk + i];
                            y1 = y1 * iLt[8 * blk + i + 1];
                        }
                        b[blk] = (i == 0) ? y0 * y0 : fma(y0, y0, b[blk]);
                        b[blk] = fma(y1, y1, b[blk]);
                    }
                }
                // lanes past the last observation contribute −0.0, the exact identity of
                // IEEE addition (x + (−0) = x for every x, ±0 and NaN included): the fold is
                // 16 unconditional adds in k order instead of 16 scalar compare-and-branch
                const double f = (k < nobs) ? fma(-0.5, tree_inplace(b), a.t_c0) : -0.0;
                // llp + f_q as fma(f_q, 1, llp): f_q·1 is exact, so one rounding of the sum
                const double one = 1.0;
                static_for<0, kResLanes>([&](auto rc) {
                    constexpr int q = decltype(rc)::value;
                    fmac_bcast<q, q == 0>(llp, f, one);
                });
            }
        } else {
            double y0 = xb0 - thp0, y1 = xb1 - thp1;
            if constexpr (!UNIT_T) {
                y0 = y0 * iLt0;
                y1 = y1 * iLt1;
            }
            const double qv = row_sumsq32(y0, y1, qlead);
            llp = a.n_tc0 - (a.S_c + a.nobs_d * qv) * 0.5;
        }
        wave_lds_sync();  // the next step's θ° write stays behind this step's reads of the row
        if (!(llp - llp == 0.0)) faults |= 1u;
        // ---- accept_reject! (run.jl:271-278)
        const double llr = ((((llp - ll) + ltd) - ltd) + 0.0) - 0.0;
        const bool acc = E > -llr;
        if constexpr (FULL)
            __builtin_nontemporal_store(d2v{thp0, thp1},
                                        reinterpret_cast<d2v *>(reinterpret_cast<char *>(a.hist_prop + slot * D * C) + po));
        th0 = acc ? thp0 : th0;
        th1 = acc ? thp1 : th1;
        tfa = acc ? tpa : tfa;
        tfb = acc ? tpb : tfb;
        if (s + 1 == a.nsteps && r == 0) a.ll_prop[chain] = llp;
        ll = acc ? llp : ll;
        nacc += acc ? 1u : 0u;
        if constexpr (FULL) {
            __builtin_nontemporal_store(d2v{th0, th1},
                                        reinterpret_cast<d2v *>(reinterpret_cast<char *>(a.hist_theta + slot * D * C) + po));
            if (r == 0) __builtin_nontemporal_store(ll, &chain_elem(a.hist_ll + slot * C, c32));
        } else {
            // mix_moments_kernel reads θ after each step of the launch from here
            *reinterpret_cast<d2v *>(reinterpret_cast<char *>(a.mom_theta + (uint64_t)s * D * C) + po) = d2v{th0, th1};
        }
        {
            const uint64_t m = __ballot(acc);  // lanes 0, 16, 32, 48 carry the wave's 4 chains
            if (lane == 0)
                nib[s * kResWaves + w] = (uint8_t)((m & 1u) | ((m >> 15) & 2u) | ((m >> 30) & 4u) | ((m >> 45) & 8u));
        }
        ra = rolling_update(ra, rg0, rg1, iter, a.W, N, a.rcp_W, acc);
    }

    // accept bits: 16 chains = 2 bytes per slot row
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < a.nsteps; t += blockDim.x) {
        const uint8_t *nb = nib + t * kResWaves;
        const uint16_t v = (uint16_t)(nb[0] | (nb[1] << 4) | (nb[2] << 8) | (nb[3] << 12));
        *reinterpret_cast<uint16_t *>(a.hist_acc + (uint64_t)(a.iter0 + t - 1) * a.row_bytes + blockIdx.x * 2u) = v;
    }
    // fault bits of any lane of the chain's row
    uint32_t f = faults;
    f |= (uint32_t)__builtin_amdgcn_mov_dpp((int)f, 0x111, 0xF, 0xF, true);  // row_shr:1
    f |= (uint32_t)__builtin_amdgcn_mov_dpp((int)f, 0x112, 0xF, 0xF, true);  // row_shr:2
    f |= (uint32_t)__builtin_amdgcn_mov_dpp((int)f, 0x114, 0xF, 0xF, true);  // row_shr:4
    f |= (uint32_t)__builtin_amdgcn_mov_dpp((int)f, 0x118, 0xF, 0xF, true);  // row_shr:8
    faults = rbcast_u32<15>(f);
    if (r == 0) {
        a.ll[chain] = ll;
        a.ra[chain] = ra;
        a.ring[2 * chain] = rg0;
        a.ring[2 * chain + 1] = rg1;
        a.nacc[chain] = nacc;
        a.faults[chain] = faults;
        if (faults) *a.fault_flag = 1u;
    }
    *reinterpret_cast<d2v *>(reinterpret_cast<char *>(a.theta) + po) = d2v{th0, th1};
}

}  // namespace emcmc
