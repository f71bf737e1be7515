// emcmc_dispatch.h — kernel tables shared by the host ABI (emcmc.hip) and the
// per-family instantiation units (inst_*.hip).  Each unit instantiates one
// family of step kernels for gfx950; splitting them lets make build the
// families in parallel.
#pragma once

#include <utility>
#include <vector>

#include "emcmc_kernels.h"
#include "emcmc_chol.h"
#include "emcmc_fused.h"
#include "emcmc_mala.h"
#include "emcmc_mix.h"
#include "emcmc_mwg.h"
#include "emcmc_block.h"

namespace emcmc {

using KernelFn = void (*)(StepParams);
using MwgFn = void (*)(MwgParams);
using MixFn = void (*)(MixParams);
using ReadjustFn = void (*)(MixReadjustParams);
using MalaFn = void (*)(MalaParams);
using MomentsFn = void (*)(MixMomentsParams);

// fused single-update kernels (rwm_gsn_diag_kernel / rwm_gsn_dense_kernel)
struct Key {
    int D, lpc, full, ll, dense, unit, occ;
};
struct Entry {
    Key k;
    KernelFn fn;
};
const std::vector<Entry> &diag_table();
const std::vector<Entry> &diag2_table();  // occ = 2 (≤ 256 registers): inst_diag2.hip
const std::vector<Entry> &chol_table();  // dense = 2 (chol) and 3 (diag_s): inst_chol.hip

// general schedule kernel (mwg_gsn_kernel)
struct MwgEntry {
    int D;
    int nu;  // 0: mwg_gsn_kernel<D> (registers, D ≤ 16); else mwg_wide_kernel<D, nu>
    MwgFn full_perobs, full_suff, acc_perobs, acc_suff;
};
const std::vector<MwgEntry> &mwg_table();

// one MALA update over all D coordinates on the built-in GsnTargetLaw (mwg_block_kernel,
// emcmc_block.h), ahead of time at the D listed in inst_block.hip; other 17 ≤ D ≤ 64,
// user updates and user laws compile at run time
struct BlockEntry {
    int D, tdense, full, ll;
    MwgFn fn;
};
const std::vector<BlockEntry> &block_table();

// GaussianRandomWalkMix / chain moments (mix_gsn_kernel, mix_moments_kernel, mix_readjust_kernel)
struct MixEntry {
    int D, full, ll, mix, adiag;
    MixFn fn;
};
const std::vector<MixEntry> &mix_table();
// the same step for a dense Σ_A / Σ_t at D ≥ 16 with the factors through the
// scalar cache (mix_chol_kernel, emcmc_mix.h; adiag = 0)
const std::vector<MixEntry> &mixchol_table();
// the same step with the chain's L_B resident in registers, 16 lanes per chain
// (mix_res_kernel, emcmc_mixres.h; D = 32, MIX, diagonal Σ_A / Σ_t)
struct MixResEntry {
    int D, full, ll, unit;
    MixFn fn;
};
const std::vector<MixResEntry> &mixres_table();
constexpr int kMixResChainsPerBlock = 16;  // = kResChainsPerBlock (inst_mix.hip checks)
size_t mixres_lds(int D, uint64_t nobs, uint64_t nsteps_max, bool perobs);
std::pair<MomentsFn, int> moments_lookup(int D);
ReadjustFn readjust_lookup(int D);

// MALA on the logistic target (mala_logistic_kernel); mode 1 = ∇ℓ initialisation
MalaFn mala_lookup(int D, bool full, int mode);

}  // namespace emcmc
