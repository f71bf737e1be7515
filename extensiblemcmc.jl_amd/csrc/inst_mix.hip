// inst_mix.hip — gfx950 instantiations of the GaussianRandomWalkMix / Haario / chain-moments
// kernels (emcmc_mix.h).
#include "emcmc_dispatch.h"
#include "emcmc_mixres.h"

namespace emcmc {

static_assert(kMixResChainsPerBlock == kResChainsPerBlock, "chains per block of mix_res_kernel");

template <int D, bool FULL, int LL, bool MIX, bool ADIAG>
MixFn mix_fn() {
    return &mix_gsn_kernel<D, FULL, LL, MIX, ADIAG>;
}
#define MIXV(D, F, L, M, A) {D, F, L, M, A, mix_fn<D, F, L, M, A>()}
#define MIX8(D, A)                                                                                         \
    MIXV(D, true, 0, true, A), MIXV(D, true, 1, true, A), MIXV(D, false, 0, true, A),                     \
        MIXV(D, false, 1, true, A), MIXV(D, true, 0, false, A), MIXV(D, true, 1, false, A),                \
        MIXV(D, false, 0, false, A), MIXV(D, false, 1, false, A)
const std::vector<MixEntry> &mix_table() {
    // dense Σ_A / Σ_t for D ≤ 8; D = 16, 32 take diagonal ones (cfg 4: σ²I, I)
    static const std::vector<MixEntry> t = {MIX8(1, true),  MIX8(2, true),  MIX8(2, false), MIX8(3, true),
                                            MIX8(3, false), MIX8(4, true),  MIX8(4, false), MIX8(8, true),
                                            MIX8(8, false), MIX8(16, true), MIX8(32, true)};
    return t;
}
template <int D, bool FULL, int LL, bool MIX>
MixFn mixchol_fn() {
    return &mix_chol_kernel<D, FULL, LL, MIX>;
}
// correlated Σ_A / Σ_t at D ≥ 16: factors through the scalar cache (the entry's
// adiag field is 0: dense)
#define MIXCHOL8(D)                                                                                         \
    {D, true, 0, true, 0, mixchol_fn<D, true, 0, true>()}, {D, true, 1, true, 0, mixchol_fn<D, true, 1, true>()},   \
        {D, false, 0, true, 0, mixchol_fn<D, false, 0, true>()},                                             \
        {D, false, 1, true, 0, mixchol_fn<D, false, 1, true>()},                                             \
        {D, true, 0, false, 0, mixchol_fn<D, true, 0, false>()},                                             \
        {D, true, 1, false, 0, mixchol_fn<D, true, 1, false>()},                                             \
        {D, false, 0, false, 0, mixchol_fn<D, false, 0, false>()},                                           \
        {D, false, 1, false, 0, mixchol_fn<D, false, 1, false>()}
const std::vector<MixEntry> &mixchol_table() {
    static const std::vector<MixEntry> t = {MIXCHOL8(16), MIXCHOL8(32)};
    return t;
}

template <int D, bool FULL, int LL, bool UNIT>
MixFn mixres_fn() {
    return &mix_res_kernel<D, FULL, LL, UNIT>;
}
#define MIXRES(D, F, L, U) {D, F, L, U, mixres_fn<D, F, L, U>()}
const std::vector<MixResEntry> &mixres_table() {
    static const std::vector<MixResEntry> t = {MIXRES(32, true, 0, false), MIXRES(32, true, 1, false),
                                               MIXRES(32, false, 0, false), MIXRES(32, false, 1, false),
                                               MIXRES(32, true, 0, true),  MIXRES(32, true, 1, true),
                                               MIXRES(32, false, 0, true), MIXRES(32, false, 1, true)};
    return t;
}
size_t mixres_lds(int D, uint64_t nobs, uint64_t nsteps_max, bool perobs) {
    return mixres_lds_bytes(D, nobs, nsteps_max, perobs);
}

template <int D>
ReadjustFn readjust_fn() {
    return &mix_readjust_kernel<D>;
}
template <int D>
std::pair<MomentsFn, int> moments_fn() {
    return {&mix_moments_kernel<D>, MomentTiles<D>::WPB};
}
std::pair<MomentsFn, int> moments_lookup(int D) {
    switch (D) {
    case 1: return moments_fn<1>();
    case 2: return moments_fn<2>();
    case 3: return moments_fn<3>();
    case 4: return moments_fn<4>();
    case 8: return moments_fn<8>();
    case 16: return moments_fn<16>();
    case 32: return moments_fn<32>();
    default: return {nullptr, 0};
    }
}

ReadjustFn readjust_lookup(int D) {
    switch (D) {
    case 1: return readjust_fn<1>();
    case 2: return readjust_fn<2>();
    case 3: return readjust_fn<3>();
    case 4: return readjust_fn<4>();
    case 8: return readjust_fn<8>();
    case 16: return readjust_fn<16>();
    case 32: return readjust_fn<32>();
    default: return nullptr;
    }
}


}  // namespace emcmc
