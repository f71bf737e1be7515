// inst_chol.hip — gfx950 instantiations of the fused single-update kernels that
// read their wave-uniform operands through the scalar cache: rwm_gsn_chol_kernel
// (correlated Σ_rw / Σ_t, key dense = 2) and rwm_gsn_diag_s_kernel (one lane per
// chain, observations as SGPR operands, key dense = 3); see emcmc_kernels.h.
// (A unit of their own: with rwm_gsn_diag_kernel<32, 1, …> in the same unit the
// ROCm 7.2 inliner crashes.)
#include "emcmc_dispatch.h"

namespace emcmc {

template <int D, bool FULL, int LL>
KernelFn chol_fn() {
    return &rwm_gsn_chol_kernel<D, FULL, LL>;
}
template <int D, bool FULL, int LL, bool UNIT>
KernelFn diag_s_fn() {
    return &rwm_gsn_diag_s_kernel<D, FULL, LL, UNIT>;
}

#define CHOL4(D)                                                                                     \
    {{D, 1, 1, 0, 2, 0, 0}, chol_fn<D, true, 0>()}, {{D, 1, 1, 1, 2, 0, 0}, chol_fn<D, true, 1>()},     \
        {{D, 1, 0, 0, 2, 0, 0}, chol_fn<D, false, 0>()}, {{D, 1, 0, 1, 2, 0, 0}, chol_fn<D, false, 1>()}
#define DIAGS(D, U)                                                                                       \
    {{D, 1, 1, 0, 3, U, 0}, diag_s_fn<D, true, 0, U>()}, {{D, 1, 1, 1, 3, U, 0}, diag_s_fn<D, true, 1, U>()}, \
        {{D, 1, 0, 0, 3, U, 0}, diag_s_fn<D, false, 0, U>()}, {{D, 1, 0, 1, 3, U, 0}, diag_s_fn<D, false, 1, U>()}

const std::vector<Entry> &chol_table() {
    static const std::vector<Entry> t = {
        CHOL4(16), CHOL4(24), CHOL4(32), DIAGS(32, true), DIAGS(32, false),
    };
    return t;
}

}  // namespace emcmc
