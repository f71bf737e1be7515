// inst_diag.hip — gfx950 instantiations of the fused single-update step kernels
// (rwm_gsn_diag_kernel, rwm_gsn_dense_kernel); see emcmc_kernels.h.
#include "emcmc_dispatch.h"

namespace emcmc {

template <int D, int LPC, bool FULL, int LL, bool UNIT, int MINW = 1>
KernelFn diag_fn() {
    return &rwm_gsn_diag_kernel<D, LPC, FULL, LL, UNIT, MINW>;
}
template <int D, bool FULL, int LL>
KernelFn dense_fn() {
    return &rwm_gsn_dense_kernel<D, FULL, LL>;
}

#define DIAGU(D, LPC, U)                                                                          \
    {{D, LPC, 1, 0, 0, U, 0}, diag_fn<D, LPC, true, 0, U>()},                                        \
        {{D, LPC, 1, 1, 0, U, 0}, diag_fn<D, LPC, true, 1, U>()},                                    \
        {{D, LPC, 0, 0, 0, U, 0}, diag_fn<D, LPC, false, 0, U>()},                                   \
        {{D, LPC, 0, 1, 0, U, 0}, diag_fn<D, LPC, false, 1, U>()}
#define DIAG4(D, LPC) DIAGU(D, LPC, false), DIAGU(D, LPC, true)
#define DENSE4(D)                                                                                    \
    {{D, 1, 1, 0, 1, 0, 0}, dense_fn<D, true, 0>()}, {{D, 1, 1, 1, 1, 0, 0}, dense_fn<D, true, 1>()},   \
        {{D, 1, 0, 0, 1, 0, 0}, dense_fn<D, false, 0>()}, {{D, 1, 0, 1, 1, 0, 0}, dense_fn<D, false, 1>()}
const std::vector<Entry> &diag_table() {
    static const std::vector<Entry> t = {
        DIAG4(1, 1),  DIAG4(2, 1),  DIAG4(3, 1),  DIAG4(4, 1),  DIAG4(8, 1),
        DIAG4(16, 1), DIAG4(16, 2), DIAG4(32, 1), DIAG4(32, 2), DIAG4(32, 4),
        DIAG4(64, 2), DIAG4(64, 4),
        DENSE4(1),    DENSE4(2),    DENSE4(3),
        DENSE4(4),    DENSE4(8),
    };
    return t;
}

}  // namespace emcmc
