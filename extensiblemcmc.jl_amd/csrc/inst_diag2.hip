// inst_diag2.hip — rwm_gsn_diag_kernel with its registers capped for 2 waves per
// SIMD (MINW = 2: ≤ 256 VGPRs + AGPRs) at the shapes whose uncapped build needs a
// few more than 256 and would run one wave per SIMD: D = 16 (LPC 1), D = 32
// (LPC 2: the cfg 2 headline kernel) and D = 64 (LPC 4).  At 65,536 chains and
// LPC = 2 the grid is 2048 waves, exactly 2 per SIMD: capped, every wave is
// resident from the start; uncapped, the grid runs as two rounds of 1024 waves
// (scripts/trace_diag.py).  A unit of its own so that `make -j` builds it beside
// inst_diag.hip.
#include "emcmc_dispatch.h"

namespace emcmc {

template <int D, int LPC, bool FULL, int LL, bool UNIT>
KernelFn diag2_fn() {
    return &rwm_gsn_diag_kernel<D, LPC, FULL, LL, UNIT, 2>;
}

#define DIAG2U(D, LPC, U)                                                                         \
    {{D, LPC, 1, 0, 0, U, 2}, diag2_fn<D, LPC, true, 0, U>()},                                       \
        {{D, LPC, 1, 1, 0, U, 2}, diag2_fn<D, LPC, true, 1, U>()},                                   \
        {{D, LPC, 0, 0, 0, U, 2}, diag2_fn<D, LPC, false, 0, U>()},                                  \
        {{D, LPC, 0, 1, 0, U, 2}, diag2_fn<D, LPC, false, 1, U>()}
#define DIAG2(D, LPC) DIAG2U(D, LPC, false), DIAG2U(D, LPC, true)

const std::vector<Entry> &diag2_table() {
    static const std::vector<Entry> t = {DIAG2(16, 1), DIAG2(32, 2), DIAG2(64, 4)};
    return t;
}

}  // namespace emcmc
