// inst_block.hip — gfx950 instantiations of mwg_block_kernel (emcmc_block.h): one MALA
// update over all D coordinates on the built-in GsnTargetLaw, dense or diagonal Σ_t,
// both history and likelihood modes.  Other D, user updates and user laws: hiprtc.
#include "emcmc_dispatch.h"

namespace emcmc {

template <int D, bool TD, bool FULL, int LL>
MwgFn block_fn() {
    return &mwg_block_kernel<D, FULL, LL, GsnSweep<TD>, MalaOnly>;
}
#define BLOCK8(D)                                                                                        \
    {D, 1, 1, 0, block_fn<D, true, true, 0>()}, {D, 1, 1, 1, block_fn<D, true, true, 1>()},             \
        {D, 1, 0, 0, block_fn<D, true, false, 0>()}, {D, 1, 0, 1, block_fn<D, true, false, 1>()},       \
        {D, 0, 1, 0, block_fn<D, false, true, 0>()}, {D, 0, 1, 1, block_fn<D, false, true, 1>()},       \
        {D, 0, 0, 0, block_fn<D, false, false, 0>()}, {D, 0, 0, 1, block_fn<D, false, false, 1>()}
const std::vector<BlockEntry> &block_table() {
    static const std::vector<BlockEntry> t = {BLOCK8(32)};
    return t;
}

}  // namespace emcmc
