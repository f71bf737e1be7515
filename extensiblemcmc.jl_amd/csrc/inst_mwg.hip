// inst_mwg.hip — gfx950 instantiations of the general schedule kernel (emcmc_mwg.h).
#include "emcmc_dispatch.h"

namespace emcmc {

template <int D, bool FULL, int LL>
MwgFn mwg_fn() {
    return &mwg_gsn_kernel<D, FULL, LL>;
}
template <int D, int NU, bool FULL, int LL>
MwgFn mwg_wide_fn() {
    return &mwg_wide_kernel<D, NU, FULL, LL>;
}
#define MWG4(D) \
    {D, 0, mwg_fn<D, true, 0>(), mwg_fn<D, true, 1>(), mwg_fn<D, false, 0>(), mwg_fn<D, false, 1>()}
#define MWGW4(D, NU)                                                                                  \
    {D, NU, mwg_wide_fn<D, NU, true, 0>(), mwg_wide_fn<D, NU, true, 1>(), mwg_wide_fn<D, NU, false, 0>(), \
     mwg_wide_fn<D, NU, false, 1>()}
const std::vector<MwgEntry> &mwg_table() {
    static const std::vector<MwgEntry> t = {MWG4(1),  MWG4(2),  MWG4(3),        MWG4(4),
                                            MWG4(8),  MWG4(16), MWGW4(32, 16), MWGW4(32, 32)};
    return t;
}


}  // namespace emcmc
