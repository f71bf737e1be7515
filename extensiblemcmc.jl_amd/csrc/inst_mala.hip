// inst_mala.hip — gfx950 instantiations of the MALA logistic kernel (emcmc_mala.h).
#include "emcmc_dispatch.h"

namespace emcmc {

template <int DB, bool FULL, int MODE>
MalaFn mala_fn() {
    return &mala_logistic_kernel<DB, FULL, MODE>;
}
MalaFn mala_lookup(int D, bool full, int mode) {
    if (mode == 1) {
        switch (D) {
        case 16: return mala_fn<1, true, 1>();
        case 32: return mala_fn<2, true, 1>();
        case 48: return mala_fn<3, true, 1>();
        case 64: return mala_fn<4, true, 1>();
        default: return nullptr;
        }
    }
    switch (D) {
    case 16: return full ? mala_fn<1, true, 0>() : mala_fn<1, false, 0>();
    case 32: return full ? mala_fn<2, true, 0>() : mala_fn<2, false, 0>();
    case 48: return full ? mala_fn<3, true, 0>() : mala_fn<3, false, 0>();
    case 64: return full ? mala_fn<4, true, 0>() : mala_fn<4, false, 0>();
    default: return nullptr;
    }
}

}  // namespace emcmc
