// emcmc.hip — libemcmc.so: C ABI (include/emcmc.h) over the gfx950 MCMC step
// kernels in emcmc_kernels.h.  Build: see extensiblemcmc.jl_amd/Makefile
// (hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared).
//
// The host side here plays the role of the reference's workspace/backend
// layer (src/workspaces.jl, src/mcmc.jl): it owns the chain state (SoA in
// HBM), factorises the Gaussian covariances once (the reference re-factorises
// at every MvNormal construction, random_walk.jl:147,167 and
// gsn_target.jl:20 — same matrices, so the same factor), and turns a schedule
// of (mcmciter, pidx) steps into fused multi-step launches.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#define EMCMC_HOST_UNIT 1  // this unit compiles the diagnostics / probe kernels
#include "../../include/emcmc.h"
#include "emcmc_kernels.h"
#include "emcmc_mala.h"
#include "emcmc_mix.h"
#include "emcmc_mwg.h"
#include "emcmc_dispatch.h"
#include "emcmc_rwblock.h"
#include "emcmc_rtc.h"

using namespace emcmc;

namespace {

constexpr uint32_t kDefaultRollWindow = 100;  // chain_statistics.jl:27
constexpr uint32_t kDefaultStepsPerLaunch = 64;
constexpr size_t kMaxLds = 160 * 1024;  // gfx950: 160 KiB of LDS per CU, all of it addressable by one workgroup

// ----------------------------------------------------------------------------
// Canonical Cholesky (lower factor L of the upper-stored symmetric Σ), the
// order oracle/emcmc_oracle.c restates.  Returns false if Σ is not positive
// definite (the reference throws PosDefException from cholesky()).
bool cholesky_upper_colmajor(const double *S, int D, std::vector<double> &L) {
    L.assign((size_t)D * D, 0.0);
    for (int j = 0; j < D; ++j) {
        double s = S[j + (size_t)j * D];
        for (int k = 0; k < j; ++k) s = s - L[(size_t)j * D + k] * L[(size_t)j * D + k];
        if (!(s > 0.0)) return false;
        const double ljj = std::sqrt(s);
        L[(size_t)j * D + j] = ljj;
        for (int i = j + 1; i < D; ++i) {
            double t = S[j + (size_t)i * D];  // Σ(j,i), upper triangle
            for (int k = 0; k < j; ++k) t = t - L[(size_t)i * D + k] * L[(size_t)j * D + k];
            L[(size_t)i * D + j] = t / ljj;
        }
    }
    return true;
}

bool is_diag_upper(const double *S, int D) {
    for (int i = 0; i < D; ++i)
        for (int j = i + 1; j < D; ++j)
            if (S[i + (size_t)j * D] != 0.0) return false;
    return true;
}

// logdet of a Cholesky factor as LinearAlgebra.logdet(::Cholesky): dd + dd
double logdet_chol(const std::vector<double> &L, int D) {
    double dd = 0.0;
    for (int i = 0; i < D; ++i) dd = dd + log_pos(L[(size_t)i * D + i]);
    return dd + dd;
}

// Distributions.mvnormal_c0: −(D·log2π + logdet)/2
double mvnormal_c0(int D, double logdet) { return -((double)D * kLog2Pi + logdet) / 2.0; }

// host restatement of the canonical blocked sum of squares (used for S_c)
double canon_sumsq_host(const double *y, int D) {
    const int BLK = (D % 8 == 0 && D >= 16) ? 8 : D;
    const int NB = D / BLK;
    std::vector<double> b(NB);
    for (int k = 0; k < NB; ++k) {
        double s = y[k * BLK] * y[k * BLK];
        for (int i = 1; i < BLK; ++i) s = std::fma(y[k * BLK + i], y[k * BLK + i], s);
        b[k] = s;
    }
    int n = NB;
    while (n > 1) {
        for (int i = 0; i < n / 2; ++i) b[i] = b[2 * i] + b[2 * i + 1];
        if (n & 1) b[n / 2] = b[n - 1];
        n = (n + 1) / 2;
    }
    return b[0];
}

struct UpdateHost {
    uint32_t kernel = 0, prior = 0, adaptation = 0;
    std::vector<uint32_t> coords;
    std::vector<double> sigma, L, invdiag;  // GaussianRandomWalk
    std::vector<double> eps;                // UniformRandomWalk ϵ
    std::vector<uint8_t> pos;               // UniformRandomWalk positivity flags (random_walk.jl:45-52)
    emcmc_unifrw_adaptation adpt{};         // AdaptationUnifRW: k and target
    std::vector<double> ascale, amin, amax, aoff;  // its per-coordinate scale/min/max/offset
    bool diag = false;
    double c0 = 0.0;
    // GaussianRandomWalkMix: Σ_B, its factor, λ; HaarioTypeAdaptation
    std::vector<double> sigma_b, LB, invdiagB;
    double c0B = 0.0, lam = 0.0, lam0 = 0.0;  // λ now / as constructed (emcmc_set_state restores it)
    // general-kernel per-chain state offsets in emcmc_handle::d_mixpool (MwgUpdate)
    uint64_t lb_off = 0, lbi_off = 0, lbc_off = 0, lbs_off = 0, hm_off = 0, hc_off = 0;
    emcmc_haario_adaptation haario{};
    emcmc_lambda_fn flam = nullptr;  // HaarioTypeAdaptation fλ (host callback; nullptr = identity)
    void *flam_ctx = nullptr;
    // EMCMC_USER_UPDATE: the source (shared by the handle's user updates) and parameters
    std::string usrc, uopts;
    std::vector<double> uparams;
    // prior (priors.jl) as MwgUpdate term slots (emcmc_mwg.h): per slot a family,
    // its parameters and host constant; MvNormal rows; factor boundaries
    uint32_t nslot = 0;
    uint64_t psrc0 = 0, pstart = 0, pend = 0, pmvn = 0;
    std::vector<uint32_t> pfam, pmvs;
    std::vector<double> pa, pb, pc, pmu, piL, pL;
};

struct TargetHost {
    uint32_t kind = EMCMC_TARGET_GSN;
    std::vector<double> labels;  // EMCMC_TARGET_LOGISTIC: y
    uint32_t dim = 0, ll_mode = 0;
    uint64_t nobs = 0;
    std::vector<double> mu, sigma, L, invdiag, obs, xbar;
    bool diag = false;
    double c0 = 0.0, S_c = 0.0;
    // EMCMC_TARGET_USER: the law's source, hiprtc options, constants, row width
    std::string src, opts;
    std::vector<double> params;
    uint32_t obs_dim = 0;
};


struct Variant {
    KernelFn fn = nullptr;
    MwgFn mfn = nullptr;  // general schedule kernel (mwg_gsn_kernel) when set
    hipFunction_t ufn = nullptr;  // the same kernel with a user law, compiled at run time (emcmc_rtc.hip)
    MixFn xfn = nullptr;  // mix / chain-moments kernel (mix_gsn_kernel) when set
    ReadjustFn rfn = nullptr;  // Haario readjust kernel
    MomentsFn mofn = nullptr;  // batched chain mean/cov (mix_moments_kernel)
    int mo_tiles = 0;
    MalaFn afn = nullptr, ainit = nullptr;  // MALA step / ∇ℓ initialisation kernels
    hipFunction_t ffn = nullptr;  // a fused single-update kernel compiled at run time (rwm_gsn_chol_kernel
                                  // at a D without an ahead-of-time instantiation)
    bool mix = false;
    bool xres = false;  // xfn is mix_res_kernel (16 lanes per chain, L_B in registers)
    bool xchol = false;  // xfn is mix_chol_kernel (dense Σ_A / Σ_t through the scalar cache)
    bool block = false;  // mfn / ufn is mwg_block_kernel (one MALA or user update over all D coordinates)
    int lpc = 1;
    int dense = 0;  // 0 rwm_gsn_diag_kernel, 1 rwm_gsn_dense_kernel, 2 rwm_gsn_chol_kernel
    bool unit = false;
    int occ = 0;
    std::string name;
};

}  // namespace

struct emcmc_handle {
    emcmc_config cfg{};
    hipStream_t stream = nullptr;
    std::string err;
    std::vector<UpdateHost> updates;
    TargetHost target;
    bool target_set = false, allocated = false;
    uint64_t stats_N = 1;  // GenericChainStats.N (chain_statistics.jl:34)
    // device buffers
    double *d_theta = nullptr, *d_ll = nullptr, *d_ra = nullptr;
    // non-null: the current θ is this FULL-history slot (the last launch of rwm_gsn_diag_kernel
    // left it there and did not write d_theta); settle_theta copies it back before any other use
    double *theta_live = nullptr;
    bool theta_live_ok = true;  // EMCMC_THETA_LIVE=0: always write the state buffer (A/B)
    uint64_t *d_ring = nullptr;
    uint32_t *d_nacc = nullptr, *d_faults = nullptr;
    // any-fault word, written by the kernels only when a chain ends a launch faulted:
    // host-mapped pinned memory, so emcmc_synchronize reads 4 B after the stream
    // drains instead of copying and scanning C fault words
    uint32_t *h_fault_flag = nullptr, *d_fault_flag = nullptr;
    double *d_ll_prop = nullptr;  // [P][C] sub_ws°.ll of each update's latest proposal
    double *d_hist_theta = nullptr, *d_hist_prop = nullptr, *d_hist_ll = nullptr;
    uint8_t *d_hist_acc = nullptr;
    double *d_consts = nullptr, *d_obs = nullptr;
    Ziggurat *d_zig = nullptr;
    double *d_scratch = nullptr;  // diagnostics
    size_t scratch_bytes = 0;
    double *d_gather = nullptr;   // history layout conversion
    size_t gather_bytes = 0;
    uint64_t row_bytes = 0;
    // general schedule path (mwg_gsn_kernel)
    double *d_mu_p = nullptr, *d_eps = nullptr, *d_tL = nullptr, *d_tiL = nullptr, *d_xbar = nullptr;
    double *d_gcache = nullptr;  // MALA: ∇ℓ(θ) carried between the steps of a launch (emcmc_mwg.h mala_carry)
    double *d_bconsts = nullptr;  // mwg_block_kernel's constant table (emcmc_block.h BlockConsts)
    uint32_t *d_aprop = nullptr, *d_aacc = nullptr, *d_steps = nullptr;
    MwgUpdate *d_mwg = nullptr;
    // user target (EMCMC_TARGET_USER): the loaded code object and the law's constants
    hipModule_t umod = nullptr;
    std::string umod_key;
    uint32_t rtc_origin = 0;  // emcmc_rtc_info of the loaded module
    double rtc_seconds = 0.0;
    double *d_uparams = nullptr;
    std::vector<uint32_t> last_iter;                    // per update: last iteration it ran (uniform)
    std::vector<std::vector<uint32_t>> steps_staging;   // host step lists alive until synchronize
    std::vector<std::vector<double>> lam_staging;       // fλ values of a run's launch cuts, alive until synchronize
    uint64_t steps_used = 0;
    // mix / chain-moments path (mix_gsn_kernel): GenericChainStats mean/cov,
    // per-chain Σ_B factor, Haario M (same for every chain)
    double *d_mean = nullptr, *d_cov = nullptr, *d_LB = nullptr, *d_iLB = nullptr, *d_c0B = nullptr;
    double *d_Lnew = nullptr;
    double *d_mean_alt = nullptr;  // the moments kernel's output mean (swapped with d_mean per launch)
    double *d_mom_consts = nullptr;  // [steps_per_launch][8] per-step scalars of the moments recurrence
    double *d_mom_scratch = nullptr;  // ACCEPT_ONLY: θ of each step of a launch, for the moments kernel
    uint32_t mix_M = 0;
    // general schedule path: GaussianRandomWalkMix / Haario per-chain pool,
    // GenericChainStats mean [D][C] / cov packed [D(D+1)/2][C], Haario M per update
    double *d_mixpool = nullptr;
    uint64_t mixpool_elems = 0;
    double *d_smean = nullptr, *d_scov = nullptr;
    std::vector<uint32_t> mwg_M;
    uint32_t nhaario = 0;
    bool mwg_pool_ready = false;
    // MALA path: carried ∇ℓ(θ) (state_pos layout), padded X and y
    double *d_grad = nullptr, *d_X = nullptr, *d_y = nullptr;
    uint32_t mala_tiles = 0;
    bool grad_valid = false;
    // dispatch
    Variant var;
    size_t lds_bytes = 0;
    // history ring (emcmc_config.history_ring) and streaming copies
    uint64_t ring = 0;     // iterations held per history buffer
    uint64_t hi_iter = 0;  // highest iteration launched
    hipStream_t cstream = nullptr;
    struct Copy {
        uint64_t lo, hi;  // iterations read
        hipEvent_t ev;
    };
    std::vector<Copy> copies;
    double *d_stage = nullptr;
    size_t stage_bytes = 0;
    // timing
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
    std::vector<hipEvent_t> ev_pool;
    double timed_ms = 0.0;
    uint64_t timed_launches = 0;
    double timed_bytes = 0.0;
    double pending_bytes = 0.0;
    // EMCMC_HOST_TIMING=1: the host side of emcmc_run / emcmc_synchronize, summed and
    // printed to stderr at emcmc_destroy (how the wall of a short window splits)
    bool host_timing = false;
    double ht_run_us = 0.0, ht_sync_us = 0.0;
    uint64_t ht_runs = 0, ht_syncs = 0;
    // how emcmc_synchronize waits: 1 (default) an event recorded behind the queued work and
    // hipEventSynchronize, ≈ 6 µs less than 0 = hipStreamSynchronize on a 150 µs window
    // (scripts/host_gap.py); EMCMC_SYNC=0 selects the latter for A/B
    int sync_mode = 1;
    hipEvent_t sync_ev = nullptr;
};

namespace {

emcmc_status fail(emcmc_handle *h, emcmc_status st, const char *fmt, ...) {
    if (h) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        h->err = buf;
    }
    return st;
}

#define HIPCHK(h, expr)                                                                       \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail((h), e_ == hipErrorOutOfMemory ? EMCMC_OUT_OF_MEMORY : EMCMC_HIP_ERROR, \
                        "%s failed: %s", #expr, hipGetErrorString(e_));                       \
    } while (0)

KernelFn lookup(int D, int lpc, bool full, int ll, int dense, bool unit, int occ = 0) {
    for (const auto *tab : {&diag_table(), &diag2_table(), &chol_table()})
        for (const auto &e : *tab)
            if (e.k.D == D && e.k.lpc == lpc && e.k.full == (int)full && e.k.ll == ll && e.k.dense == dense &&
                e.k.unit == (int)unit && e.k.occ == occ)
                return e.fn;
    return nullptr;
}

// lanes per chain: 16 coordinates per lane where D allows (measured best at
// D=32: fewer duplicated per-chain scalar ops than LPC=4, 2 waves/SIMD)
int auto_lpc(int D) {
    if (D % 16 == 0 && D >= 32) return D / 16 <= 4 ? D / 16 : 4;
    if (D % 16 == 0) return 2;
    return 1;
}

// one update, joint on coords 1:D in order
bool joint_all_coords(const emcmc_handle *h) {
    if (h->updates.size() != 1) return false;
    const UpdateHost &u = h->updates[0];
    if (u.coords.size() != h->cfg.dim) return false;
    for (uint32_t i = 0; i < h->cfg.dim; ++i)
        if (u.coords[i] != i) return false;
    return true;
}

// GaussianRandomWalkMix (± Haario), or GaussianRandomWalk with chain moments:
// the mix kernels
// the fused mix / chain-moments kernels (cfg 4): one joint update on coords 1:D,
// ImproperPrior, no positivity flags, the built-in target; everything else with
// GaussianRandomWalkMix or chain moments runs on the general kernel
bool mix_path(const emcmc_handle *h) {
    if (!joint_all_coords(h)) return false;
    if (h->target_set && h->target.kind != EMCMC_TARGET_GSN) return false;
    const UpdateHost &u = h->updates[0];
    if (u.prior != EMCMC_PRIOR_IMPROPER) return false;
    for (uint8_t f : u.pos)
        if (f) return false;
    return u.kernel == EMCMC_RW_GAUSSIAN_MIX ||
           (u.kernel == EMCMC_RW_GAUSSIAN && u.adaptation == EMCMC_ADPT_NONE && h->cfg.chain_moments);
}

// general kernel: layout of the per-chain mix / Haario pool (MwgUpdate offsets)
uint64_t mwg_pool_layout(emcmc_handle *h) {
    const uint64_t C = h->cfg.num_chains;
    uint64_t off = 0;
    h->nhaario = 0;
    for (auto &u : h->updates) {
        const uint64_t n = u.coords.size(), tn = n * (n + 1) / 2;
        u.lb_off = u.lbi_off = u.lbc_off = u.lbs_off = u.hm_off = u.hc_off = 0;
        if (u.kernel != EMCMC_RW_GAUSSIAN_MIX) continue;
        u.lb_off = off, off += tn * C;
        u.lbi_off = off, off += n * C;
        u.lbc_off = off, off += C;
        u.lbs_off = off, off += tn * C;
        if (u.adaptation == EMCMC_ADPT_HAARIO) {
            u.hm_off = off, off += n * C;
            u.hc_off = off, off += tn * C;
            ++h->nhaario;
        }
    }
    return off;
}

// (Re)start the general kernel's mix / Haario / chain-moment state: every chain's
// L_B from the user's Σ_B, Haario mean/cov and GenericChainStats mean/cov zero
// (N = 1, the phantom zero sample: chain_statistics.jl:30-35, adaptation.jl:387-395).
emcmc_status reset_mwg_pool(emcmc_handle *h) {
    const uint64_t C = h->cfg.num_chains, D = h->cfg.dim;
    // queued kernels read and write the pool on h->stream (non-blocking: the null
    // stream's copies below would not wait for them)
    if (h->allocated) HIPCHK(h, hipStreamSynchronize(h->stream));
    const uint64_t elems = mwg_pool_layout(h);
    if (elems != h->mixpool_elems) {
        if (h->d_mixpool) (void)hipFree(h->d_mixpool);
        h->d_mixpool = nullptr;
        h->mixpool_elems = elems;
        if (elems) HIPCHK(h, hipMalloc(&h->d_mixpool, elems * sizeof(double)));
    }
    if (elems) {
        std::vector<double> pool(elems, 0.0);
        for (const auto &u : h->updates) {
            if (u.kernel != EMCMC_RW_GAUSSIAN_MIX) continue;
            const uint64_t n = u.coords.size();
            for (uint64_t i = 0; i < n; ++i) {
                for (uint64_t j = 0; j <= i; ++j)
                    std::fill_n(pool.begin() + u.lb_off + (i * (i + 1) / 2 + j) * C, C, u.LB[i * n + j]);
                std::fill_n(pool.begin() + u.lbi_off + i * C, C, u.invdiagB[i]);
            }
            std::fill_n(pool.begin() + u.lbc_off, C, u.c0B);
        }
        HIPCHK(h, hipMemcpy(h->d_mixpool, pool.data(), elems * sizeof(double), hipMemcpyHostToDevice));
    }
    if (h->cfg.chain_moments) {
        const uint64_t DP = D * (D + 1) / 2;
        if (!h->d_smean) {
            HIPCHK(h, hipMalloc(&h->d_smean, D * C * sizeof(double)));
            HIPCHK(h, hipMalloc(&h->d_scov, DP * C * sizeof(double)));
        }
        HIPCHK(h, hipMemset(h->d_smean, 0, D * C * sizeof(double)));
        HIPCHK(h, hipMemset(h->d_scov, 0, DP * C * sizeof(double)));
    }
    h->mwg_M.assign(h->updates.size(), 0u);
    h->mwg_pool_ready = true;
    return EMCMC_OK;
}

// P°.θ[1:d] ← μ for every chain (workspaces.jl:225-233: P° = deepcopy(data.P))
emcmc_status reset_mu_p(emcmc_handle *h) {
    if (h->target.kind != EMCMC_TARGET_GSN && h->target.kind != EMCMC_TARGET_USER) return EMCMC_OK;
    const uint64_t C = h->cfg.num_chains, D = h->cfg.dim;
    std::vector<double> m(C * D);
    for (uint64_t c = 0; c < C; ++c)
        for (uint64_t d = 0; d < D; ++d) m[state_pos(d, c, C, (uint32_t)D)] = h->target.mu[d];
    HIPCHK(h, hipMemcpy(h->d_mu_p, m.data(), m.size() * sizeof(double), hipMemcpyHostToDevice));
    return EMCMC_OK;
}

emcmc_status ensure_alloc(emcmc_handle *h) {
    if (h->allocated) return EMCMC_OK;
    if (h->updates.empty()) return fail(h, EMCMC_STATE_ERROR, "no update added (emcmc_add_update)");
    const uint64_t C = h->cfg.num_chains, D = h->cfg.dim, M = h->cfg.num_mcmc_steps;
    const uint64_t P = h->updates.size();
    HIPCHK(h, hipMalloc(&h->d_theta, C * D * sizeof(double)));
    HIPCHK(h, hipMalloc(&h->d_ll, C * sizeof(double)));
    // per-update chain statistics [P][C] (the fused kernels use update 0)
    HIPCHK(h, hipMalloc(&h->d_ra, P * C * sizeof(double)));
    HIPCHK(h, hipMalloc(&h->d_ring, 2 * P * C * sizeof(uint64_t)));
    HIPCHK(h, hipMalloc(&h->d_nacc, P * C * sizeof(uint32_t)));
    HIPCHK(h, hipMalloc(&h->d_faults, C * sizeof(uint32_t)));
    HIPCHK(h, hipHostMalloc(reinterpret_cast<void **>(&h->h_fault_flag), sizeof(uint32_t), hipHostMallocMapped));
    HIPCHK(h, hipHostGetDevicePointer(reinterpret_cast<void **>(&h->d_fault_flag), h->h_fault_flag, 0));
    *h->h_fault_flag = 0u;
    // general schedule path: P° mean, AdaptationUnifRW state, step lists
    HIPCHK(h, hipMalloc(&h->d_mu_p, C * D * sizeof(double)));
    HIPCHK(h, hipMalloc(&h->d_aprop, P * C * sizeof(uint32_t)));
    HIPCHK(h, hipMalloc(&h->d_aacc, P * C * sizeof(uint32_t)));
    HIPCHK(h, hipMalloc(&h->d_ll_prop, P * C * sizeof(double)));
    HIPCHK(h, hipMalloc(&h->d_eps, P * kMwgMaxD * C * sizeof(double)));
    HIPCHK(h, hipMalloc(&h->d_steps, M * P * 4 * sizeof(uint32_t)));
    {
        Ziggurat zt;
        build_ziggurat(zt);
        HIPCHK(h, hipMalloc(&h->d_zig, sizeof(Ziggurat)));
        HIPCHK(h, hipMemcpy(h->d_zig, &zt, sizeof(Ziggurat), hipMemcpyHostToDevice));
    }
    if (h->updates[0].kernel == EMCMC_MALA) HIPCHK(h, hipMalloc(&h->d_grad, C * D * sizeof(double)));
    if (mix_path(h)) {  // GenericChainStats mean/cov; Σ_B factors
        const uint64_t DP = (uint64_t)packed_n((int)D);
        const UpdateHost &u = h->updates[0];
        HIPCHK(h, hipMalloc(&h->d_mean, C * D * sizeof(double)));
        HIPCHK(h, hipMalloc(&h->d_mean_alt, C * D * sizeof(double)));
        HIPCHK(h, hipMalloc(&h->d_mom_consts, (uint64_t)h->cfg.steps_per_launch * 8 * sizeof(double)));
        HIPCHK(h, hipMalloc(&h->d_cov, C * DP * sizeof(double)));
        if (u.kernel == EMCMC_RW_GAUSSIAN_MIX) {
            HIPCHK(h, hipMalloc(&h->d_LB, C * DP * sizeof(double)));
            HIPCHK(h, hipMalloc(&h->d_iLB, C * D * sizeof(double)));
            HIPCHK(h, hipMalloc(&h->d_c0B, C * sizeof(double)));
        }
        if (h->cfg.history_mode != EMCMC_HIST_FULL)
            HIPCHK(h, hipMalloc(&h->d_mom_scratch, (uint64_t)h->cfg.steps_per_launch * C * D * sizeof(double)));
    }
    h->row_bytes = ((C + 63) / 64) * 8;
    const uint64_t R = h->ring;  // history slots: a ring of R iterations (R = M unless history_ring)
    HIPCHK(h, hipMalloc(&h->d_hist_acc, R * P * h->row_bytes));
    HIPCHK(h, hipMemsetAsync(h->d_hist_acc, 0, R * P * h->row_bytes, h->stream));
    if (h->cfg.history_mode == EMCMC_HIST_FULL) {
        HIPCHK(h, hipMalloc(&h->d_hist_theta, R * P * C * D * sizeof(double)));
        HIPCHK(h, hipMalloc(&h->d_hist_prop, R * P * C * D * sizeof(double)));
        HIPCHK(h, hipMalloc(&h->d_hist_ll, R * P * C * sizeof(double)));
        // The reference preallocates its histories zero-filled in init! (workspaces.jl:413-476,
        // `zero(θ)` per slot): a slot read before its iteration ran reads 0, as there.  (The
        // zero-fill does not change the step kernels' time: DESIGN.md §6, r3 zero-fill A/B.)
        HIPCHK(h, hipMemsetAsync(h->d_hist_theta, 0, R * P * C * D * sizeof(double), h->stream));
        HIPCHK(h, hipMemsetAsync(h->d_hist_prop, 0, R * P * C * D * sizeof(double), h->stream));
        HIPCHK(h, hipMemsetAsync(h->d_hist_ll, 0, R * P * C * sizeof(double), h->stream));
    }
    h->allocated = true;
    return EMCMC_OK;
}

// Every schedule but one joint GaussianRandomWalk update on coords 1:D runs on
// mwg_gsn_kernel: per-update constants as MwgUpdate records (scalar loads),
// target factor / x̄ / observations in plain global memory.
// Dynamic LDS beyond 64 KiB in total (with the static tables) must be allowed
// per kernel.
emcmc_status allow_lds(emcmc_handle *h, const void *fn, size_t bytes) {
    if (fn && kZigLdsBytes + bytes > 64 * 1024)
        HIPCHK(h, hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    return EMCMC_OK;
}

// Load a run-time compiled code object as the handle's module (kept while the
// same kernel stays selected).
emcmc_status load_rtc_module(emcmc_handle *h, const RtcKernel &k) {
    const std::string key = std::to_string(h->cfg.device) + '|' + k.name + '|' + k.lowered + '|' +
                            std::to_string(std::hash<std::string>{}(std::string(k.code.begin(), k.code.end())));
    h->rtc_origin = k.origin;
    h->rtc_seconds = k.seconds;
    if (key == h->umod_key) return EMCMC_OK;
    // Loaded modules stay loaded for the life of the process, one per (device, code object),
    // shared by every handle that selects the kernel: a handle never unloads code another
    // handle (or a later allocation at the same addresses) could meet, and re-creating an
    // engine for a known kernel costs no load.
    static std::mutex mu;
    static std::map<std::string, hipModule_t> loaded;
    std::lock_guard<std::mutex> lock(mu);
    auto it = loaded.find(key);
    if (it == loaded.end()) {
        HIPCHK(h, hipSetDevice(h->cfg.device));
        hipModule_t m = nullptr;
        HIPCHK(h, hipModuleLoadData(&m, k.code.data()));
        it = loaded.emplace(key, m).first;
    }
    h->umod = it->second;
    h->umod_key = key;
    return EMCMC_OK;
}

// Every ahead-of-time code object of the library (one per translation unit) is loaded when
// the first handle of a device is created, before that process loads any run-time module or
// allocates any handle buffer; HIP would otherwise load a translation unit's code object at
// the first launch of one of its kernels, in the middle of a run.
void load_aot_code_objects(int device) {
    static std::mutex mu;
    static std::vector<int> done;
    std::lock_guard<std::mutex> lock(mu);
    if (std::find(done.begin(), done.end(), device) != done.end()) return;
    done.push_back(device);
    hipFuncAttributes at;
    auto touch = [&](const void *fn) {
        if (fn) (void)hipFuncGetAttributes(&at, fn);
    };
    for (const auto *tab : {&diag_table(), &diag2_table(), &chol_table()})
        if (!tab->empty()) touch(reinterpret_cast<const void *>(tab->front().fn));
    if (!mwg_table().empty()) touch(reinterpret_cast<const void *>(mwg_table().front().full_perobs));
    if (!block_table().empty()) touch(reinterpret_cast<const void *>(block_table().front().fn));
    for (const auto *tab : {&mix_table(), &mixchol_table()})
        if (!tab->empty()) touch(reinterpret_cast<const void *>(tab->front().fn));
    if (!mixres_table().empty()) touch(reinterpret_cast<const void *>(mixres_table().front().fn));
    touch(reinterpret_cast<const void *>(mala_lookup(32, true, 0)));
    touch(reinterpret_cast<const void *>(&gather_hist_kernel));
}

// mwg_block_kernel's shapes: one MALA or user update (kinds 4, 5) over coords 1:D in order,
// ImproperPrior, no chain moments / mixture state, 17 ≤ D ≤ 64, the built-in GsnTargetLaw
// over μ (d = D) or a user law
bool block_eligible(const emcmc_handle *h, bool xt) {
    const int D = (int)h->cfg.dim;
    if (xt || (h->cfg.kernel_variant & EMCMC_VARIANT_NO_BLOCK) || h->updates.size() != 1 || D < kBlockMinD || D > kMwgMaxD) return false;
    const UpdateHost &u = h->updates[0];
    if ((u.kernel != EMCMC_MALA && u.kernel != EMCMC_USER_UPDATE) || u.prior != EMCMC_PRIOR_IMPROPER ||
        u.adaptation != EMCMC_ADPT_NONE || u.coords.size() != (size_t)D)
        return false;
    for (int j = 0; j < D; ++j)
        if (u.coords[j] != (uint32_t)j) return false;
    const TargetHost &t = h->target;
    return t.kind == EMCMC_TARGET_USER || (t.kind == EMCMC_TARGET_GSN && (int)t.dim == D);
}

// BlockConsts (emcmc_block.h): L_t forward table (packed column-major, 1/L_jj on the
// diagonal) | backward table (rows D−1 … 0: 1/L_jj, L_j0 … L_j,j−1) | x̄ | 1/L_ii | observations
emcmc_status upload_block_consts(emcmc_handle *h) {
    const TargetHost &t = h->target;
    const int D = (int)h->cfg.dim;
    const size_t P = (size_t)D * (D + 1) / 2;
    std::vector<double> c(2 * P + 2 * (size_t)D + t.nobs * (size_t)D, 0.0);
    for (int j = 0; j < D; ++j)
        for (int i = j; i < D; ++i)
            c[(size_t)chol_col(D, j) + (size_t)(i - j)] = (i == j) ? t.invdiag[j] : t.L[(size_t)i * D + j];
    for (int tt = 0; tt < D; ++tt) {
        const int j = D - 1 - tt;
        double *r = c.data() + P + (size_t)chol_col(D, tt);
        r[0] = t.invdiag[j];
        for (int i = 0; i < j; ++i) r[1 + i] = t.L[(size_t)j * D + i];
    }
    std::copy(t.xbar.begin(), t.xbar.end(), c.begin() + 2 * P);
    std::copy(t.invdiag.begin(), t.invdiag.end(), c.begin() + 2 * P + D);
    std::copy(t.obs.begin(), t.obs.end(), c.begin() + 2 * P + 2 * D);
    if (h->d_bconsts) (void)hipFree(h->d_bconsts);
    h->d_bconsts = nullptr;
    HIPCHK(h, hipMalloc(&h->d_bconsts, c.size() * sizeof(double)));
    HIPCHK(h, hipMemcpy(h->d_bconsts, c.data(), c.size() * sizeof(double), hipMemcpyHostToDevice));
    return EMCMC_OK;
}

// mwg_rw_block_kernel's schedules (emcmc_rwblock.h): 1 ≤ P ≤ 8 UniformRandomWalk /
// GaussianRandomWalk updates over any coordinate subsets at 17 ≤ D ≤ 64, any prior, positivity
// flags, AdaptationUnifRW on a UniformRandomWalk; no chain moments / mixture state, no MALA or user
// updates; the built-in GsnTargetLaw over μ (d = D) or a user law.  (A single GaussianRandomWalk
// over coords 1:D with ImproperPrior and no flags on the built-in target never reaches select_mwg:
// the fused kernels take it.)
// A GaussianRandomWalk's positivity round trips keep up to six vectors of its coordinates live
// (emcmc_rwblock.h): with more than 32 flagged coordinates the kernel always needs scratch (33, 40,
// 48 measured) — the scratch gate would discard it — and at 64 the gfx950 backend aborts the process
// compiling it (LLVM ERROR: Unsupported instruction).  Such updates go to the wide kernel uncompiled.
constexpr int kRwBlockMaxGaussianPos = 32;
bool rwblock_update_ok(const UpdateHost &u) {
    if (u.kernel != EMCMC_RW_UNIFORM && u.kernel != EMCMC_RW_GAUSSIAN) return false;
    if (u.kernel == EMCMC_RW_GAUSSIAN) {
        int npos = 0;
        for (uint8_t f : u.pos) npos += f ? 1 : 0;
        if (npos > kRwBlockMaxGaussianPos) return false;
    }
    return u.adaptation == EMCMC_ADPT_NONE || (u.kernel == EMCMC_RW_UNIFORM && u.adaptation == EMCMC_ADPT_UNIF_RW);
}
bool rwblock_eligible(const std::vector<UpdateHost> &ups, uint32_t D) {
    if (D < (uint32_t)kBlockMinD || D > (uint32_t)kMwgMaxD || ups.empty() || ups.size() > (size_t)kRwMaxP)
        return false;
    for (const auto &u : ups)
        if (!rwblock_update_ok(u)) return false;
    return true;
}
bool rwblock_eligible(const emcmc_handle *h, bool xt) {
    if (xt || (h->cfg.kernel_variant & EMCMC_VARIANT_NO_BLOCK)) return false;
    const TargetHost &t = h->target;
    if (!(t.kind == EMCMC_TARGET_USER || (t.kind == EMCMC_TARGET_GSN && t.dim == h->cfg.dim))) return false;
    return rwblock_eligible(h->updates, h->cfg.dim);
}

// The compile-time schedule of eligible updates (emcmc_rwblock.h): per update its coordinates,
// kind, diagonal Σ, positivity mask, adaptation, the prior's slot structure and whether it shares
// no coordinate with another update; label: the kernel-name tag; sched_name: the generated
// struct's name (RwSched_<digest of the schedule>, so kernels of different schedules have
// different symbol names in a profile).
std::string rw_sched_source(const std::vector<UpdateHost> &ups, std::string &label, std::string &sched_name) {
    const size_t P = ups.size();
    char buf[64];
    std::string body;
    static const char *kPriorName[4] = {"ImproperPrior", "ImproperPosPrior", "ProductPrior", "StandardPrior"};
    label.clear();
    for (size_t p = 0; p < P; ++p) {
        const UpdateHost &u = ups[p];
        uint64_t pos = 0;
        for (size_t j = 0; j < u.pos.size(); ++j)
            if (u.pos[j]) pos |= 1ull << j;
        const bool uni = u.kernel == EMCMC_RW_UNIFORM;
        const bool adapt = uni && u.adaptation == EMCMC_ADPT_UNIF_RW;
        const bool slots = u.prior == EMCMC_PRIOR_PRODUCT || u.prior == EMCMC_PRIOR_STANDARD;
        bool disjoint = true;
        for (size_t q = 0; q < P && disjoint; ++q)
            if (q != p)
                for (uint32_t c : ups[q].coords)
                    if (std::find(u.coords.begin(), u.coords.end(), c) != u.coords.end()) disjoint = false;
        std::string b = "template <> struct RWSCHED::U<" + std::to_string(p) + "> {\n";
        b += "    static constexpr int n = " + std::to_string(u.coords.size()) + ";\n";
        b += "    static constexpr int coords[64] = {";
        for (size_t j = 0; j < 64; ++j) b += std::to_string(j < u.coords.size() ? u.coords[j] : 0u) + (j < 63 ? "," : "};\n");
        b += "    static constexpr uint32_t kind = " + std::to_string(u.kernel) + "u;\n";
        b += std::string("    static constexpr bool diag = ") + ((uni || u.diag) ? "true" : "false") + ";\n";
        snprintf(buf, sizeof buf, "0x%016llxull", (unsigned long long)pos);
        b += std::string("    static constexpr uint64_t pos = ") + buf + ";\n";
        b += std::string("    static constexpr bool adapt = ") + (adapt ? "true" : "false") + ";\n";
        b += std::string("    static constexpr bool disjoint = ") + (disjoint ? "true" : "false") + ";\n";
        b += "    static constexpr uint32_t prior = " + std::to_string(u.prior) + "u;\n";
        b += "    static constexpr int nslot = " + std::to_string(slots ? u.nslot : 0u) + ";\n";
        const uint64_t masks[4] = {u.psrc0, u.pstart, u.pend, u.pmvn};
        const char *mnames[4] = {"psrc0", "pstart", "pend", "pmvn"};
        for (int k = 0; k < 4; ++k) {
            snprintf(buf, sizeof buf, "0x%016llxull", (unsigned long long)(slots ? masks[k] : 0ull));
            b += std::string("    static constexpr uint64_t ") + mnames[k] + " = " + buf + ";\n";
        }
        std::string fam = "    static constexpr uint32_t fam[64] = {", mvs = "    static constexpr int mvs[64] = {";
        for (int j = 0; j < 64; ++j) {
            const bool in = slots && (uint32_t)j < u.nslot;
            fam += std::to_string(in ? u.pfam[j] : 0u) + (j < 63 ? "," : "};\n");
            mvs += std::to_string(in ? u.pmvs[j] : 0u) + (j < 63 ? "," : "};\n");
        }
        body += b + fam + mvs + "};\n";
        // kernel-name tag
        std::string l = std::string(uni ? "UniformRandomWalk" : "GaussianRandomWalk") + (uni || u.diag ? "" : "(dense)");
        bool ident = true;
        for (size_t j = 0; j < u.coords.size(); ++j) ident = ident && u.coords[j] == j;
        if (P > 1 || !ident) l += "[" + std::to_string(u.coords.size()) + "]";
        if (pos) {
            snprintf(buf, sizeof buf, ",pos=0x%llx", (unsigned long long)pos);
            l += buf;
        }
        if (adapt) l += ",AdaptationUnifRW";
        l += std::string(",") + (u.prior < 4 ? kPriorName[u.prior] : "?");
        if (slots && u.pmvn) l += "(MvNormal)";
        label += (p ? ";" : "") + l;
    }
    std::string src = "namespace emcmc {\nstruct RWSCHED {\n    static constexpr int P = " + std::to_string(P) +
                      ";\n    template <int p> struct U;\n};\n" + body + "}  // namespace emcmc\n";
    uint64_t hsh = 0xcbf29ce484222325ull;
    for (unsigned char ch : src) hsh = (hsh ^ ch) * 0x100000001b3ull;
    snprintf(buf, sizeof buf, "RwSched_%016llx", (unsigned long long)hsh);
    sched_name = buf;
    for (size_t at = src.find("RWSCHED"); at != std::string::npos; at = src.find("RWSCHED", at + 1))
        src.replace(at, 7, sched_name);
    if (P > 1) label = "P=" + std::to_string(P) + "," + label;
    return src;
}

emcmc_status select_mwg(emcmc_handle *h) {
    const int D = (int)h->cfg.dim;
    if (h->allocated) {
        // Re-selected after emcmc_set_state (a new target or variant): kernels still
        // queued on the non-blocking h->stream read the update table and the pool
        // replaced below. The pool restarts (L_B = user Σ_B, Haario M = 0, moments =
        // phantom zero sample), so the adaptation state restarts with it: N = 1 and
        // λ as constructed, as emcmc_set_state does.
        HIPCHK(h, hipStreamSynchronize(h->stream));
        h->stats_N = 1;
        for (auto &u : h->updates) u.lam = u.lam0;
    }
    const bool full = h->cfg.history_mode == EMCMC_HIST_FULL;
    const int ll = (int)h->target.ll_mode;
    Variant v;
    size_t nmax = 1;  // largest update: the wide kernel's local vector length
    for (const auto &u : h->updates) nmax = std::max(nmax, u.coords.size());
    int best_nu = 1 << 30;
    const bool user = h->target.kind == EMCMC_TARGET_USER;
    std::string usrc, uopts;  // a user update's source: compiled into the same kernel
    bool xt = h->cfg.chain_moments != 0;  // GaussianRandomWalkMix / Haario / chain moments: compiled at run time
    bool mala = false;                    // MALA updates: compiled at run time with the target's gradient
    for (const auto &u : h->updates) {
        if (u.kernel == EMCMC_USER_UPDATE) usrc = u.usrc, uopts = u.uopts;
        if (u.kernel == EMCMC_RW_GAUSSIAN_MIX) xt = true;
        if (u.kernel == EMCMC_MALA) mala = true;
    }
    if (mala && user && !rtc_defines_user_grad(h->target.src))
        return fail(h, EMCMC_UNSUPPORTED_PLUGIN,
                    "MALA needs the target's gradient (compute_gradients_and_momenta!): the user law defines none "
                    "(EMCMC_USER_GRAD { … })");
    // a schedule of 1 ≤ P ≤ 8 UniformRandomWalk / GaussianRandomWalk updates at 17 ≤ D ≤ 64 (priors,
    // positivity flags, AdaptationUnifRW, any coordinate subsets): mwg_rw_block_kernel
    // (emcmc_rwblock.h), the schedule's structure compiled in, every per-chain vector in registers
    if (usrc.empty() && !mala && rwblock_eligible(h, xt)) {
        const bool tdense = !h->target.diag;
        std::string label, sname;
        const std::string shape = rw_sched_source(h->updates, label, sname);
        RtcKernel k;
        const std::string log = rtc_compile_rwblock(D, full, user ? 0 : ll, tdense, shape, sname, label,
                                                    user ? h->target.src : "", user ? h->target.opts : "", k);
        if (!log.empty()) {
            h->err = std::string(user ? "user target does not compile:\n" : "run-time kernel build failed:\n") + log;
            return user ? EMCMC_INVALID_ARG : EMCMC_HIP_ERROR;
        }
        if (emcmc_status st = load_rtc_module(h, k)) return st;
        HIPCHK(h, hipModuleGetFunction(&v.ufn, h->umod, k.lowered.c_str()));
        // Register-resident or not at all: a schedule whose state does not fit the register
        // file (e.g. D = 64 with P°.θ, a dense 40-coordinate Σ and a dense target: 512 VGPRs,
        // 256 AGPRs, 3,322 SGPR spills, 660 B of scratch per lane) goes to the wide kernel.
        // That code object gave wrong bits on MI355X; every shape measured
        // and tested on this kernel needs no scratch.
        int scratch = 0;
        HIPCHK(h, hipFuncGetAttribute(&scratch, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, v.ufn));
        static const bool allow_scratch = [] {  // A/B builds only (EMCMC_RTC_EXTRA occupancy trials)
            const char *e = getenv("EMCMC_RW_ALLOW_SCRATCH");
            return e && *e && *e != '0';
        }();
        if (scratch == 0 || allow_scratch) {
            v.name = k.name;
            v.block = true;
            if (!user) {
                if (emcmc_status st = upload_block_consts(h)) return st;
            }
        } else {
            v.ufn = nullptr;
            h->rtc_origin = 0;
            h->rtc_seconds = 0.0;
        }
    }
    // one MALA or user update over all 17 ≤ D ≤ 64 coordinates: mwg_block_kernel (emcmc_block.h),
    // every per-chain vector in registers (the wide kernel's NU = D loops live in scratch)
    if (!v.block && block_eligible(h, xt)) {
        const bool tdense = !h->target.diag;
        if (!user && usrc.empty())
            for (const auto &e : block_table())
                if (e.D == D && e.tdense == (int)tdense && e.full == (int)full && e.ll == ll) v.mfn = e.fn;
        if (!v.mfn) {
            RtcKernel k;
            const std::string log = rtc_compile_block(D, full, user ? 0 : ll, tdense, user ? h->target.src : "",
                                                      user ? h->target.opts : "", usrc, uopts, k);
            if (!log.empty()) {
                h->err = std::string(user || !usrc.empty() ? "user target / update does not compile:\n"
                                                            : "run-time kernel build failed:\n") +
                         log;
                return (user || !usrc.empty()) ? EMCMC_INVALID_ARG : EMCMC_HIP_ERROR;
            }
            if (emcmc_status st = load_rtc_module(h, k)) return st;
            HIPCHK(h, hipModuleGetFunction(&v.ufn, h->umod, k.lowered.c_str()));
            v.name = k.name;
        } else {
            char bn[160];
            snprintf(bn, sizeof bn, "mwg_block_kernel<D=%d,%s,%s,%s,MALA>", D, full ? "FULL" : "ACCEPT_ONLY",
                     ll == LL_PER_OBS ? "PER_OBS" : "SUFFSTAT", tdense ? "DENSE_T" : "DIAG_T");
            v.name = bn;
        }
        v.block = true;
        if (!user) {
            if (emcmc_status st = upload_block_consts(h)) return st;
        }
    }
    for (const auto &e : mwg_table()) {
        if (user || !usrc.empty() || xt || mala || v.block) break;
        if (e.D != D) continue;
        if (e.nu != 0 && ((size_t)e.nu < nmax || e.nu >= best_nu)) continue;  // smallest NU that fits
        if (e.nu != 0) best_nu = e.nu;
        v.mfn = full ? (ll == LL_PER_OBS ? e.full_perobs : e.full_suff)
                     : (ll == LL_PER_OBS ? e.acc_perobs : e.acc_suff);
    }
    // a user law, or a dimension without an ahead-of-time instantiation: the
    // same kernel compiled at run time (emcmc_rtc.hip, cached per process)
    if (!v.block && (user || !usrc.empty() || xt || mala || (!v.mfn && D <= kMwgMaxD))) {
        RtcKernel k;
        const int nu = rtc_wide_nu(D, (int)nmax);
        const std::string log = user ? rtc_compile_user(h->target.src, h->target.opts, D, full, nu, k, usrc, uopts, xt,
                                                        mala)
                                     : rtc_compile_gsn(D, full, ll, nu, k, usrc, uopts, xt, mala);
        if (!log.empty()) {
            h->err = std::string(user || !usrc.empty() ? "user target / update does not compile:\n"
                                                        : "run-time kernel build failed:\n") +
                     log;
            return (user || !usrc.empty()) ? EMCMC_INVALID_ARG : EMCMC_HIP_ERROR;
        }
        if (emcmc_status st = load_rtc_module(h, k)) return st;
        HIPCHK(h, hipModuleGetFunction(&v.ufn, h->umod, k.lowered.c_str()));
        v.name = k.name;
        best_nu = 1 << 30;
    }
    if (!v.mfn && !v.ufn)
        return fail(h, EMCMC_UNSUPPORTED_PLUGIN,
                    "no general-schedule device kernel for D=%d (D ≤ 64)", D);
    (void)mwg_pool_layout(h);  // the mix / Haario offsets the table records
    std::vector<MwgUpdate> tab(h->updates.size());
    for (size_t p = 0; p < h->updates.size(); ++p) {
        const UpdateHost &u = h->updates[p];
        MwgUpdate &m = tab[p];
        std::memset(&m, 0, sizeof m);
        m.kind = u.kernel;
        m.nc = (uint32_t)u.coords.size();
        m.adapt = u.adaptation;
        for (uint32_t j = 0; j < m.nc; ++j) m.coords[j] = u.coords[j];
        if (u.kernel == EMCMC_RW_GAUSSIAN_MIX) {
            m.lam = u.lam;
            m.hk = (u.adaptation == EMCMC_ADPT_HAARIO) ? u.haario.adapt_every_k_steps : 0u;
            m.adapt = 0;  // Haario runs in mwg_post_step, not as AdaptationUnifRW
            m.lb_off = u.lb_off, m.lbi_off = u.lbi_off, m.lbc_off = u.lbc_off, m.lbs_off = u.lbs_off;
            m.hm_off = u.hm_off, m.hc_off = u.hc_off;
        }
        if (u.kernel == EMCMC_USER_UPDATE) {
            for (size_t q = 0; q < u.uparams.size(); ++q) m.L[q] = u.uparams[q];
        } else if (u.kernel == EMCMC_MALA) {  // ϵ, h and the diagonal factor ϵI of its densities
            m.eps0[0] = u.eps[0];
            m.eps0[1] = u.eps[1];
            for (uint32_t i = 0; i < m.nc; ++i) {
                m.L[i * kMwgMaxD + i] = u.L[(size_t)i * m.nc + i];
                m.iL[i] = u.invdiag[i];
            }
            m.c0 = u.c0;
            m.diag = 1u;
        } else if (u.kernel == EMCMC_RW_UNIFORM) {
            for (uint32_t j = 0; j < m.nc; ++j) m.eps0[j] = u.eps[j];
            for (uint32_t j = 0; j < m.nc; ++j) m.uc[j] = -log_any(2.0 * u.eps[j]);
            for (uint32_t j = 0; j < m.nc; ++j) m.posmask |= (u.pos.size() > j && u.pos[j]) ? (1ull << j) : 0ull;
            if (u.adaptation == EMCMC_ADPT_UNIF_RW) {
                m.k = u.adpt.adapt_every_k_steps;
                m.target = u.adpt.target_accpt_rate;
                for (uint32_t j = 0; j < m.nc; ++j) {
                    m.ascale[j] = u.ascale[j];
                    m.amin[j] = u.amin[j];
                    m.amax[j] = u.amax[j];
                    m.aoff[j] = u.aoff[j];
                }
            }
        } else {
            const int n = (int)m.nc;
            for (int i = 0; i < n; ++i)
                for (int j = 0; j <= i; ++j) m.L[i * kMwgMaxD + j] = u.L[(size_t)i * n + j];
            for (int i = 0; i < n; ++i) m.iL[i] = u.invdiag[i];
            m.c0 = u.c0;
            m.diag = u.diag ? 1u : 0u;
            for (uint32_t j = 0; j < m.nc; ++j) m.posmask |= (u.pos.size() > j && u.pos[j]) ? (1ull << j) : 0ull;
        }
        m.prior = u.prior;
        m.nslot = u.nslot;
        m.psrc0 = u.psrc0;
        m.pstart = u.pstart;
        m.pend = u.pend;
        m.pmvn = u.pmvn;
        for (uint32_t j = 0; j < u.nslot; ++j) {
            m.pfam[j] = u.pfam[j];
            m.pmvs[j] = u.pmvs[j];
            m.pa[j] = u.pa[j];
            m.pb[j] = u.pb[j];
            m.pc[j] = u.pc[j];
            m.pmu[j] = u.pmu[j];
            m.piL[j] = u.piL[j];
        }
        if (u.pmvn)
            for (uint32_t j = 0; j < u.nslot; ++j)
                for (uint32_t q = 0; q <= j; ++q) m.pL[j * kMwgMaxD + q] = u.pL[(size_t)j * kMwgMaxD + q];
    }
    if (h->d_mwg) (void)hipFree(h->d_mwg);
    HIPCHK(h, hipMalloc(&h->d_mwg, tab.size() * sizeof(MwgUpdate)));
    HIPCHK(h, hipMemcpy(h->d_mwg, tab.data(), tab.size() * sizeof(MwgUpdate), hipMemcpyHostToDevice));
    const TargetHost &t = h->target;
    auto upload = [&](double *&dst, const std::vector<double> &src) -> emcmc_status {
        if (dst) (void)hipFree(dst);
        dst = nullptr;
        HIPCHK(h, hipMalloc(&dst, std::max<size_t>(1, src.size()) * sizeof(double)));
        if (!src.empty()) HIPCHK(h, hipMemcpy(dst, src.data(), src.size() * sizeof(double), hipMemcpyHostToDevice));
        return EMCMC_OK;
    };
    emcmc_status st;
    if ((st = upload(h->d_tL, t.L)) || (st = upload(h->d_tiL, t.invdiag)) || (st = upload(h->d_xbar, t.xbar)) ||
        (st = upload(h->d_obs, t.obs)) || (st = upload(h->d_uparams, t.params)))
        return st;
    char nm[160];
    if (v.ufn || v.block)
        snprintf(nm, sizeof nm, "%s", v.name.c_str());
    else if (best_nu < (1 << 30))
        snprintf(nm, sizeof nm, "mwg_wide_kernel<D=%d,NU=%d,P=%zu,%s,%s>", D, best_nu, h->updates.size(),
                 full ? "FULL" : "ACCEPT_ONLY", ll == LL_PER_OBS ? "PER_OBS" : "SUFFSTAT");
    else
        snprintf(nm, sizeof nm, "mwg_gsn_kernel<D=%d,P=%zu,%s,%s>", D, h->updates.size(),
                 full ? "FULL" : "ACCEPT_ONLY", ll == LL_PER_OBS ? "PER_OBS" : "SUFFSTAT");
    v.name = nm;
    h->lds_bytes = 0;  // tables only, in static LDS
    h->var = v;
    if (h->allocated) return reset_mwg_pool(h);
    return EMCMC_OK;
}

bool fused_eligible(const emcmc_handle *h) {
    if (!joint_all_coords(h) || h->cfg.chain_moments) return false;
    const UpdateHost &u = h->updates[0];
    if (u.prior != EMCMC_PRIOR_IMPROPER) return false;  // priors and proposal! resampling: general kernel
    for (uint8_t f : u.pos)
        if (f) return false;  // positivity-restricted coordinates: general schedule kernel (D ≤ 64)
    return u.kernel == EMCMC_RW_GAUSSIAN && u.adaptation == EMCMC_ADPT_NONE;
}

// The fused diagonal step with the update's separable terms compiled in (emcmc_fprior.h
// FusedUpdate): ONE update over coords 0..D−1 in order on a diagonal GsnTargetLaw —
// GaussianRandomWalk with a diagonal Σ or UniformRandomWalk (positivity flags allowed on either),
// no adaptation — whose prior is ImproperPrior (with flags, or UniformRandomWalk; the flag-less
// Gaussian one is the plain fused kernel), ImproperPosPrior, or ONE ProductPrior / StandardPrior factor that
// is a Product of D univariates (no "reads θ[1]" dims-1 factor) or one MvNormal over all D; the families and positivity flags repeat across the chain's lanes (those of
// coordinate i = those of i mod D/LPC).
bool fused_prior_mvn(const UpdateHost &u) {
    return (u.prior == EMCMC_PRIOR_PRODUCT || u.prior == EMCMC_PRIOR_STANDARD) && u.pmvn != 0ull;
}
int fused_lpc(const emcmc_handle *h) {
    return h->cfg.lanes_per_chain ? (int)h->cfg.lanes_per_chain : auto_lpc((int)h->cfg.dim);
}
bool fused_prior_eligible(const emcmc_handle *h) {
    if ((h->cfg.kernel_variant & EMCMC_VARIANT_NO_FUSED_PRIOR) || !joint_all_coords(h) || h->cfg.chain_moments)
        return false;
    const UpdateHost &u = h->updates[0];
    const int D = (int)h->cfg.dim;
    const bool uni = u.kernel == EMCMC_RW_UNIFORM;
    if ((u.kernel != EMCMC_RW_GAUSSIAN && !uni) || u.adaptation != EMCMC_ADPT_NONE || !h->target.diag ||
        h->target.kind != EMCMC_TARGET_GSN || D > 64 || (!uni && !u.diag))
        return false;
    bool anypos = false;
    for (uint8_t f : u.pos) anypos = anypos || f;
    const bool slots = u.prior == EMCMC_PRIOR_PRODUCT || u.prior == EMCMC_PRIOR_STANDARD;
    // ImproperPrior without flags on a GaussianRandomWalk: the plain (ahead-of-time) fused kernel
    if (u.prior == EMCMC_PRIOR_IMPROPER ? (!uni && !anypos) : (!slots && u.prior != EMCMC_PRIOR_IMPROPER_POS))
        return false;
    if (slots && (u.nslot != (uint32_t)D || u.psrc0 || u.pstart != 1ull || u.pend != (1ull << (D - 1))))
        return false;
    const bool mvn = fused_prior_mvn(u);  // then every slot is a row of it (one factor: pmvs = 0)
    if (mvn && u.pmvn != (D == 64 ? ~0ull : (1ull << D) - 1ull)) return false;
    const int lpc = fused_lpc(h);
    if ((lpc != 1 && lpc != 2 && lpc != 4) || D % lpc) return false;
    const int dpl = D / lpc;
    // the likelihood's canonical sum (SumShape: blocks of 8, a pairwise tree over the blocks) splits
    // across the lanes only where each lane's blocks form one subtree: D/LPC = 8·2^k
    if (lpc > 1 && (dpl % 8 || ((dpl / 8) & (dpl / 8 - 1)))) return false;
    for (int i = 0; i < D; ++i) {
        if (slots && !mvn && u.pfam[i] != u.pfam[i % dpl]) return false;
        const bool pi = i < (int)u.pos.size() && u.pos[i], pj = (i % dpl) < (int)u.pos.size() && u.pos[i % dpl];
        if (pi != pj) return false;
    }
    return true;
}

// EMCMC_UNSUPPORTED_PLUGIN when the shape does not fit (its LDS or a code object that needs
// scratch): the caller falls back to the schedule kernels.
emcmc_status select_fused_prior(emcmc_handle *h) {
    const UpdateHost &u = h->updates[0];
    const TargetHost &t = h->target;
    const int D = (int)h->cfg.dim;
    const bool full = h->cfg.history_mode == EMCMC_HIST_FULL;
    const int ll = (int)t.ll_mode;
    const int lpc = fused_lpc(h);
    bool unit = true;
    for (int i = 0; i < D; ++i) unit = unit && t.invdiag[i] == 1.0;
    const bool uni = u.kernel == EMCMC_RW_UNIFORM;
    const bool slots = u.prior == EMCMC_PRIOR_PRODUCT || u.prior == EMCMC_PRIOR_STANDARD;
    const bool mvn = fused_prior_mvn(u);
    // staged in LDS; FusedUpdate::kConsts = 3 with univariate slots
    const size_t nconst = (slots && !mvn ? 7 : 4) * (size_t)D;
    const size_t obs_doubles = (ll == LL_PER_OBS) ? t.nobs * (size_t)D : 0;
    const size_t lds = lds_align16((nconst + obs_doubles) * sizeof(double));
    if (kZigLdsBytes + lds > kMaxLds) return EMCMC_UNSUPPORTED_PLUGIN;  // the schedule kernel reads them from HBM
    std::string label, sname;
    const std::string shape = rw_sched_source(h->updates, label, sname);
    // two waves per SIMD (512-thread blocks, sibling pacing) where the step fits 256 registers, else
    // one; register-resident or not at all (as mwg_rw_block_kernel, select_mwg)
    Variant v;
    int minw = 0;
    for (int w : {2, 1}) {
        RtcKernel k;
        const std::string log = rtc_compile_fused_prior(D, lpc, w, full, ll, unit, shape, sname,
                                                        uni ? label : label.substr(label.find(',') + 1), k);
        if (!log.empty()) return fail(h, EMCMC_HIP_ERROR, "run-time kernel build failed:\n%s", log.c_str());
        if (emcmc_status st = load_rtc_module(h, k)) return st;
        HIPCHK(h, hipModuleGetFunction(&v.ffn, h->umod, k.lowered.c_str()));
        int scratch = 0;
        HIPCHK(h, hipFuncGetAttribute(&scratch, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, v.ffn));
        if (scratch == 0) {
            minw = w;
            v.name = k.name;
            break;
        }
    }
    if (!minw) {
        h->rtc_origin = 0;
        h->rtc_seconds = 0.0;
        return EMCMC_UNSUPPORTED_PLUGIN;
    }
    v.lpc = lpc;
    v.dense = 0;
    v.occ = minw;
    v.unit = unit;
    // the diag kernel's constants (L_ii, 1/L_ii — UniformRandomWalk: ϵ_i, −log 2ϵ_i with the device's
    // log — 1/L_t,ii, x̄), then the prior's a, b, c per coordinate, or — an MvNormal factor, read
    // from global memory — μ, 1/L_jj, L packed lower row-major, c0 (FusedUpdate::eval_mvn)
    const size_t nmvn = mvn ? 2 * (size_t)D + (size_t)D * (D + 1) / 2 + 1 : 0;
    std::vector<double> c(nconst + nmvn);
    if (mvn) {
        double *g = c.data() + nconst;
        for (int j = 0, q = 2 * D; j < D; ++j) {
            g[j] = u.pmu[j];
            g[D + j] = u.piL[j];
            for (int m = 0; m <= j; ++m) g[q++] = u.pL[(size_t)j * kMwgMaxD + m];
        }
        g[nmvn - 1] = u.pc[D - 1];
    }
    for (int i = 0; i < D; ++i) {
        c[i] = uni ? u.eps[i] : u.L[(size_t)i * D + i];
        c[D + i] = uni ? -log_any(2.0 * u.eps[i]) : u.invdiag[i];
        c[2 * D + i] = t.invdiag[i];
        c[3 * D + i] = t.xbar[i];
        if (slots && !mvn) {
            c[4 * D + i] = u.pa[i];
            c[5 * D + i] = u.pb[i];
            c[6 * D + i] = u.pc[i];
        }
    }
    if (h->d_consts) (void)hipFree(h->d_consts);
    HIPCHK(h, hipMalloc(&h->d_consts, c.size() * sizeof(double)));
    HIPCHK(h, hipMemcpy(h->d_consts, c.data(), c.size() * sizeof(double), hipMemcpyHostToDevice));
    if (h->d_obs) (void)hipFree(h->d_obs);
    h->d_obs = nullptr;
    if (t.nobs) {
        HIPCHK(h, hipMalloc(&h->d_obs, t.obs.size() * sizeof(double)));
        HIPCHK(h, hipMemcpy(h->d_obs, t.obs.data(), t.obs.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    h->lds_bytes = lds;
    h->var = v;
    return EMCMC_OK;
}

// chains per 256-thread block of mix_readjust_kernel<D> (R lanes per chain)
int readjust_chains_per_block(int D) {
    int r = 1;
    while (r < D) r <<= 1;
    return 4 * (64 / r);
}
emcmc_status select_mix(emcmc_handle *h) {
    const int D = (int)h->cfg.dim;
    const UpdateHost &u = h->updates[0];
    const bool full = h->cfg.history_mode == EMCMC_HIST_FULL;
    const int ll = (int)h->target.ll_mode;
    const bool mix = u.kernel == EMCMC_RW_GAUSSIAN_MIX;
    const bool adiag = (u.diag && h->target.diag) || D == 1;
    // the mix / chain-moments kernels have no prior term and no proposal! redraw
    // loop: a prior or positivity flags there would be dropped silently
    if (u.prior != EMCMC_PRIOR_IMPROPER)
        return fail(h, EMCMC_UNSUPPORTED_PLUGIN,
                    "chain moments / GaussianRandomWalkMix run on device with ImproperPrior only");
    for (uint8_t f : u.pos)
        if (f)
            return fail(h, EMCMC_UNSUPPORTED_PLUGIN,
                        "chain moments / GaussianRandomWalkMix: positivity-restricted coordinates have no device "
                        "plugin on the mix kernels");
    Variant v;
    for (const auto &e : mix_table())
        if (e.D == D && e.full == (int)full && e.ll == ll && e.mix == (int)mix && e.adiag == (int)adiag) v.xfn = e.fn;
    // a dense Σ_A or Σ_t at D ≥ 16: the factors through the scalar cache
    if (!v.xfn && !adiag && !(h->cfg.kernel_variant & EMCMC_VARIANT_NO_MIX_CHOL))
        for (const auto &e : mixchol_table())
            if (e.D == D && e.full == (int)full && e.ll == ll && e.mix == (int)mix) {
                v.xfn = e.fn;
                v.xchol = true;
            }
    if (!v.xfn)
        return fail(h, EMCMC_UNSUPPORTED_PLUGIN,
                    "no mix/chain-moments kernel for D=%d with %s Σ_A/Σ_t (instantiated: D ∈ {1,2,3,4,8} any, "
                    "D ∈ {16,32} diagonal Σ_A and Σ_t)",
                    D, adiag ? "diagonal" : "dense");
    if (u.adaptation == EMCMC_ADPT_HAARIO) {
        v.rfn = readjust_lookup(D);
        if (!v.rfn) return fail(h, EMCMC_UNSUPPORTED_PLUGIN, "no Haario readjust kernel for D=%d", D);
    }
    std::tie(v.mofn, v.mo_tiles) = moments_lookup(D);
    if (!v.mofn) return fail(h, EMCMC_UNSUPPORTED_PLUGIN, "no chain-moments kernel for D=%d", D);
    v.mix = true;
    const TargetHost &t = h->target;
    // L_B resident in registers across the launch (mix_res_kernel) where instantiated
    bool unit = true;
    for (int i = 0; i < D; ++i) unit = unit && t.invdiag[i] == 1.0;
    if (mix && adiag && h->cfg.num_chains % kMixResChainsPerBlock == 0 &&
        !(h->cfg.kernel_variant & EMCMC_VARIANT_MIX_STREAM)) {
        for (const auto &e : mixres_table())
            if (e.D == D && e.full == (int)full && e.ll == ll && e.unit == (int)unit) {
                v.xfn = e.fn;
                v.xres = true;
            }
    }
    char nm[160];
    snprintf(nm, sizeof nm, "%s<D=%d,%s,%s,%s,%s%s>+mix_moments_kernel%s",
             v.xres ? "mix_res_kernel" : v.xchol ? "mix_chol_kernel" : "mix_gsn_kernel",
             D, full ? "FULL" : "ACCEPT_ONLY", ll == LL_PER_OBS ? "PER_OBS" : "SUFFSTAT", mix ? "MIX" : "GSN_MOMENTS",
             adiag ? "DIAG" : "DENSE", v.xres && unit ? ",UNIT_T" : "", v.rfn ? "+mix_readjust_kernel" : "");
    v.name = nm;
    const size_t DD = (size_t)D * D;
    std::vector<double> c;
    if (v.xchol) {
        // emcmc_mix.h mix_chol_kernel: L_A rows (packed lower, row-major, with L_ii) | L_A and
        // L_t packed column-major with 1/L_jj on the diagonal | x̄ | observations (row-major)
        const size_t P = (size_t)D * (D + 1) / 2;
        c.assign(3 * P + D + (ll == LL_PER_OBS ? t.nobs * (size_t)D : 0), 0.0);
        for (int i = 0; i < D; ++i)
            for (int j = 0; j <= i; ++j) c[(size_t)lo_idx(i, j)] = u.L[(size_t)i * D + j];
        for (int j = 0; j < D; ++j)
            for (int i = j; i < D; ++i) {
                const size_t e = (size_t)chol_col(D, j) + (size_t)(i - j);
                c[P + e] = (i == j) ? u.invdiag[j] : u.L[(size_t)i * D + j];
                c[2 * P + e] = (i == j) ? t.invdiag[j] : t.L[(size_t)i * D + j];
            }
        std::copy(t.xbar.begin(), t.xbar.end(), c.begin() + 3 * P);
        if (ll == LL_PER_OBS) std::copy(t.obs.begin(), t.obs.end(), c.begin() + 3 * P + D);
    } else {
        c.resize(2 * DD + 3 * (size_t)D);
        std::copy(u.L.begin(), u.L.end(), c.begin());
        std::copy(u.invdiag.begin(), u.invdiag.end(), c.begin() + DD);
        std::copy(t.L.begin(), t.L.end(), c.begin() + DD + D);
        std::copy(t.invdiag.begin(), t.invdiag.end(), c.begin() + 2 * DD + D);
        std::copy(t.xbar.begin(), t.xbar.end(), c.begin() + 2 * DD + 2 * D);
    }
    const size_t obs_doubles = (ll == LL_PER_OBS) ? t.nobs * (size_t)D : 0;
    const size_t lds = v.xres    ? mixres_lds(D, t.nobs, h->cfg.steps_per_launch, ll == LL_PER_OBS)
                       : v.xchol ? 0  // the ziggurat only, in static LDS
                                 : (c.size() + obs_doubles) * sizeof(double);  // + kZigLdsBytes of static LDS
    if (kZigLdsBytes + lds > kMaxLds)
        return fail(h, EMCMC_INVALID_ARG,
                    "per-observation likelihood needs %zu B of LDS (> %zu); use EMCMC_LL_SUFFSTAT for n=%llu", lds,
                    kMaxLds, (unsigned long long)t.nobs);
    if (h->d_consts) (void)hipFree(h->d_consts);
    HIPCHK(h, hipMalloc(&h->d_consts, c.size() * sizeof(double)));
    HIPCHK(h, hipMemcpy(h->d_consts, c.data(), c.size() * sizeof(double), hipMemcpyHostToDevice));
    if (h->d_obs) (void)hipFree(h->d_obs);
    h->d_obs = nullptr;
    HIPCHK(h, hipMalloc(&h->d_obs, t.obs.size() * sizeof(double)));
    HIPCHK(h, hipMemcpy(h->d_obs, t.obs.data(), t.obs.size() * sizeof(double), hipMemcpyHostToDevice));
    h->lds_bytes = lds;
    if (emcmc_status st2 = allow_lds(h, reinterpret_cast<const void *>(v.xfn), lds)) return st2;
    h->var = v;
    return EMCMC_OK;
}

// ---- MALA kernel table ---------------------------------------------------------
emcmc_status select_mala(emcmc_handle *h) {
    const int D = (int)h->cfg.dim;
    if (!joint_all_coords(h))
        return fail(h, EMCMC_UNSUPPORTED_PLUGIN, "MALA runs on device as the single joint update on coords 1:D");
    if (h->target.kind != EMCMC_TARGET_LOGISTIC)
        return fail(h, EMCMC_UNSUPPORTED_PLUGIN, "MALA on device needs the logistic-regression target");
    if (h->updates[0].prior != EMCMC_PRIOR_IMPROPER)
        return fail(h, EMCMC_UNSUPPORTED_PLUGIN,
                    "MALA on the logistic-regression kernel runs with ImproperPrior only (priors: a user law with "
                    "EMCMC_USER_GRAD on the general kernel)");
    const bool full = h->cfg.history_mode == EMCMC_HIST_FULL;
    Variant v;
    v.afn = mala_lookup(D, full, 0);
    v.ainit = mala_lookup(D, true, 1);
    if (!v.afn || !v.ainit)
        return fail(h, EMCMC_UNSUPPORTED_PLUGIN, "no MALA kernel for D=%d (instantiated: D ∈ {16,32,48,64})", D);
    char nm[160];
    snprintf(nm, sizeof nm, "mala_logistic_kernel<D=%d,%s>", D, full ? "FULL" : "ACCEPT_ONLY");
    v.name = nm;
    // X padded to whole 64-row tiles with zero rows (their ℓ terms are masked)
    const TargetHost &t = h->target;
    const uint64_t tiles = (t.nobs + kMalaTileRows - 1) / kMalaTileRows;
    std::vector<double> X(tiles * kMalaTileRows * (size_t)D, 0.0), y(tiles * kMalaTileRows, 0.0);
    std::copy(t.obs.begin(), t.obs.end(), X.begin());
    std::copy(t.labels.begin(), t.labels.end(), y.begin());
    if (h->d_X) (void)hipFree(h->d_X);
    if (h->d_y) (void)hipFree(h->d_y);
    h->d_X = h->d_y = nullptr;
    HIPCHK(h, hipMalloc(&h->d_X, X.size() * sizeof(double)));
    HIPCHK(h, hipMalloc(&h->d_y, y.size() * sizeof(double)));
    HIPCHK(h, hipMemcpy(h->d_X, X.data(), X.size() * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(h, hipMemcpy(h->d_y, y.data(), y.size() * sizeof(double), hipMemcpyHostToDevice));
    h->mala_tiles = (uint32_t)tiles;
    h->grad_valid = false;
    h->lds_bytes = 0;
    h->var = v;
    return EMCMC_OK;
}

emcmc_status select_variant(emcmc_handle *h) {
    if (!h->target_set || h->updates.empty()) return EMCMC_OK;
    // MALA: the fused MFMA kernel on the logistic-regression target (cfg 3); on any
    // other target the general kernel with the target's gradient (the built-in
    // GsnTargetLaw's or a user law's EMCMC_USER_GRAD)
    for (const auto &u : h->updates)
        if (u.kernel == EMCMC_MALA && h->target.kind == EMCMC_TARGET_LOGISTIC) return select_mala(h);
    if (h->target.kind == EMCMC_TARGET_LOGISTIC)
        return fail(h, EMCMC_UNSUPPORTED_PLUGIN, "the logistic-regression target runs on device with MALA only");
    if (h->target.kind == EMCMC_TARGET_USER) return select_mwg(h);  // mix, Haario, chain moments included
    if (mix_path(h)) {
        // the fused mix kernels where instantiated (cfg 4 shapes), else the general kernel
        const std::string keep = h->err;
        const emcmc_status st = select_mix(h);
        if (st != EMCMC_UNSUPPORTED_PLUGIN) return st;
        h->err = keep;
        return select_mwg(h);
    }
    for (const auto &u : h->updates)
        if (u.kernel == EMCMC_RW_GAUSSIAN_MIX) return select_mwg(h);
    if (h->cfg.chain_moments) return select_mwg(h);
    if (fused_prior_eligible(h)) {
        const std::string keep = h->err;
        const emcmc_status st = select_fused_prior(h);
        if (st != EMCMC_UNSUPPORTED_PLUGIN) return st;
        h->err = keep;
        return select_mwg(h);
    }
    if (!fused_eligible(h)) return select_mwg(h);
    const UpdateHost &u = h->updates[0];
    const int D = (int)h->cfg.dim;
    const bool full = h->cfg.history_mode == EMCMC_HIST_FULL;
    const int ll = (int)h->target.ll_mode;
    // a correlated Σ (proposal or target) beyond the fused dense kernel's D ≤ 8:
    // rwm_gsn_chol_kernel (factors through the scalar cache) where instantiated,
    // else the general kernel (forward substitutions from the factors, D ≤ 64)
    // (the chol kernel compiled at run time for other D ≤ kCholRtcMaxD = 64:
    // registers hold θ, θ° and one substitution vector, 6·D VGPRs)
    // The kernel's scalar-load stream is unrolled at compile time in chunks of the largest of
    // 16/8/4/2/1 doubles dividing D; above kCholRtcMaxChunks chunks per observation sweep (odd
    // D > 25, D ≡ 2 mod 4 above 38) the compile takes minutes, and the general kernel runs instead.
    const bool chol_rtc = !(u.diag && h->target.diag) && D > 8 && !lookup(D, 1, full, ll, 2, false);
    if (chol_rtc && (D > kCholRtcMaxD || chol_rtc_chunks(D) > kCholRtcMaxChunks ||
                     (h->cfg.kernel_variant & EMCMC_VARIANT_NO_RTC_CHOL)))
        return select_mwg(h);
    const bool diag = u.diag && h->target.diag;
    Variant v;
    if (diag) {
        int lpc = h->cfg.lanes_per_chain ? (int)h->cfg.lanes_per_chain : auto_lpc(D);
        bool unit = true;
        for (int i = 0; i < D; ++i) unit = unit && h->target.invdiag[i] == 1.0;
        v.unit = unit;
        // default: the 2-waves-per-SIMD register cap where instantiated (inst_diag2.hip)
        const int occ = (h->cfg.kernel_variant & EMCMC_VARIANT_UNCAPPED) ? 0 : 2;
        v.fn = lookup(D, lpc, full, ll, false, unit, occ);
        v.occ = occ;
        if (!v.fn && occ) {
            v.fn = lookup(D, lpc, full, ll, false, unit, 0);
            v.occ = 0;
        }
        if (!v.fn && !h->cfg.lanes_per_chain) {
            lpc = 1;
            v.fn = lookup(D, 1, full, ll, false, unit);
        }
        v.lpc = lpc;
        v.dense = 0;
        // one lane per chain with the observations through the scalar cache
        if ((h->cfg.kernel_variant & EMCMC_VARIANT_SCALAR_OBS) && (!h->cfg.lanes_per_chain || lpc == 1))
            if (KernelFn f = lookup(D, 1, full, ll, 3, unit)) {
                v.fn = f;
                v.lpc = 1;
                v.dense = 3;
                v.occ = 0;
            }
    } else {
        v.dense = D > 8 ? 2 : 1;
        v.fn = lookup(D, 1, full, ll, v.dense, false);
        v.lpc = 1;
        if (!v.fn && chol_rtc) {
            RtcKernel k;
            const std::string log = rtc_compile_chol(D, full, ll, k);
            if (!log.empty()) return fail(h, EMCMC_HIP_ERROR, "run-time kernel build failed:\n%s", log.c_str());
            if (emcmc_status st = load_rtc_module(h, k)) return st;
            HIPCHK(h, hipModuleGetFunction(&v.ffn, h->umod, k.lowered.c_str()));
        }
    }
    if (!v.fn && !v.ffn)
        return fail(h, EMCMC_UNSUPPORTED_PLUGIN,
                    "no device kernel for D=%d (%s, lanes_per_chain=%u); instantiated: diag D∈{1,2,3,4,8,16,32,64}, "
                    "dense D∈{1,2,3,4,8,16,24,32}",
                    D, diag ? "diagonal" : "dense", h->cfg.lanes_per_chain);
    char nm[160];
    snprintf(nm, sizeof nm, "rwm_gsn_%s_kernel<D=%d,LPC=%d,%s,%s%s%s>%s",
             v.dense == 3 ? "diag_s" : v.dense == 2 ? "chol" : v.dense ? "dense" : "diag", D, v.lpc,
             full ? "FULL" : "ACCEPT_ONLY", ll == LL_PER_OBS ? "PER_OBS" : "SUFFSTAT", v.unit ? ",UNIT_T" : "",
             v.occ == 2 ? ",MINW=2" : "", v.ffn ? "[hiprtc]" : "");
    v.name = nm;
    // constants for this variant
    std::vector<double> c;
    const TargetHost &t = h->target;
    if (v.dense == 0 || v.dense == 3) {
        c.resize(4 * (size_t)D);
        for (int i = 0; i < D; ++i) {
            c[i] = u.L[(size_t)i * D + i];
            c[D + i] = u.invdiag[i];
            c[2 * D + i] = t.invdiag[i];
            c[3 * D + i] = t.xbar[i];
        }
    } else if (v.dense == 2) {
        // packed column-major lower factors (emcmc_kernels.h, rwm_gsn_chol_kernel):
        // L_rw with its diagonal, L_rw and L_t with 1/L_jj in place of L_jj, x̄, the
        // observations row-major
        const size_t P = (size_t)D * (D + 1) / 2;
        c.resize(3 * P + (size_t)D + (ll == LL_PER_OBS ? t.nobs * (size_t)D : 0));
        for (int j = 0; j < D; ++j)
            for (int i = j; i < D; ++i) {
                const size_t e = (size_t)chol_col(D, j) + (size_t)(i - j);
                c[e] = u.L[(size_t)i * D + j];
                c[P + e] = (i == j) ? u.invdiag[j] : u.L[(size_t)i * D + j];
                c[2 * P + e] = (i == j) ? t.invdiag[j] : t.L[(size_t)i * D + j];
            }
        std::copy(t.xbar.begin(), t.xbar.end(), c.begin() + 3 * P);
        if (ll == LL_PER_OBS) std::copy(t.obs.begin(), t.obs.end(), c.begin() + 3 * P + D);
    } else {
        const size_t DD = (size_t)D * D;
        c.resize(2 * DD + 3 * (size_t)D);
        std::copy(u.L.begin(), u.L.end(), c.begin());
        std::copy(u.invdiag.begin(), u.invdiag.end(), c.begin() + DD);
        std::copy(t.L.begin(), t.L.end(), c.begin() + DD + D);
        std::copy(t.invdiag.begin(), t.invdiag.end(), c.begin() + 2 * DD + D);
        std::copy(t.xbar.begin(), t.xbar.end(), c.begin() + 2 * DD + 2 * D);
    }
    // (the chol kernel reads its constants, the diag_s kernel its observations,
    // through the scalar cache)
    const size_t obs_doubles = (ll == LL_PER_OBS && v.dense < 2) ? t.nobs * (size_t)D : 0;
    size_t lds = v.dense == 2 ? 0 : (c.size() + obs_doubles) * sizeof(double);  // + kZigLdsBytes of static LDS
    if (!v.dense) lds = lds_align16(lds);
    if (kZigLdsBytes + lds > kMaxLds) {
        // more observations than the LDS holds (≈ 350 at D = 32): stream them
        // through the scalar cache (rwm_gsn_diag_s_kernel, any n) where
        // instantiated, else the general kernel (observations from global memory)
        KernelFn f = (v.dense == 0 && ll == LL_PER_OBS) ? lookup(D, 1, full, ll, 3, v.unit) : nullptr;
        if (!f) return select_mwg(h);
        v.fn = f;
        v.lpc = 1;
        v.dense = 3;
        v.occ = 0;
        lds = c.size() * sizeof(double);
        snprintf(nm, sizeof nm, "rwm_gsn_diag_s_kernel<D=%d,LPC=1,%s,PER_OBS%s>", D, full ? "FULL" : "ACCEPT_ONLY",
                 v.unit ? ",UNIT_T" : "");
        v.name = nm;
    }
    if (h->d_consts) (void)hipFree(h->d_consts);
    HIPCHK(h, hipMalloc(&h->d_consts, c.size() * sizeof(double)));
    HIPCHK(h, hipMemcpy(h->d_consts, c.data(), c.size() * sizeof(double), hipMemcpyHostToDevice));
    if (h->d_obs) (void)hipFree(h->d_obs);
    h->d_obs = nullptr;
    if (t.nobs) {
        HIPCHK(h, hipMalloc(&h->d_obs, t.obs.size() * sizeof(double)));
        HIPCHK(h, hipMemcpy(h->d_obs, t.obs.data(), t.obs.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    h->lds_bytes = lds;
    if (emcmc_status st2 = allow_lds(h, reinterpret_cast<const void *>(v.fn), lds)) return st2;
    h->var = v;
    return EMCMC_OK;
}

// Algorithmic HBM bytes of one launch group: the step kernel
// and, on the mix / chain-moments path, the batched mean/cov kernel and the
// Haario readjust when it follows the group.
// The fused diagonal kernel in FULL history mode leaves θ in its launch's last history slot
// and does not write the state buffer too (8·D bytes per chain and launch less: 2.3% of a
// 20-step launch at D = 32); theta_live points there until something else needs d_theta.
bool theta_in_hist(const emcmc_handle *h) {
    return h->var.fn && !h->var.ffn && !h->var.mfn && !h->var.ufn && !h->var.xfn && !h->var.afn &&
           h->var.dense == 0 && h->d_hist_theta && h->cfg.history_mode == EMCMC_HIST_FULL && h->theta_live_ok;
}
emcmc_status settle_theta(emcmc_handle *h) {
    if (!h->theta_live) return EMCMC_OK;
    const uint64_t n = h->cfg.num_chains * (uint64_t)h->cfg.dim;
    HIPCHK(h, hipMemcpyAsync(h->d_theta, h->theta_live, n * sizeof(double), hipMemcpyDeviceToDevice, h->stream));
    h->theta_live = nullptr;
    return EMCMC_OK;
}

double bytes_per_launch(const emcmc_handle *h, uint64_t nsteps, bool readjust) {
    const double C = (double)h->cfg.num_chains, D = (double)h->cfg.dim;
    double per_step = (h->cfg.history_mode == EMCMC_HIST_FULL) ? (16.0 * D + 8.0 + 0.125) : 0.125;
    double state = 16.0 * D + 2 * 8 + 2 * 8 + 2 * 16 + 2 * 4 + 2 * 4;  // θ, ll, ra, ring, nacc, faults (R+W)
    if (theta_in_hist(h)) state -= 8.0 * D;  // θ read, not written back (its last history slot holds it)
    if (h->var.xfn) {
        const double DP = D * (D + 1) / 2;
        // mix_moments_kernel: θ of every step once (ACCEPT_ONLY: written by the
        // step kernel to a scratch and read back), mean and cov read + written
        per_step += (h->cfg.history_mode == EMCMC_HIST_FULL) ? 8.0 * D : 16.0 * D;
        state += 16.0 * DP + 16.0 * D;
        if (h->updates[0].kernel == EMCMC_RW_GAUSSIAN_MIX) {
            if (h->var.xres) state += 8.0 * DP + 8.0 * D;  // L_B and 1/L_B,ii, read once per launch (registers)
            else per_step += 8.0 * DP + 8.0 * D;            // L_B and 1/L_B,ii, read by every step
            state += 8.0;                                   // c0_B
        }
        // readjust: cov read, L_B / 1/L_B,ii / c0_B written
        if (readjust) state += 8.0 * DP + 8.0 * DP + 8.0 * D + 8.0;
    }
    return C * ((double)nsteps * per_step + state);
}

hipEvent_t get_event(emcmc_handle *h) {
    if (!h->ev_pool.empty()) {
        hipEvent_t e = h->ev_pool.back();
        h->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    // timing events only: no system-scope fence when one is recorded (the step kernels'
    // own end-of-dispatch release covers their results)
    (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
    return e;
}

// One step-kernel launch on the handle's stream.  With timing on, the launch
// carries its own start/stop events (hipExtLaunchKernel: the timestamps of the
// dispatch packet itself, as rocprofv3's kernel trace reports them, without the
// few µs of a separate event marker on either side).
hipError_t launch_step(emcmc_handle *h, const void *fn, dim3 grid, dim3 block, void **args, size_t lds,
                       uint64_t bytes) {
    if (!h->timing) return hipLaunchKernel(fn, grid, block, args, lds, h->stream);
    hipEvent_t e0 = get_event(h), e1 = get_event(h);
    const hipError_t e = hipExtLaunchKernel(fn, grid, block, args, lds, h->stream, e0, e1, 0);
    if (e == hipSuccess) {
        h->ev.emplace_back(e0, e1);
        h->pending_bytes += bytes;
    }
    return e;
}

// The same for a kernel of a run-time compiled module: event markers around the launch.
hipError_t launch_module(emcmc_handle *h, hipFunction_t fn, dim3 grid, dim3 block, void **args, size_t lds,
                         uint64_t bytes) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (h->timing) {
        e0 = get_event(h);
        e1 = get_event(h);
        if (hipError_t e = hipEventRecord(e0, h->stream)) return e;
    }
    if (hipError_t e = hipModuleLaunchKernel(fn, grid.x, 1, 1, block.x, 1, 1, (unsigned)lds, h->stream, args, nullptr))
        return e;
    if (h->timing) {
        if (hipError_t e = hipEventRecord(e1, h->stream)) return e;
        h->ev.emplace_back(e0, e1);
        h->pending_bytes += bytes;
    }
    return hipSuccess;
}

emcmc_status drain_timing(emcmc_handle *h) {
    for (auto &p : h->ev) {
        float ms = 0.f;
        HIPCHK(h, hipEventSynchronize(p.second));
        HIPCHK(h, hipEventElapsedTime(&ms, p.first, p.second));
        h->timed_ms += ms;
        h->timed_launches += 1;
        h->ev_pool.push_back(p.first);
        h->ev_pool.push_back(p.second);
    }
    h->ev.clear();
    h->timed_bytes += h->pending_bytes;
    h->pending_bytes = 0.0;
    return EMCMC_OK;
}

// ---- history ring -------------------------------------------------------------
// Kernels address history slot (iter−1)·P + pidx0; a launch whose iterations all
// lie in one ring epoch [e·R+1, (e+1)·R] gets history pointers shifted back by
// e·R iterations, so the same arithmetic lands in ring slot (iter−1) mod R.
struct HistPtrs {
    double *theta, *prop, *ll;
    uint8_t *acc;
};
uint64_t ring_epoch(const emcmc_handle *h, uint64_t iter) { return (iter - 1) / h->ring; }

HistPtrs shifted_hist(const emcmc_handle *h, uint64_t iter) {
    const uint64_t C = h->cfg.num_chains, D = h->cfg.dim, P = h->updates.size();
    const int64_t sh = -(int64_t)(ring_epoch(h, iter) * h->ring * P);  // slots
    HistPtrs o;
    o.theta = h->d_hist_theta ? h->d_hist_theta + sh * (int64_t)(C * D) : nullptr;
    o.prop = h->d_hist_prop ? h->d_hist_prop + sh * (int64_t)(C * D) : nullptr;
    o.ll = h->d_hist_ll ? h->d_hist_ll + sh * (int64_t)C : nullptr;
    o.acc = h->d_hist_acc + sh * (int64_t)h->row_bytes;
    return o;
}

// Before a launch writing iterations [a, b] (one epoch): the ring slots it
// overwrites held iterations [a−R, b−R]; wait for any streaming copy reading them.
emcmc_status guard_ring(emcmc_handle *h, uint64_t a, uint64_t b) {
    h->hi_iter = std::max(h->hi_iter, b);
    if (h->copies.empty() || h->ring >= h->cfg.num_mcmc_steps) return EMCMC_OK;
    const int64_t lo = (int64_t)a - (int64_t)h->ring, hi = (int64_t)b - (int64_t)h->ring;
    for (auto it = h->copies.begin(); it != h->copies.end();) {
        if (hipEventQuery(it->ev) == hipSuccess) {  // finished: forget it
            (void)hipEventDestroy(it->ev);
            it = h->copies.erase(it);
            continue;
        }
        if ((int64_t)it->hi >= lo && (int64_t)it->lo <= hi) HIPCHK(h, hipStreamWaitEvent(h->stream, it->ev, 0));
        ++it;
    }
    return EMCMC_OK;
}

// Mix / chain-moments path: maximal runs of consecutive iterations, cut at
// K steps and at Haario readjust steps (M reaches k after the run), each
// followed by the readjust kernel when due.
emcmc_status run_mix(emcmc_handle *h, const emcmc_step *steps, uint64_t num_steps) {
    const uint64_t C = h->cfg.num_chains;
    const TargetHost &t = h->target;
    UpdateHost &u = h->updates[0];
    const bool haario = u.adaptation == EMCMC_ADPT_HAARIO;
    const uint32_t k = haario ? u.haario.adapt_every_k_steps : 0;
    MixParams p{};
    p.theta = h->d_theta;
    p.ll = h->d_ll;
    p.ra = h->d_ra;
    p.ring = h->d_ring;
    p.nacc = h->d_nacc;
    p.faults = h->d_faults;
    p.fault_flag = h->d_fault_flag;
    p.ll_prop = h->d_ll_prop;
    p.mom_theta = h->d_mom_scratch;
    p.LB = h->d_LB;
    p.iLB = h->d_iLB;
    p.c0B = h->d_c0B;
    p.hist_theta = h->d_hist_theta;
    p.hist_prop = h->d_hist_prop;
    p.hist_ll = h->d_hist_ll;
    p.hist_acc = h->d_hist_acc;
    p.zig = h->d_zig;
    p.consts = h->d_consts;
    p.obs = h->d_obs;
    p.sconsts = h->d_consts;  // mix_chol_kernel's layout when it is selected
    p.C = C;
    p.row_bytes = h->row_bytes;
    p.chain0 = (uint32_t)h->cfg.first_chain_id;
    p.key0 = (uint32_t)h->cfg.seed;
    p.key1 = (uint32_t)(h->cfg.seed >> 32);
    p.W = h->cfg.roll_window;
    p.nobs = (uint32_t)t.nobs;
    p.tdiag = t.diag ? 1u : 0u;
    p.lam = u.lam;
    p.oml = 1.0 - u.lam;
    p.c0A = u.c0;
    p.t_c0 = t.c0;
    p.n_tc0 = (double)t.nobs * t.c0;
    p.S_c = t.S_c;
    p.nobs_d = (double)t.nobs;
    p.rcp_W = 1.0 / (double)h->cfg.roll_window;
    MixReadjustParams r{};
    r.cov = h->d_cov;
    r.LB = h->d_LB;
    r.iLB = h->d_iLB;
    r.c0B = h->d_c0B;
    r.faults = h->d_faults;
    r.fault_flag = h->d_fault_flag;
    r.C = C;
    r.sB = (2.38 * 2.38) / (double)h->cfg.dim;  // 2.38^2/length(rw), adaptation.jl:423
    const dim3 block(256), grid((unsigned)((C + 255) / 256));
    const dim3 rgrid_res((unsigned)(C / kMixResChainsPerBlock));  // mix_res_kernel: 16 chains per block (C % 16 == 0)
    const uint64_t K = h->cfg.steps_per_launch;
    // (running the mean/cov kernel of a launch on a second stream beside the next launch's
    // step kernel was measured 18% slower at cfg 4: DESIGN.md §6, scripts/ab/mix_overlap.patch)
    uint64_t i = 0;
    while (i < num_steps) {
        uint64_t cap = K;
        if (haario) cap = std::min<uint64_t>(cap, k - h->mix_M);
        uint64_t j = i + 1;
        while (j < num_steps && j - i < cap && steps[j].mcmciter == steps[j - 1].mcmciter + 1 &&
               ring_epoch(h, steps[j].mcmciter) == ring_epoch(h, steps[i].mcmciter))
            ++j;
        const uint64_t n = j - i;
        p.iter0 = steps[i].mcmciter;
        p.nsteps = (uint32_t)n;
        p.N0 = h->stats_N;
        {
            const HistPtrs hp = shifted_hist(h, p.iter0);
            p.hist_theta = hp.theta;
            p.hist_prop = hp.prop;
            p.hist_ll = hp.ll;
            p.hist_acc = hp.acc;
            emcmc_status gs = guard_ring(h, p.iter0, steps[j - 1].mcmciter);
            if (gs) return gs;
        }
        if (p.iter0 > 1 && h->last_iter[0] != p.iter0 - 1)  // rolling_ar[iter−1] never written → 0.0
            HIPCHK(h, hipMemsetAsync(h->d_ra, 0, C * sizeof(double), h->stream));
        h->last_iter[0] = steps[j - 1].mcmciter;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (h->timing) {
            e0 = get_event(h);
            e1 = get_event(h);
            HIPCHK(h, hipEventRecord(e0, h->stream));
        }
        void *args[] = {&p};
        HIPCHK(h, hipLaunchKernel(reinterpret_cast<const void *>(h->var.xfn), h->var.xres ? rgrid_res : grid, block,
                                  args, h->lds_bytes, h->stream));
        {  // the launch's mean/cov recurrence, from its θ history
            MixMomentsParams mp{};
            mp.theta = p.hist_theta ? p.hist_theta + (uint64_t)(p.iter0 - 1) * h->cfg.dim * C : h->d_mom_scratch;
            mp.mean = h->d_mean;
            mp.mean_out = h->d_mean_alt;
            mp.cov = h->d_cov;
            mp.C = C;
            mp.N0 = p.N0;
            mp.nsteps = p.nsteps;
            mp.kst = h->d_mom_consts;
            {
                uint64_t n0 = p.N0;
                uint32_t ns = p.nsteps;
                double *kst = h->d_mom_consts;
                void *kargs[] = {&n0, &ns, &kst};
                HIPCHK(h, hipLaunchKernel(reinterpret_cast<const void *>(&moments_consts_kernel),
                                          dim3((ns + 63) / 64), dim3(64), kargs, 0, h->stream));
            }
            void *margs[] = {&mp};
            // one block per 64 chains, one wave per unit of the packed triangle
            const dim3 mgrid((unsigned)((C + 63) / 64)), mblock((unsigned)(64 * h->var.mo_tiles));
            HIPCHK(h, hipLaunchKernel(reinterpret_cast<const void *>(h->var.mofn), mgrid, mblock, margs, 0, h->stream));
            std::swap(h->d_mean, h->d_mean_alt);
        }
        h->stats_N += n;
        bool readjusted = false;
        if (haario) {
            h->mix_M += (uint32_t)n;
            if (h->mix_M >= k) {  // time_to_update: readjust!, M = 0
                void *rargs[] = {&r};
                const int cpb = readjust_chains_per_block((int)h->cfg.dim);
                const dim3 rgrid((unsigned)((C + cpb - 1) / cpb));
                HIPCHK(h, hipLaunchKernel(reinterpret_cast<const void *>(h->var.rfn), rgrid, block, rargs, 0,
                                          h->stream));
                h->mix_M = 0;
                readjusted = true;
                if (u.flam) {  // rw.λ = adpt.fλ(rw.λ, adpt.N, mcmc_iter) (adaptation.jl:425)
                    u.lam = u.flam(u.lam, (int64_t)h->stats_N, (int64_t)steps[j - 1].mcmciter, u.flam_ctx);
                    p.lam = u.lam;
                    p.oml = 1.0 - u.lam;
                }
            }
        }
        if (h->timing) {  // the whole group: step kernel, mean/cov kernel, readjust
            HIPCHK(h, hipEventRecord(e1, h->stream));
            h->ev.emplace_back(e0, e1);
            h->pending_bytes += bytes_per_launch(h, n, readjusted);
        }
        i = j;
    }
    return EMCMC_OK;
}

// MALA: one launch per MCMC step (the X stream dominates; launch cost is
// negligible); ∇ℓ(θinit) is evaluated by the MODE-1 kernel before the first step.
emcmc_status run_mala(emcmc_handle *h, const emcmc_step *steps, uint64_t num_steps) {
    const uint64_t C = h->cfg.num_chains, D = h->cfg.dim;
    const UpdateHost &u = h->updates[0];
    const TargetHost &t = h->target;
    MalaParams p{};
    p.theta = h->d_theta;
    p.grad = h->d_grad;
    p.ll = h->d_ll;
    p.ra = h->d_ra;
    p.ring = h->d_ring;
    p.nacc = h->d_nacc;
    p.faults = h->d_faults;
    p.fault_flag = h->d_fault_flag;
    p.ll_prop = h->d_ll_prop;
    p.hist_theta = h->d_hist_theta;
    p.hist_prop = h->d_hist_prop;
    p.hist_ll = h->d_hist_ll;
    p.hist_acc = h->d_hist_acc;
    p.zig = h->d_zig;
    p.X = h->d_X;
    p.y = h->d_y;
    p.C = C;
    p.row_bytes = h->row_bytes;
    p.nrows = t.nobs;
    p.ntiles = h->mala_tiles;
    p.chain0 = (uint32_t)h->cfg.first_chain_id;
    p.key0 = (uint32_t)h->cfg.seed;
    p.key1 = (uint32_t)(h->cfg.seed >> 32);
    p.W = h->cfg.roll_window;
    const double eps = u.eps[0];
    p.eps = eps;
    p.h = (eps * eps) / 2.0;
    p.ieps = 1.0 / eps;
    {  // MvNormal(m, ϵ²I): logdet = dd + dd, dd = Σ_d log ϵ
        double dd = 0.0;
        for (uint64_t d = 0; d < D; ++d) dd = dd + log_pos(eps);
        p.c0 = mvnormal_c0((int)D, dd + dd);
    }
    p.rcp_W = 1.0 / (double)h->cfg.roll_window;
    const dim3 block(256), grid((unsigned)((C + kMalaChainsPerWG - 1) / kMalaChainsPerWG));
    if (!h->grad_valid) {
        void *args[] = {&p};
        HIPCHK(h, hipLaunchKernel(reinterpret_cast<const void *>(h->var.ainit), grid, block, args, 0, h->stream));
        h->grad_valid = true;
    }
    for (uint64_t i = 0; i < num_steps; ++i) {
        p.iter = steps[i].mcmciter;
        p.N0 = h->stats_N;
        {
            const HistPtrs hp = shifted_hist(h, p.iter);
            p.hist_theta = hp.theta;
            p.hist_prop = hp.prop;
            p.hist_ll = hp.ll;
            p.hist_acc = hp.acc;
            emcmc_status gs = guard_ring(h, p.iter, p.iter);
            if (gs) return gs;
        }
        if (p.iter > 1 && h->last_iter[0] != p.iter - 1)  // rolling_ar[iter−1] never written → 0.0
            HIPCHK(h, hipMemsetAsync(h->d_ra, 0, C * sizeof(double), h->stream));
        h->last_iter[0] = p.iter;
        void *args[] = {&p};
        HIPCHK(h, launch_step(h, reinterpret_cast<const void *>(h->var.afn), grid, block, args, 0,
                              bytes_per_launch(h, 1, false)));
        h->stats_N += 1;
    }
    return EMCMC_OK;
}

// General schedule: the step list goes to HBM (4 u32 per step, read by the
// kernel with scalar loads) and runs in launches of ≤ K steps in schedule order.
emcmc_status run_mwg(emcmc_handle *h, const emcmc_step *steps, uint64_t num_steps) {
    const uint64_t C = h->cfg.num_chains, P = h->updates.size();
    const uint64_t cap = h->cfg.num_mcmc_steps * P;
    if (num_steps == 0) return EMCMC_OK;
    if (num_steps > cap) return fail(h, EMCMC_INVALID_ARG, "more steps than M·P in one call");
    if (!h->mwg_pool_ready) {
        emcmc_status ps = reset_mwg_pool(h);
        if (ps) return ps;
    }
    std::vector<uint32_t> st(4 * num_steps);
    // HaarioTypeAdaptation: M += 1 on its own turn, readjust! at M ≥ k (flags bit 1,
    // adaptation.jl:399-426); with a user fλ the launch ends after a readjust and
    // the next one reads the new λ (cut[i]: λ of the following steps)
    std::vector<std::pair<uint64_t, std::pair<uint32_t, double>>> cuts;
    uint64_t Nh = h->stats_N;
    for (uint64_t i = 0; i < num_steps; ++i) {
        const uint32_t it = steps[i].mcmciter, q = steps[i].pidx - 1;
        st[4 * i] = it;
        st[4 * i + 1] = steps[i].pidx;
        st[4 * i + 2] = (it > 1 && h->last_iter[q] == it - 1) ? 1u : 0u;  // rolling_ar[it−1][q] was written
        st[4 * i + 3] = 0;
        h->last_iter[q] = it;
        UpdateHost &u = h->updates[q];
        ++Nh;  // adpt.N after this step's register! (= GenericChainStats.N)
        if (u.kernel == EMCMC_RW_GAUSSIAN_MIX && u.adaptation == EMCMC_ADPT_HAARIO &&
            ++h->mwg_M[q] >= u.haario.adapt_every_k_steps) {
            h->mwg_M[q] = 0;
            st[4 * i + 2] |= 2u;
            if (u.flam) {  // rw.λ = adpt.fλ(rw.λ, adpt.N, mcmc_iter) (adaptation.jl:425)
                u.lam = u.flam(u.lam, (int64_t)Nh, (int64_t)it, u.flam_ctx);
                cuts.push_back({i + 1, {q, u.lam}});
            }
        }
    }
    if (h->steps_used + num_steps > cap) h->steps_used = 0;  // earlier lists were consumed in stream order
    uint32_t *dst = h->d_steps + 4 * h->steps_used;
    HIPCHK(h, hipMemcpyAsync(dst, st.data(), st.size() * sizeof(uint32_t), hipMemcpyHostToDevice, h->stream));
    h->steps_staging.push_back(std::move(st));  // alive until emcmc_synchronize
    h->steps_used += num_steps;
    const TargetHost &t = h->target;
    MwgParams a{};
    a.theta = h->d_theta;
    a.mu_p = h->d_mu_p;
    a.ll = h->d_ll;
    a.ra = h->d_ra;
    a.ring = h->d_ring;
    a.nacc = h->d_nacc;
    a.aprop = h->d_aprop;
    a.aacc = h->d_aacc;
    a.eps = h->d_eps;
    a.faults = h->d_faults;
    a.fault_flag = h->d_fault_flag;
    a.ll_prop = h->d_ll_prop;
    a.hist_theta = h->d_hist_theta;
    a.hist_prop = h->d_hist_prop;
    a.hist_ll = h->d_hist_ll;
    a.hist_acc = h->d_hist_acc;
    a.zig = h->d_zig;
    a.updates = h->d_mwg;
    a.Lt = h->d_tL;
    a.iLt = h->d_tiL;
    a.xbar = h->d_xbar;
    a.obs = h->d_obs;
    a.user_params = h->d_uparams;
    a.C = C;
    a.row_bytes = h->row_bytes;
    a.chain0 = (uint32_t)h->cfg.first_chain_id;
    a.key0 = (uint32_t)h->cfg.seed;
    a.key1 = (uint32_t)(h->cfg.seed >> 32);
    a.P = (uint32_t)P;
    a.W = h->cfg.roll_window;
    a.nobs = (uint32_t)t.nobs;
    a.tdiag = t.diag ? 1u : 0u;
    a.t_c0 = t.c0;
    a.n_tc0 = (double)t.nobs * t.c0;
    a.S_c = t.S_c;
    a.nobs_d = (double)t.nobs;
    a.mixpool = h->d_mixpool;
    a.smean = h->d_smean;
    a.scov = h->d_scov;
    a.chain_moments = h->cfg.chain_moments ? 1u : 0u;
    a.nhaario = h->nhaario;
    a.consts = h->d_bconsts;
    if (P == 1 && h->updates[0].kernel == EMCMC_MALA) {  // one MALA update: carry ∇ℓ(θ) between steps
        if (!h->d_gcache) HIPCHK(h, hipMalloc(&h->d_gcache, C * (uint64_t)h->cfg.dim * sizeof(double)));
        a.gcache = h->d_gcache;
    }
    const dim3 block(256), grid((unsigned)((C + 255) / 256));
    const uint64_t K = h->cfg.steps_per_launch;
    size_t ci = 0;  // next λ cut
    if (!cuts.empty()) {  // the cut values stay alive until emcmc_synchronize: no host wait per readjust
        std::vector<double> lv(cuts.size());
        for (size_t k = 0; k < cuts.size(); ++k) lv[k] = cuts[k].second.second;
        h->lam_staging.push_back(std::move(lv));
    }
    const double *lam_src = cuts.empty() ? nullptr : h->lam_staging.back().data();
    for (uint64_t i = 0, n = 0; i < num_steps; i += n) {
        while (ci < cuts.size() && cuts[ci].first <= i) {  // λ after an fλ readjust, in stream order
            const uint32_t q = cuts[ci].second.first;
            HIPCHK(h, hipMemcpyAsync(reinterpret_cast<char *>(h->d_mwg + q) + offsetof(MwgUpdate, lam), lam_src + ci,
                                     sizeof(double), hipMemcpyHostToDevice, h->stream));
            ++ci;
        }
        const uint64_t lim = (ci < cuts.size()) ? cuts[ci].first : num_steps;  // end the launch at the next cut
        n = 1;  // ≤ K steps, all in one ring epoch
        while (i + n < lim && n < K && ring_epoch(h, steps[i + n].mcmciter) == ring_epoch(h, steps[i].mcmciter))
            ++n;
        a.steps = dst + 4 * i;
        a.nsteps = (uint32_t)n;
        a.N0 = h->stats_N;
        {
            uint64_t lo = steps[i].mcmciter, hi = lo;
            for (uint64_t k = i; k < i + n; ++k) {
                lo = std::min<uint64_t>(lo, steps[k].mcmciter);
                hi = std::max<uint64_t>(hi, steps[k].mcmciter);
            }
            const HistPtrs hp = shifted_hist(h, lo);
            a.hist_theta = hp.theta;
            a.hist_prop = hp.prop;
            a.hist_ll = hp.ll;
            a.hist_acc = hp.acc;
            emcmc_status gs = guard_ring(h, lo, hi);
            if (gs) return gs;
        }
        void *args[] = {&a};
        if (h->var.ufn) {  // a run-time compiled module
            HIPCHK(h, launch_module(h, h->var.ufn, grid, block, args, h->lds_bytes, bytes_per_launch(h, n, false)));
        } else {
            HIPCHK(h, launch_step(h, reinterpret_cast<const void *>(h->var.mfn), grid, block, args, h->lds_bytes,
                                  bytes_per_launch(h, n, false)));
        }
        h->stats_N += n;
    }
    return EMCMC_OK;
}

}  // namespace

// ============================================================================
extern "C" {

emcmc_status emcmc_device_count(int *count) {
    if (!count) return EMCMC_INVALID_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return EMCMC_OK;
}

emcmc_status emcmc_create(emcmc_handle **out, const emcmc_config *cfg) {
    if (!out || !cfg) return EMCMC_INVALID_ARG;
    *out = nullptr;
    if (cfg->abi_version != EMCMC_ABI_VERSION) return EMCMC_INVALID_ARG;
    if (cfg->dim == 0 || cfg->num_chains == 0 || cfg->num_mcmc_steps == 0) return EMCMC_INVALID_ARG;
    if (cfg->first_chain_id + cfg->num_chains > (1ull << 32)) return EMCMC_INVALID_ARG;  // 32-bit chain ids
    if (cfg->num_mcmc_steps >= (1ull << 32)) return EMCMC_INVALID_ARG;
    if (cfg->history_mode > EMCMC_HIST_ACCEPT_ONLY) return EMCMC_INVALID_ARG;
    if (cfg->roll_window > 128) return EMCMC_INVALID_ARG;
    // history slots and the state array are addressed with a 32-bit per-lane byte offset
    // (SlotOffset, LaneSoA) from a wave-uniform base, whatever the history mode
    if (cfg->num_chains * cfg->dim * sizeof(double) > 0xFFFFFFFFull) return EMCMC_INVALID_ARG;
    if (cfg->lanes_per_chain != 0 && cfg->lanes_per_chain != 1 && cfg->lanes_per_chain != 2 &&
        cfg->lanes_per_chain != 4)
        return EMCMC_INVALID_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return EMCMC_NO_DEVICE;
    if (cfg->device < 0 || cfg->device >= n) return EMCMC_INVALID_ARG;
    if (hipSetDevice(cfg->device) != hipSuccess) return EMCMC_HIP_ERROR;
    auto *h = new emcmc_handle();
    h->cfg = *cfg;
    if (h->cfg.roll_window == 0) h->cfg.roll_window = kDefaultRollWindow;
    if (h->cfg.steps_per_launch == 0) h->cfg.steps_per_launch = kDefaultStepsPerLaunch;
    h->ring = (h->cfg.history_ring && h->cfg.history_ring < h->cfg.num_mcmc_steps) ? h->cfg.history_ring
                                                                                    : h->cfg.num_mcmc_steps;
    if (hipStreamCreateWithFlags(&h->cstream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return EMCMC_HIP_ERROR;
    }
    if (const char *e = getenv("EMCMC_HOST_TIMING")) h->host_timing = *e && *e != '0';
    if (const char *e = getenv("EMCMC_SYNC")) h->sync_mode = atoi(e) ? 1 : 0;
    if (const char *e = getenv("EMCMC_THETA_LIVE")) h->theta_live_ok = atoi(e) != 0;
    if (h->sync_mode && hipEventCreateWithFlags(&h->sync_ev, hipEventDisableTiming) != hipSuccess) h->sync_mode = 0;
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        if (h->sync_ev) (void)hipEventDestroy(h->sync_ev);
        (void)hipStreamDestroy(h->cstream);
        delete h;
        return EMCMC_HIP_ERROR;
    }
    load_aot_code_objects(cfg->device);
    *out = h;
    return EMCMC_OK;
}

namespace {
// (family, a, b) of a univariate prior factor → the device's (a, b, c)
// (emcmc_mwg.h univariate_logpdf; restated in oracle/emcmc_oracle.c)
emcmc_status univariate_consts(emcmc_handle *h, uint32_t fam, double a, double b, double &pa, double &pb,
                               double &pc) {
    pa = a, pb = b;
    switch (fam) {
    case EMCMC_DIST_NORMAL:
    case EMCMC_DIST_LOGNORMAL:
        if (!(b > 0.0)) return fail(h, EMCMC_INVALID_ARG, "Normal/LogNormal prior: σ must be > 0");
        pc = log_pos(b);
        return EMCMC_OK;
    case EMCMC_DIST_UNIFORM:
        if (!(a < b)) return fail(h, EMCMC_INVALID_ARG, "Uniform prior: a < b");
        pc = -log_pos(b - a);
        return EMCMC_OK;
    case EMCMC_DIST_EXPONENTIAL:
        if (!(a > 0.0)) return fail(h, EMCMC_INVALID_ARG, "Exponential prior: θ must be > 0");
        pb = 1.0 / a;
        pc = log_pos(pb);
        return EMCMC_OK;
    case EMCMC_DIST_GAMMA:
        if (!(a > 0.0 && b > 0.0)) return fail(h, EMCMC_INVALID_ARG, "Gamma prior: α, θ must be > 0");
        pc = (-std::lgamma(a)) - a * log_pos(b);
        return EMCMC_OK;
    case EMCMC_DIST_BETA:
        if (!(a > 0.0 && b > 0.0)) return fail(h, EMCMC_INVALID_ARG, "Beta prior: α, β must be > 0");
        pc = (std::lgamma(a) + std::lgamma(b)) - std::lgamma(a + b);
        return EMCMC_OK;
    case EMCMC_DIST_INVERSE_GAMMA:
        if (!(a > 0.0 && b > 0.0)) return fail(h, EMCMC_INVALID_ARG, "InverseGamma prior: α, θ must be > 0");
        pc = a * log_pos(b) - std::lgamma(a);
        return EMCMC_OK;
    case EMCMC_DIST_CAUCHY:
        if (!(b > 0.0)) return fail(h, EMCMC_INVALID_ARG, "Cauchy prior: σ must be > 0");
        pc = log_pos(b);  // log σ (log π enters in Distributions.jl's order on the device)
        return EMCMC_OK;
    case EMCMC_DIST_LAPLACE:
        if (!(b > 0.0)) return fail(h, EMCMC_INVALID_ARG, "Laplace prior: θ must be > 0");
        pc = log_pos(2.0 * b);
        return EMCMC_OK;
    case EMCMC_DIST_TDIST:
        if (!(a > 0.0)) return fail(h, EMCMC_INVALID_ARG, "TDist prior: ν must be > 0");
        pb = (a + 1.0) / 2.0;
        pc = (std::lgamma((a + 1.0) / 2.0) - std::lgamma(a / 2.0)) - log_pos(a * 3.141592653589793) / 2.0;
        return EMCMC_OK;
    }
    return fail(h, EMCMC_UNSUPPORTED_PLUGIN, "prior family %u has no device plugin", fam);
}

// ProductPrior / StandardPrior → term slots (emcmc_mwg.h MwgUpdate).  The index
// list is the constructor's (priors.jl:64-79): a dims-1 factor reads θ_local[1]
// and takes one slot; a dims-k factor reads θ_local[last:last+k−1] and takes k
// slots; `last` advances by dims either way, so slot j reads θ_local[j] unless it
// belongs to a dims-1 factor.
emcmc_status build_prior_slots(emcmc_handle *h, const emcmc_update_desc *u, UpdateHost &uh) {
    const emcmc_prior_desc *pd = u->prior_params;
    const uint32_t n = u->num_coords;
    if (!pd || !pd->factors || pd->num_factors == 0)
        return fail(h, EMCMC_INVALID_ARG, "ProductPrior/StandardPrior needs prior_params factors");
    if (u->prior == EMCMC_PRIOR_STANDARD && pd->num_factors != 1)
        return fail(h, EMCMC_INVALID_ARG, "StandardPrior has exactly one distribution");
    uh.pfam.assign(kMwgMaxD, 0u);
    uh.pmvs.assign(kMwgMaxD, 0u);
    uh.pa.assign(kMwgMaxD, 0.0);
    uh.pb.assign(kMwgMaxD, 0.0);
    uh.pc.assign(kMwgMaxD, 0.0);
    uh.pmu.assign(kMwgMaxD, 0.0);
    uh.piL.assign(kMwgMaxD, 0.0);
    uh.pL.assign((size_t)kMwgMaxD * kMwgMaxD, 0.0);
    uint32_t last = 0;
    for (uint32_t f = 0; f < pd->num_factors; ++f) {
        const emcmc_prior_factor &fa = pd->factors[f];
        const uint32_t k = fa.count;
        const bool multi = fa.family == EMCMC_DIST_PRODUCT || fa.family == EMCMC_DIST_MVNORMAL;
        if (k == 0) return fail(h, EMCMC_INVALID_ARG, "prior factor %u: dims must be ≥ 1", f);
        if (u->prior == EMCMC_PRIOR_STANDARD) {
            if (!multi)
                return fail(h, EMCMC_UNSUPPORTED_PLUGIN,
                            "StandardPrior(univariate) on a coordinate vector: logpdf(dist, θ::Vector) has no "
                            "scalar value in the reference (priors.jl:39); use Product([dist]) or ProductPrior");
            if (k != n) return fail(h, EMCMC_INVALID_ARG, "StandardPrior: length(dist) must equal length(coords)");
        } else if (multi != (k > 1)) {
            return fail(h, EMCMC_UNSUPPORTED_PLUGIN,
                        multi ? "ProductPrior factor %u: a multivariate dist with dims 1 reads the scalar θ[1] "
                                "(priors.jl:68-70), a MethodError in the reference"
                              : "ProductPrior factor %u: a univariate dist over dims > 1 reads the vector "
                                "θ[last:last+dims-1] (priors.jl:72), a MethodError in the reference",
                        f);
        }
        const uint32_t st = (k == 1) ? 0u : last;
        const uint32_t s0 = last;  // first slot of this factor
        if (last + k > n)
            return fail(h, EMCMC_INVALID_ARG,
                        "ProductPrior dims sum to more than the update's %u coordinates (the reference raises a "
                        "BoundsError for a dims > 1 factor past the end; more dims-1 factors than coordinates are "
                        "not supported on device)",
                        n);
        last += k;
        uh.pstart |= 1ull << s0;
        uh.pend |= 1ull << (s0 + k - 1);
        if (k == 1) uh.psrc0 |= 1ull << s0;
        if (fa.family == EMCMC_DIST_PRODUCT) {
            if (!fa.components) return fail(h, EMCMC_INVALID_ARG, "Product prior factor needs its components");
            for (uint32_t i = 0; i < k; ++i) {
                const emcmc_prior_factor &cp = fa.components[i];
                if (cp.family == EMCMC_DIST_PRODUCT || cp.family == EMCMC_DIST_MVNORMAL || cp.count != 1)
                    return fail(h, EMCMC_UNSUPPORTED_PLUGIN, "Product components must be univariate");
                uh.pfam[s0 + i] = cp.family;
                if (emcmc_status e = univariate_consts(h, cp.family, cp.a, cp.b, uh.pa[s0 + i], uh.pb[s0 + i],
                                                       uh.pc[s0 + i]))
                    return e;
            }
        } else if (fa.family == EMCMC_DIST_MVNORMAL) {
            if (!fa.mu || !fa.sigma) return fail(h, EMCMC_INVALID_ARG, "MvNormal prior factor needs μ and Σ");
            std::vector<double> Lk;
            if (!cholesky_upper_colmajor(fa.sigma, (int)k, Lk))
                return fail(h, EMCMC_INVALID_ARG, "MvNormal prior factor %u: Σ is not positive definite", f);
            for (uint32_t i = 0; i < k; ++i) {
                const uint32_t j = st + i;
                uh.pmvn |= 1ull << j;
                uh.pmvs[j] = st;
                uh.pmu[j] = fa.mu[i];
                uh.piL[j] = 1.0 / Lk[(size_t)i * k + i];
                for (uint32_t q = 0; q <= i; ++q) uh.pL[(size_t)j * kMwgMaxD + st + q] = Lk[(size_t)i * k + q];
            }
            uh.pc[st + k - 1] = mvnormal_c0((int)k, logdet_chol(Lk, (int)k));
        } else {
            uh.pfam[s0] = fa.family;
            if (emcmc_status e = univariate_consts(h, fa.family, fa.a, fa.b, uh.pa[s0], uh.pb[s0], uh.pc[s0])) return e;
        }
    }
    uh.nslot = last;
    return EMCMC_OK;
}
}  // namespace

namespace {
// emcmc_update_desc → UpdateHost: every check and host-side factorisation of
// emcmc_add_update (h supplies D, the error text and the handle's other updates; a
// device-less handle serves emcmc_prebuild_rw_block_kernel)
emcmc_status build_update(emcmc_handle *h, const emcmc_update_desc *u, UpdateHost &uh) {
    const uint32_t D = h->cfg.dim;
    if (u->num_coords == 0 || !u->coords) return fail(h, EMCMC_INVALID_ARG, "update needs coords");
    if (u->num_coords > D) return fail(h, EMCMC_INVALID_ARG, "more coords than D");
    for (uint32_t i = 0; i < u->num_coords; ++i) {
        if (u->coords[i] >= D) return fail(h, EMCMC_INVALID_ARG, "coord %u out of range (D=%u)", u->coords[i], D);
        for (uint32_t j = 0; j < i; ++j)
            if (u->coords[j] == u->coords[i]) return fail(h, EMCMC_INVALID_ARG, "repeated coord %u", u->coords[i]);
    }
    if (u->kernel != EMCMC_RW_GAUSSIAN && u->kernel != EMCMC_RW_UNIFORM && u->kernel != EMCMC_RW_GAUSSIAN_MIX &&
        u->kernel != EMCMC_MALA && u->kernel != EMCMC_USER_UPDATE)
        return fail(h, EMCMC_UNSUPPORTED_PLUGIN, "transition kernel %u has no device plugin yet", u->kernel);
    if (u->kernel == EMCMC_USER_UPDATE) {
        const emcmc_user_update_desc *ud = u->user_update;
        if (!ud || !ud->source) return fail(h, EMCMC_INVALID_ARG, "user update: needs user_update->source");
        if (ud->num_params > (uint64_t)kMwgMaxD * kMwgMaxD || (ud->num_params && !ud->params))
            return fail(h, EMCMC_INVALID_ARG, "user update: params (≤ %d doubles)", kMwgMaxD * kMwgMaxD);
        if (u->adaptation != EMCMC_ADPT_NONE)
            return fail(h, EMCMC_UNSUPPORTED_PLUGIN, "user update: adaptation has no device plugin");
        if (h->cfg.dim > (uint32_t)kMwgMaxD)
            return fail(h, EMCMC_UNSUPPORTED_PLUGIN, "user update: D=%u > %d (general schedule kernel)", h->cfg.dim,
                        kMwgMaxD);
        for (const auto &o : h->updates)
            if (o.kernel == EMCMC_USER_UPDATE &&
                (o.usrc != ud->source || o.uopts != (ud->options ? ud->options : "")))
                return fail(h, EMCMC_UNSUPPORTED_PLUGIN,
                            "user updates of one handle share one source (dispatch on params to combine several)");
    }
    if (u->prior > EMCMC_PRIOR_STANDARD)
        return fail(h, EMCMC_UNSUPPORTED_PLUGIN, "prior %u has no device plugin", u->prior);
    if (u->adaptation != EMCMC_ADPT_NONE &&
        !((u->adaptation == EMCMC_ADPT_UNIF_RW || u->adaptation == EMCMC_ADPT_UNIF_RW_VEC) &&
          u->kernel == EMCMC_RW_UNIFORM) &&
        !(u->adaptation == EMCMC_ADPT_HAARIO && u->kernel == EMCMC_RW_GAUSSIAN_MIX))
        return fail(h, EMCMC_UNSUPPORTED_PLUGIN, "adaptation %u has no device plugin for kernel %u yet",
                    u->adaptation, u->kernel);
    std::vector<uint8_t> pos(u->num_coords, 0);
    if (u->pos)
        for (uint32_t i = 0; i < u->num_coords; ++i) {
            pos[i] = u->pos[i] ? 1 : 0;
            if (pos[i] && u->kernel != EMCMC_RW_UNIFORM && u->kernel != EMCMC_RW_GAUSSIAN &&
                u->kernel != EMCMC_RW_GAUSSIAN_MIX)
                return fail(h, EMCMC_UNSUPPORTED_PLUGIN,
                            "positivity-restricted coordinates are on device for the random walks only");
        }
    if (h->updates.size() >= 64) return fail(h, EMCMC_INVALID_ARG, "at most 64 updates");
    uh.kernel = u->kernel;
    uh.prior = u->prior;
    uh.adaptation = u->adaptation;
    uh.coords.assign(u->coords, u->coords + u->num_coords);
    uh.pos = pos;
    if (u->prior == EMCMC_PRIOR_PRODUCT || u->prior == EMCMC_PRIOR_STANDARD)
        if (emcmc_status st = build_prior_slots(h, u, uh)) return st;
    const int n = (int)u->num_coords;
    if (u->kernel == EMCMC_USER_UPDATE) {
        const emcmc_user_update_desc *ud = u->user_update;
        uh.usrc = ud->source;
        uh.uopts = ud->options ? ud->options : "";
        if (ud->num_params) uh.uparams.assign(ud->params, ud->params + ud->num_params);
    } else if (u->kernel == EMCMC_RW_GAUSSIAN || u->kernel == EMCMC_RW_GAUSSIAN_MIX) {
        if (!u->sigma) return fail(h, EMCMC_INVALID_ARG, "GaussianRandomWalk needs Σ");
        uh.sigma.assign(u->sigma, u->sigma + (size_t)n * n);
        if (!cholesky_upper_colmajor(uh.sigma.data(), n, uh.L))
            return fail(h, EMCMC_INVALID_ARG, "GaussianRandomWalk Σ is not positive definite");
        uh.invdiag.resize(n);
        for (int i = 0; i < n; ++i) uh.invdiag[i] = 1.0 / uh.L[(size_t)i * n + i];
        uh.diag = is_diag_upper(uh.sigma.data(), n);
        uh.c0 = mvnormal_c0(n, logdet_chol(uh.L, n));
        if (u->kernel == EMCMC_RW_GAUSSIAN_MIX) {  // random_walk.jl:198-206
            if (!u->sigma_b) return fail(h, EMCMC_INVALID_ARG, "GaussianRandomWalkMix needs Σ_B (sigma_b)");
            if (!(u->mix_lambda >= 0.0 && u->mix_lambda <= 1.0))
                return fail(h, EMCMC_INVALID_ARG, "GaussianRandomWalkMix: @assert 0.0 <= λ <= 1.0");
            uh.lam = uh.lam0 = u->mix_lambda;
            uh.sigma_b.assign(u->sigma_b, u->sigma_b + (size_t)n * n);
            if (!cholesky_upper_colmajor(uh.sigma_b.data(), n, uh.LB))
                return fail(h, EMCMC_INVALID_ARG, "GaussianRandomWalkMix Σ_B is not positive definite");
            uh.invdiagB.resize(n);
            for (int i = 0; i < n; ++i) uh.invdiagB[i] = 1.0 / uh.LB[(size_t)i * n + i];
            uh.c0B = mvnormal_c0(n, logdet_chol(uh.LB, n));
            if (u->adaptation == EMCMC_ADPT_HAARIO) {
                const auto *ad = static_cast<const emcmc_haario_adaptation *>(u->adaptation_params);
                if (!ad) return fail(h, EMCMC_INVALID_ARG, "HaarioTypeAdaptation parameters missing (adaptation_params)");
                if (ad->adapt_every_k_steps == 0) return fail(h, EMCMC_INVALID_ARG, "adapt_every_k_steps must be ≥ 1");
                uh.haario = *ad;
            }
        }
    } else if (u->kernel == EMCMC_MALA) {
        if (!u->epsilon || !(u->epsilon[0] > 0.0)) return fail(h, EMCMC_INVALID_ARG, "MALA needs a step size ϵ > 0");
        if (u->adaptation != EMCMC_ADPT_NONE) return fail(h, EMCMC_UNSUPPORTED_PLUGIN, "MALA adaptation");
        const double e = u->epsilon[0];
        uh.eps = {e, (e * e) / 2.0};  // ϵ, h = ϵ²/2
        // the transition density's MvNormal(·, ϵ²I) as the update's diagonal factor L = ϵI
        uh.L.assign((size_t)n * n, 0.0);
        for (int i = 0; i < n; ++i) uh.L[(size_t)i * n + i] = e;
        uh.invdiag.assign(n, 1.0 / e);
        uh.diag = true;
        uh.c0 = mvnormal_c0(n, logdet_chol(uh.L, n));
    } else {
        if (!u->epsilon) return fail(h, EMCMC_INVALID_ARG, "UniformRandomWalk needs ϵ");
        uh.eps.assign(u->epsilon, u->epsilon + n);
        for (double e : uh.eps)  // UniformRandomWalk: @assert all(ϵ .> 0.0) (random_walk.jl:50)
            if (!(e > 0.0)) return fail(h, EMCMC_INVALID_ARG, "UniformRandomWalk ϵ must be > 0");
        if (u->adaptation == EMCMC_ADPT_UNIF_RW) {
            const auto *ad = static_cast<const emcmc_unifrw_adaptation *>(u->adaptation_params);
            if (!ad) return fail(h, EMCMC_INVALID_ARG, "AdaptationUnifRW parameters missing (adaptation_params)");
            if (ad->adapt_every_k_steps == 0) return fail(h, EMCMC_INVALID_ARG, "adapt_every_k_steps must be ≥ 1");
            uh.adpt = *ad;
            uh.ascale.assign(n, ad->scale);
            uh.amin.assign(n, ad->min);
            uh.amax.assign(n, ad->max);
            uh.aoff.assign(n, ad->offset);
        } else if (u->adaptation == EMCMC_ADPT_UNIF_RW_VEC) {  // the per-coordinate form
            const auto *ad = static_cast<const emcmc_unifrw_adaptation_vec *>(u->adaptation_params);
            if (!ad || !ad->scale || !ad->min || !ad->max || !ad->offset)
                return fail(h, EMCMC_INVALID_ARG, "AdaptationUnifRW per-coordinate parameters missing");
            if (ad->adapt_every_k_steps == 0) return fail(h, EMCMC_INVALID_ARG, "adapt_every_k_steps must be ≥ 1");
            uh.adaptation = EMCMC_ADPT_UNIF_RW;  // one device form: per-coordinate arrays
            uh.adpt.adapt_every_k_steps = ad->adapt_every_k_steps;
            uh.adpt.target_accpt_rate = ad->target_accpt_rate;
            uh.ascale.assign(ad->scale, ad->scale + n);
            uh.amin.assign(ad->min, ad->min + n);
            uh.amax.assign(ad->max, ad->max + n);
            uh.aoff.assign(ad->offset, ad->offset + n);
        }
    }
    return EMCMC_OK;
}
}  // namespace

emcmc_status emcmc_add_update(emcmc_handle *h, const emcmc_update_desc *u) {
    if (!h || !u) return EMCMC_INVALID_ARG;
    if (h->allocated) return fail(h, EMCMC_STATE_ERROR, "updates must be added before set_state/run");
    UpdateHost uh;
    if (emcmc_status st = build_update(h, u, uh)) return st;
    h->updates.push_back(std::move(uh));
    return select_variant(h);
}

emcmc_status emcmc_set_target(emcmc_handle *h, const emcmc_target_desc *t) {
    if (!h || !t) return EMCMC_INVALID_ARG;
    if (t->kind != EMCMC_TARGET_GSN && t->kind != EMCMC_TARGET_LOGISTIC)
        return fail(h, EMCMC_UNSUPPORTED_PLUGIN, "target kind %u", t->kind);
    const uint32_t d = t->dim;
    if (t->kind == EMCMC_TARGET_LOGISTIC) {
        if (d != h->cfg.dim) return fail(h, EMCMC_INVALID_ARG, "logistic target: dim must equal D");
        if (!t->obs || !t->labels || t->num_obs == 0) return fail(h, EMCMC_INVALID_ARG, "logistic target needs X and y");
        TargetHost th;
        th.kind = EMCMC_TARGET_LOGISTIC;
        th.dim = d;
        th.nobs = t->num_obs;
        th.obs.assign(t->obs, t->obs + t->num_obs * d);
        th.labels.assign(t->labels, t->labels + t->num_obs);
        h->target = std::move(th);
        h->target_set = true;
        h->grad_valid = false;
        return select_variant(h);
    }
    if (d != h->cfg.dim && (uint64_t)d + (uint64_t)d * d == h->cfg.dim) {
        // the state is GsnTargetLaw's whole θ = [μ; vec Σ] (gsn_target.jl:1-13):
        // updates may write Σ entries, so the law refactorises Σ at every
        // evaluation — the shipped law csrc/laws/gsn_full.c, compiled at run time
        if (!t->mu || !t->sigma || !t->obs || t->num_obs == 0) return fail(h, EMCMC_INVALID_ARG, "null target arrays");
        if (t->ll_mode != EMCMC_LL_PER_OBS)
            return fail(h, EMCMC_UNSUPPORTED_PLUGIN, "GsnTargetLaw over [μ; vec Σ] evaluates per observation only");
        std::vector<double> th0(t->mu, t->mu + d);
        th0.insert(th0.end(), t->sigma, t->sigma + (size_t)d * d);
        const double prm = (double)d;
        emcmc_user_target_desc u{};
        u.dim = h->cfg.dim;
        u.obs_dim = d;
        u.theta0 = th0.data();
        u.num_obs = t->num_obs;
        u.obs = t->obs;
        u.num_params = 1;
        u.params = &prm;
        u.source = rtc_builtin_law("gsn_full.c");
        if (!u.source) return fail(h, EMCMC_HIP_ERROR, "the shipped GsnTargetLaw source is missing");
        return emcmc_set_user_target(h, &u);
    }
    if (d != h->cfg.dim)
        return fail(h, EMCMC_UNSUPPORTED_PLUGIN,
                    "device GsnTargetLaw needs state = μ or state = [μ; vec Σ] (d=%u, D=%u)", d, h->cfg.dim);
    if (!t->mu || !t->sigma || (t->num_obs && !t->obs)) return fail(h, EMCMC_INVALID_ARG, "null target arrays");
    if (t->num_obs == 0) return fail(h, EMCMC_INVALID_ARG, "GsnTargetLaw needs observations");
    if (t->ll_mode > EMCMC_LL_SUFFSTAT) return fail(h, EMCMC_INVALID_ARG, "ll_mode");
    TargetHost th;
    th.dim = d;
    th.ll_mode = t->ll_mode;
    th.nobs = t->num_obs;
    th.mu.assign(t->mu, t->mu + d);
    th.sigma.assign(t->sigma, t->sigma + (size_t)d * d);
    th.obs.assign(t->obs, t->obs + t->num_obs * d);
    if (!cholesky_upper_colmajor(th.sigma.data(), (int)d, th.L))
        return fail(h, EMCMC_INVALID_ARG, "GsnTargetLaw Σ is not positive definite");
    th.invdiag.resize(d);
    for (uint32_t i = 0; i < d; ++i) th.invdiag[i] = 1.0 / th.L[(size_t)i * d + i];
    th.diag = is_diag_upper(th.sigma.data(), (int)d);
    th.c0 = mvnormal_c0((int)d, logdet_chol(th.L, (int)d));
    // x̄ = (Σ_k x_k)/n and S_c = Σ_k ‖L⁻¹(x_k − x̄)‖² (canonical order, as oracle/)
    th.xbar.assign(d, 0.0);
    for (uint32_t i = 0; i < d; ++i) {
        double s = 0.0;
        for (uint64_t k = 0; k < th.nobs; ++k) s = s + th.obs[k * d + i];
        th.xbar[i] = s / (double)th.nobs;
    }
    double Sc = 0.0;
    std::vector<double> y(d);
    for (uint64_t k = 0; k < th.nobs; ++k) {
        for (uint32_t i = 0; i < d; ++i) {
            double acc = th.obs[k * d + i] - th.xbar[i];
            for (uint32_t j = 0; j < i; ++j) acc = std::fma(-th.L[(size_t)i * d + j], y[j], acc);
            y[i] = acc * th.invdiag[i];
        }
        Sc = Sc + canon_sumsq_host(y.data(), (int)d);
    }
    th.S_c = Sc;
    h->target = std::move(th);
    h->target_set = true;
    if (h->allocated) {  // P° = deepcopy(data.P): every chain's P° mean starts at μ
        emcmc_status st = reset_mu_p(h);
        if (st) return st;
    }
    return select_variant(h);
}

emcmc_status emcmc_set_user_target(emcmc_handle *h, const emcmc_user_target_desc *t) {
    if (!h || !t) return EMCMC_INVALID_ARG;
    if (!t->source) return fail(h, EMCMC_INVALID_ARG, "user target: null source");
    if (t->dim != h->cfg.dim)
        return fail(h, EMCMC_INVALID_ARG, "user target: dim %u != D %u (the law's θ is the chain state)", t->dim,
                    h->cfg.dim);
    if (t->dim > (uint32_t)kMwgMaxD)
        return fail(h, EMCMC_UNSUPPORTED_PLUGIN, "user target: D=%u > %d (general schedule kernel)", t->dim, kMwgMaxD);
    if ((t->num_obs && (!t->obs || t->obs_dim == 0)) || (t->num_params && !t->params))
        return fail(h, EMCMC_INVALID_ARG, "user target: null obs / params");
    if (t->num_obs > 0xFFFFFFFFull) return fail(h, EMCMC_INVALID_ARG, "user target: more than 2^32-1 observations");
    TargetHost th;
    th.kind = EMCMC_TARGET_USER;
    th.dim = t->dim;
    th.nobs = t->num_obs;
    th.obs_dim = t->obs_dim;
    th.mu.assign(t->dim, 0.0);
    if (t->theta0) th.mu.assign(t->theta0, t->theta0 + t->dim);
    if (t->num_obs) th.obs.assign(t->obs, t->obs + t->num_obs * t->obs_dim);
    if (t->num_params) th.params.assign(t->params, t->params + t->num_params);
    th.src = t->source;
    th.opts = t->options ? t->options : "";
    th.diag = true;
    h->target = std::move(th);
    h->target_set = true;
    if (h->allocated) {  // P° = deepcopy(data.P)
        emcmc_status st = reset_mu_p(h);
        if (st) return st;
    }
    if (h->updates.empty()) {  // compile now, so errors surface here; select_variant reuses the cache
        RtcKernel k;
        const std::string log = rtc_compile_user(h->target.src, h->target.opts, (int)t->dim,
                                                 h->cfg.history_mode == EMCMC_HIST_FULL, (int)t->dim, k);
        if (!log.empty()) {
            h->err = "user target does not compile:\n" + log;
            h->target_set = false;
            return EMCMC_INVALID_ARG;
        }
        return EMCMC_OK;
    }
    emcmc_status st = select_variant(h);
    if (st == EMCMC_INVALID_ARG) h->target_set = false;
    return st;
}

emcmc_status emcmc_check_user_target(const char *source, uint32_t dim, const char *options, char *log_out,
                                     size_t log_len) {
    if (!source) return EMCMC_INVALID_ARG;
    RtcKernel k;
    // a law with a gradient (EMCMC_USER_GRAD) is checked with MALA compiled in
    const bool mala = rtc_defines_user_grad(source);
    const std::string log = rtc_compile_user(source, options ? options : "", (int)dim, true, (int)dim, k,
                                             std::string(), std::string(), false, mala);
    if (log_out && log_len) {
        const size_t n = std::min(log.size(), log_len - 1);
        std::memcpy(log_out, log.data(), n);
        log_out[n] = '\0';
    }
    return log.empty() ? EMCMC_OK : EMCMC_INVALID_ARG;
}

emcmc_status emcmc_check_user_update(const char *source, uint32_t dim, const char *options, char *log_out,
                                     size_t log_len) {
    if (!source) return EMCMC_INVALID_ARG;
    RtcKernel k;
    const std::string log = rtc_compile_gsn((int)dim, true, 0, (int)dim, k, source, options ? options : "");
    if (log_out && log_len) {
        const size_t n = std::min(log.size(), log_len - 1);
        std::memcpy(log_out, log.data(), n);
        log_out[n] = '\0';
    }
    return log.empty() ? EMCMC_OK : EMCMC_INVALID_ARG;
}

namespace {
void copy_log(const std::string &log, char *log_out, size_t log_len) {
    if (log_out && log_len) {
        const size_t n = std::min(log.size(), log_len - 1);
        std::memcpy(log_out, log.data(), n);
        log_out[n] = '\0';
    }
}
}  // namespace

emcmc_status emcmc_prebuild_chol_kernel(uint32_t dim, uint32_t history_mode, uint32_t ll_mode, char *log_out,
                                        size_t log_len) {
    if (dim < 2 || dim > (uint32_t)kCholRtcMaxD || history_mode > 1 || ll_mode > 1) return EMCMC_INVALID_ARG;
    copy_log("", log_out, log_len);
    if (lookup((int)dim, 1, history_mode == EMCMC_HIST_FULL, (int)ll_mode, 2, false)) return EMCMC_OK;  // ahead of time
    RtcKernel k;
    const std::string log = rtc_compile_chol((int)dim, history_mode == EMCMC_HIST_FULL, (int)ll_mode, k);
    copy_log(log, log_out, log_len);
    return log.empty() ? EMCMC_OK : EMCMC_HIP_ERROR;
}

emcmc_status emcmc_prebuild_block_kernel(uint32_t dim, uint32_t history_mode, uint32_t ll_mode, int dense_target,
                                         const char *target_source, const char *target_options,
                                         const char *update_source, const char *update_options, char *log_out,
                                         size_t log_len) {
    if (dim < (uint32_t)kBlockMinD || dim > (uint32_t)kMwgMaxD || history_mode > 1 || ll_mode > 1)
        return EMCMC_INVALID_ARG;
    copy_log("", log_out, log_len);
    const bool full = history_mode == EMCMC_HIST_FULL, user = target_source && *target_source;
    const bool upd = update_source && *update_source;
    if (!user && !upd)
        for (const auto &e : block_table())
            if (e.D == (int)dim && e.tdense == (dense_target ? 1 : 0) && e.full == (int)full && e.ll == (int)ll_mode)
                return EMCMC_OK;  // ahead of time
    RtcKernel k;
    const std::string log =
        rtc_compile_block((int)dim, full, user ? 0 : (int)ll_mode, dense_target != 0, user ? target_source : "",
                          target_options ? target_options : "", upd ? update_source : "",
                          update_options ? update_options : "", k);
    copy_log(log, log_out, log_len);
    return log.empty() ? EMCMC_OK : (user || upd) ? EMCMC_INVALID_ARG : EMCMC_HIP_ERROR;
}

emcmc_status emcmc_prebuild_rw_block_kernel(uint32_t dim, uint32_t history_mode, uint32_t ll_mode, int dense_target,
                                            const emcmc_update_desc *updates, uint32_t num_updates,
                                            const char *target_source, const char *target_options, char *log_out,
                                            size_t log_len) {
    copy_log("", log_out, log_len);
    if (!updates || num_updates == 0 || dim < (uint32_t)kBlockMinD || dim > (uint32_t)kMwgMaxD || history_mode > 1 ||
        ll_mode > 1)
        return EMCMC_INVALID_ARG;
    emcmc_handle tmp;  // no device: build_update only reads cfg.dim and the updates already built
    tmp.cfg.dim = dim;
    for (uint32_t p = 0; p < num_updates; ++p) {
        UpdateHost uh;
        if (emcmc_status st = build_update(&tmp, updates + p, uh)) {
            copy_log(tmp.err, log_out, log_len);
            return st;
        }
        tmp.updates.push_back(std::move(uh));
    }
    if (!rwblock_eligible(tmp.updates, dim)) {
        copy_log("not a mwg_rw_block_kernel schedule: 1..8 UniformRandomWalk / GaussianRandomWalk updates "
                 "(AdaptationUnifRW on a UniformRandomWalk only, at most 32 positivity flags on a "
                 "GaussianRandomWalk) at 17 <= dim <= 64",
                 log_out, log_len);
        return EMCMC_INVALID_ARG;
    }
    const bool user = target_source && *target_source;
    std::string label, sname;
    const std::string shape = rw_sched_source(tmp.updates, label, sname);
    RtcKernel k;
    const std::string log = rtc_compile_rwblock((int)dim, history_mode == EMCMC_HIST_FULL, user ? 0 : (int)ll_mode,
                                                dense_target != 0, shape, sname, label, user ? target_source : "",
                                                target_options ? target_options : "", k);
    copy_log(log, log_out, log_len);
    return log.empty() ? EMCMC_OK : user ? EMCMC_INVALID_ARG : EMCMC_HIP_ERROR;
}

emcmc_status emcmc_prebuild_fused_prior_kernel(uint32_t dim, uint32_t lanes_per_chain, uint32_t history_mode,
                                               uint32_t ll_mode, int unit_target, const emcmc_update_desc *update,
                                               char *log_out, size_t log_len) {
    copy_log("", log_out, log_len);
    if (!update || dim == 0 || dim > (uint32_t)kMwgMaxD || history_mode > 1 || ll_mode > 1) return EMCMC_INVALID_ARG;
    emcmc_handle tmp;  // no device: the update, the target's kind and diagonal flag are all selection reads
    tmp.cfg.dim = dim;
    tmp.cfg.lanes_per_chain = lanes_per_chain;
    tmp.target.kind = EMCMC_TARGET_GSN;
    tmp.target.diag = true;
    UpdateHost uh;
    if (emcmc_status st = build_update(&tmp, update, uh)) {
        copy_log(tmp.err, log_out, log_len);
        return st;
    }
    tmp.updates.push_back(std::move(uh));
    if (!fused_prior_eligible(&tmp)) {
        copy_log("not a fused-prior shape: one diagonal GaussianRandomWalk or UniformRandomWalk "
                 "over coords 0..dim-1 without adaptation, with ImproperPosPrior or a ProductPrior / StandardPrior "
                 "that is one Product of dim univariates or one MvNormal over all dim coordinates (ImproperPrior too "
                 "with positivity flags or a UniformRandomWalk), families and positivity flags repeating across the chain's lanes, dim/lanes = "
                 "8·2^k with more than one lane per chain",
                 log_out, log_len);
        return EMCMC_INVALID_ARG;
    }
    std::string label, sname;
    const std::string shape = rw_sched_source(tmp.updates, label, sname);
    RtcKernel k;
    const bool uni = tmp.updates[0].kernel == EMCMC_RW_UNIFORM;
    for (int w : {2, 1}) {  // both occupancies select_fused_prior may try
        const std::string log = rtc_compile_fused_prior((int)dim, fused_lpc(&tmp), w, history_mode == EMCMC_HIST_FULL,
                                                        (int)ll_mode, unit_target != 0, shape, sname,
                                                        uni ? label : label.substr(label.find(',') + 1), k);
        if (!log.empty()) {
            copy_log(log, log_out, log_len);
            return EMCMC_HIP_ERROR;
        }
    }
    return EMCMC_OK;
}

emcmc_status emcmc_set_state(emcmc_handle *h, const double *theta, const double *ll) {
    if (!h || !theta) return EMCMC_INVALID_ARG;
    emcmc_status st = ensure_alloc(h);
    if (st) return st;
    const uint64_t C = h->cfg.num_chains, D = h->cfg.dim;
    // host row-major [C][D] → device state_pos layout
    std::vector<double> soa(C * D);
    for (uint64_t c = 0; c < C; ++c)
        for (uint64_t d = 0; d < D; ++d) soa[state_pos(d, c, C, (uint32_t)D)] = theta[c * D + d];
    HIPCHK(h, hipMemcpyAsync(h->d_theta, soa.data(), C * D * sizeof(double), hipMemcpyHostToDevice, h->stream));
    h->theta_live = nullptr;
    std::vector<double> l(C, -INFINITY);
    if (ll) std::copy(ll, ll + C, l.begin());
    HIPCHK(h, hipMemcpyAsync(h->d_ll, l.data(), C * sizeof(double), hipMemcpyHostToDevice, h->stream));
    const uint64_t P = h->updates.size();
    HIPCHK(h, hipMemsetAsync(h->d_ra, 0, P * C * sizeof(double), h->stream));
    HIPCHK(h, hipMemsetAsync(h->d_ring, 0, 2 * P * C * sizeof(uint64_t), h->stream));
    HIPCHK(h, hipMemsetAsync(h->d_nacc, 0, P * C * sizeof(uint32_t), h->stream));
    HIPCHK(h, hipMemsetAsync(h->d_faults, 0, C * sizeof(uint32_t), h->stream));
    HIPCHK(h, hipMemsetAsync(h->d_aprop, 0, P * C * sizeof(uint32_t), h->stream));
    HIPCHK(h, hipMemsetAsync(h->d_aacc, 0, P * C * sizeof(uint32_t), h->stream));
    HIPCHK(h, hipMemsetAsync(h->d_ll_prop, 0xFF, P * C * sizeof(double), h->stream));  // NaN until an update runs
    {  // per-chain ϵ of every update starts at the update's ϵ
        std::vector<double> e(P * kMwgMaxD * C, 0.0);
        for (uint64_t q = 0; q < P; ++q)
            for (size_t j = 0; j < h->updates[q].eps.size(); ++j)
                std::fill_n(e.begin() + (q * kMwgMaxD + j) * C, C, h->updates[q].eps[j]);
        HIPCHK(h, hipMemcpyAsync(h->d_eps, e.data(), e.size() * sizeof(double), hipMemcpyHostToDevice, h->stream));
        if (h->target_set) {
            st = reset_mu_p(h);
            if (st) return st;
        }
        HIPCHK(h, hipStreamSynchronize(h->stream));  // host vectors go out of scope
        *static_cast<volatile uint32_t *>(h->h_fault_flag) = 0u;  // fault words were cleared above
    }
    if (h->d_mean) {  // GenericChainStats: mean = 0, cov = 0, N = 1 (chain_statistics.jl:30-35)
        const uint64_t DP = (uint64_t)packed_n((int)D);
        HIPCHK(h, hipMemsetAsync(h->d_mean, 0, C * D * sizeof(double), h->stream));
        HIPCHK(h, hipMemsetAsync(h->d_cov, 0, C * DP * sizeof(double), h->stream));
        if (h->d_LB) {  // every chain starts from the user's Σ_B
            const UpdateHost &u = h->updates[0];
            std::vector<double> lb(C * DP), il(C * D), c0(C, u.c0B);
            for (uint64_t c = 0; c < C; ++c) {
                for (int i = 0; i < (int)D; ++i)
                    for (int j = 0; j <= i; ++j)
                        lb[state_pos((uint64_t)lo_idx(i, j), c, C, (uint32_t)DP)] = u.LB[(size_t)i * D + j];
                for (uint64_t i = 0; i < D; ++i) il[i * C + c] = u.invdiagB[i];
            }
            HIPCHK(h, hipMemcpy(h->d_LB, lb.data(), lb.size() * sizeof(double), hipMemcpyHostToDevice));
            HIPCHK(h, hipMemcpy(h->d_iLB, il.data(), il.size() * sizeof(double), hipMemcpyHostToDevice));
            HIPCHK(h, hipMemcpy(h->d_c0B, c0.data(), c0.size() * sizeof(double), hipMemcpyHostToDevice));
        }
        HIPCHK(h, hipStreamSynchronize(h->stream));
    }
    h->mix_M = 0;
    h->grad_valid = false;
    h->hi_iter = 0;
    h->stats_N = 1;
    h->last_iter.assign(P, 0u);
    for (auto &u : h->updates) u.lam = u.lam0;  // rw.λ as constructed (fλ adapts it during a run)
    if (h->var.mfn || h->var.ufn) {
        if ((st = reset_mwg_pool(h))) return st;
        if (h->nhaario) {  // the table's λ back to its constructed value
            for (size_t q = 0; q < h->updates.size(); ++q)
                if (h->updates[q].kernel == EMCMC_RW_GAUSSIAN_MIX)
                    HIPCHK(h, hipMemcpy(reinterpret_cast<char *>(h->d_mwg + q) + offsetof(MwgUpdate, lam),
                                        &h->updates[q].lam, sizeof(double), hipMemcpyHostToDevice));
        }
    }
    return EMCMC_OK;
}

namespace {
emcmc_status run_impl(emcmc_handle *h, const emcmc_step *steps, uint64_t num_steps);
double host_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

emcmc_status emcmc_run(emcmc_handle *h, const emcmc_step *steps, uint64_t num_steps) {
    if (!h || !h->host_timing) return run_impl(h, steps, num_steps);
    const double t0 = host_us();
    const emcmc_status st = run_impl(h, steps, num_steps);
    h->ht_run_us += host_us() - t0;
    ++h->ht_runs;
    return st;
}

namespace {
emcmc_status run_impl(emcmc_handle *h, const emcmc_step *steps, uint64_t num_steps) {
    if (!h || (!steps && num_steps)) return EMCMC_INVALID_ARG;
    if (!h->allocated) return fail(h, EMCMC_STATE_ERROR, "emcmc_set_state must precede emcmc_run");
    if (!h->target_set) return fail(h, EMCMC_STATE_ERROR, "emcmc_set_target must precede emcmc_run");
    if (!h->var.fn && !h->var.ffn && !h->var.mfn && !h->var.ufn && !h->var.xfn && !h->var.afn)
        return fail(h, EMCMC_UNSUPPORTED_PLUGIN, "no kernel variant selected");
    if (!h->d_zig) return fail(h, EMCMC_STATE_ERROR, "state not allocated");
    const uint32_t P = (uint32_t)h->updates.size();
    for (uint64_t i = 0; i < num_steps; ++i) {
        if (steps[i].pidx < 1 || steps[i].pidx > P) return fail(h, EMCMC_INVALID_ARG, "step %llu: pidx", (unsigned long long)i);
        if (steps[i].mcmciter < 1 || steps[i].mcmciter > h->cfg.num_mcmc_steps)
            return fail(h, EMCMC_INVALID_ARG, "step %llu: mcmciter %u outside 1..M", (unsigned long long)i,
                        steps[i].mcmciter);
    }
    const bool live = theta_in_hist(h);
    if (!live)
        if (emcmc_status s = settle_theta(h)) return s;
    if (h->var.mfn || h->var.ufn) return run_mwg(h, steps, num_steps);
    if (h->var.xfn) return run_mix(h, steps, num_steps);
    if (h->var.afn) return run_mala(h, steps, num_steps);
    const uint64_t C = h->cfg.num_chains;
    const int lpc = h->var.lpc;
    const uint64_t threads = C * (uint64_t)lpc;
    const unsigned bs = h->var.dense ? 256u : (unsigned)diag_block(h->var.occ);
    const dim3 block(bs), grid((unsigned)((threads + bs - 1) / bs));
    const TargetHost &t = h->target;
    StepParams p{};
    p.theta = h->d_theta;
    p.ll = h->d_ll;
    p.ra = h->d_ra;
    p.ring = h->d_ring;
    p.nacc = h->d_nacc;
    p.faults = h->d_faults;
    p.fault_flag = h->d_fault_flag;
    p.ll_prop = h->d_ll_prop;
    p.hist_theta = h->d_hist_theta;
    p.hist_prop = h->d_hist_prop;
    p.hist_ll = h->d_hist_ll;
    p.hist_acc = h->d_hist_acc;
    p.zig = h->d_zig;
    p.consts = h->d_consts;
    p.obs = h->d_obs;
    p.C = C;
    p.row_bytes = h->row_bytes;
    p.chain0 = (uint32_t)h->cfg.first_chain_id;
    p.key0 = (uint32_t)h->cfg.seed;
    p.key1 = (uint32_t)(h->cfg.seed >> 32);
    p.P = P;
    p.W = h->cfg.roll_window;
    p.nobs = (uint32_t)t.nobs;
    p.rw_c0 = h->updates[0].c0;
    p.t_c0 = t.c0;
    p.n_tc0 = (double)t.nobs * t.c0;
    p.S_c = t.S_c;
    p.nobs_d = (double)t.nobs;
    p.rcp_W = 1.0 / (double)h->cfg.roll_window;
    p.xcd = (h->cfg.kernel_variant & EMCMC_VARIANT_NO_XCD_ORDER) ? 0u : 1u;
    const uint64_t K = h->cfg.steps_per_launch;
    uint64_t i = 0;
    while (i < num_steps) {
        // maximal run of ≤ K consecutive iterations of the same update
        uint64_t j = i + 1;
        while (j < num_steps && j - i < K && steps[j].pidx == steps[i].pidx &&
               steps[j].mcmciter == steps[j - 1].mcmciter + 1 &&
               ring_epoch(h, steps[j].mcmciter) == ring_epoch(h, steps[i].mcmciter))
            ++j;
        const uint64_t n = j - i;
        {
            const HistPtrs hp = shifted_hist(h, steps[i].mcmciter);
            p.hist_theta = hp.theta;
            p.hist_prop = hp.prop;
            p.hist_ll = hp.ll;
            p.hist_acc = hp.acc;
            emcmc_status gs = guard_ring(h, steps[i].mcmciter, steps[j - 1].mcmciter);
            if (gs) return gs;
        }
        p.pidx0 = steps[i].pidx - 1;
        p.iter0 = steps[i].mcmciter;
        p.nsteps = (uint32_t)n;
        p.N0 = h->stats_N;
        // rolling_ar[iter−1][p] of an iteration that did not run is 0.0
        // (chain_statistics.jl:57 reads a never-written slot)
        if (p.iter0 > 1 && h->last_iter[p.pidx0] != p.iter0 - 1)
            HIPCHK(h, hipMemsetAsync(h->d_ra, 0, C * sizeof(double), h->stream));
        h->last_iter[p.pidx0] = steps[j - 1].mcmciter;
        if (live) {  // θ from the previous launch's last history slot, left in this launch's
            p.theta_in = h->theta_live ? h->theta_live : h->d_theta;
            p.theta = nullptr;
        } else {
            p.theta_in = nullptr;
            p.theta = h->d_theta;
        }
        void *args[] = {&p};
        if (h->var.ffn)
            HIPCHK(h, launch_module(h, h->var.ffn, grid, block, args, h->lds_bytes, bytes_per_launch(h, n, false)));
        else
            HIPCHK(h, launch_step(h, reinterpret_cast<const void *>(h->var.fn), grid, block, args, h->lds_bytes,
                                  bytes_per_launch(h, n, false)));
        if (live)  // slot (iter − 1)·P + pidx0 of the launch's last iteration, as the kernel addressed it
            h->theta_live = p.hist_theta + ((uint64_t)(p.iter0 + n - 2) * P + p.pidx0) * C * (uint64_t)h->cfg.dim;
        h->stats_N += n;
        i = j;
    }
    return EMCMC_OK;
}
}  // namespace

emcmc_status emcmc_synchronize(emcmc_handle *h) {
    if (!h) return EMCMC_INVALID_ARG;
    const double t0 = h->host_timing ? host_us() : 0.0;
    if (h->sync_mode == 0) {
        HIPCHK(h, hipStreamSynchronize(h->stream));
    } else {
        HIPCHK(h, hipEventRecord(h->sync_ev, h->stream));
        HIPCHK(h, hipEventSynchronize(h->sync_ev));
    }
    if (h->host_timing) {
        h->ht_sync_us += host_us() - t0;
        ++h->ht_syncs;
    }
    h->steps_staging.clear();
    h->lam_staging.clear();
    if (!h->allocated) return EMCMC_OK;
    // O(1): the kernels set the mapped flag when a chain ends a launch with a fault bit
    if (*static_cast<volatile uint32_t *>(h->h_fault_flag))
        return fail(h, EMCMC_CHAIN_FAULT, "at least one chain raised a fault (emcmc_get_faults)");
    return EMCMC_OK;
}

void emcmc_destroy(emcmc_handle *h) {
    if (!h) return;
    (void)hipSetDevice(h->cfg.device);
    if (h->host_timing)
        fprintf(stderr, "[emcmc host] emcmc_run %.2f us x %llu, emcmc_synchronize %.2f us x %llu (sync mode %d)\n",
                h->ht_runs ? h->ht_run_us / h->ht_runs : 0.0, (unsigned long long)h->ht_runs,
                h->ht_syncs ? h->ht_sync_us / h->ht_syncs : 0.0, (unsigned long long)h->ht_syncs, h->sync_mode);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->cstream) (void)hipStreamSynchronize(h->cstream);
    if (h->sync_ev) (void)hipEventDestroy(h->sync_ev);
    for (auto &c : h->copies) (void)hipEventDestroy(c.ev);
    if (h->d_stage) (void)hipFree(h->d_stage);
    if (h->cstream) (void)hipStreamDestroy(h->cstream);
    for (auto &p : h->ev) {
        (void)hipEventDestroy(p.first);
        (void)hipEventDestroy(p.second);
    }
    for (auto e : h->ev_pool) (void)hipEventDestroy(e);
    void *bufs[] = {h->d_theta,     h->d_ll,        h->d_ra,      h->d_ring,     h->d_nacc,  h->d_faults,
                    h->d_hist_theta, h->d_hist_prop, h->d_hist_ll, h->d_hist_acc, h->d_consts, h->d_obs,
                    h->d_scratch,   h->d_gather,    h->d_zig,     h->d_mu_p,     h->d_eps,   h->d_tL,
                    h->d_tiL,       h->d_xbar,      h->d_aprop,   h->d_aacc,     h->d_steps, h->d_mwg,
                    h->d_mean,      h->d_cov,       h->d_LB,      h->d_iLB,      h->d_c0B,   h->d_Lnew,
                    h->d_grad,      h->d_X,         h->d_y,       h->d_mom_scratch, h->d_mean_alt, h->d_mom_consts,
                    h->d_ll_prop,   h->d_uparams,   h->d_gcache,  h->d_bconsts};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    // h->umod belongs to the process-wide module table (load_rtc_module)
    if (h->h_fault_flag) (void)hipHostFree(h->h_fault_flag);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

const char *emcmc_last_error(const emcmc_handle *h) { return h ? h->err.c_str() : "null handle"; }

emcmc_status emcmc_get_state(emcmc_handle *h, double *theta, double *ll) {
    if (!h) return EMCMC_INVALID_ARG;
    if (!h->allocated) return fail(h, EMCMC_STATE_ERROR, "no state");
    if (emcmc_status s = settle_theta(h)) return s;
    HIPCHK(h, hipStreamSynchronize(h->stream));
    const uint64_t C = h->cfg.num_chains, D = h->cfg.dim;
    if (theta) {  // device state_pos layout → host [C][D]
        std::vector<double> soa(C * D);
        HIPCHK(h, hipMemcpy(soa.data(), h->d_theta, C * D * sizeof(double), hipMemcpyDeviceToHost));
        for (uint64_t c = 0; c < C; ++c)
            for (uint64_t d = 0; d < D; ++d) theta[c * D + d] = soa[state_pos(d, c, C, (uint32_t)D)];
    }
    if (ll) HIPCHK(h, hipMemcpy(ll, h->d_ll, C * sizeof(double), hipMemcpyDeviceToHost));
    return EMCMC_OK;
}

emcmc_status emcmc_get_chain_stats(emcmc_handle *h, double *rolling_ar, uint64_t *accepted) {
    if (!h) return EMCMC_INVALID_ARG;
    if (!h->allocated) return fail(h, EMCMC_STATE_ERROR, "no state");
    HIPCHK(h, hipStreamSynchronize(h->stream));
    const uint64_t PC = h->cfg.num_chains * h->updates.size();
    if (rolling_ar) HIPCHK(h, hipMemcpy(rolling_ar, h->d_ra, PC * sizeof(double), hipMemcpyDeviceToHost));
    if (accepted) {
        std::vector<uint32_t> a(PC);
        HIPCHK(h, hipMemcpy(a.data(), h->d_nacc, PC * sizeof(uint32_t), hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < PC; ++i) accepted[i] = a[i];
    }
    return EMCMC_OK;
}

emcmc_status emcmc_get_update_state(emcmc_handle *h, uint32_t pidx, double *epsilon, uint32_t *proposed,
                                    uint32_t *accepted) {
    if (!h) return EMCMC_INVALID_ARG;
    if (!h->allocated) return fail(h, EMCMC_STATE_ERROR, "no state");
    if (pidx < 1 || pidx > h->updates.size()) return fail(h, EMCMC_INVALID_ARG, "pidx %u", pidx);
    HIPCHK(h, hipStreamSynchronize(h->stream));
    const uint64_t C = h->cfg.num_chains, q = pidx - 1;
    const UpdateHost &u = h->updates[q];
    if (epsilon) {
        const size_t nc = u.coords.size();
        if (u.kernel != EMCMC_RW_UNIFORM) return fail(h, EMCMC_INVALID_ARG, "update %u has no ϵ", pidx);
        std::vector<double> e(nc * C);
        HIPCHK(h, hipMemcpy(e.data(), h->d_eps + q * kMwgMaxD * C, e.size() * sizeof(double), hipMemcpyDeviceToHost));
        for (uint64_t c = 0; c < C; ++c)
            for (size_t j = 0; j < nc; ++j) epsilon[c * nc + j] = e[j * C + c];
    }
    if (proposed) HIPCHK(h, hipMemcpy(proposed, h->d_aprop + q * C, C * sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (accepted) HIPCHK(h, hipMemcpy(accepted, h->d_aacc + q * C, C * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return EMCMC_OK;
}

namespace {
// [n][C] mean and packed lower [n(n+1)/2][C] cov (general kernel) → [C][n], [C][n][n]
emcmc_status copy_soa_moments(emcmc_handle *h, const double *dmean, const double *dcov, uint64_t n, double *mean,
                              double *cov) {
    const uint64_t C = h->cfg.num_chains, tn = n * (n + 1) / 2;
    if (mean) {
        std::vector<double> m(n * C);
        HIPCHK(h, hipMemcpy(m.data(), dmean, m.size() * sizeof(double), hipMemcpyDeviceToHost));
        for (uint64_t c = 0; c < C; ++c)
            for (uint64_t i = 0; i < n; ++i) mean[c * n + i] = m[i * C + c];
    }
    if (cov) {
        std::vector<double> v(tn * C);
        HIPCHK(h, hipMemcpy(v.data(), dcov, v.size() * sizeof(double), hipMemcpyDeviceToHost));
        for (uint64_t c = 0; c < C; ++c)
            for (uint64_t i = 0; i < n; ++i)
                for (uint64_t j = 0; j <= i; ++j) {
                    const double x = v[(i * (i + 1) / 2 + j) * C + c];
                    cov[(c * n + i) * n + j] = x;
                    cov[(c * n + j) * n + i] = x;
                }
    }
    return EMCMC_OK;
}
bool general_path(const emcmc_handle *h) { return h->var.mfn || h->var.ufn; }
}  // namespace

emcmc_status emcmc_get_adaptation_moments(emcmc_handle *h, uint32_t pidx, double *mean, double *cov) {
    if (!h) return EMCMC_INVALID_ARG;
    if (!h->allocated) return fail(h, EMCMC_STATE_ERROR, "no state");
    if (pidx < 1 || pidx > h->updates.size()) return fail(h, EMCMC_INVALID_ARG, "pidx %u", pidx);
    const UpdateHost &u = h->updates[pidx - 1];
    if (u.kernel != EMCMC_RW_GAUSSIAN_MIX || u.adaptation != EMCMC_ADPT_HAARIO)
        return fail(h, EMCMC_INVALID_ARG, "update %u has no HaarioTypeAdaptation", pidx);
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (general_path(h))
        return copy_soa_moments(h, h->d_mixpool + u.hm_off, h->d_mixpool + u.hc_off, u.coords.size(), mean, cov);
    return emcmc_get_chain_moments(h, mean, cov);  // the fused path (P = 1): the same recurrence on the same θ
}

emcmc_status emcmc_get_chain_moments(emcmc_handle *h, double *mean, double *cov) {
    if (!h) return EMCMC_INVALID_ARG;
    if (!h->allocated) return fail(h, EMCMC_STATE_ERROR, "no state");
    if (general_path(h)) {
        if (!h->cfg.chain_moments || !h->d_smean)
            return fail(h, EMCMC_STATE_ERROR, "chain moments are kept on device with emcmc_config.chain_moments");
        HIPCHK(h, hipStreamSynchronize(h->stream));
        return copy_soa_moments(h, h->d_smean, h->d_scov, h->cfg.dim, mean, cov);
    }
    if (!h->d_mean)
        return fail(h, EMCMC_STATE_ERROR,
                    "chain moments are kept on device only with GaussianRandomWalkMix or emcmc_config.chain_moments");
    HIPCHK(h, hipStreamSynchronize(h->stream));
    const uint64_t C = h->cfg.num_chains, D = h->cfg.dim, DP = (uint64_t)packed_n((int)D);
    if (mean) {
        std::vector<double> m(C * D);
        HIPCHK(h, hipMemcpy(m.data(), h->d_mean, m.size() * sizeof(double), hipMemcpyDeviceToHost));
        for (uint64_t c = 0; c < C; ++c)
            for (uint64_t d = 0; d < D; ++d) mean[c * D + d] = m[state_pos(d, c, C, (uint32_t)D)];
    }
    if (cov) {
        std::vector<double> v(C * DP);
        HIPCHK(h, hipMemcpy(v.data(), h->d_cov, v.size() * sizeof(double), hipMemcpyDeviceToHost));
        for (uint64_t c = 0; c < C; ++c)
            for (int i = 0; i < (int)D; ++i)
                for (int j = i; j < (int)D; ++j) {
                    const double x = v[state_pos((uint64_t)up_idx((int)D, i, j), c, C, (uint32_t)DP)];
                    cov[(c * D + i) * D + j] = x;
                    cov[(c * D + j) * D + i] = x;
                }
    }
    return EMCMC_OK;
}

emcmc_status emcmc_get_mix_state(emcmc_handle *h, uint32_t pidx, double *chol_sigma_b, uint32_t *steps_since_adapt) {
    if (!h) return EMCMC_INVALID_ARG;
    if (!h->allocated) return fail(h, EMCMC_STATE_ERROR, "no state");
    if (pidx < 1 || pidx > h->updates.size()) return fail(h, EMCMC_INVALID_ARG, "pidx %u", pidx);
    if (h->updates[pidx - 1].kernel != EMCMC_RW_GAUSSIAN_MIX)
        return fail(h, EMCMC_INVALID_ARG, "update %u is not a GaussianRandomWalkMix", pidx);
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (general_path(h)) {  // the chain's L_B in the pool, packed lower [n(n+1)/2][C]
        const UpdateHost &u = h->updates[pidx - 1];
        const uint64_t C = h->cfg.num_chains, n = u.coords.size(), tn = n * (n + 1) / 2;
        if (chol_sigma_b) {
            std::vector<double> v(tn * C);
            HIPCHK(h, hipMemcpy(v.data(), h->d_mixpool + u.lb_off, v.size() * sizeof(double), hipMemcpyDeviceToHost));
            for (uint64_t c = 0; c < C; ++c)
                for (uint64_t i = 0; i < n; ++i)
                    for (uint64_t j = 0; j < n; ++j)
                        chol_sigma_b[(c * n + i) * n + j] = (j <= i) ? v[(i * (i + 1) / 2 + j) * C + c] : 0.0;
        }
        if (steps_since_adapt) *steps_since_adapt = h->mwg_M.empty() ? 0u : h->mwg_M[pidx - 1];
        return EMCMC_OK;
    }
    if (!h->d_LB) return fail(h, EMCMC_STATE_ERROR, "no mix state");
    const uint64_t C = h->cfg.num_chains, D = h->cfg.dim, DP = (uint64_t)packed_n((int)D);
    if (chol_sigma_b) {
        std::vector<double> v(C * DP);
        HIPCHK(h, hipMemcpy(v.data(), h->d_LB, v.size() * sizeof(double), hipMemcpyDeviceToHost));
        for (uint64_t c = 0; c < C; ++c)
            for (int i = 0; i < (int)D; ++i)
                for (int j = 0; j < (int)D; ++j)
                    chol_sigma_b[(c * D + i) * D + j] =
                        (j <= i) ? v[state_pos((uint64_t)lo_idx(i, j), c, C, (uint32_t)DP)] : 0.0;
    }
    if (steps_since_adapt) *steps_since_adapt = h->mix_M;
    return EMCMC_OK;
}

emcmc_status emcmc_set_mix_lambda_fn(emcmc_handle *h, uint32_t pidx, emcmc_lambda_fn f, void *ctx) {
    if (!h || pidx < 1 || pidx > h->updates.size()) return EMCMC_INVALID_ARG;
    UpdateHost &u = h->updates[pidx - 1];
    if (u.kernel != EMCMC_RW_GAUSSIAN_MIX || u.adaptation != EMCMC_ADPT_HAARIO)
        return fail(h, EMCMC_INVALID_ARG, "fλ belongs to a GaussianRandomWalkMix update with HaarioTypeAdaptation");
    u.flam = f;
    u.flam_ctx = ctx;
    return EMCMC_OK;
}

emcmc_status emcmc_get_mix_lambda(emcmc_handle *h, uint32_t pidx, double *lambda) {
    if (!h || !lambda || pidx < 1 || pidx > h->updates.size()) return EMCMC_INVALID_ARG;
    if (h->updates[pidx - 1].kernel != EMCMC_RW_GAUSSIAN_MIX) return fail(h, EMCMC_INVALID_ARG, "not a mix update");
    *lambda = h->updates[pidx - 1].lam;
    return EMCMC_OK;
}

emcmc_status emcmc_get_faults(emcmc_handle *h, uint32_t *faults) {
    if (!h || !faults) return EMCMC_INVALID_ARG;
    if (!h->allocated) return fail(h, EMCMC_STATE_ERROR, "no state");
    HIPCHK(h, hipStreamSynchronize(h->stream));
    HIPCHK(h, hipMemcpy(faults, h->d_faults, h->cfg.num_chains * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return EMCMC_OK;
}

emcmc_status emcmc_get_proposal_ll(emcmc_handle *h, double *ll_prop) {
    if (!h || !ll_prop) return EMCMC_INVALID_ARG;
    if (!h->allocated) return fail(h, EMCMC_STATE_ERROR, "no state");
    HIPCHK(h, hipStreamSynchronize(h->stream));
    HIPCHK(h, hipMemcpy(ll_prop, h->d_ll_prop, h->updates.size() * h->cfg.num_chains * sizeof(double),
                        hipMemcpyDeviceToHost));
    return EMCMC_OK;
}

static emcmc_status hist_geometry(emcmc_handle *h, uint32_t which, void **base, size_t *row) {
    const uint64_t C = h->cfg.num_chains, D = h->cfg.dim, P = h->updates.size();
    switch (which) {
    case EMCMC_H_STATE: *base = h->d_hist_theta; *row = P * C * D * sizeof(double); break;
    case EMCMC_H_PROPOSAL: *base = h->d_hist_prop; *row = P * C * D * sizeof(double); break;
    case EMCMC_H_LL: *base = h->d_hist_ll; *row = P * C * sizeof(double); break;
    case EMCMC_H_ACCEPT: *base = h->d_hist_acc; *row = P * h->row_bytes; break;
    default: return fail(h, EMCMC_INVALID_ARG, "unknown history %u", which);
    }
    if (!*base) return fail(h, EMCMC_STATE_ERROR, "history %u not retained in this history_mode", which);
    return EMCMC_OK;
}

// STATE/PROPOSAL slots [slot0, slot0+nslots) for chains [c0, c0+nc): device
// state_pos layout → host [slot][nc][D], staged through a bounded scratch.
static emcmc_status copy_state_slots(emcmc_handle *h, const double *base, uint64_t slot0, uint64_t nslots,
                                     uint64_t c0, uint64_t nc, double *host_out) {
    const uint64_t C = h->cfg.num_chains, D = h->cfg.dim;
    const uint64_t per_slot = nc * D;
    const uint64_t cap_elems = std::max<uint64_t>(per_slot, (256ull << 20) / sizeof(double));
    const uint64_t slots_per_chunk = std::max<uint64_t>(1, cap_elems / per_slot);
    const uint64_t need = std::min(nslots, slots_per_chunk) * per_slot * sizeof(double);
    if (h->gather_bytes < need) {
        HIPCHK(h, hipStreamSynchronize(h->stream));
        if (h->d_gather) (void)hipFree(h->d_gather);
        HIPCHK(h, hipMalloc(&h->d_gather, need));
        h->gather_bytes = need;
    }
    for (uint64_t s0 = 0; s0 < nslots; s0 += slots_per_chunk) {
        const uint64_t ns = std::min(slots_per_chunk, nslots - s0);
        const uint64_t n = ns * per_slot;
        hipLaunchKernelGGL(gather_hist_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, h->stream, base, C,
                           (uint32_t)D, slot0 + s0, ns, c0, nc, h->d_gather);
        HIPCHK(h, hipGetLastError());
        HIPCHK(h, hipMemcpyAsync(host_out + s0 * per_slot, h->d_gather, n * sizeof(double), hipMemcpyDeviceToHost,
                                 h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
    }
    return EMCMC_OK;
}

// Iterations [i0, i0+n) are on device: inside 1..M and, with a ring, not yet
// overwritten (the last R iterations launched).
static emcmc_status check_resident(emcmc_handle *h, uint64_t i0, uint64_t n) {
    if (i0 < 1 || n == 0 || i0 + n - 1 > h->cfg.num_mcmc_steps)
        return fail(h, EMCMC_INVALID_ARG, "iteration window outside 1..M");
    if (h->ring < h->cfg.num_mcmc_steps && h->hi_iter > h->ring && i0 <= h->hi_iter - h->ring)
        return fail(h, EMCMC_STATE_ERROR,
                    "iteration %llu was overwritten: the history ring keeps iterations %llu..%llu",
                    (unsigned long long)i0, (unsigned long long)(h->hi_iter - h->ring + 1),
                    (unsigned long long)h->hi_iter);
    return EMCMC_OK;
}

// Calls fn(ring_iter0, count, done) over the runs of [i0, i0+n) that are
// contiguous in the ring (split where the ring wraps).
extern "C++" {
template <typename F>
static emcmc_status for_each_ring_run(const emcmc_handle *h, uint64_t i0, uint64_t n, F fn) {
    for (uint64_t done = 0; done < n;) {
        const uint64_t r = (i0 + done - 1) % h->ring;
        const uint64_t len = std::min(n - done, h->ring - r);
        emcmc_status st = fn(r, len, done);
        if (st) return st;
        done += len;
    }
    return EMCMC_OK;
}
}  // extern "C++"

emcmc_status emcmc_get_history(emcmc_handle *h, uint32_t which, uint64_t iter_first, uint64_t num_iters,
                               void *host_out, size_t host_bytes) {
    if (!h || !host_out) return EMCMC_INVALID_ARG;
    if (!h->allocated) return fail(h, EMCMC_STATE_ERROR, "no state");
    emcmc_status st = check_resident(h, iter_first, num_iters);
    if (st) return st;
    void *base = nullptr;
    size_t row = 0;
    st = hist_geometry(h, which, &base, &row);
    if (st) return st;
    if (host_bytes < row * num_iters) return fail(h, EMCMC_INVALID_ARG, "host buffer too small");
    HIPCHK(h, hipStreamSynchronize(h->stream));
    const uint64_t P = h->updates.size();
    return for_each_ring_run(h, iter_first, num_iters, [&](uint64_t r, uint64_t len, uint64_t done) {
        if (which == EMCMC_H_STATE || which == EMCMC_H_PROPOSAL)
            return copy_state_slots(h, (const double *)base, r * P, len * P, 0, h->cfg.num_chains,
                                    (double *)((uint8_t *)host_out + done * row));
        HIPCHK(h, hipMemcpy((uint8_t *)host_out + done * row, (const uint8_t *)base + r * row, row * len,
                            hipMemcpyDeviceToHost));
        return EMCMC_OK;
    });
}

emcmc_status emcmc_get_history_chains(emcmc_handle *h, uint32_t which, uint64_t iter_first, uint64_t num_iters,
                                      uint64_t chain_first, uint64_t num_chains, void *host_out, size_t host_bytes) {
    if (!h || !host_out) return EMCMC_INVALID_ARG;
    if (!h->allocated) return fail(h, EMCMC_STATE_ERROR, "no state");
    if (which == EMCMC_H_ACCEPT) return fail(h, EMCMC_INVALID_ARG, "accept bits: use emcmc_get_history");
    emcmc_status st = check_resident(h, iter_first, num_iters);
    if (st) return st;
    const uint64_t C = h->cfg.num_chains, P = h->updates.size();
    if (num_chains == 0 || chain_first + num_chains > C) return fail(h, EMCMC_INVALID_ARG, "chain window");
    void *base = nullptr;
    size_t row = 0;
    st = hist_geometry(h, which, &base, &row);
    if (st) return st;
    const size_t per_chain = (which == EMCMC_H_LL) ? sizeof(double) : h->cfg.dim * sizeof(double);
    const size_t height = num_iters * P;
    if (host_bytes < num_chains * per_chain * height) return fail(h, EMCMC_INVALID_ARG, "host buffer too small");
    HIPCHK(h, hipStreamSynchronize(h->stream));
    const size_t out_row = P * num_chains * per_chain;  // host bytes per iteration
    return for_each_ring_run(h, iter_first, num_iters, [&](uint64_t r, uint64_t len, uint64_t done) {
        uint8_t *dst = (uint8_t *)host_out + done * out_row;
        if (which != EMCMC_H_LL)
            return copy_state_slots(h, (const double *)base, r * P, len * P, chain_first, num_chains, (double *)dst);
        const size_t width = num_chains * per_chain, spitch = C * per_chain;
        const uint8_t *src = (const uint8_t *)base + r * row + chain_first * per_chain;
        HIPCHK(h, hipMemcpy2D(dst, width, src, spitch, width, len * P, hipMemcpyDeviceToHost));
        return EMCMC_OK;
    });
}

emcmc_status emcmc_history_device_ptr(emcmc_handle *h, uint32_t which, void **dptr, size_t *bytes) {
    if (!h || !dptr || !bytes) return EMCMC_INVALID_ARG;
    if (!h->allocated) return fail(h, EMCMC_STATE_ERROR, "no state");
    size_t row = 0;
    emcmc_status st = hist_geometry(h, which, dptr, &row);
    if (st) return st;
    *bytes = row * h->ring;
    return EMCMC_OK;
}

emcmc_status emcmc_stream_history(emcmc_handle *h, uint32_t which, uint64_t iter_first, uint64_t num_iters,
                                  uint64_t thin, void *host_out, size_t host_bytes) {
    if (!h || !host_out || thin == 0) return EMCMC_INVALID_ARG;
    if (!h->allocated) return fail(h, EMCMC_STATE_ERROR, "no state");
    const uint64_t last = iter_first + (num_iters - 1) * thin;
    if (num_iters == 0 || iter_first < 1 || last > h->cfg.num_mcmc_steps)
        return fail(h, EMCMC_INVALID_ARG, "iteration window outside 1..M");
    if (last > h->hi_iter) return fail(h, EMCMC_STATE_ERROR, "iteration %llu has not been run", (unsigned long long)last);
    emcmc_status st = check_resident(h, iter_first, 1);
    if (st) return st;
    void *base = nullptr;
    size_t row = 0;
    st = hist_geometry(h, which, &base, &row);
    if (st) return st;
    if (host_bytes < row * num_iters) return fail(h, EMCMC_INVALID_ARG, "host buffer too small");
    const uint64_t C = h->cfg.num_chains, D = h->cfg.dim, P = h->updates.size();
    // ordered after the compute work enqueued so far
    hipEvent_t ready = nullptr;
    HIPCHK(h, hipEventCreateWithFlags(&ready, hipEventDisableTiming));
    HIPCHK(h, hipEventRecord(ready, h->stream));
    HIPCHK(h, hipStreamWaitEvent(h->cstream, ready, 0));
    (void)hipEventDestroy(ready);
    uint8_t *out = (uint8_t *)host_out;
    if (which == EMCMC_H_STATE || which == EMCMC_H_PROPOSAL) {
        // gather each iteration's P slots (state_pos layout) into host layout on
        // the copy stream, in chunks through a staging buffer
        const uint64_t per_it = P * C * D;
        const uint64_t chunk = std::max<uint64_t>(1, (256ull << 20) / (per_it * sizeof(double)));
        const size_t need = std::min(num_iters, chunk) * per_it * sizeof(double);
        if (h->stage_bytes < need) {
            HIPCHK(h, hipStreamSynchronize(h->cstream));
            if (h->d_stage) (void)hipFree(h->d_stage);
            h->d_stage = nullptr;
            HIPCHK(h, hipMalloc(&h->d_stage, need));
            h->stage_bytes = need;
        }
        for (uint64_t k0 = 0; k0 < num_iters; k0 += chunk) {
            const uint64_t nk = std::min(chunk, num_iters - k0);
            for (uint64_t k = 0; k < nk; ++k) {
                const uint64_t it = iter_first + (k0 + k) * thin;
                const uint64_t n = per_it;
                hipLaunchKernelGGL(gather_hist_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, h->cstream,
                                   (const double *)base, C, (uint32_t)D, ((it - 1) % h->ring) * P, P, (uint64_t)0, C,
                                   h->d_stage + k * per_it);
                HIPCHK(h, hipGetLastError());
            }
            HIPCHK(h, hipMemcpyAsync(out + k0 * row, h->d_stage, nk * row, hipMemcpyDeviceToHost, h->cstream));
        }
    } else {
        for (uint64_t k = 0; k < num_iters;) {  // contiguous runs when thin == 1
            const uint64_t it = iter_first + k * thin, r = (it - 1) % h->ring;
            uint64_t len = 1;
            if (thin == 1) len = std::min(num_iters - k, h->ring - r);
            HIPCHK(h, hipMemcpyAsync(out + k * row, (const uint8_t *)base + r * row, len * row, hipMemcpyDeviceToHost,
                                     h->cstream));
            k += len;
        }
    }
    hipEvent_t done = nullptr;
    HIPCHK(h, hipEventCreateWithFlags(&done, hipEventDisableTiming));
    HIPCHK(h, hipEventRecord(done, h->cstream));
    h->copies.push_back({iter_first, last, done});
    return EMCMC_OK;
}

emcmc_status emcmc_stream_wait(emcmc_handle *h) {
    if (!h) return EMCMC_INVALID_ARG;
    HIPCHK(h, hipStreamSynchronize(h->cstream));
    for (auto &c : h->copies) (void)hipEventDestroy(c.ev);
    h->copies.clear();
    return EMCMC_OK;
}

emcmc_status emcmc_host_alloc(size_t bytes, void **ptr) {
    if (!ptr) return EMCMC_INVALID_ARG;
    *ptr = nullptr;
    if (hipHostMalloc(ptr, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) return EMCMC_OUT_OF_MEMORY;
    return EMCMC_OK;
}

emcmc_status emcmc_host_free(void *ptr) {
    if (ptr && hipHostFree(ptr) != hipSuccess) return EMCMC_HIP_ERROR;
    return EMCMC_OK;
}

}  // extern "C"

// for emcmc_comm.hip (cross-rank diagnostics)
int emcmc_internal_device(const emcmc_handle *h) { return h->cfg.device; }
uint32_t emcmc_internal_dim(const emcmc_handle *h) { return h->cfg.dim; }
void emcmc_internal_set_error(emcmc_handle *h, const std::string &msg) { h->err = msg; }

extern "C" {

emcmc_status emcmc_moments_window(emcmc_handle *h, uint64_t iter_first, uint64_t num_iters, int split,
                                  double *out3d, emcmc_moments *info) {
    if (!h || !out3d) return EMCMC_INVALID_ARG;
    if (!h->allocated) return fail(h, EMCMC_STATE_ERROR, "no state");
    if (!h->d_hist_theta) return fail(h, EMCMC_STATE_ERROR, "moments need EMCMC_HIST_FULL");
    if (iter_first < 1 || num_iters < 2 || iter_first + num_iters - 1 > h->cfg.num_mcmc_steps)
        return fail(h, EMCMC_INVALID_ARG, "iteration window");
    {
        emcmc_status rs = check_resident(h, iter_first, num_iters);
        if (rs) return rs;
        if ((iter_first - 1) % h->ring + num_iters > h->ring)
            return fail(h, EMCMC_STATE_ERROR, "moments window wraps the history ring");
    }
    const uint64_t ring0 = (iter_first - 1) % h->ring;  // ring iteration of iter_first
    const uint64_t C = h->cfg.num_chains, D = h->cfg.dim, P = h->updates.size();
    const uint32_t halves = split ? 2u : 1u;
    const size_t need = 2 * C * D * halves * sizeof(double) + 3 * D * sizeof(double) + 64;
    if (h->scratch_bytes < need) {
        HIPCHK(h, hipStreamSynchronize(h->stream));
        if (h->d_scratch) (void)hipFree(h->d_scratch);
        HIPCHK(h, hipMalloc(&h->d_scratch, need));
        h->scratch_bytes = need;
    }
    double *mean = h->d_scratch, *var = mean + C * D * halves, *o = var + C * D * halves;
    unsigned long long *cnt = reinterpret_cast<unsigned long long *>(o + 3 * D);
    const uint64_t total = C * D * halves;
    const uint64_t slot0 = ring0 * P + (P - 1);  // state after the last update of the iteration
    hipLaunchKernelGGL(chain_moments_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, h->stream,
                       h->d_hist_theta, C, (uint32_t)D, slot0, (uint32_t)P, (uint32_t)num_iters, halves, mean, var);
    HIPCHK(h, hipGetLastError());
    hipLaunchKernelGGL(moments_reduce_kernel, dim3((unsigned)D), dim3(256), 0, h->stream, mean, var, C,
                       (uint32_t)D, halves, o);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipMemsetAsync(cnt, 0, sizeof(unsigned long long), h->stream));
    const uint64_t words = num_iters * P * h->row_bytes / 8;
    hipLaunchKernelGGL(popcount_kernel, dim3(1024), dim3(256), 0, h->stream,
                       reinterpret_cast<const uint64_t *>(h->d_hist_acc + ring0 * P * h->row_bytes),
                       words, cnt);
    HIPCHK(h, hipGetLastError());
    unsigned long long acc = 0;
    HIPCHK(h, hipMemcpyAsync(out3d, o, 3 * D * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipMemcpyAsync(&acc, cnt, sizeof acc, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (info) {
        info->num_chains = C * halves;
        info->num_draws = num_iters / halves;
        info->accepted = acc;
        info->proposed = C * num_iters * P;
    }
    return EMCMC_OK;
}

emcmc_status emcmc_set_timing(emcmc_handle *h, int enable) {
    if (!h) return EMCMC_INVALID_ARG;
    h->timing = enable != 0;
    return EMCMC_OK;
}

emcmc_status emcmc_get_timing(emcmc_handle *h, double *total_ms, uint64_t *launches, double *algorithmic_bytes,
                              int reset) {
    if (!h) return EMCMC_INVALID_ARG;
    emcmc_status st = drain_timing(h);
    if (st) return st;
    if (total_ms) *total_ms = h->timed_ms;
    if (launches) *launches = h->timed_launches;
    if (algorithmic_bytes) *algorithmic_bytes = h->timed_bytes;
    if (reset) {
        h->timed_ms = 0.0;
        h->timed_launches = 0;
        h->timed_bytes = 0.0;
    }
    return EMCMC_OK;
}

emcmc_status emcmc_kernel_name(emcmc_handle *h, char *buf, size_t buflen) {
    if (!h || !buf || buflen == 0) return EMCMC_INVALID_ARG;
    snprintf(buf, buflen, "%s", h->var.name.empty() ? "(none)" : h->var.name.c_str());
    return EMCMC_OK;
}

emcmc_status emcmc_rtc_info(emcmc_handle *h, uint32_t *origin, double *seconds) {
    if (!h || !origin || !seconds) return EMCMC_INVALID_ARG;
    if (!h->var.ufn && !h->var.ffn) return fail(h, EMCMC_STATE_ERROR, "the selected kernel is compiled ahead of time");
    *origin = h->rtc_origin;
    *seconds = h->rtc_seconds;
    return EMCMC_OK;
}

emcmc_status emcmc_probe_variates(int device, uint64_t seed, uint32_t pidx0, uint32_t dim, uint64_t n,
                                  const uint32_t *chains, const uint32_t *iters, double *z, double *E) {
    if (!chains || !iters || !z || !E || dim == 0) return EMCMC_INVALID_ARG;
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || nd == 0) return EMCMC_NO_DEVICE;
    if (device < 0 || device >= nd || hipSetDevice(device) != hipSuccess) return EMCMC_INVALID_ARG;
    if (n == 0) return EMCMC_OK;
    uint32_t *dc = nullptr, *di = nullptr;
    double *dz = nullptr, *dE = nullptr;
    Ziggurat *dzig = nullptr;
    Ziggurat zt;
    build_ziggurat(zt);
    emcmc_status st = EMCMC_OK;
    if (hipMalloc(&dc, n * 4) || hipMalloc(&di, n * 4) || hipMalloc(&dz, n * dim * 8) || hipMalloc(&dE, n * 8) ||
        hipMalloc(&dzig, sizeof(Ziggurat))) {
        st = EMCMC_OUT_OF_MEMORY;
    } else if (hipMemcpy(dc, chains, n * 4, hipMemcpyHostToDevice) ||
               hipMemcpy(di, iters, n * 4, hipMemcpyHostToDevice) ||
               hipMemcpy(dzig, &zt, sizeof(Ziggurat), hipMemcpyHostToDevice)) {
        st = EMCMC_HIP_ERROR;
    } else {
        hipLaunchKernelGGL(probe_variates_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, dzig,
                           (uint32_t)seed, (uint32_t)(seed >> 32), pidx0, dim, n, dc, di, dz, dE);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
            hipMemcpy(z, dz, n * dim * 8, hipMemcpyDeviceToHost) || hipMemcpy(E, dE, n * 8, hipMemcpyDeviceToHost))
            st = EMCMC_HIP_ERROR;
    }
    (void)hipFree(dc);
    (void)hipFree(di);
    (void)hipFree(dz);
    (void)hipFree(dE);
    (void)hipFree(dzig);
    return st;
}

emcmc_status emcmc_probe_log(int device, const double *x, double *y, uint64_t n) {
    if (!x || !y) return EMCMC_INVALID_ARG;
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || nd == 0) return EMCMC_NO_DEVICE;
    if (device < 0 || device >= nd || hipSetDevice(device) != hipSuccess) return EMCMC_INVALID_ARG;
    if (n == 0) return EMCMC_OK;
    double *dx = nullptr, *dy = nullptr;
    emcmc_status st = EMCMC_OK;
    if (hipMalloc(&dx, n * 8) || hipMalloc(&dy, n * 8)) {
        st = EMCMC_OUT_OF_MEMORY;
    } else if (hipMemcpy(dx, x, n * 8, hipMemcpyHostToDevice)) {
        st = EMCMC_HIP_ERROR;
    } else {
        hipLaunchKernelGGL(probe_log_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, dx, dy, n);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
            hipMemcpy(y, dy, n * 8, hipMemcpyDeviceToHost))
            st = EMCMC_HIP_ERROR;
    }
    (void)hipFree(dx);
    (void)hipFree(dy);
    return st;
}

}  // extern "C"
