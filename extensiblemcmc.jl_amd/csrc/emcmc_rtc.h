// emcmc_rtc.h — run-time compilation of user log-likelihoods (hiprtc).
//
// The reference's plugin surface for a target is a Julia type with
// `set_parameters!(P, idx, θ)` and `loglikelihood(P, obs)`
// (src/example/gsn_target.jl:15-29, docs/src/get_started/basic_use.md:84-112);
// any law the user writes drops into `compute_ll!` (run.jl:251-260).  On the
// device the law is a function of P°.θ, written once in a C subset that both
// hiprtc (here) and gcc (the oracle, oracle/user_prelude.h) compile:
//
//     EMCMC_USER_LOGLIK {            // theta[D], D, obs, nobs, params in scope
//         double s = 0.0;
//         for (uint64_t k = 0; k < nobs; ++k) s = s + em_log(obs[k] * theta[0]);
//         return s;
//     }
//
// with + − × ÷, fma, sqrt, fabs, copysign and em_exp / em_log (the engine's
// own exp/log — NaN below 0 — restated bit for bit in oracle/oracle_math.h).  The source is
// compiled into the general schedule kernel (emcmc_mwg.h) with TGT = the
// user's law, so every update kind, prior and adaptation of that kernel runs
// with it.
#pragma once

#include <string>
#include <vector>

namespace emcmc {

struct RtcKernel {
    std::vector<char> code;  // gfx950 code object
    std::string lowered;     // mangled kernel name inside it
    std::string name;        // readable name for emcmc_kernel_name
    // how this process obtained it (emcmc_rtc_info): the process cache, the
    // on-disk code-object cache, or a hiprtc compile; seconds spent getting it
    uint32_t origin = 0;
    double seconds = 0.0;
};
// kRtcCompiledCacheRefused: compiled because the on-disk cache directory exists but is not
// private to this user (emcmc_rtc.hip private_dir; a one-time stderr warning says so)
enum : uint32_t { kRtcFromProcess = 0, kRtcFromDisk = 1, kRtcCompiled = 2, kRtcCompiledCacheRefused = 3 };

// The on-disk code-object cache: EMCMC_RTC_CACHE (a directory; "off" disables
// it), else rtc_cache/ beside libemcmc.so.  Entries are keyed by a 128-bit
// digest of everything the code depends on (program text, embedded headers,
// name expression, options, hiprtc version, target arch), so a second process,
// the other ranks of a node and later runs load instead of compiling.
std::string rtc_cache_dir();

// Compile (or fetch from the process-wide cache) the general schedule kernel
// for dimension D with the user's log-likelihood: mwg_gsn_kernel<D> for
// D ≤ 16, mwg_wide_kernel<D, NU> for 16 < D ≤ 64 (NU = 16 when every update
// has ≤ 16 coordinates — unrolled, in registers — else NU = D).  Returns "" on
// success, else the compiler's log.
int rtc_wide_nu(int D, int nmax);
// usrc / uopts: a user update's EMCMC_USER_PROPOSAL + EMCMC_USER_LTD source (empty: none)
// xt: compile GaussianRandomWalkMix / Haario / chain moments in (emcmc_mwg.h XT)
// mala: compile MALA updates in (kind 4; the target's gradient: GsnTarget::grad or
// the user law's EMCMC_USER_GRAD, which the source then defines)
std::string rtc_compile_user(const std::string &src, const std::string &opts, int D, bool full, int nu,
                             RtcKernel &out, const std::string &usrc = std::string(),
                             const std::string &uopts = std::string(), bool xt = false, bool mala = false);

// The text of a law the library ships as an EMCMC_USER_LOGLIK source
// (csrc/laws/<name>), or nullptr.
const char *rtc_builtin_law(const char *name);

// The same kernel with the built-in GsnTargetLaw (emcmc_mwg.h GsnTarget) for a
// dimension the library has no ahead-of-time instantiation of (inst_mwg.hip).
std::string rtc_compile_gsn(int D, bool full, int ll_mode, int nu, RtcKernel &out,
                            const std::string &usrc = std::string(), const std::string &uopts = std::string(),
                            bool xt = false, bool mala = false);

// Does a user law's source define a gradient body (`EMCMC_USER_GRAD { … }`)?
// Comments, string and character literals are skipped, and the name must stand
// as a whole token, so a law that only mentions the macro in a comment gets the
// "MALA needs the target's gradient" refusal instead of a compile error.
inline bool rtc_defines_user_grad(const std::string &src) {
    static const char kTok[] = "EMCMC_USER_GRAD";
    const size_t n = src.size(), tn = sizeof kTok - 1;
    auto ident = [](char c) { return c == '_' || (c >= '0' && c <= '9') || ((c | 32) >= 'a' && (c | 32) <= 'z'); };
    for (size_t i = 0; i < n;) {
        const char c = src[i];
        if (c == '/' && i + 1 < n && src[i + 1] == '/') {
            while (i < n && src[i] != '\n') ++i;
        } else if (c == '/' && i + 1 < n && src[i + 1] == '*') {
            const size_t e = src.find("*/", i + 2);
            i = (e == std::string::npos) ? n : e + 2;
        } else if (c == '"' || c == '\'') {
            for (++i; i < n && src[i] != c; ++i)
                if (src[i] == '\\') ++i;
            ++i;
        } else if (ident(c)) {
            size_t j = i;
            while (j < n && ident(src[j])) ++j;
            if (j - i == tn && src.compare(i, tn, kTok) == 0) return true;
            i = j;
        } else {
            ++i;
        }
    }
    return false;
}

// rwm_gsn_chol_kernel<D, FULL, LL> (emcmc_kernels.h) for a D without an
// ahead-of-time instantiation (inst_chol.hip: 16, 24, 32): correlated Σ_rw / Σ_t
// on the fused single-update path, any D ≤ 64 (θ, θ° and one substitution vector
// in registers: no spills to D = 40, AGPR and scratch spills above — still 20–45×
// the general kernel).
constexpr int kCholRtcMaxD = 64;
constexpr int kCholRtcMaxChunks = 400;
// chunks of one observation sweep (prefix D + the packed factor), as chol_stream
// cuts them: 16 doubles each, the prefix and the table on chunks of their own
// (≤ 4 + 130 at D = 64, so every D ≤ 64 is within the compile budget)
inline int chol_rtc_chunks(int D) { return (D + 15) / 16 + (D * (D + 1) / 2 + 15) / 16; }
std::string rtc_compile_chol(int D, bool full, int ll_mode, RtcKernel &out);

// mwg_block_kernel<D, FULL, LL, TGT, UPD> (emcmc_block.h): one MALA or user update over
// all 17 ≤ D ≤ 64 coordinates with the per-chain vectors in registers.  src: a user
// law (TGT = its loglik / grad), else the built-in GsnTargetLaw through the scalar
// cache (TGT = GsnSweep<tdense>); usrc: a user update (UPD = its proposal! /
// log_transition_density), else MALA.
std::string rtc_compile_block(int D, bool full, int ll_mode, bool tdense, const std::string &src,
                              const std::string &opts, const std::string &usrc, const std::string &uopts,
                              RtcKernel &out);

// mwg_rw_block_kernel<D, FULL, LL, TGT, RwSched> (emcmc_rwblock.h): a schedule of 1–8
// UniformRandomWalk / GaussianRandomWalk updates over any coordinate subsets at 17 ≤ D ≤ 64 with
// any prior, positivity flags and AdaptationUnifRW.  shape: the source of the schedule's
// compile-time structure `struct <shape_struct>` with one U<p> per update (emcmc.hip
// rw_sched_source); shape_name: its label in the kernel name; src / opts: a user law, else the
// built-in GsnTargetLaw (GsnSweep<tdense>).
std::string rtc_compile_rwblock(int D, bool full, int ll_mode, bool tdense, const std::string &shape,
                                const std::string &shape_struct, const std::string &shape_name,
                                const std::string &src, const std::string &opts, RtcKernel &out);

// rwm_gsn_diag_kernel<D, LPC, FULL, LL, UNIT_T, MINW, FusedPrior<shape_struct>> (emcmc_fused.h,
// emcmc_fprior.h): the fused diagonal step with a separable ProductPrior / StandardPrior of D
// univariate factors (the schedule source's U<0> gives the families).
std::string rtc_compile_fused_prior(int D, int lpc, int minw, bool full, int ll_mode, bool unit_t,
                                   const std::string &shape, const std::string &shape_struct,
                                   const std::string &shape_name, RtcKernel &out);

}  // namespace emcmc
