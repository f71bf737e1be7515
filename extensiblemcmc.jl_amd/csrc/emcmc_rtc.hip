// emcmc_rtc.hip — hiprtc driver for user log-likelihoods (see emcmc_rtc.h).
//
// The kernel headers are embedded at build time (build/gen/rtc_headers.inc,
// scripts/embed_headers.py); the user's source is wrapped between a prelude
// that defines EMCMC_USER_LOGLIK / em_exp / em_log and an epilogue that turns
// the function into the kernel's target policy (emcmc_mwg.h GsnTarget's
// interface).  Code objects are cached per (source, options, D, history mode)
// for the life of the process, so shards and repeated runs compile once.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

// the library's state_pos tile width (emcmc_kernels.h): run-time kernels must lay out
// HBM as the ahead-of-time ones do, so it is passed to every compile (and digest)
#ifndef EMCMC_SOA_TILE
#define EMCMC_SOA_TILE 32
#endif

#include <dlfcn.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "emcmc_rtc.h"
#include "rtc_headers.inc"

namespace emcmc {
namespace {

const char *const kPrelude = R"EMCMC_RTC(#include "emcmc_mwg.h"
#define EMCMC_USER_LOGLIK                                                                                  \
    extern "C" __device__ __attribute__((always_inline)) inline double emcmc_user_loglik(                 \
        const double *__restrict__ theta, int D, const double *__restrict__ obs, uint64_t nobs,            \
        const double *__restrict__ params)
#define EMCMC_USER_GRAD                                                                                    \
    extern "C" __device__ __attribute__((always_inline)) inline void emcmc_user_grad(                     \
        const double *__restrict__ theta, int D, const double *__restrict__ obs, uint64_t nobs,            \
        const double *__restrict__ params, double *__restrict__ grad)
#define EMCMC_USER_PROPOSAL                                                                                \
    extern "C" __device__ __attribute__((always_inline)) inline void emcmc_user_proposal(                 \
        const double *__restrict__ theta, double *__restrict__ theta_prop, int n,                          \
        const double *__restrict__ params, emcmc::UserRng *__restrict__ rng)
#define EMCMC_USER_LTD                                                                                     \
    extern "C" __device__ __attribute__((always_inline)) inline double emcmc_user_ltd(                    \
        const double *__restrict__ x, const double *__restrict__ y, int n, const double *__restrict__ params)
#define em_exp(x) emcmc::exp_any(x)
#define em_log(x) emcmc::log_real(x)
#define em_randn(j) emcmc::user_randn(*rng, (uint32_t)(j))
#define em_rand(j) emcmc::user_rand(*rng, (uint32_t)(j))
)EMCMC_RTC";

const char *const kEpilogue = R"EMCMC_RTC(
namespace emcmc {
// loglikelihood(P°, obs) of the user's law (gsn_target.jl:23-29's interface)
struct UserTarget {
    template <int D, int LLMODE, bool ROLL = false>
    __device__ __forceinline__ static double loglik(const MwgParams &a, const double (&mp)[D]) {
        return emcmc_user_loglik(mp, D, a.obs, (uint64_t)a.nobs, a.user_params);
    }
    // ∇ loglikelihood(P°, obs) of the user's law (EMCMC_USER_GRAD), the hook
    // MALA reads (compute_gradients_and_momenta!, updates.jl:123-133); the host
    // refuses MALA on a law without one
    template <int D, int LLMODE, bool ROLL = false>
    __device__ __forceinline__ static void grad(const MwgParams &a, const double (&mp)[D], double (&g)[D]) {
#ifdef EMCMC_HAS_USER_GRAD
        emcmc_user_grad(mp, D, a.obs, (uint64_t)a.nobs, a.user_params, g);
#else
        for (int d = 0; d < D; ++d) g[d] = __builtin_nan("");
#endif
    }
};
}  // namespace emcmc
)EMCMC_RTC";

const char *const kUpdEpilogue = R"EMCMC_RTC(
namespace emcmc {
// proposal! / log_transition_density of the user's update (updates.jl:42-93)
struct UserUpdate {
    static constexpr bool kEnabled = true;
#ifdef EMCMC_RTC_MALA
    static constexpr bool kMala = true;  // MALA updates in the same schedule
#else
    static constexpr bool kMala = false;
#endif
    __device__ __forceinline__ static void propose(UserRng &rng, const double *th, double *tp, int n,
                                                   const double *params) {
        emcmc_user_proposal(th, tp, n, params, &rng);
    }
    __device__ __forceinline__ static double ltd(const double *x, const double *y, int n, const double *params) {
        return emcmc_user_ltd(x, y, n, params);
    }
};
}  // namespace emcmc
)EMCMC_RTC";

std::mutex g_mu;
std::map<std::string, RtcKernel> g_cache;

std::string program_log(hiprtcProgram p) {
    size_t n = 0;
    if (hiprtcGetProgramLogSize(p, &n) != HIPRTC_SUCCESS || n == 0) return "";
    std::string s(n, '\0');
    if (hiprtcGetProgramLog(p, &s[0]) != HIPRTC_SUCCESS) return "";
    while (!s.empty() && s.back() == '\0') s.pop_back();
    return s;
}

}  // namespace

// src empty: the built-in GsnTarget with likelihood mode ll; else the user's law
int rtc_wide_nu(int D, int nmax) { return (D > 16 && nmax <= 16) ? 16 : D; }

namespace {

bool cache_get(const std::string &key, RtcKernel &out) {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_cache.find(key);
    if (it == g_cache.end()) return false;
    out = it->second;
    out.origin = kRtcFromProcess;
    out.seconds = 0.0;
    return true;
}

// ---- on-disk code-object cache ------------------------------------------------
// 128-bit digest: two FNV-1a-64 streams with different offsets over the same bytes
struct Digest {
    uint64_t a = 0xcbf29ce484222325ull, b = 0x84222325cbf29ce4ull;
    void add(const void *p, size_t n) {
        const unsigned char *c = static_cast<const unsigned char *>(p);
        for (size_t i = 0; i < n; ++i) {
            a = (a ^ c[i]) * 0x100000001b3ull;
            b = (b ^ c[i] ^ 0x5a) * 0x100000001b3ull;
        }
        const uint64_t len = n;  // length-delimited: ("ab","c") ≠ ("a","bc")
        const unsigned char *l = reinterpret_cast<const unsigned char *>(&len);
        for (int i = 0; i < 8; ++i) a = (a ^ l[i]) * 0x100000001b3ull, b = (b ^ l[i]) * 0x100000001b3ull;
    }
    void add(const std::string &s) { add(s.data(), s.size()); }
    std::string hex() const {
        char buf[33];
        snprintf(buf, sizeof buf, "%016llx%016llx", (unsigned long long)a, (unsigned long long)b);
        return buf;
    }
};

// Entry file: magic | lowered-name length, name | code length, code | 128-bit digest of
// (name, code).  A reader checks the digest, so a torn, truncated or zero-filled file is a
// miss (recompiled), never a code object that runs.
const char kDiskMagic[8] = {'E', 'M', 'C', 'R', 'T', 'C', '2', '\n'};

std::string payload_digest(const RtcKernel &k) {
    Digest d;
    d.add(k.lowered);
    d.add(k.code.data(), k.code.size());
    return d.hex();
}

// The cache directory is used only when it is private to this user: owned by the
// effective uid and neither group- nor world-writable (else anyone who can write it could
// plant a code object every later handle would execute).  Created 0700 when absent.
bool private_dir(const std::string &dir, bool create, bool *refused = nullptr) {
    struct stat st;
    if (stat(dir.c_str(), &st) != 0) {
        if (!create || mkdir(dir.c_str(), 0700) != 0 || stat(dir.c_str(), &st) != 0) return false;
    }
    if (!S_ISDIR(st.st_mode) || st.st_uid != geteuid() || (st.st_mode & (S_IWGRP | S_IWOTH))) {
        if (refused) *refused = true;
        // said once per process whatever EMCMC_RTC_LOG says: every run-time kernel now compiles in
        // every process (≈ 1 minute each at D ≥ 40) and the cause is the directory's owner or mode
        static std::once_flag once;
        std::call_once(once, [&] {
            fprintf(stderr,
                    "[emcmc rtc] warning: %s is not a private directory of this user (owner uid %u, euid %u, "
                    "mode %03o): the on-disk code-object cache is not used, run-time kernels compile in every "
                    "process; make it owned by the running user with mode 0700 (INTEGRATION.md)\n",
                    dir.c_str(), (unsigned)st.st_uid, (unsigned)geteuid(), (unsigned)(st.st_mode & 0777));
        });
        return false;
    }
    return true;
}

bool disk_get(const std::string &dir, const std::string &file, RtcKernel &k, bool *refused) {
    if (!private_dir(dir, false, refused)) return false;
    std::ifstream f(file, std::ios::binary);
    if (!f) return false;
    char m[8];
    uint64_t nl = 0, nc = 0;
    if (!f.read(m, 8) || std::string(m, 8) != std::string(kDiskMagic, 8)) return false;
    if (!f.read(reinterpret_cast<char *>(&nl), 8) || nl == 0 || nl > 4096) return false;
    k.lowered.resize(nl);
    if (!f.read(&k.lowered[0], (std::streamsize)nl)) return false;
    if (!f.read(reinterpret_cast<char *>(&nc), 8) || nc == 0 || nc > (1ull << 30)) return false;
    k.code.resize(nc);
    if (!f.read(k.code.data(), (std::streamsize)nc)) return false;
    char dg[32];
    if (!f.read(dg, 32) || std::string(dg, 32) != payload_digest(k)) return false;
    return f.peek() == std::char_traits<char>::eof();  // a truncated or padded file is not an entry
}

void disk_put(const std::string &dir, const std::string &file, const RtcKernel &k) {
    if (!private_dir(dir, true)) return;
    std::string tmp = file + ".tmp.XXXXXX";  // unique per writer (threads of one process included)
    const int fd = mkstemp(&tmp[0]);
    if (fd < 0) return;  // read-only location: the process cache still holds it
    FILE *f = fdopen(fd, "wb");
    if (!f) {
        close(fd);
        (void)unlink(tmp.c_str());
        return;
    }
    const uint64_t nl = k.lowered.size(), nc = k.code.size();
    const std::string dg = payload_digest(k);
    bool ok = fwrite(kDiskMagic, 1, 8, f) == 8 && fwrite(&nl, 8, 1, f) == 1 &&
              fwrite(k.lowered.data(), 1, nl, f) == nl && fwrite(&nc, 8, 1, f) == 1 &&
              fwrite(k.code.data(), 1, nc, f) == nc && fwrite(dg.data(), 1, 32, f) == 32;
    ok = (fclose(f) == 0) && ok;
    if (!ok || rename(tmp.c_str(), file.c_str()) != 0) (void)unlink(tmp.c_str());  // atomic: ranks may race
}

// EMCMC_RTC_EXTRA: extra options for every run-time compile (A/B builds of the run-time
// kernels, e.g. "-DEMCMC_CHOL_SHARED=0"); part of the disk-cache digest and of the
// process-cache key (rtc_env_extra is read once per process).
const std::vector<std::string> &rtc_env_extra() {
    static const std::vector<std::string> v = [] {
        std::vector<std::string> out;
        if (const char *e = getenv("EMCMC_RTC_EXTRA")) {
            std::istringstream is(e);
            for (std::string w; is >> w;) out.push_back(w);
        }
        return out;
    }();
    return v;
}

// Compile prog_src for gfx950 and fetch the code object of the kernel named by
// the expression ex; cache it under key.  Returns "" or the compiler's log.
// -ffp-contract=off: the parity contract with oracle/ (no implicit fma).
// Embedded headers a program includes (directly or not): its disk-cache digest covers these
// only, so editing the block kernel's header leaves the cached chol kernels valid.
const std::vector<std::string> kCholDeps = {"emcmc_tables.h", "emcmc_math.h", "emcmc_kernels.h", "emcmc_chol.h"};
const std::vector<std::string> kMwgDeps = {"emcmc_tables.h", "emcmc_math.h", "emcmc_kernels.h", "emcmc_mwg.h"};
const std::vector<std::string> kBlockDeps = {"emcmc_tables.h", "emcmc_math.h", "emcmc_kernels.h", "emcmc_mwg.h",
                                             "emcmc_block.h"};
const std::vector<std::string> kRwBlockDeps = {"emcmc_tables.h", "emcmc_math.h",  "emcmc_kernels.h",
                                               "emcmc_mwg.h",    "emcmc_block.h", "emcmc_rwblock.h"};
const std::vector<std::string> kFusedPriorDeps = {"emcmc_tables.h", "emcmc_math.h",  "emcmc_kernels.h",
                                                  "emcmc_mwg.h",    "emcmc_fused.h", "emcmc_fprior.h"};

std::string compile_kernel(const std::string &key, const std::string &prog_src, const char *file,
                           const std::string &ex, const std::string &name, const std::vector<std::string> &extra,
                           RtcKernel &out, const std::vector<std::string> &deps) {
    const auto t0 = std::chrono::steady_clock::now();
    const auto since = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
    // disk cache: the digest covers every input of the compile
    const std::string dir = rtc_cache_dir();
    std::string dfile;
    bool refused = false;  // the cache directory exists but is not private: not read, not written
    if (!dir.empty()) {
        Digest d;
        for (const auto &dep : deps)
            for (int i = 0; i < kRtcHeaderCount; ++i)
                if (dep == kRtcHeaderNames[i]) {
                    d.add(dep);
                    d.add(std::string(kRtcHeaderSrc[i]));
                }
        int vmaj = 0, vmin = 0;
        (void)hiprtcVersion(&vmaj, &vmin);
        d.add(prog_src);
        d.add(std::string(file));
        d.add(ex);
        for (const auto &w : extra) d.add(w);
        d.add("-DEMCMC_SOA_TILE=" + std::to_string(EMCMC_SOA_TILE));
        for (const auto &w : rtc_env_extra()) d.add(w);
        d.add("gfx950|-O3|-ffp-contract=off|-std=c++17|hiprtc " + std::to_string(vmaj) + "." + std::to_string(vmin) +
              "|HIP " + std::to_string(HIP_VERSION));
        dfile = dir + "/" + d.hex() + ".co";
        RtcKernel k;
        if (disk_get(dir, dfile, k, &refused)) {
            k.name = name;
            k.origin = kRtcFromDisk;
            k.seconds = since();
            {
                std::lock_guard<std::mutex> lk(g_mu);
                g_cache[key] = k;
            }
            out = std::move(k);
            return "";
        }
    }
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, prog_src.c_str(), file, kRtcHeaderCount, kRtcHeaderSrc, kRtcHeaderNames) !=
        HIPRTC_SUCCESS)
        return "hiprtcCreateProgram failed";
    hiprtcAddNameExpression(prog, ex.c_str());
    std::vector<std::string> o = {"--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17",
                                  "-DEMCMC_SOA_TILE=" + std::to_string(EMCMC_SOA_TILE)};
    for (const auto &w : rtc_env_extra()) o.push_back(w);
    o.insert(o.end(), extra.begin(), extra.end());
    std::vector<const char *> ov;
    for (const auto &w : o) ov.push_back(w.c_str());
    const hiprtcResult rc = hiprtcCompileProgram(prog, (int)ov.size(), ov.data());
    const std::string log = program_log(prog);
    if (rc != HIPRTC_SUCCESS) {
        hiprtcDestroyProgram(&prog);
        return std::string("hiprtc: ") + hiprtcGetErrorString(rc) + "\n" + log;
    }
    RtcKernel k;
    const char *low = nullptr;
    size_t n = 0;
    if (hiprtcGetLoweredName(prog, ex.c_str(), &low) != HIPRTC_SUCCESS || !low ||
        hiprtcGetCodeSize(prog, &n) != HIPRTC_SUCCESS || n == 0) {
        hiprtcDestroyProgram(&prog);
        return "hiprtc: no code object for " + ex;
    }
    k.lowered = low;
    k.code.resize(n);
    if (hiprtcGetCode(prog, k.code.data()) != HIPRTC_SUCCESS) {
        hiprtcDestroyProgram(&prog);
        return "hiprtcGetCode failed";
    }
    hiprtcDestroyProgram(&prog);
    k.name = name;
    k.origin = refused ? kRtcCompiledCacheRefused : kRtcCompiled;
    k.seconds = since();
    if (!dfile.empty() && !refused) disk_put(dir, dfile, k);
    if (getenv("EMCMC_RTC_LOG"))
        fprintf(stderr, "[emcmc rtc] compiled %s in %.1f s%s%s\n", name.c_str(), k.seconds,
                dfile.empty() ? "" : ", cached as ", dfile.c_str());
    {
        std::lock_guard<std::mutex> lk(g_mu);
        g_cache[key] = k;
    }
    out = std::move(k);
    return "";
}

}  // namespace

std::string rtc_cache_dir() {
    const char *e = getenv("EMCMC_RTC_CACHE");
    if (e && *e) return std::string(e) == "off" ? std::string() : std::string(e);
    Dl_info info;
    if (!dladdr(reinterpret_cast<void *>(&rtc_wide_nu), &info) || !info.dli_fname) return std::string();
    std::string lib = info.dli_fname;
    const size_t s = lib.rfind('/');
    return (s == std::string::npos ? std::string(".") : lib.substr(0, s)) + "/rtc_cache";
}

std::string rtc_compile(const std::string &src, const std::string &opts, int D, bool full, int ll, int nu,
                        RtcKernel &out, const std::string &usrc = std::string(), const std::string &uopts = std::string(),
                        bool xt = false, bool mala = false) {
    if (D < 1 || D > 64) return "the general schedule kernel runs 1 ≤ D ≤ 64";
    if (nu < 1 || nu > D) nu = D;
    const bool user = !src.empty(), upd = !usrc.empty();
    std::ostringstream key;
    key << D << '|' << nu << '|' << full << '|' << ll << '|' << xt << '|' << mala << '|' << opts << '|' << src << '|'
        << uopts << '|' << usrc;
    if (cache_get(key.str(), out)) return "";
    std::ostringstream expr, name;
    const char *fl = full ? "true" : "false";
    const char *tgt = user ? "emcmc::UserTarget" : "emcmc::GsnTarget";
    const char *ut = upd ? "emcmc::UserUpdate" : mala ? "emcmc::MalaOnly" : "emcmc::NoUserUpdate";
    const char *xs = xt ? "true" : "false";
    if (D <= 16) {
        expr << "emcmc::mwg_gsn_kernel<" << D << ", " << fl << ", " << ll << ", " << tgt << ", " << ut << ", " << xs
             << ">";
        name << "mwg_gsn_kernel<D=" << D;
    } else {
        expr << "emcmc::mwg_wide_kernel<" << D << ", " << nu << ", " << fl << ", " << ll << ", " << tgt << ", " << ut
             << ", " << xs << ">";
        name << "mwg_wide_kernel<D=" << D << ",NU=" << nu;
    }
    name << "," << (full ? "FULL" : "ACCEPT_ONLY") << ","
         << (user ? "UserTarget" : ll == 0 ? "PER_OBS" : "SUFFSTAT") << (upd ? ",UserUpdate" : "")
         << (xt ? ",MIX_MOMENTS" : "") << (mala ? ",MALA" : "") << "[hiprtc]>";
    std::string prog_src = std::string(kPrelude);
    if (user) prog_src += std::string("#line 1 \"user_target\"\n") + src + "\n" + kEpilogue;
    if (upd) prog_src += std::string("#line 1 \"user_update\"\n") + usrc + "\n" + kUpdEpilogue;
    std::vector<std::string> extra;
    if (mala) extra.push_back("-DEMCMC_RTC_MALA=1");
    if (user && rtc_defines_user_grad(src)) extra.push_back("-DEMCMC_HAS_USER_GRAD=1");
    for (const std::string *op : {&opts, &uopts}) {
        std::istringstream is(*op);
        for (std::string w; is >> w;) extra.push_back(w);
    }
    return compile_kernel(key.str(), prog_src, user ? "user_target.hip" : upd ? "user_update.hip" : "gsn_target.hip",
                          expr.str(), name.str(), extra, out, kMwgDeps);
}

std::string rtc_compile_user(const std::string &src, const std::string &opts, int D, bool full, int nu,
                             RtcKernel &out, const std::string &usrc, const std::string &uopts, bool xt, bool mala) {
    if (src.empty()) return "empty user source";
    return rtc_compile(src, opts, D, full, 0, nu, out, usrc, uopts, xt, mala);
}

std::string rtc_compile_chol(int D, bool full, int ll_mode, RtcKernel &out) {
    if (D < 2 || D > kCholRtcMaxD) return "rwm_gsn_chol_kernel is compiled at run time for 2 ≤ D ≤ 64";
    std::ostringstream key, expr, name;
    key << "chol|" << D << '|' << full << '|' << ll_mode;
    if (cache_get(key.str(), out)) return "";
    expr << "emcmc::rwm_gsn_chol_kernel<" << D << ", " << (full ? "true" : "false") << ", " << ll_mode << ">";
    name << "rwm_gsn_chol_kernel<D=" << D << ",LPC=1," << (full ? "FULL" : "ACCEPT_ONLY") << ","
         << (ll_mode == 0 ? "PER_OBS" : "SUFFSTAT") << ">[hiprtc]";
    return compile_kernel(key.str(), "#include \"emcmc_chol.h\"\n", "chol_kernel.hip", expr.str(), name.str(),
                          {"-ftemplate-depth=2048"}, out, kCholDeps);
}

std::string rtc_compile_block(int D, bool full, int ll_mode, bool tdense, const std::string &src,
                              const std::string &opts, const std::string &usrc, const std::string &uopts,
                              RtcKernel &out) {
    if (D < 17 || D > 64) return "mwg_block_kernel runs 17 ≤ D ≤ 64";
    const bool user = !src.empty(), upd = !usrc.empty();
    std::ostringstream key, expr, name;
    key << "block|" << D << '|' << full << '|' << ll_mode << '|' << tdense << '|' << opts << '|' << src << '|'
        << uopts << '|' << usrc;
    if (cache_get(key.str(), out)) return "";
    const char *tgt = user ? "emcmc::UserTarget" : tdense ? "emcmc::GsnSweep<true>" : "emcmc::GsnSweep<false>";
    expr << "emcmc::mwg_block_kernel<" << D << ", " << (full ? "true" : "false") << ", " << ll_mode << ", " << tgt
         << ", " << (upd ? "emcmc::UserUpdate" : "emcmc::MalaOnly") << ">";
    name << "mwg_block_kernel<D=" << D << "," << (full ? "FULL" : "ACCEPT_ONLY") << ","
         << (user ? "UserTarget" : ll_mode == 0 ? "PER_OBS" : "SUFFSTAT")
         << (user ? "" : tdense ? ",DENSE_T" : ",DIAG_T") << (upd ? ",UserUpdate" : ",MALA") << "[hiprtc]>";
    std::string prog_src = std::string(kPrelude) + "#include \"emcmc_block.h\"\n";
    if (user) prog_src += std::string("#line 1 \"user_target\"\n") + src + "\n" + kEpilogue;
    if (upd) prog_src += std::string("#line 1 \"user_update\"\n") + usrc + "\n" + kUpdEpilogue;
    std::vector<std::string> extra = {"-ftemplate-depth=2048"};
    if (!upd) extra.push_back("-DEMCMC_RTC_MALA=1");
    if (user && rtc_defines_user_grad(src)) extra.push_back("-DEMCMC_HAS_USER_GRAD=1");
    for (const std::string *op : {&opts, &uopts}) {
        std::istringstream is(*op);
        for (std::string w; is >> w;) extra.push_back(w);
    }
    return compile_kernel(key.str(), prog_src, user ? "user_target.hip" : upd ? "user_update.hip" : "block_kernel.hip",
                          expr.str(), name.str(), extra, out, kBlockDeps);
}

std::string rtc_compile_rwblock(int D, bool full, int ll_mode, bool tdense, const std::string &shape,
                                const std::string &shape_struct, const std::string &shape_name,
                                const std::string &src, const std::string &opts, RtcKernel &out) {
    if (D < 17 || D > 64) return "mwg_rw_block_kernel runs 17 ≤ D ≤ 64";
    const bool user = !src.empty();
    std::ostringstream key, expr, name;
    key << "rwblock|" << D << '|' << full << '|' << ll_mode << '|' << tdense << '|' << shape << '|' << opts << '|'
        << src;
    if (cache_get(key.str(), out)) return "";
    const char *tgt = user ? "emcmc::UserTarget" : tdense ? "emcmc::GsnSweep<true>" : "emcmc::GsnSweep<false>";
    expr << "emcmc::mwg_rw_block_kernel<" << D << ", " << (full ? "true" : "false") << ", " << ll_mode << ", " << tgt
         << ", emcmc::" << shape_struct << ">";
    name << "mwg_rw_block_kernel<D=" << D << "," << (full ? "FULL" : "ACCEPT_ONLY") << ","
         << (user ? "UserTarget" : ll_mode == 0 ? "PER_OBS" : "SUFFSTAT") << (user ? "" : tdense ? ",DENSE_T" : ",DIAG_T")
         << "," << shape_name << "[hiprtc]>";
    std::string prog_src = std::string(kPrelude) + "#include \"emcmc_rwblock.h\"\n" + shape;
    if (user) prog_src += std::string("#line 1 \"user_target\"\n") + src + "\n" + kEpilogue;
    std::vector<std::string> extra = {"-ftemplate-depth=2048"};
    if (user && rtc_defines_user_grad(src)) extra.push_back("-DEMCMC_HAS_USER_GRAD=1");
    std::istringstream is(opts);
    for (std::string w; is >> w;) extra.push_back(w);
    return compile_kernel(key.str(), prog_src, user ? "user_target.hip" : "rw_block_kernel.hip", expr.str(),
                          name.str(), extra, out, kRwBlockDeps);
}

std::string rtc_compile_fused_prior(int D, int lpc, int minw, bool full, int ll_mode, bool unit_t,
                                   const std::string &shape, const std::string &shape_struct,
                                   const std::string &shape_name, RtcKernel &out) {
    if (D < 1 || D > 64 || (lpc != 1 && lpc != 2 && lpc != 4) || D % lpc != 0 || (lpc > 1 && (D / lpc) % 8 != 0))
        return "rwm_gsn_diag_kernel with a prior: D ≤ 64, 1, 2 or 4 lanes per chain over whole 8-blocks";
    std::ostringstream key, expr, name;
    key << "fprior|" << D << '|' << lpc << '|' << minw << '|' << full << '|' << ll_mode << '|' << unit_t << '|' << shape;
    if (cache_get(key.str(), out)) return "";
    expr << "emcmc::rwm_gsn_diag_kernel<" << D << ", " << lpc << ", " << (full ? "true" : "false") << ", " << ll_mode
         << ", " << (unit_t ? "true" : "false") << ", " << minw << ", emcmc::FusedUpdate<emcmc::" << shape_struct
         << ">>";
    name << "rwm_gsn_diag_kernel<D=" << D << ",LPC=" << lpc << "," << (full ? "FULL" : "ACCEPT_ONLY") << ","
         << (ll_mode == 0 ? "PER_OBS" : "SUFFSTAT") << (unit_t ? ",UNIT_T" : "") << (minw == 2 ? ",MINW=2," : ",")
         << shape_name << "[hiprtc]>";
    const std::string prog_src = "#include \"emcmc_fprior.h\"\n" + shape;
    return compile_kernel(key.str(), prog_src, "fused_prior_kernel.hip", expr.str(), name.str(),
                          {"-ftemplate-depth=2048"}, out, kFusedPriorDeps);
}

const char *rtc_builtin_law(const char *name) {
    for (int i = 0; i < kRtcHeaderCount; ++i)
        if (std::string(kRtcHeaderNames[i]) == name) return kRtcHeaderSrc[i];
    return nullptr;
}

std::string rtc_compile_gsn(int D, bool full, int ll_mode, int nu, RtcKernel &out, const std::string &usrc,
                            const std::string &uopts, bool xt, bool mala) {
    return rtc_compile("", "", D, full, ll_mode, nu, out, usrc, uopts, xt, mala);
}

}  // namespace emcmc
