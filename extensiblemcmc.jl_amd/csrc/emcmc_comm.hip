// emcmc_comm.hip — cross-chain diagnostics over every rank of a job (include/emcmc.h:
// emcmc_comm_*, emcmc_diagnostics).  New functionality: the reference's chain statistics
// are single-chain (src/chain_statistics.jl:16-66); SURVEY.md §8(b)/(e) specifies the
// cross-chain R̂ all-gathered over RCCL.
//
// Each rank reduces its shard on device (emcmc_moments_window: per-dimension m̄, M2 and
// Σvar of its (split-)chain means and variances); the ranks exchange one record of
// 3·D + 3 doubles each with an all-gather — ncclAllGather over xGMI, or the caller's
// host all-gather — and every rank merges the records in rank order with Chan's
// pairwise update, then forms split-R̂.  The merge and R̂ are written in the order of
// extensible_mcmc/diagnostics.py (merge, rhat_from_moments), so the two agree bit for
// bit (-ffp-contract=off; every product and quotient rounded where numpy rounds it).
//
// RCCL is opened with dlopen at the first RCCL call: a process that already holds
// librccl.so.1 (torch's copy) shares it, others get the system's; a host without it
// still loads libemcmc.so and gets EMCMC_RCCL_ERROR from the RCCL calls only.
#include <dlfcn.h>
#include <link.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/emcmc.h"

// emcmc.hip: the handle's device, dimension and last-error slot
int emcmc_internal_device(const emcmc_handle *h);
uint32_t emcmc_internal_dim(const emcmc_handle *h);
void emcmc_internal_set_error(emcmc_handle *h, const std::string &msg);

namespace {

struct Rccl {
    decltype(&::ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&::ncclCommInitRank) init_rank = nullptr;
    decltype(&::ncclAllGather) all_gather = nullptr;
    decltype(&::ncclCommDestroy) destroy = nullptr;
    decltype(&::ncclGetErrorString) error_string = nullptr;
    std::string err;
    bool ok = false;
};

const Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        // The RCCL beside the HIP runtime this library is bound to: a process can hold two
        // HIP runtimes (torch's wheel bundles one, SONAME libamdhip64.so.7 like the system's,
        // and its libraries load it by another name when libemcmc.so came first), and an RCCL
        // of the other runtime cannot use this library's streams.
        std::string dir;
        Dl_info info;
        if (dladdr(reinterpret_cast<void *>(&hipGetDeviceCount), &info) && info.dli_fname) {
            dir = info.dli_fname;
            const size_t sl = dir.rfind('/');
            dir = (sl == std::string::npos) ? std::string() : dir.substr(0, sl + 1);
        }
        void *so = nullptr;
        const std::string cands[] = {dir.empty() ? "" : dir + "librccl.so.1", dir.empty() ? "" : dir + "librccl.so",
                                     "librccl.so.1", "/opt/rocm/lib/librccl.so.1"};
        for (const auto &name : cands)
            if (!name.empty() && (so = dlopen(name.c_str(), RTLD_NOW | RTLD_GLOBAL))) break;
        if (!so) {
            const char *e = dlerror();
            r.err = std::string("cannot open librccl.so.1: ") + (e ? e : "?");
            return;
        }
        r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(so, "ncclGetUniqueId"));
        r.init_rank = reinterpret_cast<decltype(r.init_rank)>(dlsym(so, "ncclCommInitRank"));
        r.all_gather = reinterpret_cast<decltype(r.all_gather)>(dlsym(so, "ncclAllGather"));
        r.destroy = reinterpret_cast<decltype(r.destroy)>(dlsym(so, "ncclCommDestroy"));
        r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(so, "ncclGetErrorString"));
        r.ok = r.get_unique_id && r.init_rank && r.all_gather && r.destroy && r.error_string;
        if (!r.ok) r.err = "librccl.so.1 lacks an nccl* entry point";
    });
    return r;
}

// Every HIP runtime image mapped into this process (dl_iterate_phdr): objects whose file
// name starts with "libamdhip64.so", one per load address.  torch's wheel bundles its own
// runtime; when libemcmc.so is loaded first, torch's libraries load theirs beside it, and
// streams, events and device pointers of one runtime mean nothing to the other (an RCCL of
// the other runtime then fails in ncclCommInitRank).
std::vector<std::string> hip_runtime_images() {
    std::vector<std::pair<uintptr_t, std::string>> seen;
    dl_iterate_phdr(
        [](struct dl_phdr_info *info, size_t, void *p) -> int {
            auto *v = static_cast<std::vector<std::pair<uintptr_t, std::string>> *>(p);
            const char *path = info->dlpi_name ? info->dlpi_name : "";
            const char *base = std::strrchr(path, '/');
            base = base ? base + 1 : path;
            if (std::strncmp(base, "libamdhip64.so", 14) != 0) return 0;
            for (const auto &e : *v)
                if (e.first == (uintptr_t)info->dlpi_addr) return 0;
            v->push_back({(uintptr_t)info->dlpi_addr, path});
            return 0;
        },
        &seen);
    std::vector<std::string> out;
    for (const auto &e : seen) out.push_back(e.second);
    return out;
}

}  // namespace

// why the last emcmc_comm_init / emcmc_comm_unique_id / handle-less merge failed (no comm
// exists to hold it)
thread_local std::string g_comm_err;

namespace {
// the refusal of a process that holds two HIP runtimes (emcmc_comm_init, emcmc_comm_unique_id)
bool two_runtimes(std::string &msg) {
    const std::vector<std::string> imgs = hip_runtime_images();
    if (imgs.size() < 2) return false;
    msg = "this process holds " + std::to_string(imgs.size()) + " HIP runtimes (";
    for (size_t i = 0; i < imgs.size(); ++i) msg += (i ? ", " : "") + imgs[i];
    msg += "): RCCL and the library's streams must share one — import torch (or the caller's HIP "
           "runtime) before libemcmc.so is loaded, or point LD_LIBRARY_PATH at one ROCm";
    return true;
}
}  // namespace

struct emcmc_comm {
    int nranks = 1, rank = 0, device = -1;
    ncclComm_t nccl = nullptr;
    hipStream_t stream = nullptr;
    double *d_buf = nullptr;  // send record + gathered records
    size_t d_cap = 0;         // doubles
    emcmc_allgather_fn fn = nullptr;
    void *ctx = nullptr;
    std::string err;
};

namespace {

emcmc_status comm_fail(emcmc_comm *c, emcmc_status st, const std::string &msg) {
    if (c) c->err = msg;
    return st;
}

// The gathered records [nranks][3D+3] merged in rank order: diagnostics.merge, then
// diagnostics.rhat_from_moments.
emcmc_status merge_records(const double *rows, int nranks, uint32_t D, uint64_t num_draws, emcmc_diag *out,
                           std::string &err) {
    const size_t rec = 3 * (size_t)D + 3;
    std::vector<double> mean(rows + 1, rows + 1 + D), m2(rows + 1 + D, rows + 1 + 2 * D),
        sv(rows + 1 + 2 * D, rows + 1 + 3 * D);
    uint64_t nch = (uint64_t)std::llround(rows[0]);
    uint64_t acc = (uint64_t)std::llround(rows[1 + 3 * D]), prop = (uint64_t)std::llround(rows[2 + 3 * D]);
    for (int r = 1; r < nranks; ++r) {
        const double *b = rows + r * rec;
        const double na = (double)nch, nb = (double)(uint64_t)std::llround(b[0]);
        if (nb == 0.0) continue;
        const double n = na + nb;
        const double fb = nb / n, fab = na * nb / n;
        for (uint32_t d = 0; d < D; ++d) {
            const double dl = b[1 + d] - mean[d];
            mean[d] = mean[d] + dl * fb;
            const double dd = dl * dl;
            m2[d] = (m2[d] + b[1 + D + d]) + dd * fab;
            sv[d] = sv[d] + b[1 + 2 * D + d];
        }
        nch = (uint64_t)n;
        acc += (uint64_t)std::llround(b[1 + 3 * D]);
        prop += (uint64_t)std::llround(b[2 + 3 * D]);
    }
    if (nch < 2) {  // B = n·M2/(m − 1): split-R̂ needs two (half-)chains over all ranks
        err = "split-R̂ needs at least 2 (half-)chains over all ranks, got " + std::to_string(nch);
        return EMCMC_INVALID_ARG;
    }
    const double mch = (double)nch, n = (double)num_draws;
    const double fB = n / ((double)nch - 1.0), fW = (double)(num_draws - 1) / n;
    double mx = -INFINITY;
    bool nan = false;
    for (uint32_t d = 0; d < D; ++d) {
        const double B = fB * m2[d];
        const double W = sv[d] / mch;
        const double vp = fW * W + B / n;
        const double rh = std::sqrt(vp / W);
        if (out->mean) out->mean[d] = mean[d];
        if (out->m2) out->m2[d] = m2[d];
        if (out->sum_var) out->sum_var[d] = sv[d];
        if (out->W) out->W[d] = W;
        if (out->B) out->B[d] = B;
        if (out->rhat) out->rhat[d] = rh;
        if (std::isnan(rh)) nan = true;
        else if (rh > mx) mx = rh;
    }
    out->num_chains = nch;
    out->num_draws = num_draws;
    out->accepted = acc;
    out->proposed = prop;
    out->accept_rate = (double)acc / (double)(prop > 1 ? prop : 1);
    out->max_rhat = nan ? NAN : mx;
    out->dim = D;
    out->nranks = (uint32_t)nranks;
    return EMCMC_OK;
}

#define RCCLCHK(c, expr)                                                                         \
    do {                                                                                         \
        ncclResult_t r_ = (expr);                                                                \
        if (r_ != ncclSuccess)                                                                   \
            return comm_fail((c), EMCMC_RCCL_ERROR, std::string(#expr) + ": " + rccl().error_string(r_)); \
    } while (0)
#define CHIPCHK(c, expr)                                                                         \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            return comm_fail((c), EMCMC_HIP_ERROR, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// all-gather `count` doubles per rank into rows (host, nranks·count)
emcmc_status gather(emcmc_comm *c, const double *send, double *rows, size_t count) {
    if (c->fn) {
        if (c->fn(send, rows, count, c->ctx) != 0) return comm_fail(c, EMCMC_RCCL_ERROR, "host all-gather failed");
        return EMCMC_OK;
    }
    const size_t need = count * (1 + (size_t)c->nranks);
    CHIPCHK(c, hipSetDevice(c->device));
    if (c->d_cap < need) {
        if (c->d_buf) (void)hipFree(c->d_buf);
        c->d_buf = nullptr;
        c->d_cap = 0;
        CHIPCHK(c, hipMalloc(&c->d_buf, need * sizeof(double)));
        c->d_cap = need;
    }
    double *d_send = c->d_buf, *d_recv = c->d_buf + count;
    CHIPCHK(c, hipMemcpyAsync(d_send, send, count * sizeof(double), hipMemcpyHostToDevice, c->stream));
    RCCLCHK(c, rccl().all_gather(d_send, d_recv, count, ncclFloat64, c->nccl, c->stream));
    CHIPCHK(c, hipMemcpyAsync(rows, d_recv, count * c->nranks * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    CHIPCHK(c, hipStreamSynchronize(c->stream));
    return EMCMC_OK;
}

}  // namespace

extern "C" {

emcmc_status emcmc_comm_unique_id(uint8_t id[EMCMC_COMM_ID_BYTES]) {
    if (!id) {
        g_comm_err = "emcmc_comm_unique_id: null id";
        return EMCMC_INVALID_ARG;
    }
    static_assert(sizeof(ncclUniqueId) == EMCMC_COMM_ID_BYTES, "ncclUniqueId size");
    if (two_runtimes(g_comm_err)) return EMCMC_HIP_ERROR;
    int nd = 0;  // RCCL aborts the process when no device is visible: refuse first
    if (hipGetDeviceCount(&nd) != hipSuccess || nd == 0) {
        g_comm_err = "emcmc_comm_unique_id: no HIP device visible";
        return EMCMC_NO_DEVICE;
    }
    if (!rccl().ok) {
        g_comm_err = rccl().err;
        return EMCMC_RCCL_ERROR;
    }
    ncclUniqueId u;
    if (const ncclResult_t r = rccl().get_unique_id(&u); r != ncclSuccess) {
        g_comm_err = std::string("ncclGetUniqueId: ") + rccl().error_string(r);
        return EMCMC_RCCL_ERROR;
    }
    std::memcpy(id, &u, sizeof u);
    return EMCMC_OK;
}

emcmc_status emcmc_comm_init(emcmc_comm **out, int nranks, int rank, int device,
                             const uint8_t id[EMCMC_COMM_ID_BYTES]) {
    if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks || device < 0) {
        g_comm_err = "emcmc_comm_init: invalid argument (null out/id, or rank/nranks/device out of range)";
        return EMCMC_INVALID_ARG;
    }
    *out = nullptr;
    if (two_runtimes(g_comm_err)) return EMCMC_HIP_ERROR;
    if (!rccl().ok) {
        g_comm_err = rccl().err;
        return EMCMC_RCCL_ERROR;
    }
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || nd == 0) {
        g_comm_err = "emcmc_comm_init: no HIP device visible";
        return EMCMC_NO_DEVICE;
    }
    if (device >= nd) {
        g_comm_err = "emcmc_comm_init: device " + std::to_string(device) + " of " + std::to_string(nd);
        return EMCMC_INVALID_ARG;
    }
    auto *c = new emcmc_comm;
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        g_comm_err = std::string("emcmc_comm_init: hipSetDevice / hipStreamCreateWithFlags: ") +
                     hipGetErrorString(hipGetLastError());
        delete c;
        return EMCMC_HIP_ERROR;
    }
    if (const ncclResult_t r = rccl().init_rank(&c->nccl, nranks, u, rank); r != ncclSuccess) {
        g_comm_err = std::string("ncclCommInitRank: ") + rccl().error_string(r);
        (void)hipStreamDestroy(c->stream);
        delete c;
        return EMCMC_RCCL_ERROR;
    }
    *out = c;
    return EMCMC_OK;
}

emcmc_status emcmc_comm_init_host(emcmc_comm **out, int nranks, int rank, emcmc_allgather_fn fn, void *ctx) {
    if (!out || !fn || nranks < 1 || rank < 0 || rank >= nranks) {
        g_comm_err = "emcmc_comm_init_host: invalid argument (null out/fn, or rank/nranks out of range)";
        return EMCMC_INVALID_ARG;
    }
    auto *c = new emcmc_comm;
    c->nranks = nranks;
    c->rank = rank;
    c->fn = fn;
    c->ctx = ctx;
    *out = c;
    return EMCMC_OK;
}

void emcmc_comm_destroy(emcmc_comm *c) {
    if (!c) return;
    if (c->nccl) {
        (void)hipSetDevice(c->device);
        if (c->stream) (void)hipStreamSynchronize(c->stream);
        rccl().destroy(c->nccl);
    }
    if (c->d_buf) (void)hipFree(c->d_buf);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char *emcmc_comm_last_error(const emcmc_comm *c) {
    if (!c) return g_comm_err.c_str();  // the calling thread's last failed init / unique id
    return c->err.c_str();
}

emcmc_status emcmc_diagnostics_merge(emcmc_comm *c, const double *record, uint32_t dim, uint64_t num_draws,
                                     emcmc_diag *out) {
    if (!record || !out || dim == 0 || num_draws < 1) return EMCMC_INVALID_ARG;
    const size_t rec = 3 * (size_t)dim + 3;
    const int nranks = c ? c->nranks : 1;
    std::vector<double> rows(rec * nranks);
    if (c) {
        emcmc_status st = gather(c, record, rows.data(), rec);
        if (st) return st;
    } else {
        std::memcpy(rows.data(), record, rec * sizeof(double));
    }
    std::string err;
    const emcmc_status st = merge_records(rows.data(), nranks, dim, num_draws, out, err);
    if (st) {
        if (c) c->err = err;
        else g_comm_err = err;
    }
    return st;
}

int emcmc_hip_runtime_images(char *paths_out, size_t len) {
    const std::vector<std::string> imgs = hip_runtime_images();
    std::string all;
    for (size_t i = 0; i < imgs.size(); ++i) all += (i ? "\n" : "") + imgs[i];
    if (paths_out && len) {
        const size_t n = std::min(all.size(), len - 1);
        std::memcpy(paths_out, all.data(), n);
        paths_out[n] = '\0';
    }
    return (int)imgs.size();
}

emcmc_status emcmc_diagnostics(emcmc_handle *h, emcmc_comm *c, uint64_t iter_first, uint64_t num_iters, int split,
                               emcmc_diag *out) {
    if (!h || !out) return EMCMC_INVALID_ARG;
    if (c && c->nccl && c->device != emcmc_internal_device(h)) {
        emcmc_internal_set_error(h, "emcmc_diagnostics: the RCCL comm is on another device than the handle");
        return EMCMC_INVALID_ARG;
    }
    const uint32_t D = emcmc_internal_dim(h);
    std::vector<double> record(3 * (size_t)D + 3);
    emcmc_moments info{};
    emcmc_status st = emcmc_moments_window(h, iter_first, num_iters, split, record.data() + 1, &info);
    if (st) return st;
    record[0] = (double)info.num_chains;
    record[1 + 3 * D] = (double)info.accepted;
    record[2 + 3 * D] = (double)info.proposed;
    st = emcmc_diagnostics_merge(c, record.data(), D, info.num_draws, out);
    if (st) emcmc_internal_set_error(h, std::string("emcmc_diagnostics: ") + (c ? c->err : g_comm_err));
    return st;
}

}  // extern "C"
