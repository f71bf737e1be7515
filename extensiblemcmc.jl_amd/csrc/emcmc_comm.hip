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
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdio>
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

}  // namespace

// why the last emcmc_comm_init / emcmc_comm_unique_id failed (no comm exists to hold it)
thread_local std::string g_comm_err;

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
void merge_records(const double *rows, int nranks, uint32_t D, uint64_t num_draws, emcmc_diag *out) {
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
    const double mch = (double)nch, n = (double)num_draws;
    const double fB = n / (double)(nch - 1), fW = (double)(num_draws - 1) / n;
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
    if (!id) return EMCMC_INVALID_ARG;
    static_assert(sizeof(ncclUniqueId) == EMCMC_COMM_ID_BYTES, "ncclUniqueId size");
    int nd = 0;  // RCCL aborts the process when no device is visible: refuse first
    if (hipGetDeviceCount(&nd) != hipSuccess || nd == 0) return EMCMC_NO_DEVICE;
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
    if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks || device < 0) return EMCMC_INVALID_ARG;
    *out = nullptr;
    if (!rccl().ok) {
        g_comm_err = rccl().err;
        return EMCMC_RCCL_ERROR;
    }
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || nd == 0) return EMCMC_NO_DEVICE;
    if (device >= nd) return EMCMC_INVALID_ARG;
    auto *c = new emcmc_comm;
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
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
    if (!out || !fn || nranks < 1 || rank < 0 || rank >= nranks) return EMCMC_INVALID_ARG;
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
    merge_records(rows.data(), nranks, dim, num_draws, out);
    return EMCMC_OK;
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
    if (st && c) emcmc_internal_set_error(h, std::string("emcmc_diagnostics: ") + c->err);
    return st;
}

}  // extern "C"
