// engine.cpp -- host side of the qvq engine: context, per-level schedule, kd-tree builds,
// RCCL exchange and the C ABI of include/qvq.h.  No kernels here; the HIP kernels and
// their launch wrappers live in k_assign.hip and k_misc.hip.
//
// Per split level (LBGIterate, src/Quantizer.cpp:98-108, one effective Lloyd step), all on
// one stream with no host round trip:
//   D == 12, K <= mf_fuse_max_k():  search (fused exact sums) -> recheck -> kd_resolve
//                                   -> reduce -> [all-reduce] -> finalize+split+tables
//   otherwise:                      search (MFMA or VALU) -> recheck -> kd_resolve -> update
//                                   -> reduce -> [all-reduce] -> finalize+split+tables
// While the GPU runs a level's search, the host builds the reference kd-tree over that
// level's codebook (which the previous finalize wrote to mapped memory) for kd_resolve.  A
// tree too large for the kernel's LDS falls back to a synchronous host resolution of the tie
// rows (resolve_host_ties).  A quantize starts with the mean kernel and ends with one
// copy_out launch into mapped memory, whose completion flag the host polls.
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <rccl/rccl.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <memory>
#include <unordered_map>
#include <vector>

#include "common.hpp"
#include "kdtree.hpp"
#include "qvq.h"
#include "wait.hpp"

namespace qvq {

// src/ColorSpace.cpp:4-6 (NORMAL) and :16-21 (SCALED, reciprocal multiply under fast-math)
static double cs_value(int cs, int b) {
    const double s = (double)(signed char)(unsigned char)b;
    return cs == QVQ_CS_NORMAL ? s : (s + 128.0) * (1.0 / 255);
}

bool make_terms(int cs, Terms &t) {
    if (cs != QVQ_CS_NORMAL && cs != QVQ_CS_SCALED) return false;
    const bool scaled = cs == QVQ_CS_SCALED;
    t.scale = scaled ? 60 : 0;
    t.vmax = 0;
    // u = (int8)b + 128 orders the bytes by value: SCALED v = fl(u * fl(1/255)),
    // NORMAL v = u - 128.  q = R*u + E with |E| <= 64 (SCALED) or E = -128 (NORMAL).
    t.R = scaled ? (int64_t)std::ldexp(1.0 / 255, 60) : 1;
    t.mu = scaled ? 0.5 : -0.5;
    t.sx = scaled ? (1.0 / 255) / 2 : 0.5;
    int64_t E[256], emax = 0;
    for (int b = 0; b < 256; b++) {
        t.v64[b] = cs_value(cs, b);
        t.v32[b] = (float)t.v64[b];
        t.vmax = std::max(t.vmax, std::fabs(t.v64[b]));
        const double qd = std::ldexp(t.v64[b], t.scale);
        if (qd != std::floor(qd)) return false;
        const int64_t u = (int64_t)(signed char)(unsigned char)b + 128;
        E[b] = (int64_t)qd - t.R * u;
        emax = std::max<int64_t>(emax, E[b] < 0 ? -E[b] : E[b]);
        t.hi[b] = (uint32_t)u;
        t.w[b] = (float)(2 * u - 255);   // v - mu = w * sx (exactly, up to fl() of v)
    }
    t.bias = emax;
    for (int b = 0; b < 256; b++) t.lo[b] = (uint32_t)(E[b] + t.bias);
    t.pad_code = scaled ? 0x80 : 0x00;
    return t.v64[t.pad_code] == 0.0;
}

}  // namespace qvq

using namespace qvq;

constexpr uint32_t SCHED_COUNTERS = 2 * 33 + 2, N_COUNTERS = SCHED_COUNTERS + 2;
// Levels whose kd-tree the device builds (k_kdbuild.hip, beside the search): K * D from this up
// (C4's 48-D levels from K = 512; C3's 12-D trees take the host well under 0.1 ms).
constexpr uint64_t KDB_MIN_KD = 16384;

namespace qvq {
// One level's tie certificate (engine.cpp certify_rows): the level's distinct tie
// rows, the split as far as its reference bits are known, the answers; with several ranks the
// rows left open and the cells they need wait for the end of the quantize (cert_finish).
struct CertState {
    std::vector<double> qs;           // distinct tie rows (nu x D values)
    uint32_t nu = 0;
    std::vector<uint32_t> of;         // tie record -> distinct row
    std::vector<uint32_t> rows, spec; // the tie records: row, speculative index
    std::vector<double> kp;           // the reference's split where known
    std::vector<uint8_t> known;
    std::vector<int64_t> ans;         // per distinct row: the reference's index, -1 open
    std::vector<uint32_t> pend;       // distinct rows still open
    std::vector<uint8_t> sel;         // [K/2] the parent cells those rows need
    uint32_t cells = 0, rounds = 0;
    bool prepared = false;            // kp / known set and the tree's replay state built (cert_init)
};
}  // namespace qvq

// QVQ_HOST_TRACE=1: a host timeline of each qvq_lbg (us since its start, per thread), printed
// to stderr at its end: the main thread's tree builds and enqueues, the checks' start, export
// and end (diagnostics for where a quantize waits).  One per context: the checks of a context
// mark it from its worker thread while the calling thread does.
struct HostTrace {
    std::atomic<bool> on{false};
    std::chrono::steady_clock::time_point t0;
    std::mutex m;
    std::vector<std::pair<double, std::string>> ev;
    void start(std::chrono::steady_clock::time_point t) {
        std::lock_guard<std::mutex> g(m);
        t0 = t;
        ev.clear();
        on.store(true, std::memory_order_release);
    }
    void mark(const std::string &what) {
        if (!on.load(std::memory_order_acquire)) return;
        std::lock_guard<std::mutex> g(m);
        const double t = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        ev.emplace_back(t, what);
    }
    std::string finish() {
        std::lock_guard<std::mutex> g(m);
        on.store(false, std::memory_order_release);
        // (t0 in steady_clock ns -- CLOCK_MONOTONIC, the clock of rocprofv3's timestamps)
        std::string out = "qvq host trace: t0_ns " +
                          std::to_string(std::chrono::duration_cast<std::chrono::nanoseconds>(t0.time_since_epoch()).count());
        for (const auto &e : ev) out += "\n  " + std::to_string((int)e.first) + " " + e.second;
        return out;
    }
};

struct qvq_ctx {
    int dev = 0;
    int num_cu = 256;
    hipStream_t stream = nullptr;
    std::string err;

    // training set
    uint64_t N = 0;
    uint32_t D = 0, Dp = 0;
    // exact mode (qvq_set_vectors_exact, or qvq_set_vectors on values that are not byte images):
    // the fp64 rows themselves and the reference's Kahan arithmetic (k_exact.hip)
    bool exact = false;
    double *d_X64 = nullptr;
    uint32_t *d_ex_keys = nullptr, *d_ex_iota = nullptr, *d_ex_order = nullptr;
    void *d_ex_temp = nullptr;
    size_t ex_temp_bytes = 0;
    uint32_t *d_ex_koff = nullptr;
    uint32_t ex_kcap = 0;
    int cs = -1;
    Terms terms;
    int mf_t = 0;            // MFMA score scale exponent
    MfThresholds mf_th{};
    uint8_t *d_codes = nullptr;
    float *d_lut32 = nullptr, *d_w = nullptr;
    double *d_lut64 = nullptr;
    uint64_t *d_plut = nullptr;
    uint32_t *d_A = nullptr, *d_flags = nullptr, *d_ties = nullptr;
    // the previous level's final assignment (qvq_lbg swaps the two each level): the input of
    // the reference-bit (Kahan) centroids a level with kd-tree ties needs
    uint32_t *d_A_alt = nullptr;
    KahanWork kw;
    double *d_kc_cent = nullptr, *d_kc_split = nullptr;   // Kahan centroids [K/2][D], their split [K][D]
    uint32_t kc_kcap = 0;
    std::vector<double> h_kc_split;   // host copy of the split for the tree build
    uint32_t *d_kc_sel = nullptr;     // [K/2] slot + 1 of the cells a tie certificate sums (0: not summed)
    uint32_t *h_kc_sel = nullptr;     // its pinned host side
    double *h_kc_out = nullptr, *dh_kc_out = nullptr;   // [K][D] mapped: the selected cells' split rows
    std::vector<double> cert_kp;      // the reference's split where known (tie certificate)
    std::vector<uint8_t> cert_known;
    std::vector<uint32_t> cert_vals;  // the certified answers (host side of their upload)
    uint64_t pub_seq = 0;          // per-level tie-count publications (h_ready[1] = seq, h_ready[2] = ties)
    double tie_abs = 0;            // the recheck's absolute tie band: centroid bits may differ by this much
    unsigned *d_counters = nullptr;   // per level: [2l] flagged rows, [2l+1] kd-tree ties; [66], [67] block counters;
                                      // [68], [69] the pruned wide search's task counters (SCHED_COUNTERS)
    uint64_t *d_hist = nullptr;       // byte histogram [256] | its all-reduced copy [256]

    // level buffers
    uint32_t Kcap = 0;
    uint32_t G = 0;   // workgroup slabs
    double *d_C64_cent = nullptr, *d_C64_split = nullptr;
    double *d_C64_split_alt = nullptr;   // qvq_lbg's next split while d_C64_split may still be needed
    float *d_C32 = nullptr;
    float *d_E32 = nullptr;   // D = 12: expanded fp32 terms for the small-K scan
    _Float16 *d_rows = nullptr;   // MFMA code-vector rows
    uint32_t *d_perm = nullptr;   // pruned search: tile order of the split codebook (finalize's prune_order)
    int32_t *d_tint = nullptr;    // ... and the tiles' projection envelopes
    uint32_t perm_k = 0;          // the K whose order d_perm holds (0: none)
    uint64_t *d_part = nullptr, *d_sums = nullptr;
    uint32_t *d_part_cnt = nullptr;
    double *d_dist_part = nullptr;
    uint64_t *d_mean = nullptr;   // MEAN_COPIES x mean sums [hi D][lo D][n]: zero between quantizes (the finalize clears them)
    uint64_t out_seq = 0;         // quantizes whose results copy_out has published
    uint32_t *d_scatter = nullptr;
    uint32_t *d_sortbuf = nullptr;   // sorted-order sums: idx [N] | ks [N]
    uint64_t scatter_bytes = 0;
    uint8_t *d_raster = nullptr;          // qvq_set_images' raster upload buffer (grown on demand)
    uint64_t raster_bytes = 0;
    uint8_t *d_decode = nullptr;          // qvq_decode scratch (grown on demand)
    uint64_t decode_bytes = 0;
    uint64_t *d_decode_stat = nullptr;    // decode: [squared error, bad-index flag]
    uint64_t *h_decode_stat = nullptr;    // pinned host copy
    // mapped pinned host memory (coherent): the split codebook finalize writes for the
    // host's tree build, its ready sequence number, and two flattened kd-tree images
    // the split codebooks the finalizes publish for the host, two halves of cb_half doubles
    // (host_cb_of): level L's codebook in half L & 1
    double *h_cb = nullptr, *dh_cb = nullptr;
    uint64_t cb_half = 0;
    uint64_t *h_ready = nullptr, *dh_ready = nullptr;
    uint64_t seq = 0;
    uint8_t *h_tree[2] = {nullptr, nullptr}, *dh_tree[2] = {nullptr, nullptr};
    uint8_t *d_tree = nullptr;   // device copy of the level's tree image (one DMA per level)
    // the level's kd-tree built on the device (k_kdbuild.hip) on kstream, beside the search:
    // scratch (vind, nodes, boxes), the mapped host image of the whole tree, its launch number
    hipStream_t kstream = nullptr;
    hipEvent_t ev_kcb = nullptr, ev_kdb = nullptr;
    uint32_t *d_kdb_vind = nullptr;
    KdbNode *d_kdb_nodes = nullptr;
    double *d_kdb_nbox = nullptr, *d_kdb_cbox = nullptr;
    uint8_t *h_kdb = nullptr, *dh_kdb = nullptr;
    uint32_t kdb_cap = 0;   // code vectors the scratch takes (0: none)
    uint64_t kdb_seq = 0;
    std::vector<double> cb_local;   // host copy of the published codebook for the tree build
    std::vector<uint32_t> cnt_local;   // ... and of its parent cells' row counts (empty: not known)
    std::unique_ptr<RefKDTree> tree;   // the last level's tree over cb_local
    KdView tree_kd;                    // and its device image (depth 0: none)
    // deferred-tie levels build their tree on this worker, off the launch path (start_tree_job)
    struct Worker {   // one host thread, jobs in order
        std::thread th;
        std::mutex m;
        std::condition_variable cv;
        std::deque<std::function<void()>> q;
        bool stop = false;
        std::atomic<int> pending{0};
    } worker;
    // helpers of the worker for the certificate's replays (persistent: their per-thread replay
    // caches stay warm); pool_run forks fn over them and the calling thread
    struct Pool {
        std::vector<std::thread> th;
        std::mutex m;
        std::condition_variable cv;
        std::function<void(uint32_t)> fn;
        std::atomic<uint64_t> epoch{0};
        std::atomic<uint32_t> want{0}, busy{0};
        std::atomic<bool> stop{false};
    } pool;
    // one rank: the CPUs of the L3 domain the first quantize ran on (host_place)
    bool place_tried = false, place_ok = false;
    cpu_set_t place;
    // the speculative Kahan check (qvq_lbg): level L's ties verified on the worker while the GPU
    // runs levels L + 1 and L + 2; four assignment buffers keep A_{L-1} (the check's cells)
    // until level L + 3, when the check is joined
    uint32_t *d_A3 = nullptr, *d_A4 = nullptr;
    uint8_t *h_tx[3] = {nullptr, nullptr, nullptr}, *dh_tx[3] = {nullptr, nullptr, nullptr};   // TieExport, level % 3
    uint32_t tx_cap = 0;
    hipStream_t vstream = nullptr;   // the check's selected Kahan sums
    struct Verify {
        bool posted = false;
        std::atomic<bool> done{true}, cancel{false};
        int status = 0;   // 0: the reference's indices are the speculative ones; 1: not shown; 2: deferred
        uint32_t K = 0, level = 0;
        uint64_t seq = 0;
        int par = 0;
        const uint32_t *A_prev = nullptr;
        std::unique_ptr<RefKDTree> tree;
        std::vector<double> cb;
        std::vector<uint32_t> cnt;   // the parent cells' row counts (empty: not known)
        CertState cs;
        hipEvent_t ev = nullptr;
    } ver[3];   // level % 3
    // several ranks: the checks whose rows wait for cells summed over every rank's rows (status
    // 2), finished together at the end of qvq_lbg; A_prev stays valid (one assignment buffer per
    // level, d_Aext)
    struct Deferred {
        uint32_t level = 0, K = 0;
        const uint32_t *A_prev = nullptr;
        std::unique_ptr<RefKDTree> tree;
        std::vector<double> cb;
        CertState cs;
    };
    std::vector<Deferred> deferred;
    std::vector<uint32_t *> d_Aext;   // assignment buffers beyond the four (several ranks: one per level)
    uint64_t *d_vote = nullptr, *h_vote = nullptr;   // the ranks' small all-reduced decisions (qvq_lbg)
    uint64_t vote_cap = 0;
    uint64_t *d_kc_chain = nullptr;   // chained Kahan sums: gather | state (k_kahan.hip)
    uint64_t kc_chain_cap = 0;
    std::atomic<bool> tree_cancel{false};
    bool tree_job = false, job_ok = false;
    int job_buf = 0;
    KdView job_kd;
    uint64_t tree_cap = 0;
    uint32_t nslabs = 0;   // slabs holding the last run_level's sums
    uint32_t col_blocks = 0;   // blocks per image column (consecutive rows run down a column); 0: no image
    bool kd_pend = false;      // run_level left its kd-tree ties to kd_reduce_kernel (pend_kd)
    PubArgs pub;               // run_level left its tie-count publication to the next reduce
    uint32_t sums_copies = 1;  // 2: run_level's tie moves are in copy 1 of d_sums (the finalize adds it)
    KdView pend_kd{};
    bool sums1_dirty = false;  // copy 1 of d_sums may hold moves (a quantize that stopped early)
    uint64_t sums_bytes = 0;
    uint32_t nsub = 0;     // ... of which the last nsub are subtracted
    int timing_level = -2;   // qvq_set_timing: -1 all levels, -2 none (default), else that level only
    bool upd[32] = {};
    hipEvent_t ev_end = nullptr;
    hipEvent_t ev_sync = nullptr;   // wait_stream
    double timeout_s = 120;         // bound of every host wait (qvq_set_timeout, QVQ_TIMEOUT_S)

    // multi-GPU: an RCCL communicator, or (tests) a host all-reduce callback
    ncclComm_t comm = nullptr;
    qvq_allreduce_fn host_ar = nullptr;
    void *host_ar_user = nullptr;
    void *h_ar_stage = nullptr;   // pinned staging of the host all-reduce
    uint64_t ar_stage_bytes = 0;
    int nranks = 1, rank = 0;
    // a bounded wait failed while work may still be queued on the stream: every later call
    // returns QVQ_ESTATE until qvq_destroy (results must not land in freed memory,
    // and the stream's scratch must not be reused under running kernels)
    bool poisoned = false;
    void *h_stage = nullptr;      // pinned staging of qvq_update's results
    uint64_t stage_bytes = 0;

    qvq_timings tm;
    HostTrace htrace;
    hipEvent_t ev[32][4];
    bool ev_ready = false;
};

namespace {

thread_local std::string g_static_err;

qvq_status fail(qvq_ctx *c, qvq_status st, const std::string &msg) {
    if (c) c->err = msg;
    else g_static_err = msg;
    return st;
}

// Entry points that use the device refuse a poisoned context (wait_failed).
#define GUARD(ctx)                                                                                    \
    do {                                                                                              \
        if (!(ctx)) return QVQ_EINVAL;                                                                \
        if ((ctx)->poisoned)                                                                          \
            return fail((ctx), QVQ_ESTATE, "context poisoned by an earlier failed wait; destroy it"); \
    } while (0)

#define HIPCHK(expr)                                                                                  \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess)                                                                         \
            return fail(ctx, QVQ_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));         \
    } while (0)

#define NCCLCHK(expr)                                                                                 \
    do {                                                                                              \
        ncclResult_t r_ = (expr);                                                                     \
        if (r_ != ncclSuccess)                                                                        \
            return fail(ctx, QVQ_ECOMM, std::string(#expr) + ": " + ncclGetErrorString(r_));          \
    } while (0)

template <typename T>
void dfree(T *&p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

uint32_t pad32(uint32_t K) { return (K + 31) & ~31u; }   // MFMA tile pairs
bool kahan_mode(const qvq_ctx *ctx);
double tie_band(const qvq_ctx *ctx);
// The path knobs a test exercises: QVQ_SEARCH=valu (the VALU search at every K) and
// QVQ_KDTREE=host (ties answered on the host); QVQ_KAHAN=0 / QVQ_SPECULATE=0 (index rule and
// schedule); QVQ_KAHAN_FAIL_LEVEL / _RANK (forced check failures).
bool env_is(const char *name, const char *val) {
    const char *v = std::getenv(name);
    return v && std::strcmp(v, val) == 0;
}
bool use_mfma(const qvq_ctx *ctx, uint32_t K) {
    return ctx->D == MF_D && mf_can_search(K) && !env_is("QVQ_SEARCH", "valu");
}
// MFMA search for D != 12 from K = 128 code vectors up: below it the VALU search wins (C4,
// D = 48: 82 vs 182 us at K = 32, 154 vs 187 at K = 64; from K = 64 or 32 the C4 levels ran
// slower, profiles/r05ak).
constexpr uint32_t WIDE_MIN_K = 128;
bool use_wide(const qvq_ctx *ctx, uint32_t K) {
    return ctx->D != MF_D && wide_can_search(ctx->Dp) && K >= WIDE_MIN_K && !env_is("QVQ_SEARCH", "valu");
}
bool use_fused(const qvq_ctx *ctx, uint32_t K) { return use_mfma(ctx, K) && K <= mf_fuse_max_k(); }
// Pruned MFMA search (k_mf32.hip PRUNE: tiles outside a chunk's provable window skipped) for
// D = 12 from K = 256 (from K = 128 it measured slower, profiles/r05ao) up to prune_order's
// capacity.  Its order is computed by the previous level's finalize.  Other D
// (assign_wide_kernel, streamed codebooks): from K = 1024; a codebook resident in LDS (small D)
// is searched unpruned: its per-wave windows measured no faster.
// The D = 12 kernel keeps one tile envelope per lane: at most 64 tiles (K <= 2048).
constexpr uint32_t PRUNE_MIN_K = 256, WPRUNE_MIN_K = 1024;
bool use_prune(const qvq_ctx *ctx, uint32_t K) {
    if (K > PRUNE_MAXK_HOST) return false;
    if (ctx->D == MF_D)
        return K >= PRUNE_MIN_K && K <= 2048 && use_mfma(ctx, K) && mf32_prune_fits(K, use_fused(ctx, K));
    if (wide_codebook_resident(ctx->Dp, K)) return false;
    return K >= WPRUNE_MIN_K && use_wide(ctx, K) && wide_prune_fits(ctx->Dp, K);
}

void free_kahan_work(KahanWork &w) {
    for (uint32_t **p : {&w.hist, &w.tot, &w.koff, &w.segoff, &w.blkoff}) dfree(*p);
    dfree(w.planes);
    dfree(w.stats);
    for (void **p : {&w.meta, &w.bsum, &w.bfn, &w.sfn, &w.bfn8, &w.tab})
        if (*p) (void)hipFree(*p), *p = nullptr;
    w.seg_cap = w.blk_cap = w.n_cap = 0;
    w.k_cap = w.d_cap = 0;
}

void free_kahan(qvq_ctx *ctx) {
    free_kahan_work(ctx->kw);
    dfree(ctx->d_kc_chain);
    ctx->kc_chain_cap = 0;
    dfree(ctx->d_kc_cent);
    dfree(ctx->d_kc_split);
    dfree(ctx->d_kc_sel);
    if (ctx->h_kc_sel) (void)hipHostFree(ctx->h_kc_sel);
    if (ctx->h_kc_out) (void)hipHostFree(ctx->h_kc_out);
    ctx->h_kc_sel = nullptr;
    ctx->h_kc_out = ctx->dh_kc_out = nullptr;
    ctx->kc_kcap = 0;
}

void free_training(qvq_ctx *ctx) {
    free_kahan(ctx);
    dfree(ctx->d_A_alt);
    dfree(ctx->d_A3);
    dfree(ctx->d_A4);
    for (uint32_t *&p : ctx->d_Aext) dfree(p);
    ctx->d_Aext.clear();
    ctx->deferred.clear();
    dfree(ctx->d_X64);
    dfree(ctx->d_ex_keys);
    dfree(ctx->d_ex_iota);
    dfree(ctx->d_ex_order);
    if (ctx->d_ex_temp) (void)hipFree(ctx->d_ex_temp);
    ctx->d_ex_temp = nullptr;
    ctx->ex_temp_bytes = 0;
    dfree(ctx->d_ex_koff);
    ctx->ex_kcap = 0;
    ctx->exact = false;
    dfree(ctx->d_sortbuf);
    dfree(ctx->d_codes);
    dfree(ctx->d_A);
    dfree(ctx->d_flags);
    dfree(ctx->d_ties);
    ctx->N = 0;
    ctx->D = ctx->Dp = 0;
}

void free_levels(qvq_ctx *ctx) {
    dfree(ctx->d_C64_cent);
    dfree(ctx->d_C64_split);
    dfree(ctx->d_C64_split_alt);
    dfree(ctx->d_C32);
    dfree(ctx->d_E32);
    dfree(ctx->d_rows);
    dfree(ctx->d_perm);
    dfree(ctx->d_tint);
    ctx->perm_k = 0;
    dfree(ctx->d_part);
    dfree(ctx->d_part_cnt);
    dfree(ctx->d_sums);
    if (ctx->h_cb) (void)hipHostFree(ctx->h_cb);
    ctx->h_cb = ctx->dh_cb = nullptr;
    for (int b = 0; b < 2; b++) {
        if (ctx->h_tree[b]) (void)hipHostFree(ctx->h_tree[b]);
        ctx->h_tree[b] = ctx->dh_tree[b] = nullptr;
    }
    dfree(ctx->d_tree);
    ctx->tree_cap = 0;
    dfree(ctx->d_kdb_vind);
    dfree(ctx->d_kdb_nodes);
    dfree(ctx->d_kdb_nbox);
    dfree(ctx->d_kdb_cbox);
    if (ctx->h_kdb) (void)hipHostFree(ctx->h_kdb);
    ctx->h_kdb = ctx->dh_kdb = nullptr;
    ctx->kdb_cap = 0;
    ctx->Kcap = 0;
}

bool device_tree_on();
// Flattened tree: root box lo[D], hi[D] | nodes[<= 2K] | vind[K].
uint64_t tree_bytes(uint32_t K, uint32_t D) {
    return 16ull * D + (2ull * K + 1) * sizeof(KdNodeDev) + 4ull * K;
}

// MFMA score scale and error bounds for the near-tie flag ("near-tie flags").
void mfma_setup(qvq_ctx *ctx) {
    const Terms &t = ctx->terms;
    const double D = ctx->D;
    // centroids are means of data values, the split scales them by 1.2 or 0.8
    double vmin = 1e300, vmax = -1e300, wmax = 0;
    for (int b = 0; b < 256; b++) {
        vmin = std::min(vmin, t.v64[b]);
        vmax = std::max(vmax, t.v64[b]);
        wmax = std::max(wmax, (double)std::fabs(t.w[b]));
    }
    const double cmin = std::min(1.2 * vmin, 0.8 * vmin), cmax = std::max(1.2 * vmax, 0.8 * vmax);
    const double cp = std::max(std::fabs(cmin - t.mu), std::fabs(cmax - t.mu));   // max |c - mu|
    const double n_max = D * cp * cp;
    const double c2_max = 2 * t.sx * cp;
    const double s_bound = n_max + D * wmax * c2_max;    // sum of |terms| of one score, unscaled
    int tt = 0;
    while (std::ldexp(n_max, tt + 1) <= 60000.0 && std::ldexp(s_bound, tt + 1) <= 120000.0) tt++;
    while (std::ldexp(n_max, tt) > 60000.0 || std::ldexp(s_bound, tt) > 120000.0) tt--;
    ctx->mf_t = tt;
    const double u = std::ldexp(1.0, -24);
    // one MFMA score: <= (slots + 1) sequential fp32 roundings over the terms (D = 12: 32
    // slots in one MFMA; wide layout: KS chained MFMAs of 32 slots), the f16 hi/lo split
    // (2^-22 relative + 2^-25 absolute per operand, scaled back), the fp32 scale/shift of
    // the score and of ||x - mu||^2, x ~ mu + w*sx (2^-53)
    const double rounds = ctx->D == MF_D ? 33.0 : 32.0 * wide_ks(ctx->Dp) + 1.0;
    const double e_acc = rounds * u * s_bound;
    const double e_rep = D * wmax * (c2_max * std::ldexp(1.0, -22) + std::ldexp(1.0, -25 - tt)) +
                         n_max * std::ldexp(1.0, -22) + std::ldexp(1.0, -25 - tt);
    const double e_conv = 4 * u * (s_bound + D * cp * cp) + 1e-12 * s_bound;
    ctx->mf_th.mfma = (float)(1.25 * (e_acc + e_rep + e_conv));
    // The same bound for one row, with sum_d |w_d| of that row in place of D * wmax (every term
    // above is linear in it): S_row = n_max + c2_max * sum|w| replaces s_bound.
    {
        const double ew = std::ldexp(1.0, -25 - tt);
        const double a0 = rounds * u * n_max + (n_max * std::ldexp(1.0, -22) + ew) + 4 * u * (n_max + D * cp * cp) +
                          1e-12 * n_max;
        const double a1 = rounds * u * c2_max + (c2_max * std::ldexp(1.0, -22) + ew) + 4 * u * c2_max + 1e-12 * c2_max;
        ctx->mf_th.m0 = (float)(1.25 * a0 * 1.0001);
        ctx->mf_th.m1 = (float)(1.25 * a1 * 1.0001);
    }
    // direct-form fp32 recompute (same bound as the VALU search)
    const double L = std::sqrt(D) * (std::max(std::fabs(vmin), std::fabs(vmax)) + std::max(std::fabs(cmin), std::fabs(cmax))) * 1.001;
    ctx->mf_th.alpha = (float)(3.0 * 4.01 * u * L);   // x in fp32 is mu + w*sx: <= 2u relative
    ctx->mf_th.beta = (float)(2.0 * ((ctx->Dp + 4) * u * 1.01 + 4e-15));
    ctx->mf_th.gamma = (float)(2.0 * 4.01 * u * u * L * L + 1e-30);
    ctx->mf_th.inv_scale = (float)std::ldexp(1.0, -tt);
    // small-K scan (assign_small_kernel): each expanded score is an fp32 fma chain from n over
    // the D terms w_d * c''_d, with n and c'' rounded to fp32 once and w exact, so its error is
    // at most (D + 1) u (1 + u)^D (n + sum_d |w_d| |c''_d|) <= (D + 2) u S_row; two scores are
    // compared.  S_row <= 2^t (n_max + c2_max sum_d |w_d|), plus a 1e-11 relative floor for the
    // reference's own fp64 rounding (as e_conv above).
    const double sc = std::ldexp(1.0, tt);
    const double ks = 2.0 * (D + 2) * u * 1.01;
    ctx->mf_th.e0 = (float)((ks * n_max + 1e-11 * s_bound) * sc * 1.0001);
    ctx->mf_th.e1 = (float)(ks * c2_max * sc * 1.0001);
    ctx->mf_th.mu = (float)t.mu;
    ctx->mf_th.sx = (float)t.sx;
}

// Allocate the per-row buffers and upload the colour-space tables.
qvq_status alloc_training(qvq_ctx *ctx, uint64_t N, uint32_t D, int cs) {
    if (N == 0 || D == 0) return fail(ctx, QVQ_EINVAL, "empty training set");
    if (N >= (1ull << 32)) return fail(ctx, QVQ_EINVAL, "more than 2^32-1 rows per rank");
    const uint32_t Dp = (D + 3) & ~3u;
    if (Dp > 64) return fail(ctx, QVQ_EINVAL, "block dimension above 64 (3*w*h) is not supported");
    // the same shape again (repeated compresses of one image size): keep every buffer
    if (!ctx->exact && ctx->d_codes && ctx->N == N && ctx->D == D && ctx->cs == cs) return QVQ_OK;
    free_training(ctx);
    free_levels(ctx);
    if (!make_terms(cs, ctx->terms)) return fail(ctx, QVQ_EUNSUPPORTED, "colour space has no exact byte sums");
    ctx->N = N;
    ctx->D = D;
    ctx->Dp = Dp;
    ctx->cs = cs;
    mfma_setup(ctx);
    HIPCHK(hipMalloc(&ctx->d_codes, N * Dp));
    HIPCHK(hipMalloc(&ctx->d_A, N * 4));
    HIPCHK(hipMalloc(&ctx->d_flags, N * 4));
    HIPCHK(hipMalloc(&ctx->d_ties, N * 4));
    uint64_t plut[256];
    for (int b = 0; b < 256; b++) plut[b] = ((uint64_t)ctx->terms.hi[b] << 32) | ctx->terms.lo[b];
    HIPCHK(hipMemcpy(ctx->d_lut32, ctx->terms.v32, sizeof(ctx->terms.v32), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(ctx->d_w, ctx->terms.w, sizeof(ctx->terms.w), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(ctx->d_lut64, ctx->terms.v64, sizeof(ctx->terms.v64), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(ctx->d_plut, plut, sizeof(plut), hipMemcpyHostToDevice));
    // the band of rows whose answer can depend on the centroids' last bits:
    // |c_kahan - c_exact| <= delta per component, so a distance moves by at most
    // 2 delta sqrt(D) sqrt(d) + D delta^2
    const double delta = cs == QVQ_CS_SCALED ? std::ldexp(1.0, -49) : 0.0;
    ctx->tie_abs = 2 * delta * std::sqrt((double)D);
    return QVQ_OK;
}

qvq_status ensure_levels(qvq_ctx *ctx, uint32_t Kmax) {
    if (ctx->Kcap >= Kmax) return QVQ_OK;
    free_levels(ctx);
    const uint64_t KD = (uint64_t)Kmax * ctx->D;
    const uint64_t Kp = pad32(Kmax);
    HIPCHK(hipMalloc(&ctx->d_C64_cent, KD * 8));
    HIPCHK(hipMalloc(&ctx->d_C64_split, KD * 8));
    HIPCHK(hipMalloc(&ctx->d_C64_split_alt, KD * 8));
    HIPCHK(hipMalloc(&ctx->d_C32, Kp * ctx->Dp * 4));
    if (ctx->D == MF_D) HIPCHK(hipMalloc(&ctx->d_E32, Kp * 16 * 4));
    HIPCHK(hipMalloc(&ctx->d_rows, Kp * 2 * cb_row_f16(ctx->D, ctx->Dp)));
    HIPCHK(hipMalloc(&ctx->d_perm, Kp * 4));
    HIPCHK(hipMalloc(&ctx->d_tint, tint_bytes((uint32_t)Kp)));
    // G per-CU slabs + two correction slabs (fused path: rows the recheck / kd-tree move, at
    // the new index (+) and at the search's provisional one (-))
    HIPCHK(hipMalloc(&ctx->d_part, (uint64_t)(ctx->G + 2) * KD * 8));
    HIPCHK(hipMalloc(&ctx->d_part_cnt, (uint64_t)(ctx->G + 2) * Kmax * 4));
    // two copies of the final sums: copy 1 takes the kd-tree ties' moves (kd_reduce_kernel) and
    // is cleared, over the level's region, by each fused search before the level's kd_reduce
    HIPCHK(hipMalloc(&ctx->d_sums, 2 * (2 * KD + Kmax) * 8));
    HIPCHK(hipMemset(ctx->d_sums, 0, 2 * (2 * KD + Kmax) * 8));
    ctx->sums_bytes = 2 * (2 * KD + Kmax) * 8;
    const unsigned mflags = hipHostMallocMapped | hipHostMallocCoherent;
    // two halves, each split rows | parent counts (host_cb_of)
    ctx->cb_half = (KD + (uint64_t)Kmax / 2 + 1 + 7) / 8 * 8;
    HIPCHK(hipHostMalloc(&ctx->h_cb, 2 * ctx->cb_half * 8, mflags));
    HIPCHK(hipHostGetDevicePointer((void **)&ctx->dh_cb, ctx->h_cb, 0));
    ctx->tree_cap = tree_bytes(Kmax, ctx->D);
    for (int b = 0; b < 2; b++) {
        HIPCHK(hipHostMalloc(&ctx->h_tree[b], ctx->tree_cap, mflags));
        HIPCHK(hipHostGetDevicePointer((void **)&ctx->dh_tree[b], ctx->h_tree[b], 0));
    }
    HIPCHK(hipMalloc(&ctx->d_tree, ctx->tree_cap));
    {   // the device tree build's scratch (levels of up to KDB_MAXK code vectors)
        const uint32_t Kb = std::min<uint32_t>(Kmax, KDB_MAXK);
        if (device_tree_on() && kd_build_fits(Kb, ctx->D) && (uint64_t)Kmax * ctx->D >= KDB_MIN_KD) {
            HIPCHK(hipMalloc(&ctx->d_kdb_vind, (uint64_t)Kb * 4));
            HIPCHK(hipMalloc(&ctx->d_kdb_nodes, 2ull * Kb * sizeof(KdbNode)));
            HIPCHK(hipMalloc(&ctx->d_kdb_nbox, 2ull * Kb * 2 * ctx->D * 8));
            HIPCHK(hipMalloc(&ctx->d_kdb_cbox, 2ull * Kb * 2 * ctx->D * 8));
            HIPCHK(hipHostMalloc(&ctx->h_kdb, kdb_host_layout(Kb, ctx->D).total, mflags));
            HIPCHK(hipHostGetDevicePointer((void **)&ctx->dh_kdb, ctx->h_kdb, 0));
            std::memset(ctx->h_kdb, 0, sizeof(KdbHeader));
            ctx->kdb_cap = Kb;
            if (!ctx->kstream) HIPCHK(hipStreamCreateWithFlags(&ctx->kstream, hipStreamNonBlocking));
            if (!ctx->ev_kcb) HIPCHK(hipEventCreateWithFlags(&ctx->ev_kcb, hipEventDisableTiming));
            if (!ctx->ev_kdb) HIPCHK(hipEventCreateWithFlags(&ctx->ev_kdb, hipEventDisableTiming));
        }
    }
    ctx->Kcap = Kmax;
    return QVQ_OK;
}

// Search tables for the K code vectors in d_C64_split.
qvq_status run_prep(qvq_ctx *ctx, uint32_t K) {
    HIPCHK(launch_prep(ctx->stream, ctx->d_C64_split, K, pad32(K), ctx->D, ctx->Dp, ctx->terms.mu, ctx->terms.sx,
                       ctx->mf_t, ctx->d_C32, ctx->d_rows, ctx->d_E32));
    return QVQ_OK;
}

// fp32 error-bound coefficients for the VALU search flag ("near-tie flags").
void valu_coeffs(const qvq_ctx *ctx, float &alpha, float &beta, float &gamma) {
    const double u = std::ldexp(1.0, -24);
    const double vmax = ctx->terms.vmax;
    const double L = std::sqrt((double)ctx->D) * (vmax + 1.2 * vmax) * 1.001;   // >= || |x| + |c| ||
    alpha = (float)(2.0 * 4.01 * u * L);
    beta = (float)(2.0 * ((ctx->Dp + 4) * u * 1.01 + 4e-15));
    gamma = (float)(2.0 * 4.01 * u * u * L * L + 1e-30);
}

// Grow a pinned host buffer (h, bytes) to at least need bytes.
qvq_status ensure_pinned(qvq_ctx *ctx, void *&h, uint64_t &bytes, uint64_t need) {
    if (bytes >= need) return QVQ_OK;
    if (h) (void)hipHostFree(h);
    h = nullptr;
    bytes = 0;
    HIPCHK(hipHostMalloc(&h, need, hipHostMallocDefault));
    bytes = need;
    return QVQ_OK;
}

qvq_status wait_stream(qvq_ctx *ctx);

// Sum of count u64 (f64 = false) or double values at device pointer buf over the ranks, in
// place, on the context's stream: ncclAllReduce over xGMI, or -- the test-only host
// communicator of qvq_comm_init_host -- a copy to pinned memory, the caller's callback, and a
// copy back (the stream is drained around the callback).  No communicator: nothing to do.
qvq_status all_reduce(qvq_ctx *ctx, void *buf, uint64_t count, bool f64) {
    if (ctx->comm) {
        NCCLCHK(ncclAllReduce(buf, buf, count, f64 ? ncclDouble : ncclUint64, ncclSum, ctx->comm, ctx->stream));
        return QVQ_OK;
    }
    if (!ctx->host_ar) return QVQ_OK;
    qvq_status st = ensure_pinned(ctx, ctx->h_ar_stage, ctx->ar_stage_bytes, count * 8);
    if (st != QVQ_OK) return st;
    HIPCHK(hipMemcpyAsync(ctx->h_ar_stage, buf, count * 8, hipMemcpyDeviceToHost, ctx->stream));
    if ((st = wait_stream(ctx)) != QVQ_OK) return st;
    const int rc = ctx->host_ar(ctx->h_ar_stage, count, f64 ? 1 : 0, ctx->host_ar_user);
    if (rc != 0) return fail(ctx, QVQ_ECOMM, "host all-reduce callback failed (" + std::to_string(rc) + ")");
    // stream-ordered: the next all-reduce's download (and callback) come after this upload
    HIPCHK(hipMemcpyAsync(buf, ctx->h_ar_stage, count * 8, hipMemcpyHostToDevice, ctx->stream));
    return QVQ_OK;
}

qvq_status all_reduce_sums(qvq_ctx *ctx, uint32_t K, uint64_t *sums = nullptr, uint32_t copies = 1) {
    if (!sums) sums = ctx->d_sums;
    return all_reduce(ctx, sums, copies * (2 * (uint64_t)K * ctx->D + K), false);
}

// Sums of a final assignment through the counting sort (k_misc.hip) from K * D = 1536 (C4 from
// K = 32: 5.52 -> 5.23 ms against 16384).
bool use_sorted_sums(const qvq_ctx *ctx, uint32_t K) {
    return (uint64_t)K * ctx->D >= 1536 && sorted_sums_fits(K) && ctx->N <= 0xFFFFFFFFull;
}

// Centroid sums under assignment d_A: slabs in d_part (ctx->nslabs of them, for the reduce),
// or with the sort straight into d_sums (ctx->nslabs = 0).
qvq_status run_update_slabs(qvq_ctx *ctx, const uint32_t *d_A, uint32_t K) {
    if (use_sorted_sums(ctx, K)) {
        if (!ctx->d_sortbuf) HIPCHK(hipMalloc(&ctx->d_sortbuf, ctx->N * 2 * sizeof(uint32_t)));
        HIPCHK(launch_sorted_sums(ctx->stream, ctx->Dp, ctx->G, ctx->d_codes, ctx->N, d_A, K, ctx->D, ctx->d_plut,
                                  ctx->d_part_cnt, reinterpret_cast<uint32_t *>(ctx->d_part), ctx->d_sortbuf,
                                  ctx->d_sortbuf + ctx->N, ctx->d_sums));
        ctx->nslabs = 0;
        return QVQ_OK;
    }
    HIPCHK(launch_update(ctx->stream, ctx->Dp, ctx->G, ctx->d_codes, ctx->N, d_A, K, ctx->D, ctx->d_plut, ctx->d_part,
                         ctx->d_part_cnt));
    ctx->nslabs = ctx->G;
    return QVQ_OK;
}

qvq_status run_update(qvq_ctx *ctx, const uint32_t *d_A, uint32_t K) {
    qvq_status st = run_update_slabs(ctx, d_A, K);
    if (st != QVQ_OK) return st;
    if (ctx->nslabs) HIPCHK(launch_reduce(ctx->stream, ctx->d_part, ctx->d_part_cnt, ctx->nslabs, 0, K, ctx->D, ctx->d_sums));
    return QVQ_OK;
}

// Reference-bit ties: the indices of the rows whose answer can depend on
// the centroids' last bits follow the reference's Kahan sums, on any rank count (several ranks:
// the chains run across the ranks, kahan_chained).  QVQ_KAHAN=0: the exact-sum codebook answers
// them (A/B).
bool kahan_mode(const qvq_ctx *ctx) {
    static const bool off = env_is("QVQ_KAHAN", "0");
    return !off && !ctx->exact;
}
// The recheck's absolute tie band: only where a reference-bit step follows (kahan_mode)
double tie_band(const qvq_ctx *ctx) { return kahan_mode(ctx) ? ctx->tie_abs : 0.0; }

qvq_status alloc_kahan_work(qvq_ctx *ctx, KahanWork &w, uint32_t Kc);

qvq_status ensure_kahan(qvq_ctx *ctx, uint32_t Kc) {
    KahanWork &w = ctx->kw;
    const uint32_t D = ctx->D;
    if (ctx->kc_kcap < Kc) {
        dfree(ctx->d_kc_cent);
        dfree(ctx->d_kc_split);
        dfree(ctx->d_kc_sel);
        if (ctx->h_kc_sel) (void)hipHostFree(ctx->h_kc_sel);
        if (ctx->h_kc_out) (void)hipHostFree(ctx->h_kc_out);
        HIPCHK(hipMalloc(&ctx->d_kc_cent, (uint64_t)Kc * D * 8));
        HIPCHK(hipMalloc(&ctx->d_kc_split, 2ull * Kc * D * 8));
        HIPCHK(hipMalloc(&ctx->d_kc_sel, (uint64_t)Kc * 4));
        HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_kc_sel), (uint64_t)Kc * 4, hipHostMallocDefault));
        HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_kc_out), 2ull * Kc * D * 8, hipHostMallocMapped));
        HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void **>(&ctx->dh_kc_out), ctx->h_kc_out, 0));
        ctx->kc_kcap = Kc;
    }
    return alloc_kahan_work(ctx, w, Kc);
}

// A Kahan workspace for N rows, Kc cells and D components (kept while it fits).
qvq_status alloc_kahan_work(qvq_ctx *ctx, KahanWork &w, uint32_t Kc) {
    const uint64_t N = ctx->N;
    const uint32_t D = ctx->D;
    if (w.n_cap == N && w.k_cap >= Kc && w.d_cap == D) return QVQ_OK;
    const uint32_t kcap = std::max(Kc, w.k_cap);
    free_kahan_work(w);
    uint64_t segs, blks;
    KahanWork::caps(N, kcap, segs, blks);
    HIPCHK(hipMalloc(&w.hist, (uint64_t)KahanWork::sort_blocks(N) * kcap * 4));
    HIPCHK(hipMalloc(&w.tot, (uint64_t)kcap * 4));
    for (uint32_t **p : {&w.koff, &w.segoff, &w.blkoff}) HIPCHK(hipMalloc(p, ((uint64_t)kcap + 1) * 4));
    HIPCHK(hipMalloc(&w.planes, (uint64_t)D * KahanWork::plane_len(N)));
    HIPCHK(hipMemset(w.planes, 0, (uint64_t)D * KahanWork::plane_len(N)));
    HIPCHK(hipMalloc(&w.meta, (uint64_t)D * segs * KahanWork::meta_bytes()));
    HIPCHK(hipMalloc(&w.bsum, (uint64_t)D * blks * 16));
    HIPCHK(hipMalloc(&w.bfn, (uint64_t)D * blks * KahanWork::fn_bytes()));
    HIPCHK(hipMalloc(&w.sfn, (uint64_t)D * segs * KahanWork::segfn_bytes()));
    HIPCHK(hipMalloc(&w.bfn8, (uint64_t)D * blks * 8 * KahanWork::fn_bytes()));
    HIPCHK(hipMalloc(&w.stats, 4 * sizeof(unsigned)));
    HIPCHK(hipMemset(w.stats, 0, 4 * sizeof(unsigned)));
    {   // the byte table: SCALED values in units of 2^-60
        uint64_t kx[256];
        for (int b = 0; b < 256; b++) kx[b] = (uint64_t)std::ldexp(ctx->terms.v64[b], 60);
        std::vector<uint8_t> tab(KahanWork::tab_bytes());
        KahanWork::make_tab(kx, tab.data());
        HIPCHK(hipMalloc(&w.tab, tab.size()));
        HIPCHK(hipMemcpy(w.tab, tab.data(), tab.size(), hipMemcpyHostToDevice));
    }
    w.n_one = (uint32_t)N;
    w.seg_cap = segs;
    w.blk_cap = blks;
    w.n_cap = N;
    w.k_cap = kcap;
    w.d_cap = D;
    return QVQ_OK;
}


// Sum over the ranks of n small u64 values (host, in place) on the context's stream, waiting for
// the result: the ranks' decisions at the end of qvq_lbg, so that every rank takes the same
// branch.  One rank: nothing to do.
qvq_status vote(qvq_ctx *ctx, uint64_t *vals, uint64_t n) {
    if (ctx->nranks <= 1 || (!ctx->comm && !ctx->host_ar) || n == 0) return QVQ_OK;
    if (ctx->vote_cap < n) {
        dfree(ctx->d_vote);
        if (ctx->h_vote) (void)hipHostFree(ctx->h_vote);
        ctx->h_vote = nullptr;
        ctx->vote_cap = 0;
        HIPCHK(hipMalloc(&ctx->d_vote, n * 8));
        HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_vote), n * 8, hipHostMallocDefault));
        ctx->vote_cap = n;
    }
    std::memcpy(ctx->h_vote, vals, n * 8);
    HIPCHK(hipMemcpyAsync(ctx->d_vote, ctx->h_vote, n * 8, hipMemcpyHostToDevice, ctx->stream));
    qvq_status st = all_reduce(ctx, ctx->d_vote, n, false);
    if (st != QVQ_OK) return st;
    HIPCHK(hipMemcpyAsync(ctx->h_vote, ctx->d_vote, n * 8, hipMemcpyDeviceToHost, ctx->stream));
    if ((st = wait_stream(ctx)) != QVQ_OK) return st;
    std::memcpy(vals, ctx->h_vote, n * 8);
    return QVQ_OK;
}

// The reference's Kahan centroids (and their split) of S cells when the rows are split over the
// ranks, each rank holding a contiguous range of the global rows, ranks in row order (DESIGN.md
// 5; src/Quantizer.cpp:59-70 sums each cell's rows in ascending global order, so a chain runs
// across the ranks).  A: this rank's rows' cells among K_in (nullptr: the mean, K_in = S = 1);
// sel: the device slot map of launch_kahan_centroids (nullptr: every cell, S = K_in).  Every
// rank calls it with the same cells and gets the same centroids in d_kc_cent [S][D] and, with
// want_split, their split in d_kc_split [2S][D] (device; ensure_kahan sizes both):
//   1. each rank sorts its rows of the cells and sums each chain exactly (its totals and row
//      counts into its slice of an all-gather, one collective): every chain's exact prefix at
//      each rank's first row;
//   2. each rank builds its segment functions at those global prefixes;
//   3. the chains pass from rank to rank: rank q advances the reference's state (sum, c) over
//      its rows and an all-reduce, the others contributing zeros, hands it on (nranks small
//      collectives);
//   4. C = sum * fl(1/n), n the cell's rows over every rank.
// splits (qvq_update_kahan_split, tests): this context's rows as virtual ranks cut at the given
// offsets, run one after another on the device (no collective).
qvq_status kahan_chained(qvq_ctx *ctx, const uint32_t *A, uint32_t K_in, const uint32_t *sel, uint32_t S,
                         bool want_split, const std::vector<uint64_t> *splits = nullptr) {
    const uint32_t D = ctx->D, Dp = ctx->Dp;
    const bool virt = splits != nullptr;
    const uint32_t R = virt ? (uint32_t)splits->size() - 1 : (uint32_t)ctx->nranks;
    const uint32_t rank = virt ? 0u : (uint32_t)ctx->rank;
    const uint32_t Ks = sel ? S : K_in;   // the sort's keys: slots, or cells
    if (!A && (K_in != 1 || S != 1 || sel)) return fail(ctx, QVQ_EINVAL, "kahan_chained: the mean is one cell");
    qvq_status st = ensure_kahan(ctx, std::max(K_in, S));   // (may reallocate the outputs below)
    if (st != QVQ_OK) return st;
    double *C_out = ctx->d_kc_cent, *split_out = want_split ? ctx->d_kc_split : nullptr;
    const uint64_t gcount = 2ull * R * S * D + (uint64_t)R * S, scount = 2ull * S * D;
    if (ctx->kc_chain_cap < gcount + scount) {
        dfree(ctx->d_kc_chain);
        ctx->kc_chain_cap = 0;
        HIPCHK(hipMalloc(&ctx->d_kc_chain, (gcount + scount) * 8));
        ctx->kc_chain_cap = gcount + scount;
    }
    uint64_t *gather = ctx->d_kc_chain, *state = gather + gcount;
    hipStream_t s = ctx->stream;
    HIPCHK(hipMemsetAsync(gather, 0, (gcount + scount) * 8, s));
    const KahanWork &w = ctx->kw;
    if (virt) {
        for (uint32_t v = 0; v < R; v++) {
            const uint64_t off = (*splits)[v], n = (*splits)[v + 1] - off;
            if (!n) continue;
            const uint8_t *codes = ctx->d_codes + off * Dp;
            const uint32_t *Av = A ? A + off : nullptr;
            HIPCHK(launch_kahan_chain_local(s, w, codes, Dp, D, n, Av, Ks, sel, K_in, gather, v, R));
            HIPCHK(launch_kahan_chain_build(s, w, D, n, Ks, gather, v));
            HIPCHK(launch_kahan_chain_eval(s, w, D, n, Ks, state, gather, v));
        }
    } else {
        HIPCHK(launch_kahan_chain_local(s, w, ctx->d_codes, Dp, D, ctx->N, A, Ks, sel, K_in, gather, rank, R));
        if (R > 1 && (st = all_reduce(ctx, gather, gcount, false)) != QVQ_OK) return st;
        HIPCHK(launch_kahan_chain_build(s, w, D, ctx->N, Ks, gather, rank));
        for (uint32_t q = 0; q < R; q++) {
            if (q == rank) HIPCHK(launch_kahan_chain_eval(s, w, D, ctx->N, Ks, state, gather, rank));
            else HIPCHK(hipMemsetAsync(state, 0, scount * 8, s));
            if (R > 1 && (st = all_reduce(ctx, state, scount, false)) != QVQ_OK) return st;
        }
    }
    HIPCHK(launch_kahan_chain_finish(s, D, Ks, state, gather, R, C_out, split_out));
    return QVQ_OK;
}

bool join_tree_job(qvq_ctx *ctx, bool cancel);

// Build the reference kd-tree over the host copy hC of the K code vectors being searched
// into tree image buffer buf (pinned host memory, DMA-copied to d_tree for kd_resolve_kernel).  An empty
// view means host resolution (tree too deep/large for the kernel's LDS, or QVQ_KDTREE=host).

// Level L's split codebook as the finalize of level L - 1 publishes it (host / device view).
// Double-buffered by level parity: the synchronous Kahan levels build a level's tree on the
// worker from this copy while the level's own finalize already publishes the next level's
// codebook (one buffer: a worker late by more than the level's search read a mix of the two,
// the r05i-r05m intermittent mismatches on palette images).
// QVQ_CB_SINGLE=1 (tests only): the one buffer of before the fix, which with
// QVQ_TREE_JOB_DELAY_MS makes the race deterministic (tests/test_gpu_kahan.py).
uint32_t cb_half_of(uint32_t level) {
    static const bool single = env_is("QVQ_CB_SINGLE", "1");
    return single ? 0u : (level & 1);
}
double *host_cb_of(const qvq_ctx *ctx, uint32_t level) { return ctx->h_cb + (uint64_t)cb_half_of(level) * ctx->cb_half; }
double *dev_cb_of(const qvq_ctx *ctx, uint32_t level) { return ctx->dh_cb + (uint64_t)cb_half_of(level) * ctx->cb_half; }

// The host part: the tree (ctx->tree over ctx->cb_local) and its flattened image in h_tree[buf];
// v.bytes = 0 when there is no device image (too large, or too deep for the kernel's LDS).
// No HIP call: the tree worker runs it.
void build_tree_host(qvq_ctx *ctx, const double *hC, uint32_t K, int buf, KdView &v,
                     const std::atomic<bool> *cancel = nullptr) {
    v = KdView{};
    // the build reads the codebook many times; mapped memory the GPU just wrote is read
    // once, sequentially, into ordinary memory first
    ctx->cb_local.assign(hC, hC + (size_t)K * ctx->D);
    if ((hC == host_cb_of(ctx, 0) || hC == host_cb_of(ctx, 1)) && K >= 2) {   // a finalize's split: the parent counts follow it
        const uint32_t *cnt = reinterpret_cast<const uint32_t *>(hC + (size_t)K * ctx->D);
        ctx->cnt_local.assign(cnt, cnt + K / 2);
    } else {
        ctx->cnt_local.clear();
    }
    ctx->htrace.mark("K" + std::to_string(K) + " codebook copied");
    ctx->tree.reset(new RefKDTree(ctx->cb_local.data(), K, (int)ctx->D, cancel));
    ctx->htrace.mark("K" + std::to_string(K) + " tree structure");
    const RefKDTree &tree = *ctx->tree;
    if (tree.cancelled()) return;
    const uint32_t D = ctx->D;
    const size_t nn = tree.num_nodes();
    KdView t;
    t.depth = tree.depth();
    t.n_nodes = (uint32_t)nn;
    const uint64_t bytes = 16ull * D + nn * sizeof(KdNodeDev) + 4ull * K;
    if (bytes > ctx->tree_cap) return;
    t.bytes = (uint32_t)bytes;
    if (!kd_resolve_fits(t, K)) return;
    double *lo = reinterpret_cast<double *>(ctx->h_tree[buf]), *hi = lo + D;
    KdNodeDev *nodes = reinterpret_cast<KdNodeDev *>(hi + D);
    uint32_t *vind = reinterpret_cast<uint32_t *>(nodes + nn);
    tree.flatten(nodes, vind, lo, hi);
    v = t;
}

// The device view of image buf (v from build_tree_host).  Every kd_resolve workgroup stages the
// image.  Big images (C4: 150+ KB) go to device memory with one DMA first (mapped reads from 16
// workgroups cost up to ~70 us); small ones are read in place (the DMA itself costs ~5 us of
// stream time per level).
void tree_view(qvq_ctx *ctx, int buf, KdView &v) {
    if (!v.bytes) {
        v = KdView{};
        return;
    }
    const uint32_t D = ctx->D;
    const double *dlo = reinterpret_cast<const double *>(ctx->dh_tree[buf]);
    constexpr uint64_t dma_min = 32768;
    if (v.bytes > dma_min) {
        if (hipMemcpyAsync(ctx->d_tree, ctx->h_tree[buf], v.bytes, hipMemcpyHostToDevice, ctx->stream) != hipSuccess) {
            v = KdView{};
            return;
        }
        dlo = reinterpret_cast<const double *>(ctx->d_tree);
    }
    v.lo = dlo;
    v.hi = dlo + D;
    v.nodes = reinterpret_cast<const KdNodeDev *>(dlo + 2 * D);
    v.vind = reinterpret_cast<const uint32_t *>(v.nodes + v.n_nodes);
}

void build_tree(qvq_ctx *ctx, const double *hC, uint32_t K, int buf, KdView &kd) {
    kd = KdView{};
    ctx->tree_kd = KdView{};
    if (env_is("QVQ_KDTREE", "host")) return;
    build_tree_host(ctx, hC, K, buf, kd);
    tree_view(ctx, buf, kd);
    ctx->tree_kd = kd;
}

CommState probe_comm(qvq_ctx *ctx, std::string &msg);
qvq_status wait_failed(qvq_ctx *ctx, qvq_status st);

// The device build of a level's tree (k_kdbuild.hip), 48-D levels from K = 512 up to KDB_MAXK:
// opt-in (QVQ_KDTREE=device).  Bit-identical to the host build (tests/test_gpu_kdbuild.py), but
// slower than it on the GPU box's host: K = 4096 3.7 ms vs 1.8 ms, K = 2048 2.2 vs 0.7 (a node
// costs ~10-20 us of dependent device round trips and barriers, and C4's trees have ~300 big
// nodes on one serial path), so the host build, overlapping the search, stays the default
// (DESIGN.md 8).
bool device_tree_on() {
    static const bool on = env_is("QVQ_KDTREE", "device");
    return on;
}
bool use_device_tree(const qvq_ctx *ctx, uint32_t K) {
    return device_tree_on() && ctx->kdb_cap >= K && !ctx->exact && kd_build_fits(K, ctx->D) &&
           (uint64_t)K * ctx->D >= KDB_MIN_KD;
}

// Enqueue the device build of the tree over the K code vectors in d_C64_split on kstream, after
// the work already on the context's stream (the finalize that wrote them); the search then runs
// beside it.
qvq_status start_device_tree(qvq_ctx *ctx, uint32_t K) {
    HIPCHK(hipEventRecord(ctx->ev_kcb, ctx->stream));
    HIPCHK(hipStreamWaitEvent(ctx->kstream, ctx->ev_kcb, 0));
    HIPCHK(launch_kd_build(ctx->kstream, ctx->d_C64_split, K, ctx->D, ctx->d_kdb_vind, ctx->d_kdb_nodes,
                           ctx->d_kdb_nbox, ctx->d_kdb_cbox, ctx->d_tree, ctx->dh_kdb, ++ctx->kdb_seq));
    HIPCHK(hipEventRecord(ctx->ev_kdb, ctx->kstream));
    return QVQ_OK;
}

// The device build's tree for the level: waits (bounded) for its image, makes the context's
// stream wait for the build (d_C64_split is rewritten by the level's finalize), and imports it as
// ctx->tree over ctx->cb_local (which the caller filled) with its device view in kd.  false: the
// build failed (the caller builds on the host).
qvq_status finish_device_tree(qvq_ctx *ctx, uint32_t K, KdView &kd, bool &ok) {
    ok = false;
    kd = KdView{};
    const KdbHeader *h = reinterpret_cast<const KdbHeader *>(ctx->h_kdb);
    std::string err;
    const qvq_status st = wait_until(
        [&] { return *reinterpret_cast<const volatile uint64_t *>(&h->seq) >= ctx->kdb_seq; },
        [&](std::string &m) {
            const hipError_t q = hipStreamQuery(ctx->kstream);
            if (q == hipSuccess) return StreamState::Drained;
            if (q == hipErrorNotReady) return StreamState::Running;
            m = hipGetErrorString(q);
            return StreamState::Failed;
        },
        [&](std::string &m) { return probe_comm(ctx, m); }, ctx->timeout_s, err);
    if (st != QVQ_OK) return wait_failed(ctx, fail(ctx, st, "device kd-tree build: " + err));
    std::atomic_thread_fence(std::memory_order_acquire);
    HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_kdb, 0));
    if (h->status != 1) return QVQ_OK;
    ctx->tree.reset(new RefKDTree(ctx->cb_local.data(), K, (int)ctx->D, ctx->h_kdb));
    KdView t;
    t.depth = (int)h->depth;
    t.n_nodes = h->n_nodes;
    const uint64_t bytes = 16ull * ctx->D + (uint64_t)h->n_nodes * sizeof(KdNodeDev) + 4ull * K;
    ok = true;
    if (bytes > ctx->tree_cap) return QVQ_OK;
    t.bytes = (uint32_t)bytes;
    if (!kd_resolve_fits(t, K)) return QVQ_OK;
    const double *dlo = reinterpret_cast<const double *>(ctx->d_tree);
    t.lo = dlo;
    t.hi = dlo + ctx->D;
    t.nodes = reinterpret_cast<const KdNodeDev *>(dlo + 2 * ctx->D);
    t.vind = reinterpret_cast<const uint32_t *>(t.nodes + t.n_nodes);
    kd = t;
    return QVQ_OK;
}

// A deferred-tie level (qvq_lbg's Kahan path) needs its tree only when it has ties, which the
// host learns after the search: the worker awaits the codebook's publication and builds the
// tree while this thread enqueues the rest of the level; join_tree_job waits for it (ties)
// or cancels it (none).
void post_job(qvq_ctx *ctx, std::function<void()> job, qvq_ctx::Worker *wk = nullptr) {
    qvq_ctx::Worker &w = wk ? *wk : ctx->worker;
    if (!w.th.joinable()) {
        w.th = std::thread([&w] {
            std::unique_lock<std::mutex> lk(w.m);
            for (;;) {
                w.cv.wait(lk, [&w] { return w.stop || !w.q.empty(); });
                if (w.stop && w.q.empty()) return;   // (queued frees still run)
                std::function<void()> job = std::move(w.q.front());
                w.q.pop_front();
                lk.unlock();
                job();
                w.pending.fetch_sub(1, std::memory_order_release);
                lk.lock();
            }
        });
        if (ctx->place_ok) pthread_setaffinity_np(w.th.native_handle(), sizeof(cpu_set_t), &ctx->place);
    }
    w.pending.fetch_add(1, std::memory_order_relaxed);
    {
        std::lock_guard<std::mutex> g(w.m);
        w.q.push_back(std::move(job));
    }
    w.cv.notify_one();
}

void start_tree_job(qvq_ctx *ctx, const double *hC, uint32_t K, int buf, uint64_t wait_seq) {
    join_tree_job(ctx, true);
    if (env_is("QVQ_KDTREE", "host")) return;
    ctx->tree_cancel.store(false);
    ctx->tree_job = true;
    ctx->job_ok = false;
    ctx->job_buf = buf;
    ctx->tree_kd = KdView{};
    const int slot = (int)__builtin_ctz(K) - 1;
    post_job(ctx, [ctx, hC, K, buf, wait_seq, slot] {
        const auto t0 = std::chrono::steady_clock::now();
        volatile uint64_t *flag = ctx->h_ready;
        while (wait_seq && *flag < wait_seq) {   // the codebook's publication (bounded by cancel)
            if (ctx->tree_cancel.load(std::memory_order_relaxed)) return;
            cpu_relax();
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        // QVQ_TREE_JOB_DELAY_MS (tests only): a worker late past the level's own finalize, the
        // interleaving of the r05m race (the finalize publishes the next level's codebook)
        static const int delay_ms = std::getenv("QVQ_TREE_JOB_DELAY_MS") ? std::atoi(std::getenv("QVQ_TREE_JOB_DELAY_MS")) : 0;
        if (delay_ms > 0) std::this_thread::sleep_for(std::chrono::milliseconds(delay_ms));
        const auto t1 = std::chrono::steady_clock::now();
        build_tree_host(ctx, hC, K, buf, ctx->job_kd, &ctx->tree_cancel);
        ctx->job_ok = !ctx->tree->cancelled();
        ctx->tm.wait_ms[slot] = std::chrono::duration<double, std::milli>(t1 - t0).count();
        ctx->tm.tree_ms[slot] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
    });
}

bool join_tree_job(qvq_ctx *ctx, bool cancel) {
    if (!ctx->tree_job) return false;
    if (cancel) ctx->tree_cancel.store(true);
    while (ctx->worker.pending.load(std::memory_order_acquire)) std::this_thread::yield();
    ctx->tree_job = false;
    if (!ctx->job_ok) {
        ctx->tree.reset();
        ctx->tree_kd = KdView{};
        return false;
    }
    KdView v = ctx->job_kd;
    tree_view(ctx, ctx->job_buf, v);
    ctx->tree_kd = v;
    return true;
}

// Copy between a caller's host buffer and device memory at DMA speed: the host range is pinned
// in place for the copy (hipHostRegister; a pageable hipMemcpy goes through bounce buffers at a
// fraction of PCIe bandwidth: the 50 MB C3 raster took ~3 ms), with a plain copy as the fallback
// (already pinned memory, or registration refused).
// Synchronous on the context's stream.
hipError_t host_copy(qvq_ctx *ctx, void *dst, const void *src, uint64_t bytes, hipMemcpyKind kind) {
    void *host = const_cast<void *>(kind == hipMemcpyHostToDevice ? src : dst);
    const bool reg = bytes >= (1u << 20) && hipHostRegister(host, bytes, hipHostRegisterDefault) == hipSuccess;
    if (!reg) (void)hipGetLastError();
    hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (reg) (void)hipHostUnregister(host);
    return e;
}

// Probes for wait_until (wait.hpp): the stream's state, and the communicator's asynchronous
// error state (RCCL reports a peer's failure there while our collective is stuck).
StreamState probe_stream(qvq_ctx *ctx, std::string &msg) {
    const hipError_t q = hipStreamQuery(ctx->stream);
    if (q == hipSuccess) return StreamState::Drained;
    if (q == hipErrorNotReady) return StreamState::Running;
    msg = hipGetErrorString(q);
    return StreamState::Failed;
}
CommState probe_comm(qvq_ctx *ctx, std::string &msg) {
    if (!ctx->comm) return CommState::None;
    ncclResult_t ae = ncclSuccess;
    const ncclResult_t r = ncclCommGetAsyncError(ctx->comm, &ae);
    if (r != ncclSuccess) ae = r;
    if (ae == ncclSuccess || ae == ncclInProgress) return CommState::Healthy;
    msg = ncclGetErrorString(ae);
    return CommState::Failed;
}
// A failed or timed-out wait: a communicator is aborted (which also releases the stream from
// a stuck RCCL kernel) and the context runs single-rank until the next qvq_comm_init.  Then
// the stream gets one more bounded chance to drain; if it does not (a timeout without a
// communicator, a kernel still running), the context is poisoned: work that may still write
// the context's scratch or copy into caller memory is queued, so every later call but
// qvq_destroy returns QVQ_ESTATE.
qvq_status wait_failed(qvq_ctx *ctx, qvq_status st) {
    if (st == QVQ_ECOMM && ctx->comm) {
        (void)ncclCommAbort(ctx->comm);
        ctx->comm = nullptr;
        ctx->nranks = 1;
        ctx->rank = 0;
    }
    using clock = std::chrono::steady_clock;
    // after an abort the RCCL kernels exit: give the stream 2 s to drain; a timeout without a
    // communicator means a long or stuck kernel: one query
    const auto until = clock::now() + std::chrono::milliseconds(st == QVQ_ECOMM ? 2000 : 0);
    hipError_t q = hipStreamQuery(ctx->stream);
    while (q == hipErrorNotReady && clock::now() < until) q = hipStreamQuery(ctx->stream);
    if (q != hipSuccess) {
        ctx->poisoned = true;
        ctx->err += " (context poisoned: destroy it)";
    }
    return st;
}

// Wait until the stream has published seq in a mapped flag (the ready number of finalize's
// codebook in h_ready, or copy_out's completion).  Bounded: a failed or drained stream, a
// communicator error, or ctx->timeout_s without progress end the wait with a status.
qvq_status wait_flag(qvq_ctx *ctx, volatile uint64_t *flag, uint64_t seq) {
    std::string err;
    const qvq_status st = wait_until([&] { return *flag >= seq; },
                                     [&](std::string &m) { return probe_stream(ctx, m); },
                                     [&](std::string &m) { return probe_comm(ctx, m); }, ctx->timeout_s, err);
    if (st != QVQ_OK) return wait_failed(ctx, fail(ctx, st, err));
    std::atomic_thread_fence(std::memory_order_acquire);
    return QVQ_OK;
}
// Wait for everything enqueued on the stream so far (an event, polled with the same bounds).
qvq_status wait_stream(qvq_ctx *ctx) {
    HIPCHK(hipEventRecord(ctx->ev_sync, ctx->stream));
    std::string err;
    hipError_t eq = hipSuccess;
    const qvq_status st = wait_until(
        [&] {
            eq = hipEventQuery(ctx->ev_sync);
            return eq != hipErrorNotReady;
        },
        [&](std::string &m) { return probe_stream(ctx, m); }, [&](std::string &m) { return probe_comm(ctx, m); },
        ctx->timeout_s, err);
    if (st != QVQ_OK) return wait_failed(ctx, fail(ctx, st, err));
    if (eq != hipSuccess) return fail(ctx, QVQ_EDEVICE, std::string("stream: ") + hipGetErrorString(eq));
    return QVQ_OK;
}
qvq_status wait_codebook(qvq_ctx *ctx, uint64_t seq) { return wait_flag(ctx, ctx->h_ready, seq); }

// Tie rows listed by the recheck when no device tree was available: answer them with the
// host tree over hC and write A; with accumulate their terms move from the search's
// provisional index to the answer (launch_fix_rows).  Synchronous.
qvq_status resolve_host_ties(qvq_ctx *ctx, const double *hC, uint32_t K, uint32_t nt, bool accumulate,
                             uint64_t *xsums = nullptr) {
    const uint32_t D = ctx->D, Dp = ctx->Dp;
    const uint64_t need = (uint64_t)nt * (8 + Dp);
    if (ctx->scatter_bytes < need) {
        dfree(ctx->d_scatter);
        HIPCHK(hipMalloc(&ctx->d_scatter, need));
        ctx->scatter_bytes = need;
    }
    uint32_t *d_rows = ctx->d_scatter, *d_vals = ctx->d_scatter + nt;
    uint8_t *d_gath = reinterpret_cast<uint8_t *>(ctx->d_scatter + 2 * (uint64_t)nt);
    std::vector<uint32_t> rows(nt), vals(nt);
    std::vector<uint8_t> code((uint64_t)nt * Dp);
    HIPCHK(launch_gather_codes(ctx->stream, ctx->d_codes, Dp, ctx->d_ties, nt, d_gath));
    HIPCHK(hipMemcpyAsync(rows.data(), ctx->d_ties, nt * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipMemcpyAsync(code.data(), d_gath, code.size(), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    std::vector<double> q(D);
    RefKDTree tree(hC, K, (int)D);
    for (uint32_t i = 0; i < nt; i++) {
        for (uint32_t d = 0; d < D; d++) q[d] = ctx->terms.v64[code[(uint64_t)i * Dp + d]];
        vals[i] = tree.nearest(q.data());
    }
    HIPCHK(hipMemcpyAsync(d_rows, rows.data(), nt * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(d_vals, vals.data(), nt * 4, hipMemcpyHostToDevice, ctx->stream));
    uint64_t *xslab = accumulate ? ctx->d_part + (uint64_t)ctx->G * K * D : nullptr;
    uint32_t *xcnt = accumulate ? ctx->d_part_cnt + (uint64_t)ctx->G * K : nullptr;
    HIPCHK(launch_fix_rows(ctx->stream, ctx->d_codes, Dp, D, ctx->d_A, d_rows, d_vals, nt, K, xslab, xcnt,
                           ctx->d_plut, xsums));
    HIPCHK(hipStreamSynchronize(ctx->stream));   // the host vectors must outlive the copies
    return QVQ_OK;
}

// One level's assignment of every row against the split codebook (d_C64_split, host copy
// hC, search tables in d_C32/d_rows), K code vectors.  wait_seq != 0: hC is published by a
// finalize still in flight.  With sums_out the exact centroid sums of the final assignment
// are left in the first ctx->nslabs slabs of d_part / d_part_cnt, the last ctx->nsub of them
// to be subtracted (fused: the search's G slabs with every row at its provisional index, slab
// G with the rows the recheck and the kd-tree move at their new index, slab G + 1 with the
// same rows at the provisional one; otherwise the update's G).
// Copy 1 of d_sums sits one capacity-sized copy in, where no level's copy 0 reaches.
uint64_t sums_cap_stride(const qvq_ctx *ctx) { return 2 * (uint64_t)ctx->Kcap * ctx->D + ctx->Kcap; }

// One rank, fused sums: the kd-tree ties go with the reduce (kd_reduce_kernel: one launch fewer
// per level).
bool kd_merge(const qvq_ctx *ctx) {
    return !ctx->comm && !ctx->host_ar;
}

qvq_status run_level(qvq_ctx *ctx, uint32_t K, int slot, bool sums_out, const double *hC, uint64_t wait_seq,
                     bool defer_ties = false) {
    const bool fused = sums_out && use_fused(ctx, K);
    ctx->kd_pend = false;
    ctx->sums_copies = 1;
    // one rank, sums from a separate pass: that pass (and its reduce) runs before the tree is
    // built -- it overlaps the host build instead of waiting behind it -- and the ties' moves are
    // then applied to the finished sums (move_row_sums)
    const bool early_upd = sums_out && !fused && (kd_merge(ctx) || defer_ties);
    uint64_t *sums1 = early_upd ? ctx->d_sums : nullptr;
    uint64_t *xslab = fused ? ctx->d_part + (uint64_t)ctx->G * K * ctx->D : nullptr;
    uint32_t *xcnt = fused ? ctx->d_part_cnt + (uint64_t)ctx->G * K : nullptr;
    ctx->nslabs = fused ? ctx->G + 2 : ctx->G;
    ctx->nsub = fused ? 1 : 0;
    unsigned *cnt = ctx->d_counters + 2 * slot;
    // HIP events around the search (each record costs a few us of GPU idle): every level,
    // one level, or none (qvq_set_timing)
    const bool timing = ctx->timing_level == -1 || ctx->timing_level == slot;
    // the level's kd-tree on the device, beside the search (every CU holds a search workgroup
    // and room for the build's)
    const bool devtree = !defer_ties && use_device_tree(ctx, K);
    qvq_status st;
    if (devtree && (st = start_device_tree(ctx, K)) != QVQ_OK) return st;
    if (timing) HIPCHK(hipEventRecord(ctx->ev[slot][0], ctx->stream));
    if (use_mfma(ctx, K)) {
        const bool prune = ctx->perm_k == K;   // the order qvq_lbg's finalize left for this level
        // one rank, fused sums: the search clears copy 1 of the final sums (the kd ties' moves,
        // added by the previous level's finalize), covering every smaller level's layout
        const bool clear1 = fused && kd_merge(ctx);
        HIPCHK(launch_assign_mfma(ctx->stream, ctx->num_cu, fused, ctx->d_codes, ctx->N, ctx->d_rows, ctx->d_E32, K,
                                  ctx->d_C32, ctx->d_plut, ctx->mf_th, ctx->d_A, ctx->d_flags, &cnt[0],
                                  ctx->d_part, ctx->d_part_cnt, prune ? ctx->d_perm : nullptr,
                                  prune ? ctx->d_tint : nullptr, clear1 ? ctx->d_sums + sums_cap_stride(ctx) : nullptr,
                                  clear1 ? (uint32_t)(2 * (uint64_t)K * ctx->D + K) : 0u));
    } else if (use_wide(ctx, K)) {
        const bool prune = ctx->perm_k == K;
        HIPCHK(launch_assign_wide(ctx->stream, ctx->num_cu, ctx->Dp, ctx->D, ctx->d_codes, ctx->N, ctx->d_rows, K,
                                  ctx->d_C32, ctx->mf_th, ctx->d_A, ctx->d_flags, &cnt[0],
                                  prune ? ctx->d_perm : nullptr, prune ? ctx->d_tint : nullptr,
                                  std::max<uint32_t>(1, (ctx->col_blocks + 32) / 64), ctx->d_counters + SCHED_COUNTERS));
    } else {
        float alpha, beta, gamma;
        valu_coeffs(ctx, alpha, beta, gamma);
        HIPCHK(launch_assign_valu(ctx->stream, ctx->num_cu, ctx->Dp, ctx->d_codes, ctx->N, ctx->d_C32, K,
                                  ctx->d_lut32, alpha, beta, gamma, ctx->d_A, ctx->d_flags, &cnt[0]));
    }
    if (timing) HIPCHK(hipEventRecord(ctx->ev[slot][1], ctx->stream));
    // the MFMA recheck from K = 512 (below it the fp32 pass over K code vectors is cheaper than
    // staging the MFMA tables, profiles/r02f)
    if (K >= 512 && use_mfma(ctx, K) && recheck_mf32_fits(K)) {
        HIPCHK(launch_recheck_mf32(ctx->stream, ctx->num_cu, ctx->d_codes, ctx->d_flags, &cnt[0], ctx->d_rows,
                                   ctx->d_C64_split, K, ctx->d_lut64, ctx->mf_th, 1e-12, tie_band(ctx), ctx->d_A, ctx->d_ties,
                                   &cnt[1], xslab, xcnt, ctx->d_plut));
    } else {
        float alpha, beta, gamma;
        valu_coeffs(ctx, alpha, beta, gamma);
        const bool pruned = ctx->perm_k == K;   // the search's order is valid for the recheck too
        HIPCHK(launch_recheck(ctx->stream, ctx->num_cu, ctx->d_codes, ctx->Dp, ctx->D, ctx->d_flags, &cnt[0],
                              ctx->d_C64_split, ctx->d_C32, K, ctx->d_lut64, alpha, beta, gamma, 1e-12, tie_band(ctx), ctx->d_A,
                              ctx->d_ties, &cnt[1], xslab, xcnt, ctx->d_plut, pruned ? ctx->d_perm : nullptr,
                              pruned ? ctx->d_tint : nullptr,
                              (float)((double)ctx->D / (ctx->terms.sx * ctx->terms.sx))));
    }
    if (defer_ties) {   // the level's tie count to the host, before the rest of the level runs
        ctx->pub_seq++;
        if (fused) {   // published by the slab reduce that follows (qvq_lbg): no launch of its own
            ctx->pub.cnt = &cnt[1];
            ctx->pub.dst = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(ctx->dh_ready) + 16);
            ctx->pub.flag = ctx->dh_ready + 1;
            ctx->pub.seq = ctx->pub_seq;
        } else {
            HIPCHK(launch_copy_out(ctx->stream, &cnt[1], reinterpret_cast<uint8_t *>(ctx->dh_ready) + 16, 4, nullptr,
                                   nullptr, 0, nullptr, nullptr, 0, ctx->dh_ready + 1, ctx->pub_seq,
                                   ctx->d_counters + 2 * 33 + 1));
        }
    }
    if (early_upd) {
        HIPCHK(hipEventRecord(ctx->ev[slot][2], ctx->stream));
        if ((st = run_update(ctx, ctx->d_A, K)) != QVQ_OK) return st;
        ctx->nslabs = 0;   // reduced already
        HIPCHK(hipEventRecord(ctx->ev[slot][3], ctx->stream));
    }
    if (defer_ties) {   // qvq_lbg answers the ties after the finalize, if there are any (tree on the worker)
        start_tree_job(ctx, hC, K, slot & 1, wait_seq);
        ctx->upd[slot] = false;
        return QVQ_OK;
    }
    // the tree build overlaps the search just enqueued
    const auto tw0 = std::chrono::steady_clock::now();
    if (wait_seq && (st = wait_codebook(ctx, wait_seq)) != QVQ_OK) return st;
    const auto tw1 = std::chrono::steady_clock::now();
    ctx->htrace.mark("K" + std::to_string(K) + " codebook seen, tree build");
    KdView kd;
    bool dev_ok = false;
    if (devtree) {   // the host copies of the codebook and parent counts, then the device's tree
        ctx->cb_local.assign(hC, hC + (size_t)K * ctx->D);
        if ((hC == host_cb_of(ctx, 0) || hC == host_cb_of(ctx, 1)) && K >= 2) {
            const uint32_t *pc = reinterpret_cast<const uint32_t *>(hC + (size_t)K * ctx->D);
            ctx->cnt_local.assign(pc, pc + K / 2);
        } else {
            ctx->cnt_local.clear();
        }
        if ((st = finish_device_tree(ctx, K, kd, dev_ok)) != QVQ_OK) return st;
        ctx->tree_kd = kd;
    }
    if (!dev_ok) build_tree(ctx, hC, K, slot & 1, kd);
    ctx->htrace.mark("K" + std::to_string(K) + (dev_ok ? " device tree in" : " tree built"));
    ctx->tm.wait_ms[slot] = std::chrono::duration<double, std::milli>(tw1 - tw0).count();
    ctx->tm.tree_ms[slot] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw1).count();
    if (kd.depth > 0 && fused && kd_merge(ctx) && kd_reduce_fits(kd, K)) {
        ctx->kd_pend = true;   // with the reduce (qvq_lbg)
        ctx->pend_kd = kd;
        ctx->sums_copies = 2;
    } else if (kd.depth > 0) {
        HIPCHK(launch_kd_resolve(ctx->stream, ctx->d_codes, ctx->Dp, ctx->D, ctx->d_ties, &cnt[1], ctx->d_C64_split,
                                 K, ctx->d_lut64, kd, ctx->d_A, xslab, xcnt, ctx->d_plut, sums1));
    } else {   // ties answered on the host
        unsigned nt = 0;
        HIPCHK(hipMemcpyAsync(&nt, &cnt[1], sizeof(nt), hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        if (nt && (st = resolve_host_ties(ctx, hC, K, nt, fused, sums1)) != QVQ_OK) return st;
    }
    ctx->upd[slot] = sums_out && !fused;
    if (ctx->upd[slot] && !early_upd) {
        HIPCHK(hipEventRecord(ctx->ev[slot][2], ctx->stream));
        if ((st = run_update_slabs(ctx, ctx->d_A, K)) != QVQ_OK) return st;
        HIPCHK(hipEventRecord(ctx->ev[slot][3], ctx->stream));
    }
    return QVQ_OK;
}

// |c_kahan - c_exact| per split component for SCALED values (the tie band's delta)
constexpr double KAHAN_DELTA = 0x1p-49;

// The ties of a Kahan level answered from the level's own tree (over the exact-sum split) and
// the reference's sums of the few cells that can matter: the reference's search
// replayed over every split the certificate allows (RefKDTree::certified_search), first with
// what is known without sums; for the rows it leaves open, the reference's Kahan centroids of
// their candidates' parent cells (every code vector within a slack of the nearest that covers
// the reference's bits; the selected cells only), the replay again; for rows still open, the
// cells of the points a collecting replay blames, and once more.  done = false, nothing
// changed, when a row stays open: the caller then computes the whole split and its tree.
uint32_t cert_threads();
// The threads a check may use: cert_threads() (one while the main thread builds a kd-tree made
// the builds faster but the checks later: C4 6.88 vs 6.52 ms, profiles/r05z).
uint32_t cert_helpers(const qvq_ctx *) { return cert_threads(); }


// QVQ_CERT_TRACE=1: the certificate's phases, us since the check saw its level's export
struct CertTrace {
    bool on = false;
    std::chrono::steady_clock::time_point t0;
    std::string s;
    void mark(const char *what) {
        if (!on) return;
        char b[64];
        std::snprintf(b, sizeof(b), " %s %.0f", what,
                      std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        s += b;
    }
};
thread_local CertTrace cert_trace;

// The split rows of the cells cell_of (their reference bits, [2][S][D]: slot | S + slot) into a
// certificate's known split; the tree's replay caches updated for those points.
void cert_apply_cells(const RefKDTree &tree, CertState &cs, uint32_t Kc, uint32_t D, const std::vector<uint32_t> &cell_of,
                      const double *split) {
    const uint32_t S = (uint32_t)cell_of.size();
    std::vector<uint32_t> changed;
    for (uint32_t t = 0; t < S; t++)
        for (uint32_t h = 0; h < 2; h++) {
            const uint32_t r = cell_of[t] + h * Kc;
            std::memcpy(&cs.kp[(size_t)r * D], &split[((size_t)h * S + t) * D], D * 8);
            std::memset(&cs.known[(size_t)r * D], 1, D);
            changed.push_back(r);
        }
    tree.cert_update(changed.data(), changed.size());   // kp / known changed on these rows
    cs.rounds++;
}

// fn(t) for t = 0 .. n - 1: t = 0 on the calling thread, the others on the pool's threads
// (for replays of tens of us and more: a helper's wake-up costs about that).  A job is one
// epoch: a helper reads the epoch, want and fn together under the lock, so it runs each epoch
// at most once and never a stale fn; a helper spawned now starts from the current epoch (it
// never sees a finished job as new).  The caller's fn(0) and the wait for busy == 0 keep every
// helper's fn(t) inside this call.
void pool_run(qvq_ctx *ctx, uint32_t n, const std::function<void(uint32_t)> &fn) {
    qvq_ctx::Pool &P = ctx->pool;
    if (n <= 1) {
        fn(0);
        return;
    }
    while (P.th.size() + 1 < n) {
        const uint32_t t = (uint32_t)P.th.size() + 1;
        uint64_t start;
        {
            std::lock_guard<std::mutex> g(P.m);
            start = P.epoch.load();
        }
        P.th.emplace_back([&P, t, start, dev = ctx->dev] {
            (void)hipSetDevice(dev);
            uint64_t seen = start;
            for (;;) {
                uint32_t want;
                std::function<void(uint32_t)> job;
                {
                    std::unique_lock<std::mutex> lk(P.m);
                    P.cv.wait(lk, [&] { return P.stop.load() || P.epoch.load() != seen; });
                    if (P.stop.load()) return;
                    seen = P.epoch.load();
                    want = P.want.load();
                    if (t < want) job = P.fn;
                }
                if (t < want) {
                    job(t);
                    P.busy.fetch_sub(1, std::memory_order_acq_rel);
                }
            }
        });
        if (ctx->place_ok) pthread_setaffinity_np(P.th.back().native_handle(), sizeof(cpu_set_t), &ctx->place);
    }
    {
        std::lock_guard<std::mutex> g(P.m);
        P.fn = fn;
        P.want.store(n);
        P.busy.store(n - 1);
        P.epoch.fetch_add(1);
    }
    P.cv.notify_all();
    fn(0);
    while (P.busy.load(std::memory_order_acquire)) std::this_thread::yield();
}

// The certificate's known split: coordinates whose reference bits are the exact sums' without
// computing them -- a cell's exact mean is 0 or 1 only when all its values are (SCALED values lie
// in [0, 1], at least 1/(255 n) from 1 otherwise; Kahan sums of 0s and 1s are exact), split by 1.2
// or 0.8, and every component of a cell of at most two rows (its Kahan sum, of one value or two,
// is the exact sum rounded once: the same centroid bits; pcnt, the finalize's parent counts).
// The tree's replay caches are reset for it; with prepare also built (the aggregates and every
// node's replayed split: the last level's check does this before its tie rows arrive).
// par (optional): the rows and the aggregates over the certificate's helper threads (the last
// level's check sets up a K = 4096, D = 48 certificate after its tree: ~0.5 ms on one thread)
void cert_init(const RefKDTree &tree, CertState &cs, const double *cb, const std::vector<uint32_t> &pcnt, uint32_t K,
               uint32_t D, bool prepare, qvq_ctx *par = nullptr) {
    const uint32_t Kc = K / 2;
    cs.kp.resize((size_t)K * D);
    cs.known.resize((size_t)K * D);
    const bool counts = pcnt.size() == Kc;
    auto rows = [&](uint32_t j0, uint32_t j1) {
        std::memcpy(&cs.kp[(size_t)j0 * D], cb + (size_t)j0 * D, (size_t)(j1 - j0) * D * 8);
        for (uint32_t j = j0; j < j1; j++) {
            const double u = j < Kc ? 1 + 0.2 : 1 - 0.2;
            const double *v = &cs.kp[(size_t)j * D];
            uint8_t *k = &cs.known[(size_t)j * D];
            const bool few = counts && pcnt[j % Kc] <= 2;
            for (uint32_t d = 0; d < D; d++) k[d] = few || v[d] == 0 || std::fabs(v[d] - u) <= 1e-14;
        }
    };
    const uint32_t nt = par && (uint64_t)K * D >= 65536 ? std::min<uint32_t>(cert_helpers(par), 8) : 1;
    if (nt > 1)
        pool_run(par, nt, [&](uint32_t t) { rows((uint32_t)((uint64_t)K * t / nt), (uint32_t)((uint64_t)K * (t + 1) / nt)); });
    else
        rows(0, K);
    tree.cert_clear();   // kp / known: this level's (the vectors are reused)
    if (prepare) tree.cert_prepare(KAHAN_DELTA, cs.kp.data(), cs.known.data());
    cs.prepared = true;
}

// The certificate over cs.nu distinct rows cs.qs (nu x D values): cs.ans[u] the reference's
// index, or -1 for a row it leaves open.  tree: the level's tree over the exact-sum split cb (K
// code vectors); A_prev: the previous level's assignment (nullptr at K = 2: the parent cell is the
// mean of every row), whose selected cells are summed on stream (sync waits for them).
// defer (several ranks): a cell's rows are split over the ranks, so no cell is
// summed here: the rows the known coordinates leave open stay in cs.pend with every cell they
// need in cs.sel (their candidates' and the blamed points'), and cert_finish completes them once
// the ranks have summed those cells together (qvq_lbg).
template <class Sync>
qvq_status certify_rows(qvq_ctx *ctx, const RefKDTree &tree, const double *cb, const std::vector<uint32_t> &pcnt,
                        uint32_t K, const uint32_t *A_prev, hipStream_t stream, Sync sync, CertState &cs, bool defer,
                        uint32_t &open_rows) {
    const uint32_t D = ctx->D, Kc = K / 2, nu = cs.nu;
    const std::vector<double> &qs = cs.qs;
    std::vector<int64_t> &ans = cs.ans;
    if (!cs.prepared) cert_init(tree, cs, cb, pcnt, K, D, false);
    std::vector<double> &kp = cs.kp;
    std::vector<uint8_t> &known = cs.known;
    ans.assign(nu, -1);
    cs.pend.clear();
    cs.sel.assign(Kc, 0);
    // rows over host threads when the replays are long (48-D: the search visits most leaves)
    const bool long_search = (uint64_t)K * D >= 65536;   // 48-D: a search visits most leaves
    const uint32_t nthr = long_search ? std::min<uint32_t>(nu, cert_threads()) : 1;   // (the most)
    auto each = [&](const std::vector<uint32_t> &rows, auto &&fn) {   // fn(u, thread slot)
        // (per phase: one thread while the main thread builds a tree, cert_helpers)
        const uint32_t nthr = long_search ? std::min<uint32_t>(nu, cert_helpers(ctx)) : 1;
        if (nthr <= 1 || rows.size() < 2) {
            for (uint32_t u : rows) fn(u, 0u);
            return;
        }
        std::atomic<size_t> next{0};
        pool_run(ctx, std::min<uint32_t>(nthr, (uint32_t)rows.size()), [&](uint32_t t) {
            for (size_t i = next++; i < rows.size(); i = next++) fn(rows[i], t);
        });
    };
    std::vector<uint32_t> open, left;
    auto replay = [&](const std::vector<uint32_t> &rows) {
        each(rows, [&](uint32_t u, uint32_t) {
            ans[u] = tree.certified_search(&qs[(size_t)u * D], KAHAN_DELTA, kp.data(), known.data());
        });
        left.clear();
        for (uint32_t u : rows)
            if (ans[u] < 0) left.push_back(u);
        open.swap(left);
    };
    // each row's candidates (every code vector within a slack of the nearest that covers the
    // reference's bits); short searches replay every row at once and list candidates for the
    // rows left open only, long ones (48-D) replay at once only rows whose candidates are known
    std::vector<std::vector<uint32_t>> cand(nu);
    std::vector<uint32_t> all(nu);
    for (uint32_t u = 0; u < nu; u++) all[u] = u;
    auto near = [&](const std::vector<uint32_t> &rows) {
        each(rows, [&](uint32_t u, uint32_t) {
            double dmin;
            tree.near_set(&qs[(size_t)u * D], 1e-9, 1e-9, cand[u], dmin);
        });
        cert_trace.mark("near");
    };
    auto all_known = [&](uint32_t j) {
        for (uint32_t d = 0; d < D; d++)
            if (!known[(size_t)j * D + d]) return false;
        return true;
    };
    std::vector<uint32_t> ready, &pend = cs.pend;
    // long searches (48-D) list candidates first and skip the replays their unknown candidates
    // doom; short ones replay first and list candidates for the rows left open only (C3's last
    // level: 2 rows, near sets 36 us of a 53 us check after the export, profiles/r05p)
    const bool near_first = long_search;
    if (near_first) {
        near(all);
        for (uint32_t u = 0; u < nu; u++) {
            bool k = true;
            for (uint32_t j : cand[u]) k = k && all_known(j);
            (k ? ready : pend).push_back(u);
        }
    } else {
        ready = all;
    }
    if (!ready.empty()) {
        replay(ready);
        pend.insert(pend.end(), open.begin(), open.end());
        cert_trace.mark("replay");
        if (!near_first) near(pend);
    }
    std::vector<uint8_t> &sel = cs.sel;
    cs.cells = cs.rounds = 0;
    auto want = [&](uint32_t j) {
        if (all_known(j)) return;
        cs.cells += !sel[j % Kc];
        sel[j % Kc] = 1;
    };
    // the reference's centroids of the selected cells (of the previous level's assignment),
    // compacted to slots; the split rows (slot | S + slot) land in mapped host memory
    std::vector<uint32_t> cell_of;
    auto launch_cells = [&](const std::vector<uint8_t> &pick) -> qvq_status {
        qvq_status s2;
        if ((s2 = ensure_kahan(ctx, Kc)) != QVQ_OK) return s2;
        cell_of.clear();
        for (uint32_t c = 0; c < Kc; c++) {
            ctx->h_kc_sel[c] = pick[c] ? (uint32_t)cell_of.size() + 1 : 0u;
            if (pick[c]) cell_of.push_back(c);
        }
        if (A_prev) {
            // the longest chain (the finalize's parent counts): short ones run step by step
            uint64_t max_rows = pcnt.size() == Kc ? 1 : 0;
            for (uint32_t c : cell_of) max_rows = max_rows ? std::max<uint64_t>(max_rows, pcnt[c]) : 0;
            HIPCHK(hipMemcpyAsync(ctx->d_kc_sel, ctx->h_kc_sel, (size_t)Kc * 4, hipMemcpyHostToDevice, stream));
            HIPCHK(launch_kahan_centroids(stream, ctx->kw, ctx->d_codes, ctx->Dp, D, ctx->N, A_prev,
                                          (uint32_t)cell_of.size(), ctx->d_kc_cent, ctx->dh_kc_out, ctx->d_kc_sel, Kc,
                                          max_rows));
        } else {   // K = 2: the one parent cell is the mean of every row
            HIPCHK(launch_kahan_centroids(stream, ctx->kw, ctx->d_codes, ctx->Dp, D, ctx->N, nullptr, 1,
                                          ctx->d_kc_cent, ctx->dh_kc_out, nullptr, 0, ctx->N));
        }
        cert_trace.mark("launched");
        return QVQ_OK;
    };
    auto finish_cells = [&]() -> qvq_status {
        qvq_status s2;
        if ((s2 = sync()) != QVQ_OK) return s2;
        cert_trace.mark("sums");
        cert_apply_cells(tree, cs, Kc, D, cell_of, ctx->h_kc_out);
        return QVQ_OK;
    };
    open.clear();
    if (!pend.empty() && (K >= 4 ? A_prev != nullptr : K == 2)) {
        // the candidates' cells on the GPU while a collecting replay finds the points whose bits
        // settle the decisions the intervals leave open (with the candidates unknown, it blames
        // them too); their cells, if new, in a second round
        qvq_status st;
        for (uint32_t u : pend)
            for (uint32_t j : cand[u]) want(j);
        std::vector<uint8_t> first = sel;
        if (cs.cells && !defer && (st = launch_cells(first)) != QVQ_OK) return st;
        std::vector<std::vector<uint32_t>> blame(std::max<uint32_t>(nthr, 1));
        each(pend, [&](uint32_t u, uint32_t t) {
            tree.certify_blame(&qs[(size_t)u * D], KAHAN_DELTA, kp.data(), known.data(), blame[t]);
        });
        const uint32_t c0 = cs.cells;
        for (const auto &b : blame)
            for (uint32_t j : b) want(j);
        cert_trace.mark("blame");
        if (defer) {   // the cells come from every rank's rows (cert_finish)
            open_rows = (uint32_t)pend.size();
            return QVQ_OK;
        }
        if (c0 && (st = finish_cells()) != QVQ_OK) return st;
        if (cs.cells > c0) {
            std::vector<uint8_t> more(Kc, 0);
            for (uint32_t c = 0; c < Kc; c++) more[c] = sel[c] && !first[c];
            if ((st = launch_cells(more)) != QVQ_OK || (st = finish_cells()) != QVQ_OK) return st;
        }
        replay(pend);
        cert_trace.mark("replay");
    } else {
        open = pend;
    }
    pend = open;
    open_rows = (uint32_t)open.size();
    return QVQ_OK;
}

// The deferred rows (certify_rows with defer) once the cells cell_of have their reference bits:
// split rows at split ([2][S][D]: slot | S + slot); returns the rows still open.
uint32_t cert_finish(const RefKDTree &tree, CertState &cs, uint32_t K, uint32_t D, const std::vector<uint32_t> &cell_of,
                     const double *split) {
    cert_apply_cells(tree, cs, K / 2, D, cell_of, split);
    tree.cert_clear();   // (every thread's cache: the replays run here, the defer's ran elsewhere)
    std::vector<uint32_t> open;
    for (uint32_t u : cs.pend) {
        cs.ans[u] = tree.certified_search(&cs.qs[(size_t)u * D], KAHAN_DELTA, cs.kp.data(), cs.known.data());
        if (cs.ans[u] < 0) open.push_back(u);
    }
    cs.pend.swap(open);
    return (uint32_t)cs.pend.size();
}

// A settled row whose reference index is not its speculative one (the quantize must be redone).
bool cert_mismatch(const CertState &cs, uint32_t K) {
    for (size_t i = 0; i < cs.rows.size(); i++) {
        const int64_t a = cs.ans[cs.of[i]];
        if (a >= 0 && (uint32_t)a != cs.spec[i]) {
            if (env_is("QVQ_KAHAN_DEBUG", "1"))
                std::fprintf(stderr, "qvq kahan: K %u row %u: speculative %u, the reference %lld\n", K, cs.rows[i],
                             cs.spec[i], (long long)a);
            return true;
        }
    }
    return false;
}

// Host threads for the certificate's replays (at most 8, half the machine's).
uint32_t cert_threads() {
    static const uint32_t n = [] {
        // (C4 at 1 / 2 / 4 / 8 helpers is within the boxes' run-to-run spread, 6.8-7.6 ms:
        // profiles/r05s, r05u)
        return std::max<uint32_t>(1, std::min<uint32_t>(8, std::thread::hardware_concurrency() / 2));
    }();
    return n;
}

// Distinct rows of n row records (code bytes at code + i * stride, D of them): their values qs,
// and of[i] = the distinct row of record i.
uint32_t distinct_rows(const qvq_ctx *ctx, const uint8_t *code, size_t stride, uint32_t n, std::vector<double> &qs,
                       std::vector<uint32_t> &of) {
    std::unordered_map<std::string, uint32_t> uniq;
    of.resize(n);
    qs.clear();
    for (uint32_t i = 0; i < n; i++) {
        const uint8_t *c = code + (size_t)i * stride;
        const auto it = uniq.emplace(std::string(reinterpret_cast<const char *>(c), ctx->D), (uint32_t)uniq.size());
        of[i] = it.first->second;
        if (it.second)
            for (uint32_t d = 0; d < ctx->D; d++) qs.push_back(ctx->terms.v64[c[d]]);
    }
    return (uint32_t)uniq.size();
}

qvq_status certify_kahan_ties(qvq_ctx *ctx, uint32_t K, unsigned nt, uint64_t *target, bool &done) {
    done = false;
    if (!ctx->tree || ctx->cb_local.size() != (size_t)K * ctx->D || K < 2) return QVQ_OK;
    const uint32_t D = ctx->D, Dp = ctx->Dp;
    const uint64_t need = (uint64_t)nt * (4 + Dp);
    if (ctx->scatter_bytes < need) {
        dfree(ctx->d_scatter);
        HIPCHK(hipMalloc(&ctx->d_scatter, need));
        ctx->scatter_bytes = need;
    }
    uint32_t *d_vals = ctx->d_scatter;
    uint8_t *d_gath = reinterpret_cast<uint8_t *>(ctx->d_scatter + nt);
    std::vector<uint8_t> code((uint64_t)nt * Dp);
    HIPCHK(launch_gather_codes(ctx->stream, ctx->d_codes, Dp, ctx->d_ties, nt, d_gath));
    HIPCHK(hipMemcpyAsync(code.data(), d_gath, code.size(), hipMemcpyDeviceToHost, ctx->stream));
    qvq_status st;
    if ((st = wait_stream(ctx)) != QVQ_OK) return st;
    CertState cs;
    cs.nu = distinct_rows(ctx, code.data(), Dp, nt, cs.qs, cs.of);
    uint32_t open = 0;
    if ((st = certify_rows(ctx, *ctx->tree, ctx->cb_local.data(), ctx->cnt_local, K, K == 2 ? nullptr : ctx->d_A_alt, ctx->stream,
                           [ctx] { return wait_stream(ctx); }, cs, false, open)) != QVQ_OK)
        return st;
    if (open) {
        if (env_is("QVQ_KAHAN_DEBUG", "1"))
            std::fprintf(stderr, "qvq kahan: K %u ties %u (%u distinct) cells %u: %u rows not certified\n", K, nt, cs.nu,
                         cs.cells, open);
        return QVQ_OK;
    }
    std::vector<uint32_t> &vals = ctx->cert_vals;   // outlives the copy (no wait)
    vals.resize(nt);
    for (uint32_t i = 0; i < nt; i++) vals[i] = (uint32_t)cs.ans[cs.of[i]];
    HIPCHK(hipMemcpyAsync(d_vals, vals.data(), nt * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(launch_fix_rows(ctx->stream, ctx->d_codes, Dp, D, ctx->d_A, ctx->d_ties, d_vals, nt, K, nullptr, nullptr,
                           ctx->d_plut, target));
    if (env_is("QVQ_KAHAN_DEBUG", "1"))
        std::fprintf(stderr, "qvq kahan: K %u ties %u (%u distinct) certified, cells summed %u in %u rounds\n", K, nt,
                     cs.nu, cs.cells, cs.rounds);
    done = true;
    return QVQ_OK;
}

// The speculative check of one level (on the worker): the level's tie rows and their
// speculative indices (exported with its codebook) against the reference's, by the certificate
// over the level's tree.  status 0: all equal; 1: a row differs or stays open (qvq_lbg then
// redoes the quantize with the synchronous Kahan levels); 2 (several ranks): the rows settled
// so far agree and the rest wait for cells summed over every rank's rows (v.cs, cert_finish).
// QVQ_KAHAN_FAIL_LEVEL=L (tests): level L's check fails (on rank QVQ_KAHAN_FAIL_RANK, default
// every rank), exercising the redo.
void verify_level(qvq_ctx *ctx, qvq_ctx::Verify &v) {
    v.status = 1;
    ctx->htrace.mark("check K" + std::to_string(v.K) + " start");
    struct End {
        qvq_ctx *c;
        const qvq_ctx::Verify &v;
        ~End() { c->htrace.mark("check K" + std::to_string(v.K) + " end, status " + std::to_string(v.status)); }
    } end_mark{ctx, v};
    (void)hipSetDevice(ctx->dev);
    // the check usually starts while the GPU still runs its level (the last level's check is
    // then all that is left of the call): the known split and the tree's aggregates before the
    // export arrives, and for short searches (D = 12: a few hundred nodes) every node's split
    // replay too (C3: the last level's 2 tie rows took ~95 us after the export, r05i)
    // (C3 1.241 -> 1.197 ms, C4 7.51 -> 7.18, profiles/r05p)
    if (!v.cs.prepared && v.tree && !v.tree->cancelled() && v.K >= 2 &&
        v.cb.size() == (size_t)v.K * ctx->D) {
        const bool full = (uint64_t)v.K * ctx->D < 65536;
        cert_init(*v.tree, v.cs, v.cb.data(), v.cnt, v.K, ctx->D, full, ctx);
        ctx->htrace.mark("check K" + std::to_string(v.K) + " known split set");
        if (!full)
            v.tree->cert_warm(KAHAN_DELTA, v.cs.kp.data(), v.cs.known.data(), cert_helpers(ctx),
                              [ctx](unsigned n, const std::function<void(unsigned)> &fn) { pool_run(ctx, n, fn); });
        ctx->htrace.mark("check K" + std::to_string(v.K) + " aggregates set");
    }
    volatile uint64_t *flag = ctx->h_ready;
    while (*flag < v.seq) {   // the export is released with the codebook's ready number
        if (v.cancel.load(std::memory_order_relaxed)) return;
        cpu_relax();
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    ctx->htrace.mark("check K" + std::to_string(v.K) + " export seen");
    static const int fail_level = std::getenv("QVQ_KAHAN_FAIL_LEVEL") ? std::atoi(std::getenv("QVQ_KAHAN_FAIL_LEVEL")) : 0;
    static const int fail_rank = std::getenv("QVQ_KAHAN_FAIL_RANK") ? std::atoi(std::getenv("QVQ_KAHAN_FAIL_RANK")) : -1;
    if (fail_level && (int)v.level == fail_level && (fail_rank < 0 || fail_rank == ctx->rank)) return;
    static const bool trace = env_is("QVQ_CERT_TRACE", "1");
    cert_trace.on = trace;
    cert_trace.t0 = std::chrono::steady_clock::now();
    cert_trace.s.clear();
    const uint32_t *tx = reinterpret_cast<const uint32_t *>(ctx->h_tx[v.par]);
    const uint32_t nt = tx[0];
    if (nt == 0) {
        v.status = 0;
        return;
    }
    if (nt > ctx->tx_cap) {
        ctx->tm.tie_overflow++;
        return;
    }
    if (!v.tree || v.tree->cancelled() || v.K < 2) return;
    const uint32_t Dp = ctx->Dp, words = 2 + Dp / 4;
    std::vector<uint32_t> rec(tx + 2, tx + 2 + (size_t)nt * words);   // out of the mapped buffer at once
    CertState &cs = v.cs;
    cs.rows.resize(nt);
    cs.spec.resize(nt);
    for (uint32_t i = 0; i < nt; i++) {
        cs.rows[i] = rec[(size_t)i * words];
        cs.spec[i] = rec[(size_t)i * words + 1];
        if (cs.rows[i] >= ctx->N || cs.spec[i] >= v.K) return;
    }
    cs.nu = distinct_rows(ctx, reinterpret_cast<const uint8_t *>(rec.data() + 2), (size_t)words * 4, nt, cs.qs, cs.of);
    uint32_t open = 0;
    // the selected cells' sums on the check's stream: a bounded poll that also ends when the
    // call cancels the check (a failed wait in qvq_lbg), so joining a cancelled check is prompt
    auto sync = [ctx, &v]() -> qvq_status {
        const auto until = std::chrono::steady_clock::now() + std::chrono::duration<double>(ctx->timeout_s);
        for (;;) {
            const hipError_t q = hipStreamQuery(ctx->vstream);
            if (q == hipSuccess) return QVQ_OK;
            if (q != hipErrorNotReady) return QVQ_EDEVICE;
            if (v.cancel.load(std::memory_order_relaxed) || std::chrono::steady_clock::now() > until)
                return QVQ_EDEVICE;
            std::this_thread::yield();
        }
    };
    const bool defer = ctx->nranks > 1;
    // (A_prev is complete: the GPU wrote the flag seen above after the levels that made it)
    if (certify_rows(ctx, *v.tree, v.cb.data(), v.cnt, v.K, v.A_prev, ctx->vstream, sync, cs, defer, open) != QVQ_OK ||
        (open && !defer))
        return;
    // QVQ_KAHAN_OPEN_LEVEL=L (tests; -1: every level): a row of level L left open with no cell
    // wanted, on rank QVQ_KAHAN_FAIL_RANK (default every rank) -- the state that no later sum can
    // settle, which must end in the redo
    static const int open_level = std::getenv("QVQ_KAHAN_OPEN_LEVEL") ? std::atoi(std::getenv("QVQ_KAHAN_OPEN_LEVEL")) : 0;
    if (open_level && (open_level < 0 || (int)v.level == open_level) && (fail_rank < 0 || fail_rank == ctx->rank) &&
        cs.nu > 0) {
        if (cs.pend.empty()) cs.pend.push_back(0);
        open = (uint32_t)cs.pend.size();
        cs.sel.assign(v.K / 2, 0);
        cs.cells = 0;
    }
    // open rows that want no cell (their candidates all known, yet a decision left open): no
    // cell summed over the ranks can settle them, so the level fails here (several ranks: a
    // deferred entry without cells would be skipped by resolve_deferred, keeping unconfirmed
    // speculative indices)
    if (open && cs.cells == 0) return;
    if (cert_mismatch(cs, v.K)) return;
    cert_trace.mark("done");
    if (env_is("QVQ_KAHAN_DEBUG", "1") || trace)
        std::fprintf(stderr, "qvq kahan: K %u ties %u (%u distinct) %s, cells %s %u in %u rounds%s%s\n", v.K, nt, cs.nu,
                     open ? "deferred" : "verified", open ? "wanted" : "summed", cs.cells, cs.rounds,
                     trace ? " | us:" : "", cert_trace.s.c_str());
    v.status = open ? 2 : 0;
}

// The check's verdict (status 0 / 1 / 2, -1: none posted); its tree and rows are released,
// except a deferred check's (status 2, several ranks), which moves to ctx->deferred.

// free_on_worker: the check's tree and state are destroyed on the worker, not here (the last
// level's at the end of a call: C4's K = 4096 tree and certificate free ~30 us of buffers, with
// the munmaps' TLB shootdowns, while the caller waits)
int join_verify(qvq_ctx *ctx, qvq_ctx::Verify &v, bool free_on_worker = false) {
    if (!v.posted) return -1;
    while (!v.done.load(std::memory_order_acquire)) std::this_thread::yield();
    v.posted = false;
    const int status = v.status;
    if (status == 2) {
        qvq_ctx::Deferred d;
        d.level = v.level;
        d.K = v.K;
        d.A_prev = v.A_prev;
        d.tree = std::move(v.tree);
        d.cb = std::move(v.cb);
        d.cs = std::move(v.cs);
        ctx->deferred.push_back(std::move(d));
    }
    if (free_on_worker && v.tree) {
        RefKDTree *t = v.tree.release();
        CertState *c = new CertState(std::move(v.cs));
        post_job(ctx, [t, c] {
            delete t;
            delete c;
        }, nullptr);
    }
    v.tree.reset();
    v.cs = CertState();
    return status;
}

// join_verify within the context's wait bounds: a failed stream or communicator, or a timeout,
// fails the call as any other wait does (wait_failed; a drained stream is no failure here: the
// check's host replays may outlast the GPU's work).  ok = not failed (status 0, 2 or none).
qvq_status join_verify_bounded(qvq_ctx *ctx, qvq_ctx::Verify &v, bool &ok, bool free_on_worker = false) {
    ok = true;
    if (!v.posted) return QVQ_OK;
    std::string err;
    const qvq_status st = wait_until(
        [&] { return v.done.load(std::memory_order_acquire); },
        [&](std::string &m) {
            const StreamState ss = probe_stream(ctx, m);
            return ss == StreamState::Drained ? StreamState::Running : ss;
        },
        [&](std::string &m) { return probe_comm(ctx, m); }, ctx->timeout_s, err);
    if (st != QVQ_OK) {
        for (auto &u : ctx->ver) u.cancel.store(true);
        return wait_failed(ctx, fail(ctx, st, err));
    }
    ok = join_verify(ctx, v, free_on_worker) != 1;
    return QVQ_OK;
}

// The speculative check's buffers (once per context): the third assignment buffer, the mapped
// tie exports, the check's stream and events, and the Kahan work for the largest level.
qvq_status ensure_speculation(qvq_ctx *ctx, uint32_t Kmax) {
    if (!ctx->d_A_alt) HIPCHK(hipMalloc(&ctx->d_A_alt, ctx->N * 4));
    if (!ctx->d_A3) HIPCHK(hipMalloc(&ctx->d_A3, ctx->N * 4));
    if (!ctx->d_A4) HIPCHK(hipMalloc(&ctx->d_A4, ctx->N * 4));
    if (!ctx->h_tx[0]) {
        ctx->tx_cap = 65536;
        const size_t bytes = 8 + (size_t)ctx->tx_cap * (8 + 64);
        for (int i = 0; i < 3; i++) {
            HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_tx[i]), bytes, hipHostMallocMapped));
            HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void **>(&ctx->dh_tx[i]), ctx->h_tx[i], 0));
        }
    }
    if (!ctx->vstream) {   // high priority: the check's few short kernels go ahead of the next search's queued blocks
        int lo = 0, hi = 0;
        if (hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess && hi != lo)
            HIPCHK(hipStreamCreateWithPriority(&ctx->vstream, hipStreamNonBlocking, hi));
        else
            HIPCHK(hipStreamCreateWithFlags(&ctx->vstream, hipStreamNonBlocking));
    }
    for (auto &v : ctx->ver)
        if (!v.ev) HIPCHK(hipEventCreateWithFlags(&v.ev, hipEventDisableTiming));
    return Kmax >= 4 ? ensure_kahan(ctx, Kmax / 2) : QVQ_OK;
}

// The ties of a level run with defer_ties (nt > 0 of them in d_ties): the reference's split
// codebook -- the previous level's centroids as Kahan sums in row order (k_kahan.hip; for the
// NORMAL colour space the exact sums are those bits already), split -- its kd-tree, and the
// ties answered against both (every distance recomputed from the reference's code vectors).
// The moves go to sums copy 1 (fused: the finalize adds it) or straight into copy 0.
qvq_status resolve_kahan_ties(qvq_ctx *ctx, uint32_t K, int slot, unsigned nt, bool fused) {
    const uint32_t D = ctx->D, Kc = K / 2;
    const double *S_ref = ctx->d_C64_split;
    qvq_status st;
    uint64_t *target = fused ? ctx->d_sums + sums_cap_stride(ctx) : ctx->d_sums;
    if (ctx->cs == QVQ_CS_SCALED) {
        bool done;
        if ((st = certify_kahan_ties(ctx, K, nt, target, done)) != QVQ_OK || done) return st;
        if ((st = ensure_kahan(ctx, Kc)) != QVQ_OK) return st;
        HIPCHK(launch_kahan_centroids(ctx->stream, ctx->kw, ctx->d_codes, ctx->Dp, D, ctx->N,
                                      K == 2 ? nullptr : ctx->d_A_alt, Kc, ctx->d_kc_cent, ctx->d_kc_split));
        S_ref = ctx->d_kc_split;
        if (env_is("QVQ_KAHAN_DEBUG", "1")) {   // blocks not composable, block misses, segment replays
            unsigned ms[4];
            HIPCHK(hipMemcpyAsync(ms, ctx->kw.stats, sizeof(ms), hipMemcpyDeviceToHost, ctx->stream));
            HIPCHK(hipMemsetAsync(ctx->kw.stats, 0, sizeof(ms), ctx->stream));
            HIPCHK(hipStreamSynchronize(ctx->stream));
            std::fprintf(stderr, "qvq kahan: K %u level ties %u blocks not composable %u block misses %u replays %u\n",
                         K, nt, ms[0], ms[1], ms[2]);
        }
    }
    ctx->h_kc_split.resize((size_t)K * D);
    HIPCHK(hipMemcpyAsync(ctx->h_kc_split.data(), S_ref, (size_t)K * D * 8, hipMemcpyDeviceToHost, ctx->stream));
    if ((st = wait_stream(ctx)) != QVQ_OK) return st;
    KdView kd;
    // the level's tree (over the exact-sum split, built during the search) is the reference's
    // tree too when no differing coordinate can move a box, cut or partition (kdtree.cpp)
    if (ctx->tree && ctx->tree_kd.depth > 0 && ctx->cb_local.size() == (size_t)K * D &&
        ctx->tree->unchanged_under(ctx->h_kc_split.data())) {
        kd = ctx->tree_kd;
        if (env_is("QVQ_KAHAN_DEBUG", "1")) std::fprintf(stderr, "qvq kahan: K %u the level's tree reused\n", K);
    } else {
        build_tree(ctx, ctx->h_kc_split.data(), K, slot & 1, kd);
    }
    unsigned *cnt = ctx->d_counters + 2 * slot;
    if (kd.depth > 0) {
        HIPCHK(launch_kd_resolve(ctx->stream, ctx->d_codes, ctx->Dp, D, ctx->d_ties, &cnt[1], S_ref, K, ctx->d_lut64,
                                 kd, ctx->d_A, nullptr, nullptr, ctx->d_plut, target));
        return QVQ_OK;
    }
    return resolve_host_ties(ctx, ctx->h_kc_split.data(), K, nt, false, target);
}

// resolve_kahan_ties on several ranks (a level with ties on any rank, every rank calls it): the
// reference's whole split from the chains over every rank's rows (kahan_chained), its kd-tree,
// this rank's ties (nt) answered against both, and the ties' moves of every rank summed (sums
// copy 1, added by the finalize that follows).
qvq_status resolve_kahan_ties_multi(qvq_ctx *ctx, uint32_t K, int slot, unsigned nt) {
    const uint32_t D = ctx->D, Kc = K / 2;
    qvq_status st;
    uint64_t *target = ctx->d_sums + sums_cap_stride(ctx);
    if ((st = kahan_chained(ctx, K == 2 ? nullptr : ctx->d_A_alt, Kc, nullptr, Kc, true)) !=
        QVQ_OK)
        return st;
    ctx->h_kc_split.resize((size_t)K * D);
    HIPCHK(hipMemcpyAsync(ctx->h_kc_split.data(), ctx->d_kc_split, (size_t)K * D * 8, hipMemcpyDeviceToHost, ctx->stream));
    if ((st = wait_stream(ctx)) != QVQ_OK) return st;
    if (nt) {
        KdView kd;
        if (ctx->tree && ctx->tree_kd.depth > 0 && ctx->cb_local.size() == (size_t)K * D &&
            ctx->tree->unchanged_under(ctx->h_kc_split.data()))
            kd = ctx->tree_kd;
        else
            build_tree(ctx, ctx->h_kc_split.data(), K, slot & 1, kd);
        unsigned *cnt = ctx->d_counters + 2 * slot;
        if (kd.depth > 0)
            HIPCHK(launch_kd_resolve(ctx->stream, ctx->d_codes, ctx->Dp, D, ctx->d_ties, &cnt[1], ctx->d_kc_split, K,
                                     ctx->d_lut64, kd, ctx->d_A, nullptr, nullptr, ctx->d_plut, target));
        else if ((st = resolve_host_ties(ctx, ctx->h_kc_split.data(), K, nt, false, target)) != QVQ_OK)
            return st;
    }
    return all_reduce_sums(ctx, K, target);
}

// Several ranks, at the end of a speculative qvq_lbg: the checks whose rows wait
// for cells summed over every rank's rows (ctx->deferred).  A vote of every rank's failure and,
// per level, of the cells its open rows need; then for each level with cells wanted (ascending,
// every rank the same), their reference bits from the chains over every rank's rows
// (kahan_chained on the level's parent assignment, alev[L - 1]) and this rank's open rows
// replayed with them (cert_finish); a second vote of the failures.  failed: in, this rank's
// failure so far; out, any rank's (the quantize is then redone on every rank).
qvq_status resolve_deferred(qvq_ctx *ctx, uint32_t bits, const std::vector<uint32_t *> &alev, bool &failed) {
    const uint32_t D = ctx->D;
    // [0] failures | per level L: its parent cells (2^(L-1)), four 16-bit counts per word
    std::vector<uint64_t> off(bits + 2, 1);
    for (uint32_t L = 1; L <= bits; L++) off[L + 1] = off[L] + ((1ull << (L - 1)) + 3) / 4;
    std::vector<uint64_t> v(off[bits + 1], 0);
    v[0] = failed ? 1 : 0;
    for (const auto &d : ctx->deferred)
        for (uint32_t c = 0; c < d.K / 2; c++)
            if (d.cs.sel[c]) v[off[d.level] + c / 4] |= 1ull << (16 * (c % 4));
    qvq_status st;
    if ((st = vote(ctx, v.data(), v.size())) != QVQ_OK) return st;
    if (v[0]) {
        failed = true;
        return QVQ_OK;
    }
    bool local_fail = false;
    std::vector<uint32_t> cell_of;
    std::vector<double> split;
    for (uint32_t L = 1; L <= bits; L++) {
        const uint32_t Kc = 1u << (L - 1);
        cell_of.clear();
        for (uint32_t c = 0; c < Kc; c++)
            if ((v[off[L] + c / 4] >> (16 * (c % 4))) & 0xFFFF) cell_of.push_back(c);
        if (cell_of.empty()) {   // no rank wants a cell here: rows still open stay open (a redo)
            for (const auto &d : ctx->deferred)
                if (d.level == L && !d.cs.pend.empty()) local_fail = true;
            continue;
        }
        ctx->tm.kahan_relays++;
        const uint32_t S = (uint32_t)cell_of.size();
        if ((st = ensure_kahan(ctx, Kc)) != QVQ_OK) return st;
        if (L >= 2) {
            for (uint32_t c = 0; c < Kc; c++) ctx->h_kc_sel[c] = 0;
            for (uint32_t t = 0; t < S; t++) ctx->h_kc_sel[cell_of[t]] = t + 1;
            HIPCHK(hipMemcpyAsync(ctx->d_kc_sel, ctx->h_kc_sel, (size_t)Kc * 4, hipMemcpyHostToDevice, ctx->stream));
            st = kahan_chained(ctx, alev[L - 1], Kc, ctx->d_kc_sel, S, true);
        } else {
            st = kahan_chained(ctx, nullptr, 1, nullptr, 1, true);
        }
        if (st != QVQ_OK) return st;
        split.resize(2ull * S * D);
        HIPCHK(hipMemcpyAsync(split.data(), ctx->d_kc_split, split.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
        if ((st = wait_stream(ctx)) != QVQ_OK) return st;
        for (auto &d : ctx->deferred) {
            if (d.level != L) continue;
            const uint32_t open = cert_finish(*d.tree, d.cs, d.K, D, cell_of, split.data());
            const bool bad = open || cert_mismatch(d.cs, d.K);
            if (env_is("QVQ_KAHAN_DEBUG", "1"))
                std::fprintf(stderr, "qvq kahan: rank %d K %u deferred rows finished over %u cells: %s\n", ctx->rank,
                             d.K, S, open ? "rows left open" : bad ? "a row differs" : "verified");
            local_fail = local_fail || bad;
        }
    }
    uint64_t f = local_fail ? 1 : 0;
    if ((st = vote(ctx, &f, 1)) != QVQ_OK) return st;
    failed = f != 0;
    return QVQ_OK;
}

// The byte histogram of the resident rows (kept on the device: qvq_lbg derives sum ||x||^2 and
// the row count from it, after summing it over the ranks).
qvq_status compute_xsq(qvq_ctx *ctx) {
    HIPCHK(launch_byte_hist(ctx->stream, ctx->d_codes, ctx->N, ctx->D, ctx->Dp, ctx->d_hist));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return QVQ_OK;
}

qvq_status check_image_args(qvq_ctx *ctx, uint32_t n_images, uint32_t xSize, uint32_t ySize, uint32_t bw,
                            uint32_t bh, uint64_t &N, uint32_t &D) {
    if (!ctx) return QVQ_EINVAL;
    if (n_images == 0 || xSize == 0 || ySize == 0 || bw == 0 || bh == 0)
        return fail(ctx, QVQ_EINVAL, "image and block sizes must be positive");
    N = (uint64_t)((xSize + bw - 1) / bw) * ((ySize + bh - 1) / bh) * n_images;
    D = 3 * bw * bh;
    return QVQ_OK;
}

qvq_status tile_into(qvq_ctx *ctx, const uint8_t *d_rgb, uint32_t n_images, uint32_t xSize, uint32_t ySize,
                     uint32_t bw, uint32_t bh) {
    ctx->col_blocks = (ySize + bh - 1) / bh;   // the pruned wide search stacks its chunks across columns
    HIPCHK(launch_tile(ctx->stream, d_rgb, ctx->d_codes, n_images, xSize, ySize, bw, bh, ctx->D, ctx->Dp,
                       ctx->terms.pad_code));
    return QVQ_OK;
}

}  // namespace

extern "C" {

QVQ_API const char *qvq_version(void) { return "qvq 0.2 (gfx950, f16 MFMA search)"; }

QVQ_API const char *qvq_last_error(const qvq_ctx *ctx) { return ctx ? ctx->err.c_str() : g_static_err.c_str(); }

QVQ_API qvq_status qvq_create(int hip_device, qvq_ctx **out) {
    if (!out) return QVQ_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(nullptr, QVQ_EDEVICE, "no HIP device");
    if (hip_device < 0 || hip_device >= n) return fail(nullptr, QVQ_EINVAL, "bad device index");
    qvq_ctx *ctx = new qvq_ctx();
    ctx->dev = hip_device;
    if (const char *t = std::getenv("QVQ_TIMING")) ctx->timing_level = std::atoi(t);   // A/B: the default per-level events
    std::memset(&ctx->tm, 0, sizeof(ctx->tm));
    auto bail = [&](hipError_t e, const char *what) {
        g_static_err = std::string(what) + ": " + hipGetErrorString(e);
        qvq_destroy(ctx);
        return QVQ_EDEVICE;
    };
    hipError_t e;
    if ((e = hipSetDevice(hip_device)) != hipSuccess) return bail(e, "hipSetDevice");
    hipDeviceProp_t prop;
    if ((e = hipGetDeviceProperties(&prop, hip_device)) != hipSuccess) return bail(e, "hipGetDeviceProperties");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        g_static_err = std::string("libqvq is built for gfx950, device is ") + prop.gcnArchName;
        qvq_destroy(ctx);
        return QVQ_EDEVICE;
    }
    ctx->num_cu = prop.multiProcessorCount;
    ctx->G = (uint32_t)ctx->num_cu;   // one search/update workgroup (and slab) per CU
    if ((e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)) != hipSuccess) return bail(e, "stream");
    if ((e = hipMalloc(&ctx->d_lut32, 256 * 4)) != hipSuccess) return bail(e, "hipMalloc");
    if ((e = hipMalloc(&ctx->d_w, 256 * 4)) != hipSuccess) return bail(e, "hipMalloc");
    if ((e = hipMalloc(&ctx->d_lut64, 256 * 8)) != hipSuccess) return bail(e, "hipMalloc");
    if ((e = hipMalloc(&ctx->d_plut, 256 * 8)) != hipSuccess) return bail(e, "hipMalloc");
    // mapped: [0, 64) the codebook ready number, [64, 1024) a quantize's small results
    if ((e = hipHostMalloc(&ctx->h_ready, 1024, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
        return bail(e, "hipHostMalloc");
    *ctx->h_ready = 0;
    if ((e = hipHostGetDevicePointer((void **)&ctx->dh_ready, ctx->h_ready, 0)) != hipSuccess)
        return bail(e, "hipHostGetDevicePointer");
    if ((e = hipMalloc(&ctx->d_counters, N_COUNTERS * sizeof(unsigned))) != hipSuccess) return bail(e, "hipMalloc");
    if ((e = hipMemset(ctx->d_counters, 0, N_COUNTERS * sizeof(unsigned))) != hipSuccess) return bail(e, "hipMemset");
    if ((e = hipMalloc(&ctx->d_hist, 512 * 8)) != hipSuccess) return bail(e, "hipMalloc");
    if ((e = hipMalloc(&ctx->d_decode_stat, 16)) != hipSuccess) return bail(e, "hipMalloc");
    if ((e = hipHostMalloc(&ctx->h_decode_stat, 16, hipHostMallocDefault)) != hipSuccess) return bail(e, "hipHostMalloc");
    if ((e = hipMalloc(&ctx->d_dist_part, 8192 * 8)) != hipSuccess) return bail(e, "hipMalloc");
    if ((e = hipMalloc(&ctx->d_mean, MEAN_COPIES * (2 * 64 + 1) * 8)) != hipSuccess) return bail(e, "hipMalloc");
    if ((e = hipMemset(ctx->d_mean, 0, MEAN_COPIES * (2 * 64 + 1) * 8)) != hipSuccess) return bail(e, "hipMemset");
    for (int l = 0; l < 32; l++)
        for (int j = 0; j < 4; j++)
            if ((e = hipEventCreate(&ctx->ev[l][j])) != hipSuccess) return bail(e, "hipEventCreate");
    if ((e = hipEventCreate(&ctx->ev_end)) != hipSuccess) return bail(e, "hipEventCreate");
    if ((e = hipEventCreateWithFlags(&ctx->ev_sync, hipEventDisableTiming)) != hipSuccess)
        return bail(e, "hipEventCreate");
    if (const char *t = std::getenv("QVQ_TIMEOUT_S")) ctx->timeout_s = std::max(0.001, std::atof(t));
    ctx->ev_ready = true;
    *out = ctx;
    return QVQ_OK;
}

QVQ_API void qvq_destroy(qvq_ctx *ctx) {
    if (!ctx) return;
    join_tree_job(ctx, true);
    for (auto &v : ctx->ver) v.cancel.store(true);
    while (ctx->worker.pending.load(std::memory_order_acquire)) std::this_thread::yield();
    {
        std::lock_guard<std::mutex> g(ctx->pool.m);
        ctx->pool.stop.store(true);
    }
    ctx->pool.cv.notify_all();
    for (auto &t : ctx->pool.th) t.join();
    {
        qvq_ctx::Worker *w = &ctx->worker;
        if (w->th.joinable()) {
            {
                std::lock_guard<std::mutex> g(w->m);
                w->stop = true;
            }
            w->cv.notify_one();
            w->th.join();
        }
    }
    (void)hipSetDevice(ctx->dev);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->kstream) {
        (void)hipStreamSynchronize(ctx->kstream);
        (void)hipStreamDestroy(ctx->kstream);
    }
    if (ctx->ev_kcb) (void)hipEventDestroy(ctx->ev_kcb);
    if (ctx->ev_kdb) (void)hipEventDestroy(ctx->ev_kdb);
    if (ctx->comm) ncclCommDestroy(ctx->comm);
    free_training(ctx);
    free_levels(ctx);
    dfree(ctx->d_lut32);
    dfree(ctx->d_w);
    dfree(ctx->d_lut64);
    dfree(ctx->d_plut);
    dfree(ctx->d_counters);
    dfree(ctx->d_hist);
    if (ctx->h_ready) (void)hipHostFree(ctx->h_ready);
    dfree(ctx->d_dist_part);
    dfree(ctx->d_mean);
    dfree(ctx->d_scatter);
    dfree(ctx->d_decode);
    dfree(ctx->d_raster);
    dfree(ctx->d_decode_stat);
    if (ctx->h_decode_stat) (void)hipHostFree(ctx->h_decode_stat);
    if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
    if (ctx->h_ar_stage) (void)hipHostFree(ctx->h_ar_stage);
    dfree(ctx->d_vote);
    if (ctx->h_vote) (void)hipHostFree(ctx->h_vote);
    if (ctx->ev_ready)
        for (int l = 0; l < 32; l++)
            for (int j = 0; j < 4; j++) (void)hipEventDestroy(ctx->ev[l][j]);
    if (ctx->ev_end) (void)hipEventDestroy(ctx->ev_end);
    if (ctx->ev_sync) (void)hipEventDestroy(ctx->ev_sync);
    for (auto &v : ctx->ver)
        if (v.ev) (void)hipEventDestroy(v.ev);
    for (uint8_t *h : ctx->h_tx)
        if (h) (void)hipHostFree(h);
    if (ctx->vstream) (void)hipStreamDestroy(ctx->vstream);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

QVQ_API uint64_t qvq_num_vectors(const qvq_ctx *ctx) { return ctx ? ctx->N : 0; }
QVQ_API uint32_t qvq_dim(const qvq_ctx *ctx) { return ctx ? ctx->D : 0; }
QVQ_API const uint32_t *qvq_assign_device(const qvq_ctx *ctx) { return ctx ? ctx->d_A : nullptr; }

QVQ_API qvq_status qvq_set_images_device(qvq_ctx *ctx, const void *d_rgb, uint32_t n_images, uint32_t xSize,
                                         uint32_t ySize, uint32_t bw, uint32_t bh, int colorspace) {
    uint64_t N;
    uint32_t D;
    qvq_status st = check_image_args(ctx, n_images, xSize, ySize, bw, bh, N, D);
    if (st != QVQ_OK) return st;
    GUARD(ctx);
    if (!d_rgb) return fail(ctx, QVQ_EINVAL, "null raster");
    HIPCHK(hipSetDevice(ctx->dev));
    if ((st = alloc_training(ctx, N, D, colorspace)) != QVQ_OK) return st;
    if ((st = tile_into(ctx, (const uint8_t *)d_rgb, n_images, xSize, ySize, bw, bh)) != QVQ_OK) return st;
    return compute_xsq(ctx);
}

QVQ_API qvq_status qvq_set_images(qvq_ctx *ctx, const uint8_t *rgb, uint32_t n_images, uint32_t xSize, uint32_t ySize,
                                  uint32_t bw, uint32_t bh, int colorspace) {
    uint64_t N;
    uint32_t D;
    qvq_status st = check_image_args(ctx, n_images, xSize, ySize, bw, bh, N, D);
    if (st != QVQ_OK) return st;
    GUARD(ctx);
    if (!rgb) return fail(ctx, QVQ_EINVAL, "null raster");
    HIPCHK(hipSetDevice(ctx->dev));
    const uint64_t bytes = (uint64_t)xSize * ySize * 3 * n_images;
    if (ctx->raster_bytes < bytes) {   // kept across calls (repeated compresses)
        dfree(ctx->d_raster);
        ctx->raster_bytes = 0;
        HIPCHK(hipMalloc(&ctx->d_raster, bytes));
        ctx->raster_bytes = bytes;
    }
    const hipError_t e = host_copy(ctx, ctx->d_raster, rgb, bytes, hipMemcpyHostToDevice);
    if (e != hipSuccess) return fail(ctx, QVQ_EDEVICE, std::string("raster upload: ") + hipGetErrorString(e));
    if ((st = alloc_training(ctx, N, D, colorspace)) != QVQ_OK) return st;
    if ((st = tile_into(ctx, ctx->d_raster, n_images, xSize, ySize, bw, bh)) != QVQ_OK) return st;
    return compute_xsq(ctx);
}

QVQ_API qvq_status qvq_set_synthetic(qvq_ctx *ctx, uint32_t S, uint64_t seed0, uint32_t n_images, uint32_t bw,
                                     uint32_t bh, int colorspace) {
    uint64_t N;
    uint32_t D;
    if (!ctx) return QVQ_EINVAL;
    GUARD(ctx);
    if (S < 2) return fail(ctx, QVQ_EINVAL, "synthetic images need S >= 2");
    qvq_status st = check_image_args(ctx, n_images, S, S, bw, bh, N, D);
    if (st != QVQ_OK) return st;
    HIPCHK(hipSetDevice(ctx->dev));
    const uint64_t npix = (uint64_t)S * S * n_images;
    uint8_t *d_rgb = nullptr;
    HIPCHK(hipMalloc(&d_rgb, npix * 3));
    st = QVQ_OK;
    const hipError_t e = launch_gen(ctx->stream, d_rgb, S, seed0, npix);
    if (e != hipSuccess) st = fail(ctx, QVQ_EDEVICE, std::string("gen_kernel: ") + hipGetErrorString(e));
    if (st == QVQ_OK) st = alloc_training(ctx, N, D, colorspace);
    if (st == QVQ_OK) st = tile_into(ctx, d_rgb, n_images, S, S, bw, bh);
    if (st == QVQ_OK) st = compute_xsq(ctx);
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(d_rgb);
    return st;
}

QVQ_API qvq_status qvq_set_vectors(qvq_ctx *ctx, const double *X, uint64_t n, uint32_t dim) {
    if (!ctx) return QVQ_EINVAL;
    GUARD(ctx);
    if (!X || n == 0 || dim == 0) return fail(ctx, QVQ_EINVAL, "empty training set");
    if (dim > 64) return fail(ctx, QVQ_EINVAL, "block dimension above 64 (3*w*h) is not supported");
    ctx->col_blocks = 0;   // rows without image geometry
    // Recognise the colour space from the values: every value must be a byte's image
    // under NORMAL or SCALED (0.0 included), so the exact sums apply.
    int cs_found = -1;
    std::vector<uint8_t> codes;
    const uint32_t Dp = (dim + 3) & ~3u;
    for (int cs : {QVQ_CS_SCALED, QVQ_CS_NORMAL}) {
        Terms t;
        make_terms(cs, t);
        std::vector<std::pair<double, uint8_t>> inv;
        for (int b = 0; b < 256; b++) inv.push_back({t.v64[b], (uint8_t)b});
        std::sort(inv.begin(), inv.end());
        codes.assign(n * Dp, t.pad_code);
        bool ok = true;
        for (uint64_t i = 0; i < n && ok; i++)
            for (uint32_t d = 0; d < dim; d++) {
                const double v = X[i * dim + d];
                auto it = std::lower_bound(inv.begin(), inv.end(), std::make_pair(v, (uint8_t)0));
                if (it == inv.end() || it->first != v || (v == 0.0 && std::signbit(v))) {   // -0.0 is no byte image
                    ok = false;
                    break;
                }
                codes[i * Dp + d] = it->second;
            }
        if (ok) {
            cs_found = cs;
            break;
        }
    }
    // other values (arbitrary fp64 data, CIE1931): the reference's own arithmetic (exact mode),
    // one rank only -- with a communicator the ranks would disagree on the mode: fail fast here
    // instead of at qvq_lbg, where peers would wait in the first all-reduce
    if (cs_found < 0) {
        if (ctx->comm || ctx->host_ar)
            return fail(ctx, QVQ_EUNSUPPORTED, "values are not byte images (exact mode runs on one rank)");
        return qvq_set_vectors_exact(ctx, X, n, dim);
    }
    HIPCHK(hipSetDevice(ctx->dev));
    qvq_status st = alloc_training(ctx, n, dim, cs_found);
    if (st != QVQ_OK) return st;
    HIPCHK(hipMemcpy(ctx->d_codes, codes.data(), codes.size(), hipMemcpyHostToDevice));
    return compute_xsq(ctx);
}

// ---------------------------------------------------------------------------------------
// Exact mode (k_exact.hip): any fp64 training set, the reference's arithmetic bit for bit --
// fp64 search in nanoflann's order with kd-tree ties, Kahan sums over each cell's rows in
// ascending order times fl(1/n) (src/Quantizer.cpp:46-87).  One rank; host-driven levels.
// ---------------------------------------------------------------------------------------
QVQ_API qvq_status qvq_set_vectors_exact(qvq_ctx *ctx, const double *X, uint64_t n, uint32_t dim) {
    if (!ctx) return QVQ_EINVAL;
    GUARD(ctx);
    if (!X || n == 0 || dim == 0) return fail(ctx, QVQ_EINVAL, "empty training set");
    if (dim > 64) return fail(ctx, QVQ_EINVAL, "block dimension above 64 (3*w*h) is not supported");
    if (n >= (1ull << 31)) return fail(ctx, QVQ_EINVAL, "exact mode: more than 2^31-1 rows");
    for (uint64_t i = 0; i < n * dim; i++)
        if (!std::isfinite(X[i])) return fail(ctx, QVQ_EINVAL, "exact mode: training values must be finite");
    HIPCHK(hipSetDevice(ctx->dev));
    free_training(ctx);
    free_levels(ctx);
    ctx->N = n;
    ctx->D = dim;
    ctx->Dp = (dim + 3) & ~3u;
    ctx->cs = -1;
    ctx->exact = true;
    HIPCHK(hipMalloc(&ctx->d_X64, n * dim * 8));
    HIPCHK(hipMalloc(&ctx->d_A, n * 4));
    HIPCHK(hipMalloc(&ctx->d_ties, n * 4));
    HIPCHK(hipMalloc(&ctx->d_ex_keys, n * 4));
    HIPCHK(hipMalloc(&ctx->d_ex_iota, n * 4));
    HIPCHK(hipMalloc(&ctx->d_ex_order, n * 4));
    ctx->ex_temp_bytes = exact_sort_temp_bytes(n);
    HIPCHK(hipMalloc(&ctx->d_ex_temp, std::max<size_t>(ctx->ex_temp_bytes, 16)));
    HIPCHK(hipMemcpy(ctx->d_X64, X, n * dim * 8, hipMemcpyHostToDevice));
    HIPCHK(launch_exact_iota(ctx->stream, ctx->d_ex_iota, n));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return QVQ_OK;
}

namespace {

qvq_status exact_single_rank(qvq_ctx *ctx) {
    if (ctx->comm || ctx->host_ar)
        return fail(ctx, QVQ_EUNSUPPORTED, "exact mode runs on one rank (Kahan sums do not split across ranks)");
    return QVQ_OK;
}

qvq_status exact_koff(qvq_ctx *ctx, uint32_t K) {
    if (ctx->ex_kcap >= K + 1) return QVQ_OK;
    dfree(ctx->d_ex_koff);
    HIPCHK(hipMalloc(&ctx->d_ex_koff, ((size_t)K + 1) * 4));
    ctx->ex_kcap = K + 1;
    return QVQ_OK;
}

// Assignment of every row against the K code vectors at d_C64_split (host copy hC): the
// fp64 argmin, exact ties answered by the host kd-tree over hC.  Returns the tie count.
qvq_status exact_assign(qvq_ctx *ctx, const double *hC, uint32_t K, unsigned &nties) {
    const uint32_t D = ctx->D;
    qvq_status st;
    unsigned *cnt = ctx->d_counters + 1;
    HIPCHK(hipMemsetAsync(cnt, 0, sizeof(unsigned), ctx->stream));
    HIPCHK(launch_exact_assign(ctx->stream, ctx->d_X64, ctx->N, D, ctx->d_C64_split, K, 1e-12, ctx->d_A, ctx->d_ties,
                               cnt));
    HIPCHK(hipMemcpyAsync(&nties, cnt, sizeof(unsigned), hipMemcpyDeviceToHost, ctx->stream));
    if ((st = wait_stream(ctx)) != QVQ_OK) return st;
    if (nties == 0) return QVQ_OK;
    const uint64_t need = (uint64_t)nties * (8 + 8ull * D);
    if (ctx->scatter_bytes < need) {
        dfree(ctx->d_scatter);
        HIPCHK(hipMalloc(&ctx->d_scatter, need));
        ctx->scatter_bytes = need;
    }
    uint32_t *d_vals = ctx->d_scatter;
    double *d_rows = reinterpret_cast<double *>(ctx->d_scatter + 2 * (uint64_t)nties);
    std::vector<uint32_t> rows(nties), vals(nties);
    std::vector<double> q((size_t)nties * D);
    HIPCHK(launch_exact_gather(ctx->stream, ctx->d_X64, D, ctx->d_ties, nties, d_rows));
    HIPCHK(hipMemcpyAsync(rows.data(), ctx->d_ties, nties * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipMemcpyAsync(q.data(), d_rows, q.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    if ((st = wait_stream(ctx)) != QVQ_OK) return st;
    RefKDTree tree(hC, K, (int)D);
    for (unsigned i = 0; i < nties; i++) vals[i] = tree.nearest(q.data() + (size_t)i * D);
    HIPCHK(hipMemcpyAsync(d_vals, vals.data(), nties * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(launch_exact_fix(ctx->stream, ctx->d_A, ctx->d_ties, d_vals, nties));
    if ((st = wait_stream(ctx)) != QVQ_OK) return st;   // the host vectors must outlive the copies
    return QVQ_OK;
}

// Centroids of assignment d_A (nullptr: the mean) into d_C64_cent, counts into cnt (device, may be null).
qvq_status exact_centroids(qvq_ctx *ctx, bool mean, uint32_t K, uint64_t *cnt) {
    qvq_status st = exact_koff(ctx, K);
    if (st != QVQ_OK) return st;
    HIPCHK(launch_exact_centroids(ctx->stream, ctx->d_X64, ctx->N, ctx->D, mean ? nullptr : ctx->d_A, K,
                                  ctx->d_ex_keys, ctx->d_ex_iota, ctx->d_ex_order, ctx->d_ex_koff, ctx->d_ex_temp,
                                  ctx->ex_temp_bytes, ctx->d_C64_cent, cnt));
    return QVQ_OK;
}

qvq_status lbg_exact(qvq_ctx *ctx, uint32_t bits, double *codebook, uint32_t *assign, double *distortion) {
    qvq_status st = exact_single_rank(ctx);
    if (st != QVQ_OK) return st;
    const auto t0 = std::chrono::steady_clock::now();
    const uint32_t Kmax = 1u << bits, D = ctx->D;
    if ((st = ensure_levels(ctx, std::max<uint32_t>(Kmax, 2))) != QVQ_OK) return st;
    std::memset(&ctx->tm, 0, sizeof(ctx->tm));
    ctx->tm.levels = (int)bits;
    // codeVectors[0] = trainingSetSum() / N (src/Quantizer.cpp:129-130)
    std::vector<double> hC((size_t)Kmax * D), hS((size_t)Kmax * D);
    if ((st = exact_centroids(ctx, true, 1, nullptr)) != QVQ_OK) return st;
    HIPCHK(hipMemcpyAsync(hC.data(), ctx->d_C64_cent, (size_t)D * 8, hipMemcpyDeviceToHost, ctx->stream));
    if ((st = wait_stream(ctx)) != QVQ_OK) return st;
    if (bits == 0) HIPCHK(hipMemsetAsync(ctx->d_A, 0, ctx->N * 4, ctx->stream));
    for (uint32_t lvl = 1; lvl <= bits; lvl++) {
        const uint32_t K = 1u << lvl, H = K / 2;
        // concat(C, C), then the halves scaled by (1 + 0.2) and (1 - 0.2) (src/Quantizer.cpp:134-138)
        for (size_t i = 0; i < (size_t)H * D; i++) {
            hS[i] = hC[i] * (double)(1 + 0.2);
            hS[(size_t)H * D + i] = hC[i] * (double)(1 - 0.2);
        }
        HIPCHK(hipMemcpyAsync(ctx->d_C64_split, hS.data(), (size_t)K * D * 8, hipMemcpyHostToDevice, ctx->stream));
        unsigned nt = 0;
        const auto ta = std::chrono::steady_clock::now();
        if ((st = exact_assign(ctx, hS.data(), K, nt)) != QVQ_OK) return st;   // synchronous
        const auto tb = std::chrono::steady_clock::now();
        ctx->tm.host_ties[lvl - 1] = nt;
        if ((st = exact_centroids(ctx, false, K, nullptr)) != QVQ_OK) return st;
        HIPCHK(hipMemcpyAsync(hC.data(), ctx->d_C64_cent, (size_t)K * D * 8, hipMemcpyDeviceToHost, ctx->stream));
        if ((st = wait_stream(ctx)) != QVQ_OK) return st;
        // wall times: assign (search + ties) and update (sort + Kahan chains + codebook copy)
        ctx->tm.assign_ms[lvl - 1] = std::chrono::duration<float, std::milli>(tb - ta).count();
        ctx->tm.update_ms[lvl - 1] =
            std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - tb).count();
    }
    // updateDistortion after the last fix (src/Quantizer.cpp:9-22)
    double dist = 0;
    HIPCHK(launch_exact_distortion(ctx->stream, ctx->d_X64, ctx->N, D, ctx->d_C64_cent, ctx->d_A, ctx->d_dist_part,
                                   ctx->d_dist_part + 4096));
    // results reach the caller only after the bounded wait succeeds (staged in pinned memory)
    if ((st = ensure_pinned(ctx, ctx->h_stage, ctx->stage_bytes, 8 + (assign ? ctx->N * 4 : 0))) != QVQ_OK) return st;
    uint8_t *stage = static_cast<uint8_t *>(ctx->h_stage);
    HIPCHK(hipMemcpyAsync(stage, ctx->d_dist_part + 4096, 8, hipMemcpyDeviceToHost, ctx->stream));
    if (assign) HIPCHK(hipMemcpyAsync(stage + 8, ctx->d_A, ctx->N * 4, hipMemcpyDeviceToHost, ctx->stream));
    if ((st = wait_stream(ctx)) != QVQ_OK) return st;
    std::memcpy(&dist, stage, 8);
    if (assign) std::memcpy(assign, stage + 8, ctx->N * 4);
    if (codebook) std::memcpy(codebook, hC.data(), (size_t)Kmax * D * 8);
    if (distortion) *distortion = dist;
    ctx->tm.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return QVQ_OK;
}

}  // namespace

// Host placement, one rank: the engine's host threads -- the caller's for the duration of
// qvq_lbg, the worker and the certificate's helpers -- on the L3 domain (CCD, SMT siblings
// included) of the CPU the first quantize ran on, within the threads' allowed CPUs.  The level's
// tree build, its check and the helpers share the codebook, the tree and its caches; spread over
// the GPU box's 16 L3 domains, C4 ran ~0.4 ms slower (profiles/r07c: 6.84 vs 6.31-6.44 ms).
static bool l3_domain(int cpu, cpu_set_t &out) {
    char path[128];
    std::snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list", cpu);
    FILE *f = std::fopen(path, "r");
    if (!f) return false;
    char buf[1024];
    const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
    std::fclose(f);
    buf[n] = 0;
    CPU_ZERO(&out);
    const char *q = buf;
    while (*q) {   // "a-b,c,..."
        char *e;
        const long a = std::strtol(q, &e, 10);
        if (e == q) break;
        long b = a;
        q = e;
        if (*q == '-') {
            b = std::strtol(q + 1, &e, 10);
            if (e == q + 1) break;
            q = e;
        }
        for (long c = a; c <= b && c < CPU_SETSIZE; c++)
            if (c >= 0) CPU_SET((int)c, &out);
        while (*q == ',' || *q == '\n' || *q == ' ') q++;
    }
    return CPU_COUNT(&out) > 0;
}

struct HostPlaceGuard {   // the caller's CPUs narrowed to ctx->place during one call
    bool set = false;
    cpu_set_t old;
    explicit HostPlaceGuard(qvq_ctx *ctx) {
        if (ctx->comm || ctx->host_ar) return;   // several ranks share the box's CPUs: left alone
        if (pthread_getaffinity_np(pthread_self(), sizeof(old), &old) != 0) return;
        if (!ctx->place_tried) {
            ctx->place_tried = true;
            cpu_set_t l3;
            const int cpu = sched_getcpu();
            if (cpu >= 0 && l3_domain(cpu, l3)) {
                CPU_AND(&ctx->place, &l3, &old);
                ctx->place_ok = CPU_COUNT(&ctx->place) > 0;
            }
            if (ctx->place_ok) {   // threads started before (the worker of an earlier call)
                if (ctx->worker.th.joinable())
                    pthread_setaffinity_np(ctx->worker.th.native_handle(), sizeof(cpu_set_t), &ctx->place);
                for (std::thread &t : ctx->pool.th)
                    pthread_setaffinity_np(t.native_handle(), sizeof(cpu_set_t), &ctx->place);
            }
        }
        if (!ctx->place_ok) return;
        cpu_set_t want;
        CPU_AND(&want, &old, &ctx->place);
        if (CPU_COUNT(&want) == 0) return;
        set = pthread_setaffinity_np(pthread_self(), sizeof(want), &want) == 0;
    }
    ~HostPlaceGuard() {
        if (set) pthread_setaffinity_np(pthread_self(), sizeof(old), &old);
    }
};

QVQ_API qvq_status qvq_lbg(qvq_ctx *ctx, uint32_t bits, double eps, double *codebook, uint32_t *assign,
                           double *distortion) {
    (void)eps;   // cannot change the outputs: one Lloyd step per level
    if (!ctx) return QVQ_EINVAL;
    GUARD(ctx);
    if (ctx->N == 0) return fail(ctx, QVQ_ESTATE, "no training set");
    if (bits > 20) return fail(ctx, QVQ_EINVAL, "bits must be <= 20");
    HIPCHK(hipSetDevice(ctx->dev));
    if (ctx->exact) return lbg_exact(ctx, bits, codebook, assign, distortion);
    const HostPlaceGuard place(ctx);
    const auto t0 = std::chrono::steady_clock::now();
    static const bool htrace = env_is("QVQ_HOST_TRACE", "1");
    if (htrace) {
        ctx->htrace.start(t0);
    }
    const uint32_t Kmax = 1u << bits;
    qvq_status st = ensure_levels(ctx, std::max<uint32_t>(Kmax, 2));
    if (st != QVQ_OK) return st;
    std::memset(&ctx->tm, 0, sizeof(ctx->tm));
    ctx->tm.levels = (int)bits;
    const Terms &T = ctx->terms;
    // codeVectors[0] = trainingSetSum() / N, then the first split (src/Quantizer.cpp:129-138).
    // The mean kernel also clears the counters and writes [sum ||x||^2, rows] for the
    // closed-form distortion (summed over all ranks below).
    double *d_dist = ctx->d_dist_part;
    // sum ||x||^2 and the row count come from the byte histogram (qvq_set_*), all-reduced as
    // integers first: the distortion is then the same bits for every rank count
    const uint64_t *hist = ctx->d_hist;
    if (ctx->comm || ctx->host_ar) {
        HIPCHK(hipMemcpyAsync(ctx->d_hist + 256, ctx->d_hist, 256 * 8, hipMemcpyDeviceToDevice, ctx->stream));
        if ((st = all_reduce(ctx, ctx->d_hist + 256, 256, false)) != QVQ_OK) return st;
        hist = ctx->d_hist + 256;
    }
    // Reference-bit (Kahan) levels, SCALED values (NORMAL values are integers: the exact sums are
    // the reference's bits).  Speculative (default): each level runs as with exact sums, its ties
    // answered by the exact-sum tree on the device, and the worker checks them against the
    // reference's rule (the certificate) while the GPU runs the next level; a
    // level whose check fails makes the quantize run again with synchronous Kahan levels (each
    // waits for its ties to be answered by the reference's rule).  Several ranks:
    // a check never sums a cell on its own (a cell's chain runs over every rank's rows); its open
    // rows wait for the end of the call, where the ranks vote, sum the cells wanted together
    // (kahan_chained) and vote again, so that every rank redoes the quantize or none does.
    // QVQ_SPECULATE=0: synchronous from the start.
    const bool kahan = kahan_mode(ctx) && ctx->cs == QVQ_CS_SCALED;
    const bool multi = ctx->nranks > 1 && (ctx->comm || ctx->host_ar);
    static const bool spec_off = env_is("QVQ_SPECULATE", "0");
    bool spec = kahan && !spec_off;
    if (spec && (st = ensure_speculation(ctx, Kmax)) != QVQ_OK) return st;
    if (kahan && !ctx->d_A_alt) HIPCHK(hipMalloc(&ctx->d_A_alt, ctx->N * 4));
    // several ranks, speculative: one assignment buffer per level, so that every level's parent
    // assignment is still there when the deferred checks finish at the end of the call
    const uint32_t npool = spec && multi ? std::max<uint32_t>(4, bits + 1) : 4;
    while (spec && 4 + ctx->d_Aext.size() < npool) {
        uint32_t *p = nullptr;
        HIPCHK(hipMalloc(&p, ctx->N * 4));
        ctx->d_Aext.push_back(p);
    }
    ctx->deferred.clear();
    struct JobGuard {   // no tree build or check outlives the call (an error return included)
        qvq_ctx *c;
        ~JobGuard() {
            join_tree_job(c, true);
            for (auto &v : c->ver) {
                v.cancel.store(true);
                join_verify(c, v);
            }
        }
    } job_guard{ctx};
    // distortion inputs, per-level counters and the codebook go to mapped pinned memory in one
    // launch (the mapped split-codebook buffer is free once the last tree is built); the copy's
    // own flag ends the wait: polling it wakes the host at once (a stream synchronize costs tens
    // of us of wake-up), and the wait is bounded (wait.hpp), so a peer rank that dies inside a
    // level's all-reduce ends this call with QVQ_ECOMM
    bool out_enqueued = false;
    uint64_t out_seq = 0;
    auto enqueue_out = [&]() -> qvq_status {
        if (ctx->timing_level == -1) HIPCHK(hipEventRecord(ctx->ev_end, ctx->stream));   // each record idles the GPU ~6 us
        uint8_t *dh_small = reinterpret_cast<uint8_t *>(ctx->dh_ready) + 64;
        static_assert(3 * sizeof(double) + 2 * 33 * sizeof(unsigned) <= 1024 - 64, "small results exceed the mapped area");
        const uint64_t cb_bytes = codebook ? (uint64_t)Kmax * ctx->D * 8 : 0;
        uint64_t *done = reinterpret_cast<uint64_t *>(dh_small + (1024 - 64 - 8));
        out_seq = ++ctx->out_seq;
        HIPCHK(launch_copy_out(ctx->stream, ctx->d_dist_part, dh_small, 3 * sizeof(double), ctx->d_counters,
                               dh_small + 3 * sizeof(double), 2 * 33 * sizeof(unsigned), ctx->d_C64_cent, ctx->dh_cb,
                               cb_bytes, done, out_seq, ctx->d_counters + 2 * 33 + 1));
        out_enqueued = true;
        return QVQ_OK;
    };
    // the published results out of the mapped buffers: distortion inputs, per-level counters,
    // the codebook (C4: 1.5 MB, ~60 us)
    double dres[3];
    unsigned stats[2 * 33];
    bool results_copied = false;
    auto copy_results = [&]() -> qvq_status {
        uint8_t *h_small = reinterpret_cast<uint8_t *>(ctx->h_ready) + 64;
        const uint64_t cb_bytes = codebook ? (uint64_t)Kmax * ctx->D * 8 : 0;
        qvq_status ws = wait_flag(ctx, reinterpret_cast<volatile uint64_t *>(h_small + (1024 - 64 - 8)), out_seq);
        if (ws != QVQ_OK) return ws;
        std::memcpy(dres, h_small, sizeof(dres));
        std::memcpy(stats, h_small + sizeof(dres), sizeof(stats));
        if (codebook) std::memcpy(codebook, ctx->h_cb, cb_bytes);
        results_copied = true;
        ctx->htrace.mark("results copied");
        return QVQ_OK;
    };
    for (;;) {   // once, or twice when a speculative check fails
    out_enqueued = false;
    results_copied = false;
    const bool tmean = ctx->timing_level == -3;   // events around the mean kernel (qvq_set_timing)
    if (tmean) HIPCHK(hipEventRecord(ctx->ev[31][0], ctx->stream));
    HIPCHK(launch_mean_sums(ctx->stream, ctx->Dp, ctx->d_codes, ctx->N, ctx->D, ctx->d_plut, ctx->d_mean,
                            ctx->d_counters, N_COUNTERS, d_dist, hist, ctx->d_lut64));
    if (tmean) HIPCHK(hipEventRecord(ctx->ev[31][1], ctx->stream));
    if ((st = all_reduce_sums(ctx, 1, ctx->d_mean, MEAN_COPIES)) != QVQ_OK) {
        (void)hipMemsetAsync(ctx->d_mean, 0, MEAN_COPIES * (2 * 64 + 1) * 8, ctx->stream);   // keep it clear for the next call
        return st;
    }
    unsigned *dist_done = ctx->d_counters + 2 * 33;
    // finalize (+ split, tables, host codebook and its ready number) / final distortion
    // (K = 1 reads the mean sums and leaves them cleared for the next quantize)
    if (ctx->sums1_dirty) {   // a quantize stopped between a kd_reduce and its finalize
        HIPCHK(hipMemsetAsync(ctx->d_sums, 0, ctx->sums_bytes, ctx->stream));
        ctx->sums1_dirty = false;
    }
    // copies 2: copy 1 holds the ties' moves (added here; the next level's search clears it)
    // the split a finalize writes: with deferred ties the level's own split must survive its
    // (speculative) finalize, so the next one goes to the other buffer and the two swap
    double *split_out = ctx->d_C64_split;
    // clear1: the finalize also clears sums copy 1 after adding it (no fused search of a later
    // level clears it: a communicator, or the synchronous Kahan levels' moves)
    auto finalize = [&](uint32_t K, bool split, uint32_t copies = 1, const unsigned *gate = nullptr,
                        const TieExport &tx = TieExport(), bool clear1 = false) {
        if (split || tx.out) ctx->seq++;
        const bool prune = split && use_prune(ctx, 2 * K);   // the next search's tile order
        ctx->perm_k = prune ? 2 * K : 0;
        return launch_finalize_prep(ctx->stream, K == 1 ? ctx->d_mean : ctx->d_sums, K, ctx->D, ctx->Dp, T.R, T.bias,
                                    T.scale,
                                    ctx->d_C64_cent, split, split_out, pad32(2 * K), T.mu, T.sx, ctx->mf_t,
                                    ctx->d_C32, ctx->d_rows, ctx->d_E32,
                                    split ? dev_cb_of(ctx, (uint32_t)__builtin_ctz(K) + 1) : nullptr, d_dist + 8,
                                    dist_done,
                                    split ? nullptr : d_dist + 2, (split || tx.out) ? ctx->dh_ready : nullptr,
                                    ctx->seq, K == 1 || (clear1 && copies > 1), K == 1 ? MEAN_COPIES : copies,
                                    prune ? ctx->d_perm : nullptr, prune ? ctx->d_tint : nullptr, K == 1 ? 0 : 1,
                                    copies > 1 ? sums_cap_stride(ctx) : 0,
                                    gate, tx);
    };
    HIPCHK(finalize(1, bits > 0));
    // with bits >= 1 the first search writes every row's index
    if (bits == 0) HIPCHK(hipMemsetAsync(ctx->d_A, 0, ctx->N * 4, ctx->stream));

    const bool sync_kahan = kahan && !spec;
    if (sync_kahan) split_out = ctx->d_C64_split_alt;
    // the assignment buffers (d_A, d_A_alt, d_A3, d_A4 and d_Aext own them together): level L
    // writes abuf[L % P]; a check of level L reads A_{L-1} until level L + 3 starts (one rank) or
    // to the end of the call (several ranks, P > bits)
    std::vector<uint32_t *> abuf = {ctx->d_A, ctx->d_A_alt, ctx->d_A3, ctx->d_A4};
    abuf.insert(abuf.end(), ctx->d_Aext.begin(), ctx->d_Aext.end());
    const uint32_t P = spec ? (uint32_t)std::min<size_t>(abuf.size(), npool) : 4;
    std::vector<uint32_t *> alev(bits + 1, nullptr);   // A_L of this call
    bool spec_failed = false, local_fail = false;
    for (uint32_t lvl = 1; lvl <= bits; lvl++) {
        const uint32_t K = 1u << lvl;
        const int slot = (int)lvl - 1;
        if (spec) {
            if (lvl >= 4) {
                bool ok;
                ctx->htrace.mark("L" + std::to_string(lvl) + " joins check K" + std::to_string(ctx->ver[lvl % 3].K));
                if ((st = join_verify_bounded(ctx, ctx->ver[lvl % 3], ok)) != QVQ_OK) return st;
                ctx->htrace.mark("L" + std::to_string(lvl) + " joined");
                if (!ok && !multi) {
                    spec_failed = true;
                    break;
                }
                local_fail = local_fail || !ok;   // several ranks: every rank runs on to the vote
            }
            ctx->d_A = abuf[lvl % P];
            ctx->d_A_alt = abuf[(lvl + P - 1) % P];
            ctx->d_A3 = abuf[(lvl + 1) % P];   // the buffers stay distinct, and owned, across calls
            ctx->d_A4 = abuf[(lvl + 2) % P];
            ctx->d_Aext.clear();   // the rest of the pool
            for (uint32_t *q : abuf)
                if (q != ctx->d_A && q != ctx->d_A_alt && q != ctx->d_A3 && q != ctx->d_A4) ctx->d_Aext.push_back(q);
        } else if (kahan) {
            std::swap(ctx->d_A, ctx->d_A_alt);   // d_A_alt: the previous level's assignment
        }
        alev[lvl] = ctx->d_A;
        if ((st = run_level(ctx, K, slot, true, host_cb_of(ctx, lvl), ctx->seq, sync_kahan)) != QVQ_OK) return st;
        if (spec) {   // the level's check: its tree now
            qvq_ctx::Verify &v = ctx->ver[lvl % 3];
            v.K = K;
            v.level = lvl;
            v.tree = std::move(ctx->tree);
            // (swapped, not moved: the joined check's buffers come back with their capacity, so
            // the next level's codebook copy writes no fresh pages -- 1.5 MB at C4's level 12)
            std::swap(v.cb, ctx->cb_local);
            std::swap(v.cnt, ctx->cnt_local);
            ctx->cb_local.clear();
            ctx->cnt_local.clear();
            v.cs = CertState();
        }
        const bool split = lvl < bits;
        {
            const uint32_t copies = ctx->sums_copies;
            if (copies > 1) ctx->sums1_dirty = true;
            const unsigned *tcnt = ctx->d_counters + 2 * ((int)lvl - 1) + 1;   // the level's ties
            if (ctx->kd_pend) {   // the level's ties and the reduce together
                HIPCHK(launch_kd_reduce(ctx->stream, ctx->d_codes, ctx->Dp, ctx->D, ctx->d_ties, tcnt,
                                        ctx->d_C64_split, K, ctx->d_lut64, ctx->pend_kd, ctx->d_A, ctx->d_plut,
                                        ctx->d_part, ctx->d_part_cnt, ctx->nslabs, ctx->nsub, ctx->d_sums,
                                        ctx->d_sums + sums_cap_stride(ctx)));
                ctx->kd_pend = false;
            } else if (ctx->nslabs) {   // nslabs 0: the sorted sums are in d_sums already
                HIPCHK(launch_reduce(ctx->stream, ctx->d_part, ctx->d_part_cnt, ctx->nslabs, ctx->nsub, K, ctx->D,
                                     ctx->d_sums, ctx->pub));
            }
            if (ctx->pub.flag) {   // run_level left the tie count to the reduce, which did not run
                if (!ctx->nslabs || ctx->kd_pend)
                    HIPCHK(launch_copy_out(ctx->stream, ctx->pub.cnt, ctx->pub.dst, 4, nullptr, nullptr, 0, nullptr,
                                           nullptr, 0, ctx->pub.flag, ctx->pub.seq, ctx->d_counters + 2 * 33 + 1));
                ctx->pub = PubArgs();
            }
            if ((st = all_reduce_sums(ctx, K)) != QVQ_OK) return st;
            TieExport tx;
            if (spec) {   // the level's tie rows and their indices go out with its codebook
                tx.rows = ctx->d_ties;
                tx.cnt = tcnt;
                tx.A = ctx->d_A;
                tx.codes = ctx->d_codes;
                tx.cap = ctx->tx_cap;
                tx.n_rows = ctx->N;
                tx.out = ctx->dh_tx[lvl % 3];
            }
            HIPCHK(finalize(K, split, copies, copies > 1 ? tcnt : nullptr, tx));
            if (copies > 1) ctx->sums1_dirty = false;
            if (spec) {   // the check of this level, on the worker
                qvq_ctx::Verify &v = ctx->ver[lvl % 3];
                v.posted = true;
                v.done.store(false);
                v.cancel.store(false);
                v.status = 1;
                v.seq = ctx->seq;
                v.par = (int)(lvl % 3);
                v.A_prev = lvl >= 2 ? ctx->d_A_alt : nullptr;
                qvq_ctx::Verify *vp = &v;
                post_job(ctx, [ctx, vp] {
                    verify_level(ctx, *vp);
                    vp->done.store(true, std::memory_order_release);
                });
                ctx->htrace.mark("L" + std::to_string(lvl) + " finalize enqueued, check posted");
            }
            if (sync_kahan) {   // the level's ties (published after its recheck)
                if ((st = wait_flag(ctx, ctx->h_ready + 1, ctx->pub_seq)) != QVQ_OK) return st;
                const unsigned nt = (unsigned)(uint32_t)ctx->h_ready[2];
                uint64_t nt_all = nt;   // every rank's ties: the ranks resolve together
                if (multi && (st = vote(ctx, &nt_all, 1)) != QVQ_OK) return st;
                join_tree_job(ctx, nt_all == 0);   // the level's tree: needed for ties only
                if (nt_all) {
                    const bool fused = use_fused(ctx, K);
                    if (multi) {   // every rank's moves in copy 1, all-reduced, added by the finalize
                        ctx->sums1_dirty = true;
                        if ((st = resolve_kahan_ties_multi(ctx, K, slot, nt)) != QVQ_OK) return st;
                        HIPCHK(finalize(K, split, 2, nullptr, TieExport(), true));
                    } else {
                        if (fused) ctx->sums1_dirty = true;
                        if ((st = resolve_kahan_ties(ctx, K, slot, nt, fused)) != QVQ_OK) return st;
                        // (without kd_reduce no fused search clears copy 1 before its next use)
                        HIPCHK(finalize(K, split, fused ? 2 : 1, fused ? tcnt : nullptr, TieExport(),
                                        fused && !kd_merge(ctx)));
                    }
                    ctx->sums1_dirty = false;
                }
                if (split) {
                    std::swap(ctx->d_C64_split, ctx->d_C64_split_alt);
                    split_out = ctx->d_C64_split_alt;
                }
            }
        }
    }
    if (spec && !spec_failed) {   // the results' copy overlaps the last checks
        if ((st = enqueue_out()) != QVQ_OK) return st;
        ctx->htrace.mark("results' copy enqueued");
        for (uint32_t l = bits >= 3 ? bits - 2 : 1; l <= bits; l++) {
            // one rank: the results leave the mapped buffers while the last check runs (a
            // failed check redoes the quantize, and the copy with it)
            if (l == bits && !multi && (st = copy_results()) != QVQ_OK) return st;
            bool ok;
            if ((st = join_verify_bounded(ctx, ctx->ver[l % 3], ok, true)) != QVQ_OK) return st;
            local_fail = local_fail || !ok;
        }
        ctx->htrace.mark("last checks joined");
        spec_failed = local_fail;
        if (multi && (st = resolve_deferred(ctx, bits, alev, spec_failed)) != QVQ_OK) return st;
    }
    ctx->deferred.clear();
    if (!spec_failed) break;
    // a check failed: every check joined, the stream drained, then the quantize again with
    // synchronous Kahan levels
    for (auto &v : ctx->ver) {
        v.cancel.store(true);
        join_verify(ctx, v);
    }
    ctx->deferred.clear();
    if ((st = wait_stream(ctx)) != QVQ_OK) return st;
    if (ctx->sums1_dirty) {
        HIPCHK(hipMemsetAsync(ctx->d_sums, 0, ctx->sums_bytes, ctx->stream));
        ctx->sums1_dirty = false;
    }
    ctx->kd_pend = false;
    ctx->pub = PubArgs();
    ctx->tm.kahan_redo++;
    spec = false;
    }
    // Returned distortion: updateDistortion after the last fix (src/Quantizer.cpp:9-22,103),
    // from the sums of the final assignment (finalize_prep_kernel without split).
    // (enqueue_out: before the last checks are joined when speculating)
    if (!out_enqueued && (st = enqueue_out()) != QVQ_OK) return st;
    if (!results_copied && (st = copy_results()) != QVQ_OK) return st;
    if (assign)   // every collective of this call is complete: a plain copy
        HIPCHK(host_copy(ctx, assign, ctx->d_A, ctx->N * 4, hipMemcpyDeviceToHost));
    // closed form: sum ||x||^2 - sum_k (2 c_k.S_k - n_k ||c_k||^2) cancels to a few ulps of
    // sum ||x||^2 when the cells are (nearly) exact; a distortion is never negative
    if (distortion) *distortion = std::max(0.0, (dres[0] - dres[2]) / (dres[1] * (double)ctx->D));
    for (uint32_t lvl = 1; lvl <= bits; lvl++) {
        // assign: the search kernel; update: the non-fused update; other: the rest of the
        // level up to the next level's search (recheck, kd-tree, reduce, finalize, tables)
        float a = 0, u = 0, whole = 0;
        const bool timed = ctx->timing_level == -1 || ctx->timing_level == (int)lvl - 1;
        if (timed) {
            (void)hipEventSynchronize(ctx->ev[lvl - 1][1]);   // complete; the runtime may not know yet
            (void)hipEventElapsedTime(&a, ctx->ev[lvl - 1][0], ctx->ev[lvl - 1][1]);
        }
        if (ctx->upd[lvl - 1]) {
            (void)hipEventSynchronize(ctx->ev[lvl - 1][3]);
            (void)hipEventElapsedTime(&u, ctx->ev[lvl - 1][2], ctx->ev[lvl - 1][3]);
        }
        if (ctx->timing_level == -1) (void)hipEventSynchronize(ctx->ev_end);
        if (ctx->timing_level == -1)
            (void)hipEventElapsedTime(&whole, ctx->ev[lvl - 1][0], lvl < bits ? ctx->ev[lvl][0] : ctx->ev_end);
        ctx->tm.assign_ms[lvl - 1] = a;
        ctx->tm.other_ms[lvl - 1] = ctx->timing_level == -1 ? std::max(0.f, whole - a - u) : 0.f;
        ctx->tm.update_ms[lvl - 1] = u;
        ctx->tm.flagged[lvl - 1] = stats[2 * (lvl - 1)];
        ctx->tm.host_ties[lvl - 1] = stats[2 * (lvl - 1) + 1];
    }
    if (ctx->timing_level == -3) {
        float m = 0;
        (void)hipEventSynchronize(ctx->ev[31][1]);
        (void)hipEventElapsedTime(&m, ctx->ev[31][0], ctx->ev[31][1]);
        ctx->tm.mean_ms = m;
    }
    (void)hipGetLastError();
    ctx->tm.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (htrace) {
        ctx->htrace.mark("return");
        std::fprintf(stderr, "%s\n", ctx->htrace.finish().c_str());
    }
    return QVQ_OK;
}

QVQ_API qvq_status qvq_assign(qvq_ctx *ctx, const double *C, uint32_t K, uint32_t *assign) {
    if (!ctx) return QVQ_EINVAL;
    GUARD(ctx);
    if (ctx->N == 0) return fail(ctx, QVQ_ESTATE, "no training set");
    if (!C || K == 0) return fail(ctx, QVQ_EINVAL, "empty codebook");
    HIPCHK(hipSetDevice(ctx->dev));
    qvq_status st = ensure_levels(ctx, K);
    if (st != QVQ_OK) return st;
    std::memset(&ctx->tm, 0, sizeof(ctx->tm));
    HIPCHK(hipMemcpy(ctx->d_C64_split, C, (uint64_t)K * ctx->D * 8, hipMemcpyHostToDevice));
    if (ctx->exact) {
        unsigned nt = 0;
        if ((st = exact_assign(ctx, C, K, nt)) != QVQ_OK) return st;
        ctx->tm.levels = 1;
        ctx->tm.host_ties[0] = nt;
        if (assign) HIPCHK(hipMemcpy(assign, ctx->d_A, ctx->N * 4, hipMemcpyDeviceToHost));
        return QVQ_OK;
    }
    HIPCHK(hipMemsetAsync(ctx->d_counters, 0, 2 * sizeof(unsigned), ctx->stream));
    if ((st = run_prep(ctx, K)) != QVQ_OK) return st;
    ctx->perm_k = 0;   // (prep writes no tile order)
    if ((st = run_level(ctx, K, 0, false, C, 0)) != QVQ_OK) return st;
    unsigned stats[2];
    HIPCHK(hipMemcpyAsync(stats, ctx->d_counters, sizeof(stats), hipMemcpyDeviceToHost, ctx->stream));
    if (assign) HIPCHK(hipMemcpyAsync(assign, ctx->d_A, ctx->N * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    ctx->tm.levels = 1;
    ctx->tm.flagged[0] = stats[0];
    ctx->tm.host_ties[0] = stats[1];
    return QVQ_OK;
}

QVQ_API qvq_status qvq_update(qvq_ctx *ctx, const uint32_t *assign, uint32_t K, double *C_out, uint64_t *counts) {
    if (!ctx) return QVQ_EINVAL;
    GUARD(ctx);
    if (ctx->N == 0) return fail(ctx, QVQ_ESTATE, "no training set");
    if (!assign || K == 0) return fail(ctx, QVQ_EINVAL, "empty assignment");
    for (uint64_t i = 0; i < ctx->N; i++)
        if (assign[i] >= K) return fail(ctx, QVQ_EINVAL, "assignment index out of range");
    HIPCHK(hipSetDevice(ctx->dev));
    qvq_status st = ensure_levels(ctx, K);
    if (st != QVQ_OK) return st;
    HIPCHK(hipMemcpy(ctx->d_A, assign, ctx->N * 4, hipMemcpyHostToDevice));
    if (ctx->exact) {
        if ((st = exact_single_rank(ctx)) != QVQ_OK) return st;
        uint64_t *d_cnt = ctx->d_sums;   // K u64 of scratch (2KD + K)
        if ((st = exact_centroids(ctx, false, K, d_cnt)) != QVQ_OK) return st;
        if (C_out) HIPCHK(hipMemcpyAsync(C_out, ctx->d_C64_cent, (uint64_t)K * ctx->D * 8, hipMemcpyDeviceToHost, ctx->stream));
        if (counts) HIPCHK(hipMemcpyAsync(counts, d_cnt, (uint64_t)K * 8, hipMemcpyDeviceToHost, ctx->stream));
        return wait_stream(ctx);
    }
    if ((st = run_update(ctx, ctx->d_A, K)) != QVQ_OK) return st;
    if ((st = all_reduce_sums(ctx, K)) != QVQ_OK) return st;
    const Terms &T = ctx->terms;
    HIPCHK(launch_finalize(ctx->stream, ctx->d_sums, K, ctx->D, T.R, T.bias, T.scale, ctx->d_C64_cent));
    // results land in context-owned pinned memory and reach the caller only after the bounded
    // wait succeeds (a failed wait can leave these copies queued: wait_failed)
    const uint64_t cB = (uint64_t)K * ctx->D * 8, nB = (uint64_t)K * 8;
    if ((st = ensure_pinned(ctx, ctx->h_stage, ctx->stage_bytes, cB + nB)) != QVQ_OK) return st;
    uint8_t *stage = static_cast<uint8_t *>(ctx->h_stage);
    HIPCHK(hipMemcpyAsync(stage, ctx->d_C64_cent, cB, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipMemcpyAsync(stage + cB, ctx->d_sums + 2 * (uint64_t)K * ctx->D, nB, hipMemcpyDeviceToHost, ctx->stream));
    if ((st = wait_stream(ctx)) != QVQ_OK) return st;   // bounded: the all-reduce may wait on peer ranks
    if (C_out) std::memcpy(C_out, stage, cB);
    if (counts) std::memcpy(counts, stage + cB, nB);
    return QVQ_OK;
}

// The reference's centroids bit for bit (Solution::fixCodeVectors, src/Quantizer.cpp:59-87):
// Kahan sums in ascending row order times fl(1/n) (k_kahan.hip).  One rank; byte rows.
QVQ_API qvq_status qvq_update_kahan(qvq_ctx *ctx, const uint32_t *assign, uint32_t K, double *C_out) {
    if (!ctx) return QVQ_EINVAL;
    GUARD(ctx);
    if (ctx->N == 0) return fail(ctx, QVQ_ESTATE, "no training set");
    if (!assign || K == 0) return fail(ctx, QVQ_EINVAL, "empty assignment");
    if (ctx->exact) return qvq_update(ctx, assign, K, C_out, nullptr);   // exact mode: the Kahan chain already
    if (ctx->cs != QVQ_CS_SCALED) return qvq_update(ctx, assign, K, C_out, nullptr);   // integers: exact = Kahan
    for (uint64_t i = 0; i < ctx->N; i++)
        if (assign[i] >= K) return fail(ctx, QVQ_EINVAL, "assignment index out of range");
    HIPCHK(hipSetDevice(ctx->dev));
    qvq_status st = ensure_levels(ctx, K);
    if (st != QVQ_OK) return st;
    if ((st = ensure_kahan(ctx, K)) != QVQ_OK) return st;
    HIPCHK(hipMemcpy(ctx->d_A, assign, ctx->N * 4, hipMemcpyHostToDevice));
    if (ctx->nranks > 1) {   // every rank's rows: the chains pass from rank to rank (kahan_chained)
        if ((st = kahan_chained(ctx, K == 1 ? nullptr : ctx->d_A, K, nullptr, K, false)) != QVQ_OK)
            return st;
    } else {
        uint64_t max_rows = ctx->N;   // the longest chain (short ones run step by step)
        if (K > 1) {
            std::vector<uint64_t> n(K, 0);
            for (uint64_t i = 0; i < ctx->N; i++) n[assign[i]]++;   // (checked < K above)
            max_rows = std::max<uint64_t>(1, *std::max_element(n.begin(), n.end()));
        }
        HIPCHK(launch_kahan_centroids(ctx->stream, ctx->kw, ctx->d_codes, ctx->Dp, ctx->D, ctx->N,
                                      K == 1 ? nullptr : ctx->d_A, K, ctx->d_kc_cent, nullptr, nullptr, 0, max_rows));
    }
    const uint64_t cB = (uint64_t)K * ctx->D * 8;
    if ((st = ensure_pinned(ctx, ctx->h_stage, ctx->stage_bytes, cB)) != QVQ_OK) return st;
    HIPCHK(hipMemcpyAsync(ctx->h_stage, ctx->d_kc_cent, cB, hipMemcpyDeviceToHost, ctx->stream));
    if ((st = wait_stream(ctx)) != QVQ_OK) return st;
    if (C_out) std::memcpy(C_out, ctx->h_stage, cB);
    if (env_is("QVQ_KAHAN_DEBUG", "1")) {
        unsigned ms[4];
        HIPCHK(hipMemcpy(ms, ctx->kw.stats, sizeof(ms), hipMemcpyDeviceToHost));
        HIPCHK(hipMemset(ctx->kw.stats, 0, sizeof(ms)));
        std::fprintf(stderr, "qvq kahan: K %u blocks not composable %u block misses %u replays %u\n", K, ms[0], ms[1],
                     ms[2]);
    }
    return QVQ_OK;
}

// Test entry: qvq_update_kahan with this context's rows cut into virtual ranks at splits[0..n]
// (0 = splits[0] <= ... <= splits[n] = N), the chained evaluation of several ranks run in turn on
// one device (kahan_chained).  The result must equal qvq_update_kahan's for any cuts.
QVQ_API qvq_status qvq_update_kahan_split(qvq_ctx *ctx, const uint32_t *assign, uint32_t K, const uint64_t *splits,
                                          uint32_t nsplits, double *C_out) {
    if (!ctx) return QVQ_EINVAL;
    GUARD(ctx);
    if (ctx->N == 0) return fail(ctx, QVQ_ESTATE, "no training set");
    if (ctx->exact || ctx->cs != QVQ_CS_SCALED) return fail(ctx, QVQ_EUNSUPPORTED, "SCALED byte rows only");
    if (!assign || K == 0 || !splits || nsplits == 0) return fail(ctx, QVQ_EINVAL, "empty assignment or splits");
    if (splits[0] != 0 || splits[nsplits] != ctx->N) return fail(ctx, QVQ_EINVAL, "splits must run from 0 to N");
    for (uint32_t i = 0; i < nsplits; i++)
        if (splits[i] > splits[i + 1]) return fail(ctx, QVQ_EINVAL, "splits must not decrease");
    for (uint64_t i = 0; i < ctx->N; i++)
        if (assign[i] >= K) return fail(ctx, QVQ_EINVAL, "assignment index out of range");
    HIPCHK(hipSetDevice(ctx->dev));
    qvq_status st = ensure_levels(ctx, K);
    if (st != QVQ_OK) return st;
    HIPCHK(hipMemcpy(ctx->d_A, assign, ctx->N * 4, hipMemcpyHostToDevice));
    const std::vector<uint64_t> cuts(splits, splits + nsplits + 1);
    if ((st = kahan_chained(ctx, K == 1 ? nullptr : ctx->d_A, K, nullptr, K, false, &cuts)) != QVQ_OK)
        return st;
    const uint64_t cB = (uint64_t)K * ctx->D * 8;
    if ((st = ensure_pinned(ctx, ctx->h_stage, ctx->stage_bytes, cB)) != QVQ_OK) return st;
    HIPCHK(hipMemcpyAsync(ctx->h_stage, ctx->d_kc_cent, cB, hipMemcpyDeviceToHost, ctx->stream));
    if ((st = wait_stream(ctx)) != QVQ_OK) return st;
    if (C_out) std::memcpy(C_out, ctx->h_stage, cB);
    return QVQ_OK;
}

// ---------------------------------------------------------------------------------------
// Decode: CompressedImage::decompress (src/Compressor.cpp:156-165) as one device gather.
// ---------------------------------------------------------------------------------------
static qvq_status check_decode_args(qvq_ctx *ctx, uint32_t K, uint64_t nblocks, uint32_t xSize, uint32_t ySize,
                                    uint32_t bw, uint32_t bh) {
    if (!ctx) return QVQ_EINVAL;
    if (K == 0 || bw == 0 || bh == 0 || xSize == 0 || ySize == 0)
        return fail(ctx, QVQ_EINVAL, "decode: K, block and image sizes must be > 0");
    // the kernel's block-row count and wrap span are 32-bit
    if ((uint64_t)ySize + bh - 1 > 0xFFFFFFFFull || (uint64_t)xSize + bw - 1 > 0xFFFFFFFFull)
        return fail(ctx, QVQ_EINVAL, "decode: image size + block size - 1 exceeds 2^32 - 1");
    const uint64_t wB = ((uint64_t)xSize + bw - 1) / bw, hB = ((uint64_t)ySize + bh - 1) / bh;
    if (nblocks != wB * hB) return fail(ctx, QVQ_EINVAL, "decode: nblocks != ceil(x/bw)*ceil(y/bh)");
    if ((uint64_t)bw * bh * 3 > 0xFFFFFFFFull) return fail(ctx, QVQ_EINVAL, "decode: block too large");
    return QVQ_OK;
}

// One decode launch on stream s (0 = the legacy null stream, ordered after every blocking
// stream's work, as in the caller's own torch/HIP code) with the context's persistent
// out-of-range flag and signed-byte squared-error accumulator; orig (may be null) is the
// original raster for the raport's MSE.  Synchronises s.
static qvq_status run_decode(qvq_ctx *ctx, hipStream_t s, const uint8_t *d_cb, uint32_t K, const uint32_t *d_A,
                             uint32_t xSize, uint32_t ySize, uint32_t bw, uint32_t bh, uint8_t *d_rgb,
                             const uint8_t *d_orig, double *mse) {
    uint64_t *d_err = ctx->d_decode_stat;   // [0] squared error, [1] bad-index flag
    hipError_t e = hipMemsetAsync(d_err, 0, 16, s);
    if (e == hipSuccess)
        e = launch_decode(s, d_cb, K, bw * bh * 3, d_A, xSize, ySize, bw, bh, d_rgb, d_orig, d_err,
                          reinterpret_cast<uint32_t *>(d_err + 1));
    if (e == hipSuccess) e = hipMemcpyAsync(ctx->h_decode_stat, d_err, 16, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return fail(ctx, QVQ_EDEVICE, std::string("decode: ") + hipGetErrorString(e));
    if (ctx->h_decode_stat[1]) return fail(ctx, QVQ_EINVAL, "decode: code-vector index out of range");
    if (mse) *mse = (double)ctx->h_decode_stat[0] / ((double)xSize * ySize * 3);
    return QVQ_OK;
}

QVQ_API qvq_status qvq_decode_device(qvq_ctx *ctx, const void *d_codebook, uint32_t K, const void *d_assign,
                                     uint64_t nblocks, uint32_t xSize, uint32_t ySize, uint32_t bw, uint32_t bh,
                                     void *d_rgb, void *stream) {
    qvq_status st = check_decode_args(ctx, K, nblocks, xSize, ySize, bw, bh);
    if (st != QVQ_OK) return st;
    GUARD(ctx);
    if (!d_codebook || !d_assign || !d_rgb) return fail(ctx, QVQ_EINVAL, "decode: null pointer");
    if ((uintptr_t)d_assign % 4) return fail(ctx, QVQ_EINVAL, "decode: assignment pointer not 4-byte aligned");
    HIPCHK(hipSetDevice(ctx->dev));
    // ordered after the engine's own queued work (e.g. the qvq_lbg that wrote d_assign) on
    // any stream the caller names, the legacy null stream included
    HIPCHK(hipEventRecord(ctx->ev_sync, ctx->stream));
    HIPCHK(hipStreamWaitEvent((hipStream_t)stream, ctx->ev_sync, 0));
    return run_decode(ctx, (hipStream_t)stream, (const uint8_t *)d_codebook, K, (const uint32_t *)d_assign, xSize,
                      ySize, bw, bh, (uint8_t *)d_rgb, nullptr, nullptr);
}

QVQ_API qvq_status qvq_decode(qvq_ctx *ctx, const uint8_t *codebook, uint32_t K, const uint32_t *assign,
                              uint64_t nblocks, uint32_t xSize, uint32_t ySize, uint32_t bw, uint32_t bh, uint8_t *rgb) {
    return qvq_decode_mse(ctx, codebook, K, assign, nblocks, xSize, ySize, bw, bh, rgb, nullptr, nullptr);
}

QVQ_API qvq_status qvq_decode_mse(qvq_ctx *ctx, const uint8_t *codebook, uint32_t K, const uint32_t *assign,
                                  uint64_t nblocks, uint32_t xSize, uint32_t ySize, uint32_t bw, uint32_t bh,
                                  uint8_t *rgb, const uint8_t *orig, double *mse) {
    qvq_status st = check_decode_args(ctx, K, nblocks, xSize, ySize, bw, bh);
    if (st != QVQ_OK) return st;
    GUARD(ctx);
    if (!codebook || !assign || (!rgb && !mse) || (mse && !orig))
        return fail(ctx, QVQ_EINVAL, "decode: null pointer");
    HIPCHK(hipSetDevice(ctx->dev));
    // one scratch allocation, grown on demand and kept: codebook | indices | raster | original
    const uint64_t cbB = (uint64_t)K * bw * bh * 3, aB = nblocks * 4, rB = (uint64_t)xSize * ySize * 3;
    const uint64_t oA = (cbB + 15) & ~15ull, oR = (oA + aB + 15) & ~15ull, oO = (oR + rB + 15) & ~15ull;
    const uint64_t need = oO + (orig ? rB : 0);
    if (ctx->decode_bytes < need) {
        dfree(ctx->d_decode);
        HIPCHK(hipMalloc(&ctx->d_decode, need));
        ctx->decode_bytes = need;
    }
    uint8_t *d = ctx->d_decode;
    HIPCHK(hipMemcpyAsync(d, codebook, cbB, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(d + oA, assign, aB, hipMemcpyHostToDevice, ctx->stream));
    if (orig) HIPCHK(hipMemcpyAsync(d + oO, orig, rB, hipMemcpyHostToDevice, ctx->stream));
    st = run_decode(ctx, ctx->stream, d, K, reinterpret_cast<const uint32_t *>(d + oA), xSize, ySize, bw, bh, d + oR,
                    orig ? d + oO : nullptr, mse);
    if (st == QVQ_OK && rgb) {
        HIPCHK(hipMemcpyAsync(rgb, d + oR, rB, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
    }
    return st;
}

QVQ_API qvq_status qvq_comm_unique_id(uint8_t id[128]) {
    static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id size");
    ncclUniqueId u;
    const ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return fail(nullptr, QVQ_ECOMM, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    std::memcpy(id, &u, 128);
    return QVQ_OK;
}

QVQ_API qvq_status qvq_comm_init(qvq_ctx *ctx, int nranks, int rank, const uint8_t id[128]) {
    GUARD(ctx);
    if (!id || nranks < 1 || rank < 0 || rank >= nranks) return QVQ_EINVAL;
    HIPCHK(hipSetDevice(ctx->dev));
    if (ctx->comm) {
        ncclCommDestroy(ctx->comm);
        ctx->comm = nullptr;
    }
    ctx->host_ar = nullptr;
    ctx->host_ar_user = nullptr;
    ctx->nranks = 1;
    ctx->rank = 0;
    // a communicator even for one rank: the caller asked for the collective path (it is
    // then a local copy per level, and the results equal the communicator-free run's)
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    NCCLCHK(ncclCommInitRank(&ctx->comm, nranks, u, rank));
    ctx->nranks = nranks;
    ctx->rank = rank;
    return QVQ_OK;
}

QVQ_API qvq_status qvq_comm_init_host(qvq_ctx *ctx, int nranks, int rank, qvq_allreduce_fn fn, void *user) {
    GUARD(ctx);
    if (!fn || nranks < 1 || rank < 0 || rank >= nranks) return QVQ_EINVAL;
    if (ctx->comm) {
        HIPCHK(hipSetDevice(ctx->dev));
        ncclCommDestroy(ctx->comm);
        ctx->comm = nullptr;
    }
    ctx->host_ar = fn;
    ctx->host_ar_user = user;
    ctx->nranks = nranks;
    ctx->rank = rank;
    return QVQ_OK;
}

QVQ_API qvq_status qvq_comm_info(const qvq_ctx *ctx, int *nranks, int *rank, int *kind) {
    if (!ctx) return QVQ_EINVAL;
    if (nranks) *nranks = ctx->nranks;
    if (rank) *rank = ctx->rank;
    if (kind) *kind = ctx->comm ? QVQ_COMM_RCCL : ctx->host_ar ? QVQ_COMM_HOST : QVQ_COMM_NONE;
    return QVQ_OK;
}

QVQ_API qvq_status qvq_set_timeout(qvq_ctx *ctx, double seconds) {
    if (!ctx || !(seconds > 0)) return QVQ_EINVAL;
    ctx->timeout_s = seconds;
    return QVQ_OK;
}

QVQ_API qvq_status qvq_set_timing(qvq_ctx *ctx, int level) {
    if (!ctx || level < -3 || level > 31) return QVQ_EINVAL;
    ctx->timing_level = level;
    return QVQ_OK;
}

QVQ_API qvq_status qvq_get_timings(const qvq_ctx *ctx, qvq_timings *out) {
    if (!ctx || !out) return QVQ_EINVAL;
    *out = ctx->tm;
    return QVQ_OK;
}

QVQ_API qvq_status qvq_host_kdtree_nn(const double *C, uint32_t K, uint32_t dim, const double *Q, uint64_t nq,
                                      uint32_t *out) {
    if (!C || !Q || !out || K == 0 || dim == 0 || dim > 64) return QVQ_EINVAL;
    RefKDTree tree(C, K, (int)dim);
    for (uint64_t i = 0; i < nq; i++) out[i] = tree.nearest(Q + i * dim);
    return QVQ_OK;
}

QVQ_API qvq_status qvq_host_kdtree_image(const double *C, uint32_t K, uint32_t dim, void *img, uint64_t bytes,
                                         uint64_t *need) {
    if (!C || !need || K == 0 || dim == 0 || dim > 64) return QVQ_EINVAL;
    *need = kdb_host_layout(K, dim).total;
    if (!img || bytes < *need) return QVQ_EINVAL;
    RefKDTree tree(C, K, (int)dim);
    if (tree.num_nodes() > 2ull * K) return QVQ_EINVAL;   // (the layout holds 2K nodes)
    std::memset(img, 0, *need);
    tree.to_device_image(static_cast<uint8_t *>(img));
    return QVQ_OK;
}

QVQ_API qvq_status qvq_kdtree_device_check(qvq_ctx *ctx, const double *C, uint32_t K, uint32_t dim, double *build_ms,
                                           uint32_t *result) {
    if (!ctx || !C || !result || K == 0 || dim == 0 || dim > 64) return QVQ_EINVAL;
    GUARD(ctx);
    if (!kd_build_fits(K, dim)) return fail(ctx, QVQ_EUNSUPPORTED, "device kd build: K or dim too large");
    HIPCHK(hipSetDevice(ctx->dev));
    const KdbHostLayout L = kdb_host_layout(K, dim);
    double *dP = nullptr, *nbox = nullptr, *cbox = nullptr;
    uint32_t *vind = nullptr;
    KdbNode *nodes = nullptr;
    uint8_t *flat = nullptr, *himg = nullptr, *dhimg = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    struct Free {
        std::function<void()> f;
        ~Free() { f(); }
    } fr{[&] {
        for (void *p : {(void *)dP, (void *)nbox, (void *)cbox, (void *)vind, (void *)nodes, (void *)flat})
            if (p) (void)hipFree(p);
        if (himg) (void)hipHostFree(himg);
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
    }};
    HIPCHK(hipMalloc(&dP, (uint64_t)K * dim * 8));
    HIPCHK(hipMalloc(&nbox, 2ull * K * 2 * dim * 8));
    HIPCHK(hipMalloc(&cbox, 2ull * K * 2 * dim * 8));
    HIPCHK(hipMalloc(&vind, (uint64_t)K * 4));
    HIPCHK(hipMalloc(&nodes, 2ull * K * sizeof(KdbNode)));
    HIPCHK(hipMalloc(&flat, tree_bytes(K, dim)));
    HIPCHK(hipHostMalloc(&himg, L.total, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer((void **)&dhimg, himg, 0));
    std::memset(himg, 0, sizeof(KdbHeader));
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipMemcpy(dP, C, (uint64_t)K * dim * 8, hipMemcpyHostToDevice));
    HIPCHK(hipEventRecord(e0, ctx->stream));
    HIPCHK(launch_kd_build(ctx->stream, dP, K, dim, vind, nodes, nbox, cbox, flat, dhimg, 1));
    HIPCHK(hipEventRecord(e1, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const KdbHeader &h = *reinterpret_cast<const KdbHeader *>(himg);
    if (build_ms) {   // the launch; phase 1, phase 2, the images (the kernel's 100 MHz stamps)
        build_ms[0] = ms;
        for (int i = 0; i < 3; i++) build_ms[1 + i] = (double)h.pad2[i] * 1e-5;
    }
    if (h.seq != 1 || h.status != 1) {
        *result = 2;   // the build gave up (capacity): the engine builds on the host then
        return QVQ_OK;
    }
    const RefKDTree dev(C, K, (int)dim, himg), host(C, K, (int)dim);
    std::string why;
    *result = host.same_as(dev, &why) ? 0u : 1u;
    if (*result) ctx->err = "device kd-tree differs: " + why;
    // the device image kd_resolve reads: the host flattening of the same tree, node ids aside
    std::vector<uint8_t> fimg(16ull * dim + (uint64_t)h.n_nodes * sizeof(KdNodeDev) + 4ull * K);
    HIPCHK(hipMemcpy(fimg.data(), flat, fimg.size(), hipMemcpyDeviceToHost));
    const double *flo = reinterpret_cast<const double *>(fimg.data());
    const KdNodeDev *fn = reinterpret_cast<const KdNodeDev *>(flo + 2 * dim);
    const uint32_t *fv = reinterpret_cast<const uint32_t *>(fn + h.n_nodes);
    const KdbNode *hn = reinterpret_cast<const KdbNode *>(himg + L.nodes);
    const uint32_t *hv = reinterpret_cast<const uint32_t *>(himg + L.vind);
    for (uint32_t i = 0; i < h.n_nodes && !*result; i++) {
        const KdNodeDev &a = fn[i];
        const KdbNode &b = hn[i];
        const bool leaf = b.child1 < 0;
        if (a.child1 != b.child1 || a.child2 != b.child2 || a.b != (int32_t)b.right ||
            a.a != (int32_t)(leaf ? b.left : ((uint32_t)b.divfeat | b.left << 8)) || (!leaf && (a.lo != b.divlow || a.hi != b.divhigh))) {
            *result = 1;
            ctx->err = "device kd_resolve image differs at node " + std::to_string(i);
        }
    }
    for (uint32_t i = 0; i < K && !*result; i++)
        if (fv[i] != hv[i]) {
            *result = 1;
            ctx->err = "device kd_resolve image vind differs";
        }
    return QVQ_OK;
}

QVQ_API qvq_status qvq_host_finalize(const uint64_t *hi, const uint64_t *lo, const uint64_t *cnt, uint32_t K,
                                     uint32_t dim, int colorspace, double *C_out) {
    Terms t;
    if (!hi || !lo || !cnt || !C_out) return QVQ_EINVAL;
    if (!make_terms(colorspace, t)) return QVQ_EUNSUPPORTED;
    for (uint64_t k = 0; k < K; k++)
        for (uint32_t d = 0; d < dim; d++)
            C_out[k * dim + d] = centroid_value(hi[k * dim + d], lo[k * dim + d], cnt[k], t.R, t.bias, t.scale);
    return QVQ_OK;
}

QVQ_API qvq_status qvq_host_wait_probe(int scenario, double timeout_s, double *elapsed_s) {
    if (scenario < 0 || scenario > 5 || !(timeout_s > 0)) return QVQ_EINVAL;
    using clock = std::chrono::steady_clock;
    const auto t0 = clock::now();
    auto after = [&](double s) { return std::chrono::duration<double>(clock::now() - t0).count() >= s; };
    std::string err;
    const qvq_status st = wait_until(
        [&] { return scenario == 0 && after(0.005); },
        [&](std::string &m) {
            if (scenario == 4) {
                m = "scripted stream fault";
                return StreamState::Failed;
            }
            return scenario == 5 ? StreamState::Drained : StreamState::Running;
        },
        [&](std::string &m) {
            if (scenario == 3 && after(0.005)) {
                m = "scripted peer failure";
                return CommState::Failed;
            }
            return scenario == 2 || scenario == 3 ? CommState::Healthy : CommState::None;
        },
        timeout_s, err);
    if (elapsed_s) *elapsed_s = std::chrono::duration<double>(clock::now() - t0).count();
    if (st != QVQ_OK) g_static_err = err;
    return st;
}

QVQ_API qvq_status qvq_host_pool_stress(uint32_t rounds, uint32_t maxn, uint64_t *errors) {
    if (!errors || maxn < 1 || maxn > 64) return QVQ_EINVAL;
    std::unique_ptr<qvq_ctx> ctx(new qvq_ctx());   // the pool only: no device work
    std::atomic<uint32_t> hits[64];
    uint64_t bad = 0;
    for (uint32_t r = 0; r < rounds; r++) {
        // n grows and shrinks (new helpers spawn while earlier epochs exist, idle ones wake late)
        const uint32_t n = 1 + (uint32_t)(((uint64_t)r * 2654435761u) >> 7) % maxn;
        for (auto &h : hits) h.store(0);
        pool_run(ctx.get(), n, [&](uint32_t t) {
            hits[t].fetch_add(1);
            if ((t + r) % 5 == 0) std::this_thread::yield();
        });
        for (uint32_t t = 0; t < 64; t++) bad += hits[t].load() != (t < n ? 1u : 0u);
    }
    {
        std::lock_guard<std::mutex> g(ctx->pool.m);
        ctx->pool.stop.store(true);
    }
    ctx->pool.cv.notify_all();
    for (auto &t : ctx->pool.th) t.join();
    *errors = bad;
    return QVQ_OK;
}

QVQ_API qvq_status qvq_host_row_terms(const uint8_t *codes, uint32_t dim, int colorspace, uint64_t *hi,
                                      uint64_t *lo) {
    Terms t;
    if (!codes || !hi || !lo) return QVQ_EINVAL;
    if (!make_terms(colorspace, t)) return QVQ_EUNSUPPORTED;
    for (uint32_t d = 0; d < dim; d++) {
        hi[d] = t.hi[codes[d]];
        lo[d] = t.lo[codes[d]];
    }
    return QVQ_OK;
}

}  // extern "C"
