// mhs_api.cpp -- C-ABI orchestration of the MI355X SpGEMM (include/mhspgemm.h).
//
// Replaces MH_spgemm (reference src/main.cu:12-72) and the Tool workspace
// (src/Tool.cu:4-69).  One call = one stream-ordered pipeline:
//
//   memset stats -> k_mask_b (Form_mask_matrix_B) -> k_analyze + bins (symbolic_binning)
//   -> symbolic bins (Calculate_C_nnz) -> scan + classify + bins + ONE readback
//   (numeric_binning) -> C.col/C.val allocation (Malloc_C_col_val) -> numeric bins
//   (Numeric) -> stream sync.
//
// The reference makes 5 binning round trips (2 blocking copies each), 3 scalar
// reads and 6 device-wide syncs per call; here the only host round
// trip is the single Stats readback that C's allocation needs anyway.
#include "mhs_internal.hpp"
#include "../../include/mhspgemm.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

using namespace mhs;

struct mhs_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    char* ws = nullptr;
    size_t ws_bytes = 0;
    char* gscratch = nullptr;
    size_t gscratch_bytes = 0;
    Stats* h_stats = nullptr;  // pinned
    Published* pub = nullptr;  // fine-grained pinned: Stats handed over by the last pre-numeric kernel
    Published* d_pub = nullptr;
    int seq = 0;
    hipEvent_t ev[8] = {};
    bool sync = true;      // MHS_OPT_SYNC
    bool groups = true;     // row groups (MHS_NO_GROUPS=1: every row alone)
    bool near = true;       // near row groups (GRP_NEAR; MHS_NO_NEAR=1: off)
    bool split = true;      // block bins split by LDS need (MHS_NO_SPLIT=1: off)
    // MHS_OPT_NUMERIC_EVENTS: ring of (start, end) events around the numeric phase
    std::vector<hipEvent_t> nev;
    long long ncalls = 0;
    int mc_list = 0;         // tile-list cap of the row cache (0: mc_list_for(M); MHS_MC_LIST)
    bool stats_zero = false; // the workspace's device Stats are zero (left so by the last k_scan)
    bool use_mcache = true;  // symbolic keeps narrow rows' tile masks for numeric (MHS_NO_MCACHE)
    bool tiny_num = true;    // numeric tiny (sort) classes (MHS_NO_TINY_NUM=1: off)
    // numeric-first tiny rows from this many rows of A on (MHS_OPT_TINY_FIRST_ROWS,
    // MHS_NFT_MIN_M; < 0: never): one hand-off more per call, so big matrices only
    long long nft_min_m = 1 << 19;
    bool sym_fork = false;   // MHS_SYM_FORK=1: rare symbolic bins on an aux stream for every call
    // ... and for every call of at least this many rows (MHS_SYM_FORK_MIN_M; < 0: never): the
    // fork's cross-stream wait (~20 us) is noise there, the rare bins' milliseconds are not
    long long sym_fork_min_m = 1 << 19;
    bool nft_slots = true;   // MHS_NFT_NO_SLOTS=1 (tests): count the rows only, as when the slots do not fit
    int nft_other_pct = 5;   // slots only when at most this share of the rows is past the tiny classes (MHS_NFT_OTHER_PCT)
    // numeric-first tiny rows without the probe below nft_min_m rows, for matrices averaging fewer
    // than this many entries a row (MHS_NFT_AUTO_AVG; 0: off): the slots are sized by their upper
    // bound (TINY_SLOT_MAX a row), so no hand-off decides them
    int nft_auto_avg = 12;
    char* slots = nullptr;   // their value slots (cached across calls)
    size_t slots_bytes = 0;
    size_t mem_budget = 0;   // MHS_OPT_MEM_BUDGET (MiB): a call's workspace + C beyond it count as OOM (tests)
    size_t c_held = 0;       // C bytes a row-chunked call holds while it lays out its second pass
    long long front_passes = 0;  // front_pass calls (row-chunked passes; mhs_ctx_chunked_calls diagnostics)
    long long chunked_calls = 0;  // calls that ran row-chunked (mhs_ctx_chunked_calls)
    long long stat[9] = {};       // path counters (mhs_ctx_stat; [0] unused: chunked_calls)
    int dense_span_max = 0;  // NM_DENSE for rows spanning <= this many 64-column tiles (MHS_DENSE_SPAN; off: occupancy)
    // output pool (caching allocator for C arrays): (buffer, allocation size)
    std::vector<std::pair<void*, size_t>> pool;
    hipEvent_t stream_ev = nullptr;  // orders a new caller stream after the previous one
    // numeric bins on several streams (MHS_NUM_STREAMS, default 4; 1 = one stream): aux
    // streams fork from the call's stream after the Stats hand-off and join it before return
    static constexpr int NAUX = 7;
    int num_streams = 4;
    hipStream_t aux[NAUX] = {};
    hipEvent_t fork_ev = nullptr, join_ev[NAUX] = {};
    hipEvent_t split_ev = nullptr;  // k_split_bins done (the split block launches wait for it)
    bool split_on = false;          // a speculated plan's phase A split its block bins (phase B's launches)
    // launch plan speculation (SpecArgs, mhs_internal.hpp): the last hand-off's Stats and the
    // operands they belong to; MHS_NO_SPEC=1 turns it off
    struct PlanKey {
        const void* p[6];
        long long M, N, MB, nnzA, nnzB, gen;
        int near, nft, mc_list, pad;  // (no implicit padding: compared bytewise)
        bool operator==(const PlanKey& o) const { return memcmp(this, &o, sizeof *this) == 0; }
    };
    bool spec = true;
    bool plan_valid = false;
    PlanKey plan_key{};
    Stats plan_h{};
    long long gen = 0;        // bumped by every mhs_ctx_set_option (options change the pipeline)
    int* d_go = nullptr;      // k_scan's verdict on a speculated plan (device int)
    bool spec_fork = false;  // MHS_SPEC_FORK=1: speculated plans also behind every forked symbolic pass (A/B)
    // speculated calls run their plan's rare symbolic rows on an aux stream beside k_sym_common
    // (scircuit-like -3.9 %, the other configs within 0.5 %: r06sf2); MHS_SPEC_FORK=0 turns it off
    bool spec_fork_rare = true;
    // a forked symbolic pass launches k_sym_common before the aux stream's rare rows (no host launch
    // ahead of the call stream's: scircuit-like -0.6 %, webbase-like -0.3 %, cage15-like -0.1 %: r06fo);
    // MHS_FORK_ORDER=0: the rare rows first
    bool fork_common_first = true;
    int spec_nss = mhs_ctx::NAUX + 1;  // streams of a speculated numeric phase (MHS_SPEC_NSS: a cap, A/B)
};

namespace {

int fail(mhs_ctx* ctx, int code, const std::string& what) {
    if (ctx) ctx->err = what;
    return code;
}

int fail_hip(mhs_ctx* ctx, hipError_t e, const char* what) {
    std::string m = std::string(what) + ": " + hipGetErrorString(e);
    (void)hipGetLastError();
    return fail(ctx, e == hipErrorOutOfMemory ? MHS_ERR_OOM : MHS_ERR_HIP, m);
}

// Spin until the device has published call `seq`'s Stats.  Every 256 polls the
// stream is queried: a fault ends the wait with the HIP error, an idle stream
// without the publication is an internal error (never spins forever).
int wait_published(mhs_ctx* ctx, hipStream_t s, const Published* pub, int seq) {
    for (unsigned polls = 1;; ++polls) {
        if (__atomic_load_n(&pub->seq, __ATOMIC_ACQUIRE) == seq) return MHS_OK;
        if ((polls & 255) == 0) {
            const hipError_t q = hipStreamQuery(s);
            if (q == hipSuccess) {
                if (__atomic_load_n(&pub->seq, __ATOMIC_ACQUIRE) == seq) return MHS_OK;
                return fail(ctx, MHS_ERR_HIP, "device did not publish the symbolic statistics");
            }
            if (q != hipErrorNotReady) return fail_hip(ctx, q, "waiting for the symbolic phase");
        }
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
    }
}

#define MHS_HIP(expr)                                                   \
    do {                                                                \
        hipError_t e_ = (expr);                                         \
        if (e_ != hipSuccess) return fail_hip(ctx, e_, #expr);          \
    } while (0)

inline size_t al(size_t x) { return (x + 255) & ~size_t(255); }

double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

hipError_t pool_get(mhs_ctx* ctx, void** p, size_t bytes) {
    if (bytes == 0) bytes = 16;
    size_t best = (size_t)-1;
    size_t bi = 0;
    for (size_t i = 0; i < ctx->pool.size(); ++i) {
        const size_t s = ctx->pool[i].second;
        if (s >= bytes && s <= 2 * bytes + (1u << 20) && s < best) {
            best = s;
            bi = i;
        }
    }
    if (best != (size_t)-1) {
        *p = ctx->pool[bi].first;
        ctx->pool.erase(ctx->pool.begin() + (long)bi);
        return hipSuccess;
    }
    hipError_t e = hipMalloc(p, bytes);
    if (e == hipErrorOutOfMemory && !ctx->pool.empty()) {
        for (auto& b : ctx->pool) (void)hipFree(b.first);
        ctx->pool.clear();
        (void)hipGetLastError();
        e = hipMalloc(p, bytes);
    }
    return e;
}

// The buffer's true size comes from the runtime (not from a side table: a buffer
// freed with mhs_csr_free and handed out again by hipMalloc at the same address
// would otherwise be filed under its old size).
void pool_put(mhs_ctx* ctx, void* p);
// C.col / C.val back to the pool (C.ptr kept)
void mhs_ctx_recycle_cols(mhs_ctx* ctx, mhs_csr* out) {
    pool_put(ctx, out->col);
    pool_put(ctx, out->val);
    out->col = nullptr;
    out->val = nullptr;
}

void pool_put(mhs_ctx* ctx, void* p) {
    if (!p) return;
    hipDeviceptr_t base = nullptr;
    size_t bytes = 0;
    if (hipMemGetAddressRange(&base, &bytes, (hipDeviceptr_t)p) != hipSuccess || base != (hipDeviceptr_t)p) {
        (void)hipGetLastError();
        (void)hipFree(p);
        return;
    }
    ctx->pool.emplace_back(p, bytes);
    // keep the pool bounded: drop the oldest buffers beyond 16 entries
    while (ctx->pool.size() > 16) {
        (void)hipFree(ctx->pool.front().first);
        ctx->pool.erase(ctx->pool.begin());
    }
}

struct Layout {
    size_t btcol, btmask, bmeta, bhi, rflop, rtflop, rlo, rhi, ctiles, sym_bin, asame, grp, bin_list, scan_part, mcache,
        stats, blkflop, spill_mask, spill_key, lofs, tslot, nft_bin, near_list, nsig, ucol, gna, bx_col, bx_val, split_list, total;
    bool near, near_b;
    long long bx_pre;  // B's entries in front of the union rows in bx_* (B is A), else 0
    long long spill_cap;
};

// near: near row groups planned; near_b: B is A (the union rows also serve B's union runs, so
// B's arrays are copied in front of them -- A != B reserves only the union rows)
Layout plan(int M, int MB, long long nnzA, long long nnzB, int mc_list, int M_total = -1, bool near = false,
            bool near_b = false) {
    Layout L{};
    size_t o = 0;
    auto take = [&](size_t bytes) {
        size_t r = o;
        o += al(bytes ? bytes : 16);
        return r;
    };
    const size_t nscan = (size_t)(M + 1 + SCAN_ITEMS - 1) / SCAN_ITEMS + 1;
    L.stats = take(sizeof(Stats));
    L.btcol = take((size_t)nnzB * 4);
    L.btmask = take((size_t)nnzB * 8);
    L.bmeta = take((size_t)MB * 16);
    L.bhi = take((size_t)MB * 4);
    L.rflop = take((size_t)M * 4);
    L.rtflop = take((size_t)M * 4);
    L.rlo = take((size_t)M * 4);
    L.rhi = take((size_t)M * 4);
    L.ctiles = take((size_t)M * 4);
    L.sym_bin = take((size_t)M);
    L.asame = take((size_t)M);
    L.grp = take((size_t)M);
    static_assert((int)NUM_NB >= (int)SYM_NB, "bin_list holds either phase's bins");
    L.bin_list = take((size_t)(NUM_NB - 1) * M * 4);
    L.blkflop = take(((size_t)analyze_blocks(nnzA, M) + 1) * 8);
    L.scan_part = take(nscan * 8 + (size_t)ZERO_INTS * 4);  // look-back words, then the row cursors and bin counters
    L.mcache = take((size_t)M * mc_stride(mc_list) * 8);
    L.spill_cap = spill_cap(nnzB);
    if (M_total > M && M_total > 0)  // a row chunk: its share of the region (spill lists belong to rows)
        L.spill_cap = std::max<long long>(SPILL_PARTS * 1024, L.spill_cap * M / M_total);
    if (const char* e = getenv("MHS_SPILL_CAP")) L.spill_cap = atoll(e) < 1 ? 1 : atoll(e);  // tests: a full region
    L.spill_mask = take((size_t)L.spill_cap * 8);
    L.spill_key = take((size_t)L.spill_cap * 4);
    L.lofs = take((size_t)M * 4);
    L.tslot = take((size_t)M * 8);
    L.nft_bin = take((size_t)M);
    L.split_list = take((size_t)M * 4);
    L.near = near;
    if (near) {  // near row groups: candidate list, union rows (see Work)
        L.near_b = near_b;
        L.bx_pre = near_b ? nnzB : 0;
        L.near_list = take((size_t)M * 4);
        L.nsig = take((size_t)M * 4);
        L.ucol = take((size_t)nnzA * 4);
        L.gna = take((size_t)M * 4);
        if (near_b) L.bx_col = take((size_t)(nnzB + 3 * nnzA) * 4);  // B's arrays + the union rows (see Work)
        L.bx_val = take((size_t)(L.bx_pre + 3 * nnzA) * 8);
    }
    L.total = o;
    return L;
}

// Device bytes the context holds for a call: its cached buffers plus C arrays a row-chunked
// call has already allocated (MHS_OPT_MEM_BUDGET counts them all).
size_t held(const mhs_ctx* ctx) { return ctx->ws_bytes + ctx->gscratch_bytes + ctx->slots_bytes + ctx->c_held; }

int ensure(mhs_ctx* ctx, char** buf, size_t* have, size_t need) {
    if (*have >= need) return MHS_OK;
    if (*buf) {
        MHS_HIP(hipStreamSynchronize(ctx->stream));
        MHS_HIP(hipFree(*buf));
        *buf = nullptr;
        *have = 0;
    }
    size_t want = need + need / 8;
    if (ctx->mem_budget && held(ctx) + want > ctx->mem_budget) want = need;
    if (ctx->mem_budget && held(ctx) + need > ctx->mem_budget)
        return fail(ctx, MHS_ERR_OOM, "workspace exceeds the context's memory budget");
    MHS_HIP(hipMalloc((void**)buf, want));
    *have = want;
    return MHS_OK;
}

// C.col / C.val of nnz entries (+ what the call already holds) within the test budget
hipError_t alloc_c(mhs_ctx* ctx, mhs_csr* out, long long nnz) {
    if (ctx->mem_budget && held(ctx) + (size_t)nnz * 12 > ctx->mem_budget) return hipErrorOutOfMemory;
    hipError_t e = pool_get(ctx, (void**)&out->col, (size_t)nnz * 4);
    if (e == hipSuccess) e = pool_get(ctx, (void**)&out->val, (size_t)nnz * 8);
    if (e != hipSuccess) {
        pool_put(ctx, out->col);
        out->col = nullptr;
    }
    return e;
}

// The call's Work over the workspace laid out by `L` (rows of this pass: M).
Work make_work(mhs_ctx* ctx, const Layout& L, int M, long long nnzA, long long nnzB, int Bn, int mc_list) {
    Work w{};
    w.btcol = (int*)(ctx->ws + L.btcol);
    w.btmask = (unsigned long long*)(ctx->ws + L.btmask);
    w.bmeta = (int4*)(ctx->ws + L.bmeta);
    w.bhi = (int*)(ctx->ws + L.bhi);
    w.rflop = (int*)(ctx->ws + L.rflop);
    w.rtflop = (int*)(ctx->ws + L.rtflop);
    w.rlo = (int*)(ctx->ws + L.rlo);
    w.rhi = (int*)(ctx->ws + L.rhi);
    w.ctiles = (int*)(ctx->ws + L.ctiles);
    w.sym_bin = (unsigned char*)(ctx->ws + L.sym_bin);
    w.asame = (unsigned char*)(ctx->ws + L.asame);
    w.grp = (unsigned char*)(ctx->ws + L.grp);
    w.groups = ctx->groups ? 1 : 0;
    w.tiny_num = ctx->tiny_num ? 1 : 0;  // per row: packed sort keys hold its column offsets in 23 bits
    (void)Bn;
    w.bin_list = (int*)(ctx->ws + L.bin_list);
    w.blkflop = (unsigned long long*)(ctx->ws + L.blkflop);
    w.nflop = M > 0 ? analyze_blocks(nnzA, M) : 0;
    w.scan_part = (int*)(ctx->ws + L.scan_part);
    w.cursors = w.scan_part + 2 * ((M + 1 + SCAN_ITEMS - 1) / SCAN_ITEMS + 1);
    w.mcache = ctx->use_mcache ? (unsigned long long*)(ctx->ws + L.mcache) : nullptr;
    w.mc_list = mc_list;
    w.spill.mask = (unsigned long long*)(ctx->ws + L.spill_mask);
    w.spill.key = (int*)(ctx->ws + L.spill_key);
    w.spill.lofs = (int*)(ctx->ws + L.lofs);
    w.spill.top = w.cursors + SPILL_CURSOR_SLOT * 8 * CURSOR_STRIDE;  // zeroed with the cursors
    w.spill.cap = L.spill_cap;
    w.tslot = (long long*)(ctx->ws + L.tslot);
    w.split_list = (int*)(ctx->ws + L.split_list);
    if (L.near) {
        w.near_list = (int*)(ctx->ws + L.near_list);
        w.nsig = (unsigned*)(ctx->ws + L.nsig);
        w.ucol = (int*)(ctx->ws + L.ucol);
        w.bx_val = (double*)(ctx->ws + L.bx_val);
        w.uval = w.bx_val + L.bx_pre;
        if (L.near_b) {  // B is A: its union runs read bx_*
            w.bx_col = (int*)(ctx->ws + L.bx_col);
            w.ucolx = w.bx_col + nnzB;
        }
        w.gna = (int*)(ctx->ws + L.gna);
    }
    w.stats = (Stats*)(ctx->ws + L.stats);
    w.gscratch = ctx->gscratch;
    w.gscratch_bytes = ctx->gscratch_bytes;
    return w;
}

std::string err_text(int err) {
    std::string m;
    if (err & ERR_UNSORTED) m += "B column indices are not sorted within a row; ";
    if (err & ERR_COL_RANGE) m += "B column index out of [0, B.N); ";
    if (err & ERR_ACOL_RANGE) m += "A column index out of [0, B.M); ";
    if (err & ERR_OVERFLOW) m += "nnz(C) exceeds INT32_MAX; ";
    return m;
}

// Everything before the numeric launches for the rows of `a` (M > 0): (mask of B), row
// analysis, symbolic bins, row_ptr scan into Cptr[0..M] + numeric bins, the Stats hand-off.
int front_pass(mhs_ctx* ctx, const Csr& a, const Csr& b, Work& w, int* Cptr, bool mask, Stats& h) {
    hipStream_t s = ctx->stream;
    if (!ctx->stats_zero) MHS_HIP(hipMemsetAsync(w.stats, 0, sizeof(Stats), s));
    ctx->stats_zero = false;
    if (mask) launch_mask_b(b, w, s);
    launch_analyze(a, w, b.M, s, Cptr);
    launch_symbolic_common(a, b, w, a.M, b.N, Cptr, s);
    launch_symbolic_rare(a, w, a.M, b.N, Cptr, s, false);
    launch_symbolic_b256(a, w, a.M, b.N, Cptr, s);
    const int seq = ++ctx->seq;
    launch_scan_classify(a.M, w, Cptr, a.ptr, s, ctx->dense_span_max, ctx->d_pub, seq, SpecArgs{});
    MHS_HIP(hipGetLastError());
    const int rc = wait_published(ctx, s, ctx->pub, seq);
    if (rc) return rc;
    memcpy(&h, (const void*)&ctx->pub->stats, sizeof(Stats));
    ctx->stats_zero = true;
    ++ctx->front_passes;
    return MHS_OK;
}

// Global-bin scratch for the numeric pass of `h` (grown on demand).
int ensure_gscratch(mhs_ctx* ctx, Work& w, const Stats& h);

constexpr int NUM_GLOBAL_GRID = 128;
#ifndef MHS_MULTI_FLOP_LOG2
#define MHS_MULTI_FLOP_LOG2 22  // numeric launches over several streams from 2^this products on (round 4: 24 -> 22, scircuit-like numeric -9 %)
#endif

#ifndef MHS_SPLIT_FLOP_LOG2
#define MHS_SPLIT_FLOP_LOG2 24  // block bins split by LDS need from 2^this products on
#endif

// Streams the numeric launches of `h` are dealt over: several heavy bins go over the aux
// streams (fork/join costs ~10-20 us, so only for at least 3 launches of a product worth it).
int numeric_streams(const mhs_ctx* ctx, const Stats& h) {
    const int nl = numeric_launches(h);
    return (nl >= 3 && h.flop >= (1ull << MHS_MULTI_FLOP_LOG2)) ? std::min(ctx->num_streams, nl) : 1;
}

// The numeric launches for `h` (grids, LDS) on the call's stream, the heavy bins dealt over
// the aux streams, which join the call's stream again.
// Phases of a numeric launch sequence: ALL (after the hand-off: every launch), and the two halves
// of a speculated plan -- SPEC_A, queued right behind k_scan before its Stats are known: the fork
// event, the block-bin split and the launches dealt to the call's stream; SPEC_B, after the host
// has seen k_scan's verdict: the aux streams' launches (their wait on the fork event then finds
// it complete -- waits on a pending one measured slower than the whole hand-off, r06b) and joins.
enum NumPhase { NUM_ALL = 0, NUM_SPEC_A = 1, NUM_SPEC_B = 2 };

int run_numeric(mhs_ctx* ctx, const Csr& a, const Csr& b, const Work& w, const Stats& h, const mhs_csr& out,
                hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr, int phase = NUM_ALL) {
    hipStream_t s = ctx->stream;
    // several heavy bins: deal them over the aux streams (fork/join costs ~10-20 us,
    // so only when there are at least 3 launches of a product worth it)
    hipStream_t ss[mhs_ctx::NAUX + 1] = {s};
    int nss = numeric_streams(ctx, h);
    if (w.go) nss = std::min(nss, ctx->spec_nss);  // (MHS_SPEC_NSS: a speculated plan on fewer streams)
    for (int i = 1; i < nss; ++i) ss[i] = ctx->aux[i - 1];
    hipError_t fe = hipSuccess;
    const bool first = phase != NUM_SPEC_B, last = phase != NUM_SPEC_A;
    if (phase == NUM_SPEC_B && nss == 1) return MHS_OK;  // (phase A launched everything)
    if (first && nss > 1 && ev0) MHS_HIP(hipEventRecord(ev0, s));  // (several streams: events of their own)
    if (first && nss > 1) MHS_HIP(hipEventRecord(ctx->fork_ev, s));
    // the aux streams wait for the fork (everything before numeric) -- set up after the first
    // numeric launch has gone out on the call's stream (launch_numeric)
    auto fork = [&]() {
        for (int i = 1; i < nss && fe == hipSuccess; ++i) fe = hipStreamWaitEvent(ss[i], ctx->fork_ev, 0);
        return fe == hipSuccess;
    };
    // block bins split by LDS need only where their two launches can run side by side (on
    // one stream the hub rows' launch would no longer overlap the others' bulk).  The partition
    // runs on the call's stream after the fork: only the split launches wait for it (split_ev),
    // the other bins start at once (wb-edu-like: 0.33 ms off the numeric phase's start)
    // (and only from 2^MHS_SPLIT_FLOP_LOG2 products: on scircuit-like the partition and its event
    // wait cost more than the split saves -- numeric 0.146 -> 0.119 ms unsplit)
    const bool want_split = nss > 1 && ctx->split && h.flop >= (1ull << MHS_SPLIT_FLOP_LOG2);
    bool split = false;
    if (first) {
        split = want_split && launch_split_bins(w, h, a.M, out.ptr, s, ctx->dense_span_max);
        if (split) MHS_HIP(hipEventRecord(ctx->split_ev, s));
        ctx->split_on = split;
        ctx->stat[MHS_STAT_SPLIT] += split;
        ctx->stat[MHS_STAT_MULTI_STREAM] += nss > 1;
    } else {
        split = ctx->split_on;  // (phase A's decision)
    }
    const int only = phase == NUM_SPEC_A ? 1 : phase == NUM_SPEC_B ? ~1 : ~0;
    const int used = launch_numeric(a, b, w, h, out.ptr, out.col, out.val, ss, nss, NUM_GLOBAL_GRID,
                                    ctx->dense_span_max, split, split ? ctx->split_ev : nullptr,
                                    nss > 1 ? std::function<bool()>(fork) : std::function<bool()>(),
                                    nss == 1 ? ev0 : nullptr, nss == 1 ? ev1 : nullptr, only);
    if (nss == 1 && (used & (1 << 30))) {  // (no launch carried them)
        if (ev0) MHS_HIP(hipEventRecord(ev0, s));
        if (ev1) MHS_HIP(hipEventRecord(ev1, s));
    }
    if (!last) {
        MHS_HIP(hipGetLastError());
        return MHS_OK;
    }
    // joins first: an error below must not leave aux-stream work behind the call's stream
    for (int i = 1; i < nss; ++i)
        if (used & (1 << i)) {
            MHS_HIP(hipEventRecord(ctx->join_ev[i - 1], ss[i]));
            MHS_HIP(hipStreamWaitEvent(s, ctx->join_ev[i - 1], 0));
        }
    if (nss > 1 && ev1) MHS_HIP(hipEventRecord(ev1, s));
    MHS_HIP(fe);
    MHS_HIP(hipGetLastError());
    return MHS_OK;
}

int ensure_gscratch(mhs_ctx* ctx, Work& w, const Stats& h) {
    if (h.num_count[NUM_GLOBAL] <= 0) return MHS_OK;
    const size_t per = (size_t)align16(h.num_global_need);
    const size_t g = (size_t)std::min(h.num_count[NUM_GLOBAL], NUM_GLOBAL_GRID);
    const int rc = ensure(ctx, &ctx->gscratch, &ctx->gscratch_bytes, per * g);
    if (rc) return rc;
    w.gscratch = ctx->gscratch;
    w.gscratch_bytes = ctx->gscratch_bytes;
    return MHS_OK;
}

void free_cached(mhs_ctx* ctx) {
    if (ctx->ws) (void)hipFree(ctx->ws);
    if (ctx->gscratch) (void)hipFree(ctx->gscratch);
    if (ctx->slots) (void)hipFree(ctx->slots);
    ctx->ws = ctx->gscratch = ctx->slots = nullptr;
    ctx->ws_bytes = ctx->gscratch_bytes = ctx->slots_bytes = 0;
    for (auto& b : ctx->pool) (void)hipFree(b.first);
    ctx->pool.clear();
    ctx->stats_zero = false;
}

// Row-chunked product, the fallback when the workspace (or the workspace and C together)
// does not fit the device.  Everything cached is given back; a counting pass runs with the
// largest chunk workspace that fits (Mc rows, halved until it does) and sizes C; the
// workspace is freed and C allocated -- C's size does not depend on the chunking, so when C
// alone does not fit the call fails right there, after one pass; then the workspace is laid
// out again for the memory C leaves (halved only while the workspace itself does not fit)
// and a second pass writes every chunk's rows at their offset in C (row_ptr rebased by one
// small kernel per chunk).  The reference has no such path: Tool::allocate and the C
// cudaMalloc simply throw (src/Tool.cu:4-45, src/main.cu:54-61).
int spgemm_chunked(mhs_ctx* ctx, const mhs_csr* A, const mhs_csr* B, mhs_csr* C, mhs_timing* t,
                   std::chrono::steady_clock::time_point T0) {
    const int M = A->M, MB = B->M;
    hipStream_t s = ctx->stream;
    MHS_HIP(hipStreamSynchronize(s));
    free_cached(ctx);
    (void)hipGetLastError();
    int Mc = M, mc_list = 0;
    Layout L{};
    const Csr b{B->M, B->N, B->nnz, B->ptr, B->col, B->val};
    auto view = [&](int c) {
        const int r0 = c * Mc, r1 = std::min(M, r0 + Mc);
        // nnz of a view only steers launch geometry: the same estimate in plan and launch
        const int est = (int)((long long)A->nnz * (r1 - r0) / (M > 0 ? M : 1));
        return Csr{r1 - r0, A->N, est, A->ptr + r0, A->col, A->val};
    };
    // the workspace for chunks of Mc rows: `first` rows, then halved until it fits (a one-row
    // workspace is tried before the call gives up)
    auto fit_workspace = [&](int first) {
        for (Mc = first;; Mc = (Mc + 1) / 2) {
            if (ctx->ws) (void)hipFree(ctx->ws);
            ctx->ws = nullptr;
            ctx->ws_bytes = 0;
            ctx->stats_zero = false;
            mc_list = ctx->mc_list > 0 ? ctx->mc_list : mc_list_for(Mc);
            L = plan(Mc, MB, A->nnz, B->nnz, mc_list, M);
            const int rc = ensure(ctx, &ctx->ws, &ctx->ws_bytes, L.total);
            if (rc != MHS_ERR_OOM) return rc;
            (void)hipGetLastError();
            if (Mc <= 1) return fail(ctx, MHS_ERR_OOM, "a one-row workspace does not fit the device");
        }
    };
    int rc = fit_workspace((M + 1) / 2);  // (the whole-M workspace has just failed)
    if (rc) return rc;
    // pass 1: counts
    int nch = (M + Mc - 1) / Mc;
    Stats h{};
    long long total = 0;
    unsigned long long flop = 0;
    {
        int* tptr = nullptr;
        MHS_HIP(pool_get(ctx, (void**)&tptr, (size_t)(Mc + 1) * 4));
        for (int c = 0; c < nch && rc == MHS_OK; ++c) {
            const Csr a = view(c);
            Work w = make_work(ctx, L, a.M, a.nnz, B->nnz, B->N, mc_list);
            rc = front_pass(ctx, a, b, w, tptr, c == 0, h);
            if (rc == MHS_OK && h.err)
                rc = fail(ctx, (h.err & ERR_OVERFLOW) ? MHS_ERR_OVERFLOW : MHS_ERR_INVALID, err_text(h.err));
            total += h.nnzC;
            flop += h.flop;
        }
        pool_put(ctx, tptr);
        if (rc) return rc;
    }
    if (total > INT_MAX) return fail(ctx, MHS_ERR_OVERFLOW, "nnz(C) exceeds INT32_MAX");
    // C before the second pass's workspace: it does not depend on the chunking
    const int Mc1 = Mc;
    free_cached(ctx);
    mhs_csr out{};
    out.M = M;
    out.N = B->N;
    out.nnz = (int)total;
    {
        hipError_t e = pool_get(ctx, (void**)&out.ptr, (size_t)(M + 1) * 4);
        if (e == hipSuccess) e = alloc_c(ctx, &out, total);
        if (e != hipSuccess) {
            pool_put(ctx, out.ptr);
            free_cached(ctx);
            (void)hipGetLastError();
            return e == hipErrorOutOfMemory ? fail(ctx, MHS_ERR_OOM, "C itself does not fit the device")
                                            : fail_hip(ctx, e, "allocating C (row-chunked)");
        }
    }
    ctx->c_held = (size_t)(M + 1) * 4 + (size_t)total * 12;
    rc = fit_workspace(Mc1);  // (pass 1 fitted Mc1 rows alone; C now sits beside it)
    ctx->c_held = 0;
    if (rc) {
        mhs_csr_free(&out);
        return rc;
    }
    nch = (M + Mc - 1) / Mc;
    // pass 2: every chunk's rows at their offset
    long long off = 0;
    int sym[NBINS] = {}, num[NBINS] = {};
    for (int c = 0; c < nch; ++c) {
        const Csr a = view(c);
        const int r0 = c * Mc;
        Work w = make_work(ctx, L, a.M, a.nnz, B->nnz, B->N, mc_list);
        rc = front_pass(ctx, a, b, w, out.ptr + r0, c == 0, h);
        if (rc == MHS_OK) rc = ensure_gscratch(ctx, w, h);
        if (rc) {
            (void)hipStreamSynchronize(s);
            mhs_csr_free(&out);
            return rc;
        }
        if (h.nnzC > 0)
            launch_numeric(a, b, w, h, out.ptr + r0, out.col + off, out.val + off, &s, 1, NUM_GLOBAL_GRID,
                           ctx->dense_span_max, false);
        launch_add_offset(out.ptr + r0, a.M + (c == nch - 1 ? 1 : 0), (int)off, s);
        MHS_HIP(hipGetLastError());
        off += h.nnzC;
        for (int i = 1; i < NBINS; ++i) {
            sym[i] += h.sym_count[i];
            num[i] += h.num_count[i];
        }
    }
    MHS_HIP(hipStreamSynchronize(s));
    *C = out;
    ++ctx->chunked_calls;
    if (t) {
        mhs_timing tm{};
        tm.total_e2e = tm.total_ref = ms_since(T0);
        tm.flop = flop;
        tm.nnzC = total;
        long long ns = 0, nn = 0;
        for (int i = 1; i < 16; ++i) {
            tm.sym_bins[i] = i < NBINS ? sym[i] : 0;
            tm.num_bins[i] = i < NBINS ? num[i] : 0;
            ns += tm.sym_bins[i];
            nn += tm.num_bins[i];
        }
        tm.sym_bins[0] = (int)(M - ns);
        tm.num_bins[0] = (int)(M - nn);
        *t = tm;
    }
    return MHS_OK;
}


}  // namespace

extern "C" {

int mhs_abi_version(void) { return MHS_ABI_VERSION; }

int mhs_ctx_create(mhs_ctx** out, int device) {
    if (!out) return MHS_ERR_INVALID;
    *out = nullptr;
    mhs_ctx* ctx = new mhs_ctx();
    ctx->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipHostMalloc((void**)&ctx->h_stats, sizeof(Stats), hipHostMallocDefault);
    if (e == hipSuccess)
        e = hipHostMalloc((void**)&ctx->pub, sizeof(Published), hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&ctx->d_pub, ctx->pub, 0);
    if (e == hipSuccess) memset(ctx->pub, 0, sizeof(Published));
    for (int i = 0; e == hipSuccess && i < 8; ++i) e = hipEventCreate(&ctx->ev[i]);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->stream_ev, hipEventDisableTiming);
    if (const char* v = getenv("MHS_NUM_STREAMS")) ctx->num_streams = std::max(1, std::min(atoi(v), mhs_ctx::NAUX + 1));
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->fork_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->split_ev, hipEventDisableTiming);
    for (int i = 0; e == hipSuccess && i + 1 < ctx->num_streams; ++i) {
        e = hipStreamCreateWithFlags(&ctx->aux[i], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->join_ev[i], hipEventDisableTiming);
    }
    if (e == hipSuccess) e = hipMalloc((void**)&ctx->d_go, 256);
    if (e == hipSuccess) e = init_kernel_attributes();
    if (e != hipSuccess) {
        fprintf(stderr, "mhs_ctx_create: %s\n", hipGetErrorString(e));
        delete ctx;
        return e == hipErrorOutOfMemory ? MHS_ERR_OOM : MHS_ERR_HIP;
    }
    ctx->stream = ctx->own_stream;
    if (const char* e = getenv("MHS_DENSE_SPAN")) ctx->dense_span_max = atoi(e);
    if (getenv("MHS_NO_MCACHE")) ctx->use_mcache = false;
    if (const char* e = getenv("MHS_MC_LIST")) ctx->mc_list = atoi(e) < MC_LIST_MIN ? MC_LIST_MIN : atoi(e);
    if (getenv("MHS_NO_GROUPS")) ctx->groups = false;
    if (getenv("MHS_NO_NEAR")) ctx->near = false;
    if (getenv("MHS_NO_SPLIT")) ctx->split = false;
    if (getenv("MHS_NO_TINY_NUM")) ctx->tiny_num = false;
    if (const char* e = getenv("MHS_NFT_MIN_M")) ctx->nft_min_m = atoll(e);
    if (getenv("MHS_NFT_NO_SLOTS")) ctx->nft_slots = false;
    if (const char* e = getenv("MHS_SYM_FORK")) ctx->sym_fork = atoi(e) != 0;
    if (const char* e = getenv("MHS_SYM_FORK_MIN_M")) ctx->sym_fork_min_m = atoll(e);
    if (const char* e = getenv("MHS_NFT_OTHER_PCT")) ctx->nft_other_pct = atoi(e);
    if (const char* e = getenv("MHS_NFT_AUTO_AVG")) ctx->nft_auto_avg = atoi(e);
    if (const char* e = getenv("MHS_NO_SPEC")) ctx->spec = atoi(e) == 0;
    if (const char* e = getenv("MHS_FORK_ORDER")) ctx->fork_common_first = atoi(e) != 0;
    if (const char* e = getenv("MHS_SPEC_FORK")) {
        ctx->spec_fork = atoi(e) == 1;
        ctx->spec_fork_rare = atoi(e) == 2;
    }
    if (const char* e = getenv("MHS_SPEC_NSS")) ctx->spec_nss = std::max(1, std::min(atoi(e), mhs_ctx::NAUX + 1));
    *out = ctx;
    return MHS_OK;
}

void mhs_ctx_destroy(mhs_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    mhs_ctx_trim(ctx);  // outstanding C buffers belong to the caller
    if (ctx->stream_ev) (void)hipEventDestroy(ctx->stream_ev);
    if (ctx->fork_ev) (void)hipEventDestroy(ctx->fork_ev);
    if (ctx->split_ev) (void)hipEventDestroy(ctx->split_ev);
    for (int i = 0; i < mhs_ctx::NAUX; ++i) {
        if (ctx->aux[i]) {
            (void)hipStreamSynchronize(ctx->aux[i]);
            (void)hipStreamDestroy(ctx->aux[i]);
        }
        if (ctx->join_ev[i]) (void)hipEventDestroy(ctx->join_ev[i]);
    }
    if (ctx->h_stats) (void)hipHostFree(ctx->h_stats);
    if (ctx->pub) (void)hipHostFree(ctx->pub);
    for (auto& ev : ctx->nev)
        if (ev) (void)hipEventDestroy(ev);
    for (auto& ev : ctx->ev)
        if (ev) (void)hipEventDestroy(ev);
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
    if (ctx->d_go) (void)hipFree(ctx->d_go);
    delete ctx;
}

const char* mhs_last_error(const mhs_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int mhs_ctx_set_stream(mhs_ctx* ctx, void* s) {
    if (!ctx) return MHS_ERR_INVALID;
    hipStream_t next = s ? (hipStream_t)s : ctx->own_stream;
    if (next != ctx->stream) {
        // the workspace is shared by every call: work queued on the old stream (an
        // unsynchronised call's numeric phase) must finish before the new stream's
        // first kernel rewrites it
        MHS_HIP(hipSetDevice(ctx->device));
        MHS_HIP(hipEventRecord(ctx->stream_ev, ctx->stream));
        MHS_HIP(hipStreamWaitEvent(next, ctx->stream_ev, 0));
        ctx->stream = next;
    }
    return MHS_OK;
}

int mhs_ctx_trim(mhs_ctx* ctx) {
    if (!ctx) return MHS_ERR_INVALID;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->ws) (void)hipFree(ctx->ws);
    if (ctx->gscratch) (void)hipFree(ctx->gscratch);
    if (ctx->slots) (void)hipFree(ctx->slots);
    ctx->ws = ctx->gscratch = ctx->slots = nullptr;
    ctx->ws_bytes = ctx->gscratch_bytes = ctx->slots_bytes = 0;
    for (auto& b : ctx->pool) (void)hipFree(b.first);
    ctx->pool.clear();
    return MHS_OK;
}

void mhs_csr_free(mhs_csr* C) {
    if (!C) return;
    if (C->ptr) (void)hipFree(C->ptr);
    if (C->col) (void)hipFree(C->col);
    if (C->val) (void)hipFree(C->val);
    std::memset(C, 0, sizeof *C);
}

void mhs_ctx_recycle(mhs_ctx* ctx, mhs_csr* C) {
    if (!C) return;
    if (!ctx) {
        mhs_csr_free(C);
        return;
    }
    pool_put(ctx, C->ptr);
    pool_put(ctx, C->col);
    pool_put(ctx, C->val);
    std::memset(C, 0, sizeof *C);
}

int mhs_spgemm(mhs_ctx* ctx, const mhs_csr* A, const mhs_csr* B, mhs_csr* C, mhs_timing* t) {
    if (!ctx) return MHS_ERR_INVALID;
    if (!A || !B || !C) return fail(ctx, MHS_ERR_INVALID, "null argument");
    if (A->M < 0 || A->N < 0 || A->nnz < 0 || B->M < 0 || B->N < 0 || B->nnz < 0)
        return fail(ctx, MHS_ERR_INVALID, "negative dimension");
    if (A->N != B->M)
        return fail(ctx, MHS_ERR_INVALID, "A.N != B.M (C = A*B needs matching inner dimension)");
    if ((A->M > 0 && !A->ptr) || (B->M > 0 && !B->ptr) || (A->nnz > 0 && (!A->col || !A->val)) ||
        (B->nnz > 0 && (!B->col || !B->val)))
        return fail(ctx, MHS_ERR_INVALID, "null device array");
    MHS_HIP(hipSetDevice(ctx->device));
    const auto T0 = std::chrono::steady_clock::now();
    hipStream_t s = ctx->stream;
    const bool timed = t != nullptr;
    mhs_timing tm{};

    const int M = A->M, N = B->N, MB = B->M;
    mhs_csr out{};
    out.M = M;
    out.N = N;

    // ---- mem_alloc: workspace (cached across calls) + C.ptr --------------------
    const int mc_list = ctx->mc_list > 0 ? ctx->mc_list : mc_list_for(M);
    const bool probe = ctx->tiny_num && ctx->nft_min_m >= 0 && M >= ctx->nft_min_m && M > 0;
    // numeric-first without the probe (short-row matrices below nft_min_m rows): every tiny row
    // is sorted once, in symbolic, into slots sized by the per-row bound
    const bool nft_auto = !probe && M > 0 && ctx->nft_min_m >= 0 && M < ctx->nft_min_m && ctx->tiny_num &&
                          ctx->nft_slots && ctx->nft_auto_avg > 0 && A->nnz < (long long)ctx->nft_auto_avg * M;
    // near row groups: with the row cache (their C patterns are compared there), not with
    // the numeric-first probe (big M), and union rows of at most 3 x 32 M values
    bool near = ctx->near && ctx->groups && ctx->use_mcache && !probe && !nft_auto && A->nnz <= (1 << 25);
    const bool same_ab = A->ptr == B->ptr && A->col == B->col && A->val == B->val;
    Layout L = plan(M, MB, A->nnz, B->nnz, mc_list, -1, near, near && same_ab);
    const char* ws_before = ctx->ws;
    int rc = ensure(ctx, &ctx->ws, &ctx->ws_bytes, L.total);
    if (rc == MHS_ERR_OOM && near) {  // near groups are an optimisation: drop them before chunking
        (void)hipGetLastError();
        near = false;
        L = plan(M, MB, A->nnz, B->nnz, mc_list, -1, false);
        rc = ensure(ctx, &ctx->ws, &ctx->ws_bytes, L.total);
    }
    if (rc == MHS_ERR_OOM && M > 1) return spgemm_chunked(ctx, A, B, C, t, T0);
    if (rc) return rc;
    if (ctx->ws != ws_before) ctx->stats_zero = false;
    {
        const hipError_t e = pool_get(ctx, (void**)&out.ptr, (size_t)(M + 1) * 4);
        if (e == hipErrorOutOfMemory && M > 1) {
            (void)hipGetLastError();
            return spgemm_chunked(ctx, A, B, C, t, T0);
        }
        if (e != hipSuccess) return fail_hip(ctx, e, "allocating C.ptr");
    }
    Work w = make_work(ctx, L, M, A->nnz, B->nnz, B->N, mc_list);
    w.near_b = L.near && same_ab;
    if (L.near) {
        w.vcheck = B->val;
        w.vcheck_n = B->nnz;
    }
    // device Stats start zeroed: the previous call's k_scan left them so, else a memset
    if (!ctx->stats_zero) MHS_HIP(hipMemsetAsync(w.stats, 0, sizeof(Stats), s));
    ctx->stats_zero = false;  // until this call's k_scan has published and cleared them
    if (M == 0) {
        MHS_HIP(hipMemsetAsync(out.ptr, 0, 4, s));
    }
    const double t_alloc = ms_since(T0);
    if (timed) MHS_HIP(hipEventRecord(ctx->ev[0], s));

    const Csr a{A->M, A->N, A->nnz, A->ptr, A->col, A->val};
    const Csr b{B->M, B->N, B->nnz, B->ptr, B->col, B->val};

    // ---- Form_mask_matrix_B ------------------------------------------------------
    launch_mask_b(b, w, s);
    if (timed) MHS_HIP(hipEventRecord(ctx->ev[1], s));
    // ---- symbolic_binning ---------------------------------------------------------
    // numeric-first tiny rows (big M): k_analyze also bins the rows that way and counts
    // them; the host picks the bin lists and sizes the candidates' value slots
    unsigned long long other = 0;
    if (probe) w.nft_bin = (unsigned char*)(ctx->ws + L.nft_bin);
    if (nft_auto) {
        const size_t n = (size_t)M * TINY_SLOT_MAX;
        if (ensure(ctx, &ctx->slots, &ctx->slots_bytes, n * 12) == MHS_OK) {
            w.nft_bin = (unsigned char*)(ctx->ws + L.nft_bin);
            w.nft = 1;
            w.sc_val = (double*)ctx->slots;
            w.sc_col = (int*)(ctx->slots + n * 8);
        } else {
            (void)hipGetLastError();
        }
    }
    const int seq_probe = probe ? ++ctx->seq : 0;
    launch_analyze(a, w, MB, s, out.ptr, probe ? ctx->d_pub : nullptr, seq_probe);
    if (probe) {
        MHS_HIP(hipGetLastError());
        rc = wait_published(ctx, s, ctx->pub, seq_probe);
        if (rc) {
            pool_put(ctx, out.ptr);
            return rc;
        }
        const unsigned long long n = ctx->pub->stats.an_slots;
        other = ctx->pub->stats.an_other;
        w.sym_big = other >= (1ull << 21);
        // slots pay where the tiny rows are (nearly) the whole product: elsewhere numeric's
        // tiny classes run beside the long rows' kernels anyway (measured: wb-edu-like +10%
        // with slots, 19% of its rows past the tiny classes; GAP-road- / delaunay-like -12% / -17%)
        if (n > 0 && ctx->nft_slots && other * 100 <= (unsigned long long)M * ctx->nft_other_pct &&
            ensure(ctx, &ctx->slots, &ctx->slots_bytes, (size_t)n * 12) == MHS_OK) {
            w.nft = 1;
            w.sc_val = (double*)ctx->slots;
            w.sc_col = (int*)(ctx->slots + (size_t)n * 8);
        } else {
            (void)hipGetLastError();
        }
        launch_bin_list(a, w, s);
    }
    if (timed) MHS_HIP(hipEventRecord(ctx->ev[2], s));
    // ---- launch plan speculation (SpecArgs): the previous call's numeric plan on the same
    // operands goes out right behind k_scan, checked on the device; not with the numeric-first
    // probe (its own hand-off) or a forked symbolic pass
    const bool fork_big = ctx->sym_fork_min_m >= 0 && M >= ctx->sym_fork_min_m;
    bool fork_sym = ((w.nft && other > 0) || ctx->sym_fork || fork_big) && ctx->num_streams > 1 && ctx->aux[0];
    mhs_ctx::PlanKey key{};
    {
        const void* ps[6] = {A->ptr, A->col, A->val, B->ptr, B->col, B->val};
        for (int i = 0; i < 6; ++i) key.p[i] = ps[i];
        key.M = M;
        key.N = N;
        key.MB = MB;
        key.nnzA = A->nnz;
        key.nnzB = B->nnz;
        key.gen = ctx->gen;
        key.near = L.near;
        key.nft = w.nft;
        key.mc_list = mc_list;
    }
    const bool plannable = ctx->spec && M > 0 && !probe && (!fork_sym || ctx->spec_fork);
    // (a plan dealt over several streams queues only its call-stream launches ahead of k_scan: see
    // NumPhase)
    const bool spec = plannable && ctx->plan_valid && ctx->plan_key == key;
    const Stats ph = ctx->plan_h;  // (a copy: this call replaces the plan)
    // a speculated call whose plan has rows in the rare symbolic bins runs them on an aux stream
    // beside k_sym_common (their 38 us ran after it on scircuit-like); the plan left them out where
    // they were empty
    if (spec && !fork_sym && ctx->spec_fork_rare && ctx->num_streams > 1 && ctx->aux[0] &&
        (ph.sym_count[SYM_WM] > 0 || ph.sym_count[SYM_B1024] > 0 || ph.sym_count[SYM_GLOBAL] > 0))
        fork_sym = true;
    ctx->plan_valid = false;  // (set again by this call's success)
    // ---- Calculate_C_nnz ------------------------------------------------------------
    // persistent grids that read their bins' sizes on the device: no host round trip.
    // Numeric-first: rows of the rare bins (long, few) run on an aux stream beside the
    // common bins -- their tail no longer idles the chip
    if (fork_sym) {
        ++ctx->stat[MHS_STAT_SYM_FORK];
        MHS_HIP(hipEventRecord(ctx->fork_ev, s));
        if (ctx->fork_common_first) {  // (the call stream's launch first: no host launch ahead of it)
            launch_symbolic_common(a, b, w, M, N, out.ptr, s, spec ? &ph : nullptr);
            MHS_HIP(hipStreamWaitEvent(ctx->aux[0], ctx->fork_ev, 0));
            launch_symbolic_rare(a, w, M, N, out.ptr, ctx->aux[0], false);
        } else {
            MHS_HIP(hipStreamWaitEvent(ctx->aux[0], ctx->fork_ev, 0));
            launch_symbolic_rare(a, w, M, N, out.ptr, ctx->aux[0], false);
            launch_symbolic_common(a, b, w, M, N, out.ptr, s, spec ? &ph : nullptr);
        }
        launch_symbolic_b256(a, w, M, N, out.ptr, s);
        MHS_HIP(hipEventRecord(ctx->join_ev[0], ctx->aux[0]));
        MHS_HIP(hipStreamWaitEvent(s, ctx->join_ev[0], 0));
        launch_near(a, w, out.ptr, s);
    } else {
        launch_symbolic_common(a, b, w, M, N, out.ptr, s, spec ? &ph : nullptr);
        // a speculated plan leaves out the rare bins' launches where the plan's bins are empty
        // (a row in one of them changes the Stats: k_scan rejects the plan, the call reruns)
        const bool rare = !spec || ph.sym_count[SYM_WM] > 0 || ph.sym_count[SYM_B1024] > 0 ||
                          ph.sym_count[SYM_GLOBAL] > 0 || (L.near && ph.near_heads > 0);
        if (rare) launch_symbolic_rare(a, w, M, N, out.ptr, s, true);  // (+ near row groups)
        if (!spec || ph.sym_count[SYM_B256] > 0) launch_symbolic_b256(a, w, M, N, out.ptr, s);
        ctx->stat[MHS_STAT_SPEC_SKIPPED] += (!rare) + (spec && ph.sym_count[SYM_B256] == 0);
    }
    MHS_HIP(hipGetLastError());
    if (timed) MHS_HIP(hipEventRecord(ctx->ev[3], s));
    // ---- numeric_binning: scan, classify, bins, one readback ------------------------
    Stats h;
    bool launched = false;  // the speculated numeric launches went out
    double t_malloc = 0;
    const int nring = (int)ctx->nev.size() / 2;
    const int slot = nring ? (int)(ctx->ncalls % nring) : 0;
    if (M > 0) {
        // the numeric bin offsets kernel publishes Stats to pinned host memory; the
        // host spins on the sequence number (no stream sync, no interrupt wake-up)
        const int seq = ++ctx->seq;
        launch_scan_classify(M, w, out.ptr, a.ptr, s, ctx->dense_span_max, ctx->d_pub, seq,
                             spec ? SpecArgs{ctx->d_go, ph} : SpecArgs{});
        MHS_HIP(hipGetLastError());
        if (timed) MHS_HIP(hipEventRecord(ctx->ev[4], s));
        if (spec) {
            const auto T5 = std::chrono::steady_clock::now();
            hipError_t e = alloc_c(ctx, &out, ph.nnzC);
            if (e == hipSuccess) {
                const int g = ensure_gscratch(ctx, w, ph);
                e = g == MHS_OK ? hipSuccess : hipErrorOutOfMemory;
                if (g != MHS_OK) mhs_ctx_recycle_cols(ctx, &out);
            }
            if (e == hipSuccess) {
                if (w.near_b && ph.near_verified > 0 && B->nnz > 0) {
                    MHS_HIP(hipMemcpyAsync(w.bx_col, B->col, (size_t)B->nnz * 4, hipMemcpyDeviceToDevice, s));
                    MHS_HIP(hipMemcpyAsync(w.bx_val, B->val, (size_t)B->nnz * 8, hipMemcpyDeviceToDevice, s));
                    w.bx_on = 1;
                }
                t_malloc = ms_since(T5);
                if (timed) MHS_HIP(hipEventRecord(ctx->ev[5], s));
                w.go = ctx->d_go;
                if (ph.nnzC > 0) {
                    out.nnz = (int)ph.nnzC;
                    rc = run_numeric(ctx, a, b, w, ph, out, nring ? ctx->nev[2 * slot] : nullptr,
                                     nring ? ctx->nev[2 * slot + 1] : nullptr, NUM_SPEC_A);
                    if (rc) {
                        (void)hipStreamSynchronize(s);
                        mhs_ctx_recycle(ctx, &out);
                        return rc;
                    }
                } else if (nring) {
                    MHS_HIP(hipEventRecord(ctx->nev[2 * slot], s));
                    MHS_HIP(hipEventRecord(ctx->nev[2 * slot + 1], s));
                }
                if (timed) MHS_HIP(hipEventRecord(ctx->ev[6], s));
                launched = true;
                ++ctx->stat[MHS_STAT_SPEC];
            } else {
                (void)hipGetLastError();  // (no room for the plan's C: the hand-off path decides)
            }
        }
        rc = wait_published(ctx, s, ctx->pub, seq);
        if (rc) {
            if (launched) (void)hipStreamSynchronize(s);
            if (launched) mhs_ctx_recycle_cols(ctx, &out);
            pool_put(ctx, out.ptr);
            return rc;
        }
        memcpy(&h, (const void*)&ctx->pub->stats, sizeof(Stats));
        ctx->stats_zero = true;  // k_scan's last block cleared them after publishing
        if (launched && !h.err && stats_same_plan(h, ph) && ph.nnzC > 0) {
            // the plan holds: its aux-stream launches and joins (phase B)
            rc = run_numeric(ctx, a, b, w, ph, out, nring ? ctx->nev[2 * slot] : nullptr,
                             nring ? ctx->nev[2 * slot + 1] : nullptr, NUM_SPEC_B);
            if (rc) {
                (void)hipStreamSynchronize(s);
                mhs_ctx_recycle(ctx, &out);
                return rc;
            }
        }
        if (launched && (h.err || !stats_same_plan(h, ph))) {
            // the plan was not this call's: its kernels returned at once (k_scan wrote go = 0);
            // every array is rewritten by a call without speculation
            MHS_HIP(hipStreamSynchronize(s));
            mhs_ctx_recycle_cols(ctx, &out);
            ++ctx->stat[MHS_STAT_SPEC_MISS];
            if (!h.err) {
                pool_put(ctx, out.ptr);
                return mhs_spgemm(ctx, A, B, C, t);  // (plan_valid is false: no speculation)
            }
            launched = false;
        }
    } else {
        MHS_HIP(hipGetLastError());
        MHS_HIP(hipMemcpyAsync(ctx->h_stats, w.stats, sizeof(Stats), hipMemcpyDeviceToHost, s));
        if (timed) MHS_HIP(hipEventRecord(ctx->ev[4], s));
        MHS_HIP(hipStreamSynchronize(s));
        h = *ctx->h_stats;
    }
    if (h.err) {
        pool_put(ctx, out.ptr);
        return fail(ctx, (h.err & ERR_OVERFLOW) ? MHS_ERR_OVERFLOW : MHS_ERR_INVALID, err_text(h.err));
    }
    out.nnz = (int)h.nnzC;
    ctx->stat[MHS_STAT_NFT] += w.nft != 0;
    ctx->stat[MHS_STAT_NEAR] += L.near && h.near_verified > 0;

    if (!launched) {
        // ---- Malloc_C_col_val ---------------------------------------------------------------
        const auto T5 = std::chrono::steady_clock::now();
        {
            const hipError_t e = alloc_c(ctx, &out, out.nnz);
            if (e != hipSuccess) {
                pool_put(ctx, out.ptr);
                (void)hipGetLastError();
                // C beside the full workspace does not fit: retry with a row-chunked workspace
                if (e == hipErrorOutOfMemory && M > 1) return spgemm_chunked(ctx, A, B, C, t, T0);
                return fail_hip(ctx, e, "allocating C.col/C.val");
            }
        }
        rc = ensure_gscratch(ctx, w, h);
        // near union runs of B (A*A, near groups verified): B's arrays copied in front of the union
        // rows (in the near check instead, for every call with candidates: cant-perturbed-like -1.5 %,
        // cant-s1-like symbolic +5 % -- candidates, no groups)
        if (rc == MHS_OK && w.near_b && h.near_verified > 0 && B->nnz > 0) {
            MHS_HIP(hipMemcpyAsync(w.bx_col, B->col, (size_t)B->nnz * 4, hipMemcpyDeviceToDevice, s));
            MHS_HIP(hipMemcpyAsync(w.bx_val, B->val, (size_t)B->nnz * 8, hipMemcpyDeviceToDevice, s));
            w.bx_on = 1;
        }
        if (rc) {
            mhs_ctx_recycle(ctx, &out);
            (void)hipGetLastError();
            if (rc == MHS_ERR_OOM && M > 1) return spgemm_chunked(ctx, A, B, C, t, T0);
            return rc;
        }
        t_malloc = ms_since(T5);

        // ---- Numeric -------------------------------------------------------------------------
        if (timed) MHS_HIP(hipEventRecord(ctx->ev[5], s));
        w.go = nullptr;
        if (out.nnz > 0) {
            rc = run_numeric(ctx, a, b, w, h, out, nring ? ctx->nev[2 * slot] : nullptr,
                             nring ? ctx->nev[2 * slot + 1] : nullptr);
            if (rc) {
                mhs_ctx_recycle(ctx, &out);
                return rc;
            }
        } else if (nring) {
            MHS_HIP(hipEventRecord(ctx->nev[2 * slot], s));
            MHS_HIP(hipEventRecord(ctx->nev[2 * slot + 1], s));
        }
        MHS_HIP(hipGetLastError());
        if (timed) MHS_HIP(hipEventRecord(ctx->ev[6], s));
    }
    ++ctx->ncalls;
    if (timed || ctx->sync) MHS_HIP(hipStreamSynchronize(s));
    *C = out;
    if (plannable) {  // the next call on these operands may speculate on this call's plan
        ctx->plan_key = key;
        ctx->plan_h = h;
        ctx->plan_valid = true;
    }

    if (timed) {
        float f = 0;
        tm.mem_alloc = t_alloc;
        MHS_HIP(hipEventElapsedTime(&f, ctx->ev[0], ctx->ev[1]));
        tm.Form_mask_matrix_B = f;
        MHS_HIP(hipEventElapsedTime(&f, ctx->ev[1], ctx->ev[2]));
        tm.symbolic_binning = f;
        MHS_HIP(hipEventElapsedTime(&f, ctx->ev[2], ctx->ev[3]));
        tm.Calculate_C_nnz = f;
        MHS_HIP(hipEventElapsedTime(&f, ctx->ev[3], ctx->ev[4]));
        tm.numeric_binning = f;
        tm.Malloc_C_col_val = t_malloc;
        MHS_HIP(hipEventElapsedTime(&f, ctx->ev[5], ctx->ev[6]));
        tm.Numeric = f;
        tm.total_e2e = ms_since(T0);
        tm.total_ref = tm.total_e2e - tm.Form_mask_matrix_B;
        tm.flop = h.flop;
        tm.nnzC = h.nnzC;
        for (int i = 0; i < 16; ++i) {
            tm.sym_bins[i] = i < NBINS ? h.sym_count[i] : 0;
            tm.num_bins[i] = i < NBINS ? h.num_count[i] : 0;
        }
        long long nonempty = 0;
        for (int i = 1; i < NBINS; ++i) nonempty += h.sym_count[i];
        tm.sym_bins[0] = (int)(M - nonempty);
        nonempty = 0;
        for (int i = 1; i < NBINS; ++i) nonempty += h.num_count[i];
        tm.num_bins[0] = (int)(M - nonempty);
        *t = tm;
    }
    return MHS_OK;
}

int mhs_transpose(mhs_ctx* ctx, const mhs_csr* A, mhs_csr* At) {
    if (!ctx || !A || !At) return fail(ctx, MHS_ERR_INVALID, "mhs_transpose: null argument");
    if (A->M < 0 || A->N < 0 || A->nnz < 0 || (A->M > 0 && !A->ptr) || (A->nnz > 0 && (!A->col || !A->val)))
        return fail(ctx, MHS_ERR_INVALID, "mhs_transpose: malformed A");
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return fail_hip(ctx, e, "hipSetDevice");
    const Csr a{A->M, A->N, A->nnz, A->ptr, A->col, A->val};
    size_t tmp_bytes = 0;
    e = transpose_csr(a, nullptr, nullptr, nullptr, nullptr, &tmp_bytes, ctx->stream);
    if (e != hipSuccess) return fail_hip(ctx, e, "transpose (scratch size)");
    mhs_csr T{A->N, A->M, A->nnz, nullptr, nullptr, nullptr};
    void* tmp = nullptr;
    e = hipMalloc((void**)&T.ptr, sizeof(int32_t) * ((size_t)A->N + 1));
    if (e == hipSuccess) e = hipMalloc((void**)&T.col, sizeof(int32_t) * (size_t)(A->nnz ? A->nnz : 1));
    if (e == hipSuccess) e = hipMalloc((void**)&T.val, sizeof(double) * (size_t)(A->nnz ? A->nnz : 1));
    if (e == hipSuccess) e = hipMalloc(&tmp, tmp_bytes ? tmp_bytes : 16);
    if (e == hipSuccess) e = transpose_csr(a, T.ptr, T.col, T.val, tmp, &tmp_bytes, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (tmp) (void)hipFree(tmp);
    if (e != hipSuccess) {
        mhs_csr_free(&T);
        return fail_hip(ctx, e, "transpose");
    }
    *At = T;
    return MHS_OK;
}

int mhs_ctx_set_option(mhs_ctx* ctx, int option, int value) {
    if (!ctx) return MHS_ERR_INVALID;
    switch (option) {
    case MHS_OPT_SYNC:
        ctx->sync = value != 0;
        return MHS_OK;
    case MHS_OPT_NUMERIC_EVENTS: {
        if (value < 0 || value > 4096) return fail(ctx, MHS_ERR_INVALID, "numeric event ring size out of [0, 4096]");
        MHS_HIP(hipSetDevice(ctx->device));
        MHS_HIP(hipStreamSynchronize(ctx->stream));
        for (auto& ev : ctx->nev) (void)hipEventDestroy(ev);
        ctx->nev.assign(2 * (size_t)value, nullptr);
        for (auto& ev : ctx->nev) MHS_HIP(hipEventCreate(&ev));
        ctx->ncalls = 0;
        return MHS_OK;
    }
    case MHS_OPT_MEM_BUDGET:
        if (value < 0) return fail(ctx, MHS_ERR_INVALID, "memory budget must be >= 0 MiB");
        ctx->mem_budget = (size_t)value << 20;
        ++ctx->gen;  // (a speculated plan belongs to the options it was made under)
        return MHS_OK;
    case MHS_OPT_SPECULATE:
        ctx->spec = value != 0;
        ctx->plan_valid = false;
        return MHS_OK;
    case MHS_OPT_TINY_FIRST_ROWS:
        ctx->nft_min_m = value;
        ++ctx->gen;
        return MHS_OK;
    default:
        return fail(ctx, MHS_ERR_INVALID, "unknown option");
    }
}

long long mhs_ctx_chunked_calls(const mhs_ctx* ctx) { return ctx ? ctx->chunked_calls : -1; }

long long mhs_ctx_stat(const mhs_ctx* ctx, int which) {
    if (!ctx || which < 0 || which > MHS_STAT_SPEC_SKIPPED) return -1;
    return which == MHS_STAT_CHUNKED ? ctx->chunked_calls : ctx->stat[which];
}

int mhs_ctx_numeric_ms(mhs_ctx* ctx, float* out, int n) {
    if (!ctx || (!out && n > 0)) return -MHS_ERR_INVALID;
    const long long ring = (long long)ctx->nev.size() / 2;
    if (ring == 0) return 0;
    long long have = ctx->ncalls < ring ? ctx->ncalls : ring;
    if (n < have) have = n;
    for (long long i = 0; i < have; ++i) {
        const long long call = ctx->ncalls - have + i;
        const int slot = (int)(call % ring);
        if (hipEventSynchronize(ctx->nev[2 * slot + 1]) != hipSuccess) return -MHS_ERR_HIP;
        float f = 0;
        if (hipEventElapsedTime(&f, ctx->nev[2 * slot], ctx->nev[2 * slot + 1]) != hipSuccess) return -MHS_ERR_HIP;
        out[i] = f;
    }
    return (int)have;
}

int mhs_probe_conflicts(mhs_ctx* ctx, uint64_t* count) {
    if (!ctx || !count) return MHS_ERR_INVALID;
    unsigned long long* dev = nullptr;
    MHS_HIP(hipSetDevice(ctx->device));
    MHS_HIP(probe_counter(&dev));
    if (!dev) return fail(ctx, MHS_ERR_INVALID, "probe statistics need the MHS_PROBE_STATS=1 build (libmhspgemm_probe.so)");
    unsigned long long v = 0;
    MHS_HIP(hipMemcpyAsync(&v, dev, sizeof v, hipMemcpyDeviceToHost, ctx->stream));
    MHS_HIP(hipMemsetAsync(dev, 0, sizeof v, ctx->stream));
    MHS_HIP(hipStreamSynchronize(ctx->stream));
    *count = v;
    return MHS_OK;
}

int mhs_memcpy(mhs_ctx* ctx, void* dst, const void* src, size_t bytes, int kind) {
    if (!ctx) return MHS_ERR_INVALID;
    if (bytes == 0) return MHS_OK;
    hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    MHS_HIP(hipSetDevice(ctx->device));
    MHS_HIP(hipMemcpyAsync(dst, src, bytes, k, ctx->stream));
    MHS_HIP(hipStreamSynchronize(ctx->stream));
    return MHS_OK;
}

int mhs_device_alloc(mhs_ctx* ctx, void** p, size_t bytes) {
    if (!ctx || !p) return MHS_ERR_INVALID;
    MHS_HIP(hipSetDevice(ctx->device));
    MHS_HIP(hipMalloc(p, bytes ? bytes : 16));
    return MHS_OK;
}

int mhs_device_free(mhs_ctx* ctx, void* p) {
    if (!ctx) return MHS_ERR_INVALID;
    if (p) MHS_HIP(hipFree(p));
    return MHS_OK;
}

int mhs_hbm_peak(mhs_ctx* ctx, size_t bytes, int iters, double* gbps) {
    if (!ctx) return MHS_ERR_INVALID;
    if (!gbps || iters <= 0 || bytes < (1u << 20))
        return fail(ctx, MHS_ERR_INVALID, "mhs_hbm_peak: needs gbps[3], iters > 0 and bytes >= 1 MiB");
    MHS_HIP(hipSetDevice(ctx->device));
    MHS_HIP(hbm_peak_run(bytes, iters, gbps));
    return MHS_OK;
}

}  // extern "C"
