// mhs_internal.hpp -- shared host/device declarations of the MI355X SpGEMM.
//
// Layout in HBM (all arrays live in the context workspace unless noted):
//   B side (per B row r, built by k_mask_b = Form_mask_matrix_B):
//     btcol[nnzB]  int32   tile column (col >> 6) of each 64-column tile of row r,
//     btmask[nnzB] uint64  bitmask of the row's columns inside that tile;
//                          row r's tiles sit at [B.ptr[r], B.ptr[r] + ntiles(r)),
//                          i.e. the tile arrays reuse B's own row_ptr (tiles(r) <= nnz(r)),
//                          so no scan and no second pass are needed.
//     bmeta[MB]    int4    {tile start (= B.ptr[r]), nnz(r), ntiles(r), lo tile}
//     bhi[MB]      int32   hi tile (lo = INT_MAX / hi = -1 for empty rows)
//   C side (per C row i, built by k_analyze):
//     rflop[M]  products of row i (saturated int32)   = the reference's "flop"
//     rtflop[M] tile products of row i               = the reference's "tile-flop"
//     rlo/rhi   tile span of row i
//     ctiles[M] distinct C tiles of row i (symbolic)
//     C.ptr     nnz of row i (symbolic), then scanned in place to the row_ptr
//   binning: bin id per row (uint8), per-block bin counts, row lists grouped by bin.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <functional>

namespace mhs {

constexpr int TILE_SHIFT = 6;  // 64-column tiles, one uint64 mask each (wave64 ballot width)
constexpr int TILE_BITS = 64;
constexpr int NBINS = 16;  // capacity of the per-bin counters
constexpr int WPB = 4;          // waves per block in the wave-per-row kernels
constexpr int LDS_MAX_C = 163840;  // gfx950: 160 KiB per workgroup (probed on the box)
constexpr int MHS_SCAN_ITEMS = 1024;
constexpr int SCAN_ITEMS = MHS_SCAN_ITEMS;  // rows per block (of 1024 threads) in the row_ptr scan and the bin lists
// Row cursors of the dynamically scheduled bin walks: a launch slot (numeric bin b: b,
// symbolic bin b: NUM_NB + b) has one cursor per XCD group, 64 bytes apart.  They live after
// k_scan's look-back words and are zeroed with them by k_analyze.
constexpr int CURSOR_SLOTS = 40;
constexpr int CURSOR_STRIDE = 16;  // ints
constexpr int CURSOR_INTS = CURSOR_SLOTS * 8 * CURSOR_STRIDE;
// Bin-list counters (round 6): the per-(block, bin) atomics of k_bin_list / k_scan that reserve a
// block's places in a bin's list, one 128-byte line per bin (they were the 16 ints of Stats'
// sym_count / num_count, one line: every block's reservations serialised on it), then k_bin_list's
// done counter.  After the cursors, zeroed with them by k_analyze; the last block of each kernel
// copies its totals into Stats.
#ifndef MHS_BINCNT_STRIDE
#define MHS_BINCNT_STRIDE 32
#endif
constexpr int BINCNT_STRIDE = MHS_BINCNT_STRIDE;  // ints (128 bytes; 1: the counters on one line, A/B)
constexpr int BINCNT_INTS = (2 * NBINS + 1) * BINCNT_STRIDE;
constexpr int ZERO_INTS = (CURSOR_INTS + BINCNT_INTS + 1) & ~1;  // cursors + bin counters, zeroed per call in 8-byte words
constexpr int SPILL_PARTS = 64;        // spill-list bump counters: cursor slots 32..39
constexpr int SPILL_CURSOR_SLOT = 32;
constexpr int BLOCK_BIG_SLOT = 28;     // cursors of the block bins' hub-row launches (28: 256, 29: 1024 threads)
static_assert(SPILL_CURSOR_SLOT * 8 + SPILL_PARTS <= CURSOR_SLOTS * 8, "spill counters fit the cursor area");

// Symbolic bins (by LDS need and tile work).
// Tiny rows: a team of W lanes per row holding K products per lane (flop <= W*K,
// nA <= W), sorted by column in registers -- no table (numeric parks the values in
// LDS by element during the sort).  Classes, smallest first; a row takes the first
// class it fits (tiny_w / tiny_k below).
constexpr int TINY_NC = 6;
constexpr int TINY_EBITS = 9;              // numeric sort key = (column << 9) | element (W*K <= 512)
constexpr int TINY_NUM_NMAX = (1 << 23) - 1;  // ... so a numeric tiny row spans < 2^23 columns (offsets from its first tile)
// Classes of the two phases (measured per phase on delaunay-, GAP-road-, mac_econ-like):
// symbolic (counts only: no segmented sums) sorts every row of at most 8 A entries in
// 8-lane teams -- eight rows per wave, so one dependent load chain (row -> A -> bmeta -> B)
// serves eight rows: (8,1) (8,4) (8,8) (32,4).  Numeric keeps its values beside the keys
// and sums segments per slot, so wide slots cost more: (4,2) (8,4) (16,4) (32,4) (64,4) (64,8).
// Measured per class: numeric class 0 as (4,2) (GAP-road-like -8 %), class 2 as
// (16,4) instead of (32,2) (delaunay-like -12 %); (4,8) for class 1 and (4,2) for symbolic
// class 0 were slower or neutral.
__host__ __device__ constexpr int tiny_w(int c) { return 4 << (c < 4 ? c : 4); }  // 4 8 16 32 64 64
__host__ __device__ constexpr int tiny_k(int c) { return c == 0 ? 2 : c == 5 ? 8 : 4; }
__host__ __device__ constexpr int tiny_ws(int c) { return c <= 2 ? 8 : c == 3 ? 32 : 64; }
__host__ __device__ constexpr int tiny_ks(int c) { return c == 0 ? 1 : (c == 2 || c == 4) ? 8 : 4; }
constexpr int TINY_FUSED_KMAX = 4;  // largest K of the numeric classes 0..3 (one fused launch)
constexpr int TINY_SLOT_MAX = 128;  // value slots of a numeric-first row: W*K of its class (0..3), at most 32*4
// Symbolic uses the classes below TINY_SYM_NC only (past 128 products a hash table
// counts faster than a sort); numeric uses the 64-lane classes for rows whose table
// would not fit the small wave bin (measured: cop20k-like 2.3x slower sorted, while
// rows that need big tables run 2x faster sorted).
constexpr int TINY_SYM_NC = 4;
// ... except scattered rows: symbolic class 4, (64,8), takes rows of at most 512 products that
// the small wave table cannot hold (k_analyze's sym_tiny_class: a hub column's B row in the
// row, web-graph rows), which otherwise count in 10 KiB waves or block tables
constexpr int TINY_SYMX_NC = 5;
constexpr int MHS_SYM_SORT64 = 1;  // symbolic class 4 on (k_analyze, k_sym_common, k_scan)
constexpr int MHS_TINY_NUM_SMALL = 4;
constexpr int TINY_NUM_SMALL = MHS_TINY_NUM_SMALL;  // numeric classes >= this only replace big-table rows
__host__ __device__ inline int tiny_class(int flop, int nA, int nc = TINY_NC) {
    if (flop <= 0) return -1;
    for (int c = 0; c < nc; ++c)
        if (flop <= tiny_w(c) * tiny_k(c) && nA <= tiny_w(c)) return c;
    return -1;
}
__host__ __device__ inline int tiny_class_sym(int flop, int nA) {
    if (flop <= 0) return -1;
    for (int c = 0; c < 4; ++c)
        if (flop <= tiny_ws(c) * tiny_ks(c) && nA <= tiny_ws(c)) return c;
    return -1;
}
enum SymBin : int {
    SYM_NONE = 0, SYM_WAVE = 1, SYM_B256 = 2, SYM_B1024 = 3, SYM_GLOBAL = 4, SYM_TINY = 5,
    SYM_WM = SYM_TINY + TINY_NC,  // wave per row with a 10 KiB table (scattered rows of a few hundred tiles)
    SYM_NB
};
// Numeric bins (by LDS need and product work).
// NUM_WSG / NUM_W16G: row groups (up to RG_MAX consecutive rows of A with one
// column pattern, processed together by one wave: every B value loaded feeds R rows).
enum NumBin : int {
    NUM_NONE = 0, NUM_WS = 1, NUM_W16 = 2, NUM_B256 = 3, NUM_B1024 = 4, NUM_GLOBAL = 5, NUM_WSG = 6,
    NUM_W16G = 7, NUM_TINY = 8,
    NUM_WSH = NUM_TINY + TINY_NC,  // NUM_WS / NUM_W16 rows in hash mode (their own kernels: see MODES)
    NUM_W16H,
    NUM_NB
};
static_assert(NUM_NB + SYM_NB <= BLOCK_BIG_SLOT && BLOCK_BIG_SLOT + 2 <= SPILL_CURSOR_SLOT, "cursor slots do not overlap");
// Row groups: rows i-1, i of A with the same column pattern (FEM dofs of one node)
// have C rows with one pattern.  Maximal runs are broken every RG_BREAK rows and cut
// into groups of at most RG_MAX rows; grp[head] = R, grp[head + o] = GRP_CONT | o.
constexpr int RG_MAX = 3;
constexpr int RG_BREAK = 96;  // a multiple of 2, 3, 4 and 6: dof blocks of those sizes stay whole
constexpr int GRP_CONT = 0x80;
// Near row groups: consecutive rows whose A patterns differ by a few entries (k_bin_list's
// candidates: rows of the small-table wave bin with the same C tile span and first column) and
// whose C patterns turn out equal (k_near, after the symbolic pass counted each row on its
// own).  Their numeric runs as a row group over the union of their A rows (ucol / uval:
// columns once, R values each, 0 where a row lacks the column).  Head: R | GRP_NEAR.
constexpr int GRP_NEAR = 0x40;
constexpr int GRP_RMASK = 0x3F;
constexpr int NEAR_WORDS = 256;   // union rows: A columns within a window of NEAR_WORDS * 64
constexpr int NEAR_UMAX = 128;    // ... and at most this many union entries

// Per-team LDS budgets (bytes).  The wave kernels carve one region per wave.
constexpr int SYM_WAVE_BYTES = 5120;   // 4 waves x 5 KiB: 8 blocks (32 waves, the CU's cap) per CU
constexpr int SYM_WAVE_WORK = 4096;     // tile products a single wave takes on
constexpr int SYM_WM_BYTES = (LDS_MAX_C - 1024) / 16;  // 16 waves of a 1024-thread block (k_sym_rare): 16 waves per CU
constexpr int SYM_B256_BYTES = 32768;
constexpr int SYM_B256_WORK = 1 << 20;
constexpr int NUM_WS_BYTES = 5120;     // 4 waves x 5 KiB = 20 KiB/block: 8 blocks (32 waves) per CU
constexpr int NUM_WS_WORK = 8192;       // products a single wave takes on
// The bigger wave bins: 10 KiB a wave, 4 blocks (16 waves) per CU (round 3: 16 KiB left 2
// blocks per CU; rows past 10 KiB now take the 256-thread block bin -- cage15-like -3 %,
// cant-s1-like -4 %, pdb1HYS-like -4 %, wb-edu-like -3..9 %, others neutral: profiles/r03)
constexpr int NUM_W16_BYTES = 10240;
constexpr int NUM_W16_WORK = 32768;
constexpr int NUM_WSG_BYTES = 10240;   // grouped rows: 4 waves x 10 KiB = 40 KiB/block (4 per CU)
constexpr int NUM_B256_BYTES = 65536;
constexpr int NUM_B256_WORK = 1 << 22;
constexpr int LDS_MAX = 163840;         // gfx950: 160 KiB per workgroup (probed on the box)
constexpr int STAGE_SUBS = 4;           // 256-thread block kernels stage 4 x 64 A entries per barrier
// ... the 1024-thread ones 12 x 64 (hub rows of thousands of short-B-row entries were bound by
// one Acol -> bmeta round trip per 256 entries and barrier)
constexpr int STAGE_SUBS_1024 = 12;
constexpr int BLOCK_HDR = 1024 + STAGE_SUBS * 65 * 16;  // per-block LDS header: reductions, counter, A-entry stage
constexpr int BLOCK_HDR_1024 = 1024 + STAGE_SUBS_1024 * 65 * 16;
__host__ __device__ constexpr int block_hdr(int T) { return T >= 1024 ? BLOCK_HDR_1024 : BLOCK_HDR; }
constexpr int WAVE_HDR = 16;            // per-wave LDS header
constexpr int B1024_BYTES = LDS_MAX - BLOCK_HDR_1024 - 1024;  // budget of the 1024-thread kernels
// Block bins split by LDS need: a launch takes the LDS of its largest row, so one hub row of
// 60 KiB would hold every 12 KiB row of the bin to 2 blocks per CU.  Rows at or below the
// split run in a launch of their own sized to them (4 blocks of 256 / 2 blocks of 1024
// threads per CU), the rest in a second launch beside it.
constexpr int B256_SPLIT = LDS_MAX / 4 - BLOCK_HDR - 2048;
constexpr int B1024_SPLIT = LDS_MAX / 2 - BLOCK_HDR_1024 - 2048;

// One 16-byte tile-table entry: OR of the masks of every B tile that maps to
// this C tile, the C-row rank of its first column, and the key (hash mode).
struct alignas(16) TileEntry {
    unsigned long long mask;
    int base;
    int key;
};

// Device-side statistics read back once per call (the only mid-call sync).
struct Stats {
    unsigned long long flop;       // total products
    long long nnzC;                // total C nnz (scan result)
    int err;                       // error bits (ERR_*)
    int scan_ticket;               // k_scan's dynamic block index (look-back order = dispatch order)
    int sym_count[NBINS];
    int num_count[NBINS];
    int num_global_need;           // max LDS-equivalent bytes of a global numeric row
    int num_block_need[2];         // max LDS bytes of a row in NUM_B256 / NUM_B1024 (launch sizing)
    int num_block_small_need[2];   // ... of the rows at or below BLOCK_SPLIT[bin] (the small launch)
    int num_block_big[2];          // rows above BLOCK_SPLIT[bin] (their own launch when both kinds exist)
    int final_done;                // k_scan_final blocks finished (last one publishes)
    unsigned long long an_slots;   // numeric-first probe: the candidates' slot entries,
    unsigned long long an_other;   // rows with products past the tiny classes,
    int an_done;                   // and k_probe_publish blocks finished
    int near_heads;                // near-group candidates listed by k_bin_list (k_near's work)
    int near_verified;             // ... of which verified (union rows built): B's near union runs
    int nonfinite;                 // the near check met an Inf / NaN in B's values: k_scan dissolves the near groups
    int num_wave_need[2];                // max LDS bytes of a group in NUM_WSG / NUM_W16G (+ WAVE_HDR)
};
// Host-visible copy of Stats (fine-grained pinned memory): the last pre-numeric
// kernel writes it and then `seq`, the host spins on `seq` instead of a stream sync.
struct Published {
    Stats stats;
    int seq;
    int pad[3];
};
// Launch plan speculation (round 6).  Every numeric launch a call makes (which kernels, their
// grids, LDS, C's size, the global-bin scratch, the near copy) is a function of the Stats the
// call's k_scan publishes.  A call on the same operands as the context's previous call
// (same device arrays and sizes) launches the previous call's numeric plan right behind k_scan
// instead of waiting for the hand-off; k_scan's last block compares the call's own Stats with
// the plan's and writes the verdict to `go`, and every numeric kernel of the plan returns at
// once unless go == 1.  The host checks the same comparison on the published Stats and, on a
// mismatch, reruns the call without speculation.  Nothing is skipped or reused on the device:
// every phase runs on every call; only the host's launch decisions are taken ahead of time.
__host__ __device__ inline bool stats_same_plan(const Stats& a, const Stats& b) {
    bool eq = a.flop == b.flop && a.nnzC == b.nnzC && a.num_global_need == b.num_global_need &&
              a.near_heads == b.near_heads && a.near_verified == b.near_verified && a.nonfinite == b.nonfinite;
    for (int i = 0; i < NBINS; ++i) eq = eq && a.sym_count[i] == b.sym_count[i] && a.num_count[i] == b.num_count[i];
    for (int k = 0; k < 2; ++k)
        eq = eq && a.num_block_need[k] == b.num_block_need[k] && a.num_block_small_need[k] == b.num_block_small_need[k] &&
             a.num_block_big[k] == b.num_block_big[k] && a.num_wave_need[k] == b.num_wave_need[k];
    return eq;
}
struct SpecArgs {
    int* go;       // nullptr: the call does not speculate
    Stats expect;  // the plan's Stats
};
constexpr int SAME_PATTERN = 0x40000000;  // bmeta.z flag: B row repeats row-1's columns
// bmeta.w of a verified near group's head (B is A; set by k_scan for the numeric pass, over
// the lo tile only k_analyze reads): NEAR_HEAD | R << 16 | nU -- see finish_chunk
constexpr int NEAR_HEAD = (int)0x80000000;
constexpr int ERR_UNSORTED = 1;
constexpr int ERR_COL_RANGE = 2;
constexpr int ERR_ACOL_RANGE = 4;
constexpr int ERR_OVERFLOW = 8;

__host__ __device__ inline int next_pow2(int x) {
    int p = 1;
    while (p < x) p <<= 1;
    return p;
}
__host__ __device__ inline int ilog2(int x) {  // x power of two
    int l = 0;
    while ((1 << l) < x) ++l;
    return l;
}
// Open-addressed table size for up to `bound` distinct keys: load <= 2/3, rounded to
// 16 slots, not to a power of two (slots come from a multiply-high range reduction):
// linear probing stays short, and a tighter table lets more rows share a CU's LDS --
// the small-row phases are bound by rows in flight, not by probes.
__host__ __device__ inline int hash_slots(int bound) {
    const int b = bound < 1 ? 1 : bound;
    return (b + ((b + 1) >> 1) + 15) & ~15;  // >= ceil(1.5 b) > b: an insert always finds a slot
}
// the power-of-two sizing the direct/hash choice of symbolic was tuned with
__host__ __device__ inline int hash_slots_pow2(int bound) {
    const int b = bound < 1 ? 1 : bound;
    const int h = next_pow2(b + (b >> 1) + 1);
    return h < 16 ? 16 : h;
}
__host__ __device__ inline long long align16(long long x) { return (x + 15) & ~15LL; }

// Symbolic tile table: direct-mapped over the row's tile span (no keys, no CAS) when
// the span is not much wider than the table a hash would need and the direct table
// does not push the row into a bigger bin than the hash would; else hashed.
__host__ __device__ inline bool sym_direct(int span, int tflop) {
    const int bound = tflop < span ? tflop : span;
    const int h = hash_slots_pow2(bound);
    return span <= 2 * h && (span <= h || (long long)span * 16 <= 4096);
}
__host__ __device__ inline long long sym_need(int span, int tflop) {
    int bound = tflop < span ? tflop : span;
    // symbolic tables: masks (8 B a slot), plus keys (4 B) when hashed -- see sym_row
    return sym_direct(span, tflop) ? align16((long long)span * 8) : align16((long long)hash_slots(bound) * 12);
}
// Numeric row modes:
//   NM_DENSE  narrow tile span: a dense accumulator over the span's columns
//             (span*64 doubles) -- a product is one ds_add_f64 at (col - base),
//             the rank compaction happens once per C entry at output time;
//   NM_DIRECT tile table direct-mapped over the span + rank-compressed accumulator
//             (n doubles): a product lands at base(tile) + popc(mask & below(col));
//   NM_HASH   scattered rows: hashed tile table + rank-compressed accumulator
//             (tiles sorted by key to assign bases).
// (A column -> rank map over the span, a uint16 per column, measured 25 % slower than
// NM_DIRECT on cant-like: dropped.)
enum NumMode : int { NM_DENSE = 0, NM_DIRECT = 1, NM_HASH = 2 };
constexpr int MCACHE_SPAN = 32;   // rows spanning <= 32 tiles: symbolic keeps their tile masks
__host__ __device__ inline long long num_need_dense(int span) { return (long long)span * (16 + 64 * 8); }
__host__ __device__ inline long long num_need_direct(int span, int n) {
    return (long long)span * 16 + align16((long long)n * 8);
}
// Hash rows rank their tiles by counting smaller keys when t <= HASH_CNT_T (t^2/64 compares
// per wave, no sort buffer); bigger tables are bitonic-sorted in a next_pow2(t) buffer
// that shares the accumulator region.
constexpr int HASH_CNT_T = 192;
__host__ __device__ inline int hash_sort_p(int t) { return t <= HASH_CNT_T ? 0 : next_pow2(t); }
__host__ __device__ inline long long num_need_hash(int t, int n) {
    const int h = hash_slots(t);
    const int p = hash_sort_p(t);
    return (long long)h * 16 + align16((long long)(n > p ? n : p) * 8);
}
// symbolic stores the OR'd tile masks of rows it tabled direct-mapped over a narrow span
__host__ __device__ inline bool mcached(int span, int tflop) { return span <= MCACHE_SPAN && sym_direct(span, tflop); }
// ... and of the other rows with at most `list` distinct tiles (a run-time cap, MC_LIST_MAX
// unless M rows of that would not fit MC_BYTES_MAX), an unordered compact list in the
// row's slot of mc_stride(list) words: masks at [0, list), tile keys (int32) after them.
// Numeric then skips the tile walk (and, hashed, the table compaction).
constexpr int MC_LIST_MIN = 16;
constexpr int MC_LIST_MAX = 128;
constexpr long long MC_BYTES_MAX = 12LL << 30;
__host__ __device__ inline int mc_stride(int list) {
    const int w = list + (list + 1) / 2;
    return w > MCACHE_SPAN ? w : MCACHE_SPAN;
}
inline int mc_list_for(long long M) {
    return M * mc_stride(MC_LIST_MAX) * 8 <= MC_BYTES_MAX ? MC_LIST_MAX : MC_LIST_MIN;
}
static_assert(MC_LIST_MIN * 12 <= MCACHE_SPAN * 8, "the smallest tile list fits the narrow rows' slot");
__host__ __device__ inline bool mlisted(int span, int tflop, int t, int list) {
    return !mcached(span, tflop) && t <= list;
}
__host__ __device__ inline int num_mode(int span, int t, int n, int dense_span_max) {
    if (span <= dense_span_max) return NM_DENSE;
    // direct-mapped (no probes, no tile sort) unless it needs more LDS than a hash table
    // at load 1/2 would: the tighter hash sizing only shrinks the rows that hash anyway
    const long long hash_half = (long long)next_pow2(2 * (t < 1 ? 1 : t)) * 16 +
                                align16((long long)(n > next_pow2(t) ? n : next_pow2(t)) * 8);
    // (round 5: direct-mapped whenever both fit the small wave bin measured neutral on cop20k-like)
    return num_need_direct(span, n) <= hash_half ? NM_DIRECT : NM_HASH;
}
// Wide rows: hash-mode rows whose table would not fit the 256-thread kernel's 64 KiB run
// in the 1024-thread kernel with windowed dense masks and global accumulation (measured:
// for smaller tables the hash kernels' occupancy wins).
__host__ __device__ inline bool num_wide(int span, int t, int n, int dense_span_max);
__host__ __device__ inline long long num_need(int span, int t, int n, int dense_span_max) {
    const int m = num_mode(span, t, n, dense_span_max);
    return m == NM_DENSE ? num_need_dense(span) : m == NM_DIRECT ? num_need_direct(span, n) : num_need_hash(t, n);
}
// Hub rows past the 256-thread hash budget rank their tiles by a span bitmap.
// Span-bitmap rows (num_row_bitmap): span/64 * 12 bytes + 16 per tile + 8 per C entry.
__host__ __device__ inline long long num_need_ranked(int span, int t, int n) {
    const long long nw = ((long long)span + 63) >> 6;
    return align16(nw * 8) + align16(nw * 4) + 2 * align16((long long)t * 8) + align16((long long)n * 8);
}
__host__ __device__ inline bool num_big_hash(int span, int t, int n, int dense_span_max) {
    return num_mode(span, t, n, dense_span_max) == NM_HASH && num_need_hash(t, n) > NUM_B256_BYTES - BLOCK_HDR;
}
__host__ __device__ inline bool num_ranked(int span, int t, int n, int dense_span_max) {
    return num_big_hash(span, t, n, dense_span_max) && num_need_ranked(span, t, n) <= B1024_BYTES;
}
__host__ __device__ inline bool num_wide(int span, int t, int n, int dense_span_max) {
    return num_big_hash(span, t, n, dense_span_max) && !num_ranked(span, t, n, dense_span_max);
}
// One row's accumulator bytes in mode m (16-aligned); a group of R rows needs the
// tables once and R accumulators.
__host__ __device__ inline long long num_acc_bytes(int m, int span, int t, int n) {
    if (m == NM_DENSE) return (long long)span * 64 * 8;
    if (m == NM_HASH) {
        const int p = hash_sort_p(t);
        return align16((long long)(n > p ? n : p) * 8);
    }
    return align16((long long)n * 8);
}
__host__ __device__ inline long long num_need_rows(int span, int t, int n, int dense_span_max, int R) {
    const int m = num_mode(span, t, n, dense_span_max);
    return num_need(span, t, n, dense_span_max) + (long long)(R - 1) * num_acc_bytes(m, span, t, n);
}

// ------------------------------------------------------------ launchers ---
struct Csr {
    int M, N, nnz;
    const int* ptr;
    const int* col;
    const double* val;
};

struct SpillLists;  // (mhs_kernels.hip) symbolic's tile lists of rows past the row-cache cap
struct SpillArea {
    unsigned long long* mask;
    int* key;
    int* lofs;
    int* top;
    long long cap;
};
// entries of the spill region: one per B nonzero (at least 1 M, at most 64 M = 768 MB)
inline long long spill_cap(long long nnzB) {
    const long long c = nnzB < (1LL << 20) ? (1LL << 20) : nnzB;
    return c > (1LL << 26) ? (1LL << 26) : c;
}

struct Work {
    // B side
    int* btcol;
    unsigned long long* btmask;
    int4* bmeta;
    int* bhi;
    // C side
    int* rflop;
    int* rtflop;
    int* rlo;
    int* rhi;
    int* ctiles;
    unsigned char* sym_bin;  // M: symbolic bin of every row (k_analyze)
    unsigned char* asame;    // M: row has the column pattern of row-1 (k_analyze)
    unsigned char* grp;      // M: row groups (k_bin_list; see RG_MAX)
    int groups;              // form row groups (0: every row alone)
    // near row groups (GRP_NEAR; nullptr: off): candidate list (head * 4 + R), union rows
    // at the head's A offset (ucol: nnz(A) ints; uval: 3 nnz(A) doubles, values of row r at
    // 3 * Aptr[head] + r * nU), union length per head
    int* near_list;
    unsigned* nsig;  // M: k_analyze's near-link signature of every row
    int* ucol;
    double* uval;
    int* gna;
    int near_b;      // B is A with near groups planned: k_scan marks the verified heads in bmeta
    // B's arrays extended by the near union rows (nnzB + 3 nnzA entries; uval = bx_val + nnzB,
    // ucolx = bx_col + nnzB): the numeric value walks read them when bx_on (B is A, groups verified)
    int* bx_col;
    double* bx_val;
    int* ucolx;
    int bx_on;
    const double* vcheck;    // B's values, checked for Inf / NaN by the near check (near groups planned)
    long long vcheck_n;
    int tiny_num;            // numeric tiny classes allowed (per row: column span <= TINY_NUM_NMAX + 1)
    // numeric-first tiny rows (big M): the symbolic tiny launch sorts them once, in the
    // numeric classes, and sums their values into slots (sc_*); numeric only copies them
    // into C.  nft_bin (M, the probe): k_analyze also bins every row that way and counts
    // the candidates; the host then picks the bin lists (nft: numeric-first, with slots).
    unsigned char* nft_bin;
    int nft;
    long long* tslot;        // M: a slot row's first entry
    int* sc_col;
    double* sc_val;
    int* bin_list;           // (NUM_NB-1) * M: bin x's rows at (x-1)*M (symbolic bins, then numeric bins)
    int* split_list;         // M: the block bins' rows split by LDS need (k_split_bins): B1024's, then B256's
    unsigned long long* blkflop;  // per-block flop partials of k_analyze
    int nflop;                    // their count
    int* scan_part;    // k_scan's look-back state: one 64-bit word per block (flag | prefix)
    int* cursors;      // CURSOR_INTS row cursors (after the look-back words), then BINCNT_INTS bin counters
    unsigned long long* mcache;   // [M][mc_stride] tile masks / tile lists (symbolic -> numeric)
    int mc_list;                  // list cap (see mlisted)
    SpillArea spill;              // tile lists of rows past mc_list (symbolic -> numeric)
    Stats* stats;
    void* gscratch;    // global-bin scratch
    size_t gscratch_bytes;
    const int* go;     // speculated numeric launches: run only when *go == 1 (k_scan's verdict); nullptr: always
    int sym_big;       // the numeric-first probe counted >= 2^21 rows past the tiny classes: big symbolic wave grid
};

void launch_mask_b(const Csr& B, const Work& w, hipStream_t s);
// Row analysis, then the symbolic bin lists -- or, with w.nft_bin (the numeric-first
// probe), the candidate counts published as `seq` (the host then calls launch_bin_list)
void launch_analyze(const Csr& A, const Work& w, int MB, hipStream_t s, int* Cptr, Published* pub = nullptr,
                    int seq = 0);
void launch_bin_list(const Csr& A, const Work& w, hipStream_t s);

int analyze_blocks(long long nnzA, int M);

void launch_symbolic_common(const Csr& A, const Csr& B, const Work& w, int M, int N, int* Cptr, hipStream_t s,
                            const Stats* plan = nullptr);
// with_near: its phase 0 checks the near row-group candidates (after k_sym_common on the
// same stream); else launch_near does, once both symbolic launches are done
void launch_symbolic_rare(const Csr& A, const Work& w, int M, int N, int* Cptr, hipStream_t s, bool with_near);
void launch_symbolic_b256(const Csr& A, const Work& w, int M, int N, int* Cptr, hipStream_t s);
// near row groups: verify k_bin_list's candidates after the symbolic pass, build union rows
void launch_near(const Csr& A, const Work& w, const int* Cptr, hipStream_t s);
void launch_scan_classify(int M, const Work& w, int* Cptr, const int* Aptr, hipStream_t s, int dense_span_max,
                          Published* pub, int seq, const SpecArgs& spec);
// fork: called once before the first launch on an aux stream (the aux streams' waits on the
// fork event; the first launch goes out on ss[0] before it); false: the waits failed, every
// later launch goes to ss[0].  ev_start / ev_stop (optional): timing events carried by the first and
// last dispatch of a single-stream phase; bit 30 of the result: not attached (several streams or
// no launch) -- the caller records them
int launch_numeric(const Csr& A, const Csr& B, const Work& w, const Stats& h, int* Cptr,
                   int* Ccol, double* Cval, const hipStream_t* ss, int nss, int global_grid, int dense_span_max,
                   bool split, hipEvent_t split_ev = nullptr, const std::function<bool()>& fork = nullptr,
                   hipEvent_t ev_start = nullptr, hipEvent_t ev_stop = nullptr, int only = ~0);
// numeric launches a call makes for these bin counts (the 32-lane tiny classes share one; a
// split block bin makes two)
int numeric_launches(const Stats& h);
// Block bins holding rows on both sides of their LDS split: partition their lists into
// w.split_list (small rows first, hub rows last) on `s`.  False when no bin splits.
bool launch_split_bins(const Work& w, const Stats& h, int M, const int* Cptr, hipStream_t s, int dense_span_max);
size_t sym_global_bytes_per_block(int N);
// p[0..n) += off (row-chunked products: a chunk's row_ptr rebased to its place in C)
void launch_add_offset(int* p, int n, int off, hipStream_t s);
// Device CSR transpose (AAT operand): tmp == nullptr -> *tmp_bytes = scratch size.
hipError_t transpose_csr(const Csr& A, int* tptr, int* tcol, double* tval, void* tmp, size_t* tmp_bytes,
                         hipStream_t s);
hipError_t init_kernel_attributes();
// device address of the probe-conflict counter (nullptr unless built with MHS_PROBE_STATS=1)
hipError_t probe_counter(unsigned long long** dev);
// mhs_hbm.hip: the streaming kernels of mhs_hbm_peak on the current device (gbps[3]: copy, read, write)
hipError_t hbm_peak_run(size_t bytes, int iters, double* gbps);

}  // namespace mhs
