// mhs_kernels.hip -- gfx950 (MI355X, CDNA4) kernels of the mask-and-hash SpGEMM.
//
// Phases (reference call path src/main.cu:12-72, inc/MH_spgemm.cuh):
//   k_mask_b          Form_mask_matrix_B (MH_spgemm.cuh:242-295, Form_mask_matrix_B.cuh):
//                     every B row -> (64-column tile, 64-bit mask) pairs.  Columns are
//                     sorted, so a tile is a run of equal col>>6 found with one wave
//                     ballot + a segmented OR scan per 64 entries: no hash, one pass,
//                     written in place of the row's own CSR slots (no scan, no malloc).
//   k_analyze         flop / tile-flop / tile span per A row (k_calculate_flop,
//                     Form_mask_matrix_B.cuh:14-95) + symbolic bin id.
//   k_bin_*           stable row binning (binning.cuh:67-155) without host round trips.
//   k_sym_*           Calculate_C_nnz (MH_spgemm.cuh:297-362, Calculate_C_nnz.cuh):
//                     OR the B tile masks of a C row into an LDS tile table (direct-
//                     mapped over the row's tile span, or open-addressed), nnz = sum popc.
//   k_scan_*          row_ptr exclusive scan (CUB ExclusiveSum, src/main.cu:55) fused
//                     with the numeric bin classification.
//   k_num_*           h_numeric (MH_spgemm.cuh:364-430, numeric.cuh): rebuild the C
//                     row's tile table, give every tile the C-row rank of its first
//                     column (prefix popcount in tile order), then every product
//                     lands at base + popc(mask & below(col)) in a dense LDS
//                     accumulator: no key CAS per product and no sort of the output,
//                     columns come out ordered by construction.
//
// Every phase is binned by row size into wave-per-row kernels (one LDS region per
// wave, no block barriers), block-per-row kernels (256 / 1024 threads, up to 160 KiB
// of LDS) and a global-memory fallback; rows are walked in XCD-grouped order so that
// neighbouring rows (which share B rows) run on one XCD's L2.
#include "mhs_internal.hpp"

#include <hip/hip_ext.h>

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <functional>
#include <type_traits>
#include <vector>

#ifndef MHS_ROW_STAMPS
#define MHS_ROW_STAMPS 0  // 1: tools/diag/stamps*.py builds -- per-row, per-phase s_memtime cycles
#endif
constexpr int MHS_RUN_MAX = 3;  // longest run a value walk merges into one accumulate (1..4)
constexpr int MHS_RUN_UNROLL = 2;  // B entries per lane issued together in a run walk (registers: occupancy)
constexpr int MHS_TILE_UNROLL = 2;  // tiles per lane issued together in a tile walk
constexpr int MHS_UNROLL = 4;  // B entries per lane issued together in the product walk
constexpr int MHS_UNROLL_BLOCK = 8;  // ... in the block kernels (measured: S1-like rows -9%; the wave kernels keep 4)
constexpr int MHS_NUM_WS_GRID = 4096;  // block cap of the small-row grouped numeric launch
constexpr int MHS_TINY64_GRID = 4096;  // block cap of the 64-lane tiny numeric launches (8192: wb-edu-like +6 %)
constexpr int MHS_NUM_W16H_GRID = 2048;  // block cap of the 10 KiB hash launch (4096: neutral at 16 KiB, profiles/r02za2_grid)
// block cap of each numeric-first symbolic tiny class: 4096, 16384 from 4 M rows (r05ab17/18:
// delaunay-like 10.26 -> 9.70 ms, GAP-road-like 4.53 -> 4.43 at 16384, but mac_econ-, scircuit-like
// +5-6 %; 512-2048 slower on every huge matrix, delaunay-like up to 19 ms)
constexpr int MHS_COPY_CAP_BIG = 65536;  // the slot copy's block cap from 4 M rows (16384 below; delaunay-like -1 %, r05ab19)
constexpr int MHS_NFT_GRID = 4096, MHS_NFT_GRID_BIG = 16384, MHS_NFT_BIG_M = 1 << 22;
constexpr int MHS_TINY_PF = 1;  // tiny teams load their next row a round ahead (GAP-road-like -3 %, mac_econ-, scircuit-like -1 %)
constexpr int MHS_SYM_WAVE_GRID = 2048;  // block cap of k_sym_common's wave rows (65536: cage15-like -3 %, cop20k-, webbase-, mac_econ-like +5 %)
constexpr int MHS_SYM_WAVE_GRID_BIG = 65536;  // ... when the probe counted >= 2^21 table rows (Work::sym_big)
constexpr int MHS_NUM_WSH_BIG = (1 << 21);  // small hash bins of at least this many rows: block cap MHS_NUM_WSH_BIG_GRID
constexpr int MHS_NUM_WSH_BIG_GRID = 65536;  // (cage15-like -2.5 % over 16384; 65536 for every bin: offshore-, webbase-like +1.5 %)
constexpr int MHS_NUM_WSX_GRID = 16384;  // ... of the small-row hash / direct launches (8192: cage15-like numeric +4.5 %, 4096: +13 %,
                                         // cant-perturbed +5 %; the grouped launch: 8192 measured +1.4 % on cant-like)
constexpr int MHS_VAL_GMIN = 4;  // narrowest lane group of a value walk
constexpr int MHS_TILE_GMIN = 4;  // narrowest lane group of a tile walk
constexpr int MHS_RUN_GMIN = 8;  // narrowest lane group of a chunk with merged runs (32 before: see DESIGN §8)
constexpr int MHS_MASK_GMAX = 64;
constexpr int MHS_AN_GMAX = 8;  // k_analyze: 8 lanes per row (several rows per wave overlap their load chains)
constexpr int MHS_GRP_UNROLL = 3;  // entries per lane issued together in a row-group walk
// Occupancy targets (waves per SIMD; 0 = the compiler's choice).  The wave kernels are
// bound by per-row latency chains, so waves in flight matter more than a few spills.
constexpr int MHS_WPE_HASH = 8;  // measured: cop20k-like numeric -18%, cage15-like -16% (vs the compiler's 6)
constexpr int MHS_SYM_B256_GRID = 1024;  // block cap of the persistent 256-thread symbolic bin launch
constexpr int MHS_WPE_HASH16 = 4;  // the 10 KiB hash bin: LDS allows 4 waves per SIMD (an 8-wave register target spilled 34 VGPRs for nothing)
// (the generic / grouped wave numeric kernel: no occupancy floor -- the compiler's choice; a
// 5-wave floor at 96 VGPRs measured slower)
constexpr int MHS_WPE_DIRECT = 0;
constexpr int MHS_WPE_TINY = 0;
#define MHS_WPE_ATTR(n) __attribute__((amdgpu_waves_per_eu((n) > 0 ? (n) : 1)))
constexpr int MHS_WPE_SYM = 8;  // symbolic wave + tiny kernels: cant-like -12%, cop20k-like -22%
#if MHS_ROW_STAMPS  // diagnostic build: per-row, per-phase s_memtime cycles (plain stores)
__device__ unsigned long long* g_rowdiag;  // [M][8]
#define MHS_STAMP0() unsigned long long tp_ = __builtin_amdgcn_s_memtime()
#define MHS_STAMP(k)                                                    \
    do {                                                                \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();    \
        if (tm.rank() == 0) g_rowdiag[(size_t)row * 8 + (k)] = t_ - tp_; \
        tp_ = t_;                                                       \
        MHS_FLIGHT_PHASE(k);                                            \
    } while (0)
#ifndef MHS_FLIGHT
#define MHS_FLIGHT 1  // the flight recorder in stamps builds (0: compiled out)
#endif
// Flight recorder (stamps builds, round 6): every wave of the numeric wave kernels writes, to
// fine-grained host memory, the row it is on, its list index, the last phase stamp it passed
// and a tick.  The host reads it while the kernels run (tools/diag/flight.py): a wave that
// never finishes shows where it is.  Plain system-scope vector stores; off unless set up.
__device__ unsigned long long* g_flight;  // [wave][4]: row | li << 32, phase, tick, calls
extern "C" int mhs_diag_flight(void* dev_ptr) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_flight), &dev_ptr, sizeof(void*));
}
__device__ __forceinline__ void flight_put(int slot, unsigned long long v) {
    if (!MHS_FLIGHT) return;
    unsigned long long* f = g_flight;
    if (!f) return;
    const long long w = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (w < 65536 && (threadIdx.x & 63) == 0)
        __hip_atomic_store(f + w * 4 + slot, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
#define MHS_FLIGHT_PHASE(k) flight_put(1, (unsigned long long)(k) + 1)
#define MHS_FLIGHT_TAKE(li) flight_put(3, (unsigned long long)(unsigned)(li))
#define MHS_FLIGHT_ROW(row, li)                                                      \
    do {                                                                             \
        flight_put(0, (unsigned long long)(unsigned)(row) | ((unsigned long long)(unsigned)(li) << 32)); \
        flight_put(1, 0ull);                                                         \
        flight_put(2, __builtin_amdgcn_s_memtime());                                 \
    } while (0)
extern "C" int mhs_diag_setup(int M, unsigned long long** dev) {
    hipError_t e = hipMalloc((void**)dev, (size_t)M * 64);
    if (e == hipSuccess) e = hipMemset(*dev, 0, (size_t)M * 64);
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_rowdiag), dev, sizeof(void*));
    return (int)e;
}
// the row stamps into a caller's buffer (e.g. fine-grained host memory, read while a kernel runs)
extern "C" int mhs_diag_set_rows(void* dev_ptr) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_rowdiag), &dev_ptr, sizeof(void*));
}
// symbolic rows (sym_row_s): [M][4] phases -- clear, tile walk, count, row cache / spill list
__device__ unsigned long long* g_symdiag;
extern "C" int mhs_diag_setup_sym(int M, unsigned long long** dev) {
    hipError_t e = hipMalloc((void**)dev, (size_t)M * 32);
    if (e == hipSuccess) e = hipMemset(*dev, 0, (size_t)M * 32);
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_symdiag), dev, sizeof(void*));
    return (int)e;
}
#define MHS_SSTAMP0() unsigned long long tps_ = __builtin_amdgcn_s_memtime()
#define MHS_SSTAMP(k)                                                     \
    do {                                                                  \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();      \
        if (tm.rank() == 0 && g_symdiag) g_symdiag[(size_t)row * 4 + (k)] = t_ - tps_; \
        tps_ = t_;                                                        \
    } while (0)
#else
#define MHS_STAMP0()
#define MHS_STAMP(k)
#define MHS_SSTAMP0()
#define MHS_SSTAMP(k)
#define MHS_FLIGHT_ROW(row, li)
#define MHS_FLIGHT_TAKE(li)
#endif
// (bisecting the round-4/5 stamps hang on cage15-like: MHS_STAMP_NUM_BODY=0 keeps the stamps out
// of num_row_body, the wave and 256-thread rows)
#if MHS_ROW_STAMPS && defined(MHS_STAMP_NUM_BODY) && !MHS_STAMP_NUM_BODY
#define MHS_BSTAMP0()
#define MHS_BSTAMP(k)
#else
#define MHS_BSTAMP0() MHS_STAMP0()
#define MHS_BSTAMP(k) MHS_STAMP(k)
#endif
// Probe guard (diagnostic builds; on with the stamps): a hash probe loop that has visited every
// slot of its table records where, the key and the table size, and stops -- a key missing from
// its table would otherwise spin forever (the round-4 stamps run on cage15-like never returned)
#ifndef MHS_PROBE_GUARD
#define MHS_PROBE_GUARD MHS_ROW_STAMPS
#endif
#if MHS_PROBE_GUARD
__device__ unsigned long long g_guard[8];  // trips, then the first trip: where, key, H, steps
__device__ bool probe_guard(int steps, int H, int where, int key) {
    if (steps <= H) return false;
    if (atomicAdd(&g_guard[0], 1ull) == 0ull) {
        g_guard[1] = (unsigned long long)where;
        g_guard[2] = (unsigned long long)(unsigned)key;
        g_guard[3] = (unsigned long long)H;
    }
    return true;
}
extern "C" int mhs_diag_guard(unsigned long long* out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_guard), sizeof(g_guard));
}
#define MHS_GUARD_DECL int guard_steps_ = 0
#define MHS_GUARD(H, where, key) \
    if (probe_guard(++guard_steps_, (H), (where), (key))) break
#else
#define MHS_GUARD_DECL
#define MHS_GUARD(H, where, key)
#endif

// k_scan / k_bin_list phase stamps (diagnostic builds, -DMHS_SCAN_STAMPS=1; tools/diag/scan_stamps.py):
// thread 0 of every block writes s_memtime at each phase boundary -- [block][16]: k_scan 0..7,
// k_bin_list 8..11
#ifndef MHS_SCAN_STAMPS
#define MHS_SCAN_STAMPS 0
#endif
#if MHS_SCAN_STAMPS
__device__ unsigned long long* g_scandiag;
extern "C" int mhs_diag_setup_scan(int nblocks, unsigned long long** dev) {
    hipError_t e = hipMalloc((void**)dev, (size_t)nblocks * 128);
    if (e == hipSuccess) e = hipMemset(*dev, 0, (size_t)nblocks * 128);
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_scandiag), dev, sizeof(void*));
    return (int)e;
}
#define MHS_SCSTAMP(b, k) \
    do { if (threadIdx.x == 0 && g_scandiag) g_scandiag[(size_t)(b) * 16 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define MHS_SCSTAMP(b, k)
#endif

namespace mhs {

// ------------------------------------------------------------------ helpers ---

constexpr int MHS_TINY_DUP = 2;  // ... and at most this many products a C column
constexpr int MHS_TINY_SPARSE_PCT = 50;  // class-4 rows with tiles >= this % of their C columns go to the sort class (0: off)
constexpr int MHS_LANE_AVG = 9;  // k_mask_b / k_analyze: a lane per row below this many entries a row on average (0: off)
__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Ordering point for LDS traffic between lanes of ONE wave: a wave's LDS
// operations are performed in issue order, so only the compiler must be kept
// from moving accesses across this point.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
    return v;
}

template <class V>
__device__ __forceinline__ V wave_sum(V v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    return v;
}

__device__ __forceinline__ int wave_incl_scan(int x) {
    const int lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        int y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    return x;
}

__device__ __forceinline__ long long wave_incl_scan64(long long x) {
    const int lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        long long y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    return x;
}

// threadIdx.x from the wave's index (an SGPR) and the lane: the fused multi-role kernels
// otherwise keep v0 (the work-item id) live throughout, and at 64 VGPRs spill it
__device__ __forceinline__ int thread_x() {
    return (__builtin_amdgcn_readfirstlane((int)threadIdx.x) & ~63) + lane_id();
}
// (an opaque lane id: recomputed where used -- hoisted, the mask held two VGPRs across
// whole kernels, and the 64-VGPR kernels spilled it to scratch)
__device__ __forceinline__ unsigned long long lanemask_lt() {
    int lane = lane_id();
    asm volatile("" : "+v"(lane));
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// Opt-in probe statistics (the reference's HASH_CONFLICT, inc/common.h:18, printed at
// src/main.cu:68-71): a build with MHS_PROBE_STATS=1 counts every probe step that met
// another key -- symbolic inserts, numeric table builds and numeric lookups -- in one
// device counter read back by mhs_probe_count().  Off (and free) in the product build.
#ifndef MHS_PROBE_STATS
#define MHS_PROBE_STATS 0
#endif
#if MHS_PROBE_STATS
__device__ unsigned long long g_probe_conflicts;
#endif
__device__ __forceinline__ void probe_conflict() {
#if MHS_PROBE_STATS
    atomicAdd(&g_probe_conflicts, 1ull);
#endif
}

// Fibonacci hash of a tile key into [0, H) (any H: multiply-high range reduction)
__device__ __forceinline__ int hslot(int key, int H) {
    return (int)__umulhi((unsigned)key * 2654435769u, (unsigned)H);
}
__device__ __forceinline__ int hnext(int s, int H) { return s + 1 < H ? s + 1 : 0; }

__device__ __forceinline__ int sat_int(long long x) { return x > INT_MAX ? INT_MAX : (int)x; }
__device__ __forceinline__ int hi_lo_span(int lo, int hi) { return hi - lo + 1; }

// Streaming stores (C): each byte is written once, so they bypass L2 allocation
// (nontemporal) and leave the XCD's 4 MiB to the B rows that neighbouring C rows share.
// Measured and dropped: stores that drop their line from L2 (`sc1`), and
// nontemporal row-cache / partial-line traffic.
template <class T>
__device__ __forceinline__ void st_stream(T* p, T v) {
    __builtin_nontemporal_store(v, p);
}
// Stores that leave partial cache lines (a tile's set bits, a tiny row's segment ends) stay
// cached: L2 merges them into whole lines; nontemporal they reach HBM as masked partial
// writes (measured: WRITE_SIZE 1.32x C's bytes on cant-like).
template <class T>
__device__ __forceinline__ void st_part(T* p, T v) {
    *p = v;
}
// The symbolic -> numeric row cache: plain (cached) stores and loads (measured: nontemporal
// made cage15-like symbolic +3.5 %, cop20k-like numeric +4 %)
template <class T>
__device__ __forceinline__ void st_cache(T* p, T v) {
    *p = v;
}
template <class T>
__device__ __forceinline__ T ld_cache(const T* p) {
    return *p;
}

// Two consecutive entries in one load (8-byte aligned doubles, 4-byte aligned ints: gfx950 loads
// them unaligned as one global_load_dwordx4 / _dwordx2)
typedef double d2u __attribute__((ext_vector_type(2), aligned(8)));
typedef int i2u __attribute__((ext_vector_type(2), aligned(4)));
typedef int i4u __attribute__((ext_vector_type(4), aligned(4)));
typedef int i4a __attribute__((ext_vector_type(4), aligned(16)));
// Lane-group width for walking the products of one row: groups of G lanes
// take one A entry each and stride its B row.  Pick G minimising the sweeps
// ceil(nA / groups) * ceil(avg B-row length / G) (ties -> wider, better
// coalesced groups); at most 64 groups so one staged chunk of 64 A entries
// feeds every group.
__device__ __forceinline__ int pick_group(long long work, int nA, int T, int gfloor = 4, int unroll = 1) {
    int gmin = T / 64;
    if (gmin < gfloor) gmin = gfloor;
    if (nA <= 0) return gmin;
    const long long avg = (work + nA - 1) / nA;
    const int U = unroll;
    int best = gmin;
    long long bc = LLONG_MAX;
    for (int g = gmin; g <= T; g <<= 1) {
        const int ng = T / g;
        // sweeps = A entries per group x load batches per entry (a batch: U entries per lane,
        // issued together -- one dependent round trip)
        const long long c = (long long)((nA + ng - 1) / ng) * ((avg + (long long)g * U - 1) / ((long long)g * U));
        if (c <= bc) {
            bc = c;
            best = g;
        }
    }
    return best;
}

// bmeta.z = tile count | SAME_PATTERN (row has the column pattern of row-1).
__device__ __forceinline__ int meta_ntiles(const int4& m) { return m.z & ~SAME_PATTERN; }
// a verified near group's head (B is A; k_scan sets it for the numeric pass, over the lo tile
// that only k_analyze reads): bmeta.w = NEAR_HEAD | R << 16 | nU
__device__ __forceinline__ bool meta_near(const int4& m) { return m.w < 0; }
__device__ __forceinline__ int meta_near_r(const int4& m) { return (m.w >> 16) & 3; }
__device__ __forceinline__ int meta_near_n(const int4& m) { return m.w & 0xFFFF; }
__device__ __forceinline__ bool meta_same(const int4& m) { return (m.z & SAME_PATTERN) != 0; }
// Runs.  A entry j continues a run when Acol[j] = Acol[j-1] + 1 and B row Acol[j]
// has the column pattern of B row Acol[j]-1 (bmeta SAME_PATTERN, e.g. the dofs of
// one FEM node).  The rows of a run are consecutive in B's CSR and equally long, so
// B row k+i starts at s + i*n.  A tile walk visits only the head of each run (the
// tile masks are the same; OR is idempotent); a value walk visits heads of runs cut
// every MHS_RUN_MAX entries and sums a_i * b_i over the run before one accumulate.
struct StagedChunk {
    int st, ln, L;  // this lane's entry: B segment start, length, run length (heads)
    double av;
    int src;        // compacted visit list: src of visit e is in lane e
    int nh, lmax;   // visits in the chunk, longest run (wave-uniform)
};

// Lanes hold the chunk entries [jb, jb+64) ∩ [.., a1) of one A row (lane 0 = jb).
// Staging is split in its loads (ChunkLoads: A.col, the previous A.col, A.val, then
// bmeta of the column) and the ballots that turn them into visits (finish_chunk), so a
// walk can issue the loads of its next chunk before it walks the current one.  Loads are
// issued together (kprev clamped, not branched on) and every lane reaches the ballots.
struct ChunkLoads {
    int k, kp;
    int4 m;
    double av;
    bool in;
};
__device__ __forceinline__ ChunkLoads load_chunk_a(int lane, int jb, int a1, const int* __restrict__ Acol,
                                                   const double* __restrict__ Aval) {
    ChunkLoads c;
    const int jl = jb + lane;
    c.in = jl < a1;
    c.k = 0;
    c.kp = 0;
    c.av = 0.0;
    c.m = make_int4(0, 0, 0, 0);
    if (c.in) {
        c.k = Acol[jl];
        c.kp = Acol[jl > 0 ? jl - 1 : 0];
        if (Aval) c.av = Aval[jl];
    }
    return c;
}
__device__ __forceinline__ void load_chunk_meta(ChunkLoads& c, const int4* __restrict__ bmeta) {
    if (c.in) c.m = bmeta[c.k];
}
// Near union runs (value walks, A*A with verified near row groups): B rows k0 .. k0+R-1 of a
// near group have patterns that differ by a few entries, so they form no SAME_PATTERN run;
// where the A row holds all R of them (consecutive lanes k0, k0+1, ..), the visit walks the
// group's union row instead, as one run of R: the value arrays are then B's extended by the
// union rows (columns at ubase + 3u, row i's values at ubase + 3u + i*nU, 0 where row k0+i
// lacks the column; u = the group head's row start, B being A).  Every union column is in
// this C row, as all R rows are in its A row.  A group head's bmeta carries NEAR_HEAD, R, nU.
// The lanes of near union runs in a staged chunk (finish_chunk): bit 0 = this lane heads one,
// bit 1 = it is in one, bit 2 = the lane before is, R above bit 8 (heads).
__device__ __attribute__((noinline)) int union_lanes(int lane, bool in, int k, int kp, int uR) {
    const unsigned long long D = __ballot(in && lane > 0 && kp == k - 1);  // lane continues lane-1's column
    const unsigned long long need = uR > 1 ? ((1ull << (uR - 1)) - 1) : 0ull;
    const bool uhead = in && uR > 1 && lane + uR - 1 <= 63 && ((D >> (lane + 1)) & need) == need;
    const unsigned long long U2 = __ballot(uhead), U3 = __ballot(uhead && uR > 2);
    const unsigned long long Uin = U2 | (U2 << 1) | (U3 << 2);
    const bool inU = (Uin >> lane) & 1ull;
    const bool prevU = lane > 0 && ((Uin >> (lane - 1)) & 1ull);
    return (uhead ? 1 : 0) | (inU ? 2 : 0) | (prevU ? 4 : 0) | (uhead ? uR << 8 : 0);
}
__device__ __forceinline__ StagedChunk finish_chunk(int lane, const ChunkLoads& c, bool tiles, int ubase = 0) {
    StagedChunk x;
    x.st = c.in ? c.m.x : 0;
    x.ln = c.in ? (tiles ? meta_ntiles(c.m) : c.m.y) : 0;
    x.av = c.av;
    const bool in = c.in;
    // union runs first (their lanes stay out of the SAME_PATTERN runs; out of line: inlined
    // twice, it cost the direct wave kernels an occupancy step)
    int uflags = 0;
    if (!tiles && ubase > 0 && __ballot(in && meta_near(c.m))) {
        uflags = union_lanes(lane, in, c.k, c.kp, in && meta_near(c.m) ? meta_near_r(c.m) : 0);
        if (uflags & 1) {
            x.st = ubase + 3 * c.m.x;
            x.ln = meta_near_n(c.m);
        }
    }
    const bool uhead = uflags & 1, inU = uflags & 2, prevU = uflags & 4;
    const int uR = uflags >> 8;
    const bool cont = in && lane > 0 && meta_same(c.m) && c.kp == c.k - 1 && !inU && !prevU;
    const unsigned long long C = __ballot(cont);
    bool head;
    if (tiles) {
        head = in && !cont;
        x.L = 1;
    } else if (MHS_RUN_MAX == 1) {
        head = in;
        x.L = 1;
    } else {
        const unsigned long long incl = (2ull << lane) - 1;  // lanes <= lane (all at 63)
        const int h = 63 - __clzll(~C & incl);               // start of this lane's run
        head = in && (lane - h) % MHS_RUN_MAX == 0;
        const unsigned long long above = lane == 63 ? 0ull : (C >> (lane + 1));
        x.L = min(MHS_RUN_MAX, 1 + __builtin_ctzll(~above));
        if (inU) {  // a union run: its head visits, its members do not
            head = uhead;
            x.L = uhead ? uR : 1;
        }
    }
    const unsigned long long Hm = __ballot(head);
    x.nh = __popcll(Hm);
    const int ci = __popcll(Hm & lanemask_lt());
    const int dst = head ? ci : x.nh + (lane - ci);  // a permutation of the lanes
    x.src = __builtin_amdgcn_ds_permute(dst << 2, lane);
    int lm = 1;
    if (!tiles && MHS_RUN_MAX > 1) {
        if (__ballot(head && x.L > 1)) lm = 2;
        if (MHS_RUN_MAX > 2 && __ballot(head && x.L > 2)) lm = 3;
        if (MHS_RUN_MAX > 3 && __ballot(head && x.L > 3)) lm = 4;
    }
    x.lmax = lm;
    return x;
}
__device__ __forceinline__ StagedChunk stage_chunk(int lane, int jb, int a1,
                                                   const int* __restrict__ Acol,
                                                   const double* __restrict__ Aval,
                                                   const int4* __restrict__ bmeta, bool tiles) {
    ChunkLoads c = load_chunk_a(lane, jb, a1, Acol, Aval);
    load_chunk_meta(c, bmeta);
    return finish_chunk(lane, c, tiles);
}

// Lane-group width of one staged chunk: nh visits of about `avg` B entries each, U entries
// per lane and load batch.  Minimises the chunk's dependent load batches
// ceil(nh / groups) * ceil(avg / (G*U)), ties to the wider group; at least gmin.
__device__ __forceinline__ int chunk_group(int nh, int avg, int U, int gmin) {
    int best = gmin, bc = INT_MAX;
    for (int g = gmin; g <= 64; g <<= 1) {
        const int ng = 64 / g;
        const int c = ((nh + ng - 1) / ng) * ((avg + g * U - 1) / (g * U));
        if (c <= bc) {
            bc = c;
            best = g;
        }
    }
    return best;
}

// XCD-grouped walk over a row list: blocks b and b+8 share an XCD (round-robin
// dispatch), so group g = b % 8 takes the g-th eighth of the list and its blocks
// stride through it.  Speed only -- any placement gives the same result.
struct RowWalk {
    int first, end, stride;
    __device__ RowWalk(int count, int teams_per_block, int team)
        : RowWalk(count, teams_per_block, team, (int)blockIdx.x, (int)gridDim.x) {}
    // blocks [0, nb) of a sub-grid (bid = index in it)
    __device__ RowWalk(int count, int teams_per_block, int team, int bid, int nb) {
        if ((nb & 7) == 0) {
            const int g = bid & 7, nbg = nb >> 3, bi = bid >> 3;
            first = (int)((long long)count * g / 8) + bi * teams_per_block + team;
            end = (int)((long long)count * (g + 1) / 8);
            stride = nbg * teams_per_block;
        } else {
            first = bid * teams_per_block + team;
            end = count;
            stride = nb * teams_per_block;
        }
    }
};

constexpr int MHS_GRP_CHUNK = 63;  // A entries staged per chunk in the grouped walk (<= 64)
static_assert(MHS_GRP_CHUNK >= 1 && MHS_GRP_CHUNK <= 64, "a chunk is one entry per lane");
constexpr int MHS_SYMWM_DYN_MAX = 32768;  // k_sym_rare's 10 KiB wave rows from the cursors up to this many rows
constexpr int MHS_DYN16_MAX = 32768;  // hash 10 KiB bins of at most this many rows: all rows from the cursor
constexpr int MHS_GUIDED_STATIC = 4;  // eighths of an XCD group's rows walked statically before the cursor
// Dynamic XCD-grouped walk: group g = blockIdx % 8 (an XCD under round-robin dispatch) owns
// the g-th eighth of the list; its waves take CH consecutive entries at a time from the
// group's cursor, in list order.  The rows in flight on an XCD stay one compact window
// (neighbouring rows share B rows in its L2) and a slow row holds back no other.
struct WaveQueue {
    int* cur;
    int begin, end, i, lim, ch;
    __device__ WaveQueue(int* cursors, int count, int chunk) : ch(chunk) {
        const int g = (int)(blockIdx.x & 7);
        begin = (int)((long long)count * g / 8);
        end = (int)((long long)count * (g + 1) / 8);
        cur = cursors + g * CURSOR_STRIDE;
        i = lim = 0;
    }
    // next list index of this wave (wave-uniform), false once the group's eighth is done
    __device__ bool next(int& idx) {
        if (i >= lim) {
            int t = 0;
            if (lane_id() == 0) t = atomicAdd(cur, ch);
            t = __builtin_amdgcn_readfirstlane(t);
            i = begin + t;
            lim = min(i + ch, end);
            if (i >= end) return false;
        }
        idx = i++;
        return true;
    }
};

// Dynamic row queue of a block team (k_sym_rare, k_num_block): thread 0 takes the next list
// index from the launch's cursor (one atomic per row: the block bins hold hundreds to a few
// thousand rows), the block reads it between two barriers.  Power-law rows differ by orders
// of magnitude in cost; a static stride left the kernel's end to the block that drew the
// heaviest rows.  (k_sym_block<256> keeps its static walk: tens of thousands of uniform rows
// on one cursor measured +12 % on cant-s1- and scircuit-like.)
struct BlockQueue {
    int* cur;
    int* slot;  // an LDS word
    int count;
    __device__ bool next(int& idx) const {
        __syncthreads();  // every thread has read the previous index
        if (threadIdx.x == 0) *slot = atomicAdd(cur, 1);
        __syncthreads();
        idx = *slot;
        return idx < count;
    }
};

// ------------------------------------------------------------------- teams ---
// A team processes one row at a time: a wave (64 lanes, wave_sync) or a whole
// block (__syncthreads; reductions through an LDS header).  GlobalTeam is a
// block whose tables live in global memory: its sync makes global stores and
// atomics visible block-wide (agent-scope fence: L1 invalidate).

struct WaveTeam {
    static constexpr int size = 64;
    __device__ int rank() const { return lane_id(); }
    __device__ void sync() const { wave_sync(); }
    __device__ int bcast0(int v) const { return __builtin_amdgcn_readfirstlane(v); }  // (lane 0 is active)
    template <class V>
    __device__ V sum(V v) const { return wave_sum(v); }
    template <class LD, class ST>
    __device__ void exclusive_scan(int L, LD load, ST store) const {
        const int lane = lane_id();
        int carry = 0;
        for (int b = 0; b < L; b += 64) {
            const int i = b + lane;
            const int x = i < L ? load(i) : 0;
            const int inc = wave_incl_scan(x);
            if (i < L) store(i, carry + inc - x);
            carry += __shfl(inc, 63);
        }
    }
};

template <int T, bool GLOBALMEM>
struct BlockTeam {
    static constexpr int size = T;
    static constexpr int W = T / 64;
    long long* scratch;  // LDS, >= W entries
    __device__ int rank() const { return threadIdx.x; }
    __device__ void sync() const {
        if constexpr (GLOBALMEM) __threadfence();
        __syncthreads();
    }
    __device__ int bcast0(int v) const {  // thread 0's v in every thread
        __syncthreads();
        if (threadIdx.x == 0) scratch[0] = v;
        __syncthreads();
        const int r = (int)scratch[0];
        __syncthreads();
        return r;
    }
    template <class V>
    __device__ V sum(V v) const {
        v = wave_sum(v);
        const int w = threadIdx.x >> 6;
        if (lane_id() == 0) scratch[w] = (long long)v;
        __syncthreads();
        long long r = 0;
#pragma unroll
        for (int i = 0; i < W; ++i) r += scratch[i];
        __syncthreads();
        return (V)r;
    }
    template <class LD, class ST>
    __device__ void exclusive_scan(int L, LD load, ST store) const {
        const int lane = lane_id(), w = threadIdx.x >> 6;
        int* ws = (int*)scratch;
        int carry = 0;
        for (int b = 0; b < L; b += T) {
            const int i = b + (int)threadIdx.x;
            const int x = i < L ? load(i) : 0;
            const int inc = wave_incl_scan(x);
            if (lane == 63) ws[w] = inc;
            __syncthreads();
            int woff = 0, tot = 0;
#pragma unroll
            for (int k = 0; k < W; ++k) {
                const int v = ws[k];
                woff += (k < w) ? v : 0;
                tot += v;
            }
            if (i < L) store(i, carry + woff + inc - x);
            carry += tot;
            __syncthreads();
        }
        if constexpr (GLOBALMEM) sync();
    }
};

template <class Team>
__device__ void team_bitonic(const Team& tm, unsigned long long* S, int P) {
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tm.rank(); i < P; i += Team::size) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const unsigned long long a = S[i], b = S[ixj];
                    const bool up = (i & k) == 0;
                    if ((a > b) == up) {
                        S[i] = b;
                        S[ixj] = a;
                    }
                }
            }
            tm.sync();
        }
    }
}

// Lane exchange v <- lane ^ d (d a power of two, a compile-time constant once the
// callers' loops are unrolled) without the LDS crossbar where the hardware has a path:
// DPP quad_perm for d = 1, 2; DPP row shifts + select for d = 4, 8 (both neighbours are
// inside the lane's 16-lane row); ds_swizzle (xor mode, no LDS memory access) for 16;
// ds_bpermute only for 32.  Every lane of the wave must be active.
__device__ __forceinline__ int xor_lanes(int v, int d) {
    const int lane = lane_id();
    if (d == 1) return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    if (d == 2) return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    if (d == 4) {
        const int up = __builtin_amdgcn_mov_dpp(v, 0x104, 0xF, 0xF, false);  // row_shl:4  (lane + 4)
        const int dn = __builtin_amdgcn_mov_dpp(v, 0x114, 0xF, 0xF, false);  // row_shr:4  (lane - 4)
        return (lane & 4) ? dn : up;
    }
    if (d == 8) {
        const int up = __builtin_amdgcn_mov_dpp(v, 0x108, 0xF, 0xF, false);  // row_shl:8
        const int dn = __builtin_amdgcn_mov_dpp(v, 0x118, 0xF, 0xF, false);  // row_shr:8
        return (lane & 8) ? dn : up;
    }
    if (d == 16) return __builtin_amdgcn_ds_swizzle(v, 0x401F);  // and 0x1F, xor 0x10
    return __shfl_xor(v, d);
}

// DPP row shift right by d (d in 1, 2, 4, 8; lanes whose source is outside their 16-lane row
// read 0), whole-wave shifts by one lane, row broadcasts (GFX9 row_bcast:15 / :31).
__device__ __forceinline__ int row_shr(int v, int d) {
    if (d == 1) return __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);
    if (d == 2) return __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);
    if (d == 4) return __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true);
    return __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true);
}
__device__ __forceinline__ int wave_shr1(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, true); }
__device__ __forceinline__ int wave_shl1(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x130, 0xF, 0xF, true); }
template <int ROWS>
__device__ __forceinline__ int row_bcast15(int v) {  // lane 15 of row r -> row r+1 (rows in ROWS), else 0
    return __builtin_amdgcn_update_dpp(0, v, 0x142, ROWS, 0xF, false);
}
template <int ROWS>
__device__ __forceinline__ int row_bcast31(int v) {  // lane 31 -> rows 2, 3 (in ROWS), else 0
    return __builtin_amdgcn_update_dpp(0, v, 0x143, ROWS, 0xF, false);
}
// Inclusive scan over teams of W lanes (aligned groups of W consecutive lanes).
template <int W>
__device__ __forceinline__ int team_incl_scan(int x, int tl) {
#pragma unroll
    for (int d = 1; d < (W < 16 ? W : 16); d <<= 1) {
        const int o = row_shr(x, d);
        x += tl >= d ? o : 0;  // (W < 16: teams share a row -- the guard keeps them apart)
    }
    if (W >= 32) x += row_bcast15<0xA>(x);
    if (W == 64) x += row_bcast31<0xC>(x);
    return x;
}

// Segmented inclusive sum over teams of W lanes: a lane with `seen` set starts a segment.
template <int W>
__device__ __forceinline__ double team_seg_scan(double sum, bool seen, int tl) {
#pragma unroll
    for (int d = 1; d < (W < 16 ? W : 16); d <<= 1) {
        const int oh = row_shr(__double2hiint(sum), d), ol = row_shr(__double2loint(sum), d);
        const int of = row_shr((int)seen, d);
        const bool add = tl >= d && !seen;
        sum += add ? __hiloint2double(oh, ol) : 0.0;
        seen = add ? of != 0 : seen;
    }
    auto carry = [&](int oh, int ol, bool rows) {
        if (rows && !seen) sum += __hiloint2double(oh, ol);
    };
    const int row = lane_id() >> 4;
    if (W == 32) {  // rows 1, 3 take lane 15 / 47 of the row below
        carry(row_bcast15<0xA>(__double2hiint(sum)), row_bcast15<0xA>(__double2loint(sum)), (row & 1) != 0);
    } else if (W == 64) {  // row 1 <- lane 15, then row 2 <- lane 31, then row 3 <- lane 47 (each
                           // already final: a lane without a head in its row continues the row below)
        carry(row_bcast15<0x2>(__double2hiint(sum)), row_bcast15<0x2>(__double2loint(sum)), row == 1);
        carry(row_bcast31<0x4>(__double2hiint(sum)), row_bcast31<0x4>(__double2loint(sum)), row == 2);
        carry(row_bcast15<0x8>(__double2hiint(sum)), row_bcast15<0x8>(__double2loint(sum)), row == 3);
    }
    return sum;
}

// Bitonic sort of W*K unsigned keys held by a team of W lanes, K per lane, ascending
// over element e = i*W + tl (slot i, team lane tl): partners at distance d < W are in
// other lanes (shuffles), at d >= W in other slots of the lane.  Compare-exchange by
// selects (no divergent branches).
template <int W, int K>
__device__ __forceinline__ void reg_bitonic(unsigned (&key)[K], int tl) {
#pragma unroll
    for (int k = 2; k <= W * K; k <<= 1) {
#pragma unroll
        for (int d = k >> 1; d > 0; d >>= 1) {
            if (d < W) {
                unsigned ok[K];
#pragma unroll
                for (int i = 0; i < K; ++i) ok[i] = (unsigned)xor_lanes((int)key[i], d);  // d < W: inside the team
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    const bool asc = ((i * W + tl) & k) == 0, low = (tl & d) == 0;
                    const bool take = (low == asc) ? ok[i] < key[i] : ok[i] > key[i];
                    key[i] = take ? ok[i] : key[i];
                }
            } else {
                const int ds = d / W;
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    if (i & ds) continue;
                    const int j = i | ds;
                    const bool asc = ((i * W + tl) & k) == 0;
                    const unsigned lo_ = key[i] < key[j] ? key[i] : key[j];
                    const unsigned hi_ = key[i] < key[j] ? key[j] : key[i];
                    key[i] = asc ? lo_ : hi_;
                    key[j] = asc ? hi_ : lo_;
                }
            }
        }
    }
}

template <bool GLOBALMEM>
__device__ __forceinline__ void acc_add(double* p, double v) {
    if constexpr (GLOBALMEM) unsafeAtomicAdd(p, v);
    else atomicAdd(p, v);  // ds_add_f64
}

// --------------------------------------------------- Form_mask_matrix_B ---
// G lanes per B row.  Per chunk of G entries: head = first entry of a tile run,
// a forward segmented OR scan collects each run's bits, the run's last lane
// (tail) writes (tile, mask) at row_start + run index.  A run that crosses a
// chunk edge is carried in `carry`.  Also checks the sorted-columns precondition.
// One B row by a lane group of G lanes (every lane of the wave calls it: shuffles and
// ballots); `valid` false for groups without a row.
template <int G, int MC>
__device__ __forceinline__ void mask_row(int row, bool valid, int N, const int* __restrict__ ptr,
                                         const int* __restrict__ col, int* __restrict__ btcol,
                                         unsigned long long* __restrict__ btmask, int4* __restrict__ bmeta,
                                         int* __restrict__ bhi, int& err) {
    const int lane = lane_id();
    const int gl = lane & (G - 1);
    const int gbase = lane & ~(G - 1);
    unsigned long long gmask = ~0ull;
    if constexpr (G < 64) gmask = ((1ull << G) - 1) << gbase;
    const int s = valid ? ptr[row] : 0;
    const int e = valid ? ptr[row + 1] : 0;
    // same column pattern as the previous row (FEM dofs of one node): later
    // phases OR its tiles once per run and fuse its products (SAME_PATTERN)
    const int ps = (valid && row > 0) ? ptr[row - 1] : 0;
    const bool same_len = valid && row > 0 && e > s && (s - ps) == (e - s);
    bool differ = false;
    int ntiles = 0, prev_col = -1;
    unsigned long long carry = 0;
    // MC chunks' columns (and the previous row's, for the same-pattern test) are loaded together,
    // plus the next group's first chunk (its first column closes the last chunk's runs): one
    // round trip per MC chunks (MC = 4 where rows average more than G entries: wb-edu-like and
    // cage15-like masks -5..7 %; rows of one chunk keep MC = 1)
    for (int b0 = s; b0 < e; b0 += MC * G) {
        int cc[MC + 1], pp[MC];
#pragma unroll
        for (int u = 0; u <= MC; ++u) {
            const int j = b0 + u * G + gl;
            cc[u] = j < e ? col[j] : INT_MAX;
            if (u < MC) pp[u] = (same_len && j < e) ? col[ps + (j - s)] : 0;
        }
#pragma unroll
        for (int u = 0; u < MC; ++u) {
            const int b = b0 + u * G;
            if (b >= e) break;
            const int j = b + gl;
            const bool in = j < e;
            const int c = cc[u];
            if (same_len && in && pp[u] != c) differ = true;
            const int first_next = __shfl(cc[u + 1], gbase);
            const int up = __shfl_up(c, 1, G);
            const int pc = (gl == 0) ? prev_col : up;
            const int tile = c >> TILE_SHIFT;
            const int ptile = pc < 0 ? -1 : (pc >> TILE_SHIFT);
            const bool head = in && tile != ptile;
            if (in && c < pc) err |= ERR_UNSORTED;
            if (in && (c < 0 || c >= N)) err |= ERR_COL_RANGE;
            // next entry's column: within the chunk from the neighbour lane, at the
            // chunk edge from the next chunk's first
            const int dn = __shfl_down(c, 1, G);
            int nc = (gl == G - 1) ? first_next : dn;
            if (j + 1 >= e) nc = INT_MAX;
            const bool tail = in && ((nc >> TILE_SHIFT) != tile || nc == INT_MAX);
            // forward segmented OR within the chunk
            unsigned long long m = in ? (1ull << (c & (TILE_BITS - 1))) : 0ull;
            if (gl == 0 && !head) m |= carry;
#pragma unroll
            for (int d = 1; d < G; d <<= 1) {
                const unsigned long long om = __shfl_up(m, d, G);
                const int ot = __shfl_up(tile, d, G);
                if (gl >= d && ot == tile) m |= om;
            }
            const unsigned long long hb = __ballot(head) & gmask;
            if (tail) {
                const unsigned long long le = (lane == 63) ? ~0ull : ((2ull << lane) - 1);
                const int pos = s + ntiles + __popcll(hb & le) - 1;
                btcol[pos] = tile;
                btmask[pos] = m;
            }
            ntiles += __popcll(hb);
            const int last = (e - b < G ? e - b : G) - 1;
            const unsigned long long lm = __shfl(m, gbase + last);
            const int lc = __shfl(c, gbase + last);
            const bool lt = __shfl((int)tail, gbase + last) != 0;
            carry = lt ? 0ull : lm;
            prev_col = lc;
        }
    }
    const bool same = same_len && (__ballot(differ) & gmask) == 0;
    if (valid && gl == 0) {
        bmeta[row] = make_int4(s, e - s, ntiles | (same ? SAME_PATTERN : 0), e > s ? (col[s] >> TILE_SHIFT) : INT_MAX);
        bhi[row] = e > s ? (col[e - 1] >> TILE_SHIFT) : -1;
    }
}

// G lanes per B row.  Per chunk of G entries: head = first entry of a tile run,
// a forward segmented OR scan collects each run's bits, the run's last lane
// (tail) writes (tile, mask) at row_start + run index.  A run that crosses a
// chunk edge is carried in `carry`.  Also checks the sorted-columns precondition.
// Rows longer than MASK_LONG chunks (power-law matrices) are deferred and then
// walked by the whole wave, one at a time: a G-lane group would hold its wave (and
// the kernel's tail) for thousands of iterations.
constexpr int MASK_LONG = 16;
template <int G, int MC>
__global__ __launch_bounds__(256) void k_mask_b(int MB, int N, const int* __restrict__ ptr,
                                                const int* __restrict__ col, int* __restrict__ btcol,
                                                unsigned long long* __restrict__ btmask,
                                                int4* __restrict__ bmeta, int* __restrict__ bhi,
                                                Stats* __restrict__ stats) {
    const int lane = lane_id();
    const int gl = lane & (G - 1);
    const int row = (int)((blockIdx.x * (unsigned)blockDim.x + threadIdx.x) / G);
    const bool valid = row < MB;
    int err = 0;
    bool lng = false;
    if constexpr (G < 64) lng = valid && ptr[row + 1] - ptr[row] > MASK_LONG * G;
    mask_row<G, MC>(row, valid && !lng, N, ptr, col, btcol, btmask, bmeta, bhi, err);
    if constexpr (G < 64) {
        for (unsigned long long lb = __ballot(lng && gl == 0); lb; lb &= lb - 1) {
            const int r = __shfl(row, __builtin_ctzll(lb));
            mask_row<64, 4>(r, true, N, ptr, col, btcol, btmask, bmeta, bhi, err);
        }
    }
    if (__any(err != 0)) {
        int werr = err;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) werr |= __shfl_xor(werr, d);
        if (lane == 0) atomicOr(&stats->err, werr);
    }
}

// Short rows (matrices averaging at most 8 entries a row): a lane per B row, 64 rows a wave.
// The lane loads U entries of its row at a time (all issued together) and builds the
// (tile, mask) runs in order in its registers -- no shuffles within a row, so one
// ptr -> col round trip serves 64 rows instead of the 8-16 of the lane groups (those kernels
// were bound by that chain: wb-edu-like 0.9 ms, GAP-road-like 0.5 ms for a few hundred MB).
// Same-pattern test: row r-1 is the lane below (its chunk i sits in the same registers), for
// lane 0 a load.  Rows past MASK_LANE_LONG entries: whole-wave walks afterwards.
constexpr int MASK_LANE_LONG = 32;
template <int U>
__global__ __launch_bounds__(256) void k_mask_lane(int MB, int N, const int* __restrict__ ptr,
                                                   const int* __restrict__ col, int* __restrict__ btcol,
                                                   unsigned long long* __restrict__ btmask,
                                                   int4* __restrict__ bmeta, int* __restrict__ bhi,
                                                   Stats* __restrict__ stats) {
    const int lane = lane_id();
    const int row = (int)(blockIdx.x * 256u + threadIdx.x);
    const bool valid = row < MB;
    const int s = valid ? ptr[row] : 0;
    const int e = valid ? ptr[row + 1] : 0;
    const int len = e - s;
    const bool lng = len > MASK_LANE_LONG;
    const bool act = valid && !lng && len > 0;
    // the previous row's length: the lane below's, lane 0 loads it
    int pl = __shfl_up(len, 1);
    if (lane == 0) pl = (valid && row > 0) ? s - ptr[row - 1] : -1;
    const bool same_len = act && row > 0 && pl == len;
    int err = 0, ntiles = 0, prev_c = -1, cur_t = -1, first_t = INT_MAX;
    unsigned long long cur_m = 0ull;
    bool differ = false;
    const int nch = act ? (len + U - 1) / U : 0;
    const int maxch = wave_max(nch);  // (uniform trip count: the shuffles need every lane)
    for (int i = 0; i < maxch; ++i) {
        int c[U];
        bool in[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = s + i * U + u;
            in[u] = act && j < e;
            c[u] = in[u] ? col[j] : INT_MAX;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int p = __shfl_up(c[u], 1);
            if (lane == 0 && same_len && in[u]) p = col[s + i * U + u - len];
            differ = differ || (same_len && in[u] && p != c[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!in[u]) continue;
            const int cc = c[u];
            if (cc < prev_c) err |= ERR_UNSORTED;
            if (cc < 0 || cc >= N) err |= ERR_COL_RANGE;
            prev_c = cc;
            const int t = cc >> TILE_SHIFT;
            if (t != cur_t) {
                if (cur_t < 0) first_t = t;
                if (cur_t >= 0) {
                    btcol[s + ntiles] = cur_t;
                    btmask[s + ntiles] = cur_m;
                    ++ntiles;
                }
                cur_t = t;
                cur_m = 0ull;
            }
            cur_m |= 1ull << (cc & (TILE_BITS - 1));
        }
    }
    if (cur_t >= 0) {
        btcol[s + ntiles] = cur_t;
        btmask[s + ntiles] = cur_m;
        ++ntiles;
    }
    if (valid && !lng) {
        bmeta[row] = make_int4(s, len, ntiles | (same_len && !differ ? SAME_PATTERN : 0), first_t);
        bhi[row] = cur_t;  // the last tile (-1: an empty row)
    }
    for (unsigned long long lb = __ballot(lng); lb; lb &= lb - 1) {
        const int r = __shfl(row, __builtin_ctzll(lb));
        mask_row<64, 4>(r, true, N, ptr, col, btcol, btmask, bmeta, bhi, err);
    }
    if (__any(err != 0)) {
        int werr = err;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) werr |= __shfl_xor(werr, d);
        if (lane == 0) atomicOr(&stats->err, werr);
    }
}

// ------------------------------------------------------------ row analysis ---

__device__ __forceinline__ int sym_bin_of(int flop, int tflop, int span) {
    if (flop == 0) return SYM_NONE;
    const long long need = sym_need(span, tflop);
    if (need <= SYM_WAVE_BYTES - WAVE_HDR && tflop <= SYM_WAVE_WORK) return SYM_WAVE;
    if (need <= SYM_WM_BYTES - WAVE_HDR && tflop <= SYM_WAVE_WORK) return SYM_WM;
    if (need <= SYM_B256_BYTES - BLOCK_HDR && tflop <= SYM_B256_WORK) return SYM_B256;
    if (need <= B1024_BYTES) return SYM_B1024;
    return SYM_GLOBAL;
}

// A row's symbolic tiny class (-1: none): tiny_class_sym's 8- and 32-lane classes, and class 4
// -- (64,8), a register sort of at most 512 products -- for a row the small wave table cannot
// hold (round 5: such rows -- a hub column's B row beside a few short ones, web-graph rows of
// a few hundred scattered tiles -- took 2-4 dependent table steps a product in 10 KiB waves
// or block tables).  Numeric recomputes it to know which rows left no masks behind.
__device__ __forceinline__ int sym_tiny_class(int flop, int nA, int tflop, int span) {
    const int c = tiny_class_sym(flop, nA);
    if (MHS_SYM_SORT64 && c < 0 && flop > 0 && flop <= tiny_ws(4) * tiny_ks(4) && nA <= tiny_ws(4) &&
        sym_bin_of(flop, tflop, span) != SYM_WAVE)
        return 4;
    return c;
}

// Stats -> fine-grained pinned host memory, then the sequence number the host spins
// on (wave 0 of one block: L1-bypassing reads, system-scope stores, release of the
// number).  One wave does it all, so the release's wait for the wave's outstanding
// stores covers every word: no block-wide system fence (an extra L2 write-back) and
// no barrier on the path to the host.
__device__ void publish_stats(const Stats* stats, Published* pub, int seq) {
    constexpr int NW = (int)(sizeof(Stats) / 4);
    static_assert(sizeof(Stats) % 4 == 0 && NW <= 1024, "Stats is copied by wave 0, zeroed by one block");
    if (threadIdx.x >= 64) return;
    const int* src = reinterpret_cast<const int*>(stats);
    int* dst = reinterpret_cast<int*>(&pub->stats);
    for (int i = threadIdx.x; i < NW; i += 64)
        __hip_atomic_store(dst + i, __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (threadIdx.x == 0) __hip_atomic_store(&pub->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Last block of a grid to reach this point (after its writes): returns true in
// every thread of that block, with the other blocks' writes visible to it.
__device__ bool last_block_done(int* done) {
    __shared__ int last;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        last = atomicAdd(done, 1) == (int)gridDim.x - 1;
    }
    __syncthreads();
    if (last) __threadfence();
    return last;
}

// One A row by a group of G lanes (all lanes of the wave call it); returns the row's
// flop in every lane of the group (0 for invalid groups).
__device__ __forceinline__ void analyze_out(int row, long long flop, long long tflop, int lo, int hi, int kfirst,
                                            bool differ, bool bad, int nA, int* __restrict__ rflop,
                                            int* __restrict__ rtflop, int* __restrict__ rlo, int* __restrict__ rhi,
                                            int* __restrict__ ctiles, unsigned char* __restrict__ sym_bin,
                                            int* __restrict__ Cptr, unsigned char* __restrict__ asame,
                                            unsigned char* __restrict__ nft_bin, int& nslots, int& nother,
                                            unsigned* __restrict__ nsig, int sort64);
template <int G, int U = (G == 64 ? 4 : 1)>
__device__ __forceinline__ long long analyze_row(int row, bool valid, int MB, const int* __restrict__ Aptr,
                                                 const int* __restrict__ Acol, const int4* __restrict__ bmeta,
                                                 const int* __restrict__ bhi, int* __restrict__ rflop,
                                                 int* __restrict__ rtflop, int* __restrict__ rlo,
                                                 int* __restrict__ rhi, int* __restrict__ ctiles,
                                                 unsigned char* __restrict__ sym_bin, int* __restrict__ Cptr,
                                                 unsigned char* __restrict__ asame, int& err,
                                                 unsigned char* __restrict__ nft_bin, int& nslots, int& nother,
                                                 unsigned* __restrict__ nsig, int sort64) {
    const int gl = lane_id() & (G - 1);
    long long flop = 0, tflop = 0;
    int lo = INT_MAX, hi = -1;
    int kfirst = -1;  // the row's first A column (lane 0 of the group)
    bool differ = true;  // row's column pattern differs from row-1's (row groups)
    bool bad = false;    // an A column outside [0, B.M): the row is never walked (MHS_ERR_INVALID)
    if (valid) {
        const int s = Aptr[row], e = Aptr[row + 1];
        const int ps = row > 0 ? Aptr[row - 1] : 0;
        differ = !(row > 0 && e > s && s - ps == e - s);
        const int dp = s - ps;
        // U entries a lane per round, their loads issued together -- one Acol -> bmeta round
        // trip per U*G entries: the whole-wave walk of a long row (hub rows of power-law
        // matrices: thousands of entries) and the lane groups of matrices whose rows average
        // more than G entries (round 4: cant-like analysis -15 %, cage15-like -13 %; rows of
        // fewer entries keep U = 1: delaunay-like +9 % at 4)
        for (int j0 = s + gl; j0 < e; j0 += G * U) {
            int k[U], kp[U];
            bool in[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int j = j0 + u * G;
                in[u] = j < e;
                const int jj = in[u] ? j : j0;  // clamped: a cache hit, not counted
                k[u] = Acol[jj];
                kp[u] = Acol[jj - dp];  // unconditional: stays in [0, nnz(A)); a guarded load would serialise
            }
            int4 m[U];
            int h[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int kc = in[u] && k[u] >= 0 && k[u] < MB ? k[u] : 0;  // (row 0: a valid slot, unused)
                m[u] = bmeta[kc];
                h[u] = bhi[kc];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (!in[u]) continue;
                differ = differ || kp[u] != k[u];
                if (j0 + u * G == s) kfirst = k[u];
                if (k[u] < 0 || k[u] >= MB) {
                    err = ERR_ACOL_RANGE;
                    bad = true;
                    continue;
                }
                flop += m[u].y;
                tflop += meta_ntiles(m[u]);
                lo = min(lo, m[u].w);
                hi = max(hi, h[u]);
            }
        }
    }
#pragma unroll
    for (int d = G / 2; d >= 1; d >>= 1) {
        flop += __shfl_xor(flop, d);
        tflop += __shfl_xor(tflop, d);
        lo = min(lo, __shfl_xor(lo, d));
        hi = max(hi, __shfl_xor(hi, d));
        const int od = __shfl_xor((int)differ, d);  // every lane shuffles (no short circuit)
        differ = differ || od != 0;
        const int ob = __shfl_xor((int)bad, d);
        bad = bad || ob != 0;
    }
    if (valid && gl == 0)
        analyze_out(row, flop, tflop, lo, hi, kfirst, differ, bad, Aptr[row + 1] - Aptr[row], rflop, rtflop, rlo, rhi,
                    ctiles, sym_bin, Cptr, asame, nft_bin, nslots, nother, nsig, sort64);
    return valid ? flop : 0;
}

// A row's analysis outputs (its lane of the group / its own lane).
__device__ __forceinline__ void analyze_out(int row, long long flop, long long tflop, int lo, int hi, int kfirst,
                                            bool differ, bool bad, int nA, int* __restrict__ rflop,
                                            int* __restrict__ rtflop, int* __restrict__ rlo, int* __restrict__ rhi,
                                            int* __restrict__ ctiles, unsigned char* __restrict__ sym_bin,
                                            int* __restrict__ Cptr, unsigned char* __restrict__ asame,
                                            unsigned char* __restrict__ nft_bin, int& nslots, int& nother,
                                            unsigned* __restrict__ nsig, int sort64) {
    {
        // a row with an out-of-range column enters no bin: the symbolic kernels gather
        // bmeta[Acol[j]] unchecked, and the host returns MHS_ERR_INVALID before numeric
        asame[row] = (unsigned char)((differ || bad) ? 0 : 1);
        const int f = bad ? 0 : sat_int(flop), tf = bad ? 0 : sat_int(tflop);
        const int span = f ? hi - lo + 1 : 0;
        rflop[row] = f;
        rtflop[row] = tf;
        rlo[row] = lo;
        rhi[row] = hi;
        // (class 4 only where numeric sorts the row too: k_scan sends it to a 64-lane tiny class,
        // so no numeric table kernel looks for masks symbolic did not keep)
        const int tc = sort64 && (long long)span * TILE_BITS - 1 <= TINY_NUM_NMAX ? sym_tiny_class(f, nA, tf, span)
                                                                                   : tiny_class_sym(f, nA);
        const int bin = tc >= 0 ? SYM_TINY + tc : sym_bin_of(f, tf, span);
        sym_bin[row] = (unsigned char)bin;
        // near row-group signature (k_bin_list links rows whose signatures match: the same
        // C tile span and first A column, both in the small-table wave bin); a collision only
        // adds a candidate that k_sym_rare's check turns down (it compares every row's span,
        // counts and row-cache words with the head's)
        if (nsig)
            nsig[row] = (bin == SYM_WAVE && nA >= 8 && !bad)
                            ? (((unsigned)lo * 0x9E3779B1u) ^ ((unsigned)hi * 0x85EBCA77u) ^
                               ((unsigned)kfirst * 0xC2B2AE3Du)) | 1u
                            : 0u;
        if (nft_bin) {
            // numeric-first candidates: the numeric classes 0..3, whose sort keys hold the
            // column relative to the row's first tile (23 bits); a wider row counts in a table
            const int tn = (long long)span * TILE_BITS - 1 <= TINY_NUM_NMAX ? tiny_class(f, nA, TINY_SYM_NC) : -1;
            // (class 4 rows sort in symbolic's class-4 range either way)
            nft_bin[row] = (unsigned char)(tn >= 0 ? SYM_TINY + tn : tc >= 0 && tc < 4 ? sym_bin_of(f, tf, span) : bin);
            nslots += tn >= 0 ? tiny_w(tn) * tiny_k(tn) : 0;
            nother += f > 0 && tn < 0;
        }
        if (bin == SYM_NONE) {
            Cptr[row] = 0;
            ctiles[row] = 0;
        }
    }
}

// G lanes per A row; rows longer than AN_LONG*G entries are deferred to whole-wave
// walks (as in k_mask_b).
constexpr int AN_LONG = 16;
// k_analyze's per-block word: flop (< 2^37: <= 64 rows of < 2^31) in the low 40 bits, then
// 8 bits of rows past the tiny classes (<= 64 per block) and 16 of numeric-first slot
// entries (<= 64 rows x 128)
constexpr int BLK_FLOP_BITS = 40, BLK_SLOT_SHIFT = 48;
constexpr unsigned long long BLK_FLOP_MASK = (1ull << BLK_FLOP_BITS) - 1;
template <int G, int U>
__global__ __launch_bounds__(256) void k_analyze(int M, int MB, const int* __restrict__ Aptr,
                                                 const int* __restrict__ Acol,
                                                 const int4* __restrict__ bmeta,
                                                 const int* __restrict__ bhi, int* __restrict__ rflop,
                                                 int* __restrict__ rtflop, int* __restrict__ rlo,
                                                 int* __restrict__ rhi, int* __restrict__ ctiles,
                                                 unsigned char* __restrict__ sym_bin, int* __restrict__ Cptr,
                                                 unsigned long long* __restrict__ blkflop,
                                                 unsigned char* __restrict__ asame,
                                                 Stats* __restrict__ stats,
                                                 unsigned long long* __restrict__ lb_state, int nlb,
                                                 unsigned char* __restrict__ nft_bin, unsigned* __restrict__ nsig, int sort64) {
    const int lane = lane_id();
    const int gl = lane & (G - 1);
    const int row = (int)((blockIdx.x * (unsigned)blockDim.x + threadIdx.x) / G);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nlb; i += gridDim.x * blockDim.x)
        lb_state[i] = 0ull;  // k_scan's look-back words (k_scan runs after every analyze block)
    const bool valid = row < M;
    int err = 0, nslots = 0, nother = 0;
    bool lng = false;
    if constexpr (G < 64) lng = valid && Aptr[row + 1] - Aptr[row] > AN_LONG * G;
    long long flop = analyze_row<G, U>(row, valid && !lng, MB, Aptr, Acol, bmeta, bhi, rflop, rtflop, rlo, rhi,
                                    ctiles, sym_bin, Cptr, asame, err, nft_bin, nslots, nother, nsig, sort64);
    flop = gl == 0 ? flop : 0;
    if constexpr (G < 64) {
        for (unsigned long long lb = __ballot(lng && gl == 0); lb; lb &= lb - 1) {
            const int r = __shfl(row, __builtin_ctzll(lb));
            const long long f = analyze_row<64>(r, true, MB, Aptr, Acol, bmeta, bhi, rflop, rtflop, rlo, rhi,
                                                ctiles, sym_bin, Cptr, asame, err, nft_bin, nslots, nother, nsig, sort64);
            flop += lane == 0 ? f : 0;
        }
    }
    // per-block flop partial (plain store; summed by k_scan), with the block's other rows and
    // numeric-first slot entries above bit BLK_FLOP_BITS (summed by k_probe_publish)
    __shared__ unsigned long long wsum[4];
    unsigned long long mine = (unsigned long long)flop;
    if (nft_bin && gl == 0)
        mine += ((unsigned long long)nother << BLK_FLOP_BITS) + ((unsigned long long)nslots << BLK_SLOT_SHIFT);
    mine = wave_sum(mine);
    if (lane == 0) wsum[threadIdx.x >> 6] = mine;
    __syncthreads();
    if (threadIdx.x == 0) blkflop[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    if (__any(err != 0) && lane == 0) atomicOr(&stats->err, ERR_ACOL_RANGE);
}

// Short rows (matrices averaging at most 8 entries a row): a lane per A row, 64 rows a wave
// (as k_mask_lane): the lane loads U of its row's columns at a time, then their bmeta / bhi
// gathers, all issued together -- one ptr -> Acol -> bmeta chain serves 64 rows.  Rows past
// AN_LANE_LONG entries: whole-wave walks afterwards.  Two per-block words (128 rows each:
// the packing of BLK_FLOP_BITS holds at most 255 other rows a word).
constexpr int AN_LANE_LONG = 32;
template <int U>
__global__ __launch_bounds__(256) void k_analyze_lane(int M, int MB, const int* __restrict__ Aptr,
                                                      const int* __restrict__ Acol, const int4* __restrict__ bmeta,
                                                      const int* __restrict__ bhi, int* __restrict__ rflop,
                                                      int* __restrict__ rtflop, int* __restrict__ rlo,
                                                      int* __restrict__ rhi, int* __restrict__ ctiles,
                                                      unsigned char* __restrict__ sym_bin, int* __restrict__ Cptr,
                                                      unsigned long long* __restrict__ blkflop,
                                                      unsigned char* __restrict__ asame, Stats* __restrict__ stats,
                                                      unsigned long long* __restrict__ lb_state, int nlb,
                                                      unsigned char* __restrict__ nft_bin, unsigned* __restrict__ nsig, int sort64) {
    const int lane = lane_id();
    const int row = (int)(blockIdx.x * 256u + threadIdx.x);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nlb; i += gridDim.x * blockDim.x)
        lb_state[i] = 0ull;  // k_scan's look-back words (k_scan runs after every analyze block)
    const bool valid = row < M;
    int err = 0, nslots = 0, nother = 0;
    const int s = valid ? Aptr[row] : 0;
    const int e = valid ? Aptr[row + 1] : 0;
    const int len = e - s;
    const bool lng = len > AN_LANE_LONG;
    const bool act = valid && !lng;
    int pl = __shfl_up(len, 1);  // the previous row's length: the lane below's, lane 0 loads it
    if (lane == 0) pl = (valid && row > 0) ? s - Aptr[row - 1] : -1;
    const bool cmp = act && row > 0 && len > 0 && pl == len;  // compare with row - 1's columns
    bool differ = !cmp, bad = false;
    long long flop = 0, tflop = 0;
    int lo = INT_MAX, hi = -1, kfirst = -1;
    const int nch = act ? (len + U - 1) / U : 0;
    const int maxch = wave_max(nch);  // (uniform trip count: the shuffles need every lane)
    for (int i = 0; i < maxch; ++i) {
        int k[U];
        bool in[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = s + i * U + u;
            in[u] = act && j < e;
            k[u] = in[u] ? Acol[j] : 0;
        }
        int4 m[U];
        int h[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int kc = in[u] && k[u] >= 0 && k[u] < MB ? k[u] : 0;  // (row 0: a valid slot, unused)
            m[u] = bmeta[kc];
            h[u] = bhi[kc];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int p = __shfl_up(k[u], 1);
            if (lane == 0 && cmp && in[u]) p = Acol[s + i * U + u - len];
            differ = differ || (in[u] && p != k[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!in[u]) continue;
            if (i == 0 && u == 0) kfirst = k[u];
            if (k[u] < 0 || k[u] >= MB) {
                err = ERR_ACOL_RANGE;
                bad = true;
                continue;
            }
            flop += m[u].y;
            tflop += meta_ntiles(m[u]);
            lo = min(lo, m[u].w);
            hi = max(hi, h[u]);
        }
    }
    if (act)
        analyze_out(row, flop, tflop, lo, hi, kfirst, differ, bad, len, rflop, rtflop, rlo, rhi, ctiles, sym_bin,
                    Cptr, asame, nft_bin, nslots, nother, nsig, sort64);
    if (!act) flop = 0;
    for (unsigned long long lb = __ballot(lng); lb; lb &= lb - 1) {
        const int r = __shfl(row, __builtin_ctzll(lb));
        const long long f = analyze_row<64>(r, true, MB, Aptr, Acol, bmeta, bhi, rflop, rtflop, rlo, rhi, ctiles,
                                            sym_bin, Cptr, asame, err, nft_bin, nslots, nother, nsig, sort64);
        flop += lane == 0 ? f : 0;
    }
    __shared__ unsigned long long wsum[4];
    unsigned long long mine = (unsigned long long)flop;
    if (nft_bin) mine += ((unsigned long long)nother << BLK_FLOP_BITS) + ((unsigned long long)nslots << BLK_SLOT_SHIFT);
    mine = wave_sum(mine);
    if (lane == 0) wsum[threadIdx.x >> 6] = mine;
    __syncthreads();
    if (threadIdx.x < 2) blkflop[2 * blockIdx.x + threadIdx.x] = wsum[2 * threadIdx.x] + wsum[2 * threadIdx.x + 1];
    if (__any(err != 0) && lane == 0) atomicOr(&stats->err, ERR_ACOL_RANGE);
}

// ----------------------------------------------------------------- binning ---
// Stable partition of rows [0, M) by bin id into one list, bin-major.

// ------------------------------------------------------- product walking ---
// for_products(team, A row [a0, a1), ...) calls f.put(f.load(idx), a_ij) for
// every entry idx of the B segment of every A entry j: the B row's CSR range
// (numeric) or its tile range (tiles == true).  A entries come in chunks of 64
// loaded with one coalesced gather (A.col, A.val, bmeta[k]); a wave hands them
// to its lane groups with shuffles, a block through a 1 KiB LDS stage.  Each
// lane issues two independent B loads before consuming them.

// Keep a load unconditional: without a use hipcc sinks a load whose value is only
// selected under a lane predicate into a branch, with an s_waitcnt vmcnt(0) there.
__device__ __forceinline__ void pin(double& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(int& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(unsigned long long& x) { asm volatile("" : "+v"(x)); }

// near union runs of a value walk (see finish_chunk): the extended arrays' union base, 0: none
template <class F>
__device__ __forceinline__ int union_base(const F& f) {
    if constexpr (F::kUnion) return f.ubase;
    return 0;
}

template <class F>
__device__ __forceinline__ void run_segment(const F& f, int s, int n, int gl, int G, double a) {
    constexpr int U = MHS_TILE_UNROLL;
    int q = gl;
    for (; q + (U - 1) * G < n; q += U * G) {
        typename F::Item x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = f.load(s + q + u * G);
#pragma unroll
        for (int u = 0; u < U; ++u) f.put(x[u], a);
    }
    if (q < n) {  // the tail (< U entries) in one batch: clamped loads, no per-entry round trip
        typename F::Item x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = f.load(s + (q + u * G < n ? q + u * G : q));
#pragma unroll
        for (int u = 0; u < U; ++u) {
            pin(x[u].tc);
            pin(x[u].m);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (q + u * G < n) f.put(x[u], a);
    }
}


// Value walk over one run of LM (compile-time bound) B rows, L (<= LM) of them
// live: B entry q of row k+i is s + i*n + q.  Loads of dead rows are clamped to
// row k (a cache hit) rather than branched around.
template <int LM, int UV = MHS_UNROLL, class F>
__device__ __forceinline__ void run_segment_run(const F& f, int s, int n, int gl, int G,
                                                const double (&a)[LM], int L) {
    constexpr int U = LM == 1 ? UV : MHS_RUN_UNROLL;
    int o[LM];
#pragma unroll
    for (int i = 0; i < LM; ++i) o[i] = i < L ? i * n : 0;
    // U entries per lane per batch, a short segment's tail included: indices past the
    // segment are clamped to the batch's first entry (a cache hit, not accumulated), so
    // a segment of <= U*G entries costs one load round trip, not one per entry
    for (int q0 = gl; q0 < n; q0 += U * G) {
        int c[U];
        double b[U][LM];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int q = q0 + u * G < n ? q0 + u * G : q0;
            c[u] = f.col(s + q);
#pragma unroll
            for (int i = 0; i < LM; ++i) b[u][i] = f.val(s + o[i] + q);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            pin(c[u]);
#pragma unroll
            for (int i = 0; i < LM; ++i) pin(b[u][i]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (q0 + u * G >= n) break;
            double v = a[0] * b[u][0];
#pragma unroll
            for (int i = 1; i < LM; ++i) v += i < L ? a[i] * b[u][i] : 0.0;
            f.add(c[u], v);
        }
    }
}

// Row group: the same walk feeding RM (compile-time bound) accumulators, R of them
// live: B entry q contributes sum_i a[r][i] * b_i to C row r.  One load per B row of
// the run serves all R rows.
template <int LM, int RM, bool FULL, class F>
__device__ __forceinline__ void run_segment_group(const F& f, int s, int n, int gl, int G,
                                                  const double (&a)[RM][LM], int L, int R, int stride) {
    // U entries per lane issued together: a group's wave is latency-bound on these
    // loads, and the grouped kernels' occupancy is set by LDS (registers to spare)
    constexpr int U = MHS_GRP_UNROLL;
    int o[LM];
#pragma unroll
    for (int i = 0; i < LM; ++i) o[i] = i < L ? i * n : 0;
    for (int q0 = gl; q0 < n; q0 += U * G) {
        int c[U];
        double b[U][LM];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int q = q0 + u * G < n ? q0 + u * G : q0;  // clamped: a cache hit, not accumulated
            c[u] = f.col(s + q);
#pragma unroll
            for (int i = 0; i < LM; ++i) b[u][i] = f.val(s + o[i] + q);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            pin(c[u]);  // (every load of the batch issues before the first use: one round trip)
#pragma unroll
            for (int i = 0; i < LM; ++i) pin(b[u][i]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (q0 + u * G >= n) break;
            double v[RM];
#pragma unroll
            for (int r = 0; r < RM; ++r) {
                v[r] = a[r][0] * b[u][0];
#pragma unroll
                for (int i = 1; i < LM; ++i) {
                    if constexpr (FULL)  // every visit of the sweep is a whole run: no masks
                        v[r] = fma(a[r][i], b[u][i], v[r]);
                    else
                        v[r] += i < L ? a[r][i] * b[u][i] : 0.0;
                }
            }
            f.add_rows(c[u], v, R, stride);
        }
    }
}

// One wave's chunks of an A row: [jb0, jb0 + 64), [jb0 + jstep, ...), ... below a1.
template <class F>
__device__ __forceinline__ void wave_chunk(const StagedChunk& x, int Grow, const F& f) {
    const int lane = lane_id();
    {
        // a chunk with merged runs loads LM rows per lane and sweep: wider groups
        // keep each load instruction within fewer cache lines
        const int G = (F::kValues && x.lmax > 1 && Grow < MHS_RUN_GMIN) ? MHS_RUN_GMIN : Grow;
        const int gs = 31 - __clz(G);  // G is a power of two
        const int grp = lane >> gs, gl = lane & (G - 1), ngrp = 64 >> gs;
        const int iters = (x.nh + ngrp - 1) / ngrp;
        for (int it = 0; it < iters; ++it) {
            // block distribution: groups run A entries far apart in the row at the same
            // time (neighbouring entries share B columns and would collide on the same
            // accumulator words)
            const int e = grp * iters + it;
            const int h = __shfl(x.src, e & 63);  // all lanes active at the shuffles
            const int s = __shfl(x.st, h);
            const int n0 = __shfl(x.ln, h);
            const int n = e < x.nh ? n0 : 0;
            if constexpr (F::kValues) {
                const int L = __shfl(x.L, h);
                if (x.lmax == 1) {
                    const double a[1] = {__shfl(x.av, h)};
                    run_segment_run<1>(f, s, n, gl, G, a, 1);
                } else if (x.lmax == 2) {
                    const double a[2] = {__shfl(x.av, h), __shfl(x.av, min(h + 1, 63))};
                    run_segment_run<2>(f, s, n, gl, G, a, L);
                } else if (x.lmax == 3) {
                    const double a[3] = {__shfl(x.av, h), __shfl(x.av, min(h + 1, 63)),
                                         __shfl(x.av, min(h + 2, 63))};
                    run_segment_run<3>(f, s, n, gl, G, a, L);
                } else {
                    const double a[4] = {__shfl(x.av, h), __shfl(x.av, min(h + 1, 63)),
                                         __shfl(x.av, min(h + 2, 63)), __shfl(x.av, min(h + 3, 63))};
                    run_segment_run<4>(f, s, n, gl, G, a, L);
                }
            } else {
                run_segment(f, s, n, gl, G, 0.0);
            }
        }
    }
}
template <class F>
__device__ __forceinline__ void wave_chunks(int jb0, int jstep, int a1, const int* __restrict__ Acol,
                                            const double* __restrict__ Aval, const int4* __restrict__ bmeta,
                                            bool tiles, int Grow, const F& f) {
    for (int jb = jb0; jb < a1; jb += jstep)
        wave_chunk(stage_chunk(lane_id(), jb, a1, Acol, Aval, bmeta, tiles), Grow, f);
}


// A wave's row walk with chunks staged in pairs (as for_products_group) and a lane-group
// width per chunk (chunk_group): a row's short last chunk takes wide groups.
template <class F>
__device__ __forceinline__ void wave_walk(int a0, int a1, const int* __restrict__ Acol, const double* __restrict__ Aval,
                                          const int4* __restrict__ bmeta, bool tiles, long long work, const F& f) {
    const int lane = lane_id();
    const int nA = a1 - a0;
    const int avg = nA > 0 ? (int)((work + nA - 1) / nA) : 1;
    // (tile walks pick by entries, U = 1: picking by their 2-entry batches made the groups
    // narrower, more visits at once, more same-address LDS atomics -- cage15-like symbolic +8 %)
    const int U = tiles ? 1 : MHS_UNROLL;
    for (int jb = a0; jb < a1; jb += 128) {
        ChunkLoads c0 = load_chunk_a(lane, jb, a1, Acol, Aval);
        ChunkLoads c1 = load_chunk_a(lane, jb + 64, a1, Acol, Aval);
        load_chunk_meta(c0, bmeta);
        load_chunk_meta(c1, bmeta);
        const StagedChunk x0 = finish_chunk(lane, c0, tiles, union_base(f));
        wave_chunk(x0, chunk_group(x0.nh, avg, U, tiles ? MHS_TILE_GMIN : MHS_VAL_GMIN), f);
        if (jb + 64 < a1) {
            const StagedChunk x1 = finish_chunk(lane, c1, tiles, union_base(f));
            wave_chunk(x1, chunk_group(x1.nh, avg, U, tiles ? MHS_TILE_GMIN : MHS_VAL_GMIN), f);
        }
    }
}

template <class F>
__device__ __forceinline__ void for_products(const WaveTeam&, int a0, int a1,
                                             const int* __restrict__ Acol,
                                             const double* __restrict__ Aval,
                                             const int4* __restrict__ bmeta, bool tiles, int Grow,
                                             const F& f, int4*) {
    wave_chunks(a0, 64, a1, Acol, Aval, bmeta, tiles, Grow, f);
}

// Row group (wave teams only): the head row's A entries are staged as usual and lane
// j also holds the a-values of rows head+1 .. head+R-1 (rows of one pattern are
// consecutive and equally long in A: entry j of row head+r sits at j + r*nA).
#ifndef MHS_GRP_PIPE
#define MHS_GRP_PIPE 0
#endif
// A full-group chunk whose every visit is one whole 3-row run that one load batch covers
// (n <= U*G: dof-3 FEM rows): the visits' batches are software-pipelined -- visit it+1's
// column and value loads issue before visit it's adds, so a lane group keeps one L2 round
// trip in flight under its LDS accumulation instead of waiting for each batch in turn.
template <int RM, class F>
__device__ __forceinline__ void group_chunk_pipe(const StagedChunk& x, const double (&avr)[RM], const F& f, int R,
                                                 int stride, int G, int grp, int gl, int iters) {
    constexpr int U = MHS_GRP_UNROLL;
    int c0[U], c1[U];
    double b0[U][3], b1[U][3];
    int h0, n0, h1 = 0, n1 = 0;
    auto issue = [&](int it, int& h, int& n, int (&c)[U], double (&b)[U][3]) {
        const int e = grp * iters + it;
        h = __shfl(x.src, e & 63);
        const int s = __shfl(x.st, h);
        const int nn = __shfl(x.ln, h);
        n = e < x.nh ? nn : 0;
        if (gl < n) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int q = gl + u * G < n ? gl + u * G : gl;  // clamped: a cache hit, not accumulated
                c[u] = f.col(s + q);
#pragma unroll
                for (int i = 0; i < 3; ++i) b[u][i] = f.val(s + i * n + q);
            }
        }
    };
    issue(0, h0, n0, c0, b0);
    for (int it = 0; it < iters; ++it) {
        if (it + 1 < iters) issue(it + 1, h1, n1, c1, b1);
        double a[RM][3];
#pragma unroll
        for (int r = 0; r < RM; ++r)
#pragma unroll
            for (int i = 0; i < 3; ++i) a[r][i] = __shfl(avr[r], min(h0 + i, 63));
        if (gl < n0) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (gl + u * G >= n0) break;
                double v[RM];
#pragma unroll
                for (int r = 0; r < RM; ++r) {
                    v[r] = a[r][0] * b0[u][0];
                    v[r] = fma(a[r][1], b0[u][1], v[r]);
                    v[r] = fma(a[r][2], b0[u][2], v[r]);
                }
                f.add_rows(c0[u], v, R, stride);
            }
        }
        h0 = h1;
        n0 = n1;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            c0[u] = c1[u];
#pragma unroll
            for (int i = 0; i < 3; ++i) b0[u][i] = b1[u][i];
        }
    }
}

template <int RC, class F>
__device__ __forceinline__ void group_chunk_r(const StagedChunk& x, const double (&avr)[RG_MAX], int avg, const F& f,
                                              int Rrt, int stride) {
    constexpr int RM = RG_MAX;
    const int R = RC ? RC : Rrt;  // RC: the group size as a constant (no per-row branches in the adds)
    const int lane = lane_id();
    // the chunk's own lane-group width (a row's short last chunk takes wide groups: one
    // load batch for its few visits instead of the row's batches per visit)
    const int G = chunk_group(x.nh, avg, MHS_GRP_UNROLL, x.lmax > 1 ? MHS_RUN_GMIN : MHS_VAL_GMIN);
    const int gs = 31 - __clz(G);
    const int grp = lane >> gs, gl = lane & (G - 1), ngrp = 64 >> gs;
    const int iters = (x.nh + ngrp - 1) / ngrp;
    if constexpr (MHS_GRP_PIPE && RC == RG_MAX && RG_MAX == 3) {
        if (x.lmax == 3 && iters > 1) {
            // lane e < nh holds visit e's head: every visit a whole 3-row run in one batch?
            const int hv = x.src;
            const int Lv = __shfl(x.L, hv), nv = __shfl(x.ln, hv);
            if (__ballot(lane < x.nh && nv > 0 && (Lv != 3 || nv > MHS_GRP_UNROLL * G)) == 0) {
                group_chunk_pipe<RM>(x, avr, f, R, stride, G, grp, gl, iters);
                return;
            }
        }
    }
    for (int it = 0; it < iters; ++it) {
        const int e = grp * iters + it;
        const int h = __shfl(x.src, e & 63);
        const int sb = __shfl(x.st, h);
        const int n0 = __shfl(x.ln, h);
        const int n = e < x.nh ? n0 : 0;
        const int L = __shfl(x.L, h);
        if (x.lmax == 1) {
            double a[RM][1];
#pragma unroll
            for (int r = 0; r < RM; ++r) a[r][0] = __shfl(avr[r], h);
            run_segment_group<1, RM, true>(f, sb, n, gl, G, a, 1, R, stride);
        } else {
            double a[RM][3];
#pragma unroll
            for (int r = 0; r < RM; ++r)
#pragma unroll
                for (int i = 0; i < 3; ++i) a[r][i] = __shfl(avr[r], min(h + i, 63));
            if (__ballot(n > 0 && L != 3) == 0)
                run_segment_group<3, RM, true>(f, sb, n, gl, G, a, 3, R, stride);
            else
                run_segment_group<3, RM, false>(f, sb, n, gl, G, a, L, R, stride);
        }
    }
}
template <class F>
__device__ __forceinline__ void group_chunk(const StagedChunk& x, const double (&avr)[RG_MAX], int avg, const F& f,
                                            int R, int stride) {
    if (R == RG_MAX) {  // full groups (FEM dof triples): no per-row branches (cant-like numeric -3 %)
        group_chunk_r<RG_MAX>(x, avr, avg, f, R, stride);
        return;
    }
    group_chunk_r<0>(x, avr, avg, f, R, stride);
}

// Row group (wave teams only): the head row's A entries are staged as usual and lane
// j also holds the a-values of rows head+1 .. head+R-1 (rows of one pattern are
// consecutive and equally long in A: entry j of row head+r sits at j + r*nA).  Chunks
// are staged in pairs: both chunks' A loads and then both bmeta loads are issued before
// the first is walked, so the second chunk's two dependent round trips overlap the
// first chunk's sweeps (a 69-entry FEM row: 63 + 6 entries).
struct GroupPair {
    ChunkLoads c0, c1;
    double avr0[RG_MAX], avr1[RG_MAX];
};
// the A-side loads of the pair at jb (chunks of MHS_GRP_CHUNK entries: 63 keeps the 3-entry
// runs of dof-3 rows whole -- a chunk edge cuts a run: a 1-entry visit in one chunk, a
// 2-entry one in the next, masked sweeps)
__device__ __forceinline__ void group_pair_a(GroupPair& p, int jb, int a1, const int* __restrict__ Acol,
                                             const double* __restrict__ Aval, int R, int nA) {
    const int lane = lane_id();
    const int ce0 = min(a1, jb + MHS_GRP_CHUNK), jb1 = ce0, ce1 = min(a1, jb1 + MHS_GRP_CHUNK);
    p.c0 = load_chunk_a(lane, jb, ce0, Acol, Aval);
    p.avr0[0] = p.c0.av;
#pragma unroll
    for (int r = 1; r < RG_MAX; ++r) p.avr0[r] = (jb + lane < ce0 && r < R) ? Aval[jb + lane + r * nA] : 0.0;
    p.c1 = load_chunk_a(lane, jb1, ce1, Acol, Aval);
    p.avr1[0] = p.c1.av;
#pragma unroll
    for (int r = 1; r < RG_MAX; ++r) p.avr1[r] = (jb1 + lane < ce1 && r < R) ? Aval[jb1 + lane + r * nA] : 0.0;
}
__device__ __forceinline__ void group_pair_meta(GroupPair& p, const int4* __restrict__ bmeta) {
    load_chunk_meta(p.c0, bmeta);
    load_chunk_meta(p.c1, bmeta);
}
// The walk of a row group whose first pair `p` is loaded (A and bmeta) by the caller -- its
// round trips overlap the row's tile-table and rank phases (num_row_body).
template <class F>
__device__ __forceinline__ void for_products_group(GroupPair& p, int a0, int a1, const int* __restrict__ Acol,
                                                   const double* __restrict__ Aval,
                                                   const int4* __restrict__ bmeta, int avg, const F& f,
                                                   int R, int nA, int stride) {
    static_assert(MHS_RUN_MAX <= 3, "grouped walks merge runs of up to 3 B rows");
    const int lane = lane_id();
    const int ub = union_base(f);
    for (int jb = a0; jb < a1; jb += 2 * MHS_GRP_CHUNK) {
        if (jb != a0) {
            group_pair_a(p, jb, a1, Acol, Aval, R, nA);
            group_pair_meta(p, bmeta);
        }
        const int jb1 = min(a1, jb + MHS_GRP_CHUNK);
        group_chunk(finish_chunk(lane, p.c0, false, ub), p.avr0, avg, f, R, stride);
        if (jb1 < a1) group_chunk(finish_chunk(lane, p.c1, false, ub), p.avr1, avg, f, R, stride);
    }
}

// A staged sub-chunk walked flattened: its nloc visits' B segments laid end to end
// (e[v] = {B start, length, A index, inclusive prefix of the lengths}), product p of
// tot to thread p mod T; the visit of p by a binary search of the prefixes in LDS.
// U products per thread issue their loads together (clamped, not branched around).
template <int T, class F>
__device__ __forceinline__ void flat_chunk(const F& f, const int4* e, int nloc, int tot,
                                           const double* __restrict__ Aval) {
    constexpr int U = 2;
    for (int p0 = threadIdx.x; p0 < tot; p0 += U * T) {
        typename F::Item x[U];
        int own[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int p = p0 + u * T < tot ? p0 + u * T : p0;
            int lo = 0, hi = nloc - 1;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (e[mid].w > p) hi = mid;
                else lo = mid + 1;
            }
            const int4 v = e[lo];
            own[u] = v.z;
            x[u] = f.load(v.x + p - (v.w - v.y));
        }
        double a[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if constexpr (F::kValues) {
                a[u] = Aval[own[u]];
                pin(x[u].c);
                pin(x[u].v);
            } else {
                a[u] = 0.0;
                pin(x[u].tc);
                pin(x[u].m);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (p0 + u * T < tot) f.put(x[u], a[u]);
    }
}

template <int T, bool GM, class F>
__device__ __forceinline__ void for_products(const BlockTeam<T, GM>&, int a0, int a1,
                                             const int* __restrict__ Acol,
                                             const double* __restrict__ Aval,
                                             const int4* __restrict__ bmeta, bool tiles, int Grow,
                                             const F& f, int4* stage) {
    // Waves 0..S-1 each stage one 64-entry sub-chunk at once (their Acol -> bmeta load
    // chains overlap; one barrier per 64*S A entries -- rows with thousands of short A
    // entries were bound by one chunk's load chain per barrier).  Sub-chunk s:
    // stage[s*65] = {visits, longest run, group width}; stage[s*65+1+e] = {B start,
    // length, A index, run length}.
    constexpr int S = T >= 1024 ? STAGE_SUBS_1024 : (T / 64) < STAGE_SUBS ? (T / 64) : STAGE_SUBS;
    const int wv = threadIdx.x >> 6;
    for (int jr = a0; jr < a1; jr += 64 * S) {
        if (wv < S) {
            const int jb = jr + 64 * wv;
            const int lane = lane_id();
            int4* sg = stage + wv * 65;
            const StagedChunk x = stage_chunk(lane, jb, a1, Acol, nullptr, bmeta, tiles);
            const int h = x.src;
            const int st = __shfl(x.st, h), ln = __shfl(x.ln, h), L = __shfl(x.L, h);
            const int G = (F::kValues && x.lmax > 1 && Grow < MHS_RUN_GMIN) ? MHS_RUN_GMIN : Grow;
            // skewed chunk (no runs; its longest B segment is over twice a lane group's
            // fair share, e.g. a hub row among short ones): walk it flattened instead
            const int lnv = lane < x.nh ? ln : 0;
            const int incl = wave_incl_scan(lnv);
            const int tot = __shfl(incl, 63);
            const int mx = wave_max(lnv);
            const int ngrp = T / G < x.nh ? T / G : x.nh;
            const bool flat = T <= 256 && x.lmax == 1 && ngrp > 1 && (long long)mx * ngrp > 2LL * tot;
            if (lane < x.nh) sg[1 + lane] = make_int4(st, ln, jb + h, flat ? incl : L);
            if (lane == 0) sg[0] = make_int4(jb < a1 ? x.nh : 0, x.lmax, G, flat ? tot : -1);
        }
        __syncthreads();
        for (int sc = 0; sc < S; ++sc) {
            const int4* sg = stage + sc * 65;
            const int4 hd = sg[0];
            const int nloc = hd.x, lmax = hd.y, G = hd.z;
            if (nloc == 0) break;  // sub-chunks past the row's end are empty (and all later ones)
            if constexpr (T <= 256) {  // (the 1024-thread kernels would spill)
                if (hd.w >= 0) {
                    flat_chunk<T>(f, sg + 1, nloc, hd.w, Aval);
                    continue;
                }
            }
            const int gs = 31 - __clz(G);  // G is a power of two
            const int grp = threadIdx.x >> gs, gl = threadIdx.x & (G - 1), ngrp = T >> gs;  // ngrp <= 64
            const int iters = (nloc + ngrp - 1) / ngrp;
            for (int it = 0; it < iters; ++it) {
                const int e = grp * iters + it;
                if (e >= nloc) continue;
                const int4 v = sg[1 + e];
                if constexpr (F::kValues) {
                    if (lmax == 1) {
                        const double a[1] = {Aval[v.z]};
                        run_segment_run<1, MHS_UNROLL_BLOCK>(f, v.x, v.y, gl, G, a, 1);
                    } else if (lmax == 2) {
                        const double a[2] = {Aval[v.z], Aval[v.z + (v.w > 1)]};
                        run_segment_run<2>(f, v.x, v.y, gl, G, a, v.w);
                    } else if (lmax == 3) {
                        const double a[3] = {Aval[v.z], Aval[v.z + (v.w > 1)], Aval[v.z + 2 * (v.w > 2)]};
                        run_segment_run<3>(f, v.x, v.y, gl, G, a, v.w);
                    } else {
                        const double a[4] = {Aval[v.z], Aval[v.z + (v.w > 1)], Aval[v.z + 2 * (v.w > 2)],
                                             Aval[v.z + 3 * (v.w > 3)]};
                        run_segment_run<4>(f, v.x, v.y, gl, G, a, v.w);
                    }
                } else {
                    run_segment(f, v.x, v.y, gl, G, 0.0);
                }
            }
        }
        __syncthreads();
    }
}

// Block teams of 1024 threads, per-wave pieces (round 5, MHS_PIECES): the row's A entries cut
// into 16 contiguous pieces, each wave walking its own in 64-entry chunks with a lane-group width
// per chunk, no stage and no barrier.  The staged walk above runs lane groups of at least T/64
// lanes, so at most 64 A entries per dependent load round trip and S of them in sequence per
// barrier: webbase-like's hub rows (4,400 entries of ~4 products) took ~84 round trips a walk
// (row stamps: ~170 k cycles per walk).  The group width counts the chunk's longest segment too
// (a hub column's long B row among short ones).  (For the 256-thread kernels the pieces measured
// slower: scircuit-like +3 %, cant-s1-like +4 %.)
constexpr int MHS_PIECES = 1;
// (round 5: single wave rows' first A chunk loaded before the tile table, as row groups do --
// cage15-like +5 %, offshore-like +10 %, cop20k-like +4 %: the 5 KiB hash kernel spills at 8 waves)
constexpr int MHS_PIECE_UNROLL = 2;  // B entries per lane issued together in a piece's value walk (registers)
__device__ __forceinline__ int chunk_group_mx(int nh, int avg, int mx, int U, int gmin) {
    int best = gmin, bc = INT_MAX;
    for (int g = gmin; g <= 64; g <<= 1) {
        const int ng = 64 / g;
        const int c0 = ((nh + ng - 1) / ng) * ((avg + g * U - 1) / (g * U));
        const int c1 = (mx + g * U - 1) / (g * U);
        const int c = c0 > c1 ? c0 : c1;
        if (c <= bc) {
            bc = c;
            best = g;
        }
    }
    return best;
}
template <int T, class F>
__device__ __forceinline__ void for_products_pieces(int a0, int a1, const int* __restrict__ Acol,
                                                    const double* __restrict__ Aval, const int4* __restrict__ bmeta,
                                                    bool tiles, int avg, const F& f) {
    constexpr int NW = T / 64;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int nA = a1 - a0;
    const int p0 = a0 + (int)((long long)nA * wv / NW), p1 = a0 + (int)((long long)nA * (wv + 1) / NW);
    const int lane = lane_id();
    const int U = tiles ? MHS_TILE_UNROLL : MHS_PIECE_UNROLL;
    for (int jb = p0; jb < p1; jb += 64) {
        ChunkLoads c = load_chunk_a(lane, jb, p1, Acol, Aval);
        load_chunk_meta(c, bmeta);
        // every entry its own visit (no run sweeps: the 1024-thread kernels' registers)
        StagedChunk x;
        x.st = c.in ? c.m.x : 0;
        x.ln = c.in ? (tiles ? meta_ntiles(c.m) : c.m.y) : 0;
        x.av = c.av;
        const unsigned long long Hm = __ballot(c.in);
        x.nh = __popcll(Hm);
        const int mx = wave_max(x.ln);
        const int G = chunk_group_mx(x.nh, avg, mx, U, tiles ? MHS_TILE_GMIN : MHS_VAL_GMIN);
        const int gs = 31 - __clz(G);  // G is a power of two
        const int grp = lane >> gs, gl = lane & (G - 1), ngrp = 64 >> gs;
        const int iters = (x.nh + ngrp - 1) / ngrp;
        for (int it = 0; it < iters; ++it) {
            const int e = grp * iters + it;  // (entries in lane order: the chunk's lanes [0, nh) hold them)
            const int st = __shfl(x.st, e & 63);
            const int n0 = __shfl(x.ln, e & 63);
            const double av = __shfl(x.av, e & 63);
            const int n = e < x.nh ? n0 : 0;
            if constexpr (F::kValues) {
                const double avs[1] = {av};
                run_segment_run<1, MHS_PIECE_UNROLL>(f, st, n, gl, G, avs, 1);
            } else {
                run_segment(f, st, n, gl, G, 0.0);
            }
        }
    }
}
struct WideTiles;
struct WideAccum;
template <class F>
__device__ constexpr bool piece_walk_ok() {
    return MHS_PIECES && !std::is_same<F, WideTiles>::value && !std::is_same<F, WideAccum>::value;
}

// Lane groups (a flattened walk -- 64 consecutive products per batch, the owner of each
// found by a search over the chunk's prefix of segment lengths -- measured slower: its
// per-batch owner search costs more instructions than it saves in coalescing).
template <class Team, class F>
__device__ __forceinline__ void walk_products(const Team& tm, int a0, int a1,
                                              const int* __restrict__ Acol,
                                              const double* __restrict__ Aval,
                                              const int4* __restrict__ bmeta, bool tiles,
                                              long long work, const F& f, int4* stage) {
    const int nA = a1 - a0;
    if constexpr (Team::size == 64 && F::kPairs) {
        wave_walk(a0, a1, Acol, Aval, bmeta, tiles, work, f);
        return;
    }
    if constexpr (Team::size >= 1024 && piece_walk_ok<F>()) {
        const int avg = nA > 0 ? (int)((work + nA - 1) / nA) : 1;
        if (nA >= 2 * Team::size) {  // (rows of at least two 64-entry chunks a wave)
            for_products_pieces<Team::size>(a0, a1, Acol, Aval, bmeta, tiles, avg, f);
            return;
        }
    }
    for_products(tm, a0, a1, Acol, Aval, bmeta, tiles,
                 pick_group(work, nA, Team::size, tiles ? MHS_TILE_GMIN : MHS_VAL_GMIN,
                            tiles ? 1 : (Team::size > 64 ? MHS_UNROLL_BLOCK : MHS_UNROLL)),  // (tile walks: by entries)
                 f, stage);
}

// ---------------------------------------------------------- tile tables ---
// Insert every B tile of the row's products into the tile table E:
//   direct: slot = tile - lo (the row's tile span), keys implicit;
//   hash:   open addressing, Fibonacci hash, linear probe, CAS on the key.
// Tables hold >= 2x the distinct tiles, so an insert always finds a slot.
struct TileBuild {
    static constexpr bool kValues = false;
    static constexpr bool kUnion = false;
    static constexpr bool kPairs = false;  // wave walks may stage chunk pairs (registers)
    TileEntry* E;
    bool direct;
    int lo, H;
    const int* __restrict__ btcol;
    const unsigned long long* __restrict__ btmask;
    struct Item {
        int tc;
        unsigned long long m;
    };
    __device__ __forceinline__ Item load(int i) const { return Item{btcol[i], btmask[i]}; }
    __device__ __forceinline__ void put(const Item& x, double) const {
        if (direct) {
            atomicOr(&E[x.tc - lo].mask, x.m);
        } else {
            int s = hslot(x.tc, H);
            MHS_GUARD_DECL;
            for (;;) {
                const int old = atomicCAS(&E[s].key, -1, x.tc);
                if (old == -1 || old == x.tc) {
                    atomicOr(&E[s].mask, x.m);
                    break;
                }
                MHS_GUARD(H, 2, x.tc);
                probe_conflict();
                s = hnext(s, H);
            }
        }
    }
};

// Numeric accumulate, one functor per row mode (compile-time: no per-product
// mode branch).  DENSE: acc[col - colbase].  DIRECT / HASH: product (c, a*b)
// -> acc[base(tile(c)) + popc(mask & below(c))], the tile found direct-mapped
// or by probing (always present: it was inserted by the tile build).
// B gathers: O32 -- the value arrays' byte offsets fit 32 bits (nnz(B) + union rows < 2^29, the
// host's choice): a load is one global_load with an SGPR base and a 32-bit VGPR offset (no 64-bit
// address arithmetic: two VALU ops and two VGPRs fewer per load in the product walks)
template <bool O32, class T>
__device__ __forceinline__ T ld_idx(const T* __restrict__ base, int i) {
    if constexpr (O32) return *(const T*)((const char*)base + (unsigned)i * (unsigned)sizeof(T));
    else return base[i];
}
template <bool GM, int MODE, bool O32 = false>
struct Accum {
    static constexpr bool kValues = true;
    static constexpr bool kUnion = true;  // near union runs (see finish_chunk)
    static constexpr bool kPairs = MODE != NM_HASH;  // (the hash kernels run at 64 VGPRs: pairs spill)
    const TileEntry* E;
    double* acc;
    int lo, H, colbase;
    const int* __restrict__ Bcol;
    const double* __restrict__ Bval;
    int ubase;          // near union runs (NumArgs::ubase; 0: none)
    struct Item {
        int c;
        double v;
    };
    __device__ __forceinline__ Item load(int i) const { return Item{ld_idx<O32>(Bcol, i), ld_idx<O32>(Bval, i)}; }
    __device__ __forceinline__ int col(int i) const { return ld_idx<O32>(Bcol, i); }
    __device__ __forceinline__ double val(int i) const { return ld_idx<O32>(Bval, i); }
    __device__ __forceinline__ void put(const Item& x, double a) const { add(x.c, a * x.v); }
    // acc[column c] += v
    __device__ __forceinline__ void add(int c, double v) const { acc_add<GM>(&acc[index(c)], v); }
    // row group: accumulator slice r (stride `stride` doubles) of column c += v[r], r < R
    template <int RM>
    __device__ __forceinline__ void add_rows(int c, const double (&v)[RM], int R, int stride) const {
        const int idx = index(c);
#pragma unroll
        for (int r = 0; r < RM; ++r)
            if (r < R) acc_add<GM>(&acc[idx + r * stride], v[r]);
    }
    __device__ __forceinline__ int index(int c) const {
        const Item x{c, 0.0};
        int idx;
        if constexpr (MODE == NM_DENSE) {
            idx = x.c - colbase;
        } else {
            const int tc = x.c >> TILE_SHIFT;
            int s;
            if constexpr (MODE == NM_DIRECT) {
                s = tc - lo;
            } else {
                s = hslot(tc, H);
            }
            uint4 q = *reinterpret_cast<const uint4*>(&E[s]);  // one ds_read_b128: mask, base, key
            if constexpr (MODE == NM_HASH) {
                MHS_GUARD_DECL;
                while ((int)q.w != tc) {
                    MHS_GUARD(H, 1, tc);
                    probe_conflict();
                    s = hnext(s, H);
                    q = *reinterpret_cast<const uint4*>(&E[s]);
                }
            }
            const unsigned long long mask = ((unsigned long long)q.y << 32) | q.x;
            const unsigned long long below = (1ull << (x.c & (TILE_BITS - 1))) - 1;
            idx = (int)q.z + __popcll(mask & below);
        }
        return idx;
    }
};

template <class Team>
__device__ __forceinline__ void build_tiles(const Team& tm, TileEntry* E, bool direct, int lo,
                                            int H, int a0, int a1,
                                            const int* __restrict__ Acol,
                                            const int4* __restrict__ bmeta,
                                            const int* __restrict__ btcol,
                                            const unsigned long long* __restrict__ btmask,
                                            int tflop, int4* stage) {
    const TileBuild f{E, direct, lo, H, btcol, btmask};
    walk_products(tm, a0, a1, Acol, nullptr, bmeta, true, tflop, f, stage);
}

template <class Team>
__device__ __forceinline__ void clear_tiles(const Team& tm, TileEntry* E, int H) {
    for (int s = tm.rank(); s < H; s += Team::size) {
        TileEntry z;
        z.mask = 0;
        z.base = 0;
        z.key = -1;
        E[s] = z;
    }
}

constexpr int WIDE_WT = 16384;  // tiles per window: 1 M columns (masks 128 KiB + bases 16 KiB)
static_assert(WIDE_WT * 9 <= B1024_BYTES, "a wide window fits the 1024-thread kernel's LDS");

// Wide-row tile walk: OR each B tile inside the window [w0, w1) into a dense mask array.
struct WideTiles {
    static constexpr bool kValues = false;
    static constexpr bool kUnion = false;
    static constexpr bool kPairs = false;  // wave walks may stage chunk pairs (registers)
    unsigned long long* masks;
    int w0, w1;
    const int* __restrict__ btcol;
    const unsigned long long* __restrict__ btmask;
    struct Item {
        int tc;
        unsigned long long m;
    };
    __device__ __forceinline__ Item load(int i) const { return Item{btcol[i], btmask[i]}; }
    __device__ __forceinline__ void put(const Item& x, double) const {
        if (x.tc >= w0 && x.tc < w1) atomicOr(&masks[x.tc - w0], x.m);
    }
};

// ------------------------------------------------------- span bitmap rank ---
// Rows too big for a 256-thread block's hash table (hub rows of power-law matrices: a
// few thousand distinct tiles scattered over a span of 10^4..10^5 tiles): a bit per tile
// of the row's span in LDS and a popcount prefix per 64-bit word give every tile its rank
// among the row's tiles in O(1) -- no hash, no probe, no CAS, no tile sort -- and per-rank
// arrays (mask, key, C-row base) hold the row compactly in column order.
//   walk 1  SpanBits      set the bit of every B tile of the row's products
//   scan    wpre[w]       = set bits in words < w
//   walk 2  RankedMasks   OR each B tile's mask into msk[rank], key[rank] = tile
// LDS: span/64 * 12 bytes + 16 bytes per distinct tile (+ 8 per C entry in numeric).
__device__ __forceinline__ int span_rank(const unsigned long long* bm, const int* wpre, int d) {
    return wpre[d >> 6] + (int)__popcll(bm[d >> 6] & ((1ull << (d & 63)) - 1));
}
struct SpanBits {
    static constexpr bool kValues = false;
    static constexpr bool kUnion = false;
    static constexpr bool kPairs = false;  // wave walks may stage chunk pairs (registers)
    unsigned long long* bm;
    int lo;
    const int* __restrict__ btcol;
    struct Item {
        int tc;
        unsigned long long m;
    };
    __device__ __forceinline__ Item load(int i) const { return Item{btcol[i], 0ull}; }
    __device__ __forceinline__ void put(const Item& x, double) const {
        const int d = x.tc - lo;
        atomicOr(&bm[d >> 6], 1ull << (d & 63));
    }
};
struct RankedMasks {
    static constexpr bool kValues = false;
    static constexpr bool kUnion = false;
    static constexpr bool kPairs = false;  // wave walks may stage chunk pairs (registers)
    const unsigned long long* bm;
    const int* wpre;
    unsigned long long* msk;
    int2* kb;  // (key, base) per rank
    int lo;
    const int* __restrict__ btcol;
    const unsigned long long* __restrict__ btmask;
    struct Item {
        int tc;
        unsigned long long m;
    };
    __device__ __forceinline__ Item load(int i) const { return Item{btcol[i], btmask[i]}; }
    __device__ __forceinline__ void put(const Item& x, double) const {
        const int r = span_rank(bm, wpre, x.tc - lo);
        atomicOr(&msk[r], x.m);
        kb[r].x = x.tc;  // every writer of rank r stores the same key
    }
};
__host__ __device__ inline long long span_bits_bytes(int span) {
    const long long nw = ((long long)span + 63) >> 6;
    return align16(nw * 8) + align16(nw * 4);
}

// Spill lists: the (mask, key) tile list of a row with more tiles than its row-cache slot
// holds (hub rows: hundreds to thousands of tiles), in one bump-allocated region; numeric
// then skips its tile walk (for span-ranked rows: both).  lofs[row] = the list's offset, or
// -1 when the region was full; written by symbolic for exactly the rows numeric asks about
// (not cached, t > mc_list), so it needs no initialisation.
struct SpillLists : SpillArea {
    __host__ __device__ SpillLists() : SpillArea{} {}
    __host__ __device__ SpillLists(const SpillArea& x) : SpillArea(x) {}
};
__device__ __forceinline__ bool spill_row(int span, int tflop, int t, int mc_list) {
    return !mcached(span, tflop) && t > mc_list;
}
// Reserve t entries (team-uniform result: offset, or -1 when full) and record it for R rows.
// The region is cut into SPILL_PARTS partitions with a bump counter each (row % SPILL_PARTS
// picks one, counters 64 B apart): one counter for every spilling row serialised the
// symbolic phase on its atomics (wb-edu-like: hundreds of thousands of rows).
__device__ __forceinline__ int spill_reserve_off(const SpillLists& sp, int row, int t) {
    const int p = row & (SPILL_PARTS - 1);
    const long long part = sp.cap / SPILL_PARTS;
    const int o = atomicAdd(sp.top + p * CURSOR_STRIDE, t);
    return (long long)o + t <= part ? (int)(p * part + o) : -1;
}
template <class Team>
__device__ __forceinline__ int spill_reserve(const Team& tm, const SpillLists& sp, int row, int R, int t) {
    int off = -1;
    if (tm.rank() == 0 && sp.mask) off = spill_reserve_off(sp, row, t);
    off = tm.bcast0(off);
    if (tm.rank() < R) sp.lofs[row + tm.rank()] = off;
    return off;
}

// ------------------------------------------------------------- symbolic ---
struct SymArgs {
    int M;
    const int* Aptr;
    const int* Acol;
    const int4* bmeta;
    const int* btcol;
    const unsigned long long* btmask;
    const int* rtflop;
    const int* rlo;
    const int* rhi;
    const int* list;  // bin x's rows at list + (x-1)*M, count in stats->sym_count[x]
    const Stats* stats;
    const unsigned char* grp;  // row groups: R of every listed head
    int bin;
    int* Cptr;
    int* ctiles;
    char* gscratch;
    long long gbytes;  // per block
    unsigned long long* mcache;
    int mc_list, mc_stride;  // row cache: tile-list cap, words per row
    int* cursors;            // all row cursors (slot NUM_NB + bin: k_sym_rare queues)
    SpillLists sp;           // tile lists of rows past the row cache's cap
};

// Symbolic tile table (counts only, no ranks): masks Mk[H], then -- hashed -- keys Kk[H]:
// 8 or 12 bytes a slot (sym_need), so more rows fit the small-table wave bin.
struct SymTileBuild {
    static constexpr bool kValues = false;
    static constexpr bool kUnion = false;
    static constexpr bool kPairs = true;  // wave walks may stage chunk pairs (registers)
    unsigned long long* Mk;
    int* Kk;
    bool direct;
    int lo, H;
    const int* __restrict__ btcol;
    const unsigned long long* __restrict__ btmask;
    struct Item {
        int tc;
        unsigned long long m;
    };
    __device__ __forceinline__ Item load(int i) const { return Item{btcol[i], btmask[i]}; }
    __device__ __forceinline__ void put(const Item& x, double) const {
        if (direct) {
            atomicOr(&Mk[x.tc - lo], x.m);
        } else {
            int s = hslot(x.tc, H);
            MHS_GUARD_DECL;
            for (;;) {
                const int old = atomicCAS(&Kk[s], -1, x.tc);
                if (old == -1 || old == x.tc) {
                    atomicOr(&Mk[s], x.m);
                    break;
                }
                MHS_GUARD(H, 3, x.tc);
                probe_conflict();
                s = hnext(s, H);
            }
        }
    }
};

// A symbolic row's scalars (loaded in the row, or batch-prefetched by sym_wave_rows)
struct SymRow {
    int row, lo, hi, tflop, a0, a1;
};
template <class Team>
__device__ void sym_row_s(const Team& tm, const SymArgs& a, const SymRow& r, TileEntry* E, int4* stage);
template <class Team>
__device__ __forceinline__ void sym_row(const Team& tm, const SymArgs& a, int row, TileEntry* E, int4* stage) {
    SymRow r;
    r.row = row;
    r.lo = __builtin_amdgcn_readfirstlane(a.rlo[row]);
    r.hi = __builtin_amdgcn_readfirstlane(a.rhi[row]);
    r.tflop = __builtin_amdgcn_readfirstlane(a.rtflop[row]);
    r.a0 = __builtin_amdgcn_readfirstlane(a.Aptr[row]);
    r.a1 = __builtin_amdgcn_readfirstlane(a.Aptr[row + 1]);
    sym_row_s(tm, a, r, E, stage);
}
template <class Team>
__device__ void sym_row_s(const Team& tm, const SymArgs& a, const SymRow& r, TileEntry* E, int4* stage) {
    const int row = r.row, lo = r.lo, hi = r.hi, tflop = r.tflop;
    MHS_SSTAMP0();
    const int span = hi - lo + 1;
    const bool direct = sym_direct(span, tflop);
    const int H = direct ? span : hash_slots(tflop < span ? tflop : span);
    unsigned long long* Mk = reinterpret_cast<unsigned long long*>(E);
    int* Kk = reinterpret_cast<int*>(Mk + H);
    for (int s = tm.rank(); s < H; s += Team::size) {
        Mk[s] = 0ull;
        if (!direct) Kk[s] = -1;
    }
    tm.sync();
    MHS_SSTAMP(0);
    walk_products(tm, r.a0, r.a1, a.Acol, nullptr, a.bmeta, true, tflop,
                  SymTileBuild{Mk, Kk, direct, lo, H, a.btcol, a.btmask}, stage);
    tm.sync();
    MHS_SSTAMP(1);
    long long n = 0;
    int t = 0;
    for (int s = tm.rank(); s < H; s += Team::size) {
        const unsigned long long m = Mk[s];
        n += __popcll(m);
        t += m != 0;
    }
    n = tm.sum(n);
    t = tm.sum(t);
    MHS_SSTAMP(2);
    const int R = __builtin_amdgcn_readfirstlane((int)a.grp[row]);  // the group's rows share the pattern
    if (tm.rank() < R) {
        a.Cptr[row + tm.rank()] = (int)n;
        a.ctiles[row + tm.rank()] = t;
    }
    // numeric reuses the OR'd masks of narrow rows (span <= 32 < team size: one store per lane)
    const int r_ = tm.rank();
    if (direct && span <= MCACHE_SPAN && r_ < span && a.mcache) {
        const unsigned long long m = Mk[r_];
        for (int g = 0; g < R; ++g) st_cache(&a.mcache[(size_t)(row + g) * a.mc_stride + r_], m);
    }
    // ... and the compacted (key, mask) list of the other rows with few tiles
    if (a.mcache && mlisted(span, tflop, t, a.mc_list) && r_ < 64) {  // the first wave compacts the table
        const int lane = lane_id();
        int k = 0;
        for (int s0 = 0; s0 < H; s0 += 64) {
            const int sl = s0 + lane;
            const unsigned long long m = sl < H ? Mk[sl] : 0ull;
            const bool occ = m != 0ull;
            const unsigned long long bal = __ballot(occ);
            if (occ) {
                const int pos = k + __popcll(bal & lanemask_lt());
                const int key = direct ? lo + sl : Kk[sl];
                for (int g = 0; g < R; ++g) {
                    unsigned long long* slot = a.mcache + (size_t)(row + g) * a.mc_stride;
                    st_cache(&slot[pos], m);
                    st_cache(&reinterpret_cast<int*>(slot + a.mc_list)[pos], key);
                }
            }
            k += __popcll(bal);
        }
    }
    // ... rows past the slot: a spill list (one copy for the group: lofs points every row at it)
    if (a.mcache && spill_row(span, tflop, t, a.mc_list)) {
        const int off = spill_reserve(tm, a.sp, row, R, t);
        if (off >= 0) {
            // every wave compacts its share of the slots (the list is unordered): a wave
            // team walks all of them, a block's waves take places with an LDS counter
            // (the stage area is free after the walk)
            const int lane = lane_id();
            int* ctr = reinterpret_cast<int*>(stage);
            if (Team::size > 64 && tm.rank() == 0) *ctr = 0;
            tm.sync();
            int k = off;
            for (int s0 = tm.rank() & ~63; s0 < H; s0 += Team::size) {
                const int sl = s0 + lane;
                const unsigned long long m = sl < H ? Mk[sl] : 0ull;
                const bool occ = m != 0ull;
                const unsigned long long bal = __ballot(occ);
                if (Team::size > 64) {
                    int at = 0;
                    if (lane == 0 && bal) at = atomicAdd(ctr, __popcll(bal));
                    k = off + __shfl(at, 0);
                }
                if (occ) {
                    const int pos = k + __popcll(bal & lanemask_lt());
                    st_cache(&a.sp.mask[pos], m);
                    st_cache(&a.sp.key[pos], direct ? lo + sl : Kk[sl]);
                }
                if (Team::size == 64) k += __popcll(bal);
            }
        }
    }
    tm.sync();
    MHS_SSTAMP(3);
}

// the small-table wave bin, blocks [0, nb) of a grid
template <int BYTES>
__device__ __forceinline__ void sym_wave_rows(const SymArgs& a, int bid, int nb) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int w = threadIdx.x >> 6;
    TileEntry* E = (TileEntry*)(smem + w * BYTES + WAVE_HDR);
    const int count = a.stats->sym_count[a.bin];
    const int* list = a.list + (long long)(a.bin - 1) * a.M;
    WaveTeam tm;
    // the wave's next 64 rows and their scalars in one batch (lane j: the row at step j), read
    // back with readlane: the list -> row scalars round trips leave the rows' chains
    const int lane = lane_id();
    const RowWalk rw(count, WPB, w, bid, nb);
    for (int b0 = rw.first; b0 < rw.end; b0 += 64 * rw.stride) {
        const int li = b0 + lane * rw.stride;
        const bool in = li < rw.end;
        const int row = in ? list[li] : 0;
        const int lo = in ? a.rlo[row] : 0, hi = in ? a.rhi[row] : 0, tf = in ? a.rtflop[row] : 0;
        const int a0 = in ? a.Aptr[row] : 0, a1 = in ? a.Aptr[row + 1] : 0;
        const int nrows = min(64, (rw.end - b0 + rw.stride - 1) / rw.stride);
        for (int j = 0; j < nrows; ++j) {
            SymRow r;
            r.row = __builtin_amdgcn_readlane(row, j);
            r.lo = __builtin_amdgcn_readlane(lo, j);
            r.hi = __builtin_amdgcn_readlane(hi, j);
            r.tflop = __builtin_amdgcn_readlane(tf, j);
            r.a0 = __builtin_amdgcn_readlane(a0, j);
            r.a1 = __builtin_amdgcn_readlane(a1, j);
            sym_row_s(tm, a, r, E, nullptr);
        }
    }
}

template <int T, bool GLOBALMEM>
__global__ __launch_bounds__(T) void k_sym_block(SymArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    BlockTeam<T, GLOBALMEM> tm{(long long*)smem};
    TileEntry* E = GLOBALMEM ? (TileEntry*)(a.gscratch + (long long)blockIdx.x * a.gbytes)
                             : (TileEntry*)(smem + block_hdr(T));
    const int count = a.stats->sym_count[a.bin];
    const int* list = a.list + (long long)(a.bin - 1) * a.M;
    int4* stage = (int4*)(smem + 1024);
    for (RowWalk rw(count, 1, 0); rw.first < rw.end; rw.first += rw.stride)
        sym_row(tm, a, __builtin_amdgcn_readfirstlane(list[rw.first]), E, stage);
}

// Every rare symbolic bin in one launch (their sizes are on the device; an empty bin
// costs nothing but its loop test): 1024-thread blocks holding all 160 KiB of LDS.
//   phase 1  rows past the 32 KiB table: direct-mapped ones in the 1024-thread block's
//            LDS table, hashed ones and rows past the LDS as wide rows (dense windows),
//   phase 2  rows for a 10 KiB table: a wave per row, 16 waves per block.
// (Rows for a 32 KiB table keep a 256-thread kernel of their own: at one block per CU
// they would have a fifth of the rows in flight.)
// Wide rows (the hashed 1024-block rows and every row past its LDS): windows of
// WIDE_WT tiles, a dense 64-bit mask per tile in LDS (no hash, no CAS, no global
// table); nnz = sum of popcounts, tiles = non-zero masks.
__device__ void sym_row_wide(const BlockTeam<1024, false>& tm, const SymArgs& a, int row, unsigned long long* masks,
                             int4* stage, int* lctr) {
    constexpr int T = 1024;
    const int lo = __builtin_amdgcn_readfirstlane(a.rlo[row]);
    const int hi = __builtin_amdgcn_readfirstlane(a.rhi[row]);
    const int tflop = __builtin_amdgcn_readfirstlane(a.rtflop[row]);
    const int a0 = __builtin_amdgcn_readfirstlane(a.Aptr[row]), a1 = __builtin_amdgcn_readfirstlane(a.Aptr[row + 1]);
    const int R = __builtin_amdgcn_readfirstlane((int)a.grp[row]);
    long long n = 0;
    int t = 0;
    if (tm.rank() == 0) *lctr = 0;
    for (int w0 = lo; w0 <= hi; w0 += WIDE_WT) {
        const int w1 = min(hi + 1, w0 + WIDE_WT), wt = w1 - w0;
        for (int sl = tm.rank(); sl < wt; sl += T) masks[sl] = 0ull;
        tm.sync();
        walk_products(tm, a0, a1, a.Acol, nullptr, a.bmeta, true, tflop, WideTiles{masks, w0, w1, a.btcol, a.btmask},
                      stage);
        tm.sync();
        if (a.mcache) {
            // the row's tile list for numeric (complete when the row ends with t <= the cap:
            // numeric's mlisted); unordered, a counter add per wave and window
            const int lane = lane_id();
            for (int s0 = tm.rank() & ~63; s0 < wt; s0 += T) {
                const int sl = s0 + lane;
                const unsigned long long m = sl < wt ? masks[sl] : 0ull;
                const unsigned long long bal = __ballot(m != 0ull);
                if (!bal) continue;
                int at = 0;
                if (lane == 0) at = atomicAdd(lctr, __popcll(bal));
                at = __shfl(at, 0);
                const int pos = at + __popcll(bal & lanemask_lt());
                if (m && pos < a.mc_list)
                    for (int g = 0; g < R; ++g) {
                        unsigned long long* slot = a.mcache + (size_t)(row + g) * a.mc_stride;
                        st_cache(&slot[pos], m);
                        st_cache(&reinterpret_cast<int*>(slot + a.mc_list)[pos], w0 + sl);
                    }
            }
        }
        long long wn = 0;
        int wtl = 0;
        for (int sl = tm.rank(); sl < wt; sl += T) {
            const unsigned long long m = masks[sl];
            wn += __popcll(m);
            wtl += m != 0ull;
        }
        n += tm.sum(wn);  // (sum syncs: the masks are free for the next window)
        t += tm.sum(wtl);
    }
    if (tm.rank() < R) {
        a.Cptr[row + tm.rank()] = (int)n;
        a.ctiles[row + tm.rank()] = t;
        if (a.mcache && spill_row(hi - lo + 1, tflop, t, a.mc_list)) a.sp.lofs[row + tm.rank()] = -1;  // no list
    }
    tm.sync();
}

// Hashed rare rows whose span bitmap fits: two tile walks (bits, then ranked masks) instead
// of one walk per window of the span.  Returns false (nothing written) when the span bitmap
// or the row's tiles do not fit the region; the caller then walks windows.
__device__ bool sym_row_bitmap(const BlockTeam<1024, false>& tm, const SymArgs& a, int row, char* region,
                               int4* stage) {
    constexpr int T = 1024;
    const int lo = __builtin_amdgcn_readfirstlane(a.rlo[row]);
    const int hi = __builtin_amdgcn_readfirstlane(a.rhi[row]);
    const int span = hi - lo + 1;
    const long long sb = span_bits_bytes(span);
    if (sb > B1024_BYTES / 2) return false;
    const int nw = (span + 63) >> 6;
    unsigned long long* bm = (unsigned long long*)region;
    int* wpre = (int*)(region + align16((long long)nw * 8));
    const int tflop = __builtin_amdgcn_readfirstlane(a.rtflop[row]);
    const int a0 = __builtin_amdgcn_readfirstlane(a.Aptr[row]), a1 = __builtin_amdgcn_readfirstlane(a.Aptr[row + 1]);
    for (int i = tm.rank(); i < nw; i += T) bm[i] = 0ull;
    tm.sync();
    walk_products(tm, a0, a1, a.Acol, nullptr, a.bmeta, true, tflop, SpanBits{bm, lo, a.btcol}, stage);
    tm.sync();
    int tl = 0;
    for (int i = tm.rank(); i < nw; i += T) tl += __popcll(bm[i]);
    const int t = tm.sum(tl);
    if (sb + align16((long long)t * 8) * 2 > B1024_BYTES) return false;  // (uniform: every thread returns)
    tm.exclusive_scan(
        nw, [&](int i) { return (int)__popcll(bm[i]); }, [&](int i, int v) { wpre[i] = v; });
    unsigned long long* msk = (unsigned long long*)(region + sb);
    int2* kb = (int2*)(region + sb + align16((long long)t * 8));
    for (int r = tm.rank(); r < t; r += T) msk[r] = 0ull;
    tm.sync();
    walk_products(tm, a0, a1, a.Acol, nullptr, a.bmeta, true, tflop,
                  RankedMasks{bm, wpre, msk, kb, lo, a.btcol, a.btmask}, stage);
    tm.sync();
    long long nl = 0;
    for (int r = tm.rank(); r < t; r += T) nl += __popcll(msk[r]);
    const long long n = tm.sum(nl);
    const int R = __builtin_amdgcn_readfirstlane((int)a.grp[row]);
    if (tm.rank() < R) {
        a.Cptr[row + tm.rank()] = (int)n;
        a.ctiles[row + tm.rank()] = t;
    }
    if (a.mcache && mlisted(span, tflop, t, a.mc_list))  // few tiles over a wide span: the list for numeric
        for (int r = tm.rank(); r < t; r += T)
            for (int g = 0; g < R; ++g) {
                unsigned long long* slot = a.mcache + (size_t)(row + g) * a.mc_stride;
                st_cache(&slot[r], msk[r]);
                st_cache(&reinterpret_cast<int*>(slot + a.mc_list)[r], kb[r].x);
            }
    if (a.mcache && spill_row(span, tflop, t, a.mc_list)) {  // in column order
        const int off = spill_reserve(tm, a.sp, row, R, t);
        if (off >= 0)
            for (int r = tm.rank(); r < t; r += T) {
                st_cache(&a.sp.mask[off + r], msk[r]);
                st_cache(&a.sp.key[off + r], kb[r].x);
            }
    }
    tm.sync();
    return true;
}

// Near groups (k_bin_list's candidate list), one wave per candidate after the symbolic
// pass: the rows' C patterns must be equal -- counts, tile spans, and the row cache's tile
// masks (direct-mapped tables only: their lists come out in tile order) -- else the rows
// stay alone.  A verified group gets its union row: the rows' A columns marked in a bitmap
// over their column window, ranked by prefix popcounts; R value slices (0 where a row lacks
// the column) staged in LDS and copied out.  Then grp marks it (head R | GRP_NEAR).
struct NearArgs {
    const int* Aptr;
    const int* Acol;
    const double* Aval;
    const int* Cptr;  // the symbolic counts (before the scan)
    const int* ctiles;
    const int* rlo;
    const int* rhi;
    const int* rflop;
    const int* rtflop;
    const unsigned long long* mcache;
    int mc_list, mc_stride;
    const int* list;
    const Stats* stats;
    unsigned char* grp;
    int* ucol;
    double* uval;
    int* gna;
    int* ucolx;     // union columns for B's near union runs (bx_col + nnzB): at 3 * A0
    int* verified;  // Stats::near_verified
    // near groups add explicit 0*b (A side) and a*0 (B's union runs) products: B's values (A's
    // when B is A) are checked for Inf / NaN by the phase's waves, and a non-finite value makes
    // k_scan dissolve every near group of the call
    const double* vcheck;
    long long vcheck_n;
    int* nonfinite;  // Stats::nonfinite
};
constexpr int MHS_NEAR_GRID = 2048;  // k_near's block cap
constexpr int NEAR_PER = 4;  // A entries a lane holds: a group's R rows of at most 256 entries
constexpr int NEAR_LDS = NEAR_WORDS * 12 + RG_MAX * NEAR_UMAX * 8;  // a wave's bitmap, word prefixes, values
static_assert(16 * NEAR_LDS <= LDS_MAX_C - 1024, "k_sym_rare's 16 waves hold their near-group regions");
// The candidate groups gw, gw + nw, ... of the list (one wave each).
__device__ void near_groups(const NearArgs& p, char* lds, int gw, int nwaves) {
    unsigned long long* bm = (unsigned long long*)lds;
    int* wpre = (int*)(bm + NEAR_WORDS);
    double* uv = (double*)(wpre + NEAR_WORDS);
    const int lane = lane_id();
    const WaveTeam tm;
    const int count = __hip_atomic_load(&p.stats->near_heads, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (count > 0 && p.vcheck) {  // the finiteness of B's values, a slice a wave (only with candidates)
        bool bad = false;
        const long long st = (long long)nwaves * 64;
        long long i = (long long)gw * 64 + lane;
        for (; i + 3 * st < p.vcheck_n; i += 4 * st) {  // four loads in flight a lane
            double x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) x[u] = p.vcheck[i + u * st];
#pragma unroll
            for (int u = 0; u < 4; ++u) bad |= !__builtin_isfinite(x[u]);
        }
        for (; i < p.vcheck_n; i += st) bad |= !__builtin_isfinite(p.vcheck[i]);
        if (__ballot(bad) && lane == 0) *p.nonfinite = 1;
    }
    bool any = false;  // this wave verified a group (Stats::near_verified: one store a wave, no atomics)
    // every step's loads are independent of each other: three round trips per group
    for (int li = gw; li < count; li += nwaves) {
        const int e = __builtin_amdgcn_readfirstlane(p.list[li]);
        const int h = e >> 2, R = e & 3;
        // 1. the rows' scalars, lane r for row h + r
        const bool rl = lane < R;
        int n = 0, t = 0, tf = 0, fl = 0, a0 = 0, a1 = 0, rlo_l = 0, rhi_l = 0;
        if (rl) {
            rlo_l = p.rlo[h + lane];
            rhi_l = p.rhi[h + lane];
            n = p.Cptr[h + lane];
            t = p.ctiles[h + lane];
            tf = p.rtflop[h + lane];
            fl = p.rflop[h + lane];
            a0 = p.Aptr[h + lane];
            a1 = p.Aptr[h + lane + 1];
        }
        const int lo = __builtin_amdgcn_readfirstlane(rlo_l);
        const int hi = __builtin_amdgcn_readfirstlane(rhi_l);
        const int span = hi - lo + 1;
        // the row cache form of each row's C pattern (1: masks over the span, 2: a tile list)
        const int f = !rl || !sym_direct(span, tf) || tiny_class_sym(fl, a1 - a0) >= 0 ? 0
                      : mcached(span, tf)                                              ? 1
                      : mlisted(span, tf, t, p.mc_list)                                ? 2
                                                                                       : 0;
        const int n0 = __builtin_amdgcn_readfirstlane(n), t0 = __builtin_amdgcn_readfirstlane(t);
        const int f0 = __builtin_amdgcn_readfirstlane(f);
        const int A0 = __builtin_amdgcn_readfirstlane(a0), A1 = __shfl(a1, R - 1);
        const int b1 = __shfl(a0, 1), b2 = __shfl(a0, 2);  // rows 1, 2 start (R > 1, > 2)
        const unsigned long long rm = (1ull << R) - 1;
        if (n0 <= 0 || f0 == 0 || !p.mcache || A1 - A0 > 64 * NEAR_PER ||
            (__ballot(rl && n == n0 && t == t0 && f == f0 && rlo_l == lo && rhi_l == hi) & rm) != rm)
            continue;
        // 2. the row cache words of rows 1.. against row 0's, and the rows' A entries
        const int words = f0 == 1 ? span : t0;
        const unsigned long long* s0 = p.mcache + (size_t)h * p.mc_stride;
        bool diff = false;
        for (int i = lane; i < (R - 1) * words; i += 64) {
            const int r = 1 + (i >= words), q = i - (r - 1) * words;
            const unsigned long long* s1 = p.mcache + (size_t)(h + r) * p.mc_stride;
            diff = diff || s0[q] != s1[q] ||
                   (f0 == 2 && reinterpret_cast<const int*>(s0 + p.mc_list)[q] != reinterpret_cast<const int*>(s1 + p.mc_list)[q]);
        }
        int c[NEAR_PER];
        double v[NEAR_PER];
        int cmin = INT_MAX, cmax = -1;
#pragma unroll
        for (int u = 0; u < NEAR_PER; ++u) {
            const int j = A0 + lane + 64 * u;
            c[u] = j < A1 ? p.Acol[j] : -1;
            v[u] = j < A1 ? p.Aval[j] : 0.0;
            if (c[u] >= 0) {
                cmin = min(cmin, c[u]);
                cmax = max(cmax, c[u]);
            }
        }
        if (__ballot(diff)) continue;
        // 3. the union row over the rows' column window (A rows need not be sorted)
        cmin = __builtin_amdgcn_readfirstlane(wave_min(cmin));
        cmax = __builtin_amdgcn_readfirstlane(wave_max(cmax));
        if (cmax - cmin >= NEAR_WORDS * 64) continue;
        const int nw = ((cmax - cmin) >> 6) + 1;
        for (int q = lane; q < nw; q += 64) bm[q] = 0ull;
        tm.sync();
#pragma unroll
        for (int u = 0; u < NEAR_PER; ++u)
            if (c[u] >= 0) atomicOr(&bm[(c[u] - cmin) >> 6], 1ull << ((c[u] - cmin) & 63));
        tm.sync();
        tm.exclusive_scan(nw, [&](int q) { return (int)__popcll(bm[q]); }, [&](int q, int x) { wpre[q] = x; });
        tm.sync();
        const int nU = __builtin_amdgcn_readfirstlane(wpre[nw - 1] + (int)__popcll(bm[nw - 1]));
        if (nU > NEAR_UMAX) continue;
        for (int q = lane; q < R * nU; q += 64) uv[q] = 0.0;
        tm.sync();
#pragma unroll
        for (int u = 0; u < NEAR_PER; ++u) {
            if (c[u] < 0) continue;
            const int j = A0 + lane + 64 * u, r = (R > 1 && j >= b1) + (R > 2 && j >= b2);
            const int d = c[u] - cmin;
            const int rk = wpre[d >> 6] + (int)__popcll(bm[d >> 6] & ((1ull << (d & 63)) - 1));
            atomicAdd(&uv[r * nU + rk], v[u]);  // (duplicate columns in a row: summed, as their products)
            p.ucol[A0 + rk] = c[u];             // (the rows that share a column write it alike)
            if (p.ucolx) p.ucolx[3LL * A0 + rk] = c[u];
        }
        tm.sync();
        for (int q = lane; q < R * nU; q += 64) p.uval[3LL * A0 + q] = uv[q];
        if (lane == 0) {
            p.gna[h] = nU;
            any = true;
            p.grp[h] = (unsigned char)(R | GRP_NEAR);
        }
        if (lane > 0 && lane < R) p.grp[h + lane] = (unsigned char)(GRP_CONT | lane);
    }
    if (__ballot(any) && lane == 0) *p.verified = 1;
}

// (the symbolic rare bins on an aux stream: the candidates checked by a launch of their own)
__global__ __launch_bounds__(256) void k_near(NearArgs p) {
    __shared__ __attribute__((aligned(16))) char lds[WPB * NEAR_LDS];
    const int w = threadIdx.x >> 6;
    near_groups(p, lds + w * NEAR_LDS, (int)blockIdx.x * WPB + w, (int)gridDim.x * WPB);
}

__global__ __launch_bounds__(1024) void k_sym_rare(SymArgs a, NearArgs np) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int4* stage = (int4*)(smem + 1024);
    BlockTeam<1024, false> tm{(long long*)smem};
    TileEntry* E = (TileEntry*)(smem + BLOCK_HDR_1024);
    __shared__ int qslot;
    // phase 0: near row groups (their rows are k_sym_common's, done before this launch)
    if (np.list) {
        near_groups(np, smem + (threadIdx.x >> 6) * NEAR_LDS, (int)blockIdx.x * 16 + (int)(threadIdx.x >> 6),
                    (int)gridDim.x * 16);
        __syncthreads();
    }
#pragma unroll 1
    for (int bin = SYM_GLOBAL; bin >= SYM_B1024; --bin) {
        const int count = a.stats->sym_count[bin];
        const int* list = a.list + (long long)(bin - 1) * a.M;
        auto one = [&](int li) {
            const int row = __builtin_amdgcn_readfirstlane(list[li]);
            const int span = __builtin_amdgcn_readfirstlane(a.rhi[row]) - __builtin_amdgcn_readfirstlane(a.rlo[row]) + 1;
            if (bin == SYM_B1024 && sym_direct(span, __builtin_amdgcn_readfirstlane(a.rtflop[row])))
                sym_row(tm, a, row, E, stage);
            else if (!sym_row_bitmap(tm, a, row, (char*)E, stage))
                sym_row_wide(tm, a, row, (unsigned long long*)E, stage, (int*)(smem + 512));
        };
        if (count == 0) continue;  // (no atomics for an empty bin: most matrices have none)
        const BlockQueue q{a.cursors + (NUM_NB + bin) * 8 * CURSOR_STRIDE, &qslot, count};
        for (int li; q.next(li);) one(li);
    }
    __syncthreads();  // phase 2 reuses the whole LDS
    const int w = threadIdx.x >> 6;
    TileEntry* Ew = (TileEntry*)(smem + w * SYM_WM_BYTES + WAVE_HDR);
    const int count = a.stats->sym_count[SYM_WM];
    const int* list = a.list + (long long)(SYM_WM - 1) * a.M;
    WaveTeam wt;
    // A bin of a few rows per wave (<= MHS_SYMWM_DYN_MAX) takes them from the XCD groups'
    // cursors: blocks leave phase 1 at different times, and the early ones' waves then take
    // the rows the late ones would have held.  (Every wave on one cursor, every call, even
    // an empty bin's: +40-95 µs per call on cant / cop20k / scircuit-like -- measured.)
    if (count > 0 && count <= MHS_SYMWM_DYN_MAX) {
        WaveQueue q(a.cursors + (NUM_NB + SYM_WM) * 8 * CURSOR_STRIDE, count, 1);
        for (int li; q.next(li);) sym_row(wt, a, __builtin_amdgcn_readfirstlane(list[li]), Ew, nullptr);
        return;
    }
    for (RowWalk rw(count, 16, w); rw.first < rw.end; rw.first += rw.stride)
        sym_row(wt, a, __builtin_amdgcn_readfirstlane(list[rw.first]), Ew, nullptr);
}

// ----------------------------------------------------- scan + classify ---

// Append a 1024-thread block's SCAN_ITEMS rows (blockIdx*SCAN_ITEMS + j, bins in
// binof[j]) to contiguous per-bin lists: bin x's rows at list + (x-1)*M, cursor
// cnt[x * BINCNT_STRIDE] (a 128-byte line per bin: on one line the blocks' reservations
// serialised -- round 6).  The block's rows keep row order; one atomic per (block, bin)
// reserves their places.
template <int NB, int PER>
__device__ void append_block_rows(const unsigned char* binof, long long M, int* __restrict__ cnt,
                                  int* __restrict__ list, int blk) {
    constexpr int ITEMS = 1024 * PER;
    static_assert(PER * 16 <= 64 && NB <= 16, "one wave scans one bin's (pass, wave) counts");
    __shared__ int wc[NB][PER * 16];  // [bin][pass*16 + wave]: members, then exclusive prefix
    __shared__ int nbase[NB];
    const int lane = lane_id(), w = threadIdx.x >> 6;
    int mybin[PER], rank[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {  // pass k = rows k*1024 + threadIdx.x of the block (row order)
        mybin[k] = binof[k * 1024 + threadIdx.x];
        rank[k] = 0;
        for (int x = 1; x < NB; ++x) {
            const unsigned long long bal = __ballot(mybin[k] == x);
            if (mybin[k] == x) rank[k] = __popcll(bal & lanemask_lt());
            if (lane == 0) wc[x][k * 16 + w] = __popcll(bal);
        }
    }
    __syncthreads();
    if (w >= 1 && w < NB) {  // wave x: exclusive prefix over (pass, wave); reserve the block's places
        const int c = lane < PER * 16 ? wc[w][lane] : 0;
        const int inc = wave_incl_scan(c);
        if (lane < PER * 16) wc[w][lane] = inc - c;
        if (lane == 63) nbase[w] = inc ? atomicAdd(&cnt[w * BINCNT_STRIDE], inc) : 0;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int x = mybin[k];
        if (x > 0)
            list[(long long)(x - 1) * M + nbase[x] + wc[x][k * 16 + w] + rank[k]] =
                blk * ITEMS + k * 1024 + threadIdx.x;
    }
}

// Row groups and the symbolic bin lists (one light pass after k_analyze, whose grid
// is too fine-grained for per-block cursor atomics).  Row i's group: the maximal run
// of same-pattern rows containing it, broken every RG_BREAK rows, cut into groups of
// RG_MAX from the run start.  Only group heads enter the symbolic lists (a group's
// rows share one C pattern).  Numeric-first tiny rows stay alone (their values come
// out of the symbolic pass).
// Numeric-first probe: sums k_analyze's per-block slot entries / other rows and hands them
// to the host (the last block publishes), which picks the bin lists.
__global__ __launch_bounds__(1024) void k_probe_publish(const unsigned long long* __restrict__ blk, int n,
                                                        Stats* __restrict__ stats, Published* pub, int seq) {
    const int per = (n + (int)gridDim.x - 1) / (int)gridDim.x;
    const int i0 = blockIdx.x * per, i1 = min(n, i0 + per);
    unsigned long long slots = 0, other = 0;
    for (int i = i0 + threadIdx.x; i < i1; i += 1024) {
        const unsigned long long x = blk[i];
        other += (x >> BLK_FLOP_BITS) & 0xFF;
        slots += x >> BLK_SLOT_SHIFT;
    }
    slots = wave_sum(slots);
    other = wave_sum(other);
    if (lane_id() == 0 && slots) atomicAdd(&stats->an_slots, slots);
    if (lane_id() == 0 && other) atomicAdd(&stats->an_other, other);
    if (last_block_done(&stats->an_done)) publish_stats(stats, pub, seq);
}

// Near-group candidates (k_bin_list): the A rows the link test reads
struct NearCand {
    const unsigned* nsig;  // k_analyze's signatures
    int* list;             // nullptr: no near groups
};

template <int PER>
__global__ __launch_bounds__(1024) void k_bin_list(int M, const unsigned char* __restrict__ bin_id,
                                                   const unsigned char* __restrict__ asame,
                                                   unsigned char* __restrict__ grp, int groups,
                                                   int* __restrict__ list, const unsigned char* __restrict__ nft_bin,
                                                   Stats* __restrict__ stats, NearCand nc, int* __restrict__ bincnt) {
    __shared__ unsigned char binof[1024 * PER];
    // links of rows [blk0 - RG_BREAK, blk0 + ITEMS + RG_MAX): a row's group reads its run back
    // to the last RG_BREAK boundary and its group forward
    constexpr int LK = 1024 * PER + RG_BREAK + RG_MAX;
    __shared__ unsigned char lk_s[LK];
    __shared__ int ncand_s, nbase_s;  // the block's near candidates: one counter add per block
    MHS_SCSTAMP(blockIdx.x, 8);
    if (threadIdx.x == 0) ncand_s = 0;
    const long long lbase = (long long)blockIdx.x * (1024 * PER) - RG_BREAK;
    // link of row r to row r-1: 1 = the same A pattern, 2 = a near candidate (see GRP_NEAR;
    // rows of the small-table wave bin only: k_sym_rare checks them after k_sym_common), 0 = none
    for (int j = threadIdx.x; j < LK; j += 1024) {
        const long long r = lbase + j;
        int l = 0;
        if (r >= 0 && r < M) {
            if (asame[r]) {
                l = 1;
            } else if (nc.list && r > 0 && !asame[r - 1] && (r + 1 >= M || !asame[r + 1])) {
                // (rows of same-pattern runs stay out: a near link would shift their groups)
                const unsigned g1 = nc.nsig[r];
                l = g1 != 0u && g1 == nc.nsig[r - 1] ? 2 : 0;
            }
        }
        lk_s[j] = (unsigned char)l;
    }
    __syncthreads();
    auto link = [&](long long r) -> int { return lk_s[r - lbase]; };
    int cand_e[PER], cand_n = 0;
    for (int j = threadIdx.x; j < 1024 * PER; j += 1024) {
        const long long i = (long long)blockIdx.x * (1024 * PER) + j;
        unsigned char b = 0;
        bool cand = false;  // head of a near candidate group (listed for k_near)
        int cR = 0;
        if (i < M) {
            int g = 1;
            // a run of same-pattern rows is tiny throughout or not at all
            const int bi = nft_bin ? nft_bin[i] : bin_id[i];
            const bool solo = nft_bin && bi >= SYM_TINY && bi < SYM_TINY + TINY_SYM_NC;
            if (groups && !solo) {
                // the run of linked rows through i is cut into groups of RG_MAX from its start
                long long h = i;
                if (link(i)) {
                    long long rs = i;
                    const long long lim = i - i % RG_BREAK;
                    while (rs > lim && link(rs)) --rs;
                    h = i - (i - rs) % RG_MAX;
                }
                int R = 1;
                bool nearg = false;
                while (R < RG_MAX && h + R < M && (h + R) % RG_BREAK != 0) {
                    const int lk = link(h + R);
                    if (!lk) break;
                    nearg = nearg || lk == 2;
                    ++R;
                }
                // near candidates: every row counted on its own by symbolic; k_near decides
                if (!nearg) g = i == h ? R : (GRP_CONT | (int)(i - h));
                cand = nearg && i == h;
                cR = R;
            }
            grp[i] = (unsigned char)g;
            b = (g & GRP_CONT) ? 0 : bi;
        }
        if (cand) cand_e[cand_n++] = (int)(i * 4 + cR);
        binof[j] = b;
    }
    int at = cand_n ? atomicAdd(&ncand_s, cand_n) : 0;
    __syncthreads();
    if (threadIdx.x == 0 && ncand_s) nbase_s = atomicAdd(&stats->near_heads, ncand_s);
    __syncthreads();
    for (int q = 0; q < cand_n; ++q) nc.list[nbase_s + at + q] = cand_e[q];
    MHS_SCSTAMP(blockIdx.x, 9);  // (classified)
    append_block_rows<SYM_NB, PER>(binof, M, bincnt, list, (int)blockIdx.x);
    MHS_SCSTAMP(blockIdx.x, 10);  // (appended)
    // the last block leaves the totals in Stats (the symbolic launches read them there)
    if (last_block_done(bincnt + 2 * NBINS * BINCNT_STRIDE) && threadIdx.x < NBINS)
        stats->sym_count[threadIdx.x] = __hip_atomic_load(bincnt + threadIdx.x * BINCNT_STRIDE, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int num_bin_of(int n, int flop, int span, int t, int* gneed,
                                          int dense_span_max, int nA, bool tiny_ok) {
    if (n == 0) return NUM_NONE;
    const int tc = tiny_ok ? tiny_class(flop, nA) : -1;
    if (tc >= 0 && tc < TINY_NUM_SMALL) return NUM_TINY + tc;
    // scattered rows of the first 64-lane class (about a tile per C column: their tables cost a
    // tile, a hash probe and a rank per column) with few repeated columns sort in registers too
    if (MHS_TINY_SPARSE_PCT > 0 && tc == TINY_NUM_SMALL && 100LL * t >= (long long)MHS_TINY_SPARSE_PCT * n &&
        (long long)MHS_TINY_DUP * n >= flop)
        return NUM_TINY + tc;
    const long long need = num_need(span, t, n, dense_span_max);
    const bool hash = num_mode(span, t, n, dense_span_max) == NM_HASH;
    if (need <= NUM_WS_BYTES - WAVE_HDR && flop <= NUM_WS_WORK) return hash ? NUM_WSH : NUM_WS;
    if (tc >= 0) return NUM_TINY + tc;  // a bigger table than the small wave bin's: sort in registers
    if (num_wide(span, t, n, dense_span_max) || num_ranked(span, t, n, dense_span_max))
        return NUM_B1024;  // rank by span bitmap, else windowed masks with global accumulation
    if (need <= NUM_W16_BYTES - WAVE_HDR && flop <= NUM_W16_WORK) return hash ? NUM_W16H : NUM_W16;
    if (need <= NUM_B256_BYTES - BLOCK_HDR && flop <= NUM_B256_WORK) return NUM_B256;
    if (need <= B1024_BYTES) return NUM_B1024;
    atomicMax(gneed, (int)(need > INT_MAX ? INT_MAX : need));
    return NUM_GLOBAL;
}

// Grouped numeric bin of a group of R rows (NUM_NONE: run its rows one by one).
__device__ __forceinline__ int num_group_bin_of(int n, int flop, int span, int t, int R, int dense_span_max,
                                                int nA, bool tiny_ok) {
    if (R < 2 || n == 0 || (tiny_ok && tiny_class(flop, nA, TINY_NUM_SMALL) >= 0))
        return NUM_NONE;  // tiny rows: one by one
    const long long need = num_need_rows(span, t, n, dense_span_max, R);
    if (need <= NUM_WSG_BYTES - WAVE_HDR && flop <= NUM_WS_WORK) return NUM_WSG;
    if (need <= NUM_W16_BYTES - WAVE_HDR && flop <= NUM_W16_WORK) return NUM_W16G;
    return NUM_NONE;
}

// Row pointer = exclusive scan of the C row nnz (items [0, M]; item M = 0 gives
// row_ptr[M]) in ONE pass with decoupled look-back: blocks take tickets in dispatch
// order (big grids), publish their aggregate, add up their predecessors' (inclusive
// prefix once one is found) and publish their own inclusive prefix.  Every predecessor
// holds an earlier ticket, so it has started and publishes without waiting on this
// block.  The same pass gives every row its numeric bin and appends it to the bin
// lists, and every block adds its share of the product total; the last block to finish
// publishes Stats to the host.
constexpr int SCAN_TICKET_MIN = 256;  // k_scan grids above this take dispatch-order tickets
constexpr unsigned long long LB_AGG = 1ull << 62, LB_INC = 2ull << 62, LB_VAL = (1ull << 62) - 1;
// LDS bytes a block-bin row's tables need (k_scan sizes the launches by it; a split launch
// filters its rows by it).
__device__ __forceinline__ int block_row_need(bool b1024, int lo, int hi, int t, int n, int dense_span_max) {
    const int span = hi_lo_span(lo, hi);
    return b1024 && num_wide(span, t, n, dense_span_max)     ? B1024_BYTES
           : b1024 && num_ranked(span, t, n, dense_span_max) ? (int)num_need_ranked(span, t, n)
                                                             : (int)num_need(span, t, n, dense_span_max);
}

template <int PER>
__global__ __launch_bounds__(1024) void k_scan(int M, int* __restrict__ Cptr,
                                               unsigned long long* __restrict__ state,
                                               const int* __restrict__ rflop,
                                               const int* __restrict__ rlo,
                                               const int* __restrict__ rhi,
                                               const int* __restrict__ ctiles,
                                               const unsigned char* __restrict__ grp,
                                               const int* __restrict__ Aptr,
                                               int* __restrict__ list, Stats* __restrict__ stats,
                                               int dense_span_max, Published* pub, int seq, int tiny_ok,
                                               const unsigned long long* __restrict__ blkflop, int nflop, int nft,
                                               long long* __restrict__ tslot, const int* __restrict__ gna,
                                               int4* __restrict__ bmeta_near,
                                               const unsigned char* __restrict__ sym_bin, SpecArgs spec,
                                               int* __restrict__ bincnt) {
    constexpr int ITEMS = 1024 * PER;  // PER consecutive rows per thread
    static_assert(PER == 1 || PER == 4, "launch_scan_classify instantiates these");
    __shared__ long long ws[16];
    __shared__ long long excl_s;
    __shared__ int bid_s;
    // the block's largest grouped-bin LDS needs [0, 2), block-bin needs [2, 4), their small
    // launches' needs [4, 6) and hub-row counts [6, 8): LDS first, one global atomic a block
    __shared__ int agg_s[8];
    const int lane = lane_id(), w = threadIdx.x >> 6;
    if (threadIdx.x < 8) agg_s[threadIdx.x] = 0;
    // grids of <= 256 blocks (M <= 256K rows) are co-resident (a 1024-thread block with
    // ~1 KiB of LDS fits any CU), so no block can wait on one that never starts: the
    // block index serves, and the ticket's atomic round trip leaves the critical path
    const bool nonfin = stats->nonfinite != 0;  // (k_sym_rare's near check, before this launch)
    int bid = blockIdx.x;
    if (gridDim.x > SCAN_TICKET_MIN) {
        if (threadIdx.x == 0) bid_s = atomicAdd(&stats->scan_ticket, 1);
        __syncthreads();
        bid = bid_s;
    }
    const int base = bid * ITEMS + threadIdx.x * PER;
    MHS_SCSTAMP(bid, 0);
    // every load of the block's rows issues here, ahead of the first barrier (the classification
    // below needs none of the prefix): one round trip for the counts and the row scalars
    unsigned long long fpart = 0;  // the block's share of k_analyze's per-block product partials
    {
        const int per = (nflop + (int)gridDim.x - 1) / (int)gridDim.x;
        const int i1 = min(nflop, (bid + 1) * per);
        for (int i = bid * per + threadIdx.x; i < i1; i += 1024) fpart += blkflop[i] & BLK_FLOP_MASK;
    }
    int v[PER], rlo_k[PER], rhi_k[PER], grp_k[PER], a0_k[PER], a1_k[PER], rfl_k[PER], ctl_k[PER], sb_k[PER];
    auto row_scalars = [&]() {
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int i = base + k;
            const bool in = i < M;
            rlo_k[k] = in ? rlo[i] : 0;
            rhi_k[k] = in ? rhi[i] : 0;
            grp_k[k] = in ? grp[i] : 0;
            a0_k[k] = in ? Aptr[i] : 0;
            a1_k[k] = in ? Aptr[i + 1] : 0;
            rfl_k[k] = in ? rflop[i] : 0;
            ctl_k[k] = in ? ctiles[i] : 0;
            sb_k[k] = in ? sym_bin[i] : 0;
        }
    };
    long long loc = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int i = base + k;
        v[k] = i < M ? Cptr[i] : 0;
        loc += v[k];
    }
    {  // total products (off the tail: the last block only publishes)
        const unsigned long long f = wave_sum(fpart);
        if (lane == 0 && f) atomicAdd(&stats->flop, f);
    }
    const long long inc = wave_incl_scan64(loc);
    if (lane == 63) ws[w] = inc;
    __syncthreads();
    long long woff = 0, total = 0;
    for (int k = 0; k < 16; ++k) {
        woff += k < w ? ws[k] : 0;
        total += ws[k];
    }
    MHS_SCSTAMP(bid, 1);  // (counts loaded, block scan done)
    // the block's aggregate goes out first: successors' look-backs need it
    if (threadIdx.x == 0 && bid > 0)
        __hip_atomic_store(&state[bid], LB_AGG | (unsigned long long)total, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    // numeric bin of every row (independent of the prefix: its loads overlap the
    // predecessors' publication instead of following the look-back)
    row_scalars();  // (loaded here, after the counts' barrier: ahead of it measured slower)
    __shared__ unsigned char nbin_of[ITEMS];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int i = base + k;
        int nbin = NUM_NONE;
        if (i < M) {
            const int n = v[k];
            const int lo = rlo_k[k], hi = rhi_k[k];
            const int span = n ? hi - lo + 1 : 0;
            int g = grp_k[k];
            int hrow = (g & GRP_CONT) ? i - (g & 0x7F) : i;
            int ghd = (g & GRP_CONT) ? grp[hrow] : g;
            if (nonfin && (ghd & GRP_NEAR)) {  // Inf / NaN in B's values: the near group's rows alone
                g = ghd = 1;
                hrow = i;
            }
            if (bmeta_near) {  // near union runs of B rows (B is A): mark a verified group's head
                const int R = g & GRP_RMASK;
                if (!(g & GRP_CONT) && (g & GRP_NEAR) && R >= 2 && R <= MHS_RUN_MAX)
                    bmeta_near[i].w = NEAR_HEAD | (R << 16) | gna[i];
            }
            // a group runs as one item when its R accumulators fit a wave bin; its
            // members decide alike (same C pattern and sizes; flop and A length: the head's)
            // and then stay out
            const int gh = ghd & GRP_RMASK;
            const int nA = a1_k[k] - a0_k[k];
            const int hflop = gh > 1 ? rflop[hrow] : rfl_k[k];
            const int hnA = gh > 1 ? Aptr[hrow + 1] - Aptr[hrow] : nA;
            // tiny sort keys hold the column relative to the row's first tile in 23 bits
            const bool tok = tiny_ok && (long long)span * TILE_BITS - 1 <= TINY_NUM_NMAX;
            // numeric-first rows (k_analyze's rule) have their values: one copy list
            const int fc = nft && tok ? tiny_class(rfl_k[k], nA, TINY_SYM_NC) : -1;
            // symbolic's scattered class (k_analyze allows it only where tok holds) kept no masks:
            // the row sorts in numeric too, on its own (a group's rows are all of the class)
            const bool s4 = sb_k[k] == SYM_TINY + 4;
            const int gb =
                fc >= 0 || s4 ? -1 : num_group_bin_of(n, hflop, span, ctl_k[k], gh, dense_span_max, hnA, tok);
            if (nft && fc < 0) tslot[i] = -1;  // (slot rows: written by the symbolic pass)
            if (gb < 0)
                nbin = NUM_TINY + (s4 ? tiny_class(rfl_k[k], nA) : fc);
            else if (gb != NUM_NONE)
                nbin = (g & GRP_CONT) ? NUM_NONE : gb;
            else
                nbin = num_bin_of(n, rfl_k[k], span, ctl_k[k], &stats->num_global_need, dense_span_max, nA,
                                  tok);
        }
        nbin_of[threadIdx.x * PER + k] = (unsigned char)nbin;
        // the grouped wave bins' launches take LDS regions sized to their largest group (a 3-row FEM
        // group needs ~7 KB of the 10 KiB region: 5 waves per SIMD instead of 4)
        {
            int gneed = 0;
            if (nbin == NUM_WSG || nbin == NUM_W16G) {
                const int gg = grp_k[k] & GRP_RMASK;
                gneed = (int)num_need_rows(rhi_k[k] - rlo_k[k] + 1, ctl_k[k], v[k], dense_span_max, gg > 1 ? gg : 1) +
                        WAVE_HDR;
            }
            // (LDS first: one global atomic per wave measured +10 us on cant-like's k_scan --
            // thousands of waves on one address)
            if (__ballot(gneed > 0)) {
                const int gs = wave_max(nbin == NUM_WSG ? gneed : 0), g16 = wave_max(nbin == NUM_W16G ? gneed : 0);
                if (lane == 0 && gs) atomicMax(&agg_s[0], gs);
                if (lane == 0 && g16) atomicMax(&agg_s[1], g16);
            }
        }
        // the block kernels' launches get the LDS their largest row needs (more blocks per
        // CU than a fixed 64 / 157 KiB when the rows are smaller)
        int need = 0;
        if (nbin == NUM_B256 || nbin == NUM_B1024)
            need = block_row_need(nbin == NUM_B1024, rlo_k[k], rhi_k[k], ctl_k[k], v[k], dense_span_max);
        const int n256 = wave_max(nbin == NUM_B256 ? need : 0), n1024 = wave_max(nbin == NUM_B1024 ? need : 0);
        if (n256 | n1024) {  // the split launches (B256_SPLIT / B1024_SPLIT)
            const int split = nbin == NUM_B256 ? B256_SPLIT : B1024_SPLIT;
            const bool blk = nbin == NUM_B256 || nbin == NUM_B1024;
            const int s256 = wave_max(nbin == NUM_B256 && need <= split ? need : 0);
            const int s1024 = wave_max(nbin == NUM_B1024 && need <= split ? need : 0);
            const int b256 = __popcll(__ballot(blk && nbin == NUM_B256 && need > split));
            const int b1024 = __popcll(__ballot(blk && nbin == NUM_B1024 && need > split));
            if (lane == 0) {
                if (n256) atomicMax(&agg_s[2], n256);
                if (n1024) atomicMax(&agg_s[3], n1024);
                if (s256) atomicMax(&agg_s[4], s256);
                if (s1024) atomicMax(&agg_s[5], s1024);
                if (b256) atomicAdd(&agg_s[6], b256);
                if (b1024) atomicAdd(&agg_s[7], b1024);
            }
        }
    }
    __syncthreads();
    MHS_SCSTAMP(bid, 2);  // (classified)
    if (threadIdx.x < 8 && agg_s[threadIdx.x]) {
        const int k = threadIdx.x, v = agg_s[k];
        if (k < 2) atomicMax(&stats->num_wave_need[k], v);
        else if (k < 4) atomicMax(&stats->num_block_need[k - 2], v);
        else if (k < 6) atomicMax(&stats->num_block_small_need[k - 4], v);
        else atomicAdd(&stats->num_block_big[k - 6], v);
    }
    if (w == 0) {
        // wave 0 looks back over 64 predecessors per round trip: lane l reads block j - l;
        // the nearest inclusive prefix ends the walk, the aggregates above it are summed
        // (a window with an unpublished block before that point is re-read)
        long long ex = 0;
        if (bid > 0) {
            // fast path (big grids: the predecessor is usually done): one load
            unsigned long long s1 = 0;
            if (lane == 0) s1 = __hip_atomic_load(&state[bid - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s1 = __shfl(s1, 0);
            for (int j = bid - 1; !(s1 & LB_INC);) {
                const int idx = j - lane;
                const unsigned long long st =
                    idx >= 0 ? __hip_atomic_load(&state[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                             : LB_INC;  // before block 0: an inclusive prefix of 0
                const unsigned long long inc_m = __ballot((st & LB_INC) != 0);
                const unsigned long long zero_m = __ballot(st == 0);
                const int fi = inc_m ? __builtin_ctzll(inc_m) : 64;
                const unsigned long long upto = fi >= 63 ? ~0ull : ((2ull << fi) - 1);
                if (zero_m & upto) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;  // a predecessor running: its aggregate comes without waiting on us
                }
                ex += wave_sum(lane <= fi ? (long long)(st & LB_VAL) : 0LL);
                if (fi < 64) break;
                j -= 64;
            }
            if (s1 & LB_INC) ex = (long long)(s1 & LB_VAL);
        }
        if (lane == 0) {
            __hip_atomic_store(&state[bid], LB_INC | (unsigned long long)(ex + total), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            excl_s = ex;
            if (bid == (int)gridDim.x - 1) {
                stats->nnzC = ex + total;
                if (ex + total > INT_MAX) atomicOr(&stats->err, ERR_OVERFLOW);
            }
        }
    }
    __syncthreads();
    MHS_SCSTAMP(bid, 3);  // (look-back done)
    long long off = excl_s + woff + inc - loc;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int i = base + k;
        if (i <= M) Cptr[i] = (int)off;
        off += v[k];
    }
    __syncthreads();
    MHS_SCSTAMP(bid, 4);  // (row_ptr written)
    append_block_rows<NUM_NB, PER>(nbin_of, M, bincnt, list, bid);
    MHS_SCSTAMP(bid, 5);  // (appended)
    if (!last_block_done(&stats->final_done)) return;
    MHS_SCSTAMP(bid, 6);  // (the last block)
    if (threadIdx.x < NBINS)  // the bins' totals (bin-list counters) into Stats
        stats->num_count[threadIdx.x] =
            __hip_atomic_load(bincnt + threadIdx.x * BINCNT_STRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (pub) {
        if (nonfin && threadIdx.x == 0) stats->near_verified = 0;  // (no union runs: nothing to copy)
        __syncthreads();
        // a speculated plan (SpecArgs): the numeric launches behind this kernel run only if the
        // call's Stats are the plan's (the host checks the same on the published copy)
        if (spec.go && threadIdx.x == 0) *spec.go = (stats->err == 0 && stats_same_plan(*stats, spec.expect)) ? 1 : 0;
        publish_stats(stats, pub, seq);
        MHS_SCSTAMP(bid, 7);  // (published)
        // the host has its copy: leave the device Stats zeroed for the next call (nothing
        // after this kernel reads them), which saves that call a memset launch
        __syncthreads();
        if (threadIdx.x < (int)(sizeof(Stats) / 4)) reinterpret_cast<int*>(stats)[threadIdx.x] = 0;
    }
}

// --------------------------------------------------------------- numeric ---
struct NumArgs {
    const int* Aptr;
    const int* Acol;
    const double* Aval;
    const int* Bcol;
    const double* Bval;
    const int4* bmeta;
    const int* btcol;
    const unsigned long long* btmask;
    const int* rflop;
    const int* rtflop;
    const int* rlo;
    const int* rhi;
    const int* ctiles;
    const int* list;  // the bin's rows (contiguous, row order within each scan block)
    int count;
    const unsigned char* grp;  // row groups (grouped bins: R of every head)
    const int* Cptr;
    int* Ccol;
    double* Cval;
    char* gscratch;
    long long gbytes;
    int dense_span_max;
    const unsigned long long* mcache;
    int mc_list, mc_stride;  // row cache: tile-list cap, words per row
    int* cursor;             // this launch's row cursors (block queue, guided / queued wave walks)
    SpillLists sp;           // tile lists of rows past the row cache's cap (symbolic -> numeric)
    int qall;                // guided bins: every row from the cursor (few rows a wave)
    const int* ucol;         // near groups' union rows (GRP_NEAR; see Work)
    const double* uval;
    const int* gna;
    int ubase;               // near union runs of B rows (A*A with verified near groups; 0: off): Bcol /
                             // Bval are then B's arrays extended by the union rows at ubase
    int wave_bytes;          // grouped wave launches: LDS bytes per wave (0: the template's)
    const int* go;           // speculated plan: run only when *go == 1 (k_scan's verdict); nullptr: always
};
// A speculated launch whose plan k_scan rejected returns before touching anything.
#define MHS_PLAN_GUARD(args) \
    if ((args).go && *(args).go != 1) return

// C output of a row (num_row_body, num_row_bitmap): values two a lane, columns four a lane, in
// 16-byte stores (8-byte aligned doubles and 4-byte aligned ints: gfx950 stores them unaligned);
// `rank` / `T`: the team's lane and size.  src (LDS) is 16-byte aligned.
__device__ __forceinline__ void store_vals(double* __restrict__ dst, const double* src, int n, int rank, int T) {
    for (int r = 2 * rank; r < n; r += 2 * T) {
        if (r + 1 < n) __builtin_nontemporal_store(*(const d2u*)(src + r), (d2u*)(dst + r));
        else st_stream(dst + r, src[r]);
    }
}
// the C row's columns (R rows of a group alike) from the staged list cb (LDS, 16-byte aligned)
__device__ __forceinline__ void store_cols(int* __restrict__ dst, const int* cb, int n, int R, int rank, int T) {
    for (int r = 4 * rank; r < n; r += 4 * T) {
        if (r + 3 < n) {
            const i4a c4 = *(const i4a*)(cb + r);
            for (int g = 0; g < R; ++g) __builtin_nontemporal_store((i4u)c4, (i4u*)(dst + g * n + r));
        } else {
            for (int k = r; k < n; ++k)
                for (int g = 0; g < R; ++g) st_stream(&dst[g * n + k], cb[k]);
        }
    }
}
// the columns of a tile table (DIRECT: tile lo + s; hashed: the entry's key) at their C-row ranks
// into cb: a lane expands a tile of <= 8 columns, a tile of more is expanded by its whole wave
// (lane = bit, the entry re-read by every lane: a broadcast LDS read)
template <bool DIRECT>
__device__ __forceinline__ void stage_cols(const TileEntry* E, int H, int lo, int* cb, int rank, int T) {
    const int lane = lane_id();
    for (int s0 = rank & ~63; s0 < H; s0 += T) {
        const int s = s0 + lane;
        unsigned long long mk = 0;
        int key = 0, base = 0;
        if (s < H) {
            const TileEntry e = E[s];
            mk = e.mask;
            key = DIRECT ? lo + s : e.key;
            base = e.base;
        }
        const bool big = __popcll(mk) > 8;
        unsigned long long bigs = __ballot(big);
        if (!big) {
            int r = base;
            while (mk) {
                cb[r++] = (key << TILE_SHIFT) + __builtin_ctzll(mk);
                mk &= mk - 1;
            }
        }
        while (bigs) {
            const int src = __builtin_ctzll(bigs);
            bigs &= bigs - 1;
            const uint4 q = *reinterpret_cast<const uint4*>(&E[s0 + src]);  // mask, base, key
            const unsigned long long m2 = ((unsigned long long)q.y << 32) | q.x;
            const int k2 = DIRECT ? lo + s0 + src : (int)q.w;
            if ((m2 >> lane) & 1ull) cb[(int)q.z + __popcll(m2 & lanemask_lt())] = (k2 << TILE_SHIFT) + lane;
        }
    }
}

// (forced inline, as num_row: left to the inliner, a grown grouped kernel called them out of
// line, and the kernel argument they take by reference went to scratch -- 304 bytes a lane,
// every field read a scratch load)
template <class Team, bool GLOBALMEM, int MODE, bool GROUPED, bool O32>
__device__ __forceinline__ void num_row_body(const Team& tm, const NumArgs& a, int row, int lo, int span, int t,
                             int c0, int n, int a0, int a1, char* region, int* counter,
                             int4* stage, int R) {
    MHS_BSTAMP0();
    const int H = MODE == NM_HASH ? hash_slots(t) : span;
    const int colbase = lo << TILE_SHIFT;
    TileEntry* E = (TileEntry*)region;
    double* acc = (double*)(region + (long long)H * 16);
    const int nacc = MODE == NM_DENSE ? span * TILE_BITS : n;
    const int tflop = __builtin_amdgcn_readfirstlane(a.rtflop[row]);
    // row group: R accumulator slices `stride` doubles apart; C row r at c0 + r*n
    const int stride = GROUPED ? (int)(num_acc_bytes(MODE, span, t, n) / 8) : 0;
    const int nclear = GROUPED ? (R - 1) * stride + nacc : nacc;

    // row groups: the first chunk pair's A loads go out now and its bmeta gathers after the tile
    // table -- both round trips overlap the table and rank phases instead of opening the walk
    // (a FEM dof-3 row of 69 entries is one pair: every A-side load of the group)
    GroupPair gp;
    bool gnear = false;
    int gnw = a1 - a0;
    const int* gcol = a.Acol;
    const double* gval = a.Aval;
    if constexpr (GROUPED) {
        gnear = (__builtin_amdgcn_readfirstlane((int)a.grp[row]) & GRP_NEAR) != 0;
        if (gnear) {
            gnw = __builtin_amdgcn_readfirstlane(a.gna[row]);
            gcol = a.ucol;
            gval = a.uval + 2LL * a0;
        }
        group_pair_a(gp, a0, a0 + gnw, gcol, gval, R, gnw);
    }
    // 1. the C row's tile table: the symbolic pass's masks when it kept them,
    //    else rebuilt (same OR pass as symbolic)
    MHS_BSTAMP(0);
    // symbolic kept the masks unless it sorted the row as a tiny one (numeric runs those
    // with tables when the tiny classes are off: N beyond the packed keys' 23 bits)
    // (symbolic's class 4 rows never come here: k_scan sorts them in numeric too)
    const bool sym_tiny = tiny_class_sym(__builtin_amdgcn_readfirstlane(a.rflop[row]), a1 - a0) >= 0;
    const int lofs = (a.mcache && !sym_tiny && spill_row(span, tflop, t, a.mc_list))
                         ? __builtin_amdgcn_readfirstlane(a.sp.lofs[row])
                         : -1;
    // hashed rows rank their tiles by a bitmap over the span (block teams / many tiles,
    // when it fits the accumulator), else by counting (few tiles), else by a sort
    const bool rank_bitmap = MODE == NM_HASH && (Team::size > 64 || t >= 64) &&
                             (long long)((span + 63) >> 6) * 12 + 16 + (long long)t * 4 <=
                                 num_acc_bytes(NM_HASH, span, t, n);
    // (a two-level bitmap over the span -- O(H) LDS work where counting costs t^2/64 -- measured
    // cage15-like numeric +3 %: more dependent LDS steps per row; the kernel is latency-bound)
    const bool rank_count = MODE == NM_HASH && !rank_bitmap &&
                            (t <= HASH_CNT_T || (long long)((t + Team::size - 1) / Team::size) * t <= 768);
    bool have_list = false;  // the count list is already in acc
    if (MODE != NM_HASH && a.mcache && mcached(span, tflop) && !sym_tiny) {
        for (int s = tm.rank(); s < span; s += Team::size) {
            TileEntry z;
            z.mask = ld_cache(&a.mcache[(size_t)row * a.mc_stride + s]);
            z.base = 0;
            z.key = -1;
            E[s] = z;
        }
        tm.sync();
    } else if (a.mcache && !sym_tiny && (mlisted(span, tflop, t, a.mc_list) || lofs >= 0)) {
        // symbolic's compacted list of the t (key, mask) pairs (the row-cache slot, or a spill
        // list); a hashed row that ranks by counting also gets its (key, slot | popc) list
        // here, no table compaction later
        const unsigned long long* slot = lofs >= 0 ? a.sp.mask + lofs : a.mcache + (size_t)row * a.mc_stride;
        const int* skey = lofs >= 0 ? a.sp.key + lofs : reinterpret_cast<const int*>(slot + a.mc_list);
        // (round 5: a lane's first entries loaded before the clear and the rest 2-4 at a time
        // measured scircuit-like / cant-s1-like +1-2 % at 256 threads and 1024, cop20k-like -2..+4 %)
        clear_tiles(tm, E, H);
        if (MODE == NM_HASH && tm.rank() == 0) *counter = 0;
        tm.sync();
        for (int r = tm.rank(); r < t; r += Team::size) {
            const unsigned long long m = ld_cache(&slot[r]);
            const int key = ld_cache(&skey[r]);
            if (MODE != NM_HASH) {
                E[key - lo].mask = m;
            } else {
                int sl = hslot(key, H);
                MHS_GUARD_DECL;
                while (atomicCAS(&E[sl].key, -1, key) != -1) {  // keys are distinct
                    MHS_GUARD(H, 4, key);
                    probe_conflict();
                    sl = hnext(sl, H);
                }
                E[sl].mask = m;
                if (rank_count) reinterpret_cast<int2*>(acc)[r] = make_int2(key, (sl << 8) | __popcll(m));
            }
        }
        have_list = MODE == NM_HASH && rank_count;
        tm.sync();
    } else {
        clear_tiles(tm, E, H);
        if (MODE == NM_HASH && tm.rank() == 0) *counter = 0;
        tm.sync();
        build_tiles(tm, E, MODE != NM_HASH, lo, H, a0, a1, a.Acol, a.bmeta, a.btcol, a.btmask,
                    tflop, stage);
        tm.sync();
    }
    MHS_BSTAMP(1);

    if constexpr (GROUPED) group_pair_meta(gp, a.bmeta);
    // 2. rank of every tile's first column = prefix popcount in tile order
    if constexpr (MODE != NM_HASH) {
        tm.exclusive_scan(
            span, [&](int i) { return (int)__popcll(E[i].mask); },
            [&](int i, int v) { E[i].base = v; });
    } else if (rank_bitmap) {
        // block teams, tables of many tiles: rank by a bitmap over the span instead of a
        // sort -- bit per occupied tile, prefix popcount of the bitmap words, then a
        // tile's rank = word prefix + popc(word & below); bases = exclusive scan of the
        // masks' popcounts in rank order.  O(H + span/64 + t), no bitonic rounds.
        const int nw = (span + 63) >> 6;
        unsigned long long* bm = (unsigned long long*)acc;  // acc is free until the accumulate
        int* wpre = (int*)(bm + nw);
        int* cnt = wpre + ((nw + 3) & ~3);
        for (int i = tm.rank(); i < nw; i += Team::size) bm[i] = 0ull;
        tm.sync();
        for (int s = tm.rank(); s < H; s += Team::size) {
            const int key = E[s].key;
            if (key != -1) atomicOr(&bm[(key - lo) >> 6], 1ull << ((key - lo) & 63));
        }
        tm.sync();
        tm.exclusive_scan(
            nw, [&](int i) { return (int)__popcll(bm[i]); }, [&](int i, int v) { wpre[i] = v; });
        tm.sync();
        auto rank_of = [&](int key) {
            const int d = key - lo;
            return wpre[d >> 6] + (int)__popcll(bm[d >> 6] & ((1ull << (d & 63)) - 1));
        };
        for (int s = tm.rank(); s < H; s += Team::size) {
            const uint4 q = *reinterpret_cast<const uint4*>(&E[s]);
            if ((int)q.w != -1) cnt[rank_of((int)q.w)] = __popcll(((unsigned long long)q.y << 32) | q.x);
        }
        tm.sync();
        tm.exclusive_scan(
            t, [&](int i) { return cnt[i]; }, [&](int i, int v) { cnt[i] = v; });
        tm.sync();
        for (int s = tm.rank(); s < H; s += Team::size) {
            const int key = E[s].key;
            if (key != -1) E[s].base = cnt[rank_of(key)];
        }
    } else if (rank_count) {
        // few tiles: rank by counting.  Compact the table into (key, slot << 8 | popc)
        // pairs (a ballot per wave, one counter add per wave), then a tile's base = the
        // popcounts of the smaller keys summed over the list -- t compares per tile on
        // broadcast LDS reads, no sort rounds (t <= n: the list fits the accumulator).
        // (Counting ranks only -- four keys a read -- and scanning the popcounts in rank order
        // measured cop20k-like numeric +5 %, cage15-like neutral.)
        int2* L = (int2*)acc;  // acc is free until the accumulate
        const int lane = lane_id();
        for (int s0 = tm.rank() & ~63; !have_list && s0 < H; s0 += Team::size) {
            const int s = s0 + lane;
            uint4 q = make_uint4(0u, 0u, 0u, 0xFFFFFFFFu);
            if (s < H) q = *reinterpret_cast<const uint4*>(&E[s]);  // mask, base, key
            const bool occ = (int)q.w != -1;
            const unsigned long long bal = __ballot(occ);
            int at = 0;
            if (lane == 0 && bal) at = atomicAdd(counter, __popcll(bal));
            at = __shfl(at, 0);
            if (occ)
                L[at + __popcll(bal & lanemask_lt())] =
                    make_int2((int)q.w, (s << 8) | __popcll(((unsigned long long)q.y << 32) | q.x));
        }
        tm.sync();
        // (sorting the keys in registers instead -- bitonic over DPP -- measured cage15-like +3 %)
        for (int i = tm.rank(); i < t; i += Team::size) {
            const int2 me = L[i];
            int base = 0, j = 0;
            for (; j + 1 < t; j += 2) {  // two entries per broadcast read
                const int4 o = *reinterpret_cast<const int4*>(&L[j]);
                base += (o.x < me.x ? (o.y & 0xFF) : 0) + (o.z < me.x ? (o.w & 0xFF) : 0);
            }
            if (j < t) {
                const int2 o = L[j];
                base += o.x < me.x ? (o.y & 0xFF) : 0;
            }
            E[me.y >> 8].base = base;
        }
    } else {
        unsigned long long* S = (unsigned long long*)acc;
        const int P = next_pow2(t);
        for (int s = tm.rank(); s < H; s += Team::size) {
            const int key = E[s].key;
            if (key != -1) {
                const int idx = atomicAdd(counter, 1);
                S[idx] = ((unsigned long long)(unsigned)key << 32) | (unsigned)s;
            }
        }
        for (int i = t + tm.rank(); i < P; i += Team::size) S[i] = ~0ull;
        tm.sync();
        team_bitonic(tm, S, P);
        tm.exclusive_scan(
            t, [&](int e) { return (int)__popcll(E[(int)(unsigned)S[e]].mask); },
            [&](int e, int v) { E[(int)(unsigned)S[e]].base = v; });
    }
    tm.sync();
    MHS_BSTAMP(2);
    for (int r = tm.rank(); r < nclear; r += Team::size) acc[r] = 0.0;
    tm.sync();
    MHS_BSTAMP(3);

    // 3. accumulate every product of the row (of the group's rows)
    {
        const Accum<GLOBALMEM, MODE, O32> f{E, acc, lo, H, colbase, a.Bcol, a.Bval, a.ubase};
        if constexpr (GROUPED) {
            const int nAr = a1 - a0;
            const int avg = nAr > 0 ? (__builtin_amdgcn_readfirstlane(a.rflop[row]) + nAr - 1) / nAr : 1;
            // a near group walks its union row (columns at the head's A offset, R value slices
            // nU apart from 3 * Aptr[head]): row r's value of union entry j at uv[a0 + j + r * nU]
            // with uv = uval + 2 * a0 (gcol / gval above).  (One call site: two inlined walks
            // doubled the registers.)
            for_products_group(gp, a0, a0 + gnw, gcol, gval, a.bmeta, avg, f, R, gnw, stride);
        } else {
            walk_products(tm, a0, a1, a.Acol, a.Aval, a.bmeta, false, a.rflop[row], f, stage);
        }
    }
    tm.sync();
    MHS_BSTAMP(4);

    // 4. write C (sorted by construction: tiles in column order, bits in order)
    if constexpr (MODE == NM_DENSE) {
        // one wave per tile, lane = bit: compaction of the dense accumulator
        const int lane = lane_id();
        const int nw = Team::size / 64, wv = tm.rank() >> 6;
        for (int s = wv; s < span; s += nw) {
            const TileEntry e = E[s];
            if ((e.mask >> lane) & 1ull) {
                const int pos = c0 + e.base + __popcll(e.mask & lanemask_lt());
                for (int g = 0; g < (GROUPED ? R : 1); ++g) {
                    st_part(&a.Ccol[pos + g * n], colbase + (s << TILE_SHIFT) + lane);
                    st_part(&a.Cval[pos + g * n], acc[g * stride + (s << TILE_SHIFT) + lane]);
                }
            }
        }
    } else {
        // C.val two a lane and C.col four a lane: 16-byte stores, half and a quarter of the store
        // instructions of one entry a lane (the accumulator slices are 16-byte aligned); the
        // columns staged in LDS by tile first (a lane per tile of <= 8 columns, else the whole
        // wave, lane = bit).  Measured (round 4): cant-like numeric -4 %, pwtk- / shipsec1-like
        // -15 %, hood-like -8 %, cage15-like -7 % -- the walks' loads and the output's stores
        // share the texture pipeline, which the 8- and 4-byte stores held
        for (int g = 0; g < (GROUPED ? R : 1); ++g)
            store_vals(a.Cval + c0 + g * n, acc + g * stride, n, tm.rank(), Team::size);
        tm.sync();
        MHS_BSTAMP(6);  // (stamps builds: the output phase split in three -- values, staging, columns)
        int* cb = (int*)acc;
        stage_cols<MODE != NM_HASH>(E, H, lo, cb, tm.rank(), Team::size);
        tm.sync();
        MHS_BSTAMP(7);
        store_cols(a.Ccol + c0, cb, n, GROUPED ? R : 1, tm.rank(), Team::size);
    }
    tm.sync();
    MHS_BSTAMP(5);
}

// Row-level scalars are made provably wave-uniform (readfirstlane) so that the
// mode dispatch and every per-row loop bound compile to scalar control flow.
// ------------------------------------------------------------ wide rows ---
// Rows whose tile tables would not fit a wave (scattered over a wide column range,
// e.g. power-law rows touching hub columns): no hash and no tile sort.  The block
// walks the row's tile span in windows of WIDE_WT tiles; per window the LDS holds a
// dense 64-bit mask per tile and a C-row base per 4 tiles (9 bytes per tile), and the
// products accumulate straight into the row's slice of C.val with global FP64
// atomics (zeroed first).  A product's rank = base4[g] + popcounts of the masks of
// the tiles before it in its group of 4 + popc(mask & below(col)).


struct WideAccum {
    static constexpr bool kValues = true;
    static constexpr bool kUnion = false;
    static constexpr bool kPairs = false;  // wave walks may stage chunk pairs (registers)
    const unsigned long long* masks;
    const int* base4;
    int w0, w1;
    double* crow;  // C.val + c0
    const int* __restrict__ Bcol;
    const double* __restrict__ Bval;
    struct Item {
        int c;
        double v;
    };
    __device__ __forceinline__ Item load(int i) const { return Item{Bcol[i], Bval[i]}; }
    __device__ __forceinline__ void put(const Item& x, double a) const { add(x.c, a * x.v); }
    __device__ __forceinline__ int col(int i) const { return Bcol[i]; }
    __device__ __forceinline__ double val(int i) const { return Bval[i]; }
    __device__ __forceinline__ void add(int c, double v) const {
        const int tc = c >> TILE_SHIFT;
        if (tc < w0 || tc >= w1) return;
        const int sl = tc - w0, g = sl >> 2;
        int idx = base4[g];
        for (int k = g << 2; k < sl; ++k) idx += __popcll(masks[k]);
        idx += __popcll(masks[sl] & ((1ull << (c & (TILE_BITS - 1))) - 1));
        unsafeAtomicAdd(&crow[idx], v);
    }
    template <int RM>
    __device__ __forceinline__ void add_rows(int, const double (&)[RM], int, int) const {}
};

template <int T>
__device__ void num_row_wide(const BlockTeam<T, false>& tm, const NumArgs& a, int row, int lo, int hi, int c0,
                             int n, int a0, int a1, char* region, int4* stage) {
    unsigned long long* masks = (unsigned long long*)region;
    int* base4 = (int*)(region + (size_t)WIDE_WT * 8);
    double* crow = a.Cval + c0;
    const int tflop = __builtin_amdgcn_readfirstlane(a.rtflop[row]);
    const int flop = __builtin_amdgcn_readfirstlane(a.rflop[row]);
    for (int r = tm.rank(); r < n; r += T) crow[r] = 0.0;
    __threadfence();  // the zeros are visible to the (memory-side) atomics below
    int carry = 0;    // C entries in earlier windows
    for (int w0 = lo; w0 <= hi; w0 += WIDE_WT) {
        const int w1 = min(hi + 1, w0 + WIDE_WT), wt = w1 - w0;
        for (int sl = tm.rank(); sl < wt; sl += T) masks[sl] = 0ull;
        tm.sync();
        walk_products(tm, a0, a1, a.Acol, nullptr, a.bmeta, true, tflop,
                      WideTiles{masks, w0, w1, a.btcol, a.btmask}, stage);
        tm.sync();
        const int ng = (wt + 3) >> 2;
        tm.exclusive_scan(
            ng,
            [&](int g) {
                int c = 0;
                for (int k = g << 2; k < min(wt, (g << 2) + 4); ++k) c += __popcll(masks[k]);
                return c;
            },
            [&](int g, int v) { base4[g] = carry + v; });
        tm.sync();
        walk_products(tm, a0, a1, a.Acol, a.Aval, a.bmeta, false, flop,
                      WideAccum{masks, base4, w0, w1, crow, a.Bcol, a.Bval}, stage);
        // column indices of the window: a thread per group of 4 tiles (scattered rows
        // hold a few bits per tile), bits in order
        int wc = 0;
        for (int g = tm.rank(); g < ng; g += T) {
            int idx = base4[g];
            for (int k = g << 2; k < min(wt, (g << 2) + 4); ++k) {
                unsigned long long m = masks[k];
                wc += __popcll(m);
                while (m) {
                    st_part(&a.Ccol[c0 + idx++], ((w0 + k) << TILE_SHIFT) + __builtin_ctzll(m));
                    m &= m - 1;
                }
            }
        }
        carry += tm.sum(wc);  // (sum syncs: the masks are free for the next window)
    }
}

// Numeric rank-by-bitmap row (block kernels): the two tile walks of sym_row_bitmap, the
// C-row base of every rank by one scan in column order, then each product lands at
// base[rank] + popc(msk[rank] & below(col)) in an LDS accumulator (no global atomics).
template <bool GM, bool O32 = false>
struct RankAccum {
    static constexpr bool kValues = true;
    static constexpr bool kUnion = false;
    static constexpr bool kPairs = false;  // wave walks may stage chunk pairs (registers)
    const unsigned long long* bm;
    const int* wpre;
    const unsigned long long* msk;
    const int2* kb;
    double* acc;
    int lo;
    const int* __restrict__ Bcol;
    const double* __restrict__ Bval;
    struct Item {
        int c;
        double v;
    };
    __device__ __forceinline__ Item load(int i) const { return Item{ld_idx<O32>(Bcol, i), ld_idx<O32>(Bval, i)}; }
    __device__ __forceinline__ int col(int i) const { return ld_idx<O32>(Bcol, i); }
    __device__ __forceinline__ double val(int i) const { return ld_idx<O32>(Bval, i); }
    __device__ __forceinline__ void put(const Item& x, double a) const { add(x.c, a * x.v); }
    __device__ __forceinline__ void add(int c, double v) const {
        const int r = span_rank(bm, wpre, (c >> TILE_SHIFT) - lo);
        const int idx = kb[r].y + (int)__popcll(msk[r] & ((1ull << (c & (TILE_BITS - 1))) - 1));
        acc_add<GM>(&acc[idx], v);
    }
    template <int RM>
    __device__ __forceinline__ void add_rows(int, const double (&)[RM], int, int) const {}
};

template <int T, bool O32>
__device__ void num_row_bitmap(const BlockTeam<T, false>& tm, const NumArgs& a, int row, int lo, int span, int t,
                               int c0, int n, int a0, int a1, char* region, int4* stage) {
    const int nw = (span + 63) >> 6;
    const long long sb = span_bits_bytes(span);
    unsigned long long* bm = (unsigned long long*)region;
    int* wpre = (int*)(region + align16((long long)nw * 8));
    unsigned long long* msk = (unsigned long long*)(region + sb);
    int2* kb = (int2*)(region + sb + align16((long long)t * 8));
    double* acc = (double*)(region + sb + 2 * align16((long long)t * 8));
    MHS_STAMP0();
    const int tflop = __builtin_amdgcn_readfirstlane(a.rtflop[row]);
    const int lofs = (a.mcache && spill_row(span, tflop, t, a.mc_list))
                         ? __builtin_amdgcn_readfirstlane(a.sp.lofs[row])
                         : -1;
    MHS_STAMP(0);
    for (int i = tm.rank(); i < nw; i += T) bm[i] = 0ull;
    for (int r = tm.rank(); r < t; r += T) msk[r] = 0ull;
    tm.sync();
    if (lofs >= 0) {
        // symbolic's spill list (column order): the bits and the ranked masks from t entries
        // instead of two walks over every product of the row
        for (int r = tm.rank(); r < t; r += T) {
            const int d = ld_cache(&a.sp.key[lofs + r]) - lo;
            atomicOr(&bm[d >> 6], 1ull << (d & 63));
        }
        tm.sync();
        tm.exclusive_scan(
            nw, [&](int i) { return (int)__popcll(bm[i]); }, [&](int i, int v) { wpre[i] = v; });
        for (int r = tm.rank(); r < t; r += T) {
            const int key = ld_cache(&a.sp.key[lofs + r]);
            const int k = span_rank(bm, wpre, key - lo);
            msk[k] = ld_cache(&a.sp.mask[lofs + r]);
            kb[k].x = key;
        }
    } else {
        walk_products(tm, a0, a1, a.Acol, nullptr, a.bmeta, true, tflop, SpanBits{bm, lo, a.btcol}, stage);
        tm.sync();
        tm.exclusive_scan(
            nw, [&](int i) { return (int)__popcll(bm[i]); }, [&](int i, int v) { wpre[i] = v; });
        walk_products(tm, a0, a1, a.Acol, nullptr, a.bmeta, true, tflop,
                      RankedMasks{bm, wpre, msk, kb, lo, a.btcol, a.btmask}, stage);
    }
    tm.sync();
    MHS_STAMP(1);
    tm.exclusive_scan(
        t, [&](int r) { return (int)__popcll(msk[r]); }, [&](int r, int v) { kb[r].y = v; });
    MHS_STAMP(2);
    for (int r = tm.rank(); r < n; r += T) acc[r] = 0.0;
    tm.sync();
    MHS_STAMP(3);
    walk_products(tm, a0, a1, a.Acol, a.Aval, a.bmeta, false, __builtin_amdgcn_readfirstlane(a.rflop[row]),
                  RankAccum<false, O32>{bm, wpre, msk, kb, acc, lo, a.Bcol, a.Bval}, stage);
    tm.sync();
    MHS_STAMP(4);
    store_vals(a.Cval + c0, acc, n, tm.rank(), T);
    tm.sync();  // the accumulator region now stages the column indices
    int* cb = (int*)acc;
    for (int r = tm.rank(); r < t; r += T) {
        unsigned long long m = msk[r];
        const int2 e = kb[r];
        int b = e.y;
        while (m) {
            cb[b++] = (e.x << TILE_SHIFT) + __builtin_ctzll(m);
            m &= m - 1;
        }
    }
    tm.sync();
    store_cols(a.Ccol + c0, cb, n, 1, tm.rank(), T);
    tm.sync();
    MHS_STAMP(5);
}

// MODES: which row bodies a kernel instantiates (the binning sends a row only to a
// kernel that has its mode): the hash body's register sort would otherwise set the
// register budget -- and the occupancy -- of the direct-mapped wave kernels too.
enum NumModes : int { MODES_ALL = 0, MODES_NOHASH = 1, MODES_HASH = 2 };

// Row-level scalars are made provably wave-uniform (readfirstlane) so that the
// mode dispatch and every per-row loop bound compile to scalar control flow.
struct NumRow {
    int row, lo, hi, t, c0, n, a0, a1;
};
template <class Team, bool GLOBALMEM, bool GROUPED = false, int MODES = MODES_ALL, bool O32 = false>
__device__ __forceinline__ void num_row_s(const Team& tm, const NumArgs& a, const NumRow& r, char* region,
                                          int* counter, int4* stage, int R = 1);
template <class Team, bool GLOBALMEM, bool GROUPED = false, int MODES = MODES_ALL, bool O32 = false>
__device__ __forceinline__ void num_row(const Team& tm, const NumArgs& a, int row, char* region, int* counter,
                        int4* stage, int R = 1) {
    NumRow r;
    r.row = row;
    r.lo = __builtin_amdgcn_readfirstlane(a.rlo[row]);
    r.hi = __builtin_amdgcn_readfirstlane(a.rhi[row]);
    r.t = __builtin_amdgcn_readfirstlane(a.ctiles[row]);
    r.c0 = __builtin_amdgcn_readfirstlane(a.Cptr[row]);
    r.n = __builtin_amdgcn_readfirstlane(a.Cptr[row + 1]) - r.c0;
    r.a0 = __builtin_amdgcn_readfirstlane(a.Aptr[row]);
    r.a1 = __builtin_amdgcn_readfirstlane(a.Aptr[row + 1]);
    num_row_s<Team, GLOBALMEM, GROUPED, MODES, O32>(tm, a, r, region, counter, stage, R);
}
template <class Team, bool GLOBALMEM, bool GROUPED, int MODES, bool O32>
__device__ __forceinline__ void num_row_s(const Team& tm, const NumArgs& a, const NumRow& r, char* region,
                                          int* counter, int4* stage, int R) {
    const int row = r.row, lo = r.lo, hi = r.hi, t = r.t, c0 = r.c0, n = r.n, a0 = r.a0, a1 = r.a1;
    const int span = hi - lo + 1;
    const int mode = num_mode(span, t, n, a.dense_span_max);
    if constexpr (MODES == MODES_HASH) {
        num_row_body<Team, GLOBALMEM, NM_HASH, GROUPED, O32>(tm, a, row, lo, span, t, c0, n, a0, a1, region, counter, stage, R);
        return;
    }
    if (mode == NM_DENSE)
        num_row_body<Team, GLOBALMEM, NM_DENSE, GROUPED, O32>(tm, a, row, lo, span, t, c0, n, a0, a1, region, counter, stage, R);
    else if (MODES == MODES_NOHASH || mode == NM_DIRECT)
        num_row_body<Team, GLOBALMEM, NM_DIRECT, GROUPED, O32>(tm, a, row, lo, span, t, c0, n, a0, a1, region, counter, stage, R);
    else
        num_row_body<Team, GLOBALMEM, NM_HASH, GROUPED, O32>(tm, a, row, lo, span, t, c0, n, a0, a1, region, counter, stage, R);
}


template <int BYTES, bool GROUPED, bool HASH, bool O32>
__device__ __forceinline__ void num_wave_rows(const NumArgs& a, int bid = -1, int nb = -1) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (bid < 0) {  // (a role of a fused launch passes its own sub-grid)
        bid = (int)blockIdx.x;
        nb = (int)gridDim.x;
    }
    const int w = threadIdx.x >> 6;
    char* reg = smem + w * (GROUPED && a.wave_bytes > 0 ? a.wave_bytes : BYTES);  // (grouped: sized to the bin)
    WaveTeam tm;
    auto one = [&](int li) {
        const int row = __builtin_amdgcn_readfirstlane(a.list[li]);
        MHS_FLIGHT_ROW(row, li);
        if constexpr (GROUPED)  // a group head: R rows of one pattern
            num_row<WaveTeam, false, true, MODES_ALL, O32>(tm, a, row, reg + WAVE_HDR, (int*)reg, nullptr,
                                                         __builtin_amdgcn_readfirstlane((int)a.grp[row]) & GRP_RMASK);
        else
            num_row<WaveTeam, false, false, HASH ? MODES_HASH : MODES_NOHASH, O32>(tm, a, row, reg + WAVE_HDR,
                                                                             (int*)reg, nullptr);
    };
    // The 10 KiB bins (16 KiB before round 3) hold the heaviest wave rows (power-law rows of hundreds of tiles, a
    // few rows per wave): a static stride leaves the launch's end to the wave that drew the
    // heaviest ones.  Guided walk: each XCD group's waves stride statically through the first
    // MHS_GUIDED_STATIC/8 of its eighth of the list (row locality, no atomics), then take the
    // rest one row at a time from the group's cursor.  Measured (profiles/r02p_guided): hash
    // bin guided with half static: wb-edu-like numeric -4 %, webbase-like -2 %, cage15-like and
    // pdb1HYS-like neutral; the whole bin from the cursor (2 rows a take): wb-edu -12 %,
    // webbase -10 %, but cage15 +3.5 %; the direct / grouped 16 KiB bins guided: pdb1HYS +10 %.
    constexpr bool guided = BYTES == NUM_W16_BYTES && HASH;
    // (round 5: the small hash bin from the XCD groups' cursors, 2-8 rows a take, measured
    // cage15-like +3 %, cop20k-like +16 %, offshore-like +14 %)
    if (guided && a.qall) {
        WaveQueue q(a.cursor, a.count, 1);
        for (int li; q.next(li);) one(li);
    } else if (guided && (gridDim.x & 7) == 0) {
        const int g = (int)(blockIdx.x & 7);
        const int begin = (int)((long long)a.count * g / 8), end = (int)((long long)a.count * (g + 1) / 8);
        const int split = begin + (int)((long long)(end - begin) * MHS_GUIDED_STATIC / 8);
        const int stride = (int)(gridDim.x >> 3) * WPB;
        for (int li = begin + (int)(blockIdx.x >> 3) * WPB + w; li < split; li += stride) one(li);
        int* cur = a.cursor + g * CURSOR_STRIDE;
        for (;;) {
            int t = 0;
            if (lane_id() == 0) t = atomicAdd(cur, 1);
            const int li = split + __builtin_amdgcn_readfirstlane(t);
            MHS_FLIGHT_TAKE(li);
            if (li >= end) break;
            one(li);
        }
    } else {
        for (RowWalk rw(a.count, WPB, w, bid, nb); rw.first < rw.end; rw.first += rw.stride) one(rw.first);
    }
}

template <int BYTES, bool GROUPED = false, bool HASH = false, bool O32 = false>
#if MHS_GRP_PIPE > 1
#define MHS_GRP_WPE MHS_WPE_ATTR(4)
#else
#define MHS_GRP_WPE
#endif
__global__ __launch_bounds__(256) MHS_GRP_WPE void k_num_wave(NumArgs a) {
    MHS_PLAN_GUARD(a);
    num_wave_rows<BYTES, GROUPED, HASH, O32>(a);
}
template <int BYTES, bool O32 = false>
__global__ __launch_bounds__(256) MHS_WPE_ATTR(BYTES > NUM_WS_BYTES ? MHS_WPE_HASH16 : MHS_WPE_HASH) void k_num_wave_hash(NumArgs a) {
    MHS_PLAN_GUARD(a);
    num_wave_rows<BYTES, false, true, O32>(a);
}
template <int BYTES, bool O32 = false>
__global__ __launch_bounds__(256) MHS_WPE_ATTR(MHS_WPE_DIRECT) void k_num_wave_direct(NumArgs a) {
    MHS_PLAN_GUARD(a);
    num_wave_rows<BYTES, false, false, O32>(a);
}

template <int T, bool GLOBALMEM, bool O32 = false>
__global__ __launch_bounds__(T) void k_num_block(NumArgs a) {
    MHS_PLAN_GUARD(a);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    BlockTeam<T, GLOBALMEM> tm{(long long*)smem};
    char* reg = GLOBALMEM ? (a.gscratch + (long long)blockIdx.x * a.gbytes) : (smem + block_hdr(T));
    int* counter = (int*)(smem + 128);
    int4* stage = (int4*)(smem + 1024);
    __shared__ int qslot;
    const BlockQueue q{a.cursor, &qslot, a.count};
    for (int li; q.next(li);) {
        const int row = __builtin_amdgcn_readfirstlane(a.list[li]);
        if constexpr (T == 1024 && !GLOBALMEM) {
            const int lo = __builtin_amdgcn_readfirstlane(a.rlo[row]);
            const int hi = __builtin_amdgcn_readfirstlane(a.rhi[row]);
            const int t = __builtin_amdgcn_readfirstlane(a.ctiles[row]);
            const int c0 = __builtin_amdgcn_readfirstlane(a.Cptr[row]);
            const int n = __builtin_amdgcn_readfirstlane(a.Cptr[row + 1]) - c0;
            if (num_ranked(hi - lo + 1, t, n, a.dense_span_max)) {
                num_row_bitmap<T, O32>(tm, a, row, lo, hi - lo + 1, t, c0, n, __builtin_amdgcn_readfirstlane(a.Aptr[row]),
                                  __builtin_amdgcn_readfirstlane(a.Aptr[row + 1]), reg, stage);
                continue;
            }
            if (num_wide(hi - lo + 1, t, n, a.dense_span_max)) {
                num_row_wide<T>(tm, a, row, lo, hi, c0, n, __builtin_amdgcn_readfirstlane(a.Aptr[row]),
                                __builtin_amdgcn_readfirstlane(a.Aptr[row + 1]), reg, stage);
                tm.sync();
                continue;
            }
        }
        num_row<BlockTeam<T, GLOBALMEM>, GLOBALMEM, false, MODES_ALL, O32>(tm, a, row, reg, counter, stage);
    }
}

// ------------------------------------------------------------- tiny rows ---
// Rows of at most W*K products (and W A entries): a team of W lanes per row holding
// K products per lane, slot-major (product p = i*W + lane in slot i).  Lane p finds
// its A entry by a binary search over the team's inclusive scan of B-row lengths,
// loads its (column, value), and the team sorts the W*K pairs by column (bitonic in
// registers: element e = i*W + lane, partners across lanes by shuffles for d < W and
// across slots in the lane for d >= W); equal columns are then adjacent: heads count
// the row (symbolic) or close a segmented sum (numeric).  No table and no LDS, and
// several rows per wave -- where a wave per row would idle most lanes through ten
// dependent loads.
struct TinyArgs {
    int M, count, bin;  // count < 0: the bin's size on the device (the symbolic launch)
    int nft;            // symbolic launch: numeric-first slot rows (the numeric classes; see k_analyze)
    const int* Aptr;
    const int* Acol;
    const double* Aval;
    const int4* bmeta;
    const int* Bcol;
    const double* Bval;
    const int* list;  // the bin's rows
    const Stats* stats;
    const unsigned char* grp;
    const int* rlo;   // numeric: the row's first tile (sort keys are columns relative to it)
    int* Cptr;
    int* ctiles;
    int* Ccol;
    double* Cval;
    // numeric-first: the symbolic launch sums the rows into value slots (class c's from
    // sbase on: W*K entries per row of its list; a wave's rows packed at the start of
    // their slots' span), the row's nnz goes to Cptr[row] and its slot to tslot[row];
    // k_tiny_copy moves them into C
    int* sc_col;
    double* sc_val;
    long long* tslot;
    long long sbase;
    int blk0[TINY_SYMX_NC + 1];  // slots: class c takes blocks [blk0[c], blk0[c+1]) (sized on the host)
    const int* go;               // numeric launches of a speculated plan (see NumArgs)
};

template <int W, int K, bool NUMERIC>
__device__ __forceinline__ void tiny_rows(const TinyArgs& a, int bid, int nb) {
    static_assert((W & (W - 1)) == 0 && W <= 64 && (K & (K - 1)) == 0 && W * K <= (1 << TINY_EBITS), "team shape");
    const int count = a.count >= 0 ? a.count : a.stats->sym_count[a.bin];
    const bool slots = NUMERIC && a.sc_col != nullptr;  // numeric-first: into value slots
    const RowWalk rw(count, 256 / W, (int)(threadIdx.x / W), bid, nb);
    extern __shared__ __attribute__((aligned(16))) char tiny_smem[];
    double* vstage = (double*)tiny_smem + (size_t)(threadIdx.x / W) * (W * K);  // numeric: W*K doubles per team
    // the wave iterates while any of its teams has a row (shuffles need every lane).  A team's
    // next row (list entry, then its A pointers) is loaded a round ahead, under this row's chain
    int it = rw.first;
    int nrow = 0, na0 = 0, na1 = 0;
    if (MHS_TINY_PF && it < rw.end) {
        nrow = a.list[it];
        na0 = a.Aptr[nrow];
        na1 = a.Aptr[nrow + 1];
    }
    for (; __ballot(it < rw.end) != 0; it += rw.stride) {
        // the lane's team masks, rebuilt every row from an opaque lane id: hoisted, they stayed
        // live across the fused kernels' class dispatch and went to scratch (64-VGPR budget)
        int lane = lane_id();
        asm volatile("" : "+v"(lane));
        const int tl = lane & (W - 1);   // lane in the team
        const int tb = lane & ~(W - 1);  // the team's first lane
        const unsigned long long tmask = W == 64 ? ~0ull : (((1ull << (W & 63)) - 1) << tb);
        const unsigned long long below = tmask & (lane == 0 ? 0ull : (~0ull >> (64 - lane)));
        const bool live = it < rw.end;
        const int row = MHS_TINY_PF ? nrow : live ? a.list[it] : 0;
        const int a0 = MHS_TINY_PF ? na0 : live ? a.Aptr[row] : 0;
        const int nA = !live ? 0 : MHS_TINY_PF ? na1 - na0 : a.Aptr[row + 1] - a0;
        const bool ln = it + rw.stride < rw.end;
        if (MHS_TINY_PF) nrow = ln ? a.list[it + rw.stride] : 0;
        long long c0 = (NUMERIC && live && !slots) ? a.Cptr[row] : 0;  // issued early: off the tail's chain
        const int cb = (NUMERIC && live) ? (a.rlo[row] << TILE_SHIFT) : 0;  // key origin (23-bit offsets)
        int st = 0, len = 0;
        double av = 0.0;
        if (tl < nA) {
            const int4 m = a.bmeta[a.Acol[a0 + tl]];
            st = m.x;
            len = m.y;
            if (NUMERIC) av = a.Aval[a0 + tl];
        }
        const int incl = team_incl_scan<W>(len, tl);  // inclusive scan of the B-row lengths over the team
        const int flop = __shfl(incl, tb + W - 1);
        const int excl = incl - len;
        // sort keys: symbolic the column; numeric (column << TINY_EBITS) | element, the
        // value parked in the team's LDS slice at its element and fetched after the sort
        unsigned key[K];
        int q[K];
        bool valid[K];
        double avs[K];
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const int p = i * W + tl;
            int j = 0;  // product p belongs to entry j: the first with incl_j > p
#pragma unroll
            for (int step = W / 2; step >= 1; step >>= 1) {
                const int x = __shfl(incl, tb + j + step - 1);
                j += x <= p ? step : 0;
            }
            valid[i] = p < flop;
            const int src = tb + (valid[i] ? j : 0);
            const int stj = __shfl(st, src);
            const int exj = __shfl(excl, src);
            avs[i] = NUMERIC ? __shfl(av, src) : 0.0;  // shuffles outside any branch: every lane
            q[i] = valid[i] ? stj + (p - exj) : 0;      // clamped: every slot's loads issue together
        }
        int bc[K];
        double bv[K];
#pragma unroll
        for (int i = 0; i < K; ++i) {
            bc[i] = a.Bcol[q[i]];
            if (NUMERIC) bv[i] = a.Bval[q[i]];
        }
        if (MHS_TINY_PF) {  // (after this row's B loads: the next row's pointers wait on its list entry)
            na0 = ln ? a.Aptr[nrow] : 0;
            na1 = ln ? a.Aptr[nrow + 1] : 0;
        }
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const unsigned c = (unsigned)bc[i];
            key[i] = !valid[i] ? 0xFFFFFFFFu : NUMERIC ? ((c - (unsigned)cb) << TINY_EBITS) | (unsigned)(i * W + tl) : c;
            if (NUMERIC) vstage[i * W + tl] = avs[i] * bv[i];
        }
        reg_bitonic<W, K>(key, tl);
        int c[K];
#pragma unroll
        for (int i = 0; i < K; ++i)
            c[i] = key[i] == 0xFFFFFFFFu ? INT_MAX : (int)(NUMERIC ? (key[i] >> TINY_EBITS) + (unsigned)cb : key[i]);
        double v[K];
        if constexpr (NUMERIC) {  // each sorted slot fetches its element's value
            wave_sync();
#pragma unroll
            for (int i = 0; i < K; ++i) {
                const int e = (int)(key[i] & ((1u << TINY_EBITS) - 1));
                v[i] = c[i] == INT_MAX ? 0.0 : vstage[e];
            }
            wave_sync();  // the slice is rewritten by the team's next row
        }
        // heads: element e differs from e-1 (slot i lane tl-1, or slot i-1 lane W-1)
        bool head[K];
        int nnz = 0, ntl = 0;
        int prev_last = INT_MAX;  // slot i-1's last element (lane W-1)
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const int up = __shfl_up(c[i], 1, W);
            const int pc = tl == 0 ? (i == 0 ? -1 : prev_last) : up;
            head[i] = c[i] != INT_MAX && pc != c[i];
            if constexpr (!NUMERIC) {
                const bool thead = c[i] != INT_MAX && (pc < 0 || (pc >> TILE_SHIFT) != (c[i] >> TILE_SHIFT));
                ntl += __popcll(__ballot(thead) & tmask);
            }
            nnz += __popcll(__ballot(head[i]) & tmask);
            prev_last = __shfl(c[i], tb + W - 1);
        }
        if (slots) {  // the wave's rows own the slots of list entries [it0, it0 + 64/W): packed
            const int x = (tl == 0 && live) ? nnz : 0;
            const int inc = wave_incl_scan(x);
            c0 = a.sbase + (long long)__shfl(it, 0) * (W * K) + __shfl(inc - x, tb);
        }
        if constexpr (!NUMERIC) {
            const int R = live ? (int)a.grp[row] : 0;  // a group head: its rows share the count
            if (tl < R) {
                a.Cptr[row + tl] = nnz;
                a.ctiles[row + tl] = ntl;
            }
        } else {
            // segmented inclusive sums (segments start at heads), carried across slots
            double carry = 0.0;  // open segment's sum at the end of slot i-1
            int rank0 = 0;       // heads in slots < i
#pragma unroll
            for (int i = 0; i < K; ++i) {
                // the lane's segment began in this slot iff a head sits at or below it in the team
                const bool seen = (__ballot(head[i]) & tmask & (below | (1ull << lane))) != 0;
                double sum = team_seg_scan<W>(v[i], head[i], tl);
                sum += seen ? 0.0 : carry;  // the segment began in an earlier slot
                const int nc = __shfl_down(c[i], 1, W);
                const int nxt = i + 1 < K ? __shfl(c[i + 1 < K ? i + 1 : i], tb) : INT_MAX;
                const int next = tl == W - 1 ? nxt : nc;
                const bool last = c[i] != INT_MAX && next != c[i];
                const unsigned long long hb = __ballot(head[i]) & tmask;
                if (live && last) {
                    const long long pos = c0 + rank0 + __popcll(hb & (below | (1ull << lane))) - 1;
                    st_part(&(slots ? a.sc_col : a.Ccol)[pos], c[i]);
                    st_part(&(slots ? a.sc_val : a.Cval)[pos], sum);
                }
                carry = __shfl(sum, tb + W - 1);
                rank0 += __popcll(hb);
            }
            if (slots && live && tl == 0) {
                a.Cptr[row] = rank0;
                a.tslot[row] = c0;
            }
        }
    }
}

template <int W, int K>
__global__ __launch_bounds__(256) MHS_WPE_ATTR(MHS_WPE_TINY) void k_tiny_num(TinyArgs a) {
    MHS_PLAN_GUARD(a);
    tiny_rows<W, K, true>(a, (int)blockIdx.x, (int)gridDim.x);
}

// The 32-lane-or-narrower numeric tiny classes in one launch: class f.c[k] takes blocks
// [f.blk0[k], f.blk0[k+1]) (sizes known on the host; multiples of 8 keep the XCD walk).
struct TinyFused {
    int nclass;
    int c[4];
    int count[4];
    int blk0[5];
};
__global__ __launch_bounds__(256) MHS_WPE_ATTR(8) void k_tiny_num_small(TinyArgs a, TinyFused f) {
    MHS_PLAN_GUARD(a);
    int k = 0;
    while (k + 1 < f.nclass && (int)blockIdx.x >= f.blk0[k + 1]) ++k;
    const int bid = (int)blockIdx.x - f.blk0[k], nb = f.blk0[k + 1] - f.blk0[k];
    a.count = f.count[k];
    a.bin = NUM_TINY + f.c[k];
    a.list += (long long)(a.bin - 1) * a.M;
    switch (f.c[k]) {
    case 0: tiny_rows<tiny_w(0), tiny_k(0), true>(a, bid, nb); break;
    case 1: tiny_rows<tiny_w(1), tiny_k(1), true>(a, bid, nb); break;
    case 2: tiny_rows<tiny_w(2), tiny_k(2), true>(a, bid, nb); break;
    default: tiny_rows<tiny_w(3), tiny_k(3), true>(a, bid, nb); break;
    }
}

// Every symbolic tiny class in one launch (the bins' sizes are on the device): blocks
// [TINY_SYM_GRID*c, TINY_SYM_GRID*(c+1)) walk class c's list.
constexpr int TINY_SYM_GRID = 1024;
__device__ __forceinline__ void tiny_sym_rows(TinyArgs a, int blk) {
    int c = blk / TINY_SYM_GRID, bid = blk % TINY_SYM_GRID, nb = TINY_SYM_GRID;
    if (a.nft) {  // numeric-first slots: the grid follows the bins' sizes, as numeric's does
        // (constant indices only: a dynamically indexed kernel argument goes to scratch)
        static_assert(TINY_SYM_NC == 4 && TINY_SYMX_NC == 5, "class ranges below");
        const int b1 = a.blk0[1], b2 = a.blk0[2], b3 = a.blk0[3], b4 = a.blk0[4], b5 = a.blk0[5];
        c = (blk >= b1) + (blk >= b2) + (blk >= b3) + (blk >= b4);
        const int lo = c == 0 ? 0 : c == 1 ? b1 : c == 2 ? b2 : c == 3 ? b3 : b4;
        const int hi = c == 0 ? b1 : c == 1 ? b2 : c == 2 ? b3 : c == 3 ? b4 : b5;
        bid = blk - lo;
        nb = hi - lo;
    }
    static_assert(TINY_NC == 6 && TINY_SYM_NC == 4 && tiny_ws(3) <= 32 && tiny_w(3) <= 32 && tiny_w(4) == 64 &&
                      tiny_w(5) == 64 && tiny_ws(4) == 64,
                  "k_tiny_sym / launch_tiny_num instantiate the classes of tiny_class()");
    a.bin = SYM_TINY + c;
    a.list += (long long)c * a.M;
    if (c == 4) {  // the scattered class counts only, in either mode
        tiny_rows<tiny_ws(4), tiny_ks(4), false>(a, bid, nb);
        return;
    }
    if (!a.nft) {
        switch (c) {
        case 0: tiny_rows<tiny_ws(0), tiny_ks(0), false>(a, bid, TINY_SYM_GRID); break;
        case 1: tiny_rows<tiny_ws(1), tiny_ks(1), false>(a, bid, TINY_SYM_GRID); break;
        case 2: tiny_rows<tiny_ws(2), tiny_ks(2), false>(a, bid, TINY_SYM_GRID); break;
        default: tiny_rows<tiny_ws(3), tiny_ks(3), false>(a, bid, TINY_SYM_GRID); break;
        }
        return;
    }
    // numeric-first: the numeric classes' shapes; class c's slots follow classes < c
    for (int k = 0; k < c; ++k) a.sbase += (long long)a.stats->sym_count[SYM_TINY + k] * (tiny_w(k) * tiny_k(k));
    switch (c) {
    case 0: tiny_rows<tiny_w(0), tiny_k(0), true>(a, bid, nb); break;
    case 1: tiny_rows<tiny_w(1), tiny_k(1), true>(a, bid, nb); break;
    case 2: tiny_rows<tiny_w(2), tiny_k(2), true>(a, bid, nb); break;
    default: tiny_rows<tiny_w(3), tiny_k(3), true>(a, bid, nb); break;
    }
}

// Numeric-first rows: C entries from their value slots, L lanes per row (two entries
// per lane in flight).
struct CopyArgs {
    const int* list;  // numeric bin lists (class c's at (NUM_TINY + c - 1) * M)
    long long M;
    const int* Cptr;
    const long long* tslot;
    const int* sc_col;
    const double* sc_val;
    int* Ccol;
    double* Cval;
    const int* go;
};
static int copy_lanes(int c) { return c == 0 ? 4 : c == 1 ? 8 : c == 2 ? 16 : 32; }

// In row order: L lanes per row over every row of A, slot rows only (tslot >= 0; k_scan
// marks the others): a wave's stores cover consecutive C rows and its loads consecutive
// slots, with no list in the chain (measured: GAP-road-like copy 1.44 -> 0.82 ms against
// walking each class's list).
template <int L>
__device__ __forceinline__ void copy_rows(const CopyArgs& a, int bid, int nb) {
    const int tl = threadIdx.x & (L - 1);
    for (long long row = ((long long)bid * 256 + threadIdx.x) / L; row < a.M; row += (long long)nb * (256 / L)) {
        const long long src = a.tslot[row];
        if (src < 0) continue;
        const int c0 = a.Cptr[row], n = a.Cptr[row + 1] - c0;
        for (int k = tl; k < n; k += 2 * L) {
            const bool two = k + L < n;
            const int x0 = a.sc_col[src + k];
            const double v0 = a.sc_val[src + k];
            const int x1 = two ? a.sc_col[src + k + L] : 0;
            const double v1 = two ? a.sc_val[src + k + L] : 0.0;
            a.Ccol[c0 + k] = x0;
            a.Cval[c0 + k] = v0;
            if (two) {
                a.Ccol[c0 + k + L] = x1;
                a.Cval[c0 + k + L] = v1;
            }
        }
    }
}
template <int L>
__global__ __launch_bounds__(256) void k_tiny_copy_rows(CopyArgs a) {
    MHS_PLAN_GUARD(a);
    copy_rows<L>(a, (int)blockIdx.x, (int)gridDim.x);
}
// The slot copy and the small hash wave bin as roles of one launch (round 6), when they are the
// numeric phase's only launches (short-row matrices: mac_econ-like): blocks [0, hash_blocks) walk
// the hash rows -- latency-bound, dispatched first -- and the rest copy the slots, HBM-bound, at
// the same time instead of one after the other on the call's stream.
template <int L, bool O32>
__global__ __launch_bounds__(256) MHS_WPE_ATTR(MHS_WPE_HASH) void k_copy_hash(CopyArgs c, NumArgs x, int hash_blocks) {
    MHS_PLAN_GUARD(x);
    if ((int)blockIdx.x < hash_blocks)
        num_wave_rows<NUM_WS_BYTES, false, true, O32>(x, (int)blockIdx.x, hash_blocks);
    else
        copy_rows<L>(c, (int)blockIdx.x - hash_blocks, (int)gridDim.x - hash_blocks);
}



// The common symbolic bins in one launch (their sizes are on the device; an empty role
// costs its blocks one load): blocks [0, wave_blocks) run the small-table wave bin,
// the rest every tiny class -- one launch less, and the two overlap.
template <int BYTES>
__global__ __launch_bounds__(256) MHS_WPE_ATTR(MHS_WPE_SYM) void k_sym_common(SymArgs a, TinyArgs t, int wave_blocks) {
    if ((int)blockIdx.x < wave_blocks)
        sym_wave_rows<BYTES>(a, (int)blockIdx.x, wave_blocks);
    else
        tiny_sym_rows(t, (int)blockIdx.x - wave_blocks);
}

// -------------------------------------------------------------- launchers ---

// Rows per block of the row_ptr scan and the bin lists: 4096 (four per thread) for big
// matrices -- a quarter of the blocks, so a quarter of the per-(block, bin) cursor atomics
// (tiny-row matrices of millions of rows were bound by them) -- 1024 below, where fewer
// blocks would leave the chip idle (measured: cant-like -6% at 4096).
constexpr int MHS_SCAN_BIG_M = (1 << 19);
static int scan_per(int M) { return M >= MHS_SCAN_BIG_M ? 4 : 1; }

constexpr int MHS_ROW_GMIN = 4;  // narrowest lane group per row in k_mask_b / k_analyze (tiny rows: 16 per wave)
static int pick_group(long long nnz, int rows, int gmax = 64) {
    const long long avg = rows > 0 ? (nnz + rows - 1) / rows : 1;
    int g = MHS_ROW_GMIN;
    while (g < avg && g < gmax) g <<= 1;
    return g;
}

static int round8(long long x, int cap) {
    long long g = x < cap ? x : cap;
    if (g < 8) g = 8;
    return (int)((g + 7) / 8 * 8);
}

// Must run on every call, even when B is unchanged: it rewrites all of bmeta, and k_scan
// marks near heads in bmeta.w (over the lo tile) for the numeric pass -- a skipped mask pass
// would let stale NEAR_HEAD bits reach k_analyze.
void launch_mask_b(const Csr& B, const Work& w, hipStream_t s) {
    if (B.M <= 0) return;
    // about four chunk iterations per row: a wave then holds several rows, whose
    // dependent load chains overlap (measured on gfx950: 64-lane rows were latency-bound)
    const long long avg = B.M > 0 ? B.nnz / B.M : 0;
    if (avg < MHS_LANE_AVG) {  // short rows: a lane per row
        const dim3 grid((B.M + 255) / 256), blk(256);
        if (avg < 4)
            hipLaunchKernelGGL(k_mask_lane<4>, grid, blk, 0, s, B.M, B.N, B.ptr, B.col, w.btcol, w.btmask, w.bmeta, w.bhi, w.stats);
        else
            hipLaunchKernelGGL(k_mask_lane<8>, grid, blk, 0, s, B.M, B.N, B.ptr, B.col, w.btcol, w.btmask, w.bmeta, w.bhi, w.stats);
        return;
    }
    // rows of < 3 entries (road networks): 2-lane groups, 32 rows per wave (GAP-road-like -3.6 %)
    // (round 6: groups widen from rows of 16 G entries on, not 8 G -- eight rows a wave for
    // cant-like's 69-entry rows, three chunk rounds instead of two: the waves overlap their
    // ptr -> col chains, cant-like pipelined steps -1.5 %, cant-perturbed-like -0.6 %)
    int G = avg < 3 ? 2 : avg < 4 ? MHS_ROW_GMIN : 8;
    while (2 * G <= avg / 8 && G < MHS_MASK_GMAX) G <<= 1;
    const int rpb = 256 / G;
    const dim3 grid((B.M + rpb - 1) / rpb), blk(256);
#define MHS_MASK(GG, MM) hipLaunchKernelGGL((k_mask_b<GG, MM>), grid, blk, 0, s, B.M, B.N, B.ptr, B.col, w.btcol, w.btmask, w.bmeta, w.bhi, w.stats)
    const bool multi = avg > G;  // rows of several chunks: four chunks a round trip
    switch (G) {
    case 2: MHS_MASK(2, 1); break;
    case 4: MHS_MASK(4, 1); break;
    case 8: if (multi) MHS_MASK(8, 4); else MHS_MASK(8, 1); break;
    case 16: if (multi) MHS_MASK(16, 4); else MHS_MASK(16, 1); break;
    case 32: if (multi) MHS_MASK(32, 4); else MHS_MASK(32, 1); break;
    default: MHS_MASK(64, 4); break;
#undef MHS_MASK
    }
}

// k_analyze: G lanes per row, 256-thread blocks.
// 2-lane groups for rows of < 3 entries on average (GAP-road-like 5.29 -> 4.97 ms)
// G = 1: k_analyze_lane (rows averaging fewer than MHS_LANE_AVG entries; two per-block words)
static void analyze_geometry(long long nnzA, int M, int* G, int* blocks) {
    const long long avg = M > 0 ? nnzA / M : 0;
    *G = avg < MHS_LANE_AVG ? 1 : avg < 3 ? 2 : pick_group(nnzA, M, MHS_AN_GMAX);
    const int rpb = 256 / *G;
    *blocks = (M + rpb - 1) / rpb;
}

int analyze_blocks(long long nnzA, int M) {  // k_analyze's per-block words
    int G, blocks;
    analyze_geometry(nnzA, M, &G, &blocks);
    return G == 1 ? 2 * blocks : blocks;
}

void launch_analyze(const Csr& A, const Work& w, int MB, hipStream_t s, int* Cptr, Published* pub, int seq) {
    if (A.M <= 0) return;
    int G, blocks;
    analyze_geometry(A.nnz, A.M, &G, &blocks);
    const dim3 grid(blocks), blk(256);
#define MHS_ANALYZE(GG, UU) hipLaunchKernelGGL((k_analyze<GG, UU>), grid, blk, 0, s, A.M, MB, A.ptr, A.col, w.bmeta, w.bhi, w.rflop, w.rtflop, w.rlo, w.rhi, w.ctiles, w.sym_bin, Cptr, w.blkflop, w.asame, w.stats, (unsigned long long*)w.scan_part, (A.M + 1 + SCAN_ITEMS - 1) / SCAN_ITEMS + 1 + ZERO_INTS / 2, w.nft_bin, (w.near_list && !w.nft_bin) ? w.nsig : nullptr, w.tiny_num && MHS_SYM_SORT64)
#define MHS_ANALYZE_LANE(UU) hipLaunchKernelGGL((k_analyze_lane<UU>), grid, blk, 0, s, A.M, MB, A.ptr, A.col, w.bmeta, w.bhi, w.rflop, w.rtflop, w.rlo, w.rhi, w.ctiles, w.sym_bin, Cptr, w.blkflop, w.asame, w.stats, (unsigned long long*)w.scan_part, (A.M + 1 + SCAN_ITEMS - 1) / SCAN_ITEMS + 1 + ZERO_INTS / 2, w.nft_bin, (w.near_list && !w.nft_bin) ? w.nsig : nullptr, w.tiny_num && MHS_SYM_SORT64)
    switch (G) {
    case 1:
        if (A.nnz < 4LL * A.M) MHS_ANALYZE_LANE(4);
        else MHS_ANALYZE_LANE(8);
        break;
    case 2: MHS_ANALYZE(2, 1); break;
    case 4: MHS_ANALYZE(4, 1); break;
    case 8:
        if (A.nnz > 8LL * A.M) MHS_ANALYZE(8, 4);  // rows of more than a group's 8 entries on average
        else MHS_ANALYZE(8, 1);
        break;
    case 16: MHS_ANALYZE(16, 1); break;
    case 32: MHS_ANALYZE(32, 1); break;
    default: MHS_ANALYZE(64, 4); break;
    }
#undef MHS_ANALYZE
#undef MHS_ANALYZE_LANE
    if (w.nft_bin && pub) {  // numeric-first probe: the counts go to the host, which picks the bin lists
        hipLaunchKernelGGL(k_probe_publish, dim3(64), dim3(1024), 0, s, (const unsigned long long*)w.blkflop,
                           G == 1 ? 2 * blocks : blocks,
                           w.stats, pub, seq);
        return;
    }
    launch_bin_list(A, w, s);
}

void launch_bin_list(const Csr& A, const Work& w, hipStream_t s) {
    const unsigned char* nb = w.nft ? w.nft_bin : nullptr;
    const NearCand nc{w.nsig, (w.groups && !nb) ? w.near_list : nullptr};
    if (scan_per(A.M) == 4)
        hipLaunchKernelGGL(k_bin_list<4>, dim3((A.M + 4095) / 4096), dim3(1024), 0, s, A.M, w.sym_bin, w.asame, w.grp,
                           w.groups, w.bin_list, nb, w.stats, nc, w.cursors + CURSOR_INTS);
    else
        hipLaunchKernelGGL(k_bin_list<1>, dim3((A.M + 1023) / 1024), dim3(1024), 0, s, A.M, w.sym_bin, w.asame, w.grp,
                           w.groups, w.bin_list, nb, w.stats, nc, w.cursors + CURSOR_INTS);
}

static NearArgs near_args(const Csr& A, const Work& w, const int* Cptr);  // (with the symbolic launchers)

void launch_near(const Csr& A, const Work& w, const int* Cptr, hipStream_t s) {
    const NearArgs p = near_args(A, w, Cptr);
    if (!p.list) return;
    // a persistent grid over the device-side candidate count (none: the waves return at once)
    const int cap = (A.M / 3 + WPB - 1) / WPB;
    hipLaunchKernelGGL(k_near, dim3(round8(cap, MHS_NEAR_GRID)), dim3(256), 0, s, p);
}

hipError_t probe_counter(unsigned long long** dev) {
#if MHS_PROBE_STATS
    return hipGetSymbolAddress((void**)dev, HIP_SYMBOL(g_probe_conflicts));
#else
    *dev = nullptr;
    return hipSuccess;
#endif
}

hipError_t init_kernel_attributes() {
    // gfx950 grants up to 160 KiB of LDS per workgroup; make the large dynamic
    // requests explicit for the block-per-row kernels.  k_sym_rare and k_num_block hold a
    // static LDS word (the row queue) and launch with at most LDS_MAX - 1024 dynamic bytes:
    // static + dynamic must stay within the 160 KiB or the attribute call fails.
    hipError_t e = hipFuncSetAttribute((const void*)k_sym_block<1024, false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX - 1024);
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void*)k_sym_rare, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX - 1024);
    const void* big[] = {(const void*)k_num_block<1024, false, false>, (const void*)k_num_block<1024, false, true>,
                         (const void*)k_num_block<256, false, false>, (const void*)k_num_block<256, false, true>};
    for (const void* k : big)
        if (e == hipSuccess) e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX - 1024);
    const void* wave[] = {(const void*)k_num_wave_direct<NUM_W16_BYTES, false>,
                          (const void*)k_num_wave_direct<NUM_W16_BYTES, true>,
                          (const void*)k_num_wave_hash<NUM_W16_BYTES, false>,
                          (const void*)k_num_wave_hash<NUM_W16_BYTES, true>,
                          (const void*)k_num_wave<NUM_W16_BYTES, true, false, false>,
                          (const void*)k_num_wave<NUM_W16_BYTES, true, false, true>};
    for (const void* k : wave)
        if (e == hipSuccess) e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    return e;
}

__global__ __launch_bounds__(256) void k_add_offset(int* __restrict__ p, int n, int off) {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) p[i] += off;
}
void launch_add_offset(int* p, int n, int off, hipStream_t s) {
    if (n <= 0 || off == 0) return;
    hipLaunchKernelGGL(k_add_offset, dim3(std::min((n + 255) / 256, 4096)), dim3(256), 0, s, p, n, off);
}

size_t sym_global_bytes_per_block(int N) {
    const int span_max = N > 0 ? ((N - 1) >> TILE_SHIFT) + 1 : 1;
    return (size_t)hash_slots(span_max) * 16;
}

// Numeric launches: the numeric-phase events (MHS_OPT_NUMERIC_EVENTS) ride on the first and last
// dispatch packet of a single-stream numeric phase (hipExtLaunchKernel) instead of event records
// of their own between the kernels -- each record measured ~5 us of idle before the next kernel
// (pipelined cant-like steps, r06b timelines).  launch_numeric sets them for the launch at hand.
namespace {
thread_local hipEvent_t t_num_start = nullptr, t_num_stop = nullptr;
}
template <typename F, typename... Args>
static void num_launch(F kernel, const dim3& g, const dim3& b, unsigned lds, hipStream_t s, Args... args) {
    hipEvent_t e0 = t_num_start, e1 = t_num_stop;
    t_num_start = t_num_stop = nullptr;
    if (e0 || e1) hipExtLaunchKernelGGL(kernel, g, b, lds, s, e0, e1, 0u, args...);
    else hipLaunchKernelGGL(kernel, g, b, lds, s, args...);
}

// Numeric tiny class c, `rows` rows.
static void launch_tiny_num(int c, int rows, const TinyArgs& t, hipStream_t s) {
#define MHS_TINY(WW, KK)                                                                                  \
    num_launch((k_tiny_num<WW, KK>), dim3(round8((rows + 256 / (WW) - 1) / (256 / (WW)), MHS_TINY64_GRID)), \
                       dim3(256), 256 * (KK) * 8, s, t)
    switch (c) {
    case 0: MHS_TINY(tiny_w(0), tiny_k(0)); break;
    case 1: MHS_TINY(tiny_w(1), tiny_k(1)); break;
    case 2: MHS_TINY(tiny_w(2), tiny_k(2)); break;
    case 3: MHS_TINY(tiny_w(3), tiny_k(3)); break;
    case 4: MHS_TINY(tiny_w(4), tiny_k(4)); break;
    default: MHS_TINY(tiny_w(5), tiny_k(5)); break;
    }
#undef MHS_TINY
}

static SymArgs sym_args(const Csr& A, const Work& w, int M, int N, int* Cptr) {
    SymArgs a;
    a.M = M;
    a.Aptr = A.ptr;
    a.Acol = A.col;
    a.bmeta = w.bmeta;
    a.btcol = w.btcol;
    a.btmask = w.btmask;
    a.rtflop = w.rtflop;
    a.rlo = w.rlo;
    a.rhi = w.rhi;
    a.list = w.bin_list;
    a.stats = w.stats;
    a.grp = w.grp;
    a.Cptr = Cptr;
    a.ctiles = w.ctiles;
    a.gscratch = (char*)w.gscratch;
    a.gbytes = (long long)sym_global_bytes_per_block(N);
    a.mcache = w.mcache;
    a.mc_list = w.mc_list;
    a.mc_stride = mc_stride(w.mc_list);
    a.cursors = w.cursors;
    a.sp = w.spill;
    a.bin = 0;
    return a;
}

// The common symbolic bins, launched right after the row analysis with persistent
// grids that read their bin's size on the device: the small-table wave bin and
// every tiny class (one launch).
void launch_symbolic_common(const Csr& A, const Csr& B, const Work& w, int M, int N, int* Cptr, hipStream_t s,
                            const Stats* plan) {
    if (M <= 0) return;
    SymArgs a = sym_args(A, w, M, N, Cptr);
    a.bin = SYM_WAVE;
    // A speculated plan (SpecArgs) gives the bins' sizes ahead of the device: the roles are sized to
    // them (an empty role launches no blocks; a bin of other counts changes the Stats, k_scan rejects
    // the plan and the call reruns with the grids below).  Without a plan every role's grid is sized
    // for M rows and its surplus blocks exit after one load.  (r06pg: mac_econ-like -2 %,
    // scircuit-like -3 %, webbase-like -0.6 %: thousands of empty blocks no longer dispatched)
    const int wave_rows = plan ? plan->sym_count[SYM_WAVE] : M;
    // (the probe counted >= 2^21 rows past the tiny classes -- table rows, nearly all in this bin: the
    // numeric hash bin's big-grid rule; r06i: cage15-like -3.2 %; wb-edu-like, 1.9 M such rows, keeps 2048)
    const int wave_blocks =
        wave_rows == 0 ? 0 : round8((wave_rows + WPB - 1) / WPB, w.sym_big ? MHS_SYM_WAVE_GRID_BIG : MHS_SYM_WAVE_GRID);
    TinyArgs t{};
    t.M = M;
    t.Aptr = A.ptr;
    t.Acol = A.col;
    t.bmeta = w.bmeta;
    t.Bcol = B.col;
    t.stats = w.stats;
    t.grp = w.grp;
    t.Cptr = Cptr;
    t.ctiles = w.ctiles;
    t.list = w.bin_list + (long long)(SYM_TINY - 1) * M;
    t.count = -1;
    t.nft = w.nft;
    if (w.nft) {
        t.Aval = A.val;
        t.Bval = B.val;
        t.rlo = w.rlo;
        t.sc_col = w.sc_col;
        t.sc_val = w.sc_val;
        t.tslot = w.tslot;
    }
    constexpr int NCL = MHS_SYM_SORT64 ? TINY_SYMX_NC : TINY_SYM_NC;
    int tiny_blocks = TINY_SYM_GRID * NCL;
    if (plan && !t.nft) {  // (class c's blocks are [1024 c, 1024 (c+1)): all of them, or none)
        int rows = 0;
        for (int c = 0; c < NCL; ++c) rows += plan->sym_count[SYM_TINY + c];
        if (rows == 0) tiny_blocks = 0;
    }
    if (t.nft) {  // (the classes' sizes are on the device: grids for M rows each, as numeric's)
        for (int c = 0; c < TINY_SYM_NC; ++c) {
            const int per = 256 / tiny_w(c);
            const int rows = plan ? plan->sym_count[SYM_TINY + c] : M;
            t.blk0[c + 1] = t.blk0[c] + (rows == 0 ? 0 : round8((rows + per - 1) / per, M >= MHS_NFT_BIG_M ? MHS_NFT_GRID_BIG : MHS_NFT_GRID));
        }
        const bool c4 = MHS_SYM_SORT64 && (!plan || plan->sym_count[SYM_TINY + 4] > 0);
        t.blk0[TINY_SYMX_NC] = t.blk0[TINY_SYM_NC] + (c4 ? TINY_SYM_GRID : 0);  // class 4: a walk
        tiny_blocks = t.blk0[TINY_SYMX_NC];
    }
    if (wave_blocks + tiny_blocks > 0)
        hipLaunchKernelGGL(k_sym_common<SYM_WAVE_BYTES>, dim3(wave_blocks + tiny_blocks), dim3(256),
                           WPB * SYM_WAVE_BYTES, s, a, t, wave_blocks);
}

// The rare bins (10 KiB waves, 32 KiB and 157 KiB block tables, global memory): one
// persistent launch that reads the bins' sizes on the device.
static NearArgs near_args(const Csr& A, const Work& w, const int* Cptr) {
    NearArgs p{};
    if (A.M <= 1 || !w.near_list || !w.groups || w.nft) return p;  // p.list == nullptr: none
    p.Aptr = A.ptr;
    p.Acol = A.col;
    p.Aval = A.val;
    p.Cptr = Cptr;
    p.ctiles = w.ctiles;
    p.rlo = w.rlo;
    p.rhi = w.rhi;
    p.rflop = w.rflop;
    p.rtflop = w.rtflop;
    p.mcache = w.mcache;
    p.mc_list = w.mc_list;
    p.mc_stride = mc_stride(w.mc_list);
    p.list = w.near_list;
    p.stats = w.stats;
    p.grp = w.grp;
    p.ucol = w.ucol;
    p.uval = w.uval;
    p.gna = w.gna;
    p.ucolx = w.near_b ? w.ucolx : nullptr;  // (B's union runs: B is A)
    p.verified = &w.stats->near_verified;
    p.vcheck = w.vcheck;
    p.vcheck_n = w.vcheck_n;
    p.nonfinite = &w.stats->nonfinite;
    return p;
}

void launch_symbolic_rare(const Csr& A, const Work& w, int M, int N, int* Cptr, hipStream_t s, bool with_near) {
    if (M <= 0) return;
    SymArgs a = sym_args(A, w, M, N, Cptr);
    const NearArgs np = with_near ? near_args(A, w, Cptr) : NearArgs{};
    hipLaunchKernelGGL(k_sym_rare, dim3(256), dim3(1024), LDS_MAX - 1024, s, a, np);
}

// The 32 KiB block bin (its own launch: at one block per CU in k_sym_rare it would hold a fifth
// of the rows in flight).  With the rare bins on an aux stream it follows the common bins on the
// call's stream, beside k_sym_rare (webbase-like: 60 us off the symbolic phase).
void launch_symbolic_b256(const Csr& A, const Work& w, int M, int N, int* Cptr, hipStream_t s) {
    if (M <= 0) return;
    SymArgs a = sym_args(A, w, M, N, Cptr);
    a.bin = SYM_B256;
    hipLaunchKernelGGL((k_sym_block<256, false>), dim3(round8(M, MHS_SYM_B256_GRID)), dim3(256), SYM_B256_BYTES, s, a);
}

void launch_scan_classify(int M, const Work& w, int* Cptr, const int* Aptr, hipStream_t s, int dense_span_max,
                          Published* pub, int seq, const SpecArgs& spec) {
    // the state words were zeroed by k_analyze (SCAN_ITEMS-row blocks: enough for either width)
    const int per = scan_per(M), nb = (M + 1 + 1024 * per - 1) / (1024 * per);
#define MHS_SCAN(P)                                                                                                \
    hipLaunchKernelGGL(k_scan<P>, dim3(nb), dim3(1024), 0, s, M, Cptr, (unsigned long long*)w.scan_part, w.rflop,  \
                       w.rlo, w.rhi, w.ctiles, w.grp, Aptr, w.bin_list, w.stats, dense_span_max, pub, seq, w.tiny_num, \
                       w.blkflop, w.nflop, w.sc_col != nullptr, w.tslot, w.gna, w.near_b ? w.bmeta : nullptr, w.sym_bin, spec, \
                       w.cursors + CURSOR_INTS + NBINS * BINCNT_STRIDE)
    if (per == 4) MHS_SCAN(4);
    else MHS_SCAN(1);
#undef MHS_SCAN
}

// Dynamic LDS of a block-kernel launch: the header plus its largest row's tables, in
// 2 KiB steps, at most the bin's budget.
static int block_lds(int need, int budget, int T) {
    if (need <= 0) return budget;
    const int b = (block_hdr(T) + need + 2047) & ~2047;
    return b < budget ? b : budget;
}

// A block bin runs as two launches when it holds rows on both sides of its LDS split.
static bool block_split_on(const Stats& h, int k) {
    const int bin = k ? NUM_B1024 : NUM_B256;
    return h.num_block_big[k] > 0 && h.num_block_big[k] < h.num_count[bin];
}

int numeric_launches(const Stats& h) {
    int n = 0, small = 0;
    for (int b = 1; b < NUM_NB; ++b) {
        if (h.num_count[b] <= 0) continue;
        if (b >= NUM_TINY && b < NUM_TINY + 4) small = 1;
        else ++n;
    }
    return n + small + block_split_on(h, 0) + block_split_on(h, 1);
}

// Partition of the split block bins' lists (one 1024-thread block per bin): rows at or below
// the bin's LDS split from the front of its part of w.split_list, hub rows from the back
// (a ballot and one LDS counter add per wave; order within a wave kept).
struct SplitArgs {
    const int* list[2];
    int count[2], split[2], base[2], on[2];
    int blk0[3];  // bin k's blocks: [blk0[k], blk0[k+1]) (1024 rows a block)
    int* out;
    int* ctr;     // per bin: small-row and big-row counters (zeroed with the row cursors)
    const int *rlo, *rhi, *ctiles, *Cptr;
    int dense_span_max;
    const int* go;
};
constexpr int SPLIT_CURSOR_SLOT = BLOCK_BIG_SLOT + 2;  // k_split_bins' counters (4 of its 8 words)
static_assert(SPLIT_CURSOR_SLOT < SPILL_CURSOR_SLOT, "split counters below the spill counters");
// A grid of 1024-row blocks per split bin (one block per bin measured 0.5 ms on wb-edu-like's
// 56 K block rows, on the block launches' critical path): LDS offsets within the block, then one
// counter add per block and kind.  Order within the small and the big rows is by block arrival
// (the block launches take their rows from a queue anyway).
__global__ __launch_bounds__(1024) void k_split_bins(SplitArgs a) {
    MHS_PLAN_GUARD(a);
    const int k = (int)blockIdx.x < a.blk0[1] ? 0 : 1;
    const int i = ((int)blockIdx.x - a.blk0[k]) * 1024 + (int)threadIdx.x;
    __shared__ int nsmall, nbig, gsmall, gbig;
    if (threadIdx.x == 0) nsmall = nbig = 0;
    __syncthreads();
    const int count = a.count[k], lane = lane_id();
    int row = 0;
    bool big = false;
    if (i < count) {
        row = a.list[k][i];
        big = block_row_need(k == 1, a.rlo[row], a.rhi[row], a.ctiles[row], a.Cptr[row + 1] - a.Cptr[row],
                             a.dense_span_max) > a.split[k];
    }
    const unsigned long long bb = __ballot(i < count && big), bs = __ballot(i < count && !big);
    int ob = 0, os = 0;
    if (lane == 0) {
        if (bb) ob = atomicAdd(&nbig, __popcll(bb));
        if (bs) os = atomicAdd(&nsmall, __popcll(bs));
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int* c = a.ctr + k * 2 * CURSOR_STRIDE;
        gsmall = nsmall ? atomicAdd(c, nsmall) : 0;
        gbig = nbig ? atomicAdd(c + CURSOR_STRIDE, nbig) : 0;
    }
    __syncthreads();
    ob = __shfl(ob, 0) + gbig;
    os = __shfl(os, 0) + gsmall;
    int* out = a.out + a.base[k];
    if (i < count) {
        if (big) out[count - 1 - (ob + __popcll(bb & lanemask_lt()))] = row;
        else out[os + __popcll(bs & lanemask_lt())] = row;
    }
}

bool launch_split_bins(const Work& w, const Stats& h, int M, const int* Cptr, hipStream_t s, int dense_span_max) {
    SplitArgs a{};
    // bin 0 of the kernel is NUM_B256 (its list after NUM_B1024's in split_list), bin 1 NUM_B1024
    const int bins[2] = {NUM_B256, NUM_B1024};
    const int splits[2] = {B256_SPLIT, B1024_SPLIT};
    for (int k = 0; k < 2; ++k) {
        a.list[k] = w.bin_list + (long long)(bins[k] - 1) * M;
        a.count[k] = h.num_count[bins[k]] > 0 ? h.num_count[bins[k]] : 0;
        a.split[k] = splits[k];
        a.on[k] = block_split_on(h, k);
        a.blk0[k + 1] = a.blk0[k] + (a.on[k] ? (a.count[k] + 1023) / 1024 : 0);
    }
    if (!a.on[0] && !a.on[1]) return false;
    a.base[1] = 0;
    a.base[0] = a.count[1];
    a.out = w.split_list;
    a.ctr = w.cursors + SPLIT_CURSOR_SLOT * 8 * CURSOR_STRIDE;
    a.rlo = w.rlo;
    a.rhi = w.rhi;
    a.ctiles = w.ctiles;
    a.Cptr = Cptr;
    a.dense_span_max = dense_span_max;
    a.go = w.go;
    hipLaunchKernelGGL(k_split_bins, dim3(a.blk0[2]), dim3(1024), 0, s, a);
    return true;
}

// Numeric launches of the non-empty bins, largest rows first, dealt round-robin over nss streams
// (launch i on ss[(i + 1) % nss], so the last, bulk wave bins tend to stay on ss[0]): one bin's
// tail overlaps the next bin's bulk (the reference runs its bins on 12 streams, src/Tool.cu:6-10).
// Measured (round 4, profiles/r04): dealing by estimated work (LPT over products and the heaviest
// row) put the hub rows' launch behind the bulk bins -- wb-edu-like +3 %, webbase-like +3 % --
// concurrent launches share the CUs, and the hub rows' 1024-thread blocks, one per CU for their
// LDS, progress only as CUs free up; started first, they hold their CUs from the start.
// Returns the mask of streams used.
namespace {
struct NumLaunch {
    std::function<void(hipStream_t)> go;
};
}  // namespace

int launch_numeric(const Csr& A, const Csr& B, const Work& w, const Stats& h, int* Cptr, int* Ccol,
                   double* Cval, const hipStream_t* ss, int nss, int global_grid, int dense_span_max, bool split,
                   hipEvent_t split_ev, const std::function<bool()>& fork, hipEvent_t ev_start, hipEvent_t ev_stop,
                   int only) {
    std::vector<NumLaunch> L;
    auto add = [&](std::function<void(hipStream_t)> go) { L.push_back(NumLaunch{std::move(go)}); };
    NumArgs a{};
    a.dense_span_max = dense_span_max;
    a.mcache = w.mcache;
    a.mc_list = w.mc_list;
    a.mc_stride = mc_stride(w.mc_list);
    a.Aptr = A.ptr;
    a.Acol = A.col;
    a.Aval = A.val;
    a.Bcol = B.col;
    a.Bval = B.val;
    a.bmeta = w.bmeta;
    a.btcol = w.btcol;
    a.btmask = w.btmask;
    a.rflop = w.rflop;
    a.rtflop = w.rtflop;
    a.rlo = w.rlo;
    a.rhi = w.rhi;
    a.ctiles = w.ctiles;
    a.Cptr = Cptr;
    a.Ccol = Ccol;
    a.Cval = Cval;
    a.gscratch = (char*)w.gscratch;
    a.gbytes = 0;
    a.grp = w.grp;
    a.cursor = w.cursors;
    a.sp = w.spill;
    a.ucol = w.ucol;
    a.uval = w.uval;
    a.gna = w.gna;
    a.go = w.go;
    // near union runs (B is A and near groups were verified): the value walks read B's arrays
    // extended by the union rows (bx_col / bx_val, filled by launch_union_b before numeric)
    if (w.bx_on) {
        a.ubase = B.nnz;
        a.Bcol = w.bx_col;
        a.Bval = w.bx_val;
    }
    // 32-bit byte offsets for the B gathers when B's value array (extended by the union rows)
    // stays below 4 GiB: nnz(B) + 3 nnz(A) < 2^29 (the reference's int32 CSR allows up to 2^31)
    const bool o32 = (long long)B.nnz + (w.bx_on ? 3LL * A.nnz : 0) < (1LL << 29);
    // a wave-bin launch over `bin`'s list (cursor slot = bin)
    auto wave_args = [&](int bin) {
        NumArgs x = a;
        x.count = h.num_count[bin];
        x.list = w.bin_list + (long long)(bin - 1) * A.M;
        x.cursor = w.cursors + bin * 8 * CURSOR_STRIDE;
        return x;
    };

    // Numeric-first rows: their copy of the slot values into C (short and HBM-bound).
    const bool copy = w.sc_col != nullptr;  // numeric-first: tiny classes 0..3 hold slot rows
    // ... fused with the small hash wave bin when those two are the whole phase (k_copy_hash)
    // (r06fc: mac_econ-like numeric 45 -> 34 us, pipelined step -5 %)
    bool fuse = copy && h.num_count[NUM_WSH] > 0;
    for (int b = 1; b < NUM_NB && fuse; ++b)
        fuse = b == NUM_WSH || (b >= NUM_TINY && b < NUM_TINY + 4) || h.num_count[b] <= 0;
    if (copy) {
        TinyFused f{};
        int ncopy = 0, cmed = 0;
        for (int c = 3; c >= 0; --c) {
            const int count = h.num_count[NUM_TINY + c];
            if (count <= 0) continue;
            ncopy += count;
            const int per = 256 / copy_lanes(c);
            f.c[f.nclass] = c;
            f.count[f.nclass] = count;
            f.blk0[f.nclass + 1] = f.blk0[f.nclass] + round8((count + per - 1) / per, 4096);
            ++f.nclass;
        }
        for (int c = 0, acc = 0; c < 4; ++c) {  // the class of the median slot row
            acc += h.num_count[NUM_TINY + c];
            if (2 * acc >= ncopy) {
                cmed = c;
                break;
            }
        }
        if (f.nclass > 0) {
            const CopyArgs ca{w.bin_list, A.M, Cptr, w.tslot, w.sc_col, w.sc_val, Ccol, Cval, w.go};
            // lanes per row by the median row's class
            const int Lw = copy_lanes(cmed) > 16 ? 16 : copy_lanes(cmed);
            const dim3 grid(round8((A.M + 256 / Lw - 1) / (256 / Lw), A.M >= MHS_NFT_BIG_M ? MHS_COPY_CAP_BIG : 16384));
            if (fuse) {
                const NumArgs x = wave_args(NUM_WSH);
                const int hb = round8((x.count + WPB - 1) / WPB, x.count >= MHS_NUM_WSH_BIG ? MHS_NUM_WSH_BIG_GRID : MHS_NUM_WSX_GRID);
                const dim3 g2(hb + grid.x);
                add([=](hipStream_t s) {
#define MHS_COPY_HASH(LL)                                                                                           \
    (o32 ? num_launch((k_copy_hash<LL, true>), g2, dim3(256), WPB * NUM_WS_BYTES, s, ca, x, hb)                      \
         : num_launch((k_copy_hash<LL, false>), g2, dim3(256), WPB * NUM_WS_BYTES, s, ca, x, hb))
                    if (Lw == 4) MHS_COPY_HASH(4);
                    else if (Lw == 8) MHS_COPY_HASH(8);
                    else MHS_COPY_HASH(16);
#undef MHS_COPY_HASH
                });
            } else {
                add([=](hipStream_t s) {
                    if (Lw == 4) num_launch(k_tiny_copy_rows<4>, grid, dim3(256), 0, s, ca);
                    else if (Lw == 8) num_launch(k_tiny_copy_rows<8>, grid, dim3(256), 0, s, ca);
                    else num_launch(k_tiny_copy_rows<16>, grid, dim3(256), 0, s, ca);
                });
            }
        } else {
            fuse = false;
        }
    }
    if (h.num_count[NUM_GLOBAL] > 0) {
        NumArgs x = wave_args(NUM_GLOBAL);
        x.gbytes = align16(h.num_global_need);
        const int g = x.count < global_grid ? x.count : global_grid;
        add([=](hipStream_t s) {
            if (o32) num_launch((k_num_block<1024, true, true>), dim3(g), dim3(1024), BLOCK_HDR_1024, s, x);
            else num_launch((k_num_block<1024, true, false>), dim3(g), dim3(1024), BLOCK_HDR_1024, s, x);
        });
    }
    // block bins: rows past the bin's LDS split (hub rows) in a launch of their own, so the
    // others run at the occupancy their own tables allow
    auto block_bin = [&](int bin, int k, int T, int grid_cap, int budget, int big_slot) {
        const int count = h.num_count[bin];
        if (count <= 0) return;
        auto go = [&](const int* list, int rows, int lds, int slot, hipEvent_t after) {
            NumArgs x = a;
            x.list = list;
            x.count = rows;
            x.cursor = w.cursors + slot * 8 * CURSOR_STRIDE;
            const dim3 grid(round8(rows, grid_cap));
            const hipStream_t s0 = ss[0];
            add([=](hipStream_t s) {
                if (after && s != s0) (void)hipStreamWaitEvent(s, after, 0);  // (k_split_bins' lists)
                if (T == 1024 && o32) num_launch((k_num_block<1024, false, true>), grid, dim3(1024), lds, s, x);
                else if (T == 1024) num_launch((k_num_block<1024, false, false>), grid, dim3(1024), lds, s, x);
                else if (o32) num_launch((k_num_block<256, false, true>), grid, dim3(256), lds, s, x);
                else num_launch((k_num_block<256, false, false>), grid, dim3(256), lds, s, x);
            });
        };
        if (split && block_split_on(h, k)) {  // k_split_bins: small rows first, hub rows last
            const int big = h.num_block_big[k];
            const int* l = w.split_list + (k ? 0 : (h.num_count[NUM_B1024] > 0 ? h.num_count[NUM_B1024] : 0));
            go(l + (count - big), big, block_lds(h.num_block_need[k], budget, T), big_slot, split_ev);
            go(l, count - big, block_lds(h.num_block_small_need[k], budget, T), bin, split_ev);
        } else {
            go(w.bin_list + (long long)(bin - 1) * A.M, count, block_lds(h.num_block_need[k], budget, T), bin, nullptr);
        }
    };
    block_bin(NUM_B1024, 1, 1024, 256, LDS_MAX - 1024, BLOCK_BIG_SLOT + 1);
    block_bin(NUM_B256, 0, 256, 1024, NUM_B256_BYTES, BLOCK_BIG_SLOT);
    if (h.num_count[NUM_W16H] > 0) {
        NumArgs x = wave_args(NUM_W16H);
        x.qall = x.count <= MHS_DYN16_MAX;  // a few rows per resident wave: the launch's end is one heavy row
        const dim3 grid(round8((x.count + WPB - 1) / WPB, MHS_NUM_W16H_GRID));
        add([=](hipStream_t s) {
            if (o32) num_launch((k_num_wave_hash<NUM_W16_BYTES, true>), grid, dim3(256), WPB * NUM_W16_BYTES, s, x);
            else num_launch((k_num_wave_hash<NUM_W16_BYTES, false>), grid, dim3(256), WPB * NUM_W16_BYTES, s, x);
        });
    }
    if (h.num_count[NUM_WSH] > 0 && !fuse) {
        const NumArgs x = wave_args(NUM_WSH);
        const dim3 grid(round8((x.count + WPB - 1) / WPB, x.count >= MHS_NUM_WSH_BIG ? MHS_NUM_WSH_BIG_GRID : MHS_NUM_WSX_GRID));
        add([=](hipStream_t s) {
            if (o32) num_launch((k_num_wave_hash<NUM_WS_BYTES, true>), grid, dim3(256), WPB * NUM_WS_BYTES, s, x);
            else num_launch((k_num_wave_hash<NUM_WS_BYTES, false>), grid, dim3(256), WPB * NUM_WS_BYTES, s, x);
        });
    }
    if (h.num_count[NUM_W16] > 0) {
        const NumArgs x = wave_args(NUM_W16);
        const dim3 grid(round8((x.count + WPB - 1) / WPB, 2048));
        add([=](hipStream_t s) {
            if (o32) num_launch((k_num_wave_direct<NUM_W16_BYTES, true>), grid, dim3(256), WPB * NUM_W16_BYTES, s, x);
            else num_launch((k_num_wave_direct<NUM_W16_BYTES, false>), grid, dim3(256), WPB * NUM_W16_BYTES, s, x);
        });
    }
    {
        TinyArgs t{};
        t.M = A.M;
        t.Aptr = A.ptr;
        t.Acol = A.col;
        t.Aval = A.val;
        t.bmeta = w.bmeta;
        t.Bcol = B.col;
        t.Bval = B.val;
        t.Cptr = Cptr;
        t.Ccol = Ccol;
        t.Cval = Cval;
        t.rlo = w.rlo;
        t.go = w.go;
        for (int c = TINY_NC - 1; c >= 4; --c) {  // 64-lane classes: kernels of their own (registers)
            const int count = h.num_count[NUM_TINY + c];
            if (count <= 0) continue;
            TinyArgs tc = t;
            tc.count = count;
            tc.bin = NUM_TINY + c;
            tc.list = w.bin_list + (long long)(tc.bin - 1) * A.M;
            add([=](hipStream_t s) { launch_tiny_num(c, count, tc, s); });
        }
        TinyFused f{};
        static_assert(tiny_w(3) <= 32 && tiny_k(0) <= TINY_FUSED_KMAX && tiny_k(1) <= TINY_FUSED_KMAX &&
                          tiny_k(2) <= TINY_FUSED_KMAX && tiny_k(3) <= TINY_FUSED_KMAX && tiny_w(4) == 64,
                      "classes 0..3 fuse (W <= 32, K <= TINY_FUSED_KMAX)");
        for (int c = 3; c >= 0 && !copy; --c) {  // (numeric-first: copied above)
            const int count = h.num_count[NUM_TINY + c];
            if (count <= 0) continue;
            const int per = 256 / tiny_w(c);
            f.c[f.nclass] = c;
            f.count[f.nclass] = count;
            f.blk0[f.nclass + 1] = f.blk0[f.nclass] + round8((count + per - 1) / per, 4096);
            ++f.nclass;
        }
        if (f.nclass > 0) {
            t.list = w.bin_list;
            add([=](hipStream_t s) {
                num_launch(k_tiny_num_small, dim3(f.blk0[f.nclass]), dim3(256), 256 * TINY_FUSED_KMAX * 8, s, t,
                                   f);
            });
        }
    }
    // grouped bins: LDS regions of their largest group's need, 256-byte steps (k_scan's num_wave_need)
    auto wave_region = [](int need, int cap) {
        const int b = (need + 255) & ~255;
        return need <= 0 || b > cap ? cap : b;
    };
    if (h.num_count[NUM_W16G] > 0) {
        NumArgs x = wave_args(NUM_W16G);
        x.wave_bytes = wave_region(h.num_wave_need[1], NUM_W16_BYTES);
        const dim3 grid(round8((x.count + WPB - 1) / WPB, 2048));
        add([=](hipStream_t s) {
            if (o32) num_launch((k_num_wave<NUM_W16_BYTES, true, false, true>), grid, dim3(256), WPB * x.wave_bytes, s, x);
            else num_launch((k_num_wave<NUM_W16_BYTES, true, false, false>), grid, dim3(256), WPB * x.wave_bytes, s, x);
        });
    }
    if (h.num_count[NUM_WSG] > 0) {
        NumArgs x = wave_args(NUM_WSG);
        x.wave_bytes = wave_region(h.num_wave_need[0], NUM_WSG_BYTES);
        const dim3 grid(round8((x.count + WPB - 1) / WPB, MHS_NUM_WS_GRID));
        add([=](hipStream_t s) {
            if (o32) num_launch((k_num_wave<NUM_WSG_BYTES, true, false, true>), grid, dim3(256), WPB * x.wave_bytes, s, x);
            else num_launch((k_num_wave<NUM_WSG_BYTES, true, false, false>), grid, dim3(256), WPB * x.wave_bytes, s, x);
        });
    }
    if (h.num_count[NUM_WS] > 0) {
        const NumArgs x = wave_args(NUM_WS);
        const dim3 grid(round8((x.count + WPB - 1) / WPB, MHS_NUM_WSX_GRID));
        add([=](hipStream_t s) {
            if (o32) num_launch((k_num_wave_direct<NUM_WS_BYTES, true>), grid, dim3(256), WPB * NUM_WS_BYTES, s, x);
            else num_launch((k_num_wave_direct<NUM_WS_BYTES, false>), grid, dim3(256), WPB * NUM_WS_BYTES, s, x);
        });
    }
    // launch i on ss[i % n]: the first (largest rows) goes out on the call's stream at once, and the
    // aux streams' waits on the fork event are set up after it (`fork`, host API calls that would
    // otherwise sit between the hand-off and the first numeric kernel: round 5, scircuit-like's
    // hand-off gap 46 -> ? us)
    // (a failed fork -- the aux streams' wait on the fork event -- sends every later launch to
    // ss[0]: no aux-stream launch may run without its dependency on the pre-numeric work)
    // `only`: the streams (bit k: ss[k]) whose launches go out in this call -- a speculated plan
    // deals the same list twice, the call stream's share first (see NumPhase in mhs_api.cpp)
    int used = 0;
    int n = nss < 1 ? 1 : (nss > 8 ? 8 : nss);
    const bool evs = n == 1 && !L.empty() && (ev_start || ev_stop) && (only & 1);  // (single stream only: see num_launch)
    bool forked = false;
    for (size_t i = 0; i < L.size(); ++i) {
        int k = n > 1 ? (int)(i % n) : 0;
        if (!((only >> k) & 1)) continue;
        if (k != 0 && !forked) {  // the aux streams' waits, before their first launch
            forked = true;
            if (fork && !fork()) {
                n = 1;  // (a failed fork: the rest on ss[0])
                k = 0;
            }
        }
        used |= 1 << k;
        if (evs && i == 0) t_num_start = ev_start;
        if (evs && i + 1 == L.size()) t_num_stop = ev_stop;
        L[i].go(ss[k]);
    }
    t_num_start = t_num_stop = nullptr;
    if (!evs && (ev_start || ev_stop)) used |= 1 << 30;  // the caller records the events itself
    if (!forked && n > 1 && fork && (only & ~1)) (void)fork();  // (the caller's error check expects the fork)
    return used;
}
}  // namespace mhs
