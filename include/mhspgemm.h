/*
 * mhspgemm.h -- C-ABI of the MI355X-native hash-accumulator SpGEMM.
 *
 * Drop-in boundary for the reference's call path (yyssys/MH-SpGEMM):
 *   void MH_spgemm(const CSR &A, CSR &B, CSR &C, Timing &Timing, Tool &tools)
 *     (/root/reference/src/main.cu:12-72)
 * which the reference's main() calls on device-resident A and B
 * (src/main.cu:110-124) and which leaves C (C.d_ptr/d_col/d_val, C.nnz)
 * on the device.  Every entry point below is extern "C", takes plain
 * pointers and sizes, and never throws; failures return an mhs_status and
 * leave a message in mhs_last_error().
 *
 * Data contract (same as the reference):
 *   - CSR, zero-based, int32 row_ptr[M+1] / col_idx[nnz], double val[nnz].
 *   - A is M x K, B is K x N (the reference computes A*A: B = A, main.cu:101).
 *   - B's column indices are sorted ascending within each row (the reference
 *     relies on it in Form_mask_matrix_B.cuh:442-447 and guarantees it in
 *     mmio_read.h:150).  Violations are detected and reported as
 *     MHS_ERR_INVALID rather than producing a wrong C.
 *   - C's pattern is structural (cancellation zeros are kept), columns are
 *     sorted ascending per row, duplicates in A or B are summed.
 *   - Values are FP64; summation order on the GPU is not fixed, so values
 *     match a sequential reference to rounding (the north-star bound is
 *     1e-6 relative), row_ptr and col_idx match bit-exactly.
 */
#ifndef MHSPGEMM_H
#define MHSPGEMM_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MHS_ABI_VERSION 10

typedef enum mhs_status {
    MHS_OK = 0,
    MHS_ERR_HIP = 1,      /* a HIP runtime call failed (reference: CHECK_ERROR throw, common.h:85-95) */
    MHS_ERR_OOM = 2,      /* device allocation failed */
    MHS_ERR_INVALID = 3,  /* bad argument, dimension mismatch, unsorted or out-of-range columns */
    MHS_ERR_OVERFLOW = 4, /* nnz(C) does not fit int32 row_ptr */
    MHS_ERR_IO = 5        /* Matrix Market read failure */
} mhs_status;

/* A CSR matrix.  For mhs_spgemm the arrays are DEVICE pointers
 * (the reference's CSR::d_ptr/d_col/d_val, inc/CSR.h:15-17). */
typedef struct mhs_csr {
    int32_t M, N, nnz;
    int32_t *ptr; /* M+1 */
    int32_t *col; /* nnz */
    double *val;  /* nnz */
} mhs_csr;

/* Per-phase times in ms, the reference's Timing fields (inc/Timing.h:3-20),
 * measured with hipEvents on the context stream, plus the two totals and
 * run statistics. */
typedef struct mhs_timing {
    double mem_alloc;          /* workspace + C.ptr allocation            */
    double Form_mask_matrix_B; /* B -> (tile col, 64-bit mask) rows       */
    double symbolic_binning;   /* row analysis + symbolic bins            */
    double Calculate_C_nnz;    /* symbolic: nnz of every C row            */
    double numeric_binning;    /* row_ptr scan + numeric bins + readback  */
    double Malloc_C_col_val;   /* C.col / C.val allocation                */
    double Numeric;            /* numeric: values + sorted columns        */
    double total_ref;          /* = getTotal(): all but Form_mask_matrix_B (src/Timing.cpp:39-41) */
    double total_e2e;          /* everything, device-resident A,B -> device-resident C */
    uint64_t flop;             /* sum over A's nonzeros of nnz(B row)   (src/main.cu:102-107) */
    int64_t nnzC;
    int32_t sym_bins[16];      /* rows per symbolic bin (0: rows not processed: empty, or in a row group) */
    int32_t num_bins[16];      /* rows per numeric bin  (0: likewise)                                  */
} mhs_timing;

typedef struct mhs_ctx mhs_ctx;

/* Context = the reference's Tool (inc/Tool.h, src/Tool.cu:4-45): stream,
 * workspace (kept across calls, grown on demand), pinned readback area.
 * One context per device; a context is not thread-safe, distinct contexts
 * may be used from distinct threads. */
int mhs_ctx_create(mhs_ctx **ctx, int device);
void mhs_ctx_destroy(mhs_ctx *ctx);
const char *mhs_last_error(const mhs_ctx *ctx);
/* Run on a caller-owned hipStream_t (e.g. PyTorch's current stream); NULL
 * restores the context's own stream. */
int mhs_ctx_set_stream(mhs_ctx *ctx, void *hip_stream);
/* Release cached workspace and pooled output buffers. */
int mhs_ctx_trim(mhs_ctx *ctx);

/* Context options (mhs_ctx_set_option):
 *   MHS_OPT_SYNC (default 1): mhs_spgemm returns after C is complete.  0: it
 *     returns once the numeric phase is queued on the context stream (C's
 *     nnz and arrays are valid; their contents are stream-ordered, as for any
 *     kernel output).  A call with a timing struct always synchronises.
 *   MHS_OPT_NUMERIC_EVENTS (default 0): keep hipEvent pairs around the numeric
 *     phase of the last `value` calls, read with mhs_ctx_numeric_ms.
 *   MHS_OPT_MEM_BUDGET (default 0 = none): treat a call's workspace, or workspace
 *     plus C, beyond `value` MiB as an out-of-memory condition (exercises the
 *     row-chunked fallback below without filling the device).
 *   MHS_OPT_TINY_FIRST_ROWS (default 524288; < 0: never): from this many rows of A
 *     on, rows of at most 128 products are summed during the symbolic phase into
 *     cached value slots and numeric only copies them into C (one sort instead of
 *     two; one more device-to-host hand-off per call, so big matrices only).  Below
 *     the threshold, matrices averaging fewer than 12 entries a row take the same
 *     path without the hand-off, with slots sized by the per-row bound (M * 128 *
 *     12 bytes, cached in the context; skipped when they do not fit the device or
 *     MHS_OPT_MEM_BUDGET).  A negative value turns both off.
 *   MHS_OPT_SPECULATE (default 1; env MHS_NO_SPEC=1 sets 0): a call on the same
 *     operands as the context's previous call (the same device arrays and sizes)
 *     queues the previous call's numeric launches behind the row_ptr scan instead of
 *     waiting for its statistics; the scan checks on the device that the call's
 *     statistics equal the plan's, the numeric kernels run only then, and a
 *     mismatch reruns the call without speculation (MHS_STAT_SPEC_MISS).  Every
 *     phase runs on every call either way.
 * Out of memory: when the workspace, C.ptr, the global-bin scratch or C beside them does
 * not fit, mhs_spgemm gives back every cached buffer and retries row-chunked: a counting
 * pass with the largest chunk workspace that fits sizes C; C is allocated before the
 * second pass's workspace (halved only while that workspace does not fit beside C).  It
 * returns MHS_ERR_OOM right after the counting pass when C itself does not fit, or when
 * a one-row workspace does not fit. */
typedef enum mhs_option { MHS_OPT_SYNC = 1, MHS_OPT_NUMERIC_EVENTS = 2, MHS_OPT_MEM_BUDGET = 3,
                           MHS_OPT_TINY_FIRST_ROWS = 4, MHS_OPT_SPECULATE = 5 } mhs_option;
int mhs_ctx_set_option(mhs_ctx *ctx, int option, int value);
/* Calls of this context that ran row-chunked (the out-of-memory fallback). */
long long mhs_ctx_chunked_calls(const mhs_ctx *ctx);
/* Path counters of this context (diagnostics, ABI v9): calls that ran
 *   MHS_STAT_CHUNKED      row-chunked (as mhs_ctx_chunked_calls),
 *   MHS_STAT_SPLIT        their numeric block bins split by LDS need (k_split_bins),
 *   MHS_STAT_SYM_FORK     the rare symbolic bins on an aux stream beside the common ones,
 *   MHS_STAT_NFT          numeric-first tiny rows (value slots filled by the symbolic pass),
 *   MHS_STAT_NEAR         near row groups verified (union rows built),
 *   MHS_STAT_MULTI_STREAM numeric launches dealt over several streams,
 *   MHS_STAT_SPEC         (ABI v10) the previous call's numeric plan launched ahead of the scan,
 *   MHS_STAT_SPEC_MISS    ... and rejected by the scan (the call reran without speculation),
 *   MHS_STAT_SPEC_SKIPPED symbolic launches left out by speculated calls (the plan's empty bins).
 * Returns -1 for a null context or an unknown counter. */
typedef enum mhs_stat { MHS_STAT_CHUNKED = 0, MHS_STAT_SPLIT = 1, MHS_STAT_SYM_FORK = 2, MHS_STAT_NFT = 3,
                        MHS_STAT_NEAR = 4, MHS_STAT_MULTI_STREAM = 5, MHS_STAT_SPEC = 6, MHS_STAT_SPEC_MISS = 7,
                        MHS_STAT_SPEC_SKIPPED = 8 } mhs_stat;
long long mhs_ctx_stat(const mhs_ctx *ctx, int which);
/* Numeric-phase durations (ms) of the last min(n, recorded) calls, oldest
 * first; waits for them.  Returns the count written, or -status on error. */
int mhs_ctx_numeric_ms(mhs_ctx *ctx, float *out, int n);

/* Hash probe conflicts (the reference's HASH_CONFLICT switch, inc/common.h:18, printed
 * at src/main.cu:68-71): probe steps that met another key in the symbolic and numeric
 * tile hash tables (inserts and lookups) since the previous call of this function, which
 * resets the count.  Only the diagnostic library libmhspgemm_probe.so (built with
 * MHS_PROBE_STATS=1) counts; the product library returns MHS_ERR_INVALID.  Synchronises
 * the context stream.  The counter is per process (shared by all contexts). */
int mhs_probe_conflicts(mhs_ctx *ctx, uint64_t *count);

/* C = A * B on the device.  A, B: device CSR.  On MHS_OK, C->M = A->M,
 * C->N = B->N, C->nnz is set and C->ptr/col/val are fresh device
 * allocations owned by the caller (free with mhs_csr_free, or hand back to
 * the context's pool with mhs_ctx_recycle).  A and B may alias.  B is not
 * modified (unlike the reference, which allocates B.d_tile* in place).
 * Returns after C is complete (the context stream is synchronised), unless
 * MHS_OPT_SYNC is 0.  t may be NULL. */
int mhs_spgemm(mhs_ctx *ctx, const mhs_csr *A, const mhs_csr *B, mhs_csr *C, mhs_timing *t);

/* At = A^T on the device (the reference's AAT operand: B = transpose(A),
 * src/main.cu:98-99 with AAT=1, inc/common.h:37; host transpose src/utils.cpp:20-46).
 * At->M = A->N, At->N = A->M; rows of At list their columns ascending; arrays are
 * fresh device allocations owned by the caller (mhs_csr_free).  Synchronous. */
int mhs_transpose(mhs_ctx *ctx, const mhs_csr *A, mhs_csr *At);

/* Free a device CSR produced by mhs_spgemm (hipFree) and zero the struct. */
void mhs_csr_free(mhs_csr *C);
/* Return C's device buffers to ctx's output pool for reuse by later calls
 * (a caching allocator: avoids hipMalloc/hipFree per call). */
void mhs_ctx_recycle(mhs_ctx *ctx, mhs_csr *C);

/* ---- host-side helpers (the reference's L1 layer) ---------------------- */

/* Host CSR (malloc'ed arrays). */
typedef struct mhs_host_csr {
    int32_t M, N, nnz;
    int32_t *ptr, *col;
    double *val;
    int32_t is_symmetric;
} mhs_host_csr;

/* readMtxFile (inc/mmio_read.h:34-159): real/integer/pattern(1.0)/complex
 * (real part); symmetric and hermitian off-diagonals mirrored, skew not;
 * duplicates kept; rows sorted by (col, val).  Returns MHS_OK or MHS_ERR_IO. */
int mhs_read_mtx(const char *path, mhs_host_csr *A);
void mhs_host_csr_free(mhs_host_csr *A);
/* Binary CSR cache (replaces re-running the fscanf loop of
 * inc/mmio_read.h:80-108 on every run).  mhs_read_mtx_cached reads `cache_path`
 * (NULL: path + ".mhscsr") when its stamp matches the .mtx's size and mtime,
 * else parses the text with mhs_read_mtx and writes the cache (best effort);
 * *from_cache (may be NULL) says which.  The cache reader checks ptr/col
 * invariants and returns MHS_ERR_IO on a truncated or corrupt file. */
int mhs_read_mtx_cached(const char *path, const char *cache_path, mhs_host_csr *A, int *from_cache);
int mhs_write_csr_bin(const char *path, const mhs_host_csr *A, int64_t src_size, int64_t src_mtime_ns);
int mhs_read_csr_bin(const char *path, mhs_host_csr *A, int64_t *src_size, int64_t *src_mtime_ns);
/* int_result of src/main.cu:102-107. */
uint64_t mhs_flop_count(int32_t nnzA, const int32_t *Acol, const int32_t *Bptr);

/* Device memory helpers for callers without their own HIP runtime binding
 * (e.g. ctypes).  kind: 0 = H2D, 1 = D2H, 2 = D2D.  Synchronous on ctx's stream. */
int mhs_memcpy(mhs_ctx *ctx, void *dst, const void *src, size_t bytes, int kind);
int mhs_device_alloc(mhs_ctx *ctx, void **p, size_t bytes);
int mhs_device_free(mhs_ctx *ctx, void *p);

/* Measured HBM bandwidth of the context's device (a diagnostic beside the 8 TB/s spec that
 * the roofline fractions are priced against; not on the SpGEMM path): streaming kernels over
 * two `bytes` buffers (>= 1 MiB; allocated and freed inside), each run `iters` times
 * between hipEvents.  gbps[0] = copy (read + write bytes), gbps[1] = read, gbps[2] = write,
 * in GB/s (1e9 B/s).  Synchronous. */
int mhs_hbm_peak(mhs_ctx *ctx, size_t bytes, int iters, double *gbps);

int mhs_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MHSPGEMM_H */
