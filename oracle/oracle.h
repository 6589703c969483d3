/*
 * oracle.h -- CPU restatement of the reference MH-SpGEMM host semantics.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (mh-spgemm_amd/) may
 * include, link or call this.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py use it, and only as the checker / the timed CPU
 * baseline ("kind": "port").
 *
 * Parity status: UNPINNED against reference-generated outputs.  The reference
 * (yyssys/MH-SpGEMM) ships no tests, no fixtures and no golden vectors for this
 * path, its kernels need nvcc, and its host code needs the CUDA runtime
 * library (libcudart), which this image does not have.
 * The restatement is instead cross-checked bit-exactly against an independent
 * implementation (scipy.sparse, committed as tests/golden/ fixtures together
 * with tests/golden/make_golden.py) and against hand-derived known answers.
 *
 * Each function cites the reference file:line whose behaviour it restates.
 */
#ifndef MHS_ORACLE_H
#define MHS_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_csr {
    int32_t M, N, nnz;
    int32_t *ptr; /* M+1 */
    int32_t *col; /* nnz */
    double *val;  /* nnz */
    int32_t is_symmetric; /* banner says "symmetric" (inc/mmio_read.h:63) */
} orc_csr;

/* Matrix Market -> CSR (inc/mmio_read.h:34-159, inc/mmio.h:128-232).
 * Returns 0 on success, a negative code on failure:
 *   -1 cannot open, -2 bad banner, -3 bad size line, -4 short read,
 *   -5 unsupported (array storage), -6 out-of-range index. */
int orc_read_mtx(const char *path, orc_csr *A);
void orc_csr_free(orc_csr *A);

/* int_result = sum over A's nonzeros of nnz(B row A.col[j]) (src/main.cu:102-107). */
unsigned long long orc_flop(int32_t nnzA, const int32_t *Acol, const int32_t *Bptr);

/* CSR transpose by counting sort (src/utils.cpp:20-46). T arrays malloc'ed. */
int orc_transpose(const orc_csr *A, orc_csr *T);

/* C = A*B, Gustavson, structural nnz (cancellation zeros kept, like the symbolic
 * phase inc/Calculate_C_nnz.cuh:410-835), columns sorted ascending per row
 * (inc/numeric.cuh:287-297), each value accumulated in double in the fixed
 * order (A entries in row order, then B entries in row order).
 * Pass 1 fills Cptr[M+1] and returns nnz(C) (or -1 on error). */
int64_t orc_spgemm_symbolic(int32_t M, int32_t N, const int32_t *Ap, const int32_t *Ai,
                            const int32_t *Bp, const int32_t *Bi, int32_t *Cp, int nthreads);
/* Pass 2 fills Ci/Cv given Cp from pass 1.  Rows [row_begin,row_end) only
 * (so the CPU baseline can time a bounded row sample); Cp must still be the
 * full pass-1 array.  Returns 0 on success. */
int orc_spgemm_numeric(int32_t M, int32_t N, const int32_t *Ap, const int32_t *Ai, const double *Av,
                       const int32_t *Bp, const int32_t *Bi, const double *Bv,
                       const int32_t *Cp, int32_t *Ci, double *Cv,
                       int32_t row_begin, int32_t row_end, int nthreads);

/* The reference checker CSR::operator== (src/CSR.cu:48-96), restated:
 *   returns  1  equal
 *            0  unequal with <= 10 errors
 *           -1  nnz differ            (reference throws "nnz not equal")
 *           -2  more than 10 errors   (reference throws "error num exceed threshold")
 *           -3  ptr[M] differ         (reference throws)
 * "self" is the left operand (its val is the relative-error base, :80). */
int orc_compare_ref(int32_t M, int32_t nnz_self, const int32_t *p_self, const int32_t *c_self,
                    const double *v_self, int32_t nnz_other, const int32_t *p_other,
                    const int32_t *c_other, const double *v_other, int verbose);

/* North-star checker: ptr and col bit-exact, val |d| <= rtol*|ref| or |d| <= atol.
 * Returns the number of mismatching entries (0 = pass), -1 if nnz differ. */
int64_t orc_compare_tol(int32_t M, int32_t nnz_ref, const int32_t *p_ref, const int32_t *c_ref,
                        const double *v_ref, int32_t nnz_got, const int32_t *p_got,
                        const int32_t *c_got, const double *v_got, double rtol, double atol);

int orc_max_threads(void);

#ifdef __cplusplus
}
#endif
#endif
