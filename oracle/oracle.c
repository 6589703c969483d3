/*
 * oracle.c -- CPU restatement of the reference MH-SpGEMM host semantics.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Parity UNPINNED against reference
 * outputs; pinned to scipy.sparse fixtures (tests/golden/) and known answers.
 *
 * Build: oracle/Makefile (gcc -O2 -fopenmp -ffp-contract=off).  The
 * -ffp-contract=off flag matters: every value is a separate multiply then add,
 * in a fixed order, which is what makes the restatement bit-reproducible and
 * bit-identical to scipy's SMMP accumulation order.
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <ctype.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

int orc_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ---------------------------------------------------------------- mmio --- */

/* Banner: "%%MatrixMarket matrix coordinate <type> <storage>", tokens lower-
 * cased, all five required (inc/mmio.h:128-202).  Type: real|complex|pattern|
 * integer; storage: general|symmetric|hermitian|skew-symmetric. */
typedef struct {
    char type;    /* 'R' 'C' 'P' 'I' */
    char storage; /* 'G' 'S' 'H' 'K' */
    int array;
} orc_banner;

static void lower(char *s) {
    for (; *s; ++s) *s = (char)tolower((unsigned char)*s);
}

static int read_banner(FILE *f, orc_banner *b) {
    char line[1025], ban[64], mtx[64], crd[64], dt[64], st[64];
    if (!fgets(line, sizeof line, f)) return -2;
    if (sscanf(line, "%63s %63s %63s %63s %63s", ban, mtx, crd, dt, st) != 5) return -2;
    lower(mtx); lower(crd); lower(dt); lower(st);
    if (strncmp(ban, "%%MatrixMarket", 14) != 0) return -2;
    if (strcmp(mtx, "matrix") != 0) return -2;
    if (strcmp(crd, "coordinate") == 0) b->array = 0;
    else if (strcmp(crd, "array") == 0) b->array = 1;
    else return -2;
    if (!strcmp(dt, "real")) b->type = 'R';
    else if (!strcmp(dt, "complex")) b->type = 'C';
    else if (!strcmp(dt, "pattern")) b->type = 'P';
    else if (!strcmp(dt, "integer")) b->type = 'I';
    else return -2;
    if (!strcmp(st, "general")) b->storage = 'G';
    else if (!strcmp(st, "symmetric")) b->storage = 'S';
    else if (!strcmp(st, "hermitian")) b->storage = 'H';
    else if (!strcmp(st, "skew-symmetric")) b->storage = 'K';
    else return -2;
    return 0;
}

/* Size line: skip '%' comment lines, then "M N nz" (inc/mmio.h:204-232). */
static int read_size(FILE *f, int *M, int *N, int *nz) {
    char line[1025];
    *M = *N = *nz = 0;
    do {
        if (!fgets(line, sizeof line, f)) return -3;
    } while (line[0] == '%');
    if (sscanf(line, "%d %d %d", M, N, nz) == 3) return 0;
    for (;;) {
        int r = fscanf(f, "%d %d %d", M, N, nz);
        if (r == EOF) return -3;
        if (r == 3) return 0;
    }
}

typedef struct { int32_t c; double v; } orc_cv;

static int cmp_cv(const void *a, const void *b) {
    const orc_cv *x = (const orc_cv *)a, *y = (const orc_cv *)b;
    if (x->c != y->c) return x->c < y->c ? -1 : 1;
    if (x->v < y->v) return -1;
    if (x->v > y->v) return 1;
    return 0;
}

/* Per-row sort by (col, val) pairs, as std::sort over pair<int,double>
 * (inc/mmio_read.h:9-31). */
static void sort_rows(int32_t M, const int32_t *ptr, int32_t *col, double *val) {
#pragma omp parallel
    {
        size_t cap = 0;
        orc_cv *buf = NULL;
#pragma omp for schedule(dynamic, 64)
        for (int32_t r = 0; r < M; ++r) {
            int32_t s = ptr[r], e = ptr[r + 1], n = e - s;
            if (n < 2) continue;
            if ((size_t)n > cap) {
                free(buf);
                cap = (size_t)n;
                buf = (orc_cv *)malloc(cap * sizeof(orc_cv));
            }
            for (int32_t j = 0; j < n; ++j) { buf[j].c = col[s + j]; buf[j].v = val[s + j]; }
            qsort(buf, (size_t)n, sizeof(orc_cv), cmp_cv);
            for (int32_t j = 0; j < n; ++j) { col[s + j] = buf[j].c; val[s + j] = buf[j].v; }
        }
        free(buf);
    }
}

/* readMtxFile (inc/mmio_read.h:34-159):
 *   - entries read with fscanf per type: real "%d %d %lg", integer "%d %d %d"
 *     (converted to double), pattern "%d %d" (value 1.0), complex
 *     "%d %d %lg %lg" (real part kept)                            (:80-102)
 *   - 1-based -> 0-based                                           (:104-105)
 *   - symmetric or hermitian: every off-diagonal entry is mirrored with the
 *     same value; skew-symmetric is NOT mirrored                   (:112-121)
 *   - CSR fill in file order, each entry followed by its mirror    (:130-146)
 *   - duplicates kept; rows sorted by (col,val)                    (:150)
 * Deviation (documented): "array" (dense) storage is rejected; the reference
 * would mis-parse it as coordinate. */
int orc_read_mtx(const char *path, orc_csr *A) {
    memset(A, 0, sizeof *A);
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    orc_banner b;
    int rc = read_banner(f, &b);
    if (rc) { fclose(f); return rc; }
    if (b.array) { fclose(f); return -5; }
    int M, N, nz;
    rc = read_size(f, &M, &N, &nz);
    if (rc) { fclose(f); return rc; }
    if (M < 0 || N < 0 || nz < 0) { fclose(f); return -3; }
    int32_t *ri = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nz > 0 ? nz : 1));
    int32_t *ci = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nz > 0 ? nz : 1));
    double *vv = (double *)malloc(sizeof(double) * (size_t)(nz > 0 ? nz : 1));
    int32_t *cnt = (int32_t *)calloc((size_t)M + 1, sizeof(int32_t));
    int sym = (b.storage == 'S' || b.storage == 'H');
    for (int i = 0; i < nz; ++i) {
        int r, c, iv, got;
        double v = 0.0, im;
        switch (b.type) {
        case 'R': got = fscanf(f, "%d %d %lg\n", &r, &c, &v); rc = (got == 3); break;
        case 'I': got = fscanf(f, "%d %d %d\n", &r, &c, &iv); v = iv; rc = (got == 3); break;
        case 'P': got = fscanf(f, "%d %d\n", &r, &c); v = 1.0; rc = (got == 2); break;
        default:  got = fscanf(f, "%d %d %lg %lg\n", &r, &c, &v, &im); rc = (got == 4); break;
        }
        if (!rc) { rc = -4; goto fail; }
        --r; --c;
        if (r < 0 || r >= M || c < 0 || c >= N) { rc = -6; goto fail; }
        ri[i] = r; ci[i] = c; vv[i] = v;
        cnt[r]++;
    }
    fclose(f);
    f = NULL;
    if (sym)
        for (int i = 0; i < nz; ++i)
            if (ri[i] != ci[i]) {
                if (ci[i] >= M) { rc = -6; goto fail; }
                cnt[ci[i]]++;
            }
    /* exclusive scan (src/utils.cpp:3-18) */
    {
        int64_t run = 0;
        for (int r = 0; r <= M; ++r) {
            int32_t c = cnt[r];
            cnt[r] = (int32_t)run;
            run += c;
        }
        if (run > 0x7fffffff) { rc = -6; goto fail; }
    }
    A->M = M; A->N = N; A->nnz = cnt[M];
    A->is_symmetric = (b.storage == 'S');
    A->ptr = cnt;
    A->col = (int32_t *)malloc(sizeof(int32_t) * (size_t)(A->nnz > 0 ? A->nnz : 1));
    A->val = (double *)malloc(sizeof(double) * (size_t)(A->nnz > 0 ? A->nnz : 1));
    {
        int32_t *off = (int32_t *)calloc((size_t)M + 1, sizeof(int32_t));
        for (int i = 0; i < nz; ++i) {
            int32_t r = ri[i], c = ci[i];
            int32_t o = cnt[r] + off[r]++;
            A->col[o] = c; A->val[o] = vv[i];
            if (sym && r != c) {
                o = cnt[c] + off[c]++;
                A->col[o] = r; A->val[o] = vv[i];
            }
        }
        free(off);
    }
    free(ri); free(ci); free(vv);
    sort_rows(A->M, A->ptr, A->col, A->val);
    return 0;
fail:
    if (f) fclose(f);
    free(ri); free(ci); free(vv); free(cnt);
    memset(A, 0, sizeof *A);
    return rc;
}

void orc_csr_free(orc_csr *A) {
    if (!A) return;
    free(A->ptr); free(A->col); free(A->val);
    memset(A, 0, sizeof *A);
}

/* ------------------------------------------------------- flop, transpose --- */

unsigned long long orc_flop(int32_t nnzA, const int32_t *Acol, const int32_t *Bptr) {
    unsigned long long s = 0;
    for (int32_t j = 0; j < nnzA; ++j) s += (unsigned long long)(Bptr[Acol[j] + 1] - Bptr[Acol[j]]);
    return s;
}

int orc_transpose(const orc_csr *A, orc_csr *T) {
    memset(T, 0, sizeof *T);
    T->M = A->N; T->N = A->M; T->nnz = A->nnz;
    T->ptr = (int32_t *)calloc((size_t)A->N + 1, sizeof(int32_t));
    T->col = (int32_t *)malloc(sizeof(int32_t) * (size_t)(A->nnz > 0 ? A->nnz : 1));
    T->val = (double *)malloc(sizeof(double) * (size_t)(A->nnz > 0 ? A->nnz : 1));
    if (!T->ptr || !T->col || !T->val) { orc_csr_free(T); return -1; }
    for (int32_t j = 0; j < A->nnz; ++j) T->ptr[A->col[j]]++;
    int32_t run = 0;
    for (int32_t c = 0; c <= A->N; ++c) { int32_t x = T->ptr[c]; T->ptr[c] = run; run += x; }
    int32_t *fill = (int32_t *)calloc((size_t)A->N + 1, sizeof(int32_t));
    for (int32_t r = 0; r < A->M; ++r)
        for (int32_t j = A->ptr[r]; j < A->ptr[r + 1]; ++j) {
            int32_t c = A->col[j];
            int32_t o = T->ptr[c] + fill[c]++;
            T->col[o] = r; T->val[o] = A->val[j];
        }
    free(fill);
    return 0;
}

/* --------------------------------------------------------------- SpGEMM --- */

static int cmp_i32(const void *a, const void *b) {
    int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
    return (x > y) - (x < y);
}

static void sort_i32(int32_t *v, int32_t n) {
    if (n < 32) {
        for (int32_t i = 1; i < n; ++i) {
            int32_t x = v[i], j = i - 1;
            while (j >= 0 && v[j] > x) { v[j + 1] = v[j]; --j; }
            v[j + 1] = x;
        }
    } else {
        qsort(v, (size_t)n, sizeof(int32_t), cmp_i32);
    }
}

int64_t orc_spgemm_symbolic(int32_t M, int32_t N, const int32_t *Ap, const int32_t *Ai,
                            const int32_t *Bp, const int32_t *Bi, int32_t *Cp, int nthreads) {
    if (nthreads <= 0) nthreads = orc_max_threads();
    int err = 0;
#pragma omp parallel num_threads(nthreads)
    {
        int32_t *mark = (int32_t *)malloc(sizeof(int32_t) * (size_t)(N > 0 ? N : 1));
        if (!mark) {
#pragma omp atomic write
            err = 1;
        } else {
            for (int32_t c = 0; c < N; ++c) mark[c] = -1;
#pragma omp for schedule(dynamic, 64)
            for (int32_t i = 0; i < M; ++i) {
                int32_t n = 0;
                for (int32_t j = Ap[i]; j < Ap[i + 1]; ++j) {
                    int32_t k = Ai[j];
                    for (int32_t q = Bp[k]; q < Bp[k + 1]; ++q) {
                        int32_t c = Bi[q];
                        if (mark[c] != i) { mark[c] = i; ++n; }
                    }
                }
                Cp[i] = n;
            }
            free(mark);
        }
    }
    if (err) return -1;
    int64_t run = 0;
    for (int32_t i = 0; i < M; ++i) { int32_t n = Cp[i]; Cp[i] = (int32_t)run; run += n; }
    Cp[M] = (int32_t)run;
    if (run > 0x7fffffff) return -1;
    return run;
}

int orc_spgemm_numeric(int32_t M, int32_t N, const int32_t *Ap, const int32_t *Ai, const double *Av,
                       const int32_t *Bp, const int32_t *Bi, const double *Bv,
                       const int32_t *Cp, int32_t *Ci, double *Cv,
                       int32_t row_begin, int32_t row_end, int nthreads) {
    if (nthreads <= 0) nthreads = orc_max_threads();
    if (row_begin < 0) row_begin = 0;
    if (row_end > M) row_end = M;
    int err = 0;
#pragma omp parallel num_threads(nthreads)
    {
        double *acc = (double *)malloc(sizeof(double) * (size_t)(N > 0 ? N : 1));
        int32_t *mark = (int32_t *)malloc(sizeof(int32_t) * (size_t)(N > 0 ? N : 1));
        if (!acc || !mark) {
#pragma omp atomic write
            err = 1;
        } else {
            for (int32_t c = 0; c < N; ++c) mark[c] = -1;
#pragma omp for schedule(dynamic, 64)
            for (int32_t i = row_begin; i < row_end; ++i) {
                int32_t *list = Ci + Cp[i];
                int32_t n = 0;
                for (int32_t j = Ap[i]; j < Ap[i + 1]; ++j) {
                    int32_t k = Ai[j];
                    double a = Av[j];
                    for (int32_t q = Bp[k]; q < Bp[k + 1]; ++q) {
                        int32_t c = Bi[q];
                        if (mark[c] != i) {
                            mark[c] = i;
                            acc[c] = 0.0;
                            list[n++] = c;
                        }
                        double p = a * Bv[q]; /* separate multiply ... */
                        acc[c] = acc[c] + p;  /* ... then add: no FMA */
                    }
                }
                sort_i32(list, n);
                for (int32_t t = 0; t < n; ++t) Cv[Cp[i] + t] = acc[list[t]];
            }
        }
        free(acc);
        free(mark);
    }
    return err ? -1 : 0;
}

/* ------------------------------------------------------------ checkers --- */

int orc_compare_ref(int32_t M, int32_t nnz_self, const int32_t *p_self, const int32_t *c_self,
                    const double *v_self, int32_t nnz_other, const int32_t *p_other,
                    const int32_t *c_other, const double *v_other, int verbose) {
    if (nnz_self != nnz_other) {
        if (verbose) printf("nnz not equal %d %d\n", nnz_self, nnz_other);
        return -1;
    }
    int err = 0;
    const double eps = 1e-9;
    for (int32_t i = 0; i < M; ++i) {
        if (err > 10) return -2;
        if (p_self[i] != p_other[i]) {
            if (verbose) printf("ptr not equal at %d rows, %d != %d\n", i, p_self[i], p_other[i]);
            err++;
        }
        for (int32_t j = p_self[i]; j < p_self[i + 1]; ++j) {
            if (err > 10) return -2;
            if (c_self[j] != c_other[j]) {
                if (verbose) printf("col not equal at %d rows, index %d != %d\n", i, c_self[j], c_other[j]);
                err++;
            }
            double d = fabs(v_self[j] - v_other[j]);
            if (!(d < eps || d < eps * fabs(v_self[j]))) {
                if (verbose) printf("val not eqaul at %d rows, value %.18le != %.18le\n", i, v_self[j], v_other[j]);
                err++;
            }
        }
    }
    if (p_self[M] != p_other[M]) {
        if (verbose) printf("ptr[M] not equal\n");
        return -3;
    }
    return err ? 0 : 1;
}

int64_t orc_compare_tol(int32_t M, int32_t nnz_ref, const int32_t *p_ref, const int32_t *c_ref,
                        const double *v_ref, int32_t nnz_got, const int32_t *p_got,
                        const int32_t *c_got, const double *v_got, double rtol, double atol) {
    if (nnz_ref != nnz_got) return -1;
    int64_t bad = 0;
    for (int32_t i = 0; i <= M; ++i) bad += (p_ref[i] != p_got[i]);
    if (bad) return bad;
    for (int32_t j = 0; j < nnz_ref; ++j) {
        if (c_ref[j] != c_got[j]) { ++bad; continue; }
        double d = fabs(v_ref[j] - v_got[j]);
        if (!(d <= atol || d <= rtol * fabs(v_ref[j]))) ++bad;
    }
    return bad;
}
