// mh_spgemm.hpp -- header-only C++ shim over the C-ABI (mhspgemm.h) that gives
// a driver written against the reference the reference's own surface:
//
//   class CSR      (inc/CSR.h:4-44, src/CSR.cu:4-135)   host + device arrays,
//                  H2D / D2H, operator== (the cuSPARSE-style checker)
//   class Timing   (inc/Timing.h, src/Timing.cpp)       7 phase fields, getTotal()
//   class Tool     (inc/Tool.h, src/Tool.cu)            here: owns the mhs_ctx
//   void MH_spgemm(const CSR&, CSR&, CSR&, Timing&, Tool&)   (src/main.cu:12-72)
//   int  readMtxFile(CSR&, const char*)                      (inc/mmio_read.h:34)
//
// Errors: the C-ABI returns codes; this shim rethrows as std::runtime_error so a
// caller's try { MH_spgemm(...) } catch (...) { "MH-SpGEMM failed!!!" } behaves as
// in the reference (src/main.cu:117-145).  B is not mutated (no d_tile* arrays).
#pragma once
#include <hip/hip_runtime.h>

#include <cassert>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>

#include "mhspgemm.h"

namespace mhs_shim {
inline void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) {
        std::printf("%s in %s\n", hipGetErrorString(e), what);
        throw std::runtime_error(what);
    }
}
}  // namespace mhs_shim

class CSR {
public:
    int M = 0, N = 0, nnz = 0;
    int* ptr = nullptr;
    int* col = nullptr;
    double* val = nullptr;
    int* d_ptr = nullptr;
    int* d_col = nullptr;
    double* d_val = nullptr;
    int isSymmetric = 0;

    CSR() = default;
    CSR(const CSR&) = delete;
    ~CSR() { release(); }

    void alloc(int r, int c, int n) {
        h_release_csr();
        M = r;
        N = c;
        nnz = n;
        ptr = new int[r + 1]();
        col = new int[n > 0 ? n : 1];
        val = new double[n > 0 ? n : 1];
    }
    // deep host copy, as the reference (src/CSR.cu:34-47)
    CSR& operator=(const CSR& A) {
        if (this == &A) return *this;
        alloc(A.M, A.N, A.nnz);
        isSymmetric = A.isSymmetric;
        std::memcpy(ptr, A.ptr, sizeof(int) * (size_t)(M + 1));
        std::memcpy(col, A.col, sizeof(int) * (size_t)nnz);
        std::memcpy(val, A.val, sizeof(double) * (size_t)nnz);
        return *this;
    }
    // CSR::operator== (src/CSR.cu:48-96): nnz mismatch throws; ptr and col exact;
    // val accepted when |d| < 1e-9 or |d| < 1e-9 * |this->val|; > 10 errors throws.
    bool operator==(const CSR& o) const {
        if (nnz != o.nnz) {
            std::printf("nnz not equal %d %d\n", nnz, o.nnz);
            throw std::runtime_error("nnz not equal");
        }
        assert(M == o.M && N == o.N);
        int err = 0;
        const double eps = 1e-9;
        for (int i = 0; i < M; i++) {
            if (err > 10) throw std::runtime_error("matrix compare: error num exceed threshold");
            if (ptr[i] != o.ptr[i]) {
                std::printf("ptr not equal at %d rows, %d != %d\n", i, ptr[i], o.ptr[i]);
                err++;
            }
            for (int j = ptr[i]; j < ptr[i + 1]; j++) {
                if (err > 10) throw std::runtime_error("matrix compare: error num exceed threshold");
                if (col[j] != o.col[j]) {
                    std::printf("col not equal at %d rows, index %d != %d\n", i, col[j], o.col[j]);
                    err++;
                }
                const double d = std::fabs(val[j] - o.val[j]);
                if (!(d < eps || d < eps * std::fabs(val[j]))) {
                    std::printf("val not eqaul at %d rows, value %.18le != %.18le\n", i, val[j], o.val[j]);
                    err++;
                }
            }
        }
        if (ptr[M] != o.ptr[M]) {
            std::printf("ptr[M] not equal\n");
            throw std::runtime_error("matrix compare: error num exceed threshold");
        }
        return err == 0;
    }
    void H2D() {
        using mhs_shim::hip_check;
        hip_check(hipMalloc((void**)&d_ptr, sizeof(int) * (size_t)(M + 1)), "hipMalloc d_ptr");
        hip_check(hipMalloc((void**)&d_col, sizeof(int) * (size_t)(nnz > 0 ? nnz : 1)), "hipMalloc d_col");
        hip_check(hipMalloc((void**)&d_val, sizeof(double) * (size_t)(nnz > 0 ? nnz : 1)), "hipMalloc d_val");
        hip_check(hipMemcpy(d_ptr, ptr, sizeof(int) * (size_t)(M + 1), hipMemcpyHostToDevice), "H2D ptr");
        hip_check(hipMemcpy(d_col, col, sizeof(int) * (size_t)nnz, hipMemcpyHostToDevice), "H2D col");
        hip_check(hipMemcpy(d_val, val, sizeof(double) * (size_t)nnz, hipMemcpyHostToDevice), "H2D val");
    }
    void D2H() {
        using mhs_shim::hip_check;
        h_release_csr();
        ptr = new int[M + 1];
        col = new int[nnz > 0 ? nnz : 1];
        val = new double[nnz > 0 ? nnz : 1];
        hip_check(hipMemcpy(ptr, d_ptr, sizeof(int) * (size_t)(M + 1), hipMemcpyDeviceToHost), "D2H ptr");
        hip_check(hipMemcpy(col, d_col, sizeof(int) * (size_t)nnz, hipMemcpyDeviceToHost), "D2H col");
        hip_check(hipMemcpy(val, d_val, sizeof(double) * (size_t)nnz, hipMemcpyDeviceToHost), "D2H val");
    }
    void h_release_csr() {
        delete[] ptr;
        delete[] col;
        delete[] val;
        ptr = col = nullptr;
        val = nullptr;
    }
    void d_release_csr() {
        if (d_ptr) (void)hipFree(d_ptr);
        if (d_col) (void)hipFree(d_col);
        if (d_val) (void)hipFree(d_val);
        d_ptr = d_col = nullptr;
        d_val = nullptr;
    }
    void release() {
        h_release_csr();
        d_release_csr();
    }
};

class Timing {
public:
    double mem_alloc = 0, Form_mask_matrix_B = 0, Calculate_C_nnz = 0, Malloc_C_col_val = 0, Numeric = 0,
           symbolic_binning = 0, numeric_binning = 0;
    double total_e2e = 0;
    unsigned long long flop = 0;

    void operator+=(const Timing& t) {
        mem_alloc += t.mem_alloc;
        Form_mask_matrix_B += t.Form_mask_matrix_B;
        Calculate_C_nnz += t.Calculate_C_nnz;
        Malloc_C_col_val += t.Malloc_C_col_val;
        Numeric += t.Numeric;
        symbolic_binning += t.symbolic_binning;
        numeric_binning += t.numeric_binning;
        total_e2e += t.total_e2e;
    }
    void operator/=(double x) {
        mem_alloc /= x;
        Form_mask_matrix_B /= x;
        Calculate_C_nnz /= x;
        Malloc_C_col_val /= x;
        Numeric /= x;
        symbolic_binning /= x;
        numeric_binning /= x;
        total_e2e /= x;
    }
    void print_step_time() const {
        std::printf("  -------------time-------------\n");
        std::printf("    mem_alloc: \t\t%.3lfms\n", mem_alloc);
        std::printf("    form_mask_matrix_B: %.3lfms\n", Form_mask_matrix_B);
        std::printf("    symbolic_binning: \t%.3lfms\n", symbolic_binning);
        std::printf("    calculate_C_nnz: \t%.3lfms\n", Calculate_C_nnz);
        std::printf("    malloc_C_col_val: \t%.3lfms\n", Malloc_C_col_val);
        std::printf("    numeric_binning: \t%.3lfms\n", numeric_binning);
        std::printf("    numeric: \t\t%.3lfms\n", Numeric);
        std::printf("  ------------------------------\n");
    }
    // src/Timing.cpp:39-41: excludes Form_mask_matrix_B
    double getTotal() const {
        return Calculate_C_nnz + Malloc_C_col_val + Numeric + symbolic_binning + numeric_binning + mem_alloc;
    }
};

class Tool {
public:
    mhs_ctx* ctx = nullptr;
    explicit Tool(int device = 0) {
        if (mhs_ctx_create(&ctx, device) != MHS_OK) throw std::runtime_error("mhs_ctx_create failed");
    }
    Tool(const Tool&) = delete;
    ~Tool() { mhs_ctx_destroy(ctx); }
    // The reference allocates per call (src/Tool.cu:4-45); the context keeps its
    // workspace across calls, release() trims it.
    void allocate(const CSR&, const CSR&) {}
    void release() { mhs_ctx_trim(ctx); }
};

inline void MH_spgemm(const CSR& A, CSR& B, CSR& C, Timing& timing, Tool& tools) {
    mhs_csr a{A.M, A.N, A.nnz, A.d_ptr, A.d_col, A.d_val};
    mhs_csr b{B.M, B.N, B.nnz, B.d_ptr, B.d_col, B.d_val};
    mhs_csr c{};
    mhs_timing t{};
    const int rc = mhs_spgemm(tools.ctx, &a, &b, &c, &t);
    if (rc != MHS_OK) {
        std::printf("%s\n", mhs_last_error(tools.ctx));
        throw std::runtime_error(mhs_last_error(tools.ctx));
    }
    C.d_release_csr();
    C.M = c.M;
    C.N = c.N;
    C.nnz = c.nnz;
    C.d_ptr = c.ptr;
    C.d_col = c.col;
    C.d_val = c.val;
    std::printf("C.nnz = %d\n", C.nnz);
    timing.mem_alloc = t.mem_alloc;
    timing.Form_mask_matrix_B = t.Form_mask_matrix_B;
    timing.symbolic_binning = t.symbolic_binning;
    timing.Calculate_C_nnz = t.Calculate_C_nnz;
    timing.numeric_binning = t.numeric_binning;
    timing.Malloc_C_col_val = t.Malloc_C_col_val;
    timing.Numeric = t.Numeric;
    timing.total_e2e = t.total_e2e;
    timing.flop = t.flop;
}

// src/utils.cpp:20-46 (B = A^T for AAT, src/main.cu:98-99) on the device: A must be
// device-resident; B gets device arrays (and host arrays, as the reference's B).
inline void matrix_transposition(const CSR& A, CSR& B, Tool& tools) {
    mhs_csr a{A.M, A.N, A.nnz, A.d_ptr, A.d_col, A.d_val};
    mhs_csr t{};
    if (mhs_transpose(tools.ctx, &a, &t) != MHS_OK) throw std::runtime_error(mhs_last_error(tools.ctx));
    B.release();
    B.M = t.M;
    B.N = t.N;
    B.nnz = t.nnz;
    B.isSymmetric = 0;
    B.d_ptr = t.ptr;
    B.d_col = t.col;
    B.d_val = t.val;
    B.D2H();
}

// cache = true: a binary CSR cache beside the file (mhs_read_mtx_cached), re-parsed
// only when the .mtx changes.
inline int readMtxFile(CSR& A, const char* filename, bool cache = false) {
    mhs_host_csr h{};
    const int rc = cache ? mhs_read_mtx_cached(filename, nullptr, &h, nullptr) : mhs_read_mtx(filename, &h);
    if (rc != MHS_OK) {
        std::printf("Could not read Matrix Market file %s.\n", filename);
        return -1;
    }
    A.alloc(h.M, h.N, h.nnz);
    A.isSymmetric = h.is_symmetric;
    std::memcpy(A.ptr, h.ptr, sizeof(int) * (size_t)(h.M + 1));
    std::memcpy(A.col, h.col, sizeof(int) * (size_t)h.nnz);
    std::memcpy(A.val, h.val, sizeof(double) * (size_t)h.nnz);
    mhs_host_csr_free(&h);
    return 0;
}
