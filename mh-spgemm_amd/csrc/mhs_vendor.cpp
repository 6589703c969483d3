// mhs_vendor.cpp -- rocSPARSE SpGEMM, the vendor row beside MH-SpGEMM (the
// reference's cuSPARSE comparison, inc/cusparse_spgemm.cuh:6-105).  Same stage
// order as the reference's cuSPARSE flow: buffer size -> nnz(C) -> allocate C ->
// compute; timed over the same span.
#include <hip/hip_runtime.h>
#include <rocsparse/rocsparse.h>

#include <chrono>
#include <cstdio>
#include <cstring>

#include "mhs_vendor.h"

namespace {

struct Fail {
    char* err;
    int len;
    int operator()(const char* what, int code) const {
        if (err && len > 0) std::snprintf(err, (size_t)len, "%s failed (%d)", what, code);
        return MHS_ERR_HIP;
    }
};

}  // namespace

#define HIPCHK(x)                                           \
    do {                                                    \
        hipError_t e_ = (x);                                \
        if (e_ != hipSuccess) { rc = fail(#x, (int)e_); goto out; } \
    } while (0)
#define RSCHK(x)                                                   \
    do {                                                           \
        rocsparse_status s_ = (x);                                 \
        if (s_ != rocsparse_status_success) { rc = fail(#x, (int)s_); goto out; } \
    } while (0)

extern "C" int mhs_vendor_spgemm(int device, const mhs_csr* A, const mhs_csr* B, mhs_csr* C, double* ms,
                                 char* err, int err_len) {
    const Fail fail{err, err_len};
    int rc = MHS_OK;
    rocsparse_handle h = nullptr;
    rocsparse_spmat_descr dA = nullptr, dB = nullptr, dC = nullptr;
    void* buf = nullptr;
    int32_t* cptr = nullptr;
    int32_t* ccol = nullptr;
    double* cval = nullptr;
    const double alpha = 1.0, beta = 0.0;
    size_t bytes = 0;
    int64_t rows = 0, cols = 0, nnz = 0;
    std::chrono::steady_clock::time_point t0, t1;
    if (!A || !B || !C || A->N != B->M) return fail("mhs_vendor_spgemm(arguments)", MHS_ERR_INVALID), MHS_ERR_INVALID;
    std::memset(C, 0, sizeof(*C));
    HIPCHK(hipSetDevice(device));
    RSCHK(rocsparse_create_handle(&h));
    RSCHK(rocsparse_create_csr_descr(&dA, A->M, A->N, A->nnz, A->ptr, A->col, A->val, rocsparse_indextype_i32,
                                     rocsparse_indextype_i32, rocsparse_index_base_zero, rocsparse_datatype_f64_r));
    RSCHK(rocsparse_create_csr_descr(&dB, B->M, B->N, B->nnz, B->ptr, B->col, B->val, rocsparse_indextype_i32,
                                     rocsparse_indextype_i32, rocsparse_index_base_zero, rocsparse_datatype_f64_r));
    // rocSPARSE wants C's row pointer at descriptor creation (cuSPARSE takes NULL and
    // the reference allocates it inside its timed span: here it is allocated just before)
    HIPCHK(hipMalloc((void**)&cptr, sizeof(int32_t) * ((size_t)A->M + 1)));
    RSCHK(rocsparse_create_csr_descr(&dC, A->M, B->N, 0, cptr, nullptr, nullptr, rocsparse_indextype_i32,
                                     rocsparse_indextype_i32, rocsparse_index_base_zero, rocsparse_datatype_f64_r));
    HIPCHK(hipDeviceSynchronize());
    t0 = std::chrono::steady_clock::now();
    RSCHK(rocsparse_spgemm(h, rocsparse_operation_none, rocsparse_operation_none, &alpha, dA, dB, &beta, dC, dC,
                           rocsparse_datatype_f64_r, rocsparse_spgemm_alg_default,
                           rocsparse_spgemm_stage_buffer_size, &bytes, nullptr));
    HIPCHK(hipMalloc(&buf, bytes ? bytes : 1));
    RSCHK(rocsparse_spgemm(h, rocsparse_operation_none, rocsparse_operation_none, &alpha, dA, dB, &beta, dC, dC,
                           rocsparse_datatype_f64_r, rocsparse_spgemm_alg_default, rocsparse_spgemm_stage_nnz,
                           &bytes, buf));
    RSCHK(rocsparse_spmat_get_size(dC, &rows, &cols, &nnz));
    if (nnz > INT32_MAX) {
        rc = fail("rocsparse nnz(C) beyond int32", (int)MHS_ERR_OVERFLOW);
        goto out;
    }
    HIPCHK(hipMalloc((void**)&ccol, sizeof(int32_t) * (size_t)(nnz ? nnz : 1)));
    HIPCHK(hipMalloc((void**)&cval, sizeof(double) * (size_t)(nnz ? nnz : 1)));
    RSCHK(rocsparse_csr_set_pointers(dC, cptr, ccol, cval));
    RSCHK(rocsparse_spgemm(h, rocsparse_operation_none, rocsparse_operation_none, &alpha, dA, dB, &beta, dC, dC,
                           rocsparse_datatype_f64_r, rocsparse_spgemm_alg_default, rocsparse_spgemm_stage_compute,
                           &bytes, buf));
    HIPCHK(hipFree(buf));
    buf = nullptr;
    HIPCHK(hipDeviceSynchronize());
    t1 = std::chrono::steady_clock::now();
    if (ms) *ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    C->M = A->M;
    C->N = B->N;
    C->nnz = (int32_t)nnz;
    C->ptr = cptr;
    C->col = ccol;
    C->val = cval;
    cptr = nullptr;
    ccol = nullptr;
    cval = nullptr;
out:
    if (buf) (void)hipFree(buf);
    if (cptr) (void)hipFree(cptr);
    if (ccol) (void)hipFree(ccol);
    if (cval) (void)hipFree(cval);
    if (dA) rocsparse_destroy_spmat_descr(dA);
    if (dB) rocsparse_destroy_spmat_descr(dB);
    if (dC) rocsparse_destroy_spmat_descr(dC);
    if (h) rocsparse_destroy_handle(h);
    return rc;
}

extern "C" void mhs_vendor_free(mhs_csr* C) {
    if (!C) return;
    if (C->ptr) (void)hipFree(C->ptr);
    if (C->col) (void)hipFree(C->col);
    if (C->val) (void)hipFree(C->val);
    std::memset(C, 0, sizeof(*C));
}
