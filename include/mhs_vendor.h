/*
 * mhs_vendor.h -- rocSPARSE SpGEMM on the same box: the vendor comparison row
 * (libmhs_vendor.so, kept out of libmhspgemm.so so the product library does not
 * depend on rocSPARSE).
 *
 * Replaces the reference's cuSPARSE path, compiled in with CUSPARSE=1
 * (inc/common.h:78):  cusparse_spgemm(CSR* a, CSR* b, CSR* c, double* time)
 * (/root/reference/inc/cusparse_spgemm.cuh:94-105, inner :6-92), called from
 * src/main.cu:148-170 and checked against MH-SpGEMM's C with CSR::operator==
 * under CHECK_RESULT (src/main.cu:186-199).
 *
 * Timing span as the reference's: from the first SpGEMM call (buffer-size
 * query) through C's allocation, the compute stage and the buffer release,
 * device-synchronised on both sides (cusparse_spgemm.cuh:30-88); the library
 * handle and descriptors are created outside it.
 */
#ifndef MHS_VENDOR_H
#define MHS_VENDOR_H
#include "mhspgemm.h"

#ifdef __cplusplus
extern "C" {
#endif

/* C = A * B with rocsparse_spgemm (CSR, int32 indices, FP64).  A, B: device CSR
 * on `device`.  On MHS_OK, C's arrays are fresh hipMalloc'd device buffers
 * (free with mhs_vendor_free) and *ms holds the timed span in milliseconds.
 * Errors: MHS_ERR_HIP (HIP or rocSPARSE failure; message in *err if non-NULL). */
int mhs_vendor_spgemm(int device, const mhs_csr *A, const mhs_csr *B, mhs_csr *C, double *ms,
                      char *err, int err_len);
/* hipFree C's arrays and zero the struct. */
void mhs_vendor_free(mhs_csr *C);

#ifdef __cplusplus
}
#endif
#endif /* MHS_VENDOR_H */
