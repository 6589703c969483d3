// mhs_transpose.hip -- device CSR transpose, the operand of the AAT mode (C = A*A^T).
//
// The reference builds B = A^T on the host before the upload when AAT is set
// (inc/common.h:37, src/main.cu:98-99, host transpose src/utils.cpp:20-46: a column
// count, a prefix sum and a row-ordered scatter, so every row of A^T lists its
// columns -- A's row indices -- ascending).  Here the same result comes from one
// stable radix sort of A's entries by column (rocPRIM: LSD radix sort is stable, and
// A's entries are in row-major order, so each column's entries keep ascending row
// order), a gather of (row, value) through the sorted entry indices, and the row
// pointer read off the sorted keys.
#include "mhs_internal.hpp"

#include <rocprim/device/device_radix_sort.hpp>

namespace mhs {

__global__ void k_tr_iota(int nnz, int* __restrict__ idx) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < nnz) idx[e] = e;
}

// row of entry e: the last i with ptr[i] <= e (binary search over the row pointer)
__device__ __forceinline__ int row_of(const int* __restrict__ ptr, int M, int e) {
    int lo = 0, hi = M;  // ptr[lo] <= e < ptr[hi]
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (ptr[mid] <= e) lo = mid;
        else hi = mid;
    }
    return lo;
}

__global__ void k_tr_gather(int M, int nnz, const int* __restrict__ Aptr, const double* __restrict__ Aval,
                            const int* __restrict__ idx, int* __restrict__ tcol, double* __restrict__ tval) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nnz) return;
    const int e = idx[k];
    tcol[k] = row_of(Aptr, M, e);
    tval[k] = Aval[e];
}

// A^T row pointer from the sorted keys (A's columns): entry k opens rows
// (key[k-1], key[k]]; the last entry closes rows (key[nnz-1], N].
__global__ void k_tr_ptr(int N, int nnz, const int* __restrict__ key, int* __restrict__ tptr) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nnz) return;
    // clamped: a column outside [0, N) (an invalid A) must not write outside tptr
    const int c = min(max(key[k], -1), N - 1);
    const int p = k > 0 ? min(max(key[k - 1], -1), N - 1) : -1;
    for (int r = p + 1; r <= c; ++r) tptr[r] = k;
    if (k == nnz - 1)
        for (int r = c + 1; r <= N; ++r) tptr[r] = nnz;
}

// tmp == nullptr: *tmp_bytes = the scratch size needed.  Else At (N x M, nnz(A)) is
// written into tptr[N+1], tcol[nnz], tval[nnz].
hipError_t transpose_csr(const Csr& A, int* tptr, int* tcol, double* tval, void* tmp, size_t* tmp_bytes,
                         hipStream_t s) {
    const size_t nnz = (size_t)A.nnz;
    const size_t a16 = 256;
    auto up = [&](size_t x) { return (x + a16 - 1) / a16 * a16; };
    size_t sort_bytes = 0;
    hipError_t e = rocprim::radix_sort_pairs((void*)nullptr, sort_bytes, (const int*)nullptr, (int*)nullptr,
                                             (const int*)nullptr, (int*)nullptr, nnz, 0,
                                             32 - __builtin_clz((unsigned)(A.N > 1 ? A.N - 1 : 1)), s);
    if (e != hipSuccess) return e;
    const size_t need = 3 * up(nnz * 4 + 4) + up(sort_bytes);
    if (!tmp) {
        *tmp_bytes = need;
        return hipSuccess;
    }
    if (*tmp_bytes < need) return hipErrorInvalidValue;
    if (nnz == 0) return hipMemsetAsync(tptr, 0, sizeof(int) * ((size_t)A.N + 1), s);
    char* p = (char*)tmp;
    int* idx_in = (int*)p;
    p += up(nnz * 4 + 4);
    int* idx_out = (int*)p;
    p += up(nnz * 4 + 4);
    int* key_out = (int*)p;
    p += up(nnz * 4 + 4);
    const unsigned grid = (unsigned)((nnz + 255) / 256);
    hipLaunchKernelGGL(k_tr_iota, dim3(grid), dim3(256), 0, s, (int)nnz, idx_in);
    e = rocprim::radix_sort_pairs((void*)p, sort_bytes, A.col, key_out, (const int*)idx_in, idx_out, nnz, 0,
                                  32 - __builtin_clz((unsigned)(A.N > 1 ? A.N - 1 : 1)), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_tr_gather, dim3(grid), dim3(256), 0, s, A.M, (int)nnz, A.ptr, A.val, idx_out, tcol, tval);
    hipLaunchKernelGGL(k_tr_ptr, dim3(grid), dim3(256), 0, s, A.N, (int)nnz, key_out, tptr);
    return hipGetLastError();
}

}  // namespace mhs
