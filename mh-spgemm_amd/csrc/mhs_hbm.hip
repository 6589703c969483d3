// mhs_hbm.hip -- measured HBM peak of the box (the 8 TB/s spec confirmed with a
// copy kernel, both figures reported beside every roofline fraction).
//
// Three streaming kernels over buffers far larger than the 256 MiB Infinity Cache, 16 bytes a
// lane (global_load/store_dwordx4), four independent 16-byte accesses in flight per lane per
// iteration, a grid of 16 blocks per CU walking the buffer in grid-stride order:
//   copy   dst[i] = src[i]         bytes = 2 x size (read + write)
//   read   xor of src (one store per block, so nothing is elided)   bytes = size
//   write  dst[i] = constant       bytes = size
// (copy and write each run with cached and with nontemporal stores: the better is reported)
// Each runs `iters` times back to back on a stream of its own between two hipEvents; the
// rate is bytes x iters / elapsed.  Not on the SpGEMM path: a diagnostic for bench.py.
#include "mhs_internal.hpp"
#include "../../include/mhspgemm.h"

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));  // 16 bytes: global_load/store_dwordx4
constexpr int HBM_T = 256;
constexpr int HBM_U = 4;  // 16-byte accesses a lane issues together

template <bool NT>
__global__ __launch_bounds__(HBM_T) void k_hbm_copy(const v4i* __restrict__ src, v4i* __restrict__ dst, long long n) {
    const long long stride = (long long)gridDim.x * HBM_T;
    long long i = (long long)blockIdx.x * HBM_T + threadIdx.x;
    for (; i + (HBM_U - 1) * stride < n; i += HBM_U * stride) {
        v4i v[HBM_U];
#pragma unroll
        for (int u = 0; u < HBM_U; ++u) v[u] = NT ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
        for (int u = 0; u < HBM_U; ++u) {
            if (NT) __builtin_nontemporal_store(v[u], dst + i + u * stride);
            else dst[i + u * stride] = v[u];
        }
    }
    for (; i < n; i += stride) dst[i] = src[i];
}

__global__ __launch_bounds__(HBM_T) void k_hbm_read(const v4i* __restrict__ src, long long n, int* __restrict__ out) {
    const long long stride = (long long)gridDim.x * HBM_T;
    long long i = (long long)blockIdx.x * HBM_T + threadIdx.x;
    int acc = 0;
    for (; i + (HBM_U - 1) * stride < n; i += HBM_U * stride) {
        v4i v[HBM_U];
#pragma unroll
        for (int u = 0; u < HBM_U; ++u) v[u] = __builtin_nontemporal_load(src + i + u * stride);
#pragma unroll
        for (int u = 0; u < HBM_U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < n; i += stride) acc ^= src[i].x;
    if (acc == 0x7FFFFFFF) out[blockIdx.x] = acc;  // (data-dependent: the loads cannot be dropped)
}

template <bool NT>
__global__ __launch_bounds__(HBM_T) void k_hbm_write(v4i* __restrict__ dst, long long n, int seed) {
    const long long stride = (long long)gridDim.x * HBM_T;
    const v4i v = v4i{seed, seed + 1, seed + 2, seed + 3};
    for (long long i = (long long)blockIdx.x * HBM_T + threadIdx.x; i < n; i += stride) {
        if (NT) __builtin_nontemporal_store(v, dst + i);
        else dst[i] = v;
    }
}

}  // namespace

extern "C" int mhs_hbm_peak(mhs_ctx* ctx, size_t bytes, int iters, double* gbps) {
    (void)ctx;
    if (!gbps || iters <= 0 || bytes < (1u << 20)) return MHS_ERR_INVALID;
    bytes &= ~(size_t)15;
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return MHS_ERR_HIP;
    const int grid = prop.multiProcessorCount * 16;
    const long long n = (long long)(bytes / 16);
    v4i *a = nullptr, *b = nullptr;
    int* sink = nullptr;
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = MHS_OK;
    hipError_t e = hipMalloc((void**)&a, bytes);
    if (e == hipSuccess) e = hipMalloc((void**)&b, bytes);
    if (e == hipSuccess) e = hipMalloc((void**)&sink, (size_t)grid * 4);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    if (e == hipSuccess) e = hipMemsetAsync(a, 1, bytes, s);
    // copy and write each with cached and with nontemporal stores; the better of the two is
    // reported (the best rate a plain streaming kernel reaches on this box)
    double best[3] = {0.0, 0.0, 0.0};
    for (int k = 0; k < 5 && e == hipSuccess; ++k) {
        auto launch = [&]() {
            switch (k) {
            case 0: hipLaunchKernelGGL(k_hbm_copy<true>, dim3(grid), dim3(HBM_T), 0, s, a, b, n); break;
            case 1: hipLaunchKernelGGL(k_hbm_copy<false>, dim3(grid), dim3(HBM_T), 0, s, a, b, n); break;
            case 2: hipLaunchKernelGGL(k_hbm_read, dim3(grid), dim3(HBM_T), 0, s, a, n, sink); break;
            case 3: hipLaunchKernelGGL(k_hbm_write<true>, dim3(grid), dim3(HBM_T), 0, s, b, n, k); break;
            default: hipLaunchKernelGGL(k_hbm_write<false>, dim3(grid), dim3(HBM_T), 0, s, b, n, k); break;
            }
        };
        launch();  // warm-up
        e = hipEventRecord(e0, s);
        for (int it = 0; it < iters && e == hipSuccess; ++it) launch();
        if (e == hipSuccess) e = hipEventRecord(e1, s);
        if (e == hipSuccess) e = hipEventSynchronize(e1);
        float ms = 0.f;
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
        const double moved = (double)bytes * (k < 2 ? 2.0 : 1.0) * iters;
        const int slot = k < 2 ? 0 : k == 2 ? 1 : 2;
        const double r = e == hipSuccess && ms > 0.f ? moved / (ms * 1e-3) / 1e9 : 0.0;
        if (r > best[slot]) best[slot] = r;
    }
    for (int k = 0; k < 3; ++k) gbps[k] = best[k];
    if (e != hipSuccess) rc = e == hipErrorOutOfMemory ? MHS_ERR_OOM : MHS_ERR_HIP;
    (void)hipGetLastError();
    if (s) (void)hipStreamSynchronize(s);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (s) (void)hipStreamDestroy(s);
    (void)hipFree(a);
    (void)hipFree(b);
    (void)hipFree(sink);
    return rc;
}
