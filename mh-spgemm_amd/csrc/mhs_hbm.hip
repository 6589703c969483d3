// mhs_hbm.hip -- measured HBM peak of the box (the 8 TB/s spec confirmed with a
// copy kernel, both figures reported beside every roofline fraction).
//
// Streaming kernels over buffers far larger than the 256 MiB Infinity Cache, 16 bytes a lane
// (global_load/store_dwordx4):
//   copy   dst[i] = src[i]         bytes = 2 x size (read + write)
//   read   xor of src (one store per block, so nothing is elided)   bytes = size
//   write  dst[i] = constant       bytes = size
// Every kernel runs in several shapes -- grid-stride or one contiguous slab per block, 2 to 16
// 16-byte accesses in flight per lane, 2 to 32 blocks per CU, cached or nontemporal; and the
// runtime's own D2D hipMemcpy / hipMemset blits -- and the best rate of each kind is reported (round 5: the round-4 single shape, grid-stride x4 at 16
// blocks per CU, read 4.7 TB/s copy where the microarchitecture guide measures 6.3).
// Each shape runs `iters` times back to back on a stream of its own between two hipEvents; the
// rate is bytes x iters / elapsed.  Not on the SpGEMM path: a diagnostic for bench.py
// (entry point mhs_hbm_peak in mhs_api.cpp).
#include "mhs_internal.hpp"

#include <cstdio>
#include <cstdlib>

namespace mhs {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));  // 16 bytes: global_load/store_dwordx4
constexpr int HBM_T = 256;

template <bool NT>
__device__ __forceinline__ v4i ld(const v4i* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(v4i* p, v4i v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// Block b owns [b*per, (b+1)*per) (SLAB) or every grid-stride U-group (!SLAB); a lane issues U
// loads, then U stores.
template <bool NT, int U, bool SLAB, int STNT = -1>  // STNT: stores' nontemporal flag (-1: as NT)
__global__ __launch_bounds__(HBM_T) void k_hbm_copy(const v4i* __restrict__ src, v4i* __restrict__ dst, long long n) {
    constexpr bool SNT = STNT < 0 ? NT : STNT != 0;
    long long i, end, stride;
    if (SLAB) {
        const long long per = (n + gridDim.x - 1) / gridDim.x;
        i = (long long)blockIdx.x * per + threadIdx.x;
        end = min(n, (long long)(blockIdx.x + 1) * per);
        stride = HBM_T;
    } else {
        i = (long long)blockIdx.x * HBM_T + threadIdx.x;
        end = n;
        stride = (long long)gridDim.x * HBM_T;
    }
    for (; i + (U - 1) * stride < end; i += U * stride) {
        v4i v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ld<NT>(src + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) st<SNT>(dst + i + u * stride, v[u]);
    }
    for (; i < end; i += stride) dst[i] = src[i];
}

template <int U, bool SLAB>
__global__ __launch_bounds__(HBM_T) void k_hbm_read(const v4i* __restrict__ src, long long n, int* __restrict__ out) {
    long long i, end, stride;
    if (SLAB) {
        const long long per = (n + gridDim.x - 1) / gridDim.x;
        i = (long long)blockIdx.x * per + threadIdx.x;
        end = min(n, (long long)(blockIdx.x + 1) * per);
        stride = HBM_T;
    } else {
        i = (long long)blockIdx.x * HBM_T + threadIdx.x;
        end = n;
        stride = (long long)gridDim.x * HBM_T;
    }
    int acc = 0;
    for (; i + (U - 1) * stride < end; i += U * stride) {
        v4i v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(src + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < end; i += stride) acc ^= src[i].x;
    if (acc == 0x7FFFFFFF) out[blockIdx.x] = acc;  // (data-dependent: the loads cannot be dropped)
}

template <bool NT, int U = 1, bool SLAB = false>
__global__ __launch_bounds__(HBM_T) void k_hbm_write(v4i* __restrict__ dst, long long n, int seed) {
    long long i, end, stride;
    if (SLAB) {
        const long long per = (n + gridDim.x - 1) / gridDim.x;
        i = (long long)blockIdx.x * per + threadIdx.x;
        end = min(n, (long long)(blockIdx.x + 1) * per);
        stride = HBM_T;
    } else {
        i = (long long)blockIdx.x * HBM_T + threadIdx.x;
        end = n;
        stride = (long long)gridDim.x * HBM_T;
    }
    const v4i v = v4i{seed, seed + 1, seed + 2, seed + 3};
    for (; i + (U - 1) * stride < end; i += U * stride) {
#pragma unroll
        for (int u = 0; u < U; ++u) st<NT>(dst + i + u * stride, v);
    }
    for (; i < end; i += stride) st<NT>(dst + i, v);
}

struct Shape {
    int kind;  // 0 copy, 1 read, 2 write
    int per_cu;
    void (*launch)(int grid, hipStream_t s, v4i* a, v4i* b, long long n, int* sink);
};

template <bool NT, int U, bool SLAB, int STNT = -1>
void l_copy(int g, hipStream_t s, v4i* a, v4i* b, long long n, int*) {
    hipLaunchKernelGGL((k_hbm_copy<NT, U, SLAB, STNT>), dim3(g), dim3(HBM_T), 0, s, a, b, n);
}
template <int U, bool SLAB>
void l_read(int g, hipStream_t s, v4i* a, v4i*, long long n, int* sink) {
    hipLaunchKernelGGL((k_hbm_read<U, SLAB>), dim3(g), dim3(HBM_T), 0, s, a, n, sink);
}
template <bool NT, int U = 1, bool SLAB = false>
void l_write(int g, hipStream_t s, v4i*, v4i* b, long long n, int*) {
    hipLaunchKernelGGL((k_hbm_write<NT, U, SLAB>), dim3(g), dim3(HBM_T), 0, s, b, n, 7);
}
// the runtime's own blit kernels, for comparison (labelled in the shape list)
void l_blit_copy(int, hipStream_t s, v4i* a, v4i* b, long long n, int*) {
    (void)hipMemcpyAsync(b, a, (size_t)n * 16, hipMemcpyDeviceToDevice, s);
}
void l_blit_fill(int, hipStream_t s, v4i*, v4i* b, long long n, int*) { (void)hipMemsetAsync(b, 3, (size_t)n * 16, s); }

const Shape kShapes[] = {
    {0, 16, l_copy<true, 4, false>},  {0, 16, l_copy<false, 4, false>}, {0, 8, l_copy<true, 8, false>},
    {0, 8, l_copy<false, 8, false>},  {0, 4, l_copy<true, 8, true>},    {0, 8, l_copy<true, 8, true>},
    {0, 8, l_copy<false, 8, true>},   {0, 16, l_copy<true, 4, true>},   {0, 4, l_copy<true, 16, false>},
    {0, 2, l_copy<true, 16, true>},   {0, 32, l_copy<true, 2, false>},  {0, 32, l_copy<false, 2, false>},
    {1, 16, l_read<4, false>},        {1, 8, l_read<8, false>},         {1, 8, l_read<8, true>},
    {2, 16, l_write<true>},           {2, 16, l_write<false>},          {2, 4, l_write<true>},
    {2, 32, l_write<false>},          {2, 8, l_write<true, 4>},         {2, 2, l_write<true, 4>},
    {2, 4, l_write<false, 4>},        {0, 1, l_blit_copy},              {2, 1, l_blit_fill},
    // slabs for the writes and fewer, longer-lived blocks for the copies (round 5: the write
    // side held the copy at ~5.5 TB/s where the runtime's fill reached 6.5)
    {2, 1, l_write<true, 4, true>},   {2, 2, l_write<true, 4, true>},   {2, 4, l_write<false, 4, true>},
    {2, 8, l_write<true, 8, true>},   {0, 1, l_copy<true, 8, true>},    {0, 2, l_copy<true, 8, true>},
    {0, 2, l_copy<false, 8, true>},   {0, 1, l_copy<true, 16, true>},   {0, 4, l_copy<false, 16, true>},
    {0, 16, l_copy<true, 4, true, 0>}, {0, 8, l_copy<true, 4, true, 0>}, {0, 4, l_copy<true, 8, true, 0>},
    {0, 16, l_copy<false, 4, true, 1>}, {0, 32, l_copy<true, 2, true>}, {0, 16, l_copy<true, 2, true>},
};

}  // namespace

hipError_t hbm_peak_run(size_t bytes, int iters, double* gbps) {
    bytes &= ~(size_t)15;
    int dev = 0;
    hipDeviceProp_t prop;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipGetDeviceProperties(&prop, dev);
    if (e != hipSuccess) return e;
    const int cus = prop.multiProcessorCount;
    const long long n = (long long)(bytes / 16);
    v4i *a = nullptr, *b = nullptr;
    int* sink = nullptr;
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    e = hipMalloc((void**)&a, bytes);
    if (e == hipSuccess) e = hipMalloc((void**)&b, bytes);
    if (e == hipSuccess) e = hipMalloc((void**)&sink, (size_t)cus * 16 * 4);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    if (e == hipSuccess) e = hipMemsetAsync(a, 1, bytes, s);
    if (e == hipSuccess) e = hipMemsetAsync(b, 2, bytes, s);
    double best[3] = {0.0, 0.0, 0.0};
    for (const Shape& sh : kShapes) {
        if (e != hipSuccess) break;
        const int grid = cus * sh.per_cu;
        sh.launch(grid, s, a, b, n, sink);  // warm-up
        e = hipEventRecord(e0, s);
        for (int it = 0; it < iters && e == hipSuccess; ++it) sh.launch(grid, s, a, b, n, sink);
        if (e == hipSuccess) e = hipGetLastError();
        if (e == hipSuccess) e = hipEventRecord(e1, s);
        if (e == hipSuccess) e = hipEventSynchronize(e1);
        float ms = 0.f;
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
        const double moved = (double)bytes * (sh.kind == 0 ? 2.0 : 1.0) * iters;
        const double r = e == hipSuccess && ms > 0.f ? moved / (ms * 1e-3) / 1e9 : 0.0;
        if (r > best[sh.kind]) best[sh.kind] = r;
        if (getenv("MHS_HBM_VERBOSE"))
            fprintf(stderr, "hbm shape %d (kind %d, %d blocks/CU): %.1f GB/s\n", (int)(&sh - kShapes), sh.kind,
                    sh.per_cu, r);
    }
    for (int k = 0; k < 3; ++k) gbps[k] = best[k];
    if (s) (void)hipStreamSynchronize(s);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (s) (void)hipStreamDestroy(s);
    (void)hipFree(a);
    (void)hipFree(b);
    (void)hipFree(sink);
    return e;
}

}  // namespace mhs
