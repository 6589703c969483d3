// LDS throughput microbenchmark (gfx950): cycles per wave-instruction of ds_add_f64 (atomic,
// distinct addresses per lane), a ds_read_b64 + v_add_f64 + ds_write_b64 read-modify-write,
// and ds_add_f64 with 4 lanes per address -- one CU-filling launch each, timed with events.
// build: /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o tools/micro/lds_atomics tools/micro/lds_atomics.hip
// (the binary is git-ignored; results: profiles/r03/micro_lds_atomics.txt)
#include <hip/hip_runtime.h>
#include <cstdio>
template <int MODE>
__global__ __launch_bounds__(256) void k(double* out, int iters) {
    __shared__ double acc[4096];
    for (int i = threadIdx.x; i < 4096; i += 256) acc[i] = 0.0;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double v = 1.0 + threadIdx.x;
    for (int it = 0; it < iters; ++it) {
        const int base = ((it * 7) & 15) * 256 + w * 64;
        if (MODE == 0) atomicAdd(&acc[base + lane], v);                 // distinct addresses
        else if (MODE == 1) acc[base + lane] += v;                      // plain RMW (one wave per slice)
        else if (MODE == 2) atomicAdd(&acc[base + (lane >> 2)], v);     // 4 lanes per address
        else atomicAdd(&acc[base + ((lane * 9) & 63)], v);              // distinct, scrambled banks
    }
    __syncthreads();
    double s = 0;
    for (int i = threadIdx.x; i < 4096; i += 256) s += acc[i];
    if (s == -1.0) out[blockIdx.x] = s;
}
int main() {
    double* out;
    hipMalloc(&out, 1 << 20);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int iters = 4096, blocks = 256 * 8;  // 8 blocks x 4 waves per CU: 8 waves per SIMD
    const char* names[] = {"ds_add_f64 distinct", "rmw read+add+write", "ds_add_f64 4 lanes/addr", "ds_add_f64 scrambled"};
    for (int m = 0; m < 4; ++m) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            if (m == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters);
            if (m == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters);
            if (m == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters);
            if (m == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, iters);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            // wave-instructions per CU: 32 waves x iters; cycles per CU at 2.4 GHz
            const double cyc = ms * 1e-3 * 2.4e9;
            if (rep) printf("%-26s %8.3f ms  %6.2f CU-cycles per wave-instruction\n", names[m], ms, cyc / (32.0 * iters));
        }
    }
    return 0;
}
