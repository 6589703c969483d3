// Device property probe for the MI355X box (tools only; not part of the product path).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k_lds_add(double* out, int n) {
  extern __shared__ double acc[];
  for (int i = threadIdx.x; i < n; i += blockDim.x) acc[i] = 0.0;
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * n; i += blockDim.x) atomicAdd(&acc[i % n], 1.0);
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) out[i] = acc[i];
}
int main() {
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  printf("name=%s gcn=%s CUs=%d sharedPerBlock=%zu maxSharedPerMP=%zu sharedOptin=%zu warp=%d clock=%d memclk=%d busw=%d l2=%d regsPerBlock=%d maxThreadsPerMP=%d totalGlobalMem=%zu\n",
    p.name, p.gcnArchName, p.multiProcessorCount, p.sharedMemPerBlock, p.maxSharedMemoryPerMultiProcessor,
    p.sharedMemPerBlockOptin, p.warpSize, p.clockRate, p.memoryClockRate, p.memoryBusWidth, p.l2CacheSize,
    p.regsPerBlock, p.maxThreadsPerMultiProcessor, p.totalGlobalMem);
  double* d; hipMalloc(&d, 4096 * 8);
  hipError_t e = hipFuncSetAttribute((const void*)k_lds_add, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  printf("setattr 160K: %s\n", hipGetErrorString(e));
  hipLaunchKernelGGL(k_lds_add, dim3(1), dim3(256), 160 * 1024, 0, d, 4096);
  e = hipDeviceSynchronize();
  double h[4]; hipMemcpy(h, d, 32, hipMemcpyDeviceToHost);
  printf("lds add 160K launch: %s  out[0]=%g (expect 64)\n", hipGetErrorString(e), h[0]);
  return 0;
}
