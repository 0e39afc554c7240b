// Probe: the largest dynamic LDS allocation one workgroup may use on this device.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void touch(float *out, int n) {
  extern __shared__ float lds[];
  for (int i = threadIdx.x; i < n; i += blockDim.x) lds[i] = (float)i;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = lds[n - 1];
}
int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  printf("sharedMemPerBlock %zu maxSharedMemoryPerMultiProcessor %zu sharedMemPerBlockOptin %zu\n", p.sharedMemPerBlock,
         p.maxSharedMemoryPerMultiProcessor, p.sharedMemPerBlockOptin);
  float *o;
  hipMalloc(&o, 1024 * 4);
  for (size_t kb : {64, 96, 128, 158, 160}) {
    const size_t bytes = kb * 1024;
    hipError_t a = hipFuncSetAttribute((const void *)touch, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    hipLaunchKernelGGL(touch, dim3(256), dim3(768), bytes, 0, o, (int)(bytes / 4));
    hipError_t e = hipGetLastError();
    hipError_t s = hipDeviceSynchronize();
    float v = 0;
    hipMemcpy(&v, o, 4, hipMemcpyDeviceToHost);
    printf("%zu KB: setattr %d launch %d sync %d value %.0f (want %zu)\n", kb, (int)a, (int)e, (int)s, v, bytes / 4 - 1);
  }
  return 0;
}
