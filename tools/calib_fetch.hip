// FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access widths the GRU kernels use.
// Streams exactly 1 GiB through 4-byte-per-lane loads (the buffer_load_b32 pattern of the saved
// activations) and through 16-byte-per-lane loads, and writes 1 GiB with 4-byte-per-lane stores;
// run under `rocprofv3 --pmc FETCH_SIZE` (and WRITE_SIZE) to get the counter-to-bytes factor.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void rd_b32(const float* __restrict__ x, float* __restrict__ out, size_t n) {
  float s = 0.0f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += x[i];
  if (s == 1234.5f) out[0] = s;
}

__global__ void rd_b128(const float4* __restrict__ x, float* __restrict__ out, size_t n4) {
  float s = 0.0f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = x[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 1234.5f) out[0] = s;
}

__global__ void wr_b32(float* __restrict__ y, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) y[i] = 1.0f;
}

int main() {
  const size_t bytes = 1ull << 30, n = bytes / 4;
  float *x, *y, *o;
  if (hipMalloc(&x, bytes) != hipSuccess || hipMalloc(&y, bytes) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  hipMemset(x, 0, bytes);
  for (int r = 0; r < 2; ++r) {
    hipLaunchKernelGGL(rd_b32, dim3(8192), dim3(256), 0, 0, x, o, n);
    hipLaunchKernelGGL(rd_b128, dim3(8192), dim3(256), 0, 0, reinterpret_cast<const float4*>(x), o, n / 4);
    hipLaunchKernelGGL(wr_b32, dim3(8192), dim3(256), 0, 0, y, n);
  }
  hipDeviceSynchronize();
  printf("calib done: %zu bytes per kernel\n", bytes);
  hipFree(x);
  hipFree(y);
  hipFree(o);
  return 0;
}
