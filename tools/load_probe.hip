// Load-path probe (round 5): a CU's rate for the backward memory part's loads (16 bytes per lane, eight 128-byte row
// segments of [unit][M] arrays per wave instruction) as a function of loads in flight per wave and cache policy.
//   hipcc -O3 --offload-arch=gfx950 tools/load_probe.hip -o /tmp/load_probe && /tmp/load_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
typedef float f4v __attribute__((ext_vector_type(4)));

// DEPTH blocks of 8 loads per lane issued before one wait; AUX: 0 default, 2 nt
template <int DEPTH, int AUX>
__global__ void __launch_bounds__(512, 1) k_load(const float* __restrict__ in, float* __restrict__ sink, long M, int iters,
                                                unsigned long long* cyc) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hi = lane >> 5, col = lane & 31;
  const long c0 = (long)blockIdx.x * iters * 64;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in), 0, -1, 0x00020000);
  f4v acc = {0.0f, 0.0f, 0.0f, 0.0f};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; it += DEPTH) {
    f4v v[DEPTH][8];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int h = j >> 2, g4 = j & 3;
        const int u = 32 * wave + 4 * hi + (col & 3) + 8 * g4;
        const long cb = c0 + 64L * (it + d);
        const unsigned vo = (unsigned)(((long)u * M + 32 * h + (col & 28)) * 4);
        v[d][j] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)vo, (int)(cb * 4), AUX));
      }
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += v[d][j];
  }
  __syncthreads();
  if (tid == 0) cyc[blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
  if (acc.x + acc.y + acc.z + acc.w == 1.2345e-30f) sink[tid] = acc.x;   // keeps the loads (never true)
}

template <int DEPTH, int AUX>
int run(const float* in, float* sink, long M, int iters, unsigned long long* cyc, int g) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL((k_load<DEPTH, AUX>), dim3(g), dim3(512), 0, 0, in, sink, M, iters, cyc);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  unsigned long long h[256];
  CHECK(hipMemcpy(h, cyc, g * 8, hipMemcpyDeviceToHost));
  double mc = 0;
  for (int i = 0; i < g; ++i) mc += (double)h[i] / g;
  const double bytes_wg = (double)iters * 64 * 256 * 4;
  printf("{\"depth_kb_per_wave\": %d, \"aux\": %d, \"workgroups\": %d, \"ms\": %.4f, \"GBps\": %.1f, "
         "\"B_per_clk_per_cu\": %.2f, \"cycles_per_wait\": %.0f}\n", 8 * DEPTH, AUX, g, best, bytes_wg * g / best / 1e6,
         bytes_wg / mc, mc / (iters / DEPTH));
  return 0;
}

int main() {
  const int iters = 192;
  const long M = 256L * iters * 64;
  float *in, *sink;
  unsigned long long* cyc;
  CHECK(hipMalloc(&in, 256L * M * 4));
  CHECK(hipMemset(in, 0, 256L * M * 4));
  CHECK(hipMalloc(&sink, 4096));
  CHECK(hipMalloc(&cyc, 256 * 8));
  for (int g : {8, 256}) {
    run<1, 0>(in, sink, M, iters, cyc, g);
    run<1, 2>(in, sink, M, iters, cyc, g);
    run<2, 0>(in, sink, M, iters, cyc, g);
    run<2, 2>(in, sink, M, iters, cyc, g);
    run<4, 2>(in, sink, M, iters, cyc, g);
  }
  return 0;
}
