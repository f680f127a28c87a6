// Load-path probe 2 (round 5): a CU's load rate vs how many rows (cache lines) one wave instruction touches.  Every
// instruction moves 1 KB (16 bytes per lane) as R rows x (1 KB / R) contiguous bytes of rows far apart (the [unit][M]
// arrays of the GRU kernels); 8 instructions per wave between waits (8 KB per wave in flight).  Every byte is read
// once (a 1 GB footprint: row stride = 256 workgroups x iters x the bytes a workgroup reads per row), so the loads come
// from HBM.
//   hipcc -O3 --offload-arch=gfx950 tools/load_probe2.hip -o /tmp/load_probe2 && /tmp/load_probe2
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
typedef float f4v __attribute__((ext_vector_type(4)));

// LOG2R: rows per instruction = 2^LOG2R (lane l: row l >> (6 - LOG2R), 16-byte piece l & (2^(6-LOG2R) - 1))
template <int LOG2R>
__global__ void __launch_bounds__(512, 1) k_load(const float* __restrict__ in, float* __restrict__ sink, long M,
                                                int iters, unsigned long long* cyc) {
  constexpr int R = 1 << LOG2R, PPR = 64 / R;   // rows per instruction, 16-byte pieces per row
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = lane / PPR, piece = lane % PPR;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in), 0, -1, 0x00020000);
  // per iteration a wave covers 8 instructions x R rows x (PPR * 16) bytes; columns advance by PPR * 4 per iteration
  const long c0 = (long)blockIdx.x * iters * PPR * 4;
  f4v acc = {0.0f, 0.0f, 0.0f, 0.0f};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    f4v v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int u = (wave * 8 + j) * R + row;   // up to 64 * R rows
      const unsigned vo = (unsigned)(((long)u * M + 4 * piece) * 4);
      v[j] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)vo, (int)((c0 + (long)it * PPR * 4) * 4), 0));
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += v[j];
  }
  __syncthreads();
  if (tid == 0) cyc[blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
  if (acc.x + acc.y + acc.z + acc.w == 1.2345e-30f) sink[tid] = acc.x;   // keeps the loads (never true)
}

template <int LOG2R>
int run(const float* in, float* sink, long M, int iters, unsigned long long* cyc, int g) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(k_load<LOG2R>, dim3(g), dim3(512), 0, 0, in, sink, M, iters, cyc);
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
  const double bytes_wg = (double)iters * 8 * 8 * 1024;
  printf("{\"rows_per_instr\": %d, \"bytes_per_row\": %d, \"workgroups\": %d, \"ms\": %.4f, \"GBps\": %.1f, "
         "\"B_per_clk_per_cu\": %.2f}\n", 1 << LOG2R, 1024 >> LOG2R, g, best, bytes_wg * g / best / 1e6, bytes_wg / mc);
  return 0;
}

int main() {
  const int iters = 64;
  float *in, *sink;
  unsigned long long* cyc;
  CHECK(hipMalloc(&in, (1L << 30) + (1L << 20)));   // 64 x R rows x (256 x iters x 1024 / R bytes) = 1 GB for every R
  CHECK(hipMemset(in, 0, (1L << 30) + (1L << 20)));
  CHECK(hipMalloc(&sink, 4096));
  CHECK(hipMalloc(&cyc, 256 * 8));
  // row stride in floats: 256 workgroups x iters x (PPR x 4 floats) per row
  auto ms = [&](int log2r) { return 256L * iters * (64 >> log2r) * 4; };
  for (int g : {8, 256}) {
    run<0>(in, sink, ms(0), iters, cyc, g);
    run<2>(in, sink, ms(2), iters, cyc, g);
    run<3>(in, sink, ms(3), iters, cyc, g);
    run<4>(in, sink, ms(4), iters, cyc, g);
    run<6>(in, sink, ms(6), iters, cyc, g);
  }
  return 0;
}
