// Memory-pattern probe for the GRU backward's memory part (tools/layout_probe.py): 2560 workgroups of 512 threads
// (8 waves), each walking T = 20 steps of 64 rows x 256 units, loading 4 saved arrays per step with the backward's
// lane mapping (16-byte loads of 4 rows of one unit, a 3-slot ring of quads) and storing 5 arrays (dword, lane =
// row), in two layouts:
//   plain   [unit][M]                      (M = K*T*R columns, the current layout)
//   blocked [M/64][unit][64]               (a 64-row block's 256 units contiguous: 64 KiB per array per step)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <bool BLOCKED>
__global__ void __launch_bounds__(512, 1) probe(const float* __restrict__ in, float* __restrict__ out, long M, int R,
                                               int T, float* __restrict__ sink) {
  const int tid = threadIdx.x, lane = tid & 63, hi = lane >> 5, col = lane & 31;
  const int wave = tid >> 6;
  const int nb = R / 64;
  const int k = blockIdx.x / nb;
  const int r0 = (blockIdx.x - k * nb) * 64;
  const int ub = 32 * wave + 4 * hi;
  float acc = 0.0f;
  auto addr = [&](int arr, int unit, long c) -> long {   // element (unit, column c) of array arr
    if (BLOCKED) return (long)arr * 256 * M + ((c >> 6) * 256 + unit) * 64 + (c & 63);
    return ((long)arr * 256 + unit) * M + c;
  };
  for (int t = 0; t < T; ++t) {
    const long ctr = ((long)k * T + t) * R + r0;
    float4 ring[3][4];
    auto load_q = [&](int qi, float4 (&v)[4]) {
      const int h = qi >> 2, g4 = qi & 3;
      const int unit = ub + (col & 3) + 8 * g4;
      const long c = ctr + 32 * h + (col & 28);
#pragma unroll
      for (int a = 0; a < 4; ++a) v[a] = *reinterpret_cast<const float4*>(in + addr(a, unit, c));
    };
    load_q(0, ring[0]);
    load_q(1, ring[1]);
#pragma unroll
    for (int qi = 0; qi < 8; ++qi) {
      if (qi + 2 < 8) load_q(qi + 2, ring[(qi + 2) % 3]);
      float4(&v)[4] = ring[qi % 3];
      float s = 0.0f;
#pragma unroll
      for (int a = 0; a < 4; ++a) s += v[a].x + v[a].y + v[a].z + v[a].w;
      acc += s;
      const int h = qi >> 2, g4 = qi & 3;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int unit = ub + 8 * g4 + j;
        const long c = ctr + 32 * h + col;
        out[addr(0, unit, c)] = s;
        out[addr(1, unit, c)] = s + 1.0f;
      }
    }
    // the contraction phase's three cotangent stores
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int unit = ub + 8 * (q >> 2) + (q & 3);
        const long c = ctr + 32 * h + col;
        out[addr(2, unit, c)] = acc;
        out[addr(3, unit, c)] = acc;
        out[addr(4, unit, c)] = acc;
      }
    __builtin_amdgcn_s_barrier();
  }
  if (acc == 12345.0f) sink[0] = acc;
}

int main() {
  const int R = 32768, T = 20, K = 5;
  const long M = (long)K * T * R;
  float *in, *out, *sink;
  hipMalloc(&in, sizeof(float) * 4 * 256 * M);
  hipMalloc(&out, sizeof(float) * 5 * 256 * M);
  hipMalloc(&sink, 4);
  hipMemset(in, 0, sizeof(float) * 4 * 256 * M);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const double bytes = (4.0 + 5.0) * 256 * 4 * M;
  for (int rep = 0; rep < 2; ++rep)
    for (int blocked = 0; blocked < 2; ++blocked) {
      hipEventRecord(a);
      for (int it = 0; it < 3; ++it) {
        if (blocked) hipLaunchKernelGGL(probe<true>, dim3(K * R / 64), dim3(512), 0, 0, in, out, M, R, T, sink);
        else hipLaunchKernelGGL(probe<false>, dim3(K * R / 64), dim3(512), 0, 0, in, out, M, R, T, sink);
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      ms /= 3;
      printf("{\"layout\": \"%s\", \"ms\": %.3f, \"TB_per_s\": %.2f}\n", blocked ? "blocked" : "plain", ms,
             bytes / ms / 1e9);
    }
  return 0;
}
