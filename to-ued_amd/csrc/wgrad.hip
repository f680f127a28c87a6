// LPG weight-gradient reductions on CDNA4 matrix cores: C[ra x rb] = A[ra x K] . B[rb x K]^T with both
// operands K-contiguous and K = K_upd * T * R (3.28M at the C2 shape) -- a short-and-wide GEMM whose whole
// cost is the reduction over K.  Replaces the library GEMMs of the LPG backward (lpg.py: the gate-weight
// gradient [h_in; x; 1] . [dr; dz; dhn]^T, the input-gate gradient [x; 1] . dn^T and the head gradient
// DH . [relu(h_out); 1]^T).
//
// Layout: one workgroup per (128-column tile of B rows, K chunk).  It holds ALL ra rows of A (NRT tiles of
// 16 rows; ra <= 16 or ra <= 272) against its 128 B rows: every A k-slab is staged once through LDS (by
// LDS-DMA, double-buffered; two workgroups per CU cover each other's slab waits) and read by the eight
// waves (one 16-row B tile each), every B row streams from HBM exactly once per chunk.
// The f32 16x16x4 MFMA (v_mfma_f32_16x16x4_f32, exact f32 fma, 32 cycles/SIMD) runs with the k order
// permuted per lane: lane l (k-group g = l >> 4) covers k0 + 8g + e of a 32-k slab at step e, for A and B
// alike, so each lane's B operands are two contiguous 16-byte loads per slab (full 128-byte lines per row).
// Partial sums per K chunk go to a workspace and a second kernel adds them in chunk order: the result is
// deterministic (no atomics).
#include "common.h"

typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace {

TOUED_DEV floatx4 mfma16(float a, float b, floatx4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

TOUED_DEV float f4(const float4& v, int e) { return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w; }

template <int NRT>
__global__ void __launch_bounds__(512, 2) k_wgrad(const float* __restrict__ A, long lda, int ra,
                                                  const float* __restrict__ B, long ldb, int rb, long K, long kchunk,
                                                  float* __restrict__ part) {
  constexpr int RA = NRT * 16;               // A rows held (zero-padded past ra)
  __shared__ float4 As[2][RA * 8];           // [buffer][row][8 float4 = one 32-k slab]
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, c16 = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ct = blockIdx.x, sc = blockIdx.y;
  const long kb = (long)sc * kchunk;
  const long ke = kb + kchunk < K ? kb + kchunk : K;
  const int nslab = (int)((ke - kb) / 32);
  const int brow = ct * 128 + wave * 16 + c16;
  const bool bok = brow < rb;
  const float4* Bp = reinterpret_cast<const float4*>(B + (long)(bok ? brow : 0) * ldb + kb) + 2 * g;
  // A slab s -> LDS buffer by LDS-DMA (global_load_lds_dwordx4): one wave instruction moves 8 rows x 128 B
  // into the lane-linear [row][8 float4] image.  Rows past ra read row ra-1 instead: they only feed C rows
  // that are never written out.
  auto stage_a = [&](int s, int buf) {
    for (int j = wave; j < RA / 8; j += 8) {
      int row = 8 * j + (lane >> 3);
      row = row < ra ? row : ra - 1;
      const float* src = A + (long)row * lda + kb + 32L * s + 4 * (lane & 7);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(As[buf] + 64 * j), 16, 0, 0);
    }
  };
  floatx4 acc[NRT];
#pragma unroll
  for (int i = 0; i < NRT; ++i) acc[i] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
  if (nslab > 0) stage_a(0, 0);
  float4 b0 = Bp[0], b1 = Bp[1];
  __syncthreads();
  for (int s = 0; s < nslab; ++s) {
    const int buf = s & 1;
    const int sn = s + 1 < nslab ? s + 1 : s;
    stage_a(sn, buf ^ 1);
    const float4 nb0 = Bp[8 * sn], nb1 = Bp[8 * sn + 1];
    // A operand of row tile i at step e: A[16i + c16][k0 + 8g + e] (two ds_read_b128 per tile and slab).
    // Tiles go in pairs (consecutive MFMAs never wait on each other's accumulator) and the next pair's
    // LDS reads are issued before the current pair's MFMAs.
    const float4* al = As[buf] + c16 * 8 + 2 * g;
    float4 x0 = al[0], x1 = al[1], y0 = al[128], y1 = al[129];
#pragma unroll
    for (int i = 0; i < NRT; i += 2) {
      const float4 cx0 = x0, cx1 = x1, cy0 = y0, cy1 = y1;
      if (i + 2 < NRT) { x0 = al[(i + 2) * 128]; x1 = al[(i + 2) * 128 + 1]; }
      if (i + 3 < NRT) { y0 = al[(i + 3) * 128]; y1 = al[(i + 3) * 128 + 1]; }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float bv = e < 4 ? f4(b0, e) : f4(b1, e - 4);
        acc[i] = mfma16(e < 4 ? f4(cx0, e) : f4(cx1, e - 4), bv, acc[i]);
        if (i + 1 < NRT) acc[i + 1] = mfma16(e < 4 ? f4(cy0, e) : f4(cy1, e - 4), bv, acc[i + 1]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    b0 = nb0; b1 = nb1;
    __syncthreads();   // drains the slab's LDS-DMA (vmcnt(0)) before the buffers swap
  }
  // D map: lane l, reg r -> C[16i + 4g + r][brow]
  const int rbp = gridDim.x * 128;
  float* out = part + (long)sc * RA * rbp;
#pragma unroll
  for (int i = 0; i < NRT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) out[(long)(16 * i + 4 * g + r) * rbp + brow] = acc[i][r];
}

// C[i][j] = sum over chunks (in chunk order) of part[s][i][j], i < ra, j < rb
__global__ void k_wgrad_reduce(const float* __restrict__ part, int S, int RA, int rbp, int ra, int rb,
                               float* __restrict__ C) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)ra * rb) return;
  const int i = (int)(idx / rb), j = (int)(idx - (long)i * rb);
  float s = 0.0f;
  for (int c = 0; c < S; ++c) s += part[((long)c * RA + i) * rbp + j];
  C[idx] = s;
}

struct Plan {
  int nrt, ncol, S;
  long kchunk;
};

static Plan plan(int ra, int rb, long K) {
  Plan p;
  p.nrt = ra <= 16 ? 1 : 17;
  p.ncol = (rb + 127) / 128;
  int cus = 256;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
    cus = 256;
  // NRT = 17: two workgroups per CU (125 VGPRs, 68 KB LDS each), as many K chunks as fill them in one
  // round.  NRT = 1 is a bandwidth-bound stream over B: four workgroups per CU keep enough loads in flight.
  int S = (p.nrt == 1 ? 4 : 2) * cus / p.ncol;
  if (S < 1) S = 1;
  long slabs = K / 32;
  if (S > slabs) S = (int)(slabs > 0 ? slabs : 1);
  p.kchunk = ((slabs + S - 1) / S) * 32;
  p.S = (int)((K + p.kchunk - 1) / p.kchunk);
  if (p.S < 1) p.S = 1;
  return p;
}

}  // namespace

extern "C" {

size_t toued_wgrad_workspace_floats(int ra, int rb, long K) {
  if (ra <= 0 || rb <= 0 || K <= 0) return 0;
  const Plan p = plan(ra, rb, K);
  return (size_t)p.S * p.nrt * 16 * p.ncol * 128;
}

int toued_wgrad(int ra, int rb, long K, const float* A, long lda, const float* B, long ldb, float* C, float* work,
                size_t work_floats, hipStream_t stream) {
  TOUED_REQUIRE(ra >= 1 && ra <= 272 && rb >= 1 && K >= 0, "toued_wgrad: ra=%d (1..272) rb=%d K=%ld", ra, rb, K);
  TOUED_REQUIRE(K % 32 == 0, "toued_wgrad: K=%ld must be a multiple of 32", K);
  TOUED_REQUIRE(lda % 4 == 0 && ldb % 4 == 0, "toued_wgrad: lda=%ld ldb=%ld must be multiples of 4 (16-byte rows)",
                lda, ldb);
  TOUED_REQUIRE(A && B && C, "toued_wgrad: null operand");
  if (K == 0) {
    TOUED_REQUIRE(hipMemsetAsync(C, 0, sizeof(float) * ra * rb, stream) == hipSuccess, "toued_wgrad: memset failed");
    return 0;
  }
  const Plan p = plan(ra, rb, K);
  const size_t need = (size_t)p.S * p.nrt * 16 * p.ncol * 128;
  TOUED_REQUIRE(work && work_floats >= need, "toued_wgrad: workspace of %zu floats needed (got %zu)", need, work_floats);
  const dim3 grid(p.ncol, p.S);
  if (p.nrt == 1)
    hipLaunchKernelGGL(k_wgrad<1>, grid, dim3(512), 0, stream, A, lda, ra, B, ldb, rb, K, p.kchunk, work);
  else
    hipLaunchKernelGGL(k_wgrad<17>, grid, dim3(512), 0, stream, A, lda, ra, B, ldb, rb, K, p.kchunk, work);
  const long n = (long)ra * rb;
  hipLaunchKernelGGL(k_wgrad_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, work, p.S, p.nrt * 16,
                     p.ncol * 128, ra, rb, C);
  TOUED_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
