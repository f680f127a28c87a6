// LPG weight-gradient reductions on CDNA4 matrix cores: C[ra x rb] = A[ra x K] . B[rb x K]^T with both
// operands K-contiguous and K = K_upd * T * R (3.28M at the C2 shape) -- a short-and-wide GEMM whose whole
// cost is the reduction over K.  Replaces the library GEMMs of the LPG backward (lpg.py: the gate-weight
// gradient [h_in; x; 1] . [dr; dz; dhn]^T, the input-gate gradient [x; 1] . dn^T and the head gradient
// DH . [relu(h_out); 1]^T).
//
// Main reduction (ra <= 272, k_wgrad_x6): f32-accurate products on the bf16 matrix cores.  Every f32
// operand is split exactly into three bf16 pieces, x = x0 + x1 + x2 (round-to-nearest at each stage; the
// three 8-bit significands cover f32's 24), and a.b is formed from the six piece products whose weight is
// at least 2^-16 of a0.b0: a0b0 + a0b1 + a1b0 + a0b2 + a1b1 + a2b0.  Every piece product is exact and the
// MFMA accumulates in f32; the three dropped products are below 2^-24 relative, so the result carries the
// error of an f32 GEMM (same test bound as the f32-MFMA kernel) at 6 x 16 = 96 bf16-MFMA cycles per
// 32x16x16 block instead of the f32 MFMA's 256.
// One 512-thread workgroup per (256 B rows, K chunk), one per CU: it stages each 32-k slab of ALL ra
// A rows through LDS once (loaded as f32, split, written as three bf16 images, double-buffered, XOR-swizzled
// for conflict-free 16-byte fragment reads) and each wave streams its own 32 B rows from HBM (split in
// registers), so B is read exactly once per chunk.  v_mfma_f32_16x16x32_bf16, 17 A tiles x 2 B tiles of
// accumulators per wave.
//
// Small reductions (ra <= 16, k_wgrad<1>): HBM-bound streams over B on the f32 16x16x4 MFMA, with the k
// order permuted per lane (lane l, k-group g = l >> 4, covers k0 + 8g + e of a 32-k slab at step e) so each
// lane's operands are two contiguous 16-byte loads per slab.  (k_wgrad<17> is the former f32 main kernel,
// kept for comparison: TOUED_WGRAD_F32=1.)
// Partial sums per K chunk go to a workspace and a second kernel adds them in chunk order: the result is
// deterministic (no atomics).
#include <stdlib.h>
#include "common.h"

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));


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

// ------------------------------------------------------------------ f32-accurate bf16 split kernel
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int X6_RA = 272;          // A rows held (17 tiles of 16, zero-padded past ra)
constexpr int X6_NW = 4;            // waves per workgroup: one per SIMD (512-register budget)
constexpr int X6_BT = 3;            // B tiles of 16 rows per wave
constexpr int X6_CT = 16 * X6_BT * X6_NW;   // B rows per workgroup (192)
constexpr int X6_AQ = X6_RA * 8;    // float4 per 32-k A slab (2176)
constexpr int X6_NS = (X6_AQ + 64 * X6_NW - 1) / (64 * X6_NW);   // staging rounds per thread (9)

TOUED_DEV floatx4 mfma_bf(bf16x8 a, bf16x8 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// element e of the three pieces: x = p0 + p1 + p2 exactly (each stage rounds to nearest; the residual
// subtractions are exact)
template <typename V>
TOUED_DEV void split3_bf16(float x, V& p0, V& p1, V& p2, int e) {
  const __bf16 h = (__bf16)x;
  const float r1 = x - (float)h;
  const __bf16 m = (__bf16)r1;
  p0[e] = h;
  p1[e] = m;
  p2[e] = (__bf16)(r1 - (float)m);
}

// LDS image of one 32-k A slab piece: [row][4 k-octets of 8 bf16], octet o of row r at slot o ^ f((r >> 2) & 3)
// with f = (0, 2, 3, 1).  A fragment read (lane l: row 16i + (l & 15), octet l >> 4) is a ds_read_b128, which
// gfx950 serves in the lane groups {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} (+32): each group holds rows
// {0-3, 12-15} of one octet and rows {4-11} of the other, and f sends those 16 (row, octet) pairs to 16 distinct
// bank quads (the former o ^ ((r >> 2) & 3) paired rows 0/4 and 12/8 on one quad: 2-way conflicts on every read).
// The staging writes (ds_write_b64, 16 contiguous lanes = two whole rows) stay conflict-free under any in-row
// permutation.
TOUED_DEV int x6_slot(int row, int oct) { return row * 4 + (oct ^ ((0x78 >> (2 * ((row >> 2) & 3))) & 3)); }

// Software pipeline per 32-k slab s (A image `buf` in LDS, B pieces bp in registers):
//   slab start: load the raw A slab s+1 (9 float4 per thread);
//   A tile i (i = 0..16): issue the LDS fragment reads of tile i+1, then the 18 MFMAs of tile i (3 B tiles x 6
//   piece products), interleaved one-for-one with the side work of that tile:
//     tiles 0-5:  split half a B tile of slab s+1 (raw loads issued during slab s-1) into bpn;
//     tile 6:     issue the raw B loads of slab s+2;
//     tiles 8-16: split one staging round of A slab s+1 into the idle LDS image.
//   barrier.  Loads run a slab ahead, LDS fragment reads a tile ahead, and every split hides under MFMAs.
__global__ void __launch_bounds__(64 * X6_NW, 1) k_wgrad_x6(const float* __restrict__ A, long lda, int ra,
                                                             const float* __restrict__ B, long ldb, int rb, long K,
                                                             long kchunk, float* __restrict__ part) {
  constexpr int NT = 64 * X6_NW;
  // XCD-aware tile order: blocks b and b + 8 share an XCD (round-robin dealing), so block b takes linear slot
  // L = (first slot of its XCD's contiguous range) + b / 8 and the ncol column tiles of one K chunk (consecutive
  // L) run on one XCD, where they read each A slab through the same L2.
  const int G = gridDim.x, ncol = (rb + X6_CT - 1) / X6_CT;
  const int xcd = blockIdx.x & 7;
  const int L = xcd * (G >> 3) + (xcd < (G & 7) ? xcd : (G & 7)) + (blockIdx.x >> 3);
  static_assert(X6_NS == 9 && 2 * X6_BT <= 8, "schedule below: 9 staging rounds at tiles 8-16, B splits before");
  __shared__ bf16x8 As[2][3][X6_RA * 4];   // [buffer][piece][slot]: 104,448 B
  const int tid = threadIdx.x, lane = tid & 63, q16 = lane & 15, oct = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ct = L % ncol, sc = L / ncol;
  const long kb = (long)sc * kchunk;
  const long ke = kb + kchunk < K ? kb + kchunk : K;
  const int nslab = (int)((ke - kb) / 32);
  // this lane's B rows (tiles t): fragment = B[row][k0 + 8 oct .. +7] = two float4
  const float4* Bp[X6_BT];
  int brow[X6_BT];
#pragma unroll
  for (int t = 0; t < X6_BT; ++t) {
    brow[t] = ct * X6_CT + 16 * (X6_BT * wave + t) + q16;
    Bp[t] = reinterpret_cast<const float4*>(B + (long)(brow[t] < rb ? brow[t] : 0) * ldb + kb) + 2 * oct;
  }
  // A staging: float4 i = tid + NT j (row i >> 3, k-quad i & 7) of the slab.  The last round covers only part
  // of the slab: the other threads repeat the element of their previous round (same address, same data) so
  // that every load and LDS write is unconditional (no exec branch, no vmcnt(0) inside the loop).  Rows past
  // ra repeat row ra-1: they only feed C rows that are never written out.
  float4 ast[X6_NS];
  auto a_index = [&](int j) {
    const int i = tid + NT * j;
    return j < X6_NS - 1 || i < X6_AQ ? i : i - NT;
  };
  auto load_a = [&](int s) {
#pragma unroll
    for (int j = 0; j < X6_NS; ++j) {
      const int i = a_index(j);
      const int row = (i >> 3) < ra ? (i >> 3) : ra - 1;
      ast[j] = *reinterpret_cast<const float4*>(A + (long)row * lda + kb + 32L * s + 4 * (i & 7));
    }
  };
  auto write_a = [&](int buf, int j) {
    const int i = a_index(j);
    const int row = i >> 3, kq = i & 7;
    const int slot = x6_slot(row, kq >> 1);
    bf16x4 p[3];
#pragma unroll
    for (int e = 0; e < 4; ++e) split3_bf16(f4(ast[j], e), p[0], p[1], p[2], e);
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) reinterpret_cast<bf16x4*>(&As[buf][pc][slot])[kq & 1] = p[pc];
  };
  float4 bq[X6_BT][2];
  auto issue_b = [&](int s) {
#pragma unroll
    for (int t = 0; t < X6_BT; ++t) { bq[t][0] = Bp[t][8 * s]; bq[t][1] = Bp[t][8 * s + 1]; }
  };
  auto split_b = [&](bf16x8 (&dst)[X6_BT][3], int t, int half) {
#pragma unroll
    for (int e = 0; e < 4; ++e) split3_bf16(f4(bq[t][half], e), dst[t][0], dst[t][1], dst[t][2], 4 * half + e);
  };
  floatx4 acc[17][X6_BT];
#pragma unroll
  for (int i = 0; i < 17; ++i)
#pragma unroll
    for (int t = 0; t < X6_BT; ++t) acc[i][t] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};

  auto slab = [&](int s, bf16x8 (&bp)[X6_BT][3], bf16x8 (&bpn)[X6_BT][3]) {
    const int buf = s & 1;
    load_a(s + 1 < nslab ? s + 1 : s);
    const bf16x8* a0p = As[buf][0];
    const bf16x8* a1p = As[buf][1];
    const bf16x8* a2p = As[buf][2];
    bf16x8 a[3];
    {
      const int slot = x6_slot(q16, oct);
      a[0] = a0p[slot]; a[1] = a1p[slot]; a[2] = a2p[slot];
    }
#pragma unroll
    for (int i = 0; i < 17; ++i) {
      bf16x8 an[3];
      if (i + 1 < 17) {
        const int slot = x6_slot(16 * (i + 1) + q16, oct);
        an[0] = a0p[slot]; an[1] = a1p[slot]; an[2] = a2p[slot];
      }
#pragma unroll
      for (int t = 0; t < X6_BT; ++t) {
        floatx4 c = acc[i][t];
        c = mfma_bf(a[2], bp[t][0], c);
        c = mfma_bf(a[1], bp[t][1], c);
        c = mfma_bf(a[0], bp[t][2], c);
        c = mfma_bf(a[1], bp[t][0], c);
        c = mfma_bf(a[0], bp[t][1], c);
        c = mfma_bf(a[0], bp[t][0], c);
        acc[i][t] = c;
      }
      if (i < 2 * X6_BT) split_b(bpn, i >> 1, i & 1);
      if (i == 2 * X6_BT) issue_b(s + 2 < nslab ? s + 2 : nslab - 1);
      if (i >= 8) write_a(buf ^ 1, i - 8);
      if (i + 1 < 17) {
        __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);   // next tile's fragment reads first
      }
#pragma unroll
      for (int m = 0; m < 6 * X6_BT; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // one MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);   // one VALU of the side work
      }
      __builtin_amdgcn_sched_barrier(0);
      if (i + 1 < 17) { a[0] = an[0]; a[1] = an[1]; a[2] = an[2]; }
    }
    lds_barrier();
  };

  bf16x8 bpa[X6_BT][3], bpb[X6_BT][3];
  if (nslab > 0) {
    load_a(0);
    issue_b(0);
#pragma unroll
    for (int j = 0; j < X6_NS; ++j) write_a(0, j);
#pragma unroll
    for (int t = 0; t < X6_BT; ++t) { split_b(bpa, t, 0); split_b(bpa, t, 1); }
    issue_b(nslab > 1 ? 1 : 0);
  }
  __syncthreads();
  for (int s = 0; s < nslab; ++s) {
    slab(s, bpa, bpb);
#pragma unroll
    for (int t = 0; t < X6_BT; ++t)
#pragma unroll
      for (int pc = 0; pc < 3; ++pc) bpa[t][pc] = bpb[t][pc];   // (a two-slab unrolled swap spills)
  }
  // D map: lane l, reg r -> C[16i + 4 oct + r][brow]
  const int rbp = ncol * X6_CT;
  float* out = part + (long)sc * X6_RA * rbp;
#pragma unroll
  for (int t = 0; t < X6_BT; ++t)
#pragma unroll
    for (int i = 0; i < 17; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(long)(16 * i + 4 * oct + r) * rbp + brow[t]] = acc[i][t][r];
}

// ------------------------------------------------------------------ block-floating-point fp16-pair kernel
// k_wgrad_h3: the main reduction on scaled fp16 pairs, three products per element pair instead of six.  Every
// operand is scaled by a power of two so that its magnitude stays below 2^14 and split exactly into
// y = x0 + x1 (x0 = fp16(y), x1 = fp16(y - x0): 22 significand bits); a0b0 + a0b1 + a1b0 are exact products
// accumulated in f32, the dropped a1b1 is below 2^-22 relative.  Scales:
//   * A row i: 2^14 for the rows known to be bounded by 1 (the GRU carry h_in), else 2^(14 - e_i) from the
//     row's measured maximum |a| < 2^e_i (k_wgrad_rowmax; the x feature rows) -- rows 256.. of [h_in; x; 1];
//   * B (the gate cotangents, per column m of very different magnitude): the backward writes each column's
//     exponent t_m (2^t_m max_j |B[j][m]| < 2^14); a workgroup's K chunk uses c = min_m t_m over its columns,
//     so the chunk's largest column sits below 2^14 and a column 2^d smaller keeps 22 bits while d < 24 and an
//     absolute error below 2^-38 of the chunk maximum beyond -- f32-accumulation class.
// The partial sums are unscaled exactly (powers of two) before the chunk-ordered reduction.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

TOUED_DEV floatx4 mfma_h(f16x8 a, f16x8 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

template <typename V>
TOUED_DEV void split2_f16(float y, V& p0, V& p1, int e) {
  const _Float16 h = (_Float16)y;
  p0[e] = h;
  p1[e] = (_Float16)(y - (float)h);
}
// the same pieces of y = x * s (s a power of two: the product is exact) in two VALU instructions, each a
// v_fma_mixlo_f16: h = fp16(x s), l = fp16(fma(x, s, -h)) with h read back as f16 -- the f32 product, the f32 of h
// and the subtraction of the plain form cost three more, and beside one wave's MFMAs the VALU issue is the bound
template <typename V>
TOUED_DEV void split2_f16s(float x, float s, V& p0, V& p1, int e) {
  const _Float16 h = (_Float16)__builtin_fmaf(x, s, 0.0f);
  p0[e] = h;
  p1[e] = (_Float16)__builtin_fmaf(x, s, -(float)h);
}

// exponent e with 2^e > |x| >= 2^(e-1) (frexp), for the scale 2^(14 - e)
TOUED_DEV int scale_exp_of(float mx) {
  if (!(mx > 0.0f) || !(mx <= 3.0e38f)) return 0;
  int e;
  frexpf(mx, &e);
  return min(126, max(-126, 14 - e));
}

// bits[row - r0] = max over k of |A[row][k]| as float bits (non-negative floats order like ints)
__global__ void __launch_bounds__(256) k_wgrad_rowmax(const float* __restrict__ A, long lda, int r0, long K,
                                                      long kper, int* __restrict__ bits) {
  const int row = r0 + blockIdx.y;
  const long kb = (long)blockIdx.x * kper, ke = kb + kper < K ? kb + kper : K;
  const float* a = A + (long)row * lda;
  float m = 0.0f;
  for (long k = kb + threadIdx.x * 4; k < ke; k += 256 * 4) {
    const float4 v = *reinterpret_cast<const float4*>(a + k);
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(&bits[blockIdx.y], __float_as_int(m));
}

#ifdef WG_STAMPS
// timing instrumentation (tools/wgrad_stamps.py): lane 0 of each wave of workgroups < 64 records s_memtime at the
// start of each of the first 64 slabs, after tile 7, before and after the slab barrier
__device__ unsigned long long g_wg_stamps[64 * 8 * 64 * 4];
#define WG_STAMP(s, ph)                                                                                 \
  do {                                                                                                  \
    if (blockIdx.x < 64 && lane == 0 && (s) < 64)                                                       \
      g_wg_stamps[((blockIdx.x * 8 + wave) * 64 + (s)) * 4 + (ph)] = __builtin_amdgcn_s_memtime();      \
  } while (0)
#else
#define WG_STAMP(s, ph) do {} while (0)
#endif

#ifdef H3_PLACE
// placement instrumentation (tools/h3_place.py): per launch (ring of 64) and workgroup, the XCC the workgroup ran on,
// its HW_ID word, and its start and end times (s_memrealtime, 100 MHz)
__device__ unsigned long long g_h3_place[64 * 256 * 4];
__device__ unsigned int g_h3_launch;
#endif

// cache policy of the streamed B loads (buffer aux bits; 2 = nt): B is read once, A (each slab read by the chunk's
// column tiles, ideally from L2) is what should stay in L2
#ifndef H3_B_AUX
#define H3_B_AUX 0
#endif
#ifndef H3_BR2
#define H3_BR2 1
#endif
// NW waves per workgroup, BT B tiles of 16 rows per wave: <4, 3> one wave per SIMD (acc 17 x 3, 512-register
// budget), <8, 2> two waves per SIMD (acc 17 x 2 in 256 registers) so that one wave's waits are the other's issue.
// LAY (toued_wgrad_bfp_slab): bit 1 = B in 32-column slab blocks of 256 rows (k_gru_bwd6n<true>'s DG): row r of block
// r >> 8, column k at (r >> 8) * 256 K + ((k >> 5) * 256 + (r & 255)) * 32 + (k & 31) floats; bit 0 = A's rows 0..255
// (the GRU's h_in) in slab blocks at A, ((k >> 5) * 256 + r) * 32 + (k & 31), its rows 256.. in [ra][lda] rows
template <int NW, int BT, int LAY>
__global__ void __launch_bounds__(64 * NW, 1) k_wgrad_h3(const float* __restrict__ A, long lda, int ra,
                                                        int a_unit_rows, const int* __restrict__ rowmax_bits,
                                                        const float* __restrict__ B, long ldb, int rb,
                                                        const int8_t* __restrict__ colexp, long K, long kchunk,
                                                        float* __restrict__ part, int ntiles, int* __restrict__ qctr,
                                                        int* __restrict__ visits) {
  constexpr int NT = 64 * NW;
  constexpr int CT = 16 * BT * NW;                          // B rows per workgroup
  constexpr bool BSL = (LAY & 2) != 0, ASL = (LAY & 1) != 0;
  static_assert(!BSL || CT == 256, "slab-block B: one 256-row block per column tile");
  constexpr int NS = (X6_AQ + NT - 1) / NT;                 // A staging rounds per thread
  static_assert(NS <= 17 && 2 * BT < 17 - NS, "side-work schedule: B splits, B issue, then the staging rounds");
  const int ncol = (rb + CT - 1) / CT;
#ifdef H3_PLACE
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
#endif
  // Tile queues, one per XCD: XCD x owns the linear slots [base(x), base(x) + cnt(x)) (consecutive slots are the
  // ncol column tiles of one K chunk, which read each A slab through that XCD's L2).  A workgroup takes the next slot
  // of the XCD it runs on (XCC_ID), or of the next XCD with slots left.  The grid has more workgroups than tiles: a
  // workgroup the dispatcher could not place at launch (a CU of its shader engine held by the eval chain beside this
  // kernel) starts after the first ones finish, finds the queues empty and leaves -- instead of a tile of its own
  // in a second round (6.9 vs 4.0 ms with a fixed blockIdx -> tile map; tools/h3_place.py).
  // The ranges hold whole K chunks (all ncol column tiles of a chunk on one XCD, so its A slabs come through one L2
  // only; ranges cut inside a chunk had two XCDs fetch that chunk's A); a workgroup stealing from another XCD takes
  // that XCD's slots from the back, so a chunk is split between two XCDs at most at the end of a range.
  __shared__ int s_slot;
  if (threadIdx.x == 0) {
    const int x = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7;   // HW_REG_XCC_ID
    const int nch = ntiles / ncol, per = nch >> 3, rem = nch & 7;
    int got = -1;
    for (int y = 0; y < 8 && got < 0; ++y) {
      const int q = (x + y) & 7;
      const int cnt = ncol * (per + (q < rem ? 1 : 0));
      if (cnt == 0) continue;
      // one word per queue: slots claimed from the front (low 16 bits) and from the back (high 16 bits); a claim
      // succeeds while the two together are below cnt, so every slot goes out exactly once
      const int old = atomicAdd(&qctr[q], y == 0 ? 1 : 1 << 16);
      const int f = old & 0xFFFF, b = old >> 16;
      if (f + b < cnt) got = ncol * (q * per + (q < rem ? q : rem)) + (y == 0 ? f : cnt - 1 - b);
    }
    s_slot = got;
    // tests only (toued_dbg_wgrad_visits): count each claimed tile, so a tile claimed twice or never shows
    if (visits && got >= 0) atomicAdd(&visits[got], 1);
  }
  __syncthreads();
  const int L = s_slot;
  if (L < 0) return;
  __shared__ f16x8 As[2][2][X6_RA * 4];    // [buffer][piece][slot]: 69,632 B
  __shared__ float asc[X6_RA];             // 2^s_i of A row i
  __shared__ int cred[NW];
  const int tid = threadIdx.x, lane = tid & 63, q16 = lane & 15, oct = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ct = L % ncol, sc = L / ncol;
  const long kb = (long)sc * kchunk;
  const long ke = kb + kchunk < K ? kb + kchunk : K;
  const int nslab = (int)((ke - kb) / 32);
  // chunk B exponent c = min over the chunk's columns (127 = an all-zero column, no constraint)
  int cm = 127;
  for (long m = kb + 16L * tid; m < ke; m += 16L * NT) {
    const int4 v = *reinterpret_cast<const int4*>(colexp + m);
    const int w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int b = 0; b < 4; ++b) cm = min(cm, (int)(int8_t)(w4[q] >> (8 * b)));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cm = min(cm, __shfl_xor(cm, o, 64));
  if (lane == 0) cred[wave] = cm;
  for (int i = tid; i < X6_RA; i += NT) {
    const int r = i < ra ? i : ra - 1;
    asc[i] = r < a_unit_rows ? 16384.0f : ldexpf(1.0f, scale_exp_of(__int_as_float(rowmax_bits[r - a_unit_rows])));
  }
  __syncthreads();
  int cexp = cred[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) cexp = min(cexp, cred[w]);
  if (cexp == 127) cexp = 0;
  const float bsc = ldexpf(1.0f, cexp);
  // B tile t through its own (wave-uniform) descriptor at the tile's first row and the chunk's first column, with
  // 32-bit lane offsets (rows past rb read row rb - 1: they only feed C rows that are never written out).  A
  // fragment's 8 k of lane octet o are k-quads o and o + 4 of the slab (both operands permuted alike: the sum is
  // over all 32), so each B load instruction reads 64 contiguous bytes of each of its 16 rows.
  __amdgpu_buffer_rsrc_t rsB[BT];
  unsigned boff[BT];
  int brow[BT];
#pragma unroll
  for (int t = 0; t < BT; ++t) {
    const int tb = ct * CT + 16 * (BT * wave + t);
    const int tbc = tb < rb ? tb : rb - 1;
    brow[t] = tb + q16;
    const int rr = brow[t] < rb ? brow[t] : rb - 1;
    if (BSL) {   // the tile's rows within its block's slab (128 bytes each); the slab in the scalar offset
      rsB[t] = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(B + (long)ct * 256 * K + (kb >> 5) * 256 * 32), 0,
                                                 -1, 0x00020000);
      boff[t] = (unsigned)((rr - ct * 256) * 128 + 16 * oct);
    } else {
      rsB[t] = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(B + (long)tbc * ldb + kb), 0, -1, 0x00020000);
      boff[t] = (unsigned)(((long)(rr - tbc) * ldb + 4 * oct) * 4);
    }
  }
  float4 ast[NS];
  // the last round's threads past the slab's 272 rows redo row 271's k-quads (identical values, benign duplicate LDS
  // writes); they must stay in rows >= 256 so that a round is uniformly slab-block or row-major A (ASL)
  auto a_index = [&](int j) {
    const int i = tid + NT * j;
    return j < NS - 1 || i < X6_AQ ? i : X6_AQ - 8 + (i & 7);
  };
  // A through a buffer descriptor: per round one 32-bit lane offset (row, k-quad), the slab's column in the scalar
  // offset (64-bit row pointers per round, loop-invariant, were spilled and reloaded every slab)
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A), 0, -1, 0x00020000);
  // ASL: rounds j < JS stage rows 0..255 (uniform per round: round j holds rows j NT / 8 .. (j + 1) NT / 8 - 1) from the
  // slab blocks: the chunk's first block in the descriptor, the slab's block in the scalar offset
  constexpr int JS = ASL ? 2048 / NT : 0;
  static_assert(!ASL || (2048 % NT == 0 && JS <= NS - 1), "slab-block A: rounds split at row 256");
  const __amdgpu_buffer_rsrc_t rsAs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A + (ASL ? (kb >> 5) * 256 * 32 : 0)), 0, -1, 0x00020000);
  unsigned avo[NS];
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const int i = a_index(j);
    const int row = (i >> 3) < ra ? (i >> 3) : ra - 1;
    avo[j] = j < JS ? (unsigned)((row * 32 + 4 * (i & 7)) * 4) : (unsigned)(((long)row * lda + 4 * (i & 7)) * 4);
  }
  auto load_a = [&](int s) {
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const u32x4 x = j < JS ? __builtin_amdgcn_raw_buffer_load_b128(rsAs, (int)avo[j], 32768 * s, 0)
                             : __builtin_amdgcn_raw_buffer_load_b128(rsA, (int)avo[j], (int)((kb + 32L * s) * 4), 0);
      ast[j] = make_float4(__uint_as_float(x.x), __uint_as_float(x.y), __uint_as_float(x.z), __uint_as_float(x.w));
    }
  };
  // this thread's staging rows are the same in every slab: their scales live in registers (an LDS read per round
  // would sit on the in-order LDS counter in front of the fragment reads)
  float asr[NS];
  auto write_a = [&](int buf, int j) {
    const int i = a_index(j);
    const int row = i >> 3, kq = i & 7;
    const int slot = x6_slot(row, kq & 3);
    const float s = asr[j];
    f16x4 p0, p1;
#pragma unroll
    for (int e = 0; e < 4; ++e) split2_f16s(f4(ast[j], e), s, p0, p1, e);
    reinterpret_cast<f16x4*>(&As[buf][0][slot])[kq >> 2] = p0;
    reinterpret_cast<f16x4*>(&As[buf][1][slot])[kq >> 2] = p1;
  };
  float4 bq[BT][2];
  auto issue_b = [&](int s) {
#pragma unroll
    for (int t = 0; t < BT; ++t)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rsB[t], (int)boff[t], (BSL ? 32768 : 128) * s + 64 * hf,
                                                              H3_B_AUX);
        bq[t][hf] = make_float4(__uint_as_float(x.x), __uint_as_float(x.y), __uint_as_float(x.z), __uint_as_float(x.w));
      }
  };
  auto split_b = [&](f16x8 (&dst)[BT][2], int t, int half) {
#pragma unroll
    for (int e = 0; e < 4; ++e) split2_f16s(f4(bq[t][half], e), bsc, dst[t][0], dst[t][1], 4 * half + e);
  };
  floatx4 acc[17][BT];
#pragma unroll
  for (int i = 0; i < 17; ++i)
#pragma unroll
    for (int t = 0; t < BT; ++t) acc[i][t] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};

  auto slab = [&](int s, f16x8 (&bp)[BT][2], f16x8 (&bpn)[BT][2]) {
    WG_STAMP(s, 0);
    const int buf = s & 1;
    load_a(s + 1 < nslab ? s + 1 : s);
    const f16x8* a0p = As[buf][0];
    const f16x8* a1p = As[buf][1];
    // A fragments two tiles ahead (the LDS reads of tile i + 2 go out with tile i's MFMAs)
    // A fragments LA tiles ahead through an (LA + 1)-slot ring (the LDS reads of tile i + LA go out with tile i's
    // MFMAs): two ahead with one wave per SIMD, one ahead with two (the partner wave covers the rest; registers)
    constexpr int LA = NW == 4 ? 2 : 1;
    f16x8 fr[LA + 1][2];
#pragma unroll
    for (int d = 0; d < LA; ++d) {
      const int slot = x6_slot(16 * d + q16, oct);
      fr[d][0] = a0p[slot]; fr[d][1] = a1p[slot];
    }
#pragma unroll
    for (int i = 0; i < 17; ++i) {
      if (i + LA < 17) {
        const int slot = x6_slot(16 * (i + LA) + q16, oct);
        fr[(i + LA) % (LA + 1)][0] = a0p[slot]; fr[(i + LA) % (LA + 1)][1] = a1p[slot];
      }
      const f16x8(&a)[2] = fr[i % (LA + 1)];
#pragma unroll
      for (int t = 0; t < BT; ++t) {
        floatx4 c = acc[i][t];
        c = mfma_h(a[1], bp[t][0], c);
        c = mfma_h(a[0], bp[t][1], c);
        c = mfma_h(a[0], bp[t][0], c);
        acc[i][t] = c;
      }
      // all of the next slab's B splits in the first tile, the loads of the slab after next in the second: those
      // loads get 16 tiles to land instead of 13 (the kernel waits on its B stream: 4.62-4.66 vs 4.70-4.73 ms)
      if (i == 0)
#pragma unroll
        for (int t = 0; t < BT; ++t) { split_b(bpn, t, 0); split_b(bpn, t, 1); }
      if (i == 1) issue_b(s + 2 < nslab ? s + 2 : nslab - 1);
      if (i == 8) WG_STAMP(s, 1);
      if (i >= 17 - NS) write_a(buf ^ 1, i - (17 - NS));
      if (i + LA < 17) {
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // the fragment reads of tile i + LA first
      }
#pragma unroll
      for (int m = 0; m < 3 * BT; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // one MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);   // side-work VALU
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    WG_STAMP(s, 2);
    lds_barrier();
    WG_STAMP(s, 3);
  };

#if H3_BR2
  // B's raw slabs through a two-buffer register ring instead of split-ahead pieces (same registers: raw x 2 + one
  // piece set instead of raw + two piece sets): slab s+2's loads go out at tile 1 of slab s and are split at the end of
  // slab s+1, two slabs in flight instead of one; the split of the next slab's pieces sits after the last tile's MFMAs
  float4 bq2[2][BT][2];
  auto issue_into = [&](float4 (&dst)[BT][2], int s) {
#pragma unroll
    for (int t = 0; t < BT; ++t)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rsB[t], (int)boff[t], (BSL ? 32768 : 128) * s + 64 * hf,
                                                              H3_B_AUX);
        dst[t][hf] = make_float4(__uint_as_float(x.x), __uint_as_float(x.y), __uint_as_float(x.z), __uint_as_float(x.w));
      }
  };
  auto split_from = [&](const float4 (&src)[BT][2], f16x8 (&dst)[BT][2]) {
#pragma unroll
    for (int t = 0; t < BT; ++t)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int e = 0; e < 4; ++e) split2_f16s(f4(src[t][hf], e), bsc, dst[t][0], dst[t][1], 4 * hf + e);
  };
  auto slab2 = [&](int s, f16x8 (&bp)[BT][2], const float4 (&nxt)[BT][2], float4 (&fill)[BT][2]) {
    const int buf = s & 1;
    load_a(s + 1 < nslab ? s + 1 : s);
    const f16x8* a0p = As[buf][0];
    const f16x8* a1p = As[buf][1];
    constexpr int LA = NW == 4 ? 2 : 1;
    f16x8 fr[LA + 1][2];
#pragma unroll
    for (int d = 0; d < LA; ++d) {
      const int slot = x6_slot(16 * d + q16, oct);
      fr[d][0] = a0p[slot]; fr[d][1] = a1p[slot];
    }
#pragma unroll
    for (int i = 0; i < 17; ++i) {
      if (i + LA < 17) {
        const int slot = x6_slot(16 * (i + LA) + q16, oct);
        fr[(i + LA) % (LA + 1)][0] = a0p[slot]; fr[(i + LA) % (LA + 1)][1] = a1p[slot];
      }
      const f16x8(&a)[2] = fr[i % (LA + 1)];
#pragma unroll
      for (int t = 0; t < BT; ++t) {
        floatx4 c = acc[i][t];
        c = mfma_h(a[1], bp[t][0], c);
        c = mfma_h(a[0], bp[t][1], c);
        c = mfma_h(a[0], bp[t][0], c);
        acc[i][t] = c;
      }
      if (i == 1) issue_into(fill, s + 2 < nslab ? s + 2 : nslab - 1);
      if (i >= 17 - NS) write_a(buf ^ 1, i - (17 - NS));
      if (i == 16) split_from(nxt, bp);   // the last tile's MFMAs have read bp
      if (i + LA < 17) {
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      }
#pragma unroll
      for (int m = 0; m < 3 * BT; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    lds_barrier();
  };
#pragma unroll
  for (int j = 0; j < NS; ++j) asr[j] = asc[a_index(j) >> 3];
  f16x8 bpc[BT][2];
  if (nslab > 0) {
    load_a(0);
    issue_into(bq2[0], 0);
    issue_into(bq2[1], nslab > 1 ? 1 : 0);
#pragma unroll
    for (int j = 0; j < NS; ++j) write_a(0, j);
    split_from(bq2[0], bpc);
  }
  __syncthreads();
  int s2 = 0;
  for (; s2 + 1 < nslab; s2 += 2) {
    slab2(s2, bpc, bq2[1], bq2[0]);
    slab2(s2 + 1, bpc, bq2[0], bq2[1]);
  }
  if (s2 < nslab) slab2(s2, bpc, bq2[1], bq2[0]);
#else
  f16x8 bpa[BT][2], bpb[BT][2];
#pragma unroll
  for (int j = 0; j < NS; ++j) asr[j] = asc[a_index(j) >> 3];
  if (nslab > 0) {
    load_a(0);
    issue_b(0);
#pragma unroll
    for (int j = 0; j < NS; ++j) write_a(0, j);
#pragma unroll
    for (int t = 0; t < BT; ++t) { split_b(bpa, t, 0); split_b(bpa, t, 1); }
    issue_b(nslab > 1 ? 1 : 0);
  }
  __syncthreads();
  for (int s = 0; s < nslab; ++s) {
    slab(s, bpa, bpb);
#pragma unroll
    for (int t = 0; t < BT; ++t)
#pragma unroll
      for (int pc = 0; pc < 2; ++pc) bpa[t][pc] = bpb[t][pc];
  }
#endif
  // D map: lane l, reg r -> C[16i + 4 oct + r][brow]; unscale by 2^-(s_row + c) (two exact steps)
  const int rbp = ncol * CT;
  float* out = part + (long)sc * X6_RA * rbp;
  const float ib = ldexpf(1.0f, -cexp);
#pragma unroll
  for (int i = 0; i < 17; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float ia = 1.0f / asc[16 * i + 4 * oct + r];
#pragma unroll
      for (int t = 0; t < BT; ++t) out[(long)(16 * i + 4 * oct + r) * rbp + brow[t]] = (acc[i][t][r] * ia) * ib;
    }
#ifdef H3_PLACE
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x < 256) {
    const unsigned slot = g_h3_launch & 63u;
    unsigned long long* e = g_h3_place + ((size_t)slot * 256 + blockIdx.x) * 4;
    e[0] = (unsigned long long)__builtin_amdgcn_s_getreg((3 << 11) | 20);   // XCC_ID[3:0]
    e[1] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
    e[2] = t_start;
    e[3] = __builtin_amdgcn_s_memrealtime();
  }
#endif
}

// C[i][j] = sum over chunks (in chunk order) of part[s][i][j], i < ra, j < rb
__global__ void k_wgrad_reduce(const float* __restrict__ part, int S, int RA, int rbp, int ra, int rb,
                               float* __restrict__ C, int ldc) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)ra * rb) return;
  const int i = (int)(idx / rb), j = (int)(idx - (long)i * rb);
  float s = 0.0f;
  for (int c = 0; c < S; ++c) s += part[((long)c * RA + i) * rbp + j];
  C[(long)i * ldc + j] = s;
}

// Many chunks (the small HBM-stream reductions split K ~500 ways): one wave per output element, lane l sums
// chunks l, l + 64, ... in order, then a fixed xor-butterfly across the wave -- still deterministic, and
// ~S/64 dependent loads per lane instead of S.
__global__ void k_wgrad_reduce_wave(const float* __restrict__ part, int S, int RA, int rbp, int ra, int rb,
                                    float* __restrict__ C, int ldc) {
  const long idx = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (idx >= (long)ra * rb) return;
  const int i = (int)(idx / rb), j = (int)(idx - (long)i * rb);
  float s = 0.0f;
  for (int c = lane; c < S; c += 64) s += part[((long)c * RA + i) * rbp + j];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  if (lane == 0) C[(long)i * ldc + j] = s;
}

// Row sums of A [ra][K] (row stride lda) into C[i * ldc]: per (K chunk, row) partials in a fixed order (float4 loads,
// 256 threads, a block tree), then one wave per row over the chunks.  Deterministic.
__global__ void __launch_bounds__(256) k_rowsum_part(const float* __restrict__ A, long lda, long K, long kchunk,
                                                     float* __restrict__ part) {
  const int c = blockIdx.x, i = blockIdx.y, ra = gridDim.y;
  const long kb = (long)c * kchunk, ke = kb + kchunk < K ? kb + kchunk : K;
  const float4* a4 = reinterpret_cast<const float4*>(A + (long)i * lda + kb);
  const long n4 = (ke - kb) / 4;
  float s = 0.0f;
  for (long m = threadIdx.x; m < n4; m += 256) {
    const float4 v = a4[m];
    s += (v.x + v.y) + (v.z + v.w);
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[(long)c * ra + i] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void k_rowsum_final(const float* __restrict__ part, int S, int ra, float* __restrict__ C, int ldc) {
  const int i = blockIdx.x, lane = threadIdx.x;
  float s = 0.0f;
  for (int c = lane; c < S; c += 64) s += part[(long)c * ra + i];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  if (lane == 0) C[(long)i * ldc] = s;
}

struct Plan {
  int nrt, ncol, S, ct;   // ct: B rows per workgroup (column-tile width of the partial-sum workspace)
  bool x6;
  long kchunk;
};

static bool wgrad_f32_forced() {
  static const bool f = [] {
    const char* e = getenv("TOUED_WGRAD_F32");
    return e && e[0] == '1';
  }();
  return f;
}

static Plan plan(int ra, int rb, long K) {
  Plan p;
  p.nrt = ra <= 16 ? 1 : 17;
  p.x6 = p.nrt == 17 && !wgrad_f32_forced();
  p.ct = p.x6 ? X6_CT : 128;
  p.ncol = (rb + p.ct - 1) / p.ct;
  int cus = 256;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
    cus = 256;
  {
    const int rsv = toued::current_ctx()->reserved_cus.load();
    cus = cus - rsv > cus / 2 ? cus - rsv : cus / 2;
  }
  // x6: one workgroup per CU (104 KB LDS), as many K chunks as fill the CUs in one round.  f32 NRT = 17:
  // two workgroups per CU (125 VGPRs, 68 KB LDS each).  NRT = 1 is a bandwidth-bound stream over B: four
  // workgroups per CU keep enough loads in flight.
  int S = (p.x6 ? 1 : p.nrt == 1 ? 4 : 2) * cus / p.ncol;
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

#ifdef H3_PLACE
int toued_dbg_h3_place(unsigned long long* host, unsigned* launches) {
  if (hipMemcpyFromSymbol(launches, HIP_SYMBOL(g_h3_launch), sizeof(unsigned)) != hipSuccess) return 1;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_h3_place), sizeof(g_h3_place)) == hipSuccess ? 0 : 1;
}
__global__ void k_h3_next() { if (threadIdx.x == 0) atomicAdd(&g_h3_launch, 1u); }
#endif
#ifdef WG_STAMPS
int toued_dbg_wgrad_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wg_stamps), sizeof(g_wg_stamps)) == hipSuccess ? 0 : 1;
}
#endif

int toued_set_reserved_cus(int n) {
  return toued::current_ctx()->reserved_cus.exchange(n > 0 ? n : 0);
}

size_t toued_wgrad_workspace_floats(int ra, int rb, long K) {
  if (ra <= 0 || rb <= 0 || K <= 0) return 0;
  const Plan p = plan(ra, rb, K);
  return (size_t)p.S * p.nrt * 16 * p.ncol * p.ct;
}

static int wgrad_ldc(int ra, int rb, long K, const float* A, long lda, const float* B, long ldb, float* C, int ldc,
                     float* work, size_t work_floats, hipStream_t stream);

int toued_wgrad(int ra, int rb, long K, const float* A, long lda, const float* B, long ldb, float* C, float* work,
                size_t work_floats, hipStream_t stream) {
  return wgrad_ldc(ra, rb, K, A, lda, B, ldb, C, rb, work, work_floats, stream);
}

// C [ra][rb] with row stride ldc (the backward's head block [9][257] takes its 256 unit columns from here and the
// bias column from toued_rowsum_into)
int toued_wgrad_ldc(int ra, int rb, long K, const float* A, long lda, const float* B, long ldb, float* C, int ldc,
                    float* work, size_t work_floats, hipStream_t stream) {
  return wgrad_ldc(ra, rb, K, A, lda, B, ldb, C, ldc, work, work_floats, stream);
}

// rows sums: the chunks and the partials' floats the workspace needs
static long rowsum_chunk(long K) {
  long kc = ((K + 255) / 256 + 31) / 32 * 32;
  return kc < 32 ? 32 : kc;
}
size_t toued_rowsum_workspace_floats(int ra, long K) {
  return K > 0 ? (size_t)((K + rowsum_chunk(K) - 1) / rowsum_chunk(K)) * ra : 0;
}
int toued_rowsum_into(int ra, long K, const float* A, long lda, float* C, int ldc, float* work, size_t work_floats,
                      hipStream_t stream) {
  TOUED_REQUIRE(ra >= 1 && K >= 0 && K % 4 == 0 && lda % 4 == 0, "toued_rowsum_into: ra=%d K=%ld lda=%ld", ra, K, lda);
  TOUED_REQUIRE(work_floats >= toued_rowsum_workspace_floats(ra, K), "toued_rowsum_into: workspace too small");
  if (K == 0) {
    for (int i = 0; i < ra; ++i)
      TOUED_REQUIRE(hipMemsetAsync(C + (long)i * ldc, 0, sizeof(float), stream) == hipSuccess, "memset failed");
    return 0;
  }
  const long kc = rowsum_chunk(K);
  const int S = (int)((K + kc - 1) / kc);
  hipLaunchKernelGGL(k_rowsum_part, dim3(S, ra), dim3(256), 0, stream, A, lda, K, kc, work);
  hipLaunchKernelGGL(k_rowsum_final, dim3(ra), dim3(64), 0, stream, work, S, ra, C, ldc);
  TOUED_CHECK_LAUNCH();
  return 0;
}

static int wgrad_ldc(int ra, int rb, long K, const float* A, long lda, const float* B, long ldb, float* C, int ldc,
                     float* work, size_t work_floats, hipStream_t stream) {
  TOUED_REQUIRE(ra >= 1 && ra <= 272 && rb >= 1 && K >= 0, "toued_wgrad: ra=%d (1..272) rb=%d K=%ld", ra, rb, K);
  TOUED_REQUIRE(K % 32 == 0, "toued_wgrad: K=%ld must be a multiple of 32", K);
  TOUED_REQUIRE(lda % 4 == 0 && ldb % 4 == 0, "toued_wgrad: lda=%ld ldb=%ld must be multiples of 4 (16-byte rows)",
                lda, ldb);
  TOUED_REQUIRE(A && B && C, "toued_wgrad: null operand");
  if (K == 0) {
    for (int i = 0; i < ra; ++i)
      TOUED_REQUIRE(hipMemsetAsync(C + (long)i * ldc, 0, sizeof(float) * rb, stream) == hipSuccess,
                    "toued_wgrad: memset failed");
    return 0;
  }
  const Plan p = plan(ra, rb, K);
  const size_t need = (size_t)p.S * p.nrt * 16 * p.ncol * p.ct;
  TOUED_REQUIRE(work && work_floats >= need, "toued_wgrad: workspace of %zu floats needed (got %zu)", need, work_floats);
  const dim3 grid(p.ncol, p.S);
  if (p.x6)
    hipLaunchKernelGGL(k_wgrad_x6, dim3(p.ncol * p.S), dim3(64 * X6_NW), 0, stream, A, lda, ra, B, ldb, rb, K, p.kchunk, work);
  else if (p.nrt == 1)
    hipLaunchKernelGGL(k_wgrad<1>, grid, dim3(512), 0, stream, A, lda, ra, B, ldb, rb, K, p.kchunk, work);
  else
    hipLaunchKernelGGL(k_wgrad<17>, grid, dim3(512), 0, stream, A, lda, ra, B, ldb, rb, K, p.kchunk, work);
  const long n = (long)ra * rb;
  if (p.S > 128)
    hipLaunchKernelGGL(k_wgrad_reduce_wave, dim3((unsigned)((n * 64 + 255) / 256)), dim3(256), 0, stream, work, p.S,
                       p.nrt * 16, p.ncol * p.ct, ra, rb, C, ldc);
  else
    hipLaunchKernelGGL(k_wgrad_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, work, p.S,
                       p.nrt * 16, p.ncol * p.ct, ra, rb, C, ldc);
  TOUED_CHECK_LAUNCH();
  return 0;
}

// Main LPG weight-gradient reduction on block-floating-point fp16 pairs (k_wgrad_h3): rows [0, a_unit_rows) of A
// must be bounded by 1 in magnitude; col_exp[m] is B column m's scale exponent (127 = zero column).
// k_wgrad_h3<8, 2> (two waves per SIMD) unless TOUED_WGRAD_NW4=1 selects <4, 3> (one wave per SIMD, comparison
// runs): 4.59-4.67 ms against 4.75-4.88 at the C2 shape, per-slab stamps 23.4 against 29.8 cycles per B row
static bool wgrad_h8() {
  static const bool f = [] {
    const char* e = getenv("TOUED_WGRAD_NW4");
    return !(e && e[0] == '1');
  }();
  return f;
}

// CUs the plan's tiles leave unused (TOUED_H3_SLACK, default 16) and workgroups launched beyond the tiles
// (TOUED_H3_EXTRA, default 16).  Measured (tools/h3_place.py, tools/h3_timing.py, 25 launches each beside the eval
// chain): the dispatcher deals workgroups to XCDs and shader engines in turn and dispatches them in order, so one
// workgroup it cannot place (its engine's free CUs taken) holds back every later one until a CU frees -- a tile in
// a second round (6.9 instead of 4.0 ms).  With 16 tiles fewer than the free CUs and the grid at the free CUs, the
// held-back workgroups are spares: 0 of 25 launches slow (8 / 16: 14 of 25; 8 / 8: 6 of 17; a fixed
// blockIdx -> tile map: 7 of 22, all 17 without HIP timing events in the stream)
static int h3_slack() {
  static const int v = [] {
    const char* e = getenv("TOUED_H3_SLACK");
    return e ? atoi(e) : 16;
  }();
  return v;
}

static int h3_extra() {
  static const int v = [] {
    const char* e = getenv("TOUED_H3_EXTRA");
    return e ? atoi(e) : 16;
  }();
  return v;
}

// the k_wgrad_h3 variant's plan: B rows per workgroup, column tiles and K chunks (one workgroup per CU)
static Plan plan_bfp(int ra, int rb, long K) {
  Plan p = plan(ra > 16 ? ra : 17, rb, K);
  p.ct = wgrad_h8() ? 16 * 2 * 8 : X6_CT;
  p.ncol = (rb + p.ct - 1) / p.ct;
  int cus = 256;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
    cus = 256;
  {
    const int rsv = toued::current_ctx()->reserved_cus.load();
    cus = cus - rsv > cus / 2 ? cus - rsv : cus / 2;
  }
  cus = cus - h3_slack() > cus / 2 ? cus - h3_slack() : cus / 2;
  int S = cus / p.ncol;
  if (S < 1) S = 1;
  const long slabs = K / 32;
  if (S > slabs) S = (int)(slabs > 0 ? slabs : 1);
  p.kchunk = ((slabs + S - 1) / S) * 32;
  p.S = (int)((K + p.kchunk - 1) / p.kchunk);
  if (p.S < 1) p.S = 1;
  return p;
}

// tests only: per-tile claim counters of the next toued_wgrad_bfp launches (visits[tile] += 1 per claim; nullptr
// switches it off), and the tile count of the last launch
static int* g_dbg_visits = nullptr;
static int g_dbg_visits_cap = 0;
static int g_dbg_last_ntiles = 0;
int toued_dbg_wgrad_visits(int* visits, int capacity) {
  g_dbg_visits = capacity > 0 ? visits : nullptr;
  g_dbg_visits_cap = capacity > 0 ? capacity : 0;
  return 0;
}
int toued_dbg_wgrad_last_ntiles(void) { return g_dbg_last_ntiles; }

size_t toued_wgrad_bfp_workspace_floats(int ra, int rb, long K) {
  if (ra <= 0 || rb <= 0 || K <= 0) return 0;
  const Plan p = plan_bfp(ra, rb, K);
  return (size_t)p.S * 17 * 16 * p.ncol * p.ct + X6_RA + 8;
}

}  // extern "C"

static int wgrad_bfp(int ra, int rb, long K, const float* A, long lda, int a_unit_rows, const float* B, long ldb,
                     int layout, const int8_t* col_exp, float* C, float* work, size_t work_floats, hipStream_t stream) {
  TOUED_REQUIRE(ra > 16 && ra <= X6_RA && rb >= 1 && a_unit_rows >= 0 && a_unit_rows <= ra,
                "toued_wgrad_bfp: ra=%d (17..%d) rb=%d a_unit_rows=%d", ra, X6_RA, rb, a_unit_rows);
  TOUED_REQUIRE(K > 0 && K % 32 == 0, "toued_wgrad_bfp: K=%ld must be a positive multiple of 32", K);
  TOUED_REQUIRE(lda % 4 == 0 && ldb % 4 == 0, "toued_wgrad_bfp: lda=%ld ldb=%ld must be multiples of 4", lda, ldb);
  TOUED_REQUIRE((double)ra * lda * 4.0 < 4294967295.0, "toued_wgrad_bfp: A (%d rows x %ld) exceeds the 4 GiB buffer range",
                ra, lda);
  TOUED_REQUIRE(A && B && C && col_exp, "toued_wgrad_bfp: null operand");
  TOUED_REQUIRE((reinterpret_cast<uintptr_t>(col_exp) & 15) == 0, "toued_wgrad_bfp: col_exp must be 16-byte aligned");
  const Plan p = plan_bfp(ra, rb, K);
  TOUED_REQUIRE(p.kchunk % 16 == 0, "toued_wgrad_bfp: chunk %ld", p.kchunk);
  const size_t need = (size_t)p.S * 17 * 16 * p.ncol * p.ct;
  TOUED_REQUIRE(work && work_floats >= need + X6_RA + 8, "toued_wgrad_bfp: workspace of %zu floats needed (got %zu)",
                need + X6_RA + 8, work_floats);
  int* bits = reinterpret_cast<int*>(work + need);
  int* qctr = bits + X6_RA;                                // the eight per-XCD tile queue counters
  const int nmeas = ra - a_unit_rows;
  TOUED_REQUIRE(hipMemsetAsync(bits, 0, sizeof(int) * (X6_RA + 8), stream) == hipSuccess, "toued_wgrad_bfp: memset");
  const int ntiles = p.ncol * p.S, grid = ntiles + h3_extra();
  if (nmeas > 0) {
    const long kper = 65536;
    hipLaunchKernelGGL(k_wgrad_rowmax, dim3((unsigned)((K + kper - 1) / kper), nmeas), dim3(256), 0, stream, A, lda,
                       a_unit_rows, K, kper, bits);
  }
  int* visits = g_dbg_visits && ntiles <= g_dbg_visits_cap ? g_dbg_visits : nullptr;
  g_dbg_last_ntiles = ntiles;
  if (layout == 3)
    hipLaunchKernelGGL((k_wgrad_h3<8, 2, 3>), dim3(grid), dim3(512), 0, stream, A, lda, ra, a_unit_rows, bits, B,
                       ldb, rb, col_exp, K, p.kchunk, work, ntiles, qctr, visits);
  else if (layout == 2)
    hipLaunchKernelGGL((k_wgrad_h3<8, 2, 2>), dim3(grid), dim3(512), 0, stream, A, lda, ra, a_unit_rows, bits, B,
                       ldb, rb, col_exp, K, p.kchunk, work, ntiles, qctr, visits);
  else if (layout == 1)
    hipLaunchKernelGGL((k_wgrad_h3<8, 2, 1>), dim3(grid), dim3(512), 0, stream, A, lda, ra, a_unit_rows, bits, B,
                       ldb, rb, col_exp, K, p.kchunk, work, ntiles, qctr, visits);
  else if (wgrad_h8())
    hipLaunchKernelGGL((k_wgrad_h3<8, 2, 0>), dim3(grid), dim3(512), 0, stream, A, lda, ra, a_unit_rows, bits, B,
                       ldb, rb, col_exp, K, p.kchunk, work, ntiles, qctr, visits);
  else
    hipLaunchKernelGGL((k_wgrad_h3<X6_NW, X6_BT, 0>), dim3(grid), dim3(64 * X6_NW), 0, stream, A, lda, ra,
                       a_unit_rows, bits, B, ldb, rb, col_exp, K, p.kchunk, work, ntiles, qctr, visits);
#ifdef H3_PLACE
  hipLaunchKernelGGL(k_h3_next, dim3(1), dim3(64), 0, stream);
#endif
  const long n = (long)ra * rb;
  hipLaunchKernelGGL(k_wgrad_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, work, p.S, 17 * 16,
                     p.ncol * p.ct, ra, rb, C, rb);
  TOUED_CHECK_LAUNCH();
  return 0;
}

extern "C" {
int toued_wgrad_bfp(int ra, int rb, long K, const float* A, long lda, int a_unit_rows, const float* B, long ldb,
                    const int8_t* col_exp, float* C, float* work, size_t work_floats, hipStream_t stream) {
  return wgrad_bfp(ra, rb, K, A, lda, a_unit_rows, B, ldb, 0, col_exp, C, work, work_floats, stream);
}

// The same with operands in 32-column slab blocks (the split-precision GRU pair's layouts): layout bit 0 = A's rows
// [0, 256) in slab blocks at A ([K/32][256][32]; its rows 256.. stay [ra][lda] rows at A), bit 1 = B in slab blocks
// of 256 rows, [rb/256][K/32][256][32] (ldb unused).  The two-waves-per-SIMD kernel; bit 1 needs rb % 256 == 0,
// bit 0 ra > 256 and a_unit_rows == 256.
int toued_wgrad_bfp_slab(int ra, int rb, long K, const float* A, long lda, int a_unit_rows, const float* B, long ldb,
                         int layout, const int8_t* col_exp, float* C, float* work, size_t work_floats,
                         hipStream_t stream) {
  TOUED_REQUIRE(layout >= 0 && layout <= 3, "toued_wgrad_bfp_slab: layout=%d (0..3)", layout);
  TOUED_REQUIRE(!(layout & 2) || (rb % 256 == 0 && rb > 0), "toued_wgrad_bfp_slab: rb=%d must be a multiple of 256", rb);
  TOUED_REQUIRE(!(layout & 1) || (ra > 256 && a_unit_rows == 256),
                "toued_wgrad_bfp_slab: slab-block A needs ra > 256 (got %d) and a_unit_rows == 256 (got %d)", ra,
                a_unit_rows);
  TOUED_REQUIRE(layout == 0 || wgrad_h8(), "toued_wgrad_bfp_slab: slab blocks need the 256-row tiles (not TOUED_WGRAD_NW4=1)");
  TOUED_REQUIRE((double)K * 256.0 * 4.0 < 4294967295.0, "toued_wgrad_bfp_slab: a 256-row block of K=%ld exceeds 4 GiB", K);
  return wgrad_bfp(ra, rb, K, A, lda, a_unit_rows, B, (layout & 2) ? 4 : ldb, layout, col_exp, C, work, work_floats,
                   stream);
}

}  // extern "C"
