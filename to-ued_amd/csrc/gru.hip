// LPG reverse-time GRU (models/lpg.py:11-36 LPGGRU + :79-85 heads) on CDNA4 matrix cores.
//
// Rows = agents x workers (32,768 at N=512) share the LPG parameters, so every time step is a dense
// [rows x 272] x [272 x 1024] contraction (h: 256 recurrent units, + x features and a bias row; columns
// r | z | W_hn h + b_hn | W_in x + b_in) and the VJP a [rows x 768] x [768 x 256] one.
//
// Arithmetic: f32-class products on the 16-bit matrix cores, f32 accumulation:
//   * recurrent products (forward carry k-steps, the three backward gate passes): power-of-two-scaled fp16
//     pairs (y = 2^s x, x0 = fp16(y), x1 = fp16(y - x0)), a0b0 + a0b1 + a1b0 on v_mfma_f32_32x32x16_f16 --
//     weight rows scaled per unit (k_fwd6_scales / k_bwd6_scales), the carry by 2^14 (|h| < 1), backward
//     cotangent rows by a per-batch-row 2^t from an LDS row-max exchange; every scale is exact;
//   * the forward's input k-step [x; 1]: exact three-piece bf16 split, six products of weight >= 2^-16.
// Accuracy vs float64 equals the all-bf16-triple kernels' (tools/gru_accuracy.py, tests/test_gpu_meta.py).
//
// Forward (k_gru_fwd6): one 512-thread workgroup per 64 rows for the whole reverse scan; the carry lives in
// LDS as two fp16 pieces of 2^14 h + a bf16 residual that keeps h_in exact.  Backward (k_gru_bwd6n): one
// 512-thread workgroup per (k, 64 rows), t ascending, lockstep memory part then contraction through one LDS
// cotangent image; dr, dz, dhn are stored to HBM beside the contraction's MFMAs.
//
// f32 fallbacks (v_mfma_f32_32x32x2_f32, one 32-row tile per workgroup): k_gru_fwd<SAVE, NT> (also the
// per-candidate ES forward) and k_gru_bwd<1> for row counts that do not split into 64-row blocks, and every
// GRU kernel under TOUED_GRU_F32=1 (comparison runs).
//
// MFMA operand/result maps (cdna_hip_programming.md §3):
//   f32 32x32x2:  A: lane l holds A[i = l&31][k = l>>5];  B: lane l holds B[k = l>>5][j = l&31]
//   bf16 32x32x16: A: lane l holds A[i = l&31][k = 8(l>>5) + e];  B: B[k = 8(l>>5) + e][j = l&31], e = 0..7
//   D (both): reg q of lane l is D[i = (q&3) + 8*(q>>2) + 4*(l>>5)][j = l&31]
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include "common.h"

extern "C" size_t toued_wgrad_workspace_floats(int ra, int rb, long K);
extern "C" int toued_wgrad(int ra, int rb, long K, const float* A, long lda, const float* B, long ldb, float* C,
                           float* work, size_t work_floats, hipStream_t stream);
extern "C" int toued_wgrad_ldc(int ra, int rb, long K, const float* A, long lda, const float* B, long ldb, float* C,
                               int ldc, float* work, size_t work_floats, hipStream_t stream);
extern "C" size_t toued_rowsum_workspace_floats(int ra, long K);
extern "C" int toued_rowsum_into(int ra, long K, const float* A, long lda, float* C, int ldc, float* work,
                                 size_t work_floats, hipStream_t stream);

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

#define HU 256          // GRU width (lpg_gru_width)
#define RB 32           // batch rows per workgroup
#define LDH 33          // padded LDS row length
#define NAUG 8          // augmented K rows: x (F <= 7) + bias row
#define KQF 33          // fwd k-quads: 32 over h + 1 over the augmented rows
#define NTILE_F 32      // fwd A tiles: r[8] z[8] nh[8] ni[8]

struct EtaOff {         // flat LPG parameter offsets (oracle/lpg.py layout)
  int pi_b, pi_w, y_b, y_w, hn_b, hn_w, hr_w, hz_w, in_b, in_w, ir_b, ir_w, iz_b, iz_w, e1_b, e1_w, e2_b, e2_w;
};

namespace {

TOUED_DEV floatx16 mfma32(float a, float b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// Streamed [256][M] tensors: raw buffer ops with a wave-uniform descriptor built from the
// array base + the register's (uniform) unit/column offset, and ONE 32-bit per-lane byte
// offset shared by every array (cdna_hip_programming.md T8/T20) -- no per-array 64-bit
// VGPR addresses.  The host guarantees 256*M*4 < 2^32 (toued_gru_* check).
TOUED_DEV __amdgpu_buffer_rsrc_t rsrc_of(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, -1 /* 4 GiB */, 0x00020000);
}
// element (unit u = lane unit base + qu, column c) at base + u*M + c: lane part in vbyte, uniform part in soff
TOUED_DEV float ld_u(__amdgpu_buffer_rsrc_t r, unsigned vbyte, unsigned soff) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)vbyte, (int)soff, 0));
}
// Cache policy of the streamed [256][M] stores and loads (buffer-instruction aux bits: 2 = nt, non-temporal).  The
// saves, cotangents and relu rows are written once and read once by a later kernel, never from L2: nt stores measured
// forward 1.24 -> 1.21 ms, backward 9.47 -> 9.27 (sc0 / sc1 no change); nt on the backward's saved-activation loads
// another 9.54 -> 9.22-9.32.
#ifndef GRU_ST_AUX
#define GRU_ST_AUX 2
#endif
#ifndef GRU_LD_AUX
#define GRU_LD_AUX 2
#endif
TOUED_DEV void st_u(__amdgpu_buffer_rsrc_t r, unsigned vbyte, unsigned soff, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)vbyte, (int)soff, GRU_ST_AUX);
}
TOUED_DEV int qunit(int q) { return (q & 3) + 8 * (q >> 2); }

// 16-byte raw buffer ops: the four consecutive units (q & 3) of a register quad in the m-major layout
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));   // packed FP32 pairs (v_pk_*_f32)
TOUED_DEV void ld4(__amdgpu_buffer_rsrc_t r, unsigned vbyte, unsigned soff, float* v) {
  const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(r, (int)vbyte, (int)soff, GRU_LD_AUX);
  v[0] = __uint_as_float(x.x); v[1] = __uint_as_float(x.y); v[2] = __uint_as_float(x.z); v[3] = __uint_as_float(x.w);
}
// (quad_transpose, the 4x4 lane-quad / register-quad transpose: common.h)

TOUED_DEV float sigm(float x) { return 1.0f / (1.0f + __expf(-x)); }
// v_rcp_f32 (1 ulp) instead of the IEEE division sequence: the forward's gate maths is on the critical path
TOUED_DEV float sigm_r(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
TOUED_DEV float tanh_r(float x) {
  const float e = __expf(-2.0f * fabsf(x));
  return copysignf((1.0f - e) * __builtin_amdgcn_rcpf(1.0f + e), x);
}
TOUED_DEV float tanh_f(float x) {
  const float e = __expf(-2.0f * fabsf(x));
  const float t = (1.0f - e) / (1.0f + e);
  return copysignf(t, x);
}

// The n gate of the split-precision kernels: n = tanh(W_in x + b_in + r * (W_hn h + b_hn)).  The input part
// ain = W_in x + b_in is one f32 MFMA chain (v_mfma_f32_32x32x2f32, K = 8: x_0..x_{F-1}, 0.., 1) in the gate
// maths' accumulator layout (lane = row, register q = unit 32 wave + 4 hi + qunit(q)), issued identically by the
// forward (k_gru_fwd6) and the backward (k_gru_bwd6n), so the backward recomputes n bit for bit from the saved r
// and W_hn h + b_hn instead of reading a saved n: 1 KiB per column less written by the forward and read by the
// backward.  wI[kk] = A[i = unit 32 wave + (l & 31)][k = 2 kk + (l >> 5)] = W_in[k][u] (k < F), b_in[u] (k = 7).
TOUED_DEV void load_win_frags(float (&wI)[4], const float* eta, const EtaOff& o, int F, int wave, int lane) {
  const int u = 32 * wave + (lane & 31);
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const int k = 2 * kk + (lane >> 5);
    wI[kk] = k < F ? eta[o.in_w + k * HU + u] : k == 7 ? eta[o.in_b + u] : 0.0f;
  }
}
// B[k = 2 kk + hi][j = row] from this lane's row inputs (xk(k) = x_k for k < F)
template <typename XK>
TOUED_DEV floatx16 gate_ain(const float (&wI)[4], int F, int hi, XK xk) {
  floatx16 a;
#pragma unroll
  for (int q = 0; q < 16; ++q) a[q] = 0.0f;
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const int k = 2 * kk + hi;
    const float xkv = hi ? xk(2 * kk + 1) : xk(2 * kk);   // static indices (a lane-dependent one puts xk's array in scratch)
    a = mfma32(wI[kk], k < F ? xkv : k == 7 ? 1.0f : 0.0f, a);
  }
  return a;
}
TOUED_DEV float gate_n(float ain, float rg, float hn) { return tanh_r(__builtin_fmaf(rg, hn, ain)); }

// 1/x for a power of two x = 2^k (normal, -126 <= k <= 126): exact, by the exponent field (an IEEE division costs
// ten VALU instructions)
TOUED_DEV float inv_pow2(float x) { return __int_as_float((254 << 23) - __float_as_int(x)); }
// the lane id derived afresh where it is used (volatile: never hoisted): a lane-dependent LDS address kept
// live across a long loop body gets spilled, and its reload's wait drains every outstanding buffer access
// (vmcnt counts the stores too)
TOUED_DEV int lane_now() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
// x of lane l ^ 32, with the source lane re-derived here (__shfl_xor's lane arithmetic, kept live across the step loop
// by the compiler, was spilled; its reload in the gate maths waited for every outstanding save store)
TOUED_DEV float xor32(float x) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute((lane_now() ^ 32) << 2, __float_as_int(x)));
}

// ------------------------------------------------------------------ packing
// fwdA[(tile*KQF + kq)*64 + lane] = float4 over kk = 4kq..4kq+3 of A[i=l&31][k=2kk+(l>>5)]
__global__ void k_pack_fwd(const float* __restrict__ eta, EtaOff o, int F, float4* __restrict__ out,
                           long eta_stride, long out_stride4) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= NTILE_F * KQF * 64) return;
  eta += (long)blockIdx.y * eta_stride;            // candidate blockIdx.y (ES); 0 for the shared eta
  out += (long)blockIdx.y * out_stride4;
  const int lane = gid & 63, kq = (gid >> 6) % KQF, tile = gid / (64 * KQF);
  const int g = tile >> 3, u = 32 * (tile & 7) + (lane & 31);
  float v[4];
  for (int e = 0; e < 4; ++e) {
    const int k = 2 * (4 * kq + e) + (lane >> 5);
    float x = 0.0f;
    if (k < HU) {
      if (g == 0) x = eta[o.hr_w + k * HU + u];
      else if (g == 1) x = eta[o.hz_w + k * HU + u];
      else if (g == 2) x = eta[o.hn_w + k * HU + u];
    } else {
      const int f = k - HU;
      if (f < F) {
        if (g == 0) x = eta[o.ir_w + f * HU + u];
        else if (g == 1) x = eta[o.iz_w + f * HU + u];
        else if (g == 3) x = eta[o.in_w + f * HU + u];
      } else if (f == F) {
        x = g == 0 ? eta[o.ir_b + u] : g == 1 ? eta[o.iz_b + u] : g == 2 ? eta[o.hn_b + u] : eta[o.in_b + u];
      }
    }
    v[e] = x;
  }
  out[gid] = make_float4(v[0], v[1], v[2], v[3]);
}

// bwdA[((ut*3 + g)*32 + kq)*64 + lane]: A[i = u (input unit) ][k = c (gate unit)] = W_g[u][c]
__global__ void k_pack_bwd(const float* __restrict__ eta, EtaOff o, float4* __restrict__ out) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= 8 * 3 * 32 * 64) return;
  const int lane = gid & 63, kq = (gid >> 6) & 31, g = (gid >> 11) % 3, ut = gid / (64 * 32 * 3);
  const int u = 32 * ut + (lane & 31);
  const int base = g == 0 ? o.hr_w : g == 1 ? o.hz_w : o.hn_w;
  float v[4];
  for (int e = 0; e < 4; ++e) {
    const int c = 2 * (4 * kq + e) + (lane >> 5);
    v[e] = eta[base + u * HU + c];
  }
  out[gid] = make_float4(v[0], v[1], v[2], v[3]);
}

// bwd6 fragments [ks][unit tile ut][gate g][piece] (1 KiB each), appended after the f32 ones: lane l holds
// A[i = input unit 32 ut + (l & 31)][k = gate unit 16 ks + 8 (l >> 5) + e] = W_g[i][k], split in three bf16
#define B6_NF (16 * 8 * 3 * 3)
#define B6_SCALES (B6_NF * 256)            // float offset of the per-input-unit scales 2^s of W_z, W_hn [256]
#define B6_FLOATS (B6_SCALES + HU)
// One k-major LDS buffer ([unit][row], pitch RB*NT + 1; h^T in the forward, a gate cotangent in the
// backward) of NT row tiles out to its row-major [unit][M] array: per instruction lane l stores row
// RB*h + (l & 31) of unit 32*wave + 2i + (l >> 5), so every wave instruction writes 2 units x 128
// contiguous bytes; the LDS reads (consecutive rows of a unit) are conflict-free.  Dword stores: a VALU write to
// the data VGPRs of a preceding 16-byte buffer store needs wait states that hipcc does not insert when the store
// has an SGPR soffset (observed on gfx950: the first dword of some 16-byte stores replaced by the next value
// written to its register); dword stores carry no such hazard.
template <int NT>
TOUED_DEV void store_gate_lds(const float* buf, __amdgpu_buffer_rsrc_t rs, long M, long col0, int wave, int lane) {
  constexpr int LDT = RB * NT + 1;
  const unsigned so = (unsigned)(col0 * 4);
#pragma unroll
  for (int h = 0; h < NT; ++h) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int unit = 32 * wave + 2 * i + (lane >> 5), r = RB * h + (lane & 31);
      st_u(rs, (unsigned)(((long)unit * M + r) * 4), so, buf[unit * LDT + r]);
    }
  }
}

// The split-precision pair's saves (k_gru_fwd6 writes them, k_gru_bwd6n reads them; the forward's pointers at its
// update's first block; the input rows x that follow h_in stay [F][M] rows):
//  * h_in -- also the main weight-gradient reduction's A operand (toued_wgrad_bfp_slab layout bit 0) -- in 32-column
//    slab blocks [M / 32][256][32] (element (u, c) at ((c >> 5) * 256 + u) * 32 + (c & 31)): the reduction's A slab
//    (256 units x 32 columns) is 32 KB of contiguous memory and each of its 16-byte loads four columns of one unit.
//    Byte offsets of unit ub_ + uq, column c0 + 32 h + col_ (c0 a multiple of 32): lane part slab_vbyte, uniform part
//    slab_soff.  The backward loads four rows of one unit per lane and transposes them across a lane quad.
//  * r, z, W_hn h + b_hn -- read only by the backward -- in 32-column unit-quad blocks [M / 32][64][32][4] (element
//    (u, c) at (c >> 5) * 8192 + ((u >> 2) * 32 + (c & 31)) * 4 + (u & 3)): a lane of the forward's gate maths and of
//    the backward's memory part holds four consecutive units (a register quad) of one batch row, so each (array, quad)
//    is one 16-byte load with no lane transposes (round 6: the backward 7.78 -> 7.35 ms with all four arrays so; the
//    reduction's A staging then needed a lane-quad transpose per load and lost 3.77 -> 4.15 ms, so h_in stays in
//    slab blocks).  Byte offsets of register quad g4 of unit base ub_ (a multiple of 4), column c0 + 32 h + col_: lane
//    part quad_vbyte, uniform part quad_soff.
// Both keep a wave instruction's accesses in 512-byte or longer contiguous runs (HBM serves 128-byte row segments at
// ~4.0 TB/s, contiguous KBs at ~5.9: tools/load_probe2.hip).
// HIN_SLAB=0 (comparison builds): h_in in [256][M] rows (toued_gru_hin_slab() reports it to the host)
#ifndef HIN_SLAB
#define HIN_SLAB 1
#endif
TOUED_DEV unsigned slab_vbyte(int ub_, int col_) { return (unsigned)(ub_ * 128 + col_ * 4); }
TOUED_DEV unsigned slab_soff(long c0, int h, int uq) { return (unsigned)(((c0 >> 5) + h) * 32768L + uq * 128); }
TOUED_DEV unsigned quad_vbyte(int ub_, int col_) { return (unsigned)(((ub_ >> 2) * 32 + col_) * 16); }
TOUED_DEV unsigned quad_soff(long c0, int h, int g4) { return (unsigned)(((c0 >> 5) + h) * 32768L + g4 * 1024); }
// 16-byte store of a register quad (the r, z, hn saves).  Two wait states follow it before the scheduler may place
// anything that rewrites its data registers: on gfx950 a buffer_store_dwordx4 whose data VGPRs the next one or two
// instructions overwrite stored nondeterministic values (round 6, tools/det_fwd_diff.py: thousands of saved r / z / hn
// elements differed between identical forwards; the compiler inserts no wait state there).  b64 / b32 stores and
// b128 followed by s_nop 1 or s_nop 4 were bit-identical over repeated runs; the s_nop 1 form keeps b128's speed
// (forward 1.166-1.168 ms, b64 pairs 1.218-1.226, profiles/r06/r06t7_ab.log).
TOUED_DEV void st4(__amdgpu_buffer_rsrc_t r, unsigned vbyte, unsigned soff, const float (&v)[4]) {
  const u32x4 x = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
  __builtin_amdgcn_raw_buffer_store_b128(x, r, (int)vbyte, (int)soff, GRU_ST_AUX);
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 1");
  __builtin_amdgcn_sched_barrier(0);
}

// ------------------------------------------------------------------ forward
struct FwdArgs {
  int R, T, W, F;
  const float* X; long xs_f, xs_col;   // X[f*xs_f + (t*R + r)*xs_col]
  const uint8_t* done;                 // [N][T][W]
  const float4* A;                     // packed fwd fragments (f32 MFMA)
  const void* A6;                      // packed fwd fragments (bf16 split pieces, k_gru_fwd6)
  const float* eta; EtaOff o;
  float* pi_hat; float* y_hat;         // [T][R], [T][8][R]
  float* s_hin; float* s_r; float* s_z; float* s_n; float* s_hn;  // [256][M] with column base added
  long M;
  int rpc;                             // rows per parameter candidate (inference mode, ES)
  long a_stride4, eta_stride;          // per-candidate strides of A (float4 units) and eta (floats)
  int stagger;                         // inference mode: s_sleep(127) quanta half of the first round waits at start
};

#define NWAVE 8         // 512-thread workgroups: wave w owns units [32w, 32w+32)
#define NGRP (2 * NWAVE)

// NT row tiles of 32 rows per workgroup.  NT = 2 (one workgroup per CU, 256 VGPRs): every packed weight
// fragment feeds 8 MFMAs instead of 4, halving the L2 fragment stream and the per-step fixed costs.  A
// barrier after the contraction lets each lane overwrite its own h_in slot with the next carry in place, so
// h_out never sits in registers across the barrier (no spills at 256 VGPRs).
template <bool SAVE, int NT>
__global__ void __launch_bounds__(512, NT == 1 ? 4 : 1) k_gru_fwd(FwdArgs p) {
  constexpr int RBT = RB * NT;          // rows per workgroup
  constexpr int LDT = RBT + 1;          // padded LDS row (k-major [unit][row])
  __shared__ float hT[(HU + NAUG) * LDT];
  __shared__ float wh[HU * 9];
  __shared__ float hp[NGRP * 9 * RBT];
  __shared__ float hout[9 * RBT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hi = lane >> 5, col = lane & 31;
  const int r0 = blockIdx.x * RBT;
  const int R = p.R, T = p.T, W = p.W, F = p.F;
  int a_[NT], w_[NT];
#pragma unroll
  for (int h = 0; h < NT; ++h) {
    a_[h] = (r0 + RB * h) / W;
    w_[h] = r0 + RB * h + col - a_[h] * W;
  }
  const int cand = SAVE ? 0 : r0 / p.rpc;
  const float* eta = p.eta + (long)cand * p.eta_stride;
  for (int i = tid; i < HU * 9; i += 512) {
    const int u = i / 9, oo = i - u * 9;
    wh[i] = oo == 0 ? eta[p.o.pi_w + u] : eta[p.o.y_w + u * 8 + (oo - 1)];
  }
  for (int i = tid; i < (HU + NAUG) * LDT; i += 512) hT[i] = 0.0f;
  __syncthreads();
  if (tid < RBT) {
    const int t = T - 1;
    for (int f = 0; f < NAUG; ++f)
      hT[(HU + f) * LDT + tid] = f < F ? p.X[f * p.xs_f + ((size_t)t * R + r0 + tid) * p.xs_col] : (f == F ? 1.0f : 0.0f);
  }
  __syncthreads();
  const float bpi = eta[p.o.pi_b];
  const float4* Ab = p.A + (long)cand * p.a_stride4 + lane;
  const __amdgpu_buffer_rsrc_t rs_hin = rsrc_of(p.s_hin), rs_r = rsrc_of(p.s_r), rs_z = rsrc_of(p.s_z),
                               rs_n = rsrc_of(p.s_n), rs_hn = rsrc_of(p.s_hn);
  for (int s = 0; s < T; ++s) {
    const int t = T - 1 - s;
    floatx16 acc[4][NT];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int h = 0; h < NT; ++h)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[g][h][q] = 0.0f;
    // ---- recurrent contraction over the 256 h rows (kq 0..31): r, z, nh tiles of unit tile `wave`
    float4 an[3];
#pragma unroll
    for (int g = 0; g < 3; ++g) an[g] = Ab[((8 * g + wave) * KQF + 0) * 64];
#pragma unroll 2
    for (int kq = 0; kq < 32; ++kq) {
      float4 ac[3];
#pragma unroll
      for (int g = 0; g < 3; ++g) ac[g] = an[g];
      if (kq + 1 < 32) {
#pragma unroll
        for (int g = 0; g < 3; ++g) an[g] = Ab[((8 * g + wave) * KQF + kq + 1) * 64];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int h = 0; h < NT; ++h) {
          const float b = hT[(2 * (4 * kq + e) + hi) * LDT + RB * h + col];
#pragma unroll
          for (int g = 0; g < 3; ++g) {
            const float av = e == 0 ? ac[g].x : e == 1 ? ac[g].y : e == 2 ? ac[g].z : ac[g].w;
            acc[g][h] = mfma32(av, b, acc[g][h]);
          }
        }
      }
    }
    // ---- augmented rows (x features + bias): kq = 32 for all four gate kinds
    {
      float4 ag[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) ag[g] = Ab[((8 * g + wave) * KQF + 32) * 64];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int h = 0; h < NT; ++h) {
          const float b = hT[(HU + 2 * e + hi) * LDT + RB * h + col];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const float av = e == 0 ? ag[g].x : e == 1 ? ag[g].y : e == 2 ? ag[g].z : ag[g].w;
            acc[g][h] = mfma32(av, b, acc[g][h]);
          }
        }
      }
    }
    // ---- h_in(t) leaves from LDS (16-byte row quads) before hT is overwritten with h_in(t-1)
    if (SAVE) store_gate_lds<NT>(hT, rs_hin, p.M, (long)t * R + r0, wave, lane);
    __syncthreads();   // all MFMA and h_in reads of hT done: the carry can overwrite it in place
    if (t >= 1 && tid < RBT) {
      for (int f = 0; f < F; ++f)
        hT[(HU + f) * LDT + tid] = p.X[f * p.xs_f + ((size_t)(t - 1) * R + r0 + tid) * p.xs_col];
    }
    // ---- gate maths (lane = row, register q = unit offset)
    const long cbase = (long)t * R;                              // uniform column base
    const float* whl = wh + (32 * wave + 4 * hi) * 9;
#pragma unroll
    for (int h = 0; h < NT; ++h) {
      const unsigned vbyte = (unsigned)(((long)(32 * wave + 4 * hi) * p.M + r0 + RB * h + col) * 4);
      float* hTl = hT + (32 * wave + 4 * hi) * LDT + RB * h + col;
      const bool dn = (t >= 1) ? p.done[((size_t)a_[h] * T + (t - 1)) * W + w_[h]] != 0 : false;
      float hp_loc[9];
#pragma unroll
      for (int oo = 0; oo < 9; ++oo) hp_loc[oo] = 0.0f;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const float rg = sigm(acc[0][h][q]);
        const float zg = sigm(acc[1][h][q]);
        const float hn = acc[2][h][q];
        const float ng = tanh_f(acc[3][h][q] + rg * hn);
        const float hin = hTl[qunit(q) * LDT];    // h_in(t) (masked carry)
        const float hh = (1.0f - zg) * ng + zg * hin;
        hTl[qunit(q) * LDT] = dn ? 0.0f : hh;    // next-step carry h_in(t-1) = where(d_{t-1}, 0, h_out(t))
        if (SAVE) {
          const unsigned so = (unsigned)(((long)qunit(q) * p.M + cbase) * 4);
          st_u(rs_r, vbyte, so, rg);
          st_u(rs_z, vbyte, so, zg);
          st_u(rs_n, vbyte, so, ng);
          st_u(rs_hn, vbyte, so, hn);
        }
        const float rl = fmaxf(hh, 0.0f);
#pragma unroll
        for (int oo = 0; oo < 9; ++oo) hp_loc[oo] += rl * whl[qunit(q) * 9 + oo];
      }
#pragma unroll
      for (int oo = 0; oo < 9; ++oo) hp[((2 * wave + hi) * 9 + oo) * RBT + RB * h + col] = hp_loc[oo];
    }
    __syncthreads();   // head partials and the carry visible
    for (int i = tid; i < 9 * RBT; i += 512) {
      const int oo = i / RBT, c = i - oo * RBT;
      float v = oo == 0 ? bpi : eta[p.o.y_b + oo - 1];
#pragma unroll
      for (int gq = 0; gq < NGRP; ++gq) v += hp[(gq * 9 + oo) * RBT + c];
      hout[i] = v;
    }
    __syncthreads();
    if (tid < RBT) {
      const long ob = (long)t * R + r0 + tid;
      p.pi_hat[ob] = hout[tid];
      float m = -__builtin_inff();
      for (int j = 0; j < 8; ++j) m = fmaxf(m, hout[(j + 1) * RBT + tid]);
      float e[8], ssum = 0.0f;
      for (int j = 0; j < 8; ++j) { e[j] = __expf(hout[(j + 1) * RBT + tid] - m); ssum += e[j]; }
      const float inv = 1.0f / ssum;
      for (int j = 0; j < 8; ++j) p.y_hat[((long)t * 8 + j) * R + r0 + tid] = e[j] * inv;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ forward on the 16-bit matrix cores
// k_gru_fwd6: one 512-thread workgroup owns 64 rows (two 32-row tiles) for the whole T-step scan; wave w owns
// units [32w, 32w + 32), so its accumulators are {r, z, W_hn h + b_hn, W_in x + b_in} x 2 row tiles.  Per step:
//   contraction over k = 256 h units (16 k-steps of 16, fp16 pairs) + one augmented k-step [x (F <= 7); 1; 0...]
//     (bf16 triples): A fragments (weights scaled, split and packed by k_pack_fwd6, 16 B per lane and piece)
//     stream from L2 one k-step ahead; B fragments (fp16 pieces of 2^14 h in LDS [row][unit], 528-byte rows:
//     the 16 lanes of a read hit 16 distinct bank quads) are read one k-step ahead; each A fragment feeds both
//     row tiles;
//   barrier; exact power-of-two unscale; gate maths in the accumulator layout (lane = row, register = unit);
//   h_in rebuilt exactly ((x0 + x1) + r == 2^14 h); the new carry split and written back in place (each
//   (row, unit) has one owner lane); saves r, z, n, W_hn h + b_hn, h_in for the backward; head partials;
//   barrier; head reduce + softmax.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

#define F6_HP 264        // carry image row pitch (16-bit elements): 528 B
#define F6_NFH (16 * 8 * 3 * 2)     // h-part fragments [ks][unit tile][gate r|z|hn][fp16 piece], 1 KiB each
#define F6_NFA (8 * 4 * 3)          // augmented fragments [unit tile][gate r|z|hn|ni][bf16 piece]
#define F6_SCALES ((F6_NFH + F6_NFA) * 256)   // float offset of the per-(gate, unit) weight scales 2^s [4][256]
// f32 fragments of the augmented k-step (input weights and biases of r, z and the hn bias, scaled by 2^s):
// [unit tile][gate r|z|hn][lane] float4 over kk = 0..3 of A[i = unit][k = 2 kk + (l >> 5)] (k < F: W_g[k][u],
// k = 7: the bias), for the f32-MFMA input k-step (FWD_AUG32)
#define F6_A32 (F6_SCALES + 4 * HU)
#define F6_FLOATS (F6_A32 + 8 * 3 * 64 * 4)   // packed size in floats (1 KiB fragment = 256 floats)
#define F6_NGRP (16 * 8 * 3 + 8 * 4 + 8 * 3)  // k_pack_fwd6's fragment groups: h part, bf16 augmented, f32 augmented
#define HSCALE 16384.0f  // carry scale 2^14: |h| < 1 -> |2^14 h| < 2^14, inside the fp16 range

template <typename V>
TOUED_DEV void split3v(float x, V& p0, V& p1, V& p2, int e) {
  const __bf16 h = (__bf16)x;
  const float r1 = x - (float)h;
  const __bf16 m = (__bf16)r1;
  p0[e] = h;
  p1[e] = m;
  p2[e] = (__bf16)(r1 - (float)m);
}

// fp16 pair of an f32 value y (|y| < 65504): y ~ x0 + x1 to 2^-22 relative (normal range)
template <typename V>
TOUED_DEV void split2h(float y, V& x0, V& x1, int e) {
  const _Float16 a = (_Float16)y;
  x0[e] = a;
  x1[e] = (_Float16)(y - (float)a);
}

// carry piece triple of h: fp16 x0, x1 of y = 2^14 h (the MFMA operand) and the bf16 residual r = y - x0 - x1,
// so that (x0 + x1) + r == y exactly for |h| >= 2^-24 (r then has <= 8 significant bits; below, |r| < 2^-25
// and the reconstruction error is < 2^-47 absolute in h)
TOUED_DEV void split_carry(float h, f16x4& x0, f16x4& x1, bf16x4& r, int e) {
  const float y = h * HSCALE;
  const _Float16 a = (_Float16)y;
  const float d = y - (float)a;
  const _Float16 b = (_Float16)d;
  x0[e] = a;
  x1[e] = b;
  r[e] = (__bf16)(d - (float)b);
}

// per-(gate, output unit) weight scale 2^s: s = 14 - e with max_k |W_g[k][u]| < 2^e (clamped to [-30, 20]), so
// the scaled row's fp16 pieces stay below 2^14 and its small entries keep their relative precision; the ni gate
// (no h part) uses s = 0.  One thread per (gate, unit) and candidate (blockIdx.y).
__global__ void __launch_bounds__(256) k_fwd6_scales(const float* __restrict__ eta, EtaOff o, float* __restrict__ out,
                                                     long eta_stride, long out_stride) {
  // block (gate, 64-unit group, candidate): thread = (unit, k quarter); coalesced over units
  __shared__ float red[4][64];
  const int g = blockIdx.x >> 2, u = 64 * (blockIdx.x & 3) + (threadIdx.x & 63), kq = threadIdx.x >> 6;
  eta += (long)blockIdx.y * eta_stride;
  out += (long)blockIdx.y * out_stride;
  float m = 0.0f;
  if (g < 3) {
    const int base = g == 0 ? o.hr_w : g == 1 ? o.hz_w : o.hn_w;
    for (int k = 64 * kq; k < 64 * kq + 64; ++k) m = fmaxf(m, fabsf(eta[base + k * HU + u]));
  }
  red[kq][threadIdx.x & 63] = m;
  __syncthreads();
  if (kq == 0) {
    m = fmaxf(fmaxf(red[0][threadIdx.x], red[1][threadIdx.x]), fmaxf(red[2][threadIdx.x], red[3][threadIdx.x]));
    int sc = 0;
    if (m > 0.0f && m <= 3.0e38f) {
      int e;
      frexpf(m, &e);          // m < 2^e
      sc = min(20, max(-30, 14 - e));
    }
    out[g * HU + u] = ldexpf(1.0f, sc);
  }
}

// one thread per (fragment group, lane): fragment group = (ks, ut, g) for the h part or (ut, g) for the
// augmented rows; lane l holds A[i = unit 32 ut + (l & 31)][k = 8 (l >> 5) + e], e = 0..7.  Every row is
// scaled by its 2^s (k_fwd6_scales, at F6_SCALES of the same buffer): the h part as two fp16 pieces, the
// augmented rows (input weights and biases, multiplied with 2^14 x on the B side) as three bf16 pieces.
__global__ void k_pack_fwd6(const float* __restrict__ eta, EtaOff o, int F, bf16x8* __restrict__ out,
                            long eta_stride, long out_stride16) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  eta += (long)blockIdx.y * eta_stride;            // candidate blockIdx.y (ES); 0 for the shared eta
  out += (long)blockIdx.y * out_stride16;
  const float* scl = reinterpret_cast<const float*>(out) + F6_SCALES;
  const int ngrp_h = 16 * 8 * 3, ngrp = ngrp_h + 8 * 4;
  if (gid >= F6_NGRP * 64) return;
  const int lane = gid & 63, grp = gid >> 6;
  if (grp < ngrp_h) {
    const int g = grp % 3, ut = (grp / 3) % 8, ks = grp / 24;
    const int u = 32 * ut + (lane & 31);
    const int base = g == 0 ? o.hr_w : g == 1 ? o.hz_w : o.hn_w;
    const float sg = scl[g * HU + u];
    f16x8 pc[2];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 16 * ks + 8 * (lane >> 5) + e;
      split2h(eta[base + k * HU + u] * sg, pc[0], pc[1], e);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) out[(long)(grp * 2 + q) * 64 + lane] = __builtin_bit_cast(bf16x8, pc[q]);
  } else if (grp >= ngrp) {
    // the f32 augmented fragments (FWD_AUG32)
    const int ga = grp - ngrp, g = ga % 3, ut = ga / 3;
    const int u = 32 * ut + (lane & 31);
    const float sg = scl[g * HU + u];
    float v[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int k = 2 * kk + (lane >> 5);
      float x = 0.0f;
      if (k < F) {
        if (g == 0) x = eta[o.ir_w + k * HU + u];
        else if (g == 1) x = eta[o.iz_w + k * HU + u];
      } else if (k == 7) {
        x = g == 0 ? eta[o.ir_b + u] : g == 1 ? eta[o.iz_b + u] : eta[o.hn_b + u];
      }
      v[kk] = x * sg;   // a power of two: exact
    }
    reinterpret_cast<float4*>(out)[F6_A32 / 4 + (ut * 3 + g) * 64 + lane] = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    const int ga = grp - ngrp_h, g = ga % 4, ut = ga / 4;
    const int u = 32 * ut + (lane & 31);
    const float sg = scl[g * HU + u];
    bf16x8 pc[3];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int f = 8 * (lane >> 5) + e;
      float x = 0.0f;
      if (f < F) {
        if (g == 0) x = eta[o.ir_w + f * HU + u];
        else if (g == 1) x = eta[o.iz_w + f * HU + u];
        else if (g == 3) x = eta[o.in_w + f * HU + u];
      } else if (f == F) {
        x = g == 0 ? eta[o.ir_b + u] : g == 1 ? eta[o.iz_b + u] : g == 2 ? eta[o.hn_b + u] : eta[o.in_b + u];
      }
      split3v(x * sg, pc[0], pc[1], pc[2], e);
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) out[(long)(F6_NFH + ga * 3 + q) * 64 + lane] = pc[q];
  }
}

// per-input-unit scale 2^s of the backward's fp16 weight rows: s = 14 - e with
// max_k max(|W_r[i][k]|, |W_z[i][k]|, |W_hn[i][k]|) < 2^e, clamped to [-30, 20] (the forward's k_fwd6_scales rule)
__global__ void __launch_bounds__(256) k_bwd6_scales(const float* __restrict__ eta, EtaOff o, float* __restrict__ out) {
  // one wave per input unit i: lane-strided contiguous reads of the three rows, wave max
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (i >= HU) return;
  float m = 0.0f;
  for (int k = lane; k < HU; k += 64)
    m = fmaxf(m, fmaxf(fabsf(eta[o.hr_w + i * HU + k]),
                       fmaxf(fabsf(eta[o.hz_w + i * HU + k]), fabsf(eta[o.hn_w + i * HU + k]))));
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) m = fmaxf(m, __shfl_xor(m, d));
  if (lane == 0) {
    int sc = 0;
    if (m > 0.0f && m <= 3.0e38f) {
      int e;
      frexpf(m, &e);
      sc = min(20, max(-30, 14 - e));
    }
    out[i] = ldexpf(1.0f, sc);
  }
}

// backward A fragments A[i = input unit 32 ut + (l & 31)][k = gate unit 16 ks + 8 (l >> 5) + e] = W_g[i][k] of
// the three gates, row i scaled by its 2^s (k_bwd6_scales), as two fp16 pieces in piece slots 0, 1 of the
// [ks][ut][g][piece] layout (slot 2 unused)
__global__ void k_pack_bwd6(const float* __restrict__ eta, EtaOff o, __bf16* __restrict__ out8) {
  typedef __bf16 v8 __attribute__((ext_vector_type(8)));
  v8* out = reinterpret_cast<v8*>(out8);
  const float* scl = reinterpret_cast<const float*>(out8) + B6_SCALES;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= 16 * 8 * 3 * 64) return;
  const int lane = gid & 63, grp = gid >> 6;
  const int g = grp % 3, ut = (grp / 3) % 8, ks = grp / 24;
  const int u = 32 * ut + (lane & 31);
  const int base = g == 0 ? o.hr_w : g == 1 ? o.hz_w : o.hn_w;
  const float sg = scl[u];
  f16x8 pc[2];
#pragma unroll
  for (int e = 0; e < 8; ++e) split2h(eta[base + u * HU + 16 * ks + 8 * (lane >> 5) + e] * sg, pc[0], pc[1], e);
#pragma unroll
  for (int q = 0; q < 2; ++q) out[(long)(grp * 3 + q) * 64 + lane] = __builtin_bit_cast(v8, pc[q]);
}

TOUED_DEV floatx16 mfma_bf32(bf16x8 a, bf16x8 b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// a.b from two fp16 pieces each, a1 b1 (< 2^-22 relative) dropped, smallest products first
TOUED_DEV floatx16 mfma3h(const f16x8 (&a)[2], const f16x8 (&b)[2], floatx16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[0], c, 0, 0, 0);
  return c;
}
// a.b from the pieces, smallest products first
TOUED_DEV floatx16 mfma6(const bf16x8 (&a)[3], const bf16x8 (&b)[3], floatx16 c) {
  c = mfma_bf32(a[2], b[0], c);
  c = mfma_bf32(a[1], b[1], c);
  c = mfma_bf32(a[0], b[2], c);
  c = mfma_bf32(a[1], b[0], c);
  c = mfma_bf32(a[0], b[1], c);
  c = mfma_bf32(a[0], b[0], c);
  return c;
}

#ifdef FWD_STAMPS
// timing instrumentation (tools/fwd_stamps.py, built by tools/build_variant.py gru.hip FWD_STAMPS=1): thread 0 of
// workgroups < 64 records s_memtime at 6 points of every step (of the last launch of either instance)
__device__ unsigned long long g_fwd_stamps[64 * 32 * 6];
#define FWD_STAMP(ph)                                                                                  \
  do {                                                                                                 \
    if (blockIdx.x < 64 && tid == 0 && s < 32)                                                         \
      g_fwd_stamps[(blockIdx.x * 32 + s) * 6 + (ph)] = __builtin_amdgcn_s_memtime();                   \
  } while (0)
// the ping-pong schedule (FWD_PP): lane 0 of waves 0 and 4 record the start and end of each of their three pieces of
// work per step (half 0: contraction k 0-7, k 8-15 + heads, gate maths; half 1: gate maths of the step before,
// k 0-7, k 8-15), ordered clock reads
__device__ unsigned long long g_fwd_pp[64 * 32 * 2 * 6];
// the lockstep gate maths' inside (thread 0): after the done flags + gate_ain, after row tile 0, after row tile 1
__device__ unsigned long long g_fwd_gm[64 * 32 * 4];
#define GM_STAMP(k)                                                                                    \
  do {                                                                                                 \
    if (blockIdx.x < 64 && tid == 0 && s < 32) g_fwd_gm[(blockIdx.x * 32 + s) * 4 + (k)] = fwd_clock(); \
  } while (0)
TOUED_DEV unsigned long long fwd_clock() {
  unsigned long long c;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c));
  return c;
}
#define PP_STAMP(s_, k)                                                                                \
  do {                                                                                                 \
    if (blockIdx.x < 64 && lane == 0 && (wave & 3) == 0 && (s_) >= 0 && (s_) < 32)                     \
      g_fwd_pp[((blockIdx.x * 32 + (s_)) * 2 + grp) * 6 + (k)] = fwd_clock();                          \
  } while (0)
#else
#define FWD_STAMP(ph) do {} while (0)
#define PP_STAMP(s_, k) do {} while (0)
#define GM_STAMP(k) do {} while (0)
#endif

#ifndef FWD_AUG32
#define FWD_AUG32 1
#endif
#ifndef FWD_NOSAVE
#define FWD_NOSAVE 0   // timing studies only: 1 = no saves, 2 = h_in only (the backward then reads stale data)
#endif
#ifndef FWD_HDEFER
#define FWD_HDEFER 1   // the head reduce + softmax of step s at the end of step s + 1's contraction (wave 0)
#endif
#ifndef FWD_XFIRST
#define FWD_XFIRST 0   // comparison runs: x(t) issued before the ring's lead fragments (the round-4 order)
#endif
#ifndef FWD_PP
#define FWD_PP 0       // the two halves of the workgroup one interval apart (gate maths beside the partner's MFMAs)
#endif
#ifndef FWD_PP_PRIO
#define FWD_PP_PRIO 0  // FWD_PP: the gate maths' issue priority over the partner wave's contraction
#endif
#ifndef FWD_XOR32
#define FWD_XOR32 0    // the gate maths' head-partial fold through xor32 (no spilled lane index, no store drain)
#endif
#ifndef FWD_LANEB
#define FWD_LANEB 0
#endif
#ifndef FWD_CAND0
#define FWD_CAND0 0    // timing study only: the per-candidate instance reads candidate 0's fragments everywhere
#endif
template <bool SAVE>
__global__ void __launch_bounds__(512, 1) k_gru_fwd6(FwdArgs p) {
  constexpr bool A32 = FWD_AUG32 && !SAVE;   // the per-candidate (ES) instance: f32-MFMA augmented k-step
  // carry image [row][unit]: slots 0, 1 the fp16 pieces of 2^14 h (MFMA B operand), slot 2 the bf16 residual
  __shared__ __attribute__((aligned(16))) __bf16 hB[3][64 * F6_HP];
  __shared__ __attribute__((aligned(16))) float wh[HU * 12];          // head weights [unit][pi | y0..y7 | pad]
  __shared__ __attribute__((aligned(16))) float usc[4 * HU];          // accumulator unscale 2^-(s + 14) [gate][unit]
  // head partials [wave][output][row]; FWD_HDEFER: two buffers (step parity), reduced by wave 0 at the end of the next
  // step's contraction, where it waits for the other waves' MFMAs anyway
  __shared__ float hp[(FWD_HDEFER ? 2 : 1) * 8 * 9 * 64];
  __shared__ float hout[FWD_HDEFER ? 1 : 9 * 64];
  __shared__ float wIs[8 * 4 * 64];     // gate_ain's W_in fragments [wave][kk][lane] (registers are the bound)
  __shared__ float hbias[9];            // pi_b, y_b[0..7] (the head reduce reads them from LDS)
  const int tid = threadIdx.x, lane = tid & 63, hi = lane >> 5, col = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r0 = blockIdx.x * 64;
  const int R = p.R, T = p.T, W = p.W, F = p.F;
  int a_[2], w_[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    a_[h] = (r0 + RB * h) / W;
    w_[h] = r0 + RB * h + col - a_[h] * W;
  }
  // per-candidate parameters in the ES inference mode (rows [c * rpc, (c + 1) * rpc) use candidate c)
  const int cand = SAVE ? 0 : r0 / p.rpc;
  const float* eta = p.eta + (long)cand * p.eta_stride;
  // FWD_CAND0 (timing study only, wrong results): every workgroup streams candidate 0's packed fragments, which then
  // stay L2-resident -- the per-candidate fragment stream's cost is the difference to the production kernel
  const float* A6c = reinterpret_cast<const float*>(p.A6) + (long)(FWD_CAND0 ? 0 : cand) * p.a_stride4 * 4;
  for (int i = tid; i < HU * 12; i += 512) {
    const int u = i / 12, oo = i - u * 12;
    wh[i] = oo == 0 ? eta[p.o.pi_w + u] : oo < 9 ? eta[p.o.y_w + u * 8 + (oo - 1)] : 0.0f;
  }
  for (int i = tid; i < 4 * HU; i += 512) usc[i] = 1.0f / (A6c[F6_SCALES + i] * HSCALE);   // powers of two: exact
  if (tid < 9) hbias[tid] = tid == 0 ? eta[p.o.pi_b] : eta[p.o.y_b + tid - 1];
  {
    float wI[4];
    load_win_frags(wI, eta, p.o, F, wave, lane);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) wIs[(wave * 4 + kk) * 64 + lane] = wI[kk];
  }
  {
    uint4* z = reinterpret_cast<uint4*>(&hB[0][0]);
    for (int i = tid; i < 3 * 64 * F6_HP / 8; i += 512) z[i] = make_uint4(0u, 0u, 0u, 0u);
  }
  // x(t) of row `row` -> the augmented image: [x_0 .. x_{F-1}, 1, 0 ...]
  // per-row global reads through wave-uniform buffer descriptors with 32-bit offsets (64-bit per-lane
  // addresses kept across the step loop spill)
  const __amdgpu_buffer_rsrc_t rs_X = rsrc_of(p.X);
  const __amdgpu_buffer_rsrc_t rs_done = rsrc_of(reinterpret_cast<const float*>(p.done));
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rs_A = rsrc_of(A6c);
  const unsigned vA = (unsigned)lane * 16;
  auto ldA = [&](int frag) {
    const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs_A, (int)vA, frag * 1024, 0);
    return __builtin_bit_cast(bf16x8, x);
  };
  auto ldAh = [&](int frag) {
    const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs_A, (int)vA, frag * 1024, 0);
    return __builtin_bit_cast(f16x8, x);
  };
  const __amdgpu_buffer_rsrc_t rs_hin = rsrc_of(p.s_hin), rs_r = rsrc_of(p.s_r), rs_z = rsrc_of(p.s_z),
                               rs_hn = rsrc_of(p.s_hn);
  // ES candidates: the per-candidate fragment stream from the Infinity Cache is what a step's contraction waits on,
  // and the gate maths leave it idle; half of the first round's workgroups (alternate CUs of every XCD) start about
  // half a step late so the two halves contract at different times (later rounds inherit the offset)
  if (p.stagger > 0 && blockIdx.x < 256 && ((blockIdx.x >> 3) & 1))
    for (int i = 0; i < p.stagger; ++i) __builtin_amdgcn_s_sleep(127);
  // FWD_HDEFER: step s_'s heads from its partials (wave 0, lane = row): the bias plus the eight waves' partials in
  // wave order, then pi_hat and the softmax of the eight y logits -- the arithmetic of the reduce below, in one lane
  auto head_out = [&](int s_) {
    const int tl = lane_now(), t_ = T - 1 - s_;
    const float* hb = hp + (s_ & 1) * 4608;
    float v[9];
#pragma unroll
    for (int oo = 0; oo < 9; ++oo) {
      v[oo] = hbias[oo];
#pragma unroll
      for (int gq = 0; gq < 8; ++gq) v[oo] += hb[(gq * 9 + oo) * 64 + tl];
    }
    p.pi_hat[(long)t_ * R + r0 + tl] = v[0];
    float m = -__builtin_inff();
    for (int j = 0; j < 8; ++j) m = fmaxf(m, v[j + 1]);
    float e[8], ssum = 0.0f;
    for (int j = 0; j < 8; ++j) { e[j] = __expf(v[j + 1] - m); ssum += e[j]; }
    const float inv = 1.0f / ssum;
    for (int j = 0; j < 8; ++j) p.y_hat[((long)t_ * 8 + j) * R + r0 + tl] = e[j] * inv;
  };
if constexpr (FWD_PP && SAVE) {   // (C2 instance only: the per-candidate one spills with it)
  // ---- ping-pong schedule: the workgroup's two halves (waves 0-3 own units 0-127 = k-steps 0-7 of the carry, waves
  // 4-7 units 128-255 = k-steps 8-15) run one interval apart, three intervals per step with a barrier after each:
  //   interval   waves 0-3 (half 0)                          waves 4-7 (half 1)
  //   1          contraction k 0-7 of step s (own units)     gate maths of step s-1: writes units 128-255
  //   2          contraction k 8-15 + augmented of step s    contraction k 0-7 of step s
  //   3          gate maths of step s: writes units 0-127    contraction k 8-15 + augmented of step s
  // so each SIMD (waves w and w + 4) has one wave's gate maths (VALU, saves) beside its partner's matrix work in two
  // of the three intervals, where the lockstep order runs them one after the other.  Every interval reads carry units
  // that no wave writes in it (the table above), so the carry stays single-buffered in place; the k-order of the
  // contraction is unchanged.  Heads: step s's partials (both halves) are complete after interval 1 of step s + 1;
  // wave 0 reduces them in its interval 2 (FWD_HDEFER's double buffer).
  static_assert(FWD_HDEFER, "FWD_PP defers the heads");
  const int grp = wave >> 2;
  floatx16 acc[3][2];   // r, z, W_hn h + b_hn (the n gate's input part is gate_ain, on the VALU)
  float xv[2][7];
  f16x8 A0[3][2], A1[3][2], B[2][2];
  auto fragA = [&](int ks, int g, int q) { return ((ks * 8 + wave) * 3 + g) * 2 + q; };
  auto fragAug = [&](int g, int q) { return F6_NFH + (wave * 4 + g) * 3 + q; };
  auto load_B = [&](int ks, int h) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
      B[h][q] = *reinterpret_cast<const f16x8*>(&hB[q][(RB * h + col) * F6_HP + 16 * ks + 8 * hi]);
  };
  // one k-step: refill its A ring slot two k-steps ahead (reload), load the next k-step's B fragments (nextB)
  auto kstep = [&](int ks, f16x8 (&Ar)[3][2], bool reload, bool nextB) {
#pragma unroll
    for (int g = 0; g < 3; ++g) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        acc[g][h] = mfma3h(Ar[g], B[h], acc[g][h]);
        if (g == 2 && nextB) load_B(ks + 1, h);
      }
      if (reload) {
#pragma unroll
        for (int q = 0; q < 2; ++q) Ar[g][q] = ldAh(fragA(ks + 2, g, q));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // the contraction's first half: x(t), the ring's lead fragments, k-steps 0-7 (carry units 0-127)
  auto c_first = [&](int s) {
    const int t = T - 1 - s;
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[g][h][q] = 0.0f;
      {
        auto ring = [&] {
  #pragma unroll
          for (int g = 0; g < 3; ++g)
  #pragma unroll
            for (int q = 0; q < 2; ++q) {
              A0[g][q] = ldAh(fragA(0, g, q));
              A1[g][q] = ldAh(fragA(1, g, q));
            }
        };
        if (!FWD_XFIRST) ring();
  #pragma unroll
        for (int h = 0; h < 2; ++h)
  #pragma unroll
          for (int f = 0; f < 7; ++f) {
            const int fc = f < F ? f : F - 1;
            xv[h][f] = ld_u(rs_X, (unsigned)((RB * h + col) * p.xs_col * 4),
                            (unsigned)((fc * p.xs_f + ((long)t * R + r0) * p.xs_col) * 4));
          }
        if (FWD_XFIRST) ring();
      }
    load_B(0, 0);
    load_B(0, 1);
#pragma nounroll
    for (int kp = 0; kp < 3; ++kp) {
      kstep(2 * kp, A0, true, true);
      kstep(2 * kp + 1, A1, true, true);
    }
    kstep(6, A0, true, true);
    kstep(7, A1, true, false);   // (k-step 8's B: units 128-143, written by the other half in this interval)
  };
  // the second half: k-steps 8-15 (carry units 128-255) and the augmented k-step
  auto c_second = [&](int s) {
    load_B(8, 0);
    load_B(8, 1);
#pragma nounroll
    for (int kp = 4; kp < 7; ++kp) {
      kstep(2 * kp, A0, true, true);
      kstep(2 * kp + 1, A1, true, true);
    }
    kstep(14, A0, false, true);
      f16x8 (&A)[3][2] = A1;   // k-step 15
      if (A32) {
        // the augmented k-step on the f32 MFMA (exact products): A = the scaled input weights and biases (one 16-byte
        // fragment per gate, 3 KB per wave-step instead of the bf16 triple's 12 KB: the ES candidates' per-step stream
        // from the Infinity Cache is what this kernel waits on), B = 2^14 [x_k (k < F), 1 (k = 7)]
        float4 a32[3];
  #pragma unroll
        for (int g = 0; g < 3; ++g)
          a32[g] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  rs_A, (int)vA, (F6_A32 + (wave * 3 + g) * 256) * 4, 0));
  #pragma unroll
        for (int g = 0; g < 3; ++g) {
  #pragma unroll
          for (int h = 0; h < 2; ++h) acc[g][h] = mfma3h(A[g], B[h], acc[g][h]);
          __builtin_amdgcn_sched_barrier(0);
        }
  #pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const int k = 2 * kk + hi;
          float bx[2];
  #pragma unroll
          for (int h = 0; h < 2; ++h) {
            // static indices: the lane's k = 2 kk + hi picks between two registers (a lane-dependent index puts xv in
            // scratch: 64 bytes per lane, C4's forward 2.22 -> 2.65 ms while xv lived outside the step loop)
            const float xs = hi ? xv[h][2 * kk + 1 < 7 ? 2 * kk + 1 : 6] : xv[h][2 * kk];
            bx[h] = (k < F ? xs : (k == 7 ? 1.0f : 0.0f)) * HSCALE;
          }
  #pragma unroll
          for (int g = 0; g < 3; ++g) {
            const float av = kk == 0 ? a32[g].x : kk == 1 ? a32[g].y : kk == 2 ? a32[g].z : a32[g].w;
  #pragma unroll
            for (int h = 0; h < 2; ++h) acc[g][h] = mfma32(av, bx[h], acc[g][h]);
          }
        }
      } else {
      // last carry k-step; each gate's augmented fragments (three bf16 pieces) load behind its MFMAs
      bf16x8 Aa[3][3], Ba[2][3];
  #pragma unroll
      for (int g = 0; g < 3; ++g) {
  #pragma unroll
        for (int h = 0; h < 2; ++h) acc[g][h] = mfma3h(A[g], B[h], acc[g][h]);
  #pragma unroll
        for (int q = 0; q < 3; ++q) Aa[g][q] = ldA(fragAug(g, q));
        __builtin_amdgcn_sched_barrier(0);
      }
      // augmented k-step: B = bf16 pieces of 2^14 [x, 1, 0 ...]
  #pragma unroll
      for (int h = 0; h < 2; ++h)
  #pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = hi ? 0.0f : e < F ? xv[h][e < 7 ? e : 6] : (e == F ? 1.0f : 0.0f);
          split3v(v * HSCALE, Ba[h][0], Ba[h][1], Ba[h][2], e);
        }
  #pragma unroll
      for (int g = 0; g < 3; ++g) {
  #pragma unroll
        for (int h = 0; h < 2; ++h) acc[g][h] = mfma6(Aa[g], Ba[h], acc[g][h]);
      }
      }
  };
  auto g_maths = [&](int s) {
    const int t = T - 1 - s;
    // (FWD_PP_PRIO: the gate maths' VALU ahead of the partner's MFMA issue on the SIMD)
    if (FWD_PP_PRIO) __builtin_amdgcn_s_setprio(FWD_PP_PRIO);
      // ---- gate maths (lane = row 32h + col, register q = unit 32 wave + 4 hi + qunit(q))
      floatx16 ain[2];
      // done flags d_{t-1} of the lane's two rows, issued before the saves so their wait drains nothing else
      // (lane offset re-derived here: a spilled copy's reload would wait on every outstanding access)
      bool dnf[2];
  #pragma unroll
      for (int h = 0; h < 2; ++h)
        dnf[h] = (t >= 1) ? __builtin_amdgcn_raw_buffer_load_b8(
                                rs_done, lane_now() & 31, (int)(((long)a_[h] * T + (t - 1)) * W + r0 + RB * h - a_[h] * W),
                                0) != 0
                          : false;
      float wI[4];
      {
        const int ln = lane_now();
  #pragma unroll
        for (int kk = 0; kk < 4; ++kk) wI[kk] = wIs[(wave * 4 + kk) * 64 + ln];
      }
  #pragma unroll
      for (int h = 0; h < 2; ++h) ain[h] = gate_ain(wI, F, hi, [&](int k) { return xv[h][k < 7 ? k : 6]; });
      const long cbase = (long)t * R;
      const int ub = 32 * wave + 4 * hi;
      const float4* whl = reinterpret_cast<const float4*>(wh + ub * 12);
  #pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int row = RB * h + col;
        const bool dn = dnf[h];
        const unsigned vq = quad_vbyte(ub, col), vslab = slab_vbyte(ub, col);
        float hp_loc[9];
  #pragma unroll
        for (int oo = 0; oo < 9; ++oo) hp_loc[oo] = 0.0f;
  #pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          // four consecutive units ub + 8 g4 .. +3 of this row: h_in pieces, then the new carry's pieces
          const int ho = row * F6_HP + ub + 8 * g4;
          const f16x4 h0 = *reinterpret_cast<const f16x4*>(&hB[0][ho]);
          const f16x4 h1 = *reinterpret_cast<const f16x4*>(&hB[1][ho]);
          const bf16x4 hr = *reinterpret_cast<const bf16x4*>(&hB[2][ho]);
          // the saves of this register quad: h_in (rebuilt exactly from its pieces) per unit in its slab blocks; r, z,
          // hn one 16-byte store each in their unit-quad blocks (quad_soff) after the gate maths
          const unsigned sq = quad_soff(cbase + r0, h, g4);
          float sv[3][4];
          float us[3][4];
  #pragma unroll
          for (int g = 0; g < 3; ++g) {
            const float4 v = *reinterpret_cast<const float4*>(&usc[g * HU + ub + 8 * g4]);
            us[g][0] = v.x; us[g][1] = v.y; us[g][2] = v.z; us[g][3] = v.w;
          }
          f16x4 n0, n1;
          bf16x4 nr;
  #pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int q = 4 * g4 + e;
            const float rg = sigm_r(acc[0][h][q] * us[0][e]);
            const float zg = sigm_r(acc[1][h][q] * us[1][e]);
            const float hn = acc[2][h][q] * us[2][e];
            const float ng = gate_n(ain[h][q], rg, hn);
            const float hin = (((float)h0[e] + (float)h1[e]) + (float)hr[e]) * (1.0f / HSCALE);   // exact
            const float hh = (1.0f - zg) * ng + zg * hin;
            split_carry(dn ? 0.0f : hh, n0, n1, nr, e);   // carry h_in(t-1) = where(d_{t-1}, 0, h_out(t))
            sv[0][e] = rg;
            sv[1][e] = zg;
            sv[2][e] = hn;   // n is recomputed by the backward (gate_n)
            if (SAVE && FWD_NOSAVE != 1) {   // (FWD_NOSAVE, timing studies only: 1 = no saves, 2 = h_in only)
              if (HIN_SLAB) st_u(rs_hin, vslab, slab_soff(cbase + r0, h, qunit(q)), hin);
              else st_u(rs_hin, (unsigned)(((long)ub * p.M + r0 + row) * 4), (unsigned)(((long)qunit(q) * p.M + cbase) * 4), hin);
            }
            const float rl = fmaxf(hh, 0.0f);
            const float4 w0 = whl[qunit(q) * 3], w1 = whl[qunit(q) * 3 + 1], w2 = whl[qunit(q) * 3 + 2];
            hp_loc[0] += rl * w0.x; hp_loc[1] += rl * w0.y; hp_loc[2] += rl * w0.z;
            hp_loc[3] += rl * w0.w; hp_loc[4] += rl * w1.x; hp_loc[5] += rl * w1.y;
            hp_loc[6] += rl * w1.z; hp_loc[7] += rl * w1.w; hp_loc[8] += rl * w2.x;
          }
          if (SAVE && FWD_NOSAVE == 0) {   // (FWD_NOSAVE, timing studies only: 1 = no saves, 2 = h_in only)
            st4(rs_r, vq, sq, sv[0]);
            st4(rs_z, vq, sq, sv[1]);
            st4(rs_hn, vq, sq, sv[2]);
          }
          *reinterpret_cast<f16x4*>(&hB[0][ho]) = n0;
          *reinterpret_cast<f16x4*>(&hB[1][ho]) = n1;
          *reinterpret_cast<bf16x4*>(&hB[2][ho]) = nr;
        }
        // lanes l and l + 32 hold the same row: fold the two halves, one lane writes
  #pragma unroll
        for (int oo = 0; oo < 9; ++oo) {
          const float o = __shfl_xor(hp_loc[oo], 32);
          if (hi == 0) hp[(FWD_HDEFER ? (s & 1) * 4608 : 0) + (wave * 9 + oo) * 64 + row] = hp_loc[oo] + o;
        }
      }
    if (FWD_PP_PRIO) __builtin_amdgcn_s_setprio(0);
  };
  // (each half's three roles in program order, so the ring and B registers are dead across the gate maths)
  if (grp == 0) {
    for (int s = 0; s < T; ++s) {
      PP_STAMP(s, 0);
      c_first(s);
      PP_STAMP(s, 1);
      lds_barrier();
      PP_STAMP(s, 2);
      c_second(s);
      if (wave == 0 && s > 0) head_out(s - 1);
      PP_STAMP(s, 3);
      lds_barrier();
      PP_STAMP(s, 4);
      g_maths(s);
      PP_STAMP(s, 5);
      lds_barrier();
    }
    lds_barrier();   // (the other half's last gate maths)
    if (wave == 0) head_out(T - 1);
  } else {
    for (int s = 0; s < T; ++s) {
      PP_STAMP(s, 0);
      if (s > 0) g_maths(s - 1);
      PP_STAMP(s, 1);
      lds_barrier();
      PP_STAMP(s, 2);
      c_first(s);
      PP_STAMP(s, 3);
      lds_barrier();
      PP_STAMP(s, 4);
      c_second(s);
      PP_STAMP(s, 5);
      lds_barrier();
    }
    g_maths(T - 1);
    lds_barrier();
  }
} else {
  for (int s = 0; s < T; ++s) {
    const int t = T - 1 - s;
    FWD_STAMP(0);
    floatx16 acc[3][2];   // r, z, W_hn h + b_hn (the n gate's input part is gate_ain, on the VALU)
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[g][h][q] = 0.0f;
    // ---- contraction: 16 fp16 k-steps over the carry + one augmented bf16 k-step.  Each gate's A fragments
    // (unit tile `wave`) are refilled for the next k-step right after their last MFMA, each row tile's B
    // fragments right after theirs; the partner wave on the SIMD covers what latency remains.
    // this lane's row inputs x(t) for the augmented k-step [x_0 .. x_{F-1}, 1, 0 ...] (F <= 7), split into B fragments
    // at the end of the contraction (lanes 32-63 hold k = 8..15: zero); A fragments through a two-k-step ring (A0: even
    // k-steps, A1: odd): each L2 fragment load has a whole k-step of the wave's MFMAs (plus the partner wave's) to land
    // instead of one gate's.  (Declared in the step: hoisted out of the loop, the C4 per-candidate instance ran 2.61-2.69
    // instead of 2.22 ms.)  The ring's first two k-steps go out ahead of x (FWD_XFIRST=0: the first ring wait does not
    // wait for x's HBM loads; 1.207-1.216 ms either order at C2)
    float xv[2][7];
    f16x8 A0[3][2], A1[3][2], B[2][2];

    auto fragA = [&](int ks, int g, int q) { return ((ks * 8 + wave) * 3 + g) * 2 + q; };
    auto fragAug = [&](int g, int q) { return F6_NFH + (wave * 4 + g) * 3 + q; };
    {
      auto ring = [&] {
#pragma unroll
        for (int g = 0; g < 3; ++g)
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            A0[g][q] = ldAh(fragA(0, g, q));
            A1[g][q] = ldAh(fragA(1, g, q));
          }
      };
      if (!FWD_XFIRST) ring();
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int f = 0; f < 7; ++f) {
          const int fc = f < F ? f : F - 1;
          xv[h][f] = ld_u(rs_X, (unsigned)((RB * h + col) * p.xs_col * 4),
                          (unsigned)((fc * p.xs_f + ((long)t * R + r0) * p.xs_col) * 4));
        }
      if (FWD_XFIRST) ring();
    }
    auto load_B = [&](int ks, int h) {
      // (FWD_LANEB: the lane's row and half re-derived instead of a register kept across the step loop -- no spill,
      // but the contraction issued slower: 1.150-1.152 vs 1.131-1.136 ms, r06t34)
      const int ln = FWD_LANEB ? lane_now() : lane;
      const int cl = ln & 31, hl = ln >> 5;
#pragma unroll
      for (int q = 0; q < 2; ++q)
        B[h][q] = *reinterpret_cast<const f16x8*>(&hB[q][(RB * h + cl) * F6_HP + 16 * ks + 8 * hl]);
    };
    load_B(0, 0);
    load_B(0, 1);
    auto kstep = [&](int ks, f16x8 (&Ar)[3][2], bool reload) {
#pragma unroll
      for (int g = 0; g < 3; ++g) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          acc[g][h] = mfma3h(Ar[g], B[h], acc[g][h]);
          if (g == 2) load_B(ks + 1, h);
        }
        if (reload) {
#pragma unroll
          for (int q = 0; q < 2; ++q) Ar[g][q] = ldAh(fragA(ks + 2, g, q));
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    // (a rolled loop over k-step pairs: a full unroll hoists ~300 fragment offsets into SGPRs, which spill)
#pragma nounroll
    for (int kp = 0; kp < 7; ++kp) {
      kstep(2 * kp, A0, true);
      kstep(2 * kp + 1, A1, true);
    }
    kstep(14, A0, false);
    f16x8 (&A)[3][2] = A1;   // k-step 15
    if (A32) {
      // the augmented k-step on the f32 MFMA (exact products): A = the scaled input weights and biases (one 16-byte
      // fragment per gate, 3 KB per wave-step instead of the bf16 triple's 12 KB: the ES candidates' per-step stream
      // from the Infinity Cache is what this kernel waits on), B = 2^14 [x_k (k < F), 1 (k = 7)]
      float4 a32[3];
#pragma unroll
      for (int g = 0; g < 3; ++g)
        a32[g] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                                rs_A, (int)vA, (F6_A32 + (wave * 3 + g) * 256) * 4, 0));
#pragma unroll
      for (int g = 0; g < 3; ++g) {
#pragma unroll
        for (int h = 0; h < 2; ++h) acc[g][h] = mfma3h(A[g], B[h], acc[g][h]);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int k = 2 * kk + hi;
        float bx[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          // static indices: the lane's k = 2 kk + hi picks between two registers (a lane-dependent index puts xv in
          // scratch: 64 bytes per lane, C4's forward 2.22 -> 2.65 ms while xv lived outside the step loop)
          const float xs = hi ? xv[h][2 * kk + 1 < 7 ? 2 * kk + 1 : 6] : xv[h][2 * kk];
          bx[h] = (k < F ? xs : (k == 7 ? 1.0f : 0.0f)) * HSCALE;
        }
#pragma unroll
        for (int g = 0; g < 3; ++g) {
          const float av = kk == 0 ? a32[g].x : kk == 1 ? a32[g].y : kk == 2 ? a32[g].z : a32[g].w;
#pragma unroll
          for (int h = 0; h < 2; ++h) acc[g][h] = mfma32(av, bx[h], acc[g][h]);
        }
      }
    } else {
    // last carry k-step; each gate's augmented fragments (three bf16 pieces) load behind its MFMAs
    bf16x8 Aa[3][3], Ba[2][3];
#pragma unroll
    for (int g = 0; g < 3; ++g) {
#pragma unroll
      for (int h = 0; h < 2; ++h) acc[g][h] = mfma3h(A[g], B[h], acc[g][h]);
#pragma unroll
      for (int q = 0; q < 3; ++q) Aa[g][q] = ldA(fragAug(g, q));
      __builtin_amdgcn_sched_barrier(0);
    }
    // augmented k-step: B = bf16 pieces of 2^14 [x, 1, 0 ...]
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = hi ? 0.0f : e < F ? xv[h][e < 7 ? e : 6] : (e == F ? 1.0f : 0.0f);
        split3v(v * HSCALE, Ba[h][0], Ba[h][1], Ba[h][2], e);
      }
#pragma unroll
    for (int g = 0; g < 3; ++g) {
#pragma unroll
      for (int h = 0; h < 2; ++h) acc[g][h] = mfma6(Aa[g], Ba[h], acc[g][h]);
    }
    }
    if (FWD_HDEFER && s > 0 && wave == 0) head_out(s - 1);   // (wave 0 leads its SIMD: it waits here anyway)
    FWD_STAMP(1);
    lds_barrier();   // every wave done reading hB / xB: the carry and x(t-1) overwrite them in place
    FWD_STAMP(2);
    // ---- gate maths (lane = row 32h + col, register q = unit 32 wave + 4 hi + qunit(q))
    floatx16 ain[2];
    // done flags d_{t-1} of the lane's two rows, issued before the saves so their wait drains nothing else
    // (lane offset re-derived here: a spilled copy's reload would wait on every outstanding access)
    bool dnf[2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
      dnf[h] = (t >= 1) ? __builtin_amdgcn_raw_buffer_load_b8(
                              rs_done, lane_now() & 31, (int)(((long)a_[h] * T + (t - 1)) * W + r0 + RB * h - a_[h] * W),
                              0) != 0
                        : false;
    float wI[4];
    {
      const int ln = lane_now();
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) wI[kk] = wIs[(wave * 4 + kk) * 64 + ln];
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) ain[h] = gate_ain(wI, F, hi, [&](int k) { return xv[h][k < 7 ? k : 6]; });
    const long cbase = (long)t * R;
    const int ub = 32 * wave + 4 * hi;
    const float4* whl = reinterpret_cast<const float4*>(wh + ub * 12);
    GM_STAMP(0);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = RB * h + col;
      const bool dn = dnf[h];
      const unsigned vq = quad_vbyte(ub, col), vslab = slab_vbyte(ub, col);
      float hp_loc[9];
#pragma unroll
      for (int oo = 0; oo < 9; ++oo) hp_loc[oo] = 0.0f;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        // four consecutive units ub + 8 g4 .. +3 of this row: h_in pieces, then the new carry's pieces
        const int ho = row * F6_HP + ub + 8 * g4;
        const f16x4 h0 = *reinterpret_cast<const f16x4*>(&hB[0][ho]);
        const f16x4 h1 = *reinterpret_cast<const f16x4*>(&hB[1][ho]);
        const bf16x4 hr = *reinterpret_cast<const bf16x4*>(&hB[2][ho]);
        // the saves of this register quad: h_in (rebuilt exactly from its pieces) per unit in its slab blocks; r, z,
        // hn one 16-byte store each in their unit-quad blocks (quad_soff) after the gate maths
        const unsigned sq = quad_soff(cbase + r0, h, g4);
        float sv[3][4];
        float us[3][4];
#pragma unroll
        for (int g = 0; g < 3; ++g) {
          const float4 v = *reinterpret_cast<const float4*>(&usc[g * HU + ub + 8 * g4]);
          us[g][0] = v.x; us[g][1] = v.y; us[g][2] = v.z; us[g][3] = v.w;
        }
        f16x4 n0, n1;
        bf16x4 nr;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int q = 4 * g4 + e;
          const float rg = sigm_r(acc[0][h][q] * us[0][e]);
          const float zg = sigm_r(acc[1][h][q] * us[1][e]);
          const float hn = acc[2][h][q] * us[2][e];
          const float ng = gate_n(ain[h][q], rg, hn);
          const float hin = (((float)h0[e] + (float)h1[e]) + (float)hr[e]) * (1.0f / HSCALE);   // exact
          const float hh = (1.0f - zg) * ng + zg * hin;
          split_carry(dn ? 0.0f : hh, n0, n1, nr, e);   // carry h_in(t-1) = where(d_{t-1}, 0, h_out(t))
          sv[0][e] = rg;
          sv[1][e] = zg;
          sv[2][e] = hn;   // n is recomputed by the backward (gate_n)
          if (SAVE && FWD_NOSAVE != 1) {   // (FWD_NOSAVE, timing studies only: 1 = no saves, 2 = h_in only)
            if (HIN_SLAB) st_u(rs_hin, vslab, slab_soff(cbase + r0, h, qunit(q)), hin);
            else st_u(rs_hin, (unsigned)(((long)ub * p.M + r0 + row) * 4), (unsigned)(((long)qunit(q) * p.M + cbase) * 4), hin);
          }
          const float rl = fmaxf(hh, 0.0f);
          const float4 w0 = whl[qunit(q) * 3], w1 = whl[qunit(q) * 3 + 1], w2 = whl[qunit(q) * 3 + 2];
          hp_loc[0] += rl * w0.x; hp_loc[1] += rl * w0.y; hp_loc[2] += rl * w0.z;
          hp_loc[3] += rl * w0.w; hp_loc[4] += rl * w1.x; hp_loc[5] += rl * w1.y;
          hp_loc[6] += rl * w1.z; hp_loc[7] += rl * w1.w; hp_loc[8] += rl * w2.x;
        }
        if (SAVE && FWD_NOSAVE == 0) {   // (FWD_NOSAVE, timing studies only: 1 = no saves, 2 = h_in only)
          st4(rs_r, vq, sq, sv[0]);
          st4(rs_z, vq, sq, sv[1]);
          st4(rs_hn, vq, sq, sv[2]);
        }
        *reinterpret_cast<f16x4*>(&hB[0][ho]) = n0;
        *reinterpret_cast<f16x4*>(&hB[1][ho]) = n1;
        *reinterpret_cast<bf16x4*>(&hB[2][ho]) = nr;
      }
      // lanes l and l + 32 hold the same row: fold the two halves, one lane writes
#pragma unroll
      for (int oo = 0; oo < 9; ++oo) {
        const float o = FWD_XOR32 ? xor32(hp_loc[oo]) : __shfl_xor(hp_loc[oo], 32);
        const int rw = FWD_XOR32 ? RB * h + (lane_now() & 31) : row;   // (re-derived: no spilled address either)
        if (hi == 0) hp[(FWD_HDEFER ? (s & 1) * 4608 : 0) + (wave * 9 + oo) * 64 + rw] = hp_loc[oo] + o;
      }
      GM_STAMP(1 + h);
    }
    FWD_STAMP(3);
    lds_barrier();   // head partials, the carry and x(t-1) visible
    FWD_STAMP(4);
    if (FWD_HDEFER) {
      FWD_STAMP(5);
      continue;
    }
    for (int i = 64 * wave + lane_now(); i < 9 * 64; i += 512) {
      const int oo = i >> 6, c = i & 63;
      float v = hbias[oo];
#pragma unroll
      for (int gq = 0; gq < 8; ++gq) v += hp[(gq * 9 + oo) * 64 + c];
      hout[i] = v;
    }
    lds_barrier();
    if (tid < 64) {
      const int tl = lane_now();   // == tid (wave 0)
      const long ob = (long)t * R + r0 + tl;
      p.pi_hat[ob] = hout[tl];
      float m = -__builtin_inff();
      for (int j = 0; j < 8; ++j) m = fmaxf(m, hout[(j + 1) * 64 + tl]);
      float e[8], ssum = 0.0f;
      for (int j = 0; j < 8; ++j) { e[j] = __expf(hout[(j + 1) * 64 + tl] - m); ssum += e[j]; }
      const float inv = 1.0f / ssum;
      for (int j = 0; j < 8; ++j) p.y_hat[((long)t * 8 + j) * R + r0 + tl] = e[j] * inv;
    }
    FWD_STAMP(5);
  }
  if (FWD_HDEFER && wave == 0) head_out(T - 1);   // the last step's heads (its partials visible: the loop's barrier)
}
}

// ------------------------------------------------------------------ backward
struct BwdArgs {
  int R, T, W, K;
  const uint8_t* done; long done_stride_k;     // per k: [N][T][W]
  const float4* A;                             // packed bwd fragments (f32 MFMA, k_gru_bwd<1>)
  const void* A6;                              // packed bwd fragments (bf16 split pieces, k_gru_bwd6n)
  const float* eta; EtaOff o;
  const float* y_hat; const float* d_pi_hat; const float* d_y_hat;   // [K][T][(8)][R]
  const float* s_hin; const float* s_r; const float* s_z; const float* s_n; const float* s_hn;  // [256][M]
  long M;
  float* DG;        // [4][256][M]: dr_pre, dz_pre, d(hn), dn_pre
  float* RH;        // [256][M] relu(h_out)
  float* DH;        // [9][M] head cotangents (d pi_hat, d y_logits)
  float* dX3; float* dX4;   // [K][T][R]
  int8_t* CE;       // [M] (optional, lockstep kernel): column m's cotangent scale exponent for the weight-gradient
                    // reduction (2^CE[m] max over dr, dz, dhn of column m < 2^14; 127 = all zero)
  int F;            // LPG input width (lockstep kernel: x rows at s_hin + 256 M, n recomputed by gate_n)
  float* SP;        // fused small products (k_gru_bwd6n<true>): per-workgroup partials [n_wg][SP_FLOATS]
  int stagger, stagger_mode;   // k_gru_bwd6n: s_sleep(127) quanta some first-round workgroups wait at start
  int wg_base;                 // k_gru_bwd6n: this launch's first workgroup in the whole grid (TOUED_BWD_HALVES)
};
// fused small weight-gradient products: per workgroup C[16][256] (rows 0..F-1: X . dn^T, row F: the ones row,
// rows F+1..F+9: DH . relu(h_out)^T) then the head cotangents' row sums [9][64 rows]
#define SP_C (16 * HU)
#define SP_FLOATS (SP_C + 9 * 64)

// NT row tiles of 32 rows per workgroup.  NT = 2: one workgroup per CU (150 KB LDS, 256 VGPRs), every
// packed W_h^T fragment feeds 8 MFMAs instead of 4 (half the L2 fragment stream per FLOP).
template <int NT>
__global__ void __launch_bounds__(512, NT == 1 ? 4 : 1) k_gru_bwd(BwdArgs p) {
  constexpr int RBT = RB * NT;          // rows per workgroup
  constexpr int LDT = RBT + 1;          // padded LDS row (k-major [unit][row])
  __shared__ float dgT[2 * HU * LDT];   // [dr | dz], then dhn in slot 0
  __shared__ float wi34[2 * 3 * HU];
  __shared__ float hv[9 * RBT];
  __shared__ float dxp[NGRP * 2 * RBT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hi = lane >> 5, col = lane & 31;
  const int nb = p.R / RBT;
  const int k = blockIdx.x / nb;
  const int r0 = (blockIdx.x - k * nb) * RBT;
  const int R = p.R, T = p.T, W = p.W;
  int a_[NT], w_[NT];
#pragma unroll
  for (int h = 0; h < NT; ++h) {
    const int row = r0 + RB * h + col;
    a_[h] = (r0 + RB * h) / W;
    w_[h] = row - a_[h] * W;
  }
  // W_i rows for the embedding inputs (f = 3: pyt, f = 4: pyt1), per gate kind r, z, n
  for (int i = tid; i < 2 * 3 * HU; i += 512) {
    const int f = 3 + i / (3 * HU), g = (i / HU) % 3, u = i % HU;
    const int base = g == 0 ? p.o.ir_w : g == 1 ? p.o.iz_w : p.o.in_w;
    wi34[i] = f < p.F ? p.eta[base + f * HU + u] : 0.0f;   // (inputs 3, 4 exist when F >= 5)
  }
  float dh[NT][16];
#pragma unroll
  for (int h = 0; h < NT; ++h)
#pragma unroll
    for (int q = 0; q < 16; ++q) dh[h][q] = 0.0f;
  float wA[5];    // A fragments of W_heads^T for this wave's unit tile: A[i=l&31][k=2kk+(l>>5)]
#pragma unroll
  for (int kk = 0; kk < 5; ++kk) {
    const int o = 2 * kk + hi, u = 32 * wave + col;
    wA[kk] = o < 9 ? (o == 0 ? p.eta[p.o.pi_w + u] : p.eta[p.o.y_w + u * 8 + (o - 1)]) : 0.0f;
  }
  const uint8_t* done = p.done + (long)k * p.done_stride_k;
  const float4* Ab = p.A + lane;
  const __amdgpu_buffer_rsrc_t rs_hin = rsrc_of(p.s_hin), rs_r = rsrc_of(p.s_r), rs_z = rsrc_of(p.s_z),
                               rs_n = rsrc_of(p.s_n), rs_hn = rsrc_of(p.s_hn), rs_rh = rsrc_of(p.RH);
  const __amdgpu_buffer_rsrc_t rs_dg[4] = {rsrc_of(p.DG), rsrc_of(p.DG + 1L * HU * p.M),
                                           rsrc_of(p.DG + 2L * HU * p.M), rsrc_of(p.DG + 3L * HU * p.M)};
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    const long ctr = ((long)k * T + t) * R;          // column base in [.][K*T*R]
    if (tid < RBT) {
      const long o = ctr + r0 + tid;       // global column
      float yh[8], dy[8], s = 0.0f;
      for (int j = 0; j < 8; ++j) {
        yh[j] = p.y_hat[((long)k * T * 8 + (long)t * 8 + j) * R + r0 + tid];
        dy[j] = p.d_y_hat[((long)k * T * 8 + (long)t * 8 + j) * R + r0 + tid];
        s += yh[j] * dy[j];
      }
      const float dpi = p.d_pi_hat[o];
      hv[tid] = dpi;
      p.DH[o] = dpi;
      for (int j = 0; j < 8; ++j) {
        const float v = yh[j] * (dy[j] - s);
        hv[(j + 1) * RBT + tid] = v;
        p.DH[(long)(j + 1) * p.M + o] = v;
      }
    }
    __syncthreads();
    float dhn_r[NT][16];
    const float* wil = wi34 + 32 * wave + 4 * hi;
#pragma unroll
    for (int h = 0; h < NT; ++h) {
      // head VJP W_heads . hv on MFMA: A[i = unit][k = head output o] (constant per lane, wA),
      // B[k = o][j = row] from hv; the result has the accumulator layout (lane = row, reg = unit).
      floatx16 hacc;
#pragma unroll
      for (int q = 0; q < 16; ++q) hacc[q] = 0.0f;
#pragma unroll
      for (int kk = 0; kk < 5; ++kk) {
        const int o = 2 * kk + hi;
        hacc = mfma32(wA[kk], o < 9 ? hv[o * RBT + RB * h + col] : 0.0f, hacc);
      }
      // transposed 16-byte accesses: lane col moves unit (32w + 4hi + 8g4 + (col & 3)) for the four rows
      // r0 + RB*h + (col & 28) .. +3 of this step's columns
      const unsigned vq = (unsigned)((((long)(32 * wave + 4 * hi + (col & 3))) * p.M + r0 + RB * h + (col & 28)) * 4);
      float dx3 = 0.0f, dx4 = 0.0f;
      // one unit quad (four consecutive units) per iteration: five 16-byte loads + transposes, the gate
      // maths, five dword stores per unit (+ two LDS writes per unit)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const unsigned so = (unsigned)(((long)8 * g4 * p.M + ctr) * 4);
        float v_hin[4], v_r[4], v_z[4], v_n[4], v_hn[4];
        ld4(rs_hin, vq, so, v_hin);
        ld4(rs_r, vq, so, v_r);
        ld4(rs_z, vq, so, v_z);
        ld4(rs_n, vq, so, v_n);
        ld4(rs_hn, vq, so, v_hn);
        quad_transpose(v_hin, lane);
        quad_transpose(v_r, lane);
        quad_transpose(v_z, lane);
        quad_transpose(v_n, lane);
        quad_transpose(v_hn, lane);
        float* o_rh = v_hin; float* o_dr = v_r; float* o_dz = v_z; float* o_dhn = v_n; float* o_dn = v_hn;  // reused in place
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int q = 4 * g4 + j;
          const float hin = v_hin[j], rg = v_r[j], zg = v_z[j], ng = v_n[j], hn = v_hn[j];
          const float hout = (1.0f - zg) * ng + zg * hin;
          const float d = dh[h][q] + (hout > 0.0f ? hacc[q] : 0.0f);
          const float dn_ = d * (1.0f - zg);
          const float dz = d * (hin - ng);
          const float dnp = dn_ * (1.0f - ng * ng);
          const float dhn = dnp * rg;
          const float drp = dnp * hn * rg * (1.0f - rg);
          const float dzp = dz * zg * (1.0f - zg);
          dh[h][q] = d * zg;   // direct path; the W_h^T contraction is added below
          const int lo = (32 * wave + 4 * hi + qunit(q)) * LDT + RB * h + col;   // B operands straight to LDS
          dgT[lo] = drp;
          dgT[HU * LDT + lo] = dzp;
          dhn_r[h][q] = dhn;
          o_rh[j] = fmaxf(hout, 0.0f); o_dr[j] = drp; o_dz[j] = dzp; o_dhn[j] = dhn; o_dn[j] = dnp;
          const int qu = qunit(q);
          dx3 += drp * wil[0 * HU + qu] + dzp * wil[1 * HU + qu] + dnp * wil[2 * HU + qu];
          dx4 += drp * wil[3 * HU + qu] + dzp * wil[4 * HU + qu] + dnp * wil[5 * HU + qu];
        }
        {
          const unsigned vb = (unsigned)(((long)(32 * wave + 4 * hi) * p.M + r0 + RB * h + col) * 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const unsigned so1 = (unsigned)(((long)qunit(4 * g4 + j) * p.M + ctr) * 4);
            st_u(rs_rh, vb, so1, o_rh[j]);
            st_u(rs_dg[3], vb, so1, o_dn[j]);          // dr, dz, dhn leave from LDS (store_gate_lds)
          }
        }
      }
      dxp[((2 * wave + hi) * 2 + 0) * RBT + RB * h + col] = dx3;
      dxp[((2 * wave + hi) * 2 + 1) * RBT + RB * h + col] = dx4;
    }
    floatx16 acc[NT];
#pragma unroll
    for (int h = 0; h < NT; ++h)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[h][q] = 0.0f;
    // dh_prev = dr . W_hr^T + dz . W_hz^T (both in LDS) then + dhn . W_hn^T (dhn to LDS slot 0)
#pragma unroll 1
    for (int g = 0; g < 3; ++g) {
      if (g == 2) {
        __syncthreads();     // all waves done reading slot 0 (dr)
#pragma unroll
        for (int h = 0; h < NT; ++h) {
          float* dgl = dgT + (32 * wave + 4 * hi) * LDT + RB * h + col;
#pragma unroll
          for (int q = 0; q < 16; ++q) dgl[qunit(q) * LDT] = dhn_r[h][q];
        }
      }
      if (g != 1) __syncthreads();
      // the gate cotangents just completed in LDS go out as 16-byte row-quad stores (LDS does the
      // transpose): dr and dz before the first contraction, dhn before the third
      if (g == 0) {
        store_gate_lds<NT>(dgT, rs_dg[0], p.M, ctr + r0, wave, lane);
        store_gate_lds<NT>(dgT + HU * LDT, rs_dg[1], p.M, ctr + r0, wave, lane);
      } else if (g == 2) {
        store_gate_lds<NT>(dgT, rs_dg[2], p.M, ctr + r0, wave, lane);
      }
      const float* dgs = dgT + (g == 1 ? HU * LDT : 0);
      float4 an = Ab[((wave * 3 + g) * 32 + 0) * 64];
#pragma unroll 2
      for (int kq = 0; kq < 32; ++kq) {
        const float4 av = an;
        if (kq + 1 < 32) an = Ab[((wave * 3 + g) * 32 + kq + 1) * 64];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float x = e == 0 ? av.x : e == 1 ? av.y : e == 2 ? av.z : av.w;
#pragma unroll
          for (int h = 0; h < NT; ++h) {
            const float b = dgs[(2 * (4 * kq + e) + hi) * LDT + RB * h + col];
            acc[h] = mfma32(x, b, acc[h]);
          }
        }
      }
    }
    __syncthreads();
    if (tid < RBT) {
      float s3 = 0.0f, s4 = 0.0f;
      for (int gq = 0; gq < NGRP; ++gq) { s3 += dxp[(gq * 2 + 0) * RBT + tid]; s4 += dxp[(gq * 2 + 1) * RBT + tid]; }
      p.dX3[ctr + r0 + tid] = s3;
      p.dX4[ctr + r0 + tid] = s4;
    }
    // carry to h_out(t+1): h_in(t) = where(d_t, 0, h_out(t+1))
#pragma unroll
    for (int h = 0; h < NT; ++h) {
      const bool dn = done[((size_t)a_[h] * T + t) * W + w_[h]] != 0;
#pragma unroll
      for (int q = 0; q < 16; ++q) dh[h][q] = dn ? 0.0f : dh[h][q] + acc[h][q];
    }
    __syncthreads();
  }
}


#ifdef BWD_STAMPS
// timing instrumentation (tools/bwd_stamps.py, built by tools/build_variant.py gru.hip BWD_STAMPS=1): wave 0 lane 0
// of workgroups < 64 records s_memtime at 8 points of every step
__device__ unsigned long long g_bwd_stamps[64 * 32 * 8];
#define BWD_STAMP(ph)                                                                                  \
  do {                                                                                                 \
    if (blockIdx.x < 64 && tid == 0 && t < 32)                                                         \
      g_bwd_stamps[(blockIdx.x * 32 + t) * 8 + (ph)] = __builtin_amdgcn_s_memtime();                   \
  } while (0)
// per-wave stamps of the same workgroups: memory part start / end of every wave, and the wave's SIMD (HW_ID 5:4)
#define BWD_NWS 8
__device__ unsigned long long g_bwd_wstamps[64 * 32 * 8 * BWD_NWS];
__device__ int g_bwd_wsimd[64 * 8];
#define BWD_WSTAMP(ph)                                                                                 \
  do {                                                                                                 \
    if (blockIdx.x < 64 && lane_now() == 0 && t < 32)                                                  \
      g_bwd_wstamps[((blockIdx.x * 32 + t) * 8 + wave) * BWD_NWS + (ph)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define BWD_STAMP(ph) do {} while (0)
#define BWD_WSTAMP(ph) do {} while (0)
#endif

// Backward in lockstep (k_gru_bwd6n): one 512-thread workgroup per (k, 64 rows), both 32-row tiles in
// every wave, so each pre-split W_g fragment (L2) feeds both tiles: half the fragment traffic of the two-group
// kernel, which was the vector-memory bottleneck once the contraction moved to the bf16 matrix cores.  Wave w
// owns units [32w, 32w + 32).  Per step:
//   memory part: 16-byte saved-activation loads + quad transposes, gate maths; every cotangent (dr, dz,
//     d(W_hn h + b_hn), dn) and relu(h_out) leaves as per-unit dword stores (lane = row: 128-byte rows);
//     dr is split once into three bf16 pieces in the one LDS cotangent image, dz and dhn wait in registers;
//   contraction: dh_prev = sum_g W_g . dg_g with the pieces as B fragments (no per-wave re-split), the image
//     refilled with dz, then dhn, between the three gate passes.
//   SMALL (F <= 6): the two small weight-gradient products GI = [X; 1] . dn^T and DH . relu(h_out)^T accumulate in
//     the kernel (16x16x4 f32 MFMA, exact f32 products) instead of streaming dn and relu(h_out) to HBM for a later
//     reduction: see small_mfma below.
#ifndef BWD_MPRIO
#define BWD_MPRIO 0
#endif
// BWD_TRECOMP (timing study only, wrong results): the gate pre-activations W_hr h, W_hz h and
// W_hn h recomputed on the matrix pipe at the top of every step (the forward's 16 carry k-steps: 3 gates x 2 row tiles
// x scaled fp16 pairs, A fragments through a two-k-step L2 ring, B from the image) and the memory part loading only
// h_in: a lower bound on the step of a recompute backward (no h_in image build, no augmented input k-step)
#ifndef BWD_TRECOMP
#define BWD_TRECOMP 0
#endif
// BWD_PK: the memory part's per-element gate maths on element pairs (packed FP32: v_pk_{add,mul,fma}_f32, two
// elements per instruction; 350 fewer VALU instructions in the kernel, k_gru_bwd6n 7.42 -> 7.27-7.34 ms, round 6
// profiles/r06/r06t12_ab.log; the same head-partial pairing in the forward measured no gain and was dropped)
#ifndef BWD_PK
#define BWD_PK 1
#endif
template <bool SMALL>
__global__ void __launch_bounds__(512, 1) k_gru_bwd6n(BwdArgs p) {
  constexpr int RBT = 2 * RB;
  constexpr int PP = HU + 8;                       // piece image row pitch (bf16): 528 B
  __shared__ __attribute__((aligned(16))) __bf16 dgB[3][RBT * PP];   // one cotangent, three pieces [row][unit]
  __shared__ float wi34[2 * 3 * HU];
  __shared__ float hv[9 * RBT];                    // head cotangents [output][row]
  __shared__ __attribute__((aligned(8))) float dxp[8 * RBT * 2];   // [wave][row][dx3 | dx4]
  __shared__ __attribute__((aligned(16))) float wsc[HU];          // 2^s of W_g row i (fp16 A scale)
  __shared__ float rmx[8 * RBT];                   // per-wave row maxima of |dr|, |dz|, |dhn| (fp16 B scale)
  __shared__ float wIs[8 * 4 * 64];                // gate_ain's W_in fragments [wave][kk][lane] (read at each tile)
  __shared__ float wAs[8 * 5 * 64];                // W_heads^T A fragments [wave][kk][lane] (read at each tile)
  __shared__ int dns[RBT];                         // done flags of the step's rows (loaded with the head cotangents)
  // SMALL: the A operand of the small products per row pair s of the step: Atab[s][lane] = A[i = lane & 15][k = lane
  // >> 4] with k = 0, 1: [x; 1] of rows 2s, 2s+1 (i < F, i == F) and k = 2, 3: the head cotangents of rows 2s, 2s+1
  // (i = F+1 .. F+9); and the head cotangents' running row sums over the steps (the heads' bias column)
  __shared__ __attribute__((aligned(16))) float Atab[SMALL ? 32 * 64 : 4];
  __shared__ float hvs[SMALL ? 9 * RBT : 1];
  __shared__ floatx4 accl[SMALL ? 8 * 2 * 64 : 1];
  // dr in f32 while the memory part streams ([row][unit], pitch DRP), over image slots 1 and 2
  constexpr int DRP = HU + 4;
  static_assert(RBT * DRP * 4 <= 2 * RBT * PP * 2, "dr staging exceeds image slots 1-2");
  float* drs = reinterpret_cast<float*>(&dgB[1][0]);
  const int tid = threadIdx.x, lane = tid & 63, hi = lane >> 5, col = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nb = p.R / RBT;
  const int bid = blockIdx.x + p.wg_base;
  const int k = bid / nb;
  const int r0 = (bid - k * nb) * RBT;
  const int R = p.R, T = p.T, W = p.W;
#ifdef BWD_STAMPS
  if (blockIdx.x < 64 && (tid & 63) == 0)
    g_bwd_wsimd[blockIdx.x * 8 + wave] = __builtin_amdgcn_s_getreg((1 << 11) | (4 << 6) | 4);   // HW_ID SIMD_ID
#endif
  for (int i = tid; i < 2 * 3 * HU; i += 512) {
    // BWD_PK: [gate][unit] pairs (input 3, input 4) for the packed dX3 / dX4 accumulation; else [input][gate][unit]
    const int f = BWD_PK ? 3 + (i & 1) : 3 + i / (3 * HU), g = BWD_PK ? (i >> 1) / HU : (i / HU) % 3,
              u = BWD_PK ? (i >> 1) % HU : i % HU;
    const int base = g == 0 ? p.o.ir_w : g == 1 ? p.o.iz_w : p.o.in_w;
    wi34[i] = f < p.F ? p.eta[base + f * HU + u] : 0.0f;   // (inputs 3, 4 exist when F >= 5)
  }
  for (int i = tid; i < HU; i += 512) wsc[i] = reinterpret_cast<const float*>(p.A6)[B6_SCALES + i];
  const int F = p.F;
  {
    float wI[4];   // n gate input weights (gate_ain), kept in LDS: registers are the bound here
    load_win_frags(wI, p.eta, p.o, F, wave, lane);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) wIs[(wave * 4 + kk) * 64 + lane] = wI[kk];
  }
  // W_heads^T A fragments of unit tile `wave`: A[i = unit][k = head output 2kk + hi]
#pragma unroll
  for (int kk = 0; kk < 5; ++kk) {
    const int o = 2 * kk + hi, u = 32 * wave + col;
    wAs[(wave * 5 + kk) * 64 + lane] = o < 9 ? (o == 0 ? p.eta[p.o.pi_w + u] : p.eta[p.o.y_w + u * 8 + (o - 1)]) : 0.0f;
  }
  float dh[2][16];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int q = 0; q < 16; ++q) dh[h][q] = 0.0f;
  // SMALL: the running accumulators C[i][unit 32 wave + 16 uh + (l & 15)] of the wave's two 16-unit halves wait in
  // LDS between the steps ([wave][uh][lane] float4): the register file has no room for them across the step
  if (SMALL) {
    for (int i = tid; i < 9 * RBT; i += 512) hvs[i] = 0.0f;
    for (int i = tid; i < 8 * 2 * 64; i += 512) accl[i] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
  }
  // SMALL: dn_pre, relu(h_out) and DH stay on chip (optional debug stores behind a runtime branch measured 336 B of
  // scratch per lane: the kernel is at the 256-VGPR bound); the tests take the relu decisions from the unfused kernel
  constexpr bool st_rh = !SMALL, st_dn = !SMALL;
  const __amdgpu_buffer_rsrc_t rs_hin = rsrc_of(p.s_hin), rs_r = rsrc_of(p.s_r), rs_z = rsrc_of(p.s_z),
                               rs_hn = rsrc_of(p.s_hn), rs_rh = rsrc_of(SMALL ? p.s_hin : p.RH);
  const __amdgpu_buffer_rsrc_t rs_x = rsrc_of(p.s_hin + (size_t)HU * p.M);   // the rows' inputs x [F][M]
  const __amdgpu_buffer_rsrc_t rs_dg[4] = {rsrc_of(p.DG), rsrc_of(p.DG + 1L * HU * p.M),
                                           rsrc_of(p.DG + 2L * HU * p.M),
                                           rsrc_of(SMALL ? p.DG : p.DG + 3L * HU * p.M)};
  constexpr bool st_DH = !SMALL;
  const __amdgpu_buffer_rsrc_t rs_yh = rsrc_of(p.y_hat), rs_dyh = rsrc_of(p.d_y_hat), rs_dpi = rsrc_of(p.d_pi_hat),
                               rs_DH = rsrc_of(SMALL ? p.dX3 : p.DH), rs_dx3 = rsrc_of(p.dX3), rs_dx4 = rsrc_of(p.dX4),
                               rs_done = rsrc_of(reinterpret_cast<const float*>(p.done + (long)k * p.done_stride_k));
  // head cotangents of step t (softmax VJP of y_hat, d pi_hat) -> hv, DH
  auto head_cot = [&](int t) {
    if (tid < RBT) {
      const int tl = lane_now();   // == tid (wave 0)
      const unsigned vrw = (unsigned)tl * 4;
      int dnv;
      {
        // the row's done flag, read at the carry: loaded here, with nothing behind it to drain
        const int rw = r0 + tl, a = rw / W;
        dnv = __builtin_amdgcn_raw_buffer_load_b8(rs_done, (a * T + t) * W + rw - a * W, 0, 0);
      }
      const long o = ((long)k * T + t) * R + r0;
      float yh[8], dy[8], s = 0.0f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {   // all 17 loads in flight at once (the other waves wait at the barrier)
        const unsigned so = (unsigned)((((long)k * T * 8 + (long)t * 8 + j) * R + r0) * 4);
        yh[j] = ld_u(rs_yh, vrw, so);
        dy[j] = ld_u(rs_dyh, vrw, so);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += yh[j] * dy[j];
      const float dpi = ld_u(rs_dpi, vrw, (unsigned)(o * 4));
      float xr[6];   // SMALL: this row's inputs x_0 .. x_{F-1} (F <= 6)
      if (SMALL) {
#pragma unroll
        for (int f = 0; f < 6; ++f)
          xr[f] = ld_u(rs_x, vrw, (unsigned)(((long)(f < F ? f : 0) * p.M + o) * 4));
      }
      dns[tl] = dnv;
      hv[tl] = dpi;
      if (st_DH) st_u(rs_DH, vrw, (unsigned)(o * 4), dpi);
      float hvv[9];
      hvv[0] = dpi;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = yh[j] * (dy[j] - s);
        hv[(j + 1) * RBT + tl] = v;
        hvv[j + 1] = v;
        if (st_DH) st_u(rs_DH, vrw, (unsigned)(((long)(j + 1) * p.M + o) * 4), v);
      }
      if (SMALL) {
        // row tl = 2 s + par: lanes 16 par + i (k = par: [x; 1; 0]) and 32 + 16 par + i (k = 2 + par: head
        // cotangents at i = F + 1 ..): zeros, then the entries at their (uniform, runtime) positions
        float* at = Atab + (tl >> 1) * 64 + 16 * (tl & 1);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (c >= 2) *reinterpret_cast<float4*>(at + 4 * c) = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
          *reinterpret_cast<float4*>(at + 32 + 4 * c) = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
        at[6] = 0.0f;
        at[7] = 0.0f;
        *reinterpret_cast<float4*>(at) = make_float4(0 < F ? xr[0] : 0.0f, 1 < F ? xr[1] : 0.0f, 2 < F ? xr[2] : 0.0f,
                                                     3 < F ? xr[3] : 0.0f);
        *reinterpret_cast<float2*>(at + 4) = make_float2(4 < F ? xr[4] : 0.0f, 5 < F ? xr[5] : 0.0f);
        at[F] = 1.0f;
#pragma unroll
        for (int o9 = 0; o9 < 9; ++o9) at[32 + F + 1 + o9] = hvv[o9];
#pragma unroll
        for (int o9 = 0; o9 < 9; ++o9) hvs[o9 * RBT + tl] += hvv[o9];
      }
    }
  };
  // contraction of one gate's cotangent image with W_g: two scaled fp16 pieces of each operand, three
  // products, A fragments through a 2-deep ring from L2
  const __amdgpu_buffer_rsrc_t rs_A = rsrc_of(reinterpret_cast<const float*>(p.A6));
  const unsigned vA = (unsigned)lane * 16;
  floatx16 acc[2];
  auto ldAh = [&](int ks, int g, int q) {
    const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs_A, (int)vA,
                                                          (int)((((ks * 8 + wave) * 3 + g) * 3 + q) * 1024), 0);
    return __builtin_bit_cast(f16x8, x);
  };
#ifndef BWD_RD
#define BWD_RD 4
#endif
#ifndef BWD_SPREAD
#define BWD_SPREAD 0
#endif
  // BWD_SPREAD: the pass's 32 DG stores per lane (one gate's cotangent of both row tiles, held in registers) go two per
  // k-step between the MFMAs, where the vector memory pipe carries only the A ring, instead of as a burst in front of
  // the pass (the store path takes ~11 B/clk per CU: a 64 KB burst per CU held the waves ~5.7 k cycles per gate).
  // Slot s = 2 RD gi + i of ring group gi (i static): row tile h = s >> 4, register q = s & 15; the queue qv is rotated
  // by 2 RD after each rolled group so that its indices stay static.
  // SMALL (the fused path, read only by toued_wgrad_bfp_slab): each gate's cotangent DG_g in 32-column slab blocks,
  // [M / 32][256][32] (element (u, c) at ((c >> 5) * 256 + u) * 32 + (c & 31)): a reduction workgroup's B slab (256
  // rows x 32 columns) is then 32 KB of contiguous HBM instead of 256 rows x 128 bytes 4 M bytes apart, which HBM
  // serves at ~4.0 instead of ~5.9 TB/s (tools/load_probe2.hip).  Else [256][M] rows.  Offsets of unit u's 4 bytes at
  // row r0 + RB h + col of this step: lane part (unit base ub_, col) and uniform part (unit offset uq, tile h)
  auto dg_vbyte = [&](int ub_, int col_) {
    return SMALL ? (unsigned)(ub_ * 128 + col_ * 4) : (unsigned)(((long)ub_ * p.M + r0 + col_) * 4);
  };
  auto dg_soff = [&](long ctr_, int uq, int h) {
    return SMALL ? (unsigned)((((ctr_ + r0) >> 5) + h) * 32768L + uq * 128)
                 : (unsigned)((((long)uq * p.M + ctr_) * 4) + 128 * h);
  };
  auto store_slot = [&](int gst, long ctr_, int gi, int i, float v) {
    const int s_ = 2 * BWD_RD * gi + i, h = s_ >> 4, e = s_ & 3, g4 = (s_ & 15) >> 2;
    const int ln = lane_now();
    st_u(rs_dg[gst], dg_vbyte(32 * wave + 4 * (ln >> 5), ln & 31), dg_soff(ctr_, e + 8 * g4, h), v);
  };
  // pre: called once in the pass after its last ring reload (k-step 16 - RD): loads issued there stay outstanding
  // behind every ring wait of the pass (vmcnt counts in issue order), so they cost the pass nothing
  // BWD_SPLACE: where the DG stores go.  vmcnt counts loads and stores in issue order, so a ring load issued behind a
  // 64 KB store burst is waited for only once the burst has drained (HBM-write-bound when every CU stores at once):
  // with the stores right in front of a pass, its first MFMAs waited for them.  Here each pass's first RD ring slots
  // are loaded ahead of the stores -- in the previous pass's last RD k-steps, into the slots those k-steps free (no
  // extra registers), or before the dr split's stores -- and the dz / dhn stores go out at the end of the previous
  // pass (dz_r, dhn_r are live there anyway), so a burst drains during the barrier, the refill and RD k-steps.
#ifndef BWD_SPLACE
#define BWD_SPLACE 0
#endif
  static_assert(!BWD_SPLACE || (!BWD_SPREAD && 16 % BWD_RD == 0), "BWD_SPLACE: burst stores, RD dividing 16");
  f16x8 ring[BWD_RD][2];
  auto preload_ring = [&](int g) {
#pragma unroll
    for (int i = 0; i < BWD_RD; ++i)
#pragma unroll
      for (int q = 0; q < 2; ++q) ring[i][q] = ldAh(i, g, q);
  };
  // nextg >= 0 (BWD_SPLACE): the last RD k-steps load pass nextg's first RD slots; post() runs after the last k-step
  // inpass(j): called after each of the last four k-steps (j = 0..3, the unrolled tail without ring reloads), where the
  // matrix pipe paces the wave and VALU / LDS work rides beside it (BWD_INPASS: the next gate's first piece)
  auto contract_h = [&](int g, int sb, int sb1, float (&qv)[32], long ctr_, auto&& pre, bool preloaded, int nextg,
                        auto&& post, auto&& inpass) {   // sb, sb1: the image slots of the two fp16 pieces
    constexpr int RD = BWD_RD;                    // A-fragment ring depth (k-steps in flight from L2)
    static_assert(!BWD_SPREAD || 16 % RD == 0, "the spread stores: 2 per k-step, 2 RD per ring group");
    f16x8 B[2][2];
    if (!preloaded) preload_ring(g);
    const int ln = lane_now(), bl = (ln & 31) * PP + 8 * (ln >> 5);
    auto ldB = [&](int ks, int h) {
#pragma unroll
      for (int q = 0; q < 2; ++q) B[h][q] = *reinterpret_cast<const f16x8*>(&dgB[q ? sb1 : sb][bl + RB * h * PP + 16 * ks]);
    };
    ldB(0, 0);
    ldB(0, 1);
    auto kstep = [&](int ks, f16x8 (&Ar)[2], bool reload, int gi, int j) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        acc[h] = mfma3h(Ar, B[h], acc[h]);
        if (ks + 1 < 16) ldB(ks + 1, h);
        if (BWD_SPREAD && h == 0) {
          store_slot(g, ctr_, gi, 2 * j, qv[2 * j]);
          store_slot(g, ctr_, gi, 2 * j + 1, qv[2 * j + 1]);
        }
      }
      if (reload) {
#pragma unroll
        for (int q = 0; q < 2; ++q) Ar[q] = ldAh(ks + RD, g, q);
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    // whole groups of RD k-steps that all refill their slot (slots named statically), then the tail
    constexpr int NG = (16 - RD) / RD;
#pragma nounroll
    for (int gi = 0; gi < NG; ++gi) {
#pragma unroll
      for (int j = 0; j < RD; ++j) kstep(gi * RD + j, ring[j], true, gi, j);
      if (BWD_SPREAD) {
#pragma unroll
        for (int i = 0; i < 32 - 2 * RD; ++i) qv[i] = qv[i + 2 * RD];
      }
    }
#pragma unroll
    for (int ks = NG * RD; ks < 16; ++ks) {
      kstep(ks, ring[ks % RD], ks + RD < 16, NG, ks - NG * RD);
      if (ks == 16 - RD) {   // (16 - RD >= NG RD: always in the unrolled tail)
        pre();
        __builtin_amdgcn_sched_barrier(0);
      }
      if (BWD_SPLACE && nextg >= 0 && ks >= 16 - RD) {   // this k-step's slot is free: pass nextg's slot ks - (16 - RD)
#pragma unroll
        for (int q = 0; q < 2; ++q) ring[ks % RD][q] = ldAh(ks - (16 - RD), nextg, q);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (ks >= 12) {
        inpass(ks - 12);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    post();
  };
  // scaled fp16 pieces of the four units u0 .. u0 + 3 of row `row` into image slots 0, 1
#ifndef BWD_INPASS
#define BWD_INPASS 0
#endif
#ifndef BWD_TREFILL
#define BWD_TREFILL 0   // timing studies only (wrong results): 1 = refills without LDS writes, 2 = without the split
#endif
  auto put4h = [&](int row, int u0, const float (&v)[4], float sc) {
    f16x4 x0, x1;
    if (BWD_TREFILL == 2) {
#pragma unroll
      for (int e = 0; e < 4; ++e) { x0[e] = (_Float16)0.0f; x1[e] = (_Float16)0.0f; }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) split2h(v[e] * sc, x0, x1, e);
    }
    if (BWD_TREFILL != 1) {
      *reinterpret_cast<f16x4*>(&dgB[0][row * PP + u0]) = x0;
      *reinterpret_cast<f16x4*>(&dgB[1][row * PP + u0]) = x1;
    }
  };
  // BWD_INPASS: one of the two pieces (which) into image slot `slot`
  auto put1h = [&](int slot, int which, int row, int u0, const float (&v)[4], float sc) {
    f16x4 x0, x1;
#pragma unroll
    for (int e = 0; e < 4; ++e) split2h(v[e] * sc, x0, x1, e);
    *reinterpret_cast<f16x4*>(&dgB[slot][row * PP + u0]) = which ? x1 : x0;
  };
  // SMALL: the wave's dn and relu(h_out) of one row tile and one 16-unit half go through a wave-private [row][unit]
  // f32 block in image slot 0 (free during the memory part) as the B operand B[k][j = unit] of 16x16x4 f32 MFMAs over
  // the tile's 16 row pairs, k = 0, 1: dn of rows 2s, 2s+1; k = 2, 3: relu(h_out) of rows 2s, 2s+1, against Atab's
  // A[i][k] ([x; 1] rows for k < 2, head cotangent rows for k >= 2).  Unit quads are XOR-swizzled by (row >> 2) & 3
  // (conflict-free 16-byte writes and dword reads); the second array sits 544 floats after the first (other banks).
  float* priv = reinterpret_cast<float*>(&dgB[0][0]) + 1056 * wave;
  auto small_mfma = [&](int h, int g4, const float (&dnq)[4], const float (&rhq)[4]) {
    const int ln = lane_now(), row = ln & 31, c = 2 * (g4 & 1) + (ln >> 5);
    const int wo = row * 16 + ((c ^ ((row >> 2) & 3)) << 2);
    *reinterpret_cast<float4*>(priv + wo) = make_float4(dnq[0], dnq[1], dnq[2], dnq[3]);
    *reinterpret_cast<float4*>(priv + 544 + wo) = make_float4(rhq[0], rhq[1], rhq[2], rhq[3]);
    if (g4 & 1) {
      const int l2 = lane_now(), kk = l2 >> 4, j = l2 & 15;
      const int rb = (kk >> 1) * 544 + (kk & 1) * 16 + (j & 3);
      floatx4& al = accl[(wave * 2 + (g4 >> 1)) * 64 + l2];
      floatx4 acc = al;
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) {
        const float b = priv[rb + 32 * s2 + ((((j >> 2) ^ ((s2 >> 1) & 3))) << 2)];
        const float a = Atab[(16 * h + s2) * 64 + l2];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
      }
      al = acc;
    }
  };
#ifndef BWD_NR
#define BWD_NR 3
#endif
  constexpr int NR = BWD_NR;
  const int ub = 32 * wave + 4 * hi;               // lane's unit base (register q adds qunit(q))
  float vr[NR][4][4];   // NR-slot ring: quads i+1 .. i+NR-1 in flight while quad i is processed (NR = 2: 10.11 ms)
  auto load_q = [&](long ctr_, int h, int g4, float (&v)[4][4]) {
    // r, z, hn of the lane's register quad g4 (its row, four consecutive units) from their unit-quad blocks
    // (quad_soff): one 16-byte load each; h_in from its slab blocks (slab_soff): four rows of unit ub + (col & 3) +
    // 8 g4 per lane (eight consecutive units x 32 rows, 1 KB contiguous per wave instruction), lane-quad transposed
    // in the memory part
    const unsigned vq = quad_vbyte(ub, col), sq = quad_soff(ctr_ + r0, h, g4);
    if (HIN_SLAB) ld4(rs_hin, slab_vbyte(ub + (col & 3), col & 28), slab_soff(ctr_ + r0, h, 8 * g4), v[0]);
    else ld4(rs_hin, (unsigned)((((long)(ub + (col & 3))) * p.M + r0 + RB * h + (col & 28)) * 4),
             (unsigned)(((long)8 * g4 * p.M + ctr_) * 4), v[0]);
    if (!BWD_TRECOMP) {
      ld4(rs_r, vq, sq, v[1]);
      ld4(rs_z, vq, sq, v[2]);
      ld4(rs_hn, vq, sq, v[3]);
    }
  };
  // the rows' inputs x(t) as gate_ain's B fragments (lane = row RB h + col, k = 2 kk + hi): n is recomputed.
  // Tile 0's go out with the first quads, tile 1's beside the ring loads of quad 3.
  float xa[4], xb[4];
  auto load_x = [&](long ctr_, int h, float (&x)[4]) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int ln = lane_now(), k = 2 * kk + (ln >> 5);
      // k (lane-dependent) goes in the VGPR offset: a lane-dependent soffset compiles to a waterfall loop
      x[kk] = ld_u(rs_x, (unsigned)((((long)(k < F ? k : 0)) * p.M + RB * h + (ln & 31)) * 4), (unsigned)((ctr_ + r0) * 4));
    }
  };
  // the first NR - 1 quads and tile 0's x of step t: quads [0, BWD_PF) (and x when BWD_PFX) in the previous step's dhn
  // pass after its last ring reload, so that they land during that pass, the tail and the head; the rest at the top of
  // the step's memory part
#ifndef BWD_PF
#define BWD_PF 0
#endif
#ifndef BWD_PFX
#define BWD_PFX 0
#endif
  static_assert(BWD_PF >= 0 && BWD_PF <= NR - 1, "BWD_PF: at most the ring's NR - 1 leading quads");
  auto load_first = [&](long ctr_, bool pre) {
    if (pre == (bool)BWD_PFX) load_x(ctr_, 0, xa);
#pragma unroll
    for (int qi = 0; qi < NR - 1; ++qi)
      if (pre == (qi < BWD_PF)) load_q(ctr_, qi >> 2, qi & 3, vr[qi]);
  };
  // TOUED_BWD_STAGGER (study): first-round workgroups start late by phase * stagger quanta (~8 k cycles each), phase
  // by mode: 0 = alternate CUs of every XCD, 1 = alternate XCDs, 2 = four phases over the CUs of every XCD
  if (p.stagger > 0 && blockIdx.x < 256) {
    const int ph = p.stagger_mode == 0 ? (blockIdx.x >> 3) & 1 : p.stagger_mode == 1 ? blockIdx.x & 1 : (blockIdx.x >> 3) & 3;
    for (int i = 0; i < ph * p.stagger; ++i) __builtin_amdgcn_s_sleep(127);
  }
  load_first((long)k * T * R, true);
  for (int t = 0; t < T; ++t) {
    const long ctr = ((long)k * T + t) * R;
    BWD_STAMP(0);
    head_cot(t);
    lds_barrier();
    BWD_STAMP(1);
    BWD_WSTAMP(0);
    floatx16 rc[3][2];   // BWD_TRECOMP: the recomputed r, z, W_hn h (+ b_hn) accumulators
    if (BWD_TRECOMP) {
#pragma unroll
      for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int q = 0; q < 16; ++q) rc[g][h][q] = 0.0f;
      f16x8 Ra0[3][2], Ra1[3][2], Rb[2][2];
      const int ln = lane_now(), bl = (ln & 31) * PP + 8 * (ln >> 5);
      auto ldRB = [&](int ks, int h) {
#pragma unroll
        for (int q = 0; q < 2; ++q) Rb[h][q] = *reinterpret_cast<const f16x8*>(&dgB[q][bl + RB * h * PP + 16 * ks]);
      };
#pragma unroll
      for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          Ra0[g][q] = ldAh(0, g, q);
          Ra1[g][q] = ldAh(1, g, q);
        }
      ldRB(0, 0);
      ldRB(0, 1);
      auto rstep = [&](int ks, f16x8 (&Ar)[3][2], bool reload) {
#pragma unroll
        for (int g = 0; g < 3; ++g) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            rc[g][h] = mfma3h(Ar[g], Rb[h], rc[g][h]);
            if (g == 2 && ks + 1 < 16) ldRB(ks + 1, h);
          }
          if (reload) {
#pragma unroll
            for (int q = 0; q < 2; ++q) Ar[g][q] = ldAh(ks + 2, g, q);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      };
#pragma nounroll
      for (int kp = 0; kp < 7; ++kp) {
        rstep(2 * kp, Ra0, true);
        rstep(2 * kp + 1, Ra1, true);
      }
      rstep(14, Ra0, false);
      rstep(15, Ra1, false);
      lds_barrier();   // the image read before the memory part's f32 dr staging overwrites it
    }
    // ---- memory part: the eight unit quads (two row tiles x four) as a software pipeline, quad i+1's five
    // 16-byte loads in flight while quad i is transposed and processed (twice the bytes in flight per wave)
    float dz_r[2][16], dhn_r[2][16];
    // LDS addresses below are re-derived from lane_now() where used (see lane_now)
    auto ubn = [&] { return 32 * wave + 4 * (lane_now() >> 5); };
    auto rown = [&](int h) { return RB * h + (lane_now() & 31); };
    // four units ub + 8 g4 .. +3 of this lane's row RB h + col (register quad g4 of tile h): per-unit dword
    // stores, lane = row (128-byte segments).  (Transposed back to 16-byte stores of four rows, as the loads are,
    // they measured no faster: 9.82-10.0 ms against 9.75-9.88.)
    auto st_q = [&](__amdgpu_buffer_rsrc_t rs, int h, int g4, const float (&v)[4]) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        st_u(rs, (unsigned)(((long)ub * p.M + r0 + RB * h + col) * 4),
             (unsigned)(((long)qunit(4 * g4 + e) * p.M + ctr) * 4), v[e]);
    };
    load_first(ctr, false);
    floatx16 ain;
    floatx16 hacc;
    float dx3 = 0.0f, dx4 = 0.0f;
    float rmr[2] = {0.0f, 0.0f};   // running row maxima of |dr|
#pragma unroll
    for (int qi = 0; qi < 8; ++qi) {
      const int h = qi >> 2, g4 = qi & 3;
      // BWD_MPRIO (timing study): the two waves of a SIMD (w, w + 4) take turns at the higher issue priority, one quad
      // each (1), or the younger wave leads (2), instead of the older wave leading the whole memory part
      if (BWD_MPRIO == 1) {
        if (((qi + (wave >> 2)) & 1) == 0) __builtin_amdgcn_s_setprio(2); else __builtin_amdgcn_s_setprio(1);
      } else if (BWD_MPRIO == 2 && qi == 0) {
        if (wave >= 4) __builtin_amdgcn_s_setprio(2); else __builtin_amdgcn_s_setprio(1);
      }
      float (&v)[4][4] = vr[qi % NR];
      if (qi + NR - 1 < 8) load_q(ctr, (qi + NR - 1) >> 2, (qi + NR - 1) & 3, vr[(qi + NR - 1) % NR]);
      if (qi == 3) load_x(ctr, 1, xb);
      __builtin_amdgcn_sched_barrier(0);
      if (g4 == 0) {
        // head VJP W_heads . hv on MFMA for this row tile (lane = row, register = unit)
#pragma unroll
        for (int q = 0; q < 16; ++q) hacc[q] = 0.0f;
#pragma unroll
        for (int kk = 0; kk < 5; ++kk) {
          const int ln = lane_now(), o = 2 * kk + (ln >> 5);
          hacc = mfma32(wAs[(wave * 5 + kk) * 64 + ln], o < 9 ? hv[o * RBT + RB * h + (ln & 31)] : 0.0f, hacc);
        }
        float wI[4];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) wI[kk] = wIs[(wave * 4 + kk) * 64 + lane];
        ain = gate_ain(wI, F, hi, [&](int k) { return h ? xb[k >> 1] : xa[k >> 1]; });
        dx3 = 0.0f;
        dx4 = 0.0f;
      }
      quad_transpose(v[0], lane);   // h_in: four rows of one unit -> four units of the lane's row
      const float* wil = wi34 + ubn();
      float drq[4], rhq[4], dnq[4];
      if (BWD_PK) {
        // the same gate maths on element pairs: v_pk_{add,mul,fma}_f32 carry two elements per instruction (the
        // transcendentals and selects stay per element)
        const f2v* wil2 = reinterpret_cast<const f2v*>(wi34) + ubn();
        f2v dx34 = {dx3, dx4};
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          const int j0 = 2 * pp, q0 = 4 * g4 + j0;
          const f2v hin = {v[0][j0], v[0][j0 + 1]}, rg = {v[1][j0], v[1][j0 + 1]}, zg = {v[2][j0], v[2][j0 + 1]},
                    hn = {v[3][j0], v[3][j0 + 1]};
          const f2v ng = {gate_n(ain[q0], rg.x, hn.x), gate_n(ain[q0 + 1], rg.y, hn.y)};
          const f2v omz = 1.0f - zg;
          const f2v hout = omz * ng + zg * hin;
          const f2v hac = {hout.x > 0.0f ? hacc[q0] : 0.0f, hout.y > 0.0f ? hacc[q0 + 1] : 0.0f};
          const f2v d = f2v{dh[h][q0], dh[h][q0 + 1]} + hac;
          const f2v dn_ = d * omz;
          const f2v dz = d * (hin - ng);
          const f2v dnp = dn_ * (1.0f - ng * ng);
          const f2v dhn = dnp * rg;
          const f2v drp = dnp * hn * rg * (1.0f - rg);
          const f2v dzp = dz * zg * omz;
          const f2v dhv = d * zg;   // direct path; the W_h^T contraction accumulates onto it below
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int q = q0 + e, qu = qunit(q);
            dh[h][q] = dhv[e];
            drq[j0 + e] = drp[e];
            dz_r[h][q] = dzp[e];
            dhn_r[h][q] = dhn[e];
            rhq[j0 + e] = fmaxf(hout[e], 0.0f);
            dnq[j0 + e] = dnp[e];
            dx34 += f2v{drp[e], drp[e]} * wil2[0 * HU + qu] + f2v{dzp[e], dzp[e]} * wil2[1 * HU + qu] +
                    f2v{dnp[e], dnp[e]} * wil2[2 * HU + qu];
          }
        }
        dx3 = dx34.x;
        dx4 = dx34.y;
      }
#pragma unroll
      for (int jj = 0; jj < (BWD_PK ? 0 : 4); ++jj) {
        const int q = 4 * g4 + jj;
        const float hin = v[0][jj];
        const float rg = BWD_TRECOMP ? sigm_r(rc[0][h][q] * 0.5f) : v[1][jj];
        const float zg = BWD_TRECOMP ? sigm_r(rc[1][h][q] * 0.5f) : v[2][jj];
        const float hn = BWD_TRECOMP ? rc[2][h][q] * 0.5f : v[3][jj];
        const float ng = gate_n(ain[q], rg, hn);
        const float hout = (1.0f - zg) * ng + zg * hin;
        const float d = dh[h][q] + (hout > 0.0f ? hacc[q] : 0.0f);
        const float dn_ = d * (1.0f - zg);
        const float dz = d * (hin - ng);
        const float dnp = dn_ * (1.0f - ng * ng);
        const float dhn = dnp * rg;
        const float drp = dnp * hn * rg * (1.0f - rg);
        const float dzp = dz * zg * (1.0f - zg);
        dh[h][q] = d * zg;   // direct path; the W_h^T contraction accumulates onto it below
        drq[jj] = drp;
        dz_r[h][q] = dzp;
        dhn_r[h][q] = dhn;
        const int qu = qunit(q);
        dx3 += drp * wil[0 * HU + qu] + dzp * wil[1 * HU + qu] + dnp * wil[2 * HU + qu];
        dx4 += drp * wil[3 * HU + qu] + dzp * wil[4 * HU + qu] + dnp * wil[5 * HU + qu];
        rhq[jj] = fmaxf(hout, 0.0f);
        dnq[jj] = dnp;
      }
      if (st_rh) st_q(rs_rh, h, g4, rhq);
      if (st_dn) st_q(rs_dg[3], h, g4, dnq);   // dr, dz and dhn leave beside the contraction passes
      if (SMALL) small_mfma(h, g4, dnq, rhq);
      *reinterpret_cast<float4*>(&drs[rown(h) * DRP + ubn() + 8 * g4]) = make_float4(drq[0], drq[1], drq[2], drq[3]);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) rmr[h] = fmaxf(rmr[h], fabsf(drq[jj]));
      if (g4 == 3) {
        // lanes l and l + 32 hold the same row: fold the halves, one float2 per (wave, row)
        const float f3 = dx3 + __shfl_xor(dx3, 32), f4 = dx4 + __shfl_xor(dx4, 32);
        const int ln = lane_now();
        if (ln < 32) *reinterpret_cast<float2*>(dxp + (wave * RBT + RB * h + ln) * 2) = make_float2(f3, f4);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (BWD_MPRIO) __builtin_amdgcn_s_setprio(0);
    BWD_STAMP(2);
    BWD_WSTAMP(1);
    // row maxima of |dr|, |dz|, |dhn| over this wave's units (the fp16 B scale of the three passes)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float m = rmr[h];
#pragma unroll
      for (int q = 0; q < 16; ++q) m = fmaxf(m, fmaxf(fabsf(dz_r[h][q]), fabsf(dhn_r[h][q])));
      m = fmaxf(m, __shfl_xor(m, 32));
      const int ln = lane_now();
      if (ln < 32) rmx[wave * RBT + RB * h + ln] = m;
    }
    lds_barrier();   // dr staged, row maxima visible
    BWD_STAMP(3);
    // row scale 2^t (t = 14 - e, max_u max(|dr|, |dz|, |dhn|) < 2^e, clamped to [-40, 40]): the three passes
    // accumulate in the frame 2^(s_i + t_row), unscaled exactly (powers of two) after the hn pass
    float bs[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float m = 0.0f;
      const int cl = lane_now() & 31;
#pragma unroll
      for (int w8 = 0; w8 < 8; ++w8) m = fmaxf(m, rmx[w8 * RBT + RB * h + cl]);
      int sc = 0, ce = 127;
      if (m > 0.0f && m <= 3.0e38f) {
        int e;
        frexpf(m, &e);
        sc = min(40, max(-40, 14 - e));
        ce = min(126, max(-126, 14 - e));
      }
      bs[h] = ldexpf(1.0f, sc);
      if (p.CE && wave == 0 && lane_now() < 32) p.CE[ctr + r0 + rown(h)] = (int8_t)ce;
    }
    // a lane's four units ub + 8 g4 .. +3 of batch row `row` of gate cotangent g to DG, issued beside the
    // contraction's MFMAs where the memory pipe is otherwise idle
    auto store_dg = [&](int g, int row, int g4, const float (&v)[4]) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        st_u(rs_dg[g], dg_vbyte(ub, col), dg_soff(ctr, qunit(4 * g4 + e), row >= RB ? 1 : 0), v[e]);
    };
    // dr -> fp16 pieces: x0 straight into slot 0, x1 held until every lane has read its staged f32 values
    // (slot 1 overlaps the staging)
    float qv[32];   // the pass's DG store queue (BWD_SPREAD): dr, then dz, then dhn, [h][4 g4 + e]
    if (BWD_SPLACE) preload_ring(0);   // ahead of the dr stores below
    {
      f16x4 x1h[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int row = rown(h), un = ubn();
          const float4 v = *reinterpret_cast<const float4*>(&drs[row * DRP + un + 8 * g4]);
          const float v4[4] = {v.x, v.y, v.z, v.w};
          f16x4 x0;
#pragma unroll
          for (int e = 0; e < 4; ++e) split2h(v4[e] * bs[h], x0, x1h[h][g4], e);
          *reinterpret_cast<f16x4*>(&dgB[0][row * PP + un + 8 * g4]) = x0;
          if (BWD_SPREAD) {
#pragma unroll
            for (int e = 0; e < 4; ++e) qv[16 * h + 4 * g4 + e] = v4[e];
          } else {
            store_dg(0, RB * h, g4, v4);
          }
        }
      lds_barrier();
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4)
          *reinterpret_cast<f16x4*>(&dgB[1][rown(h) * PP + ubn() + 8 * g4]) = x1h[h][g4];
      lds_barrier();
    }
    // ---- contraction: dr, then dz, then dhn (scaled fp16 pairs) through the one image, accumulated onto the
    // direct path dh (taken into the accumulator frame 2^(s_i + t_row), exact: powers of two), so dh's registers
    // are free while the contraction's fragments are live
    const int un0 = ubn();
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const float4 w4 = *reinterpret_cast<const float4*>(&wsc[un0 + 8 * g4]);
      const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[h][4 * g4 + e] = dh[h][4 * g4 + e] * (wv[e] * bs[h]);
    }
    BWD_STAMP(4);
    BWD_WSTAMP(2);
    // BWD_INPASS: dz's first piece goes to the idle slot 2 during pass dr, dhn's to slot 1 (dr's second piece, read
    // through) during pass dz; the refills write only the second pieces: pass dz reads slots (2, 0), pass dhn (1, 2)
    auto inpass_put = [&](int j, int slot, const float (&src)[2][16]) {
#pragma unroll
      for (int i = 2 * j; i < 2 * j + 2; ++i) {   // (h, g4) = (i >> 2, i & 3): eight quads over the four k-steps
        const int h = i >> 2, g4 = i & 3;
        const float v4[4] = {src[h][4 * g4], src[h][4 * g4 + 1], src[h][4 * g4 + 2], src[h][4 * g4 + 3]};
        put1h(slot, 0, rown(h), ubn() + 8 * g4, v4, bs[h]);
      }
    };
    contract_h(0, 0, 1, qv, ctr, [] {}, (bool)BWD_SPLACE, BWD_SPLACE ? 1 : -1, [&] {
      if (BWD_SPLACE) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const float v4[4] = {dz_r[h][4 * g4], dz_r[h][4 * g4 + 1], dz_r[h][4 * g4 + 2], dz_r[h][4 * g4 + 3]};
            store_dg(1, RB * h, g4, v4);
          }
      }
    }, [&](int j) {
      if (BWD_INPASS) inpass_put(j, 2, dz_r);
    });
    BWD_WSTAMP(3);
    lds_barrier();
    BWD_WSTAMP(4);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const float v4[4] = {dz_r[h][4 * g4], dz_r[h][4 * g4 + 1], dz_r[h][4 * g4 + 2], dz_r[h][4 * g4 + 3]};
        if (BWD_INPASS) put1h(0, 1, rown(h), ubn() + 8 * g4, v4, bs[h]);
        else put4h(rown(h), ubn() + 8 * g4, v4, bs[h]);
        if (BWD_SPREAD) {
#pragma unroll
          for (int e = 0; e < 4; ++e) qv[16 * h + 4 * g4 + e] = v4[e];
        } else if (!BWD_SPLACE) {
          store_dg(1, RB * h, g4, v4);
        }
      }
    lds_barrier();
    BWD_STAMP(5);
    BWD_WSTAMP(5);
    contract_h(1, BWD_INPASS ? 2 : 0, BWD_INPASS ? 0 : 1, qv, ctr, [] {}, (bool)BWD_SPLACE, BWD_SPLACE ? 2 : -1, [&] {
      if (BWD_SPLACE) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const float v4[4] = {dhn_r[h][4 * g4], dhn_r[h][4 * g4 + 1], dhn_r[h][4 * g4 + 2], dhn_r[h][4 * g4 + 3]};
            store_dg(2, RB * h, g4, v4);
          }
      }
    }, [&](int j) {
      if (BWD_INPASS) inpass_put(j, 1, dhn_r);
    });
    BWD_WSTAMP(6);
    lds_barrier();
    BWD_WSTAMP(7);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const float v4[4] = {dhn_r[h][4 * g4], dhn_r[h][4 * g4 + 1], dhn_r[h][4 * g4 + 2], dhn_r[h][4 * g4 + 3]};
        if (BWD_INPASS) put1h(2, 1, rown(h), ubn() + 8 * g4, v4, bs[h]);
        else put4h(rown(h), ubn() + 8 * g4, v4, bs[h]);
        if (BWD_SPREAD) {
#pragma unroll
          for (int e = 0; e < 4; ++e) qv[16 * h + 4 * g4 + e] = v4[e];
        } else if (!BWD_SPLACE) {
          store_dg(2, RB * h, g4, v4);
        }
      }
    lds_barrier();
    BWD_STAMP(6);
    contract_h(2, BWD_INPASS ? 1 : 0, BWD_INPASS ? 2 : 1, qv, ctr, [&] {
      if (t + 1 < T) load_first(ctr + R, true);
    }, (bool)BWD_SPLACE, -1, [] {}, [](int) {});
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const float4 w4 = *reinterpret_cast<const float4*>(&wsc[32 * wave + 4 * (lane_now() >> 5) + 8 * g4]);
      const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[h][4 * g4 + e] *= inv_pow2(wv[e] * bs[h]);
    }
    if (tid < RBT) {
      const int tl = lane_now();   // == tid (wave 0)
      float s3 = 0.0f, s4 = 0.0f;
#pragma unroll
      for (int w8 = 0; w8 < 8; ++w8) {
        const float2 v = *reinterpret_cast<const float2*>(dxp + (w8 * RBT + tl) * 2);
        s3 += v.x;
        s4 += v.y;
      }
      st_u(rs_dx3, (unsigned)tl * 4, (unsigned)((ctr + r0) * 4), s3);
      st_u(rs_dx4, (unsigned)tl * 4, (unsigned)((ctr + r0) * 4), s4);
    }
    // carry to h_out(t+1): h_in(t) = where(d_t, 0, h_out(t+1))
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const bool dn = dns[RB * h + (lane_now() & 31)] != 0;
#pragma unroll
      for (int q = 0; q < 16; ++q) dh[h][q] = dn ? 0.0f : acc[h][q];
    }
    BWD_STAMP(7);
    lds_barrier();   // hv, dxp and the image are rewritten next step
  }
  if (SMALL) {
    // this workgroup's partials: C[i = 4 (l >> 4) + r][unit 32 wave + 16 uh + (l & 15)], then the head rows' sums
    float* out = p.SP + (size_t)bid * SP_FLOATS;
    const int ln = lane_now();
#pragma unroll
    for (int uh = 0; uh < 2; ++uh) {
      const floatx4 a = accl[(wave * 2 + uh) * 64 + ln];
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(4 * (ln >> 4) + r) * HU + 32 * wave + 16 * uh + (ln & 15)] = a[r];
    }
    for (int i = tid; i < 9 * RBT; i += 512) out[SP_C + i] = hvs[i];
  }
}

// TOUED_BWD_HALVES: holds its stream for q s_sleep(127) quanta
__global__ void k_sleep_quanta(int q) {
  for (int i = 0; i < q; ++i) __builtin_amdgcn_s_sleep(127);
}

// Sum of the fused small products' per-workgroup partials in a fixed order (deterministic): level 1, block (chunk c of
// 64 workgroups, 256 outputs) -> part2[c][out]; level 2 (k_small_final) the chunks in order, and the head bias column
// over the 64 rows, into GI = [8][256] ([x; 1; 0] . dn^T) | [9][257] (DH . [relu(h_out); 1]^T)
#define SR_CHUNK 64
__global__ void __launch_bounds__(256) k_small_part(const float* __restrict__ sp, int n_wg, float* __restrict__ part2) {
  const int o = blockIdx.x * 256 + threadIdx.x;
  if (o >= SP_FLOATS) return;
  const int c = blockIdx.y, w0 = c * SR_CHUNK, w1 = min(n_wg, w0 + SR_CHUNK);
  float a = 0.0f;
  for (int w = w0; w < w1; ++w) a += sp[(size_t)w * SP_FLOATS + o];
  part2[(size_t)c * SP_FLOATS + o] = a;
}
__global__ void __launch_bounds__(256) k_small_final(const float* __restrict__ part2, int n_chunk, int F,
                                                     float* __restrict__ GI) {
  const int o = blockIdx.x * 256 + threadIdx.x;   // output element of GI
  if (o >= 8 * HU + 9 * (HU + 1)) return;
  float a = 0.0f;
  if (o < 8 * HU) {                               // [x; 1; 0] . dn^T
    const int i = o / HU, u = o % HU;
    if (i <= F)
      for (int c = 0; c < n_chunk; ++c) a += part2[(size_t)c * SP_FLOATS + i * HU + u];
  } else {
    const int e = o - 8 * HU, oo = e / (HU + 1), u = e % (HU + 1);
    if (u < HU) {
      for (int c = 0; c < n_chunk; ++c) a += part2[(size_t)c * SP_FLOATS + (F + 1 + oo) * HU + u];
    } else {                                       // bias column: sum of the head cotangents over every row
      for (int c = 0; c < n_chunk; ++c) {
        float rs = 0.0f;
        for (int r = 0; r < 64; ++r) rs += part2[(size_t)c * SP_FLOATS + SP_C + oo * 64 + r];
        a += rs;
      }
    }
  }
  GI[o] = a;
}

}  // namespace

extern "C" {

int toued_gru_pack(const float* eta, const int* off, int F, float* fwdA, float* bwdA, hipStream_t stream) {
  TOUED_REQUIRE(F >= 1 && F <= 7, "toued_gru_pack: F=%d", F);
  EtaOff o;
  memcpy(&o, off, sizeof(EtaOff));
  const int n1 = NTILE_F * KQF * 64, n2 = 8 * 3 * 32 * 64, n3 = F6_NGRP * 64;
  hipLaunchKernelGGL(k_pack_fwd, dim3((n1 + 255) / 256), dim3(256), 0, stream, eta, o, F,
                     reinterpret_cast<float4*>(fwdA), 0L, 0L);
  hipLaunchKernelGGL(k_fwd6_scales, dim3(16), dim3(256), 0, stream, eta, o, fwdA + (size_t)n1 * 4 + F6_SCALES, 0L, 0L);
  hipLaunchKernelGGL(k_pack_fwd6, dim3((n3 + 255) / 256), dim3(256), 0, stream, eta, o, F,
                     reinterpret_cast<bf16x8*>(fwdA + (size_t)n1 * 4), 0L, 0L);
  hipLaunchKernelGGL(k_pack_bwd, dim3((n2 + 255) / 256), dim3(256), 0, stream, eta, o,
                     reinterpret_cast<float4*>(bwdA));
  hipLaunchKernelGGL(k_bwd6_scales, dim3(HU / 4), dim3(256), 0, stream, eta, o, bwdA + (size_t)n2 * 4 + B6_SCALES);
  hipLaunchKernelGGL(k_pack_bwd6, dim3((16 * 8 * 3 * 64 + 255) / 256), dim3(256), 0, stream, eta, o,
                     reinterpret_cast<__bf16*>(bwdA + (size_t)n2 * 4));
  TOUED_CHECK_LAUNCH();
  return 0;
}

// which: 0 = forward fragments (f32 MFMA, then the bf16-split pieces), 1 = backward, 2 = one candidate's forward
// fragments in a toued_gru_pack_fwd_multi buffer (the same layout as 0)
size_t toued_gru_packed_floats(int which) {
  const size_t f32_part = (size_t)NTILE_F * KQF * 64 * 4;
  return which == 1 ? (size_t)8 * 3 * 32 * 64 * 4 + B6_FLOATS : f32_part + F6_FLOATS;
}

static bool gru_f32_forced() {
  static const bool f = [] {
    const char* e = getenv("TOUED_GRU_F32");
    return e && e[0] == '1';
  }();
  return f;
}

static int gru_fwd_launch(int R, int T, int W, int F, const float* X, long xs_f, long xs_col, const uint8_t* done,
                          const float* fwdA, const float* eta, const int* off, float* pi_hat, float* y_hat,
                          float* s_hin, float* s_r, float* s_z, float* s_n, float* s_hn, long M, int save, int rpc,
                          long eta_stride, hipStream_t stream) {
  FwdArgs p;
  p.R = R; p.T = T; p.W = W; p.F = F; p.X = X; p.xs_f = xs_f; p.xs_col = xs_col; p.done = done;
  p.A = reinterpret_cast<const float4*>(fwdA); p.eta = eta;
  p.A6 = fwdA + (size_t)NTILE_F * KQF * 64 * 4;
  memcpy(&p.o, off, sizeof(EtaOff));
  p.pi_hat = pi_hat; p.y_hat = y_hat; p.s_hin = s_hin; p.s_r = s_r; p.s_z = s_z; p.s_n = s_n; p.s_hn = s_hn; p.M = M;
  p.rpc = rpc; p.a_stride4 = (long)toued_gru_packed_floats(2) / 4; p.eta_stride = eta_stride;
  // 3 quanta (~24 k cycles, about half a step): gru_fwd_multi 2.399 -> 2.363 ms at C4 (2 and 5: 2.372 / 2.363)
  static const int stagger = getenv("TOUED_FWD_STAGGER") ? atoi(getenv("TOUED_FWD_STAGGER")) : 3;
  // the SAVE instance (shared, L2-resident fragments) gains nothing from it: 1.064 ms vs 1.071 / 1.076 at 3 / 5
  static const int stagger_save = getenv("TOUED_FWD_STAGGER_SAVE") ? atoi(getenv("TOUED_FWD_STAGGER_SAVE")) : 0;
  p.stagger = save ? stagger_save : stagger;
  // two row tiles per workgroup when the rows (and, for per-candidate parameters, each candidate's rows)
  // split into 64-row blocks
  const bool nt2 = R % (2 * RB) == 0 && (rpc == 0 || rpc % (2 * RB) == 0);
  // (round 5's k_gru_fwd6h, the SAVE instance as two 32-row workgroups per CU, measured 1.24 vs 1.18 ms and was
  // removed in round 6; the f32 fallback pair below keeps its own saves, n included)
  if (nt2 && !gru_f32_forced()) {
    if (save) hipLaunchKernelGGL(k_gru_fwd6<true>, dim3(R / (2 * RB)), dim3(512), 0, stream, p);
    else hipLaunchKernelGGL(k_gru_fwd6<false>, dim3(R / (2 * RB)), dim3(512), 0, stream, p);
  } else if (save) {
    if (nt2) hipLaunchKernelGGL((k_gru_fwd<true, 2>), dim3(R / (2 * RB)), dim3(512), 0, stream, p);
    else hipLaunchKernelGGL((k_gru_fwd<true, 1>), dim3(R / RB), dim3(512), 0, stream, p);
  } else {
    if (nt2) hipLaunchKernelGGL((k_gru_fwd<false, 2>), dim3(R / (2 * RB)), dim3(512), 0, stream, p);
    else hipLaunchKernelGGL((k_gru_fwd<false, 1>), dim3(R / RB), dim3(512), 0, stream, p);
  }
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_gru_fwd(int R, int T, int W, int F, const float* X, long xs_f, long xs_col, const uint8_t* done,
                  const float* fwdA, const float* eta, const int* off, float* pi_hat, float* y_hat, float* s_hin,
                  float* s_r, float* s_z, float* s_n, float* s_hn, long M, hipStream_t stream) {
  TOUED_REQUIRE(R % RB == 0 && W % RB == 0, "toued_gru_fwd: rows R=%d and workers W=%d must be multiples of 32", R, W);
  TOUED_REQUIRE(F >= 1 && F <= 7 && T >= 1, "toued_gru_fwd: F=%d T=%d", F, T);
  TOUED_REQUIRE((double)M * 264.0 * 4.0 < 4294967295.0, "toued_gru_fwd: M=%ld columns exceed the 4 GiB buffer range "
                "(use --num_mini_batches to split the agent batch)", M);
  TOUED_REQUIRE(s_hin && s_r && s_z && s_n && s_hn, "toued_gru_fwd: saved-activation buffers required");
  return gru_fwd_launch(R, T, W, F, X, xs_f, xs_col, done, fwdA, eta, off, pi_hat, y_hat, s_hin, s_r, s_z, s_n, s_hn,
                        M, 1, 0, 0, stream);
}

int toued_gru_pack_fwd_multi(const float* eta, long eta_stride, int n, const int* off, int F, float* fwdA,
                             hipStream_t stream) {
  TOUED_REQUIRE(F >= 1 && F <= 7 && n >= 0, "toued_gru_pack_fwd_multi: F=%d n=%d", F, n);
  if (n == 0) return 0;
  EtaOff o;
  memcpy(&o, off, sizeof(EtaOff));
  const int n1 = NTILE_F * KQF * 64;
  const long cstride = (long)toued_gru_packed_floats(2);   // floats per candidate
  hipLaunchKernelGGL(k_pack_fwd, dim3((n1 + 255) / 256, n), dim3(256), 0, stream, eta, o, F,
                     reinterpret_cast<float4*>(fwdA), eta_stride, cstride / 4);
  const int n3 = F6_NGRP * 64;
  hipLaunchKernelGGL(k_fwd6_scales, dim3(16, n), dim3(256), 0, stream, eta, o, fwdA + (size_t)n1 * 4 + F6_SCALES,
                     eta_stride, cstride);
  hipLaunchKernelGGL(k_pack_fwd6, dim3((n3 + 255) / 256, n), dim3(256), 0, stream, eta, o, F,
                     reinterpret_cast<bf16x8*>(fwdA + (size_t)n1 * 4), eta_stride, cstride / 4);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_gru_fwd_multi(int R, int T, int W, int F, int rows_per_cand, const float* X, long xs_f, long xs_col,
                        const uint8_t* done, const float* fwdA, const float* eta, long eta_stride, const int* off,
                        float* pi_hat, float* y_hat, hipStream_t stream) {
  TOUED_REQUIRE(R % RB == 0 && W % RB == 0, "toued_gru_fwd_multi: rows R=%d and workers W=%d must be multiples of 32",
                R, W);
  TOUED_REQUIRE(rows_per_cand > 0 && rows_per_cand % RB == 0 && R % rows_per_cand == 0,
                "toued_gru_fwd_multi: rows_per_cand=%d must be a multiple of 32 dividing R=%d", rows_per_cand, R);
  TOUED_REQUIRE(F >= 1 && F <= 7 && T >= 1, "toued_gru_fwd_multi: F=%d T=%d", F, T);
  return gru_fwd_launch(R, T, W, F, X, xs_f, xs_col, done, fwdA, eta, off, pi_hat, y_hat, nullptr, nullptr, nullptr,
                        nullptr, nullptr, 0, 0, rows_per_cand, eta_stride, stream);
}

// 1 when toued_gru_bwd runs the lockstep split-precision kernel for R rows, which writes col_exp
int toued_gru_bwd_col_exp(int R) { return R % (2 * RB) == 0 && !gru_f32_forced() ? 1 : 0; }

int toued_gru_bwd(int R, int T, int W, int K, const uint8_t* done, long done_stride_k, const float* bwdA,
                  const float* eta, const int* off, const float* y_hat, const float* d_pi_hat, const float* d_y_hat,
                  const float* s_hin, const float* s_r, const float* s_z, const float* s_n, const float* s_hn, long M,
                  float* DG, float* RH, float* DH, float* dX3, float* dX4, int8_t* col_exp, hipStream_t stream) {
  TOUED_REQUIRE(R % RB == 0 && W % RB == 0, "toued_gru_bwd: rows R=%d and workers W=%d must be multiples of 32", R, W);
  TOUED_REQUIRE((double)M * 264.0 * 4.0 < 4294967295.0, "toued_gru_bwd: M=%ld columns exceed the 4 GiB buffer range",
                M);
  BwdArgs p{};
  p.R = R; p.T = T; p.W = W; p.K = K; p.done = done; p.done_stride_k = done_stride_k;
  p.A = reinterpret_cast<const float4*>(bwdA); p.eta = eta;
  p.A6 = bwdA + (size_t)8 * 3 * 32 * 64 * 4;
  memcpy(&p.o, off, sizeof(EtaOff));
  p.y_hat = y_hat; p.d_pi_hat = d_pi_hat; p.d_y_hat = d_y_hat;
  p.s_hin = s_hin; p.s_r = s_r; p.s_z = s_z; p.s_n = s_n; p.s_hn = s_hn; p.M = M;
  p.DG = DG; p.RH = RH; p.DH = DH; p.dX3 = dX3; p.dX4 = dX4; p.CE = col_exp;
  p.F = (p.o.ir_b - p.o.in_w) / HU;   // in_w [F][256] is followed by ir_b in the flat layout (lpg.LPGLayout)
  TOUED_REQUIRE(p.F >= 1 && p.F <= 7 && p.o.ir_b - p.o.in_w == p.F * HU, "toued_gru_bwd: LPG layout F=%d", p.F);
  p.SP = nullptr;
  if (toued_gru_bwd_col_exp(R))
    hipLaunchKernelGGL(k_gru_bwd6n<false>, dim3(K * (R / (2 * RB))), dim3(512), 0, stream, p);
  else
    hipLaunchKernelGGL(k_gru_bwd<1>, dim3(K * (R / RB)), dim3(512), 0, stream, p);
  TOUED_CHECK_LAUNCH();
  return 0;
}

// 1 when the forward / backward for R rows keep r, z, W_hn h + b_hn in 32-column slab blocks (the split-precision pair)
int toued_gru_slab_saves(int R) { return toued_gru_bwd_col_exp(R); }
// 1 when the slab saves include h_in (A's first 256 rows' region; 0 only in HIN_SLAB=0 comparison builds)
int toued_gru_hin_slab(void) { return HIN_SLAB; }

// 1 when toued_gru_bwd_fused applies: the lockstep kernel (R a multiple of 64) with F + 10 <= 16 A rows
int toued_gru_bwd_fused_fits(int R, int F) { return toued_gru_bwd_col_exp(R) && F >= 1 && F <= 6 ? 1 : 0; }

size_t toued_gru_bwd_fused_work_floats(int R, int K) {
  const long n_wg = (long)K * (R / (2 * RB)), n_chunk = (n_wg + SR_CHUNK - 1) / SR_CHUNK;
  return (size_t)(n_wg + n_chunk) * SP_FLOATS;
}

// The backward with the small weight-gradient products fused (k_gru_bwd6n<true>): writes the three contraction
// cotangents DG = [dr_pre; dz_pre; d(hn)] (the main reduction's B operand), the column exponents, dX3/dX4, and GI =
// [8][256] ([x; 1; 0] . dn^T) | [9][257] (DH . [relu(h_out); 1]^T) through per-workgroup partials reduced in a fixed
// order.  dn_pre, relu(h_out) and DH are not streamed to HBM.
int toued_gru_bwd_fused(int R, int T, int W, int K, const uint8_t* done, long done_stride_k, const float* bwdA,
                        const float* eta, const int* off, const float* y_hat, const float* d_pi_hat,
                        const float* d_y_hat, const float* s_hin, const float* s_r, const float* s_z,
                        const float* s_hn, long M, float* DG3, float* dX3, float* dX4, int8_t* col_exp, float* GI,
                        float* work, size_t work_floats, hipStream_t stream) {
  TOUED_REQUIRE(R % (2 * RB) == 0 && W % RB == 0 && !gru_f32_forced(),
                "toued_gru_bwd_fused: rows R=%d must be a multiple of 64 (W=%d), split-precision kernels", R, W);
  TOUED_REQUIRE((double)M * 264.0 * 4.0 < 4294967295.0, "toued_gru_bwd_fused: M=%ld columns exceed the 4 GiB range",
                M);
  TOUED_REQUIRE(M == (long)K * T * R, "toued_gru_bwd_fused: M=%ld != K*T*R", M);
  TOUED_REQUIRE(work_floats >= toued_gru_bwd_fused_work_floats(R, K), "toued_gru_bwd_fused: workspace %zu < %zu",
                work_floats, toued_gru_bwd_fused_work_floats(R, K));
  TOUED_REQUIRE(col_exp != nullptr, "toued_gru_bwd_fused: col_exp is required");
  BwdArgs p{};
  p.R = R; p.T = T; p.W = W; p.K = K; p.done = done; p.done_stride_k = done_stride_k;
  p.A = reinterpret_cast<const float4*>(bwdA); p.eta = eta;
  p.A6 = bwdA + (size_t)8 * 3 * 32 * 64 * 4;
  memcpy(&p.o, off, sizeof(EtaOff));
  p.y_hat = y_hat; p.d_pi_hat = d_pi_hat; p.d_y_hat = d_y_hat;
  p.s_hin = s_hin; p.s_r = s_r; p.s_z = s_z; p.s_n = nullptr; p.s_hn = s_hn; p.M = M;
  p.DG = DG3; p.RH = nullptr; p.DH = nullptr; p.dX3 = dX3; p.dX4 = dX4; p.CE = col_exp;
  p.F = (p.o.ir_b - p.o.in_w) / HU;
  TOUED_REQUIRE(p.F >= 1 && p.F <= 6 && p.o.ir_b - p.o.in_w == p.F * HU, "toued_gru_bwd_fused: LPG layout F=%d", p.F);
  const int n_wg = K * (R / (2 * RB)), n_chunk = (n_wg + SR_CHUNK - 1) / SR_CHUNK;
  p.SP = work;
  {
    static const char* e = getenv("TOUED_BWD_STAGGER");   // "quanta[,mode]" (study; default off)
    p.stagger = e ? atoi(e) : 0;
    p.stagger_mode = e && strchr(e, ',') ? atoi(strchr(e, ',') + 1) : 0;
  }
  float* part2 = work + (size_t)n_wg * SP_FLOATS;
  // TOUED_BWD_HALVES=q (study): the grid as two launches on two CU-masked streams (alternate CUs), the second half q
  // s_sleep quanta (~8 k cycles each) late, so the two halves' memory parts and passes stay out of phase
  static const int halves = getenv("TOUED_BWD_HALVES") ? atoi(getenv("TOUED_BWD_HALVES")) : -1;
  if (halves >= 0 && n_wg >= 2) {
    static hipStream_t sh[2] = {nullptr, nullptr};
    static hipEvent_t ev[3];
    if (!sh[0]) {
      int dev = 0, ncu = 0;
      TOUED_REQUIRE(hipGetDevice(&dev) == hipSuccess &&
                        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess,
                    "toued_gru_bwd_fused: device query failed");
      uint32_t m[2][16] = {};
      for (int c = 0; c < ncu && c < 512; ++c) m[c & 1][c >> 5] |= 1u << (c & 31);
      const uint32_t nw = (uint32_t)((ncu + 31) / 32);
      for (int h = 0; h < 2; ++h)
        TOUED_REQUIRE(hipExtStreamCreateWithCUMask(&sh[h], nw, m[h]) == hipSuccess, "CU-masked stream");
      for (int i = 0; i < 3; ++i) TOUED_REQUIRE(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) == hipSuccess, "ev");
    }
    (void)hipEventRecord(ev[0], stream);
    const int n1 = n_wg / 2;
    for (int h = 0; h < 2; ++h) {
      (void)hipStreamWaitEvent(sh[h], ev[0], 0);
      BwdArgs q = p;
      q.wg_base = h ? n1 : 0;
      q.stagger = 0;
      if (h && halves > 0) hipLaunchKernelGGL(k_sleep_quanta, dim3(1), dim3(64), 0, sh[h], halves);
      hipLaunchKernelGGL(k_gru_bwd6n<true>, dim3(h ? n_wg - n1 : n1), dim3(512), 0, sh[h], q);
      (void)hipEventRecord(ev[1 + h], sh[h]);
      (void)hipStreamWaitEvent(stream, ev[1 + h], 0);
    }
  } else {
    hipLaunchKernelGGL(k_gru_bwd6n<true>, dim3(n_wg), dim3(512), 0, stream, p);
  }
  hipLaunchKernelGGL(k_small_part, dim3((SP_FLOATS + 255) / 256, n_chunk), dim3(256), 0, stream, work, n_wg, part2);
  hipLaunchKernelGGL(k_small_final, dim3((8 * HU + 9 * (HU + 1) + 255) / 256), dim3(256), 0, stream, part2, n_chunk,
                     p.F, GI);
  TOUED_CHECK_LAUNCH();
  return 0;
}

#ifdef FWD_STAMPS
int toued_dbg_fwd_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fwd_stamps), sizeof(g_fwd_stamps)) == hipSuccess ? 0 : 1;
}
int toued_dbg_fwd_gm_stamps(unsigned long long* host) {   // [64 workgroups][32 steps][4]
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fwd_gm), sizeof(g_fwd_gm)) == hipSuccess ? 0 : 1;
}
int toued_dbg_fwd_pp_stamps(unsigned long long* host) {   // [64 workgroups][32 steps][2 halves][6]
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fwd_pp), sizeof(g_fwd_pp)) == hipSuccess ? 0 : 1;
}
#endif

#ifdef BWD_STAMPS
int toued_dbg_bwd_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_bwd_stamps), sizeof(g_bwd_stamps)) == hipSuccess ? 0 : 1;
}
int toued_dbg_bwd_wstamps(unsigned long long* host, int* simd) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_bwd_wstamps), sizeof(g_bwd_wstamps)) == hipSuccess &&
                 hipMemcpyFromSymbol(simd, HIP_SYMBOL(g_bwd_wsimd), sizeof(g_bwd_wsimd)) == hipSuccess
             ? 0
             : 1;
}
#endif

size_t toued_gru_bwd_small_work_floats(long M) {
  return std::max(toued_wgrad_workspace_floats(8, HU, M),
                  std::max(toued_wgrad_workspace_floats(9, HU, M), toued_rowsum_workspace_floats(9, M)));
}

// the backward's small weight-gradient reductions (HBM streams over dn, relu(h_out) and the head cotangents):
// GI = [8][256] ([X; 1; 0] . dn^T) | [9][257] (DH . [relu(h_out); 1]^T).  (Folding them into the lockstep
// kernel was measured: its register file is full and the spills cost more than the 7 GB of streams saved.)
// The head block's bias column (DH's row sums) is a separate row-sum reduction: as a 257th B row it made the
// column tiles of 128 rows three instead of two, each K chunk 1.5x longer (1.04 vs 0.65 ms per launch).
int toued_gru_bwd_small(long M, const float* s_hin, const float* DG, const float* RH, const float* DH, float* GI,
                        float* work, size_t work_floats, hipStream_t stream) {
  TOUED_REQUIRE(work_floats >= toued_gru_bwd_small_work_floats(M), "toued_gru_bwd_small: workspace %zu < %zu floats",
                work_floats, toued_gru_bwd_small_work_floats(M));
  int rc = toued_wgrad(8, HU, M, s_hin + (size_t)HU * M, M, DG + (size_t)3 * HU * M, M, GI, work, work_floats, stream);
  if (rc) return rc;
  // TOUED_HEADS_SPLIT=0: the bias as a 257th B row (comparison runs).  The row sums go first: issued between the
  // head product and the main reduction they left k_wgrad_h3 at 5.9-7.1 ms instead of 4.0-4.1 (measured, same box;
  // padding the final row-sum grid to a multiple of 8 workgroups changed nothing)
  static const bool split = [] {
    const char* e = getenv("TOUED_HEADS_SPLIT");
    return !(e && e[0] == '0');
  }();
  if (!split) return toued_wgrad(9, HU + 1, M, DH, M, RH, M, GI + 8 * HU, work, work_floats, stream);
  rc = toued_rowsum_into(9, M, DH, M, GI + 8 * HU + HU, HU + 1, work, work_floats, stream);
  if (rc) return rc;
  return toued_wgrad_ldc(9, HU, M, DH, M, RH, M, GI + 8 * HU, HU + 1, work, work_floats, stream);
}

}  // extern "C"
