// Wave-level building blocks shared by the deterministic per-agent row kernels (a2c.hip, agent.hip): DPP lane
// exchanges, a DPP wave sum, and a 2048-key bitonic sort held in registers.  Internal linkage (device code only).
#pragma once
#include "common.h"

namespace {

// DPP moves for patterns whose every source lane is valid (quad permutes, row rotates and mirrors): the old value
// is never used, so it is left undefined (no zeroing move ahead of each DPP)
template <int CTRL>
TOUED_DEV uint32_t dpp_u(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
TOUED_DEV float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

// x of lane ^ M: one VALU move for M = 1, 2 (DPP quad permutes) and M = 8 (row_ror:8 -- rotating a 16-lane row by 8
// is xor 8), an LDS-crossbar swizzle for M = 4 and 16 (bit mode: and 0x1F, xor M), a permute for M = 32.  All 64
// lanes must be active.
template <int M>
TOUED_DEV uint32_t lane_xor(uint32_t x, int lane) {
  (void)lane;
  if constexpr (M == 1) {
    return dpp_u<0xB1>(x);                                 // quad_perm [1, 0, 3, 2]
  } else if constexpr (M == 2) {
    return dpp_u<0x4E>(x);                                 // quad_perm [2, 3, 0, 1]
  } else if constexpr (M == 8) {
    return dpp_u<0x128>(x);                                // row_ror:8
  } else if constexpr (M == 4 || M == 16) {
    return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (M << 10));
  } else {
    return (uint32_t)__shfl_xor((int)x, M, 64);
  }
}

// Unsigned median of three (one v_med3_u32): with c = 0 it is min(a, b), with c = ~0u max(a, b), so a compare-exchange
// whose direction is a per-lane mask costs one instruction per element.
TOUED_DEV uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) { return max(min(a, b), min(max(a, b), c)); }

// 0 or ~0u: bit B of v
template <int B>
TOUED_DEV uint32_t bitmask_of(uint32_t v) { return (uint32_t)(-(int)((v >> B) & 1u)); }

// Wave sum, every lane gets it: the xor butterfly 1, 2, 4, 8, 16, 32 with the first four steps as DPP moves (quad
// permutes, half-row and row mirrors: after the quad sums, lane i's mirror partner holds the same partial as its xor
// partner), xor 16 as a swizzle and the last step on the two half sums -- the same additions in the same order as
// the __shfl_xor butterfly (bit-identical), without its six LDS-crossbar permutes.  All 64 lanes must be active.
TOUED_DEV float wsum_dpp(float v) {
  v += dpp_f<0xB1>(v);    // xor 1
  v += dpp_f<0x4E>(v);    // xor 2
  v += dpp_f<0x141>(v);   // row_half_mirror: the other quad of the 8
  v += dpp_f<0x140>(v);   // row_mirror: the other 8 of the row
  v += __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v), 0x401F));   // xor 16
  const float lo = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
  const float hi = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
  return lo + hi;
}

// Bitonic sort of 2048 keys in LDS by NT threads (256 or 512), in registers: wave w holds keys [WB w, WB w + WB),
// WB = 64 KPL, lane l the KPL = 2048 / NT keys WB w + KPL l + r.  Stages with partner distance j < KPL are
// compare-selects between a lane's own registers, KPL <= j < WB exchange registers between lanes (lane_xor), and
// the stages with j >= WB exchange whole blocks through LDS between waves.  Every element keeps min or max of itself
// and its partner i ^ j: min when (i & j == 0) == ascending, ascending = (i & k == 0).  The keep-min/keep-max choice
// is a per-lane mask (0 / ~0u) and the exchange one umed3 per element.
template <int NT, int K, int J>
TOUED_DEV void bitonic_stage(uint32_t (&x)[2048 / NT], uint32_t* key, int lane, int wv) {
  constexpr int KPL = 2048 / NT, WB = 64 * KPL, NQ = KPL / 4;
  constexpr int LK = __builtin_ctz(K);
  const uint32_t base = (uint32_t)(WB * wv + KPL * lane);   // element index of register 0
  if constexpr (J < KPL) {
#pragma unroll
    for (int r = 0; r < KPL; ++r) {
      if ((r & J) == 0) {
        // descending mask: bit LK of the element index (r's own bits when K < KPL, else base's)
        const uint32_t desc = K < KPL ? ((r & K) ? ~0u : 0u) : bitmask_of<LK>(base);
        const uint32_t a = x[r], b = x[r | J];
        x[r] = umed3(a, b, desc);
        x[r | J] = umed3(a, b, ~desc);
      }
    }
  } else if constexpr (J < WB) {
    constexpr int M = J / KPL, LM = __builtin_ctz(M);
    // keep max when (lane is the upper partner) != (descending); K > J >= KPL, so desc does not depend on r
    const uint32_t keep = bitmask_of<LM>((uint32_t)lane) ^ bitmask_of<LK>(base);
#pragma unroll
    for (int r = 0; r < KPL; ++r) {
      const uint32_t p = lane_xor<M>(x[r], lane);
      x[r] = umed3(x[r], p, keep);
    }
  } else {
    uint4* kv = reinterpret_cast<uint4*>(key);
    const int me = (WB * wv + KPL * lane) / 4, pa = (WB * (wv ^ (J / WB)) + KPL * lane) / 4;
#pragma unroll
    for (int q = 0; q < NQ; ++q) kv[me + q] = make_uint4(x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
    __syncthreads();
    uint32_t p[KPL];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint4 v = kv[pa + q];
      p[4 * q] = v.x; p[4 * q + 1] = v.y; p[4 * q + 2] = v.z; p[4 * q + 3] = v.w;
    }
    const uint32_t keep = ((wv & (J / WB)) ? ~0u : 0u) ^ bitmask_of<LK>(base);
#pragma unroll
    for (int r = 0; r < KPL; ++r) x[r] = umed3(x[r], p[r], keep);
    __syncthreads();   // every partner read before the next stage's writes
  }
}

template <int NT, int K, int J>
TOUED_DEV void bitonic_merge(uint32_t (&x)[2048 / NT], uint32_t* key, int lane, int wv) {
  bitonic_stage<NT, K, J>(x, key, lane, wv);
  if constexpr (J > 1) bitonic_merge<NT, K, J / 2>(x, key, lane, wv);
}

template <int NT, int K>
TOUED_DEV void bitonic_levels(uint32_t (&x)[2048 / NT], uint32_t* key, int lane, int wv) {
  bitonic_merge<NT, K, K / 2>(x, key, lane, wv);
  if constexpr (K < 2048) bitonic_levels<NT, 2 * K>(x, key, lane, wv);
}

// Begins and ends with a workgroup barrier; the sorted keys are back in `key`.
template <int NT>
TOUED_DEV void sort2048_reg(uint32_t* key, int tid) {
  constexpr int KPL = 2048 / NT, WB = 64 * KPL, NQ = KPL / 4;
  const int lane = tid & 63, wv = tid >> 6;
  __syncthreads();
  uint4* kv = reinterpret_cast<uint4*>(key);
  const int me = (WB * wv + KPL * lane) / 4;
  uint32_t x[KPL];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const uint4 v = kv[me + q];
    x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
  }
  bitonic_levels<NT, 2>(x, key, lane, wv);
#pragma unroll
  for (int q = 0; q < NQ; ++q) kv[me + q] = make_uint4(x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
  __syncthreads();
}

}  // namespace
