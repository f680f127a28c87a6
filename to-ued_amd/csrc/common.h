// Shared device helpers for the TO-UED MI355X hot path (gfx950 / CDNA4).
//
//  * threefry2x32-20 and the jax.random key-derivation helpers (split, random
//    bits, uniform) — integer-exact restatement of jax 0.4.13's PRNG, the one
//    every env transition and level index depends on.
//  * Portable f32 exp/log: the exact op sequence of oracle/pmath.py, so that
//    GPU and oracle agree bit-for-bit on everything that steers sampling.
//    This TU family is compiled with -ffp-contract=off.
//  * The packed level layout (int32[64] per level) and env-state SoA layout.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <atomic>

#define TOUED_DEV __device__ __forceinline__

// ----------------------------------------------------------------------------
// Packed level record (oracle/levels.py pack_levels)
enum {
  L_MAX_STEPS = 0, L_GRID = 1, L_START = 2, L_NOBJS = 3, L_RANDRESP = 4, L_LIFETIME = 5,
  L_BUFID = 6, L_OBJ_IDS = 8, L_STATIC = 16, L_REW = 24, L_PTERM = 32, L_PRESP = 40,
  L_WALLS = 48,
  // the EnvParams per-type tables (obj_rewards, obj_p_terminate, obj_p_respawn, zero past max_n_obj_types) and
  // auto_collect, kept so that a level round-trips to the reference's Level pytree (checkpoints)
  L_TREW = 64, L_TPTERM = 69, L_TPRESP = 74, L_AUTOC = 79, LEVEL_WORDS = 80
};
#define TOUED_MAX_TYPES 5
// Env state, SoA over workers: field f of worker i at state[f * n + i].
enum { S_TIME = 0, S_POS = 1, S_EXISTS = 2, S_TERM = 3, S_OBJ = 4, S_FIELDS = 12 };
#define TOUED_MAX_OBJS 8

struct EnvSpec {
  int max_grid;   // max_grid_size
  int n_max;      // max_n_objs
  int n_types;    // max_n_obj_types
  int tabular;    // 1 = tabular observation / static respawn
};

// ----------------------------------------------------------------------------
// threefry2x32-20 (jax/_src/prng.py _threefry2x32_lowering)
// 4x4 transpose between a lane quad (four consecutive rows: lanes 4i..4i+3) and a register quad (four
// consecutive units): before, lane row j holds units u0..u0+3; after, lane u0+i's data (for rows j0..j0+3)
// sits in lane j0+i.  Two DPP quad_perm exchange stages; the transpose is its own inverse.
TOUED_DEV float dpp_swap(float v, int ctrl_sel) {
  const int x = __float_as_int(v);
  return __int_as_float(ctrl_sel == 2 ? __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false)     // [2,3,0,1]
                                      : __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false));   // [1,0,3,2]
}
TOUED_DEV void quad_transpose(float* a, int lane) {
  const bool b1 = (lane & 2) != 0, b0 = (lane & 1) != 0;
  float r0 = dpp_swap(b1 ? a[0] : a[2], 2), r1 = dpp_swap(b1 ? a[1] : a[3], 2);
  if (b1) { a[0] = r0; a[1] = r1; } else { a[2] = r0; a[3] = r1; }
  r0 = dpp_swap(b0 ? a[0] : a[1], 1);
  r1 = dpp_swap(b0 ? a[2] : a[3], 1);
  if (b0) { a[0] = r0; a[2] = r1; } else { a[1] = r0; a[3] = r1; }
}

TOUED_DEV uint32_t rotl32(uint32_t v, uint32_t r) { return (v << r) | (v >> (32u - r)); }

// Workgroup barrier for LDS-only communication: waits for this wave's LDS (and scalar) accesses and meets the other
// waves, without __syncthreads()'s workgroup-scope release fence, which also waits for every outstanding global load
// and store of the wave (vmcnt(0)).  In the MFMA kernels that stream stores and prefetch loads across their phases
// that drain sat on every barrier (k_gru_bwd6n stamps: ~20 % of a step).  Only where no wave reads global memory that
// another wave of the workgroup wrote inside the kernel.
TOUED_DEV void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

TOUED_DEV uint2 threefry(uint32_t k0, uint32_t k1, uint32_t x0, uint32_t x1) {
  const uint32_t k2 = k0 ^ k1 ^ 0x1BD11BDAu;
  x0 += k0;
  x1 += k1;
#define TF_R(r) { x0 += x1; x1 = rotl32(x1, r); x1 ^= x0; }
  TF_R(13) TF_R(15) TF_R(26) TF_R(6)  x0 += k1; x1 += k2 + 1u;
  TF_R(17) TF_R(29) TF_R(16) TF_R(24) x0 += k2; x1 += k0 + 2u;
  TF_R(13) TF_R(15) TF_R(26) TF_R(6)  x0 += k0; x1 += k1 + 3u;
  TF_R(17) TF_R(29) TF_R(16) TF_R(24) x0 += k1; x1 += k2 + 4u;
  TF_R(13) TF_R(15) TF_R(26) TF_R(6)  x0 += k2; x1 += k0 + 5u;
#undef TF_R
  return make_uint2(x0, x1);
}

// Element j of threefry_2x32(key, iota(count)) (odd counts padded with a 0 counter).
TOUED_DEV uint32_t random_bits_at(uint2 key, uint32_t count, uint32_t j) {
  const uint32_t nb = (count + 1u) >> 1;
  const uint32_t b = (j < nb) ? j : j - nb;
  const uint32_t hi = b + nb;
  const uint2 y = threefry(key.x, key.y, b, hi < count ? hi : 0u);
  return (j < nb) ? y.x : y.y;
}

// jax.random.split(key, num)[i]
TOUED_DEV uint2 split_at(uint2 key, uint32_t num, uint32_t i) {
  return make_uint2(random_bits_at(key, 2u * num, 2u * i), random_bits_at(key, 2u * num, 2u * i + 1u));
}

// split(key) -> (a, b): blocks (0,2),(1,3); out = [b0.x, b1.x, b0.y, b1.y]
TOUED_DEV void split2(uint2 key, uint2& a, uint2& b) {
  const uint2 y0 = threefry(key.x, key.y, 0u, 2u);
  const uint2 y1 = threefry(key.x, key.y, 1u, 3u);
  a = make_uint2(y0.x, y1.x);
  b = make_uint2(y0.y, y1.y);
}

// split(key, 3): blocks (0,3),(1,4),(2,5); out = [b0.x,b1.x,b2.x,b0.y,b1.y,b2.y]
TOUED_DEV void split3(uint2 key, uint2& a, uint2& b, uint2& c) {
  const uint2 y0 = threefry(key.x, key.y, 0u, 3u);
  const uint2 y1 = threefry(key.x, key.y, 1u, 4u);
  const uint2 y2 = threefry(key.x, key.y, 2u, 5u);
  a = make_uint2(y0.x, y1.x);
  b = make_uint2(y2.x, y0.y);
  c = make_uint2(y1.y, y2.y);
}

// random_bits(key, 32, ()) : single element -> block (0, 0 pad), first output.
TOUED_DEV uint32_t bits1(uint2 key) { return threefry(key.x, key.y, 0u, 0u).x; }

TOUED_DEV float bits_to_unit(uint32_t bits) {
  return __uint_as_float((bits >> 9) | 0x3F800000u) - 1.0f;
}

// jax.random.uniform(minval, maxval): max(lo, f*(hi-lo)+lo), no contraction.
TOUED_DEV float uniform_from_bits(uint32_t bits, float lo, float hi) {
  const float f = bits_to_unit(bits);
  return fmaxf(lo, __fadd_rn(__fmul_rn(f, __fsub_rn(hi, lo)), lo));
}

// ----------------------------------------------------------------------------
// Portable math (oracle/pmath.py)
TOUED_DEV float pow2i(int k) { return __uint_as_float((uint32_t)(k + 127) << 23); }

TOUED_DEV float pexp_core(float x) {
  const float k = rintf(__fmul_rn(x, 1.44269504088896341f));
  float r = __fsub_rn(x, __fmul_rn(k, 0.693145751953125f));
  r = __fsub_rn(r, __fmul_rn(k, 1.428606765330187045e-06f));
  const float C[8] = {1.0f, 1.0f, 0.5f, (float)(1.0 / 6.0), (float)(1.0 / 24.0), (float)(1.0 / 120.0),
                      (float)(1.0 / 720.0), (float)(1.0 / 5040.0)};
  float p = C[7];
#pragma unroll
  for (int i = 6; i >= 0; --i) p = __fadd_rn(__fmul_rn(p, r), C[i]);
  int ki = (int)k;
  ki = ki < -200 ? -200 : (ki > 200 ? 200 : ki);
  const int k1 = (ki >= 0) ? (ki / 2) : -((-ki + 1) / 2);  // floor division
  const int k2 = ki - k1;
  const int c1 = k1 < -126 ? -126 : (k1 > 127 ? 127 : k1);
  const int c2 = k2 < -126 ? -126 : (k2 > 127 ? 127 : k2);
  return __fmul_rn(__fmul_rn(p, pow2i(c1)), pow2i(c2));
}

// branch-free: the special cases are selected after the main path (computed on 0 for them), so a wave runs one
// straight-line sequence instead of three divergent branches per call
TOUED_DEV float pexp(float x) {
  const bool nan = x != x, hi = x > 88.72283905206835f, lo = x < -103.972084f;
  const float r = pexp_core((nan || hi || lo) ? 0.0f : x);
  return nan ? x : (hi ? __builtin_inff() : (lo ? 0.0f : r));
}

// pexp on a softmax argument x - max (x <= 0, -inf or NaN): the same value as pexp(x) for every such x, with the
// overflow test and the exponent clamps dropped -- for k = rint(x log2 e) in [-150, 0] (x >= -103.97) the +-200 and
// [-126, 127] clamps are the identity and floor(k / 2) is k >> 1; below -103.97 the result is selected to 0 whatever
// the core computed (k is floored at -200 first, so the conversion stays defined).  About 9 VALU fewer per call.
TOUED_DEV float pexp_le0(float x) {
  const float k = rintf(__fmul_rn(x, 1.44269504088896341f));
  float r = __fsub_rn(x, __fmul_rn(k, 0.693145751953125f));
  r = __fsub_rn(r, __fmul_rn(k, 1.428606765330187045e-06f));
  const float C[8] = {1.0f, 1.0f, 0.5f, (float)(1.0 / 6.0), (float)(1.0 / 24.0), (float)(1.0 / 120.0),
                      (float)(1.0 / 720.0), (float)(1.0 / 5040.0)};
  float p = C[7];
#pragma unroll
  for (int i = 6; i >= 0; --i) p = __fadd_rn(__fmul_rn(p, r), C[i]);
  const int ki = (int)fmaxf(k, -200.0f);
  const int k1 = ki >> 1, k2 = ki - k1;
  const float v = __fmul_rn(__fmul_rn(p, pow2i(k1)), pow2i(k2));
  return x != x ? x : (x < -103.972084f ? 0.0f : v);
}

TOUED_DEV float plog(float x) {
  if (x != x) return x;
  if (x == 0.0f) return -__builtin_inff();
  if (x < 0.0f) return __builtin_nanf("");
  if (__builtin_isinf(x)) return x;
  const bool sub = x < 1.17549435e-38f;
  const float xs = sub ? __fmul_rn(x, 8388608.0f) : x;
  const uint32_t bits = __float_as_uint(xs);
  int e = (int)((bits >> 23) & 0xFFu) - 127;
  if (sub) e -= 23;
  float m = __uint_as_float((bits & 0x7FFFFFu) | 0x3F800000u);
  if (m > 1.41421356237f) { m = __fmul_rn(m, 0.5f); e += 1; }
  const float f = __fsub_rn(m, 1.0f);
  const float s = __fdiv_rn(f, __fadd_rn(2.0f, f));
  const float z = __fmul_rn(s, s);
  const float w = __fmul_rn(z, z);
  const float t1 = __fmul_rn(w, __fadd_rn(0.40000972152f, __fmul_rn(w, 0.24279078841f)));
  const float t2 = __fmul_rn(z, __fadd_rn(0.66666662693f, __fmul_rn(w, 0.28498786688f)));
  const float R = __fadd_rn(t2, t1);
  const float hfsq = __fmul_rn(__fmul_rn(0.5f, f), f);
  const float dk = (float)e;
  const float inner = __fadd_rn(__fmul_rn(s, __fadd_rn(hfsq, R)), __fmul_rn(dk, 1.428606765330187045e-06f));
  return __fsub_rn(__fmul_rn(dk, 0.693145751953125f), __fsub_rn(__fsub_rn(hfsq, inner), f));
}

// erf_inv float32 (M. Giles' single-precision approximation, as XLA lowers lax.erf_inv)
TOUED_DEV float erfinv_giles(float x) {
  float w = -plog((1.0f - x) * (1.0f + x));
  float p;
  if (w < 5.0f) {
    w = w - 2.5f;
    p = 2.81022636e-08f;
    p = 3.43273939e-07f + p * w; p = -3.5233877e-06f + p * w; p = -4.39150654e-06f + p * w;
    p = 0.00021858087f + p * w; p = -0.00125372503f + p * w; p = -0.00417768164f + p * w;
    p = 0.246640727f + p * w; p = 1.50140941f + p * w;
  } else {
    w = sqrtf(w) - 3.0f;
    p = -0.000200214257f;
    p = 0.000100950558f + p * w; p = 0.00134934322f + p * w; p = -0.00367342844f + p * w;
    p = 0.00573950773f + p * w; p = -0.0076224613f + p * w; p = 0.00943887047f + p * w;
    p = 1.00167406f + p * w; p = 2.83297682f + p * w;
  }
  return p * x;
}

// ----------------------------------------------------------------------------
// Error reporting for the C ABI
struct toued_ctx {
  std::atomic<int> reserved_cus{0};   // CUs the weight-gradient reductions' split-K plans leave free (toued_set_reserved_cus)
  std::atomic<int> users{0};          // host threads that have this context current (toued_ctx_set_current)
};
// Device error word (capi.hip): a kernel whose bounded wait expires ORs one of these bits into it instead of hanging;
// the host reads it with toued_device_error_check, which turns a set bit into -3 + toued_last_error().
#define TOUED_DEVERR_A2C_DRAW_WAIT 1u   // k_a2c_chain<SELF>: a draw wave's flag wait for the key wave gave up
namespace toued {
void set_error(const char* fmt, ...);
toued_ctx* current_ctx();   // the calling thread's current context, else the process default (capi.hip)
unsigned* dev_err_word();   // the device error word (allocated by the first toued_device_error_check; nullptr before)
}
#define TOUED_CHECK_LAUNCH()                                                   \
  do {                                                                         \
    hipError_t _e = hipGetLastError();                                         \
    if (_e != hipSuccess) {                                                    \
      toued::set_error("%s: launch failed: %s", __func__, hipGetErrorString(_e)); \
      return -2;                                                               \
    }                                                                          \
  } while (0)
#define TOUED_REQUIRE(cond, ...)                                               \
  do {                                                                         \
    if (!(cond)) {                                                             \
      toued::set_error(__VA_ARGS__);                                           \
      return -1;                                                               \
    }                                                                          \
  } while (0)
