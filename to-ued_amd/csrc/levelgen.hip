// Device level generator — restates environments/environments.py:22-37 and
// environments/gridworld/configs.py:12-126 (+ the mode tables at :148-707,
// encoded host-side into a ModeProgram by toued/modes.py).
//
// One lane per level: the work is integer-RNG heavy and branchy (per-level
// sampler dispatch, a stable sort for the wall permutation, a Gumbel top-k for
// start/object cells), and N is small (N agents or the 4000-level PLR buffer),
// so a thread per level with the program in a uniform constant buffer is the
// right shape.  Output: packed level records (int32[64], common.h layout).
#include "common.h"

namespace {

enum { SK_CONST = 0, SK_LOG_UNIFORM_INT = 1, SK_LOG_UNIFORM = 2, SK_UNIFORM = 3, SK_UNIFORM_FIRST_POS = 4,
       SK_CHOICE_ARANGE = 5, SK_WALL_IDXS = 6 };

struct ParamSpec {
  int kind, n;      // sampler kind, element count (vector samplers) / n_walls
  float flo, fhi;   // float bounds (lo, hi) — log samplers take log() of these on device
  int ilo, ihi;     // integer bounds (choice_arange) / max_grid (wall_idxs)
  int ival;         // scalar constant
  int data_off;     // offset of constant list data in ModeSpec::fdata / idata
};

struct ModeSpec {
  int n_ids, max_n, n_types, max_grid, tabular, n_walls_const, pad0, pad1;
  int obj_ids[8];
  ParamSpec rew, pterm, presp, max_steps, n_objs, grid, walls;
  float fdata[24];   // constant type tables: rew @0, pterm @8, presp @16
  int idata[176];    // constant wall list
};

struct ModeProgram {
  int manual, n_sub, dst_max_n, dst_n_types, dst_max_grid, pad0, pad1, pad2;
  ParamSpec lifetime;
  ModeSpec sub[10];
};

TOUED_DEV uint32_t mulmod_span(uint32_t span) {
  uint32_t m = 65536u % span;
  return (m * m) % span;
}

// jax.random.randint(key, (), 0, span)
TOUED_DEV int randint0(uint2 key, uint32_t span) {
  uint2 k1, k2;
  split2(key, k1, k2);
  const uint32_t hb = bits1(k1), lb = bits1(k2);
  if (span == 0u) span = 1u;
  const uint32_t off = ((hb % span) * mulmod_span(span) + (lb % span)) % span;
  return (int)off;
}

TOUED_DEV int log_uniform_int(uint2 key, float lo, float hi) {
  const float u = uniform_from_bits(bits1(key), plog(lo), plog(hi));
  return (int)rintf(pexp(u));
}

// Vector samplers writing n floats into out (configs.py:98-121, random.uniform)
TOUED_DEV void sample_vec(const ParamSpec& ps, const float* cdata, uint2 key, float* out) {
  switch (ps.kind) {
    case SK_CONST:
      for (int j = 0; j < ps.n; ++j) out[j] = cdata[ps.data_off + j];
      break;
    case SK_LOG_UNIFORM: {
      const float lo = plog(ps.flo), hi = plog(ps.fhi);
      for (int j = 0; j < ps.n; ++j)
        out[j] = pexp(uniform_from_bits(random_bits_at(key, (uint32_t)ps.n, (uint32_t)j), lo, hi));
    } break;
    case SK_UNIFORM:
      for (int j = 0; j < ps.n; ++j)
        out[j] = uniform_from_bits(random_bits_at(key, (uint32_t)ps.n, (uint32_t)j), ps.flo, ps.fhi);
      break;
    case SK_UNIFORM_FIRST_POS: {
      uint2 k1, k2;
      split2(key, k1, k2);
      out[0] = uniform_from_bits(bits1(k1), 0.0f, ps.fhi);
      for (int j = 0; j < ps.n - 1; ++j)
        out[j + 1] = uniform_from_bits(random_bits_at(k2, (uint32_t)(ps.n - 1), (uint32_t)j), ps.flo, ps.fhi);
    } break;
    default:
      for (int j = 0; j < ps.n; ++j) out[j] = 0.0f;
  }
}

// Scalar int params (configs.py:83-88: callables get an extra split)
TOUED_DEV int sample_scalar(const ParamSpec& ps, uint2 key) {
  if (ps.kind == SK_CONST) return ps.ival;
  uint2 a, b;
  split2(key, a, b);
  if (ps.kind == SK_LOG_UNIFORM_INT) return log_uniform_int(b, ps.flo, ps.fhi);
  if (ps.kind == SK_CHOICE_ARANGE) return ps.ilo + randint0(b, (uint32_t)(ps.ihi - ps.ilo));
  return 0;
}

// Generate one concrete-mode level (configs.py:12-53) and pack it for the destination kwargs.
TOUED_DEV void gen_level(const ModeSpec& m, const ModeProgram& prog, uint2 rng, int lifetime, int buffer_id,
                         int* out) {
  float rew[8] = {0}, pterm[8] = {0}, presp[8] = {0};
  uint2 sub;
  split2(rng, rng, sub);
  sample_vec(m.rew, m.fdata, sub, rew);
  split2(rng, rng, sub);
  sample_vec(m.pterm, m.fdata, sub, pterm);
  split2(rng, rng, sub);
  sample_vec(m.presp, m.fdata, sub, presp);
  split2(rng, rng, sub);
  const int max_steps = sample_scalar(m.max_steps, sub);
  split2(rng, rng, sub);
  const int n_objs = sample_scalar(m.n_objs, sub);
  split2(rng, rng, sub);
  const int grid = sample_scalar(m.grid, sub);
  // walls
  split2(rng, rng, sub);
  uint32_t wall_bits[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int mg2 = m.max_grid * m.max_grid;
  if (m.walls.kind == SK_CONST) {
    for (int j = 0; j < m.walls.n; ++j) {
      const int c = m.idata[m.walls.data_off + j];
      wall_bits[c >> 5] |= 1u << (c & 31);
    }
  } else {
    // _sample_param extra split, then uniform_wall_idxs = permutation(key, mg2)[:n_walls]
    // (1 shuffle round for mg2 <= 1600: key, subkey = split(key); stable sort by random bits).
    uint2 a, b;
    split2(sub, a, b);
    uint2 k0, sk;
    split2(b, k0, sk);
    const int nw = m.walls.n;
    uint32_t bv[16];
    int bi[16];
    for (int j = 0; j < 16; ++j) { bv[j] = 0xffffffffu; bi[j] = 0x7fffffff; }
    for (int c = 0; c < mg2; ++c) {
      const uint32_t v = random_bits_at(sk, (uint32_t)mg2, (uint32_t)c);
      if (v < bv[nw - 1] || (v == bv[nw - 1] && c < bi[nw - 1])) {
        uint32_t cv = v;
        int ci = c;
        for (int j = 0; j < nw; ++j) {
          const bool before = (cv < bv[j]) || (cv == bv[j] && ci < bi[j]);
          if (before) { const uint32_t tv = bv[j]; const int ti = bi[j]; bv[j] = cv; bi[j] = ci; cv = tv; ci = ti; }
        }
      }
    }
    for (int j = 0; j < nw; ++j) wall_bits[bi[j] >> 5] |= 1u << (bi[j] & 31);
  }
  // start + object cells: choice(all_pos, (max_n+1,), replace=False, p=valid) with p unnormalised
  split2(rng, rng, sub);
  const int K = m.max_n + 1;
  float gv[9];
  int gi[9];
  for (int j = 0; j < 9; ++j) { gv[j] = __builtin_inff(); gi[j] = 0x7fffffff; }
  const float tiny = 1.17549435e-38f;
  const int g2grid = grid * grid;
  for (int c = 0; c < mg2; ++c) {
    const bool valid = (c < g2grid) && !((wall_bits[c >> 5] >> (c & 31)) & 1u);
    const float u = uniform_from_bits(random_bits_at(sub, (uint32_t)mg2, (uint32_t)c), tiny, 1.0f);
    const float negg = plog(-plog(u));            // -gumbel
    const float g = valid ? __fsub_rn(negg, 0.0f) : __builtin_inff();   // - log(1) / - log(0)
    if (g < gv[K - 1] || (g == gv[K - 1] && c < gi[K - 1])) {
      float cv = g;
      int ci = c;
      for (int j = 0; j < K; ++j) {
        const bool before = (cv < gv[j]) || (cv == gv[j] && ci < gi[j]);
        if (before) { const float tv = gv[j]; const int ti = gi[j]; gv[j] = cv; gi[j] = ci; cv = tv; ci = ti; }
      }
    }
  }
  // pack (oracle/levels.py pack_levels) into the destination kwargs
  for (int w = 0; w < LEVEL_WORDS; ++w) out[w] = 0;
  out[L_MAX_STEPS] = max_steps;
  out[L_GRID] = grid;
  out[L_START] = gi[0];
  out[L_NOBJS] = n_objs;
  out[L_RANDRESP] = m.tabular ? 0 : 1;
  out[L_LIFETIME] = lifetime;
  out[L_BUFID] = buffer_id;
  for (int i = 0; i < prog.dst_max_n; ++i) {
    const int id = (i < m.max_n) ? (i < m.n_ids ? m.obj_ids[i] : -1) : -1;
    out[L_OBJ_IDS + i] = id;
    out[L_STATIC + i] = (i < m.max_n) ? gi[1 + i] : 0;
    const int rid = id < 0 ? id + prog.dst_n_types : id;
    const bool in_src = rid < m.n_types;   // zero-padded type tables beyond the source mode's types
    out[L_REW + i] = __float_as_int(in_src ? rew[rid] : 0.0f);
    out[L_PTERM + i] = __float_as_int(in_src ? pterm[rid] : 0.0f);
    out[L_PRESP + i] = __float_as_int(in_src ? presp[rid] : 0.0f);
  }
  for (int w = 0; w < 8; ++w) out[L_WALLS + w] = (int)wall_bits[w];
  for (int j = 0; j < prog.dst_n_types && j < TOUED_MAX_TYPES; ++j) {
    const bool in_src = j < m.n_types;
    out[L_TREW + j] = __float_as_int(in_src ? rew[j] : 0.0f);
    out[L_TPTERM + j] = __float_as_int(in_src ? pterm[j] : 0.0f);
    out[L_TPRESP + j] = __float_as_int(in_src ? presp[j] : 0.0f);
  }
  out[L_AUTOC] = 1;   // every ENV_MODE_PARAMS entry sets auto_collect=True (configs.py:29)
}

__global__ void __launch_bounds__(64) k_level_gen(const ModeProgram* __restrict__ prog_g,
                                                  const uint32_t* __restrict__ keys,
                                                  const int* __restrict__ buffer_ids, int* __restrict__ out,
                                                  int* __restrict__ sub_mode, int n,
                                                  const uint8_t* __restrict__ mask) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || (mask && !mask[i])) return;
  const ModeProgram& prog = *prog_g;
  const uint2 key = make_uint2(keys[2 * i], keys[2 * i + 1]);
  uint2 p_rng, l_rng;
  split2(key, p_rng, l_rng);
  int s = 0;
  uint2 rng = p_rng;
  if (prog.manual) {
    uint2 sub_rng;
    split2(p_rng, sub_rng, rng);
    s = randint0(sub_rng, (uint32_t)prog.n_sub);
  }
  // lifetime (configs.py:606-637) from l_rng
  int lifetime;
  if (prog.lifetime.kind == SK_CONST) lifetime = prog.lifetime.ival;
  else lifetime = log_uniform_int(l_rng, prog.lifetime.flo, prog.lifetime.fhi);
  gen_level(prog.sub[s], prog, rng, lifetime, buffer_ids ? buffer_ids[i] : 0, out + (size_t)i * LEVEL_WORDS);
  if (sub_mode) sub_mode[i] = s;
}

}  // namespace

extern "C" {

size_t toued_mode_program_bytes(void) { return sizeof(ModeProgram); }

int toued_level_gen(const void* program, const uint32_t* keys, const int* buffer_ids, int* levels_out,
                    int* sub_mode_out, int n, hipStream_t stream) {
  TOUED_REQUIRE(n >= 0, "toued_level_gen: n=%d", n);
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_level_gen, dim3((n + 63) / 64), dim3(64), 0, stream,
                     reinterpret_cast<const ModeProgram*>(program), keys, buffer_ids, levels_out, sub_mode_out, n,
                     nullptr);
  TOUED_CHECK_LAUNCH();
  return 0;
}

// the same, writing only the levels i with mask[i] != 0 (in place: the level sampler's where(terminated, new, old))
int toued_level_gen_masked(const void* program, const uint32_t* keys, const int* buffer_ids, int* levels_out, int n,
                           const uint8_t* mask, hipStream_t stream) {
  TOUED_REQUIRE(n >= 0 && mask, "toued_level_gen_masked: n=%d mask=%p", n, (const void*)mask);
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_level_gen, dim3((n + 63) / 64), dim3(64), 0, stream,
                     reinterpret_cast<const ModeProgram*>(program), keys, buffer_ids, levels_out, nullptr, n, mask);
  TOUED_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
