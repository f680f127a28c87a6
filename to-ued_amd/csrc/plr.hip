// Prioritised level replay buffer logic (environments/level_sampler.py:169-234, 331-408) — HIP for gfx950.
//
// The buffer (B <= 8192 levels) is small, so each operation is ONE workgroup of 1024 threads that
// keeps its sort keys in LDS: a bitonic sort of 64-bit (order-preserving float bits, index) keys is a
// stable argsort with jax's comparator (lax.sort canonicalises -0 -> +0 and NaN, ties by index).
//
//   k_plr_reset_ids  _reset_lowest_scoring (:338-341): argsort(where(active, inf, where(new, -inf, score)))[:N]
//   k_plr_sample     _replay_from_buffer (:363-385, rank or proportional), _sample_random_from_buffer
//                    (:396-407), and the replay/random selection (:212-227): bernoulli count, the
//                    n_replayable guard, permutation(use_replay), where(use, replay, random)
#include "common.h"

namespace {

constexpr int kThreads = 1024;
constexpr int kMaxSort = 8192;

// Order-preserving map of a float to uint32 after jax's canonicalisation.
TOUED_DEV uint32_t sort_key(float x) {
  if (x == 0.0f) x = 0.0f;
  uint32_t b = __float_as_uint(x);
  if (x != x) b = 0x7FC00000u;
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

// Ascending bitonic sort of s[0..P) (P a power of two), whole block participates.
TOUED_DEV void bitonic(uint64_t* s, int P) {
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < (P >> 1); i += blockDim.x) {
        const int lo = ((i & ~(j - 1)) << 1) | (i & (j - 1));
        const int hi = lo + j;
        const bool asc = (lo & k) == 0;
        const uint64_t a = s[lo], b = s[hi];
        if ((a > b) == asc) { s[lo] = b; s[hi] = a; }
      }
      __syncthreads();
    }
  }
}

TOUED_DEV int pow2_ceil(int n) {
  int p = 1;
  while (p < n) p <<= 1;
  return p;
}

TOUED_DEV void fill_keys(uint64_t* s, int B, int P, const float* key_of) {
  for (int i = threadIdx.x; i < P; i += blockDim.x)
    s[i] = (i < B) ? (((uint64_t)sort_key(key_of[i]) << 32) | (uint32_t)i) : ~0ull;
}

TOUED_DEV int block_count(bool v, int* red) {
  int c = __builtin_popcountll(__ballot(v));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  int s = 0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  return s;
}

// -gumbel(key, (B,))[i] - log(p)   (random.choice replace=False, p given: Gumbel top-k)
TOUED_DEV float gumbel_key(uint2 key, int B, int i, float p) {
  const float tiny = 1.17549435e-38f;
  const float u = uniform_from_bits(random_bits_at(key, (uint32_t)B, (uint32_t)i), tiny, 1.0f);
  const float g = -plog(-plog(u));
  return __fsub_rn(-g, plog(p));
}

}  // namespace

__global__ void __launch_bounds__(kThreads) k_plr_reset_ids(int B, int N, const float* __restrict__ score,
                                                            const uint8_t* __restrict__ active,
                                                            const uint8_t* __restrict__ fresh, int* __restrict__ ids) {
  __shared__ uint64_t s[kMaxSort];
  __shared__ float f[kMaxSort];
  const int P = pow2_ceil(B);
  for (int i = threadIdx.x; i < B; i += blockDim.x) {
    float x = fresh[i] ? -__builtin_inff() : score[i];
    f[i] = active[i] ? __builtin_inff() : x;
  }
  __syncthreads();
  fill_keys(s, B, P, f);
  bitonic(s, P);
  for (int i = threadIdx.x; i < N; i += blockDim.x) ids[i] = (int)(uint32_t)s[i];
}

// keys: [3][2] = replay_rng, random_rng, select_rng (the sampler's rng after split(rng, 3)).
// out: chosen[N], replay[N], random[N], use[N] (int32).
__global__ void __launch_bounds__(kThreads) k_plr_sample(int B, int N, const float* __restrict__ score,
                                                         const uint8_t* __restrict__ active,
                                                         const uint8_t* __restrict__ fresh,
                                                         const uint32_t* __restrict__ keys, int proportional,
                                                         float temperature, float p_replay, int* __restrict__ chosen,
                                                         int* __restrict__ rep, int* __restrict__ rnd,
                                                         int* __restrict__ use_out) {
  __shared__ uint64_t s[kMaxSort];
  __shared__ float f[kMaxSort];
  __shared__ int red[16];
  __shared__ float total;
  const int P = pow2_ceil(B);
  const int tid = threadIdx.x;
  // ---- replay (level_sampler.py:363-385)
  for (int i = tid; i < B; i += blockDim.x) {
    const bool inv = fresh[i] || active[i];
    f[i] = inv ? 0.0f : pexp(__fdiv_rn(score[i], temperature));
  }
  int n_invalid = 0;
  for (int base = 0; base < B; base += blockDim.x) {
    const int i = base + tid;
    n_invalid += block_count(i < B && (fresh[i] || active[i]), red);
  }
  __syncthreads();
  if (tid == 0) {
    float acc = 0.0f;
    for (int i = 0; i < B; ++i) acc = __fadd_rn(acc, f[i]);
    total = acc;
  }
  __syncthreads();
  const bool uniform_p = (B - n_invalid) < N;
  for (int i = tid; i < B; i += blockDim.x) f[i] = uniform_p ? 1.0f : __fdiv_rn(f[i], total);
  __syncthreads();
  const uint2 k_rep = make_uint2(keys[0], keys[1]);
  if (proportional) {
    uint2 k0, k1;
    split2(k_rep, k0, k1);
    for (int i = tid; i < B; i += blockDim.x) f[i] = gumbel_key(k1, B, i, f[i]);
    __syncthreads();
    fill_keys(s, B, P, f);
    bitonic(s, P);
    for (int i = tid; i < N; i += blockDim.x) rep[i] = (int)(uint32_t)s[i];
  } else {
    fill_keys(s, B, P, f);
    bitonic(s, P);
    for (int i = tid; i < N; i += blockDim.x) rep[i] = (int)(uint32_t)s[B - 1 - i];  // flip(argsort(p))[:N]
  }
  __syncthreads();
  // ---- random new levels (level_sampler.py:396-407)
  int n_new = 0;
  for (int base = 0; base < B; base += blockDim.x) {
    const int i = base + tid;
    n_new += block_count(i < B && fresh[i] && !active[i], red);
  }
  const uint2 k_rnd = make_uint2(keys[2], keys[3]);
  for (int i = tid; i < B; i += blockDim.x) {
    const float p = __fdiv_rn((fresh[i] && !active[i]) ? 1.0f : 0.0f, (float)n_new);
    f[i] = gumbel_key(k_rnd, B, i, p);
  }
  __syncthreads();
  fill_keys(s, B, P, f);
  bitonic(s, P);
  for (int i = tid; i < N; i += blockDim.x) rnd[i] = (int)(uint32_t)s[i];
  __syncthreads();
  // ---- selection (level_sampler.py:212-227)
  const uint2 k_sel = make_uint2(keys[4], keys[5]);
  uint2 rng1, k_bern, rng2, k_perm;
  split2(k_sel, rng1, k_bern);
  split2(rng1, rng2, k_perm);
  int n_rep = 0;
  for (int base = 0; base < N; base += blockDim.x) {
    const int i = base + tid;
    bool b = false;
    if (i < N) b = uniform_from_bits(random_bits_at(k_bern, (uint32_t)N, (uint32_t)i), 0.0f, 1.0f) < p_replay;
    n_rep += block_count(b, red);
  }
  const bool replayable = (B - n_invalid) >= N;
  // permutation(k_perm, use) = jax _shuffle: per round (key, sub) = split(key), stable sort by
  // random_bits(sub, (N,)); ceil(3 ln N / ln(2^32-1)) rounds (1 for N <= ~1.6k).
  int* cur = reinterpret_cast<int*>(f);
  for (int i = tid; i < N; i += blockDim.x) cur[i] = i;
  const int rounds = N > 1 ? (int)ceil(3.0 * log((double)N) / log(4294967295.0)) : 0;
  const int PN = pow2_ceil(N);
  uint2 kk = k_perm;
  for (int r = 0; r < rounds; ++r) {
    uint2 knext, ksub;
    split2(kk, knext, ksub);
    kk = knext;
    for (int i = tid; i < PN; i += blockDim.x)
      s[i] = (i < N) ? (((uint64_t)random_bits_at(ksub, (uint32_t)N, (uint32_t)i) << 32) | (uint32_t)i) : ~0ull;
    bitonic(s, PN);
    for (int i = tid; i < N; i += blockDim.x) s[i] = (uint64_t)(uint32_t)cur[(uint32_t)s[i]];
    __syncthreads();
    for (int i = tid; i < N; i += blockDim.x) cur[i] = (int)(uint32_t)s[i];
    __syncthreads();
  }
  for (int i = tid; i < N; i += blockDim.x) {
    const bool u = (cur[i] < n_rep) && replayable;
    use_out[i] = u ? 1 : 0;
    chosen[i] = u ? rep[i] : rnd[i];
  }
  (void)rng2;
}

extern "C" {

int toued_plr_reset_ids(int B, int N, const float* score, const uint8_t* active, const uint8_t* fresh, int* ids,
                        hipStream_t stream) {
  TOUED_REQUIRE(B > 0 && B <= kMaxSort && N >= 0 && N <= B, "toued_plr_reset_ids: need 0 <= N <= B <= %d",
                kMaxSort);
  if (N == 0) return 0;
  hipLaunchKernelGGL(k_plr_reset_ids, dim3(1), dim3(kThreads), 0, stream, B, N, score, active, fresh, ids);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_plr_sample(int B, int N, const float* score, const uint8_t* active, const uint8_t* fresh,
                     const uint32_t* keys, int proportional, float temperature, float p_replay, int* chosen,
                     int* rep, int* rnd, int* use_out, hipStream_t stream) {
  TOUED_REQUIRE(B > 0 && B <= kMaxSort && N >= 0 && N <= B, "toued_plr_sample: need 0 <= N <= B <= %d", kMaxSort);
  TOUED_REQUIRE(temperature > 0.0f, "toued_plr_sample: temperature must be > 0");
  if (N == 0) return 0;
  hipLaunchKernelGGL(k_plr_sample, dim3(1), dim3(kThreads), 0, stream, B, N, score, active, fresh, keys,
                     proportional, temperature, p_replay, chosen, rep, rnd, use_out);
  TOUED_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
