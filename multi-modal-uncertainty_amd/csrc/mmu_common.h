// Shared device helpers for the MMBT hot-path kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));

#define MMU_LDS(T) __attribute__((address_space(3))) T

static __device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
static __device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

// ---------------------------------------------------------------- counter-based RNG
// SplitMix64 finaliser of (seed + ctr * golden): stateless, so forward and backward
// regenerate the same dropout mask from (seed, element counter).
static __device__ __forceinline__ uint32_t mmu_lowbias32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
// 32-bit stream key of a 64-bit dropout seed (wave-uniform: folded into scalar code)
static __device__ __forceinline__ uint32_t mmu_seed32(uint64_t seed) {
  return mmu_lowbias32((uint32_t)seed ^ mmu_lowbias32((uint32_t)(seed >> 32) ^ 0x68bc21ebu));
}
// keep-mask for 4 consecutive elements [4*q, 4*q+4) of a stream: 16 random bits each,
// from two 32-bit hashes of (2q, 2q+1) ^ key (4 integer multiplies per quad).
// An element is dropped when its 16-bit draw is < thr16 (= round(p * 65536)).
static __device__ __forceinline__ uint32_t mmu_keep4(uint64_t seed, uint64_t quad, uint32_t thr16) {
  const uint32_t x = (((uint32_t)quad << 1) ^ ((uint32_t)(quad >> 31) * 0x9E3779B8u)) ^ mmu_seed32(seed);
  const uint32_t h0 = mmu_lowbias32(x), h1 = mmu_lowbias32(x ^ 1u);
  return ((h0 & 0xFFFFu) >= thr16 ? 1u : 0u) | ((h0 >> 16) >= thr16 ? 2u : 0u) |
         ((h1 & 0xFFFFu) >= thr16 ? 4u : 0u) | ((h1 >> 16) >= thr16 ? 8u : 0u);
}
// Graph replays (mmu_set_seed_offset): a captured launch keeps the seed it was captured with,
// so every dropout kernel folds in a device counter the replayed graph advances; off == NULL
// (eager launches) and *off == 0 both leave the seed as given.
static __device__ __forceinline__ uint64_t mmu_eff_seed(uint64_t seed, const uint64_t* off) {
  return off ? seed ^ (*off * 0x9E3779B97F4A7C15ull) : seed;
}
static __device__ __forceinline__ bool mmu_keep1(uint64_t seed, uint64_t idx, uint32_t thr16) {
  const uint64_t quad = idx >> 2;
  const uint32_t x = (((uint32_t)quad << 1) ^ ((uint32_t)(quad >> 31) * 0x9E3779B8u)) ^ mmu_seed32(seed);
  const uint32_t h = mmu_lowbias32(x ^ (uint32_t)((idx >> 1) & 1));
  return ((h >> (16 * (idx & 1))) & 0xFFFFu) >= thr16;
}

// ---------------------------------------------------------------- math
// GELU (erf form, as pytorch_pretrained_bert's gelu) and its derivative from ONE
// branch-free evaluation: erf(x) = 1 - t*P(t)*exp(-x^2), t = 1/(1 + 0.3275911 x), x >= 0
// (Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7), so Phi(z) and phi(z) share the exp.
// The 1/sqrt(2) of x and the 1/2 of Phi = (1 + erf) / 2 are folded into the constants (two
// multiplies per element fewer in the FFN1 epilogue, which is VALU-bound).
static __device__ __forceinline__ void gelu_pair(float z, float& g, float& dg) {
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f * 0.70710678118654752f, fabsf(z), 1.0f));
  float P = fmaf(0.5f * 1.061405429f, t, 0.5f * -1.453152027f);
  P = fmaf(P, t, 0.5f * 1.421413741f);
  P = fmaf(P, t, 0.5f * -0.284496736f);
  P = fmaf(P, t, 0.5f * 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(z * z * -0.72134752044448170f);  // exp(-z^2/2) = exp(-x^2)
  const float h = (t * P) * e;                                             // = 1 - Phi(|z|)
  const float phi = z >= 0.f ? 1.0f - h : h;                               // Phi(z)
  g = z * phi;
  dg = fmaf(z * 0.39894228040143268f, e, phi);                             // Phi(z) + z phi(z)
}
static __device__ __forceinline__ float gelu_erf(float z) {
  float g, dg;
  gelu_pair(z, g, dg);
  return g;
}

static __device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
static __device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// bijective XCD-aware block remap: blocks that share an XCD (orig % 8) get a
// contiguous range of logical ids, so neighbouring tiles share that XCD's L2.
static __device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  int q = nwg >> 3, r = nwg & 7, xcd = orig & 7, idx = orig >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}
