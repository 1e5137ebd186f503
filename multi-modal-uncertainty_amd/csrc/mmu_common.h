// Shared device helpers for the MMBT hot-path kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));

#define MMU_LDS(T) __attribute__((address_space(3))) T

static __device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
static __device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

// ---------------------------------------------------------------- counter-based RNG
// SplitMix64 finaliser of (seed + ctr * golden): stateless, so forward and backward
// regenerate the same dropout mask from (seed, element counter).
static __device__ __forceinline__ uint64_t mmu_mix64(uint64_t seed, uint64_t ctr) {
  uint64_t z = seed + ctr * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// keep-mask for 4 consecutive elements [4*q, 4*q+4) of a stream: 16 random bits each.
// An element is dropped when its 16-bit draw is < thr16 (= round(p * 65536)).
static __device__ __forceinline__ uint32_t mmu_keep4(uint64_t seed, uint64_t quad, uint32_t thr16) {
  uint64_t z = mmu_mix64(seed, quad);
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) m |= (((uint32_t)(z >> (16 * i)) & 0xFFFFu) >= thr16 ? 1u : 0u) << i;
  return m;
}
static __device__ __forceinline__ bool mmu_keep1(uint64_t seed, uint64_t idx, uint32_t thr16) {
  uint64_t z = mmu_mix64(seed, idx >> 2);
  return ((uint32_t)(z >> (16 * (idx & 3))) & 0xFFFFu) >= thr16;
}

// ---------------------------------------------------------------- math
static __device__ __forceinline__ float gelu_erf(float z) {
  return 0.5f * z * (1.0f + erff(z * 0.70710678118654752f));
}
static __device__ __forceinline__ float gelu_erf_grad(float z) {
  return 0.5f * (1.0f + erff(z * 0.70710678118654752f)) + z * 0.39894228040143268f * __expf(-0.5f * z * z);
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
