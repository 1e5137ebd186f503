// FLAVA fusion-transformer kernel (gfx950): attention over the SEQUENCE = batch axis.
//
// src/model.py:193,205-207 hands nn.MultiheadAttention (batch_first=False) an [B, L, E]
// tensor, so the softmax runs over the B samples for every token position l and head h:
// sequence length S = B, "batch" = (l, h) pairs.  With token-major rows r = s*N + n
// (s = sample, n = token position, N = tokens per sample) the s-th sequence element of
// (n, h) is row s*N + n, columns h*D (q), E + h*D (k), 2E + h*D (v) of the fused in_proj
// output QKV [S*N, ld].  D = E / heads (256 for FLAVA's 3 heads).
//
// Flash-style, one workgroup per (64 sequence elements, n, h), 4 waves of 16 queries (or
// keys), v_mfma_f32_16x16x32_bf16 throughout:
//   fwd : S^T = K Q^T ;  O^T += V^T P^T         (keys on accumulator rows, queries on lanes)
//   dQ  : S^T, dP^T = V dO^T ; dQ^T += K^T dS^T
//   dKdV: S = Q K^T, dP = dO V^T (keys on lanes) ; dV^T += dO^T P ; dK^T += Q^T dS
// The softmax / dS values feed the second product straight from the accumulators: a
// 16x16 accumulator holds 4 consecutive rows per lane group g = lane>>4, so two adjacent
// subtiles give lane group g the 8 contraction indices {32c + 4g + j, 32c + 16 + 4g + j},
// j < 4 -- the transposed operand is read from a transposed LDS image in that same order.
// Scores are kept in log2 units (c = scale * log2 e); LSE2 = m + log2(sum) per query.
// No mask and no attention dropout: nn.MultiheadAttention's dropout defaults to 0 and the
// block passes attn_mask=None (src/model.py:193,214).
#include "mmu_common.h"
#include "mmu_internal.h"

namespace mmu {

constexpr float SA_LOG2E = 1.4426950408889634f;
constexpr int SA_T = 64;  // sequence elements per tile

template <int D>
struct SeqGeo {
  static constexpr int ROW = D * 2;          // bytes per row-major row
  static constexpr int CH = D / 8;           // 16-B chunks per row
  static constexpr int SWZ = CH < 16 ? CH - 1 : 15;
  static constexpr int TROW = SA_T * 2 + 16;  // bytes per transposed row (64 elements + pad)
  static constexpr int TILE = SA_T * ROW;     // row-major tile bytes
  static constexpr int TTILE = D * TROW;      // transposed tile bytes
};

// row-major tile, chunk c of row r at c ^ (r & SWZ): conflict-free 16-lane fragment reads
template <int D>
static __device__ __forceinline__ int rm_off(int r, int c) {
  return r * SeqGeo<D>::ROW + ((c ^ (r & SeqGeo<D>::SWZ)) << 4);
}

// stage rows [r0, r0+64) of column block `col` (D wide) of a strided row set into a
// row-major swizzled tile (coalesced: consecutive threads take consecutive chunks)
template <int D>
static __device__ __forceinline__ void stage_rm(char* dst, const bf16* base, int64_t rs, int col, int r0, int S) {
  constexpr int CH = SeqGeo<D>::CH;
  for (int i = threadIdx.x; i < SA_T * CH; i += 256) {
    const int r = i / CH, c = i - r * CH;
    bf16x8 v = bf16x8{};
    if (r0 + r < S) v = *(const bf16x8*)(base + (int64_t)(r0 + r) * rs + col + 8 * c);
    *(bf16x8*)(dst + rm_off<D>(r, c)) = v;
  }
}
// stage the same rows transposed: dst[d][r] (consecutive threads take consecutive rows, so
// each 2-B LDS write of a wave covers one transposed row contiguously)
template <int D>
static __device__ __forceinline__ void stage_tr(char* dst, const bf16* base, int64_t rs, int col, int r0, int S) {
  constexpr int CH = SeqGeo<D>::CH, TROW = SeqGeo<D>::TROW;
  for (int i = threadIdx.x; i < SA_T * CH; i += 256) {
    const int r = i & (SA_T - 1), c = i >> 6;
    bf16x8 v = bf16x8{};
    if (r0 + r < S) v = *(const bf16x8*)(base + (int64_t)(r0 + r) * rs + col + 8 * c);
#pragma unroll
    for (int e = 0; e < 8; ++e) *(bf16*)(dst + (8 * c + e) * TROW + 2 * r) = v[e];
  }
}
// fragment of a row-major tile: lane holds tile[row0 + (l&15)][32ks + 8(l>>4) + j]
template <int D>
static __device__ __forceinline__ bf16x8 rm_frag(const char* s, int row0, int ks, int l) {
  return *(const bf16x8*)(s + rm_off<D>(row0 + (l & 15), 4 * ks + (l >> 4)));
}
// transposed-image fragment in the accumulator order: lane holds T[d0 + (l&15)][idx(c, g, j)],
// idx = 32c + 4g + j (j < 4), 32c + 16 + 4g + (j - 4) (j >= 4)
template <int D>
static __device__ __forceinline__ bf16x8 tr_frag(const char* s, int d0, int c, int l) {
  const char* row = s + (d0 + (l & 15)) * SeqGeo<D>::TROW + 2 * (32 * c + 4 * (l >> 4));
  const bf16x4 lo = *(const bf16x4*)row, hi = *(const bf16x4*)(row + 32);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
// accumulator subtiles (2c, 2c+1) -> bf16 operand in the same contraction order
static __device__ __forceinline__ bf16x8 acc_pair(const f32x4& a, const f32x4& b) {
  return bf16x8{f2bf(a[0]), f2bf(a[1]), f2bf(a[2]), f2bf(a[3]), f2bf(b[0]), f2bf(b[1]), f2bf(b[2]), f2bf(b[3])};
}
static __device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------------------------ forward
template <int D>
__global__ __launch_bounds__(256) void seqattn_fwd_kernel(SeqAttnParams p) {
  using G = SeqGeo<D>;
  __shared__ __attribute__((aligned(16))) char smem[G::TILE + G::TTILE];
  char* Ks = smem;
  char* Vt = smem + G::TILE;
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6, g = l >> 4;
  const int nh = blockIdx.y, n = nh / p.heads, h = nh - n * p.heads;
  const int S = p.S;
  const int64_t rs = (int64_t)p.N * p.ld_qkv;
  const bf16* base = p.qkv + (int64_t)n * p.ld_qkv;
  const int q = blockIdx.x * SA_T + 16 * w + (l & 15);
  const float c = p.scale * SA_LOG2E;
  bf16x8 qf[D / 32];
#pragma unroll
  for (int ks = 0; ks < D / 32; ++ks)
    qf[ks] = q < S ? *(const bf16x8*)(base + (int64_t)q * rs + h * D + 32 * ks + 8 * g) : bf16x8{};
  f32x4 o[D / 16];
#pragma unroll
  for (int i = 0; i < D / 16; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -__builtin_huge_valf(), lsum = 0.f;
  for (int k0 = 0; k0 < S; k0 += SA_T) {
    __syncthreads();
    stage_rm<D>(Ks, base, rs, p.E + h * D, k0, S);
    stage_tr<D>(Vt, base, rs, 2 * p.E + h * D, k0, S);
    __syncthreads();
    f32x4 s[4];
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      s[st] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < D / 32; ++ks) s[st] = mfma16(rm_frag<D>(Ks, 16 * st, ks, l), qf[ks], s[st]);
    }
    float mx = -__builtin_huge_valf();
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool ok = k0 + 16 * st + 4 * g + i < S;
        s[st][i] = ok ? s[st][i] * c : -__builtin_huge_valf();
        mx = fmaxf(mx, s[st][i]);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mnew = fmaxf(m, mx);
    const float alpha = __builtin_amdgcn_exp2f(m - mnew);
    m = mnew;
    lsum *= alpha;
#pragma unroll
    for (int i = 0; i < D / 16; ++i) o[i] *= alpha;
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s[st][i] = __builtin_amdgcn_exp2f(s[st][i] - m);
        lsum += s[st][i];
      }
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2) {
      const bf16x8 pf = acc_pair(s[2 * c2], s[2 * c2 + 1]);
#pragma unroll
      for (int ds = 0; ds < D / 16; ++ds) o[ds] = mfma16(tr_frag<D>(Vt, 16 * ds, c2, l), pf, o[ds]);
    }
  }
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  if (q < S) {
    const float inv = 1.0f / lsum;
    bf16* orow = p.out + ((int64_t)q * p.N + n) * p.ld_out + h * D + 4 * g;
#pragma unroll
    for (int ds = 0; ds < D / 16; ++ds)
      *(bf16x4*)(orow + 16 * ds) = bf16x4{f2bf(o[ds][0] * inv), f2bf(o[ds][1] * inv), f2bf(o[ds][2] * inv),
                                          f2bf(o[ds][3] * inv)};
    if (g == 0) p.lse2[(int64_t)nh * S + q] = m + __log2f(lsum);
  }
}

// ------------------------------------------------------------------------------ backward
// delta[nh][s] = sum_d dO[s,n,hD+d] O[s,n,hD+d]: one wave per (row, head)
template <int D>
__global__ __launch_bounds__(256) void seqattn_delta_kernel(SeqAttnParams p) {
  const int l = threadIdx.x & 63;
  const int64_t item = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // (row r = s*N + n) * heads + h
  const int64_t rows = (int64_t)p.S * p.N;
  if (item >= rows * p.heads) return;
  const int64_t r = item / p.heads;
  const int h = (int)(item - r * p.heads);
  float acc = 0.f;
  for (int d = l; d < D; d += 64)
    acc += bf2f(p.dout[r * p.ld_do + h * D + d]) * bf2f(p.o[r * p.ld_o + h * D + d]);
  acc = wave_sum(acc);
  if (l == 0) {
    const int64_t s = r / p.N, n = r - s * p.N;
    p.delta[(n * p.heads + h) * p.S + s] = acc;
  }
}

template <int D>
__global__ __launch_bounds__(256) void seqattn_dq_kernel(SeqAttnParams p) {
  using G = SeqGeo<D>;
  __shared__ __attribute__((aligned(16))) char smem[2 * G::TILE + G::TTILE];
  char* Ks = smem;
  char* Vs = smem + G::TILE;
  char* Kt = smem + 2 * G::TILE;
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6, g = l >> 4;
  const int nh = blockIdx.y, n = nh / p.heads, h = nh - n * p.heads;
  const int S = p.S;
  const int64_t rs = (int64_t)p.N * p.ld_qkv, rso = (int64_t)p.N * p.ld_do;
  const bf16* base = p.qkv + (int64_t)n * p.ld_qkv;
  const bf16* dob = p.dout + (int64_t)n * p.ld_do;
  const int q = blockIdx.x * SA_T + 16 * w + (l & 15);
  const float c = p.scale * SA_LOG2E;
  const bool qv = q < S;
  bf16x8 qf[D / 32], df[D / 32];
#pragma unroll
  for (int ks = 0; ks < D / 32; ++ks) {
    qf[ks] = qv ? *(const bf16x8*)(base + (int64_t)q * rs + h * D + 32 * ks + 8 * g) : bf16x8{};
    df[ks] = qv ? *(const bf16x8*)(dob + (int64_t)q * rso + h * D + 32 * ks + 8 * g) : bf16x8{};
  }
  const float lse = qv ? p.lse2[(int64_t)nh * S + q] : 0.f;
  const float dl = qv ? p.delta[(int64_t)nh * S + q] : 0.f;
  f32x4 dq[D / 16];
#pragma unroll
  for (int i = 0; i < D / 16; ++i) dq[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < S; k0 += SA_T) {
    __syncthreads();
    stage_rm<D>(Ks, base, rs, p.E + h * D, k0, S);
    stage_rm<D>(Vs, base, rs, 2 * p.E + h * D, k0, S);
    stage_tr<D>(Kt, base, rs, p.E + h * D, k0, S);
    __syncthreads();
    f32x4 s[4], dp[4];
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      s[st] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[st] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < D / 32; ++ks) {
        s[st] = mfma16(rm_frag<D>(Ks, 16 * st, ks, l), qf[ks], s[st]);
        dp[st] = mfma16(rm_frag<D>(Vs, 16 * st, ks, l), df[ks], dp[st]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {  // dS = P (dP - delta)
        const bool ok = qv && k0 + 16 * st + 4 * g + i < S;
        const float pr = ok ? __builtin_amdgcn_exp2f(s[st][i] * c - lse) : 0.f;
        s[st][i] = pr * (dp[st][i] - dl);
      }
    }
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2) {
      const bf16x8 sf = acc_pair(s[2 * c2], s[2 * c2 + 1]);
#pragma unroll
      for (int ds = 0; ds < D / 16; ++ds) dq[ds] = mfma16(tr_frag<D>(Kt, 16 * ds, c2, l), sf, dq[ds]);
    }
  }
  if (qv) {
    bf16* row = p.out + ((int64_t)q * p.N + n) * p.ld_out + h * D + 4 * g;
#pragma unroll
    for (int ds = 0; ds < D / 16; ++ds)
      *(bf16x4*)(row + 16 * ds) = bf16x4{f2bf(dq[ds][0] * p.scale), f2bf(dq[ds][1] * p.scale),
                                         f2bf(dq[ds][2] * p.scale), f2bf(dq[ds][3] * p.scale)};
  }
}

template <int D>
__global__ __launch_bounds__(256) void seqattn_dkdv_kernel(SeqAttnParams p) {
  using G = SeqGeo<D>;
  __shared__ __attribute__((aligned(16))) char smem[2 * G::TILE + 2 * G::TTILE + 2 * SA_T * 4];
  char* Qs = smem;
  char* Ds = smem + G::TILE;
  char* Qt = smem + 2 * G::TILE;
  char* Dt = Qt + G::TTILE;
  float* lse_s = (float*)(Dt + G::TTILE);
  float* dl_s = lse_s + SA_T;
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6, g = l >> 4;
  const int nh = blockIdx.y, n = nh / p.heads, h = nh - n * p.heads;
  const int S = p.S;
  const int64_t rs = (int64_t)p.N * p.ld_qkv, rso = (int64_t)p.N * p.ld_do;
  const bf16* base = p.qkv + (int64_t)n * p.ld_qkv;
  const bf16* dob = p.dout + (int64_t)n * p.ld_do;
  const int key = blockIdx.x * SA_T + 16 * w + (l & 15);
  const bool kv = key < S;
  const float c = p.scale * SA_LOG2E;
  bf16x8 kf[D / 32], vf[D / 32];
#pragma unroll
  for (int ks = 0; ks < D / 32; ++ks) {
    kf[ks] = kv ? *(const bf16x8*)(base + (int64_t)key * rs + p.E + h * D + 32 * ks + 8 * g) : bf16x8{};
    vf[ks] = kv ? *(const bf16x8*)(base + (int64_t)key * rs + 2 * p.E + h * D + 32 * ks + 8 * g) : bf16x8{};
  }
  f32x4 dk[D / 16], dv[D / 16];
#pragma unroll
  for (int i = 0; i < D / 16; ++i) {
    dk[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    dv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  for (int q0 = 0; q0 < S; q0 += SA_T) {
    __syncthreads();
    stage_rm<D>(Qs, base, rs, h * D, q0, S);
    stage_rm<D>(Ds, dob, rso, h * D, q0, S);
    stage_tr<D>(Qt, base, rs, h * D, q0, S);
    stage_tr<D>(Dt, dob, rso, h * D, q0, S);
    if (threadIdx.x < SA_T) {
      const int qq = q0 + threadIdx.x;
      lse_s[threadIdx.x] = qq < S ? p.lse2[(int64_t)nh * S + qq] : 0.f;
      dl_s[threadIdx.x] = qq < S ? p.delta[(int64_t)nh * S + qq] : 0.f;
    }
    __syncthreads();
    f32x4 s[4], dp[4];
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      s[st] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[st] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < D / 32; ++ks) {
        s[st] = mfma16(rm_frag<D>(Qs, 16 * st, ks, l), kf[ks], s[st]);
        dp[st] = mfma16(rm_frag<D>(Ds, 16 * st, ks, l), vf[ks], dp[st]);
      }
      const f32x4 ls = *(const f32x4*)(lse_s + 16 * st + 4 * g);
      const f32x4 dd = *(const f32x4*)(dl_s + 16 * st + 4 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i) {  // element (query 16st + 4g + i, key): P and dS
        const bool ok = kv && q0 + 16 * st + 4 * g + i < S;
        const float pr = ok ? __builtin_amdgcn_exp2f(s[st][i] * c - ls[i]) : 0.f;
        s[st][i] = pr;
        dp[st][i] = pr * (dp[st][i] - dd[i]);
      }
    }
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2) {
      const bf16x8 pf = acc_pair(s[2 * c2], s[2 * c2 + 1]);
      const bf16x8 sf = acc_pair(dp[2 * c2], dp[2 * c2 + 1]);
#pragma unroll
      for (int ds = 0; ds < D / 16; ++ds) {
        dv[ds] = mfma16(tr_frag<D>(Dt, 16 * ds, c2, l), pf, dv[ds]);
        dk[ds] = mfma16(tr_frag<D>(Qt, 16 * ds, c2, l), sf, dk[ds]);
      }
    }
  }
  if (kv) {
    bf16* row = p.out + ((int64_t)key * p.N + n) * p.ld_out + h * D + 4 * g;
#pragma unroll
    for (int ds = 0; ds < D / 16; ++ds) {
      *(bf16x4*)(row + p.E + 16 * ds) = bf16x4{f2bf(dk[ds][0] * p.scale), f2bf(dk[ds][1] * p.scale),
                                               f2bf(dk[ds][2] * p.scale), f2bf(dk[ds][3] * p.scale)};
      *(bf16x4*)(row + 2 * p.E + 16 * ds) = bf16x4{f2bf(dv[ds][0]), f2bf(dv[ds][1]), f2bf(dv[ds][2]),
                                                   f2bf(dv[ds][3])};
    }
  }
}

// ------------------------------------------------------------------------------ launchers
#define SEQ_DISPATCH(KER, grid, P, s)                                                         \
  switch (P.D) {                                                                              \
    case 64: hipLaunchKernelGGL(KER<64>, grid, dim3(256), 0, s, P); break;                    \
    case 128: hipLaunchKernelGGL(KER<128>, grid, dim3(256), 0, s, P); break;                  \
    default: hipLaunchKernelGGL(KER<256>, grid, dim3(256), 0, s, P); break;                   \
  }

void seqattn_fwd_launch(const SeqAttnParams& p, hipStream_t s) {
  const dim3 grid((unsigned)((p.S + SA_T - 1) / SA_T), (unsigned)(p.N * p.heads));
  SEQ_DISPATCH(seqattn_fwd_kernel, grid, p, s);
}

void seqattn_bwd_launch(const SeqAttnParams& p, hipStream_t s) {
  const int64_t items = (int64_t)p.S * p.N * p.heads;
  const dim3 gd((unsigned)((items + 3) / 4));
  SEQ_DISPATCH(seqattn_delta_kernel, gd, p, s);
  const dim3 grid((unsigned)((p.S + SA_T - 1) / SA_T), (unsigned)(p.N * p.heads));
  SEQ_DISPATCH(seqattn_dq_kernel, grid, p, s);
  SEQ_DISPATCH(seqattn_dkdv_kernel, grid, p, s);
}
#undef SEQ_DISPATCH

}  // namespace mmu
