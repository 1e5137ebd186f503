// MFMA bf16 GEMM with fused epilogues for the BERT block (gfx950).
//
// C[m,n] = sum_k A(m,k) B(n,k): both operands are staged global -> registers -> LDS
// in their STORED orientation (coalesced 16-B loads either way) and the MFMA
// fragments are read back with
//   * ds_read_b128            when the operand is K-contiguous  (XOR-swizzled 128-B rows)
//   * 2 x ds_read_b64_tr_b16  when it is M/N-contiguous         (XOR-swizzled 256-B rows)
// so forward (X.W^T), data-grad (dY.W) and weight-grad (dY^T.X) products are the
// same kernel with no transposed copies in HBM.  Both LDS images were checked
// bank-conflict free for their read instruction (docs: DESIGN.md §GEMM).
//
// Tile 128x128x64, 4 waves (2x2), each wave 64x64 = 4x4 v_mfma_f32_16x16x32_bf16
// tiles, two LDS stages, one barrier per K-tile.  The product is issued as
// mfma(Bfrag, Afrag) so each lane's accumulator holds 4 CONSECUTIVE n of one m:
// epilogue loads/stores are 8-B (bf16) / 16-B (f32) per lane.
#include "mmu_common.h"
#include "mmu_internal.h"

namespace mmu {

constexpr int BM = 128, BN = 128, BKT = 64;
constexpr int STAGE_BYTES = (BM * BKT + BN * BKT) * 2;  // 32 KiB

static __device__ __forceinline__ int sw_mn(int r) { return (r & 7) ^ (((r >> 3) & 1) << 2); }

// ---- global -> registers (4 x 16 B per thread per operand tile)
template <bool KMAJ>
static __device__ __forceinline__ void g_load(uint4 (&r)[4], const bf16* __restrict__ P, int64_t ld,
                                              int64_t r0, int64_t rlim, int64_t k0, int64_t klim, int t) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (KMAJ) {  // tile [128 rows][64 k]
      int row = (t >> 3) + 32 * i, c = t & 7;
      int64_t gr = r0 + row;
      r[i] = gr < rlim ? *(const uint4*)(P + gr * ld + k0 + 8 * c) : make_uint4(0, 0, 0, 0);
    } else {     // tile [64 k][128 rows]
      int kr = (t >> 4) + 16 * i, c = t & 15;
      int64_t gk = k0 + kr;
      r[i] = gk < klim ? *(const uint4*)(P + gk * ld + r0 + 8 * c) : make_uint4(0, 0, 0, 0);
    }
  }
}

template <bool KMAJ>
static __device__ __forceinline__ void s_store(char* s, const uint4 (&r)[4], int t) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int off;
    if (KMAJ) {
      int row = (t >> 3) + 32 * i, c = t & 7;
      off = row * 128 + ((c ^ (row & 7)) << 4);
    } else {
      int kr = (t >> 4) + 16 * i, c = t & 15;
      off = kr * 256 + (((c >> 1) ^ sw_mn(kr)) << 5) + ((c & 1) << 4);
    }
    *(uint4*)(s + off) = r[i];
  }
}

// fragment for v_mfma_f32_16x16x32_bf16: lane l holds operand[row0 + (l&15)][k = 32ks + 8(l>>4) + j]
template <bool KMAJ>
static __device__ __forceinline__ bf16x8 s_frag(const char* s, int row0, int ks, int l) {
  if (KMAJ) {
    int row = row0 + (l & 15), c = 4 * ks + (l >> 4);
    return *(const bf16x8*)(s + row * 128 + ((c ^ (row & 7)) << 4));
  } else {
    int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
    int b = row0 >> 4;
    int k0 = 32 * ks + 8 * g + q, k1 = k0 + 4;
    const char* a0 = s + k0 * 256 + ((b ^ sw_mn(k0)) << 5) + 8 * p;
    const char* a1 = s + k1 * 256 + ((b ^ sw_mn(k1)) << 5) + 8 * p;
    bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((MMU_LDS(bf16x4)*)a0);
    bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((MMU_LDS(bf16x4)*)a1);
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

template <bool AK, bool BKM, int EPI, bool OUT_F32>
__global__ __launch_bounds__(256) void gemm_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];
  const int t = threadIdx.x, l = t & 63, w = t >> 6, wm = w >> 1, wn = w & 1;
  const int nwg = p.tiles_m * p.tiles_n;
  const int pid = xcd_remap(blockIdx.x, nwg);
  const int tm = pid / p.tiles_n, tn = pid - tm * p.tiles_n;
  const int64_t z = blockIdx.z;
  const bf16* __restrict__ A = p.A + z * p.sA;
  const bf16* __restrict__ B = p.B + z * p.sB;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[4], rb[4];
  // split-K: slice blockIdx.y owns k in [kb, ke); kchunk is a multiple of the K tile
  const int64_t kb = (int64_t)blockIdx.y * p.kchunk;
  const int64_t ke = kb + p.kchunk < p.K ? kb + p.kchunk : p.K;
  const int nk = (int)((ke - kb + BKT - 1) / BKT);
  g_load<AK>(ra, A, p.lda, m0, p.M, kb, ke, t);
  g_load<BKM>(rb, B, p.ldb, n0, p.N, kb, ke, t);
  s_store<AK>(smem, ra, t);
  s_store<BKM>(smem + BM * BKT * 2, rb, t);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const char* sa = smem + (kt & 1) * STAGE_BYTES;
    const char* sb = sa + BM * BKT * 2;
    const bool more = kt + 1 < nk;
    if (more) {
      g_load<AK>(ra, A, p.lda, m0, p.M, kb + (int64_t)(kt + 1) * BKT, ke, t);
      g_load<BKM>(rb, B, p.ldb, n0, p.N, kb + (int64_t)(kt + 1) * BKT, ke, t);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fb[4], fa[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fb[i] = s_frag<BKM>(sb, 64 * wn + 16 * i, ks, l);
#pragma unroll
      for (int j = 0; j < 4; ++j) fa[j] = s_frag<AK>(sa, 64 * wm + 16 * j, ks, l);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      char* dst = smem + ((kt + 1) & 1) * STAGE_BYTES;
      s_store<AK>(dst, ra, t);
      s_store<BKM>(dst + BM * BKT * 2, rb, t);
    }
    __syncthreads();
  }

  // ------------------------------------------------------------------ epilogue
  if (p.splitk > 1) {  // raw partial product -> this slice's f32 slab; summed by splitk_reduce_kernel
    float* slab = p.ws + (z * p.splitk + blockIdx.y) * p.M * p.N;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t n = n0 + 64 * wn + 16 * i + 4 * (l >> 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t m = m0 + 64 * wm + 16 * j + (l & 15);
        if (m < p.M) *(float4*)(slab + m * p.N + n) = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      }
    }
    return;
  }
  const float* bias = p.bias ? p.bias + z * p.bias_bstride : nullptr;
  const bf16* res = p.residual ? (const bf16*)p.residual + z * p.res_bstride : nullptr;
  bf16* aux = p.aux ? (bf16*)p.aux + z * p.aux_bstride : nullptr;
  const float scale = p.drop_p > 0.f ? 1.0f / (1.0f - p.drop_p) : 1.0f;
  const uint32_t thr = (uint32_t)(p.drop_p * 65536.0f + 0.5f);
  float cs[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) cs[i][r] = 0.f;

#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t n = n0 + 64 * wn + 16 * i + 4 * (l >> 4);
    float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (bias && EPI != MMU_EPI_DGELU && EPI != MMU_EPI_ADD_RES) bv = *(const float4*)(bias + n);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t m = m0 + 64 * wm + 16 * j + (l & 15);
      if (m >= p.M) continue;
      float v[4] = {acc[i][j][0] + bv.x, acc[i][j][1] + bv.y, acc[i][j][2] + bv.z, acc[i][j][3] + bv.w};
      if (EPI == MMU_EPI_BIAS_GELU) {
        bf16x4 zq = {f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
        *(bf16x4*)(aux + m * p.ldx + n) = zq;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = gelu_erf(v[r]);
      } else if (EPI == MMU_EPI_BIAS_DROP_RES) {
        if (p.drop_p > 0.f) {
          // counter over the whole batched output: batch item z, row m, column n
          uint32_t keep = mmu_keep4(p.seed, (uint64_t)((z * p.M + m) * p.N + n) >> 2, thr);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = ((keep >> r) & 1) ? v[r] * scale : 0.f;
        }
        bf16x4 rv = *(const bf16x4*)(res + m * p.ldr + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += bf2f(rv[r]);
      } else if (EPI == MMU_EPI_DGELU) {
        bf16x4 zv = *(const bf16x4*)(aux + m * p.ldx + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] *= gelu_erf_grad(bf2f(zv[r]));
      } else if (EPI == MMU_EPI_ADD_RES) {
        bf16x4 rv = *(const bf16x4*)(res + m * p.ldr + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += bf2f(rv[r]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[i][r] += v[r];
      if (OUT_F32) {
        float* C = (float*)p.C + z * p.sC + m * p.ldc + n;
        if (p.accumulate) {
          float4 o = *(float4*)C;
          v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
        }
        *(float4*)C = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        bf16* C = (bf16*)p.C + z * p.sC + m * p.ldc + n;
        *(bf16x4*)C = bf16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
      }
    }
  }
  if (p.colsum) {
    float* part = p.colsum + z * p.colsum_bstride + ((int64_t)tm * 2 + wm) * p.N;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = cs[i][r];
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        s += __shfl_xor(s, 4, 64);
        s += __shfl_xor(s, 8, 64);
        cs[i][r] = s;
      }
      if ((l & 15) == 0) {
        const int64_t n = n0 + 64 * wn + 16 * i + 4 * (l >> 4);
        *(float4*)(part + n) = make_float4(cs[i][0], cs[i][1], cs[i][2], cs[i][3]);
      }
    }
  }
}

template <bool AK, bool BKM, int EPI, bool F32>
static void launch_t(const GemmParams& p, int batch, hipStream_t s) {
  dim3 grid(p.tiles_m * p.tiles_n, p.splitk, batch);
  hipLaunchKernelGGL((gemm_kernel<AK, BKM, EPI, F32>), grid, dim3(256), 0, s, p);
}

// C[z] (+)= sum over the split-K slabs of batch item z (fixed slice order: deterministic)
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, float* __restrict__ C,
                                                            int64_t M, int64_t N, int64_t ldc, int64_t sC,
                                                            int splitk, int accumulate) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;  // float4 index within one batch item
  const int64_t z = blockIdx.y;
  if (q * 4 >= M * N) return;
  const int64_t e = q * 4, m = e / N, n = e - m * N;
  const float* s = ws + z * splitk * M * N + e;
  float4 a = *(const float4*)s;
  for (int k = 1; k < splitk; ++k) {
    const float4 b = *(const float4*)(s + k * M * N);
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  }
  float* c = C + z * sC + m * ldc + n;
  if (accumulate) {
    const float4 o = *(const float4*)c;
    a.x += o.x; a.y += o.y; a.z += o.z; a.w += o.w;
  }
  *(float4*)c = a;
}

void splitk_reduce_launch(const GemmParams& p, int batch, hipStream_t s) {
  const int64_t q = (p.M * p.N) / 4;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((q + 255) / 256), batch), dim3(256), 0, s, p.ws,
                     (float*)p.C, p.M, p.N, p.ldc, p.sC, p.splitk, p.accumulate);
}

template <int EPI, bool F32>
static void launch_e(const GemmParams& p, bool ak, bool bk, int batch, hipStream_t s) {
  if (ak && bk) launch_t<true, true, EPI, F32>(p, batch, s);
  else if (ak && !bk) launch_t<true, false, EPI, F32>(p, batch, s);
  else if (!ak && !bk) launch_t<false, false, EPI, F32>(p, batch, s);
  else launch_t<false, true, EPI, F32>(p, batch, s);
}

void gemm_launch(const GemmParams& p, bool ak, bool bk, bool f32out, int batch, hipStream_t s) {
  switch (p.kind) {
    case MMU_EPI_STORE:
      if (f32out) launch_e<MMU_EPI_STORE, true>(p, ak, bk, batch, s);
      else launch_e<MMU_EPI_STORE, false>(p, ak, bk, batch, s);
      break;
    case MMU_EPI_BIAS_GELU: launch_e<MMU_EPI_BIAS_GELU, false>(p, ak, bk, batch, s); break;
    case MMU_EPI_BIAS_DROP_RES: launch_e<MMU_EPI_BIAS_DROP_RES, false>(p, ak, bk, batch, s); break;
    case MMU_EPI_DGELU: launch_e<MMU_EPI_DGELU, false>(p, ak, bk, batch, s); break;
    case MMU_EPI_ADD_RES: launch_e<MMU_EPI_ADD_RES, false>(p, ak, bk, batch, s); break;
  }
}

// ------------------------------------------------------------------ column sums
// grid (ceil(N/256), ceil(parts/64)): each thread sums 64 partial rows of one column and adds
// the result into out with one float atomic (out zeroed first when not accumulating)
constexpr int COLSUM_ROWS = 64;
__global__ __launch_bounds__(256) void colsum_reduce_kernel(const float* __restrict__ part, int64_t parts, int64_t N,
                                                            float* __restrict__ out) {
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const int64_t r0 = (int64_t)blockIdx.y * COLSUM_ROWS;
  const int64_t r1 = r0 + COLSUM_ROWS < parts ? r0 + COLSUM_ROWS : parts;
  float s = 0.f;
  for (int64_t r = r0; r < r1; ++r) s += part[r * N + n];
  atomicAdd(out + n, s);
}

void colsum_reduce_launch(const float* part, int64_t parts, int64_t N, float* out, int acc, hipStream_t s) {
  if (!acc) (void)hipMemsetAsync(out, 0, sizeof(float) * N, s);
  hipLaunchKernelGGL(colsum_reduce_kernel,
                     dim3((unsigned)((N + 255) / 256), (unsigned)((parts + COLSUM_ROWS - 1) / COLSUM_ROWS)),
                     dim3(256), 0, s, part, parts, N, out);
}

// bf16 [M,N] -> partial[ceil(M/256), N]: each block sums 256 rows for 512 columns (8 per lane-column pass)
__global__ __launch_bounds__(256) void colsum_bf16_kernel(const bf16* __restrict__ X, int64_t M, int64_t N,
                                                          int64_t ld, float* __restrict__ part) {
  const int64_t r0 = (int64_t)blockIdx.y * 256;
  const int64_t c = ((int64_t)blockIdx.x * 64 + (threadIdx.x & 63)) * 8;
  const int wv = threadIdx.x >> 6;
  __shared__ float red[4][64 * 8];
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c < N) {
    for (int64_t r = r0 + wv; r < r0 + 256 && r < M; r += 4) {
      bf16x8 v = *(const bf16x8*)(X + r * ld + c);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += bf2f(v[e]);
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[wv][(threadIdx.x & 63) * 8 + e] = s[e];
  __syncthreads();
  if (wv == 0 && c < N) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      int q = (threadIdx.x & 63) * 8 + e;
      part[blockIdx.y * N + c + e] = red[0][q] + red[1][q] + red[2][q] + red[3][q];
    }
  }
}

void colsum_bf16_launch(const bf16* X, int64_t M, int64_t N, int64_t ld, float* part, float* out, int acc,
                        hipStream_t s) {
  int64_t parts = (M + 255) / 256;
  hipLaunchKernelGGL(colsum_bf16_kernel, dim3((unsigned)((N / 8 + 63) / 64), (unsigned)parts), dim3(256), 0, s,
                     X, M, N, ld, part);
  colsum_reduce_launch(part, parts, N, out, acc, s);
}

}  // namespace mmu
