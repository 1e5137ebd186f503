// MFMA bf16 GEMM with fused epilogues for the BERT block (gfx950).
//
// C[m,n] = sum_k A(m,k) B(n,k): both operands are staged into LDS in their STORED
// orientation (16-B coalesced loads either way) and the v_mfma_f32_16x16x32_bf16
// fragments are read back with
//   * ds_read_b128            when the operand is K-contiguous  (XOR-swizzled 128-B rows)
//   * 2 x ds_read_b64_tr_b16  when it is M/N-contiguous         (XOR-swizzled 32-B blocks)
// so forward (X.W^T), data-grad (dY.W) and weight-grad (dY^T.X) products are one
// kernel with no transposed copies in HBM.  Every LDS image was enumerated bank-
// conflict free for its read instruction.
//
// Two tilings:
//  * "big"   256x256x64, 8 waves (2 M x 4 N, 128x64 each), global->LDS by buffer_load...lds
//            (LDS-DMA: no VGPR staging; swizzle applied to the per-lane SOURCE address;
//            buffer range checks zero-fill every row/k beyond the operand), 2 LDS stages,
//            one barrier per K-tile.  Used whenever M and N are >= 256.
//  * "small" 128x128x64, 4 waves, register-staged (small / ragged problems).
// The product is issued as mfma(Bfrag, Afrag), so every lane's accumulator holds 4
// CONSECUTIVE n of one m: 8-B (bf16) / 16-B (f32) epilogue accesses.
// Split-K (weight gradients: K = tokens, few output tiles): grid.y slices write f32
// slabs, summed in slice order by splitk_reduce_kernel (deterministic).
#include "mmu_common.h"
#include "mmu_internal.h"

namespace mmu {

constexpr int BKT = 64;

static __device__ __forceinline__ int sw_mn(int r) { return (r & 7) ^ (((r >> 3) & 1) << 2); }

// ---------------------------------------------------------------- fragment reads
// lane l holds operand[row0 + (l&15)][k = 32ks + 8(l>>4) + j], j = 0..7
template <bool KMAJ, int ROWB>  // ROWB: bytes per LDS row of an M/N-major tile (256 or 512)
static __device__ __forceinline__ bf16x8 s_frag(const char* s, int row0, int ks, int l) {
  if (KMAJ) {
    const int row = row0 + (l & 15), c = 4 * ks + (l >> 4);
    return *(const bf16x8*)(s + row * 128 + ((c ^ (row & 7)) << 4));
  } else {
    const int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
    const int b = row0 >> 4;
    const int k0 = 32 * ks + 8 * g + q, k1 = k0 + 4;
    const char* a0 = s + k0 * ROWB + ((b ^ sw_mn(k0)) << 5) + 8 * p;
    const char* a1 = s + k1 * ROWB + ((b ^ sw_mn(k1)) << 5) + 8 * p;
    bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((MMU_LDS(bf16x4)*)a0);
    bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((MMU_LDS(bf16x4)*)a1);
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

// ---------------------------------------------------------------- shared epilogue
// one (m, n..n+3) quad of the output; returns the final values (for column sums)
template <int EPI, bool OUT_F32>
static __device__ __forceinline__ void epi_quad(const GemmParams& p, int64_t z, int64_t m, int64_t n, f32x4 a,
                                                const float* bias, const bf16* res, bf16* aux, float scale,
                                                uint32_t thr, float (&v)[4]) {
  float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
  if (bias && EPI != MMU_EPI_DGELU && EPI != MMU_EPI_ADD_RES) bv = *(const float4*)(bias + n);
  v[0] = a[0] + bv.x; v[1] = a[1] + bv.y; v[2] = a[2] + bv.z; v[3] = a[3] + bv.w;
  if (EPI == MMU_EPI_BIAS_GELU) {
    *(bf16x4*)(aux + m * p.ldx + n) = bf16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = gelu_erf(v[r]);
  } else if (EPI == MMU_EPI_BIAS_DROP_RES) {
    if (thr) {  // counter over the whole batched output: batch item z, row m, column n
      const uint32_t keep = mmu_keep4(p.seed, (uint64_t)((z * p.M + m) * p.N + n) >> 2, thr);
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = ((keep >> r) & 1) ? v[r] * scale : 0.f;
    }
    const bf16x4 rv = *(const bf16x4*)(res + m * p.ldr + n);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] += bf2f(rv[r]);
  } else if (EPI == MMU_EPI_DGELU) {
    const bf16x4 zv = *(const bf16x4*)(aux + m * p.ldx + n);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] *= gelu_erf_grad(bf2f(zv[r]));
  } else if (EPI == MMU_EPI_ADD_RES) {
    const bf16x4 rv = *(const bf16x4*)(res + m * p.ldr + n);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] += bf2f(rv[r]);
  }
  if (OUT_F32) {
    float* C = (float*)p.C + z * p.sC + m * p.ldc + n;
    float o[4] = {v[0], v[1], v[2], v[3]};
    if (p.accumulate) {
      const float4 c = *(float4*)C;
      o[0] += c.x; o[1] += c.y; o[2] += c.z; o[3] += c.w;
    }
    *(float4*)C = make_float4(o[0], o[1], o[2], o[3]);
  } else {
    *(bf16x4*)((bf16*)p.C + z * p.sC + m * p.ldc + n) = bf16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
  }
}

// column sums of a wave's (16-row groups x NI n-quads) block -> atomicAdd into colsum[N]
template <int NI>
static __device__ __forceinline__ void colsum_flush(float (&cs)[NI][4], float* out, int64_t nbase, int l) {
#pragma unroll
  for (int i = 0; i < NI; ++i) {
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
      const int64_t n = nbase + 16 * i + 4 * (l >> 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) atomicAdd(out + n + r, cs[i][r]);
    }
  }
}

// the shared epilogue over a wave's accumulator block acc[NI][NJ] (n-subtile i, m-subtile j)
template <int EPI, bool OUT_F32, int NI, int NJ>
static __device__ __forceinline__ void epilogue_block(const GemmParams& p, int64_t z, int64_t mw, int64_t nw,
                                                      f32x4 (&acc)[NI][NJ], int l) {
  if (p.splitk > 1) {  // raw partial product -> this slice's f32 slab (summed by splitk_reduce_kernel)
    float* slab = p.ws + (z * p.splitk + blockIdx.y) * p.M * p.N;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int64_t n = nw + 16 * i + 4 * (l >> 4);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int64_t m = mw + 16 * j + (l & 15);
        if (m < p.M && n < p.N) *(float4*)(slab + m * p.N + n) = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      }
    }
    return;
  }
  const float* bias = p.bias ? p.bias + z * p.bias_bstride : nullptr;
  const bf16* res = p.residual ? (const bf16*)p.residual + z * p.res_bstride : nullptr;
  bf16* aux = p.aux ? (bf16*)p.aux + z * p.aux_bstride : nullptr;
  const float scale = p.drop_p > 0.f ? 1.0f / (1.0f - p.drop_p) : 1.0f;
  const uint32_t thr = (uint32_t)(p.drop_p * 65536.0f + 0.5f);
  float cs[NI][4];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) cs[i][r] = 0.f;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int64_t n = nw + 16 * i + 4 * (l >> 4);
    if (n >= p.N) continue;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int64_t m = mw + 16 * j + (l & 15);
      if (m >= p.M) continue;
      float v[4];
      epi_quad<EPI, OUT_F32>(p, z, m, n, acc[i][j], bias, res, aux, scale, thr, v);
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[i][r] += v[r];
    }
  }
  if (p.colsum) colsum_flush<NI>(cs, p.colsum + z * p.colsum_bstride, nw, l);
}

// ================================================================ small: 128x128, register staged
constexpr int SBM = 128, SBN = 128;
constexpr int S_STAGE = (SBM * BKT + SBN * BKT) * 2;  // 32 KiB

template <bool KMAJ>
static __device__ __forceinline__ void g_load(uint4 (&r)[4], const bf16* __restrict__ P, int64_t ld, int64_t r0,
                                              int64_t rlim, int64_t k0, int64_t klim, int t) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (KMAJ) {  // tile [128 rows][64 k]
      const int row = (t >> 3) + 32 * i, c = t & 7;
      const int64_t gr = r0 + row;
      r[i] = gr < rlim ? *(const uint4*)(P + gr * ld + k0 + 8 * c) : make_uint4(0, 0, 0, 0);
    } else {     // tile [64 k][128 rows]
      const int kr = (t >> 4) + 16 * i, c = t & 15;
      const int64_t gk = k0 + kr;
      r[i] = (gk < klim && r0 + 8 * c < rlim) ? *(const uint4*)(P + gk * ld + r0 + 8 * c) : make_uint4(0, 0, 0, 0);
    }
  }
}

template <bool KMAJ>
static __device__ __forceinline__ void s_store(char* s, const uint4 (&r)[4], int t) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int off;
    if (KMAJ) {
      const int row = (t >> 3) + 32 * i, c = t & 7;
      off = row * 128 + ((c ^ (row & 7)) << 4);
    } else {
      const int kr = (t >> 4) + 16 * i, c = t & 15;
      off = kr * 256 + (((c >> 1) ^ sw_mn(kr)) << 5) + ((c & 1) << 4);
    }
    *(uint4*)(s + off) = r[i];
  }
}

template <bool AK, bool BKM, int EPI, bool OUT_F32>
__global__ __launch_bounds__(256) void gemm_small_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * S_STAGE];
  const int t = threadIdx.x, l = t & 63, w = t >> 6, wm = w >> 1, wn = w & 1;
  const int nwg = p.tiles_m * p.tiles_n;
  const int pid = xcd_remap(blockIdx.x, nwg);
  const int tm = pid / p.tiles_n, tn = pid - tm * p.tiles_n;
  const int64_t z = blockIdx.z;
  const bf16* __restrict__ A = p.A + z * p.sA;
  const bf16* __restrict__ B = p.B + z * p.sB;
  const int64_t m0 = (int64_t)tm * SBM, n0 = (int64_t)tn * SBN;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint4 ra[4], rb[4];
  const int64_t kb = (int64_t)blockIdx.y * p.kchunk;
  const int64_t ke = kb + p.kchunk < p.K ? kb + p.kchunk : p.K;
  const int nk = (int)((ke - kb + BKT - 1) / BKT);
  g_load<AK>(ra, A, p.lda, m0, p.M, kb, ke, t);
  g_load<BKM>(rb, B, p.ldb, n0, p.N, kb, ke, t);
  s_store<AK>(smem, ra, t);
  s_store<BKM>(smem + SBM * BKT * 2, rb, t);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const char* sa = smem + (kt & 1) * S_STAGE;
    const char* sb = sa + SBM * BKT * 2;
    const bool more = kt + 1 < nk;
    if (more) {
      g_load<AK>(ra, A, p.lda, m0, p.M, kb + (int64_t)(kt + 1) * BKT, ke, t);
      g_load<BKM>(rb, B, p.ldb, n0, p.N, kb + (int64_t)(kt + 1) * BKT, ke, t);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fb[4], fa[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fb[i] = s_frag<BKM, 256>(sb, 64 * wn + 16 * i, ks, l);
#pragma unroll
      for (int j = 0; j < 4; ++j) fa[j] = s_frag<AK, 256>(sa, 64 * wm + 16 * j, ks, l);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      char* dst = smem + ((kt + 1) & 1) * S_STAGE;
      s_store<AK>(dst, ra, t);
      s_store<BKM>(dst + SBM * BKT * 2, rb, t);
    }
    __syncthreads();
  }
  epilogue_block<EPI, OUT_F32, 4, 4>(p, z, m0 + 64 * wm, n0 + 64 * wn, acc, l);
}

// ================================================================ big: 256x256, LDS-DMA
constexpr int BBM = 256, BBN = 256;
constexpr int B_TILE = BBM * BKT * 2;  // 32 KiB per operand per stage
constexpr int B_STAGE = 2 * B_TILE;

// one operand tile (256 rows x 64 k) via 4 x 1 KiB buffer_load...lds per wave (8 waves).
// K-major: LDS [256 rows][128 B], chunk c of row r at physical chunk c ^ (r & 7).
// M/N-major: LDS [64 k][512 B], 32-B block b of k-row r at physical block b ^ sw_mn(r).
// Every lane's LDS slot is fixed (base + 16*lane); the swizzle picks which SOURCE it loads.
template <bool KMAJ>
static __device__ __forceinline__ void dma_tile(char* s, __amdgpu_buffer_rsrc_t rsrc, int64_t ld, int64_t r0,
                                                int64_t k0, int w, int l) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = w * 4 + i;  // 1 KiB piece of the 32 KiB tile
    uint32_t src;
    if (KMAJ) {
      const int row = piece * 8 + (l >> 3), c = (l & 7) ^ (row & 7);
      src = (uint32_t)(((r0 + row) * ld + k0 + 8 * c) * 2);
    } else {
      const int kr = piece * 2 + (l >> 5), j = l & 31;
      const int b = (j >> 1) ^ sw_mn(kr);
      src = (uint32_t)(((k0 + kr) * ld + r0 + 16 * b + 8 * (j & 1)) * 2);
    }
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (MMU_LDS(void)*)(s + piece * 1024), 16, src, 0, 0, 0);
  }
}

template <bool AK, bool BKM, int EPI, bool OUT_F32>
__global__ __launch_bounds__(512) void gemm_big_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * B_STAGE];
  const int t = threadIdx.x, l = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w >> 2, wn = w & 3;
  const int nwg = p.tiles_m * p.tiles_n;
  const int pid = xcd_remap(blockIdx.x, nwg);
  const int tm = pid / p.tiles_n, tn = pid - tm * p.tiles_n;
  const int64_t z = blockIdx.z;
  const int64_t m0 = (int64_t)tm * BBM, n0 = (int64_t)tn * BBN;
  // operand byte ranges: rows (K-major) or k-rows (M/N-major) beyond the operand read as zero
  const int64_t a_bytes = (AK ? p.M * p.lda : p.K * p.lda) * 2;
  const int64_t b_bytes = (BKM ? p.N * p.ldb : p.K * p.ldb) * 2;
  // (host guarantees both spans < 4 GiB: 32-bit num_records / voffset)
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.A + z * p.sA), 0, (int)(uint32_t)a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.B + z * p.sB), 0, (int)(uint32_t)b_bytes, 0x00020000);

  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int64_t kb = (int64_t)blockIdx.y * p.kchunk;
  const int64_t ke = kb + p.kchunk < p.K ? kb + p.kchunk : p.K;
  const int nk = (int)((ke - kb + BKT - 1) / BKT);
  dma_tile<AK>(smem, ra, p.lda, m0, kb, w, l);
  dma_tile<BKM>(smem + B_TILE, rb, p.ldb, n0, kb, w, l);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const char* sa = smem + (kt & 1) * B_STAGE;
    const char* sb = sa + B_TILE;
    if (kt + 1 < nk) {
      char* d = smem + ((kt + 1) & 1) * B_STAGE;
      const int64_t k1 = kb + (int64_t)(kt + 1) * BKT;
      dma_tile<AK>(d, ra, p.lda, m0, k1, w, l);
      dma_tile<BKM>(d + B_TILE, rb, p.ldb, n0, k1, w, l);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fb[4], fa[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) fb[i] = s_frag<BKM, 512>(sb, 64 * wn + 16 * i, ks, l);
#pragma unroll
      for (int j = 0; j < 8; ++j) fa[j] = s_frag<AK, 512>(sa, 128 * wm + 16 * j, ks, l);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  epilogue_block<EPI, OUT_F32, 4, 8>(p, z, m0 + 128 * wm, n0 + 64 * wn, acc, l);
}

// ---------------------------------------------------------------- launch
template <bool AK, bool BKM, int EPI, bool F32>
static void launch_t(const GemmParams& p, bool big, int batch, hipStream_t s) {
  dim3 grid(p.tiles_m * p.tiles_n, p.splitk, batch);
  if (big) hipLaunchKernelGGL((gemm_big_kernel<AK, BKM, EPI, F32>), grid, dim3(512), 0, s, p);
  else hipLaunchKernelGGL((gemm_small_kernel<AK, BKM, EPI, F32>), grid, dim3(256), 0, s, p);
}

template <int EPI, bool F32>
static void launch_e(const GemmParams& p, bool ak, bool bk, bool big, int batch, hipStream_t s) {
  if (ak && bk) launch_t<true, true, EPI, F32>(p, big, batch, s);
  else if (ak && !bk) launch_t<true, false, EPI, F32>(p, big, batch, s);
  else if (!ak && !bk) launch_t<false, false, EPI, F32>(p, big, batch, s);
  else launch_t<false, true, EPI, F32>(p, big, batch, s);
}

void gemm_launch(const GemmParams& p, bool ak, bool bk, bool f32out, bool big, int batch, hipStream_t s) {
  switch (p.kind) {
    case MMU_EPI_STORE:
      if (f32out) launch_e<MMU_EPI_STORE, true>(p, ak, bk, big, batch, s);
      else launch_e<MMU_EPI_STORE, false>(p, ak, bk, big, batch, s);
      break;
    case MMU_EPI_BIAS_GELU: launch_e<MMU_EPI_BIAS_GELU, false>(p, ak, bk, big, batch, s); break;
    case MMU_EPI_BIAS_DROP_RES: launch_e<MMU_EPI_BIAS_DROP_RES, false>(p, ak, bk, big, batch, s); break;
    case MMU_EPI_DGELU: launch_e<MMU_EPI_DGELU, false>(p, ak, bk, big, batch, s); break;
    case MMU_EPI_ADD_RES: launch_e<MMU_EPI_ADD_RES, false>(p, ak, bk, big, batch, s); break;
  }
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

// bf16 [M,N] column sums: each block sums 256 rows x 512 columns, one atomic per column
__global__ __launch_bounds__(256) void colsum_bf16_kernel(const bf16* __restrict__ X, int64_t M, int64_t N,
                                                          int64_t ld, float* __restrict__ out) {
  const int64_t r0 = (int64_t)blockIdx.y * 256;
  const int64_t c = ((int64_t)blockIdx.x * 64 + (threadIdx.x & 63)) * 8;
  const int wv = threadIdx.x >> 6;
  __shared__ float red[4][64 * 8];
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c < N) {
    for (int64_t r = r0 + wv; r < r0 + 256 && r < M; r += 4) {
      const bf16x8 v = *(const bf16x8*)(X + r * ld + c);
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
      const int q = (threadIdx.x & 63) * 8 + e;
      atomicAdd(out + c + e, red[0][q] + red[1][q] + red[2][q] + red[3][q]);
    }
  }
}

void colsum_bf16_launch(const bf16* X, int64_t M, int64_t N, int64_t ld, float* part, float* out, int acc,
                        hipStream_t s) {
  (void)part;
  if (!acc) (void)hipMemsetAsync(out, 0, sizeof(float) * N, s);
  hipLaunchKernelGGL(colsum_bf16_kernel, dim3((unsigned)((N / 8 + 63) / 64), (unsigned)((M + 255) / 256)),
                     dim3(256), 0, s, X, M, N, ld, out);
}

}  // namespace mmu
