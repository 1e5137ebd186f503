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
#include <cstdlib>

namespace mmu {

constexpr int BKT = 64;

// Diagnostic build only (make EXTRA=-DMMU_GEMM_STAMPS OUT=../../ab/stamps.so): wave 0 of every
// big-kernel workgroup records s_memtime at start, after the first K-tile landed, after the
// K loop and after the epilogue (tools/gemm_stamps.py reads them back).
#ifdef MMU_GEMM_STAMPS
__device__ uint64_t g_gemm_stamps[1 << 16][4];
#define GEMM_STAMP(i)                                                                       \
  do {                                                                                      \
    if (threadIdx.x == 0) {                                                                 \
      const int lin_ = (int)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)); \
      if (lin_ < (1 << 16)) g_gemm_stamps[lin_][i] = __builtin_amdgcn_s_memtime();          \
    }                                                                                       \
  } while (0)
#else
#define GEMM_STAMP(i) \
  do {                \
  } while (0)
#endif

static __device__ __forceinline__ int sw_mn(int r) { return (r & 7) ^ (((r >> 3) & 1) << 2); }

// ---------------------------------------------------------------- tile order
// Grouped order: pids walk GROUP_M tile rows column by column, so the ~32 tiles an XCD
// runs at once (consecutive pids after xcd_remap) form an 8 x 4 block sharing 8 A and 4 B
// panels instead of ~3 x 12 (row-major at N = 3072), which cut the L2 misses of the wide
// products (rocprofv3 FETCH_SIZE, profiles/).
// GROUP_M = p.group_m (host heuristic in capi.hip; 1 = plain row-major order).
static __device__ __forceinline__ void tile_of(int pid, int tiles_m, int tiles_n, int group_m, int& tm, int& tn) {
  const int per_group = group_m * tiles_n;
  const int g = pid / per_group, first = g * group_m;
  const int gm = tiles_m - first < group_m ? tiles_m - first : group_m;
  const int r = pid - g * per_group;
  tm = first + r % gm;
  tn = r / gm;
}
// The dispatcher deals workgroups to the 8 XCDs round-robin by LINEAR id (x fastest, then
// y = split-K slice, then z = batch item).  Remap the linear id so each XCD holds a
// contiguous run of pids, and order pids batch item > slice > tile: blocks of one slice
// (which share A / B K-ranges) then sit on one XCD's L2.
static __device__ __forceinline__ void block_tile(const GemmParams& p, int64_t& z, int& slice, int& tm, int& tn) {
  const int ntiles = p.tiles_m * p.tiles_n;
  const int per_z = ntiles * (int)gridDim.y;
  const int lin = (int)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z));
  const int pid = xcd_remap(lin, per_z * (int)gridDim.z);
  z = pid / per_z;
  const int r = pid - (int)z * per_z;
  slice = r / ntiles;
  tile_of(r - slice * ntiles, p.tiles_m, p.tiles_n, p.group_m, tm, tn);
}

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
// A wave's accumulators hold 4 consecutive n of one m per lane (16 rows per register
// group), which as direct stores is 16 scattered 8-B pieces per instruction.  The
// epilogue therefore turns each 64-row x 64-col f32 block around in the wave's own
// 16 KiB of the (now idle) staging LDS -- written as acc quads, 16-B chunk c of row r at
// c ^ (r & 15) (conflict-free ds_write_b128 and ds_read_b128) -- and reads it back as 8
// consecutive columns per lane, 8 lanes per row: every global access of the epilogue
// (residual / aux loads, bf16 or f32 stores, split-K slabs) is then a 16-B-per-lane
// access covering full 128-B lines.

// one (m, n..n+7) octet: epilogue math + store; v holds acc (+ bias) on entry.  The row's
// addresses arrive precomputed (epilogue_block: a per-lane base + a wave-uniform row offset, so
// no per-row 64-bit VALU multiplies): cdst = &C[z][m][n], xdst = &aux[z][m][n], qd = the
// dropout quad counter ((z M + m) N + n) / 4
template <int EPI, bool OUT_F32>
static __device__ __forceinline__ void epi_oct(const GemmParams& p, void* cdst, bf16* xdst, uint64_t qd,
                                               float (&v)[8], const float (&in)[8], float scale, uint32_t thr,
                                               uint64_t seed) {
  if (EPI == MMU_EPI_BIAS_GELU) {  // C = gelu(z); aux (optional) = gelu'(z) for the backward
    float d[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) gelu_pair(v[r], v[r], d[r]);
    if (xdst) {
      bf16x8 o;
#pragma unroll
      for (int r = 0; r < 8; ++r) o[r] = f2bf(d[r]);
      *(bf16x8*)xdst = o;
    }
  } else if (EPI == MMU_EPI_BIAS_DROP_RES) {
    if (thr) {  // counter over the whole batched output: batch item z, row m, column n (quads)
      const uint32_t keep = mmu_keep4(seed, qd, thr) | (mmu_keep4(seed, qd + 1, thr) << 4);
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = ((keep >> r) & 1) ? v[r] * scale : 0.f;
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] += in[r];  // residual (f32 when C is f32: the hidden stream)
  } else if (EPI == MMU_EPI_BIAS_DROP_QGELU) {  // FLAVA mlp: u = dropout(z); C = u*sigmoid(1.702u)
    uint32_t keep = 0xFFu;                         // aux (optional) = dC/dz = keep*scale*qgelu'(u)
    if (thr) keep = mmu_keep4(seed, qd, thr) | (mmu_keep4(seed, qd + 1, thr) << 4);
    float d[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const float kz = ((keep >> r) & 1) ? scale : 0.f;
      const float u = v[r] * kz;
      const float sg = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(u * -2.4554669595930157f));  // 1.702 log2 e
      v[r] = u * sg;
      d[r] = kz * fmaf(1.702f * u * sg, 1.0f - sg, sg);
    }
    if (xdst) {
      bf16x8 o;
#pragma unroll
      for (int r = 0; r < 8; ++r) o[r] = f2bf(d[r]);
      *(bf16x8*)xdst = o;
    }
  } else if (EPI == MMU_EPI_DGELU) {  // in = aux = gelu'(z) saved by the forward epilogue
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] *= in[r];
  } else if (EPI == MMU_EPI_ADD_RES) {
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] += in[r];  // residual
  }
  if (OUT_F32) {
    float4* C = (float4*)cdst;
    float4 lo = make_float4(v[0], v[1], v[2], v[3]), hi = make_float4(v[4], v[5], v[6], v[7]);
    if (p.accumulate) {
      const float4 c0 = C[0], c1 = C[1];
      lo.x += c0.x; lo.y += c0.y; lo.z += c0.z; lo.w += c0.w;
      hi.x += c1.x; hi.y += c1.y; hi.z += c1.z; hi.w += c1.w;
    }
    C[0] = lo;
    C[1] = hi;
  } else {
    bf16x8 o;
#pragma unroll
    for (int r = 0; r < 8; ++r) o[r] = f2bf(v[r]);
    *(bf16x8*)cdst = o;
  }
}

// the epilogue of a wave's 16*NJ-row x 64-col block acc[4][NJ] (n-subtile i, m-subtile j)
// through the wave-private LDS region ws (PJ * 4 KiB: passes of 16*PJ rows; the caller has
// passed a barrier that retires every staging read of it)
template <int EPI_, bool OUT_F32, int NJ, int PJ = 4>
static __device__ __forceinline__ void epilogue_block(const GemmParams& p, int64_t z, int slice, int64_t mw,
                                                      int64_t nw, f32x4 (&acc)[4][NJ], int l, char* ws) {
  // STORE_BNB / ADD_RES_BNB: the STORE / ADD_RES epilogue + the backward reduction of the
  // BatchNorm whose dY this C is, {sum g, sum g (x - mean)} with g = C (as stored) * ReLU mask
  constexpr bool BNB = EPI_ == MMU_EPI_STORE_BNB || EPI_ == MMU_EPI_ADD_RES_BNB;
  constexpr int EPI = EPI_ == MMU_EPI_STORE_BNB ? MMU_EPI_STORE : EPI_ == MMU_EPI_ADD_RES_BNB ? MMU_EPI_ADD_RES : EPI_;
  if (nw >= p.N) return;  // (N % 128 == 0: a 64-column wave block is all in or all out)
  const int q = l & 7, rr = l >> 3;
  const int64_t n = nw + 8 * q;
  // raw partial product -> this slice's f32 slab (splitk_reduce_kernel); split-K is EPI_STORE only
  const bool slab = EPI == MMU_EPI_STORE && p.splitk > 1;
  float* slab_base = slab ? p.ws + (z * p.splitk + slice) * p.M * p.N : nullptr;
  const float* bias = (!slab && p.bias && EPI != MMU_EPI_DGELU && EPI != MMU_EPI_ADD_RES)
                          ? p.bias + z * p.bias_bstride : nullptr;
  const bf16* res = p.residual ? (const bf16*)p.residual + z * p.res_bstride : nullptr;
  bf16* aux = p.aux ? (bf16*)p.aux + z * p.aux_bstride : nullptr;
  const float scale = p.drop_p > 0.f ? 1.0f / (1.0f - p.drop_p) : 1.0f;
  const uint32_t thr = (uint32_t)(p.drop_p * 65536.0f + 0.5f);
  float bv[8];
  {
    float4 b0 = make_float4(0.f, 0.f, 0.f, 0.f), b1 = b0;
    if (bias) { b0 = *(const float4*)(bias + n); b1 = *(const float4*)(bias + n + 4); }
    bv[0] = b0.x; bv[1] = b0.y; bv[2] = b0.z; bv[3] = b0.w; bv[4] = b1.x; bv[5] = b1.y; bv[6] = b1.z; bv[7] = b1.w;
  }
  // STORE_STATS: the BatchNorm statistics of the bf16 output, {sum, sum of squares} per column
  // and 64-row block into the float2 table p.colsum [ceil(M / 64)][N] (one pass = 64 rows)
  constexpr bool STATS = EPI == MMU_EPI_STORE_STATS;
  const bool want_cs = !STATS && !BNB && p.colsum != nullptr && !slab;
  constexpr bool TAB = STATS || BNB;  // a float2 [ceil(M / 64)][N] table row per pass
  float mu[8];
  const int64_t b_l = BNB ? (mw + rr) * p.N + n : 0;  // bn_x / bn_mask (>> 3) offset of the lane's row
  if (BNB) {
    const float4 m0 = *(const float4*)(p.bn_mean + n), m1 = *(const float4*)(p.bn_mean + n + 4);
    mu[0] = m0.x; mu[1] = m0.y; mu[2] = m0.z; mu[3] = m0.w; mu[4] = m1.x; mu[5] = m1.y; mu[6] = m1.z; mu[7] = m1.w;
  }
  float cs[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) cs[r] = 0.f;
  constexpr bool LOADS = EPI == MMU_EPI_BIAS_DROP_RES || EPI == MMU_EPI_DGELU || EPI == MMU_EPI_ADD_RES;
  // BIAS_DROP_RES into an f32 C reads an f32 residual: the encoder's f32 hidden stream
  constexpr bool RES32 = OUT_F32 && EPI == MMU_EPI_BIAS_DROP_RES;
  const bf16* src = EPI == MMU_EPI_DGELU ? (const bf16*)aux : res;
  const float* src32 = RES32 && p.residual ? (const float*)p.residual + z * p.res_bstride : nullptr;
  const int64_t lds_ = EPI == MMU_EPI_DGELU ? p.ldx : p.ldr;
  // the lane's row mw + rr: per-lane bases computed once; row mw + rr + d adds the wave-uniform
  // d * ld (scalar multiplies) -- a per-row m * ld is a 64-bit VALU multiply per pointer
  const int64_t m_l = mw + rr;
  const int64_t in_l = m_l * lds_ + n;
  const int64_t c_l = z * p.sC + m_l * p.ldc + n;
  constexpr bool XST = EPI == MMU_EPI_BIAS_GELU || EPI == MMU_EPI_BIAS_DROP_QGELU;  // aux stores
  constexpr bool DRP = EPI == MMU_EPI_BIAS_DROP_RES || EPI == MMU_EPI_BIAS_DROP_QGELU;
  const int64_t x_l = XST ? m_l * p.ldx + n : 0;
  const int64_t s_l = EPI == MMU_EPI_STORE ? m_l * p.N + n : 0;
  const int64_t q_l = DRP ? (z * p.M + m_l) * p.N + n : 0;
  const uint64_t seed = DRP && thr ? mmu_eff_seed(p.seed, p.seed_off) : 0;
  // residual = LN(residual rows): per-column gamma / beta here, per-row mean / rstd per pass
  const bool res_ln = RES32 && p.res_ln_w != nullptr && !slab;
  float lw[8], lb[8];
  if (RES32) {
    float4 w0 = make_float4(1.f, 1.f, 1.f, 1.f), w1 = w0, b0 = make_float4(0.f, 0.f, 0.f, 0.f), b1 = b0;
    if (res_ln) {
      const float* lw_ = p.res_ln_w + z * p.res_ln_bstride;
      const float* lb_ = p.res_ln_b + z * p.res_ln_bstride;
      w0 = *(const float4*)(lw_ + n); w1 = *(const float4*)(lw_ + n + 4);
      b0 = *(const float4*)(lb_ + n); b1 = *(const float4*)(lb_ + n + 4);
    }
    lw[0] = w0.x; lw[1] = w0.y; lw[2] = w0.z; lw[3] = w0.w; lw[4] = w1.x; lw[5] = w1.y; lw[6] = w1.z; lw[7] = w1.w;
    lb[0] = b0.x; lb[1] = b0.y; lb[2] = b0.z; lb[3] = b0.w; lb[4] = b1.x; lb[5] = b1.y; lb[6] = b1.z; lb[7] = b1.w;
  }
  static_assert(!TAB || PJ == 4, "STORE_STATS / *_BNB: one epilogue pass = one 64-row table block");
#pragma unroll
  for (int pass = 0; pass < NJ / PJ; ++pass) {
    float st1[8], st2[8];
    if (TAB) {
#pragma unroll
      for (int e = 0; e < 8; ++e) st1[e] = st2[e] = 0.f;
    }
    // the pass's residual / aux rows are requested up front: one memory latency per pass
    bf16x8 in[RES32 ? 1 : 2 * PJ];
    uint32_t rmk[EPI == MMU_EPI_ADD_RES ? 2 * PJ : 1];  // residual gate (p.res_mask), 0xFF = none
    float4 in32[RES32 ? 2 * PJ : 1][2];
    float rmu[RES32 ? 2 * PJ : 1], rrs[RES32 ? 2 * PJ : 1];
#pragma unroll
    for (int it = 0; it < 2 * PJ; ++it) {
      const int d = 16 * PJ * pass + 8 * it;  // row offset from the lane's first row (uniform)
      const int64_t m = m_l + d;
      if (RES32) {
        rmu[it] = 0.f;
        rrs[it] = 1.f;
        if (!slab && m < p.M) {
          const float* s32 = src32 + in_l + d * lds_;
          in32[it][0] = *(const float4*)s32;
          in32[it][1] = *(const float4*)(s32 + 4);
          if (res_ln) {
            rmu[it] = p.res_ln_mean[z * p.M + m];
            rrs[it] = p.res_ln_rstd[z * p.M + m];
          }
        } else {
          in32[it][0] = in32[it][1] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      } else if (LOADS && !slab && m < p.M) {
        in[it] = *(const bf16x8*)(src + in_l + d * lds_);
        if (EPI == MMU_EPI_ADD_RES) rmk[it] = p.res_mask ? (uint32_t)p.res_mask[(in_l + d * lds_) >> 3] : 0xFFu;
      } else {
        in[it] = bf16x8{};
        if (EPI == MMU_EPI_ADD_RES) rmk[it] = 0;
      }
    }
#pragma unroll
    for (int jj = 0; jj < PJ; ++jj) {
      const int r = 16 * jj + (l & 15);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ch = 4 * i + (l >> 4);
        *(f32x4*)(ws + r * 256 + ((ch ^ (r & 15)) << 4)) = acc[i][PJ * pass + jj];
      }
    }
    // the BatchNorm input rows + mask bytes (after the acc spill: those registers are free)
    bf16x8 bx[BNB ? 2 * PJ : 1];
    uint32_t bm[BNB ? 2 * PJ : 1];
    if (BNB) {
#pragma unroll
      for (int it = 0; it < 2 * PJ; ++it) {
        const int d = 16 * PJ * pass + 8 * it;
        if (!slab && m_l + d < p.M) {
          const int64_t o = b_l + (int64_t)d * p.N;
          bx[it] = *(const bf16x8*)(p.bn_x + o);
          bm[it] = p.bn_mask ? (uint32_t)p.bn_mask[o >> 3] : 0xFFu;
        } else {
          bx[it] = bf16x8{};
          bm[it] = 0;
        }
      }
    }
#pragma unroll
    for (int it = 0; it < 2 * PJ; ++it) {
      const int r = rr + 8 * it;
      const int d = 16 * PJ * pass + 8 * it;
      const int64_t m = m_l + d;
      const float4 lo = *(const float4*)(ws + r * 256 + (((2 * q) ^ (r & 15)) << 4));
      const float4 hi = *(const float4*)(ws + r * 256 + (((2 * q + 1) ^ (r & 15)) << 4));
      if (m >= p.M) continue;
      if (slab) {
        float4* sd = (float4*)(slab_base + s_l + d * p.N);
        sd[0] = lo;
        sd[1] = hi;
        continue;
      }
      float v[8] = {lo.x + bv[0], lo.y + bv[1], lo.z + bv[2], lo.w + bv[3],
                    hi.x + bv[4], hi.y + bv[5], hi.z + bv[6], hi.w + bv[7]};
      float inf[8];
      if (RES32) {
        inf[0] = in32[it][0].x; inf[1] = in32[it][0].y; inf[2] = in32[it][0].z; inf[3] = in32[it][0].w;
        inf[4] = in32[it][1].x; inf[5] = in32[it][1].y; inf[6] = in32[it][1].z; inf[7] = in32[it][1].w;
        if (res_ln) {  // the LayerNorm output, as mmu_layernorm_fwd_f32 computes it
#pragma unroll
          for (int e = 0; e < 8; ++e) inf[e] = fmaf((inf[e] - rmu[it]) * rrs[it], lw[e], lb[e]);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 8; ++r) inf[r] = LOADS ? bf2f(in[RES32 ? 0 : it][r]) : 0.f;
        if (EPI == MMU_EPI_ADD_RES) {
#pragma unroll
          for (int r = 0; r < 8; ++r) inf[r] = ((rmk[EPI == MMU_EPI_ADD_RES ? it : 0] >> r) & 1) ? inf[r] : 0.f;
        }
      }
      void* cdst = OUT_F32 ? (void*)((float*)p.C + c_l + d * p.ldc) : (void*)((bf16*)p.C + c_l + d * p.ldc);
      epi_oct<EPI, OUT_F32>(p, cdst, (XST && aux) ? aux + x_l + d * p.ldx : nullptr,
                            DRP ? (uint64_t)(q_l + d * p.N) >> 2 : 0, v, inf, scale, thr, seed);
      if (want_cs) {
#pragma unroll
        for (int e = 0; e < 8; ++e) cs[e] += v[e];
      }
      if (STATS) {  // over the values as stored (bf16), as the statistics pass would read them
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float y = bf2f(f2bf(v[e]));
          st1[e] += y;
          st2[e] = fmaf(y, y, st2[e]);
        }
      }
      if (BNB) {  // g over the stored (bf16) values, as the reduction pass would read them
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float g = ((bm[BNB ? it : 0] >> e) & 1) ? bf2f(f2bf(v[e])) : 0.f;
          st1[e] += g;
          st2[e] = fmaf(g, bf2f(bx[BNB ? it : 0][e]) - mu[e], st2[e]);
        }
      }
    }
    if (TAB) {  // lanes sharing q hold the same 8 columns: reduce over rr (8 rows each)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
#pragma unroll
        for (int o = 8; o < 64; o <<= 1) {
          st1[e] += __shfl_xor(st1[e], o, 64);
          st2[e] += __shfl_xor(st2[e], o, 64);
        }
      }
      const int64_t prow = (mw + 64 * pass) >> 6;
      if (rr == 0 && mw + 64 * pass < p.M) {
        float4* d = (float4*)(p.colsum + 2 * (prow * p.N + n));
#pragma unroll
        for (int e = 0; e < 4; ++e) d[e] = make_float4(st1[2 * e], st2[2 * e], st1[2 * e + 1], st2[2 * e + 1]);
      }
    }
  }
  if (want_cs) {  // lanes sharing q hold the same 8 columns: reduce over rr, one atomic per column
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float s = cs[e];
      s += __shfl_xor(s, 8, 64);
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      cs[e] = s;
    }
    if (rr == 0) {
      if (p.cs_part) {  // this wave block's partial row (16 NJ rows), folded by colsum_reduce_kernel
        if (mw >= p.M) return;  // (a block wholly past M has no table row)
        float4* d = (float4*)(p.cs_part + ((mw - p.cs_m0) / p.cs_rows) * p.N + n);
        d[0] = make_float4(cs[0], cs[1], cs[2], cs[3]);
        d[1] = make_float4(cs[4], cs[5], cs[6], cs[7]);
      } else {
        float* out = p.colsum + z * p.colsum_bstride + n;
#pragma unroll
        for (int e = 0; e < 8; ++e) atomicAdd(out + e, cs[e]);
      }
    }
  }
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
  int tm, tn, slice;
  int64_t z;
  block_tile(p, z, slice, tm, tn);
  const bf16* __restrict__ A = p.A + z * p.sA;
  const bf16* __restrict__ B = p.B + z * p.sB;
  const int64_t m0 = (int64_t)tm * SBM, n0 = (int64_t)tn * SBN;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint4 ra[4], rb[4];
  const int64_t kb = (int64_t)slice * p.kchunk;
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
  epilogue_block<EPI, OUT_F32, 4>(p, z, slice, m0 + 64 * wm, n0 + 64 * wn, acc, l, smem + w * 16384);
}

// ---------------------------------------------------------------- conv, 128x128 tiles
// The implicit-im2col forward / data-gradient product of a 3x3 or 1x1 (any stride) conv with
// FEW output channels (64 / 128: ResNet layer1 / layer2 conv2), on the small kernel's 128x128
// tiles, 4 waves, register staging: the A rows (output pixels) are gathered per tap while
// they are loaded (16 B per lane, padding and rows past M read as zero); B = the filter
// K-major [N][9 C].  C % 64 == 0 (a 64-deep k-step lies in one tap), N % 64 == 0 (a 64-col
// wave block is all in or all out: N = 64 runs half the tile's columns).  Split-K over
// (tap, channel) steps into f32 slabs as the 256x256 conv kernel does.
struct ConvRows4 {
  int base[4], h[4], w[4];  // img * H (-1: row past M), input h, w of tap (0, 0) of the thread's 4 rows
};
static __device__ __forceinline__ void conva_g_load(uint4 (&r)[4], const bf16* __restrict__ X, const GemmParams& p,
                                                    const ConvRows4& cr, int64_t k0, int t) {
  const int H = p.conv_h, W = p.conv_w, C = p.conv_c;
  const int tap = (int)(k0 / C), ci0 = (int)(k0 - (int64_t)tap * C);
  const int dh = tap / p.conv_ks, dw = tap - dh * p.conv_ks;
  const bool kin = k0 < p.K;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = t & 7;
    const int hh = cr.h[i] + dh, ww = cr.w[i] + dw;
    const bool ok = kin && cr.base[i] >= 0 && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
    r[i] = ok ? *(const uint4*)(X + ((int64_t)(cr.base[i] + hh) * W + ww) * C + ci0 + 8 * c) : make_uint4(0, 0, 0, 0);
  }
}

template <int EPI>
__global__ __launch_bounds__(256) void gemm_conva_small_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * S_STAGE];
  const int t = threadIdx.x, l = t & 63, w = t >> 6, wm = w >> 1, wn = w & 1;
  int tm, tn, slice;
  int64_t z;
  block_tile(p, z, slice, tm, tn);
  const int64_t m0 = (int64_t)tm * SBM, n0 = (int64_t)tn * SBN;
  ConvRows4 cr;
  {
    const int Wo = p.conv_wo, HWo = p.conv_ho * Wo;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t pix = m0 + (t >> 3) + 32 * i;  // g_load<true>'s row of piece i
      const int img = (int)(pix / HWo), rem = (int)(pix - (int64_t)img * HWo);
      const int ho = rem / Wo;
      cr.base[i] = pix < p.M ? img * p.conv_h : -1;
      cr.h[i] = ho * p.conv_s - p.conv_pad;
      cr.w[i] = (rem - ho * Wo) * p.conv_s - p.conv_pad;
    }
  }
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint4 ra[4], rb[4];
  const int64_t kb = (int64_t)slice * p.kchunk;
  const int64_t ke = kb + p.kchunk < p.K ? kb + p.kchunk : p.K;
  const int nk = (int)((ke - kb + BKT - 1) / BKT);
  conva_g_load(ra, p.A, p, cr, kb, t);
  g_load<true>(rb, p.B, p.ldb, n0, p.N, kb, ke, t);
  s_store<true>(smem, ra, t);
  s_store<true>(smem + SBM * BKT * 2, rb, t);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const char* sa = smem + (kt & 1) * S_STAGE;
    const char* sb = sa + SBM * BKT * 2;
    const bool more = kt + 1 < nk;
    if (more) {
      const int64_t k1 = kb + (int64_t)(kt + 1) * BKT;
      conva_g_load(ra, p.A, p, cr, k1, t);
      g_load<true>(rb, p.B, p.ldb, n0, p.N, k1, ke, t);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fb[4], fa[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fb[i] = s_frag<true, 256>(sb, 64 * wn + 16 * i, ks, l);
#pragma unroll
      for (int j = 0; j < 4; ++j) fa[j] = s_frag<true, 256>(sa, 64 * wm + 16 * j, ks, l);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      char* dst = smem + ((kt + 1) & 1) * S_STAGE;
      s_store<true>(dst, ra, t);
      s_store<true>(dst + SBM * BKT * 2, rb, t);
    }
    __syncthreads();
  }
  epilogue_block<EPI, false, 4>(p, z, slice, m0 + 64 * wm, n0 + 64 * wn, acc, l, smem + w * 16384);
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

// B tile (64 k-rows = output pixels x 256 n = one tap's channels ci0..ci0+255) of the conv
// weight gradient, gathered from the NHWC map (rsrc): pixel (img, h, w) reads the input
// pixel (h + dh, w + dw) of the block's tap; padding (and pixels >= K) read as zero through
// an offset past the buffer's range.  Same lane-linear LDS image as dma_tile<false>.
static __device__ __forceinline__ void dma_tile_convb(char* s, __amdgpu_buffer_rsrc_t rsrc, const GemmParams& p,
                                                      int dh, int dw, int64_t ci0, int64_t k0, int w, int l) {
  const int H = p.conv_h, W = p.conv_w, C = p.conv_c, s_ = p.conv_s;
  const int Wo = p.conv_wo, HW = p.conv_ho * Wo;
  const float rhw = 1.0f / (float)HW, rw = 1.0f / (float)Wo;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = w * 4 + i;
    const int kr = piece * 2 + (l >> 5), j = l & 31;
    const int b = (j >> 1) ^ sw_mn(kr);
    const int pix = (int)k0 + kr;
    // pix / HW and rem / W by float reciprocal + one correction (exact for pix < 2^24)
    int img = (int)((float)pix * rhw);
    int rem = pix - img * HW;
    if (rem < 0) { --img; rem += HW; } else if (rem >= HW) { ++img; rem -= HW; }
    int hh = (int)((float)rem * rw);
    int ww = rem - hh * Wo;
    if (ww < 0) { --hh; ww += Wo; } else if (ww >= Wo) { ++hh; ww -= Wo; }
    hh = hh * s_ + dh;
    ww = ww * s_ + dw;
    const bool ok = pix < p.K && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
    const uint32_t src = ok ? (uint32_t)(((((int64_t)img * H + hh) * W + ww) * C + ci0 + 16 * b + 8 * (j & 1)) * 2)
                            : 0x7FFFFFF0u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (MMU_LDS(void)*)(s + piece * 1024), 16, src, 0, 0, 0);
  }
}

// A tile (256 rows = output pixels x 64 k = channels ci0..ci0+63 of one tap) of a 3x3 or
// 1x1 convolution as an implicit GEMM, gathered from the NHWC map (rsrc): output pixel
// (img, ho, wo) reads input pixel (s ho - pad + dh, s wo - pad + dw) of tap (dh, dw);
// padding and rows >= M read as zero.
// Each lane's 4 rows are fixed for the block (pbase / ph / pw, from conv_rows_init); only
// the tap and channel offset move with k.  Same lane-linear LDS image as dma_tile<true>.
struct ConvRows {
  int base[4], h[4], w[4];  // img * H (-1: row past M), input h, w of tap (0, 0) of the lane's rows
};
static __device__ __forceinline__ ConvRows conv_rows_init(const GemmParams& p, int64_t m0, int w, int l) {
  ConvRows r;
  const int Wo = p.conv_wo, HWo = p.conv_ho * Wo;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (w * 4 + i) * 8 + (l >> 3);
    const int64_t pix = m0 + row;
    const int img = (int)(pix / HWo), rem = (int)(pix - (int64_t)img * HWo);
    const int ho = rem / Wo;
    r.base[i] = pix < p.M ? img * p.conv_h : -1;
    r.h[i] = ho * p.conv_s - p.conv_pad;
    r.w[i] = (rem - ho * Wo) * p.conv_s - p.conv_pad;
  }
  return r;
}
static __device__ __forceinline__ void dma_tile_conva(char* s, __amdgpu_buffer_rsrc_t rsrc, const GemmParams& p,
                                                      const ConvRows& r, int64_t k0, int w, int l) {
  const int H = p.conv_h, W = p.conv_w, C = p.conv_c;
  const int tap = (int)(k0 / C), ci0 = (int)(k0 - (int64_t)tap * C);
  const int dh = tap / p.conv_ks, dw = tap - dh * p.conv_ks;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = w * 4 + i;
    const int row = piece * 8 + (l >> 3), c = (l & 7) ^ (row & 7);
    const int hh = r.h[i] + dh, ww = r.w[i] + dw;
    const bool ok = r.base[i] >= 0 && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W && k0 < p.K;
    const uint32_t src = ok ? (uint32_t)((((int64_t)(r.base[i] + hh) * W + ww) * C + ci0 + 8 * c) * 2) : 0x7FFFFFF0u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (MMU_LDS(void)*)(s + piece * 1024), 16, src, 0, 0, 0);
  }
}

// GATHER = 1: the conv weight-gradient product (B gathered by dma_tile_convb);
// GATHER = 2: the conv forward / data-gradient product (A gathered by dma_tile_conva)
template <bool AK, bool BKM, int EPI, bool OUT_F32, int GATHER>
static __device__ __forceinline__ void gemm_big_body(const GemmParams& p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * B_STAGE];
  const int t = threadIdx.x, l = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w >> 2, wn = w & 3;
  int tm, tn, slice;
  int64_t z;
  GEMM_STAMP(0);
  block_tile(p, z, slice, tm, tn);
  const int64_t m0 = (int64_t)tm * BBM, n0 = (int64_t)tn * BBN;
  // operand byte ranges: rows (K-major) or k-rows (M/N-major) beyond the operand read as zero
  // (gathered conv operands: the whole input map, conv_in_bytes)
  const int64_t a_bytes = GATHER == 2 ? p.conv_in_bytes : (AK ? p.M * p.lda : p.K * p.lda) * 2;
  const int64_t b_bytes = GATHER == 1 ? p.conv_in_bytes : (BKM ? p.N * p.ldb : p.K * p.ldb) * 2;
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

  const int64_t kb = (int64_t)slice * p.kchunk;
  const int64_t ke = kb + p.kchunk < p.K ? kb + p.kchunk : p.K;
  const int nk = (int)((ke - kb + BKT - 1) / BKT);
  // conv gather: the block's tap (n0 / C: a 256-column tile lies in one tap) and channels
  const int tap = GATHER == 1 ? (int)(n0 / p.conv_c) : 0;
  const int dh = GATHER == 1 ? tap / p.conv_ks - p.conv_pad : 0;
  const int dw = GATHER == 1 ? tap % p.conv_ks - p.conv_pad : 0;
  const int64_t ci0 = GATHER == 1 ? n0 - (int64_t)tap * p.conv_c : 0;
  auto dma_b = [&](char* d, int64_t k) {
    if (GATHER == 1) dma_tile_convb(d, rb, p, dh, dw, ci0, k, w, l);
    else dma_tile<BKM>(d, rb, p.ldb, n0, k, w, l);
  };
  ConvRows crow;
  if (GATHER == 2) crow = conv_rows_init(p, m0, w, l);
  auto dma_a = [&](char* d, int64_t k) {
    if (GATHER == 2) dma_tile_conva(d, ra, p, crow, k, w, l);
    else dma_tile<AK>(d, ra, p.lda, m0, k, w, l);
  };
  dma_a(smem, kb);
  dma_b(smem + B_TILE, kb);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  GEMM_STAMP(1);
  for (int kt = 0; kt < nk; ++kt) {
    const char* sa = smem + (kt & 1) * B_STAGE;
    const char* sb = sa + B_TILE;
    if (kt + 1 < nk) {
      char* d = smem + ((kt + 1) & 1) * B_STAGE;
      const int64_t k1 = kb + (int64_t)(kt + 1) * BKT;
      dma_a(d, k1);
      dma_b(d + B_TILE, k1);
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
  GEMM_STAMP(2);
  epilogue_block<EPI, OUT_F32, 8>(p, z, slice, m0 + 128 * wm, n0 + 64 * wn, acc, l, smem + w * 16384);
#ifdef MMU_GEMM_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  GEMM_STAMP(3);
}

template <bool AK, bool BKM, int EPI, bool OUT_F32>
__global__ __launch_bounds__(512) void gemm_big_kernel(GemmParams p) {
  gemm_big_body<AK, BKM, EPI, OUT_F32, 0>(p);
}

// dW[co][tap][ci] (+)= sum over pixels dY[pixel][co] * X[pixel shifted by tap][ci]
__global__ __launch_bounds__(512) void gemm_convw_kernel(GemmParams p) {
  gemm_big_body<false, false, MMU_EPI_STORE, true, 1>(p);
}

// Y[pixel][n] = sum over (tap, c) of X[pixel shifted by tap][c] * Wk[n][tap * C + c] (bf16 out)
template <int EPI>
__global__ __launch_bounds__(512) void gemm_conva_kernel(GemmParams p) {
  gemm_big_body<true, true, EPI, false, 2>(p);
}

// ================================================================ wide: 256x384, LDS-DMA (round 6)
// The BERT products with both operands K-major and N % 384 == 0 (QKV 2304, W1 3072, Wo / W2 /
// the data gradients 768) on a 256 x 384 x 64 tile: 80 KiB per stage, the 2-stage ring fills all
// 160 KiB of LDS.  Per 64-deep K-step a CU moves 80 KiB into LDS for 1.5x the MACs of the 256^2
// tile's 64 KiB (76.8 vs 64 MAC per filled byte): the 256^2 K loop is bound by that fill (DESIGN
// §3 GEMM), not by the MFMAs.  8 waves as 4 (M) x 2 (N), 64 x 192 per wave: 48 accumulators of
// 16x16, A fragments held per k-half, B fragments streamed 4 at a time.  The epilogue is the
// shared one, three 64-column blocks per wave.
constexpr int WBM = 256, WBN = 384;
constexpr int W_TA = WBM * BKT * 2;   // 32 KiB
constexpr int W_TB = WBN * BKT * 2;   // 48 KiB
constexpr int W_STAGE = W_TA + W_TB;  // 80 KiB

// P x 1 KiB pieces per wave of a K-major [8 * 8 * P rows][64 k] tile (image as dma_tile<true>)
template <int P>
static __device__ __forceinline__ void dma_kmaj(char* s, __amdgpu_buffer_rsrc_t rsrc, int64_t ld, int64_t r0,
                                                int64_t k0, int w, int l) {
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const int piece = w * P + i;
    const int row = piece * 8 + (l >> 3), c = (l & 7) ^ (row & 7);
    const uint32_t src = (uint32_t)(((r0 + row) * ld + k0 + 8 * c) * 2);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (MMU_LDS(void)*)(s + piece * 1024), 16, src, 0, 0, 0);
  }
}

template <int EPI, bool OUT_F32>
__global__ __launch_bounds__(512) void gemm_wide_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * W_STAGE];
  const int t = threadIdx.x, l = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w >> 1, wn = w & 1;
  int tm, tn, slice;
  int64_t z;
  block_tile(p, z, slice, tm, tn);
  const int64_t m0 = (int64_t)tm * WBM, n0 = (int64_t)tn * WBN;
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.A + z * p.sA), 0, (int)(uint32_t)(p.M * p.lda * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.B + z * p.sB), 0, (int)(uint32_t)(p.N * p.ldb * 2), 0x00020000);
  f32x4 acc[3][4][4];  // [64-column block][n-subtile][m-subtile]
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[c][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (int)(p.K / BKT);  // (host: K % 64 == 0, no split-K)
  dma_kmaj<4>(smem, ra, p.lda, m0, 0, w, l);
  dma_kmaj<6>(smem + W_TA, rb, p.ldb, n0, 0, w, l);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const char* sa = smem + (kt & 1) * W_STAGE;
    const char* sb = sa + W_TA;
    if (kt + 1 < nk) {
      char* d = smem + ((kt + 1) & 1) * W_STAGE;
      const int64_t k1 = (int64_t)(kt + 1) * BKT;
      dma_kmaj<4>(d, ra, p.lda, m0, k1, w, l);
      dma_kmaj<6>(d + W_TA, rb, p.ldb, n0, k1, w, l);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fa[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) fa[j] = s_frag<true, 512>(sa, 64 * wm + 16 * j, ks, l);
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        bf16x8 fb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) fb[i] = s_frag<true, 512>(sb, 192 * wn + 64 * c + 16 * i, ks, l);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[c][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[c][i][j], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // 32-row epilogue passes (16 for the f32 hidden-stream residual): the other blocks' 128
  // accumulators stay live beside a pass's prefetched rows
  constexpr int PJ = (OUT_F32 && EPI == MMU_EPI_BIAS_DROP_RES) ? 1 : 2;
#pragma unroll
  for (int c = 0; c < 3; ++c)
    epilogue_block<EPI, OUT_F32, 4, PJ>(p, z, 0, m0 + 64 * wm, n0 + 192 * wn + 64 * c, acc[c], l, smem + w * 16384);
}

// The split-K slab sum of a conv whose epilogue also tabulates (STORE_STATS / STORE_BNB): one block
// per 64 rows x 64 columns sums the slabs in slice order into the bf16 C, as
// splitk_reduce_bf16_kernel does, and forms the block's table row from the stored values:
// {sum, sum of squares} of C (STATS) or {sum g, sum g (x - mean)} with g = C * ReLU mask (BNB) --
// the float2 [ceil(M / 64)][N] layout of the epilogues, in the same pass (round 6; was a
// reduce launch + a tabulating launch over C)
template <bool BNB>
__global__ __launch_bounds__(256) void splitk_reduce_tab_kernel(const GemmParams p) {
  // block = 64 rows x 64 columns (grid ceil(M/64) x N/64: enough blocks for the small split-K maps);
  // thread = one column octet (t & 7) x rows rs, rs + 32 (rs = t >> 3)
  __shared__ float red[4][2][8][8];
  const int t = threadIdx.x, oc = t & 7, rs = t >> 3, l = t & 63, w = t >> 6;
  const int64_t M = p.M, N = p.N, n = (int64_t)blockIdx.y * 64 + 8 * oc, r0 = (int64_t)blockIdx.x * 64;
  bf16* C = (bf16*)p.C;
  float a[8], b[8], mu[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = b[e] = mu[e] = 0.f;
  if (BNB) {
#pragma unroll
    for (int e = 0; e < 8; ++e) mu[e] = p.bn_mean[n + e];
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int64_t m = r0 + rs + 32 * h;
    if (m >= M) continue;
    const int64_t o = m * N + n;
    const float* sl = p.ws + o;
    float4 lo = *(const float4*)sl, hi = *(const float4*)(sl + 4);
    for (int k = 1; k < p.splitk; ++k) {
      const float4 c = *(const float4*)(sl + k * M * N), d = *(const float4*)(sl + k * M * N + 4);
      lo.x += c.x; lo.y += c.y; lo.z += c.z; lo.w += c.w;
      hi.x += d.x; hi.y += d.y; hi.z += d.z; hi.w += d.w;
    }
    const bf16x8 v = {f2bf(lo.x), f2bf(lo.y), f2bf(lo.z), f2bf(lo.w), f2bf(hi.x), f2bf(hi.y), f2bf(hi.z), f2bf(hi.w)};
    *(bf16x8*)(C + m * p.ldc + n) = v;
    if (BNB) {
      const bf16x8 x = *(const bf16x8*)(p.bn_x + o);
      const uint32_t mk = p.bn_mask ? (uint32_t)p.bn_mask[o >> 3] : 0xFFu;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float g = ((mk >> e) & 1) ? bf2f(v[e]) : 0.f;
        a[e] += g;
        b[e] = fmaf(g, bf2f(x[e]) - mu[e], b[e]);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float y = bf2f(v[e]);
        a[e] += y;
        b[e] = fmaf(y, y, b[e]);
      }
    }
  }
  // lanes sharing oc within a wave: xor 8, 16, 32; then the 4 waves through LDS
#pragma unroll
  for (int e = 0; e < 8; ++e) {
#pragma unroll
    for (int x = 8; x < 64; x <<= 1) {
      a[e] += __shfl_xor(a[e], x, 64);
      b[e] += __shfl_xor(b[e], x, 64);
    }
  }
  if (l < 8) {
#pragma unroll
    for (int e = 0; e < 8; ++e) { red[w][0][oc][e] = a[e]; red[w][1][oc][e] = b[e]; }
  }
  __syncthreads();
  if (t < 64) {  // thread (oc, e) = (t >> 3, t & 7) writes one column's pair
    const int c = t >> 3, e = t & 7;
    const float sa = red[0][0][c][e] + red[1][0][c][e] + red[2][0][c][e] + red[3][0][c][e];
    const float sb = red[0][1][c][e] + red[1][1][c][e] + red[2][1][c][e] + red[3][1][c][e];
    const int64_t col = (int64_t)blockIdx.y * 64 + 8 * c + e;
    *(float2*)(p.colsum + 2 * ((int64_t)blockIdx.x * N + col)) = make_float2(sa, sb);
  }
}

// sum of the split-K slabs of one (M x N) product into a bf16 C (slice order: deterministic)
__global__ __launch_bounds__(256) void splitk_reduce_bf16_kernel(const float* __restrict__ ws, bf16* __restrict__ C,
                                                                 int64_t M, int64_t N, int64_t ldc, int splitk) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;  // 8 consecutive elements per thread
  if (q * 8 >= M * N) return;
  const int64_t e = q * 8, m = e / N, n = e - m * N;
  const float* s = ws + e;
  float4 a = *(const float4*)s, b = *(const float4*)(s + 4);
  for (int k = 1; k < splitk; ++k) {
    const float4 c = *(const float4*)(s + k * M * N), d = *(const float4*)(s + k * M * N + 4);
    a.x += c.x; a.y += c.y; a.z += c.z; a.w += c.w;
    b.x += d.x; b.y += d.y; b.z += d.z; b.w += d.w;
  }
  const bf16x8 o = {f2bf(a.x), f2bf(a.y), f2bf(a.z), f2bf(a.w), f2bf(b.x), f2bf(b.y), f2bf(b.z), f2bf(b.w)};
  *(bf16x8*)(C + m * ldc + n) = o;
}

void conv3x3_implicit_launch(const GemmParams& p, bool small, hipStream_t s) {
  // p.kind == MMU_EPI_STORE_STATS: the epilogue also writes the output's BatchNorm statistics
  // table (p.colsum); split-K forms the output in the reduce kernel, which then tabulates it
  // (p.kind == MMU_EPI_STORE_BNB, a data gradient: the reduction table of the BatchNorm before it)
  const bool stats = p.kind == MMU_EPI_STORE_STATS && p.splitk == 1;
  const bool bnb = p.kind == MMU_EPI_STORE_BNB && p.splitk == 1;
  const dim3 grid(p.tiles_m * p.tiles_n, p.splitk, 1);
  if (small) {
    if (stats) hipLaunchKernelGGL(gemm_conva_small_kernel<MMU_EPI_STORE_STATS>, grid, dim3(256), 0, s, p);
    else if (bnb) hipLaunchKernelGGL(gemm_conva_small_kernel<MMU_EPI_STORE_BNB>, grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL(gemm_conva_small_kernel<MMU_EPI_STORE>, grid, dim3(256), 0, s, p);
  } else {
    if (stats) hipLaunchKernelGGL(gemm_conva_kernel<MMU_EPI_STORE_STATS>, grid, dim3(512), 0, s, p);
    else if (bnb) hipLaunchKernelGGL(gemm_conva_kernel<MMU_EPI_STORE_BNB>, grid, dim3(512), 0, s, p);
    else hipLaunchKernelGGL(gemm_conva_kernel<MMU_EPI_STORE>, grid, dim3(512), 0, s, p);
  }
  if (p.splitk > 1) {
    const dim3 tab((unsigned)((p.M + 63) / 64), (unsigned)(p.N / 64));  // (N % 64 == 0: conv_implicit)
    if (p.kind == MMU_EPI_STORE_STATS) {
      hipLaunchKernelGGL(splitk_reduce_tab_kernel<false>, tab, dim3(256), 0, s, p);
    } else if (p.kind == MMU_EPI_STORE_BNB) {
      hipLaunchKernelGGL(splitk_reduce_tab_kernel<true>, tab, dim3(256), 0, s, p);
    } else {
      const int64_t q = p.M * p.N / 8;
      hipLaunchKernelGGL(splitk_reduce_bf16_kernel, dim3((unsigned)((q + 255) / 256)), dim3(256), 0, s, p.ws,
                         (bf16*)p.C, p.M, p.N, p.ldc, p.splitk);
    }
  }
}

void conv3x3_wgrad_launch(const GemmParams& p, hipStream_t s) {
  hipLaunchKernelGGL(gemm_convw_kernel, dim3(p.tiles_m * p.tiles_n, p.splitk, 1), dim3(512), 0, s, p);
  if (p.splitk > 1) splitk_reduce_launch(p, 1, s);
}

// ---------------------------------------------------------------- launch
template <bool AK, bool BKM, int EPI, bool F32>
static void launch_t(const GemmParams& p, bool big, int batch, hipStream_t s) {
  dim3 grid(p.tiles_m * p.tiles_n, p.splitk, batch);
  if (big) {
    hipLaunchKernelGGL((gemm_big_kernel<AK, BKM, EPI, F32>), grid, dim3(512), 0, s, p);
  } else {
    hipLaunchKernelGGL((gemm_small_kernel<AK, BKM, EPI, F32>), grid, dim3(256), 0, s, p);
  }
}

template <int EPI, bool F32>
static void launch_e(const GemmParams& p, bool ak, bool bk, bool big, int batch, hipStream_t s) {
  if (ak && bk) launch_t<true, true, EPI, F32>(p, big, batch, s);
  else if (ak && !bk) launch_t<true, false, EPI, F32>(p, big, batch, s);
  else if (!ak && !bk) launch_t<false, false, EPI, F32>(p, big, batch, s);
  else launch_t<false, true, EPI, F32>(p, big, batch, s);
}

// ---------------------------------------------------------------- split tail rows (round 6)
// The last tile row of a product whose last round of tiles is nearly empty (M = 256 x 513 at
// batch 256: 1026 tiles of 256 x 384 on 256 CUs) runs as split-K partial products of the small
// tiling into f32 slabs; this kernel sums a 64 x 64 block's slabs in slice order straight into the
// MFMA accumulator layout -- acc[i][j], lane l = C[m0 + 16 j + (l & 15)][n0 + 16 i + 4 (l >> 4) + 0..3]
// -- and runs the shared epilogue on it, so every epilogue kind finishes the tail rows exactly as
// the tile kernels do (only the f32 summation order of the K slices differs).
template <int EPI, bool OUT_F32>
__global__ __launch_bounds__(64) void splitk_epilogue_kernel(GemmParams p, const float* __restrict__ slabs,
                                                             int64_t m_base, int64_t rows, int splitk) {
  __shared__ __attribute__((aligned(16))) char ws[16384];
  const int l = threadIdx.x;
  const int64_t mr = (int64_t)blockIdx.x * 64, n0 = (int64_t)blockIdx.y * 64;
  const int64_t slab = rows * p.N;
  f32x4 acc[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t r = mr + 16 * j + (l & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
      if (r < rows) {
        const float* s = slabs + r * p.N + n0 + 16 * i + 4 * (l >> 4);
        a = *(const f32x4*)s;
        for (int k = 1; k < splitk; ++k) a += *(const f32x4*)(s + k * slab);
      }
      acc[i][j] = a;
    }
  }
  epilogue_block<EPI, OUT_F32, 4>(p, 0, 0, m_base + mr, n0, acc, l, ws);
}

bool splitk_epilogue_launch(const GemmParams& p, bool f32out, const float* slabs, int64_t m_base, int64_t rows,
                            int splitk, hipStream_t s) {
  const dim3 grid((unsigned)((rows + 63) / 64), (unsigned)(p.N / 64)), blk(64);
  switch (p.kind) {
    case MMU_EPI_STORE:
      if (f32out) hipLaunchKernelGGL((splitk_epilogue_kernel<MMU_EPI_STORE, true>), grid, blk, 0, s, p, slabs, m_base, rows, splitk);
      else hipLaunchKernelGGL((splitk_epilogue_kernel<MMU_EPI_STORE, false>), grid, blk, 0, s, p, slabs, m_base, rows, splitk);
      return true;
    case MMU_EPI_BIAS_GELU:
      hipLaunchKernelGGL((splitk_epilogue_kernel<MMU_EPI_BIAS_GELU, false>), grid, blk, 0, s, p, slabs, m_base, rows, splitk);
      return true;
    case MMU_EPI_BIAS_DROP_RES:
      if (f32out) hipLaunchKernelGGL((splitk_epilogue_kernel<MMU_EPI_BIAS_DROP_RES, true>), grid, blk, 0, s, p, slabs, m_base, rows, splitk);
      else hipLaunchKernelGGL((splitk_epilogue_kernel<MMU_EPI_BIAS_DROP_RES, false>), grid, blk, 0, s, p, slabs, m_base, rows, splitk);
      return true;
    case MMU_EPI_DGELU:
      hipLaunchKernelGGL((splitk_epilogue_kernel<MMU_EPI_DGELU, false>), grid, blk, 0, s, p, slabs, m_base, rows, splitk);
      return true;
    case MMU_EPI_ADD_RES:
      hipLaunchKernelGGL((splitk_epilogue_kernel<MMU_EPI_ADD_RES, false>), grid, blk, 0, s, p, slabs, m_base, rows, splitk);
      return true;
    default: return false;
  }
}

// the 256 x 384 tiling (host: both operands K-major, N % 384 == 0, no split-K; kinds below)
bool gemm_wide_launch(const GemmParams& p, bool f32out, int batch, hipStream_t s) {
  const dim3 grid(p.tiles_m * p.tiles_n, 1, batch), blk(512);
  switch (p.kind) {
    case MMU_EPI_STORE:
      if (f32out) hipLaunchKernelGGL((gemm_wide_kernel<MMU_EPI_STORE, true>), grid, blk, 0, s, p);
      else hipLaunchKernelGGL((gemm_wide_kernel<MMU_EPI_STORE, false>), grid, blk, 0, s, p);
      return true;
    case MMU_EPI_BIAS_GELU: hipLaunchKernelGGL((gemm_wide_kernel<MMU_EPI_BIAS_GELU, false>), grid, blk, 0, s, p); return true;
    case MMU_EPI_BIAS_DROP_RES:
      if (f32out) hipLaunchKernelGGL((gemm_wide_kernel<MMU_EPI_BIAS_DROP_RES, true>), grid, blk, 0, s, p);
      else hipLaunchKernelGGL((gemm_wide_kernel<MMU_EPI_BIAS_DROP_RES, false>), grid, blk, 0, s, p);
      return true;
    case MMU_EPI_DGELU: hipLaunchKernelGGL((gemm_wide_kernel<MMU_EPI_DGELU, false>), grid, blk, 0, s, p); return true;
    case MMU_EPI_ADD_RES: hipLaunchKernelGGL((gemm_wide_kernel<MMU_EPI_ADD_RES, false>), grid, blk, 0, s, p); return true;
    default: return false;
  }
}

void gemm_launch(const GemmParams& p, bool ak, bool bk, bool f32out, bool big, int batch, hipStream_t s) {
  switch (p.kind) {
    case MMU_EPI_STORE:
      if (f32out) launch_e<MMU_EPI_STORE, true>(p, ak, bk, big, batch, s);
      else launch_e<MMU_EPI_STORE, false>(p, ak, bk, big, batch, s);
      break;
    case MMU_EPI_BIAS_GELU: launch_e<MMU_EPI_BIAS_GELU, false>(p, ak, bk, big, batch, s); break;
    case MMU_EPI_BIAS_DROP_RES:
      if (f32out) launch_e<MMU_EPI_BIAS_DROP_RES, true>(p, ak, bk, big, batch, s);
      else launch_e<MMU_EPI_BIAS_DROP_RES, false>(p, ak, bk, big, batch, s);
      break;
    case MMU_EPI_DGELU: launch_e<MMU_EPI_DGELU, false>(p, ak, bk, big, batch, s); break;
    case MMU_EPI_ADD_RES: launch_e<MMU_EPI_ADD_RES, false>(p, ak, bk, big, batch, s); break;
    case MMU_EPI_BIAS_DROP_QGELU: launch_e<MMU_EPI_BIAS_DROP_QGELU, false>(p, ak, bk, big, batch, s); break;
    case MMU_EPI_STORE_STATS:  // (the 1x1 conv forward: X rows . W^T, both K-major)
      if (big) launch_t<true, true, MMU_EPI_STORE_STATS, false>(p, true, batch, s);
      else launch_t<true, true, MMU_EPI_STORE_STATS, false>(p, false, batch, s);
      break;
    case MMU_EPI_STORE_BNB:  // (the 1x1 conv data gradient: dY rows . W, B N-major)
      launch_t<true, false, MMU_EPI_STORE_BNB, false>(p, big, batch, s);
      break;
    case MMU_EPI_ADD_RES_BNB:
      launch_t<true, false, MMU_EPI_ADD_RES_BNB, false>(p, big, batch, s);
      break;
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
  // 4 slabs' loads in flight per thread, added in slice order
  int k = 1;
  for (; k + 4 <= splitk; k += 4) {
    float4 b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) b[u] = *(const float4*)(s + (k + u) * M * N);
#pragma unroll
    for (int u = 0; u < 4; ++u) { a.x += b[u].x; a.y += b[u].y; a.z += b[u].z; a.w += b[u].w; }
  }
  for (; k < splitk; ++k) {
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
constexpr int COLSUM_ROWS = 16;  // 16 rows per thread: enough blocks to fill the chip for 1-2 K partial rows
__global__ __launch_bounds__(256) void colsum_reduce_kernel(const float* __restrict__ part, int64_t parts, int64_t N,
                                                            float* __restrict__ out) {
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const int64_t r0 = (int64_t)blockIdx.y * COLSUM_ROWS;
  const int64_t r1 = r0 + COLSUM_ROWS < parts ? r0 + COLSUM_ROWS : parts;
  float s = 0.f;
#pragma unroll 8
  for (int64_t r = r0; r < r1; ++r) s += part[r * N + n];
  atomicAdd(out + n, s);
}

void colsum_reduce_launch(const float* part, int64_t parts, int64_t N, float* out, int acc, hipStream_t s) {
  if (!acc) (void)hipMemsetAsync(out, 0, sizeof(float) * N, s);
  hipLaunchKernelGGL(colsum_reduce_kernel,
                     dim3((unsigned)((N + 255) / 256), (unsigned)((parts + COLSUM_ROWS - 1) / COLSUM_ROWS)),
                     dim3(256), 0, s, part, parts, N, out);
}

// up to COLSUM_MULTI independent reductions of one width N in one launch (grid.z = the job): the
// bias / LayerNorm-parameter gradients a BERT layer's backward forms together (round 6: 9 launches
// per layer -> 3)
__global__ __launch_bounds__(256) void colsum_reduce_multi_kernel(const ColsumJobs jobs, int64_t N) {
  const int z = blockIdx.z;
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t parts = jobs.parts[z];
  const int64_t r0 = (int64_t)blockIdx.y * COLSUM_ROWS;
  if (n >= N || r0 >= parts) return;
  const int64_t r1 = r0 + COLSUM_ROWS < parts ? r0 + COLSUM_ROWS : parts;
  const float* part = jobs.part[z];
  float s = 0.f;
#pragma unroll 8
  for (int64_t r = r0; r < r1; ++r) s += part[r * N + n];
  atomicAdd(jobs.out[z] + n, s);
}

void colsum_reduce_multi_launch(const ColsumJobs& jobs, int n, int64_t N, int acc, hipStream_t s) {
  int64_t most = 0;
  for (int z = 0; z < n; ++z) {
    if (!acc) (void)hipMemsetAsync(jobs.out[z], 0, sizeof(float) * N, s);
    most = jobs.parts[z] > most ? jobs.parts[z] : most;
  }
  hipLaunchKernelGGL(colsum_reduce_multi_kernel,
                     dim3((unsigned)((N + 255) / 256), (unsigned)((most + COLSUM_ROWS - 1) / COLSUM_ROWS), (unsigned)n),
                     dim3(256), 0, s, jobs, N);
}

// column sums of a bf16 [M, N] matrix: block = 64 octets of columns x rpb rows (4 waves, 4
// loads in flight each).  With a scratch table the blocks write per-block partial rows
// (no atomics) that colsum_reduce_kernel folds, so the row blocks can be short enough to put
// ~1 K blocks on the chip; without one, rpb = 1024 rows and one float atomic per column per
// block (short blocks would pile hundreds of same-address atomics into the L2 queue).
constexpr int COLSUM_BF16_ROWS = 1024;
constexpr int COLSUM_BF16_MIN_ROWS = 64;
__global__ __launch_bounds__(256) void colsum_bf16_kernel(const bf16* __restrict__ X, int64_t M, int64_t N,
                                                          int64_t ld, int64_t rpb, float* __restrict__ part,
                                                          float* __restrict__ out) {
  const int64_t r0 = (int64_t)blockIdx.y * rpb;
  const int64_t r1 = r0 + rpb < M ? r0 + rpb : M;
  const int64_t c = ((int64_t)blockIdx.x * 64 + (threadIdx.x & 63)) * 8;
  const int wv = threadIdx.x >> 6;
  __shared__ float red[4][64 * 8];
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c < N) {
    int64_t r = r0 + wv;
    for (; r + 12 < r1; r += 16) {
      bf16x8 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *(const bf16x8*)(X + (r + 4 * u) * ld + c);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int e = 0; e < 8; ++e) s[e] += bf2f(v[u][e]);
    }
    for (; r < r1; r += 4) {
      const bf16x8 v = *(const bf16x8*)(X + r * ld + c);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += bf2f(v[e]);
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[wv][(threadIdx.x & 63) * 8 + e] = s[e];
  __syncthreads();
  if (wv == 0 && c < N) {
    float t[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int q = (threadIdx.x & 63) * 8 + e;
      t[e] = red[0][q] + red[1][q] + red[2][q] + red[3][q];
    }
    if (part) {
      float4* d = (float4*)(part + (int64_t)blockIdx.y * N + c);
      d[0] = make_float4(t[0], t[1], t[2], t[3]);
      d[1] = make_float4(t[4], t[5], t[6], t[7]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) atomicAdd(out + c + e, t[e]);
    }
  }
}

void colsum_bf16_launch(const bf16* X, int64_t M, int64_t N, int64_t ld, float* part, float* out, int acc,
                        hipStream_t s) {
  const int64_t gx = (N / 8 + 63) / 64;
  int64_t rpb = COLSUM_BF16_ROWS;
  if (part) {  // ~1 K blocks: rows per block a multiple of 16 in [64, 1024]
    rpb = (M * gx + 1023) / 1024;
    rpb = (rpb + 15) / 16 * 16;
    rpb = rpb < COLSUM_BF16_MIN_ROWS ? COLSUM_BF16_MIN_ROWS : rpb > COLSUM_BF16_ROWS ? COLSUM_BF16_ROWS : rpb;
  }
  const int64_t gy = (M + rpb - 1) / rpb;
  if (part && gy > 1) {
    hipLaunchKernelGGL(colsum_bf16_kernel, dim3((unsigned)gx, (unsigned)gy), dim3(256), 0, s, X, M, N, ld, rpb, part,
                       (float*)nullptr);
    colsum_reduce_launch(part, gy, N, out, acc, s);
    return;
  }
  if (!acc) (void)hipMemsetAsync(out, 0, sizeof(float) * N, s);
  hipLaunchKernelGGL(colsum_bf16_kernel, dim3((unsigned)gx, (unsigned)gy), dim3(256), 0, s, X, M, N, ld, rpb,
                     (float*)nullptr, out);
}

// ------------------------------------------------------------------ batched transpose
// one 64 x 64 tile per workgroup through LDS (row pitch 65 elements: conflict-free column
// reads), 16-B global reads and 8-B writes; blockIdx.z = job, tiles outside a job's shape exit.
// Job = {src, dst, rows, cols, src row pitch, dst row pitch} (pitches 0: dense)
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const int64_t* __restrict__ jobs) {
  const int64_t* j = jobs + 6 * blockIdx.z;
  const bf16* __restrict__ src = (const bf16*)j[0];
  bf16* __restrict__ dst = (bf16*)j[1];
  const int64_t rows = j[2], cols = j[3];
  const int64_t sld = j[4] ? j[4] : cols, dld = j[5] ? j[5] : rows;
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  if (r0 >= rows || c0 >= cols) return;
  __shared__ bf16 tile[64][65];
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // 64 rows x 8 octets = 512 loads of 16 B
    const int idx = t + 256 * i, r = idx >> 3, c = (idx & 7) * 8;
    const int64_t gr = r0 + r, gc = c0 + c;
    if (gr < rows && gc + 8 <= cols) {
      const bf16x8 v = *(const bf16x8*)(src + gr * sld + gc);
#pragma unroll
      for (int e = 0; e < 8; ++e) tile[r][c + e] = v[e];
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) tile[r][c + e] = (gr < rows && gc + e < cols) ? src[gr * sld + gc + e] : bf16(0.f);
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // 64 dst rows (= src cols) x 16 quads of 8 B
    const int idx = t + 256 * i, c = idx >> 4, r = (idx & 15) * 4;
    const int64_t gc = c0 + c, gr = r0 + r;
    if (gc >= cols) continue;
    if (gr + 4 <= rows) {
      bf16x4 v = {tile[r][c], tile[r + 1][c], tile[r + 2][c], tile[r + 3][c]};
      *(bf16x4*)(dst + gc * dld + gr) = v;
    } else {
      for (int e = 0; e < 4; ++e)
        if (gr + e < rows) dst[gc * dld + gr + e] = tile[r + e][c];
    }
  }
}

void transpose_bf16_batched_launch(const int64_t* jobs, int n_jobs, int64_t max_rows, int64_t max_cols,
                                   hipStream_t s) {
  hipLaunchKernelGGL(transpose_bf16_kernel,
                     dim3((unsigned)((max_cols + 63) / 64), (unsigned)((max_rows + 63) / 64), (unsigned)n_jobs),
                     dim3(256), 0, s, jobs);
}

}  // namespace mmu

#ifdef MMU_GEMM_STAMPS
extern "C" int mmu_debug_gemm_stamps(uint64_t* host, int blocks) {
  if (blocks > (1 << 16)) blocks = 1 << 16;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(mmu::g_gemm_stamps), sizeof(uint64_t) * 4 * blocks, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
#endif
