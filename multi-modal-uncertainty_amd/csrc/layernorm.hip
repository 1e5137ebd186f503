// Row LayerNorm over the 768-wide hidden state (gfx950), forward and backward.
//
// BertLayerNorm of BertSelfOutput / BertOutput in the encoder (src/mmbt.py:124-126):
// y = (x - mean) / sqrt(var + eps) * w + b, biased variance, eps 1e-12.
// One wave per row, 4 contiguous bf16 per lane per 256-column slab (8-B accesses).
// The backward also undoes the dropout of the producing GEMM epilogue
// (MMU_EPI_BIAS_DROP_RES: same (seed, m*H+n) quad stream) and emits per-block
// partial column sums for dgamma / dbeta / dbias, so the LN-affine and the Linear
// bias gradients cost no extra pass over the activations.
#include <cstdlib>
#include "mmu_common.h"
#include "mmu_internal.h"

namespace mmu {

constexpr int LN_FWD_ROWS = 16;  // rows per block: 4 waves x 4 rows, two in flight per wave

// rows are grouped: row r uses the affine params of group r / group_rows (stride pstride);
// one group == the plain LN, K groups == K ensemble members in one launch
template <int NV>  // H = 256 * NV
__global__ __launch_bounds__(256) void ln_fwd_kernel(const bf16* __restrict__ X, const float* __restrict__ w,
                                                     const float* __restrict__ b, bf16* __restrict__ Y,
                                                     float* __restrict__ mean, float* __restrict__ rstd,
                                                     int64_t rows, float eps, int64_t group_rows, int64_t pstride) {
  constexpr int H = 256 * NV;
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  auto load = [&](int64_t row, bf16x4 (&x)[NV]) {
#pragma unroll
    for (int i = 0; i < NV; ++i) x[i] = *(const bf16x4*)(X + row * H + 256 * i + 4 * l);
  };
  auto process = [&](int64_t row, const bf16x4 (&x)[NV]) {
    float v[NV][4];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[i][e] = bf2f(x[i][e]); s += v[i][e]; }
    const float mu = wave_sum(s) / H;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) { float d = v[i][e] - mu; q += d * d; }
    const float rs = rsqrtf(wave_sum(q) / H + eps);
    const float* wr = w + (row / group_rows) * pstride;
    const float* br = b + (row / group_rows) * pstride;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = 256 * i + 4 * l;
      float4 ww = *(const float4*)(wr + c), bb = *(const float4*)(br + c);
      bf16x4 y = {f2bf((v[i][0] - mu) * rs * ww.x + bb.x), f2bf((v[i][1] - mu) * rs * ww.y + bb.y),
                  f2bf((v[i][2] - mu) * rs * ww.z + bb.z), f2bf((v[i][3] - mu) * rs * ww.w + bb.w)};
      *(bf16x4*)(Y + row * H + c) = y;
    }
    if (l == 0 && mean) { mean[row] = mu; rstd[row] = rs; }
  };
  const int64_t r0 = (int64_t)blockIdx.x * LN_FWD_ROWS;
  const int64_t rend = r0 + LN_FWD_ROWS < rows ? r0 + LN_FWD_ROWS : rows;
  for (int64_t row = r0 + wv; row < rend; row += 8) {
    bf16x4 xa[NV], xb[NV];
    const bool two = row + 4 < rend;
    load(row, xa);
    if (two) load(row + 4, xb);
    process(row, xa);
    if (two) process(row + 4, xb);
  }
}

// forward, 16-B accesses: a wave owns a PAIR of rows (2 x 32 NV chunks of 8 bf16 = NV slabs
// of 64 lanes: chunk q = 64 i + l of slab i is row q / (32 NV), columns 8 (q % (32 NV)) ..+7),
// two pairs in flight per wave; the rows' sums are two masked wave reductions.  Needs both
// rows of a pair in one parameter group (group_rows even, or one group).  (The same layout
// for the backward measured slower than its row-per-wave kernel: 8 f32 column accumulators
// per chunk x 3 quantities hold it at 2 waves / SIMD.)
constexpr int LN2_PAIRS = 8;  // pairs per block: 4 waves x 2
template <int NV>  // H = 256 * NV
__global__ __launch_bounds__(256) void ln_fwd2_kernel(const bf16* __restrict__ X, const float* __restrict__ w,
                                                      const float* __restrict__ b, bf16* __restrict__ Y,
                                                      float* __restrict__ mean, float* __restrict__ rstd,
                                                      int64_t rows, float eps, int64_t group_rows, int64_t pstride) {
  constexpr int H = 256 * NV, CPR = 32 * NV;  // chunks per row
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int cc[NV];
  bool hb[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int q = 64 * i + l;
    hb[i] = q >= CPR;
    cc[i] = 8 * (hb[i] ? q - CPR : q);
  }
  const int64_t p0 = (int64_t)blockIdx.x * LN2_PAIRS;
  const int64_t np = (rows + 1) / 2;
  const int64_t pend = p0 + LN2_PAIRS < np ? p0 + LN2_PAIRS : np;
  for (int64_t pr = p0 + wv; pr < pend; pr += 8) {
    bf16x8 xa[NV], xb[NV];
    const bool two = pr + 4 < pend;
    auto load = [&](int64_t pp, bf16x8 (&x)[NV]) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int64_t row = 2 * pp + (hb[i] ? 1 : 0);
        x[i] = row < rows ? *(const bf16x8*)(X + row * H + cc[i]) : bf16x8{};
      }
    };
    auto process = [&](int64_t pp, const bf16x8 (&x)[NV]) {
      float v[NV][8];
      float sa = 0.f, sb = 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) { v[i][e] = bf2f(x[i][e]); s += v[i][e]; }
        if (hb[i]) sb += s; else sa += s;
      }
      const float mua = wave_sum(sa) / H, mub = wave_sum(sb) / H;
      float qa = 0.f, qb = 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const float mu = hb[i] ? mub : mua;
        float q = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) { const float d = v[i][e] - mu; q += d * d; }
        if (hb[i]) qb += q; else qa += q;
      }
      const float rsa = rsqrtf(wave_sum(qa) / H + eps), rsb = rsqrtf(wave_sum(qb) / H + eps);
      const int64_t ra = 2 * pp;
      const float* wr = w + (ra / group_rows) * pstride;
      const float* br = b + (ra / group_rows) * pstride;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int64_t row = ra + (hb[i] ? 1 : 0);
        if (row >= rows) continue;
        const float mu = hb[i] ? mub : mua, rs = hb[i] ? rsb : rsa;
        const float4 w0 = *(const float4*)(wr + cc[i]), w1 = *(const float4*)(wr + cc[i] + 4);
        const float4 b0 = *(const float4*)(br + cc[i]), b1 = *(const float4*)(br + cc[i] + 4);
        const float ww[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
        const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
        bf16x8 y;
#pragma unroll
        for (int e = 0; e < 8; ++e) y[e] = f2bf((v[i][e] - mu) * rs * ww[e] + bb[e]);
        *(bf16x8*)(Y + row * H + cc[i]) = y;
      }
      if (mean && l == 0) {
        mean[ra] = mua;
        rstd[ra] = rsa;
        if (ra + 1 < rows) { mean[ra + 1] = mub; rstd[ra + 1] = rsb; }
      }
    };
    load(pr, xa);
    if (two) load(pr + 4, xb);
    process(pr, xa);
    if (two) process(pr + 4, xb);
  }
}

// forward of the f32 hidden stream (the BERT encoder's LN input S = residual + branch, kept
// in f32 so that the 24 post-LN residual adds of the 12 layers are not rounded to bf16):
// one wave per row, 4 consecutive f32 per lane per 256-column slab (16-B loads), writes the
// bf16 row (the next GEMM's operand) and, when Y32 is given, the f32 row (the next residual)
template <int NV>  // H = 256 * NV
__global__ __launch_bounds__(256) void ln_fwd32_kernel(const float* __restrict__ X, const float* __restrict__ w,
                                                       const float* __restrict__ b, bf16* __restrict__ Y,
                                                       float* __restrict__ Y32, float* __restrict__ mean,
                                                       float* __restrict__ rstd, int64_t rows, float eps,
                                                       int64_t group_rows, int64_t pstride) {
  constexpr int H = 256 * NV;
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  auto load = [&](int64_t row, float4 (&x)[NV]) {
#pragma unroll
    for (int i = 0; i < NV; ++i) x[i] = *(const float4*)(X + row * H + 256 * i + 4 * l);
  };
  auto process = [&](int64_t row, const float4 (&x)[NV]) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) s += (x[i].x + x[i].y) + (x[i].z + x[i].w);
    const float mu = wave_sum(s) / H;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const float d0 = x[i].x - mu, d1 = x[i].y - mu, d2 = x[i].z - mu, d3 = x[i].w - mu;
      q += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
    }
    const float rs = rsqrtf(wave_sum(q) / H + eps);
    const float* wr = w + (row / group_rows) * pstride;
    const float* br = b + (row / group_rows) * pstride;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = 256 * i + 4 * l;
      const float4 ww = *(const float4*)(wr + c), bb = *(const float4*)(br + c);
      const float4 y = make_float4((x[i].x - mu) * rs * ww.x + bb.x, (x[i].y - mu) * rs * ww.y + bb.y,
                                   (x[i].z - mu) * rs * ww.z + bb.z, (x[i].w - mu) * rs * ww.w + bb.w);
      *(bf16x4*)(Y + row * H + c) = bf16x4{f2bf(y.x), f2bf(y.y), f2bf(y.z), f2bf(y.w)};
      if (Y32) *(float4*)(Y32 + row * H + c) = y;
    }
    if (l == 0 && mean) { mean[row] = mu; rstd[row] = rs; }
  };
  const int64_t r0 = (int64_t)blockIdx.x * LN_FWD_ROWS;
  const int64_t rend = r0 + LN_FWD_ROWS < rows ? r0 + LN_FWD_ROWS : rows;
  for (int64_t row = r0 + wv; row < rend; row += 8) {
    float4 xa[NV], xb[NV];
    const bool two = row + 4 < rend;
    load(row, xa);
    if (two) load(row + 4, xb);
    process(row, xa);
    if (two) process(row + 4, xb);
  }
}

static __device__ __forceinline__ void ld4f(const bf16* p, float (&o)[4]) {
  const bf16x4 v = *(const bf16x4*)p;
  o[0] = bf2f(v[0]); o[1] = bf2f(v[1]); o[2] = bf2f(v[2]); o[3] = bf2f(v[3]);
}
static __device__ __forceinline__ void ld4f(const float* p, float (&o)[4]) {
  const float4 v = *(const float4*)p;
  o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}

// block = 4 waves; each wave walks rows_per_part/4 rows, TWO rows per step (both rows' loads
// in flight before either reduction: the loop is latency-bound on one row at a time);
// partial column sums reduced through one reused LDS buffer (16 KiB: occupancy)
template <int NV, typename XT>  // H = 256 * NV; XT: the LN input's type (bf16, or f32 for the hidden stream)
__global__ __launch_bounds__(256) void ln_bwd_kernel(const bf16* __restrict__ dY, const XT* __restrict__ X,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const float* __restrict__ w, bf16* __restrict__ dX,
                                                     bf16* __restrict__ dXd, const bf16* __restrict__ dR,
                                                     float drop_p, uint64_t seed, const uint64_t* seed_off,
                                                     float* __restrict__ pdw, float* __restrict__ pdb,
                                                     float* __restrict__ pdbias, int64_t rows, int rpp) {
  constexpr int H = 256 * NV, nv = NV;
  __shared__ float red[4][H];
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float scale = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
  const uint32_t thr = (uint32_t)(drop_p * 65536.0f + 0.5f);
  float aw[NV][4], ab[NV][4], ac[NV][4], ww[NV][4];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      aw[i][e] = ab[i][e] = ac[i][e] = 0.f;
      ww[i][e] = w[256 * i + 4 * l + e];
    }
  struct Row {
    bf16x4 a[NV];
    float x[NV][4];
    float mu, rs;
  };
  auto load = [&](int64_t row, Row& R) {
    R.mu = mean[row];
    R.rs = rstd[row];
#pragma unroll
    for (int i = 0; i < NV; ++i)
      if (i < nv) {
        R.a[i] = *(const bf16x4*)(dY + row * H + 256 * i + 4 * l);
        ld4f(X + row * H + 256 * i + 4 * l, R.x[i]);
      }
  };
  auto process = [&](int64_t row, const Row& R) {
    float g[NV][4], xh[NV][4], dy[NV][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
      if (i < nv) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          dy[i][e] = bf2f(R.a[i][e]);
          xh[i][e] = (R.x[i][e] - R.mu) * R.rs;
          g[i][e] = dy[i][e] * ww[i][e];
          s1 += g[i][e];
          s2 += g[i][e] * xh[i][e];
        }
      }
    s1 = wave_sum(s1) / H;
    s2 = wave_sum(s2) / H;
#pragma unroll
    for (int i = 0; i < NV; ++i)
      if (i < nv) {
        const int c = 256 * i + 4 * l;
        float dx[4];
        bf16x4 rr{};
        if (dR) rr = *(const bf16x4*)(dR + row * H + c);  // pre-LN block: + the residual's gradient
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          dx[e] = R.rs * (g[i][e] - s1 - xh[i][e] * s2);
          if (dR) dx[e] += bf2f(rr[e]);
          aw[i][e] += dy[i][e] * xh[i][e];
          ab[i][e] += dy[i][e];
        }
        *(bf16x4*)(dX + row * H + c) = bf16x4{f2bf(dx[0]), f2bf(dx[1]), f2bf(dx[2]), f2bf(dx[3])};
        if (dXd) {
          uint32_t keep = thr ? mmu_keep4(mmu_eff_seed(seed, seed_off), (uint64_t)(row * H + c) >> 2, thr) : 0xFu;
#pragma unroll
          for (int e = 0; e < 4; ++e) dx[e] = ((keep >> e) & 1) ? dx[e] * scale : 0.f;
          *(bf16x4*)(dXd + row * H + c) = bf16x4{f2bf(dx[0]), f2bf(dx[1]), f2bf(dx[2]), f2bf(dx[3])};
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) ac[i][e] += dx[e];
      }
  };
  const int64_t r0 = (int64_t)blockIdx.x * rpp;
  const int64_t rend = r0 + rpp < rows ? r0 + rpp : rows;
  for (int64_t row = r0 + wv; row < rend; row += 8) {
    Row A, Bq;
    const bool two = row + 4 < rend;
    load(row, A);
    if (two) load(row + 4, Bq);
    process(row, A);
    if (two) process(row + 4, Bq);
  }
  // partial column sums: three passes through one [4 waves][H] buffer
  float* outs[3] = {pdw, pdb, pdbias};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
#pragma unroll
    for (int i = 0; i < NV; ++i)
      if (i < nv)
#pragma unroll
        for (int e = 0; e < 4; ++e) red[wv][256 * i + 4 * l + e] = k == 0 ? aw[i][e] : (k == 1 ? ab[i][e] : ac[i][e]);
    __syncthreads();
    if (outs[k])
      for (int c = threadIdx.x; c < H; c += 256)
        outs[k][(int64_t)blockIdx.x * H + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
    __syncthreads();
  }
}

void layernorm_fwd_launch(const bf16* X, const float* w, const float* b, bf16* Y, float* mean, float* rstd,
                          int64_t rows, int64_t H, float eps, int64_t group_rows, int64_t pstride, hipStream_t s) {
  if ((group_rows % 2 == 0 || group_rows >= rows || pstride == 0) && H % 256 == 0 && H <= 1024) {
    const dim3 g2((unsigned)(((rows + 1) / 2 + LN2_PAIRS - 1) / LN2_PAIRS));
#define LNF2(NV) hipLaunchKernelGGL(ln_fwd2_kernel<NV>, g2, dim3(256), 0, s, X, w, b, Y, mean, rstd, rows, eps, \
                                    group_rows, pstride)
    switch (H / 256) {
      case 1: LNF2(1); break;
      case 2: LNF2(2); break;
      case 3: LNF2(3); break;
      default: LNF2(4); break;
    }
#undef LNF2
    return;
  }
  const dim3 g((unsigned)((rows + LN_FWD_ROWS - 1) / LN_FWD_ROWS));
#define LNF(NV) hipLaunchKernelGGL(ln_fwd_kernel<NV>, g, dim3(256), 0, s, X, w, b, Y, mean, rstd, rows, eps, \
                                   group_rows, pstride)
  switch (H / 256) {
    case 1: LNF(1); break;
    case 2: LNF(2); break;
    case 3: LNF(3); break;
    default: LNF(4); break;
  }
#undef LNF
}

void layernorm_fwd32_launch(const float* X, const float* w, const float* b, bf16* Y, float* Y32, float* mean,
                            float* rstd, int64_t rows, int64_t H, float eps, int64_t group_rows, int64_t pstride,
                            hipStream_t s) {
  const dim3 g((unsigned)((rows + LN_FWD_ROWS - 1) / LN_FWD_ROWS));
#define LNF32(NV) hipLaunchKernelGGL(ln_fwd32_kernel<NV>, g, dim3(256), 0, s, X, w, b, Y, Y32, mean, rstd, rows, eps, \
                                     group_rows, pstride)
  switch (H / 256) {
    case 1: LNF32(1); break;
    case 2: LNF32(2); break;
    case 3: LNF32(3); break;
    default: LNF32(4); break;
  }
#undef LNF32
}

template <typename XT>
static void ln_bwd_launch_t(const bf16* dY, const XT* X, const float* mean, const float* rstd, const float* w,
                            bf16* dX, bf16* dXdrop, const bf16* dR, float drop_p, uint64_t seed,
                            const uint64_t* seed_off, float* pdw, float* pdb, float* pdbias, int64_t rows, int64_t H,
                            int64_t rpp, hipStream_t s) {
  const dim3 g((unsigned)((rows + rpp - 1) / rpp));
#define LNB(NV) hipLaunchKernelGGL((ln_bwd_kernel<NV, XT>), g, dim3(256), 0, s, dY, X, mean, rstd, w, dX, dXdrop, dR, \
                                   drop_p, seed, seed_off, pdw, pdb, pdbias, rows, (int)rpp)
  switch (H / 256) {
    case 1: LNB(1); break;
    case 2: LNB(2); break;
    case 3: LNB(3); break;
    default: LNB(4); break;
  }
#undef LNB
}

void layernorm_bwd_launch(const bf16* dY, const void* X, bool x_f32, const float* mean, const float* rstd,
                          const float* w, bf16* dX, bf16* dXdrop, const bf16* dR, float drop_p, uint64_t seed,
                          const uint64_t* seed_off, float* pdw, float* pdb, float* pdbias, int64_t rows, int64_t H,
                          int64_t rpp, hipStream_t s) {
  if (x_f32)
    ln_bwd_launch_t(dY, (const float*)X, mean, rstd, w, dX, dXdrop, dR, drop_p, seed, seed_off, pdw, pdb, pdbias, rows,
                    H, rpp, s);
  else
    ln_bwd_launch_t(dY, (const bf16*)X, mean, rstd, w, dX, dXdrop, dR, drop_p, seed, seed_off, pdw, pdb, pdbias, rows,
                    H, rpp, s);
}

}  // namespace mmu
