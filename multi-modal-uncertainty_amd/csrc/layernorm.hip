// Row LayerNorm over the 768-wide hidden state (gfx950), forward and backward.
//
// BertLayerNorm of BertSelfOutput / BertOutput in the encoder (src/mmbt.py:124-126):
// y = (x - mean) / sqrt(var + eps) * w + b, biased variance, eps 1e-12.
// One wave per row, 4 contiguous bf16 per lane per 256-column slab (8-B accesses).
// The backward also undoes the dropout of the producing GEMM epilogue
// (MMU_EPI_BIAS_DROP_RES: same (seed, m*H+n) quad stream) and emits per-block
// partial column sums for dgamma / dbeta / dbias, so the LN-affine and the Linear
// bias gradients cost no extra pass over the activations.
#include "mmu_common.h"
#include "mmu_internal.h"

namespace mmu {

constexpr int MAXV = 4;  // up to 4 slabs of 256 columns -> H <= 1024

// rows are grouped: row r uses the affine params of group r / group_rows (stride pstride);
// one group == the plain LN, K groups == K ensemble members in one launch
__global__ __launch_bounds__(256) void ln_fwd_kernel(const bf16* __restrict__ X, const float* __restrict__ w,
                                                     const float* __restrict__ b, bf16* __restrict__ Y,
                                                     float* __restrict__ mean, float* __restrict__ rstd,
                                                     int64_t rows, int H, float eps, int64_t group_rows,
                                                     int64_t pstride) {
  const int l = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  w += (row / group_rows) * pstride;
  b += (row / group_rows) * pstride;
  const int nv = H / 256;
  float v[MAXV][4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
    if (i < nv) {
      bf16x4 x = *(const bf16x4*)(X + row * H + 256 * i + 4 * l);
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[i][e] = bf2f(x[e]); s += v[i][e]; }
    }
  const float mu = wave_sum(s) / H;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
    if (i < nv)
#pragma unroll
      for (int e = 0; e < 4; ++e) { float d = v[i][e] - mu; q += d * d; }
  const float rs = rsqrtf(wave_sum(q) / H + eps);
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
    if (i < nv) {
      const int c = 256 * i + 4 * l;
      float4 ww = *(const float4*)(w + c), bb = *(const float4*)(b + c);
      bf16x4 y = {f2bf((v[i][0] - mu) * rs * ww.x + bb.x), f2bf((v[i][1] - mu) * rs * ww.y + bb.y),
                  f2bf((v[i][2] - mu) * rs * ww.z + bb.z), f2bf((v[i][3] - mu) * rs * ww.w + bb.w)};
      *(bf16x4*)(Y + row * H + c) = y;
    }
  if (l == 0 && mean) { mean[row] = mu; rstd[row] = rs; }
}

// block = 4 waves; each wave walks rows_per_part/4 rows; partial sums reduced through LDS
__global__ __launch_bounds__(256) void ln_bwd_kernel(const bf16* __restrict__ dY, const bf16* __restrict__ X,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const float* __restrict__ w, bf16* __restrict__ dX,
                                                     bf16* __restrict__ dXd, float drop_p, uint64_t seed,
                                                     float* __restrict__ pdw, float* __restrict__ pdb,
                                                     float* __restrict__ pdbias, int64_t rows, int H, int rpp) {
  __shared__ float red[3][4][1024];
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nv = H / 256;
  const float scale = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
  const uint32_t thr = (uint32_t)(drop_p * 65536.0f + 0.5f);
  float aw[MAXV][4], ab[MAXV][4], ac[MAXV][4], ww[MAXV][4];
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      aw[i][e] = ab[i][e] = ac[i][e] = 0.f;
      ww[i][e] = i < nv ? w[256 * i + 4 * l + e] : 0.f;
    }
  const int64_t r0 = (int64_t)blockIdx.x * rpp;
  for (int64_t row = r0 + wv; row < r0 + rpp && row < rows; row += 4) {
    const float mu = mean[row], rs = rstd[row];
    float g[MAXV][4], xh[MAXV][4], dy[MAXV][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i)
      if (i < nv) {
        bf16x4 a = *(const bf16x4*)(dY + row * H + 256 * i + 4 * l);
        bf16x4 x = *(const bf16x4*)(X + row * H + 256 * i + 4 * l);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          dy[i][e] = bf2f(a[e]);
          xh[i][e] = (bf2f(x[e]) - mu) * rs;
          g[i][e] = dy[i][e] * ww[i][e];
          s1 += g[i][e];
          s2 += g[i][e] * xh[i][e];
        }
      }
    s1 = wave_sum(s1) / H;
    s2 = wave_sum(s2) / H;
#pragma unroll
    for (int i = 0; i < MAXV; ++i)
      if (i < nv) {
        const int c = 256 * i + 4 * l;
        float dx[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          dx[e] = rs * (g[i][e] - s1 - xh[i][e] * s2);
          aw[i][e] += dy[i][e] * xh[i][e];
          ab[i][e] += dy[i][e];
        }
        *(bf16x4*)(dX + row * H + c) = bf16x4{f2bf(dx[0]), f2bf(dx[1]), f2bf(dx[2]), f2bf(dx[3])};
        if (dXd) {
          uint32_t keep = thr ? mmu_keep4(seed, (uint64_t)(row * H + c) >> 2, thr) : 0xFu;
#pragma unroll
          for (int e = 0; e < 4; ++e) dx[e] = ((keep >> e) & 1) ? dx[e] * scale : 0.f;
          *(bf16x4*)(dXd + row * H + c) = bf16x4{f2bf(dx[0]), f2bf(dx[1]), f2bf(dx[2]), f2bf(dx[3])};
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) ac[i][e] += dx[e];
      }
  }
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
    if (i < nv)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = 256 * i + 4 * l + e;
        red[0][wv][c] = aw[i][e];
        red[1][wv][c] = ab[i][e];
        red[2][wv][c] = ac[i][e];
      }
  __syncthreads();
  for (int c = threadIdx.x; c < H; c += 256) {
    const int64_t o = (int64_t)blockIdx.x * H + c;
    if (pdw) pdw[o] = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
    if (pdb) pdb[o] = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
    if (pdbias) pdbias[o] = red[2][0][c] + red[2][1][c] + red[2][2][c] + red[2][3][c];
  }
}

void layernorm_fwd_launch(const bf16* X, const float* w, const float* b, bf16* Y, float* mean, float* rstd,
                          int64_t rows, int64_t H, float eps, int64_t group_rows, int64_t pstride, hipStream_t s) {
  hipLaunchKernelGGL(ln_fwd_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, X, w, b, Y, mean, rstd,
                     rows, (int)H, eps, group_rows, pstride);
}

void layernorm_bwd_launch(const bf16* dY, const bf16* X, const float* mean, const float* rstd, const float* w,
                          bf16* dX, bf16* dXdrop, float drop_p, uint64_t seed, float* pdw, float* pdb,
                          float* pdbias, int64_t rows, int64_t H, int64_t rpp, hipStream_t s) {
  hipLaunchKernelGGL(ln_bwd_kernel, dim3((unsigned)((rows + rpp - 1) / rpp)), dim3(256), 0, s, dY, X, mean, rstd,
                     w, dX, dXdrop, drop_p, seed, pdw, pdb, pdbias, rows, (int)H, (int)rpp);
}

}  // namespace mmu
