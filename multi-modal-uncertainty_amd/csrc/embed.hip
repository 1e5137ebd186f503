// Modality-token embedding + text gather + concat / control gather (gfx950).
//
// One pass builds the encoder input rows the reference assembles from
//   ImageBertEmbeddings   src/mmbt.py:58-83   ([CLS] | Linear(img) | [SEP], pos 0..N+1, type 0, LN)
//   BertEmbeddings        src/mmbt.py:121     (word[id] + pos[t] + type[seg], LN)
//   torch.cat             src/mmbt.py:122     (img tokens then text)
//   encoder_input[:, idx] src/mmbt.py:229     (forward_control gather, one index set per call)
// and the additive key mask (src/mmbt.py:101-112,203-216) for every output row, so
// the [B, L, 768] activation is written exactly once, already in its final order.
// Also: AdaptiveAvgPool2d((N,1)) of the ResNet map (src/mmbt.py:30,42-44) and the
// embedding backward (LN backward + word-row atomics + batch reductions).
#include "mmu_common.h"
#include "mmu_internal.h"

namespace mmu {


static __device__ __forceinline__ void add_row(float (&acc)[3][4], const float* __restrict__ src, int l) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    float4 a = *(const float4*)(src + 256 * i + 4 * l);
    acc[i][0] += a.x; acc[i][1] += a.y; acc[i][2] += a.z; acc[i][3] += a.w;
  }
}

// pre-LN embedding sum of source position s for batch row b (H == 768)
static __device__ __forceinline__ void embed_sum(float (&e)[3][4], const EmbedParams& p, int64_t b, int64_t s,
                                                 int l, float& km) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) e[i][k] = 0.f;
  const int64_t H = p.H, nimg = p.n_img;
  km = 0.f;
  if (s <= nimg + 1) {
    if (s == 0) add_row(e, p.word + p.cls_id * H, l);
    else if (s == nimg + 1) add_row(e, p.word + p.sep_id * H, l);
    else add_row(e, p.proj + (b * nimg + (s - 1)) * H, l);
    add_row(e, p.pos + s * H, l);
    add_row(e, p.type, l);
  } else {
    const int64_t t = s - nimg - 2;
    const int64_t id = p.ids[b * p.T + t], sg = p.seg[b * p.T + t];
    add_row(e, p.word + id * H, l);
    add_row(e, p.pos + t * H, l);
    add_row(e, p.type + sg * H, l);
    if (p.txt_mask && p.txt_mask[b * p.T + t] == 0) km = -10000.0f;
  }
}

__global__ __launch_bounds__(256) void embed_fwd_kernel(EmbedParams p) {
  const int l = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t total = p.V * p.B * p.Lout;
  if (row >= total) return;
  const int64_t j = row % p.Lout, vb = row / p.Lout, b = vb % p.B, v = vb / p.B;
  const int64_t s = p.idx ? p.idx[v * p.Lout + j] : j;
  float e[3][4], km;
  embed_sum(e, p, b, s, l, km);
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) sum += e[i][k];
  const float mu = wave_sum(sum) / 768.f;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) { float d = e[i][k] - mu; q += d * d; }
  const float rs = rsqrtf(wave_sum(q) / 768.f + p.eps);
  // dropout: ImageBertEmbeddings.dropout (p = args.dropout) on the image-segment rows,
  // BertEmbeddings.dropout (0.1) on text rows; element counter row*768 + col
  const float dp = s <= p.n_img + 1 ? p.drop_img : p.drop_txt;
  const uint32_t thr = (uint32_t)(dp * 65536.0f + 0.5f);
  const float dsc = dp > 0.f ? 1.0f / (1.0f - dp) : 1.0f;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int c = 256 * i + 4 * l;
    float4 w = *(const float4*)(p.ln_w + c), bb = *(const float4*)(p.ln_b + c);
    float y[4] = {(e[i][0] - mu) * rs * w.x + bb.x, (e[i][1] - mu) * rs * w.y + bb.y,
                  (e[i][2] - mu) * rs * w.z + bb.z, (e[i][3] - mu) * rs * w.w + bb.w};
    if (thr) {
      const uint32_t keep = mmu_keep4(mmu_eff_seed(p.seed, p.seed_off), (uint64_t)(row * 768 + c) >> 2, thr);
#pragma unroll
      for (int k = 0; k < 4; ++k) y[k] = ((keep >> k) & 1) ? y[k] * dsc : 0.f;
    }
    *(bf16x4*)(p.X + row * 768 + c) = bf16x4{f2bf(y[0]), f2bf(y[1]), f2bf(y[2]), f2bf(y[3])};
    if (p.X32) *(float4*)(p.X32 + row * 768 + c) = make_float4(y[0], y[1], y[2], y[3]);  // the f32 hidden stream
  }
  if (l == 0) {
    p.keymask[row] = km;
    if (p.mean) { p.mean[row] = mu; p.rstd[row] = rs; }
  }
}

void embed_fwd_launch(const EmbedParams& p, hipStream_t s) {
  const int64_t total = p.V * p.B * p.Lout;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3((unsigned)((total + 3) / 4)), dim3(256), 0, s, p);
}

// ---------------------------------------------------------------- backward
// One pass over the rows, position-major: a block = 4 consecutive source positions (one per wave)
// x EBW_B samples, so each wave sums its position's gradient over its samples in registers.  Per
// row: LN backward (dropout of the forward regenerated), the word-row scatter for text rows (f32
// atomics, 256 contiguous bytes per instruction), the image rows' dproj.  Per wave: its position
// sum into the position row / [CLS] / [SEP] word rows (f32 atomics, ceil(B / EBW_B) adds per
// address).  Per block: partial rows of dgamma, dbeta and the two token-type rows, folded by
// colsum_reduce.  (Round 6: the batch sums used to go through an f32 [B, S, H] copy of the row
// gradients and a second kernel walking it column-wise: 0.69 ms at B = 256 for 0.4 GB.)
constexpr int EBW_B = 16;  // samples per block
__global__ __launch_bounds__(256) void embed_bwd_rows_kernel(EmbedBwdParams q, EmbedParams p) {
  __shared__ float red[4][4][768];                            // aw, ab, type-0, type-1 per wave
  __shared__ __attribute__((aligned(16))) float xch[4][768];  // per wave: a text row's dx, re-read lane-contiguous
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t S = q.n_img + 2 + q.T, H = 768;
  const int64_t nblk = (int64_t)gridDim.x * gridDim.y;
  const int64_t blk = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
  float* part = q.ws;
  const int64_t s = (int64_t)blockIdx.x * 4 + wv;
  const int64_t b0 = (int64_t)blockIdx.y * EBW_B;
  const bool live = s < S;
  const bool text = s >= q.n_img + 2, img = s >= 1 && s <= q.n_img;
  const float dp = s <= q.n_img + 1 ? q.drop_img : q.drop_txt;
  const uint32_t thr = (uint32_t)(dp * 65536.0f + 0.5f);
  const float dsc = dp > 0.f ? 1.0f / (1.0f - dp) : 1.0f;
  float aw[3][4], ab[3][4], w[3][4], tot[3][4], t1[3][4];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      aw[i][k] = ab[i][k] = tot[i][k] = t1[i][k] = 0.f;
      w[i][k] = q.ln_w[256 * i + 4 * l + k];
    }
  for (int64_t b = b0; live && b < b0 + EBW_B && b < q.B; ++b) {
    const int64_t row = b * S + s;
    float e[3][4], km;
    embed_sum(e, p, b, s, l, km);
    const float mu = q.mean[row], rs = q.rstd[row];
    float g[3][4], xh[3][4], s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      bf16x4 d = *(const bf16x4*)(q.dX + row * H + 256 * i + 4 * l);
      const uint32_t keep = thr ? mmu_keep4(mmu_eff_seed(q.seed, q.seed_off), (uint64_t)(row * H + 256 * i + 4 * l) >> 2, thr) : 0xFu;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float dy = ((keep >> k) & 1) ? bf2f(d[k]) * dsc : 0.f;
        xh[i][k] = (e[i][k] - mu) * rs;
        g[i][k] = dy * w[i][k];
        s1 += g[i][k];
        s2 += g[i][k] * xh[i][k];
        aw[i][k] += dy * xh[i][k];
        ab[i][k] += dy;
      }
    }
    s1 = wave_sum(s1) / 768.f;
    s2 = wave_sum(s2) / 768.f;
    const bool seg1 = text && q.seg[b * q.T + (s - q.n_img - 2)] != 0;
    float* wrow = text ? q.d_word + q.ids[b * q.T + (s - q.n_img - 2)] * H : nullptr;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int c = 256 * i + 4 * l;
      float dx[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        dx[k] = rs * (g[i][k] - s1 - xh[i][k] * s2);
        tot[i][k] += dx[k];
        if (seg1) t1[i][k] += dx[k];
      }
      if (text) {
        *(float4*)(&xch[wv][c]) = make_float4(dx[0], dx[1], dx[2], dx[3]);
      } else if (img) {
        *(float4*)(q.d_proj + (b * q.n_img + (s - 1)) * H + c) = make_float4(dx[0], dx[1], dx[2], dx[3]);
      }
    }
    if (text) {  // word-row scatter: every atomic instruction adds 256 contiguous bytes (lane l ->
                 // column 64 j + l); 16-B-strided lanes ran the memory-side atomics at a fraction
                 // of their rate.  The row sits in this wave's own LDS slice: in-order LDS, no barrier.
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int j = 0; j < 12; ++j) atomicAdd(wrow + 64 * j + l, xch[wv][64 * j + l]);
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (live) {  // this position's sum over the block's samples: position row, [CLS] / [SEP] word rows
               // (through the wave's LDS slice: lane-contiguous 256-B atomic instructions)
    const int64_t posr = text ? s - q.n_img - 2 : s;
    float* wr = s == 0 ? q.d_word + q.cls_id * H : (s == q.n_img + 1 ? q.d_word + q.sep_id * H : nullptr);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < 3; ++i)
      *(float4*)(&xch[wv][256 * i + 4 * l]) = make_float4(tot[i][0], tot[i][1], tot[i][2], tot[i][3]);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      const float v = xch[wv][64 * j + l];
      atomicAdd(q.d_pos + posr * H + 64 * j + l, v);
      if (wr) atomicAdd(wr + 64 * j + l, v);
    }
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = 256 * i + 4 * l + k;
      red[0][wv][c] = aw[i][k];
      red[1][wv][c] = ab[i][k];
      red[2][wv][c] = tot[i][k] - t1[i][k];  // token type 0 (every image-segment row, text rows with seg 0)
      red[3][wv][c] = t1[i][k];
    }
  __syncthreads();
  for (int c = threadIdx.x; c < 768; c += 256)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      part[(r * nblk + blk) * H + c] = (red[r][0][c] + red[r][1][c]) + (red[r][2][c] + red[r][3][c]);
}

int64_t embed_bwd_blocks(int64_t B, int64_t S) { return ((S + 3) / 4) * ((B + EBW_B - 1) / EBW_B); }

void embed_bwd_launch(const EmbedBwdParams& q, hipStream_t s) {
  EmbedParams p{};
  p.ids = q.ids; p.seg = q.seg; p.txt_mask = nullptr; p.idx = nullptr;
  p.proj = q.proj; p.word = q.word; p.pos = q.pos; p.type = q.type;
  p.cls_id = q.cls_id; p.sep_id = q.sep_id; p.V = 1; p.B = q.B; p.T = q.T; p.n_img = q.n_img;
  p.Lout = q.n_img + 2 + q.T; p.H = 768;
  const int64_t nblk = embed_bwd_blocks(q.B, p.Lout);
  hipLaunchKernelGGL(embed_bwd_rows_kernel, dim3((unsigned)((p.Lout + 3) / 4), (unsigned)((q.B + EBW_B - 1) / EBW_B)),
                     dim3(256), 0, s, q, p);
  const float* part = q.ws;
  ColsumJobs jobs{};
  float* outs[4] = {q.d_ln_w, q.d_ln_b, q.d_type, q.d_type + 768};
  for (int z = 0; z < 4; ++z) {
    jobs.part[z] = part + z * nblk * 768;
    jobs.parts[z] = nblk;
    jobs.out[z] = outs[z];
  }
  colsum_reduce_multi_launch(jobs, 4, 768, 1, s);
}

// ---------------------------------------------------------------- AdaptiveAvgPool2d((n,1))
// bin i covers rows [floor(i*Hh/n), ceil((i+1)*Hh/n)), all columns
__global__ __launch_bounds__(256) void row_pool_fwd_kernel(const bf16* __restrict__ f, int64_t B, int Hh, int Ww,
                                                           int64_t C, int n, float* __restrict__ out) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;  // over B * C/8
  const int64_t c8 = C / 8;
  if (idx >= B * c8) return;
  const int64_t b = idx / c8, c = (idx % c8) * 8;
  for (int i = 0; i < n; ++i) {
    const int y0 = (i * Hh) / n, y1 = ((i + 1) * Hh + n - 1) / n;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int y = y0; y < y1; ++y)
      for (int x = 0; x < Ww; ++x) {
        bf16x8 v = *(const bf16x8*)(f + ((b * Hh + y) * Ww + x) * C + c);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += bf2f(v[e]);
      }
    const float inv = 1.0f / ((y1 - y0) * Ww);
    float* o = out + (b * n + i) * C + c;
    *(float4*)o = make_float4(acc[0] * inv, acc[1] * inv, acc[2] * inv, acc[3] * inv);
    *(float4*)(o + 4) = make_float4(acc[4] * inv, acc[5] * inv, acc[6] * inv, acc[7] * inv);
  }
}

__global__ __launch_bounds__(256) void row_pool_bwd_kernel(const float* __restrict__ d, int64_t B, int Hh, int Ww,
                                                           int64_t C, int n, bf16* __restrict__ df) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;  // over B*Hh * C/8
  const int64_t c8 = C / 8;
  if (idx >= B * Hh * c8) return;
  const int64_t by = idx / c8, c = (idx % c8) * 8, b = by / Hh;
  const int y = (int)(by % Hh);
  float g[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < n; ++i) {
    const int y0 = (i * Hh) / n, y1 = ((i + 1) * Hh + n - 1) / n;
    if (y < y0 || y >= y1) continue;
    const float inv = 1.0f / ((y1 - y0) * Ww);
    const float* s = d + (b * n + i) * C + c;
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] += s[e] * inv;
  }
  bf16x8 v;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = f2bf(g[e]);
  for (int x = 0; x < Ww; ++x) *(bf16x8*)(df + ((b * Hh + y) * Ww + x) * C + c) = v;
}

void row_pool_fwd_launch(const bf16* fmap, int64_t B, int64_t Hh, int64_t Ww, int64_t C, int64_t n, float* out,
                         hipStream_t s) {
  const int64_t tot = B * (C / 8);
  hipLaunchKernelGGL(row_pool_fwd_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, fmap, B, (int)Hh,
                     (int)Ww, C, (int)n, out);
}
void row_pool_bwd_launch(const float* dout, int64_t B, int64_t Hh, int64_t Ww, int64_t C, int64_t n, bf16* dfmap,
                         hipStream_t s) {
  const int64_t tot = B * Hh * (C / 8);
  hipLaunchKernelGGL(row_pool_bwd_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, dout, B, (int)Hh,
                     (int)Ww, C, (int)n, dfmap);
}

}  // namespace mmu
