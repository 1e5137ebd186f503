// ResNet-152 stem convolution (7x7, stride 2, pad 3, 3 -> 64 channels) on channels-last bf16
// images (gfx950): the image encoder's conv embed of the reference (torchvision resnet
// child 0, src/mmbt.py:19-21,42).  Its 3 input channels make it a bad fit for the
// 64-deep implicit-GEMM conv kernels, so it gets its own pair:
//
//   forward  Y[p][o]  = sum_k W[o][k] col[k][p]          k = tap * 4 + c  (tap = kh*7 + kw,
//   filter   dW[o][k] = sum_p dY[p][o] col[k][p]          c padded 3 -> 4, taps padded 49 -> 56)
//
// A tile is 2 output rows x 64 output columns (128 pixels).  Its input patch (9 rows x 133
// columns x 4 channels, zero outside the image and in the padding channel) is staged in LDS;
// the 224-deep contraction runs as 7 K-steps of v_mfma_f32_16x16x32_bf16 whose im2col
// operand is two 8-B LDS reads per lane (two consecutive taps of one pixel).  Blocks are
// persistent (a grid-stride loop over tiles) so the filter is loaded into LDS once per block.
//   forward: 4 waves, each 32 pixels x 64 channels; the output goes through a per-wave LDS
//            staging tile so every store is a 16-B lane over the wave's contiguous 4 KiB.
//   filter : 4 waves, each 16 output channels x all 224 k (ordered (kh, kw padded to 8, c));
//            the dY rows are staged as loaded ([pixel][channel], 16-B coalesced) and both
//            operands, whose contraction runs over pixels, come from transposed LDS reads
//            (dY^T from the dY rows, im2col^T straight from the patch); per-block f32
//            partials [64][224] are summed in block order by stem_wgrad_reduce_kernel.
// Both kernels prefetch the next tile's patch (and dY rows) into registers under the
// current tile's MFMAs.
#include "mmu_common.h"
#include "mmu_internal.h"

namespace mmu {

namespace {
constexpr int ST_TR = 2, ST_TC = 64;                       // output rows x cols per tile
constexpr int ST_PR = 2 * ST_TR + 5, ST_PC = 2 * ST_TC + 6;  // input patch rows (9) x cols (134: col 133
                                                           // is read only by the filter gradient's
                                                           // padded 8th tap of a row, weight zero)
constexpr int ST_KP = 224;                                 // 56 taps x 4 channels
constexpr int ST_WROW = 272;                               // LDS filter row: 136 dwords = 8 mod 64, conflict-free b128 reads
constexpr int ST_OROW = 72;                                // LDS output staging row, bf16
constexpr int ST_TROW = 136;                               // LDS transposed rows ([.][pixel]), bf16
constexpr int ST_PATCH = ST_PR * ST_PC * 4;                // bf16 elements

struct StemGeo {
  int img, ho0, wo0;
};
static __device__ __forceinline__ StemGeo stem_tile(const StemParams& p, int64_t tile) {
  const int per_img = p.tiles_r * p.tiles_c;
  StemGeo s;
  s.img = (int)(tile / per_img);
  const int rem = (int)(tile - (int64_t)s.img * per_img);
  const int tr = rem / p.tiles_c;
  s.ho0 = ST_TR * tr;
  s.wo0 = ST_TC * (rem - tr * p.tiles_c);
  return s;
}

// input patch of a tile, prefetched into registers and then written to an LDS buffer
// [row][col][4]; channel 3 of every patch pixel is zeroed once per buffer (stem_zero_patch)
// and never written again.  The 28 threads t = 28 row + u of a patch row take its values
// e = u + 28 i (i < ST_PLOAD) in the image's own [col][3] order: consecutive threads read
// consecutive values (coalesced), and as 28 = 3 * 9 + 1 the column / channel of the next
// value follow by a carry instead of a division.
constexpr int ST_RVALS = ST_PC * 3;                        // 402 values per patch row
constexpr int ST_PTHR = 28;                                // threads per patch row
constexpr int ST_PLOAD = (ST_RVALS + ST_PTHR - 1) / ST_PTHR;  // 15
static __device__ __forceinline__ void stem_zero_patch(bf16* Ps) {
  for (int e = threadIdx.x; e < ST_PATCH; e += 256) Ps[e] = (bf16)0.f;
}
static __device__ __forceinline__ void stem_fetch_patch(const StemParams& p, const StemGeo& s, bf16 (&v)[ST_PLOAD]) {
  const int t = threadIdx.x, row = t / ST_PTHR, u = t - row * ST_PTHR;
  const int hi = 2 * s.ho0 - 3 + row, wi0 = 2 * s.wo0 - 3;
  const bool row_ok = t < ST_PR * ST_PTHR && hi >= 0 && hi < p.H;
  const bf16* src = p.X + (((int64_t)s.img * p.H + (row_ok ? hi : 0)) * p.W + wi0) * 3 + u;
  int col = u / 3, c = u - 3 * col;
#pragma unroll
  for (int i = 0; i < ST_PLOAD; ++i) {
    const int wi = wi0 + col;
    v[i] = (row_ok && u + ST_PTHR * i < ST_RVALS && wi >= 0 && wi < p.W) ? src[ST_PTHR * i] : (bf16)0.f;
    col += 9;
    if (++c == 3) { c = 0; ++col; }
  }
}
static __device__ __forceinline__ void stem_store_patch(const bf16 (&v)[ST_PLOAD], bf16* Ps) {
  const int t = threadIdx.x, row = t / ST_PTHR, u = t - row * ST_PTHR;
  if (t >= ST_PR * ST_PTHR) return;
  int col = u / 3, c = u - 3 * col;
  bf16* dst = Ps + row * ST_PC * 4;
#pragma unroll
  for (int i = 0; i < ST_PLOAD; ++i) {
    if (u + ST_PTHR * i < ST_RVALS) dst[col * 4 + c] = v[i];
    col += 9;
    if (++c == 3) { c = 0; ++col; }
  }
}

static __device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
}  // namespace

__global__ __launch_bounds__(256) void stem_fwd_kernel(StemParams p) {
  __shared__ __attribute__((aligned(16))) bf16 Ws[64 * ST_WROW];
  __shared__ __attribute__((aligned(16))) bf16 Ps[2][ST_PATCH];
  __shared__ __attribute__((aligned(16))) bf16 Os[4][32 * ST_OROW];
  const int t = threadIdx.x, l = t & 63, w = t >> 6, g = l >> 4, j = l & 15;
  // filter [64][7][7][3] -> Ws[o][tap * 4 + c] (padding taps / channel zero)
  for (int i = t; i < 64 * ST_KP; i += 256) {
    const int o = i / ST_KP, k = i - o * ST_KP, tap = k >> 2, c = k & 3;
    Ws[o * ST_WROW + k] = (tap < 49 && c < 3) ? p.Wt[(o * 49 + tap) * 3 + c] : (bf16)0.f;
  }
  stem_zero_patch(Ps[0]);
  stem_zero_patch(Ps[1]);
  const int r = w >> 1, cb = 32 * (w & 1);  // this wave: output row r, columns cb .. cb+31 of the tile
  bf16* O = Os[w];
  bf16 pv[ST_PLOAD];
  int64_t tile = blockIdx.x;
  if (tile < p.n_tiles) stem_fetch_patch(p, stem_tile(p, tile), pv);
  __syncthreads();  // zeroed patch buffers
  int buf = 0;
  for (; tile < p.n_tiles; tile += gridDim.x) {
    const StemGeo s = stem_tile(p, tile);
    stem_store_patch(pv, Ps[buf]);
    __syncthreads();  // this tile's patch (and, the first time, the filter) is in LDS
    if (tile + gridDim.x < p.n_tiles) stem_fetch_patch(p, stem_tile(p, tile + gridDim.x), pv);  // in flight
    const bf16* P = Ps[buf];
    f32x4 acc[2][4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < ST_KP / 32; ++ks) {
      bf16x8 wa[4];
#pragma unroll
      for (int cs = 0; cs < 4; ++cs) wa[cs] = *(const bf16x8*)&Ws[(16 * cs + j) * ST_WROW + 32 * ks + 8 * g];
      // taps 8 ks + 2 g and + 1 (beyond 48: padding, the filter there is zero; read tap 48)
      int t0 = 8 * ks + 2 * g, t1 = t0 + 1;
      t0 = t0 > 48 ? 48 : t0;
      t1 = t1 > 48 ? 48 : t1;
      const int kh0 = t0 / 7, kw0 = t0 - 7 * kh0, kh1 = t1 / 7, kw1 = t1 - 7 * kh1;
#pragma unroll
      for (int ps = 0; ps < 2; ++ps) {
        const int col = cb + 16 * ps + j;
        const bf16x4 v0 = *(const bf16x4*)&P[((2 * r + kh0) * ST_PC + 2 * col + kw0) * 4];
        const bf16x4 v1 = *(const bf16x4*)&P[((2 * r + kh1) * ST_PC + 2 * col + kw1) * 4];
        const bf16x8 b = bf16x8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
#pragma unroll
        for (int cs = 0; cs < 4; ++cs) acc[ps][cs] = mfma16(wa[cs], b, acc[ps][cs]);
      }
    }
    // D lane: channels 16 cs + 4 g + i of pixel 16 ps + j -> this wave's staging [pixel][channel]
#pragma unroll
    for (int ps = 0; ps < 2; ++ps)
#pragma unroll
      for (int cs = 0; cs < 4; ++cs)
        *(bf16x4*)&O[(16 * ps + j) * ST_OROW + 16 * cs + 4 * g] =
            bf16x4{f2bf(acc[ps][cs][0]), f2bf(acc[ps][cs][1]), f2bf(acc[ps][cs][2]), f2bf(acc[ps][cs][3])};
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int ho = s.ho0 + r;
    if (ho < p.Ho) {
      bf16* yrow = p.Y + (((int64_t)s.img * p.Ho + ho) * p.Wo + s.wo0 + cb) * 64;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = l + 64 * i, px = q >> 3, part = q & 7;
        if (s.wo0 + cb + px < p.Wo)
          *(bf16x8*)&yrow[px * 64 + part * 8] = *(const bf16x8*)&O[px * ST_OROW + part * 8];
      }
    }
    buf ^= 1;
  }
}

// transposed 16x16x32 operand from LDS (ds_read_b64_tr_b16, cdna_hip_programming.md T10): lane
// 4q + p of each 16-lane group g gives the address of block row q, columns 4p .. 4p+3; the
// block rows are the group's 8 contraction indices (two reads of 4), the 16 columns the
// operand's 16 rows / columns, so lane j of the group gets column j for all 8 indices.
static __device__ __forceinline__ bf16x8 stem_tr(const bf16* a0, const bf16* a1) {
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((MMU_LDS(bf16x4)*)a0);
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((MMU_LDS(bf16x4)*)a1);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// Filter gradient, K ordered k = (kh * 8 + kw) * 4 + c (kw padded to 8): a 16-column subtile
// kt = (kh, half) is taps kw = 4 half .. 4 half + 3 of one kernel row = 16 CONSECUTIVE bf16 of
// a patch pixel's row, so the im2col operand is read straight from the patch by transposed
// reads (block rows = 4 output pixels, at stride 2 input columns), no im2col tile is built.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void stem_wgrad_kernel(
    StemParams p, float* __restrict__ ws) {
  __shared__ __attribute__((aligned(16))) bf16 Ps[2][ST_PATCH];
  __shared__ __attribute__((aligned(16))) bf16 Dp[2][128 * ST_OROW];   // dY tile [pixel][channel]
  const int t = threadIdx.x, l = t & 63, w = t >> 6, g = l >> 4, q = (l >> 2) & 3, pp = l & 3;
  f32x4 acc[ST_KP / 16];
#pragma unroll
  for (int a = 0; a < ST_KP / 16; ++a) acc[a] = f32x4{0.f, 0.f, 0.f, 0.f};
  stem_zero_patch(Ps[0]);
  stem_zero_patch(Ps[1]);
  // next tile in registers: its patch values and its dY rows (2 x 64 pixels x 128 B: 4 x 16 B
  // per thread, coalesced)
  bf16 pv[ST_PLOAD];
  bf16x8 dv[4];
  auto fetch = [&](int64_t tile) {
    const StemGeo s = stem_tile(p, tile);
    stem_fetch_patch(p, s, pv);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int qq = t + 256 * i, px = qq >> 3, part = qq & 7, rr = px >> 6, cc = px & 63;
      const int ho = s.ho0 + rr, wo = s.wo0 + cc;
      dv[i] = (ho < p.Ho && wo < p.Wo)
                  ? *(const bf16x8*)&p.dY[(((int64_t)s.img * p.Ho + ho) * p.Wo + wo) * 64 + 8 * part]
                  : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  };
  int64_t tile = blockIdx.x;
  if (tile < p.n_tiles) fetch(tile);
  __syncthreads();  // zeroed patch buffers
  int buf = 0;
  for (; tile < p.n_tiles; tile += gridDim.x) {
    stem_store_patch(pv, Ps[buf]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int qq = t + 256 * i, px = qq >> 3, part = qq & 7;
      *(bf16x8*)&Dp[buf][px * ST_OROW + 8 * part] = dv[i];
    }
    __syncthreads();
    if (tile + gridDim.x < p.n_tiles) fetch(tile + gridDim.x);  // in flight under this tile
    const bf16* P = Ps[buf];
    const bf16* D = Dp[buf];
#pragma unroll 1
    for (int ks = 0; ks < 4; ++ks) {  // 4 x 32 pixels: this group's pixels 32 ks + 8 g + q (+ 4)
      const int px0 = 32 * ks + 8 * g + q, px1 = px0 + 4;
      // A = dY^T: rows = channels 16 w .. 16 w + 15
      const bf16x8 a = stem_tr(&D[px0 * ST_OROW + 16 * w + 4 * pp], &D[px1 * ST_OROW + 16 * w + 4 * pp]);
      const int r0 = px0 >> 6, c0 = px0 & 63, r1 = px1 >> 6, c1 = px1 & 63;
#pragma unroll
      for (int kt = 0; kt < ST_KP / 16; ++kt) {
        const int kh = kt >> 1, kw = 4 * (kt & 1) + pp;
        const bf16x8 b = stem_tr(&P[((2 * r0 + kh) * ST_PC + 2 * c0 + kw) * 4],
                                 &P[((2 * r1 + kh) * ST_PC + 2 * c1 + kw) * 4]);
        acc[kt] = mfma16(a, b, acc[kt]);
      }
    }
    buf ^= 1;
  }
  // D lane: channels 16 w + 4 g + i, k = 16 kt + (l & 15) -> this block's partial slab [64][224]
  float* slab = ws + (int64_t)blockIdx.x * 64 * ST_KP;
#pragma unroll
  for (int kt = 0; kt < ST_KP / 16; ++kt)
#pragma unroll
    for (int i = 0; i < 4; ++i) slab[(16 * w + 4 * g + i) * ST_KP + 16 * kt + (l & 15)] = acc[kt][i];
}

// dW[o][tap][c] (+)= sum over the block slabs, in a fixed order (deterministic): a block per
// (o, 16 consecutive outputs), 16 slab slices per output summed by one thread each (8 loads in
// flight), then the 16 slices added in slice order
__global__ __launch_bounds__(256) void stem_wgrad_reduce_kernel(const float* __restrict__ ws, int nslabs,
                                                                 float* __restrict__ dW, int accumulate) {
  __shared__ float red[16][17];
  const int o = blockIdx.y, j = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int r = blockIdx.x * 16 + j;  // output (tap, c) index within o: 0 .. 146
  float s = 0.f;
  if (r < 147) {
    const int tap = r / 3, c = r - 3 * tap, kh = tap / 7, kw = tap - 7 * kh;
    const float* src = ws + o * ST_KP + (kh * 8 + kw) * 4 + c;
#pragma unroll 8
    for (int b = sl; b < nslabs; b += 16) s += src[(int64_t)b * 64 * ST_KP];
  }
  red[sl][j] = s;
  __syncthreads();
  if (sl == 0 && r < 147) {
    float tot = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) tot += red[k][j];
    float* d = dW + o * 147 + r;
    *d = accumulate ? *d + tot : tot;
  }
}

static int stem_grid(int64_t n_tiles, int per_cu) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  const int64_t g = (int64_t)cus * per_cu;
  return (int)(n_tiles < g ? n_tiles : g);
}

void stem_fill_geometry(StemParams& p) {
  p.Ho = (p.H - 1) / 2 + 1;
  p.Wo = (p.W - 1) / 2 + 1;
  p.tiles_r = (p.Ho + ST_TR - 1) / ST_TR;
  p.tiles_c = (p.Wo + ST_TC - 1) / ST_TC;
  p.n_tiles = (int64_t)p.n * p.tiles_r * p.tiles_c;
}

int64_t stem_wgrad_ws_floats(int64_t n_tiles) { return (int64_t)stem_grid(n_tiles, 2) * 64 * ST_KP; }

void stem_fwd_launch(const StemParams& p, hipStream_t s) {
  hipLaunchKernelGGL(stem_fwd_kernel, dim3(stem_grid(p.n_tiles, 2)), dim3(256), 0, s, p);
}

void stem_wgrad_launch(const StemParams& p, float* dW, int accumulate, float* ws, hipStream_t s) {
  const int nb = stem_grid(p.n_tiles, 2);
  hipLaunchKernelGGL(stem_wgrad_kernel, dim3(nb), dim3(256), 0, s, p, ws);
  hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3((147 + 15) / 16, 64), dim3(256), 0, s, ws, nb, dW, accumulate);
}

}  // namespace mmu
