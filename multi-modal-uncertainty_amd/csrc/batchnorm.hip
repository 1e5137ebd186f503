// BatchNorm2d (+ residual add) (+ ReLU) over channels-last bf16 activations (gfx950).
//
// The ResNet-152 image trunk (src/mmbt.py:19-21, torchvision Bottleneck) runs every
// conv output through BatchNorm2d, most of them followed by ReLU and one per block by
// the residual add + ReLU.  These kernels do that in as few passes over HBM as the math
// allows, on the NHWC image [rows = N*H*W][C] the MIOpen convs produce:
//   forward  (train): stats pass (read X)            -> per-block f32 sum / sum of squares
//                     finalize (per channel, f64)    -> scale, shift, running stats, mean/invstd
//                     apply pass (read X [+skip])    -> Y = act(X*scale + shift [+ skip])
//                                                       [+ ReLU mask: one bit per element, Y > 0]
//   forward  (eval):  finalize from running stats    -> apply pass
//   backward:         reduce pass (read dY, M, X)    -> per-block sum(g), sum(g*(x-mean)), g = dY*[Y>0]
//                     finalize                       -> dgamma, dbeta (accumulated), dx coefficients
//                     apply pass (read dY, M, X)     -> dX = k1*g + k2*x + k0  [, dSkip = g]
// The ReLU mask M ([rows][C/8] bytes, bit e of byte (r, c/8) = Y[r][c+e] > 0) replaces the
// backward's two reads of Y (2 B per element each) by two 1/8-B reads: the backward moves
// 10.25 instead of 14 B per element (without a mask it reads Y itself).
// Semantics of torch.nn.BatchNorm2d in training mode: biased variance normalises, the
// running variance is updated with the unbiased one, momentum-weighted.
// Cross-rank statistics (data-parallel training with the reference's whole-batch BatchNorm):
// each pass splits at its finalize -- the reduce pass's block partials are summed into
// per-channel f64 sums (+ the row count) that the caller all-reduces across ranks, and the
// finalize + apply then run from the exchanged sums (SyncBatchNorm semantics: the weight /
// bias gradients stay per-rank, summed by the gradient all-reduce like every other one).
//
// Work split: a block owns a chunk of CH <= 512 channels (grid.y) and a range of rows
// (grid.x) sized to 4 K - 64 K elements (~1 K blocks per launch, see bn_grid); a thread owns 8 consecutive channels (16-B bf16
// accesses, a row chunk is read as CH*2 contiguous bytes) of every rpi-th row.  Per-thread
// f32 partials are reduced over the block in LDS and stored as one (sum, sum2) pair per
// channel and block -- no atomics: ~1-3 K blocks x 2C float atomics on the same addresses
// serialise in the L2 atomic units (measured 4-10x slower than the apply pass).  The
// finalize sums the block partials per channel in f64 (32 slices per channel + LDS).
#include <stdlib.h>
#include "mmu_common.h"
#include "mmu_internal.h"

namespace mmu {

constexpr int BN_THREADS = 256;
constexpr int64_t BN_ELEMS_PER_BLOCK = 64 * 1024;
constexpr int64_t BN_MAX_PART_ELEMS = 1 << 20;  // (block, channel) partial pairs: 8 MiB of scratch

struct BnGeom {
  int tpr, rpi, cg, rs, c0;  // threads per row, rows per iteration, channel group, row slot, first channel
  int64_t r0, r1;            // the block's row range
};
static __device__ __forceinline__ BnGeom bn_geom(int CH, int64_t rows, int64_t rows_per_blk) {
  BnGeom g;
  g.tpr = CH >> 3;
  g.rpi = BN_THREADS / g.tpr;
  g.cg = threadIdx.x % g.tpr;
  g.rs = threadIdx.x / g.tpr;
  g.c0 = blockIdx.y * CH + 8 * g.cg;
  g.r0 = (int64_t)blockIdx.x * rows_per_blk;
  g.r1 = g.r0 + rows_per_blk < rows ? g.r0 + rows_per_blk : rows;
  return g;
}

// per-thread (a[8], b[8]) partials -> block sums per channel -> part[blockIdx.x][c] = {a, b}.
// LDS as [value][e][thread]: every write and read is one float per lane at consecutive
// addresses (the [thread][e] layout, 8 floats per lane, was ~3.6 bank-conflict cycles per LDS
// instruction in the step's PMC pass, profiles/r3_pmc_step_v3.txt)
static __device__ __forceinline__ void bn_block_reduce(const BnGeom& g, int C, const float (&a)[8],
                                                       const float (&b)[8], float2* __restrict__ part) {
  __shared__ float red[2][8][BN_THREADS];
  const int t = threadIdx.x;
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[0][e][t] = a[e]; red[1][e][t] = b[e]; }
  __syncthreads();
  if (t < g.tpr) {
    float sa[8], sb[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { sa[e] = 0.f; sb[e] = 0.f; }
    for (int r = 0; r < g.rpi; ++r) {
      const int o = r * g.tpr + t;
#pragma unroll
      for (int e = 0; e < 8; ++e) { sa[e] += red[0][e][o]; sb[e] += red[1][e][o]; }
    }
    float2* dst = part + (int64_t)blockIdx.x * C + g.c0;
#pragma unroll
    for (int e = 0; e < 8; ++e) dst[e] = make_float2(sa[e], sb[e]);
  }
}

// sum the nparts block partials of 4 channels per block: 32 slices x 8 (channel, component)
// columns, f64, then LDS; returns true (and the two totals) in the thread that owns channel c.
// (32 slices: the finalize is a dependent-load chain of nparts / slices loads per thread;
// with 8 slices it cost ~9 us per BN, 2.9 ms per step over the trunk's 310 launches.)
constexpr int BN_FIN_CH = 4;
static __device__ __forceinline__ bool bn_sum_parts(const float2* __restrict__ part, int nparts, int C, int& c,
                                                    double& s1, double& s2) {
  __shared__ double red[32][2 * BN_FIN_CH];
  const int t = threadIdx.x, col = t & (2 * BN_FIN_CH - 1), sl = t / (2 * BN_FIN_CH);
  c = blockIdx.x * BN_FIN_CH + (col >> 1);
  const int comp = col & 1;
  double acc = 0.0;
  if (c < C) {
    const float* p = (const float*)part + 2 * (int64_t)c + comp;
#pragma unroll 4
    for (int k = sl; k < nparts; k += 32) acc += (double)p[(int64_t)k * 2 * C];
  }
  red[sl][col] = acc;
  __syncthreads();
  if (sl != 0 || comp != 0 || c >= C) return false;
  s1 = 0.0;
  s2 = 0.0;
#pragma unroll
  for (int k = 0; k < 32; ++k) { s1 += red[k][col]; s2 += red[k][col + 1]; }
  return true;
}

__global__ __launch_bounds__(BN_THREADS) void bn_stats_kernel(const bf16* __restrict__ X, int64_t rows, int C, int CH,
                                                               int64_t rows_per_blk, float2* __restrict__ part) {
  const BnGeom g = bn_geom(CH, rows, rows_per_blk);
  float s[8], q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s[e] = 0.f; q[e] = 0.f; }
  if (g.rs < g.rpi) {
#pragma unroll 4
    for (int64_t r = g.r0 + g.rs; r < g.r1; r += g.rpi) {
      const bf16x8 v = *(const bf16x8*)(X + r * C + g.c0);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float f = bf2f(v[e]);
        s[e] += f;
        q[e] = fmaf(f, f, q[e]);
      }
    }
  }
  bn_block_reduce(g, C, s, q, part);
}

// per channel: coef = {scale, shift}; batch (partials) or running statistics
// the two per-channel totals of a pass: from the block partials, or (gsum != nullptr) from the
// exchanged cross-rank sums {s1[C], s2[C], rows} (then *n = their row count)
static __device__ __forceinline__ bool bn_channel_sums(const float2* __restrict__ part, int nparts,
                                                       const double* __restrict__ gsum, int C, int& c, double& s1,
                                                       double& s2, double* n) {
  if (!gsum) return bn_sum_parts(part, nparts, C, c, s1, s2);
  if (threadIdx.x >= BN_FIN_CH) return false;
  c = blockIdx.x * BN_FIN_CH + threadIdx.x;
  if (c >= C) return false;
  s1 = gsum[c];
  s2 = gsum[C + c];
  *n = gsum[2 * C];
  return true;
}

// the local per-channel sums of a reduce pass for the exchange: sums = {s1[C], s2[C], rows};
// the backward's (sinvstd != nullptr) also accumulates this rank's dweight / dbias
__global__ __launch_bounds__(BN_THREADS) void bn_local_sums_kernel(const float2* __restrict__ part, int nparts,
                                                                    int64_t rows, int C, double* __restrict__ sums,
                                                                    const float* sinvstd, float* dw, float* db) {
  int c;
  double s1, s2;
  if (!bn_sum_parts(part, nparts, C, c, s1, s2)) return;
  sums[c] = s1;
  sums[C + c] = s2;
  if (c == 0) sums[2 * C] = (double)rows;
  if (sinvstd) {
    if (dw) dw[c] += (float)(s2 * (double)sinvstd[c]);
    if (db) db[c] += (float)s1;
  }
}

__global__ __launch_bounds__(BN_THREADS) void bn_fwd_finalize_kernel(
    const float2* __restrict__ part, int nparts, const double* __restrict__ gsum, int64_t rows, int C,
    const float* w, const float* b, float* rmean, float* rvar, int training, float momentum, float eps,
    float* smean, float* sinvstd, int64_t* nbt, float* __restrict__ coef) {
  int c;
  double s1 = 0.0, s2 = 0.0, n = (double)rows;
  if (training) {
    if (!bn_channel_sums(part, nparts, gsum, C, c, s1, s2, &n)) return;
  } else {
    const int t = threadIdx.x;
    if (t >= BN_FIN_CH) return;
    c = blockIdx.x * BN_FIN_CH + t;
    if (c >= C) return;
  }
  double mean, var;
  if (training) {
    mean = s1 / n;
    var = s2 / n - mean * mean;
    if (var < 0.0) var = 0.0;
  } else {
    mean = rmean[c];
    var = rvar[c];
  }
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float ww = w ? w[c] : 1.0f, bb = b ? b[c] : 0.0f;
  const float scale = ww * invstd;
  coef[c] = scale;
  coef[C + c] = bb - (float)mean * scale;
  if (training) {
    if (smean) { smean[c] = (float)mean; sinvstd[c] = invstd; }
    // momentum < 0: torch's cumulative moving average (momentum=None), factor 1 / num_batches_tracked
    // read on the device -- the caller has already counted this pass, so there is no increment here
    // (every channel reads the same count; no host sync, so the pass can be graph-captured)
    const float mom = momentum < 0.f ? 1.0f / (float)*nbt : momentum;
    if (rmean) {
      rmean[c] = (1.0f - mom) * rmean[c] + mom * (float)mean;
      rvar[c] = (1.0f - mom) * rvar[c] + mom * (float)(var * n / (n - 1.0));
    }
    if (nbt && c == 0 && momentum >= 0.f) *nbt += 1;
  }
}

// The trunk's residual stream carried past bf16 (round 5): the block output v (f32 in the
// apply pass) is stored as its bf16 rounding y plus an 8-bit residue r = rint((v - y) * 2^15 /
// 2^e), e = the binary exponent of y (|v - y| <= half an ulp of y = 2^(e-8), so |r| <= 128,
// clamped to 127); the
// next block's skip reads y + r * 2^(e-15), i.e. the stream to ~2^-15 of its value instead of
// bf16's 2^-8, for 1 extra byte written and read per element.  The convs still read y (their
// operands are bf16 anyway).  What it buys: tools/trunk_precision.py (a CPU emulation of the
// trunk's storage points) and tests/test_mmbt_gpu.py.
static __device__ __forceinline__ float bn_res_scale(float y) {  // 2^(e - 15), 0 for y == 0 / denormal
  return __uint_as_float(__float_as_uint(y) & 0x7f800000u) * (1.0f / 32768.0f);
}
static __device__ __forceinline__ int8_t bn_res_encode(float v, float y) {
  const uint32_t eb = __float_as_uint(y) & 0x7f800000u;
  if (eb == 0u || eb >= (254u << 23)) return 0;
  const float inv = __uint_as_float((254u << 23) - eb);  // 2^-e
  const float q = (v - y) * inv * 32768.0f;
  return (int8_t)(int)rintf(fminf(fmaxf(q, -127.0f), 127.0f));
}

template <bool SKIP, bool RELU, bool MASK, bool RIN, bool ROUT>
__global__ __launch_bounds__(BN_THREADS) void bn_apply_kernel(const bf16* __restrict__ X, const bf16* __restrict__ S,
                                                               bf16* __restrict__ Y, int64_t rows, int C, int CH,
                                                               int64_t rows_per_blk, const float* __restrict__ coef,
                                                               uint8_t* __restrict__ M, const int8_t* __restrict__ SR,
                                                               int8_t* __restrict__ YR) {
  const BnGeom g = bn_geom(CH, rows, rows_per_blk);
  if (g.rs >= g.rpi) return;
  float sc[8], sh[8];
  {
    const float4 a0 = *(const float4*)(coef + g.c0), a1 = *(const float4*)(coef + g.c0 + 4);
    const float4 b0 = *(const float4*)(coef + C + g.c0), b1 = *(const float4*)(coef + C + g.c0 + 4);
    sc[0] = a0.x; sc[1] = a0.y; sc[2] = a0.z; sc[3] = a0.w; sc[4] = a1.x; sc[5] = a1.y; sc[6] = a1.z; sc[7] = a1.w;
    sh[0] = b0.x; sh[1] = b0.y; sh[2] = b0.z; sh[3] = b0.w; sh[4] = b1.x; sh[5] = b1.y; sh[6] = b1.z; sh[7] = b1.w;
  }
#pragma unroll 4
  for (int64_t r = g.r0 + g.rs; r < g.r1; r += g.rpi) {
    const int64_t o = r * C + g.c0;
    const bf16x8 x = *(const bf16x8*)(X + o);
    bf16x8 sk;
    if (SKIP) sk = *(const bf16x8*)(S + o);
    uint2 sr = make_uint2(0u, 0u);
    if (SKIP && RIN) sr = *(const uint2*)(SR + o);
    bf16x8 y;
    uint32_t bits = 0;
    uint32_t yr[2] = {0u, 0u};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = fmaf(bf2f(x[e]), sc[e], sh[e]);
      if (SKIP) {
        const float s = bf2f(sk[e]);
        v += s;
        if (RIN) {
          const int8_t q = (int8_t)(((e < 4 ? sr.x : sr.y) >> (8 * (e & 3))) & 0xffu);
          v = fmaf((float)q, bn_res_scale(s), v);
        }
      }
      if (RELU) v = fmaxf(v, 0.f);
      y[e] = f2bf(v);
      if (MASK) bits |= (bf2f(y[e]) > 0.f ? 1u : 0u) << e;
      if (ROUT) yr[e >> 2] |= (uint32_t)(uint8_t)bn_res_encode(v, bf2f(y[e])) << (8 * (e & 3));
    }
    *(bf16x8*)(Y + o) = y;
    if (MASK) M[o >> 3] = (uint8_t)bits;
    if (ROUT) *(uint2*)(YR + o) = make_uint2(yr[0], yr[1]);
  }
}

// g = dY * [Y > 0] from the ReLU mask byte (MASK), from Y (RELU only), or dY
template <bool RELU, bool MASK>
static __device__ __forceinline__ void bn_relu_grad(const bf16* __restrict__ dY, const bf16* __restrict__ Y,
                                                    const uint8_t* __restrict__ M, int64_t o, float (&gv)[8]) {
  const bf16x8 dy = *(const bf16x8*)(dY + o);
  if (RELU && MASK) {
    const uint32_t bits = M[o >> 3];
#pragma unroll
    for (int e = 0; e < 8; ++e) gv[e] = ((bits >> e) & 1u) ? bf2f(dy[e]) : 0.f;
  } else if (RELU) {
    const bf16x8 y = *(const bf16x8*)(Y + o);
#pragma unroll
    for (int e = 0; e < 8; ++e) gv[e] = bf2f(y[e]) > 0.f ? bf2f(dy[e]) : 0.f;
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) gv[e] = bf2f(dy[e]);
  }
}

// backward reduce: part = {sum g, sum g*(x-mean)},  g = dY * [Y > 0] (RELU)
template <bool RELU, bool MASK>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_reduce_kernel(const bf16* __restrict__ dY,
                                                                    const bf16* __restrict__ Y,
                                                                    const uint8_t* __restrict__ M,
                                                                    const bf16* __restrict__ X, int64_t rows, int C,
                                                                    int CH, int64_t rows_per_blk,
                                                                    const float* __restrict__ smean,
                                                                    float2* __restrict__ part) {
  const BnGeom g = bn_geom(CH, rows, rows_per_blk);
  float s[8], q[8], mu[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s[e] = 0.f; q[e] = 0.f; }
  if (g.rs < g.rpi) {
    const float4 m0 = *(const float4*)(smean + g.c0), m1 = *(const float4*)(smean + g.c0 + 4);
    mu[0] = m0.x; mu[1] = m0.y; mu[2] = m0.z; mu[3] = m0.w; mu[4] = m1.x; mu[5] = m1.y; mu[6] = m1.z; mu[7] = m1.w;
#pragma unroll 4
    for (int64_t r = g.r0 + g.rs; r < g.r1; r += g.rpi) {
      const int64_t o = r * C + g.c0;
      const bf16x8 x = *(const bf16x8*)(X + o);
      float gv[8];
      bn_relu_grad<RELU, MASK>(dY, Y, M, o, gv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s[e] += gv[e];
        q[e] = fmaf(gv[e], bf2f(x[e]) - mu[e], q[e]);
      }
    }
  }
  bn_block_reduce(g, C, s, q, part);
}

// coef = {k1, k2, k0}: dx = k1*g + k2*x + k0 ; dweight += dgamma, dbias += dbeta
// (gsum: the exchanged cross-rank sums; dweight / dbias were accumulated from the local ones)
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_finalize_kernel(const float2* __restrict__ part, int nparts,
                                                                      const double* __restrict__ gsum,
                                                                      int64_t rows, int C, const float* w,
                                                                      const float* smean, const float* sinvstd,
                                                                      float* dw, float* db, float* __restrict__ coef) {
  int c;
  double dbeta, sgx, n = (double)rows;
  if (!bn_channel_sums(part, nparts, gsum, C, c, dbeta, sgx, &n)) return;
  const double invstd = sinvstd[c], mean = smean[c];
  const double dgamma = sgx * invstd;
  const double a = (w ? (double)w[c] : 1.0) * invstd;
  const double k2 = -a * invstd * dgamma / n;
  coef[c] = (float)a;
  coef[C + c] = (float)k2;
  coef[2 * C + c] = (float)(-a * dbeta / n - k2 * mean);
  if (dw) dw[c] += (float)dgamma;
  if (db) db[c] += (float)dbeta;
}

template <bool RELU, bool MASK, bool DSKIP>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_apply_kernel(const bf16* __restrict__ dY,
                                                                   const bf16* __restrict__ Y,
                                                                   const uint8_t* __restrict__ M,
                                                                   const bf16* __restrict__ X, int64_t rows, int C,
                                                                   int CH, int64_t rows_per_blk,
                                                                   const float* __restrict__ coef,
                                                                   bf16* __restrict__ dX, bf16* __restrict__ dS) {
  const BnGeom g = bn_geom(CH, rows, rows_per_blk);
  if (g.rs >= g.rpi) return;
  float k1[8], k2[8], k0[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    k1[e] = coef[g.c0 + e];
    k2[e] = coef[C + g.c0 + e];
    k0[e] = coef[2 * C + g.c0 + e];
  }
#pragma unroll 4
  for (int64_t r = g.r0 + g.rs; r < g.r1; r += g.rpi) {
    const int64_t o = r * C + g.c0;
    const bf16x8 x = *(const bf16x8*)(X + o);
    float gv[8];
    bn_relu_grad<RELU, MASK>(dY, Y, M, o, gv);
    bf16x8 dx, gs;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      dx[e] = f2bf(fmaf(k1[e], gv[e], fmaf(k2[e], bf2f(x[e]), k0[e])));
      gs[e] = f2bf(gv[e]);
    }
    *(bf16x8*)(dX + o) = dx;
    if (DSKIP) *(bf16x8*)(dS + o) = gs;
  }
}

// ------------------------------------------------------------------------------ launchers
struct BnGrid {
  int CH;
  int64_t rpb;
  dim3 grid;
};
// channel chunk: the largest of 512, 256, ..., 8 dividing C.  Rows per block: the tensor
// split into ~BN_TARGET_BLOCKS blocks, but each block between BN_MIN and 64 K elements (a
// multiple of the rows per iteration), and few enough row blocks that blocks x C partial
// pairs fit BN_MAX_PART_ELEMS.  (A fixed 64 K elements per block left the trunk's small
// tensors on 24-200 blocks -- e.g. layer3's 256-channel 14x14 maps at batch 32 -- i.e. on
// a tenth of the CUs, latency-bound.)
// The 8 K-element floor (was 4 K) halves the block partials the finalize sums on the small
// maps: batch-32 BN 6.08 -> 5.41-5.47 ms per step, batch 256 unchanged
// (profiles/r3_bn_grid_sweep.txt).
static BnGrid bn_grid(int64_t rows, int C) {
  const int64_t target = 1024, min_elems = 8192;
  BnGrid g;
  g.CH = 512;
  while (C % g.CH) g.CH >>= 1;
  const int rpi = BN_THREADS / (g.CH / 8);
  int64_t per = rows * (int64_t)C / target;
  per = per < min_elems ? min_elems : per > BN_ELEMS_PER_BLOCK ? BN_ELEMS_PER_BLOCK : per;
  int64_t rpb = (per + g.CH - 1) / g.CH;
  rpb = (rpb + rpi - 1) / rpi * rpi;
  const int64_t max_parts = BN_MAX_PART_ELEMS / C;
  if ((rows + rpb - 1) / rpb > max_parts) rpb = ((rows + max_parts - 1) / max_parts + rpi - 1) / rpi * rpi;
  g.rpb = rpb;
  g.grid = dim3((unsigned)((rows + rpb - 1) / rpb), (unsigned)(C / g.CH));
  return g;
}

int64_t batchnorm_ws_bytes(int64_t C) { return BN_MAX_PART_ELEMS * 8 + ((3 * C + 3) & ~3) * 4; }

void batchnorm_fwd_launch(const BnFwdParams& q, hipStream_t s) {
  const BnGrid G = bn_grid(q.rows, q.C);
  float* coef = (float*)q.ws;
  // the statistics: the producing conv's table (q.parts, its epilogue's 64-row blocks), or this
  // launch's own stats pass into the workspace
  const float2* part = q.parts ? (const float2*)q.parts : (const float2*)(coef + ((3 * q.C + 3) & ~3));
  const int nparts = q.parts ? (int)q.nparts : (int)G.grid.x;
  const dim3 fin((q.C + BN_FIN_CH - 1) / BN_FIN_CH);
  if (q.training && !q.gsum && !q.parts)
    hipLaunchKernelGGL(bn_stats_kernel, G.grid, dim3(BN_THREADS), 0, s, q.X, q.rows, q.C, G.CH, G.rpb,
                       (float2*)part);
  if (q.lsum) {  // cross-rank statistics, first half: the local sums for the exchange
    hipLaunchKernelGGL(bn_local_sums_kernel, fin, dim3(BN_THREADS), 0, s, part, nparts, q.rows, q.C, q.lsum,
                       nullptr, nullptr, nullptr);
    return;
  }
  hipLaunchKernelGGL(bn_fwd_finalize_kernel, fin, dim3(BN_THREADS), 0, s, part, nparts, q.gsum, q.rows, q.C,
                     q.w, q.b, q.rmean, q.rvar, q.training, q.momentum, q.eps, q.smean, q.sinvstd, q.nbt, coef);
  const bool sk = q.skip != nullptr, mk = q.relu && q.mask != nullptr;
#define BN_APPLY(SK, RL, MK, RI, RO)                                                                           \
  hipLaunchKernelGGL((bn_apply_kernel<SK, RL, MK, RI, RO>), G.grid, dim3(BN_THREADS), 0, s, q.X, q.skip, q.Y,    \
                     q.rows, q.C, G.CH, G.rpb, coef, q.mask, q.skip_res, q.y_res)
  if (q.y_res) {  // the residual stream's producers (capi checks the combinations)
    if (sk && mk) BN_APPLY(true, true, true, true, true);       // bn3 (train): skip + stream residue
    else if (sk && q.relu) BN_APPLY(true, true, false, true, true);  // bn3 (eval)
    else BN_APPLY(false, false, false, false, true);            // the downsample's BatchNorm
  }
  else if (sk && mk) BN_APPLY(true, true, true, false, false);
  else if (sk && q.relu) BN_APPLY(true, true, false, false, false);
  else if (sk) BN_APPLY(true, false, false, false, false);
  else if (mk) BN_APPLY(false, true, true, false, false);
  else if (q.relu) BN_APPLY(false, true, false, false, false);
  else BN_APPLY(false, false, false, false, false);
#undef BN_APPLY
}

void batchnorm_bwd_launch(const BnBwdParams& q, hipStream_t s) {
  const BnGrid G = bn_grid(q.rows, q.C);
  float* coef = (float*)q.ws;
  // the reduction: the table of the product that formed dY (q.parts), or this launch's own pass
  const float2* part = q.parts ? (const float2*)q.parts : (const float2*)(coef + ((3 * q.C + 3) & ~3));
  const int nparts = q.parts ? (int)q.nparts : (int)G.grid.x;
  const bool mk = q.relu && q.mask != nullptr;
  const dim3 fin((q.C + BN_FIN_CH - 1) / BN_FIN_CH);
  if (!q.gsum && !q.parts) {
#define BN_BREDUCE(RL, MK)                                                                                   \
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<RL, MK>), G.grid, dim3(BN_THREADS), 0, s, q.dY, q.Y, q.mask, q.X, \
                     q.rows, q.C, G.CH, G.rpb, q.smean, (float2*)part)
    if (mk) BN_BREDUCE(true, true);
    else if (q.relu) BN_BREDUCE(true, false);
    else BN_BREDUCE(false, false);
#undef BN_BREDUCE
  }
  if (q.lsum) {  // cross-rank statistics, first half: local sums (+ this rank's dweight / dbias)
    hipLaunchKernelGGL(bn_local_sums_kernel, fin, dim3(BN_THREADS), 0, s, part, nparts, q.rows, q.C, q.lsum,
                       q.sinvstd, q.dw, q.db);
    return;
  }
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, fin, dim3(BN_THREADS), 0, s, part, nparts, q.gsum, q.rows, q.C,
                     q.w, q.smean, q.sinvstd, q.gsum ? nullptr : q.dw, q.gsum ? nullptr : q.db, coef);
  const bool ds = q.dS != nullptr;
#define BN_BAPPLY(RL, MK, DS)                                                                                     \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<RL, MK, DS>), G.grid, dim3(BN_THREADS), 0, s, q.dY, q.Y, q.mask, q.X,  \
                     q.rows, q.C, G.CH, G.rpb, coef, q.dX, q.dS)
  if (mk && ds) BN_BAPPLY(true, true, true);
  else if (mk) BN_BAPPLY(true, true, false);
  else if (q.relu && ds) BN_BAPPLY(true, false, true);
  else if (q.relu) BN_BAPPLY(true, false, false);
  else if (ds) BN_BAPPLY(false, false, true);
  else BN_BAPPLY(false, false, false);
#undef BN_BAPPLY
}

}  // namespace mmu
