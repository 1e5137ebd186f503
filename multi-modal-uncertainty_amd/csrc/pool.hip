// MaxPool2d(kernel 3, stride 2, padding 1) of the ResNet-152 stem (torchvision resnet
// child 3, src/mmbt.py:19-21) on the channels-last bf16 map, forward and backward (gfx950).
//
// PyTorch's NHWC max pool stores an int64 flat index per output element (8 B) and its
// backward runs as its own scatter pass; here the forward keeps the argmax as ONE BYTE per
// output element (its position 0..8 in the 3x3 window) and the backward is a gather: every
// input pixel sums dY over the <= 2 x 2 windows that cover it and chose it.  Semantics as
// torch's kernels: windows clipped to the image, maximum scanned row-major with
// `v > max || isnan(v)` (the FIRST maximal element wins ties; NaN propagates), the gradient
// of a window goes to its argmax only, accumulated in f32 and rounded to bf16 once.
// A thread owns 8 channels (16-B accesses) of one output (forward) or input (backward) pixel.
#include "mmu_common.h"
#include "mmu_internal.h"

namespace mmu {

__global__ __launch_bounds__(256) void maxpool3s2_fwd_kernel(const bf16* __restrict__ x, int64_t B, int H, int W,
                                                             int C, int OH, int OW, bf16* __restrict__ y,
                                                             uint8_t* __restrict__ am) {
  const int c8 = C >> 3;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;  // over B * OH * OW * C/8
  if (idx >= B * OH * OW * c8) return;
  const int cg = (int)(idx % c8);
  const int64_t pix = idx / c8;
  const int ox = (int)(pix % OW), oy = (int)((pix / OW) % OH);
  const int64_t b = pix / ((int64_t)OW * OH);
  float mx[8];
  uint32_t arg[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { mx[e] = -__builtin_huge_valf(); arg[e] = 0xFF; }
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int iy = 2 * oy - 1 + kh;
    if (iy < 0 || iy >= H) continue;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int ix = 2 * ox - 1 + kw;
      if (ix < 0 || ix >= W) continue;
      const bf16x8 v = *(const bf16x8*)(x + (((b * H + iy) * W + ix) * C) + 8 * cg);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float f = bf2f(v[e]);
        if (arg[e] == 0xFF || f > mx[e] || __builtin_isnan(f)) {  // the first in-image element seeds
          mx[e] = f;
          arg[e] = (uint32_t)(3 * kh + kw);
        }
      }
    }
  }
  bf16x8 o;
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = f2bf(mx[e]);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    lo |= arg[e] << (8 * e);
    hi |= arg[4 + e] << (8 * e);
  }
  *(bf16x8*)(y + pix * C + 8 * cg) = o;
  *(uint2*)(am + pix * C + 8 * cg) = make_uint2(lo, hi);
}

__global__ __launch_bounds__(256) void maxpool3s2_bwd_kernel(const bf16* __restrict__ dy,
                                                             const uint8_t* __restrict__ am, int64_t B, int H,
                                                             int W, int C, int OH, int OW, bf16* __restrict__ dx) {
  const int c8 = C >> 3;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;  // over B * H * W * C/8
  if (idx >= B * H * W * c8) return;
  const int cg = (int)(idx % c8);
  const int64_t pix = idx / c8;
  const int ix = (int)(pix % W), iy = (int)((pix / W) % H);
  const int64_t b = pix / ((int64_t)W * H);
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  // the windows covering (iy, ix): 2 oy - 1 <= iy <= 2 oy + 1, same for x
  const int oy0 = iy >> 1, oy1 = (iy + 1) >> 1, ox0 = ix >> 1, ox1 = (ix + 1) >> 1;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int oy = a ? oy1 : oy0;
    if ((a && oy1 == oy0) || oy >= OH) continue;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int ox = c ? ox1 : ox0;
      if ((c && ox1 == ox0) || ox >= OW) continue;
      const uint32_t me = (uint32_t)(3 * (iy - (2 * oy - 1)) + (ix - (2 * ox - 1)));
      const int64_t o = ((b * OH + oy) * OW + ox) * C + 8 * cg;
      const uint2 wsel = *(const uint2*)(am + o);
      const bf16x8 g = *(const bf16x8*)(dy + o);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t sel = ((e < 4 ? wsel.x : wsel.y) >> (8 * (e & 3))) & 0xFF;
        if (sel == me) acc[e] += bf2f(g[e]);
      }
    }
  }
  bf16x8 out;
#pragma unroll
  for (int e = 0; e < 8; ++e) out[e] = f2bf(acc[e]);
  *(bf16x8*)(dx + pix * C + 8 * cg) = out;
}

void maxpool3s2_fwd_launch(const bf16* x, int64_t B, int H, int W, int C, int OH, int OW, bf16* y, uint8_t* am,
                           hipStream_t s) {
  const int64_t n = B * OH * OW * (C / 8);
  hipLaunchKernelGGL(maxpool3s2_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, B, H, W, C, OH,
                     OW, y, am);
}

void maxpool3s2_bwd_launch(const bf16* dy, const uint8_t* am, int64_t B, int H, int W, int C, int OH, int OW,
                           bf16* dx, hipStream_t s) {
  const int64_t n = B * H * W * (C / 8);
  hipLaunchKernelGGL(maxpool3s2_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, dy, am, B, H, W, C,
                     OH, OW, dx);
}

}  // namespace mmu
