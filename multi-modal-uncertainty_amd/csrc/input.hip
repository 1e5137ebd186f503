// Input pipeline tail on the GPU.
//
// The reference's image transform (src/dataset.py:488-498) ends in ToTensor + Normalize on
// the host: every 224x224 crop leaves the DataLoader worker as 602 KB of f32.  Here the
// workers stop after decode / resize / center-crop and ship the crop as uint8 HWC (150 KB);
// this kernel does  x = (u8 / 255 - mean[c]) / std[c]  on the device and writes the
// channels-last [B, 3, 224, 224] image the trunk consumes (NHWC with C = 3 is the same
// bytes as the HWC crops, so the kernel is a flat elementwise map; channel = index % 3).
// HBM-bound: 1 B read + 2 or 4 B written per element.
#include "mmu_common.h"
#include "mmu_internal.h"

namespace mmu {

constexpr int IMG_PER_THREAD = 16;  // one 16-B load of u8

template <bool OUT_BF16>
__global__ __launch_bounds__(256) void image_normalize_kernel(const uint8_t* __restrict__ in, int64_t n,
                                                              float s0, float s1, float s2, float b0, float b1,
                                                              float b2, void* __restrict__ out) {
  const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * IMG_PER_THREAD;
  if (i0 >= n) return;
  // per-channel affine y = u8 * s[c] + b[c] with s = 1 / (255 std), b = -mean / std
  const float sc[3] = {s0, s1, s2}, bc[3] = {b0, b1, b2};
  uint8_t v[IMG_PER_THREAD];
  if (i0 + IMG_PER_THREAD <= n) {
    *(uint4*)v = *(const uint4*)(in + i0);
  } else {
#pragma unroll
    for (int j = 0; j < IMG_PER_THREAD; ++j) v[j] = i0 + j < n ? in[i0 + j] : 0;
  }
  const int c0 = (int)(i0 % 3);
  float y[IMG_PER_THREAD];
#pragma unroll
  for (int j = 0; j < IMG_PER_THREAD; ++j) {
    const int c = (c0 + j) % 3;
    y[j] = fmaf((float)v[j], sc[c], bc[c]);
  }
  if (i0 + IMG_PER_THREAD <= n) {
    if (OUT_BF16) {
      bf16x8 o0, o1;
#pragma unroll
      for (int j = 0; j < 8; ++j) { o0[j] = f2bf(y[j]); o1[j] = f2bf(y[8 + j]); }
      bf16x8* d = (bf16x8*)((bf16*)out + i0);
      d[0] = o0;
      d[1] = o1;
    } else {
      float4* d = (float4*)((float*)out + i0);
#pragma unroll
      for (int j = 0; j < 4; ++j) d[j] = make_float4(y[4 * j], y[4 * j + 1], y[4 * j + 2], y[4 * j + 3]);
    }
  } else {
    for (int j = 0; j < IMG_PER_THREAD && i0 + j < n; ++j) {
      if (OUT_BF16) ((bf16*)out)[i0 + j] = f2bf(y[j]);
      else ((float*)out)[i0 + j] = y[j];
    }
  }
}

void image_normalize_launch(const uint8_t* in, int64_t n, const float* mean, const float* stdv, void* out,
                            bool out_bf16, hipStream_t s) {
  float sc[3], bc[3];
  for (int c = 0; c < 3; ++c) {
    sc[c] = 1.0f / (255.0f * stdv[c]);
    bc[c] = -mean[c] / stdv[c];
  }
  const int64_t threads = (n + IMG_PER_THREAD - 1) / IMG_PER_THREAD;
  const dim3 grid((unsigned)((threads + 255) / 256));
  if (out_bf16)
    hipLaunchKernelGGL(image_normalize_kernel<true>, grid, dim3(256), 0, s, in, n, sc[0], sc[1], sc[2], bc[0], bc[1],
                       bc[2], out);
  else
    hipLaunchKernelGGL(image_normalize_kernel<false>, grid, dim3(256), 0, s, in, n, sc[0], sc[1], sc[2], bc[0], bc[1],
                       bc[2], out);
}

}  // namespace mmu
