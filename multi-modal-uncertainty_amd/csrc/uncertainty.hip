// Ensemble / MC-dropout uncertainty reduction (gfx950).
//
// North-star metrics.  Convention of the reference analysis code:
// softmax per member / pass, then the mean over members (notebooks/food101_robustness.py:25-36,
// notebooks/utils.py:22-23).  One 128-thread block per sample reduces R = K*T logit rows.
#include "mmu_common.h"
#include "mmu_internal.h"

namespace mmu {

__global__ __launch_bounds__(128) void uncertainty_kernel(const float* __restrict__ logits, const int64_t* __restrict__ y,
                                                          int64_t R, int64_t C, float* __restrict__ p_bar,
                                                          float* __restrict__ nll, float* __restrict__ conf,
                                                          float* __restrict__ correct) {
  __shared__ float red[2];
  __shared__ float acc[1024];
  const int64_t s = blockIdx.x;
  const int t = threadIdx.x;
  for (int c = t; c < C; c += 128) acc[c] = 0.f;
  for (int64_t r = 0; r < R; ++r) {
    const float* z = logits + (s * R + r) * C;
    float mx = -__builtin_huge_valf();
    for (int c = t; c < C; c += 128) mx = fmaxf(mx, z[c]);
    mx = wave_max(mx);
    if ((t & 63) == 0) red[t >> 6] = mx;
    __syncthreads();
    mx = fmaxf(red[0], red[1]);
    __syncthreads();
    float sm = 0.f;
    for (int c = t; c < C; c += 128) sm += __expf(z[c] - mx);
    sm = wave_sum(sm);
    if ((t & 63) == 0) red[t >> 6] = sm;
    __syncthreads();
    const float inv = 1.0f / (red[0] + red[1]);
    __syncthreads();
    for (int c = t; c < C; c += 128) acc[c] += __expf(z[c] - mx) * inv;
  }
  __syncthreads();
  const float invR = 1.0f / (float)R;
  float best = -1.f;
  int arg = 0;
  for (int c = t; c < C; c += 128) {
    const float pb = acc[c] * invR;
    p_bar[s * C + c] = pb;
    if (pb > best) { best = pb; arg = c; }
  }
  // argmax: first index of the maximum (ties -> lowest class, like torch/numpy argmax)
  for (int o = 32; o > 0; o >>= 1) {
    float ob = __shfl_xor(best, o, 64);
    int oa = __shfl_xor(arg, o, 64);
    if (ob > best || (ob == best && oa < arg)) { best = ob; arg = oa; }
  }
  __shared__ float bb[2];
  __shared__ int ba[2];
  if ((t & 63) == 0) { bb[t >> 6] = best; ba[t >> 6] = arg; }
  __syncthreads();
  if (t == 0) {
    float b0 = bb[0];
    int a0 = ba[0];
    if (bb[1] > b0 || (bb[1] == b0 && ba[1] < a0)) { b0 = bb[1]; a0 = ba[1]; }
    const int64_t yy = y[s];
    nll[s] = -logf(fmaxf(acc[yy] * invR, 1e-12f));
    conf[s] = b0;
    correct[s] = a0 == yy ? 1.f : 0.f;
  }
}

// bin b holds conf in (b/n, (b+1)/n]; conf == 0 -> bin 0
__global__ void ece_bins_kernel(const float* __restrict__ conf, const float* __restrict__ correct, int64_t S,
                                int n_bins, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= S) return;
  int b = (int)ceilf(conf[i] * n_bins) - 1;
  b = b < 0 ? 0 : (b >= n_bins ? n_bins - 1 : b);
  atomicAdd(out + 3 * b, 1.f);
  atomicAdd(out + 3 * b + 1, conf[i]);
  atomicAdd(out + 3 * b + 2, correct[i]);
}

void uncertainty_launch(const float* logits, const int64_t* y, int64_t S, int64_t R, int64_t C, float* p_bar,
                        float* nll, float* conf, float* correct, hipStream_t s) {
  hipLaunchKernelGGL(uncertainty_kernel, dim3((unsigned)S), dim3(128), 0, s, logits, y, R, C, p_bar, nll, conf, correct);
}

void ece_bins_launch(const float* conf, const float* correct, int64_t S, int64_t n_bins, float* out, hipStream_t s) {
  (void)hipMemsetAsync(out, 0, sizeof(float) * 3 * n_bins, s);
  hipLaunchKernelGGL(ece_bins_kernel, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, s, conf, correct, S,
                     (int)n_bins, out);
}

}  // namespace mmu
