// Fused multi-tensor BertAdam (gfx950).
//
// pytorch_pretrained_bert 0.6.x BertAdam as constructed at train.py:142-147:
// per-tensor clip_grad_norm_(p, max_grad_norm), m/v moments without bias
// correction, decoupled weight decay added to the update, lr * warmup_linear(
// step / t_total) with the step read BEFORE its increment.  Three launches over the
// flat f32 parameter / gradient / moment buffers (HBM-bound, ~28 B per element):
//   1. per-chunk sum of squares of the gradient
//   2. per tensor: norm -> clip coefficient (x grad_scale), scheduled lr, step += 1
//   3. per chunk: moment + parameter update, optional bf16 weight copy for the GEMMs
// Tensor table (7 int64 each): offset, numel, group, bf16_offset, active,
// first_chunk, n_chunks.  Chunk table (3 int64 each): tensor, start, len.
#include "mmu_common.h"
#include "mmu_internal.h"

namespace mmu {

struct AdamDev {
  float *params, *m, *v;
  const float* grads;
  bf16* bf16_copy;
  const int64_t* table;
  const int64_t* chunks;
  int32_t* steps;
  int64_t n_tensors, n_chunks;
  float lr_decay, lr_nodecay, wd, warmup, t_total, b1, b2, eps, max_grad_norm, grad_scale;
  float* ws;  // [n_chunks] partial sq-norms, then [n_tensors][2] (coef, lr_eff)
};

__global__ __launch_bounds__(256) void adam_sqnorm_kernel(AdamDev a) {
  const int64_t ci = blockIdx.x;
  const int64_t tid = a.chunks[3 * ci], start = a.chunks[3 * ci + 1], len = a.chunks[3 * ci + 2];
  if (!a.table[7 * tid + 4]) {
    if (threadIdx.x == 0) a.ws[ci] = 0.f;
    return;
  }
  const float* g = a.grads + a.table[7 * tid] + start;
  float s = 0.f;
  // 16-B loads over the aligned body, scalar head (to 16-B alignment) and tail
  const int64_t head = ((16 - ((uintptr_t)g & 15)) & 15) / 4 < len ? ((16 - ((uintptr_t)g & 15)) & 15) / 4 : len;
  for (int64_t i = threadIdx.x; i < head; i += 256) { const float x = g[i]; s += x * x; }
  const int64_t nv = (len - head) / 4;
  const float4* g4 = (const float4*)(g + head);
  for (int64_t i = threadIdx.x; i < nv; i += 256) {
    const float4 x = g4[i];
    s += x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
  }
  for (int64_t i = head + 4 * nv + threadIdx.x; i < len; i += 256) { const float x = g[i]; s += x * x; }
  __shared__ float red[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) a.ws[ci] = red[0] + red[1] + red[2] + red[3];
}

__global__ void adam_coef_kernel(AdamDev a) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= a.n_tensors) return;
  const int64_t* T = a.table + 7 * t;
  float* out = a.ws + a.n_chunks + 2 * t;
  if (!T[4]) { out[0] = 1.f; out[1] = 0.f; return; }
  double sq = 0.0;
  for (int64_t c = T[5]; c < T[5] + T[6]; ++c) sq += a.ws[c];
  // the optimizer's gradient is grads * grad_scale (data parallelism's 1/world): its norm
  // scales with it, and the update multiplies by grad_scale * clip coefficient
  const double nrm = sqrt(sq) * (double)a.grad_scale;
  double coef = 1.0;
  if (a.max_grad_norm > 0.f) {
    const double cc = a.max_grad_norm / (nrm + 1e-6);
    if (cc < 1.0) coef = cc;
  }
  coef *= (double)a.grad_scale;
  const int32_t st = a.steps[t];
  double sched = 1.0;
  if (a.t_total > 0.f) {
    const double x = (double)st / a.t_total, w = a.warmup;
    sched = x < w ? x / w : fmax((x - 1.0) / (w - 1.0), 0.0);
  }
  const double lr = T[2] == 0 ? a.lr_decay : a.lr_nodecay;
  out[0] = (float)coef;
  out[1] = (float)(lr * sched);
  a.steps[t] = st + 1;
}

__global__ __launch_bounds__(256) void adam_update_kernel(AdamDev a) {
  const int64_t ci = blockIdx.x;
  const int64_t tid = a.chunks[3 * ci], start = a.chunks[3 * ci + 1], len = a.chunks[3 * ci + 2];
  const int64_t* T = a.table + 7 * tid;
  if (!T[4]) return;
  const float coef = a.ws[a.n_chunks + 2 * tid], lr = a.ws[a.n_chunks + 2 * tid + 1];
  const float wd = T[2] == 0 ? a.wd : 0.f;
  const int64_t off = T[0] + start;
  float* p = a.params + off;
  float* m = a.m + off;
  float* v = a.v + off;
  const float* g = a.grads + off;
  bf16* cp = T[3] >= 0 ? a.bf16_copy + T[3] + start : nullptr;
  const float b1 = a.b1, b2 = a.b2, c1 = 1.f - a.b1, c2 = 1.f - a.b2, eps = a.eps;
  auto one = [&](float pi, float gi, float mi, float vi, float& po, float& mo, float& vo) {
    const float gr = gi * coef;
    mo = b1 * mi + c1 * gr;
    vo = b2 * vi + c2 * gr * gr;
    float u = mo / (sqrtf(vo) + eps);
    if (wd > 0.f) u += wd * pi;
    po = pi - lr * u;
  };
  // 16-B accesses (8-B bf16 stores) when the chunk's f32 offset and its bf16 copy offset are
  // multiples of 4 elements (every tensor but a few odd-sized biases), else scalar
  const bool vec = (off & 3) == 0 && (!cp || ((T[3] + start) & 3) == 0);
  const int64_t nv = vec ? len / 4 : 0;
  for (int64_t i = threadIdx.x; i < nv; i += 256) {
    const float4 pv = ((const float4*)p)[i], gv = ((const float4*)g)[i];
    const float4 mv = ((const float4*)m)[i], vv = ((const float4*)v)[i];
    float4 po, mo, vo;
    one(pv.x, gv.x, mv.x, vv.x, po.x, mo.x, vo.x);
    one(pv.y, gv.y, mv.y, vv.y, po.y, mo.y, vo.y);
    one(pv.z, gv.z, mv.z, vv.z, po.z, mo.z, vo.z);
    one(pv.w, gv.w, mv.w, vv.w, po.w, mo.w, vo.w);
    ((float4*)m)[i] = mo;
    ((float4*)v)[i] = vo;
    ((float4*)p)[i] = po;
    if (cp) ((bf16x4*)cp)[i] = bf16x4{f2bf(po.x), f2bf(po.y), f2bf(po.z), f2bf(po.w)};
  }
  for (int64_t i = 4 * nv + threadIdx.x; i < len; i += 256) {
    float po, mo, vo;
    one(p[i], g[i], m[i], v[i], po, mo, vo);
    m[i] = mo;
    v[i] = vo;
    p[i] = po;
    if (cp) cp[i] = f2bf(po);
  }
}

int bertadam_launch(const AdamParams& P, hipStream_t s, const char** err) {
  (void)err;
  AdamDev a;
  a.params = P.params; a.m = P.m; a.v = P.v; a.grads = P.grads; a.bf16_copy = P.bf16_copy;
  a.table = P.table; a.steps = P.steps; a.n_tensors = P.n_tensors;
  // the chunk table follows the tensor table: caller packs [7*n_tensors | 3*n_chunks]; total = n_chunks
  a.chunks = P.table + 7 * P.n_tensors;
  a.n_chunks = P.total;
  a.lr_decay = P.lr_decay; a.lr_nodecay = P.lr_nodecay; a.wd = P.wd; a.warmup = P.warmup;
  a.t_total = P.t_total; a.b1 = P.b1; a.b2 = P.b2; a.eps = P.eps; a.max_grad_norm = P.max_grad_norm;
  a.grad_scale = P.grad_scale;
  a.ws = P.ws;
  hipLaunchKernelGGL(adam_sqnorm_kernel, dim3((unsigned)a.n_chunks), dim3(256), 0, s, a);
  hipLaunchKernelGGL(adam_coef_kernel, dim3((unsigned)((a.n_tensors + 255) / 256)), dim3(256), 0, s, a);
  hipLaunchKernelGGL(adam_update_kernel, dim3((unsigned)a.n_chunks), dim3(256), 0, s, a);
  return 0;
}

}  // namespace mmu
