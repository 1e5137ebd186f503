// Internal launcher interfaces between capi.cpp and the .hip translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/mmu.h"

typedef __bf16 bf16;

namespace mmu {

// mmu_set_seed_offset's device counter (capi.hip), copied into every dropout launch
extern const uint64_t* g_seed_off;

struct GemmParams {
  const bf16* A;
  const bf16* B;
  void* C;
  int64_t lda, ldb, ldc, M, N, K, sA, sB, sC;
  int tiles_m, tiles_n;
  int group_m;  // tile-order group height (gemm.hip tile_of)
  // epilogue (flattened mmu_epilogue)
  int kind, accumulate;
  const float* bias;
  int64_t bias_bstride;
  const void* residual;
  int64_t ldr, res_bstride;
  void* aux;
  int64_t ldx, aux_bstride;
  float* colsum;
  int64_t colsum_bstride;
  float drop_p;
  uint64_t seed;
  const uint64_t* seed_off;  // per-replay seed counter (mmu_set_seed_offset), or NULL
  // f32 residual = LN(residual rows) recomputed per element (mmu_epilogue res_ln_*)
  const float *res_ln_mean, *res_ln_rstd, *res_ln_w, *res_ln_b;
  int64_t res_ln_bstride;
  // split-K (EPI_STORE, f32 C, no bias/colsum): grid.y slices of kchunk, slabs in ws
  int splitk;
  int64_t kchunk;
  float* ws;
  // conv_ks x conv_ks (3 or 1) / stride conv_s / pad conv_pad convolutions of an NHWC map
  // [img * conv_h * conv_w pixels][conv_c] (conv_in_bytes) into conv_ho x conv_wo outputs:
  // weight gradient (gemm_convw_kernel): B[out pixel][tap * conv_c + ci] gathered;
  // forward / data gradient (gemm_conva_kernel): A[out pixel][tap * conv_c + c] gathered
  int conv_h, conv_w, conv_c, conv_ho, conv_wo, conv_ks, conv_s, conv_pad;
  int64_t conv_in_bytes;
  // STORE_BNB / ADD_RES_BNB: the BatchNorm whose dY this product forms (input rows [M][N],
  // ReLU mask [M][N/8] or null, batch mean [N]); its backward reduction table goes to colsum
  const bf16* bn_x;
  const uint8_t* bn_mask;
  const float* bn_mean;
  const uint8_t* res_mask;  // ADD_RES: residual gated by a ReLU mask [M][N/8] (ldr == N)
  // column sums (colsum, batch 1) as plain stores of per-wave-block partial rows instead of float
  // atomics: row (m_wave - cs_m0) / cs_rows of the [parts][N] table cs_part (the host folds it)
  float* cs_part;
  int64_t cs_m0;
  int cs_rows;
};
void conv3x3_wgrad_launch(const GemmParams& p, hipStream_t s);
void conv3x3_implicit_launch(const GemmParams& p, bool small, hipStream_t s);  // small: 128x128 tiles
struct StemParams {  // csrc/stem.hip
  const bf16* X;     // [n, H, W, 3]
  const bf16* Wt;    // [64][7][7][3]
  const bf16* dY;    // [n, Ho, Wo, 64] (filter gradient)
  bf16* Y;           // [n, Ho, Wo, 64] (forward)
  int n, H, W, Ho, Wo, tiles_r, tiles_c;
  int64_t n_tiles;
};
void stem_fill_geometry(StemParams& p);
int64_t stem_wgrad_ws_floats(int64_t n_tiles);
void stem_fwd_launch(const StemParams& p, hipStream_t s);
void stem_wgrad_launch(const StemParams& p, float* dW, int accumulate, float* ws, hipStream_t s);

void splitk_reduce_launch(const GemmParams& p, int batch, hipStream_t s);
void gemm_launch(const GemmParams& p, bool a_kmajor, bool b_kmajor, bool f32out, bool big, int batch, hipStream_t s);
bool gemm_wide_launch(const GemmParams& p, bool f32out, int batch, hipStream_t s);
bool splitk_epilogue_launch(const GemmParams& p, bool f32out, const float* slabs, int64_t m_base, int64_t rows,
                            int splitk, hipStream_t s);
void transpose_bf16_batched_launch(const int64_t* jobs, int n_jobs, int64_t max_rows, int64_t max_cols,
                                   hipStream_t s);
void colsum_reduce_launch(const float* part, int64_t parts, int64_t N, float* out, int acc, hipStream_t s);
constexpr int COLSUM_MULTI = 4;
struct ColsumJobs {  // (passed by value: graph-capturable)
  const float* part[COLSUM_MULTI];
  int64_t parts[COLSUM_MULTI];
  float* out[COLSUM_MULTI];
};
void colsum_reduce_multi_launch(const ColsumJobs& jobs, int n, int64_t N, int acc, hipStream_t s);
void colsum_bf16_launch(const bf16* X, int64_t M, int64_t N, int64_t ld, float* part, float* out, int acc,
                        hipStream_t s);

struct AttnParams {
  const bf16* qkv;
  int64_t ld_qkv;
  const float* keymask;
  const bf16* o;
  int64_t ld_o;
  const bf16* dout;
  int64_t ld_do;
  float* lse;
  float* delta;
  bf16* out;   // O (fwd) or dQKV (bwd)
  int64_t ld_out;
  uint64_t* dropmask;  // [batch*heads][L][ceil(L/64)] keep bits: written by fwd, read by bwd
  float* colsum;       // bwd (optional): dQKV column-sum partials, see mmu_attention_bwd
  int batch, L, heads;
  float drop_p;
  uint64_t seed;
  const uint64_t* seed_off;
};
void attention_fwd_launch(const AttnParams& p, hipStream_t s);
void attention_bwd_launch(const AttnParams& p, hipStream_t s);

void layernorm_fwd_launch(const bf16* X, const float* w, const float* b, bf16* Y, float* mean, float* rstd,
                          int64_t rows, int64_t H, float eps, int64_t group_rows, int64_t pstride, hipStream_t s);
void layernorm_fwd32_launch(const float* X, const float* w, const float* b, bf16* Y, float* Y32, float* mean,
                            float* rstd, int64_t rows, int64_t H, float eps, int64_t group_rows, int64_t pstride,
                            hipStream_t s);
void layernorm_bwd_launch(const bf16* dY, const void* X, bool x_f32, const float* mean, const float* rstd,
                          const float* w, bf16* dX, bf16* dXdrop, const bf16* dR, float drop_p, uint64_t seed,
                          const uint64_t* seed_off, float* pdw, float* pdb, float* pdbias, int64_t rows, int64_t H,
                          int64_t rows_per_part, hipStream_t s);

// FLAVA attention over the sequence (= batch) axis, flava.hip
struct SeqAttnParams {
  const bf16* qkv;
  int64_t ld_qkv;
  const bf16* o;
  int64_t ld_o;
  const bf16* dout;
  int64_t ld_do;
  bf16* out;  // O (fwd) or dQKV (bwd)
  int64_t ld_out;
  float* lse2;   // [N*heads][S] log2-sum-exp2 of the log2-scaled scores
  float* delta;  // bwd workspace [N*heads][S]
  int S, N, heads, E, D;
  float scale;
};
void seqattn_fwd_launch(const SeqAttnParams& p, hipStream_t s);
void seqattn_bwd_launch(const SeqAttnParams& p, hipStream_t s);

struct EmbedParams {
  const int64_t *ids, *seg, *txt_mask, *idx;
  const float *proj, *word, *pos, *type, *ln_w, *ln_b;
  float eps, drop_txt, drop_img;
  uint64_t seed;
  const uint64_t* seed_off;
  int64_t cls_id, sep_id, V, B, T, n_img, Lout, H;
  bf16* X;
  float* X32;  // optional f32 copy of X (the encoder's f32 hidden stream)
  float *keymask, *mean, *rstd;
};
void embed_fwd_launch(const EmbedParams& p, hipStream_t s);
struct EmbedBwdParams {
  const bf16* dX;
  const int64_t *ids, *seg;
  const float *proj, *word, *pos, *type, *ln_w, *mean, *rstd;
  int64_t cls_id, sep_id, B, T, n_img, H;
  float drop_txt, drop_img;
  uint64_t seed;
  const uint64_t* seed_off;
  float *d_word, *d_pos, *d_type, *d_ln_w, *d_ln_b, *d_proj, *ws;
};
void embed_bwd_launch(const EmbedBwdParams& p, hipStream_t s);
int64_t embed_bwd_blocks(int64_t B, int64_t S);
void image_normalize_launch(const uint8_t* in, int64_t n, const float* mean, const float* stdv, void* out,
                            bool out_bf16, hipStream_t s);
void maxpool3s2_fwd_launch(const bf16* x, int64_t B, int H, int W, int C, int OH, int OW, bf16* y, uint8_t* am,
                           hipStream_t s);
void maxpool3s2_bwd_launch(const bf16* dy, const uint8_t* am, int64_t B, int H, int W, int C, int OH, int OW,
                           bf16* dx, hipStream_t s);
void row_pool_fwd_launch(const bf16* fmap, int64_t B, int64_t Hh, int64_t Ww, int64_t C, int64_t n, float* out,
                         hipStream_t s);
void row_pool_bwd_launch(const float* dout, int64_t B, int64_t Hh, int64_t Ww, int64_t C, int64_t n, bf16* dfmap,
                         hipStream_t s);

struct AdamParams {
  float *params, *m, *v;
  const float* grads;
  bf16* bf16_copy;
  const int64_t* table;
  int32_t* steps;
  int64_t n_tensors, total;
  float lr_decay, lr_nodecay, wd, warmup, t_total, b1, b2, eps, max_grad_norm, grad_scale;
  float* ws;
  int64_t ws_floats;
};
int bertadam_launch(const AdamParams& p, hipStream_t s, const char** err);

struct BnFwdParams {
  const bf16 *X, *skip;
  bf16* Y;
  int64_t rows;
  int C;
  const float *w, *b;
  float *rmean, *rvar;
  int training, relu;
  float momentum, eps;
  float *smean, *sinvstd;
  int64_t* nbt;
  void* ws;
  uint8_t* mask;  // optional ReLU mask out ([rows][C/8] bytes, bit = Y > 0)
  const int8_t* skip_res;  // the residual stream's 8-bit residue of skip (with y_res only)
  int8_t* y_res;           // write Y's 8-bit residue (the block output / the downsample's output)
  double* lsum;        // cross-rank statistics: write the local sums {s1[C], s2[C], rows} and stop
  const double* gsum;  // cross-rank statistics: finalize + apply from the exchanged sums
  const float* parts;  // the producing conv's statistics table (float2 [nparts][C]): no stats pass
  int64_t nparts;
};
void batchnorm_fwd_launch(const BnFwdParams& q, hipStream_t s);
struct BnBwdParams {
  const bf16 *dY, *Y, *X;
  int64_t rows;
  int C;
  const float *w, *smean, *sinvstd;
  int relu;
  bf16 *dX, *dS;
  float *dw, *db;
  void* ws;
  const uint8_t* mask;  // optional ReLU mask (read instead of Y)
  double* lsum;        // as BnFwdParams: {sum g, sum g*(x-mean), rows} (+= dweight / dbias) and stop
  const double* gsum;  // finalize + apply from the exchanged sums
  const float* parts;  // or the reduction table of the product that formed dY (float2 [nparts][C])
  int64_t nparts;
};
void batchnorm_bwd_launch(const BnBwdParams& q, hipStream_t s);
int64_t batchnorm_ws_bytes(int64_t C);

void uncertainty_launch(const float* logits, const int64_t* y, int64_t S, int64_t R, int64_t C, float* p_bar,
                        float* nll, float* conf, float* correct, hipStream_t s);
void ece_bins_launch(const float* conf, const float* correct, int64_t S, int64_t n_bins, float* out, hipStream_t s);

}  // namespace mmu
