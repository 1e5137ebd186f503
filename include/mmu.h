/*
 * mmu.h -- C-ABI of libmmu_hip.so, the MI355X (gfx950) kernels of the MMBT
 * multimodal train / uncertainty-eval hot path.
 *
 * Reference being replaced (wooginawunan/multi-modal-uncertainty @ /root/reference,
 * pure PyTorch; its math lives in torchvision + pytorch_pretrained_bert 0.6.x):
 * every entry point below names the reference call it replaces (file:line).
 *
 * Conventions
 *   - Plain pointers + int64 sizes; no framework types.  All device buffers are
 *     owned by the caller; the library never allocates or frees device memory.
 *   - Work is enqueued on the caller's `stream` (a hipStream_t); no device sync.
 *   - Return 0 on success, nonzero on a bad argument / launch failure; the
 *     message is in mmu_last_error() (thread-local).
 *   - bf16 = IEEE bfloat16 bits (uint16), f32 = float.  Master weights, biases,
 *     LayerNorm params and all gradients of parameters are f32.
 *   - "additive key mask" = per (row, key) float added to the attention scores,
 *     0 for a real token and -10000 for a pad (src/mmbt.py:101-112).
 */
#ifndef MMU_H
#define MMU_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* mmu_stream_t; /* hipStream_t */

enum { MMU_BF16 = 0, MMU_F32 = 1 };

/* ------------------------------------------------------------------ status */
/* ABI version: bumped whenever an entry's argument list or buffer contract changes.  2 (round 5):
 * the residual stream's residue pointers inside mmu_batchnorm_fwd / _fwd_sums and the grad_scale
 * argument of mmu_bertadam_step.  3 (round 6): mmu_embed_bwd's workspace size is
 * mmu_embed_bwd_ws_floats().  4 (round 6): mmu_epilogue grows bn_x / bn_mask / bn_mean (the
 * BatchNorm-backward epilogues STORE_BNB / ADD_RES_BNB).  Callers compare mmu_version() with the
 * header they were built against. */
#define MMU_ABI_VERSION 4
int mmu_version(void);
const char* mmu_last_error(void);

/* Dropout under HIP-graph replay (round 5).  A captured launch replays the seed it was
 * captured with; with a device counter set here (uint64, caller-owned, NULL = off) every
 * dropout launch made afterwards folds *counter into its seed when it RUNS
 * (seed ^ counter * 0x9E3779B97F4A7C15), so a graph that advances the counter once per
 * replay draws fresh masks each step while forward and backward of one step agree.
 * A counter of 0 reproduces the eager masks bit for bit.  Process-wide setting.
 * (No reference counterpart: the reference draws torch's RNG per dropout call.) */
int mmu_set_seed_offset(const uint64_t* dev_counter);

/* ------------------------------------------------------------------ GEMM
 * C[m,n] (op)= sum_k A(m,k) * B(n,k), batched over `batch` with element strides.
 *   A(m,k) = A[m*lda + k] if a_kmajor else A[k*lda + m]      (bf16)
 *   B(n,k) = B[n*ldb + k] if b_kmajor else B[k*ldb + n]      (bf16)
 * Replaces the nn.Linear forward / backward products of pytorch_pretrained_bert
 * BertSelfAttention (query/key/value), BertSelfOutput.dense, BertIntermediate.dense,
 * BertOutput.dense (encoder call: src/mmbt.py:124-126) and the image projection
 * ImageBertEmbeddings.img_embeddings (src/mmbt.py:51,71).
 * Constraints: N % 128 == 0; K % 64 == 0 when an operand is K-major;
 *              M % 128 == 0 when A is M-major (not K-major).
 */
enum {
  MMU_EPI_STORE = 0,        /* C = acc (+bias[n]) (+C if accumulate)                     */
  MMU_EPI_BIAS_GELU = 1,    /* z = acc+bias; C = gelu_erf(z); aux (optional) = gelu'(z)  */
  MMU_EPI_BIAS_DROP_RES = 2,/* C = residual + dropout(acc+bias); with c_dtype MMU_F32 the
                               residual is f32 too (the encoder's f32 hidden stream)    */
  MMU_EPI_DGELU = 3,        /* C = acc * aux   (aux = the forward's gelu'(z))            */
  MMU_EPI_ADD_RES = 4,      /* C = acc + residual                                        */
  MMU_EPI_BIAS_DROP_QGELU = 5,/* u = dropout(acc+bias); C = u*sigmoid(1.702u); aux (optional)
                               = keep/(1-p) * d(u*sigmoid(1.702u))/du: FLAVA ResidualAttentionBlock
                               mlp c_fc -> Dropout -> QuickGELU (src/model.py:183-185,196-198) */
  MMU_EPI_STORE_STATS = 6,    /* C = acc (+bias) in bf16, and `colsum` = a float2 table
                               [ceil(M/64)][N] of {sum, sum of squares} of the stored C per column
                               and 64-row block: the training BatchNorm statistics of a conv
                               output, produced by the conv's own epilogue (round 6;
                               mmu_batchnorm_fwd_parts consumes it).  batch 1, no split-K. */
  MMU_EPI_STORE_BNB = 7,
  MMU_EPI_ADD_RES_BNB = 8,  /* STORE / ADD_RES into a bf16 C that is the output gradient dY of a
                               training BatchNorm (+ReLU) whose input was bn_x [M, N] bf16 (ReLU
                               mask bn_mask [M, N/8] u8 as mmu_batchnorm_fwd wrote it, or NULL =
                               no ReLU; batch mean bn_mean [N] f32), and `colsum` = a float2 table
                               [ceil(M/64)][N] of {sum g, sum g (bn_x - mean)} per column and
                               64-row block, g = the stored C * mask: the reduction of that
                               BatchNorm's backward, produced by the epilogue of the product that
                               forms its dY (the next conv's data gradient; round 6,
                               mmu_batchnorm_bwd_parts consumes it).  batch 1, ldc == N, A K-major
                               and B N-major (the 1x1 conv dX = dY_next . W).                  */
};
typedef struct mmu_epilogue {
  int32_t kind;
  int32_t accumulate;       /* STORE only: C += result (f32 C)                         */
  const float* bias;        /* [N] f32 or NULL                                          */
  int64_t bias_bstride;
  const void* residual;     /* bf16 [M, ldr] (f32 for BIAS_DROP_RES into an f32 C)      */
  int64_t ldr, res_bstride;
  void* aux;                /* bf16 [M, ldx]: GELU derivative (written or read)         */
  int64_t ldx, aux_bstride;
  float* colsum;            /* f32 [N] per batch: += column sums of the final C (bias grads) */
  int64_t colsum_bstride;
  float drop_p;             /* BIAS_DROP_RES                                            */
  uint64_t seed;            /* dropout stream: element (z, m, n) uses counter (z*M+m)*N+n */
  float* workspace;         /* optional f32 scratch: lets a STORE/f32/no-bias product split K
                               over workgroups (weight gradients); slabs summed in slice
                               order, so results stay deterministic.
                               Stream-ordered: one workspace per stream.                */
  int64_t workspace_floats;
  /* BIAS_DROP_RES into an f32 C only (optional, all four or none): the f32 residual is the
     LayerNorm OUTPUT recomputed from its f32 input, residual[m][n] =
     (r[m][n] - res_ln_mean[m]) * res_ln_rstd[m] * res_ln_w[n] + res_ln_b[n], with r the
     `residual` rows -- the encoder passes the previous LayerNorm's input (kept for its
     backward anyway) instead of materialising its f32 output.                          */
  const float* res_ln_mean;
  const float* res_ln_rstd;
  const float* res_ln_w;
  const float* res_ln_b;
  int64_t res_ln_bstride;   /* batched products: w / b of batch item z at + z * res_ln_bstride
                               (mean / rstd at + z * M)                                  */
  const void* bn_x;         /* STORE_BNB / ADD_RES_BNB only (ABI 4): see those kinds      */
  const uint8_t* bn_mask;
  const float* bn_mean;
  const uint8_t* res_mask;  /* ADD_RES / ADD_RES_BNB (ABI 4, optional): the residual is gated by
                               a ReLU mask [M, N/8] u8 (bit e of byte (m, n/8) keeps residual[m][n+e];
                               needs ldr == N) -- an identity Bottleneck's skip gradient g = dY3 * mask3
                               read from bn3's dY and mask instead of a materialised dSkip      */
} mmu_epilogue;

int mmu_gemm(const void* A, int64_t lda, int a_kmajor,
             const void* B, int64_t ldb, int b_kmajor,
             void* C, int64_t ldc, int c_dtype,
             int64_t M, int64_t N, int64_t K,
             int64_t batch, int64_t strideA, int64_t strideB, int64_t strideC,
             const mmu_epilogue* epi, mmu_stream_t stream);

/* Sum `parts` rows of a [parts, N] f32 partial table into out[N] (+= if accumulate). */
int mmu_colsum_reduce(const float* partial, int64_t parts, int64_t N, float* out,
                      int accumulate, mmu_stream_t stream);
/* n (1..4) independent mmu_colsum_reduce jobs of one width N in one launch: job z sums parts[z]
 * rows of partial[z] into out[z] (host arrays of n entries; the pointers are device memory). */
int mmu_colsum_reduce_multi(int n, const float* const* partial, const int64_t* parts, float* const* out, int64_t N,
                            int accumulate, mmu_stream_t stream);
/* Column sums of a bf16 [M, N] matrix into out[N] f32 (+= if accumulate): the bias grads
 * of the FLAVA blocks' projections (src/model.py).  `partial` (may be NULL): f32 scratch
 * of at least ceil(M / 64) * N floats; with it the row blocks are sized for ~1 K
 * workgroups and fold through per-block partial rows (mmu_colsum_reduce), without it
 * 1024-row blocks add into out by float atomics. */
int mmu_colsum_bf16(const void* X, int64_t M, int64_t N, int64_t ldx, float* partial,
                    float* out, int accumulate, mmu_stream_t stream);

/* Batched bf16 transpose: for each of n_jobs jobs (a device table of 6 int64 per job:
 * src pointer, dst pointer, rows, cols, src row pitch, dst row pitch; a pitch of 0 means
 * dense: cols / rows), dst[c*dpitch + r] = src[r*spitch + c].  Keeps the K-major
 * (transposed) bf16 copies of the BERT layer weights that the data-gradient products
 * dX = dY.W read as their B operand (the backward of the nn.Linear layers inside
 * pytorch_pretrained_bert BertLayer, src/mmbt.py:124-126), and the flipped, transposed
 * 3x3 filters of the conv data gradient (one job per tap); max_rows / max_cols bound the
 * jobs' shapes (grid size). */
int mmu_transpose_bf16_batched(const int64_t* jobs, int n_jobs, int64_t max_rows, int64_t max_cols,
                               mmu_stream_t stream);

/* ------------------------------------------------------------------ attention
 * softmax(Q K^T / sqrt(64) + keymask) (dropout) V for 12 x 64 heads, Q/K/V read from
 * the token-major fused projection QKV[rows, ld_qkv] (q at col h*64, k at 768+h*64,
 * v at 1536+h*64).  Replaces pytorch_pretrained_bert BertSelfAttention scores /
 * softmax / dropout / context (inside the encoder call src/mmbt.py:124-126).
 *   O   [rows, ld_o] bf16 (col h*64)   LSE [batch*heads, L] f32 (natural log-sum-exp
 *   of the scaled+masked scores).  keymask [batch, L] f32 additive.
 *   dropmask (may be NULL): [batch*heads, L, ceil(L/64)] u64 keep bits of the
 *   attention-probs dropout (bit k of word j = key 64j+k kept), written when
 *   drop_p > 0 for the backward to read.
 */
int mmu_attention_fwd(const void* QKV, int64_t ld_qkv, const float* keymask,
                      void* O, int64_t ld_o, float* LSE,
                      int64_t batch, int64_t L, int64_t heads,
                      float drop_p, uint64_t seed, uint64_t* dropmask, mmu_stream_t stream);
/* dQKV [rows, ld_dqkv] bf16 from dO; `delta` workspace [batch*heads, L] f32;
 * dropmask = the forward's (required when drop_p > 0).
 * dbias_parts (may be NULL): f32 [(ceil(L/128) + 2 ceil(L/64)) * batch, heads*64] receives
 * per-block column sums of dQ (rows [0, nqb*batch)), dK (next nkb*batch rows) and dV (last
 * nkb*batch rows), every element written; summing each row range (mmu_colsum_reduce) gives
 * the Q / K / V bias gradients without another pass over dQKV. */
int mmu_attention_bwd(const void* QKV, int64_t ld_qkv, const float* keymask,
                      const void* O, int64_t ld_o, const void* dO, int64_t ld_do,
                      const float* LSE, float* delta, void* dQKV, int64_t ld_dqkv,
                      int64_t batch, int64_t L, int64_t heads,
                      float drop_p, uint64_t seed, const uint64_t* dropmask, float* dbias_parts,
                      mmu_stream_t stream);

/* ------------------------------------------------------------------ LayerNorm
 * y = LN(x) * w + b over the last dim (768), eps; x, y bf16 [rows, H]; saves
 * mean/rstd f32 [rows].  BertLayerNorm of BertSelfOutput / BertOutput
 * (src/mmbt.py:124-126).
 */
int mmu_layernorm_fwd(const void* X, const float* w, const float* b, void* Y,
                      float* mean, float* rstd, int64_t rows, int64_t H, float eps,
                      int64_t group_rows, int64_t param_stride, mmu_stream_t stream);
/* group_rows / param_stride: row r uses w/b + (r / group_rows) * param_stride, so the K
 * members of a deep ensemble normalise in one launch (group_rows <= 0: one group).
 * mean/rstd may both be NULL (inference). */
/* Backward of y = LN(x): dX = LN'(dY) (+ dRes), optional dXdrop = dropout_bwd(dX)
 * (same (seed, m*H+n) stream as the producing BIAS_DROP_RES epilogue), and partial
 * column sums [ceil(rows/rows_per_part), H] for dgamma, dbeta and dbias
 * (= column sum of dXdrop, or of dX when no dropout output). */
int mmu_layernorm_bwd(const void* dY, const void* X, const float* mean, const float* rstd,
                      const float* w, void* dX, void* dXdrop, float drop_p, uint64_t seed,
                      float* part_dw, float* part_db, float* part_dbias,
                      int64_t rows, int64_t H, int64_t rows_per_part, mmu_stream_t stream);

/* The encoder's f32 hidden stream (post-LN BertLayer, src/mmbt.py:124-126): the LN input
 * S = residual + dropout(branch) stays f32 (written by an f32 BIAS_DROP_RES epilogue), so
 * that the 24 residual adds of the 12 layers are never rounded to bf16.
 * mmu_layernorm_fwd_f32: X f32 [rows, H] -> Y bf16 (the next GEMM's operand) and, when
 * Y32 != NULL, Y32 f32 (the next residual); group_rows / param_stride as above.
 * mmu_layernorm_bwd_f32: mmu_layernorm_bwd with an f32 X. */
int mmu_layernorm_fwd_f32(const float* X, const float* w, const float* b, void* Y, float* Y32,
                          float* mean, float* rstd, int64_t rows, int64_t H, float eps,
                          int64_t group_rows, int64_t param_stride, mmu_stream_t stream);
int mmu_layernorm_bwd_f32(const void* dY, const float* X, const float* mean, const float* rstd,
                          const float* w, void* dX, void* dXdrop, float drop_p, uint64_t seed,
                          float* part_dw, float* part_db, float* part_dbias,
                          int64_t rows, int64_t H, int64_t rows_per_part, mmu_stream_t stream);

/* Pre-LN block backward (FLAVA ResidualAttentionBlock, src/model.py:210-212: x + f(LN(x))):
 * dX = LN'(dY) + dRes; part_dbias = column sums of that total dX (the bias gradient of the
 * Linear whose output was added to the residual stream).  No dropout output. */
int mmu_layernorm_bwd_res(const void* dY, const void* X, const float* mean, const float* rstd,
                          const float* w, const void* dRes, void* dX,
                          float* part_dw, float* part_db, float* part_dbias,
                          int64_t rows, int64_t H, int64_t rows_per_part, mmu_stream_t stream);

/* ------------------------------------------------------------------ FLAVA attention
 * nn.MultiheadAttention(x, x, x) with batch_first=False applied to an [S, N, E] tensor
 * (src/model.py:193,205-207; the block receives [B, L, E], so the sequence axis is the
 * BATCH: S = B samples, N = L token positions).  QKV [S*N, ld_qkv] bf16 = the in_proj
 * output, row s*N + n, q at col h*D, k at E + h*D, v at 2E + h*D (E = heads*D).
 * softmax(Q K^T / sqrt(D)) V per (n, h); no mask, no dropout (module defaults).
 *   O [S*N, ld_o] bf16 (col h*D); LSE2 [N*heads, S] f32 = log2-sum-exp2 of the scores
 *   scaled by log2(e)/sqrt(D) (for the backward).  D in {64, 128, 256}. */
int mmu_seqattn_fwd(const void* QKV, int64_t ld_qkv, void* O, int64_t ld_o, float* LSE2,
                    int64_t S, int64_t N, int64_t heads, int64_t head_dim, mmu_stream_t stream);
/* dQKV [S*N, ld_dqkv] bf16 (every element written); delta workspace [N*heads, S] f32. */
int mmu_seqattn_bwd(const void* QKV, int64_t ld_qkv, const void* O, int64_t ld_o,
                    const void* dO, int64_t ld_do, const float* LSE2, float* delta,
                    void* dQKV, int64_t ld_dqkv, int64_t S, int64_t N, int64_t heads,
                    int64_t head_dim, mmu_stream_t stream);

/* ------------------------------------------------------------------ embeddings
 * Modality-token embed + text gather + concat/gather, one pass
 * (ImageBertEmbeddings src/mmbt.py:58-83, BertEmbeddings src/mmbt.py:121,
 *  torch.cat src/mmbt.py:122, control gather src/mmbt.py:198-229).
 * Source sequence s of length S = n_img+2+T: s=0 [CLS], 1..n_img image proj rows,
 * n_img+1 [SEP] (positions 0..n_img+1, token type 0), then text t at position t,
 * type seg[b,t].  Output row (v,b,j) embeds source position idx[v*Lout + j]
 * (idx == NULL: identity, Lout == S) and is LayerNorm'ed.  X [V*B*Lout, H] bf16,
 * X32 (optional, may be NULL) the same rows in f32 (the encoder's f32 hidden stream);
 * keymask [V*B, Lout] f32 additive; mean/rstd (optional) f32 [V*B*Lout] for backward.
 * Dropout after the LN: drop_img on the image-segment rows (ImageBertEmbeddings.dropout,
 * args.dropout), drop_txt on text rows (BertEmbeddings.dropout 0.1); counter row*768+col.
 * Tables f32: word [vocab,H], pos [maxpos,H], type [2,H]; proj f32 [B, n_img, H].
 */
int mmu_embed_fwd(const int64_t* ids, const int64_t* seg, const int64_t* txt_mask,
                  const float* proj, const float* word, const float* pos, const float* type,
                  const float* ln_w, const float* ln_b, float eps,
                  int64_t cls_id, int64_t sep_id,
                  const int64_t* idx, int64_t V, int64_t B, int64_t T, int64_t n_img, int64_t Lout,
                  int64_t H, float drop_txt, float drop_img, uint64_t seed,
                  void* X, float* X32, float* keymask, float* mean, float* rstd, mmu_stream_t stream);
/* Backward of mmu_embed_fwd for the identity variant (training): recomputes the
 * pre-LN sums, LN backward, then scatters: word rows by atomics, position / type
 * / [CLS] / [SEP] by batch reduction, image rows to dproj f32 [B, n_img, H].
 * ws: f32 workspace of at least mmu_embed_bwd_ws_floats(B, T, n_img) floats (ABI 3; ABI 2 took
 * B*S*H + 2*ceil(B*S/64)*H, which is larger for every B > 1). */
int64_t mmu_embed_bwd_ws_floats(int64_t B, int64_t T, int64_t n_img);
int mmu_embed_bwd(const void* dX, const int64_t* ids, const int64_t* seg,
                  const float* proj, const float* word, const float* pos, const float* type,
                  const float* ln_w, const float* mean, const float* rstd,
                  int64_t cls_id, int64_t sep_id, int64_t B, int64_t T, int64_t n_img, int64_t H,
                  float drop_txt, float drop_img, uint64_t seed, float* d_word, float* d_pos, float* d_type, float* d_ln_w, float* d_ln_b,
                  float* d_proj, float* ws, mmu_stream_t stream);

/* Image transform tail of the Food-101 pipeline (src/dataset.py:488-498: ToTensor +
 * Normalize) on the device: in = uint8 crops [B,H,W,3] (HWC, as decoded), n = B*H*W*3;
 * out = (in/255 - mean[c]) / std[c] with c = index % 3, i.e. the channels-last
 * [B,3,H,W] image, f32 (out_dtype MMU_F32) or bf16 (MMU_BF16).  mean / std: 3 host floats. */
int mmu_image_normalize(const uint8_t* in, int64_t n, const float* mean, const float* stdv, void* out,
                        int out_dtype, mmu_stream_t stream);

/* MaxPool2d(3, stride 2, padding 1) of the ResNet stem (torchvision resnet child 3,
 * src/mmbt.py:19-21): x NHWC bf16 [B,H,W,C] -> y [B,OH,OW,C] + argmax (uint8 position 0..8
 * in the window, same layout as y); backward: dy + argmax -> dx [B,H,W,C] (every element
 * written).  C % 8 == 0, OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1. */
int mmu_maxpool_fwd(const void* x, int64_t B, int64_t H, int64_t W, int64_t C, void* y, uint8_t* argmax,
                    mmu_stream_t stream);
int mmu_maxpool_bwd(const void* dy, const uint8_t* argmax, int64_t B, int64_t H, int64_t W, int64_t C, void* dx,
                    mmu_stream_t stream);

/* AdaptiveAvgPool2d((n,1)) + flatten + transpose of the ResNet map
 * (src/mmbt.py:30,42-44): fmap NHWC bf16 [B,Hh,Ww,C] -> out f32 [B,n,C]; and its backward. */
int mmu_row_pool_fwd(const void* fmap, int64_t B, int64_t Hh, int64_t Ww, int64_t C, int64_t n,
                     float* out, mmu_stream_t stream);
int mmu_row_pool_bwd(const float* dout, int64_t B, int64_t Hh, int64_t Ww, int64_t C, int64_t n,
                     void* dfmap, mmu_stream_t stream);

/* ------------------------------------------------------------------ 3x3 conv weight gradient
 * dW (+)= dConv2d(3x3, stride 1, pad 1)/dW of the ResNet-152 bottleneck conv2 (torchvision
 * Bottleneck.conv2, src/mmbt.py:19-21) on channels-last bf16 maps: X [n_img*H*W, Cin] (the
 * conv input), dY [n_img*H*W, Cout] (its output gradient); dW f32 [Cout][3][3][Cin] (the
 * channels-last filter), += when accumulate.  One implicit-im2col MFMA GEMM (M = Cout,
 * N = 9 Cin, K = pixels; the B operand gathered per tap with zero padding), split-K over
 * the pixels into ws (f32, may be NULL: no split).  Cin % 256 == 0, Cout % 128 == 0. */
int mmu_conv3x3_wgrad(const void* dY, const void* X, float* dW, int64_t n_img, int64_t H, int64_t W,
                      int64_t Cin, int64_t Cout, int accumulate, float* ws, int64_t ws_floats,
                      mmu_stream_t stream);

/* 3x3 / stride-1 / pad-1 convolution as one implicit-im2col MFMA GEMM (the A operand
 * gathered per tap, padding read as zero): Y[pixel][n] = sum over taps t = 3 kh + kw and
 * channels c of X[pixel + (kh - 1, kw - 1)][c] * Wk[n][t * C + c], bf16 in / out,
 * f32 accumulate; X [n_img*H*W, C] and Y [n_img*H*W, N] NHWC rows.  The forward of
 * Bottleneck.conv2 is (X = x, Wk = the channels-last filter [Cout][3][3][Cin]); its data
 * gradient is (X = dY, Wk = the flipped filter transposed to [Cin][3][3][Cout]).
 * C % 64 == 0, N % 128 == 0, N >= 256.  `ws` (optional, ws_floats f32): when the output has
 * too few 256x256 tiles to fill the chip (small batches: e.g. layer3 at batch 32 is 25
 * tiles), the taps / channels are split over workgroups into f32 slabs of ws and summed in
 * slice order into Y (deterministic). */
int mmu_conv3x3_implicit(const void* X, const void* Wk, void* Y, int64_t n_img, int64_t H, int64_t W,
                         int64_t C, int64_t N, float* ws, int64_t ws_floats, mmu_stream_t stream);

/* The same two products for the strided convs of the ResNet-152 trunk (the first block of
 * layer2..4: Bottleneck.conv2 3x3 / stride 2 / pad 1 and the downsample 1x1 / stride 2,
 * src/mmbt.py:19-21): ksize 3 (pad 1) or 1 (pad 0), any stride 1..4; X [n_img*H*W, C] the
 * input map, Y / dY [n_img*Ho*Wo, N] with Ho = (H + 2 pad - ksize) / stride + 1 (Wo alike).
 * mmu_conv_implicit: forward (Wk [N][ksize][ksize][C]), C % 64 == 0, N % 64 == 0.
 * mmu_conv_wgrad: filter gradient dW f32 [Cout][ksize][ksize][Cin], Cin % 256 == 0,
 * Cout % 128 == 0.  mmu_conv3x3_* above are (ksize 3, stride 1) of these. */
int mmu_conv_implicit(const void* X, const void* Wk, void* Y, int64_t n_img, int64_t H, int64_t W, int64_t C,
                      int64_t N, int64_t ksize, int64_t stride, float* ws, int64_t ws_floats,
                      mmu_stream_t stream);
/* mmu_conv_implicit that also writes the training BatchNorm statistics of Y: stats = float2
 * [ceil(Npix / 64)][N] {sum, sum of squares} per output channel and 64-pixel block of the bf16
 * Y (MMU_EPI_STORE_STATS; with split-K they come from a pass over Y after its reduction). */
int mmu_conv_implicit_stats(const void* X, const void* Wk, void* Y, int64_t n_img, int64_t H, int64_t W, int64_t C,
                            int64_t N, int64_t ksize, int64_t stride, float* stats, float* ws, int64_t ws_floats,
                            mmu_stream_t stream);
/* mmu_conv3x3_implicit whose output is the data gradient dX of a 3x3 conv that a training
 * BatchNorm (+ReLU) fed: also writes that BatchNorm's backward reduction table (stats = float2
 * [ceil(Npix / 64)][N] {sum g, sum g (bn_x - bn_mean)}, g = dX * bn_mask; see
 * MMU_EPI_STORE_BNB).  bn_x [Npix, N] bf16, bn_mask [Npix, N/8] u8 or NULL, bn_mean [N] f32.
 * With split-K the table comes from a pass over dX after its reduction. */
int mmu_conv3x3_implicit_bnb(const void* X, const void* Wk, void* Y, int64_t n_img, int64_t H, int64_t W, int64_t C,
                             int64_t N, const void* bn_x, const uint8_t* bn_mask, const float* bn_mean,
                             float* stats, float* ws, int64_t ws_floats, mmu_stream_t stream);
int mmu_conv_wgrad(const void* dY, const void* X, float* dW, int64_t n_img, int64_t H, int64_t W, int64_t Cin,
                   int64_t Cout, int64_t ksize, int64_t stride, int accumulate, float* ws, int64_t ws_floats,
                   mmu_stream_t stream);

/* ResNet-152 stem convolution, 7x7 / stride 2 / pad 3, 3 -> 64 channels (torchvision resnet
 * child 0, the image encoder's conv embed: src/mmbt.py:19-21,42), on channels-last bf16:
 * X [n_img, H, W, 3], Wk [64][7][7][3] (the channels-last filter), Y [n_img, Ho, Wo, 64] with
 * Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1; f32 accumulate.  One persistent kernel: tiles of
 * 2 x 64 output pixels, the input patch in LDS, 16x16x32 bf16 MFMAs over the 3-channel taps
 * padded to 4 (K = 224). */
int mmu_stem_conv_fwd(const void* X, const void* Wk, void* Y, int64_t n_img, int64_t H, int64_t W,
                      mmu_stream_t stream);
/* Its filter gradient: dW f32 [64][7][7][3] (+)= sum over pixels of dY (x) im2col(X) (dY
 * [n_img, Ho, Wo, 64] bf16), += when accumulate.  Per-block f32 partials go to ws
 * (>= mmu_stem_conv_wgrad_ws_floats(n_img, H, W) floats) and are summed in block order. */
int64_t mmu_stem_conv_wgrad_ws_floats(int64_t n_img, int64_t H, int64_t W);
int mmu_stem_conv_wgrad(const void* dY, const void* X, float* dW, int64_t n_img, int64_t H, int64_t W,
                        int accumulate, float* ws, int64_t ws_floats, mmu_stream_t stream);

/* ------------------------------------------------------------------ BatchNorm (image trunk)
 * BatchNorm2d [+ residual add] [+ ReLU] of the ResNet-152 trunk (torchvision
 * Bottleneck bn1/bn2/bn3 + downsample, src/mmbt.py:19-21) on channels-last bf16
 * activations X [rows = N*H*W, C] (C % 8 == 0, C <= 2048):
 *   Y = act(X * scale + shift [+ skip]),  act = ReLU when relu != 0.
 * training: batch statistics (biased variance), running_mean / running_var updated
 *   with momentum (unbiased variance), *num_batches_tracked += 1 (each may be NULL);
 *   momentum < 0 = torch's momentum=None (cumulative moving average): the factor is
 *   1 / *num_batches_tracked, which the caller has ALREADY incremented for this pass (required,
 *   not incremented again here),
 *   save_mean / save_invstd [C] f32 written for the backward.
 * eval: running statistics.  weight / bias may be NULL (affine = False).
 * relu_mask (may be NULL; needs relu): [rows, C/8] u8 written with bit e of byte (r, c/8)
 *   = Y[r, c+e] > 0, for the backward to read instead of Y (1/16 of its bytes).
 * y_res / skip_res (may be NULL): the residual stream past bf16 -- y_res [rows, C] i8 is written
 *   with the 8-bit residue of each output, r = rint((v - Y) * 2^15 / 2^e) (v the f32 value, e
 *   the binary exponent of Y); a skip is then read as skip + skip_res * 2^(e(skip) - 15).  Two
 *   uses: a Bottleneck's bn3 (skip, relu, skip_res and y_res all given) and the downsample's
 *   BatchNorm (no skip, no relu, y_res only).
 * ws: device scratch of >= mmu_batchnorm_ws_bytes(C) bytes (per-block partial sums +
 * per-channel coefficients, ~8 MiB), 16-B aligned.
 */
int64_t mmu_batchnorm_ws_bytes(int64_t C);
int mmu_batchnorm_fwd(const void* X, const void* skip, void* Y, int64_t rows, int64_t C,
                      const float* weight, const float* bias, float* running_mean, float* running_var,
                      int64_t* num_batches_tracked, int training, float momentum, float eps, int relu,
                      float* save_mean, float* save_invstd, void* relu_mask, const void* skip_res, void* y_res,
                      void* ws, int64_t ws_bytes, mmu_stream_t stream);
/* Training-mode forward whose batch statistics were produced by the conv before it
 * (MMU_EPI_STORE_STATS / mmu_conv_implicit_stats: parts = float2 [nparts][C] block partials of
 * X's {sum, sum of squares} per channel): no statistics pass; finalize (running stats,
 * save_mean / save_invstd) and apply as mmu_batchnorm_fwd with training = 1. */
int mmu_batchnorm_fwd_parts(const void* X, const void* skip, void* Y, int64_t rows, int64_t C, const float* parts,
                            int64_t nparts, const float* weight, const float* bias, float* running_mean,
                            float* running_var, int64_t* num_batches_tracked, float momentum, float eps, int relu,
                            float* save_mean, float* save_invstd, void* relu_mask, const void* skip_res, void* y_res,
                            void* ws, int64_t ws_bytes, mmu_stream_t stream);
/* Training-mode backward.  g = dY * [Y > 0] when relu, from relu_mask when given (the
 * forward's mask), else from Y (the forward's output); g = dY without relu;
 * dX [rows, C] bf16; dSkip (may be NULL) = g, the gradient of the residual input;
 * dweight / dbias (may be NULL) f32 [C] are ACCUMULATED (+=). */
int mmu_batchnorm_bwd(const void* dY, const void* Y, const void* relu_mask, const void* X, int64_t rows,
                      int64_t C, const float* weight, const float* save_mean, const float* save_invstd, int relu,
                      void* dX, void* dSkip, float* dweight, float* dbias, void* ws, int64_t ws_bytes,
                      mmu_stream_t stream);

/* Training-mode backward whose reduction {sum g, sum g (x - mean)} was produced by the product
 * that formed dY (MMU_EPI_STORE_BNB / ADD_RES_BNB, mmu_conv3x3_implicit_bnb: parts = float2
 * [nparts][C] block partials): no reduction pass; finalize (dweight / dbias +=) and apply as
 * mmu_batchnorm_bwd. */
int mmu_batchnorm_bwd_parts(const void* dY, const void* Y, const void* relu_mask, const void* X, int64_t rows,
                            int64_t C, const float* parts, int64_t nparts, const float* weight,
                            const float* save_mean, const float* save_invstd, int relu, void* dX, void* dSkip,
                            float* dweight, float* dbias, void* ws, int64_t ws_bytes, mmu_stream_t stream);

/* Cross-rank (synchronised) BatchNorm: data-parallel training that keeps the reference's
 * whole-batch statistics (src/mmbt.py:19-21 normalises the trunk over the full batch of one
 * device; under DP the batch is split over ranks).  Each training pass is split at its
 * per-channel reduction and the caller sums `sums` over the ranks between the two calls
 * (one all-reduce of 2C+1 doubles; torch.nn.SyncBatchNorm's exchange):
 *   sums [2C+1] f64 = {s1[0..C), s2[0..C), rows}
 *   forward:  mmu_batchnorm_stats (s1 = sum x, s2 = sum x^2 over the local rows), exchange,
 *             mmu_batchnorm_fwd_sums (the training forward of mmu_batchnorm_fwd with the
 *             statistics of the exchanged sums: mean, biased variance over sums[2C] rows;
 *             running stats from the unbiased variance of the same)
 *   backward: mmu_batchnorm_bwd_reduce (s1 = sum g, s2 = sum g (x - mean); dweight / dbias
 *             += this rank's dgamma = s2 * invstd, dbeta = s1, may be NULL), exchange,
 *             mmu_batchnorm_bwd_sums (dX [, dSkip] from the exchanged sums).
 * Arguments otherwise as mmu_batchnorm_fwd / mmu_batchnorm_bwd. */
int mmu_batchnorm_stats(const void* X, int64_t rows, int64_t C, double* sums, void* ws, int64_t ws_bytes,
                        mmu_stream_t stream);
int mmu_batchnorm_fwd_sums(const void* X, const void* skip, void* Y, int64_t rows, int64_t C, const double* sums,
                           const float* weight, const float* bias, float* running_mean, float* running_var,
                           int64_t* num_batches_tracked, float momentum, float eps, int relu, float* save_mean,
                           float* save_invstd, void* relu_mask, const void* skip_res, void* y_res, void* ws,
                           int64_t ws_bytes, mmu_stream_t stream);
int mmu_batchnorm_bwd_reduce(const void* dY, const void* Y, const void* relu_mask, const void* X, int64_t rows,
                             int64_t C, const float* save_mean, const float* save_invstd, int relu, double* sums,
                             float* dweight, float* dbias, void* ws, int64_t ws_bytes, mmu_stream_t stream);
int mmu_batchnorm_bwd_sums(const void* dY, const void* Y, const void* relu_mask, const void* X, int64_t rows,
                           int64_t C, const double* sums, const float* weight, const float* save_mean,
                           const float* save_invstd, int relu, void* dX, void* dSkip, void* ws, int64_t ws_bytes,
                           mmu_stream_t stream);

/* ------------------------------------------------------------------ BertAdam
 * Fused multi-tensor BertAdam (pytorch_pretrained_bert 0.6.x, constructed at
 * train.py:142-147; stepped at src/framework.py:303): per-tensor clip
 * (max_grad_norm), m/v update without bias correction, decoupled weight decay
 * (group 0 only), lr * warmup_linear(step/t_total) with the per-tensor step read
 * before its increment, optional bf16 copy of the updated weight for the GEMMs.
 * table (int64, device): 7 per tensor {offset, numel, group (0 decay / 1 no decay),
 *   bf16_offset (-1 = none), active (0 = skipped like a None grad), first_chunk,
 *   n_chunks}, followed by 3 per chunk {tensor, start, len}.
 * steps int32 [n_tensors] (device, incremented); ws f32 >= n_chunks + 2*n_tensors.
 * grad_scale: the gradient the optimizer sees is grads * grad_scale (clip norm included) --
 * data parallelism's 1/world applied here instead of a separate pass over the summed grads.
 */
int mmu_bertadam_step(float* params, const float* grads, float* m, float* v, void* bf16_copy,
                      const int64_t* table, int32_t* steps, int64_t n_tensors, int64_t n_chunks,
                      float lr_decay, float lr_nodecay, float wd, float warmup, float t_total,
                      float b1, float b2, float eps, float max_grad_norm, float grad_scale,
                      float* ws, int64_t ws_floats, mmu_stream_t stream);

/* ------------------------------------------------------------------ uncertainty
 * logits f32 [S, R, C] (R = members x passes per sample) ->
 * p_bar f32 [S, C] = mean_r softmax(logits[s, r]); per-sample nll [S] = -log p_bar[y];
 * conf [S], correct [S].  ECE is then binned from conf/correct (mmu_ece_bins).
 * North-star metrics; softmax-then-mean convention of
 * notebooks/food101_robustness.py:25-36.
 */
int mmu_uncertainty(const float* logits, const int64_t* y, int64_t S, int64_t R, int64_t C,
                    float* p_bar, float* nll, float* conf, float* correct, mmu_stream_t stream);
/* 15-style equal-width bins: out f32 [3*n_bins] = (count, sum conf, sum correct). */
int mmu_ece_bins(const float* conf, const float* correct, int64_t S, int64_t n_bins,
                 float* out, mmu_stream_t stream);

/* ------------------------------------------------------------------ timing
 * Device-time of every mmu_gemm launch while enabled, bracketed by HIP events on
 * the launch stream (bench.py roofline).  Reads back (host sync) only in _read.
 */
int mmu_timing_enable(int on);
/* paused != 0: launches are not recorded (already recorded ones are kept) -- the
 * ResNet 1x1-conv products run through mmu_gemm but are not BERT-layer GEMMs. */
int mmu_timing_pause(int paused);
int mmu_timing_read(double* total_ms, int64_t* launches, double* flops);

#ifdef __cplusplus
}
#endif
#endif /* MMU_H */
