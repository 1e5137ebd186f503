// Flash-style BERT self-attention (12 heads x 64) for gfx950, fwd + bwd.
//
// Replaces pytorch_pretrained_bert BertSelfAttention's scores / softmax / dropout /
// context product (called inside the encoder, src/mmbt.py:124-126).  Semantics:
//   P = softmax(Q K^T / 8 + keymask),  O = dropout(P) V     (keymask: 0 or -10000)
// Keys beyond L (tile tails) are excluded exactly (-inf), rows beyond L are not stored.
//
// All products use v_mfma_f32_32x32x16_bf16 in the "swapped" orientation: the
// score tile is S^T = K Q^T (keys on registers, queries on lanes), so each lane
// owns one query row: softmax max/sum are in-lane plus one xor-32 shuffle, and
// P feeds the next MFMA straight from its accumulator registers (no LDS trip).
//   fwd : S^T = K.Q^T ; O^T += V^T.P^T           (V^T fragment by ds_read_b64_tr_b16)
//   dQ  : S^T, dP^T = V.dO^T ; dQ^T += K^T.dS^T
//   dKdV: S = Q.K^T, dP = dO.V^T (keys on lanes) ; dV += P^T.dO ; dK += dS^T.Q
// LDS tiles are [rows][64 d] bf16 (128-B rows) with the 16-B chunk index XORed by
// f(row) = ((row>>1)&1)<<2 | ((row>>3)&3): conflict-free for both the row reads
// (ds_read_b128) and the transposed reads (checked by enumeration).
//
// Dropout: element (q, key) of head-row bh draws 16 bits from
// lowbias32(((q*Lp + key) >> 1) ^ seed_bh), low/high half by key parity; dropped
// when < round(p*65536).  The forward hashes and stores the keep bits as one u64
// per (bh, query, 64-key tile) in `dropmask`; dQ and dKdV read those bits.
#include "mmu_common.h"
#include "mmu_internal.h"
#include <cstdlib>
#include <type_traits>
#include <utility>

namespace mmu {

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;
constexpr float NEG_INF = -__builtin_huge_valf();

static __device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
static __device__ __forceinline__ uint32_t seed_for(uint64_t seed, int bh) {
  return lowbias32((uint32_t)seed ^ lowbias32((uint32_t)(seed >> 32) + 0x9E3779B9u * (uint32_t)(bh + 1)));
}
// keep bits for keys (key, key+1) of query q (key even)
static __device__ __forceinline__ uint32_t drop_pair(uint32_t sbh, uint32_t q, uint32_t key, uint32_t Lp) {
  return lowbias32(((q * Lp + key) >> 1) ^ sbh);
}

// max of three as v_max3_f32, compiler-visible: its operands come straight out of MFMA
// accumulators, and only the compiler's hazard recognizer knows how long to wait before reading
// them (an asm v_max3_f32 here, rounds 1-4, read the S tile right behind its MFMA -- a stale
// value, harmless only because the deferred-max softmax is invariant to the subtracted max)
static __device__ __forceinline__ float max3f(float a, float b, float c) {
  return __builtin_fmaxf(__builtin_fmaxf(a, b), c);
}
// (m & a) | (~m & b), written so that hipcc emits ONE v_bitop3_b32 (gfx950).  Not inline asm: the
// operands here come straight out of MFMA accumulators, and the hazard recognizer does not see
// inside an asm statement -- an asm v_bfi_b32 reading an MFMA result two instructions after the
// MFMA read it before the MFMA had written it (the 13 % dK error of a round-5 dropout test)
static __device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
  return (m & a) | (~m & b);
}
// the keep bit `pos` of word w as an all-ones / zero mask (v_bfe_i32).  In asm so that the
// optimizer cannot see that the mask is 0 / -1: it would turn the bfi above into a compare
// and a v_cndmask (one VALU more per element)
static __device__ __forceinline__ uint32_t keepmask(uint32_t w, uint32_t pos) {
  uint32_t r;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(r) : "v"(w), "v"(pos));
  return r;
}
// f(integral_constant<int, R>) for R = 0, 1, ... in order (compile-time indices, C++17)
template <typename F, int... R>
static __device__ __forceinline__ void static_for(F&& f, std::integer_sequence<int, R...>) {
  (f(std::integral_constant<int, R>{}), ...);
}
template <int POS>  // (a compile-time bit position as an inline constant, not a VGPR)
static __device__ __forceinline__ uint32_t keepmask(uint32_t w) {
  uint32_t r;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(r) : "v"(w), "n"(POS));
  return r;
}
static __host__ __device__ __forceinline__ uint32_t drop_thr(float p) { return (uint32_t)(p * 65536.0f + 0.5f); }

static __device__ __forceinline__ int fsw(int r) { return (((r >> 1) & 1) << 2) | ((r >> 3) & 3); }
static __device__ __forceinline__ int tile_off(int row, int chunk) { return row * 128 + ((chunk ^ fsw(row)) << 4); }

// operand fragment of v_mfma_f32_32x32x16_bf16, K-contiguous tile: lane l holds
// tile[row0 + (l&31)][16ks + 8(l>>5) + j]
static __device__ __forceinline__ bf16x8 row_frag(const char* s, int row0, int ks, int l) {
  return *(const bf16x8*)(s + tile_off(row0 + (l & 31), 2 * ks + (l >> 5)));
}
// transposed fragment matching an accumulator used as the other operand: lane l holds
// tile[row0 + 16s + 8(j>>2) + 4h + (j&3)][col0 + (l&31)], h = l>>5  (row0 includes 16s)
static __device__ __forceinline__ bf16x8 tr_frag(const char* s, int row0, int col0, int l) {
  const int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3, h = g >> 1;
  const int col = col0 + 16 * (g & 1) + 4 * p;  // element column
  const int r0 = row0 + 4 * h + q, r1 = r0 + 8;
  const int cb = col * 2;
  const char* a0 = s + tile_off(r0, cb >> 4) + (cb & 15);
  const char* a1 = s + tile_off(r1, cb >> 4) + (cb & 15);
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((MMU_LDS(bf16x4)*)a0);
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((MMU_LDS(bf16x4)*)a1);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
// 8 accumulator registers (8s..8s+7) -> bf16 operand fragment
static __device__ __forceinline__ bf16x8 acc_frag(const f32x16& a, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = f2bf(a[8 * s + j]);
  return r;
}
static __device__ __forceinline__ bf16x8 scale_frag(uint4 u, float sc) {
  bf16x8 v = *(bf16x8*)&u;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = f2bf(bf2f(v[j]) * sc);
  return v;
}

// Buffer descriptor from provably wave-uniform inputs: with the base / size words in
// VGPRs hipcc wraps EVERY buffer op in a readfirstlane "waterfall" loop (~10 instructions
// and a branch per DMA; 68 such loops in the dK/dV kernel).  Inputs derived from the
// kernel arguments and blockIdx are uniform; readfirstlane makes that visible.
static __device__ __forceinline__ __amdgpu_buffer_rsrc_t urs(const void* base, int bytes) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane(bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, n, 0x00020000);
}

// ---- LDS-DMA helpers (buffer_load ... lds: lane-linear LDS destination, per-lane source)
static __device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (MMU_LDS(void)*)lds, 16, off, 0, 0, 0);
}
// A tile's descriptor: the buffer [base, base + bytes) advanced by the tile's byte offset `off`
// (wave-uniform: SALU work), so the lanes' offsets within a tile stay loop-invariant VGPRs and
// the range check still sees rows past the buffer (the scalar-offset operand of a buffer load is
// outside the range check, so a per-tile row offset cannot go there: past-the-end rows would be
// read instead of returning zero)
// (bytes - off clamped at 0: an empty buffer -- e.g. no keep words without dropout -- reads zeros
// and keeps the wave's per-tile DMA count, which its vmcnt waits assume)
static __device__ __forceinline__ __amdgpu_buffer_rsrc_t urs_at(const void* base, int bytes, int off) {
  return urs((const char*)base + off, bytes > off ? bytes - off : 0);
}
static __device__ __forceinline__ void dma4(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (MMU_LDS(void)*)lds, 4, off, 0, 0, 0);
}
static __device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// (query / key block, batch-head) of this workgroup.  The grid is (blocks per head-row,
// B * heads); the dispatcher deals workgroups to the 8 XCDs round-robin by linear id, so
// without a remap the blocks of one head-row (which all stream the same K / V, or Q / dO,
// rows) land on different XCDs and each XCD's L2 fetches them again.  xcd_remap gives each
// XCD a contiguous range of linear work ids: the blocks of a head-row share one L2.
static __device__ __forceinline__ void block_coords(int& bx, int& bh) {
  const int gx = gridDim.x;
  const int wid = xcd_remap(blockIdx.y * gx + blockIdx.x, gx * gridDim.y);
  bh = wid / gx;
  bx = wid - bh * gx;
}

// ---------------------------------------------------------------- forward ring geometry
constexpr int FWD_NS = 2;                      // K/V ring depth (tiles)
constexpr int FWD_TILE = 64 * 128;             // 64 keys x 64 d bf16
constexpr int FWD_STAGE = 2 * FWD_TILE + 256;  // K tile, V tile, key-mask row
constexpr int FWD_MAX_NKV = 9;                 // L <= 576 (BERT: 512 text + image tokens)

// ---------------------------------------------------------------- forward v2 (lean softmax)
// attn_fwd_dma_kernel's ring and tiling with the per-element VALU work cut down (the v1
// forward issued ~750 VALU per 16 MFMAs per tile and measured VALU-busy ~88 %):
//  * K and V rows are DMA'd into LDS in a key permutation kappa (within each 32-key half,
//    LDS row 8a + 4h + b holds key 16h + 4a + b), so the S^T accumulator register r of
//    half-wave h holds key 16h + r: each lane's 16 keys per half are CONTIGUOUS (mask row
//    read as 4 x 16 B, dropout counters consecutive, keep bits a 16-bit field).  P^T and V
//    share the permutation, so P V is unchanged;
//  * the key-mask row enters as the S accumulator's initial value, so S' = S/8 + mask
//    costs no VALU; p = exp2(fma(S', log2e, -m log2e)): one FMA + one v_exp per element;
//  * deferred max (rescale O and l only when a row's max grew by > 8 in log2 units, so
//    P <= 2^8 between rescales; wave-uniform branch);
//  * the row sum stays per half-wave until the end (one shuffle per block, not per tile);
//  * the partial last key tile is a separate instantiation (no key < L tests in full
//    tiles), and when at most 32 of its keys are live only that half is computed;
//  * dropout: one full hash per 16 keys of a row, 16-bit draws of each key pair from a
//    multiply of it; compare / select / keep-bit shift-in (v_addc) as 3 VALU per element;
//  * O leaves through LDS as 16-B row stores.
// Needs ceil(L/64) <= FWD_MAX_NKV and ld_out % 8 == 0.
constexpr float DEFER_LOG2 = 8.0f;
// 24-bit odd multipliers of the per-pair draws (v_mul_u32_u24: full rate; the 32-bit
// v_mul_lo_u32 of the earlier draws is a quarter-rate op, 20 of them per tile)
constexpr uint32_t kDropMul24[8] = {0x9E3779u, 0x85EBCBu, 0xC2B2AFu, 0xA7D4EBu,
                                    0x965667u, 0xD3A265u, 0xFD7047u, 0xB55A4Fu};

// 32 bits of pair i's two 16-bit draws from the block hash hb: rotate hb by 4i (so every
// pair multiplies a different 24-bit window), 24-bit multiply, fold the high half into
// the low one.  Measured over 2^22 random hb: per-key drop rates 0.1 +- 3e-4, the 120
// pairwise correlations of the 16 decisions within noise (max |r| 1.4e-3 vs 1/sqrt(N) =
// 4.9e-4), joint drop counts binomial (tools/dropout_draws.py).
static __device__ __forceinline__ uint32_t pair_draw(uint32_t hb, int i) {
  const uint32_t src = i ? __builtin_amdgcn_alignbit(hb, hb, 4 * i) : hb;  // rotr(hb, 4i)
  const uint32_t x = __umul24(src, kDropMul24[i]);
  return x ^ (x >> 16);
}

static __device__ __forceinline__ int kperm(int i) {  // LDS row i of a 32-key half -> key
  return (((i >> 2) & 1) << 4) | (((i >> 3) & 3) << 2) | (i & 3);
}

// keep decisions of key pair (2i, 2i+1) from one 32-bit hash (low half -> even key):
// zero the dropped P values and shift the two keep bits into w (odd key first, so that a
// descending walk leaves bit k of w = element k)
// the same decisions without the keep bits (inference: no backward reads them)
static __device__ __forceinline__ void drop_pair_zero(uint32_t hsh, uint32_t thr, uint32_t thr_hi, float e0,
                                                      float e1, float& o0, float& o1) {
  asm("v_cmp_le_u32 vcc, %[th], %[h]\n\t"
      "v_cndmask_b32 %[o1], 0, %[e1], vcc\n\t"
      "v_cmp_le_u16 vcc, %[t], %[h]\n\t"
      "v_cndmask_b32 %[o0], 0, %[e0], vcc"
      : [o0] "=&v"(o0), [o1] "=&v"(o1)
      : [e0] "v"(e0), [e1] "v"(e1), [h] "v"(hsh), [t] "s"(thr), [th] "s"(thr_hi)
      : "vcc");
}

// the kept values go to fresh registers (o0, o1): the undropped e0 / e1 stay live for the
// row sum without the copies an in-place ("+v") operand costs (32 v_mov per tile)
static __device__ __forceinline__ void drop_pair_apply(uint32_t hsh, uint32_t thr, uint32_t thr_hi, float e0,
                                                       float e1, float& o0, float& o1, uint32_t& w) {
  asm("v_cmp_le_u32 vcc, %[th], %[h]\n\t"
      "v_cndmask_b32 %[o1], 0, %[e1], vcc\n\t"
      "v_addc_co_u32 %[w], vcc, %[w], %[w], vcc\n\t"
      "v_cmp_le_u16 vcc, %[t], %[h]\n\t"
      "v_cndmask_b32 %[o0], 0, %[e0], vcc\n\t"
      "v_addc_co_u32 %[w], vcc, %[w], %[w], vcc"
      : [o0] "=&v"(o0), [o1] "=&v"(o1), [w] "+v"(w)
      : [e0] "v"(e0), [e1] "v"(e1), [h] "v"(hsh), [t] "s"(thr), [th] "s"(thr_hi)
      : "vcc");
}

// STORE = false: dropout without the keep-bit words (p.dropmask ignored): MC-dropout
// inference, where no backward reads them; fewer live registers -> 3 waves / SIMD
template <bool DROP, int WPE, bool NOHOIST, bool STORE = true>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void attn_fwd_v2_kernel(AttnParams p) {
  __shared__ __attribute__((aligned(16))) char smem[FWD_NS * FWD_STAGE + 4 * 32 * FWD_MAX_NKV * 8];
  uint64_t* kbuf_all = (uint64_t*)(smem + FWD_NS * FWD_STAGE);
  const int t = threadIdx.x, l = t & 63, l_ = l, h = l >> 5;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  int bx, bh;
  block_coords(bx, bh);
  const int b = bh / p.heads, hd = bh - b * p.heads;
  const int L = p.L, HD = p.heads * 64;
  const int q0w = bx * 128 + 32 * w, q = q0w + (l & 31);
  const bool wave_live = q0w < L;
  const bf16* base = p.qkv + (int64_t)b * L * p.ld_qkv + hd * 64;
  const uint32_t thr = drop_thr(p.drop_p), thr_hi = thr << 16;
  const int nkv = (L + 63) / 64;
  uint64_t* kbuf = kbuf_all + w * 32 * nkv;
  const bool store_bits = STORE && DROP && p.dropmask != nullptr;
  // dropout counter base of row q: seed_bh + 4 (q nkv) + 2h  (+ 4j + s2 per tile half)
  const uint32_t ctr = seed_for(mmu_eff_seed(p.seed, p.seed_off), bh) + 4u * (uint32_t)q * (uint32_t)nkv + 2u * (uint32_t)h;

  const void* kv_base = p.qkv + (int64_t)b * L * p.ld_qkv;
  const int kv_bytes = (int)(L * p.ld_qkv * 2);
  const void* m_base = p.keymask + (int64_t)b * L;
  bf16x8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    uint4 u = q < L ? *(const uint4*)(base + (int64_t)q * p.ld_qkv + 16 * ks + 8 * h) : make_uint4(0, 0, 0, 0);
    qf[ks] = scale_frag(u, 0.125f);
  }
  f32x16 o[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) { o[0][i] = 0.f; o[1][i] = 0.f; }
  float m_run = NEG_INF, nml = 0.f;  // nml = -m_run * log2e
  // row-sum partials as scalar f32 (packed v_pk_add_f32 / v_pk_fma_f32 beside MFMAs cost more
  // issue cycles than two scalar ops: MI355X_MICROARCH 'price of one filler beside MFMAs')
  float lsum[4] = {0.f, 0.f, 0.f, 0.f};

  // per tile: waves 0,1 -> K pieces, waves 2,3 -> V pieces (4 each, rows in kperm order);
  // wave 0 also the (unpermuted) mask row.  The lane's source offsets within a tile are
  // loop-invariant; the tile's row offset goes in the DMA's scalar offset
  uint32_t kv_off[4];
#pragma unroll
  for (int pc = 0; pc < 4; ++pc) {
    const int piece = 4 * (w & 1) + pc;
    const int row = 8 * piece + (l >> 3), c = (l & 7) ^ fsw(row);
    const int key = (row & 32) | kperm(row & 31);
    kv_off[pc] = (uint32_t)((key * p.ld_qkv + (w < 2 ? HD : 2 * HD) + hd * 64 + 8 * c) * 2);
  }
  const uint32_t m_off = (uint32_t)(16 * l);
  auto issue = [&](int j) {
    char* st = smem + (j % FWD_NS) * FWD_STAGE;
    const int k0 = j * 64;
    char* dst = st + (w < 2 ? 0 : FWD_TILE);
    const __amdgpu_buffer_rsrc_t rt = urs_at(kv_base, kv_bytes, k0 * p.ld_qkv * 2);
#pragma unroll
    for (int pc = 0; pc < 4; ++pc) dma16(rt, dst + (4 * (w & 1) + pc) * 1024, kv_off[pc]);
    if (w == 0 && l < 16) dma16(urs_at(m_base, L * 4, k0 * 4), st + 2 * FWD_TILE, m_off);
  };
  auto wait_for = [&](int ahead) {
    if (w == 0) {
      if (ahead >= 1) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (ahead >= 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  };

  // one 64-key tile; PARTIAL: keys >= L exist in it (the last tile only).  Register r of
  // sc[s2] holds key 64j + 32 s2 + 16h + r.
  auto tile = [&](int j, auto partial_tag, const char* st) {
    constexpr bool PARTIAL = decltype(partial_tag)::value;
    const char* Ks = st;
    const char* Vs = st + FWD_TILE;
    const float* mk = (const float*)(st + 2 * FWD_TILE);
    const bool two = !PARTIAL || L - 64 * j > 32;  // second 32-key half has live keys
    // NOHOIST: re-derive the lane's LDS addresses per tile instead of keeping ~30 hoisted
    // lane constants live across the loop (they spill at the 3-wave register cap)
    int l = l_;
    if (NOHOIST) asm volatile("" : "+v"(l));
    f32x16 sc[2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 mv = *(const f32x4*)(mk + 32 * s2 + 16 * h + 4 * g);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = mv[e];
          if (PARTIAL && 64 * j + 32 * s2 + 16 * h + 4 * g + e >= L) v = NEG_INF;
          sc[s2][4 * g + e] = v;
        }
      }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      sc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(Ks, 0, ks, l), qf[ks], sc[0], 0, 0, 0);
    if (two) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        sc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(Ks, 32, ks, l), qf[ks], sc[1], 0, 0, 0);
    }
    float mx = max3f(sc[0][0], sc[0][1], sc[0][2]);
#pragma unroll
    for (int r = 3; r < 15; r += 2) mx = max3f(mx, sc[0][r], sc[0][r + 1]);
    mx = __builtin_fmaxf(mx, sc[0][15]);
    if (two) {
#pragma unroll
      for (int r = 0; r < 16; r += 2) mx = max3f(mx, sc[1][r], sc[1][r + 1]);
    }
    mx = __builtin_fmaxf(mx, __shfl_xor(mx, 32, 64));
    // deferred max: rescale only when a row's max grew by more than DEFER_LOG2 (log2 units)
    const bool upd = (mx - m_run) * LOG2E > DEFER_LOG2;  // m_run = -inf: true
    if (__builtin_amdgcn_ballot_w64(upd)) {
      const float mnew = upd ? mx : m_run;
      const float alpha = upd ? __builtin_amdgcn_exp2f((m_run - mnew) * LOG2E) : 1.0f;  // exp2(-inf) = 0
#pragma unroll
      for (int i = 0; i < 4; ++i) lsum[i] *= alpha;
#pragma unroll
      for (int i = 0; i < 16; ++i) { o[0][i] *= alpha; o[1][i] *= alpha; }
      m_run = mnew;
      nml = -mnew * LOG2E;
    }
    // per 32-key half: exponentials, dropout, then its P V MFMAs (the second half's VALU
    // overlaps the first half's MFMAs; fewer live registers)
    // dropout stream of (row q, tile j, half s2, half-wave h): counter ctr + 4j + s2
    const uint32_t c0 = ctr + 4u * (uint32_t)j;
    uint32_t wb[2] = {0u, 0u};  // bit r of wb[s2] = keep(register r of sc[s2])
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      if (s2 == 1 && !two) break;
      // exponent arguments and the row sum as scalar f32 (4 partial sums per lane)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float e = __builtin_amdgcn_exp2f(fmaf(sc[s2][i], LOG2E, nml));
        sc[s2][i] = e;
        lsum[i & 3] += e;
      }
      if (DROP) {
        // one full hash per (row, tile, half, half-wave); its 8 pairs' 32-bit draws come
        // from pair_draw (3 full-rate VALU per pair instead of a 7-VALU hash)
        const uint32_t hb = lowbias32(c0 + (uint32_t)s2);
#pragma unroll
        for (int i = 7; i >= 0; --i) {
          const uint32_t hsh = pair_draw(hb, i);
          float o0, o1;
          if (STORE) drop_pair_apply(hsh, thr, thr_hi, sc[s2][2 * i], sc[s2][2 * i + 1], o0, o1, wb[s2]);
          else drop_pair_zero(hsh, thr, thr_hi, sc[s2][2 * i], sc[s2][2 * i + 1], o0, o1);
          sc[s2][2 * i] = o0;
          sc[s2][2 * i + 1] = o1;
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        // (partial tile: keys 8-15 and 24-31 of the half all past L -- L = 513 -- skip their
        // P V step: their P is exactly 0)
        if (PARTIAL && u == 1 && 64 * j + 32 * s2 + 8 >= L) break;
        const bf16x8 pf = acc_frag(sc[s2], u);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
          o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(Vs, 32 * s2 + 16 * u, 32 * dt, l), pf, o[dt], 0, 0, 0);
      }
    }
    if (store_bits) {  // row word: keys 16h..16h+15 <- wb[0], keys 32+16h.. <- wb[1]
      const uint64_t mine = ((uint64_t)(wb[1] & 0xFFFFu) << (32 + 16 * h)) | ((uint64_t)(wb[0] & 0xFFFFu) << (16 * h));
      const uint32_t lo = (uint32_t)mine | (uint32_t)__shfl_xor((int)(uint32_t)mine, 32, 64);
      const uint32_t hi = (uint32_t)(mine >> 32) | (uint32_t)__shfl_xor((int)(uint32_t)(mine >> 32), 32, 64);
      if (h == 0) kbuf[(l & 31) * nkv + j] = ((uint64_t)hi << 32) | lo;
    }
  };

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int j = 0; j < FWD_NS - 1 && j < nkv; ++j) issue(j);
  // full tiles in the loop, the partial last tile (if any) peeled after it: one tile body
  // per loop keeps the O / row-sum registers in place across iterations (a full / partial
  // select inside the loop made hipcc shuffle them with ~18 v_mov_b64 per tile)
  const int nfull = L / 64;
  auto step = [&](int j) {
    const int ahead = nkv - 1 - j < FWD_NS - 2 ? nkv - 1 - j : FWD_NS - 2;
    wait_for(ahead);
    raw_barrier();
    if (j + FWD_NS - 1 < nkv) issue(j + FWD_NS - 1);
  };
  // full tiles unrolled by the ring depth: the stage base is a constant folded into the
  // ds_read immediate offsets (a runtime (j % 2) * stage base cost ~25 address VALU per tile)
  static_assert(FWD_NS == 2, "the forward loop is unrolled by its ring depth");
  for (int j = 0; j < nfull; j += 2) {
    step(j);
    if (wave_live) tile(j, std::integral_constant<bool, false>{}, smem);
    if (j + 1 < nfull) {
      step(j + 1);
      if (wave_live) tile(j + 1, std::integral_constant<bool, false>{}, smem + FWD_STAGE);
    }
  }
  if (nfull < nkv) {
    step(nfull);
    if (wave_live) tile(nfull, std::integral_constant<bool, true>{}, smem + (nfull % FWD_NS) * FWD_STAGE);
  }
  raw_barrier();  // every wave is done with the ring: it becomes the O staging area
  if (!wave_live) return;
  if (store_bits) {  // this wave's 32 rows x nkv words are contiguous in the dropmask
    uint64_t* dst = p.dropmask + ((int64_t)bh * L + q0w) * nkv;
    const int rows = L - q0w < 32 ? L - q0w : 32;
    for (int i = l; i < rows * nkv; i += 64) dst[i] = kbuf[i];
  }
  const float l_run = (lsum[0] + lsum[1]) + (lsum[2] + lsum[3]);
  const float lsum_row = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = (DROP ? 1.0f / (1.0f - p.drop_p) : 1.0f) / lsum_row;
  // O rows through LDS: [32 rows][128 B] per wave, 16-B chunk c of row r at c ^ (r & 7)
  char* os = smem + w * 4096;
  const int qr = l & 31;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const bf16x4 v = {f2bf(o[dt][4 * g] * inv), f2bf(o[dt][4 * g + 1] * inv), f2bf(o[dt][4 * g + 2] * inv),
                        f2bf(o[dt][4 * g + 3] * inv)};
      *(bf16x4*)(os + qr * 128 + (((4 * dt + g) ^ (qr & 7)) << 4) + 8 * h) = v;
    }
  if (h == 0 && q < L) p.lse[(int64_t)bh * L + q] = m_run + logf(lsum_row);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's LDS rows are written (wave-private)
  bf16* ob = p.out + hd * 64;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = (l >> 3) + 8 * i, c = l & 7;
    if (q0w + r < L)
      *(uint4*)(ob + ((int64_t)b * L + q0w + r) * p.ld_out + 8 * c) = *(const uint4*)(os + r * 128 + ((c ^ (r & 7)) << 4));
  }
}

void attention_fwd_launch(const AttnParams& p, hipStream_t s) {
  dim3 grid((p.L + 127) / 128, p.batch * p.heads);
  if (drop_thr(p.drop_p) && !p.dropmask) {
    // inference dropout (MC-dropout passes): no keep bits to store, 3 waves / SIMD
    hipLaunchKernelGGL((attn_fwd_v2_kernel<true, 3, true, false>), grid, dim3(256), 0, s, p);
  } else if (drop_thr(p.drop_p)) {
    // training dropout at 2 waves / SIMD (at the 3-wave register cap it spills lane-constant
    // LDS addresses around the loop: 0.89 vs 0.59 ms at B = 256, L = 513, p = 0.1)
    hipLaunchKernelGGL((attn_fwd_v2_kernel<true, 2, false>), grid, dim3(256), 0, s, p);
  } else {
    hipLaunchKernelGGL((attn_fwd_v2_kernel<false, 3, false>), grid, dim3(256), 0, s, p);
  }
}

// ------------------------------------------------------------------ dK/dV, LDS-DMA ring
// Same math and tiles as attn_dkdv_kernel, but the per-query-tile operands (Q and dO rows,
// -LSE, delta, keep bits) arrive by buffer_load...lds into a 4-deep LDS ring, issued 3
// tiles ahead: the register-staged version waits for each tile's HBM/L2 round trip
// behind one tile of compute.  Lane-linear DMA images: Q / dO chunk swizzle applied to the
// SOURCE address (same image as TileLoader writes); rows past L read as zero through the
// per-(batch item) buffer range (zero Q and dO rows contribute nothing).  K is pre-scaled
// by 1/8 in registers (exact), so dK gets the 1/8 at the end.  One raw s_barrier per tile
// (no __syncthreads: it would drain the DMA queue).
constexpr int DK_NS = 4;                                   // ring depth
constexpr int DK_TILE = 32 * 128;                          // 32 rows x 64 d bf16
constexpr int DK_ROWS = 32 * 4 + 32 * 4 + 32 * 8;          // -lse (as lse), -delta, keep words
constexpr int DK_STAGE = 2 * DK_TILE + DK_ROWS;            // 8704 B


// DROP is a template parameter: a runtime `drop ? keepword : ~0` select around the LDS read
// made hipcc branch around every one of the 16 per-tile keep-word loads.
template <bool DROP>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2))) void attn_dkdv_dma_kernel(AttnParams p) {
  __shared__ __attribute__((aligned(16))) char smem[DK_NS * DK_STAGE];
  const int t = threadIdx.x, l = t & 63, h = l >> 5;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  int bx, bh;
  block_coords(bx, bh);
  const int b = bh / p.heads, hd = bh - b * p.heads;
  const int L = p.L, HD = p.heads * 64;
  const int k0w = bx * 64 + 32 * w, key = k0w + (l & 31);
  const bool wave_live = k0w < L, kv = key < L;
  const bool drop = DROP;
  const float zs = drop ? 1.0f / (1.0f - p.drop_p) : 1.0f;
  const int lane31 = l & 31;
  const int nkv = (L + 63) / 64;
  const float mkey = kv ? p.keymask[(int64_t)b * L + key] * LOG2E : NEG_INF;
  const bf16* base = p.qkv + (int64_t)b * L * p.ld_qkv + hd * 64;

  // operand buffers of this (batch item, head): rows beyond L are out of range -> zero
  const void* q_base = p.qkv + (int64_t)b * L * p.ld_qkv;
  const int q_bytes = (int)(L * p.ld_qkv * 2);
  const void* do_base = p.dout + (int64_t)b * L * p.ld_do;
  const int do_bytes = (int)(L * p.ld_do * 2);
  const void* l_base = p.lse + (int64_t)bh * L;
  const void* d_base = p.delta + (int64_t)bh * L;
  const void* k_base = drop ? (const void*)(p.dropmask + (int64_t)bh * L * nkv) : nullptr;

  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    uint4 u = kv ? *(const uint4*)(base + (int64_t)key * p.ld_qkv + HD + 16 * ks + 8 * h) : make_uint4(0, 0, 0, 0);
    uint4 v = kv ? *(const uint4*)(base + (int64_t)key * p.ld_qkv + 2 * HD + 16 * ks + 8 * h) : make_uint4(0, 0, 0, 0);
    kf[ks] = scale_frag(u, -0.125f);  // exact; S enters negated: the accumulator starts at +lse
    vf[ks] = *(bf16x8*)&v;
  }
  f32x16 dk[2], dv[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) { dk[0][i] = 0.f; dk[1][i] = 0.f; dv[0][i] = 0.f; dv[1][i] = 0.f; }

  const int nq = (L + 31) / 32;
  // per tile: wave 0 -> Q pieces 0..3, lse, delta (6 DMAs); wave 1 -> dO pieces 0..3, keep (5).
  // Lane offsets within a tile are loop-invariant; the tile's row offset goes in the scalar offset
  uint32_t pc_off[4];
  const int ldr = w == 0 ? p.ld_qkv : p.ld_do;
#pragma unroll
  for (int pc = 0; pc < 4; ++pc) {
    const int row = 8 * pc + (l >> 3), c = (l & 7) ^ fsw(row);
    pc_off[pc] = (uint32_t)((row * ldr + hd * 64 + 8 * c) * 2);
  }
  const uint32_t row_off = (uint32_t)(16 * l), kw_off = (uint32_t)((((l >> 1) * nkv + bx) * 8) + 4 * (l & 1));
  auto issue = [&](int i) {
    char* st = smem + (i % DK_NS) * DK_STAGE;
    const int q0 = i * 32;
    if (w == 0) {
      const __amdgpu_buffer_rsrc_t rt = urs_at(q_base, q_bytes, q0 * p.ld_qkv * 2);
#pragma unroll
      for (int pc = 0; pc < 4; ++pc) dma16(rt, st + pc * 1024, pc_off[pc]);
      if (l < 8) {
        dma16(urs_at(l_base, L * 4, q0 * 4), st + 2 * DK_TILE, row_off);
        dma16(urs_at(d_base, L * 4, q0 * 4), st + 2 * DK_TILE + 128, row_off);
      }
    } else {
      const __amdgpu_buffer_rsrc_t rt = urs_at(do_base, do_bytes, q0 * p.ld_do * 2);
#pragma unroll
      for (int pc = 0; pc < 4; ++pc) dma16(rt, st + DK_TILE + pc * 1024, pc_off[pc]);
      // keep word of query row q0 + l/2 for this key block: 4 B per lane (low / high half)
      dma4(urs_at(k_base, drop ? L * nkv * 8 : 0, q0 * nkv * 8), st + 2 * DK_TILE + 256, kw_off);
    }
  };
  // vmcnt: this wave's DMAs per tile (6 or 5) times the tiles allowed to stay in flight
  auto wait_for = [&](int ahead) {
    if (w == 0) {
      if (ahead >= 2) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (ahead >= 2) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  };
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // K / V fragment loads
  for (int i = 0; i < DK_NS - 1 && i < nq; ++i) issue(i);
  // one query tile; the loop below is unrolled by the ring depth so the stage is a compile-time
  // constant folded into the ds_read immediate offsets (a runtime (i % 4) * stage base cost 32
  // address VALU per tile)
  auto qtile = [&](int i, auto sg_tag) {
    constexpr int SG = decltype(sg_tag)::value;
    // tiles i+1, i+2 may stay in flight; tile i must have landed for every wave
    const int ahead = nq - 1 - i < DK_NS - 2 ? nq - 1 - i : DK_NS - 2;
    wait_for(ahead);
    raw_barrier();
    if (i + DK_NS - 1 < nq) issue(i + DK_NS - 1);  // into the stage tile i-1 used (all waves are past it)
    const char* st = smem + SG * DK_STAGE;
    const char* Qs = st;
    const char* Ds = st + DK_TILE;
    const float* lse = (const float*)(st + 2 * DK_TILE);
    const float* dlt = lse + 32;
    const uint32_t* kbit = (const uint32_t*)(st + 2 * DK_TILE + 256) + w;  // [32 rows][2 halves], this wave's half
    if (wave_live) {
      // row constants of the 16 query rows a lane's registers hold: r -> row (r&3) + 8(r>>2) + 4h,
      // i.e. four runs of 4 consecutive rows -> 16-B LDS reads (keep words: stride-2 pairs)
      f32x4 l4[4], nd4[4];  // +lse, -delta/zs of the 16 rows (dQ stores delta so)
      uint32_t kwr[16];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        l4[j] = *(const f32x4*)(lse + 8 * j + 4 * h);
        nd4[j] = *(const f32x4*)(dlt + 8 * j + 4 * h);
        if (DROP)
#pragma unroll
          for (int i2 = 0; i2 < 4; ++i2) kwr[4 * j + i2] = kbit[2 * (8 * j + 4 * h + i2)];
      }
      // the accumulators start at the row constants: sc = lse - S (K negated), dp = dP - delta/zs.
      // p = exp2(-log2e sc + mask);  dS / zs = p (keep ? dp : -delta/zs),  dropped P / zs =
      // keep ? p : 0 -- the keep bit as an all-ones / zero mask (v_bfe_i32 of the row's keep
      // word at this lane's key) bit-selecting; the 1/(1-p) of both goes into dK / dV at the end
      f32x16 sc, dp;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        sc[r] = l4[r >> 2][r & 3];
        dp[r] = nd4[r >> 2][r & 3];
      }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(Qs, 0, ks, l), kf[ks], sc, 0, 0, 0);
        dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(Ds, 0, ks, l), vf[ks], dp, 0, 0, 0);
      }
      f32x16 pz;  // dropped P / zs (for dV)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float pr = __builtin_amdgcn_exp2f(fmaf(sc[r], -LOG2E, mkey));
        if (DROP) {
          const uint32_t m = keepmask(kwr[r], lane31);
          pz[r] = __uint_as_float(m & __float_as_uint(pr));
          sc[r] = pr * __uint_as_float(bfi(m, __float_as_uint(dp[r]), __float_as_uint(nd4[r >> 2][r & 3])));
        } else {
          pz[r] = pr;
          sc[r] = pr * dp[r];
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        // a last query tile whose live rows all sit in its first 16 (L = 513: one) skips the
        // second 16: their Q / dO rows are the zeros past L, which add exactly nothing
        if (s2 == 1 && 32 * i + 16 >= L) break;
        bf16x8 pf = acc_frag(pz, s2), sf = acc_frag(sc, s2);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          dv[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pf, tr_frag(Ds, 16 * s2, 32 * dt, l), dv[dt], 0, 0, 0);
          dk[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sf, tr_frag(Qs, 16 * s2, 32 * dt, l), dk[dt], 0, 0, 0);
        }
      }
    }
  };
  for (int i0 = 0; i0 < nq; i0 += DK_NS) {
    qtile(i0, std::integral_constant<int, 0>{});
    if (i0 + 1 < nq) qtile(i0 + 1, std::integral_constant<int, 1>{});
    if (i0 + 2 < nq) qtile(i0 + 2, std::integral_constant<int, 2>{});
    if (i0 + 3 < nq) qtile(i0 + 3, std::integral_constant<int, 3>{});
  }
  static_assert(DK_NS == 4, "the dK/dV loop is unrolled by its ring depth");
  // dK = (1/8) zs sum dS' Q, dV = zs sum P' dO (the primes: the loop's values, 1/zs of the true ones)
  const float dks = 0.125f * zs;
  if (p.colsum) {  // bias-gradient partials of K and V: this block's 64 keys, per column
    // each lane holds ONE column (32 dt + l&31) for 16 keys: in-lane sum + the other half-wave
    float* red = (float*)smem;  // [2 waves][K 64 | V 64]
    raw_barrier();              // every wave is done with the ring
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      float sk = 0.f, sv = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const bool ok = k0w + (r & 3) + 8 * (r >> 2) + 4 * h < L;
        sk += ok ? dk[dt][r] : 0.f;
        sv += ok ? dv[dt][r] : 0.f;
      }
      sk += __shfl_xor(sk, 32, 64);
      sv += __shfl_xor(sv, 32, 64);
      if (h == 0) {
        red[w * 128 + 32 * dt + l] = sk * dks;
        red[w * 128 + 64 + 32 * dt + l] = sv * zs;
      }
    }
    raw_barrier();
    if (t < 128) {
      const int nqb = (L + 127) / 128, nkb = (L + 63) / 64, B = p.batch;
      const float v = red[t] + red[128 + t];
      const int64_t row = (int64_t)nqb * B + (t < 64 ? 0 : (int64_t)nkb * B) + (int64_t)bx * B + b;
      p.colsum[row * HD + hd * 64 + (t & 63)] = v;
    }
  }
  if (!wave_live) return;
  bf16* outb = p.out + (int64_t)b * L * p.ld_out + hd * 64;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int kk = k0w + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (kk < L) {
        const int64_t off = (int64_t)kk * p.ld_out + 32 * dt + (l & 31);
        outb[off + HD] = f2bf(dk[dt][r] * dks);
        outb[off + 2 * HD] = f2bf(dv[dt][r] * zs);
      }
    }
}

// ------------------------------------------------------------------ dQ, LDS-DMA ring
// attn_dq_kernel with its K / V tiles, key-mask row and (per wave) keep words arriving by
// buffer_load...lds into a 3-deep ring, issued 2 tiles ahead, one raw barrier per tile.
// Keys past L read as zero K / V rows and mask 0: their P is finite but multiplies zero K
// rows (dQ += dS K) and zero V rows (dP), so they add nothing.
constexpr int DQ_NS = 3;  // (the main loop below is unrolled by exactly 3)
constexpr int DQ_TILE = 64 * 128;                         // 64 keys x 64 d bf16
constexpr int DQ_STAGE = 2 * DQ_TILE + 256 + 4 * 256;     // K, V, mask row, 4 waves x 32 keep words

// 3 waves / SIMD: with the softmax math scalar (no v_pk_*_f32) the kernel needs 158 VGPRs
// (218 with the packed pairs), under the 168 of the 3-wave budget (profiles/r4_attn_scalar_ab.txt)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void attn_dq_dma_kernel(AttnParams p) {
  __shared__ __attribute__((aligned(16))) char smem[DQ_NS * DQ_STAGE];
  const int t = threadIdx.x, l = t & 63, h = l >> 5;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  int bx, bh;
  block_coords(bx, bh);
  const int b = bh / p.heads, hd = bh - b * p.heads;
  const int L = p.L, HD = p.heads * 64;
  const int q0w = bx * 128 + 32 * w, q = q0w + (l & 31);
  const bool wave_live = q0w < L, qv = q < L;
  const bool drop = drop_thr(p.drop_p) != 0;
  const float zs = drop ? 1.0f / (1.0f - p.drop_p) : 1.0f;
  const int nkv = (L + 63) / 64;
  const bf16* base = p.qkv + (int64_t)b * L * p.ld_qkv + hd * 64;

  const void* kv_base = p.qkv + (int64_t)b * L * p.ld_qkv;
  const int kv_bytes = (int)(L * p.ld_qkv * 2);
  const void* m_base = p.keymask + (int64_t)b * L;
  const void* k_base = drop ? (const void*)(p.dropmask + (int64_t)bh * L * nkv) : nullptr;
  const int k_bytes = drop ? (int)(L * nkv * 8) : 0;

  bf16x8 qf[4], df[4];
  const bf16* dob = p.dout + ((int64_t)b * L + q) * p.ld_do + hd * 64;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    uint4 u = qv ? *(const uint4*)(base + (int64_t)q * p.ld_qkv + 16 * ks + 8 * h) : make_uint4(0, 0, 0, 0);
    qf[ks] = scale_frag(u, 0.125f);
    uint4 v = qv ? *(const uint4*)(dob + 16 * ks + 8 * h) : make_uint4(0, 0, 0, 0);
    df[ks] = *(bf16x8*)&v;
  }
  // delta = rowsum(dO * O) of this head, from the dO fragments already in registers and the
  // same 32 columns of O (the half-waves hold the two halves of the row); written for the
  // dK/dV kernel that runs next (replaces the separate attn_delta_kernel pass over O and dO)
  float dsum = 0.f;
  {
    const bf16* ob = p.o + ((int64_t)b * L + q) * p.ld_o + hd * 64;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      uint4 u = qv ? *(const uint4*)(ob + 16 * ks + 8 * h) : make_uint4(0, 0, 0, 0);
      const bf16x8 ov = *(bf16x8*)&u;
#pragma unroll
      for (int e = 0; e < 8; ++e) dsum = fmaf(bf2f(ov[e]), bf2f(df[ks][e]), dsum);
    }
    dsum += __shfl_xor(dsum, 32, 64);
    // stored as -delta/zs: the dK/dV kernel starts its dP accumulators there and selects it for
    // the dropped entries (dS / zs = p (keep ? dP - delta/zs : -delta/zs))
    if (qv && h == 0) p.delta[(int64_t)bh * L + q] = -dsum / zs;
  }
  // -lse log2e: the exponent's per-row constant (p = exp2(log2e S' - lse log2e), S' = S/8 + mask)
  const float nlse2 = qv ? -p.lse[(int64_t)bh * L + q] * LOG2E : -__builtin_huge_valf();
  const float ndz = -dsum / zs;
  const uint32_t ndz_bits = __float_as_uint(ndz);
  f32x16 dq[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) { dq[0][i] = 0.f; dq[1][i] = 0.f; }

  // per tile: waves 0,1 -> K pieces (4 each), waves 2,3 -> V pieces; wave 0 also the mask row;
  // every wave the keep words of its 32 query rows (4 B per lane)
  // (lane offsets within a tile loop-invariant; the tile's row / word offset in the scalar offset)
  uint32_t kv_off[4];
#pragma unroll
  for (int pc = 0; pc < 4; ++pc) {
    const int piece = 4 * (w & 1) + pc;
    const int row = 8 * piece + (l >> 3), c = (l & 7) ^ fsw(row);
    kv_off[pc] = (uint32_t)((row * p.ld_qkv + (w < 2 ? HD : 2 * HD) + hd * 64 + 8 * c) * 2);
  }
  const uint32_t m_off = (uint32_t)(16 * l), kw_off = (uint32_t)(((q0w + (l >> 1)) * nkv * 8) + 4 * (l & 1));
  auto issue = [&](int j) {
    char* st = smem + (j % DQ_NS) * DQ_STAGE;
    const int k0 = j * 64;
    char* dst = st + (w < 2 ? 0 : DQ_TILE);
    const __amdgpu_buffer_rsrc_t rt = urs_at(kv_base, kv_bytes, k0 * p.ld_qkv * 2);
#pragma unroll
    for (int pc = 0; pc < 4; ++pc) dma16(rt, dst + (4 * (w & 1) + pc) * 1024, kv_off[pc]);
    if (w == 0 && l < 16) dma16(urs_at(m_base, L * 4, k0 * 4), st + 2 * DQ_TILE, m_off);
    dma4(urs_at(k_base, k_bytes, j * 8), st + 2 * DQ_TILE + 256 + w * 256, kw_off);
  };
  auto wait_for = [&](int ahead) {
    if (w == 0) {
      if (ahead >= 1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (ahead >= 1) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  };
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int j = 0; j < DQ_NS - 1 && j < nkv; ++j) issue(j);
  // the loop is unrolled by the ring depth so each tile's stage is a compile-time constant
  // and folds into the ds_read immediate offsets (a runtime (j % 3) * stage base cost ~37
  // address VALU per tile)
  auto tile_step = [&](int j, auto sg_tag) {
    constexpr int SG = decltype(sg_tag)::value;
    const int ahead = nkv - 1 - j < DQ_NS - 2 ? nkv - 1 - j : DQ_NS - 2;
    wait_for(ahead);
    raw_barrier();
    if (j + DQ_NS - 1 < nkv) issue(j + DQ_NS - 1);
    const char* st = smem + SG * DQ_STAGE;  // compile-time stage: constant LDS offsets
    const char* Ks = st;
    const char* Vs = st + DQ_TILE;
    const float* mk = (const float*)(st + 2 * DQ_TILE);
    const uint32_t* kwords = (const uint32_t*)(st + 2 * DQ_TILE + 256 + w * 256);  // [32 rows][lo, hi]
    if (wave_live) {
      // keep bits of this lane's query row, pre-shifted by 4h (as in attn_dq_kernel)
      const uint64_t kw = drop ? ((uint64_t)kwords[2 * (l & 31) + 1] << 32 | kwords[2 * (l & 31)]) : ~0ull;
      const uint64_t kwh = kw >> (4 * h);
#pragma unroll
      for (int st2 = 0; st2 < 2; ++st2) {
        // a last tile whose live keys all sit in its first half (L = 513: one) skips the second:
        // its K / V rows are the zeros past L, which add exactly nothing to dQ
        if (st2 == 1 && 64 * j + 32 >= L) break;
        const uint32_t kw32 = (uint32_t)(kwh >> (32 * st2));
        // S starts at the mask: register r holds key kl = 32 st2 + 8 (r >> 2) + 4 h + (r & 3),
        // so each group of 4 registers takes 4 contiguous mask entries (one f32x4 read)
        f32x16 sc, dp;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 mv = *(const f32x4*)(mk + 32 * st2 + 8 * g + 4 * h);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            sc[4 * g + e] = mv[e];
            dp[4 * g + e] = ndz;
          }
        }
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(Ks, 32 * st2, ks, l), qf[ks], sc, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(Vs, 32 * st2, ks, l), df[ks], dp, 0, 0, 0);
        }
        // p = exp2(log2e S' - lse log2e);  dS^T / zs = p * (keep ? dP - delta/zs : -delta/zs):
        // dp started at -delta/zs; the keep bit becomes an all-ones / zero mask (v_bfe_i32) that
        // bit-selects it against -delta/zs (without dropout kw is all ones).  The zs of dS goes
        // into dQ's final scale.
        auto one = [&](auto r_tag) {
          constexpr int r = decltype(r_tag)::value;
          const float pr = __builtin_amdgcn_exp2f(fmaf(sc[r], LOG2E, nlse2));
          const uint32_t m = keepmask<(r & 3) + 8 * (r >> 2)>(kw32);
          sc[r] = pr * __uint_as_float(bfi(m, __float_as_uint(dp[r]), ndz_bits));
        };
        static_for(one, std::make_integer_sequence<int, 16>{});
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          bf16x8 sf = acc_frag(sc, s2);
#pragma unroll
          for (int dt = 0; dt < 2; ++dt)
            dq[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(Ks, 32 * st2 + 16 * s2, 32 * dt, l), sf, dq[dt],
                                                             0, 0, 0);
        }
      }
    }
    };
  for (int j0 = 0; j0 < nkv; j0 += DQ_NS) {
    tile_step(j0, std::integral_constant<int, 0>{});
    if (j0 + 1 < nkv) tile_step(j0 + 1, std::integral_constant<int, 1>{});
    if (j0 + 2 < nkv) tile_step(j0 + 2, std::integral_constant<int, 2>{});
  }
  if (p.colsum) {  // bias-gradient partials of Q: this block's 128 queries, per column
    // lane (query l&31) holds columns 32 dt + 8 g + 4 h + e: rows to LDS, then column sums.
    // Rows padded to 68 floats: at a 64-float stride the 16 lanes of each 16-B write phase
    // hit the same 4 banks (the PMC pass counted 1.3 conflict cycles per LDS instruction).
    constexpr int RS = 68;
    static_assert(4 * 32 * RS * 4 <= DQ_NS * DQ_STAGE, "dQ column-sum rows exceed the ring's LDS");
    float* rows = (float*)smem;  // [4 waves][32 queries][RS]
    raw_barrier();               // every wave is done with the ring
    float* mine = rows + w * 32 * RS + (l & 31) * RS;
    const float sc = qv ? 0.125f * zs : 0.f;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *(float4*)(mine + 32 * dt + 8 * g + 4 * h) =
            make_float4(dq[dt][4 * g] * sc, dq[dt][4 * g + 1] * sc, dq[dt][4 * g + 2] * sc, dq[dt][4 * g + 3] * sc);
    raw_barrier();
    if (t < 64) {
      float v = 0.f;
      for (int r = 0; r < 128; ++r) v += rows[r * RS + t];
      p.colsum[((int64_t)bx * p.batch + b) * HD + hd * 64 + t] = v;
    }
  }
  if (!qv) return;
  bf16* ob = p.out + ((int64_t)b * L + q) * p.ld_out + hd * 64;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float s = 0.125f * zs;
      bf16x4 v = {f2bf(dq[dt][4 * g] * s), f2bf(dq[dt][4 * g + 1] * s), f2bf(dq[dt][4 * g + 2] * s),
                  f2bf(dq[dt][4 * g + 3] * s)};
      *(bf16x4*)(ob + 32 * dt + 8 * g + 4 * h) = v;
    }
}

void attention_bwd_launch(const AttnParams& p, hipStream_t s) {
  // the dQ kernel also computes (and stores) delta = rowsum(dO * O) for the dK/dV kernel
  hipLaunchKernelGGL(attn_dq_dma_kernel, dim3((p.L + 127) / 128, p.batch * p.heads), dim3(256), 0, s, p);
  if (drop_thr(p.drop_p))
    hipLaunchKernelGGL(attn_dkdv_dma_kernel<true>, dim3((p.L + 63) / 64, p.batch * p.heads), dim3(128), 0, s, p);
  else
    hipLaunchKernelGGL(attn_dkdv_dma_kernel<false>, dim3((p.L + 63) / 64, p.batch * p.heads), dim3(128), 0, s, p);
}

}  // namespace mmu
