// extern "C" boundary of libmmu_hip.so (declared in include/mmu.h).
// Validates arguments, flattens structs into kernel params, launches on the caller's
// stream, and reports failures through a thread-local message (mmu_last_error).
#include <stdarg.h>
#include <stdio.h>
#include <map>
#include <tuple>
#include <mutex>
#include <string>
#include <vector>
#include "mmu_internal.h"
#include <cstdlib>
#include <cmath>

using namespace mmu;

static thread_local std::string g_err;

namespace mmu {
const uint64_t* g_seed_off = nullptr;
}

int mmu_set_seed_offset(const uint64_t* dev_counter) {
  g_seed_off = dev_counter;
  return 0;
}

static int fail(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return 1;
}

static int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail("%s: launch failed: %s", what, hipGetErrorString(e));
  return 0;
}

// ------------------------------------------------------------------ timing of mmu_gemm
namespace {
struct Timing {
  std::mutex mu;
  bool on = false;
  bool paused = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pool, used;
  std::vector<double> flops;
} g_t;

std::pair<hipEvent_t, hipEvent_t> take_events() {
  std::lock_guard<std::mutex> lk(g_t.mu);
  std::pair<hipEvent_t, hipEvent_t> ev;
  if (!g_t.pool.empty()) {
    ev = g_t.pool.back();
    g_t.pool.pop_back();
  } else {
    (void)hipEventCreate(&ev.first);
    (void)hipEventCreate(&ev.second);
  }
  return ev;
}
// per-(device, stream) f32 scratch for the split tail rows of mmu_gemm: 32 MiB, allocated on first
// use outside stream capture (NULL: the product runs without the tail split)
constexpr int64_t TAIL_WS_FLOATS = 8ll << 20;
// (slot 0: the split tail's slabs, slot 1: the column-sum partial rows)
float* tail_workspace(int64_t floats, hipStream_t s, int slot = 0) {
  static std::mutex mu;
  static std::map<std::tuple<int, hipStream_t, int>, float*> bufs;
  if (floats > TAIL_WS_FLOATS) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  auto it = bufs.find({dev, s, slot});
  if (it != bufs.end()) return it->second;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return nullptr;
  void* b = nullptr;
  if (hipMalloc(&b, sizeof(float) * TAIL_WS_FLOATS) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  bufs[{dev, s, slot}] = (float*)b;
  return (float*)b;
}
}  // namespace

extern "C" {

int mmu_version(void) { return MMU_ABI_VERSION; }
const char* mmu_last_error(void) { return g_err.c_str(); }

int mmu_timing_enable(int on) {
  std::lock_guard<std::mutex> lk(g_t.mu);
  g_t.on = on != 0;
  for (auto& e : g_t.used) g_t.pool.push_back(e);
  g_t.used.clear();
  g_t.flops.clear();
  return 0;
}

int mmu_timing_pause(int paused) {
  std::lock_guard<std::mutex> lk(g_t.mu);
  g_t.paused = paused != 0;
  return 0;
}

int mmu_timing_read(double* total_ms, int64_t* launches, double* flops) {
  std::lock_guard<std::mutex> lk(g_t.mu);
  double tot = 0.0, fl = 0.0;
  for (size_t i = 0; i < g_t.used.size(); ++i) {
    (void)hipEventSynchronize(g_t.used[i].second);
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, g_t.used[i].first, g_t.used[i].second) != hipSuccess) return fail("timing: elapsed");
    tot += ms;
    fl += g_t.flops[i];
  }
  *total_ms = tot;
  *launches = (int64_t)g_t.used.size();
  *flops = fl;
  return 0;
}

int mmu_gemm(const void* A, int64_t lda, int a_kmajor, const void* B, int64_t ldb, int b_kmajor, void* C,
             int64_t ldc, int c_dtype, int64_t M, int64_t N, int64_t K, int64_t batch, int64_t strideA,
             int64_t strideB, int64_t strideC, const mmu_epilogue* epi, mmu_stream_t stream) {
  if (!A || !B || !C) return fail("mmu_gemm: null operand");
  if (M <= 0 || N <= 0 || K <= 0 || batch <= 0) return fail("mmu_gemm: bad shape M=%ld N=%ld K=%ld", M, N, K);
  if (N % 128) return fail("mmu_gemm: N=%ld must be a multiple of 128", N);
  if ((a_kmajor || b_kmajor) && K % 64) return fail("mmu_gemm: K=%ld must be a multiple of 64 for a K-major operand", K);
  if (!a_kmajor && M % 128) return fail("mmu_gemm: M=%ld must be a multiple of 128 when A is M-major", M);
  if ((lda % 8) || (ldb % 8) || (ldc % 4)) return fail("mmu_gemm: leading dims must be 16-B aligned");
  if (c_dtype != MMU_BF16 && c_dtype != MMU_F32) return fail("mmu_gemm: bad c_dtype");
  GemmParams p{};
  p.A = (const bf16*)A; p.B = (const bf16*)B; p.C = C;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.M = M; p.N = N; p.K = K;
  p.sA = strideA; p.sB = strideB; p.sC = strideC;
  // big (256x256, LDS-DMA) tiling needs >= 256 rows/cols and 32-bit buffer offsets per operand
  // (spans include the rows a 256-tile / 64-deep K-tile may address past the end, so the
  // 32-bit buffer offsets of those out-of-range reads never wrap back into the operand)
  const int64_t a_span = 2 * (a_kmajor ? (M + 256) * lda : (K + 64) * lda);
  const int64_t b_span = 2 * (b_kmajor ? (N + 256) * ldb : (K + 64) * ldb);
  const bool big = M >= 256 && N >= 256 && a_span < (1ll << 32) - 4096 && b_span < (1ll << 32) - 4096;
  const int tile = big ? 256 : 128;
  p.tiles_m = (int)((M + tile - 1) / tile);
  p.tiles_n = (int)((N + tile - 1) / tile);
  // tile-order group height, measured on the BERT shapes (tools/gemm_bench.py; group-height
  // sweeps in profiles/r1_gemm_group_sweep.txt): row-major for <= 3 column tiles, 2 with an N-major B (dY.W2), 8 for the
  // wide forward products (QKV 0.496 -> 0.457 ms, W1+GELU 0.888 -> 0.832 ms)
  int kind = MMU_EPI_STORE;
  if (epi) kind = epi->kind;
  // (and 2 for the dGELU product dY2.W2, whose epilogue streams the [M, 3072] gelu' rows:
  // 0.888 -> 0.756 ms with a K-major B, profiles/r2_gemm_group_dz.txt)
  p.group_m = p.tiles_n <= 3 ? 1 : ((b_kmajor && kind != MMU_EPI_DGELU) ? 8 : 2);
  if (epi) {
    kind = epi->kind;
    p.accumulate = epi->accumulate;
    p.bias = epi->bias; p.bias_bstride = epi->bias_bstride;
    p.residual = epi->residual; p.ldr = epi->ldr; p.res_bstride = epi->res_bstride;
    p.aux = epi->aux; p.ldx = epi->ldx; p.aux_bstride = epi->aux_bstride;
    p.colsum = epi->colsum; p.colsum_bstride = epi->colsum_bstride;
    p.drop_p = epi->drop_p; p.seed = epi->seed; p.seed_off = g_seed_off;
    p.res_ln_mean = epi->res_ln_mean; p.res_ln_rstd = epi->res_ln_rstd;
    p.res_ln_w = epi->res_ln_w; p.res_ln_b = epi->res_ln_b; p.res_ln_bstride = epi->res_ln_bstride;
    p.bn_x = (const bf16*)epi->bn_x; p.bn_mask = epi->bn_mask; p.bn_mean = epi->bn_mean;
    p.res_mask = epi->res_mask;
  }
  p.kind = kind;
  if (kind < 0 || kind > MMU_EPI_ADD_RES_BNB) return fail("mmu_gemm: bad epilogue kind %d", kind);
  if ((kind == MMU_EPI_STORE_BNB || kind == MMU_EPI_ADD_RES_BNB) &&
      (!p.colsum || !p.bn_x || !p.bn_mean || batch != 1 || !a_kmajor || b_kmajor || p.accumulate || p.bias ||
       ldc != N || c_dtype != MMU_BF16))
    return fail("mmu_gemm: *_BNB needs the table (colsum), bn_x, bn_mean, batch 1, K-major A, N-major B, "
                "bf16 C with ldc == N, no bias / accumulate");
  if (kind == MMU_EPI_STORE_STATS && (!p.colsum || batch != 1 || !a_kmajor || !b_kmajor || p.accumulate))
    return fail("mmu_gemm: STORE_STATS needs the stats table (colsum), batch 1, K-major A and B, no accumulate");
  if (kind != MMU_EPI_STORE && kind != MMU_EPI_BIAS_DROP_RES && c_dtype != MMU_BF16)
    return fail("mmu_gemm: fused epilogues other than BIAS_DROP_RES write bf16");
  if (kind == MMU_EPI_BIAS_DROP_RES && c_dtype == MMU_F32 && (ldc % 4 || (epi && epi->ldr % 4)))
    return fail("mmu_gemm: f32 hidden-stream epilogue needs 16-B aligned rows");
  {
    const int nln = !!p.res_ln_mean + !!p.res_ln_rstd + !!p.res_ln_w + !!p.res_ln_b;
    if (nln && (nln != 4 || kind != MMU_EPI_BIAS_DROP_RES || c_dtype != MMU_F32))
      return fail("mmu_gemm: res_ln_* (all four) only with BIAS_DROP_RES into an f32 C");
  }
  if (kind == MMU_EPI_DGELU && !p.aux) return fail("mmu_gemm: DGELU epilogue needs aux");
  if ((kind == MMU_EPI_BIAS_DROP_RES || kind == MMU_EPI_ADD_RES || kind == MMU_EPI_ADD_RES_BNB) && !p.residual)
    return fail("mmu_gemm: epilogue needs residual");
  if (p.res_mask && ((kind != MMU_EPI_ADD_RES && kind != MMU_EPI_ADD_RES_BNB) || epi->ldr != N || batch != 1))
    return fail("mmu_gemm: res_mask only with ADD_RES / ADD_RES_BNB, batch 1, ldr == N");
  if (p.accumulate && c_dtype != MMU_F32) return fail("mmu_gemm: accumulate needs f32 C");
  if (p.drop_p < 0.f || p.drop_p >= 1.f) return fail("mmu_gemm: drop_p out of range");
  // split-K for long-K / few-tile products (the weight gradients: K = tokens, M x N = a weight matrix)
  p.splitk = 1;
  p.kchunk = K;
  if (kind == MMU_EPI_STORE && c_dtype == MMU_F32 && !p.bias && !p.colsum && epi && epi->workspace && K >= 1024) {
    const int64_t tiles = (int64_t)p.tiles_m * p.tiles_n * batch;
    // slice cap 64 / minimum slice depth 1024 (profiles/r2_splitk_cap_ab.txt); short reductions
    // (the batch-32 ResNet filter gradients: K = 1.5-25 K pixels over 4-16 tiles) go down to
    // 256-deep slices so that they still fill the chip
    const int64_t max_split = 64, min_k = K >= 32768 ? 1024 : 256;
    int64_t want = (640 + tiles - 1) / tiles;
    if (want > K / min_k) want = K / min_k;
    if (want > max_split) want = max_split;
    const int64_t cap = epi->workspace_floats / (batch * M * N);
    if (want > cap) want = cap;
    if (want >= 2) {
      int64_t chunk = (K + want - 1) / want;
      chunk = (chunk + 63) / 64 * 64;
      p.kchunk = chunk;
      p.splitk = (int)((K + chunk - 1) / chunk);
      p.ws = epi->workspace;
    }
  }
  // 256 x 384 tiling (gemm_wide_kernel): both operands K-major, N % 384 == 0, no split-K, and at
  // least MMU_GEMM_WIDE_MIN_TILES of its tiles (default 4 per CU: the bench's M = 131 k rows;
  // fewer, larger tiles leave CUs idle on small products).  MMU_GEMM_WIDE=0 turns it off.
  // (read per call, ~1 us: tests switch them inside one process)
  const char* wide_env = getenv("MMU_GEMM_WIDE");
  const char* wide_min_env = getenv("MMU_GEMM_WIDE_MIN_TILES");
  const int wide_mode = wide_env ? atoi(wide_env) : 1;
  const int64_t wide_min = wide_min_env ? (int64_t)atoll(wide_min_env) : (int64_t)1024;
  // (the dGELU product stays on 256 x 256: its aux-row loads and column-sum atomics per 64-row
  // block ran it 15-22 % slower on the wide tile, profiles/r6_gemm_wide_ab.txt)
  const bool tail_kind = kind == MMU_EPI_STORE || kind == MMU_EPI_BIAS_GELU || kind == MMU_EPI_BIAS_DROP_RES ||
                         kind == MMU_EPI_DGELU || kind == MMU_EPI_ADD_RES;
  const bool wide_kind = tail_kind && kind != MMU_EPI_DGELU;
  // Default rule (MMU_GEMM_WIDE=1), same-box A/B: the wide products N >= 2304 (QKV -3 %, FFN1 + GELU
  // -8 % with the split tail); N = 768 stays on 256 x 256 (equal or 2 % slower: its 1026 wide tiles
  // end in a round of 2).  MMU_GEMM_WIDE=2 takes every kind and width (tests).
  const bool wide = (wide_mode == 2 ? tail_kind : wide_mode == 1 && wide_kind && N >= 2304) && big && a_kmajor &&
                    b_kmajor && N % 384 == 0 && p.splitk == 1 &&
                    2 * (M + 256) * lda < (1ll << 32) - 4096 && 2 * (N + 384) * ldb < (1ll << 32) - 4096 &&
                    (M + 255) / 256 * (N / 384) * batch >= wide_min;
  if (wide) {
    p.tiles_m = (int)((M + 255) / 256);
    p.tiles_n = (int)(N / 384);
    p.group_m = p.tiles_n <= 2 ? 1 : (kind != MMU_EPI_DGELU ? 8 : 2);
  }
  // Split tail rows: when the last round of 256-row tiles holds whole tile rows and is at most an
  // eighth full (M = 256 x 513 at batch 256: 1026 wide / 1539 big tiles on 256 CUs), those rows
  // run as split-K partial products of the small tiling into a per-stream f32 scratch, and
  // splitk_epilogue_kernel sums them and applies the same epilogue.  On by default for the wide
  // tiling (MMU_GEMM_TAIL=1), whose tail round is 1.5 big tiles long; 2 = for the 256 x 256 tiling
  // too (tests: there it costs +10-20 us, the 256^2 tail round is short), 0 = off.
  const char* tail_env = getenv("MMU_GEMM_TAIL");
  const int tail_mode = tail_env ? atoi(tail_env) : 1;
  int64_t tail_rows = 0, m_main = M, tail_chunk = K;
  int tail_split = 1;
  float* tail_ws = nullptr;
  if ((tail_mode == 2 || (tail_mode == 1 && wide)) && big && batch == 1 && p.splitk == 1 && tail_kind &&
      a_kmajor && K >= 512) {
    const int64_t tiles = (int64_t)p.tiles_m * p.tiles_n, left = tiles % 256;
    if (tiles > 256 && left > 0 && left % p.tiles_n == 0 && left * 8 <= 256) {
      m_main = (int64_t)(p.tiles_m - left / p.tiles_n) * 256;
      tail_rows = M - m_main;
      const int64_t st = (tail_rows + 127) / 128 * (N / 128);  // small tiles over the tail rows
      int64_t sk = 256 / st;
      if (sk > K / 256) sk = K / 256;  // >= 4 K-steps per slice
      if (sk < 1) sk = 1;
      tail_chunk = ((K + sk - 1) / sk + 63) / 64 * 64;
      tail_split = (int)((K + tail_chunk - 1) / tail_chunk);
      // (a single slice would make the small kernel store its raw product into C: no split then)
      tail_ws = tail_split >= 2 ? tail_workspace((int64_t)tail_split * tail_rows * N, (hipStream_t)stream) : nullptr;
      if (!tail_ws) {
        tail_rows = 0;
        m_main = M;
      }
    }
  }
  hipStream_t s = (hipStream_t)stream;
  bool timed;
  std::pair<hipEvent_t, hipEvent_t> ev;
  {
    std::lock_guard<std::mutex> lk(g_t.mu);
    timed = g_t.on && !g_t.paused;
  }
  if (timed) {
    ev = take_events();
    (void)hipEventRecord(ev.first, s);
  }
  // column sums as partial rows (no float atomics: 50 us of the 0.74 ms dZ product at batch 256,
  // 180 us on the wide tile; profiles/r6_gemm_colsum_ab.txt), folded by one colsum_reduce launch.
  // Rows of 16 NJ per wave block: 128 on the 256 x 256 tile, 64 on the others.  MMU_GEMM_CS_PART=0: atomics.
  const char* csp_env = getenv("MMU_GEMM_CS_PART");
  const bool cs_rows_ok = p.colsum && batch == 1 && p.splitk == 1 && kind != MMU_EPI_STORE_STATS &&
                          kind != MMU_EPI_STORE_BNB && kind != MMU_EPI_ADD_RES_BNB && (!csp_env || atoi(csp_env) != 0);
  const int cs_rows_main = (big && !wide) ? 128 : 64;
  const int64_t cs_parts_main = (m_main + cs_rows_main - 1) / cs_rows_main;
  const int64_t cs_parts = cs_parts_main + (tail_rows + 63) / 64;
  float* cs_part = cs_rows_ok ? tail_workspace(cs_parts * N, s, 1) : nullptr;
  if (cs_part) {
    p.cs_part = cs_part;
    p.cs_m0 = 0;
    p.cs_rows = cs_rows_main;
  }
  {
    GemmParams pm = p;
    if (tail_rows) pm.tiles_m = (int)(m_main / 256);
    if (!(wide && gemm_wide_launch(pm, c_dtype == MMU_F32, (int)batch, s)))
      gemm_launch(pm, a_kmajor != 0, b_kmajor != 0, c_dtype == MMU_F32, big, (int)batch, s);
  }
  if (tail_rows) {
    GemmParams pt = p;
    pt.A = p.A + m_main * lda;
    pt.M = tail_rows;
    pt.kind = MMU_EPI_STORE;
    pt.accumulate = 0;
    pt.splitk = tail_split;
    pt.kchunk = tail_chunk;
    pt.ws = tail_ws;
    pt.tiles_m = (int)((tail_rows + 127) / 128);
    pt.tiles_n = (int)(N / 128);
    pt.group_m = 1;
    pt.cs_part = nullptr;
    gemm_launch(pt, true, b_kmajor != 0, true, false, 1, s);
    GemmParams pe = p;
    if (cs_part) {
      pe.cs_part = cs_part + cs_parts_main * N;
      pe.cs_m0 = m_main;
      pe.cs_rows = 64;
    }
    splitk_epilogue_launch(pe, c_dtype == MMU_F32, tail_ws, m_main, tail_rows, tail_split, s);
  }
  if (cs_part) colsum_reduce_launch(cs_part, cs_parts, N, p.colsum, 1, s);
  if (p.splitk > 1) splitk_reduce_launch(p, (int)batch, s);
  if (timed) {
    (void)hipEventRecord(ev.second, s);
    std::lock_guard<std::mutex> lk(g_t.mu);
    g_t.used.push_back(ev);
    g_t.flops.push_back(2.0 * (double)M * (double)N * (double)K * (double)batch);
  }
  return check_launch("mmu_gemm");
}

int mmu_transpose_bf16_batched(const int64_t* jobs, int n_jobs, int64_t max_rows, int64_t max_cols,
                               mmu_stream_t stream) {
  if (!jobs || n_jobs <= 0 || n_jobs > 65535 || max_rows <= 0 || max_cols <= 0)
    return fail("mmu_transpose_bf16_batched: bad args");
  transpose_bf16_batched_launch(jobs, n_jobs, max_rows, max_cols, (hipStream_t)stream);
  return check_launch("mmu_transpose_bf16_batched");
}

int mmu_colsum_reduce(const float* partial, int64_t parts, int64_t N, float* out, int accumulate,
                      mmu_stream_t stream) {
  if (!partial || !out || parts <= 0 || N <= 0) return fail("mmu_colsum_reduce: bad args");
  colsum_reduce_launch(partial, parts, N, out, accumulate, (hipStream_t)stream);
  return check_launch("mmu_colsum_reduce");
}

int mmu_colsum_reduce_multi(int n, const float* const* partial, const int64_t* parts, float* const* out, int64_t N,
                            int accumulate, mmu_stream_t stream) {
  if (n <= 0 || n > COLSUM_MULTI || !partial || !parts || !out || N <= 0)
    return fail("mmu_colsum_reduce_multi: bad args (1 <= n <= %d)", COLSUM_MULTI);
  ColsumJobs jobs{};
  for (int z = 0; z < n; ++z) {
    if (!partial[z] || !out[z] || parts[z] <= 0) return fail("mmu_colsum_reduce_multi: bad job %d", z);
    jobs.part[z] = partial[z];
    jobs.parts[z] = parts[z];
    jobs.out[z] = out[z];
  }
  colsum_reduce_multi_launch(jobs, n, N, accumulate, (hipStream_t)stream);
  return check_launch("mmu_colsum_reduce_multi");
}

int mmu_colsum_bf16(const void* X, int64_t M, int64_t N, int64_t ldx, float* partial, float* out, int accumulate,
                    mmu_stream_t stream) {
  if (!X || !out || M <= 0 || N <= 0 || N % 8 || ldx % 8) return fail("mmu_colsum_bf16: bad args");
  colsum_bf16_launch((const bf16*)X, M, N, ldx, partial, out, accumulate, (hipStream_t)stream);
  return check_launch("mmu_colsum_bf16");
}

static int attn_common(int64_t ld_qkv, int64_t batch, int64_t L, int64_t heads, float drop_p) {
  if (batch <= 0 || L <= 0 || heads <= 0) return fail("attention: bad shape");
  if (ld_qkv < 3 * heads * 64 || ld_qkv % 8) return fail("attention: ld_qkv too small / unaligned");
  if (drop_p < 0.f || drop_p >= 1.f) return fail("attention: drop_p out of range");
  if ((int64_t)batch * heads > 65535 * 64) return fail("attention: batch*heads too large");
  if (L > 576) return fail("attention: L=%ld > 576 (the kernels stage ceil(L/64) <= 9 key tiles)", L);
  return 0;
}

int mmu_attention_fwd(const void* QKV, int64_t ld_qkv, const float* keymask, void* O, int64_t ld_o, float* LSE,
                      int64_t batch, int64_t L, int64_t heads, float drop_p, uint64_t seed, uint64_t* dropmask,
                      mmu_stream_t stream) {
  if (!QKV || !keymask || !O || !LSE) return fail("mmu_attention_fwd: null pointer");
  if (attn_common(ld_qkv, batch, L, heads, drop_p)) return 1;
  if (ld_o < heads * 64 || ld_o % 8) return fail("mmu_attention_fwd: bad ld_o");
  if (batch * heads > 65535) return fail("mmu_attention_fwd: batch*heads > 65535");
  AttnParams p{};
  p.qkv = (const bf16*)QKV; p.ld_qkv = ld_qkv; p.keymask = keymask; p.out = (bf16*)O; p.ld_out = ld_o;
  p.lse = LSE; p.batch = (int)batch; p.L = (int)L; p.heads = (int)heads; p.drop_p = drop_p; p.seed = seed;
  p.seed_off = g_seed_off;
  p.dropmask = dropmask;
  attention_fwd_launch(p, (hipStream_t)stream);
  return check_launch("mmu_attention_fwd");
}

int mmu_attention_bwd(const void* QKV, int64_t ld_qkv, const float* keymask, const void* O, int64_t ld_o,
                      const void* dO, int64_t ld_do, const float* LSE, float* delta, void* dQKV, int64_t ld_dqkv,
                      int64_t batch, int64_t L, int64_t heads, float drop_p, uint64_t seed,
                      const uint64_t* dropmask, float* dbias_parts, mmu_stream_t stream) {
  if (!QKV || !keymask || !O || !dO || !LSE || !delta || !dQKV) return fail("mmu_attention_bwd: null pointer");
  if ((uint32_t)(drop_p * 65536.0f + 0.5f) != 0 && !dropmask)
    return fail("mmu_attention_bwd: dropout needs the forward's dropmask");
  if (attn_common(ld_qkv, batch, L, heads, drop_p)) return 1;
  if (ld_dqkv < 3 * heads * 64 || ld_do % 8 || ld_o % 8 || ld_dqkv % 4) return fail("mmu_attention_bwd: bad ld");
  if (batch * heads > 65535) return fail("mmu_attention_bwd: batch*heads > 65535");
  AttnParams p{};
  p.qkv = (const bf16*)QKV; p.ld_qkv = ld_qkv; p.keymask = keymask; p.o = (const bf16*)O; p.ld_o = ld_o;
  p.dout = (const bf16*)dO; p.ld_do = ld_do; p.lse = (float*)LSE; p.delta = delta; p.out = (bf16*)dQKV;
  p.ld_out = ld_dqkv; p.batch = (int)batch; p.L = (int)L; p.heads = (int)heads; p.drop_p = drop_p; p.seed = seed;
  p.seed_off = g_seed_off;
  p.dropmask = (uint64_t*)dropmask;
  p.colsum = dbias_parts;
  attention_bwd_launch(p, (hipStream_t)stream);
  return check_launch("mmu_attention_bwd");
}

int mmu_layernorm_fwd(const void* X, const float* w, const float* b, void* Y, float* mean, float* rstd, int64_t rows,
                      int64_t H, float eps, int64_t group_rows, int64_t param_stride, mmu_stream_t stream) {
  if (!X || !w || !b || !Y) return fail("mmu_layernorm_fwd: null pointer");
  if ((mean == nullptr) != (rstd == nullptr)) return fail("mmu_layernorm_fwd: mean/rstd must both be given or NULL");
  if (rows <= 0 || H <= 0 || H % 256 || H > 1024) return fail("mmu_layernorm_fwd: H=%ld must be 256/512/768/1024", H);
  if (group_rows <= 0) group_rows = rows;
  if (param_stride < 0) return fail("mmu_layernorm_fwd: bad param_stride");
  layernorm_fwd_launch((const bf16*)X, w, b, (bf16*)Y, mean, rstd, rows, H, eps, group_rows, param_stride,
                       (hipStream_t)stream);
  return check_launch("mmu_layernorm_fwd");
}

int mmu_layernorm_bwd(const void* dY, const void* X, const float* mean, const float* rstd, const float* w, void* dX,
                      void* dXdrop, float drop_p, uint64_t seed, float* part_dw, float* part_db, float* part_dbias,
                      int64_t rows, int64_t H, int64_t rows_per_part, mmu_stream_t stream) {
  if (!dY || !X || !mean || !rstd || !w || !dX) return fail("mmu_layernorm_bwd: null pointer");
  if (rows <= 0 || H <= 0 || H % 256 || H > 1024 || rows_per_part <= 0) return fail("mmu_layernorm_bwd: bad shape");
  if (drop_p < 0.f || drop_p >= 1.f) return fail("mmu_layernorm_bwd: drop_p out of range");
  layernorm_bwd_launch((const bf16*)dY, X, false, mean, rstd, w, (bf16*)dX, (bf16*)dXdrop, nullptr, drop_p, seed,
                       g_seed_off, part_dw, part_db, part_dbias, rows, H, rows_per_part, (hipStream_t)stream);
  return check_launch("mmu_layernorm_bwd");
}

int mmu_layernorm_fwd_f32(const float* X, const float* w, const float* b, void* Y, float* Y32, float* mean,
                          float* rstd, int64_t rows, int64_t H, float eps, int64_t group_rows, int64_t param_stride,
                          mmu_stream_t stream) {
  if (!X || !w || !b || !Y) return fail("mmu_layernorm_fwd_f32: null pointer");
  if ((mean == nullptr) != (rstd == nullptr)) return fail("mmu_layernorm_fwd_f32: mean/rstd must both be given or NULL");
  if (rows <= 0 || H <= 0 || H % 256 || H > 1024) return fail("mmu_layernorm_fwd_f32: H=%ld must be 256/512/768/1024", H);
  if (group_rows <= 0) group_rows = rows;
  if (param_stride < 0) return fail("mmu_layernorm_fwd_f32: bad param_stride");
  layernorm_fwd32_launch(X, w, b, (bf16*)Y, Y32, mean, rstd, rows, H, eps, group_rows, param_stride,
                         (hipStream_t)stream);
  return check_launch("mmu_layernorm_fwd_f32");
}

int mmu_layernorm_bwd_f32(const void* dY, const float* X, const float* mean, const float* rstd, const float* w,
                          void* dX, void* dXdrop, float drop_p, uint64_t seed, float* part_dw, float* part_db,
                          float* part_dbias, int64_t rows, int64_t H, int64_t rows_per_part, mmu_stream_t stream) {
  if (!dY || !X || !mean || !rstd || !w || !dX) return fail("mmu_layernorm_bwd_f32: null pointer");
  if (rows <= 0 || H <= 0 || H % 256 || H > 1024 || rows_per_part <= 0) return fail("mmu_layernorm_bwd_f32: bad shape");
  if (drop_p < 0.f || drop_p >= 1.f) return fail("mmu_layernorm_bwd_f32: drop_p out of range");
  layernorm_bwd_launch((const bf16*)dY, X, true, mean, rstd, w, (bf16*)dX, (bf16*)dXdrop, nullptr, drop_p, seed,
                       g_seed_off, part_dw, part_db, part_dbias, rows, H, rows_per_part, (hipStream_t)stream);
  return check_launch("mmu_layernorm_bwd_f32");
}

int mmu_layernorm_bwd_res(const void* dY, const void* X, const float* mean, const float* rstd, const float* w,
                          const void* dRes, void* dX, float* part_dw, float* part_db, float* part_dbias, int64_t rows,
                          int64_t H, int64_t rows_per_part, mmu_stream_t stream) {
  if (!dY || !X || !mean || !rstd || !w || !dX || !dRes) return fail("mmu_layernorm_bwd_res: null pointer");
  if (rows <= 0 || H <= 0 || H % 256 || H > 1024 || rows_per_part <= 0) return fail("mmu_layernorm_bwd_res: bad shape");
  layernorm_bwd_launch((const bf16*)dY, X, false, mean, rstd, w, (bf16*)dX, nullptr, (const bf16*)dRes, 0.f, 0,
                       nullptr, part_dw, part_db, part_dbias, rows, H, rows_per_part, (hipStream_t)stream);
  return check_launch("mmu_layernorm_bwd_res");
}

static int seqattn_check(const char* what, int64_t ld_qkv, int64_t S, int64_t N, int64_t heads, int64_t D) {
  if (S <= 0 || N <= 0 || heads <= 0) return fail("%s: bad shape", what);
  if (D != 64 && D != 128 && D != 256) return fail("%s: head_dim %ld not in {64, 128, 256}", what, D);
  if (ld_qkv < 3 * heads * D || ld_qkv % 8) return fail("%s: ld_qkv too small / unaligned", what);
  if (N * heads > 65535) return fail("%s: N*heads > 65535", what);
  return 0;
}

int mmu_seqattn_fwd(const void* QKV, int64_t ld_qkv, void* O, int64_t ld_o, float* LSE2, int64_t S, int64_t N,
                    int64_t heads, int64_t head_dim, mmu_stream_t stream) {
  if (!QKV || !O || !LSE2) return fail("mmu_seqattn_fwd: null pointer");
  if (seqattn_check("mmu_seqattn_fwd", ld_qkv, S, N, heads, head_dim)) return 1;
  if (ld_o < heads * head_dim || ld_o % 4) return fail("mmu_seqattn_fwd: bad ld_o");
  SeqAttnParams p{};
  p.qkv = (const bf16*)QKV; p.ld_qkv = ld_qkv;
  p.out = (bf16*)O; p.ld_out = ld_o;
  p.lse2 = LSE2;
  p.S = (int)S; p.N = (int)N; p.heads = (int)heads; p.D = (int)head_dim; p.E = (int)(heads * head_dim);
  p.scale = 1.0f / sqrtf((float)head_dim);
  seqattn_fwd_launch(p, (hipStream_t)stream);
  return check_launch("mmu_seqattn_fwd");
}

int mmu_seqattn_bwd(const void* QKV, int64_t ld_qkv, const void* O, int64_t ld_o, const void* dO, int64_t ld_do,
                    const float* LSE2, float* delta, void* dQKV, int64_t ld_dqkv, int64_t S, int64_t N, int64_t heads,
                    int64_t head_dim, mmu_stream_t stream) {
  if (!QKV || !O || !dO || !LSE2 || !delta || !dQKV) return fail("mmu_seqattn_bwd: null pointer");
  if (seqattn_check("mmu_seqattn_bwd", ld_qkv, S, N, heads, head_dim)) return 1;
  if (ld_dqkv < 3 * heads * head_dim || ld_dqkv % 4 || ld_o % 4 || ld_do % 8) return fail("mmu_seqattn_bwd: bad ld");
  SeqAttnParams p{};
  p.qkv = (const bf16*)QKV; p.ld_qkv = ld_qkv;
  p.o = (const bf16*)O; p.ld_o = ld_o;
  p.dout = (const bf16*)dO; p.ld_do = ld_do;
  p.out = (bf16*)dQKV; p.ld_out = ld_dqkv;
  p.lse2 = (float*)LSE2; p.delta = delta;
  p.S = (int)S; p.N = (int)N; p.heads = (int)heads; p.D = (int)head_dim; p.E = (int)(heads * head_dim);
  p.scale = 1.0f / sqrtf((float)head_dim);
  seqattn_bwd_launch(p, (hipStream_t)stream);
  return check_launch("mmu_seqattn_bwd");
}


int mmu_embed_fwd(const int64_t* ids, const int64_t* seg, const int64_t* txt_mask, const float* proj, const float* word,
                  const float* pos, const float* type, const float* ln_w, const float* ln_b, float eps, int64_t cls_id,
                  int64_t sep_id, const int64_t* idx, int64_t V, int64_t B, int64_t T, int64_t n_img, int64_t Lout,
                  int64_t H, float drop_txt, float drop_img, uint64_t seed, void* X, float* X32, float* keymask,
                  float* mean, float* rstd, mmu_stream_t stream) {
  if (H != 768) return fail("mmu_embed_fwd: H must be 768");
  if (!word || !pos || !type || !ln_w || !ln_b || !X || !keymask || !proj) return fail("mmu_embed_fwd: null pointer");
  if (T > 0 && (!ids || !seg)) return fail("mmu_embed_fwd: text ids/segments missing");
  if (V <= 0 || B <= 0 || Lout <= 0 || n_img <= 0) return fail("mmu_embed_fwd: bad shape");
  if (!idx && Lout != n_img + 2 + T) return fail("mmu_embed_fwd: identity variant needs Lout == n_img+2+T");
  EmbedParams p{};
  p.ids = ids; p.seg = seg; p.txt_mask = txt_mask; p.idx = idx; p.proj = proj; p.word = word; p.pos = pos;
  p.type = type; p.ln_w = ln_w; p.ln_b = ln_b; p.eps = eps; p.cls_id = cls_id; p.sep_id = sep_id; p.V = V; p.B = B;
  p.T = T; p.n_img = n_img; p.Lout = Lout; p.H = H; p.X = (bf16*)X; p.X32 = X32;
  if (drop_txt < 0.f || drop_txt >= 1.f || drop_img < 0.f || drop_img >= 1.f) return fail("mmu_embed_fwd: bad dropout");
  p.drop_txt = drop_txt; p.drop_img = drop_img; p.seed = seed; p.seed_off = g_seed_off; p.keymask = keymask; p.mean = mean; p.rstd = rstd;
  embed_fwd_launch(p, (hipStream_t)stream);
  return check_launch("mmu_embed_fwd");
}

int64_t mmu_embed_bwd_ws_floats(int64_t B, int64_t T, int64_t n_img) {
  return 4 * embed_bwd_blocks(B, n_img + 2 + T) * 768;
}

int mmu_embed_bwd(const void* dX, const int64_t* ids, const int64_t* seg, const float* proj, const float* word,
                  const float* pos, const float* type, const float* ln_w, const float* mean, const float* rstd,
                  int64_t cls_id, int64_t sep_id, int64_t B, int64_t T, int64_t n_img, int64_t H, float drop_txt,
                  float drop_img, uint64_t seed, float* d_word,
                  float* d_pos, float* d_type, float* d_ln_w, float* d_ln_b, float* d_proj, float* ws,
                  mmu_stream_t stream) {
  if (H != 768) return fail("mmu_embed_bwd: H must be 768");
  if (!dX || !ids || !seg || !proj || !word || !pos || !type || !ln_w || !mean || !rstd || !d_word || !d_pos ||
      !d_type || !d_ln_w || !d_ln_b || !d_proj || !ws)
    return fail("mmu_embed_bwd: null pointer");
  EmbedBwdParams q{};
  q.dX = (const bf16*)dX; q.ids = ids; q.seg = seg; q.proj = proj; q.word = word; q.pos = pos; q.type = type;
  q.ln_w = ln_w; q.mean = mean; q.rstd = rstd; q.cls_id = cls_id; q.sep_id = sep_id; q.B = B; q.T = T;
  q.n_img = n_img; q.H = H; q.drop_txt = drop_txt; q.drop_img = drop_img; q.seed = seed; q.seed_off = g_seed_off; q.d_word = d_word; q.d_pos = d_pos; q.d_type = d_type; q.d_ln_w = d_ln_w;
  q.d_ln_b = d_ln_b; q.d_proj = d_proj; q.ws = ws;
  embed_bwd_launch(q, (hipStream_t)stream);
  return check_launch("mmu_embed_bwd");
}

int mmu_image_normalize(const uint8_t* in, int64_t n, const float* mean, const float* stdv, void* out,
                        int out_dtype, mmu_stream_t stream) {
  if (!in || !out || !mean || !stdv || n < 0) return fail("mmu_image_normalize: bad args");
  if (out_dtype != MMU_BF16 && out_dtype != MMU_F32) return fail("mmu_image_normalize: bad out_dtype");
  for (int c = 0; c < 3; ++c)
    if (!(stdv[c] > 0.f)) return fail("mmu_image_normalize: std must be > 0");
  if (n == 0) return 0;
  image_normalize_launch(in, n, mean, stdv, out, out_dtype == MMU_BF16, (hipStream_t)stream);
  return check_launch("mmu_image_normalize");
}

int mmu_maxpool_fwd(const void* x, int64_t B, int64_t H, int64_t W, int64_t C, void* y, uint8_t* argmax,
                    mmu_stream_t stream) {
  if (!x || !y || !argmax || B <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8 || H > 65536 || W > 65536)
    return fail("mmu_maxpool_fwd: bad args");
  maxpool3s2_fwd_launch((const bf16*)x, B, (int)H, (int)W, (int)C, (int)((H - 1) / 2 + 1), (int)((W - 1) / 2 + 1),
                        (bf16*)y, argmax, (hipStream_t)stream);
  return check_launch("mmu_maxpool_fwd");
}

int mmu_maxpool_bwd(const void* dy, const uint8_t* argmax, int64_t B, int64_t H, int64_t W, int64_t C, void* dx,
                    mmu_stream_t stream) {
  if (!dy || !dx || !argmax || B <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8 || H > 65536 || W > 65536)
    return fail("mmu_maxpool_bwd: bad args");
  maxpool3s2_bwd_launch((const bf16*)dy, argmax, B, (int)H, (int)W, (int)C, (int)((H - 1) / 2 + 1),
                        (int)((W - 1) / 2 + 1), (bf16*)dx, (hipStream_t)stream);
  return check_launch("mmu_maxpool_bwd");
}

int mmu_row_pool_fwd(const void* fmap, int64_t B, int64_t Hh, int64_t Ww, int64_t C, int64_t n, float* out,
                     mmu_stream_t stream) {
  if (!fmap || !out || C % 8 || n <= 0 || n > Hh) return fail("mmu_row_pool_fwd: bad args");
  row_pool_fwd_launch((const bf16*)fmap, B, Hh, Ww, C, n, out, (hipStream_t)stream);
  return check_launch("mmu_row_pool_fwd");
}

int mmu_row_pool_bwd(const float* dout, int64_t B, int64_t Hh, int64_t Ww, int64_t C, int64_t n, void* dfmap,
                     mmu_stream_t stream) {
  if (!dout || !dfmap || C % 8 || n <= 0 || n > Hh) return fail("mmu_row_pool_bwd: bad args");
  row_pool_bwd_launch(dout, B, Hh, Ww, C, n, (bf16*)dfmap, (hipStream_t)stream);
  return check_launch("mmu_row_pool_bwd");
}

// conv geometry shared by the gathered conv products: ksize 3 (pad 1) or 1 (pad 0), stride >= 1
static int conv_geometry(GemmParams& p, int64_t n_img, int64_t H, int64_t W, int64_t C, int64_t ks, int64_t st,
                         int64_t& Mo, const char* who) {
  if (n_img <= 0 || H <= 0 || W <= 0 || C <= 0 || (ks != 1 && ks != 3) || st < 1 || st > 4)
    return fail("%s: bad geometry (n=%ld H=%ld W=%ld C=%ld ksize=%ld stride=%ld)", who, n_img, H, W, C, ks, st);
  const int64_t pad = ks / 2, Ho = (H + 2 * pad - ks) / st + 1, Wo = (W + 2 * pad - ks) / st + 1;
  const int64_t in_bytes = 2 * n_img * H * W * C;
  if (in_bytes >= 0x7FFF0000ll) return fail("%s: input map too large for 32-bit buffer offsets", who);
  p.conv_h = (int)H; p.conv_w = (int)W; p.conv_c = (int)C;
  p.conv_ho = (int)Ho; p.conv_wo = (int)Wo; p.conv_ks = (int)ks; p.conv_s = (int)st; p.conv_pad = (int)pad;
  p.conv_in_bytes = in_bytes;
  Mo = n_img * Ho * Wo;
  return 0;
}

int mmu_conv_wgrad(const void* dY, const void* X, float* dW, int64_t n_img, int64_t H, int64_t W, int64_t Cin,
                   int64_t Cout, int64_t ksize, int64_t stride, int accumulate, float* ws, int64_t ws_floats,
                   mmu_stream_t stream) {
  if (!dY || !X || !dW) return fail("mmu_conv_wgrad: null pointer");
  if (Cin % 256 || Cout % 128 || Cin <= 0 || Cout <= 0)
    return fail("mmu_conv_wgrad: needs Cin %% 256 == 0, Cout %% 128 == 0 (Cin=%ld Cout=%ld)", Cin, Cout);
  GemmParams p{};
  int64_t K;
  if (conv_geometry(p, n_img, H, W, Cin, ksize, stride, K, "mmu_conv_wgrad")) return 1;
  if (K >= (1 << 24) || 2 * (K + 64) * Cout >= (1ll << 31))
    return fail("mmu_conv_wgrad: map too large for 32-bit buffer offsets");
  const int64_t T = ksize * ksize;
  p.A = (const bf16*)dY; p.lda = Cout;  // A = dY^T: M-major [K out pixels][Cout]
  p.B = (const bf16*)X; p.ldb = Cin;    // B gathered: [K out pixels][T Cin]
  p.C = dW; p.ldc = T * Cin;            // dW [Cout][ks][ks][Cin] f32 (channels-last filter)
  p.M = Cout; p.N = T * Cin; p.K = K;
  p.tiles_m = (int)((Cout + 255) / 256);
  p.tiles_n = (int)(T * Cin / 256);
  p.group_m = 1;
  p.kind = MMU_EPI_STORE;
  p.accumulate = accumulate;
  // split-K over the pixels (few output tiles): ~640 blocks, >= 1024 pixels per slice
  const int64_t tiles = (int64_t)p.tiles_m * p.tiles_n;
  int64_t want = (640 + tiles - 1) / tiles;
  // (the 2-tile 1x1 downsample, Cin 256 -> Cout 512: up to 128 slices of >= 256 pixels)
  const bool few = tiles <= 4;
  if (want > K / (few ? 256 : 1024)) want = K / (few ? 256 : 1024);
  if (want > (few ? 128 : 32)) want = few ? 128 : 32;
  if (ws && want > ws_floats / (p.M * p.N)) want = ws_floats / (p.M * p.N);
  p.splitk = 1;
  p.kchunk = K;
  if (ws && want >= 2) {
    int64_t chunk = ((K + want - 1) / want + 63) / 64 * 64;
    p.kchunk = chunk;
    p.splitk = (int)((K + chunk - 1) / chunk);
    p.ws = ws;
  }
  conv3x3_wgrad_launch(p, (hipStream_t)stream);
  return check_launch("mmu_conv_wgrad");
}

int mmu_conv3x3_wgrad(const void* dY, const void* X, float* dW, int64_t n_img, int64_t H, int64_t W, int64_t Cin,
                      int64_t Cout, int accumulate, float* ws, int64_t ws_floats, mmu_stream_t stream) {
  return mmu_conv_wgrad(dY, X, dW, n_img, H, W, Cin, Cout, 3, 1, accumulate, ws, ws_floats, stream);
}

static int stem_params(StemParams& p, int64_t n_img, int64_t H, int64_t W, const char* who) {
  if (n_img <= 0 || H < 1 || W < 1 || n_img * H * W * 3 >= (1ll << 31) || n_img > (1 << 20))
    return fail("%s: bad image batch %ld x %ld x %ld", who, n_img, H, W);
  p.n = (int)n_img; p.H = (int)H; p.W = (int)W;
  stem_fill_geometry(p);
  if ((int64_t)p.n * p.Ho * p.Wo * 64 >= (1ll << 31)) return fail("%s: output too large", who);
  return 0;
}

int mmu_stem_conv_fwd(const void* X, const void* Wk, void* Y, int64_t n_img, int64_t H, int64_t W,
                      mmu_stream_t stream) {
  if (!X || !Wk || !Y) return fail("mmu_stem_conv_fwd: null pointer");
  StemParams p{};
  if (stem_params(p, n_img, H, W, "mmu_stem_conv_fwd")) return 1;
  p.X = (const bf16*)X; p.Wt = (const bf16*)Wk; p.Y = (bf16*)Y;
  stem_fwd_launch(p, (hipStream_t)stream);
  return check_launch("mmu_stem_conv_fwd");
}

int64_t mmu_stem_conv_wgrad_ws_floats(int64_t n_img, int64_t H, int64_t W) {
  StemParams p{};
  if (stem_params(p, n_img, H, W, "mmu_stem_conv_wgrad_ws_floats")) return -1;
  return stem_wgrad_ws_floats(p.n_tiles);
}

int mmu_stem_conv_wgrad(const void* dY, const void* X, float* dW, int64_t n_img, int64_t H, int64_t W,
                        int accumulate, float* ws, int64_t ws_floats, mmu_stream_t stream) {
  if (!dY || !X || !dW || !ws) return fail("mmu_stem_conv_wgrad: null pointer");
  StemParams p{};
  if (stem_params(p, n_img, H, W, "mmu_stem_conv_wgrad")) return 1;
  if (ws_floats < stem_wgrad_ws_floats(p.n_tiles))
    return fail("mmu_stem_conv_wgrad: ws needs %ld floats", stem_wgrad_ws_floats(p.n_tiles));
  p.X = (const bf16*)X; p.dY = (const bf16*)dY;
  stem_wgrad_launch(p, dW, accumulate, ws, (hipStream_t)stream);
  return check_launch("mmu_stem_conv_wgrad");
}

static int conv_implicit(const void* X, const void* Wk, void* Y, int64_t n_img, int64_t H, int64_t W, int64_t C,
                         int64_t N, int64_t ksize, int64_t stride, float* stats, float* ws, int64_t ws_floats,
                         mmu_stream_t stream, const void* bn_x = nullptr, const uint8_t* bn_mask = nullptr,
                         const float* bn_mean = nullptr) {
  if (!X || !Wk || !Y) return fail("mmu_conv_implicit: null pointer");
  if (C % 64 || N % 64 || N <= 0)
    return fail("mmu_conv_implicit: needs C %% 64 == 0, N %% 64 == 0 (C=%ld N=%ld)", C, N);
  GemmParams p{};
  int64_t M;
  if (conv_geometry(p, n_img, H, W, C, ksize, stride, M, "mmu_conv_implicit")) return 1;
  const int64_t T = ksize * ksize;
  if (M < 256 || 2 * (M + 256) * N >= (1ll << 31) || 2 * (N + 256) * T * C >= (1ll << 31))
    return fail("mmu_conv_implicit: map size out of range");
  // 256x256 tiles (LDS-DMA gather) for N >= 256 with N % 128 == 0; 128x128 register-staged
  // tiles for the narrow convs (N = 64 / 128 / ...)
  const bool small = N < 256 || N % 128;
  const int tm_ = small ? 128 : 256, tn_ = small ? 128 : 256;
  p.A = (const bf16*)X; p.lda = C;       // A gathered: [M out pixels][T C]
  p.B = (const bf16*)Wk; p.ldb = T * C;  // B K-major [N][T C]
  p.C = Y; p.ldc = N;                    // Y [M pixels][N] bf16
  p.M = M; p.N = N; p.K = T * C;
  p.tiles_m = (int)((M + tm_ - 1) / tm_);
  p.tiles_n = (int)((N + tn_ - 1) / tn_);
  p.group_m = 1;
  p.kind = !stats ? MMU_EPI_STORE : bn_x ? MMU_EPI_STORE_BNB : MMU_EPI_STORE_STATS;
  p.colsum = stats;
  p.bn_x = (const bf16*)bn_x; p.bn_mask = bn_mask; p.bn_mean = bn_mean;
  p.splitk = 1;
  p.kchunk = p.K;
  // split K (taps x channels) when the map has fewer tiles than half the CUs: ~512 blocks, >= 4
  // 64-deep steps per slice, slabs bounded by the workspace
  const int64_t tiles = (int64_t)p.tiles_m * p.tiles_n;
  if (ws && tiles < 128) {
    int64_t want = (512 + tiles - 1) / tiles;
    if (want > p.K / 256) want = p.K / 256;
    if (want > ws_floats / (M * N)) want = ws_floats / (M * N);
    if (want >= 2) {
      const int64_t chunk = ((p.K + want - 1) / want + 63) / 64 * 64;
      p.kchunk = chunk;
      p.splitk = (int)((p.K + chunk - 1) / chunk);
      p.ws = ws;
    }
  }
  conv3x3_implicit_launch(p, small, (hipStream_t)stream);
  return check_launch("mmu_conv_implicit");
}

int mmu_conv_implicit(const void* X, const void* Wk, void* Y, int64_t n_img, int64_t H, int64_t W, int64_t C,
                      int64_t N, int64_t ksize, int64_t stride, float* ws, int64_t ws_floats, mmu_stream_t stream) {
  return conv_implicit(X, Wk, Y, n_img, H, W, C, N, ksize, stride, nullptr, ws, ws_floats, stream);
}

int mmu_conv_implicit_stats(const void* X, const void* Wk, void* Y, int64_t n_img, int64_t H, int64_t W, int64_t C,
                            int64_t N, int64_t ksize, int64_t stride, float* stats, float* ws, int64_t ws_floats,
                            mmu_stream_t stream) {
  if (!stats) return fail("mmu_conv_implicit_stats: null stats table");
  return conv_implicit(X, Wk, Y, n_img, H, W, C, N, ksize, stride, stats, ws, ws_floats, stream);
}

int mmu_conv3x3_implicit(const void* X, const void* Wk, void* Y, int64_t n_img, int64_t H, int64_t W, int64_t C,
                         int64_t N, float* ws, int64_t ws_floats, mmu_stream_t stream) {
  return conv_implicit(X, Wk, Y, n_img, H, W, C, N, 3, 1, nullptr, ws, ws_floats, stream);
}

int mmu_conv3x3_implicit_bnb(const void* X, const void* Wk, void* Y, int64_t n_img, int64_t H, int64_t W, int64_t C,
                             int64_t N, const void* bn_x, const uint8_t* bn_mask, const float* bn_mean,
                             float* stats, float* ws, int64_t ws_floats, mmu_stream_t stream) {
  if (!stats || !bn_x || !bn_mean) return fail("mmu_conv3x3_implicit_bnb: null table / bn_x / bn_mean");
  return conv_implicit(X, Wk, Y, n_img, H, W, C, N, 3, 1, stats, ws, ws_floats, stream, bn_x, bn_mask, bn_mean);
}

int64_t mmu_batchnorm_ws_bytes(int64_t C) { return batchnorm_ws_bytes(C); }

static int bn_common(int64_t rows, int64_t C, void* ws, int64_t ws_bytes, const char* who) {
  if (rows <= 0 || C <= 0 || C % 8 || C > 2048) return fail("%s: C=%ld must be a multiple of 8, <= 2048", who, C);
  if (!ws || ws_bytes < batchnorm_ws_bytes(C) || ((uintptr_t)ws & 15))
    return fail("%s: ws must be >= mmu_batchnorm_ws_bytes(C) bytes, 16-B aligned", who);
  return 0;
}

// the residual stream's residue (y_res / skip_res): the block output (skip + ReLU, the skip's
// residue read) or the downsample's BatchNorm (no skip, no ReLU)
static int bn_res_check(const void* skip, int relu, const void* relu_mask, const void* skip_res, const void* y_res,
                        const char* who) {
  if (skip_res && !y_res) return fail("%s: skip_res needs y_res", who);
  if (!y_res) return 0;
  if (skip && (!relu || !skip_res)) return fail("%s: y_res with a skip needs relu and skip_res", who);
  if (!skip && (relu || relu_mask)) return fail("%s: y_res without a skip takes no relu", who);
  return 0;
}

int mmu_batchnorm_fwd(const void* X, const void* skip, void* Y, int64_t rows, int64_t C, const float* weight,
                      const float* bias, float* running_mean, float* running_var, int64_t* num_batches_tracked,
                      int training, float momentum, float eps, int relu, float* save_mean, float* save_invstd,
                      void* relu_mask, const void* skip_res, void* y_res, void* ws, int64_t ws_bytes,
                      mmu_stream_t stream) {
  if (!X || !Y) return fail("mmu_batchnorm_fwd: null pointer");
  if (relu_mask && !relu) return fail("mmu_batchnorm_fwd: relu_mask needs relu");
  if (bn_res_check(skip, relu, relu_mask, skip_res, y_res, "mmu_batchnorm_fwd")) return 1;
  if (bn_common(rows, C, ws, ws_bytes, "mmu_batchnorm_fwd")) return 1;
  if ((running_mean == nullptr) != (running_var == nullptr))
    return fail("mmu_batchnorm_fwd: running_mean / running_var must both be given or NULL");
  if ((save_mean == nullptr) != (save_invstd == nullptr))
    return fail("mmu_batchnorm_fwd: save_mean / save_invstd must both be given or NULL");
  if (training && rows < 2) return fail("mmu_batchnorm_fwd: training needs more than 1 value per channel");
  if (!training && !running_mean) return fail("mmu_batchnorm_fwd: eval needs running statistics");
  if (training && momentum < 0.f && !num_batches_tracked)
    return fail("mmu_batchnorm_fwd: momentum < 0 (cumulative average) needs num_batches_tracked");
  BnFwdParams q{};
  q.X = (const bf16*)X; q.skip = (const bf16*)skip; q.Y = (bf16*)Y; q.rows = rows; q.C = (int)C;
  q.w = weight; q.b = bias; q.rmean = running_mean; q.rvar = running_var; q.nbt = num_batches_tracked;
  q.training = training; q.relu = relu; q.momentum = momentum; q.eps = eps;
  q.smean = save_mean; q.sinvstd = save_invstd; q.ws = ws; q.mask = (uint8_t*)relu_mask;
  q.skip_res = (const int8_t*)skip_res; q.y_res = (int8_t*)y_res;
  batchnorm_fwd_launch(q, (hipStream_t)stream);
  return check_launch("mmu_batchnorm_fwd");
}

int mmu_batchnorm_bwd(const void* dY, const void* Y, const void* relu_mask, const void* X, int64_t rows, int64_t C,
                      const float* weight, const float* save_mean, const float* save_invstd, int relu, void* dX,
                      void* dSkip, float* dweight, float* dbias, void* ws, int64_t ws_bytes, mmu_stream_t stream) {
  if (!dY || !X || !dX || !save_mean || !save_invstd) return fail("mmu_batchnorm_bwd: null pointer");
  if (relu && !Y && !relu_mask) return fail("mmu_batchnorm_bwd: relu needs the forward output Y or its relu_mask");
  if (bn_common(rows, C, ws, ws_bytes, "mmu_batchnorm_bwd")) return 1;
  BnBwdParams q{};
  q.dY = (const bf16*)dY; q.Y = (const bf16*)Y; q.X = (const bf16*)X; q.rows = rows; q.C = (int)C; q.w = weight;
  q.smean = save_mean; q.sinvstd = save_invstd; q.relu = relu; q.dX = (bf16*)dX; q.dS = (bf16*)dSkip;
  q.dw = dweight; q.db = dbias; q.ws = ws; q.mask = (const uint8_t*)relu_mask;
  batchnorm_bwd_launch(q, (hipStream_t)stream);
  return check_launch("mmu_batchnorm_bwd");
}

int mmu_batchnorm_bwd_parts(const void* dY, const void* Y, const void* relu_mask, const void* X, int64_t rows,
                            int64_t C, const float* parts, int64_t nparts, const float* weight,
                            const float* save_mean, const float* save_invstd, int relu, void* dX, void* dSkip,
                            float* dweight, float* dbias, void* ws, int64_t ws_bytes, mmu_stream_t stream) {
  if (!dY || !X || !dX || !save_mean || !save_invstd || !parts || nparts <= 0)
    return fail("mmu_batchnorm_bwd_parts: null pointer / no partials");
  if (relu && !Y && !relu_mask) return fail("mmu_batchnorm_bwd_parts: relu needs the forward output Y or its relu_mask");
  if (bn_common(rows, C, ws, ws_bytes, "mmu_batchnorm_bwd_parts")) return 1;
  BnBwdParams q{};
  q.dY = (const bf16*)dY; q.Y = (const bf16*)Y; q.X = (const bf16*)X; q.rows = rows; q.C = (int)C; q.w = weight;
  q.smean = save_mean; q.sinvstd = save_invstd; q.relu = relu; q.dX = (bf16*)dX; q.dS = (bf16*)dSkip;
  q.dw = dweight; q.db = dbias; q.ws = ws; q.mask = (const uint8_t*)relu_mask;
  q.parts = parts; q.nparts = nparts;
  batchnorm_bwd_launch(q, (hipStream_t)stream);
  return check_launch("mmu_batchnorm_bwd_parts");
}

int mmu_batchnorm_stats(const void* X, int64_t rows, int64_t C, double* sums, void* ws, int64_t ws_bytes,
                        mmu_stream_t stream) {
  if (!X || !sums) return fail("mmu_batchnorm_stats: null pointer");
  if (bn_common(rows, C, ws, ws_bytes, "mmu_batchnorm_stats")) return 1;
  BnFwdParams q{};
  q.X = (const bf16*)X; q.rows = rows; q.C = (int)C; q.training = 1; q.ws = ws; q.lsum = sums;
  batchnorm_fwd_launch(q, (hipStream_t)stream);
  return check_launch("mmu_batchnorm_stats");
}

int mmu_batchnorm_fwd_sums(const void* X, const void* skip, void* Y, int64_t rows, int64_t C, const double* sums,
                           const float* weight, const float* bias, float* running_mean, float* running_var,
                           int64_t* num_batches_tracked, float momentum, float eps, int relu, float* save_mean,
                           float* save_invstd, void* relu_mask, const void* skip_res, void* y_res, void* ws,
                           int64_t ws_bytes, mmu_stream_t stream) {
  if (!X || !Y || !sums) return fail("mmu_batchnorm_fwd_sums: null pointer");
  if (relu_mask && !relu) return fail("mmu_batchnorm_fwd_sums: relu_mask needs relu");
  if (bn_res_check(skip, relu, relu_mask, skip_res, y_res, "mmu_batchnorm_fwd_sums")) return 1;
  if (bn_common(rows, C, ws, ws_bytes, "mmu_batchnorm_fwd_sums")) return 1;
  if ((running_mean == nullptr) != (running_var == nullptr))
    return fail("mmu_batchnorm_fwd_sums: running_mean / running_var must both be given or NULL");
  if ((save_mean == nullptr) != (save_invstd == nullptr))
    return fail("mmu_batchnorm_fwd_sums: save_mean / save_invstd must both be given or NULL");
  if (momentum < 0.f && !num_batches_tracked)
    return fail("mmu_batchnorm_fwd_sums: momentum < 0 (cumulative average) needs num_batches_tracked");
  BnFwdParams q{};
  q.X = (const bf16*)X; q.skip = (const bf16*)skip; q.Y = (bf16*)Y; q.rows = rows; q.C = (int)C;
  q.w = weight; q.b = bias; q.rmean = running_mean; q.rvar = running_var; q.nbt = num_batches_tracked;
  q.training = 1; q.relu = relu; q.momentum = momentum; q.eps = eps;
  q.smean = save_mean; q.sinvstd = save_invstd; q.ws = ws; q.mask = (uint8_t*)relu_mask; q.gsum = sums;
  q.skip_res = (const int8_t*)skip_res; q.y_res = (int8_t*)y_res;
  batchnorm_fwd_launch(q, (hipStream_t)stream);
  return check_launch("mmu_batchnorm_fwd_sums");
}

int mmu_batchnorm_fwd_parts(const void* X, const void* skip, void* Y, int64_t rows, int64_t C, const float* parts,
                            int64_t nparts, const float* weight, const float* bias, float* running_mean,
                            float* running_var, int64_t* num_batches_tracked, float momentum, float eps, int relu,
                            float* save_mean, float* save_invstd, void* relu_mask, const void* skip_res, void* y_res,
                            void* ws, int64_t ws_bytes, mmu_stream_t stream) {
  if (!X || !Y || !parts || nparts <= 0) return fail("mmu_batchnorm_fwd_parts: null pointer / no partials");
  if (relu_mask && !relu) return fail("mmu_batchnorm_fwd_parts: relu_mask needs relu");
  if (bn_res_check(skip, relu, relu_mask, skip_res, y_res, "mmu_batchnorm_fwd_parts")) return 1;
  if (bn_common(rows, C, ws, ws_bytes, "mmu_batchnorm_fwd_parts")) return 1;
  if ((running_mean == nullptr) != (running_var == nullptr))
    return fail("mmu_batchnorm_fwd_parts: running_mean / running_var must both be given or NULL");
  if ((save_mean == nullptr) != (save_invstd == nullptr))
    return fail("mmu_batchnorm_fwd_parts: save_mean / save_invstd must both be given or NULL");
  if (rows < 2) return fail("mmu_batchnorm_fwd_parts: training needs more than 1 value per channel");
  if (momentum < 0.f && !num_batches_tracked)
    return fail("mmu_batchnorm_fwd_parts: momentum < 0 (cumulative average) needs num_batches_tracked");
  BnFwdParams q{};
  q.X = (const bf16*)X; q.skip = (const bf16*)skip; q.Y = (bf16*)Y; q.rows = rows; q.C = (int)C;
  q.w = weight; q.b = bias; q.rmean = running_mean; q.rvar = running_var; q.nbt = num_batches_tracked;
  q.training = 1; q.relu = relu; q.momentum = momentum; q.eps = eps;
  q.smean = save_mean; q.sinvstd = save_invstd; q.ws = ws; q.mask = (uint8_t*)relu_mask;
  q.skip_res = (const int8_t*)skip_res; q.y_res = (int8_t*)y_res;
  q.parts = parts; q.nparts = nparts;
  batchnorm_fwd_launch(q, (hipStream_t)stream);
  return check_launch("mmu_batchnorm_fwd_parts");
}

int mmu_batchnorm_bwd_reduce(const void* dY, const void* Y, const void* relu_mask, const void* X, int64_t rows,
                             int64_t C, const float* save_mean, const float* save_invstd, int relu, double* sums,
                             float* dweight, float* dbias, void* ws, int64_t ws_bytes, mmu_stream_t stream) {
  if (!dY || !X || !sums || !save_mean || !save_invstd) return fail("mmu_batchnorm_bwd_reduce: null pointer");
  if (relu && !Y && !relu_mask) return fail("mmu_batchnorm_bwd_reduce: relu needs the forward output Y or its relu_mask");
  if (bn_common(rows, C, ws, ws_bytes, "mmu_batchnorm_bwd_reduce")) return 1;
  BnBwdParams q{};
  q.dY = (const bf16*)dY; q.Y = (const bf16*)Y; q.X = (const bf16*)X; q.rows = rows; q.C = (int)C;
  q.smean = save_mean; q.sinvstd = save_invstd; q.relu = relu; q.dw = dweight; q.db = dbias; q.ws = ws;
  q.mask = (const uint8_t*)relu_mask; q.lsum = sums;
  batchnorm_bwd_launch(q, (hipStream_t)stream);
  return check_launch("mmu_batchnorm_bwd_reduce");
}

int mmu_batchnorm_bwd_sums(const void* dY, const void* Y, const void* relu_mask, const void* X, int64_t rows,
                           int64_t C, const double* sums, const float* weight, const float* save_mean,
                           const float* save_invstd, int relu, void* dX, void* dSkip, void* ws, int64_t ws_bytes,
                           mmu_stream_t stream) {
  if (!dY || !X || !dX || !sums || !save_mean || !save_invstd) return fail("mmu_batchnorm_bwd_sums: null pointer");
  if (relu && !Y && !relu_mask) return fail("mmu_batchnorm_bwd_sums: relu needs the forward output Y or its relu_mask");
  if (bn_common(rows, C, ws, ws_bytes, "mmu_batchnorm_bwd_sums")) return 1;
  BnBwdParams q{};
  q.dY = (const bf16*)dY; q.Y = (const bf16*)Y; q.X = (const bf16*)X; q.rows = rows; q.C = (int)C; q.w = weight;
  q.smean = save_mean; q.sinvstd = save_invstd; q.relu = relu; q.dX = (bf16*)dX; q.dS = (bf16*)dSkip; q.ws = ws;
  q.mask = (const uint8_t*)relu_mask; q.gsum = sums;
  batchnorm_bwd_launch(q, (hipStream_t)stream);
  return check_launch("mmu_batchnorm_bwd_sums");
}

int mmu_bertadam_step(float* params, const float* grads, float* m, float* v, void* bf16_copy, const int64_t* table,
                      int32_t* steps, int64_t n_tensors, int64_t n_chunks, float lr_decay, float lr_nodecay, float wd,
                      float warmup, float t_total, float b1, float b2, float eps, float max_grad_norm,
                      float grad_scale, float* ws, int64_t ws_floats, mmu_stream_t stream) {
  if (!params || !grads || !m || !v || !table || !steps || !ws) return fail("mmu_bertadam_step: null pointer");
  if (n_tensors <= 0 || n_chunks <= 0) return fail("mmu_bertadam_step: empty table");
  if (ws_floats < n_chunks + 2 * n_tensors) return fail("mmu_bertadam_step: workspace too small");
  if (!(grad_scale > 0.f)) return fail("mmu_bertadam_step: grad_scale must be > 0");
  AdamParams p{};
  p.params = params; p.grads = grads; p.m = m; p.v = v; p.bf16_copy = (bf16*)bf16_copy; p.table = table;
  p.steps = steps; p.n_tensors = n_tensors; p.total = n_chunks; p.lr_decay = lr_decay; p.lr_nodecay = lr_nodecay;
  p.wd = wd; p.warmup = warmup; p.t_total = t_total; p.b1 = b1; p.b2 = b2; p.eps = eps;
  p.max_grad_norm = max_grad_norm; p.grad_scale = grad_scale; p.ws = ws; p.ws_floats = ws_floats;
  const char* e = nullptr;
  if (bertadam_launch(p, (hipStream_t)stream, &e)) return fail("mmu_bertadam_step: %s", e ? e : "failed");
  return check_launch("mmu_bertadam_step");
}

int mmu_uncertainty(const float* logits, const int64_t* y, int64_t S, int64_t R, int64_t C, float* p_bar, float* nll,
                    float* conf, float* correct, mmu_stream_t stream) {
  if (!logits || !y || !p_bar || !nll || !conf || !correct) return fail("mmu_uncertainty: null pointer");
  if (S <= 0 || R <= 0 || C <= 0 || C > 1024) return fail("mmu_uncertainty: bad shape (C <= 1024)");
  uncertainty_launch(logits, y, S, R, C, p_bar, nll, conf, correct, (hipStream_t)stream);
  return check_launch("mmu_uncertainty");
}

int mmu_ece_bins(const float* conf, const float* correct, int64_t S, int64_t n_bins, float* out, mmu_stream_t stream) {
  if (!conf || !correct || !out || S <= 0 || n_bins <= 0) return fail("mmu_ece_bins: bad args");
  ece_bins_launch(conf, correct, S, n_bins, out, (hipStream_t)stream);
  return check_launch("mmu_ece_bins");
}

}  // extern "C"
