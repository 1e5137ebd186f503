// Microbenchmark: how fast can one CU move operand tiles from L2 / HBM into LDS?
//   mode 0: buffer_load ... lds (LDS-DMA, what mmu_gemm's main loop uses)
//   mode 1: global_load_dwordx4 into VGPRs + ds_write_b128
//   mode 2: half of each 64 KiB stage by each path
// 512 threads (8 waves, like the 256x256 GEMM tile), 2 x 64 KiB LDS stages, one block per CU,
// each iteration fills one 64 KiB stage then waits + barriers (the GEMM's per-K-step pattern).
//   hipcc --offload-arch=gfx950 -O3 tools/lds_bw.hip -o tools/lds_bw && tools/lds_bw
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define LDSP(T) __attribute__((address_space(3))) T

static __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, int bytes) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, bytes, 0x00020000);
}

// mode 3: LDS-DMA with one stage in flight ahead (issue stage it+1, then wait for stage it
// with a counted vmcnt(8)): does overlap raise the rate (latency-bound) or not (bandwidth)?
__global__ __launch_bounds__(512) void bw_ahead_kernel(const char* src, int src_bytes, int iters, uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) char lds[2][65536];
  const int t = threadIdx.x, w = t >> 6, l = t & 63;
  const __amdgpu_buffer_rsrc_t r = rsrc(src, src_bytes);
  const int nst = src_bytes / 65536;
  uint32_t acc = 0;
  auto issue = [&](int it) {
    char* st = lds[it & 1];
    const uint32_t base = (uint32_t)(((blockIdx.x * 7 + it) % nst) * 65536);
#pragma unroll
    for (int i = 0; i < 8; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDSP(void)*)(st + (w * 8 + i) * 1024), 16,
                                               base + (w * 8 + i) * 1024 + l * 16, 0, 0, 0);
  };
  issue(0);
  for (int it = 0; it < iters; ++it) {
    __syncthreads();  // everyone is done reading the stage issue(it + 1) overwrites
    if (it + 1 < iters) {
      issue(it + 1);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    acc += *(const uint32_t*)(lds[it & 1] + ((t * 131) & 65535 & ~3));
  }
  if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

template <int MODE>
__global__ __launch_bounds__(512) void bw_kernel(const char* src, int src_bytes, int iters, uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) char lds[2][65536];
  const int t = threadIdx.x, w = t >> 6, l = t & 63;
  const __amdgpu_buffer_rsrc_t r = rsrc(src, src_bytes);
  const int nst = src_bytes / 65536;
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) {
    char* st = lds[it & 1];
    const uint32_t base = (uint32_t)(((blockIdx.x * 7 + it) % nst) * 65536);
    uint4 v[8];
    if (MODE != 0) {
#pragma unroll
      for (int i = (MODE == 2 ? 4 : 0); i < 8; ++i)
        v[i] = *(const uint4*)(src + base + (w * 8 + i) * 1024 + l * 16);
    }
    if (MODE != 1) {
#pragma unroll
      for (int i = 0; i < (MODE == 2 ? 4 : 8); ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDSP(void)*)(st + (w * 8 + i) * 1024), 16,
                                                 base + (w * 8 + i) * 1024 + l * 16, 0, 0, 0);
    }
    if (MODE != 0) {
#pragma unroll
      for (int i = (MODE == 2 ? 4 : 0); i < 8; ++i) *(uint4*)(st + (w * 8 + i) * 1024 + l * 16) = v[i];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    acc += *(const uint32_t*)(st + ((t * 131) & 65535 & ~3));
  }
  if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

// mode "gemm": the operand stream of one mmu_gemm big-tile launch without the MFMAs -- per
// K-step each block DMAs its A tile (256 rows x 64 k) and B tile (256 cols x 64 k), both
// K-major, 2-stage ring, tiles in mmu_gemm's grouped + XCD-remapped order.
static __device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  int q = nwg >> 3, r = nwg & 7, xcd = orig & 7, idx = orig >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}
__global__ __launch_bounds__(512) void gemm_stream_kernel(const char* A, const char* B, int M, int N, int K,
                                                          int group_m, int lda, uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) char lds[2][65536];
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  const int tiles_m = (M + 255) / 256, tiles_n = N / 256;
  const int pid = xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = group_m * tiles_n, g = pid / per_group, first = g * group_m;
  const int gm = tiles_m - first < group_m ? tiles_m - first : group_m;
  const int rr = pid - g * per_group, tm = first + rr % gm, tn = rr / gm;
  const __amdgpu_buffer_rsrc_t ra = rsrc(A + (int64_t)tm * 256 * lda * 2, (M - tm * 256 < 256 ? M - tm * 256 : 256) * lda * 2);
  const __amdgpu_buffer_rsrc_t rb = rsrc(B + (int64_t)tn * 256 * K * 2, 256 * K * 2);
  const int nk = K / 64;
  auto issue = [&](int ks) {
    char* st = lds[ks & 1];
    // 256 rows x 128 B per operand: 8 lanes per row, 64 rows per wave-instruction, 4 each
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 64 * i + 8 * w + (l >> 3), c = l & 7;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (LDSP(void)*)(st + (64 * i + 8 * w) * 128), 16,
                                               (uint32_t)((row * lda + 64 * ks + 8 * c) * 2), 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (LDSP(void)*)(st + 32768 + (64 * i + 8 * w) * 128), 16,
                                               (uint32_t)((row * K + 64 * ks + 8 * c) * 2), 0, 0, 0);
    }
  };
  uint32_t acc = 0;
  issue(0);
  for (int ks = 0; ks < nk; ++ks) {
    __syncthreads();
    if (ks + 1 < nk) {
      issue(ks + 1);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    acc += *(const uint32_t*)(lds[ks & 1] + ((t * 131) & 65535 & ~3));
  }
  if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

// the same stream with BK = 32 (32 KiB stages) and a NS-deep ring: NS - 1 stages in flight
template <int NS>
__global__ __launch_bounds__(512) void gemm_stream_ring_kernel(const char* A, const char* B, int M, int N, int K,
                                                               int group_m, int lda, uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) char lds[NS][32768];
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  const int tiles_m = (M + 255) / 256, tiles_n = N / 256;
  const int pid = xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = group_m * tiles_n, g = pid / per_group, first = g * group_m;
  const int gm = tiles_m - first < group_m ? tiles_m - first : group_m;
  const int rr = pid - g * per_group, tm = first + rr % gm, tn = rr / gm;
  const __amdgpu_buffer_rsrc_t ra = rsrc(A + (int64_t)tm * 256 * lda * 2, (M - tm * 256 < 256 ? M - tm * 256 : 256) * lda * 2);
  const __amdgpu_buffer_rsrc_t rb = rsrc(B + (int64_t)tn * 256 * K * 2, 256 * K * 2);
  const int nk = K / 32;
  auto issue = [&](int ks) {
    char* st = lds[ks % NS];
    // 256 rows x 64 B per operand: 4 lanes per row, 128 rows per wave-instruction, 2 each
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = 128 * i + 16 * w + (l >> 2), c = l & 3;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (LDSP(void)*)(st + (128 * i + 16 * w) * 64), 16,
                                               (uint32_t)((row * lda + 32 * ks + 8 * c) * 2), 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (LDSP(void)*)(st + 16384 + (128 * i + 16 * w) * 64), 16,
                                               (uint32_t)((row * K + 32 * ks + 8 * c) * 2), 0, 0, 0);
    }
  };
  uint32_t acc = 0;
  for (int j = 0; j < NS - 1 && j < nk; ++j) issue(j);
  for (int ks = 0; ks < nk; ++ks) {
    __syncthreads();
    if (ks + NS - 1 < nk) {
      issue(ks + NS - 1);
      if (NS == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      if (NS == 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      if (NS == 4) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    acc += *(const uint32_t*)(lds[ks % NS] + ((t * 131) & 32767 & ~3));
  }
  if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

template <int NS>
static void gemm_stream_ring(int cus, const char* A, const char* B, int M, int N, int K, int group_m, uint32_t* sink,
                             hipEvent_t e0, hipEvent_t e1) {
  const int tiles = ((M + 255) / 256) * (N / 256);
  hipLaunchKernelGGL(gemm_stream_ring_kernel<NS>, dim3(tiles), dim3(512), 0, 0, A, B, M, N, K, group_m, K, sink);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  hipLaunchKernelGGL(gemm_stream_ring_kernel<NS>, dim3(tiles), dim3(512), 0, 0, A, B, M, N, K, group_m, K, sink);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double ksteps = (double)tiles * (K / 64) / cus;
  printf("gemm stream BK 32 ring %d M %6d N %5d K %5d group %d: %7.1f us, %6.0f cycles per 64-deep K per CU\n", NS, M,
         N, K, group_m, ms * 1e3, ms * 1e-3 * 2.4e9 / ksteps);
  fflush(stdout);
}

static void gemm_stream(int cus, const char* A, const char* B, int M, int N, int K, int group_m, int lda,
                        uint32_t* sink, hipEvent_t e0, hipEvent_t e1) {
  const int tiles = ((M + 255) / 256) * (N / 256);
  hipLaunchKernelGGL(gemm_stream_kernel, dim3(tiles), dim3(512), 0, 0, A, B, M, N, K, group_m, lda, sink);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  hipLaunchKernelGGL(gemm_stream_kernel, dim3(tiles), dim3(512), 0, 0, A, B, M, N, K, group_m, lda, sink);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double ksteps = (double)tiles * (K / 64) / cus;  // K-steps per CU (one block per CU at a time)
  printf("gemm stream M %6d N %5d K %5d lda %5d group %d: %7.1f us, %6.0f cycles per K-step per CU at 2.4 GHz "
         "(MFMA-bound K-step: 2048)\n", M, N, K, lda, group_m, ms * 1e3, ms * 1e-3 * 2.4e9 / ksteps);
  fflush(stdout);
}

int main() {
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int sizes[3] = {1 << 20, 32 << 20, 1 << 30};
  char* src;
  uint32_t* sink;
  hipMalloc(&src, sizes[2]);
  hipMemset(src, 1, sizes[2]);
  hipMalloc(&sink, 1 << 20);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 2000;
  for (int s = 0; s < 1; ++s) {
    for (int mode = 0; mode < 4; ++mode) {
      auto launch = [&]() {
        if (mode == 0) hipLaunchKernelGGL(bw_kernel<0>, dim3(cus), dim3(512), 0, 0, src, sizes[s], iters, sink);
        if (mode == 1) hipLaunchKernelGGL(bw_kernel<1>, dim3(cus), dim3(512), 0, 0, src, sizes[s], iters, sink);
        if (mode == 2) hipLaunchKernelGGL(bw_kernel<2>, dim3(cus), dim3(512), 0, 0, src, sizes[s], iters, sink);
        if (mode == 3) hipLaunchKernelGGL(bw_ahead_kernel, dim3(cus), dim3(512), 0, 0, src, sizes[s], iters, sink);
      };
      launch();
      hipDeviceSynchronize();
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      const double bytes = (double)cus * iters * 65536.0;
      const double per_cu_clk = bytes / (ms * 1e-3) / cus / 2.4e9;
      printf("src %5d MiB  mode %d (%s): %8.1f GB/s chip, %5.1f B/clk/CU at 2.4 GHz, %6.0f cycles per 64 KiB stage\n",
             sizes[s] >> 20, mode, mode == 0 ? "LDS-DMA     " : mode == 1 ? "VGPR + ds_wr" : mode == 2 ? "half / half " : "DMA 1 ahead ",
             bytes / (ms * 1e-3) / 1e9, per_cu_clk, 65536.0 / per_cu_clk);
      fflush(stdout);
    }
  }
  // the BERT FFN1 (N = 3072, K = 768) and FFN2 (N = 768, K = 3072) operand streams at B = 256
  char *A, *B;
  hipMalloc(&A, (size_t)131328 * 3200 * 2);
  hipMalloc(&B, (size_t)3072 * 3072 * 2);
  hipMemset(A, 1, (size_t)131328 * 3200 * 2);
  hipMemset(B, 1, (size_t)3072 * 3072 * 2);
  gemm_stream(cus, A, B, 131328, 3072, 768, 8, 768, sink, e0, e1);
  gemm_stream_ring<2>(cus, A, B, 131328, 3072, 768, 8, sink, e0, e1);
  gemm_stream_ring<3>(cus, A, B, 131328, 3072, 768, 8, sink, e0, e1);
  gemm_stream_ring<4>(cus, A, B, 131328, 3072, 768, 8, sink, e0, e1);
  gemm_stream(cus, A, B, 131328, 768, 3072, 1, 3072, sink, e0, e1);
  gemm_stream_ring<2>(cus, A, B, 131328, 768, 3072, 1, sink, e0, e1);
  gemm_stream_ring<3>(cus, A, B, 131328, 768, 3072, 1, sink, e0, e1);
  gemm_stream_ring<4>(cus, A, B, 131328, 768, 3072, 1, sink, e0, e1);
  hipFree(A);
  hipFree(B);
  hipFree(src);
  hipFree(sink);
  return 0;
}
