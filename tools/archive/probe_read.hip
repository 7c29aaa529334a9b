// Read-bandwidth probe: how fast can one MI355X stream a C3-sized (6.4 GB)
// buffer?  Plain global_load_dwordx4 grid-stride reads (the achievable ceiling
// for the fused gradient kernel's genotype stream) and LDS-DMA 1 KiB pieces
// (the fx kernel's load path).  Profiling tool only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) k_read(const v4u* __restrict__ p, size_t n16, unsigned* out) {
  unsigned s = 0;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x, st = (size_t)gridDim.x * 256;
#pragma unroll 4
  for (; i < n16; i += st) {
    const v4u v = __builtin_nontemporal_load(p + i);
    s ^= v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  if (s == 0x12345678u) out[0] = s;
}

// contiguous per-block ranges of `per` bytes, 4 KiB per iteration per block
__global__ void __launch_bounds__(256) k_read_blocked(const v4u* __restrict__ p, size_t per16, size_t n16, unsigned* out) {
  unsigned s = 0;
  const size_t b0 = (size_t)blockIdx.x * per16;
  for (size_t i = b0 + threadIdx.x; i < b0 + per16 && i < n16; i += 256) {
    const v4u v = p[i];
    s ^= v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  if (s == 0x12345678u) out[0] = s;
}


// LDS-DMA streaming shaped like k_fused_grad_fx's stream: each wave owns tiles
// tt = wave0, wave0 + NWT, ... of 8 KiB (8 x 1 KiB glds16 pieces), two LDS slots
// (one tile ahead), an optional one-dword-per-line L2 prefetch PF tiles ahead.
__device__ __forceinline__ void glds16p(const void* gsrc, const void* lds_dst) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)lds_dst);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m0), "v"(gsrc) : "memory", "m0");
}
template <int PF>
__global__ void __launch_bounds__(256, 2) k_dma(const char* __restrict__ base, int tiles_per_wg, unsigned* out) {
  __shared__ __attribute__((aligned(16))) char s_x[4][2][8192];
  __shared__ char pad[12000];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const char* src = base + (size_t)blockIdx.x * tiles_per_wg * 8192 + lane * 16;
  const char* pfs = base + (size_t)blockIdx.x * tiles_per_wg * 8192 + lane * 128;
  uint32_t pfd = 0, s = 0;
  int sl = 0;
  for (int c = 0; c < 8; ++c) glds16p(src + (size_t)wave * 8192 + c * 1024, &s_x[wave][0][c * 1024]);
  for (int tt = wave; tt < tiles_per_wg; tt += 4, sl ^= 1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s ^= *(volatile uint32_t*)&s_x[wave][sl][lane * 4];
    if (tt + 4 < tiles_per_wg)
      for (int c = 0; c < 8; ++c) glds16p(src + (size_t)(tt + 4) * 8192 + c * 1024, &s_x[wave][sl ^ 1][c * 1024]);
    if (PF && tt + 4 * PF < tiles_per_wg)
      asm volatile("global_load_dword %0, %1, off" : "+v"(pfd) : "v"(pfs + (size_t)(tt + 4 * PF) * 8192) : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if ((s ^ pfd) == 0x12345678u) out[0] = s + pad[threadIdx.x];
}
template <int PF>
void run_dma(const char* p, size_t bytes, unsigned* o, int tiles_per_wg) {
  const int grid = (int)(bytes / 8192 / tiles_per_wg);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e9;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(a);
    hipLaunchKernelGGL(k_dma<PF>, dim3(grid), dim3(256), 0, 0, p, tiles_per_wg, o);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  printf("lds-dma PF=%d tiles/wg=%d grid=%d: %.3f ms  %.0f GB/s\n", PF, tiles_per_wg, grid, best,
         (double)grid * tiles_per_wg * 8192 / best / 1e6);
}

int main(int argc, char** argv) {
  const size_t bytes = argc > 1 ? strtoull(argv[1], 0, 10) : 6400000000ull;
  v4u* p;
  unsigned* o;
  hipMalloc(&p, bytes);
  hipMalloc(&o, 4);
  hipMemset(p, 1, bytes);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const size_t n16 = bytes / 16;
  for (int grid : {1024, 2048, 4096, 8192}) {
    float best = 1e9;
    for (int r = 0; r < 5; ++r) {
      hipEventRecord(a);
      hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, p, n16, o);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    printf("grid-stride grid=%d: %.3f ms  %.0f GB/s\n", grid, best, bytes / best / 1e6);
  }
  for (size_t per : {24576ull * 4, 98304ull * 4, 786432ull}) {
    const size_t per16 = per / 16;
    const size_t grid = (n16 + per16 - 1) / per16;
    float best = 1e9;
    for (int r = 0; r < 5; ++r) {
      hipEventRecord(a);
      hipLaunchKernelGGL(k_read_blocked, dim3((unsigned)grid), dim3(256), 0, 0, p, per16, n16, o);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    printf("blocked %zu B per block (%zu blocks): %.3f ms  %.0f GB/s\n", per, grid, best, bytes / best / 1e6);
  }
  for (int t : {96, 384, 782, 1536}) run_dma<0>((const char*)p, bytes, o, t);
  return 0;
}
