// Streaming-read ceiling probe (tools only, not part of the product).
//
// How fast can one MI355X read a C3-sized genotype image (782 000 tiles x 8 KiB)
// with (a) plain per-lane 16-byte vector loads and (b) the fx kernels' access
// pattern: LDS-DMA of 1 KiB pieces, one 8 KiB tile per wave, NW waves per
// workgroup, tiles two ahead in a double-buffered LDS slot, optional dependent
// VALU work per tile standing in for the forward/backward.  The gap between (a),
// (b) and the kernels' own launch times says how much of the fx gradient launch is
// stream shape rather than compute.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/_stream_probe tools/stream_probe.hip
//   tools/_stream_probe [tiles=782000] [reps=10]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

typedef unsigned v4u __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) k_vload(const v4u* __restrict__ p, int64_t n16, unsigned* out) {
  v4u acc = {0u, 0u, 0u, 0u};
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const v4u a = __builtin_nontemporal_load(p + i), b = __builtin_nontemporal_load(p + i + stride);
    const v4u c = __builtin_nontemporal_load(p + i + 2 * stride), d = __builtin_nontemporal_load(p + i + 3 * stride);
    acc ^= a ^ b ^ c ^ d;
  }
  for (; i < n16; i += stride) acc ^= __builtin_nontemporal_load(p + i);
  const unsigned r = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (r == 0x9e3779b9u) out[0] = r;  // keeps the loads alive
}

__device__ __forceinline__ uint32_t lds_off(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void glds16(const void* gsrc, const void* lds_dst) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(lds_off(lds_dst));
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt" ::"s"(m0), "v"(gsrc) : "memory", "m0");
}
template <int K>
__device__ __forceinline__ void vmw() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K) : "memory");
}

// NW waves per workgroup; workgroup w owns tiles [w * tpw, (w + 1) * tpw) (wave v takes
// every NW-th); a tile is 8 pieces of 1 KiB; tiles two ahead (slot sl ^ 1 in flight)
template <int NW>
__global__ void __launch_bounds__(64 * NW) k_dma(const char* __restrict__ x, int64_t ntiles, int64_t tpw, int work,
                                                 unsigned* out) {
  __shared__ __attribute__((aligned(16))) char s_x[NW][2][8192];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int64_t tb = (int64_t)blockIdx.x * tpw, te = tb + tpw < ntiles ? tb + tpw : ntiles;
  const char* src = x + lane * 16;
  unsigned acc = lane;
  float f = (float)lane;
  int64_t tt = tb + wave;
  int sl = 0;
  if (tt < te) {
    for (int c = 0; c < 8; ++c) glds16(src + tt * 8192 + c * 1024, &s_x[wave][0][c * 1024]);
    if (tt + NW < te)
      for (int c = 0; c < 8; ++c) glds16(src + (tt + NW) * 8192 + c * 1024, &s_x[wave][1][c * 1024]);
  }
  for (; tt < te; tt += NW, sl ^= 1) {
    if (tt + NW < te) vmw<8>(); else vmw<0>();
    acc ^= *reinterpret_cast<const unsigned*>(&s_x[wave][sl][lane * 4]);
    for (int i = 0; i < work; ++i) f = fmaf(f, 1.0001f, 0.5f);  // dependent VALU standing in for compute
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (tt + 2 * NW < te)
      for (int c = 0; c < 8; ++c) glds16(src + (tt + 2 * NW) * 8192 + c * 1024, &s_x[wave][sl][c * 1024]);
  }
  if (acc == 0x9e3779b9u || f == 1.2345f) out[0] = acc;
}

int main(int argc, char** argv) {
  const int64_t ntiles = argc > 1 ? atoll(argv[1]) : 782000;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const int64_t bytes = ntiles * 8192;
  char* x;
  unsigned* out;
  CK(hipMalloc(&x, bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(x, 0x5a, bytes));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch) {
    for (int r = 0; r < 2; ++r) launch();
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-40s %8.4f ms  %7.1f GB/s\n", name, ms, bytes / (ms * 1e6));
    fflush(stdout);
  };
  printf("image %.3f GB, %d CUs\n", bytes / 1e9, cus);
  for (int gm : {4, 8, 16}) {
    char nm[64];
    snprintf(nm, sizeof nm, "vload 256 thr, %d WG/CU", gm);
    timeit(nm, [&] { k_vload<<<cus * gm, 256>>>((const v4u*)x, bytes / 16, out); });
  }
  for (int work : {0, 200, 400}) {
    for (int wpc : {2, 4}) {  // workgroups per CU (LDS: 64 KiB per 4-wave workgroup)
      const int64_t nwg = (int64_t)cus * wpc;
      const int64_t tpw = (ntiles + nwg - 1) / nwg;
      char nm[64];
      snprintf(nm, sizeof nm, "dma 4 waves, %d WG/CU, work %d", wpc, work);
      timeit(nm, [&] { k_dma<4><<<nwg, 256>>>(x, ntiles, tpw, work, out); });
    }
    {  // the fx grid shape: 1000 workgroups of 782 tiles
      const int64_t tpw = 782, nwg = (ntiles + tpw - 1) / tpw;
      char nm[64];
      snprintf(nm, sizeof nm, "dma 4 waves, %lld WG x 782, work %d", (long long)nwg, work);
      timeit(nm, [&] { k_dma<4><<<nwg, 256>>>(x, ntiles, tpw, work, out); });
    }
  }
  CK(hipDeviceSynchronize());
  return 0;
}
