// kernel_util.h — device helpers shared by the fused gradient kernels:
// wave reductions, LDS-DMA / LDS-store inline asm, the transposing LDS read,
// f32 exponent tricks and the signed-digit split used by the i8 MFMA paths.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bann_internal.h"

typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));

// LDS image of one branch's head parameters, padded to 4x4 (zeros outside the
// real widths, so padded units stay exactly 0 and contribute nothing).
struct HeadLds {
  float W[BANN_MAXL][4][4];  // W_l[j][k], l >= 1
  float bias[BANN_MAXL][4];  // b_l (l >= 1), c0 for l = 0
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

#define LDS_BARRIER()                                      \
  do {                                                     \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     \
    __builtin_amdgcn_s_barrier();                          \
    asm volatile("" ::: "memory");                         \
  } while (0)

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// LDS stores issued through inline asm: hipcc's wait-count pass does not see
// them, so it does not drain in-flight LDS-DMA (vmcnt(0)) in front of every
// store as it does for a ds_write it cannot disambiguate from the DMA target.
// Their completion is ordered by the explicit lgkmcnt(0) of LDS_BARRIER.
__device__ __forceinline__ uint32_t lds_off(const void* p) { return (uint32_t)(uintptr_t)p; }
// LDS-DMA through inline asm as well: the wave's own counted "s_waitcnt vmcnt"
// (explicit, below) is then the only wait on it.  M0 = wave-uniform LDS base;
// the data lands at M0 + 16 * lane (4 * lane for the dword form).
__device__ __forceinline__ void glds16(const void* gsrc, const void* lds_dst) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(lds_off(lds_dst));
#ifndef BANN_GLDS_NT
#define BANN_GLDS_NT 1  // the genotype / target streams are read once per launch: non-temporal (-2 % fx, A/B)
#endif
#if BANN_GLDS_NT
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt" ::"s"(m0), "v"(gsrc) : "memory", "m0");
#else
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m0), "v"(gsrc) : "memory", "m0");
#endif
}
// the same with a wave-uniform 64-bit base in SGPRs and a per-lane 32-bit byte offset (the
// global_load "saddr" form: one address VGPR, no 64-bit address arithmetic per piece)
__device__ __forceinline__ void glds16_s(const void* sbase, uint32_t voff, const void* lds_dst) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(lds_off(lds_dst));
#if BANN_GLDS_NT
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt" ::"s"(m0), "v"(voff), "s"(sbase)
               : "memory", "m0");
#else
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(m0), "v"(voff), "s"(sbase)
               : "memory", "m0");
#endif
}
__device__ __forceinline__ void glds4(const void* gsrc, const void* lds_dst) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(lds_off(lds_dst));
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dword %1, off" ::"s"(m0), "v"(gsrc) : "memory", "m0");
}
__device__ __forceinline__ void lds_st_f32(float* p, float v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(lds_off(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_st_v4f(v4f* p, v4f v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(lds_off(p)), "v"(v) : "memory");
}

__device__ __forceinline__ uint32_t fbits(float x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ float fpow2(uint32_t biased_exp) { return __builtin_bit_cast(float, biased_exp << 23); }

typedef unsigned short v2u16 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t max_u16x2(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(v2u16, a), __builtin_bit_cast(v2u16, b)));
}
// wave-wide max of two packed u16 lanes (DPP row reductions, result uniform)
__device__ __forceinline__ uint32_t wave_max_u16x2(uint32_t v) {
  v = max_u16x2(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false));   // quad [1,0,3,2]
  v = max_u16x2(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false));   // quad [2,3,0,1]
  v = max_u16x2(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xF, 0xF, false));  // row_half_mirror
  v = max_u16x2(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xF, 0xF, false));  // row_mirror
  v = max_u16x2(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x142, 0xA, 0xF, false));  // row_bcast15
  v = max_u16x2(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x143, 0xC, 0xF, false));  // row_bcast31
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

typedef int v2i __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) v2i lds_v2i;
__device__ __forceinline__ v4i lds_tr8_pair(const char* p0, const char* p1) {
  const v2i a = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(p0));
  const v2i b = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(p1));
  return v4i{a.x, a.y, b.x, b.y};
}

// four signed 7-bit digits of v (|v| < 64), most significant first, packed LE
__device__ __forceinline__ uint32_t digits4(float v) {
  uint32_t w = 0;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const float r = __builtin_rintf(v);
    w |= ((uint32_t)(int)r & 0xFFu) << (8 * d);
    v = (v - r) * 128.f;
  }
  return w;
}
