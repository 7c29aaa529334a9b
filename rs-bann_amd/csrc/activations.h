// activations.h — h(x) and dh/dx of activation_functions.rs:22-45.
#pragma once
#include <hip/hip_runtime.h>

__device__ __forceinline__ float act_h(float x, int act) {
  switch (act) {
    case 0:  // Tanh
      return tanhf(x);
    case 1:  // ReLU: x * (x > 0)
      return x > 0.f ? x : 0.f;
    case 2:  // LeakyReLU: x * (x > 0) + 0.01 x * afsign(x)   (afsign = 1 for x < 0)
      return x > 0.f ? x : 0.01f * x;
    case 3:  // SiLU: x * sigmoid(x)
      return x / (1.f + __expf(-x));
    default:  // Identity
      return x;
  }
}

// derivative given the pre-activation x and the activation hx = h(x)
__device__ __forceinline__ float act_dh(float x, float hx, int act) {
  switch (act) {
    case 0:  // 1 - tanh(x)^2
      return 1.f - hx * hx;
    case 1:  // (x > 0)
      return x > 0.f ? 1.f : 0.f;
    case 2:  // (x > 0) + 0.01 * afsign(x): 1 / 0.01 / 0 at x == 0
      return x > 0.f ? 1.f : (x < 0.f ? 0.01f : 0.f);
    case 3: {  // f + sigmoid(x) (1 - f)
      const float s = 1.f / (1.f + __expf(-x));
      return hx + s * (1.f - hx);
    }
    default:
      return 1.f;
  }
}

// tanh with ~2 ulp error and no library call: odd minimax polynomial for
// |x| < 0.625 (f32-evaluated max rel. error 1.4e-7), 1 - 2/(e^{2|x|}+1) above
// (no cancellation there: the result is >= 0.55).
__device__ __forceinline__ float fast_tanh(float x) {
  const float ax = fabsf(x);
  const float x2 = x * x;
  float p = -0.0056647793389856815f;
  p = fmaf(p, x2, 0.020595693960785866f);
  p = fmaf(p, x2, -0.05372268706560135f);
  p = fmaf(p, x2, 0.13331151008605957f);
  p = fmaf(p, x2, -0.3333326280117035f);
  p = fmaf(p, x2, 1.0f);
  const float small = x * p;
  const float e = __expf(2.f * fminf(ax, 20.f));
  const float big = copysignf(1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f), x);  // v_rcp_f32 (1 ulp)
  return ax < 0.625f ? small : big;  // branch-free select
}

// tanh in five instructions: 1 - 2 / (2^(2x log2 e) + 1) with v_exp_f32 and
// v_rcp_f32 (1 ulp each); absolute error <= ~2.4e-7 everywhere, saturates to
// +-1 for large |x| (exp -> inf or 0).  The relative error grows only where
// |tanh x| is tiny, which the norm-relative parity of every gradient tensor
// absorbs (tests/test_gpu_parity.py).
__device__ __forceinline__ float tanh5(float x) {
  const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);  // 2 log2(e)
  return fmaf(-2.f, __builtin_amdgcn_rcpf(e + 1.f), 1.f);
}

// tanh and its derivative without cancellation: with r = 1 / (e^{2|x|} + 1) <= 1/2,
// tanh x = sign(x) (1 - 2 r) and 1 - tanh^2 x = 4 r (1 - r), where 1 - r >= 1/2:
// accurate relative to the derivative itself where tanh saturates (1 - h^2 from the
// rounded h loses it there: |h| = 1 - 1e-3 leaves ~3e-5 relative error)
__device__ __forceinline__ float tanh_r(float x, float& r) {
  const float e = __builtin_amdgcn_exp2f(fabsf(x) * 2.8853900817779268f);  // 2 log2(e); inf -> r = 0
  r = __builtin_amdgcn_rcpf(e + 1.f);
  return copysignf(fmaf(-2.f, r, 1.f), x);
}
__device__ __forceinline__ float dtanh_r(float r) { return (4.f * r) * (1.f - r); }

// compile-time activation (fused kernel): h and dh/dx without branches on the code
template <int ACT>
__device__ __forceinline__ float act_h_t(float x) {
  if constexpr (ACT == 0) return tanh5(x);
  else if constexpr (ACT == 1) return x > 0.f ? x : 0.f;
  else if constexpr (ACT == 2) return x > 0.f ? x : 0.01f * x;
  else if constexpr (ACT == 3) return x * __builtin_amdgcn_rcpf(1.f + __expf(-x));
  else return x;
}
template <int ACT>
__device__ __forceinline__ float act_dh_t(float x, float hx) {
  if constexpr (ACT == 0) return 1.f - hx * hx;
  else if constexpr (ACT == 1) return x > 0.f ? 1.f : 0.f;
  else if constexpr (ACT == 2) return x > 0.f ? 1.f : (x < 0.f ? 0.01f : 0.f);
  else if constexpr (ACT == 3) {
    const float s = __builtin_amdgcn_rcpf(1.f + __expf(-x));
    return hx + s * (1.f - hx);
  } else return 1.f;
}
