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
