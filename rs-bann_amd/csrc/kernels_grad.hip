// kernels_grad.hip — generic (any widths / depth / marker count) log-density
// gradient of the branch network: BranchSampler::backpropagate
// (branch_sampler.rs:813-875) with forward_feed (743-782) in the reference op
// order, f32 standardized inputs, double accumulation.  Reads the same 2-bit
// tile image ("u2t", kernels_fx.hip) as the fused kernels.
#include "activations.h"
#include <stdlib.h>

#include <type_traits>

#include "bann_internal.h"
#include "kernel_util.h"


// Ablation switches for profiling builds only (make ABLATE=n): 1 = skip the head,
// 2 = skip the VALU backward, 4 = skip the MFMA forward.  0 in every shipped build.
#ifndef BANN_ABLATE
#define BANN_ABLATE 0
#endif

// ===========================================================================
// generic path
// ===========================================================================
// standardized genotype of individual `row`, marker j from the u2t tile image
// (kernels_fx.hip header): tile row >> 6, marker row in window j >> 4 at position
// ((j & 15) + 8 (w & 1)) & 15 with the 8-byte halves swapped at positions >= 8.
__device__ __forceinline__ float x_std_at(const uint8_t* xb, int nchunks, int64_t row, int j, float mu, float sig) {
  const int64_t tile = row >> 6;
  const int r = (int)(row & 63), Q = r >> 2, p = r & 3;
  const int w = j >> 4, P = ((j & 15) + 8 * (w & 1)) & 15;
  const uint8_t byte = xb[tile * (int64_t)nchunks * 1024 + (16 * w + P) * 16 + (Q ^ (P & 8))];
  const float g = (float)((byte >> (2 * p)) & 3);
  // bed.rs:353: (raw - means) / stds ; zero-variance markers contribute 0 (documented deviation)
  return sig > 0.f ? (g - mu) / sig : 0.f;
}

__global__ void k_generic_fwd0(DevState st, const int32_t* __restrict__ blist) {
  const int b = blist[blockIdx.y];
  const BranchDev bd = st.br[b];
  const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t npad = (int64_t)st.nfrag * 16;
  if (row >= npad) return;
  const uint8_t* xb = st.xu2 + bd.x_off;
  const float* W0 = st.theta + bd.p_off + bd.woff[0];
  const float* b0 = st.theta + bd.p_off + bd.boff[0];
  const float* mu = st.mu + bd.mk_off;
  const float* sg = st.sigma + bd.mk_off;
  const int w0 = bd.widths[0], m = bd.m;
  float* z = st.scr + bd.scr_off + bd.scr_z[0] + row * w0;
  for (int k = 0; k < w0; ++k) {
    double acc = 0.0;
    for (int j = 0; j < m; ++j) acc += (double)x_std_at(xb, bd.nchunks, row, j, mu[j], sg[j]) * (double)W0[k * m + j];
    z[k] = (float)acc + b0[k];  // mid_layer_pre_activation: matmul + tile(bias)
  }
}

__global__ void k_generic_head(DevState st, const int32_t* __restrict__ blist) {
  const int b = blist[blockIdx.y];
  const BranchDev bd = st.br[b];
  const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t npad = (int64_t)st.nfrag * 16;
  if (row >= npad) return;
  const int L = bd.L, act = bd.act;
  const float* th = st.theta + bd.p_off;
  float* S = st.scr + bd.scr_off;
  // forward: activations of layer 0, then hidden/summary layers (branch_sampler.rs:743-758)
  {
    const int w = bd.widths[0];
    float* z = S + bd.scr_z[0] + row * w;
    float* a = S + bd.scr_a[0] + row * w;
    for (int k = 0; k < w; ++k) a[k] = act_h(z[k], act);
  }
  for (int l = 1; l < L - 1; ++l) {
    const int wi = bd.win[l], wo = bd.widths[l];
    const float* ap = S + bd.scr_a[l - 1] + row * wi;
    float* z = S + bd.scr_z[l] + row * wo;
    float* a = S + bd.scr_a[l] + row * wo;
    const float* W = th + bd.woff[l];
    const float* bb = th + bd.boff[l];
    for (int k = 0; k < wo; ++k) {
      double acc = 0.0;
      for (int j = 0; j < wi; ++j) acc += (double)ap[j] * (double)W[k * wi + j];
      z[k] = (float)acc + bb[k];
      a[k] = act_h(z[k], act);
    }
  }
  // output neuron (775-782, no bias) and error (821)
  const int wl = bd.win[L - 1];
  const float* aS = S + bd.scr_a[L - 2] + row * wl;
  const float* Wo = th + bd.woff[L - 1];
  double acc = 0.0;
  for (int j = 0; j < wl; ++j) acc += (double)aS[j] * (double)Wo[j];
  const float out = (float)acc;
  const bool valid = row < st.n;
  const float e = valid ? out - st.y[bd.y_off + row] : 0.f;
  if (valid) st.pred[bd.y_off + row] = out;
  S[bd.scr_d[L - 1] + row] = e;
  // backward deltas (844-866): delta_l = dhdx(z_l) * (delta_{l+1} W_{l+1}^T)
  for (int l = L - 2; l >= 0; --l) {
    const int w = bd.widths[l], wn = bd.widths[l + 1];
    const float* z = S + bd.scr_z[l] + row * w;
    const float* a = S + bd.scr_a[l] + row * w;
    const float* dn = S + bd.scr_d[l + 1] + row * wn;
    const float* Wn = th + bd.woff[l + 1];  // (w x wn), element (k, kk) at kk * w + k
    float* d = S + bd.scr_d[l] + row * w;
    for (int k = 0; k < w; ++k) {
      double err = 0.0;
      for (int kk = 0; kk < wn; ++kk) err += (double)dn[kk] * (double)Wn[kk * w + k];
      d[k] = act_dh(z[k], a[k], act) * (float)err;
    }
  }
}

__global__ void k_generic_reduce(DevState st, const int32_t* __restrict__ blist) {
  const int b = blist[blockIdx.y];
  const BranchDev bd = st.br[b];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > bd.P) return;
  const float* S = st.scr + bd.scr_off;
  const int64_t n = st.n;
  const int L = bd.L;
  double acc = 0.0;
  if (i == bd.P) {  // rss (823-828)
    const float* e = S + bd.scr_d[L - 1];
    for (int64_t r = 0; r < n; ++r) acc += (double)e[r] * (double)e[r];
    st.rss_part[(int64_t)b * st.max_splits] = acc;
    return;
  }
  // locate parameter i
  int l = 0;
  bool is_bias = false;
  for (int q = 0; q < L; ++q)
    if (i >= bd.woff[q] && i < bd.woff[q] + bd.win[q] * bd.widths[q]) l = q;
  if (i >= bd.boff[0]) {
    is_bias = true;
    for (int q = 0; q < L - 1; ++q)
      if (i >= bd.boff[q] && i < bd.boff[q] + bd.widths[q]) l = q;
  }
  if (is_bias) {  // db_l = sum_rows delta_l
    const int w = bd.widths[l], k = i - bd.boff[l];
    const float* d = S + bd.scr_d[l];
    for (int64_t r = 0; r < n; ++r) acc += (double)d[r * w + k];
  } else {
    const int wi = bd.win[l], wo = bd.widths[l];
    const int loc = i - bd.woff[l];
    const int k = loc / wi, j = loc - k * wi;
    const float* d = S + bd.scr_d[l];
    if (l == 0) {  // dW0 = X^T delta0 (863-866)
      const uint8_t* xb = st.xu2 + bd.x_off;
      const float mu = st.mu[bd.mk_off + j], sg = st.sigma[bd.mk_off + j];
      for (int64_t r = 0; r < n; ++r)
        acc += (double)x_std_at(xb, bd.nchunks, r, j, mu, sg) * (double)d[r * wo + k];
    } else {  // dW_l = A_{l-1}^T delta_l (830-835, 849-852)
      const float* a = S + bd.scr_a[l - 1];
      for (int64_t r = 0; r < n; ++r) acc += (double)a[r * wi + j] * (double)d[r * wo + k];
    }
  }
  st.part[bd.part_off + i] = (float)acc;
}

void launch_generic_grad(const DevState& st, const int32_t* branches, int32_t nb, int32_t max_m, int32_t max_p,
                         hipStream_t s) {
  (void)max_m;
  if (nb <= 0) return;
  const int64_t npad = (int64_t)st.nfrag * 16;
  dim3 g1((unsigned)((npad + 255) / 256), (unsigned)nb);
  hipLaunchKernelGGL(k_generic_fwd0, g1, dim3(256), 0, s, st, branches);
  hipLaunchKernelGGL(k_generic_head, g1, dim3(256), 0, s, st, branches);
  dim3 g2((unsigned)((max_p + 1 + 255) / 256), (unsigned)nb);
  hipLaunchKernelGGL(k_generic_reduce, g2, dim3(256), 0, s, st, branches);
}

