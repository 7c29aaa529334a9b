// kernels_feed.hip — forward_feed with every layer kept (branch_sampler.rs:743-782):
// the pre-activations Z_l and activations A_l = h(Z_l) of one branch, for
// Net::activations (net.rs:509-518) and the reports built on it.  Not on the
// HMC path (the fused kernels never materialise hidden layers): one launch per
// layer, plain f32 FMAs, layer 0 reading the branch's 2-bit tile image.
//
// Layouts (ArrayFire column-major, as forward_feed's arrays): Z_l, A_l are
// [w_l][n] (element (i, k) at k n + i).
#include "activations.h"
#include "bann_internal.h"

#define FEED_KB 8    // output columns per thread (one decoded genotype feeds 8 FMAs)
#define FEED_T 256   // threads per workgroup: 4 waves = 4 tiles of 64 individuals

// genotype of individual i at marker row j of a branch's tile image: tile
// i >> 6, chunk j >> 6, row r = j & 63 in window w = r >> 4 at position
// P = ((r & 15) + 8 (w & 1)) & 15, the 8-byte halves swapped for P >= 8
// (k_pack_tiles, kernels_data.hip); byte (i & 63) >> 2 holds individuals 4q..4q+3
__device__ __forceinline__ int tile_genotype(const uint8_t* __restrict__ img, int64_t tile_stride, int64_t i,
                                             int j) {
  const int c = j >> 6, r = j & 63, w = r >> 4;
  const int P = ((r & 15) + 8 * (w & 1)) & 15;
  const int ii = (int)(i & 63), q = ii >> 2;
  const int64_t at = (i >> 6) * tile_stride + 1024 * c + (16 * w + P) * 16 + (P >= 8 ? (q ^ 8) : q);
  return (img[at] >> (2 * (ii & 3))) & 3;
}

// Z0 = X W0 + b0 with X = (g - mu) / sigma (bed.rs:325-355; sigma = 0 markers contribute 0)
__global__ void __launch_bounds__(FEED_T) k_feed0(DevState st, int b, float* __restrict__ pre,
                                                  float* __restrict__ act) {
  const BranchDev bd = st.br[b];
  const int64_t n = st.n;
  const int64_t i = (int64_t)blockIdx.x * FEED_T + threadIdx.x;
  const int k0 = blockIdx.y * FEED_KB, m = bd.m, w0 = bd.widths[0];
  if (i >= n) return;
  const float* W = st.theta + bd.p_off + bd.woff[0];
  const float* mu = st.mu + bd.mk_off;
  const float* sg = st.sigma + bd.mk_off;
  const uint8_t* img = st.xu2 + bd.x_off;
  const int64_t tstride = 1024 * (int64_t)bd.nchunks;
  float acc[FEED_KB];
#pragma unroll
  for (int kk = 0; kk < FEED_KB; ++kk) acc[kk] = 0.f;
  for (int j = 0; j < m; ++j) {
    const float s = sg[j];
    const float x = s > 0.f ? ((float)tile_genotype(img, tstride, i, j) - mu[j]) / s : 0.f;
#pragma unroll
    for (int kk = 0; kk < FEED_KB; ++kk)
      if (k0 + kk < w0) acc[kk] = fmaf(x, W[(int64_t)(k0 + kk) * m + j], acc[kk]);
  }
  const float* bias = st.theta + bd.p_off + bd.boff[0];
#pragma unroll
  for (int kk = 0; kk < FEED_KB; ++kk) {
    const int k = k0 + kk;
    if (k >= w0) break;
    const float z = acc[kk] + bias[k];
    if (pre) pre[(int64_t)k * n + i] = z;
    act[(int64_t)k * n + i] = act_h(z, bd.act);
  }
}

// layer l >= 1: Z_l = A_{l-1} W_l + b_l, A_l = h(Z_l); the output layer
// (l = L-1) has no bias and no activation (output_neuron_activation, 775-782)
__global__ void __launch_bounds__(FEED_T) k_feed(DevState st, int b, int l, const float* __restrict__ in,
                                                 float* __restrict__ pre, float* __restrict__ act) {
  const BranchDev bd = st.br[b];
  const int64_t n = st.n;
  const int64_t i = (int64_t)blockIdx.x * FEED_T + threadIdx.x;
  const int k0 = blockIdx.y * FEED_KB, wi = bd.win[l], wo = bd.widths[l];
  if (i >= n) return;
  const float* W = st.theta + bd.p_off + bd.woff[l];
  float acc[FEED_KB];
#pragma unroll
  for (int kk = 0; kk < FEED_KB; ++kk) acc[kk] = 0.f;
  for (int j = 0; j < wi; ++j) {
    const float x = in[(int64_t)j * n + i];
#pragma unroll
    for (int kk = 0; kk < FEED_KB; ++kk)
      if (k0 + kk < wo) acc[kk] = fmaf(x, W[(int64_t)(k0 + kk) * wi + j], acc[kk]);
  }
  const bool out_layer = l == bd.L - 1;
#pragma unroll
  for (int kk = 0; kk < FEED_KB; ++kk) {
    const int k = k0 + kk;
    if (k >= wo) break;
    if (out_layer) {
      act[(int64_t)k * n + i] = acc[kk];
    } else {
      const float z = acc[kk] + st.theta[bd.p_off + bd.boff[l] + k];
      if (pre) pre[(int64_t)k * n + i] = z;
      act[(int64_t)k * n + i] = act_h(z, bd.act);
    }
  }
}

// pre: [sum_{l < L-1} w_l][n] (may be null), act: [sum_l w_l][n], layer after layer
void launch_forward_feed(const DevState& st, int b, const BranchDev& bd, float* pre, float* act, hipStream_t s) {
  const int64_t n = st.n;
  const unsigned gx = (unsigned)((n + FEED_T - 1) / FEED_T);
  int64_t ao = 0, po = 0;
  for (int l = 0; l < bd.L; ++l) {
    const int wo = bd.widths[l];
    const dim3 grid(gx, (unsigned)((wo + FEED_KB - 1) / FEED_KB));
    float* p = (pre && l < bd.L - 1) ? pre + po : nullptr;
    if (l == 0)
      hipLaunchKernelGGL(k_feed0, grid, dim3(FEED_T), 0, s, st, b, p, act);
    else
      hipLaunchKernelGGL(k_feed, grid, dim3(FEED_T), 0, s, st, b, l, act + ao - (int64_t)bd.win[l] * n, p, act + ao);
    ao += (int64_t)wo * n;
    if (l < bd.L - 1) po += (int64_t)wo * n;
  }
}
