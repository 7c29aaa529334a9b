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
                                             int j, bool f3m1) {
  const int c = j >> 6, r = j & 63, w = r >> 4;
  const int P = ((r & 15) + 8 * (w & 1)) & 15;
  const int ii = (int)(i & 63), q = ii >> 2;
  const int64_t at = (i >> 6) * tile_stride + 1024 * c + (16 * w + P) * 16 + (P >= 8 ? (q ^ 8) : q);
  const int v = (img[at] >> (2 * (ii & 3))) & 3;
  return (f3m1 && (ii & 3) == 3) ? ((v + 1) & 3) : v;  // field 3 stored as code - 1 (tile_f3m1)
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
  const bool f3m1 = tile_f3m1(bd.fused);
  float acc[FEED_KB];
#pragma unroll
  for (int kk = 0; kk < FEED_KB; ++kk) acc[kk] = 0.f;
  for (int j = 0; j < m; ++j) {
    const float s = sg[j];
    const float x = s > 0.f ? ((float)tile_genotype(img, tstride, i, j, f3m1) - mu[j]) / s : 0.f;
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

// ---- effect_sizes (branch_sampler.rs:784-811) --------------------------------
// The backward chain of forward_feed's layers seeded with the branch OUTPUT
// times W_out^T (792-797) -- not with the error -- and with no absolute value
// (the doc comment's "absolute values" is not what the code computes):
//   err_S = out W_out^T,  err_{l} = (h'(Z_l) * err_{l+1}) W_l^T  (l = L-2 .. 0)
// so err_0 is n x m: out_i d out_i / d x_ij per individual i and marker j.  Layouts as
// forward_feed: [w][n] (ArrayFire column-major n x w).

// err[k][i] = out[i] W_out[k] (a single product: exact, as matmul of n x 1 by 1 x S)
__global__ void __launch_bounds__(FEED_T) k_effect_seed(DevState st, int b, const float* __restrict__ out,
                                                        float* __restrict__ err) {
  const BranchDev bd = st.br[b];
  const int64_t n = st.n;
  const int64_t i = (int64_t)blockIdx.x * FEED_T + threadIdx.x;
  if (i >= n) return;
  const float* wo = st.theta + bd.p_off + bd.woff[bd.L - 1];
  const float o = out[i];
  for (int k = 0; k < bd.win[bd.L - 1]; ++k) err[(int64_t)k * n + i] = o * wo[k];
}

// err_out[j][i] = sum_k h'(Z_l[k][i]) err_in[k][i] W_l(j, k), k ascending
// (801-807: delta = dhdx(pre_l) * error; error = delta W_l^T)
__global__ void __launch_bounds__(FEED_T) k_effect_back(DevState st, int b, int l, const float* __restrict__ pre,
                                                        const float* __restrict__ act, const float* __restrict__ ein,
                                                        float* __restrict__ eout) {
  const BranchDev bd = st.br[b];
  const int64_t n = st.n;
  const int64_t i = (int64_t)blockIdx.x * FEED_T + threadIdx.x;
  const int j0 = blockIdx.y * FEED_KB, wi = bd.win[l], wo = bd.widths[l];
  if (i >= n) return;
  const float* W = st.theta + bd.p_off + bd.woff[l];
  float acc[FEED_KB];
#pragma unroll
  for (int jj = 0; jj < FEED_KB; ++jj) acc[jj] = 0.f;
  for (int k = 0; k < wo; ++k) {
    const int64_t at = (int64_t)k * n + i;
    const float d = act_dh(pre[at], act[at], bd.act) * ein[at];
#pragma unroll
    for (int jj = 0; jj < FEED_KB; ++jj)
      if (j0 + jj < wi) acc[jj] = fmaf(d, W[(int64_t)k * wi + j0 + jj], acc[jj]);
  }
#pragma unroll
  for (int jj = 0; jj < FEED_KB; ++jj)
    if (j0 + jj < wi) eout[(int64_t)(j0 + jj) * n + i] = acc[jj];
}

// population form (net.rs:529-543: sum over individuals / n): column j of err_0
// summed over i is sum_k W0(j, k) s_k with s_k = sum_i delta_0[k][i], so the
// n x m matrix is never formed.  s_k: one workgroup per column, f64, fixed order.
__global__ void __launch_bounds__(FEED_T) k_effect_colsum(DevState st, int b, const float* __restrict__ pre,
                                                          const float* __restrict__ act,
                                                          const float* __restrict__ ein, double* __restrict__ s) {
  const BranchDev bd = st.br[b];
  const int64_t n = st.n;
  const int k = blockIdx.x;
  double v = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += FEED_T) {
    const int64_t at = (int64_t)k * n + i;
    v += (double)(act_dh(pre[at], act[at], bd.act) * ein[at]);
  }
  __shared__ double red[FEED_T];
  red[threadIdx.x] = v;
  __syncthreads();
  for (int w = FEED_T / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) s[k] = red[0];
}

// pop[j] = sum_k W0(j, k) s_k / n
__global__ void __launch_bounds__(FEED_T) k_effect_pop(DevState st, int b, const double* __restrict__ s,
                                                       float* __restrict__ pop) {
  const BranchDev bd = st.br[b];
  const int j = blockIdx.x * FEED_T + threadIdx.x;
  if (j >= bd.m) return;
  const float* W = st.theta + bd.p_off + bd.woff[0];
  double v = 0.0;
  for (int k = 0; k < bd.widths[0]; ++k) v += (double)W[(int64_t)k * bd.m + j] * s[k];
  pop[j] = (float)(v / (double)st.n);
}

// pre / act: forward_feed's layers (launch_forward_feed); ea / eb: two [max w_l][n]
// buffers; full: the n x m effect-size matrix ([m][n]) or null; pop: m floats
// (the column means) or null, with s: w_0 doubles
void launch_effect_sizes(const DevState& st, int b, const BranchDev& bd, const float* pre, const float* act,
                         float* ea, float* eb, float* full, double* s, float* pop, hipStream_t strm) {
  const int64_t n = st.n;
  const int L = bd.L;
  const unsigned gx = (unsigned)((n + FEED_T - 1) / FEED_T);
  int64_t po[BANN_MAXL], ao[BANN_MAXL];
  int64_t p = 0, a = 0;
  for (int l = 0; l < L; ++l) {
    po[l] = p;
    ao[l] = a;
    a += (int64_t)bd.widths[l] * n;
    if (l < L - 1) p += (int64_t)bd.widths[l] * n;
  }
  hipLaunchKernelGGL(k_effect_seed, dim3(gx), dim3(FEED_T), 0, strm, st, b, act + ao[L - 1], ea);
  float* ein = ea;
  float* eout = eb;
  for (int l = L - 2; l >= 1; --l) {
    const dim3 grid(gx, (unsigned)((bd.win[l] + FEED_KB - 1) / FEED_KB));
    hipLaunchKernelGGL(k_effect_back, grid, dim3(FEED_T), 0, strm, st, b, l, pre + po[l], act + ao[l], ein, eout);
    float* t = ein;
    ein = eout;
    eout = t;
  }
  if (full) {
    const dim3 grid(gx, (unsigned)((bd.m + FEED_KB - 1) / FEED_KB));
    hipLaunchKernelGGL(k_effect_back, grid, dim3(FEED_T), 0, strm, st, b, 0, pre, act, ein, full);
  }
  if (pop) {
    hipLaunchKernelGGL(k_effect_colsum, dim3((unsigned)bd.widths[0]), dim3(FEED_T), 0, strm, st, b, pre, act, ein, s);
    hipLaunchKernelGGL(k_effect_pop, dim3((unsigned)((bd.m + FEED_T - 1) / FEED_T)), dim3(FEED_T), 0, strm, st, b, s,
                       pop);
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
