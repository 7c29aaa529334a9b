// kernels_grad.hip — log-density gradient of the branch network (the hot path).
//
// Replaces BranchSampler::backpropagate (branch_sampler.rs:813-875) with its
// forward_feed (743-782) and the rss it stores (823-828), for many branches per
// launch.  Two implementations write the same per-split partial sums of
// d(rss/2)/d(theta) in param_vec order (params.rs:700-715):
//
//  * k_fused_grad  — single pass over the packed int8 genotypes.  Per 64
//    individuals x 64 markers: the masked first layer Z0 = X W0 runs on
//    v_mfma_i32_16x16x64_i8 with W0/sigma split into four signed 7-bit digits
//    per column (N = 4 columns x 4 digits = 16); exact integer products, one
//    f32 rounding per 64-marker chunk.  The small head (hidden/summary/output
//    layers, the error e = f - y, rss, the back-propagated delta0) runs per
//    individual in one wave; dW0 = X^T delta0 accumulates on VALU from the SAME
//    genotype registers, so every genotype byte is read from HBM exactly once
//    per gradient evaluation (the reference reads the f32 block twice in
//    backpropagate plus once more in neg_hamiltonian).  Standardization
//    (g - mu)/sigma is folded: Z0 = G (W0/sigma) + (b0 - mu^T W0/sigma) and
//    dW0 = (G^T delta0 - mu (sum delta0)) / sigma.
//  * k_generic_*   — straightforward multi-pass kernels (any widths/depth),
//    reference op order, f32 standardized inputs, double accumulation.
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
__device__ __forceinline__ float x_std_at(const int8_t* xb, int nchunks, int64_t row, int j, float mu, float sig) {
  const int64_t f = row >> 4;
  const int c = j >> 6;
  const int lane = (int)(row & 15) + 16 * ((j & 63) >> 4);
  const float g = (float)xb[((f * nchunks + c) * 64 + lane) * 16 + (j & 15)];
  // bed.rs:353: (raw - means) / stds ; zero-variance markers contribute 0 (documented deviation)
  return sig > 0.f ? (g - mu) / sig : 0.f;
}

__global__ void k_generic_fwd0(DevState st, const int32_t* __restrict__ blist) {
  const int b = blist[blockIdx.y];
  const BranchDev bd = st.br[b];
  const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t npad = (int64_t)st.nfrag * 16;
  if (row >= npad) return;
  const int8_t* xb = st.xpk + bd.x_off;
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
      const int8_t* xb = st.xpk + bd.x_off;
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

// ===========================================================================
// fused path
// ===========================================================================

// One work item = fragments [frag_begin, frag_end) of one branch.  Wave w owns
// marker chunk w for the whole item: its A operand (W0/sigma digits) and its
// dW0 accumulators stay in registers.  Per tile of 4 fragments (64
// individuals): every wave streams its 4 x 1 KiB slab (prefetched one tile
// ahead into a ping-pong register buffer; loads are branch-free so the counted
// s_waitcnt keeps the next tile in flight), runs 4 MFMAs, publishes partial Z0
// through LDS; wave 0 runs the head for the 64 individuals; every wave then
// accumulates its dW0 block from the same genotype registers.
template <int NL, int NWMAX, int ACT>
__global__ void __launch_bounds__(64 * NWMAX) k_fused_grad(DevState st, const GradItem* __restrict__ items,
                                                           int write_pred) {
  constexpr int NH = NL - 1;  // layers with activations (0 .. L-2)
  constexpr int T = BANN_TILE_FRAGS;
  __shared__ float s_zp[NWMAX][T][16][4];  // per-chunk partial Z0
  __shared__ v4f s_delta[T][16];           // delta0 of the tile
  __shared__ HeadLds s_hd;
  __shared__ float s_db0[4];

  const GradItem it = items[blockIdx.x];
  const BranchDev& bd = st.br[it.branch];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int nch = bd.nchunks;
  const bool has_chunk = wave < nch;
  const int64_t n = st.n;

  // ---- head parameters into LDS (zero padded) ----
  for (int t = threadIdx.x; t < BANN_MAXL * 20; t += blockDim.x) {
    const int l = t / 20, r = t - l * 20;
    float v = 0.f;
    if (l >= 1 && l < NL) {
      if (r < 16) {
        const int j = r >> 2, k = r & 3;
        if (j < bd.win[l] && k < bd.widths[l]) v = st.theta[bd.p_off + bd.woff[l] + k * bd.win[l] + j];
        s_hd.W[l][j][k] = v;
      } else {
        const int k = r - 16;
        if (l < NL - 1 && k < bd.widths[l]) v = st.theta[bd.p_off + bd.boff[l] + k];
        s_hd.bias[l][k] = v;
      }
    } else if (l == 0 && r >= 16) {
      const int k = r - 16;
      s_hd.bias[0][k] = (k < bd.widths[0]) ? st.fc[it.branch].c0[k] : 0.f;
    }
  }
  const int mych = has_chunk ? wave : nch - 1;  // chunk-less waves re-read a valid slab (never used)
  const float scale = st.fc[it.branch].scale[lane >> 4];
  const v4i adig = *reinterpret_cast<const v4i*>(st.dig + bd.dig_off + ((int64_t)mych * 64 + lane) * 16);
  __syncthreads();

  const int64_t frag_bytes = (int64_t)nch * 1024;
  const int8_t* xw = st.xpk + bd.x_off + ((int64_t)mych * 64 + lane) * 16;
  const int fend = it.frag_end, flast = fend - 1;
  const float* ybr = st.y + bd.y_off;

  float acc[16][4];
#pragma unroll
  for (int j = 0; j < 16; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[j][k] = 0.f;

  // head accumulators (meaningful in wave 0 only)
  double rss = 0.0;
  float db[NH][4], dWo[4];
  float dW[NL > 2 ? NL - 2 : 1][4][4];  // dW_l for l = 1 .. L-2
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    dWo[k] = 0.f;
#pragma unroll
    for (int l = 0; l < NH; ++l) db[l][k] = 0.f;
#pragma unroll
    for (int l = 0; l < (NL > 2 ? NL - 2 : 1); ++l)
#pragma unroll
      for (int j = 0; j < 4; ++j) dW[l][j][k] = 0.f;
  }

  // branch-free loads: fragments past the item end are clamped to its last one
  auto load_tile = [&](int f0, v4i (&xv)[T], float& yv) {
#pragma unroll
    for (int q = 0; q < T; ++q) {
      const int f = min(f0 + q, flast);
      xv[q] = *reinterpret_cast<const v4i*>(xw + (int64_t)f * frag_bytes);
    }
    const int64_t row = (int64_t)min(f0 + (lane >> 4), flast) * 16 + (lane & 15);
    yv = ybr[row < n ? row : n - 1];
  };

  auto do_tile = [&](int f0, const v4i (&xv)[T], float yv) {
    // ---- forward, masked first layer on MFMA: partial Z0 of this chunk ----
    if (has_chunk) {
#pragma unroll
      for (int q = 0; q < T; ++q) {
#if BANN_ABLATE & 4
        v4i d = xv[q];
#else
        v4i d = __builtin_amdgcn_mfma_i32_16x16x64_i8(adig, xv[q], v4i{0, 0, 0, 0}, 0, 0, 0);
#endif
        // lane l: individual (l & 15), column k = l >> 4, digits d[0..3]
        const float zp = scale * ((float)d[0] + (float)d[1] * 0x1p-7f + (float)d[2] * 0x1p-14f +
                                  (float)d[3] * 0x1p-21f);
        s_zp[wave][q][lane & 15][lane >> 4] = zp;
      }
    }
    __syncthreads();

    // ---- head: one individual per lane of wave 0 ----
    if (wave == 0) {
      const int q = lane >> 4, rr = lane & 15;
      const int f = f0 + q;
      const int64_t row = (int64_t)f * 16 + rr;
      const bool valid = (f < fend) && (row < n);
#if BANN_ABLATE & 1
      const v4f p0 = *reinterpret_cast<const v4f*>(&s_zp[0][q][rr][0]);
      s_delta[q][rr] = p0 * 1e-3f;
      (void)valid;
      (void)yv;
#else
      float z[NH][4], a[NH][4];
#pragma unroll
      for (int k = 0; k < 4; ++k) z[0][k] = s_hd.bias[0][k];
#pragma unroll
      for (int w = 0; w < NWMAX; ++w) {
        if (w < nch) {
          const v4f p = *reinterpret_cast<const v4f*>(&s_zp[w][q][rr][0]);
#pragma unroll
          for (int k = 0; k < 4; ++k) z[0][k] += p[k];
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) a[0][k] = act_h_t<ACT>(z[0][k]);
#pragma unroll
      for (int l = 1; l < NH; ++l) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float s = s_hd.bias[l][k];
#pragma unroll
          for (int j = 0; j < 4; ++j) s = fmaf(a[l - 1][j], s_hd.W[l][j][k], s);
          z[l][k] = s;
          a[l][k] = act_h_t<ACT>(s);
        }
      }
      float out = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) out = fmaf(a[NH - 1][j], s_hd.W[NL - 1][j][0], out);
      const float e = valid ? out - yv : 0.f;
      if (write_pred && valid) st.pred[bd.y_off + row] = out;
      rss += (double)e * (double)e;
      float err[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dWo[j] = fmaf(a[NH - 1][j], e, dWo[j]);
        err[j] = e * s_hd.W[NL - 1][j][0];
      }
#pragma unroll
      for (int l = NH - 1; l >= 0; --l) {
        float d[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          d[k] = act_dh_t<ACT>(z[l][k], a[l][k]) * err[k];
          db[l][k] += d[k];
        }
        if (l >= 1) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float sj = 0.f;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              dW[l - 1][j][k] = fmaf(a[l - 1][j], d[k], dW[l - 1][j][k]);
              sj = fmaf(d[k], s_hd.W[l][j][k], sj);
            }
            err[j] = sj;
          }
        } else {
          s_delta[q][rr] = v4f{d[0], d[1], d[2], d[3]};
        }
      }
#endif
    }
    __syncthreads();

    // ---- backward, masked first layer on VALU: acc[j][k] += x_j * delta0_k ----
#if BANN_ABLATE & 2
    if (has_chunk) {
#pragma unroll
      for (int q = 0; q < T; ++q) {
        const v4f dl = s_delta[q][lane & 15];
        asm volatile("" ::"v"(xv[q]), "v"(dl));
      }
    }
#else
    if (has_chunk) {
#pragma unroll
      for (int q = 0; q < T; ++q) {
        const v4f dl = s_delta[q][lane & 15];
#pragma unroll
        for (int w4 = 0; w4 < 4; ++w4) {
          const uint32_t word = (uint32_t)xv[q][w4];
#pragma unroll
          for (int bq = 0; bq < 4; ++bq) {
            const float x = (float)((word >> (8 * bq)) & 0xFFu);
#pragma unroll
            for (int k = 0; k < 4; ++k) acc[w4 * 4 + bq][k] = fmaf(x, dl[k], acc[w4 * 4 + bq][k]);
          }
        }
      }
    }
#endif
  };

  v4i xa[T], xb[T];
  float ya, yb;
  load_tile(it.frag_begin, xa, ya);
  for (int f0 = it.frag_begin;; f0 += 2 * T) {
    load_tile(f0 + T, xb, yb);
    do_tile(f0, xa, ya);
    if (f0 + T >= fend) break;
    load_tile(f0 + 2 * T, xa, ya);
    do_tile(f0 + T, xb, yb);
    if (f0 + 2 * T >= fend) break;
  }

  // ---- head sums: reduce over the 64 rows-lanes of wave 0 and publish ----
  float* part = st.part + bd.part_off + (int64_t)it.split * bd.P;
  if (wave == 0) {
    const double rs = wave_sum_d(rss);
    float db0s[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) db0s[k] = wave_sum(db[0][k]);
    if (lane == 0) {
      st.rss_part[(int64_t)it.branch * st.max_splits + it.split] = rs;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s_db0[k] = db0s[k];
        if (k < bd.widths[0]) part[bd.boff[0] + k] = db0s[k];
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float v = wave_sum(dWo[j]);
      if (lane == 0 && j < bd.win[NL - 1]) part[bd.woff[NL - 1] + j] = v;
    }
#pragma unroll
    for (int l = 1; l < NH; ++l) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float v = wave_sum(db[l][k]);
        if (lane == 0 && k < bd.widths[l]) part[bd.boff[l] + k] = v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float w = wave_sum(dW[l - 1][j][k]);
          if (lane == 0 && j < bd.win[l] && k < bd.widths[l]) part[bd.woff[l] + k * bd.win[l] + j] = w;
        }
      }
    }
  }
  __syncthreads();

  // ---- dW0 partial: reduce acc over the 16 individuals-lanes of each marker group ----
  if (has_chunk) {
#pragma unroll
    for (int j = 0; j < 16; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float v = acc[j][k];
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        v += __shfl_xor(v, 8);
        acc[j][k] = v;
      }
    const int rr = lane & 15;
    float mine[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 16; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) mine[k] = (j == rr) ? acc[j][k] : mine[k];
    const int sidx = wave * 64 + (lane >> 4) * 16 + rr;
    if (sidx < bd.m) {
      const float mu = st.mu[bd.mk_off + sidx], sg = st.sigma[bd.mk_off + sidx];
      const int w0 = bd.widths[0];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (k < w0) part[bd.woff[0] + k * bd.m + sidx] = sg > 0.f ? (mine[k] - mu * s_db0[k]) / sg : 0.f;
    }
  }
}


// ---------------------------------------------------------------------------
// Pipelined variant (default): wave 0 is a dedicated HEAD wave, waves 1..NW own
// the marker chunks.  One barrier per tile; in iteration t the chunk waves run
// forward(t) and backward(t-1) while the head wave runs head(t-1)... precisely:
//   chunk wave, iteration t:  DMA X(t+D) -> wait X(t) -> MFMA fwd(t) -> zp[t&1]
//                              BARRIER(t)
//                              bwd(t-1) with delta[(t-1)&1] and X(t-1) (LDS ring)
//   head wave,  iteration t:  BARRIER(t) -> head(t) from zp[t&1] -> delta[t&1]
// so the latency-bound per-individual head overlaps the chunk waves' streaming
// MFMA/VALU work instead of stalling them, and the head's registers and the
// chunk waves' dW0 accumulators are never live in the same wave.
// ---------------------------------------------------------------------------
template <int NL, int NWMAX, int ACT, int R>
__global__ void __launch_bounds__(64 * (NWMAX + 1))
    k_fused_grad_pipe(DevState st, const GradItem* __restrict__ items, int write_pred) {
  static_assert(R == 3, "the slot-unrolled loops below assume a 3-slot ring");
  constexpr int NH = NL - 1;
  constexpr int T = BANN_TILE_FRAGS;
  constexpr int D = R - 2;  // prefetch distance in tiles
  constexpr int SLAB = 1024;
  // Every LDS-DMA target is its OWN __shared__ object and every slot index is a
  // compile-time constant: hipcc can then prove that a ds_read of slot s does
  // not alias the DMA in flight into slot s+D and keeps the counted vmcnt wait
  // (with one shared array it drains the prefetch with vmcnt(0) before every read).
  __shared__ __attribute__((aligned(16))) char xr0[NWMAX * T * SLAB];
  __shared__ __attribute__((aligned(16))) char xr1[NWMAX * T * SLAB];
  __shared__ __attribute__((aligned(16))) char xr2[NWMAX * T * SLAB];
  __shared__ __attribute__((aligned(16))) float yr0[64];
  __shared__ __attribute__((aligned(16))) float yr1[64];
  __shared__ __attribute__((aligned(16))) float yr2[64];
  __shared__ __attribute__((aligned(16))) float s_zp[2][NWMAX][T][16][4];
  __shared__ __attribute__((aligned(16))) v4f s_delta[2][T][16];
  __shared__ __attribute__((aligned(16))) HeadLds s_hd;
  __shared__ __attribute__((aligned(16))) float s_db0[4];

  const GradItem it = items[blockIdx.x];
  const BranchDev& bd = st.br[it.branch];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int nch = bd.nchunks;
  const int64_t n = st.n;
  const int fbeg = it.frag_begin, fend = it.frag_end, flast = fend - 1;
  const int ntiles = (fend - fbeg + T - 1) / T;

  for (int t = threadIdx.x; t < BANN_MAXL * 20; t += blockDim.x) {
    const int l = t / 20, r = t - l * 20;
    float v = 0.f;
    if (l >= 1 && l < NL) {
      if (r < 16) {
        const int j = r >> 2, k = r & 3;
        if (j < bd.win[l] && k < bd.widths[l]) v = st.theta[bd.p_off + bd.woff[l] + k * bd.win[l] + j];
        s_hd.W[l][j][k] = v;
      } else {
        const int k = r - 16;
        if (l < NL - 1 && k < bd.widths[l]) v = st.theta[bd.p_off + bd.boff[l] + k];
        s_hd.bias[l][k] = v;
      }
    } else if (l == 0 && r >= 16) {
      const int k = r - 16;
      s_hd.bias[0][k] = (k < bd.widths[0]) ? st.fc[it.branch].c0[k] : 0.f;
    }
  }
  __syncthreads();

  float* part = st.part + bd.part_off + (int64_t)it.split * bd.P;

  if (wave == 0) {
    // ===================== head wave =====================
    const int64_t y_off = bd.y_off;
    const float* ybr = st.y + y_off;
    float* predb = st.pred + y_off;
    auto yslot = [&](auto sc) -> float* {
      constexpr int s = decltype(sc)::value;
      if constexpr (s == 0) return yr0;
      else if constexpr (s == 1) return yr1;
      else return yr2;
    };
    auto issue_y = [&](int t, auto sc) {
      const int64_t row = (int64_t)min(fbeg + t * T + (lane >> 4), flast) * 16 + (lane & 15);
      glds4(ybr + (row < n ? row : n - 1), yslot(sc));
    };
    double rss = 0.0;
    float db[NH][4], dWo[4];
    float dW[NL > 2 ? NL - 2 : 1][4][4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      dWo[k] = 0.f;
#pragma unroll
      for (int l = 0; l < NH; ++l) db[l][k] = 0.f;
#pragma unroll
      for (int l = 0; l < (NL > 2 ? NL - 2 : 1); ++l)
#pragma unroll
        for (int j = 0; j < 4; ++j) dW[l][j][k] = 0.f;
    }
    issue_y(0, std::integral_constant<int, 0>{});
    // iteration t uses y slot t % 3 and zp / delta buffer t & 1
    auto head_iter = [&](int t, auto sc) {
      constexpr int s = decltype(sc)::value;
      if (t < ntiles) issue_y(t + D, std::integral_constant<int, (s + D) % R>{});
      LDS_BARRIER();
      if (t == ntiles) return;
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D) : "memory");  // y(t) landed (y(t+D) may fly)
      const int q = lane >> 4, rr = lane & 15;
      const int f = fbeg + t * T + q;
      const int64_t row = (int64_t)f * 16 + rr;
      const bool valid = (f < fend) && (row < n);
      const float yv = yslot(sc)[lane];
      const int zb = t & 1;
#if BANN_ABLATE & 1
      {
        const v4f p0 = *reinterpret_cast<const v4f*>(&s_zp[zb][0][q][rr][0]);
        lds_st_v4f(&s_delta[zb][q][rr], p0 * 1e-3f);
        (void)valid;
        (void)yv;
      }
#else
      float z[NH][4], a[NH][4];
      v4f zs = *reinterpret_cast<const v4f*>(&s_hd.bias[0][0]);
#pragma unroll
      for (int w = 0; w < NWMAX; ++w) {
        const v4f p = *reinterpret_cast<const v4f*>(&s_zp[zb][w][q][rr][0]);  // chunk-less waves wrote 0
        zs += p;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        z[0][k] = zs[k];
        a[0][k] = act_h_t<ACT>(z[0][k]);
      }
#pragma unroll
      for (int l = 1; l < NH; ++l) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float sacc = s_hd.bias[l][k];
#pragma unroll
          for (int j = 0; j < 4; ++j) sacc = fmaf(a[l - 1][j], s_hd.W[l][j][k], sacc);
          z[l][k] = sacc;
          a[l][k] = act_h_t<ACT>(sacc);
        }
      }
      float out = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) out = fmaf(a[NH - 1][j], s_hd.W[NL - 1][j][0], out);
      const float e = valid ? out - yv : 0.f;
      if (write_pred && valid) predb[row] = out;
      rss += (double)e * (double)e;
      float err[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dWo[j] = fmaf(a[NH - 1][j], e, dWo[j]);
        err[j] = e * s_hd.W[NL - 1][j][0];
      }
#pragma unroll
      for (int l = NH - 1; l >= 0; --l) {
        float d[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          d[k] = act_dh_t<ACT>(z[l][k], a[l][k]) * err[k];
          db[l][k] += d[k];
        }
        if (l >= 1) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float sj = 0.f;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              dW[l - 1][j][k] = fmaf(a[l - 1][j], d[k], dW[l - 1][j][k]);
              sj = fmaf(d[k], s_hd.W[l][j][k], sj);
            }
            err[j] = sj;
          }
        } else {
          lds_st_v4f(&s_delta[zb][q][rr], v4f{d[0], d[1], d[2], d[3]});
        }
      }
#endif
    };
    for (int t = 0; t <= ntiles; t += 3) {
      head_iter(t, std::integral_constant<int, 0>{});
      if (t + 1 > ntiles) break;
      head_iter(t + 1, std::integral_constant<int, 1>{});
      if (t + 2 > ntiles) break;
      head_iter(t + 2, std::integral_constant<int, 2>{});
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const double rs = wave_sum_d(rss);
    float db0s[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) db0s[k] = wave_sum(db[0][k]);
    if (lane == 0) {
      st.rss_part[(int64_t)it.branch * st.max_splits + it.split] = rs;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s_db0[k] = db0s[k];
        if (k < bd.widths[0]) part[bd.boff[0] + k] = db0s[k];
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float v = wave_sum(dWo[j]);
      if (lane == 0 && j < bd.win[NL - 1]) part[bd.woff[NL - 1] + j] = v;
    }
#pragma unroll
    for (int l = 1; l < NH; ++l) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float v = wave_sum(db[l][k]);
        if (lane == 0 && k < bd.widths[l]) part[bd.boff[l] + k] = v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float w = wave_sum(dW[l - 1][j][k]);
          if (lane == 0 && j < bd.win[l] && k < bd.widths[l]) part[bd.woff[l] + k * bd.win[l] + j] = w;
        }
      }
    }
    __syncthreads();  // s_db0 visible to the chunk waves
  } else {
    // ===================== chunk waves =====================
    const int cw = wave - 1;
    const bool has_chunk = cw < nch;
    const int mych = has_chunk ? cw : nch - 1;
    float scale = has_chunk ? st.fc[it.branch].scale[lane >> 4] : 0.f;  // chunk-less: zp = 0
    v4i adig = *reinterpret_cast<const v4i*>(st.dig + bd.dig_off + ((int64_t)mych * 64 + lane) * 16);
    // retire these loads now and hide their provenance, so the compiler's wait
    // model does not re-wait on them (with vmcnt(0)) while the asm DMAs fly
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("" : "+v"(adig), "+v"(scale));
    const int64_t frag_bytes = (int64_t)nch * 1024;
    const int8_t* xw = st.xpk + bd.x_off + ((int64_t)mych * 64 + lane) * 16;
    auto xslot = [&](auto sc) -> char* {
      constexpr int s = decltype(sc)::value;
      if constexpr (s == 0) return xr0 + cw * T * SLAB;
      else if constexpr (s == 1) return xr1 + cw * T * SLAB;
      else return xr2 + cw * T * SLAB;
    };
    auto issue_x = [&](int t, auto sc) {
      char* base = xslot(sc);
#pragma unroll
      for (int q = 0; q < T; ++q) {
        const int f = min(fbeg + t * T + q, flast);
        glds16(xw + (int64_t)f * frag_bytes, base + q * SLAB);
      }
    };
    float acc[16][4];
#pragma unroll
    for (int j = 0; j < 16; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[j][k] = 0.f;
    issue_x(0, std::integral_constant<int, 0>{});
    auto chunk_iter = [&](int t, auto sc) {
      constexpr int s = decltype(sc)::value;
      if (t < ntiles) {
        issue_x(t + D, std::integral_constant<int, (s + D) % R>{});  // clamped: always valid
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(T * D) : "memory");  // X(t) landed, X(t+D) in flight
        const v4i* xs = reinterpret_cast<const v4i*>(xslot(sc)) + lane;
#pragma unroll
        for (int q = 0; q < T; ++q) {
          const v4i xv = xs[q * 64];
#if BANN_ABLATE & 4
          v4i d = xv;
#else
          v4i d = __builtin_amdgcn_mfma_i32_16x16x64_i8(adig, xv, v4i{0, 0, 0, 0}, 0, 0, 0);
#endif
          const float zp = scale * ((float)d[0] + (float)d[1] * 0x1p-7f + (float)d[2] * 0x1p-14f +
                                    (float)d[3] * 0x1p-21f);
          lds_st_f32(&s_zp[t & 1][cw][q][lane & 15][lane >> 4], zp);
        }
      }
      LDS_BARRIER();
      if (t >= 1 && has_chunk) {
        const int tb = t - 1;
        const v4i* xs = reinterpret_cast<const v4i*>(xslot(std::integral_constant<int, (s + R - 1) % R>{})) + lane;
#pragma unroll
        for (int q = 0; q < T; ++q) {
          const v4f dl = s_delta[tb & 1][q][lane & 15];
          const v4i xv = xs[q * 64];
#if BANN_ABLATE & 2
          asm volatile("" ::"v"(xv), "v"(dl));
#else
#pragma unroll
          for (int w4 = 0; w4 < 4; ++w4) {
            const uint32_t word = (uint32_t)xv[w4];
#pragma unroll
            for (int bq = 0; bq < 4; ++bq) {
              const float x = (float)((word >> (8 * bq)) & 0xFFu);
#pragma unroll
              for (int k = 0; k < 4; ++k) acc[w4 * 4 + bq][k] = fmaf(x, dl[k], acc[w4 * 4 + bq][k]);
            }
          }
#endif
        }
      }
    };
    for (int t = 0; t <= ntiles; t += 3) {
      chunk_iter(t, std::integral_constant<int, 0>{});
      if (t + 1 > ntiles) break;
      chunk_iter(t + 1, std::integral_constant<int, 1>{});
      if (t + 2 > ntiles) break;
      chunk_iter(t + 2, std::integral_constant<int, 2>{});
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // s_db0 published by the head wave
    if (has_chunk) {
#pragma unroll
      for (int j = 0; j < 16; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float v = acc[j][k];
          v += __shfl_xor(v, 1);
          v += __shfl_xor(v, 2);
          v += __shfl_xor(v, 4);
          v += __shfl_xor(v, 8);
          acc[j][k] = v;
        }
      const int rr = lane & 15;
      float mine[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 16; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k) mine[k] = (j == rr) ? acc[j][k] : mine[k];
      const int sidx = cw * 64 + (lane >> 4) * 16 + rr;
      if (sidx < bd.m) {
        const float mu = st.mu[bd.mk_off + sidx], sg = st.sigma[bd.mk_off + sidx];
        const int w0 = bd.widths[0];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (k < w0) part[bd.woff[0] + k * bd.m + sidx] = sg > 0.f ? (mine[k] - mu * s_db0[k]) / sg : 0.f;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// MFMA-backward variant ("mx"): the pipelined schedule of k_fused_grad_pipe,
// with dW0 = G^T delta0 ALSO on v_mfma_i32_16x16x64_i8 instead of VALU FMAs.
//
// The backward contracts over individuals, so its genotype operand is the
// TRANSPOSE of the forward's (a lane needs 16 individuals of one marker, the
// packed layout gives 16 markers of one individual).  The tile is already in
// LDS (LDS-DMA ring), so the transpose is free: ds_read_b64_tr_b8 delivers,
// per 16-lane group, column i of an 8-row x 16-byte block to lane i.
//   * B (K = 64 individuals x N = 16 markers of sub-tile u): group g reads
//     fragment g; read h covers individuals 8h .. 8h+7 of that fragment.
//   * A (M = 4 columns x 4 digits, K = 64 individuals): the head wave writes
//     delta0 of its individual as 16 signed digits (byte 4c + d) in a row of an
//     [individual][16 B] image; the same transposed read yields A.
// delta0 is quantised per tile and column with a power-of-two scale
// s_c = 2^(E_c - 132) (E_c = the largest f32 exponent field in the column):
// delta/s_c < 64, four digits of 7 bits carry 27 significant bits, so the
// integer products are exact and the only roundings are the per-tile f32
// accumulations (one per sub-tile and digit set).
// The fragment stride in LDS is padded to 1152 B (and 384 B in the digit
// image) so the two 16-lane groups of a half-wave read disjoint bank halves.
// ---------------------------------------------------------------------------

template <int NL, int NWMAX, int ACT>
__global__ void __launch_bounds__(64 * (NWMAX + 1))
    k_fused_grad_mx(DevState st, const GradItem* __restrict__ items, int write_pred) {
  constexpr int R = 3;
  constexpr int NH = NL - 1;
  constexpr int T = BANN_TILE_FRAGS;
  static_assert(T == 4, "the backward MFMA contracts over exactly 4 fragments (64 individuals)");
  constexpr int D = R - 2;       // prefetch distance in tiles
  constexpr int SLAB = 1152;     // 1 KiB fragment slab + 128 B bank padding
  constexpr int DROW = 384;      // digit image: 16 rows x 16 B + 128 B padding per fragment
  __shared__ __attribute__((aligned(16))) char xr0[NWMAX * T * SLAB];
  __shared__ __attribute__((aligned(16))) char xr1[NWMAX * T * SLAB];
  __shared__ __attribute__((aligned(16))) char xr2[NWMAX * T * SLAB];
  __shared__ __attribute__((aligned(16))) float yr0[64];
  __shared__ __attribute__((aligned(16))) float yr1[64];
  __shared__ __attribute__((aligned(16))) float yr2[64];
  __shared__ __attribute__((aligned(16))) float s_zp[2][NWMAX][T][16][4];
  __shared__ __attribute__((aligned(16))) char s_dig[2][T * DROW];
  __shared__ __attribute__((aligned(16))) float s_scl[2][4];
  __shared__ __attribute__((aligned(16))) HeadLds s_hd;
  __shared__ __attribute__((aligned(16))) float s_db0[4];

  const GradItem it = items[blockIdx.x];
  const BranchDev& bd = st.br[it.branch];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int nch = bd.nchunks;
  const int64_t n = st.n;
  const int fbeg = it.frag_begin, fend = it.frag_end, flast = fend - 1;
  const int ntiles = (fend - fbeg + T - 1) / T;

  for (int t = threadIdx.x; t < BANN_MAXL * 20; t += blockDim.x) {
    const int l = t / 20, r = t - l * 20;
    float v = 0.f;
    if (l >= 1 && l < NL) {
      if (r < 16) {
        const int j = r >> 2, k = r & 3;
        if (j < bd.win[l] && k < bd.widths[l]) v = st.theta[bd.p_off + bd.woff[l] + k * bd.win[l] + j];
        s_hd.W[l][j][k] = v;
      } else {
        const int k = r - 16;
        if (l < NL - 1 && k < bd.widths[l]) v = st.theta[bd.p_off + bd.boff[l] + k];
        s_hd.bias[l][k] = v;
      }
    } else if (l == 0 && r >= 16) {
      const int k = r - 16;
      s_hd.bias[0][k] = (k < bd.widths[0]) ? st.fc[it.branch].c0[k] : 0.f;
    }
  }
  __syncthreads();

  float* part = st.part + bd.part_off + (int64_t)it.split * bd.P;

  if (wave == 0) {
    // ===================== head wave =====================
    const int64_t y_off = bd.y_off;
    const float* ybr = st.y + y_off;
    float* predb = st.pred + y_off;
    auto yslot = [&](auto sc) -> float* {
      constexpr int s = decltype(sc)::value;
      if constexpr (s == 0) return yr0;
      else if constexpr (s == 1) return yr1;
      else return yr2;
    };
    auto issue_y = [&](int t, auto sc) {
      const int64_t row = (int64_t)min(fbeg + t * T + (lane >> 4), flast) * 16 + (lane & 15);
      glds4(ybr + (row < n ? row : n - 1), yslot(sc));
    };
    double rss = 0.0;
    float db[NH][4], dWo[4];
    float dW[NL > 2 ? NL - 2 : 1][4][4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      dWo[k] = 0.f;
#pragma unroll
      for (int l = 0; l < NH; ++l) db[l][k] = 0.f;
#pragma unroll
      for (int l = 0; l < (NL > 2 ? NL - 2 : 1); ++l)
#pragma unroll
        for (int j = 0; j < 4; ++j) dW[l][j][k] = 0.f;
    }
    issue_y(0, std::integral_constant<int, 0>{});
    auto head_iter = [&](int t, auto sc) {
      constexpr int s = decltype(sc)::value;
      if (t < ntiles) issue_y(t + D, std::integral_constant<int, (s + D) % R>{});
      LDS_BARRIER();
      if (t == ntiles) return;
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D) : "memory");  // y(t) landed (y(t+D) may fly)
      const int q = lane >> 4, rr = lane & 15;
      const int f = fbeg + t * T + q;
      const int64_t row = (int64_t)f * 16 + rr;
      const bool valid = (f < fend) && (row < n);
      const float yv = yslot(sc)[lane];
      const int zb = t & 1;
      float d[4];
#if BANN_ABLATE & 1
      {
        const v4f p0 = *reinterpret_cast<const v4f*>(&s_zp[zb][0][q][rr][0]);
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] = valid ? p0[k] * 1e-3f - yv : 0.f;
      }
#else
      float z[NH][4], a[NH][4];
      v4f zs = *reinterpret_cast<const v4f*>(&s_hd.bias[0][0]);
#pragma unroll
      for (int w = 0; w < NWMAX; ++w) {
        const v4f p = *reinterpret_cast<const v4f*>(&s_zp[zb][w][q][rr][0]);  // chunk-less waves wrote 0
        zs += p;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        z[0][k] = zs[k];
        a[0][k] = act_h_t<ACT>(z[0][k]);
      }
#pragma unroll
      for (int l = 1; l < NH; ++l) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float sacc = s_hd.bias[l][k];
#pragma unroll
          for (int j = 0; j < 4; ++j) sacc = fmaf(a[l - 1][j], s_hd.W[l][j][k], sacc);
          z[l][k] = sacc;
          a[l][k] = act_h_t<ACT>(sacc);
        }
      }
      float out = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) out = fmaf(a[NH - 1][j], s_hd.W[NL - 1][j][0], out);
      const float e = valid ? out - yv : 0.f;
      if (write_pred && valid) predb[row] = out;
      rss += (double)e * (double)e;
      float err[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dWo[j] = fmaf(a[NH - 1][j], e, dWo[j]);
        err[j] = e * s_hd.W[NL - 1][j][0];
      }
#pragma unroll
      for (int l = NH - 1; l >= 0; --l) {
        float dl[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          dl[k] = act_dh_t<ACT>(z[l][k], a[l][k]) * err[k];
          db[l][k] += dl[k];
        }
        if (l >= 1) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float sj = 0.f;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              dW[l - 1][j][k] = fmaf(a[l - 1][j], dl[k], dW[l - 1][j][k]);
              sj = fmaf(dl[k], s_hd.W[l][j][k], sj);
            }
            err[j] = sj;
          }
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) d[k] = dl[k];
        }
      }
#endif
      // ---- delta0 -> per-column power-of-two scale + 4 digits (A image) ----
      const uint32_t e01 = wave_max_u16x2(((fbits(d[0]) >> 23) & 0xFFu) | (((fbits(d[1]) >> 23) & 0xFFu) << 16));
      const uint32_t e23 = wave_max_u16x2(((fbits(d[2]) >> 23) & 0xFFu) | (((fbits(d[3]) >> 23) & 0xFFu) << 16));
      const uint32_t E[4] = {e01 & 0xFFFFu, e01 >> 16, e23 & 0xFFFFu, e23 >> 16};
      v4i w;
      v4f scl;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool ok = E[k] >= 6u;   // columns below 2^-121 (or all zero) contribute 0
        const float inv = ok ? fpow2(259u - E[k]) : 0.f;
        scl[k] = ok ? fpow2(E[k] - 5u) : 0.f;
        w[k] = (int)digits4(d[k] * inv);
      }
      asm volatile("ds_write_b128 %0, %1" ::"v"(lds_off(&s_dig[zb][q * DROW + rr * 16])), "v"(w) : "memory");
      if (lane == 0) lds_st_v4f(reinterpret_cast<v4f*>(&s_scl[zb][0]), scl);
    };
    for (int t = 0; t <= ntiles; t += 3) {
      head_iter(t, std::integral_constant<int, 0>{});
      if (t + 1 > ntiles) break;
      head_iter(t + 1, std::integral_constant<int, 1>{});
      if (t + 2 > ntiles) break;
      head_iter(t + 2, std::integral_constant<int, 2>{});
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const double rs = wave_sum_d(rss);
    float db0s[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) db0s[k] = wave_sum(db[0][k]);
    if (lane == 0) {
      st.rss_part[(int64_t)it.branch * st.max_splits + it.split] = rs;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s_db0[k] = db0s[k];
        if (k < bd.widths[0]) part[bd.boff[0] + k] = db0s[k];
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float v = wave_sum(dWo[j]);
      if (lane == 0 && j < bd.win[NL - 1]) part[bd.woff[NL - 1] + j] = v;
    }
#pragma unroll
    for (int l = 1; l < NH; ++l) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float v = wave_sum(db[l][k]);
        if (lane == 0 && k < bd.widths[l]) part[bd.boff[l] + k] = v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float wv = wave_sum(dW[l - 1][j][k]);
          if (lane == 0 && j < bd.win[l] && k < bd.widths[l]) part[bd.woff[l] + k * bd.win[l] + j] = wv;
        }
      }
    }
    __syncthreads();  // s_db0 visible to the chunk waves
  } else {
    // ===================== chunk waves =====================
    const int cw = wave - 1;
    const bool has_chunk = cw < nch;
    const int mych = has_chunk ? cw : nch - 1;
    float scale = has_chunk ? st.fc[it.branch].scale[lane >> 4] : 0.f;  // chunk-less: zp = 0
    v4i adig = *reinterpret_cast<const v4i*>(st.dig + bd.dig_off + ((int64_t)mych * 64 + lane) * 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("" : "+v"(adig), "+v"(scale));
    const int64_t frag_bytes = (int64_t)nch * 1024;
    const int8_t* xw = st.xpk + bd.x_off + ((int64_t)mych * 64 + lane) * 16;
    auto xslot = [&](auto sc) -> char* {
      constexpr int s = decltype(sc)::value;
      if constexpr (s == 0) return xr0 + cw * T * SLAB;
      else if constexpr (s == 1) return xr1 + cw * T * SLAB;
      else return xr2 + cw * T * SLAB;
    };
    auto issue_x = [&](int t, auto sc) {
      char* base = xslot(sc);
#if BANN_ABLATE & 8
      (void)base;
      return;  // compute-only profiling build: no genotype traffic
#endif
#pragma unroll
      for (int q = 0; q < T; ++q) {
        const int f = min(fbeg + t * T + q, flast);
        glds16(xw + (int64_t)f * frag_bytes, base + q * SLAB);
      }
    };
    // transposed-read address of this lane inside a fragment-padded image:
    // group g = lane >> 4 -> fragment g; lane 2r + p -> row r, bytes 8p .. 8p+7
    const int tr_off = (lane & 15) / 2 * 16 + 8 * (lane & 1);
    float dw[4] = {0.f, 0.f, 0.f, 0.f};  // dW0 (G^T delta0) of column lane>>4, marker 16u + (lane & 15)
    issue_x(0, std::integral_constant<int, 0>{});
    auto chunk_iter = [&](int t, auto sc) {
      constexpr int s = decltype(sc)::value;
      if (t < ntiles) {
        issue_x(t + D, std::integral_constant<int, (s + D) % R>{});  // clamped: always valid
#if !(BANN_ABLATE & 8)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(T * D) : "memory");  // X(t) landed, X(t+D) in flight
#endif
        const char* xs = xslot(sc) + lane * 16;
#pragma unroll
        for (int q = 0; q < T; ++q) {
          const v4i xv = *reinterpret_cast<const v4i*>(xs + q * SLAB);
#if BANN_ABLATE & 4
          v4i d = xv;
#else
          v4i d = __builtin_amdgcn_mfma_i32_16x16x64_i8(adig, xv, v4i{0, 0, 0, 0}, 0, 0, 0);
#endif
          const float zp = scale * ((float)d[0] + (float)d[1] * 0x1p-7f + (float)d[2] * 0x1p-14f +
                                    (float)d[3] * 0x1p-21f);
          lds_st_f32(&s_zp[t & 1][cw][q][lane & 15][lane >> 4], zp);
        }
      }
      LDS_BARRIER();
      if (t >= 1 && has_chunk) {
        const int tb = t - 1;
        const char* xs = xslot(std::integral_constant<int, (s + R - 1) % R>{}) + (lane >> 4) * SLAB + tr_off;
        const char* ds = &s_dig[tb & 1][0] + (lane >> 4) * DROW + tr_off;
        const v4i A = lds_tr8_pair(ds, ds + 8 * 16);
        const float sc_c = s_scl[tb & 1][lane >> 4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const v4i B = lds_tr8_pair(xs + u * 256, xs + u * 256 + 8 * 16);
#if BANN_ABLATE & 2
          asm volatile("" ::"v"(A), "v"(B));
#else
          const v4i g = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B, v4i{0, 0, 0, 0}, 0, 0, 0);
          const float v = (float)g[0] + (float)g[1] * 0x1p-7f + (float)g[2] * 0x1p-14f + (float)g[3] * 0x1p-21f;
          dw[u] = fmaf(sc_c, v, dw[u]);
#endif
        }
      }
    };
    for (int t = 0; t <= ntiles; t += 3) {
      chunk_iter(t, std::integral_constant<int, 0>{});
      if (t + 1 > ntiles) break;
      chunk_iter(t + 1, std::integral_constant<int, 1>{});
      if (t + 2 > ntiles) break;
      chunk_iter(t + 2, std::integral_constant<int, 2>{});
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // s_db0 published by the head wave
    if (has_chunk) {
      const int c = lane >> 4;
      if (c < bd.widths[0]) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int sidx = cw * 64 + u * 16 + (lane & 15);
          if (sidx < bd.m) {
            const float mu = st.mu[bd.mk_off + sidx], sg = st.sigma[bd.mk_off + sidx];
            part[bd.woff[0] + c * bd.m + sidx] = sg > 0.f ? (dw[u] - mu * s_db0[c]) / sg : 0.f;
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Register-staged variant ("rx", default): the genotype tile goes straight
// from HBM into VGPRs (global_load_dwordx4, prefetched one tile ahead in a
// ping-pong register pair; the compiler's counted vmcnt waits keep the next
// tile in flight), feeds the forward MFMA from registers, and is written to
// LDS only for the backward's transposed read.  LDS per workgroup is one tile
// image per chunk wave (32 KiB) plus the partial-Z0 / digit exchange (~20 KiB),
// so TWO workgroups share a CU: two head waves, two pipelines, 18 waves.
//
// U2 = genotypes stored as 2-bit codes in HBM (4x fewer bytes than int8):
// per (tile of 4 fragments, chunk) a lane holds 4 words, one per fragment;
// genotype j = 4k + b of the lane's 16 sits at bits 8b + 2k, so byte-group k
// unpacks as (w >> 2k) & 0x03030303 -- the B operand in two VALU ops per VGPR.
// Backward-image rows of odd fragments are rotated by 8 rows (128 B), which
// puts the two 16-lane groups of every transposed read on disjoint banks.
// ---------------------------------------------------------------------------
template <int NL, int ACT, bool U2>
__global__ void __launch_bounds__(576, 6)
    k_fused_grad_rx(DevState st, const GradItem* __restrict__ items, int write_pred) {
  constexpr int NW = 8;
  constexpr int NH = NL - 1;
  constexpr int T = BANN_TILE_FRAGS;
  static_assert(T == 4, "the backward MFMA contracts over exactly 4 fragments (64 individuals)");
  constexpr int DROW = 384;
  __shared__ __attribute__((aligned(16))) char s_img[NW][T * 1024];
  __shared__ __attribute__((aligned(16))) float s_zp[2][NW][T][16][4];
  __shared__ __attribute__((aligned(16))) char s_dig[2][T * DROW];
  __shared__ __attribute__((aligned(16))) float s_scl[2][4];
  __shared__ __attribute__((aligned(16))) HeadLds s_hd;
  __shared__ __attribute__((aligned(16))) float s_db0[4];

  const GradItem it = items[blockIdx.x];
  const BranchDev& bd = st.br[it.branch];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int nch = bd.nchunks;
  const int64_t n = st.n;
  const int fbeg = it.frag_begin, fend = it.frag_end, flast = fend - 1;
  const int ntiles = (fend - fbeg + T - 1) / T;

  for (int t = threadIdx.x; t < BANN_MAXL * 20; t += blockDim.x) {
    const int l = t / 20, r = t - l * 20;
    float v = 0.f;
    if (l >= 1 && l < NL) {
      if (r < 16) {
        const int j = r >> 2, k = r & 3;
        if (j < bd.win[l] && k < bd.widths[l]) v = st.theta[bd.p_off + bd.woff[l] + k * bd.win[l] + j];
        s_hd.W[l][j][k] = v;
      } else {
        const int k = r - 16;
        if (l < NL - 1 && k < bd.widths[l]) v = st.theta[bd.p_off + bd.boff[l] + k];
        s_hd.bias[l][k] = v;
      }
    } else if (l == 0 && r >= 16) {
      const int k = r - 16;
      s_hd.bias[0][k] = (k < bd.widths[0]) ? st.fc[it.branch].c0[k] : 0.f;
    }
  }
  __syncthreads();

  float* part = st.part + bd.part_off + (int64_t)it.split * bd.P;

  if (wave == 0) {
    // ===================== head wave =====================
    const float* ybr = st.y + bd.y_off;
    float* predb = st.pred + bd.y_off;
    auto load_y = [&](int t) -> float {
      const int64_t row = (int64_t)min(fbeg + t * T + (lane >> 4), flast) * 16 + (lane & 15);
      return ybr[row < n ? row : n - 1];
    };
    double rss = 0.0;
    float db[NH][4], dWo[4];
    float dW[NL > 2 ? NL - 2 : 1][4][4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      dWo[k] = 0.f;
#pragma unroll
      for (int l = 0; l < NH; ++l) db[l][k] = 0.f;
#pragma unroll
      for (int l = 0; l < (NL > 2 ? NL - 2 : 1); ++l)
#pragma unroll
        for (int j = 0; j < 4; ++j) dW[l][j][k] = 0.f;
    }
    auto head_tile = [&](int t, float yv) {
      const int q = lane >> 4, rr = lane & 15;
      const int f = fbeg + t * T + q;
      const int64_t row = (int64_t)f * 16 + rr;
      const bool valid = (f < fend) && (row < n);
      const int zb = t & 1;
      float d[4];
#if BANN_ABLATE & 1
      {
        const v4f p0 = *reinterpret_cast<const v4f*>(&s_zp[zb][0][q][rr][0]);
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] = valid ? p0[k] * 1e-3f - yv : 0.f;
      }
#else
      float z[NH][4], a[NH][4];
      v4f zs = *reinterpret_cast<const v4f*>(&s_hd.bias[0][0]);
#pragma unroll
      for (int w = 0; w < NW; ++w) zs += *reinterpret_cast<const v4f*>(&s_zp[zb][w][q][rr][0]);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        z[0][k] = zs[k];
        a[0][k] = act_h_t<ACT>(z[0][k]);
      }
#pragma unroll
      for (int l = 1; l < NH; ++l) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float sacc = s_hd.bias[l][k];
#pragma unroll
          for (int j = 0; j < 4; ++j) sacc = fmaf(a[l - 1][j], s_hd.W[l][j][k], sacc);
          z[l][k] = sacc;
          a[l][k] = act_h_t<ACT>(sacc);
        }
      }
      float out = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) out = fmaf(a[NH - 1][j], s_hd.W[NL - 1][j][0], out);
      const float e = valid ? out - yv : 0.f;
      if (write_pred && valid) predb[row] = out;
      rss += (double)e * (double)e;
      float err[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dWo[j] = fmaf(a[NH - 1][j], e, dWo[j]);
        err[j] = e * s_hd.W[NL - 1][j][0];
      }
#pragma unroll
      for (int l = NH - 1; l >= 0; --l) {
        float dl[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          dl[k] = act_dh_t<ACT>(z[l][k], a[l][k]) * err[k];
          db[l][k] += dl[k];
        }
        if (l >= 1) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float sj = 0.f;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              dW[l - 1][j][k] = fmaf(a[l - 1][j], dl[k], dW[l - 1][j][k]);
              sj = fmaf(dl[k], s_hd.W[l][j][k], sj);
            }
            err[j] = sj;
          }
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) d[k] = dl[k];
        }
      }
#endif
      // delta0 -> per-column power-of-two scale + 4 digits (see k_fused_grad_mx)
      const uint32_t e01 = wave_max_u16x2(((fbits(d[0]) >> 23) & 0xFFu) | (((fbits(d[1]) >> 23) & 0xFFu) << 16));
      const uint32_t e23 = wave_max_u16x2(((fbits(d[2]) >> 23) & 0xFFu) | (((fbits(d[3]) >> 23) & 0xFFu) << 16));
      const uint32_t E[4] = {e01 & 0xFFFFu, e01 >> 16, e23 & 0xFFFFu, e23 >> 16};
      v4i w;
      v4f scl;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool ok = E[k] >= 6u;
        const float inv = ok ? fpow2(259u - E[k]) : 0.f;
        scl[k] = ok ? fpow2(E[k] - 5u) : 0.f;
        w[k] = (int)digits4(d[k] * inv);
      }
      *reinterpret_cast<v4i*>(&s_dig[zb][q * DROW + rr * 16]) = w;
      if (lane == 0) *reinterpret_cast<v4f*>(&s_scl[zb][0]) = scl;
    };
    float ya = load_y(0), yb = 0.f;
    for (int t = 0;; t += 2) {
      if (t < ntiles) yb = load_y(t + 1);
      LDS_BARRIER();
      if (t == ntiles) break;
      head_tile(t, ya);
      if (t + 1 < ntiles) ya = load_y(t + 2);
      LDS_BARRIER();
      if (t + 1 == ntiles) break;
      head_tile(t + 1, yb);
    }
    const double rs = wave_sum_d(rss);
    float db0s[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) db0s[k] = wave_sum(db[0][k]);
    if (lane == 0) {
      st.rss_part[(int64_t)it.branch * st.max_splits + it.split] = rs;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s_db0[k] = db0s[k];
        if (k < bd.widths[0]) part[bd.boff[0] + k] = db0s[k];
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float v = wave_sum(dWo[j]);
      if (lane == 0 && j < bd.win[NL - 1]) part[bd.woff[NL - 1] + j] = v;
    }
#pragma unroll
    for (int l = 1; l < NH; ++l) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float v = wave_sum(db[l][k]);
        if (lane == 0 && k < bd.widths[l]) part[bd.boff[l] + k] = v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float wv = wave_sum(dW[l - 1][j][k]);
          if (lane == 0 && j < bd.win[l] && k < bd.widths[l]) part[bd.woff[l] + k * bd.win[l] + j] = wv;
        }
      }
    }
    __syncthreads();  // s_db0 visible to the chunk waves
  } else {
    // ===================== chunk waves =====================
    const int cw = wave - 1;
    const bool has_chunk = cw < nch;
    const int mych = has_chunk ? cw : nch - 1;
    const float scale = has_chunk ? st.fc[it.branch].scale[lane >> 4] : 0.f;  // chunk-less: zp = 0
    const v4i adig = *reinterpret_cast<const v4i*>(st.dig + bd.dig_off + ((int64_t)mych * 64 + lane) * 16);
    // genotype sources (branch-free clamped loads: past the item end re-read its last tile)
    const int tb0 = fbeg / T, tlast = flast / T;
    const v4i* xu2 = reinterpret_cast<const v4i*>(st.xu2 + bd.x_off) + (int64_t)mych * 64 + lane;
    const int8_t* xi8 = st.xpk + bd.x_off + ((int64_t)mych * 64 + lane) * 16;
    const int64_t frag_bytes = (int64_t)nch * 1024;
    typedef v4i XReg[U2 ? 1 : T];
    auto load_tile = [&](int t, XReg& xv) {
#if BANN_ABLATE & 8
      // compute-only profiling build: no genotype traffic
#pragma unroll
      for (int q = 0; q < (U2 ? 1 : T); ++q) xv[q] = v4i{t, lane, q, 0x01010101};
      return;
#endif
      if constexpr (U2) {
        xv[0] = xu2[(int64_t)min(tb0 + t, tlast) * nch * 64];
      } else {
#pragma unroll
        for (int q = 0; q < T; ++q)
          xv[q] = *reinterpret_cast<const v4i*>(xi8 + (int64_t)min(fbeg + t * T + q, flast) * frag_bytes);
      }
    };
    auto unpack = [&](const XReg& xv, v4i (&xu)[T]) {
      if constexpr (U2) {
#pragma unroll
        for (int q = 0; q < T; ++q) {
          const uint32_t wq = (uint32_t)xv[0][q];
          xu[q] = v4i{(int)(wq & 0x03030303u), (int)((wq >> 2) & 0x03030303u), (int)((wq >> 4) & 0x03030303u),
                      (int)((wq >> 6) & 0x03030303u)};
        }
      } else {
#pragma unroll
        for (int q = 0; q < T; ++q) xu[q] = xv[q];
      }
    };
    char* img = s_img[cw];
    const int g = lane >> 4, tq = (lane & 15) >> 1, tp = lane & 1;
    const int rot = 8 * (g & 1);
    float dw[4] = {0.f, 0.f, 0.f, 0.f};  // dW0 (G^T delta0) of column lane>>4, marker 16u + (lane & 15)

    auto fwd = [&](int t, const v4i (&xu)[T]) {
#pragma unroll
      for (int q = 0; q < T; ++q) {
#if BANN_ABLATE & 4
        const v4i d = xu[q];
#else
        const v4i d = __builtin_amdgcn_mfma_i32_16x16x64_i8(adig, xu[q], v4i{0, 0, 0, 0}, 0, 0, 0);
#endif
        s_zp[t & 1][cw][q][lane & 15][lane >> 4] =
            scale * ((float)d[0] + (float)d[1] * 0x1p-7f + (float)d[2] * 0x1p-14f + (float)d[3] * 0x1p-21f);
      }
    };
    auto bwd = [&](int tb) {
      const char* ds = &s_dig[tb & 1][0] + g * DROW + tq * 16 + 8 * tp;
      const v4i A = lds_tr8_pair(ds, ds + 8 * 16);
      const float sc_c = s_scl[tb & 1][g];
      const char* xs = img + g * 1024 + 8 * tp;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r0 = (16 * u + tq + rot) & 63, r1 = (16 * u + 8 + tq + rot) & 63;
        const v4i B = lds_tr8_pair(xs + r0 * 16, xs + r1 * 16);
#if BANN_ABLATE & 2
        asm volatile("" ::"v"(A), "v"(B));
#else
        const v4i gacc = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B, v4i{0, 0, 0, 0}, 0, 0, 0);
        const float v =
            (float)gacc[0] + (float)gacc[1] * 0x1p-7f + (float)gacc[2] * 0x1p-14f + (float)gacc[3] * 0x1p-21f;
        dw[u] = fmaf(sc_c, v, dw[u]);
#endif
      }
    };
    auto write_img = [&](const v4i (&xu)[T]) {
#pragma unroll
      for (int q = 0; q < T; ++q)
        *reinterpret_cast<v4i*>(img + q * 1024 + ((lane + 8 * (q & 1)) & 63) * 16) = xu[q];
    };

    XReg xa, xb;
    load_tile(0, xa);
    for (int t = 0;; t += 2) {
      v4i xu[T];
      if (t < ntiles) {
        load_tile(t + 1, xb);
        unpack(xa, xu);
        fwd(t, xu);
      }
      LDS_BARRIER();
      if (t >= 1 && has_chunk) bwd(t - 1);
      if (t == ntiles) break;
      write_img(xu);

      v4i xv[T];
      if (t + 1 < ntiles) {
        load_tile(t + 2, xa);
        unpack(xb, xv);
        fwd(t + 1, xv);
      }
      LDS_BARRIER();
      if (has_chunk) bwd(t);
      if (t + 1 == ntiles) break;
      write_img(xv);
    }
    __syncthreads();  // s_db0 published by the head wave
    if (has_chunk) {
      const int c = lane >> 4;
      if (c < bd.widths[0]) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int sidx = cw * 64 + u * 16 + (lane & 15);
          if (sidx < bd.m) {
            const float mu = st.mu[bd.mk_off + sidx], sg = st.sigma[bd.mk_off + sidx];
            part[bd.woff[0] + c * bd.m + sidx] = sg > 0.f ? (dw[u] - mu * s_db0[c]) / sg : 0.f;
          }
        }
      }
    }
  }
}

// BANN_FUSED_VARIANT: "fx" (default: wave-per-tile, int32 accumulation over
// chunks and tiles, kernels_fx.hip), "rx" (register-staged, MFMA backward,
// 2 WG/CU), "mx" (LDS-DMA ring, MFMA backward), "pipe" (LDS-DMA ring, VALU
// backward) or "reg" (register-staged lockstep, VALU backward).
// BANN_GENO_FORMAT = "u2" (default for fx / rx: 2-bit genotype codes in HBM) or "i8".
static int fused_variant() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("BANN_FUSED_VARIANT");
    if (!e || !e[0] || (e[0] == 'f' && e[1] == 'x')) v = 5;
    else if (e[0] == 'r' && e[1] == 'x') v = 4;
    else if (e[0] == 'm') v = 3;
    else if (e[0] == 'p') v = 2;
    else v = 0;
  }
  return v;
}

int fused_prefers_u2() {
  static int u = -1;
  if (u < 0) {
    const char* e = getenv("BANN_GENO_FORMAT");
    u = (fused_variant() >= 4 && !(e && e[0] == 'i')) ? 1 : 0;
  }
  return u;
}

int fused_u2_layout() { return fused_variant() == 5 ? 1 : 0; }

const char* fused_kernel_family() {
  switch (fused_variant()) {
    case 5: return "k_fused_grad_fx";
    case 4: return "k_fused_grad_rx";
    case 3: return "k_fused_grad_mx";
    case 2: return "k_fused_grad_pipe";
    default: return "k_fused_grad";
  }
}

template <int NL, int ACT>
static void launch_fused_t(const DevState& st, const GradItem* items, int32_t nitems, int32_t nwaves, int wp,
                           hipStream_t s) {
  if (fused_variant() == 4 && nwaves <= 8) {
    if (st.u2)
      hipLaunchKernelGGL((k_fused_grad_rx<NL, ACT, true>), dim3(nitems), dim3(64 * 9), 0, s, st, items, wp);
    else
      hipLaunchKernelGGL((k_fused_grad_rx<NL, ACT, false>), dim3(nitems), dim3(64 * 9), 0, s, st, items, wp);
    return;
  }
  if (fused_variant() == 3 && nwaves <= 8) {
    hipLaunchKernelGGL((k_fused_grad_mx<NL, 8, ACT>), dim3(nitems), dim3(64 * 9), 0, s, st, items, wp);
    return;
  }
  if (fused_variant() == 2 && nwaves <= 8) {  // > 8 chunks: the LDS ring would not fit; use the reg kernel
    hipLaunchKernelGGL((k_fused_grad_pipe<NL, 8, ACT, 3>), dim3(nitems), dim3(64 * 9), 0, s, st, items, wp);
    return;
  }
  if (nwaves <= 8)
    hipLaunchKernelGGL((k_fused_grad<NL, 8, ACT>), dim3(nitems), dim3(64 * nwaves), 0, s, st, items, wp);
  else
    hipLaunchKernelGGL((k_fused_grad<NL, 16, ACT>), dim3(nitems), dim3(64 * nwaves), 0, s, st, items, wp);
}

template <int NL>
static void launch_fused_nl(const DevState& st, const GradItem* items, int32_t nitems, int32_t nwaves, int act,
                            int wp, hipStream_t s) {
  switch (act) {
    case 0: launch_fused_t<NL, 0>(st, items, nitems, nwaves, wp, s); break;
    case 1: launch_fused_t<NL, 1>(st, items, nitems, nwaves, wp, s); break;
    case 2: launch_fused_t<NL, 2>(st, items, nitems, nwaves, wp, s); break;
    case 3: launch_fused_t<NL, 3>(st, items, nitems, nwaves, wp, s); break;
    default: launch_fused_t<NL, 4>(st, items, nitems, nwaves, wp, s); break;
  }
}

void launch_fused_grad(const DevState& st, const GradItem* items, int32_t nitems, int32_t nwaves, int32_t L,
                       int32_t act, int full8, int write_pred, hipStream_t s) {
  if (nitems <= 0) return;
  if (fused_variant() == 5 && st.u2 && nwaves <= 8) {
    launch_fused_grad_fx(st, items, nitems, L, act, full8, write_pred, s);
    return;
  }
  switch (L) {
    case 2: launch_fused_nl<2>(st, items, nitems, nwaves, act, write_pred, s); break;
    case 3: launch_fused_nl<3>(st, items, nitems, nwaves, act, write_pred, s); break;
    case 4: launch_fused_nl<4>(st, items, nitems, nwaves, act, write_pred, s); break;
    default: break;
  }
}
