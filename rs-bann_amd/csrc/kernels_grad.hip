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
#include "bann_internal.h"

typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));

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

template <int NL, int NWMAX>
__global__ void __launch_bounds__(64 * NWMAX) k_fused_grad(DevState st, const GradItem* __restrict__ items,
                                                           int write_pred) {
  constexpr int NH = NL - 1;  // layers with activations (0 .. L-2)
  __shared__ float s_zp[NWMAX][BANN_TILE_FRAGS][16][4];  // per-chunk partial Z0
  __shared__ v4f s_delta[BANN_TILE_FRAGS][16];           // delta0 of the tile
  __shared__ HeadLds s_hd;
  __shared__ float s_db0[4];

  const GradItem it = items[blockIdx.x];
  const BranchDev& bd = st.br[it.branch];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nch = bd.nchunks;
  const bool has_chunk = wave < nch;
  const int act = bd.act;
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
  float scale = 0.f;
  v4i adig = {0, 0, 0, 0};
  if (has_chunk) {
    scale = st.fc[it.branch].scale[lane >> 4];
    adig = *reinterpret_cast<const v4i*>(st.dig + bd.dig_off + ((int64_t)wave * 64 + lane) * 16);
  }
  __syncthreads();

  const int8_t* xb = st.xpk + bd.x_off;
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

  auto load_tile = [&](int f0, v4i (&xv)[BANN_TILE_FRAGS]) {
#pragma unroll
    for (int q = 0; q < BANN_TILE_FRAGS; ++q) {
      const int f = f0 + q;
      if (has_chunk && f < it.frag_end)
        xv[q] = *reinterpret_cast<const v4i*>(xb + (((int64_t)f * nch + wave) * 64 + lane) * 16);
      else
        xv[q] = v4i{0, 0, 0, 0};
    }
  };

  v4i xcur[BANN_TILE_FRAGS], xnext[BANN_TILE_FRAGS];
  load_tile(it.frag_begin, xcur);
  for (int f0 = it.frag_begin; f0 < it.frag_end; f0 += BANN_TILE_FRAGS) {
    if (f0 + BANN_TILE_FRAGS < it.frag_end) load_tile(f0 + BANN_TILE_FRAGS, xnext);

    // ---- forward, masked first layer on MFMA: partial Z0 of this chunk ----
    if (has_chunk) {
#pragma unroll
      for (int q = 0; q < BANN_TILE_FRAGS; ++q) {
        v4i d = __builtin_amdgcn_mfma_i32_16x16x64_i8(adig, xcur[q], v4i{0, 0, 0, 0}, 0, 0, 0);
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
      const bool valid = (f < it.frag_end) && (row < n);
      float z[NH][4], a[NH][4];
#pragma unroll
      for (int k = 0; k < 4; ++k) z[0][k] = s_hd.bias[0][k];
      for (int w = 0; w < nch; ++w) {
        const v4f p = *reinterpret_cast<const v4f*>(&s_zp[w][q][rr][0]);
#pragma unroll
        for (int k = 0; k < 4; ++k) z[0][k] += p[k];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) a[0][k] = act_h(z[0][k], act);
#pragma unroll
      for (int l = 1; l < NH; ++l) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float s = s_hd.bias[l][k];
#pragma unroll
          for (int j = 0; j < 4; ++j) s = fmaf(a[l - 1][j], s_hd.W[l][j][k], s);
          z[l][k] = s;
          a[l][k] = act_h(s, act);
        }
      }
      float out = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) out = fmaf(a[NH - 1][j], s_hd.W[NL - 1][j][0], out);
      const float e = valid ? out - st.y[bd.y_off + row] : 0.f;
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
          d[k] = act_dh(z[l][k], a[l][k], act) * err[k];
          db[l][k] += d[k];
        }
        if (l >= 1) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float s = 0.f;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              dW[l - 1][j][k] = fmaf(a[l - 1][j], d[k], dW[l - 1][j][k]);
              s = fmaf(d[k], s_hd.W[l][j][k], s);
            }
            err[j] = s;
          }
        } else {
          s_delta[q][rr] = v4f{d[0], d[1], d[2], d[3]};
        }
      }
    }
    __syncthreads();

    // ---- backward, masked first layer on VALU: acc[j][k] += x_j * delta0_k ----
    if (has_chunk) {
#pragma unroll
      for (int q = 0; q < BANN_TILE_FRAGS; ++q) {
        const v4f dl = s_delta[q][lane & 15];
#pragma unroll
        for (int w4 = 0; w4 < 4; ++w4) {
          const uint32_t word = (uint32_t)xcur[q][w4];
#pragma unroll
          for (int bq = 0; bq < 4; ++bq) {
            const float x = (float)((word >> (8 * bq)) & 0xFFu);
#pragma unroll
            for (int k = 0; k < 4; ++k) acc[w4 * 4 + bq][k] = fmaf(x, dl[k], acc[w4 * 4 + bq][k]);
          }
        }
      }
    }
#pragma unroll
    for (int q = 0; q < BANN_TILE_FRAGS; ++q) xcur[q] = xnext[q];
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
    const int s = wave * 64 + (lane >> 4) * 16 + rr;
    if (s < bd.m) {
      const float mu = st.mu[bd.mk_off + s], sg = st.sigma[bd.mk_off + s];
      const int w0 = bd.widths[0];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (k < w0) part[bd.woff[0] + k * bd.m + s] = sg > 0.f ? (mine[k] - mu * s_db0[k]) / sg : 0.f;
    }
  }
}

template <int NL>
static void launch_fused_nl(const DevState& st, const GradItem* items, int32_t nitems, int32_t nwaves, int wp,
                            hipStream_t s) {
  if (nwaves <= 8)
    hipLaunchKernelGGL((k_fused_grad<NL, 8>), dim3(nitems), dim3(64 * nwaves), 0, s, st, items, wp);
  else
    hipLaunchKernelGGL((k_fused_grad<NL, 16>), dim3(nitems), dim3(64 * nwaves), 0, s, st, items, wp);
}

void launch_fused_grad(const DevState& st, const GradItem* items, int32_t nitems, int32_t nwaves, int32_t L,
                       int write_pred, hipStream_t s) {
  if (nitems <= 0) return;
  switch (L) {
    case 2: launch_fused_nl<2>(st, items, nitems, nwaves, write_pred, s); break;
    case 3: launch_fused_nl<3>(st, items, nitems, nwaves, write_pred, s); break;
    case 4: launch_fused_nl<4>(st, items, nitems, nwaves, write_pred, s); break;
    default: break;
  }
}
