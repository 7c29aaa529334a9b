// kernels_gx.hip — "gx": the layered gradient path for every branch shape the
// fused single-pass kernels do not take (fx/fxl: every width <= 4; wx: one hidden
// layer <= 32 x 32 over <= 128 markers): any depth, any widths, any marker count
// -- among them the reference's default architecture, hidden and summary widths
// m_b / 2 (cli.rs:365-375, rs-bann.rs:433-435).
//
// BranchSampler::backpropagate (branch_sampler.rs:813-875) with forward_feed
// (743-782) as a chain of batched GEMMs over the branches of one scratch group.
// Every GEMM runs on the f32 MFMA (v_mfma_f32_16x16x4_f32: f32 products, 64
// flop/clk/SIMD, the f32 peak), accumulating in f32 inside 64-deep K blocks and
// in f64 across them, so long reductions (m markers, n individuals) do not grow
// the f32 error with K:
//   PREP    Wp_l = W_l as [out][in] rows padded to 4; Wp_0 = W0 / sigma and
//           c0 = b0 - sum_j mu_j Wp_0[.][j] (f64): standardisation folded into W0
//   FWD0    Z0 = G Wp_0^T + c0 (G decoded from the 2-bit tile image)   -> A0 = h(Z0), H0 = h'(Z0)
//   FWD l   Z_l = A_{l-1} Wp_l^T + b_l                                  -> A_l, H_l
//           (H_l = h'(Z_l) is stored for SiLU only: for tanh, ReLU, leaky ReLU and
//           identity h' is a function of A_l, formed where it is used)
//   HEAD    out = A_s w_out (775-782), e = out - y, rss (823-828), pred,
//           dW_out = A_s^T e (830-835), delta_s = H_s * e w_out (844-847, in place over H_s)
//   BWD l   delta_{l-1} = H_{l-1} * (delta_l Wp_l)          (855-861, in place over H_{l-1})
//   GRAD l  dW_l = A_{l-1}^T delta_l, db_l = 1^T delta_l    (849-852; K = individuals, row splits)
//   GRAD0   dW0 = (G^T delta0 - mu (1^T delta0)) / sigma, db0 (863-866)
// Every workgroup computes a 64 x 64 output tile with 4 waves (32 x 32 each, four
// 16 x 16 accumulators); operands are staged through registers into a
// double-buffered LDS image [row][k] with 68-float rows (the MFMA's one-float A/B
// reads -- lane (i, q) at row i, k = 4 s + q -- hit 64 distinct banks).  Tiles are
// numbered so that consecutive ones share an operand block (the row block of a
// forward, the row range of a gradient split) and are mapped to ONE XCD, so the
// shared block is read from HBM once into that XCD's L2.
//
// Scratch (per branch, f32, offsets in BranchDev::gx_*): Wp_l, bias_l, A_l and
// H_l of [rows][ld_l] for every hidden/summary layer, the head's per-tile f64
// partials, rows = 64 * ntile (rows >= n
// carry zero genotypes; their error is 0, so they add nothing to any gradient).
// Gradients go to the branch's partial slabs part[split][P] (reduced in a fixed
// order by k_update), the rss to rss_part: bitwise reproducible.
#include <stdlib.h>

#include <type_traits>

#include "activations.h"
#include "bann_internal.h"
#include "kernel_util.h"

#ifndef GX_ABL
#define GX_ABL 0
#endif
#define GX_T 64                // output tile edge, K block depth
#define GX_PREP_Y 16           // k_gx_prep workgroups per branch
#define GX_LD 68               // LDS row stride (floats)
#define GX_LDS (GX_T * GX_LD)  // floats per operand block
#ifndef GX_NBUF
#define GX_NBUF 1              // LDS stages: 1 = 35 KiB per workgroup (4 per CU), 2 = double-buffered (2 per CU)
#endif

namespace {

__device__ __forceinline__ int64_t gx_rows(const DevState& st) { return (int64_t)((st.nfrag + 3) / 4) * 64; }
__device__ __forceinline__ float* gx_base(const DevState& st, const BranchDev& bd) { return st.scr + bd.scr_off; }

// the tile numbering of a phase for one branch (must match gx_tiles on the host)
// (tile edges TM x TN: 64 x 64, the hidden FWD / BWD of k_gx_gemm_x3 128 x 128)
__device__ __forceinline__ void gx_dims(const DevState& st, const BranchDev& bd, int ph, int l, int& tmc, int& tnc,
                                        int& ns, int TM = 64, int TN = 64) {
  const int ntile = (st.nfrag + 3) / 4;
  const int rt = (ntile * 64 + TM - 1) / TM;
  ns = 1;
  if (ph == GX_FWD0) {
    tmc = ntile;
    tnc = (bd.widths[0] + 63) / 64;
  } else if (ph == GX_FWD) {
    tmc = rt;
    tnc = (bd.widths[l] + TN - 1) / TN;
  } else if (ph == GX_BWD) {
    tmc = rt;
    tnc = (bd.widths[l - 1] + TN - 1) / TN;
  } else if (ph == GX_GRAD) {
    tmc = (bd.widths[l - 1] + TM - 1) / TM;
    tnc = (bd.widths[l] + TN - 1) / TN;
    ns = bd.nsplits;
  } else {  // GX_GRAD0
    tmc = bd.nchunks;
    tnc = (bd.widths[0] + 63) / 64;
    ns = bd.nsplits;
  }
}

// a 64 x 64 block of a row-major f32 matrix M[r][c] (row stride ld, a multiple of
// 4): element (r, c) of the block = M[r0 + r][c0 + c] when r0 + r < rmax and
// c0 + c < cmax, else 0.  Thread t holds rows (t + 256 u) >> 4, columns 4 (t & 15).
// The loads are only issued here; the edge masking waits until blk_fix, after the
// K block's MFMAs (masking right after the load would make the compiler wait for
// the data there and expose the full memory latency every block).  blk_fix
// recomputes the bounds instead of keeping them in registers.
struct Blk {
  v4f v[4];
};
struct BlkBounds {
  int64_t r0, rmax;
  int c0, cmax;
};
__device__ __forceinline__ int blk_nv(const BlkBounds& k, int u) {
  const int e = threadIdx.x + 256 * u;
  const int64_t r = k.r0 + (e >> 4);
  const int c = k.c0 + 4 * (e & 15);
  return r < k.rmax ? min(max(k.cmax - c, 0), 4) : 0;
}
__device__ __forceinline__ void blk_load(Blk& s, const float* __restrict__ M, int64_t ld, const BlkBounds& k) {
  const int t = threadIdx.x;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = t + 256 * u;
    v4f x = {0.f, 0.f, 0.f, 0.f};
    if (blk_nv(k, u) > 0) x = *(const v4f*)(M + (k.r0 + (e >> 4)) * ld + k.c0 + 4 * (e & 15));  // rows padded to 4
    s.v[u] = x;
  }
}
__device__ __forceinline__ void blk_fix(Blk& s, const BlkBounds& k) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int nv = blk_nv(k, u);
    if (nv < 2) s.v[u].y = 0.f;
    if (nv < 3) s.v[u].z = 0.f;
    if (nv < 4) s.v[u].w = 0.f;
  }
}
// LDS [r][c] (the block's rows are the MFMA rows, its columns the K index)
__device__ __forceinline__ void blk_store(Blk& s, const BlkBounds& k, float* L) {
  blk_fix(s, k);
  const int t = threadIdx.x;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = t + 256 * u;
    *(v4f*)(L + (e >> 4) * GX_LD + 4 * (e & 15)) = s.v[u];
  }
}
// LDS [c][r] (the block's columns are the MFMA rows, its rows the K index)
__device__ __forceinline__ void blk_store_t(Blk& s, const BlkBounds& k, float* L) {
  blk_fix(s, k);
  const int t = threadIdx.x;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = t + 256 * u;
    const int r = e >> 4, c = 4 * (e & 15);
    L[(c + 0) * GX_LD + r] = s.v[u].x;
    L[(c + 1) * GX_LD + r] = s.v[u].y;
    L[(c + 2) * GX_LD + r] = s.v[u].z;
    L[(c + 3) * GX_LD + r] = s.v[u].w;
  }
}

// one 1 KiB chunk image (64 marker rows x 64 individuals of one tile; u2t layout,
// kernels_fx.hip header): thread t holds the dword at byte 4 t -- physical row
// position pos = t >> 2, i.e. logical marker row 16 w + ((P - 8 (w & 1)) & 15)
// (w = pos >> 4, P = pos & 15), and individuals 16 dq .. 16 dq + 15 at bits 2 s,
// dq = (t & 3) ^ (P >= 8 ? 2 : 0) (the swapped 8-byte halves).
__device__ __forceinline__ uint32_t geno_load(const uint8_t* __restrict__ img) {
  return *(const uint32_t*)(img + 4 * threadIdx.x);
}
__device__ __forceinline__ void geno_pos(int& jl, int& dq) {
  const int t = threadIdx.x, pos = t >> 2, w = pos >> 4, P = pos & 15;
  jl = 16 * w + ((P - 8 * (w & 1)) & 15);
  dq = (t & 3) ^ ((P >> 3) << 1);
}
// LDS [individual][marker] (FWD0: individuals are the MFMA rows)
__device__ __forceinline__ void geno_store_im(uint32_t g, float* L) {
  int jl, dq;
  geno_pos(jl, dq);
#pragma unroll
  for (int s = 0; s < 16; ++s) L[(16 * dq + s) * GX_LD + jl] = (float)((g >> (2 * s)) & 3u);
}
// LDS [marker][individual] (GRAD0: markers are the MFMA rows)
__device__ __forceinline__ void geno_store_mi(uint32_t g, float* L) {
  int jl, dq;
  geno_pos(jl, dq);
  float* p = L + jl * GX_LD + 16 * dq;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t b = g >> (8 * q);
    *(v4f*)(p + 4 * q) = v4f{(float)(b & 3u), (float)((b >> 2) & 3u), (float)((b >> 4) & 3u), (float)((b >> 6) & 3u)};
  }
}

}  // namespace

// a lane of the same row of 16 (DPP control CTRL)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// h'(z) as a function of a = h(z) for the activations where it is one (tanh:
// 1 - a^2; ReLU / leaky ReLU: a > 0 <=> z > 0; identity): those layers store A_l
// only, and the backward phases form H_l from it (SiLU keeps H_l)
__device__ __forceinline__ bool dh_from_a(int act) { return act != 3; }
// the same without branches: h' = base(a) - tq a^2 with base = bp (a > 0), bn (a < 0),
// bz (a = 0) and the four constants of the activation (identical values)
struct DhA {
  float tq, bp, bn, bz;
};
__device__ __forceinline__ DhA dh_a_consts(int act) {
  switch (act) {
    case 0: return DhA{1.f, 1.f, 1.f, 1.f};
    case 1: return DhA{0.f, 1.f, 0.f, 0.f};
    case 2: return DhA{0.f, 1.f, 0.01f, 0.f};
    default: return DhA{0.f, 1.f, 1.f, 1.f};
  }
}
__device__ __forceinline__ float dh_a(float a, const DhA& k) {
  const float base = a > 0.f ? k.bp : (a < 0.f ? k.bn : k.bz);
  return k.tq != 0.f ? 1.f - a * a : base;
}
__device__ __forceinline__ float act_dh_a(float a, int act) {
  switch (act) {
    case 0: return 1.f - a * a;
    case 1: return a > 0.f ? 1.f : 0.f;
    case 2: return a > 0.f ? 1.f : (a < 0.f ? 0.01f : 0.f);
    default: return 1.f;
  }
}

// the epilogue of a TM x TN output tile (TM = 32 AX, TN = 32 AY; 64 x 64 unless
// k_gx_gemm_x3 says otherwise): lane holds rows ar + 16 X + 4 lq + y and columns
// bc + 16 Y + li of accumulator x = AY X + Y (f32 acc, or the f64 dacc when F64).
// FWD0 / FWD: A = h(Z + b), H = h'(Z + b); BWD: delta_{l-1} = H * acc in place;
// GRAD / GRAD0: the weight gradient into the split's partial slab (GRAD0 with the
// standardisation, column sums cs_col of delta0 in LDS) and, in the tm == 0 tiles,
// db from the column sum cs of thread t < TN.
// BWD: the h' operands of the lane's outputs (A_{l-1}, or H_{l-1} for SiLU), column
// and row clamped into the layer (the clamped ones are not used)
template <int AX, int AY>
__device__ __forceinline__ void gx_bwd_hload(const DevState& st, const BranchDev& bd, const float* S, int l, int tm,
                                             int tn, int wo, int ar, int bc, int li, int lq, float* hv) {
  constexpr int TM = 32 * AX, TN = 32 * AY;
  const int64_t rmax = gx_rows(st);
  const float* Hsrc = S + (dh_from_a(bd.act) ? bd.gx_a[l - 1] : bd.gx_h[l - 1]);
  const int64_t ld = bd.gx_ld[l - 1];
#pragma unroll
  for (int x = 0; x < AX * AY; ++x) {
    const int X = x / AY, Y = x % AY;
    const int jc = min(TN * tn + bc + 16 * Y + li, wo - 1);
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      const int64_t row = min(TM * (int64_t)tm + ar + 16 * X + 4 * lq + y, rmax - 1);
      hv[4 * x + y] = Hsrc[row * ld + jc];
    }
  }
}

template <int PH, bool F64, int AX = 2, int AY = 2>
__device__ __forceinline__ void gx_epilogue(const DevState& st, const BranchDev& bd, float* S, int l, int tm, int tn,
                                            int split, int wi, int wo, int ar, int bc, int li, int lq,
                                            const v4f (&acc)[AX * AY], const double (&dacc)[AX * AY][4], double cs,
                                            const double* cs_col, bool lazy = false, double cs2 = 0.0,
                                            const float* pre = nullptr) {
  constexpr int TM = 32 * AX, TN = 32 * AY;
  const int t = threadIdx.x;
  const int64_t rmax = gx_rows(st);  // FWD / BWD: rows past the last tile (TM = 128) are not written
  if constexpr (PH == GX_FWD0 || PH == GX_FWD) {
    const int lay = PH == GX_FWD0 ? 0 : l;
    const float* bias = S + bd.gx_b[lay];
    float* Ao = S + bd.gx_a[lay];
    float* Ho = S + bd.gx_h[lay];
    const int64_t ld = bd.gx_ld[lay];
    // the summary layer (lazy head, k_gx_head): the wave's partial of out = A_s w_out
    // over its TN / 2 columns, per row
    const bool head = PH == GX_FWD && l == bd.L - 2 && dh_from_a(bd.act);
    const float* wout = S + bd.gx_w[bd.L - 1];
    float po[AX][4];
#pragma unroll
    for (int X = 0; X < AX; ++X) po[X][0] = po[X][1] = po[X][2] = po[X][3] = 0.f;
    // the lane's columns' bias and w_out (pre: loaded by the caller before its K loop)
    float bq[AY], wq[AY];
#pragma unroll
    for (int Y = 0; Y < AY; ++Y) {
      const int j = TN * tn + bc + 16 * Y + li;
      bq[Y] = pre ? pre[Y] : (j < wo ? bias[j] : 0.f);
      wq[Y] = pre ? pre[AY + Y] : (head && j < wo ? wout[j] : 0.f);
    }
    // the activation as a compile-time kind (activations.h)
    auto out = [&](auto kind) {
      constexpr int ACT = decltype(kind)::value;
#pragma unroll
      for (int x = 0; x < AX * AY; ++x) {
        const int X = x / AY, Y = x % AY;
        const int j = TN * tn + bc + 16 * Y + li;
        if (j >= wo) continue;
        const float bj = bq[Y];
        const float wj = wq[Y];
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          const int64_t row = TM * (int64_t)tm + ar + 16 * X + 4 * lq + y;
          if (TM > 64 && row >= rmax) continue;
          const float z = (F64 ? (float)dacc[x][y] : acc[x][y]) + bj;  // mid_layer_pre_activation: matmul + bias
          const float a = ACT == 0 ? fast_tanh(z) : act_h_t<ACT>(z);  // tanh to ~2 ulp (layer outputs feed GEMMs)
          Ao[row * ld + j] = a;
          if constexpr (ACT == 3) Ho[row * ld + j] = act_dh_t<ACT>(z, a);
          po[X][y] += a * wj;  // columns 16 Y + li, Y in order
        }
      }
    };
    switch (bd.act) {
      case 0: out(std::integral_constant<int, 0>{}); break;
      case 1: out(std::integral_constant<int, 1>{}); break;
      case 2: out(std::integral_constant<int, 2>{}); break;
      case 3: out(std::integral_constant<int, 3>{}); break;
      default: out(std::integral_constant<int, 4>{}); break;
    }
    if (head) {  // fixed butterfly over the 16 column lanes; lane li = 0 writes slot 2 tn + (column half)
      float* op = S + bd.gx_op + (int64_t)(2 * tn + (bc != 0 ? 1 : 0)) * rmax;
#pragma unroll
      for (int X = 0; X < AX; ++X)
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          float v = po[X][y];
          v += dpp_f<0xB1>(v);   // quad_perm [1, 0, 3, 2]
          v += dpp_f<0x4E>(v);   // quad_perm [2, 3, 0, 1]
          v += dpp_f<0x141>(v);  // row_half_mirror
          v += dpp_f<0x140>(v);  // row_mirror: every lane of the 16 holds the same sum
          const int64_t row = TM * (int64_t)tm + ar + 16 * X + 4 * lq + y;
          if (li == 0 && (TM == 64 || row < rmax)) op[row] = v;
        }
    }
  } else if constexpr (PH == GX_BWD) {
    float* Hd = S + bd.gx_h[l - 1];
    const float* Ad = S + bd.gx_a[l - 1];
    const int64_t ld = bd.gx_ld[l - 1];
    const int act = bd.act;
    const bool fa = dh_from_a(act);
    // every h' operand is loaded first, unconditionally (gx_bwd_hload), so the loads
    // issue back to back: one memory latency per tile instead of one per guarded
    // group (BWD1 at c3def: 3.2 -> 2.9 ms per group).  Measured and not kept: the
    // same loads issued during the last K block's MFMAs (3.27 ms)
    float hv[AX * AY][4];
    gx_bwd_hload<AX, AY>(st, bd, S, l, tm, tn, wo, ar, bc, li, lq, &hv[0][0]);
#pragma unroll
    for (int x = 0; x < AX * AY; ++x) {
      const int X = x / AY, Y = x % AY;
      const int j = TN * tn + bc + 16 * Y + li;
      if (j >= wo) continue;
#pragma unroll
      for (int y = 0; y < 4; ++y) {
        const int64_t row = TM * (int64_t)tm + ar + 16 * X + 4 * lq + y;
        if (TM > 64 && row >= rmax) continue;
        const float h = fa ? act_dh_a(hv[x][y], act) : hv[x][y];
        // delta = h'(z) * (delta_next W^T); lazy head: the accumulator lacks e of the row
        Hd[row * ld + j] = h * (lazy ? pre[4 * X + y] * acc[x][y] : acc[x][y]);
      }
    }
  } else {
    float* part = st.part + bd.part_off + (int64_t)split * bd.P;
    const int lay = PH == GX_GRAD ? l : 0;
    const int win = bd.win[lay];
    // GRAD0: sigma and mu of the lane's 4 AX markers, loaded together (index clamped)
    float sgv[AX][4], muv[AX][4];
    if constexpr (PH == GX_GRAD0) {
#pragma unroll
      for (int X = 0; X < AX; ++X)
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          const int ic = min(TM * tm + ar + 16 * X + 4 * lq + y, wi - 1);
          sgv[X][y] = st.sigma[bd.mk_off + ic];
          muv[X][y] = st.mu[bd.mk_off + ic];
        }
    }
#pragma unroll
    for (int x = 0; x < AX * AY; ++x) {
      const int X = x / AY, Y = x % AY;
      const int j = TN * tn + bc + 16 * Y + li;
      if (j >= wo) continue;
#pragma unroll
      for (int y = 0; y < 4; ++y) {
        const int i = TM * tm + ar + 16 * X + 4 * lq + y;
        if (i >= wi) continue;
        double v = dacc[x][y];
        if (PH == GX_GRAD && lazy) v *= (double)pre[Y];  // lazy head: times w_out of the column
        if constexpr (PH == GX_GRAD0) {  // X = (g - mu) / sigma; zero-variance markers contribute 0
          const float sg = sgv[X][y];
          v = sg > 0.f ? (v - (double)muv[X][y] * cs_col[bc + 16 * Y + li]) / (double)sg : 0.0;
        }
        part[bd.woff[lay] + (int64_t)j * win + i] = (float)v;  // param_vec: W_l[out j][in i]
      }
    }
    if (tm == 0 && t < TN && TN * tn + t < wo) {
      part[bd.boff[lay] + TN * tn + t] = (float)cs;                // db_l
      if (lazy) part[bd.woff[bd.L - 1] + TN * tn + t] = (float)cs2;  // dW_out = A_s^T e (lazy head)
    }
  }
}

// ---------------------------------------------------------------------------
// the GEMM phases
// ---------------------------------------------------------------------------
// GRAD (two staged operands + f64 accumulators) at 3 workgroups per CU: 4 would spill
template <int PH>
__global__ void __launch_bounds__(256, GX_NBUF == 1 ? (PH == GX_GRAD ? 3 : 4) : 2)
    k_gx_gemm(DevState st, const int32_t* __restrict__ blist, const int32_t* __restrict__ prefix, int nb, int l,
              int total, int per) {
  __shared__ float As[GX_NBUF][GX_LDS];
  __shared__ float Bs[GX_NBUF][GX_LDS];
  __shared__ double cs_s[GX_T];
  // XCD-aware numbering: workgroup i runs on XCD i % 8, so the logical tiles of
  // one XCD are the contiguous range [xcd * per, (xcd + 1) * per)
  const int q = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (q >= total) return;
  int lo = 0, hi = nb;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (prefix[mid] <= q) lo = mid;
    else hi = mid;
  }
  const int b = blist[lo];
  const BranchDev& bd = st.br[b];
  int tmc, tnc, ns;
  gx_dims(st, bd, PH, l, tmc, tnc, ns);
  int r = q - prefix[lo];
  const int split = r / (tmc * tnc);
  r -= split * tmc * tnc;
  const int tm = r / tnc, tn = r % tnc;
  const int64_t rows = gx_rows(st);
  float* S = gx_base(st, bd);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int ar = 32 * (wv >> 1), bc = 32 * (wv & 1);

  // K range (in blocks of 64) and the operands of this phase
  int kb0 = 0, kb1;
  int64_t kcount;  // valid K
  const float* Am = nullptr;
  const float* Bm = nullptr;
  int64_t lda = 0, ldb = 0;
  int wi = 0, wo = 0;  // GEMM output M / N extent (rows of the output are individuals for FWD/BWD)
  const uint8_t* img = st.xu2 + bd.x_off;
  const int64_t tstride = (int64_t)bd.nchunks * 1024;
  if constexpr (PH == GX_FWD0) {
    kcount = bd.m;
    kb1 = bd.nchunks;
    Bm = S + bd.gx_w[0];
    ldb = bd.gx_wld[0];
    wo = bd.widths[0];
  } else if constexpr (PH == GX_FWD) {
    kcount = bd.widths[l - 1];
    kb1 = (int)((kcount + 63) / 64);
    Am = S + bd.gx_a[l - 1];
    lda = bd.gx_ld[l - 1];
    Bm = S + bd.gx_w[l];
    ldb = bd.gx_wld[l];
    wo = bd.widths[l];
  } else if constexpr (PH == GX_BWD) {
    kcount = bd.widths[l];
    kb1 = (int)((kcount + 63) / 64);
    Am = S + bd.gx_h[l];  // delta_l
    lda = bd.gx_ld[l];
    Bm = S + bd.gx_w[l];  // Wp_l [k = out][j = in]: loaded transposed
    ldb = bd.gx_wld[l];
    wo = bd.widths[l - 1];
  } else {  // GRAD / GRAD0: K = the split's rows
    const int ntile = (st.nfrag + 3) / 4;
    kb0 = (int)((int64_t)ntile * split / ns);
    kb1 = (int)((int64_t)ntile * (split + 1) / ns);
    kcount = rows;
    if constexpr (PH == GX_GRAD) {
      Am = S + bd.gx_a[l - 1];
      lda = bd.gx_ld[l - 1];
      wi = bd.widths[l - 1];
      Bm = S + bd.gx_h[l];
      ldb = bd.gx_ld[l];
      wo = bd.widths[l];
    } else {
      wi = bd.m;
      Bm = S + bd.gx_h[0];
      ldb = bd.gx_ld[0];
      wo = bd.widths[0];
    }
  }
  const bool want_cs = (PH == GX_GRAD0) || (PH == GX_GRAD && tm == 0);

  // stage K block kb into registers
  Blk ra, rb;
  uint32_t rg = 0;
  // the operand blocks of K block kb
  auto bnd_a = [&](int kb) -> BlkBounds {
    if constexpr (PH == GX_GRAD) return BlkBounds{64 * (int64_t)kb, rows, 64 * tm, wi};
    return BlkBounds{64 * (int64_t)tm, rows, 64 * kb, (int)kcount};
  };
  auto bnd_b = [&](int kb) -> BlkBounds {
    if constexpr (PH == GX_FWD0 || PH == GX_FWD) return BlkBounds{64 * (int64_t)tn, wo, 64 * kb, (int)kcount};
    if constexpr (PH == GX_BWD) return BlkBounds{64 * (int64_t)kb, kcount, 64 * tn, wo};
    return BlkBounds{64 * (int64_t)kb, rows, 64 * tn, wo};
  };
  auto load = [&](int kb) {
    if constexpr (PH == GX_FWD0) rg = geno_load(img + (int64_t)tm * tstride + (int64_t)kb * 1024);
    if constexpr (PH == GX_GRAD0) rg = geno_load(img + (int64_t)kb * tstride + (int64_t)tm * 1024);
    if constexpr (PH == GX_FWD || PH == GX_BWD || PH == GX_GRAD) blk_load(ra, Am, lda, bnd_a(kb));
    blk_load(rb, Bm, ldb, bnd_b(kb));
  };
  auto store = [&](int buf, int kb) {
    if constexpr (PH == GX_FWD0) {
      geno_store_im(rg, As[buf]);
      blk_store(rb, bnd_b(kb), Bs[buf]);
    } else if constexpr (PH == GX_FWD) {
      blk_store(ra, bnd_a(kb), As[buf]);
      blk_store(rb, bnd_b(kb), Bs[buf]);
    } else if constexpr (PH == GX_BWD) {
      blk_store(ra, bnd_a(kb), As[buf]);
      blk_store_t(rb, bnd_b(kb), Bs[buf]);
    } else if constexpr (PH == GX_GRAD) {
      blk_store_t(ra, bnd_a(kb), As[buf]);
      blk_store_t(rb, bnd_b(kb), Bs[buf]);
    } else {
      geno_store_mi(rg, As[buf]);
      blk_store_t(rb, bnd_b(kb), Bs[buf]);
    }
  };

  v4f acc[4];
  double dacc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    acc[x] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int y = 0; y < 4; ++y) dacc[x][y] = 0.0;
  }
  // f64 accumulation across K blocks where K is long (m markers, n individuals);
  // the hidden-layer GEMMs (K = a layer width) keep the f32 MFMA chain
  constexpr bool F64 = PH != GX_FWD && PH != GX_BWD;
  double cs = 0.0;  // want_cs: column sum of the B block (delta) over the K range, thread t < 64 = column t
  if (kb0 < kb1) {
    load(kb0);
    store(0, kb0);
  }
  __syncthreads();
  for (int kb = kb0; kb < kb1; ++kb) {
    const int buf = GX_NBUF == 1 ? 0 : (kb - kb0) & 1;
    if (kb + 1 < kb1) load(kb + 1);
    const float* A = As[buf];
    const float* B = Bs[buf];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int ko = 4 * s + lq;
      const float a0 = A[(ar + li) * GX_LD + ko], a1 = A[(ar + 16 + li) * GX_LD + ko];
      const float b0 = B[(bc + li) * GX_LD + ko], b1 = B[(bc + 16 + li) * GX_LD + ko];
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[1], 0, 0, 0);
      acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[2], 0, 0, 0);
      acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[3], 0, 0, 0);
    }
    if (want_cs && t < GX_T) {
      const float* Br = B + t * GX_LD;
      float c = 0.f;
#pragma unroll 16
      for (int k = 0; k < GX_T; ++k) c += Br[k];
      cs += (double)c;
    }
    if constexpr (F64) {
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        dacc[x][0] += (double)acc[x].x;
        dacc[x][1] += (double)acc[x].y;
        dacc[x][2] += (double)acc[x].z;
        dacc[x][3] += (double)acc[x].w;
        acc[x] = v4f{0.f, 0.f, 0.f, 0.f};
      }
    }
    if (GX_NBUF == 1) __syncthreads();  // every wave is done with the stage before it is refilled
    if (kb + 1 < kb1) store(GX_NBUF == 1 ? 0 : buf ^ 1, kb + 1);
    __syncthreads();
  }

  if constexpr (PH == GX_GRAD0) {
    if (t < GX_T) cs_s[t] = cs;
    __syncthreads();
  }
  gx_epilogue<PH, F64>(st, bd, S, l, tm, tn, split, wi, wo, ar, bc, li, lq, acc, dacc, cs, cs_s);
}

// ---------------------------------------------------------------------------
// the masked layer on the bf16 MFMA ("b3"): FWD0 (Z0 = G Wp_0^T) and GRAD0
// (G^T delta0).  The genotype codes 0..2 are exact in bf16; the f32 operand x
// is split into three bf16 planes hi + mid + lo (hi = bf16(x), mid =
// bf16(x - hi), lo = bf16(x - hi - mid): 24 significant bits), so one 32-deep
// K step is 3 v_mfma_f32_16x16x32_bf16 (48 cycles) where the f32 MFMA needs 8
// (256 cycles): 5.3x the masked layer's rate, products exact, f32 accumulation
// inside 64-deep K blocks and f64 across them as in k_gx_gemm.  The f32 path
// stays selectable (BANN_GX_EXACT=1: exact f32 products).
// LDS images [row][k] with 72-element rows (conflict-free 16-byte fragment reads).
// ---------------------------------------------------------------------------
#define GX_LDH 80  // bf16 row stride (elements): 40 dwords, conflict-free row and transposing reads (below)
#ifndef GX_F64_EVERY
#define GX_F64_EVERY 4  // 64-deep K blocks per f32 accumulation before the f64 sum (256 rows / markers)
#endif
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

namespace {
// x = hi + mid + lo exactly, by truncation: hi = the top 8 significant bits, mid
// the next 8 of the (exact) remainder, lo the last 8 (representable as is): two
// ANDs and two subtractions, no conversions; each plane is the high half of an
// f32 word
__device__ __forceinline__ void split3(float x, __bf16& hi, __bf16& mi, __bf16& lo) {
  const uint32_t hb = __float_as_uint(x) & 0xFFFF0000u;
  const float r = x - __uint_as_float(hb);  // exact
  const uint32_t mb = __float_as_uint(r) & 0xFFFF0000u;
  const uint32_t lb = __float_as_uint(r - __uint_as_float(mb));  // exact, <= 8 significant bits
  hi = __builtin_bit_cast(__bf16, (uint16_t)(hb >> 16));
  mi = __builtin_bit_cast(__bf16, (uint16_t)(mb >> 16));
  lo = __builtin_bit_cast(__bf16, (uint16_t)(lb >> 16));
}
}  // namespace

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;
namespace {
// 16-lane-group transposing read (T10): lane 4q + p of a group gives the address of
// row q, columns 4p .. 4p+3 of a 4 x 16 block; lane i receives column i, row q in
// element q.  Two of them stacked = one 8-deep bf16 MFMA fragment along the rows.
__device__ __forceinline__ bf16x8 tr16_pair(const __bf16* p0, const __bf16* p1) {
  const v4s a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p0));
  const v4s b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p1));
  typedef short v8s __attribute__((ext_vector_type(8)));
  const v8s r = v8s{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, r);
}
}  // namespace

// K slot of logical k (0..63) of a 64-deep K block in the b3 stages: the K slots
// 8 lq + j of half ks are k = 32 ks + 16 (j >> 2) + 4 lq + (j & 3), so the two
// 16-lane groups of a transposing read (rows 4 lq + tq) take rows 0-3 / 4-7 of an
// 8-row bank window; operands read along their rows store logical K group c (4
// consecutive k) at this element offset
__device__ __forceinline__ int b3_kpos(int c) { return 32 * (c >> 3) + 8 * (c & 3) + 4 * ((c >> 2) & 1); }

// LDS: the genotype chunk as G[marker][individual] (16 consecutive individuals per
// thread: two 16-byte stores; GRAD0, whose K is the individuals, four 8-byte stores
// at b3_kpos); FWD0 takes its A fragments (rows = individuals,
// K = markers) from it by transposing reads and its B fragments from the W0 planes
// [column][marker] (pre-split by k_gx_prep); GRAD0 takes A (rows = markers, K =
// individuals) by row reads and B from the delta0 planes [individual][column]
// (split on staging, 8-byte stores) by transposing reads.
template <int PH>
__global__ void __launch_bounds__(256, PH == GX_GRAD0 ? 3 : 4)
    k_gx_gemm_b3(DevState st, const int32_t* __restrict__ blist, const int32_t* __restrict__ prefix, int nb,
                 int total, int per) {
  __shared__ __attribute__((aligned(16))) __bf16 Gs[GX_T * GX_LDH];     // [marker][individual]
  __shared__ __attribute__((aligned(16))) __bf16 Bs[3][GX_T * GX_LDH];  // FWD0 [column][marker], GRAD0 [individual][column]
  const int q = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (q >= total) return;
  int lo_ = 0, hi_ = nb;
  while (hi_ - lo_ > 1) {
    const int mid = (lo_ + hi_) >> 1;
    if (prefix[mid] <= q) lo_ = mid;
    else hi_ = mid;
  }
  const int b = blist[lo_];
  const BranchDev& bd = st.br[b];
  int tmc, tnc, ns;
  gx_dims(st, bd, PH, 0, tmc, tnc, ns);
  int r = q - prefix[lo_];
  const int split = r / (tmc * tnc);
  r -= split * tmc * tnc;
  const int tm = r / tnc, tn = r % tnc;
  const int64_t rows = gx_rows(st);
  float* S = gx_base(st, bd);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int ar = 32 * (wv >> 1), bc = 32 * (wv & 1);
  const uint8_t* img = st.xu2 + bd.x_off;
  const int64_t tstride = (int64_t)bd.nchunks * 1024;
  const int wo = bd.widths[0];
  const int m64 = 64 * bd.nchunks;
  int kb0 = 0, kb1;
  if constexpr (PH == GX_FWD0) {
    kb1 = bd.nchunks;
  } else {
    const int ntile = (st.nfrag + 3) / 4;
    kb0 = (int)((int64_t)ntile * split / ns);
    kb1 = (int)((int64_t)ntile * (split + 1) / ns);
  }
  const __bf16* W0p = reinterpret_cast<const __bf16*>(S + bd.gx_w0p);
  const float* Dm = S + bd.gx_h[0];
  const int64_t ldd = bd.gx_ld[0];
  Blk rb;
  v4i rw[6];
  uint32_t rg = 0;
  auto load = [&](int kb) {
    if constexpr (PH == GX_FWD0) {
      rg = geno_load(img + (int64_t)tm * tstride + (int64_t)kb * 1024);
#pragma unroll
      for (int u = 0; u < 6; ++u) {  // 3 planes x 64 columns x 8 pieces of 8 markers
        const int e = t + 256 * u, pl = e >> 9, row = (e >> 3) & 63, pc = e & 7;
        const int col = 64 * tn + row;
        v4i v = v4i{0, 0, 0, 0};
        if (col < wo) v = *reinterpret_cast<const v4i*>(W0p + ((int64_t)pl * wo + col) * m64 + 64 * kb + 8 * pc);
        rw[u] = v;
      }
    } else {
      rg = geno_load(img + (int64_t)kb * tstride + (int64_t)tm * 1024);
      blk_load(rb, Dm, ldd, BlkBounds{64 * (int64_t)kb, rows, 64 * tn, wo});
    }
  };
  double csp[4] = {0.0, 0.0, 0.0, 0.0};  // GRAD0: column sums of delta0, columns 4 (t & 15) + x
  float cspf[4] = {0.f, 0.f, 0.f, 0.f};  //   their f32 part since the last f64 sum (with dacc's)
  auto store = [&](int kb) {
    int jl, dq;
    geno_pos(jl, dq);
    {
      bf16x8 v0, v1;
#pragma unroll
      for (int s2 = 0; s2 < 8; ++s2) {
        v0[s2] = (__bf16)(float)((rg >> (2 * s2)) & 3u);
        v1[s2] = (__bf16)(float)((rg >> (2 * s2 + 16)) & 3u);
      }
      if constexpr (PH == GX_FWD0) {
        *(bf16x8*)&Gs[jl * GX_LDH + 16 * dq] = v0;
        *(bf16x8*)&Gs[jl * GX_LDH + 16 * dq + 8] = v1;
      } else {
        *(bf16x4*)&Gs[jl * GX_LDH + b3_kpos(4 * dq)] = bf16x4{v0[0], v0[1], v0[2], v0[3]};
        *(bf16x4*)&Gs[jl * GX_LDH + b3_kpos(4 * dq + 1)] = bf16x4{v0[4], v0[5], v0[6], v0[7]};
        *(bf16x4*)&Gs[jl * GX_LDH + b3_kpos(4 * dq + 2)] = bf16x4{v1[0], v1[1], v1[2], v1[3]};
        *(bf16x4*)&Gs[jl * GX_LDH + b3_kpos(4 * dq + 3)] = bf16x4{v1[4], v1[5], v1[6], v1[7]};
      }
    }
    if constexpr (PH == GX_FWD0) {
#pragma unroll
      for (int u = 0; u < 6; ++u) {
        const int e = t + 256 * u, pl = e >> 9, row = (e >> 3) & 63, pc = e & 7;
        *(v2i*)&Bs[pl][row * GX_LDH + b3_kpos(2 * pc)] = v2i{rw[u][0], rw[u][1]};
        *(v2i*)&Bs[pl][row * GX_LDH + b3_kpos(2 * pc + 1)] = v2i{rw[u][2], rw[u][3]};
      }
    } else {
      blk_fix(rb, BlkBounds{64 * (int64_t)kb, rows, 64 * tn, wo});
#pragma unroll
      for (int u = 0; u < 4; ++u) {  // Bs[p][individual][column], four columns per store
        const int e = t + 256 * u, rr = e >> 4, c4 = 4 * (e & 15);
        bf16x4 h4, m4, l4;
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          __bf16 hh, mm, ll;
          split3(rb.v[u][x], hh, mm, ll);
          h4[x] = hh;
          m4[x] = mm;
          l4[x] = ll;
          cspf[x] += rb.v[u][x];
        }
        *(bf16x4*)&Bs[0][rr * GX_LDH + c4] = h4;
        *(bf16x4*)&Bs[1][rr * GX_LDH + c4] = m4;
        *(bf16x4*)&Bs[2][rr * GX_LDH + c4] = l4;
      }
    }
  };

  v4f acc[4];
  double dacc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    acc[x] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int y = 0; y < 4; ++y) dacc[x][y] = 0.0;
  }
  const int tq = li >> 2, tp = li & 3;  // transposing reads: lane 4 tq + tp
  if (kb0 < kb1) load(kb0);
  for (int kb = kb0; kb < kb1; ++kb) {
    store(kb);
    __syncthreads();
    if (kb + 1 < kb1) load(kb + 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ko = 32 * ks + 8 * lq;          // this lane group's 8 K slots (row reads)
      const int kr = 32 * ks + 4 * lq + tq;     // their rows 0-3 (+ 16: 4-7) in transposing reads
      bf16x8 a0, a1;
      if constexpr (PH == GX_FWD0) {  // rows = individuals, K = markers: transposed from Gs
        a0 = tr16_pair(&Gs[kr * GX_LDH + ar + 4 * tp], &Gs[(kr + 16) * GX_LDH + ar + 4 * tp]);
        a1 = tr16_pair(&Gs[kr * GX_LDH + ar + 16 + 4 * tp], &Gs[(kr + 16) * GX_LDH + ar + 16 + 4 * tp]);
      } else {  // rows = markers, K = individuals: row reads
        a0 = *(const bf16x8*)&Gs[(ar + li) * GX_LDH + ko];
        a1 = *(const bf16x8*)&Gs[(ar + 16 + li) * GX_LDH + ko];
      }
#pragma unroll
      for (int pl = 2; pl >= 0; --pl) {  // small planes first
        bf16x8 b0, b1;
        if constexpr (PH == GX_FWD0) {  // B[k = marker][n = column] from Bs[column][marker]
          b0 = *(const bf16x8*)&Bs[pl][(bc + li) * GX_LDH + ko];
          b1 = *(const bf16x8*)&Bs[pl][(bc + 16 + li) * GX_LDH + ko];
        } else {  // B[k = individual][n = column] transposed from Bs[individual][column]
          b0 = tr16_pair(&Bs[pl][kr * GX_LDH + bc + 4 * tp], &Bs[pl][(kr + 16) * GX_LDH + bc + 4 * tp]);
          b1 = tr16_pair(&Bs[pl][kr * GX_LDH + bc + 16 + 4 * tp], &Bs[pl][(kr + 16) * GX_LDH + bc + 16 + 4 * tp]);
        }
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b1, acc[1], 0, 0, 0);
        acc[2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b0, acc[2], 0, 0, 0);
        acc[3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, acc[3], 0, 0, 0);
      }
    }
    if (((kb - kb0) & (GX_F64_EVERY - 1)) == GX_F64_EVERY - 1 || kb + 1 == kb1) {  // f64 across 256-deep K
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        dacc[x][0] += (double)acc[x].x;
        dacc[x][1] += (double)acc[x].y;
        dacc[x][2] += (double)acc[x].z;
        dacc[x][3] += (double)acc[x].w;
        acc[x] = v4f{0.f, 0.f, 0.f, 0.f};
        if constexpr (PH == GX_GRAD0) {
          csp[x] += (double)cspf[x];
          cspf[x] = 0.f;
        }
      }
    }
    __syncthreads();  // every wave is done with the stage before it is refilled
  }

  if constexpr (PH == GX_FWD0) {
    gx_epilogue<GX_FWD0, true>(st, bd, S, 0, tm, tn, split, 0, wo, ar, bc, li, lq, acc, dacc, 0.0, nullptr);
  } else {
    // column sums: 16 threads per column group, added in thread order (deterministic)
    double* cs_s = reinterpret_cast<double*>(&Bs[0][0]);  // [16][64], the staging is free now
#pragma unroll
    for (int x = 0; x < 4; ++x) cs_s[(t >> 4) * 64 + 4 * (t & 15) + x] = csp[x];
    __syncthreads();
    double* cs_f = reinterpret_cast<double*>(&Gs[0]);  // [64]
    if (t < GX_T) {
      double c = 0.0;
      for (int k = 0; k < 16; ++k) c += cs_s[k * 64 + t];
      cs_f[t] = c;
    }
    __syncthreads();
    float* part = st.part + bd.part_off + (int64_t)split * bd.P;
    const int wi = bd.m, win = bd.m;
    float sgv[2][4], muv[2][4];  // the lane's eight markers, loaded together (index clamped)
#pragma unroll
    for (int X = 0; X < 2; ++X)
#pragma unroll
      for (int y = 0; y < 4; ++y) {
        const int ic = min(64 * tm + ar + 16 * X + 4 * lq + y, wi - 1);
        sgv[X][y] = st.sigma[bd.mk_off + ic];
        muv[X][y] = st.mu[bd.mk_off + ic];
      }
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int jc = bc + 16 * (x & 1) + li;
      const int j = 64 * tn + jc;
      if (j >= wo) continue;
      const double cs = cs_f[jc];
#pragma unroll
      for (int y = 0; y < 4; ++y) {
        const int i = 64 * tm + ar + 16 * (x >> 1) + 4 * lq + y;
        if (i >= wi) continue;
        const float sg = sgv[x >> 1][y];
        const double v = sg > 0.f ? (dacc[x][y] - (double)muv[x >> 1][y] * cs) / (double)sg : 0.0;
        part[bd.woff[0] + (int64_t)j * win + i] = (float)v;
      }
    }
    if (tm == 0 && t < GX_T && 64 * tn + t < wo) part[bd.boff[0] + 64 * tn + t] = (float)cs_f[t];  // db0
  }
}

// ---------------------------------------------------------------------------
// the hidden-layer GEMMs on the bf16 MFMA ("x3"): FWD l, BWD l and GRAD l with
// BOTH f32 operands split into three bf16 planes (x = x0 + x1 + x2, 24
// significant bits, split3) and the six plane products of weight >= 2^-16:
//   a b = a0 b0 + (a0 b1 + a1 b0) + (a0 b2 + a1 b1 + a2 b0) + O(2^-24 |a b|),
// every product keeps f32's accuracy; a 32-deep K step is six
// v_mfma_f32_16x16x32_bf16 (96 cycles) where the f32 MFMA takes eight 16x16x4
// (256 cycles).  K blocks of 32: the 3 + 3 planes of a stage take 30 KiB, four
// workgroups per CU.  An operand whose MFMA rows are contiguous in memory (FWD:
// A_{l-1} and Wp_l; BWD: delta_l) is staged [row][k] and read as 16-byte
// fragments; the others (BWD: Wp_l read transposed; GRAD: A_{l-1} and delta_l,
// K = individuals) are staged [k][row] and read with ds_read_b64_tr_b16.  f32
// accumulation inside a K block, f64 across blocks where K is long (GRAD: the
// rows).  BANN_GX_EXACT=1 keeps k_gx_gemm (f32 MFMA) for every phase.
// ---------------------------------------------------------------------------
#define GX_KB 32  // K block depth
#define GX_RK 40  // [row][k] stride (bf16 elements): 80-byte rows

namespace {
// LDS geometry of a staged operand block of R (MFMA) rows x 32 K as three bf16 planes:
// [row][k] rows of GX_RK, or [k][row] rows of KRS = R + 16.  Bank conflicts
// (MI355X_MICROARCH.md LDS table; PMC: SQ_LDS_BANK_CONFLICT was 20-45 % of the
// phases' LDS cycles before this layout):
//  - [row][k]: the 16-byte K chunk q of row r sits at chunk q ^ rk_sw(r), which
//    makes the fragment reads (ds_read_b128, lane groups {0-3,12-15,20-27}, ...)
//    conflict-free at the 80-byte stride;
//  - [k][row]: the K slots 8 lq + j of a fragment are rows 16 (j >> 2) + 4 lq +
//    (j & 3) (kr_row), so the two 16-lane groups of a transposing read take rows
//    0-3 / 4-7 of an 8-row window (conflict-free at R + 16); a [row][k] operand
//    paired with a [k][row] one (BWD's A) stores logical k at that K slot (PERM).
template <int R, bool RK>
struct Geo {
  static constexpr int KRS = R + 16;
  static constexpr int PL = RK ? R * GX_RK : GX_KB * KRS;  // elements per plane
};
__device__ __forceinline__ int rk_sw(int r) { return ((r >> 2) ^ (r >> 3)) & 1; }
// element offset of logical K group c (4 consecutive k) of [row][k] row r
template <bool PERM>
__device__ __forceinline__ int rk_off(int r, int c) {
  const int p = PERM ? 8 * (c & 3) + 4 * (c >> 2) : 4 * c;  // K slot of logical k = 4 c
  return r * GX_RK + 8 * ((p >> 3) ^ rk_sw(r)) + (p & 7);
}
// an R (MFMA rows) x 32 (K) block of an f32 matrix, R / 32 x 4 consecutive elements
// per thread.  RK: M[r][k], thread e = t + 256 u holds row e >> 3, k 4 (e & 7) .. +3.
// KR: M[k][r], thread e holds k e / (R / 4), rows 4 (e % (R / 4)) .. +3.  Elements
// outside r < rmax, k < kmax are 0 (masked at the store, as blk_fix).
template <int R>
struct Blk2 {
  v4f v[R / 32];
};
struct Blk2Bounds {
  int64_t r0, rmax, k0, kmax;
};
template <bool RK, int R>
__device__ __forceinline__ int blk2_nv(const Blk2Bounds& k, int u) {
  const int e = threadIdx.x + 256 * u;
  if constexpr (RK) {
    const int64_t r = k.r0 + (e >> 3), c = k.k0 + 4 * (e & 7);
    return r < k.rmax ? (int)min(max(k.kmax - c, (int64_t)0), (int64_t)4) : 0;
  } else {
    const int64_t kk = k.k0 + e / (R / 4), r = k.r0 + 4 * (e % (R / 4));
    return kk < k.kmax ? (int)min(max(k.rmax - r, (int64_t)0), (int64_t)4) : 0;
  }
}
template <bool RK, int R>
__device__ __forceinline__ void blk2_load(Blk2<R>& s, const float* __restrict__ M, int64_t ld, const Blk2Bounds& k) {
#pragma unroll
  for (int u = 0; u < R / 32; ++u) {
    const int e = threadIdx.x + 256 * u;
    v4f x = {0.f, 0.f, 0.f, 0.f};
    if (blk2_nv<RK, R>(k, u) > 0)
      x = RK ? *(const v4f*)(M + (k.r0 + (e >> 3)) * ld + k.k0 + 4 * (e & 7))    // rows padded to 4
             : *(const v4f*)(M + (k.k0 + e / (R / 4)) * ld + k.r0 + 4 * (e % (R / 4)));
    s.v[u] = x;
  }
}
// mask, split into the three planes P[3][PL] and store; csp (KR only) += the
// masked values per row of the thread's four
template <bool RK, bool CS, int R, bool PERM = false>
__device__ __forceinline__ void blk2_store(Blk2<R>& s, const Blk2Bounds& k, __bf16* P, double (&csp)[4]) {
  constexpr int PL = Geo<R, RK>::PL, KRS = Geo<R, RK>::KRS;
#pragma unroll
  for (int u = 0; u < R / 32; ++u) {
    const int e = threadIdx.x + 256 * u;
    const int nv = blk2_nv<RK, R>(k, u);
    v4f x = s.v[u];
    if (nv < 1) x.x = 0.f;
    if (nv < 2) x.y = 0.f;
    if (nv < 3) x.z = 0.f;
    if (nv < 4) x.w = 0.f;
    bf16x4 h4, m4, l4;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      __bf16 hh, mm, ll;
      split3(x[c], hh, mm, ll);
      h4[c] = hh;
      m4[c] = mm;
      l4[c] = ll;
      if constexpr (CS) csp[c] += (double)x[c];
    }
    const int off = RK ? rk_off<PERM>(e >> 3, e & 7) : (e / (R / 4)) * KRS + 4 * (e % (R / 4));
    *(bf16x4*)&P[off] = h4;
    *(bf16x4*)&P[PL + off] = m4;
    *(bf16x4*)&P[2 * PL + off] = l4;
  }
}
// the bf16x8 fragment (MFMA rows rb .. rb + 15, K slots 8 lq .. 8 lq + 7) of plane pl
template <bool RK, int R>
__device__ __forceinline__ bf16x8 frag3(const __bf16* P, int pl, int rb, int li, int lq) {
  constexpr int PL = Geo<R, RK>::PL, KRS = Geo<R, RK>::KRS;
  if constexpr (RK) {
    return *(const bf16x8*)&P[pl * PL + (rb + li) * GX_RK + 8 * (lq ^ rk_sw(li))];  // rb: a multiple of 16
  } else {
    const int tq = li >> 2, tp = li & 3;
    return tr16_pair(&P[pl * PL + (4 * lq + tq) * KRS + rb + 4 * tp],
                     &P[pl * PL + (16 + 4 * lq + tq) * KRS + rb + 4 * tp]);
  }
}
}  // namespace

// tile shape of k_gx_gemm_x3 per phase: wave tiles of 16 AX x 16 AY, 2 x 2 waves.
// FWD takes 64 x 128 tiles: its A block (activations, split into planes while
// staging) feeds twice the MFMAs of a 64 x 64 tile, 3 workgroups per CU (c3def
// FWD1: 2.78 -> 2.50 ms per 40-branch group).  Measured and not kept: 128 x 128
// (2 per CU: FWD 2.59, BWD 3.16 -> 3.59 ms), BWD at 64 x 128 (3.17: flat).
// gx_tiles and the head's slot count follow these.
template <int PH>
struct X3Shape {
  static constexpr int AX = 2, AY = PH == GX_BWD ? 2 : 4;
};
template <int PH>
__global__ void __launch_bounds__(256, PH == GX_FWD ? 3 : (PH == GX_GRAD ? 2 : 4))
    k_gx_gemm_x3(DevState st, const int32_t* __restrict__ blist, const int32_t* __restrict__ prefix, int nb, int l,
                 int total, int per) {
  constexpr int AX = X3Shape<PH>::AX, AY = X3Shape<PH>::AY, TM = 32 * AX, TN = 32 * AY;
  constexpr bool ARK = PH != GX_GRAD;  // A staged [row][k]
  constexpr bool BRK = PH == GX_FWD;   // B staged [row][k]
  constexpr bool F64 = PH == GX_GRAD;
  constexpr int PLA = Geo<TM, ARK>::PL, PLB = Geo<TN, BRK>::PL, KRSB = Geo<TN, BRK>::KRS;
  __shared__ __attribute__((aligned(16))) __bf16 As[3 * PLA];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[3 * PLB];
  __shared__ double cs_s[PH == GX_GRAD ? 1024 / TN : 1][TN];  // GRAD's column sums only
  const int q = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);  // XCD-aware numbering (k_gx_gemm)
  if (q >= total) return;
  int lo_ = 0, hi_ = nb;
  while (hi_ - lo_ > 1) {
    const int mid = (lo_ + hi_) >> 1;
    if (prefix[mid] <= q) lo_ = mid;
    else hi_ = mid;
  }
  const int b = blist[lo_];
  const BranchDev& bd = st.br[b];
  int tmc, tnc, ns;
  gx_dims(st, bd, PH, l, tmc, tnc, ns, TM, TN);
  int r = q - prefix[lo_];
  const int split = r / (tmc * tnc);
  r -= split * tmc * tnc;
  const int tm = r / tnc, tn = r % tnc;
  const int64_t rows = gx_rows(st);
  float* S = gx_base(st, bd);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int ar = (TM / 2) * (wv >> 1), bc = (TN / 2) * (wv & 1);
  // lazy head (k_gx_head): delta_s = h'(A_s) * e * w_out is never stored.  BWD_s:
  // A = h'(A_s), B = the w_out-scaled planes of Wp_s (k_gx_prep), the epilogue
  // multiplies row i by e_i; GRAD_s: B = h'(A_s) * e (e of the block's rows, per K
  // block), the epilogue multiplies column j by w_out_j; its column sums give db_s
  // (times w_out) and dW_out = A_s^T e (f64, from the raw A_s values)
  const bool lazy = PH != GX_FWD && l == bd.L - 2 && dh_from_a(bd.act);
  const float* ev = S + bd.gx_e;
  const float* wout = S + bd.gx_w[bd.L - 1];

  int64_t kb0 = 0, kb1, kcount;
  const float* Am;
  const float* Bm;
  int64_t lda, ldb;
  int wi = 0, wo;
  if constexpr (PH == GX_FWD) {  // Z_l = A_{l-1} Wp_l^T: A [individual][in], B = Wp_l [out][in]
    kcount = bd.widths[l - 1];
    Am = S + bd.gx_a[l - 1];
    lda = bd.gx_ld[l - 1];
    Bm = S + bd.gx_w[l];
    ldb = bd.gx_wld[l];
    wo = bd.widths[l];
  } else if constexpr (PH == GX_BWD) {  // delta_l Wp_l: A = delta_l [individual][out], B = Wp_l [out = k][in]
    kcount = bd.widths[l];
    Am = S + (lazy ? bd.gx_a[l] : bd.gx_h[l]);
    lda = bd.gx_ld[l];
    Bm = S + bd.gx_w[l];
    ldb = bd.gx_wld[l];
    wo = bd.widths[l - 1];
  } else {  // GRAD: dW_l = A_{l-1}^T delta_l over the split's rows (K = individuals)
    const int ntile = (st.nfrag + 3) / 4;
    kcount = rows;
    Am = S + bd.gx_a[l - 1];
    lda = bd.gx_ld[l - 1];
    wi = bd.widths[l - 1];
    Bm = S + (lazy ? bd.gx_a[l] : bd.gx_h[l]);
    ldb = bd.gx_ld[l];
    wo = bd.widths[l];
    kb0 = 2 * ((int64_t)ntile * split / ns);  // 64-row tiles -> 32-deep K blocks
    kb1 = 2 * ((int64_t)ntile * (split + 1) / ns);
  }
  if constexpr (PH != GX_GRAD) kb1 = (kcount + GX_KB - 1) / GX_KB;
  // the operand blocks of K block kb: rows of the A block are output rows (TM tm ..),
  // rows of the B block output columns (TN tn ..)
  auto bnd_a = [&](int64_t kb) {
    return Blk2Bounds{TM * (int64_t)tm, PH == GX_GRAD ? (int64_t)wi : rows, GX_KB * kb, kcount};
  };
  auto bnd_b = [&](int64_t kb) { return Blk2Bounds{TN * (int64_t)tn, (int64_t)wo, GX_KB * kb, kcount}; };
  Blk2<TM> ra;
  Blk2<TN> rb;
  double csa[4] = {0.0, 0.0, 0.0, 0.0}, csp[4] = {0.0, 0.0, 0.0, 0.0};  // GRAD: column sums of delta_l
  // FWD / BWD: B = Wp_l from its pre-split planes [3][out][r32(in)] (k_gx_prep): TN / 64
  // 16-byte pieces of 8 elements per plane and thread, copied to the stage as is.
  // FWD stages it [out][in] (piece p: out row p >> 2, in 8 (p & 3) ..), BWD [out = k][in]
  // (piece p: out row p / (TN / 8), in 8 (p % (TN / 8)) ..); rows past the layer and
  // pieces past the in width are zero (the planes' padding covers the rest of a piece)
  constexpr bool BP = PH != GX_GRAD;
  constexpr int NP = TN / 64;
  v4i rbp[NP][3];
  const __bf16* Wp3 = BP ? reinterpret_cast<const __bf16*>(S + (PH == GX_BWD && lazy ? bd.gx_wps : bd.gx_wp[l]))
                         : nullptr;
  const int64_t l3 = BP ? ((bd.win[l] + 31) & ~31) : 0, p3 = BP ? (int64_t)bd.widths[l] * l3 : 0;
  auto load_bp = [&](int64_t kb) {
#pragma unroll
    for (int v = 0; v < NP; ++v) {
      const int pc = t + 256 * v;
      int64_t row, col;
      bool ok;
      if constexpr (PH == GX_FWD) {
        row = TN * (int64_t)tn + (pc >> 2);
        col = GX_KB * kb + 8 * (pc & 3);
        ok = row < wo;
      } else {
        row = GX_KB * kb + pc / (TN / 8);
        col = TN * (int64_t)tn + 8 * (pc % (TN / 8));
        ok = row < kcount && col < wo;
      }
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        rbp[v][pl] = ok ? *reinterpret_cast<const v4i*>(Wp3 + pl * p3 + row * l3 + col) : v4i{0, 0, 0, 0};
    }
  };
  auto store_bp = [&]() {
#pragma unroll
    for (int v = 0; v < NP; ++v) {
      const int pc = t + 256 * v;
      const int off = PH == GX_FWD ? (pc >> 2) * GX_RK + 8 * ((pc & 3) ^ rk_sw(pc >> 2))
                                   : (pc / (TN / 8)) * KRSB + 8 * (pc % (TN / 8));
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<v4i*>(&Bs[pl * PLB + off]) = rbp[v][pl];
    }
  };
  const bool want_cs = PH == GX_GRAD && tm == 0;

  v4f acc[AX * AY];
  double dacc[AX * AY][4];
#pragma unroll
  for (int x = 0; x < AX * AY; ++x) {
    acc[x] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int y = 0; y < 4; ++y) dacc[x][y] = 0.0;
  }
  float le[4] = {0.f, 0.f, 0.f, 0.f};
  double csq[4] = {0.0, 0.0, 0.0, 0.0};  // GRAD_s, tm == 0: dW_out column sums
  auto lazy_load = [&](int64_t kb) {
    if constexpr (PH == GX_GRAD) {
#pragma unroll
      for (int u = 0; u < TN / 32; ++u) le[u] = ev[GX_KB * kb + (t + 256 * u) / (TN / 4)];
    }
  };
  const DhA dk = dh_a_consts(bd.act);
  const bool tanh_act = bd.act == 0;
  auto lazy_h = [&](auto& rr) {  // rr = h'(A_s) (* e of the row: GRAD)
    constexpr int NU = sizeof(rr.v) / sizeof(v4f);
    if (tanh_act) {
#pragma unroll
      for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float a = rr.v[u][c];
          rr.v[u][c] = PH == GX_GRAD ? (1.f - a * a) * le[u] : 1.f - a * a;
        }
    } else {
#pragma unroll
      for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float h = dh_a(rr.v[u][c], dk);
          rr.v[u][c] = PH == GX_GRAD ? h * le[u] : h;
        }
    }
  };
  auto lazy_dwo = [&](const Blk2<TN>& rr) {
#pragma unroll
    for (int u = 0; u < TN / 32; ++u)
#pragma unroll
      for (int c = 0; c < 4; ++c) csq[c] += (double)rr.v[u][c] * (double)le[u];
  };
  // values the epilogue needs, loaded before the K loop (gx_epilogue): FWD the bias
  // and w_out of the lane's AY columns, lazy BWD_s the e of its 4 AX rows, lazy
  // GRAD_s w_out of its AY columns
  float pre[4 * AX > 2 * AY ? 4 * AX : 2 * AY];
#pragma unroll
  for (int i = 0; i < (int)(sizeof(pre) / sizeof(float)); ++i) pre[i] = 0.f;
  if constexpr (PH == GX_FWD) {
    const bool head = l == bd.L - 2 && dh_from_a(bd.act);
#pragma unroll
    for (int Y = 0; Y < AY; ++Y) {
      const int j = TN * tn + bc + 16 * Y + li;
      pre[Y] = j < wo ? S[bd.gx_b[l] + j] : 0.f;
      pre[AY + Y] = head && j < wo ? wout[j] : 0.f;
    }
  } else if constexpr (PH == GX_BWD) {
    if (lazy)
#pragma unroll
      for (int X = 0; X < AX; ++X)
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          const int64_t row = TM * (int64_t)tm + ar + 16 * X + 4 * lq + y;
          pre[4 * X + y] = row < rows ? ev[row] : 0.f;
        }
  } else {
    if (lazy)
#pragma unroll
      for (int Y = 0; Y < AY; ++Y) {
        const int j = TN * tn + bc + 16 * Y + li;
        pre[Y] = j < wo ? wout[j] : 0.f;
      }
  }
  auto load = [&](int64_t kb) {
    if (lazy) lazy_load(kb);
    blk2_load<ARK, TM>(ra, Am, lda, bnd_a(kb));
    if constexpr (BP) load_bp(kb);
    else blk2_load<BRK, TN>(rb, Bm, ldb, bnd_b(kb));
  };
  auto stage = [&](int64_t kb) {
    if constexpr (PH == GX_BWD) {
      if (lazy) lazy_h(ra);
    } else if constexpr (PH == GX_GRAD) {
      if (lazy) {
        if (want_cs) lazy_dwo(rb);
        lazy_h(rb);
      }
    }
    blk2_store<ARK, false, TM, PH == GX_BWD>(ra, bnd_a(kb), As, csa);  // BWD: A [row][k] beside B [k][row]
    if constexpr (BP) store_bp();
    else if (want_cs) blk2_store<BRK, true, TN>(rb, bnd_b(kb), Bs, csp);
    else blk2_store<BRK, false, TN>(rb, bnd_b(kb), Bs, csp);
  };
  auto compute = [&](int64_t kb) {
    bf16x8 a[AX][3];
#pragma unroll
    for (int X = 0; X < AX; ++X)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) a[X][pl] = frag3<ARK, TM>(As, pl, ar + 16 * X, li, lq);
#pragma unroll
    for (int Y = 0; Y < AY; ++Y) {
      bf16x8 bq[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) bq[pl] = frag3<BRK, TN>(Bs, pl, bc + 16 * Y, li, lq);
#pragma unroll
      for (int X = 0; X < AX; ++X) {
        v4f& c = acc[AY * X + Y];
        // small products first
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[X][2], bq[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[X][1], bq[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[X][0], bq[2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[X][1], bq[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[X][0], bq[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[X][0], bq[0], c, 0, 0, 0);
      }
    }
    if constexpr (F64) {
      if ((kb & (2 * GX_F64_EVERY - 1)) == 2 * GX_F64_EVERY - 1) {  // f64 across 256-deep K
#pragma unroll
        for (int x = 0; x < AX * AY; ++x) {
          dacc[x][0] += (double)acc[x].x;
          dacc[x][1] += (double)acc[x].y;
          dacc[x][2] += (double)acc[x].z;
          dacc[x][3] += (double)acc[x].w;
          acc[x] = v4f{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
  };
  if (kb0 < kb1) load(kb0);
  for (int64_t kb = kb0; kb < kb1; ++kb) {
    stage(kb);
    __syncthreads();
    if (kb + 1 < kb1) load(kb + 1);  // lands during this block's MFMAs
    compute(kb);
    __syncthreads();  // every wave is done with the stage before it is refilled
  }
  if constexpr (F64) {  // an odd block count leaves one block in acc
#pragma unroll
    for (int x = 0; x < AX * AY; ++x) {
      dacc[x][0] += (double)acc[x].x;
      dacc[x][1] += (double)acc[x].y;
      dacc[x][2] += (double)acc[x].z;
      dacc[x][3] += (double)acc[x].w;
    }
  }
  double cs = 0.0, cs2 = 0.0;
  if (want_cs) {  // 1024 / TN threads per 4-column group, added in thread order (deterministic)
    constexpr int RW = TN / 4;
#pragma unroll
    for (int x = 0; x < 4; ++x) cs_s[t / RW][4 * (t % RW) + x] = csp[x];
    __syncthreads();
    if (t < TN)
      for (int k = 0; k < 1024 / TN; ++k) cs += cs_s[k][t];
    if (lazy) {  // db_s = w_out * (column sums of h'(A_s) e); the dW_out column sums, same order
      cs *= (t < TN && TN * tn + t < wo) ? (double)wout[TN * tn + t] : 0.0;
      __syncthreads();
#pragma unroll
      for (int x = 0; x < 4; ++x) cs_s[t / RW][4 * (t % RW) + x] = csq[x];
      __syncthreads();
      if (t < TN)
        for (int k = 0; k < 1024 / TN; ++k) cs2 += cs_s[k][t];
    }
  }
  gx_epilogue<PH, F64, AX, AY>(st, bd, S, l, tm, tn, split, wi, wo, ar, bc, li, lq, acc, dacc, cs, nullptr, lazy, cs2,
                               PH == GX_FWD || lazy ? pre : nullptr);
}

// ---------------------------------------------------------------------------
// PREP: padded weights, W0 / sigma, c0 = b0 - mu^T (W0 / sigma) (f64), biases
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_gx_prep(DevState st, const int32_t* __restrict__ blist) {
  // grid (branches, GX_PREP_Y): every element is independent (computed from theta),
  // so the y blocks of a branch split every loop below
  const int b = blist[blockIdx.x];
  const BranchDev& bd = st.br[b];
  float* S = gx_base(st, bd);
  const float* th = st.theta + bd.p_off;
  const float* mu = st.mu + bd.mk_off;
  const float* sg = st.sigma + bd.mk_off;
  const int64_t g0 = (int64_t)blockIdx.y * 256 + threadIdx.x, gs = (int64_t)gridDim.y * 256;
  auto wval = [&](int l, int k, int j) -> float {  // Wp_l[k][j]: W_l (layer 0: W0 / sigma), 0 past the in width
    if (j >= bd.win[l]) return 0.f;
    const float v = th[bd.woff[l] + (int64_t)k * bd.win[l] + j];
    return l == 0 ? (sg[j] > 0.f ? v / sg[j] : 0.f) : v;
  };
  for (int l = 0; l < bd.L; ++l) {  // padded weights [out][gx_wld[l]]
    const int ld = bd.gx_wld[l];
    float* Wp = S + bd.gx_w[l];
    const int64_t tot = (int64_t)bd.widths[l] * ld;
    for (int64_t e = g0; e < tot; e += gs) Wp[e] = wval(l, (int)(e / ld), (int)(e % ld));
  }
  {  // W0 / sigma as three bf16 planes [3][w0][64 nchunks], zero padded (k_gx_gemm_b3)
    const int m64 = 64 * bd.nchunks;
    __bf16* P3 = reinterpret_cast<__bf16*>(S + bd.gx_w0p);
    const int64_t tot = (int64_t)bd.widths[0] * m64;
    for (int64_t e = g0; e < tot; e += gs) {
      __bf16 hh, mm, ll;
      split3(wval(0, (int)(e / m64), (int)(e % m64)), hh, mm, ll);
      P3[e] = hh;
      P3[tot + e] = mm;
      P3[2 * tot + e] = ll;
    }
  }
  for (int l = 1; l < bd.L - 1; ++l) {  // Wp_l as three bf16 planes [3][w_l][r32(win_l)], zero padded (k_gx_gemm_x3)
    const int l3 = (bd.win[l] + 31) & ~31;
    __bf16* P3 = reinterpret_cast<__bf16*>(S + bd.gx_wp[l]);
    const int64_t tot = (int64_t)bd.widths[l] * l3;
    for (int64_t e = g0; e < tot; e += gs) {
      __bf16 hh, mm, ll;
      split3(wval(l, (int)(e / l3), (int)(e % l3)), hh, mm, ll);
      P3[e] = hh;
      P3[tot + e] = mm;
      P3[2 * tot + e] = ll;
    }
  }
  if (bd.L >= 3 && dh_from_a(bd.act)) {  // lazy head: w_out[k] Wp_s[k][j] as three planes (k_gx_gemm_x3 BWD_s)
    const int l = bd.L - 2, l3 = (bd.win[l] + 31) & ~31;
    const float* wo = th + bd.woff[bd.L - 1];
    __bf16* P3 = reinterpret_cast<__bf16*>(S + bd.gx_wps);
    const int64_t tot = (int64_t)bd.widths[l] * l3;
    for (int64_t e = g0; e < tot; e += gs) {
      const int k = (int)(e / l3);
      __bf16 hh, mm, ll;
      split3(wo[k] * wval(l, k, (int)(e % l3)), hh, mm, ll);
      P3[e] = hh;
      P3[tot + e] = mm;
      P3[2 * tot + e] = ll;
    }
  }
  // c0 = b0 - sum_j mu_j Wp_0[k][j] (f64): one wave per unit, lane-strided partials
  // added in a fixed order; the other biases
  {
    const int lane = threadIdx.x & 63;
    const int gw = (int)blockIdx.y * 4 + (threadIdx.x >> 6), nw = (int)gridDim.y * 4;
    for (int k = gw; k < bd.widths[0]; k += nw) {
      double acc = 0.0;
      for (int j = lane; j < bd.m; j += 64) acc += (double)mu[j] * (double)wval(0, k, j);
      acc = wave_sum_d(acc);
      if (lane == 0) S[bd.gx_b[0] + k] = (float)((double)th[bd.boff[0] + k] - acc);
    }
  }
  for (int l = 1; l < bd.L - 1; ++l)
    for (int64_t k = g0; k < bd.widths[l]; k += gs) S[bd.gx_b[l] + k] = th[bd.boff[l] + k];
}

// ---------------------------------------------------------------------------
// HEAD: output neuron, error, rss, predictions, dW_out, delta of the summary layer.
// grid (row tiles, branches): wave w takes rows w, w + 4, ... of the tile (lanes
// across the summary units, coalesced), then thread t takes units t, t + 256, ...
// over the tile's 64 rows.  dW_out and the rss leave per-tile f64 partials in the
// scratch; k_gx_head_red adds them per split in tile order (deterministic).
// ---------------------------------------------------------------------------
// Lazy head (fuse, the bf16-plane path, a summary layer after a hidden one and an
// activation whose h' is a function of A): the summary layer's FWD epilogue left
// the per-wave partials of out in gx_op, so the head only adds them (in slot order),
// forms e, pred and the rss, and writes e; BWD_s and GRAD_s form delta_s while
// staging and GRAD_s adds dW_out: A_s is not read here and delta_s never stored.
__device__ __forceinline__ bool gx_lazy_head(const BranchDev& bd, int fuse) {
  return fuse && bd.L >= 3 && dh_from_a(bd.act);
}
__global__ void __launch_bounds__(256) k_gx_head(DevState st, const int32_t* __restrict__ blist, int fuse) {
  __shared__ float e_s[GX_T];
  __shared__ double r_s[4];
  const int b = blist[blockIdx.y];
  const BranchDev& bd = st.br[b];
  const int tile = blockIdx.x;
  if (tile >= (st.nfrag + 3) / 4) return;
  float* S = gx_base(st, bd);
  const int sl = bd.L - 2, Sw = bd.widths[sl];
  if (gx_lazy_head(bd, fuse)) {
    const int t = threadIdx.x;
    if (t >= GX_T) return;
    const int64_t rows = gx_rows(st), row = 64 * (int64_t)tile + t;
    constexpr int TNF = 32 * X3Shape<GX_FWD>::AY;  // the summary layer's FWD tiles (k_gx_gemm_x3)
    const int ns = 2 * ((Sw + TNF - 1) / TNF);
    const float* op = S + bd.gx_op + row;
    double acc = 0.0;
    for (int k = 0; k < ns; ++k) acc += (double)op[k * rows];
    const float out = (float)acc;
    float e = 0.f;
    if (row < st.n) {
      e = out - st.y[bd.y_off + row];
      st.pred[bd.y_off + row] = out;
    }
    S[bd.gx_e + row] = e;
    const double rss = wave_sum_d((double)e * (double)e);
    if (t == 0) ((double*)(S + bd.gx_rss))[tile] = rss;
    return;
  }
  const float* A = S + bd.gx_a[sl];
  float* H = S + bd.gx_h[sl];
  const int64_t ld = bd.gx_ld[sl];
  const float* wout = S + bd.gx_w[bd.L - 1];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t r0 = 64 * (int64_t)tile;
  double rss = 0.0;
  for (int i = wv; i < GX_T; i += 4) {
    const int64_t row = r0 + i;
    const float* a = A + row * ld;
    double acc = 0.0;
    for (int k = lane; k < Sw; k += 64) acc += (double)a[k] * (double)wout[k];
    const float out = (float)wave_sum_d(acc);  // out = A_s w_out (the output layer has no bias)
    float e = 0.f;
    if (row < st.n) {
      e = out - st.y[bd.y_off + row];
      if (lane == 0) st.pred[bd.y_off + row] = out;
      rss += (double)e * (double)e;  // lane-uniform: counted once below
    }
    if (lane == 0) e_s[i] = e;
  }
  if (lane == 0) r_s[wv] = rss;
  __syncthreads();
  double* dwo = (double*)(S + bd.gx_dwo) + (int64_t)tile * Sw;
  const int act = bd.act;
  const bool fa = dh_from_a(act);
  for (int k = t; k < Sw; k += 256) {
    const float wk = wout[k];
    double d = 0.0;
#pragma unroll 8
    for (int i = 0; i < GX_T; ++i) {
      const float ei = e_s[i];
      const int64_t o = (r0 + i) * ld + k;
      const float a_o = A[o];
      d += (double)a_o * (double)ei;
      const float h = fa ? act_dh_a(a_o, act) : H[o];
      H[o] = h * (ei * wk);  // delta_s = h'(z_s) * (e w_out^T)
    }
    dwo[k] = d;
  }
  if (t == 0) ((double*)(S + bd.gx_rss))[tile] = ((r_s[0] + r_s[1]) + r_s[2]) + r_s[3];
}

// grid (splits, branches): dW_out and rss of each split, tiles in order
__global__ void __launch_bounds__(256) k_gx_head_red(DevState st, const int32_t* __restrict__ blist, int fuse) {
  const int b = blist[blockIdx.y];
  const BranchDev& bd = st.br[b];
  const int split = blockIdx.x;
  if (split >= bd.nsplits) return;
  const int ntile = (st.nfrag + 3) / 4;
  const int t0 = (int)((int64_t)ntile * split / bd.nsplits), t1 = (int)((int64_t)ntile * (split + 1) / bd.nsplits);
  const float* S = gx_base(st, bd);
  const int Sw = bd.widths[bd.L - 2];
  const double* dwo = (const double*)(S + bd.gx_dwo);
  float* part = st.part + bd.part_off + (int64_t)split * bd.P + bd.woff[bd.L - 1];
  for (int k = threadIdx.x; k < Sw && !gx_lazy_head(bd, fuse); k += 256) {  // lazy: GRAD_s writes dW_out
    double d = 0.0;
    for (int tl = t0; tl < t1; ++tl) d += dwo[(int64_t)tl * Sw + k];
    part[k] = (float)d;
  }
  if (threadIdx.x == 0) {
    const double* rs = (const double*)(S + bd.gx_rss);
    double r = 0.0;
    for (int tl = t0; tl < t1; ++tl) r += rs[tl];
    st.rss_part[(int64_t)b * st.max_splits + split] = r;
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
void launch_gx_prep(const DevState& st, const int32_t* blist, int nb, hipStream_t s) {
  if (nb > 0) hipLaunchKernelGGL(k_gx_prep, dim3(nb, GX_PREP_Y), dim3(256), 0, s, st, blist);
}
static bool gx_exact() {
  const char* ex = getenv("BANN_GX_EXACT");  // 1: every phase on the exact-f32 MFMA path
  return ex && atoi(ex) != 0;
}
void launch_gx_head(const DevState& st, const int32_t* blist, int nb, int max_splits, hipStream_t s) {
  if (nb <= 0) return;
  const int fuse = gx_exact() ? 0 : 1;  // the lazy head pairs with the bf16-plane BWD / GRAD (k_gx_gemm_x3)
  hipLaunchKernelGGL(k_gx_head, dim3((st.nfrag + 3) / 4, nb), dim3(256), 0, s, st, blist, fuse);
  hipLaunchKernelGGL(k_gx_head_red, dim3(max_splits, nb), dim3(256), 0, s, st, blist, fuse);
}
void launch_gx_gemm(const DevState& st, int ph, int l, const int32_t* blist, const int32_t* prefix, int nb,
                    int total, hipStream_t s) {
  if (nb <= 0 || total <= 0) return;
  const int per = (total + 7) / 8;
  const dim3 g(8 * per), blk(256);
  const bool exact = gx_exact();
  if (!exact && ph == GX_FWD0) {
    hipLaunchKernelGGL(k_gx_gemm_b3<GX_FWD0>, g, blk, 0, s, st, blist, prefix, nb, total, per);
    return;
  }
  if (!exact && ph == GX_GRAD0) {
    hipLaunchKernelGGL(k_gx_gemm_b3<GX_GRAD0>, g, blk, 0, s, st, blist, prefix, nb, total, per);
    return;
  }
  if (!exact) {
    switch (ph) {
      case GX_FWD: hipLaunchKernelGGL(k_gx_gemm_x3<GX_FWD>, g, blk, 0, s, st, blist, prefix, nb, l, total, per); return;
      case GX_BWD: hipLaunchKernelGGL(k_gx_gemm_x3<GX_BWD>, g, blk, 0, s, st, blist, prefix, nb, l, total, per); return;
      case GX_GRAD: hipLaunchKernelGGL(k_gx_gemm_x3<GX_GRAD>, g, blk, 0, s, st, blist, prefix, nb, l, total, per); return;
      default: break;
    }
  }
  switch (ph) {
    case GX_FWD0: hipLaunchKernelGGL(k_gx_gemm<GX_FWD0>, g, blk, 0, s, st, blist, prefix, nb, l, total, per); break;
    case GX_FWD: hipLaunchKernelGGL(k_gx_gemm<GX_FWD>, g, blk, 0, s, st, blist, prefix, nb, l, total, per); break;
    case GX_BWD: hipLaunchKernelGGL(k_gx_gemm<GX_BWD>, g, blk, 0, s, st, blist, prefix, nb, l, total, per); break;
    case GX_GRAD: hipLaunchKernelGGL(k_gx_gemm<GX_GRAD>, g, blk, 0, s, st, blist, prefix, nb, l, total, per); break;
    default: hipLaunchKernelGGL(k_gx_gemm<GX_GRAD0>, g, blk, 0, s, st, blist, prefix, nb, l, total, per); break;
  }
}

// tiles of phase (ph, l) for one branch: the numbering of gx_dims above
int64_t gx_tiles(const BranchDev& d, int ph, int l, int32_t nfrag) {
  const int64_t ntile = (nfrag + 3) / 4;
  auto cd = [](int64_t a) { return (a + 63) / 64; };
  const bool x3 = !gx_exact();  // k_gx_gemm_x3's tile shapes (X3Shape), else 64 x 64
  const int64_t tmf = x3 ? 32 * X3Shape<GX_FWD>::AX : 64, tnf = x3 ? 32 * X3Shape<GX_FWD>::AY : 64;
  const int64_t tmb = x3 ? 32 * X3Shape<GX_BWD>::AX : 64, tnb = x3 ? 32 * X3Shape<GX_BWD>::AY : 64;
  const int64_t tmg = x3 ? 32 * X3Shape<GX_GRAD>::AX : 64, tng = x3 ? 32 * X3Shape<GX_GRAD>::AY : 64;
  auto c = [](int64_t a, int64_t e) { return (a + e - 1) / e; };
  switch (ph) {
    case GX_FWD0: return ntile * cd(d.widths[0]);
    case GX_FWD: return (l >= 1 && l < d.L - 1) ? c(64 * ntile, tmf) * c(d.widths[l], tnf) : 0;
    case GX_BWD: return (l >= 1 && l < d.L - 1) ? c(64 * ntile, tmb) * c(d.widths[l - 1], tnb) : 0;
    case GX_GRAD:
      return (l >= 1 && l < d.L - 1) ? c(d.widths[l - 1], tmg) * c(d.widths[l], tng) * d.nsplits : 0;
    default: return (int64_t)d.nchunks * cd(d.widths[0]) * d.nsplits;
  }
}
