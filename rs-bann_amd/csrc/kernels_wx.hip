// kernels_wx.hip — fused gradient kernel for WIDE branches ("wx"): one hidden
// layer (three weight matrices: W0 m x W, W1 W x S, w2 S x 1), W <= 32,
// S <= 32, m <= 128 markers, 2-bit genotypes.  The C5 shape of BASELINE.json
// (W = S = 32) and the reference train-new defaults at small m.
//
// Replaces BranchSampler::backpropagate (branch_sampler.rs:813-875) with its
// forward_feed (743-782) and rss (823-828) for every wide branch of a plan in
// one launch, and writes the same per-slab partials d(rss/2)/d(theta) in
// param_vec order (params.rs:700-715) as the 4-wide fx kernel.
//
// One WAVE owns a 64-individual tile of one branch (like fx); the four waves of
// a workgroup take interleaved tiles of one (branch, split) item and each wave
// writes its OWN partial slab (slab = 4 split + wave), so waves never wait for
// each other after the prologue.  Per tile:
//   1. masked layer forward, exact: Z0 = G (W0/sigma) + c0 on
//      v_mfma_i32_16x16x64_i8 (W0/sigma as 4 signed 7-bit digits per column,
//      8 column blocks of 4; the 2-bit genotype fields are the B operand, kept
//      in place as in fx).  Lane (g, i) ends with Z0[ind 4i+q][col 4mb+g].
//   2. hidden GEMM forward Z1^T = W1^T A0^T on MFMA: that Z0 layout IS the B
//      operand of v_mfma_f32_16x16x4_f32 (K = 4 columns of a block) and, with
//      the K slots of a lane group read as columns 4j+g, of the bf16
//      v_mfma_f32_16x16x32_bf16 -- no lane movement.
//   3. head: A1 = h(Z1 + b1), f = A1 w2 (lane-local + a 4x4 register/lane-group
//      transpose), e = f - y, delta1 = h'(Z1) e w2.
//   4. err0 = delta1 W1^T on MFMA (delta1 is in the accumulator layout, which
//      is again the B operand; the A-operand rows are permuted so the result
//      lands in the Z0 layout), delta0 = h'(Z0) err0.
//   5. dW1 = A0^T delta1 on MFMA (K = individuals): A0^T and delta1^T go through
//      a wave-private LDS image (b128 rows, conflict-free), read back with the
//      individuals on the K slots.
//   6. masked layer backward dW0 = G^T delta0 on v_mfma_i32_16x16x64_i8:
//      delta0 as 4 digits at a per-tile, per-column power-of-two scale (27
//      significant bits), transposed to the fx digit image; the unpacked
//      genotype window is shared by the 8 column blocks; int32 digit sums are
//      converted to f32 once per tile and window.
// FP32 (BF = 0): the hidden GEMMs on v_mfma_f32_16x16x4_f32 (exact f32 fmaf
// chains, the vector rate).  BF16 (BF = 1, opt-in: C5's "bf16 hidden GEMM on
// MFMA vs fp32"): on v_mfma_f32_16x16x32_bf16, 16x the rate, bf16 operand
// rounding (~3e-3 relative on the hidden-layer gradients).
#include "activations.h"
#include "bann_internal.h"
#include "kernel_util.h"

#define WX_WAVES 4
#define WX_MAXCH 2     // <= 128 markers (register budget of the dW0 accumulators)
#define WX_MB 8        // column blocks of 4 (W <= 32)
#define WX_SLOT (WX_MAXCH * 1024)
#define WX_RS 68       // f32 row stride (floats) of the transposed staging images
#define WX_RSH 72      // bf16 row stride (elements)
#define WX_STAGE (32 * WX_RS * 4)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

namespace {

__device__ __forceinline__ float comb4w(v4i d) {  // sum_d D_d 2^(-7 d)
  return (float)d[0] + (float)d[1] * 0x1p-7f + (float)d[2] * 0x1p-14f + (float)d[3] * 0x1p-21f;
}

// signed digits of V = rint(x 2^e), |V| < 2^25 (see kernels_fx.hip digits4_fx)
__device__ __forceinline__ uint32_t digits4_wx(float x, int e) {
  const int V = (int)__builtin_rintf(__builtin_amdgcn_ldexpf(x, e));
  const uint32_t u = (uint32_t)V;
  uint32_t w = __builtin_amdgcn_ubfe(u, 21, 8);
  w |= __builtin_amdgcn_ubfe(u, 14, 7) << 8;
  w |= __builtin_amdgcn_ubfe(u, 7, 7) << 16;
  w |= (u & 127u) << 24;
  return w;
}

__device__ __forceinline__ void swp32(uint32_t& a, uint32_t& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  a = (uint32_t)r[0];
  b = (uint32_t)r[1];
}
__device__ __forceinline__ void swp16(uint32_t& a, uint32_t& b) {
  const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  a = (uint32_t)r[0];
  b = (uint32_t)r[1];
}
// 4x4 transpose between the register index and the lane group (lane >> 4):
// afterwards lane L register k holds what lane (k, L & 15) had in register L >> 4
__device__ __forceinline__ void xpose4(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
  swp32(a, c);
  swp32(b, d);
  swp16(a, b);
  swp16(c, d);
}
__device__ __forceinline__ void xpose4f(float& a, float& b, float& c, float& d) {
  uint32_t x = fbits(a), y = fbits(b), z = fbits(c), w = fbits(d);
  xpose4(x, y, z, w);
  a = __builtin_bit_cast(float, x);
  b = __builtin_bit_cast(float, y);
  c = __builtin_bit_cast(float, z);
  d = __builtin_bit_cast(float, w);
}

// all-reduce over the 16 lanes of a row (DPP; fixed order, result in every lane)
__device__ __forceinline__ float row_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(fbits(v), fbits(v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(fbits(v), fbits(v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(fbits(v), fbits(v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(fbits(v), fbits(v), 0x140, 0xF, 0xF, false));
  return v;
}
__device__ __forceinline__ uint32_t row_max_u(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xF, 0xF, false));
  return v;
}

__device__ __forceinline__ bf16x8 pack8(const float (&v)[8]) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)v[j];
  return r;
}

}  // namespace

template <int ACT, int BF>
__global__ void __launch_bounds__(64 * WX_WAVES, 1)
    k_fused_grad_wx(DevState st, const GradItem* __restrict__ items, int write_pred) {
  __shared__ __attribute__((aligned(16))) char s_w0[WX_MAXCH * WX_MB * 1024];
  __shared__ __attribute__((aligned(16))) char s_x[WX_WAVES][2][WX_SLOT];
  __shared__ __attribute__((aligned(16))) float s_y[WX_WAVES][2][64];
  __shared__ __attribute__((aligned(16))) char s_st[WX_WAVES][2][WX_STAGE];

  const GradItem it = items[blockIdx.x];
  const int b = it.branch;
  const BranchDev& bd = st.br[b];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i = lane & 15;
  const int nch = bd.nchunks;
  const int m = bd.m, w0 = bd.widths[0], S = bd.widths[1];
  const int64_t n = st.n;
  const int tb = it.frag_begin >> 2, te = (it.frag_end + 3) >> 2;
  const float* th = st.theta + bd.p_off;

  // ---- prologue: W0 digit image -> LDS (shared by the four waves) ----
  for (int t = threadIdx.x; t < nch * WX_MB * 64; t += 64 * WX_WAVES)
    *reinterpret_cast<v4i*>(&s_w0[t * 16]) = *reinterpret_cast<const v4i*>(st.dig + bd.dig_off + (int64_t)t * 16);

  // per-lane constants (zero outside the real widths: padded units stay exactly 0)
  float zs[WX_MB], c0v[WX_MB];
#pragma unroll
  for (int mb = 0; mb < WX_MB; ++mb) {
    const int c = 4 * mb + g;
    zs[mb] = c < w0 ? st.fc[b].scale[c] : 0.f;
    c0v[mb] = c < w0 ? st.fc[b].c0[c] : 0.f;
  }
  float b1v[2][4], w2v[2][4];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int s = 16 * nb + 4 * g + r;
      b1v[nb][r] = s < S ? th[bd.boff[1] + s] : 0.f;
      w2v[nb][r] = s < S ? th[bd.woff[2] + s] : 0.f;
    }
  auto W1at = [&](int c, int s) { return (c < w0 && s < S) ? th[bd.woff[1] + s * w0 + c] : 0.f; };
  // hidden-GEMM operand images of W1 (see the header comment for the maps)
  float wf[2][WX_MB], we[2][2][4];
  bf16x8 wfb[2], web[2];
  if constexpr (BF) {
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = W1at(4 * j + g, 16 * nb + i);
      wfb[nb] = pack8(v);
    }
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = W1at(4 * (4 * cb + (i & 3)) + (i >> 2), 16 * (j >> 2) + 4 * g + (j & 3));
      web[cb] = pack8(v);
    }
  } else {
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int mb = 0; mb < WX_MB; ++mb) wf[nb][mb] = W1at(4 * mb + g, 16 * nb + i);
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int r = 0; r < 4; ++r) we[cb][nb][r] = W1at(4 * (4 * cb + (i & 3)) + (i >> 2), 16 * nb + 4 * g + r);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- per-lane LDS offsets (the fx image conventions) ----
  const int tq = i >> 1, tp = lane & 1, gsw = g & 1;
  const uint32_t fo0 = (uint32_t)((16 * g + tq + 8 * gsw) * 16 + 8 * (tp ^ gsw));
  const uint32_t fo1 = (uint32_t)((16 * g + tq + 8 * (1 ^ gsw)) * 16 + 8 * (tp ^ 1 ^ gsw));
  const int pe = i, po = (i + 8) & 15;
  const uint32_t boe = (uint32_t)(pe * 16 + 4 * (2 * ((g >> 1) ^ (pe >> 3)) + (g & 1)));
  const uint32_t boo = (uint32_t)(po * 16 + 4 * (2 * ((g >> 1) ^ (po >> 3)) + (g & 1)));
  const int iota = 4 * i + g;  // this lane's own individual within the tile
  char* const sA = &s_st[wave][0][0];  // A0^T staging, later the delta0 digit image
  char* const sD = &s_st[wave][1][0];  // delta1^T staging
  char* const sd_w = sA + (i >> 2) * 256 + (4 * g + (i & 3)) * 16;
  const char* const sd_r = sA + g * 256 + tq * 16 + 8 * tp;
  const float* ybr = st.y + bd.y_off;
  float* predb = st.pred + bd.y_off;
  const char* xsrc = reinterpret_cast<const char*>(st.xu2) + bd.x_off + lane * 16;
  const int64_t tile_bytes = (int64_t)nch * 1024;
  auto issue_chunk = [&](int tt, int sl, int c) {
    glds16(xsrc + (int64_t)tt * tile_bytes + c * 1024, &s_x[wave][sl][c * 1024]);
  };
  auto issue_y = [&](int tt, int sl) {
    const int64_t row = 64 * (int64_t)tt + iota;
    glds4(ybr + (row < n ? row : n - 1), &s_y[wave][sl][0]);
  };

  // ---- accumulators ----
  float dW0a[4 * WX_MAXCH][WX_MB];
#pragma unroll
  for (int u = 0; u < 4 * WX_MAXCH; ++u)
#pragma unroll
    for (int mb = 0; mb < WX_MB; ++mb) dW0a[u][mb] = 0.f;
  float db0a[WX_MB], db1a[2][4], dW2a[2][4];
  v4f dW1a[2][2];
#pragma unroll
  for (int mb = 0; mb < WX_MB; ++mb) db0a[mb] = 0.f;
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int r = 0; r < 4; ++r) db1a[nb][r] = dW2a[nb][r] = 0.f;
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) dW1a[cb][sb] = v4f{0.f, 0.f, 0.f, 0.f};
  double rss = 0.0;

  int tt = tb + wave, sl = 0;
  if (tt < te) {
    for (int c = 0; c < nch; ++c) issue_chunk(tt, 0, c);
    issue_y(tt, 0);
  }
  for (; tt < te; tt += WX_WAVES, sl ^= 1) {
    const bool more = tt + WX_WAVES < te;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const char* xs = &s_x[wave][sl][0];

    // ---- 1. masked layer forward (exact int32 over the chunks) ----
    float z0[WX_MB][4], a0[WX_MB][4];
    {
      v4i fa[WX_MB][4];
#pragma unroll
      for (int mb = 0; mb < WX_MB; ++mb)
#pragma unroll
        for (int q = 0; q < 4; ++q) fa[mb][q] = v4i{0, 0, 0, 0};
#pragma unroll
      for (int c = 0; c < WX_MAXCH; ++c) {
        if (c < nch) {
          if (more) issue_chunk(tt + WX_WAVES, sl ^ 1, c);
          const v4u X = (v4u)lds_tr8_pair(xs + c * 1024 + fo0, xs + c * 1024 + fo1);
          const v4i B0 = (v4i)(X & 0x03030303u);
          const v4i B1 = (v4i)(X & 0x0C0C0C0Cu);
          const v4i B2 = (v4i)(X & 0x30303030u);
          const v4i B3 = (v4i)((X >> 2u) & 0x30303030u);
#pragma unroll
          for (int mb = 0; mb < WX_MB; ++mb) {
            const v4i A = *reinterpret_cast<const v4i*>(&s_w0[((c * WX_MB + mb) * 64 + lane) * 16]);
            fa[mb][0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B0, fa[mb][0], 0, 0, 0);
            fa[mb][1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B1, fa[mb][1], 0, 0, 0);
            fa[mb][2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B2, fa[mb][2], 0, 0, 0);
            fa[mb][3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B3, fa[mb][3], 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int mb = 0; mb < WX_MB; ++mb) {
        z0[mb][0] = zs[mb] * comb4w(fa[mb][0]) + c0v[mb];
        z0[mb][1] = (0.25f * zs[mb]) * comb4w(fa[mb][1]) + c0v[mb];
        z0[mb][2] = (0.0625f * zs[mb]) * comb4w(fa[mb][2]) + c0v[mb];
        z0[mb][3] = (0.0625f * zs[mb]) * comb4w(fa[mb][3]) + c0v[mb];
#pragma unroll
        for (int q = 0; q < 4; ++q) a0[mb][q] = act_h_t<ACT>(z0[mb][q]);
      }
    }
    // A0^T -> LDS rows c = 4mb + g, individuals 4i .. 4i+3
#pragma unroll
    for (int mb = 0; mb < WX_MB; ++mb) {
      if constexpr (BF) {
        bf16x4 h4 = {(__bf16)a0[mb][0], (__bf16)a0[mb][1], (__bf16)a0[mb][2], (__bf16)a0[mb][3]};
        *reinterpret_cast<bf16x4*>(sA + ((4 * mb + g) * WX_RSH + 4 * i) * 2) = h4;
      } else {
        *reinterpret_cast<v4f*>(sA + ((4 * mb + g) * WX_RS + 4 * i) * 4) =
            v4f{a0[mb][0], a0[mb][1], a0[mb][2], a0[mb][3]};
      }
    }

    // ---- 2. hidden GEMM forward: Z1^T = W1^T A0^T ----
    v4f z1[2][4];
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v4f acc = v4f{0.f, 0.f, 0.f, 0.f};
        if constexpr (BF) {
          float v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = a0[j][q];
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfb[nb], pack8(v), acc, 0, 0, 0);
        } else {
#pragma unroll
          for (int mb = 0; mb < WX_MB; ++mb) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[nb][mb], a0[mb][q], acc, 0, 0, 0);
        }
        z1[nb][q] = acc;
      }

    // ---- 3. head ----
    float a1[2][4][4];
    float p[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) p[q] = 0.f;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          z1[nb][q][r] += b1v[nb][r];
          a1[nb][q][r] = act_h_t<ACT>(z1[nb][q][r]);
          p[q] = fmaf(a1[nb][q][r], w2v[nb][r], p[q]);
        }
    xpose4f(p[0], p[1], p[2], p[3]);  // lane L: partials of individual 4i + (L >> 4) from the 4 groups
    const float out = (p[0] + p[1]) + (p[2] + p[3]);
    const int64_t row = 64 * (int64_t)tt + iota;
    const bool valid = row < n;
    const float yv = s_y[wave][sl][lane];
    if (more) issue_y(tt + WX_WAVES, sl ^ 1);
    const float e = valid ? out - yv : 0.f;
    if (write_pred && valid) predb[row] = out;
    rss += (double)e * (double)e;
    float eq[4] = {e, e, e, e};
    xpose4f(eq[0], eq[1], eq[2], eq[3]);  // eq[q] = e of individual 4i + q
    float d1[2][4][4];
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float sw = 0.f, sd = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          d1[nb][q][r] = act_dh_t<ACT>(z1[nb][q][r], a1[nb][q][r]) * (eq[q] * w2v[nb][r]);
          sw = fmaf(a1[nb][q][r], eq[q], sw);
          sd += d1[nb][q][r];
        }
        dW2a[nb][r] += sw;
        db1a[nb][r] += sd;
        // delta1^T -> LDS row s = 16 nb + 4 g + r, individuals 4i .. 4i+3
        if constexpr (BF) {
          bf16x4 h4 = {(__bf16)d1[nb][0][r], (__bf16)d1[nb][1][r], (__bf16)d1[nb][2][r], (__bf16)d1[nb][3][r]};
          *reinterpret_cast<bf16x4*>(sD + ((16 * nb + 4 * g + r) * WX_RSH + 4 * i) * 2) = h4;
        } else {
          *reinterpret_cast<v4f*>(sD + ((16 * nb + 4 * g + r) * WX_RS + 4 * i) * 4) =
              v4f{d1[nb][0][r], d1[nb][1][r], d1[nb][2][r], d1[nb][3][r]};
        }
      }

    // ---- 4. err0 = delta1 W1^T (result in the Z0 layout), delta0 ----
    float d0[WX_MB][4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        v4f acc = v4f{0.f, 0.f, 0.f, 0.f};
        if constexpr (BF) {
          float v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = d1[j >> 2][q][j & 3];
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(web[cb], pack8(v), acc, 0, 0, 0);
        } else {
#pragma unroll
          for (int nb = 0; nb < 2; ++nb)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              acc = __builtin_amdgcn_mfma_f32_16x16x4f32(we[cb][nb][r], d1[nb][q][r], acc, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int mb = 4 * cb + r;
          d0[mb][q] = act_dh_t<ACT>(z0[mb][q], a0[mb][q]) * acc[r];
        }
      }
#pragma unroll
    for (int mb = 0; mb < WX_MB; ++mb) db0a[mb] += (d0[mb][0] + d0[mb][1]) + (d0[mb][2] + d0[mb][3]);

    // ---- 5. dW1 = A0^T delta1 (K = individuals, from the LDS images) ----
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        if constexpr (BF) {
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            const bf16x8 A = *reinterpret_cast<const bf16x8*>(sA + ((16 * cb + i) * WX_RSH + 32 * ks + 8 * g) * 2);
            const bf16x8 B = *reinterpret_cast<const bf16x8*>(sD + ((16 * sb + i) * WX_RSH + 32 * ks + 8 * g) * 2);
            dW1a[cb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, B, dW1a[cb][sb], 0, 0, 0);
          }
        } else {
#pragma unroll
          for (int t4 = 0; t4 < 4; ++t4) {
            const v4f A = *reinterpret_cast<const v4f*>(sA + ((16 * cb + i) * WX_RS + 16 * g + 4 * t4) * 4);
            const v4f B = *reinterpret_cast<const v4f*>(sD + ((16 * sb + i) * WX_RS + 16 * g + 4 * t4) * 4);
#pragma unroll
            for (int e4 = 0; e4 < 4; ++e4)
              dW1a[cb][sb] = __builtin_amdgcn_mfma_f32_16x16x4f32(A[e4], B[e4], dW1a[cb][sb], 0, 0, 0);
          }
        }
      }

    // ---- 6. delta0 digits (per-tile, per-column scale), masked layer backward ----
    int R[WX_MB];
#pragma unroll
    for (int mb = 0; mb < WX_MB; ++mb) {
      const uint32_t mx = row_max_u(max(max(fbits(d0[mb][0]) & 0x7FFFFFFFu, fbits(d0[mb][1]) & 0x7FFFFFFFu),
                                        max(fbits(d0[mb][2]) & 0x7FFFFFFFu, fbits(d0[mb][3]) & 0x7FFFFFFFu)));
      R[mb] = (int)((mx >> 23) & 0xFFu) + 2;  // |delta0| < 2^(R - 128): digits carry 27 bits
      uint32_t dq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) dq[q] = digits4_wx(d0[mb][q], 153 - R[mb]);
      xpose4(dq[0], dq[1], dq[2], dq[3]);  // lane L: the 4 columns of block mb for individual iota
      // (the A0^T image in sA was consumed by step 5 above: in-order LDS per wave)
      *reinterpret_cast<v4u*>(sd_w + mb * 1024) = v4u{dq[0], dq[1], dq[2], dq[3]};
    }
    v4i Ab[WX_MB];
#pragma unroll
    for (int mb = 0; mb < WX_MB; ++mb) Ab[mb] = lds_tr8_pair(sd_r + mb * 1024, sd_r + mb * 1024 + 8 * 16);
#pragma unroll
    for (int u = 0; u < 4 * WX_MAXCH; ++u) {
      if (u < 4 * nch) {
        const uint32_t wv = *reinterpret_cast<const uint32_t*>(xs + 256 * u + ((u & 1) ? boo : boe));
        const v4i Bv = v4i{(int)(wv & 0x03030303u), (int)((wv >> 2) & 0x03030303u), (int)((wv >> 4) & 0x03030303u),
                           (int)((wv >> 6) & 0x03030303u)};
#pragma unroll
        for (int mb = 0; mb < WX_MB; ++mb) {
          const v4i t = __builtin_amdgcn_mfma_i32_16x16x64_i8(Ab[mb], Bv, v4i{0, 0, 0, 0}, 0, 0, 0);
          dW0a[u][mb] = fmaf(comb4w(t), __builtin_amdgcn_ldexpf(1.f, R[mb] - 132), dW0a[u][mb]);
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- epilogue: this wave's own partial slab (no cross-wave reduction) ----
  const int slab = wave;  // the item's 4 slabs: one per wave
  float* part = st.part + it.part_at + (int64_t)slab * bd.P;
  float db0[WX_MB];
#pragma unroll
  for (int mb = 0; mb < WX_MB; ++mb) db0[mb] = row_sum(db0a[mb]);
#pragma unroll
  for (int u = 0; u < 4 * WX_MAXCH; ++u) {
    const int j = 16 * u + i;
    if (u < 4 * nch && j < m) {
      const float mu = st.mu[bd.mk_off + j], sg = st.sigma[bd.mk_off + j];
#pragma unroll
      for (int mb = 0; mb < WX_MB; ++mb) {
        const int c = 4 * mb + g;
        if (c < w0) part[bd.woff[0] + c * m + j] = sg > 0.f ? (dW0a[u][mb] - mu * db0[mb]) / sg : 0.f;
      }
    }
  }
  if (i == 0) {
#pragma unroll
    for (int mb = 0; mb < WX_MB; ++mb)
      if (4 * mb + g < w0) part[bd.boff[0] + 4 * mb + g] = db0[mb];
  }
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int sb = 0; sb < 2; ++sb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = 16 * cb + 4 * g + r, s = 16 * sb + i;
        if (c < w0 && s < S) part[bd.woff[1] + s * w0 + c] = dW1a[cb][sb][r];
      }
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int s = 16 * nb + 4 * g + r;
      const float v1 = row_sum(db1a[nb][r]), v2 = row_sum(dW2a[nb][r]);
      if (i == 0 && s < S) {
        part[bd.boff[1] + s] = v1;
        part[bd.woff[2] + s] = v2;
      }
    }
  const double rs = wave_sum_d(rss);
  if (lane == 0) st.rss_part[it.rss_at + slab] = rs;
}

template <int BF>
static void launch_wx_bf(const DevState& st, const GradItem* items, int32_t nitems, int act, int wp, hipStream_t s) {
  const dim3 grid((unsigned)nitems), block(64 * WX_WAVES);
  switch (act) {
    case 0: hipLaunchKernelGGL((k_fused_grad_wx<0, BF>), grid, block, 0, s, st, items, wp); break;
    case 1: hipLaunchKernelGGL((k_fused_grad_wx<1, BF>), grid, block, 0, s, st, items, wp); break;
    case 2: hipLaunchKernelGGL((k_fused_grad_wx<2, BF>), grid, block, 0, s, st, items, wp); break;
    case 3: hipLaunchKernelGGL((k_fused_grad_wx<3, BF>), grid, block, 0, s, st, items, wp); break;
    default: hipLaunchKernelGGL((k_fused_grad_wx<4, BF>), grid, block, 0, s, st, items, wp); break;
  }
}

void launch_fused_grad_wx(const DevState& st, const GradItem* items, int32_t nitems, int32_t act, int bf16,
                          int write_pred, hipStream_t s) {
  if (nitems <= 0) return;
  if (bf16) launch_wx_bf<1>(st, items, nitems, act, write_pred, s);
  else launch_wx_bf<0>(st, items, nitems, act, write_pred, s);
}
