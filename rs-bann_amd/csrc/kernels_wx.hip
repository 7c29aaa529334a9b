// kernels_wx.hip — fused gradient kernel for WIDE branches ("wx"): one hidden
// layer (three weight matrices: W0 m x W, W1 W x S, w2 S x 1), W <= 32,
// S <= 32, m <= 128 markers, 2-bit genotypes.  The C5 shape of BASELINE.json
// (W = S = 32) and the reference train-new defaults at small m.
//
// Replaces BranchSampler::backpropagate (branch_sampler.rs:813-875) with its
// forward_feed (743-782) and rss (823-828) for every wide branch of a plan in
// one launch, and writes the same per-split partials d(rss/2)/d(theta) in
// param_vec order (params.rs:700-715) as the 4-wide fx kernel.
//
// One workgroup = TWO waves that share each 64-individual tile of one (branch,
// split) item; wave h owns half of every layer: hidden units c in [16h, 16h+16)
// (column blocks mb = 4h .. 4h+3) and summary units s in [16h, 16h+16).  Half
// the accumulators and operand images per wave keep a wave under 256 registers,
// so two waves share a SIMD and one wave's VALU phases (activations, digits,
// conversions) run beside the other's MFMA chains.  Per tile:
//   1. masked layer forward, exact, own columns: Z0 = G (W0/sigma) + c0 on
//      v_mfma_i32_16x16x64_i8 (W0/sigma as 4 signed 7-bit digits per column,
//      the 2-bit genotype fields as the B operand, kept in place as in fx).
//      Lane (g, i) ends with Z0[ind 4i+q][col 4mb+g].  A0 = h(Z0) -> the A0^T
//      image in LDS (rows = hidden units).                          barrier
//   2. hidden GEMM, own summary units: Z1^T = W1^T A0^T on
//      v_mfma_f32_16x16x4_f32 (K = the 32 hidden units, read from the A0^T
//      image) or v_mfma_f32_16x16x32_bf16 (opt-in).
//   3. head: A1 = h(Z1 + b1), the output's partial sum over own units -> LDS;
//                                                                barrier
//      f = partial_0 + partial_1 (same order in both waves), e = f - y,
//      delta1 = h'(Z1) e w2 (own units) -> the delta1^T image.       barrier
//   4. err0 = delta1 W1^T for own hidden units on MFMA (K = all 32 summary
//      units from the delta1^T image; A-operand rows permuted so the result
//      lands in the Z0 layout), delta0 = h'(Z0) err0.
//   5. dW1 (own hidden rows) = A0^T delta1 on MFMA (K = individuals).
//   6. masked layer backward, own columns: dW0 = G^T delta0 on
//      v_mfma_i32_16x16x64_i8, delta0 as 4 digits at a per-tile, per-column
//      power-of-two scale (27 significant bits); the digit image overwrites the
//      wave's own A0^T rows (no other wave reads them after the first barrier).
// The two waves write disjoint parts of the item's one partial slab.
// FP32 (BF = 0, BANN_WX_EXACT=1): the hidden GEMMs on v_mfma_f32_16x16x4_f32
// (exact f32 fmaf chains, the vector rate).  BF16 (BF = 1, opt-in: C5's "bf16
// hidden GEMM on MFMA vs fp32"): on v_mfma_f32_16x16x32_bf16, 16x the rate,
// bf16 operand rounding (~3e-3 relative on the hidden-layer gradients).
// The default wide kernel is k_fused_grad_wx3 below: the same phases with the
// hidden GEMMs on the bf16 MFMA at f32 accuracy (three planes per operand).
#include "activations.h"
#include "bann_internal.h"
#include "kernel_util.h"

#define WX_WAVES 2     // waves per workgroup (the two halves of a tile)
#define WX_MAXCH 2     // <= 128 markers
#define WX_MB 8        // column blocks of 4 (W <= 32)
#define WX_SLOT (WX_MAXCH * 1024)
#define WX_RS 68       // f32 row stride (floats) of the transposed images
#define WX_RSH 72      // bf16 row stride (elements)
#define WX_IMG (32 * WX_RS * 4)  // bytes of one 32-row transposed image

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

namespace {

// 2^7 sum_d D_d 2^(-7 d) from the digit sums of one tile (|D| < 2^19): the
// pairs D0 2^7 + D1 and D2 2^7 + D3 are exact in int32, two conversions
__device__ __forceinline__ float comb4p(v4i d) {
  return (float)((d[0] << 7) + d[1]) + (float)((d[2] << 7) + d[3]) * 0x1p-14f;
}

// signed digits of V = rint(x 2^e), |V| < 2^27 (see kernels_fx.hip digits4_fx)
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
// element q of eight bf16x4 rows as one bf16x8 operand (the K slots j = 0..7)
__device__ __forceinline__ bf16x8 gather8(const bf16x4 (&r)[8], int q) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = r[j][q];
  return o;
}

}  // namespace

template <int ACT, int BF>
__global__ void __launch_bounds__(64 * WX_WAVES, 2)
    k_fused_grad_wx(DevState st, const GradItem* __restrict__ items, int write_pred) {
  __shared__ __attribute__((aligned(16))) char s_w0[WX_MAXCH * WX_MB * 1024];  // W0/sigma digits, all columns
  __shared__ __attribute__((aligned(16))) char s_x[2][WX_SLOT];               // tile images (double-buffered)
  __shared__ __attribute__((aligned(16))) float s_y[2][64];
  __shared__ __attribute__((aligned(16))) char s_a[WX_IMG];   // A0^T (rows = hidden units), then delta0 digits
  __shared__ __attribute__((aligned(16))) char s_d[WX_IMG];   // delta1^T (rows = summary units)
  __shared__ __attribute__((aligned(16))) float s_po[2][64];  // the output's partial sum of each half

  const GradItem it = items[blockIdx.x];
  const int b = it.branch;
  const BranchDev& bd = st.br[b];
  const int h = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // this wave's half
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i = lane & 15;
  const int nch = bd.nchunks;
  const int m = bd.m, w0 = bd.widths[0], S = bd.widths[1];
  const int64_t n = st.n;
  const int tb = it.frag_begin >> 2, te = (it.frag_end + 3) >> 2;
  const float* th = st.theta + bd.p_off;

  // ---- prologue: W0 digit image -> LDS ----
  for (int t = threadIdx.x; t < nch * WX_MB * 64; t += 64 * WX_WAVES)
    *reinterpret_cast<v4i*>(&s_w0[t * 16]) = *reinterpret_cast<const v4i*>(st.dig + bd.dig_off + (int64_t)t * 16);

  // per-lane constants of this half (zero outside the real widths: padded units stay exactly 0)
  float zs[4], c0v[4], b1v[4], w2v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = 4 * (4 * h + k) + g;  // own hidden unit of column block 4h + k
    zs[k] = c < w0 ? st.fc[b].scale[c] : 0.f;
    c0v[k] = c < w0 ? st.fc[b].c0[c] : 0.f;
    const int s = 16 * h + 4 * g + k;   // own summary unit of register k
    b1v[k] = s < S ? th[bd.boff[1] + s] : 0.f;
    w2v[k] = s < S ? th[bd.woff[2] + s] : 0.f;
  }
  auto W1at = [&](int c, int s) { return (c < w0 && s < S) ? th[bd.woff[1] + s * w0 + c] : 0.f; };
  // hidden-GEMM operands: wf = W1^T rows of own summary units (K = hidden unit
  // 4 mb + g); we = W1 rows permuted so err0 lands in the Z0 layout of own blocks
  float wf[WX_MB], we[2][4];
  bf16x8 wfb, web;
  if constexpr (BF) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = W1at(4 * j + g, 16 * h + i);
    wfb = pack8(v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = W1at(4 * (4 * h + (i & 3)) + (i >> 2), 16 * (j >> 2) + 4 * g + (j & 3));
    web = pack8(v);
  } else {
#pragma unroll
    for (int mb = 0; mb < WX_MB; ++mb) wf[mb] = W1at(4 * mb + g, 16 * h + i);
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) we[nb][r] = W1at(4 * (4 * h + (i & 3)) + (i >> 2), 16 * nb + 4 * g + r);
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
  const int iota = 4 * i + g;  // this lane's own individual within the tile (head)
  // delta0 digit image (4 KiB): f32 mode -- the wave's own A0^T rows (hidden units
  // 16h .. 16h+15, which only this wave reads after the A0^T barrier); bf16 mode --
  // behind the half-size bf16 images (wave 0 in s_a, wave 1 in s_d)
  char* const sdig = BF ? (h == 0 ? s_a : s_d) + 32 * WX_RSH * 2 : s_a + 16 * h * WX_RS * 4;
  char* const sd_w = sdig + (i >> 2) * 256 + (4 * g + (i & 3)) * 16;
  const char* const sd_r = sdig + g * 256 + tq * 16 + 8 * tp;
  const float* ybr = st.y + bd.y_off;
  float* predb = st.pred + bd.y_off;
  const char* xsrc = reinterpret_cast<const char*>(st.xu2) + bd.x_off + lane * 16;
  const int64_t tile_bytes = (int64_t)nch * 1024;
  // wave h streams chunk h of the next tile (and wave 0 its targets)
  auto issue_tile = [&](int tt, int sl) {
    if (h < nch) glds16(xsrc + (int64_t)tt * tile_bytes + h * 1024, &s_x[sl][h * 1024]);
    if (h == 0) {
      const int64_t row = 64 * (int64_t)tt + iota;
      glds4(ybr + (row < n ? row : n - 1), &s_y[sl][0]);
    }
  };

  // ---- accumulators (own half) ----
  float dW0a[4 * WX_MAXCH][4];
#pragma unroll
  for (int u = 0; u < 4 * WX_MAXCH; ++u)
#pragma unroll
    for (int k = 0; k < 4; ++k) dW0a[u][k] = 0.f;
  float db0a[4], db1a[4], dW2a[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) db0a[k] = db1a[k] = dW2a[k] = 0.f;
  v4f dW1a[2] = {v4f{0.f, 0.f, 0.f, 0.f}, v4f{0.f, 0.f, 0.f, 0.f}};
  double rss = 0.0;

  int tt = tb, sl = 0;
  if (tt < te) issue_tile(tt, 0);
  for (; tt < te; ++tt, sl ^= 1) {
    const bool more = tt + 1 < te;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // both chunks and the targets landed; the previous tile's images are consumed
    if (more) issue_tile(tt + 1, sl ^ 1);
    const char* xs = &s_x[sl][0];

    // ---- 1. masked layer forward, own column blocks (exact int32 over the chunks) ----
    float z0[4][4], a0[4][4];
    {
      v4i fa[4][4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int q = 0; q < 4; ++q) fa[k][q] = v4i{0, 0, 0, 0};
#pragma unroll
      for (int c = 0; c < WX_MAXCH; ++c) {
        if (c < nch) {
          const v4u X = (v4u)lds_tr8_pair(xs + c * 1024 + fo0, xs + c * 1024 + fo1);
          const v4i B0 = (v4i)(X & 0x03030303u);
          const v4i B1 = (v4i)(X & 0x0C0C0C0Cu);
          const v4i B2 = (v4i)(X & 0x30303030u);
          const v4i B3 = (v4i)((X >> 2u) & 0x30303030u);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const v4i A = *reinterpret_cast<const v4i*>(&s_w0[((c * WX_MB + 4 * h + k) * 64 + lane) * 16]);
            fa[k][0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B0, fa[k][0], 0, 0, 0);
            fa[k][1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B1, fa[k][1], 0, 0, 0);
            fa[k][2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B2, fa[k][2], 0, 0, 0);
            fa[k][3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B3, fa[k][3], 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        // comb4p carries 2^7; fields 1-3 stay in place (x 4, x 16, x 16)
        z0[k][0] = (0x1p-7f * zs[k]) * comb4p(fa[k][0]) + c0v[k];
        z0[k][1] = (0x1p-9f * zs[k]) * comb4p(fa[k][1]) + c0v[k];
        z0[k][2] = (0x1p-11f * zs[k]) * comb4p(fa[k][2]) + c0v[k];
        z0[k][3] = (0x1p-11f * zs[k]) * comb4p(fa[k][3]) + c0v[k];
#pragma unroll
        for (int q = 0; q < 4; ++q) a0[k][q] = act_h_t<ACT>(z0[k][q]);
      }
    }
    // own A0^T rows c = 4 (4h + k) + g, individuals 4i .. 4i+3
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = 4 * (4 * h + k) + g;
      if constexpr (BF) {
        bf16x4 h4 = {(__bf16)a0[k][0], (__bf16)a0[k][1], (__bf16)a0[k][2], (__bf16)a0[k][3]};
        *reinterpret_cast<bf16x4*>(s_a + (c * WX_RSH + 4 * i) * 2) = h4;
      } else {
        *reinterpret_cast<v4f*>(s_a + (c * WX_RS + 4 * i) * 4) = v4f{a0[k][0], a0[k][1], a0[k][2], a0[k][3]};
      }
    }
    LDS_BARRIER();  // the full A0^T image

    // ---- 2. hidden GEMM, own summary units: Z1^T = W1^T A0^T (K = 32 hidden units) ----
    v4f z1[4];
    if constexpr (BF) {
      bf16x4 ra[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) ra[j] = *reinterpret_cast<const bf16x4*>(s_a + ((4 * j + g) * WX_RSH + 4 * i) * 2);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        z1[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfb, gather8(ra, q), v4f{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    } else {
      v4f ra[WX_MB];
#pragma unroll
      for (int mb = 0; mb < WX_MB; ++mb) ra[mb] = *reinterpret_cast<const v4f*>(s_a + ((4 * mb + g) * WX_RS + 4 * i) * 4);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v4f acc = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int mb = 0; mb < WX_MB; ++mb) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[mb], ra[mb][q], acc, 0, 0, 0);
        z1[q] = acc;
      }
    }

    // ---- 3. head: lane (g, i) register r of z1[q] = Z1[s = 16h + 4g + r][ind 4i + q] ----
    float a1[4][4], p[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      p[q] = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        z1[q][r] += b1v[r];
        a1[q][r] = act_h_t<ACT>(z1[q][r]);
        p[q] = fmaf(a1[q][r], w2v[r], p[q]);
      }
    }
    xpose4f(p[0], p[1], p[2], p[3]);  // lane L: partials of individual iota from the 4 groups
    s_po[h][lane] = (p[0] + p[1]) + (p[2] + p[3]);
    LDS_BARRIER();  // both halves' partial outputs
    const float out = s_po[0][lane] + s_po[1][lane];
    const int64_t row = 64 * (int64_t)tt + iota;
    const bool valid = row < n;
    const float yv = s_y[sl][lane];
    const float e = valid ? out - yv : 0.f;
    if (h == 0 && write_pred && valid) predb[row] = out;
    rss += (double)e * (double)e;
    float eq[4] = {e, e, e, e};
    xpose4f(eq[0], eq[1], eq[2], eq[3]);  // eq[q] = e of individual 4i + q
    float d1[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float sw = 0.f, sd = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        d1[q][r] = act_dh_t<ACT>(z1[q][r], a1[q][r]) * (eq[q] * w2v[r]);
        sw = fmaf(a1[q][r], eq[q], sw);
        sd += d1[q][r];
      }
      dW2a[r] += sw;
      db1a[r] += sd;
      // delta1^T row s = 16h + 4g + r, individuals 4i .. 4i+3
      const int s = 16 * h + 4 * g + r;
      if constexpr (BF) {
        bf16x4 h4 = {(__bf16)d1[0][r], (__bf16)d1[1][r], (__bf16)d1[2][r], (__bf16)d1[3][r]};
        *reinterpret_cast<bf16x4*>(s_d + (s * WX_RSH + 4 * i) * 2) = h4;
      } else {
        *reinterpret_cast<v4f*>(s_d + (s * WX_RS + 4 * i) * 4) = v4f{d1[0][r], d1[1][r], d1[2][r], d1[3][r]};
      }
    }
    LDS_BARRIER();  // the full delta1^T image

    // ---- 4. err0 = delta1 W1^T for own hidden units (result in the Z0 layout), delta0 ----
    float d0[4][4];
    {
      v4f acc[4];
      if constexpr (BF) {
        bf16x4 rd[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          rd[j] = *reinterpret_cast<const bf16x4*>(s_d + ((16 * (j >> 2) + 4 * g + (j & 3)) * WX_RSH + 4 * i) * 2);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(web, gather8(rd, q), v4f{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      } else {
        v4f rd[2][4];
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            rd[nb][r] = *reinterpret_cast<const v4f*>(s_d + ((16 * nb + 4 * g + r) * WX_RS + 4 * i) * 4);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v4f a = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int nb = 0; nb < 2; ++nb)
#pragma unroll
            for (int r = 0; r < 4; ++r) a = __builtin_amdgcn_mfma_f32_16x16x4f32(we[nb][r], rd[nb][r][q], a, 0, 0, 0);
          acc[q] = a;
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int k = 0; k < 4; ++k) d0[k][q] = act_dh_t<ACT>(z0[k][q], a0[k][q]) * acc[q][k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) db0a[k] += (d0[k][0] + d0[k][1]) + (d0[k][2] + d0[k][3]);

    // ---- 5. dW1 rows c = 16h + 4g + r: A0^T delta1 (K = individuals, from the images) ----
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) {
      if constexpr (BF) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 A = *reinterpret_cast<const bf16x8*>(s_a + ((16 * h + i) * WX_RSH + 32 * ks + 8 * g) * 2);
          const bf16x8 B = *reinterpret_cast<const bf16x8*>(s_d + ((16 * sb + i) * WX_RSH + 32 * ks + 8 * g) * 2);
          dW1a[sb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, B, dW1a[sb], 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int t4 = 0; t4 < 4; ++t4) {
          const v4f A = *reinterpret_cast<const v4f*>(s_a + ((16 * h + i) * WX_RS + 16 * g + 4 * t4) * 4);
          const v4f B = *reinterpret_cast<const v4f*>(s_d + ((16 * sb + i) * WX_RS + 16 * g + 4 * t4) * 4);
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4) dW1a[sb] = __builtin_amdgcn_mfma_f32_16x16x4f32(A[e4], B[e4], dW1a[sb], 0, 0, 0);
        }
      }
    }

    // ---- 6. delta0 digits (per-tile, per-column scale) over the own A0^T rows, masked backward ----
    float sc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t mx = row_max_u(max(max(fbits(d0[k][0]) & 0x7FFFFFFFu, fbits(d0[k][1]) & 0x7FFFFFFFu),
                                        max(fbits(d0[k][2]) & 0x7FFFFFFFu, fbits(d0[k][3]) & 0x7FFFFFFFu)));
      const int R = (int)((mx >> 23) & 0xFFu) + 2;  // |delta0| < 2^(R - 128): digits carry 27 bits
      sc[k] = __builtin_amdgcn_ldexpf(1.f, R - 139);  // comb4p carries 2^7
      uint32_t dq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) dq[q] = digits4_wx(d0[k][q], 153 - R);
      xpose4(dq[0], dq[1], dq[2], dq[3]);  // lane L: the 4 columns of block 4h + k for individual iota
      *reinterpret_cast<v4u*>(sd_w + k * 1024) = v4u{dq[0], dq[1], dq[2], dq[3]};
    }
    v4i Ab[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) Ab[k] = lds_tr8_pair(sd_r + k * 1024, sd_r + k * 1024 + 8 * 16);
#pragma unroll
    for (int u = 0; u < 4 * WX_MAXCH; ++u) {
      if (u < 4 * nch) {
        const uint32_t wv = *reinterpret_cast<const uint32_t*>(xs + 256 * u + ((u & 1) ? boo : boe));
        const v4i Bv = v4i{(int)(wv & 0x03030303u), (int)((wv >> 2) & 0x03030303u), (int)((wv >> 4) & 0x03030303u),
                           (int)((wv >> 6) & 0x03030303u)};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const v4i t = __builtin_amdgcn_mfma_i32_16x16x64_i8(Ab[k], Bv, v4i{0, 0, 0, 0}, 0, 0, 0);
          dW0a[u][k] = fmaf(comb4p(t), sc[k], dW0a[u][k]);
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- epilogue: this half's part of the item's partial slab ----
  float* part = st.part + it.part_at;
  float db0[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) db0[k] = row_sum(db0a[k]);
#pragma unroll
  for (int u = 0; u < 4 * WX_MAXCH; ++u) {
    const int j = 16 * u + i;
    if (u < 4 * nch && j < m) {
      const float mu = st.mu[bd.mk_off + j], sg = st.sigma[bd.mk_off + j];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = 4 * (4 * h + k) + g;
        if (c < w0) part[bd.woff[0] + c * m + j] = sg > 0.f ? (dW0a[u][k] - mu * db0[k]) / sg : 0.f;
      }
    }
  }
  if (i == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (4 * (4 * h + k) + g < w0) part[bd.boff[0] + 4 * (4 * h + k) + g] = db0[k];
  }
#pragma unroll
  for (int sb = 0; sb < 2; ++sb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = 16 * h + 4 * g + r, s = 16 * sb + i;
      if (c < w0 && s < S) part[bd.woff[1] + s * w0 + c] = dW1a[sb][r];
    }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int s = 16 * h + 4 * g + r;
    const float v1 = row_sum(db1a[r]), v2 = row_sum(dW2a[r]);
    if (i == 0 && s < S) {
      part[bd.boff[1] + s] = v1;
      part[bd.woff[2] + s] = v2;
    }
  }
  const double rs = wave_sum_d(rss);
  if (h == 0 && lane == 0) st.rss_part[it.rss_at] = rs;
}

// ===========================================================================
// k_fused_grad_wx3 (default wide kernel): the same six phases with the three
// hidden GEMMs (Z1, err0, dW1) on v_mfma_f32_16x16x32_bf16 at f32 accuracy.
// Both f32 operands are split into three bf16 planes by truncation (x = x0 + x1
// + x2 exactly, 24 significant bits; kernels_gx.hip split3) and the six plane
// products of weight >= 2^-16 are accumulated in f32:
//   a b = a0 b0 + (a0 b1 + a1 b0) + (a0 b2 + a1 b1 + a2 b0) + O(2^-24 |a b|),
// so a 32-deep K step is 6 bf16 MFMAs (96 cycles) instead of 8 f32 16x16x4
// (256 cycles).  The W1 operands are split once per item (registers); A0 and
// delta1 are split by the wave that produces them and stored as planes.
// A workgroup holds TWO tile pairs (4 waves; pair p takes tiles tb + p, tb + p
// + 2, ...) so the 16 KiB W0 digit image is shared by both: 74 KiB per
// workgroup, 2 per CU = 2 waves per SIMD as in k_fused_grad_wx.  The pairs'
// accumulators are added in pair order at the end (one partial slab per item).
// Plane images, per pair: A0 and delta1 as [half][plane][row][16 bf16]; row
// 16 q + i holds individual 4 i + q; within half h of the A0 image position
// 4 g + k holds hidden unit 16 h + 4 k + g (the order a lane of the Z0 layout
// owns them in: one 8-byte store per plane and individual), delta1 is in
// natural summary order; the four 8-byte pieces of a 32-byte half-row are
// swizzled by row (bank-conflict-free stores and reads).  Z1 / err0 read their B
// operand as two pieces per plane (8 K slots), dW1 (K = individuals) both
// operands with ds_read_b64_tr_b16 down the rows.  After its dW1 a wave's half
// of the A0 planes is dead and takes its delta0 digit image.
// ===========================================================================
#define WX3_PAIRS 2
#define WX3_PLANE (64 * 32)       // bytes of one (half, plane): 64 rows x 16 bf16
#define WX3_HALF (3 * WX3_PLANE)  // one half of a plane image (6 KiB)
#define WX3_IMG (2 * WX3_HALF)    // one plane image (12 KiB)

typedef short v4s_wx __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s_wx lds_v4s_wx;

namespace {
// x = x0 + x1 + x2 by truncation (each plane the high half of an f32 word) for
// four values: three bf16x4 planes as two dwords each
__device__ __forceinline__ void split3x4(const float (&x)[4], v2u (&pl)[3]) {
  uint32_t hb[4], mb[4], lb[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    hb[c] = fbits(x[c]) & 0xFFFF0000u;
    const float r = x[c] - __builtin_bit_cast(float, hb[c]);  // exact
    mb[c] = fbits(r) & 0xFFFF0000u;
    lb[c] = fbits(r - __builtin_bit_cast(float, mb[c]));  // exact, <= 8 significant bits
  }
  // high halves of two words -> one dword (v_perm_b32: the low halves are ignored)
  auto hh = [](uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x07060302u); };
  pl[0] = v2u{hh(hb[0], hb[1]), hh(hb[2], hb[3])};
  pl[1] = v2u{hh(mb[0], mb[1]), hh(mb[2], mb[3])};
  pl[2] = v2u{hh(lb[0], lb[1]), hh(lb[2], lb[3])};
}
__device__ __forceinline__ void split3x8(const float (&x)[8], bf16x8 (&pl)[3]) {
  v2u a[3], b[3];
  split3x4({x[0], x[1], x[2], x[3]}, a);
  split3x4({x[4], x[5], x[6], x[7]}, b);
#pragma unroll
  for (int p = 0; p < 3; ++p) pl[p] = __builtin_bit_cast(bf16x8, v4u{a[p].x, a[p].y, b[p].x, b[p].y});
}
// signed 8-bit digits of V = rint(x 2^e), |V| < 2^27, least significant first:
// V = e3 2^24 + e2 2^16 + e1 2^8 + e0 with e0..e2 in [-128, 127] -- offsetting
// the three low bytes by 128 makes them carry-free, flipping their top bits
// gives the signed digits (two VALU instead of the 7-bit field extracts)
__device__ __forceinline__ uint32_t digits8_wx(float x, int e) {
  const int V = (int)__builtin_rintf(__builtin_amdgcn_ldexpf(x, e));
  return ((uint32_t)V + 0x00808080u) ^ 0x00808080u;
}
// 2^-16 sum_d D_d 2^(8 d) from the digit sums of one tile (|D| <= 2^14): the
// pairs D3 2^8 + D2 and D1 2^8 + D0 are exact in int32 and in f32
__device__ __forceinline__ float comb8(v4i d) {
  return (float)((d[3] << 8) + d[2]) + (float)((d[1] << 8) + d[0]) * 0x1p-16f;
}
// sum of the six plane products (small terms first), accumulated onto acc
__device__ __forceinline__ v4f mm6(const bf16x8 (&a)[3], const bf16x8 (&b)[3], v4f acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc, 0, 0, 0);
  return acc;
}
// transposing read of 8 rows (two ds_read_b64_tr_b16): lane 4 uq + up of a
// 16-lane group addresses row uq, columns 4 up .. 4 up + 3; lane li receives
// column li of rows 0..3 (p0) and 4..7 (p1) as K slots 0..7
__device__ __forceinline__ bf16x8 tr16x2(const char* p0, const char* p1) {
  const v4s_wx a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_wx*)(p0));
  const v4s_wx b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_wx*)(p1));
  typedef short v8s __attribute__((ext_vector_type(8)));
  return __builtin_bit_cast(bf16x8, v8s{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]});
}
// f64 all-reduce over the 16 lanes of a row (fixed xor order, result in every lane)
__device__ __forceinline__ double row_sum_d(double v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o);
  return v;
}
// two 8-byte pieces (ds_read_b64 each) as one 8-deep bf16 fragment
__device__ __forceinline__ bf16x8 rd_pieces(const char* base, uint32_t o0, uint32_t o1) {
  const v2u a = *reinterpret_cast<const v2u*>(base + o0);
  const v2u c = *reinterpret_cast<const v2u*>(base + o1);
  return __builtin_bit_cast(bf16x8, v4u{a.x, a.y, c.x, c.y});
}
}  // namespace

template <int ACT, int NCH>
__global__ void __launch_bounds__(64 * 2 * WX3_PAIRS, 2)
    k_fused_grad_wx3(DevState st, const GradItem* __restrict__ items, int write_pred) {
  __shared__ __attribute__((aligned(16))) char s_w0[WX_MAXCH * WX_MB * 1024];  // W0/sigma digits, all columns
  __shared__ __attribute__((aligned(16))) char s_img[WX3_PAIRS][2][WX3_IMG];  // per pair: A0 planes, delta1 planes
  __shared__ __attribute__((aligned(16))) char s_x[WX3_PAIRS][2][WX_SLOT];    // tile images (double-buffered)
  __shared__ __attribute__((aligned(16))) float s_y[WX3_PAIRS][2][64];
  __shared__ __attribute__((aligned(16))) float s_po[WX3_PAIRS][2][64];

  const GradItem it = items[blockIdx.x];
  const int b = it.branch;
  const BranchDev& bd = st.br[b];
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = wv & 1, pr = wv >> 1;  // this wave's half and tile pair
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i = lane & 15;
  constexpr int nch = NCH;  // marker chunks of 64 (bd.nchunks, checked at launch)
  const int m = bd.m, w0 = bd.widths[0], S = bd.widths[1];
  const int64_t n = st.n;
  const int tb = it.frag_begin >> 2, te = (it.frag_end + 3) >> 2;
  const float* th = st.theta + bd.p_off;

  for (int t = threadIdx.x; t < nch * WX_MB * 64; t += 64 * 2 * WX3_PAIRS)
    *reinterpret_cast<v4i*>(&s_w0[t * 16]) = *reinterpret_cast<const v4i*>(st.dig + bd.dig_off + (int64_t)t * 16);

  float zs[4], c0v[4], b1v[4], w2v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = 4 * (4 * h + k) + g;
    zs[k] = c < w0 ? st.fc[b].scale[c] : 0.f;
    c0v[k] = c < w0 ? st.fc[b].c0[c] : 0.f;
    const int s = 16 * h + 4 * g + k;
    b1v[k] = s < S ? th[bd.boff[1] + s] : 0.f;
    w2v[k] = s < S ? th[bd.woff[2] + s] : 0.f;
  }
  auto W1at = [&](int c, int s) { return (c < w0 && s < S) ? th[bd.woff[1] + s * w0 + c] : 0.f; };
  // W1 planes.  Z1 (A = W1^T rows of own summary units 16 h + i): K slot 8 g + j
  // is A0 image position p = 8 g + j, hidden unit 16 (p >> 4) + 4 (p & 3) + ((p >> 2) & 3).
  // err0 (A rows permuted so the result lands in the Z0 layout): row i = hidden
  // unit 16 h + 4 (i & 3) + (i >> 2), K slot 8 g + j = summary unit 8 g + j.
  bf16x8 wz[3], we3[3];
  {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int p = 8 * g + j;
      v[j] = W1at(16 * (p >> 4) + 4 * (p & 3) + ((p >> 2) & 3), 16 * h + i);
    }
    split3x8(v, wz);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = W1at(16 * h + 4 * (i & 3) + (i >> 2), 8 * g + j);
    split3x8(v, we3);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int tq = i >> 1, tp = lane & 1, gsw = g & 1;
  const uint32_t fo0 = (uint32_t)((16 * g + tq + 8 * gsw) * 16 + 8 * (tp ^ gsw));
  const uint32_t fo1 = (uint32_t)((16 * g + tq + 8 * (1 ^ gsw)) * 16 + 8 * (tp ^ 1 ^ gsw));
  const int pe = i, po = (i + 8) & 15;
  const uint32_t boe = (uint32_t)(pe * 16 + 4 * (2 * ((g >> 1) ^ (pe >> 3)) + (g & 1)));
  const uint32_t boo = (uint32_t)(po * 16 + 4 * (2 * ((g >> 1) ^ (po >> 3)) + (g & 1)));
  const int iota = 4 * i + g;
  char* const sA = s_img[pr][0];
  char* const sD = s_img[pr][1];
  // 8-byte piece P of plane row rho sits at position P ^ swz((rho >> 2) & 3) of its
  // 32-byte half-row (swz swaps the two bits): the stores (16 lanes = 16 rows, one
  // piece each, banks mod 32) and the Z1 / err0 reads (32 lanes, mod 64) are then
  // conflict-free (row-major without it: 4-way on the stores)
  auto swz = [](int v) { return ((v & 1) << 1) | (v >> 1); };
  const int sw_i = swz((i >> 2) & 3);
  const uint32_t wr_off = (uint32_t)(h * WX3_HALF + i * 32 + 8 * (g ^ sw_i));  // + 512 q: own half, row 16 q + i
  const uint32_t rd_off0 = (uint32_t)((g >> 1) * WX3_HALF + i * 32 + 8 * ((2 * (g & 1)) ^ sw_i));  // K slots 8 g .. + 3
  const uint32_t rd_off1 = (uint32_t)((g >> 1) * WX3_HALF + i * 32 + 8 * ((2 * (g & 1) + 1) ^ sw_i));  // 8 g + 4 ..
  // dW1 (K = individuals): K slots 8 g + j of block ks are rows 32 ks + 16 (j >> 2) + 4 g
  // + (j & 3) -- the two 16-lane groups of a 32-lane bank group read rows 0-3 / 4-7
  // of an 8-row bank window (conflict-free); + 512 for j >= 4, + 1024 ks
  const uint32_t tr_off = (uint32_t)((4 * g + (i >> 2)) * 32 + 8 * ((i & 3) ^ swz(g)));
  char* const sdig = sA + h * WX3_HALF;  // delta0 digits: the own (dead) half of the A0 planes
  char* const sd_w = sdig + (i >> 2) * 256 + (4 * g + (i & 3)) * 16;
  const char* const sd_r = sdig + g * 256 + tq * 16 + 8 * tp;
  const float* ybr = st.y + bd.y_off;
  float* predb = st.pred + bd.y_off;
  const char* xsrc = reinterpret_cast<const char*>(st.xu2) + bd.x_off + lane * 16;
  const int64_t tile_bytes = (int64_t)nch * 1024;
  auto issue_tile = [&](int tt, int sl) {
    if (h < nch) glds16(xsrc + (int64_t)tt * tile_bytes + h * 1024, &s_x[pr][sl][h * 1024]);
    if (h == 0) {
      const int64_t row = 64 * (int64_t)tt + iota;
      glds4(ybr + (row < n ? row : n - 1), &s_y[pr][sl][0]);
    }
  };

  float dW0a[4 * WX_MAXCH][4];
#pragma unroll
  for (int u = 0; u < 4 * WX_MAXCH; ++u)
#pragma unroll
    for (int k = 0; k < 4; ++k) dW0a[u][k] = 0.f;
  // bias gradients are column sums that cancel strongly (n-term sums of h'(z) e
  // terms of either sign): their per-lane partials are kept in f64
  double db0a[4], db1a[4];
  float dW2a[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    db0a[k] = db1a[k] = 0.0;
    dW2a[k] = 0.f;
  }
  v4f dW1a[2] = {v4f{0.f, 0.f, 0.f, 0.f}, v4f{0.f, 0.f, 0.f, 0.f}};
  double rss = 0.0;

  // rounds of WX3_PAIRS tiles; a pair without a tile in the last round runs on
  // its stale slot with every row invalid (e = 0: it adds exactly nothing)
  const int nrounds = (te - tb + WX3_PAIRS - 1) / WX3_PAIRS;
  int sl = 0;
  if (tb + pr < te) issue_tile(tb + pr, 0);
  for (int rd = 0; rd < nrounds; ++rd, sl ^= 1) {
    const int tt = tb + WX3_PAIRS * rd + pr;
    const bool live = tt < te;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tt + WX3_PAIRS < te) issue_tile(tt + WX3_PAIRS, sl ^ 1);
    const char* xs = &s_x[pr][sl][0];

    // ---- 1. masked layer forward (as k_fused_grad_wx) ----
    float z0[4][4], a0[4][4];
    {
      v4i fa[4][4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int q = 0; q < 4; ++q) fa[k][q] = v4i{0, 0, 0, 0};
#pragma unroll
      for (int c = 0; c < WX_MAXCH; ++c) {
        if (c < nch) {
          const v4u X = (v4u)lds_tr8_pair(xs + c * 1024 + fo0, xs + c * 1024 + fo1);
          const v4i B0 = (v4i)(X & 0x03030303u);
          const v4i B1 = (v4i)(X & 0x0C0C0C0Cu);
          const v4i B2 = (v4i)(X & 0x30303030u);
          const v4i B3 = (v4i)((X >> 2u) & 0x30303030u);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const v4i A = *reinterpret_cast<const v4i*>(&s_w0[((c * WX_MB + 4 * h + k) * 64 + lane) * 16]);
            fa[k][0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B0, fa[k][0], 0, 0, 0);
            fa[k][1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B1, fa[k][1], 0, 0, 0);
            fa[k][2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B2, fa[k][2], 0, 0, 0);
            fa[k][3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B3, fa[k][3], 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        z0[k][0] = (0x1p-7f * zs[k]) * comb4p(fa[k][0]) + c0v[k];
        z0[k][1] = (0x1p-9f * zs[k]) * comb4p(fa[k][1]) + c0v[k];
        z0[k][2] = (0x1p-11f * zs[k]) * comb4p(fa[k][2]) + c0v[k];
        z0[k][3] = (0x1p-11f * zs[k]) * comb4p(fa[k][3]) + c0v[k];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if constexpr (ACT == 0) {  // z0 keeps r (tanh_r) for the derivative
            float r;
            a0[k][q] = tanh_r(z0[k][q], r);
            z0[k][q] = r;
          } else {
            a0[k][q] = act_h_t<ACT>(z0[k][q]);
          }
        }
      }
    }
    // A0 planes: own half, individual 4 i + q, positions 4 g .. 4 g + 3 (hidden 16 h + 4 k + g)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v2u pl[3];
      split3x4({a0[0][q], a0[1][q], a0[2][q], a0[3][q]}, pl);
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<v2u*>(sA + wr_off + p * WX3_PLANE + 512 * q) = pl[p];
    }
    LDS_BARRIER();  // the full A0 planes of the pair

    // ---- 2. Z1^T = W1^T A0^T, own summary units (K = the 32 hidden units) ----
    v4f z1[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      bf16x8 bq[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) bq[p] = rd_pieces(sA + p * WX3_PLANE + 512 * q, rd_off0, rd_off1);
      z1[q] = mm6(wz, bq, v4f{0.f, 0.f, 0.f, 0.f});
    }

    // ---- 3. head (as k_fused_grad_wx) ----
    float a1[4][4], pp[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      pp[q] = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        z1[q][r] += b1v[r];
        if constexpr (ACT == 0) {  // z1 keeps r (tanh_r)
          float rr;
          a1[q][r] = tanh_r(z1[q][r], rr);
          z1[q][r] = rr;
        } else {
          a1[q][r] = act_h_t<ACT>(z1[q][r]);
        }
        pp[q] = fmaf(a1[q][r], w2v[r], pp[q]);
      }
    }
    xpose4f(pp[0], pp[1], pp[2], pp[3]);
    s_po[pr][h][lane] = (pp[0] + pp[1]) + (pp[2] + pp[3]);
    LDS_BARRIER();  // both halves' partial outputs
    const float out = s_po[pr][0][lane] + s_po[pr][1][lane];
    const int64_t row = 64 * (int64_t)tt + iota;
    const bool valid = live && row < n;
    const float yv = s_y[pr][sl][lane];
    const float e = valid ? out - yv : 0.f;
    if (h == 0 && write_pred && valid) predb[row] = out;
    rss += (double)e * (double)e;
    float eq[4] = {e, e, e, e};
    xpose4f(eq[0], eq[1], eq[2], eq[3]);
    float d1[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float sw = 0.f, sd = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        d1[q][r] = (ACT == 0 ? dtanh_r(z1[q][r]) : act_dh_t<ACT>(z1[q][r], a1[q][r])) * (eq[q] * w2v[r]);
        sw = fmaf(a1[q][r], eq[q], sw);
        sd += d1[q][r];
      }
      dW2a[r] += sw;
      db1a[r] += (double)sd;
    }
    // delta1 planes: own half, individual 4 i + q, summary units 16 h + 4 g .. + 3
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v2u pl[3];
      split3x4({d1[q][0], d1[q][1], d1[q][2], d1[q][3]}, pl);
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<v2u*>(sD + wr_off + p * WX3_PLANE + 512 * q) = pl[p];
    }
    LDS_BARRIER();  // the full delta1 planes of the pair

    // ---- 4. err0 = delta1 W1^T, own hidden units in the Z0 layout; delta0 ----
    float d0[4][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      bf16x8 bq[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) bq[p] = rd_pieces(sD + p * WX3_PLANE + 512 * q, rd_off0, rd_off1);
      const v4f acc = mm6(we3, bq, v4f{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int k = 0; k < 4; ++k) d0[k][q] = (ACT == 0 ? dtanh_r(z0[k][q]) : act_dh_t<ACT>(z0[k][q], a0[k][q])) * acc[k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) db0a[k] += (double)((d0[k][0] + d0[k][1]) + (d0[k][2] + d0[k][3]));

    // ---- 5. dW1 = A0^T delta1 (rows: own hidden units in position order, K = individuals) ----
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 ta[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const char* a = sA + h * WX3_HALF + p * WX3_PLANE + 1024 * ks + tr_off;
        ta[p] = tr16x2(a, a + 512);
      }
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        bf16x8 tdl[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          const char* d = sD + sb * WX3_HALF + p * WX3_PLANE + 1024 * ks + tr_off;
          tdl[p] = tr16x2(d, d + 512);
        }
        dW1a[sb] = mm6(ta, tdl, dW1a[sb]);
      }
    }

    // ---- 6. delta0 digits over the own dead A0 half, masked backward (as k_fused_grad_wx) ----
    float sc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t mx = row_max_u(max(max(fbits(d0[k][0]) & 0x7FFFFFFFu, fbits(d0[k][1]) & 0x7FFFFFFFu),
                                        max(fbits(d0[k][2]) & 0x7FFFFFFFu, fbits(d0[k][3]) & 0x7FFFFFFFu)));
      const int R = (int)((mx >> 23) & 0xFFu) + 2;
      sc[k] = __builtin_amdgcn_ldexpf(1.f, R - 137);  // comb8 carries 2^-16
      uint32_t dq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) dq[q] = digits8_wx(d0[k][q], 153 - R);
      xpose4(dq[0], dq[1], dq[2], dq[3]);
      *reinterpret_cast<v4u*>(sd_w + k * 1024) = v4u{dq[0], dq[1], dq[2], dq[3]};
    }
    v4i Ab[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) Ab[k] = lds_tr8_pair(sd_r + k * 1024, sd_r + k * 1024 + 8 * 16);
#pragma unroll
    for (int u = 0; u < 4 * WX_MAXCH; ++u) {
      if (u < 4 * nch) {
        const uint32_t wvv = *reinterpret_cast<const uint32_t*>(xs + 256 * u + ((u & 1) ? boo : boe));
        const v4i Bv = v4i{(int)(wvv & 0x03030303u), (int)((wvv >> 2) & 0x03030303u),
                           (int)((wvv >> 4) & 0x03030303u), (int)((wvv >> 6) & 0x03030303u)};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const v4i t = __builtin_amdgcn_mfma_i32_16x16x64_i8(Ab[k], Bv, v4i{0, 0, 0, 0}, 0, 0, 0);
          dW0a[u][k] = fmaf(comb8(t), sc[k], dW0a[u][k]);
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wave is past its last tile: the plane images are free

  // ---- the two pairs' accumulators, added in pair order ----
  constexpr int NV = 4 * 4 * WX_MAXCH + 4 + 8;
  float* red = reinterpret_cast<float*>(&s_img[0][0][0]);
  double* redd = reinterpret_cast<double*>(red + 2 * NV * 64);  // [half][9][lane]: rss, db0a, db1a
  {
    float* o = red + h * NV * 64 + lane;
    if (pr == 1) {
      int v = 0;
#pragma unroll
      for (int u = 0; u < 4 * WX_MAXCH; ++u)
#pragma unroll
        for (int k = 0; k < 4; ++k) o[64 * v++] = dW0a[u][k];
#pragma unroll
      for (int k = 0; k < 4; ++k) o[64 * v++] = dW2a[k];
#pragma unroll
      for (int sb = 0; sb < 2; ++sb)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[64 * v++] = dW1a[sb][r];
      double* od = redd + h * 9 * 64 + lane;
      od[0] = rss;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        od[64 * (1 + k)] = db0a[k];
        od[64 * (5 + k)] = db1a[k];
      }
    }
    __syncthreads();
    if (pr == 1) return;
    int v = 0;
#pragma unroll
    for (int u = 0; u < 4 * WX_MAXCH; ++u)
#pragma unroll
      for (int k = 0; k < 4; ++k) dW0a[u][k] += o[64 * v++];
#pragma unroll
    for (int k = 0; k < 4; ++k) dW2a[k] += o[64 * v++];
#pragma unroll
    for (int sb = 0; sb < 2; ++sb)
#pragma unroll
      for (int r = 0; r < 4; ++r) dW1a[sb][r] += o[64 * v++];
    const double* od = redd + h * 9 * 64 + lane;
    rss += od[0];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      db0a[k] += od[64 * (1 + k)];
      db1a[k] += od[64 * (5 + k)];
    }
  }

  // ---- epilogue: this half's part of the item's partial slab ----
  float* part = st.part + it.part_at;
  double db0[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) db0[k] = row_sum_d(db0a[k]);
#pragma unroll
  for (int u = 0; u < 4 * WX_MAXCH; ++u) {
    const int j = 16 * u + i;
    if (u < 4 * nch && j < m) {
      const float mu = st.mu[bd.mk_off + j], sg = st.sigma[bd.mk_off + j];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = 4 * (4 * h + k) + g;
        if (c < w0)
          part[bd.woff[0] + c * m + j] = sg > 0.f ? (float)(((double)dW0a[u][k] - (double)mu * db0[k]) / sg) : 0.f;
      }
    }
  }
  if (i == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (4 * (4 * h + k) + g < w0) part[bd.boff[0] + 4 * (4 * h + k) + g] = (float)db0[k];
  }
  // dW1 lane (n = i, g): rows 4 g + r = A0 positions 16 h + 4 g + r = hidden 16 h + 4 r + g
#pragma unroll
  for (int sb = 0; sb < 2; ++sb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = 16 * h + 4 * r + g, s = 16 * sb + i;
      if (c < w0 && s < S) part[bd.woff[1] + s * w0 + c] = dW1a[sb][r];
    }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int s = 16 * h + 4 * g + r;
    const double v1 = row_sum_d(db1a[r]);
    const float v2 = row_sum(dW2a[r]);
    if (i == 0 && s < S) {
      part[bd.boff[1] + s] = (float)v1;
      part[bd.woff[2] + s] = v2;
    }
  }
  const double rs = wave_sum_d(rss);
  if (h == 0 && lane == 0) st.rss_part[it.rss_at] = rs;
}

bool wx_exact() {
  const char* ex = getenv("BANN_WX_EXACT");  // 1: the hidden GEMMs on the exact-f32 MFMA (k_fused_grad_wx)
  return ex && atoi(ex) != 0;
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

template <int NCH>
static void launch_wx3(const DevState& st, const GradItem* items, int32_t nitems, int act, int wp, hipStream_t s) {
  const dim3 grid((unsigned)nitems), block(64 * 2 * WX3_PAIRS);
  switch (act) {
    case 0: hipLaunchKernelGGL((k_fused_grad_wx3<0, NCH>), grid, block, 0, s, st, items, wp); break;
    case 1: hipLaunchKernelGGL((k_fused_grad_wx3<1, NCH>), grid, block, 0, s, st, items, wp); break;
    case 2: hipLaunchKernelGGL((k_fused_grad_wx3<2, NCH>), grid, block, 0, s, st, items, wp); break;
    case 3: hipLaunchKernelGGL((k_fused_grad_wx3<3, NCH>), grid, block, 0, s, st, items, wp); break;
    default: hipLaunchKernelGGL((k_fused_grad_wx3<4, NCH>), grid, block, 0, s, st, items, wp); break;
  }
}

// mode: 0 = exact f32 MFMA hidden GEMMs (k_fused_grad_wx, BANN_WX_EXACT=1), 1 =
// bf16 MFMA (opt-in, reduced precision), 2 = f32-accurate bf16 planes (default)
void launch_fused_grad_wx(const DevState& st, const GradItem* items, int32_t nitems, int32_t act, int mode,
                          int nch, int write_pred, hipStream_t s) {
  if (nitems <= 0) return;
  if (mode == 1) {
    launch_wx_bf<1>(st, items, nitems, act, write_pred, s);
  } else if (mode == 0) {
    launch_wx_bf<0>(st, items, nitems, act, write_pred, s);
  } else {
    if (nch == 1) launch_wx3<1>(st, items, nitems, act, write_pred, s);
    else launch_wx3<2>(st, items, nitems, act, write_pred, s);
  }
}
