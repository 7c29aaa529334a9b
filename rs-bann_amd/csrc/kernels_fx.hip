// kernels_fx.hip — the "fx" fused gradient kernel (default): one WAVE owns a
// 64-individual tile of one branch across ALL of its marker chunks.
//
// Replaces BranchSampler::backpropagate (branch_sampler.rs:813-875) with its
// forward_feed (743-782) and the rss it stores (823-828), for every branch of a
// plan in one launch, and writes the same per-split partial slabs as the other
// fused variants (d(rss/2)/d(theta) in param_vec order, params.rs:700-715).
//
// Why this shape (measured on the chunk-wave kernels it replaces): with one
// wave per 64-marker chunk, every tile needs a cross-wave exchange of partial
// Z0 and of delta0 (two barriers), the per-individual head serialises on one
// wave, and every MFMA result is converted to f32 on its own -- issue- and
// latency-bound at 2.4 TB/s of 2-bit genotypes.  Here:
//   * the forward accumulates Z0 over all chunks in the MFMA's int32
//     accumulator (exact), converted once per tile;
//   * the head runs in every wave, one individual per lane;
//   * dW0 = G^T delta0 accumulates over ALL tiles of the item in int32 digit
//     sums with a per-column running power-of-two scale (rescaled exactly by
//     digit carry in the rare case a tile's |delta0| outgrows it), converted to
//     f32 once at the end;
//   * waves never wait for each other inside the tile loop: each streams its
//     own tiles into its own LDS slots (LDS-DMA, two tiles ahead, counted
//     vmcnt) -- the only barriers are the final workgroup reduction.
//
// Genotype tile image (HBM == LDS, 16 B per marker row, "u2t" layout):
//   row j (marker) = 16 quads Q; quad Q = individuals 4Q .. 4Q+3 as 2-bit
//   codes at bits 2p (p = individual - 4Q).  Rows are stored in 16-row windows
//   w = j >> 4 at position P = ((j & 15) + 8 (w & 1)) & 15, and the two 8-byte
//   halves of a row at position P >= 8 are swapped (bank-conflict-free reads).
//   * forward B operand (K = 64 markers, N = 16 individuals): two
//     ds_read_b64_tr_b8 per chunk give lane (g, i) the quad-i byte of the 16
//     markers of window 4c + g; (x >> 2q) & 0x03030303 is the i8 operand of
//     individual 4i + q ("fragment" q).
//   * backward B operand (K = 64 individuals, N = 16 markers): one ds_read_b32
//     gives lane (r, n) quads 4r .. 4r+3 of marker 16u + n; (w >> 2p) &
//     0x03030303 holds individuals 16r + 4b + p (byte b), K slot 16r + 4p + b.
//     Fields p = 1, 2 are used in place (w & 0x0C0C0C0C = 4 x code, w &
//     0x30303030 = 16 x code); the delta0 digits of those individuals are taken
//     at a 4^p smaller scale, so the MFMA sum is unchanged.  The delta0 digit
//     operand A is written in the same K order.
#include <stdlib.h>
#include <type_traits>

#include "activations.h"
#include "bann_internal.h"
#include "kernel_util.h"
#include "update_core.h"

#define FX_WAVES 4        // waves per workgroup (one work item, tiles interleaved)
#define FX_SLOT 8192      // one tile image at <= 8 chunks (512 markers x 16 B)
#define FX_DROW 256       // delta0 digit image: 16 rows x 16 B per K group (read twice per tile)

// Profiling builds only (tools/build_ab.sh <tag> "-DFX_STAMPS=1" / "-DFX_ABL=<bits>"); both 0 in the
// product, where they generate no code.  FX_STAMPS: per-phase shader-cycle sums of k_fused_grad_fx
// (s_memtime) into DevState::dbg, printed at bann_ctx_destroy under BANN_STAMPS=1: p0 wait for the
// tile, p1 forward, p2 head, p3 delta0 digits, p4 backward, p5 loop overhead, p6 realtime (100 MHz),
// p7 loop cycles.  FX_ABL (results wrong, timing only): 1 forward without the 2-bit unpack, 2 backward
// without it, 4 no head (delta0 = z0), 8 no MFMAs (the operands XORed into the accumulators), 16 no
// genotype / target stream (the loop computes on whatever the slots hold).
//
// Field 3 of every fx / fxl / fxh tile image is stored as code - 1 (k_pack_tiles, PackJob::f3m1):
// read as a signed int8, a genotype byte is then f0 + 4 f1 + 16 f2 + 64 (f3 - 1) (codes <= 2, so
// the 2-bit field holds -1 .. 1).  The forward takes CUMULATIVE fragments -- x & 0x03, x & 0x0F,
// x & 0x3F and the raw byte: 3 ANDs per dword instead of 5 -- and recovers the in-place fields
// exactly in int32 once per tile: F1 = C1 - C0, F2 = C2 - C1, F3 = C3 - C2 with C3 started at
// 64 sum_k A (the W0-digit row sums over the wave's chunks, fx_rowsum64), so F_q = 4^q S_q as
// before and z keeps its bits.  The backward keeps field 3 in place too (x & 0xC0 = 64 (f3 - 1):
// one AND instead of a shift and an AND), with the delta0 digits of K-group 3 pre-divided by 64;
// the -1 comes back as 64 sum_(i in group 3) digit_i, one MFMA per tile against FX_ONES3, added
// to every marker's digit sums at the end.
#ifndef FX_STAMPS
#define FX_STAMPS 0
#endif
// the backward's genotype-window prefetch depth and its per-window scheduling barrier (round 6,
// kbench and C3 line A/B on one box: PD 8 -> 12 without the barrier, fx 1.181 / 1.190 -> 1.173 /
// 1.169 ms, 780.7 / 774.5 -> 785.4 / 787.1 steps/s; a barrier-free PD 8: 1.175 / 1.177; measured and
// not kept: the forward at priority 0, the head at 2, the backward at 1, the forward three chunks
// ahead, PD 4 or 16, no barrier per forward chunk -- tools/gpu_kab.sh, profiles/r06_fx_knobs.txt)
#ifndef FXT_PD
#define FXT_PD 12  // backward: genotype window reads this many windows ahead
#endif
#ifndef FXT_SBB
#define FXT_SBB 0  // a scheduling barrier after each backward window (1: the round-5 schedule)
#endif
#ifndef FX_ABL
#define FX_ABL 0
#endif
#if FX_STAMPS
#define FX_STAMP(i)                                            \
  do {                                                         \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    ph[i] += t_ - t_last;                                      \
    t_last = t_;                                               \
  } while (0)
#else
#define FX_STAMP(i) \
  do {              \
  } while (0)
#endif
#if FX_ABL & 8
#define FX_MFMA(a, b, c) ((c) + ((a) ^ (b)))
#else
#define FX_MFMA(a, b, c) __builtin_amdgcn_mfma_i32_16x16x64_i8((a), (b), (c), 0, 0, 0)
#endif
// The stream runs TWO tiles ahead in the same two slots: chunk c of tile t + 2
// is issued into tile t's slot as soon as tile t's backward has read chunk c's
// last window (the target piece once the head has read the target), so a piece
// has a whole tile more to land than when it is issued in the forward (the
// one-tile-ahead and burst variants measured slower: DESIGN.md 4)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

#define FX_ONES3 (v4i{0, 0, 0, 0x40404040})  // 64 in every K slot of field 3 (the backward's group 3)

// one chunk of the forward: the four cumulative fragments of a quad-byte operand
__device__ __forceinline__ void fx_fwd_chunk(v4i A, v4u X, v4i (&facc)[4]) {
  facc[0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, (v4i)(X & 0x03030303u), facc[0], 0, 0, 0);
  facc[1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, (v4i)(X & 0x0F0F0F0Fu), facc[1], 0, 0, 0);
  facc[2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, (v4i)(X & 0x3F3F3F3Fu), facc[2], 0, 0, 0);
  facc[3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, (v4i)X, facc[3], 0, 0, 0);
}
// cumulative sums -> in-place fields F_q = 4^q S_q (facc[3] started at fx_rowsum64)
__device__ __forceinline__ void fx_fwd_fields(v4i (&facc)[4]) {
  facc[3] -= facc[2];
  facc[2] -= facc[1];
  facc[1] -= facc[0];
}
// 64 sum_k A[.][k] for the digit operands of chunks [0, nc): facc[3]'s start
__device__ __forceinline__ v4i fx_rowsum64_acc(v4i A, v4i acc) {
  return __builtin_amdgcn_mfma_i32_16x16x64_i8(A, v4i{0x40404040, 0x40404040, 0x40404040, 0x40404040}, acc, 0, 0, 0);
}
// the backward's fragments of one window dword: every field in place (x 1, 4, 16, and
// 64 (f3 - 1)); the delta0 digits of K-group p carry 4^-p (p = 3: 64^-1)
__device__ __forceinline__ v4i fx_bwd_unpack(uint32_t wv) {
  return v4i{(int)(wv & 0x03030303u), (int)(wv & 0x0C0C0C0Cu), (int)(wv & 0x30303030u), (int)(wv & 0xC0C0C0C0u)};
}

__device__ __forceinline__ float ufl(float v) {  // make a wave-uniform value scalar
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}

// all but the youngest k vector-memory operations of this wave are complete
__device__ __forceinline__ void vm_wait(int k) {
  switch (k) {
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

__device__ __forceinline__ float sgpr_f(float v) {  // a wave-uniform value, pinned to a scalar register
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}

__device__ __forceinline__ float comb4(v4i d) {  // sum_d D_d 2^(-7 d)
  return (float)d[0] + (float)d[1] * 0x1p-7f + (float)d[2] * 0x1p-14f + (float)d[3] * 0x1p-21f;
}

// delta0 digits: V = rint(x 2^e), |V| < 2^27, as four signed 8-bit digits
// V = d0 + d1 2^8 + d2 2^16 + d3 2^24 (byte d = digit d, d0..d2 in [-128, 127],
// d3 in [-8, 8]): offsetting the three low bytes by 128 and flipping their top
// bits is the whole recoding, 2 VALU
__device__ __forceinline__ uint32_t digits4_fx(float x, int e) {
  const int V = (int)__builtin_rintf(__builtin_amdgcn_ldexpf(x, e));
  return ((uint32_t)V + 0x00808080u) ^ 0x00808080u;
}

// value(G) of digit sums G (digit d weighs 2^(8 d)), rounded once: the digit sums
// grow past 2^24 over an item's tiles (in-place fields weigh up to 48), where a
// per-digit float conversion would round each one
__device__ __forceinline__ float comb4_exact(v4i G) {
  const int64_t N = (int64_t)G[0] + ((int64_t)G[1] << 8) + ((int64_t)G[2] << 16) + ((int64_t)G[3] << 24);
  return (float)N;
}
// the same for two digit-sum vectors (a window's sums and the item's K-group-3 correction)
__device__ __forceinline__ float comb4_exact2(v4i G, v4i H) {
  const int64_t N = (int64_t)G[0] + ((int64_t)G[1] << 8) + ((int64_t)G[2] << 16) + ((int64_t)G[3] << 24) +
                    (int64_t)H[0] + ((int64_t)H[1] << 8) + ((int64_t)H[2] << 16) + ((int64_t)H[3] << 24);
  return (float)N;
}

// value(G) * 2^-sh for digit sums G, sh >= 0: form N in int64 (|G_d| < 2^31),
// shift it, and re-split into 8-bit digits (exact up to the dropped low bits, < 1
// of the new unit).  Branch- and loop-free so the accumulators are updated in place.
__device__ __forceinline__ v4i shr_digits(v4i G, int sh) {
  const int64_t N = (int64_t)G[0] + ((int64_t)G[1] << 8) + ((int64_t)G[2] << 16) + ((int64_t)G[3] << 24);
  const int64_t M = N >> (sh < 63 ? sh : 63);
  return v4i{(int)(M & 255), (int)((M >> 8) & 255), (int)((M >> 16) & 255), (int)(M >> 24)};
}

__device__ __forceinline__ void swap32(float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b),
                                                  false, false);
  a = __builtin_bit_cast(float, (unsigned)r[0]);
  b = __builtin_bit_cast(float, (unsigned)r[1]);
}
__device__ __forceinline__ void swap16(float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b),
                                                  false, false);
  a = __builtin_bit_cast(float, (unsigned)r[0]);
  b = __builtin_bit_cast(float, (unsigned)r[1]);
}

// NCH: 8 = every branch of the launch has exactly 8 chunks (no per-chunk guards,
// so the LDS reads of a whole phase issue back to back); 0 = any count <= 8.

// UPD: the instantiation with the fused update tail (bann_api.hip fuse_update plans);
// the default one carries no tail code at all (its registers: the tail's live values
// made the tile loop spill scalar registers to vector lanes)
template <int NL, int ACT, int NCH, int UPD>
__global__ void __launch_bounds__(64 * FX_WAVES, NL == 4 ? 1 : 2)
    k_fused_grad_fx(DevState st, const GradItem* __restrict__ items, int write_pred, int upd_mode, int upd_step,
                    int32_t* __restrict__ upd_cnt, const FoldJob* __restrict__ folds) {
  constexpr int NH = NL - 1;  // layers with activations
  constexpr int NW = FX_WAVES;
  constexpr int NS = 8 + (NH - 1) * 20;  // head statistics per wave
  __shared__ __attribute__((aligned(16))) char s_x[NW][2][FX_SLOT];
  __shared__ __attribute__((aligned(16))) char s_dig[NW][4 * FX_DROW];
  __shared__ __attribute__((aligned(16))) float s_y[NW][2][64];
  __shared__ __attribute__((aligned(16))) char s_w0[8 * 1024];  // W0/sigma digits (A operand), per chunk
  __shared__ __attribute__((aligned(16))) float s_hw[NL][20];  // head: W_l (4 x 4) then b_l (4) per layer
  __shared__ float s_hs[NW][NS];
  __shared__ double s_rss[NW];

  const GradItem it = items[blockIdx.x];
  const int b = it.branch;
  const BranchDev& bd = st.br[b];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int nch = NCH ? NCH : bd.nchunks;
  const int64_t n = st.n;
  const int tb = it.frag_begin >> 2, te = (it.frag_end + 3) >> 2;

  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 1, tp = lane & 1;
  // ---- per-lane LDS offsets ----
  const int gsw = g & 1;
  const uint32_t fo0 = (uint32_t)((16 * g + tq + 8 * gsw) * 16 + 8 * (tp ^ gsw));
  const uint32_t fo1 = (uint32_t)((16 * g + tq + 8 * (1 ^ gsw)) * 16 + 8 * (tp ^ 1 ^ gsw));
  const int pe = i16, po = (i16 + 8) & 15;
  const uint32_t boe = (uint32_t)(pe * 16 + 4 * (2 * ((g >> 1) ^ (pe >> 3)) + (g & 1)));
  const uint32_t boo = (uint32_t)(po * 16 + 4 * (2 * ((g >> 1) ^ (po >> 3)) + (g & 1)));
  const int iota = 4 * i16 + g;  // individual of this lane in the head (after the transpose)
  char* const sd = &s_dig[wave][0];
  char* const sd_w = sd + (i16 >> 2) * FX_DROW + (4 * g + (i16 & 3)) * 16;  // row K(iota)
  const char* const sd_r = sd + g * FX_DROW + tq * 16 + 8 * tp;
  // the tile's targets -- or, in network mode, the network's output error, the same
  // n-vector for every branch (bann_network_hmc_step)
  const bool net_err = st.nete != nullptr;
  const float* ybr = net_err ? st.nete : st.y + bd.y_off;
  float* predb = st.pred + bd.y_off;
  const int64_t tile_bytes = (int64_t)nch * 1024;
  // the stream's base in scalar registers: each piece is one global_load_lds in the saddr
  // form (one address VGPR, no 64-bit address arithmetic per piece: -0.7 % per launch)
  const uint64_t xb = (uint64_t)(uintptr_t)(reinterpret_cast<const char*>(st.xu2) + bd.x_off);
  const char* xbase_s = reinterpret_cast<const char*>(
      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(xb >> 32)) << 32) |
      (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)xb));

  // LDS-DMA of the NEXT tile is spread over the current tile's forward phase
  // (one 1 KiB piece per chunk, the target piece in the head): issued in one
  // burst the pieces back-pressure the wave for thousands of cycles.
  // the last chunk's padding rows (markers >= m) are not streamed (C3: 12 of 512 rows):
  // their W0 digits are zero, so whatever the slot holds there adds nothing to Z0, and
  // their dW0 rows are dropped.  Lane L moves record L of a chunk: window L >> 4 at
  // position L & 15 holds row 16 (L >> 4) + ((L & 15) - 8 ((L >> 4) & 1)) & 15.
  // (Row 0 is never padding, so the wave's instruction -- one vmcnt count -- always issues.)
  const bool pad_row = 64 * (nch - 1) + 16 * (lane >> 4) + (((lane & 15) - 8 * ((lane >> 4) & 1)) & 15) >= bd.m;
  auto issue_chunk = [&](int tt, int sl, int c) {
    if (FX_ABL & 16) return;
    if (c == nch - 1 && pad_row) return;
    glds16_s(xbase_s + (uint64_t)tt * (uint64_t)tile_bytes + (uint64_t)(c * 1024), (uint32_t)lane * 16u,
             &s_x[wave][sl][c * 1024]);
  };
  auto issue_y = [&](int tt, int sl) {
    if (FX_ABL & 16) return;
    const int64_t row = 64 * (int64_t)tt + iota;
    glds4(ybr + (row < n ? row : n - 1), &s_y[wave][sl][0]);
  };
  // the item's first two tiles are issued before the prologue's loads, so their HBM latency
  // overlaps the W0-digit and head-weight loads (a solo item -- the sequential driver's
  // one-branch steps -- has one tile per wave: the launch was that latency longer)
  int tt = tb + wave, sl = 0;
  if (tt < te) {
    for (int c = 0; c < nch; ++c) issue_chunk(tt, 0, c);
    issue_y(tt, 0);
    if (tt + NW < te) {
      for (int c = 0; c < nch; ++c) issue_chunk(tt + NW, 1, c);
      issue_y(tt + NW, 1);
    }
  }
  // ---- branch constants: head weights (LDS, then scalar registers), W0 digits, column scale ----
  const float* th = st.theta + bd.p_off;
  for (int t = threadIdx.x; t < NL * 20; t += 64 * NW) {
    const int l = t / 20, r = t - l * 20;
    float v = 0.f;
    if (r < 16) {  // Wh[l][j][k] = W_l[j][k] (l >= 1), zero padded to 4 x 4
      const int j = r >> 2, k = r & 3;
      if (l >= 1 && j < bd.win[l] && k < bd.widths[l]) v = th[bd.woff[l] + k * bd.win[l] + j];
    } else {  // bias[0] = c0 (folded standardisation), bias[l] = b_l
      const int k = r - 16;
      if (l == 0 && k < bd.widths[0]) v = st.fc[b].c0[k];
      if (l >= 1 && l < NH && k < bd.widths[l]) v = th[bd.boff[l] + k];
    }
    s_hw[l][r] = v;
  }
  float zscale = st.fc[b].scale[g];
  for (int c = wave; c < nch; c += NW)  // W0 digit image -> LDS (shared by the four waves)
    *reinterpret_cast<v4i*>(&s_w0[c * 1024 + lane * 16]) =
        *reinterpret_cast<const v4i*>(st.dig + bd.dig_off + ((int64_t)c * 64 + lane) * 16);
  // retire the prologue loads and hide their provenance: inside the tile loop the
  // only vector-memory waits are the explicit, counted ones on this wave's DMAs
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("" : "+v"(zscale));
  __syncthreads();
  v4i rowsum64 = v4i{0, 0, 0, 0};  // the forward's facc[3] start (field 3 stored as code - 1)
  for (int c = 0; c < nch; ++c) rowsum64 = fx_rowsum64_acc(*reinterpret_cast<const v4i*>(&s_w0[c * 1024 + lane * 16]), rowsum64);
  // head weights as wave-uniform values: scalar registers for the whole item (the
  // per-tile LDS broadcasts serialised the head on their latencies)
  float uW[NL][4][4], uB[NH][4];
#pragma unroll
  for (int l = 0; l < NL; ++l) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        uW[l][j][k] = (l >= 1 && (l < NL - 1 || k == 0)) ? sgpr_f(s_hw[l][4 * j + k]) : 0.f;
    if (l < NH)
#pragma unroll
      for (int k = 0; k < 4; ++k) uB[l][k] = sgpr_f(s_hw[l][16 + k]);
  }


  // ---- accumulators ----
  v4i acc[32];  // dW0 digit sums per 16-marker window u (lane: column g, marker 16u + i16)
#pragma unroll
  for (int u = 0; u < 32; ++u) acc[u] = v4i{0, 0, 0, 0};
  v4i acc3 = v4i{0, 0, 0, 0};  // 64 sum over K-group 3 of the digits: field 3's -1, every marker
  int R[4] = {0, 0, 0, 0};  // running delta0 scale exponent per column (0 = unset)
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

#if FX_STAMPS
  unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ntl = 0;
  const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime(), mt0 = __builtin_amdgcn_s_memtime();
  unsigned long long t_last = mt0;
#endif
  for (; tt < te; tt += NW, sl ^= 1) {
    const bool more = tt + NW < te;
    const bool more2 = tt + 2 * NW < te;  // tile tt + 2 NW goes into this slot
    // tile tt (issued during tile tt - NW) has landed.  (An L2 prefetch of the
    // tile after it measured +3 %: with 8 waves/CU the L2 is already the DMA's
    // working set.)
    // the nch + 1 pieces of tile tt + NW are younger (loads return in order; a
    // younger pred store still outstanding only makes this wait longer)
    FX_STAMP(5);
    vm_wait(more ? nch + 1 : 0);
    FX_STAMP(0);
    const char* xs = &s_x[wave][sl][0];

    // ---- forward: Z0 of 64 individuals, exact int32 over all chunks ----
    // (software pipelined: the LDS reads of chunk c + 1 fly while chunk c's
    // four MFMAs issue; sched barriers keep the compiler from hoisting more)
    v4i facc[4] = {v4i{0, 0, 0, 0}, v4i{0, 0, 0, 0}, v4i{0, 0, 0, 0}, rowsum64};
    // the forward at raised priority too (with the stream issued in the backward:
    // -1.2 % per launch, A/B on one box)
    __builtin_amdgcn_s_setprio(1);
    {
      constexpr int FD = 2;  // two chunks ahead: an LDS read's latency exceeds one chunk's 4 MFMAs
      v4u Xq[FD];
      v4i Aq[FD];
#pragma unroll
      for (int c = 0; c < FD; ++c) {
        Xq[c] = v4u{0u, 0u, 0u, 0u};
        Aq[c] = v4i{0, 0, 0, 0};
        if (NCH != 0 || c < nch) {
          Xq[c] = (v4u)lds_tr8_pair(xs + c * 1024 + fo0, xs + c * 1024 + fo1);
          Aq[c] = *reinterpret_cast<const v4i*>(&s_w0[c * 1024 + lane * 16]);
        }
      }
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        if (NCH == 0 && c >= nch) continue;
        const v4u Xc = Xq[c % FD];
        const v4i Ac = Aq[c % FD];
        if (c + FD < 8 && (NCH != 0 || c + FD < nch)) {
          Xq[c % FD] = (v4u)lds_tr8_pair(xs + (c + FD) * 1024 + fo0, xs + (c + FD) * 1024 + fo1);
          Aq[c % FD] = *reinterpret_cast<const v4i*>(&s_w0[(c + FD) * 1024 + lane * 16]);
        }
        // the cumulative fragments x & 0x03, x & 0x0F, x & 0x3F, x (header)
#if FX_ABL & 1
        const v4i B0 = (v4i)Xc, B1 = (v4i)Xc, B2 = (v4i)Xc, B3 = (v4i)Xc;
#else
        const v4i B0 = (v4i)(Xc & 0x03030303u);
        const v4i B1 = (v4i)(Xc & 0x0F0F0F0Fu);
        const v4i B2 = (v4i)(Xc & 0x3F3F3F3Fu);
        const v4i B3 = (v4i)Xc;
#endif
        facc[0] = FX_MFMA(Ac, B0, facc[0]);
        facc[1] = FX_MFMA(Ac, B1, facc[1]);
        facc[2] = FX_MFMA(Ac, B2, facc[2]);
        facc[3] = FX_MFMA(Ac, B3, facc[3]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    FX_STAMP(1);
    // the head + digit phase is a dependent VALU chain: at raised priority it
    // takes the SIMD's issue slots ahead of the partner wave's independent
    // MFMA/unpack stream (measured -1 %)
    __builtin_amdgcn_s_setprio(1);
    // lane (column g, slot i16) holds individual 4 i16 + q in register q; transpose
    // so that lane L holds all four columns of individual 4 (L & 15) + (L >> 4)
    fx_fwd_fields(facc);  // F_q = 4^q S_q, exact
    float z0 = zscale * comb4(facc[0]), z1 = (0.25f * zscale) * comb4(facc[1]);
    float z2 = (0.0625f * zscale) * comb4(facc[2]), z3 = (0.015625f * zscale) * comb4(facc[3]);
    swap32(z0, z2);
    swap32(z1, z3);
    swap16(z0, z1);
    swap16(z2, z3);

    // ---- head: one individual per lane ----
    const int64_t row = 64 * (int64_t)tt + iota;
    const bool valid = row < n;
    const float yv = s_y[wave][sl][lane];
    float d[4];
#if FX_ABL & 4
    d[0] = z0 + yv, d[1] = z1, d[2] = z2, d[3] = z3;
    if (write_pred && valid) predb[row] = z0;
    rss += (double)z1;
#else
    {
      const auto& Wh = uW;
      const auto& Bh = uB;
      float z[NH][4], a[NH][4];
      z[0][0] = z0 + Bh[0][0];
      z[0][1] = z1 + Bh[0][1];
      z[0][2] = z2 + Bh[0][2];
      z[0][3] = z3 + Bh[0][3];
#pragma unroll
      for (int k = 0; k < 4; ++k) a[0][k] = act_h_t<ACT>(z[0][k]);
#pragma unroll
      for (int l = 1; l < NH; ++l) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float s = Bh[l][k];
#pragma unroll
          for (int j = 0; j < 4; ++j) s = fmaf(a[l - 1][j], Wh[l][j][k], s);
          z[l][k] = s;
          a[l][k] = act_h_t<ACT>(s);
        }
      }
      float out = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) out = fmaf(a[NH - 1][j], Wh[NL - 1][j][0], out);
      const float e = valid ? (net_err ? yv : out - yv) : 0.f;
      if (write_pred && valid) predb[row] = out;
      rss += (double)e * (double)e;
      float err[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dWo[j] = fmaf(a[NH - 1][j], e, dWo[j]);
        err[j] = e * Wh[NL - 1][j][0];
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
              sj = fmaf(dl[k], Wh[l][j][k], sj);
            }
            err[j] = sj;
          }
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) d[k] = dl[k];
        }
      }
    }
#endif

    if (more2) {  // the target has been read (yv in a register): its slot takes tile tt + 2 NW's
      asm volatile("" ::"v"(yv));
      issue_y(tt + 2 * NW, sl);
    }
    __builtin_amdgcn_sched_barrier(0);
    FX_STAMP(2);
    // the backward's first genotype windows: their LDS reads fly under the digit phase
    constexpr int PD = FXT_PD;
    uint32_t wq[PD];
#pragma unroll
    for (int u = 0; u < PD; ++u)
      wq[u] = (NCH != 0 || u < 4 * nch) ? *reinterpret_cast<const uint32_t*>(xs + 256 * u + ((u & 1) ? boo : boe)) : 0u;
    // ---- delta0 -> signed digits at the running per-column scale 2^(R - 132) ----
    // running scale check: a column needs a (new) scale only when some lane's
    // |delta| reaches 2^(R - 126) (or R is unset); then the exact wave max of
    // the exponent fields sets it (rare after the first tile)
    int dl[4] = {0, 0, 0, 0};
    bool grow = false;
    {
      bool lane_need = false;  // one ballot for the four columns (no compare -> branch chain)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int ek = (int)((fbits(d[k]) >> 23) & 0xFFu);
        lane_need |= ek > (R[k] ? R[k] : 5);
      }
      if (__builtin_amdgcn_ballot_w64(lane_need) != 0) {
        const uint32_t e01 = wave_max_u16x2(((fbits(d[0]) >> 23) & 0xFFu) | (((fbits(d[1]) >> 23) & 0xFFu) << 16));
        const uint32_t e23 = wave_max_u16x2(((fbits(d[2]) >> 23) & 0xFFu) | (((fbits(d[3]) >> 23) & 0xFFu) << 16));
        const int E[4] = {(int)(e01 & 0xFFFFu), (int)(e01 >> 16), (int)(e23 & 0xFFFFu), (int)(e23 >> 16)};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (E[k] >= 6 && (R[k] == 0 || E[k] > R[k])) {  // first scale, or |delta| outgrew it
            if (R[k] != 0) {
              dl[k] = E[k] + 2 - R[k];
              grow = true;
            }
            R[k] = E[k] + 2;
          }
        }
      }
    }
    if (grow) {  // rare: rescale the digit sums of the grown columns exactly
      const int sh = g == 0 ? dl[0] : g == 1 ? dl[1] : g == 2 ? dl[2] : dl[3];
#pragma unroll
      for (int u = 0; u < 32; ++u)
        if (NCH != 0 || u < 4 * nch) acc[u] = shr_digits(acc[u], sh);
      acc3 = shr_digits(acc3, sh);
    }
    v4u w;
    // this lane's individual sits in K-group p = g of the backward operand, whose
    // genotype codes stay in place (x 4^p): pre-divide its digits by 4^p
    const int kslot_sh = 2 * g;
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = digits4_fx(d[k], 153 - kslot_sh - (R[k] ? R[k] : 255));
    *reinterpret_cast<v4u*>(sd_w) = w;

    __builtin_amdgcn_sched_barrier(0);
    FX_STAMP(3);
    __builtin_amdgcn_s_setprio(0);
    // ---- backward: dW0 digit sums += G^T delta0 (reads 4 windows ahead) ----
    const v4i A = lds_tr8_pair(sd_r, sd_r + 8 * 16);
    acc3 = FX_MFMA(A, FX_ONES3, acc3);
    {
      // every field in place (x 1, 4, 16, 64 (f3 - 1); the digits carry 4^-p): 4 VALU
      auto unpack = [](uint32_t wv) -> v4i {
#if FX_ABL & 2
        return v4i{(int)wv, (int)wv, (int)wv, (int)wv};
#else
        return fx_bwd_unpack(wv);
#endif
      };
      // window u + 2 is unpacked beside window u's MFMA: the MFMA's B operand was
      // written two iterations earlier, so no VALU -> MFMA hazard padding per window
      v4i Bn = unpack(wq[0]), Bn2 = unpack(wq[1]);
#pragma unroll
      for (int u = 0; u < 32; ++u) {
        if (NCH == 0 && u >= 4 * nch) continue;
        const v4i Bv = Bn;
        Bn = Bn2;
        if (u + 2 < 32 && (NCH != 0 || u + 2 < 4 * nch)) Bn2 = unpack(wq[(u + 2) % PD]);
        if (more2 && (u & 3) == 1) {  // window 4c + 3, chunk c's last, is unpacked: refill chunk c
          asm volatile("" ::"v"(Bn2[0]), "v"(Bn2[1]), "v"(Bn2[2]), "v"(Bn2[3]));
          issue_chunk(tt + 2 * NW, sl, u >> 2);
        }
        if (u + PD < 32 && (NCH != 0 || u + PD < 4 * nch))  // slot of window u, consumed two iterations ago
          wq[u % PD] = *reinterpret_cast<const uint32_t*>(xs + 256 * (u + PD) + (((u + PD) & 1) ? boo : boe));
        acc[u] = FX_MFMA(A, Bv, acc[u]);
        if (FXT_SBB) __builtin_amdgcn_sched_barrier(0);
      }
    }
    FX_STAMP(4);
#if FX_STAMPS
    ++ntl;
#endif
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if FX_STAMPS
  ph[6] = __builtin_amdgcn_s_memrealtime() - rt0;
  ph[7] = __builtin_amdgcn_s_memtime() - mt0;
  if (lane == 0 && st.dbg) {
    for (int i = 0; i < 8; ++i) atomicAdd(&st.dbg[i], ph[i]);
    atomicAdd(&st.dbg[15], ntl);
  }
#endif

  // ---- workgroup reduction (fixed order: deterministic) ----
  {
    const double rs = wave_sum_d(rss);
    float hs[NS];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      hs[k] = wave_sum(db[0][k]);
      hs[4 + k] = wave_sum(dWo[k]);
    }
#pragma unroll
    for (int l = 1; l < NH; ++l)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        hs[8 + (l - 1) * 20 + k] = wave_sum(db[l][k]);
#pragma unroll
        for (int j = 0; j < 4; ++j) hs[8 + (l - 1) * 20 + 4 + 4 * j + k] = wave_sum(dW[l - 1][j][k]);
      }
    if (lane == 0) {
      s_rss[wave] = rs;
#pragma unroll
      for (int q = 0; q < NS; ++q) s_hs[wave][q] = hs[q];
    }
  }
  __syncthreads();  // every wave is done with its tile slots
  {
    const int Rl = g == 0 ? R[0] : g == 1 ? R[1] : g == 2 ? R[2] : R[3];
    float* red = reinterpret_cast<float*>(&s_x[wave][0][0]);
#pragma unroll
    for (int u = 0; u < 32; ++u)
      if (u < 4 * nch) red[u * 64 + lane] = Rl ? __builtin_amdgcn_ldexpf(comb4_exact2(acc[u], acc3), Rl - 153) : 0.f;
  }
  __syncthreads();
  float* part = st.part + it.part_at;
  // a fused update with more than one workgroup per branch: the partials are handed
  // to the branch's last arriving workgroup inside the launch, stored write-through
  // (sc1: no release fence needed; MI355X_MICROARCH.md, inter-workgroup visibility)
  const bool pub = UPD && upd_cnt != nullptr && (folds != nullptr || bd.nsplits > 1);
  auto pst = [&](float* a, float v) {
    if (pub)
      __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      *a = v;
  };
  float db0[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) db0[k] = (s_hs[0][k] + s_hs[1][k]) + (s_hs[2][k] + s_hs[3][k]);
  const int m = bd.m;
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) {
    const int u = wave * 8 + jj;
    if (u < 4 * nch) {
      const int idx = u * 64 + lane;
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) s += reinterpret_cast<const float*>(&s_x[w][0][0])[idx];
      const int mk = 16 * u + i16, c = g;
      if (mk < m && c < bd.widths[0]) {
        const float mu = st.mu[bd.mk_off + mk], sg = st.sigma[bd.mk_off + mk];
        const float dbc = c == 0 ? db0[0] : c == 1 ? db0[1] : c == 2 ? db0[2] : db0[3];
        pst(part + bd.woff[0] + c * m + mk, sg > 0.f ? (s - mu * dbc) / sg : 0.f);
      }
    }
  }
  if (wave == 0 && lane < NS) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += s_hs[w][lane];
    const int q = lane;
    if (q < 4) {
      if (q < bd.widths[0]) pst(part + bd.boff[0] + q, v);
    } else if (q < 8) {
      const int j = q - 4;
      if (j < bd.win[NL - 1]) pst(part + bd.woff[NL - 1] + j, v);
    } else {
      const int l = 1 + (q - 8) / 20, r = (q - 8) % 20;
      if (r < 4) {
        if (r < bd.widths[l]) pst(part + bd.boff[l] + r, v);
      } else {
        const int j = (r - 4) >> 2, k = (r - 4) & 3;
        if (j < bd.win[l] && k < bd.widths[l]) pst(part + bd.woff[l] + k * bd.win[l] + j, v);
      }
    }
  }
  if (wave == 0 && lane == 0) {
    const double rs = (s_rss[0] + s_rss[1]) + (s_rss[2] + s_rss[3]);
    if (pub)
      __hip_atomic_store(st.rss_part + it.rss_at, rs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      st.rss_part[it.rss_at] = rs;
  }
  if constexpr (UPD) {
    // fused leapfrog update (bann_api.hip build_plan): the last of the branch's
    // workgroups to finish updates it here, with the update kernel's arithmetic and
    // reduction order (update_small as 512 virtual threads), instead of a second
    // launch -- after folding the branch's slabs first in a solo plan (folds: the
    // fold launch's order).  A branch of one split (no folds) has one workgroup:
    // this one, whose slab its own waves see after a workgroup barrier.  Otherwise
    // every wave drains its write-through partial stores, one lane counts the
    // arrival (agent scope), and the last arriver acquires before reading the slabs.
    __shared__ int s_last;
    __shared__ double s_redd[4 * 8];
    if (pub) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int narr = folds ? folds[it.fold_ix].nslab : bd.nsplits;
    if (threadIdx.x == 0)
      s_last = !pub || __hip_atomic_fetch_add(&upd_cnt[b], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == narr - 1;
    __syncthreads();
    if (s_last) {
      if (pub) {
        if (threadIdx.x == 0) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          upd_cnt[b] = 0;  // for the next launch (ordered by the kernel boundary)
        }
        __syncthreads();
      }
      if (folds) {
        fold_solo_all<64 * FX_WAVES>(st, folds[it.fold_ix], bd);
        __syncthreads();  // slab 0 and its rss, written by this workgroup, read by update_small
      }
      float* s_th = reinterpret_cast<float*>(&s_x[0][0][0]);  // the tile slots are free: P <= 2048 floats
      update_small<64 * FX_WAVES, 1, 2>(st, b, bd, upd_mode, false, upd_step, s_redd, s_th);
    }
  }
}

template <int NL, int NCH, int UPD>
static void launch_fx_nlu(const DevState& st, const GradItem* items, int32_t nitems, int act, int wp, int um, int us,
                          int32_t* cnt, const FoldJob* fo, hipStream_t s) {
  const dim3 grid((unsigned)nitems), block(64 * FX_WAVES);
  switch (act) {
    case 0: hipLaunchKernelGGL((k_fused_grad_fx<NL, 0, NCH, UPD>), grid, block, 0, s, st, items, wp, um, us, cnt, fo); break;
    case 1: hipLaunchKernelGGL((k_fused_grad_fx<NL, 1, NCH, UPD>), grid, block, 0, s, st, items, wp, um, us, cnt, fo); break;
    case 2: hipLaunchKernelGGL((k_fused_grad_fx<NL, 2, NCH, UPD>), grid, block, 0, s, st, items, wp, um, us, cnt, fo); break;
    case 3: hipLaunchKernelGGL((k_fused_grad_fx<NL, 3, NCH, UPD>), grid, block, 0, s, st, items, wp, um, us, cnt, fo); break;
    default: hipLaunchKernelGGL((k_fused_grad_fx<NL, 4, NCH, UPD>), grid, block, 0, s, st, items, wp, um, us, cnt, fo); break;
  }
}
template <int NL, int NCH>
static void launch_fx_nl(const DevState& st, const GradItem* items, int32_t nitems, int act, int wp, int um, int us,
                         int32_t* cnt, const FoldJob* fo, hipStream_t s) {
  if (cnt)
    launch_fx_nlu<NL, NCH, 1>(st, items, nitems, act, wp, um, us, cnt, fo, s);
  else
    launch_fx_nlu<NL, NCH, 0>(st, items, nitems, act, wp, um, us, nullptr, nullptr, s);
}

// full8: every branch of this launch group has exactly 8 chunks; upd_cnt != null:
// the fused leapfrog update in the launch's tail (mode upd_mode, step upd_step),
// folds != null: a solo plan's fold jobs, run by the tail before the update
void launch_fused_grad_fx(const DevState& st, const GradItem* items, int32_t nitems, int32_t L, int32_t act,
                          int full8, int write_pred, int upd_mode, int upd_step, int32_t* upd_cnt,
                          const FoldJob* folds, hipStream_t s) {
  if (nitems <= 0) return;
  const int wp = write_pred, um = upd_mode, us = upd_step;
  const FoldJob* fo = upd_cnt ? folds : nullptr;
  switch (L * 2 + (full8 ? 1 : 0)) {
    case 4: launch_fx_nl<2, 0>(st, items, nitems, act, wp, um, us, upd_cnt, fo, s); break;
    case 5: launch_fx_nl<2, 8>(st, items, nitems, act, wp, um, us, upd_cnt, fo, s); break;
    case 6: launch_fx_nl<3, 0>(st, items, nitems, act, wp, um, us, upd_cnt, fo, s); break;
    case 7: launch_fx_nl<3, 8>(st, items, nitems, act, wp, um, us, upd_cnt, fo, s); break;
    case 8: launch_fx_nl<4, 0>(st, items, nitems, act, wp, um, us, upd_cnt, fo, s); break;
    case 9: launch_fx_nl<4, 8>(st, items, nitems, act, wp, um, us, upd_cnt, fo, s); break;
    default: break;
  }
}

// ===========================================================================
// Forward-only fx pass: f_b(theta) of every individual (forward_feed,
// branch_sampler.rs:743-782, at the output neuron), no target, no backward.
// Network-joint HMC needs the summed branch outputs before any branch can form
// its output error, so each of its leapfrog steps starts with this pass; the
// prediction paths (bann_predict*, stale rows before a target rebuild) use it
// too.  Same tiles, work items, W0 digits and head as k_fused_grad_fx; the
// stream runs two tiles ahead in the wave's two slots, the refill of a slot is
// issued once the forward has read it (the head's prediction store first, so
// the counted wait at the top never waits on a piece younger than the tile).
// ===========================================================================
#ifndef FWD_NU
#define FWD_NU 3  // 8-chunk forward: half-tile units per wave (0: whole-tile slots, the A/B variant)
#endif
#ifndef FWD_ABL
#define FWD_ABL 0  // timing ablations of the ring forward (tools only; results wrong): 1 no MFMA, 2 no head, 4 no stream,
                  // 8 predictions stored by wave 0 only
#endif
#ifndef FWD_PB
#define FWD_PB 8  // ring forward: tiles per prediction write burst (1: one store per tile, counted in the waits:
                  // kbench 1.134 vs 1.173 ms, but 1.203 vs 1.181 ms inside the network trajectory)
#endif
#ifndef FWD_PBC
#define FWD_PBC 0  // PB > 1: count the bursts' stores in the waits too
#endif
#ifndef FWD_NS
#define FWD_NS 2  // tile slots per wave: the stream runs FWD_NS tiles ahead (2: two workgroups per CU;
                  // round 5, network line A/B: 379.6 / 381.2 vs 376.0 / 377.2 steps/s with 4, 376.6 / 378.2 with 3)
#endif
// all but the youngest k (0 .. 31) vector-memory operations of this wave are complete
__device__ __forceinline__ void vm_wait_n(int k) {
#define VMW(i) \
  case i: asm volatile("s_waitcnt vmcnt(" #i ")" ::: "memory"); break;
  switch (k) {
    VMW(1) VMW(2) VMW(3) VMW(4) VMW(5) VMW(6) VMW(7) VMW(8) VMW(9) VMW(10) VMW(11) VMW(12) VMW(13) VMW(14)
    VMW(15) VMW(16) VMW(17) VMW(18) VMW(19) VMW(20) VMW(21) VMW(22) VMW(23) VMW(24) VMW(25) VMW(26) VMW(27)
    VMW(28) VMW(29) VMW(30) VMW(31)
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
#undef VMW
}

// NU > 0 (8-chunk tiles): the half-tile ring, NU units of 4 KiB per wave and the W0 digits in
// registers (no LDS copy), so that 4 NU KiB per wave set the workgroups per CU
template <int NL, int ACT, int NCH, int NU>
__global__ void __launch_bounds__(64 * FX_WAVES, NU > 0 ? 2 : (FWD_NS <= 2 ? 2 : 1))
    k_forward_fx(DevState st, const GradItem* __restrict__ items) {
  constexpr int NH = NL - 1;
  constexpr int NW = FX_WAVES;
  constexpr int NS = FWD_NS;
  static_assert(NU == 0 || NCH == 8, "the half-tile ring needs 8-chunk tiles");
  __shared__ __attribute__((aligned(16))) char s_x[NW][NU > 0 ? 1 : NS][NU > 0 ? NU * 4096 : FX_SLOT];
  __shared__ __attribute__((aligned(16))) char s_w0[NU > 0 ? 16 : 8 * 1024];
  __shared__ __attribute__((aligned(16))) float s_hw[NL][20];

  const GradItem it = items[blockIdx.x];
  const int b = it.branch;
  const BranchDev& bd = st.br[b];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int nch = NCH ? NCH : bd.nchunks;
  const int64_t n = st.n;
  const int tb = it.frag_begin >> 2, te = (it.frag_end + 3) >> 2;

  const float* th = st.theta + bd.p_off;
  for (int t = threadIdx.x; t < NL * 20; t += 64 * NW) {
    const int l = t / 20, r = t - l * 20;
    float v = 0.f;
    if (r < 16) {
      const int j = r >> 2, k = r & 3;
      if (l >= 1 && j < bd.win[l] && k < bd.widths[l]) v = th[bd.woff[l] + k * bd.win[l] + j];
    } else {
      const int k = r - 16;
      if (l == 0 && k < bd.widths[0]) v = st.fc[b].c0[k];
      if (l >= 1 && l < NH && k < bd.widths[l]) v = th[bd.boff[l] + k];
    }
    s_hw[l][r] = v;
  }
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 1, tp = lane & 1;
  float zscale = st.fc[b].scale[g];
  v4i Areg[NU > 0 ? 8 : 1];  // the ring's W0 digit operands, one per chunk
  if constexpr (NU > 0) {
#pragma unroll
    for (int c = 0; c < 8; ++c) Areg[c] = *reinterpret_cast<const v4i*>(st.dig + bd.dig_off + ((int64_t)c * 64 + lane) * 16);
  } else {
    for (int c = wave; c < nch; c += NW)
      *reinterpret_cast<v4i*>(&s_w0[c * 1024 + lane * 16]) =
          *reinterpret_cast<const v4i*>(st.dig + bd.dig_off + ((int64_t)c * 64 + lane) * 16);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("" : "+v"(zscale));
  __syncthreads();
  v4i rowsum64 = v4i{0, 0, 0, 0};  // facc[3]'s start (field 3 stored as code - 1)
  if constexpr (NU > 0) {
#pragma unroll
    for (int c = 0; c < 8; ++c) rowsum64 = fx_rowsum64_acc(Areg[c], rowsum64);
  } else {
    for (int c = 0; c < nch; ++c) rowsum64 = fx_rowsum64_acc(*reinterpret_cast<const v4i*>(&s_w0[c * 1024 + lane * 16]), rowsum64);
  }
  float uWm[NL][4][4], uB[NH][4];  // head weights W_l[j][k] (l >= 1; output layer: k = 0) and biases, scalar
#pragma unroll
  for (int l = 0; l < NL; ++l) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        uWm[l][j][k] = (l >= 1 && (l < NL - 1 || k == 0)) ? sgpr_f(s_hw[l][4 * j + k]) : 0.f;
    if (l < NH)
#pragma unroll
      for (int k = 0; k < 4; ++k) uB[l][k] = sgpr_f(s_hw[l][16 + k]);
  }

  const int gsw = g & 1;
  const uint32_t fo0 = (uint32_t)((16 * g + tq + 8 * gsw) * 16 + 8 * (tp ^ gsw));
  const uint32_t fo1 = (uint32_t)((16 * g + tq + 8 * (1 ^ gsw)) * 16 + 8 * (tp ^ 1 ^ gsw));
  const int iota = 4 * i16 + g;
  float* predb = st.pred + bd.y_off;
  const char* xsrc = reinterpret_cast<const char*>(st.xu2) + bd.x_off + lane * 16;
  const int64_t tile_bytes = (int64_t)nch * 1024;
  // the last chunk's padding rows are not streamed (as in k_fused_grad_fx)
  const bool pad_row = 64 * (nch - 1) + 16 * (lane >> 4) + (((lane & 15) - 8 * ((lane >> 4) & 1)) & 15) >= bd.m;
  auto issue_chunk = [&](int tt, int sl, int c) {
    if (c == nch - 1 && pad_row) return;
    if constexpr (NU == 0) glds16(xsrc + (int64_t)tt * tile_bytes + c * 1024, &s_x[wave][sl][c * 1024]);
  };

  // the head of one tile: in-place fields -> z (one individual per lane) -> f
  auto head_out = [&](v4i (&facc)[4]) -> float {
    fx_fwd_fields(facc);
    float z0 = zscale * comb4(facc[0]), z1 = (0.25f * zscale) * comb4(facc[1]);
    float z2 = (0.0625f * zscale) * comb4(facc[2]), z3 = (0.015625f * zscale) * comb4(facc[3]);
    swap32(z0, z2);
    swap32(z1, z3);
    swap16(z0, z1);
    swap16(z2, z3);
    float a[4];
    a[0] = act_h_t<ACT>(z0 + uB[0][0]);
    a[1] = act_h_t<ACT>(z1 + uB[0][1]);
    a[2] = act_h_t<ACT>(z2 + uB[0][2]);
    a[3] = act_h_t<ACT>(z3 + uB[0][3]);
#pragma unroll
    for (int l = 1; l < NH; ++l) {
      float an[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float s = uB[l][k];
#pragma unroll
        for (int j = 0; j < 4; ++j) s = fmaf(a[j], uWm[l][j][k], s);
        an[k] = act_h_t<ACT>(s);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) a[k] = an[k];
    }
    float out = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) out = fmaf(a[j], uWm[NL - 1][j][0], out);
    return out;
  };
  if constexpr (NU > 0) {
    // Half-tile ring: NU slots of one 4-chunk unit each (unit u = half u & 1 of the wave's
    // tile u >> 1); NU - 1 units are in flight while one is read.  A wave owns a contiguous
    // run of the item's tiles and writes its predictions PB tiles at a time (PB x 256 bytes,
    // back to back): single 256-byte stores between the stream's reads cost the launch a
    // fifth of its time (profiles/r05_fwd_store_ablation.md).
    constexpr int PB = FWD_PB;
    char* const xw = &s_x[wave][0][0];
    const int q = (te - tb + NW - 1) / NW;
    const int tw0 = tb + wave * q;
    const int nt = te - tw0 < 0 ? 0 : (te - tw0 < q ? te - tw0 : q);
    const int nu = 2 * nt;
    auto issue_unit = [&](int u) {
      if constexpr (FWD_ABL & 4) return;
      const int64_t tt = tw0 + (u >> 1);
      char* dst = xw + (u % NU) * 4096;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int cc = 4 * (u & 1) + c;
        if (cc == nch - 1 && pad_row) continue;
        glds16(xsrc + tt * tile_bytes + cc * 1024, dst + c * 1024);
      }
    };
    for (int u = 0; u < NU && u < nu; ++u) issue_unit(u);
    for (int k0 = 0; k0 < nt; k0 += PB) {
      float obuf[PB];
#pragma unroll
      for (int j = 0; j < PB; ++j) {
        const int k = k0 + j;
        obuf[j] = 0.f;
        if (PB > 1 && k >= nt) break;
        v4i facc[4] = {v4i{0, 0, 0, 0}, v4i{0, 0, 0, 0}, v4i{0, 0, 0, 0}, rowsum64};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int u = 2 * k + h;
          // younger than unit u: the units issued after it (through u + NU - 1, four pieces
          // each) and, with one prediction store per tile (PB = 1), the stores of tiles kb
          // that ended after u was issued (tile kb stores right after issuing unit
          // 2 kb + 1 + NU): kb in [ceil((u - NU - 1) / 2), floor((u - 2) / 2)].  Vector memory
          // operations leave vmcnt in issue order on gfx9 (loads, stores and LDS-DMA alike),
          // so counting them is exact; a wait that left the stores out would also wait for
          // them, i.e. for the whole ring behind a store to HBM (profiles/r05_fwd_store_ablation.md).
          // The stores of tiles before a wave's last are full (every row < n), so each is one
          // issued instruction.
          const int last = u + NU - 1 < nu - 1 ? u + NU - 1 : nu - 1;
          int younger_st = 0;
          if constexpr ((PB == 1 || FWD_PBC) && !(FWD_ABL & 8)) {
            const int lo = u - NU - 1 <= 0 ? 0 : (u - NU) >> 1, hi = (u - 2) >> 1;
            if (u >= 2)  // PB > 1: the tiles that end a burst (kb % PB == PB - 1) store PB rows of 64
              for (int kb = lo; kb <= hi; ++kb) younger_st += (PB == 1 || kb % PB == PB - 1) ? PB : 0;
          }
          if constexpr (!(FWD_ABL & 4)) vm_wait_n(4 * (last - u) + younger_st);
          const char* xs = xw + (u % NU) * 4096;
          v4u Xq[2];
#pragma unroll
          for (int c = 0; c < 2; ++c) Xq[c] = (v4u)lds_tr8_pair(xs + c * 1024 + fo0, xs + c * 1024 + fo1);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const v4u Xc = Xq[c % 2];
            if (c + 2 < 4) Xq[c % 2] = (v4u)lds_tr8_pair(xs + (c + 2) * 1024 + fo0, xs + (c + 2) * 1024 + fo1);
            if constexpr (FWD_ABL & 1) {
              facc[c] ^= (v4i)Xc;
            } else {
              fx_fwd_chunk(Areg[4 * h + c], Xc, facc);
            }
            __builtin_amdgcn_sched_barrier(0);
          }
          // every read of this unit's slot has returned (the MFMAs consumed them): refill it
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          if (u + NU < nu) issue_unit(u + NU);
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (FWD_ABL & 2) {
          obuf[j] = (float)(facc[0].x ^ facc[1].y ^ facc[2].z ^ facc[3].w);
        } else {
          obuf[j] = head_out(facc);
        }
      }
#pragma unroll
      for (int j = 0; j < PB; ++j) {
        const int64_t row = 64 * (int64_t)(tw0 + k0 + j) + iota;
        if (k0 + j < nt && row < n && (!(FWD_ABL & 8) || wave == 0)) predb[row] = obuf[j];
      }
    }
  } else {
  // ring of NS slots: tile i of this wave in slot i % NS; the prologue fills the
  // ring, each iteration refills the slot it consumed with the tile NS ahead
  int tt = tb + wave, sl = 0;
  for (int j = 0; j < NS; ++j)
    if (tt + j * NW < te)
      for (int c = 0; c < nch; ++c) issue_chunk(tt + j * NW, j, c);
  for (; tt < te; tt += NW, sl = (sl + 1) % NS) {
    int ahead = 0;  // later tiles of the ring in flight: their pieces are younger than this tile's
    for (int j = 1; j < NS; ++j) ahead += tt + j * NW < te;
    vm_wait_n(ahead * nch);
    const char* xs = &s_x[wave][sl][0];
    v4i facc[4] = {v4i{0, 0, 0, 0}, v4i{0, 0, 0, 0}, v4i{0, 0, 0, 0}, rowsum64};
    {
      constexpr int FD = 2;
      v4u Xq[FD];
      v4i Aq[FD];
#pragma unroll
      for (int c = 0; c < FD; ++c) {
        Xq[c] = v4u{0u, 0u, 0u, 0u};
        Aq[c] = v4i{0, 0, 0, 0};
        if (NCH != 0 || c < nch) {
          Xq[c] = (v4u)lds_tr8_pair(xs + c * 1024 + fo0, xs + c * 1024 + fo1);
          Aq[c] = *reinterpret_cast<const v4i*>(&s_w0[c * 1024 + lane * 16]);
        }
      }
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        if (NCH == 0 && c >= nch) continue;
        const v4u Xc = Xq[c % FD];
        const v4i Ac = Aq[c % FD];
        if (c + FD < 8 && (NCH != 0 || c + FD < nch)) {
          Xq[c % FD] = (v4u)lds_tr8_pair(xs + (c + FD) * 1024 + fo0, xs + (c + FD) * 1024 + fo1);
          Aq[c % FD] = *reinterpret_cast<const v4i*>(&s_w0[(c + FD) * 1024 + lane * 16]);
        }
        fx_fwd_chunk(Ac, Xc, facc);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    {
      const float out = head_out(facc);
      const int64_t row = 64 * (int64_t)tt + iota;
      if (row < n) predb[row] = out;
    }
    // every read of this slot has returned (the MFMAs consumed them): refill it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (tt + NS * NW < te)
      for (int c = 0; c < nch; ++c) issue_chunk(tt + NS * NW, sl, c);
  }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int NL, int NCH>
static void launch_fwd_nl(const DevState& st, const GradItem* items, int32_t nitems, int act, hipStream_t s) {
  const dim3 grid((unsigned)nitems), block(64 * FX_WAVES);
  switch (act) {
    case 0: hipLaunchKernelGGL((k_forward_fx<NL, 0, NCH, NCH == 8 ? FWD_NU : 0>), grid, block, 0, s, st, items); break;
    case 1: hipLaunchKernelGGL((k_forward_fx<NL, 1, NCH, NCH == 8 ? FWD_NU : 0>), grid, block, 0, s, st, items); break;
    case 2: hipLaunchKernelGGL((k_forward_fx<NL, 2, NCH, NCH == 8 ? FWD_NU : 0>), grid, block, 0, s, st, items); break;
    case 3: hipLaunchKernelGGL((k_forward_fx<NL, 3, NCH, NCH == 8 ? FWD_NU : 0>), grid, block, 0, s, st, items); break;
    default: hipLaunchKernelGGL((k_forward_fx<NL, 4, NCH, NCH == 8 ? FWD_NU : 0>), grid, block, 0, s, st, items); break;
  }
}

void launch_forward_fx(const DevState& st, const GradItem* items, int32_t nitems, int32_t L, int32_t act, int full8,
                       hipStream_t s) {
  if (nitems <= 0) return;
  switch (L * 2 + (full8 ? 1 : 0)) {
    case 4: launch_fwd_nl<2, 0>(st, items, nitems, act, s); break;
    case 5: launch_fwd_nl<2, 8>(st, items, nitems, act, s); break;
    case 6: launch_fwd_nl<3, 0>(st, items, nitems, act, s); break;
    case 7: launch_fwd_nl<3, 8>(st, items, nitems, act, s); break;
    case 8: launch_fwd_nl<4, 0>(st, items, nitems, act, s); break;
    case 9: launch_fwd_nl<4, 8>(st, items, nitems, act, s); break;
    default: break;
  }
}

// ===========================================================================
// Network-mode forward with per-group output sums (bann_network_hmc_step; fx branches of
// 8 chunks).  A network step needs sum_b f_b only, not the branch outputs.  A work item is a
// GROUP of up to 8 R branches over one range of T <= GS_TMAX tiles; its 8 waves take the
// group in R passes of 8 branches (wave w: branch 8 r + w of the item's list), each branch
// through the half-tile ring of k_forward_fx (its W0 digits in registers, its head weights in
// scalar registers), PB = 8 tiles of outputs in registers.  Per block of 8 tiles the waves
// put them in LDS (double-buffered, one barrier); thread t then adds tile t >> 6, individual
// t & 63 over the 8 waves in wave order and accumulates it into the item's LDS sum over the
// passes in pass order (the same thread every pass: deterministic, no second barrier).  The
// item's row -- one per 8 R branches -- is stored once, at the end.  Measured (round 6,
// profiles/r06_net_gsum_ab.txt): per-branch rows (200 MB per launch) cost the forward
// 0.26 ms, one row per 8 branches written block by block (25 MB) still 0.11 ms -- the
// stores interleaved with the read stream, not their waits -- so the rows are few and late.
// The per-branch rows the trajectory's end needs come from the last step's per-branch
// forward (bann_dist.hip).
// ===========================================================================
#define GS_TMAX 100  // tiles per item (the LDS sum: 25 KiB)
template <int NL, int ACT>
__global__ void __launch_bounds__(64 * 8, 1)
    k_forward_gsum(DevState st, const NetGroupItem* __restrict__ items, const int32_t* __restrict__ blist,
                   float* __restrict__ gsum) {
  constexpr int NH = NL - 1;
  constexpr int NW = 8;
  constexpr int NU = 3;   // half-tile units per wave in the ring
  constexpr int PB = 8;   // tiles per block
  __shared__ __attribute__((aligned(16))) char s_x[NW][NU * 4096];
  __shared__ __attribute__((aligned(16))) float s_o[2][NW][PB][64];
  __shared__ __attribute__((aligned(16))) float s_acc[GS_TMAX][64];
  __shared__ float s_hw[NW][NL][20];

  const NetGroupItem* itp = items + blockIdx.x;  // fields read in place (a private copy indexed by
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // the wave would go to LDS)
  const int lane = threadIdx.x & 63;
  const int tb = itp->tile_begin, nt = itp->tile_end - itp->tile_begin;
  const int nbr = itp->nbr, loff = itp->list_off;
  const int passes = (nbr + NW - 1) / NW;
  const int64_t n = st.n;
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 1, tp = lane & 1;
  const int gsw = g & 1;
  const uint32_t fo0 = (uint32_t)((16 * g + tq + 8 * gsw) * 16 + 8 * (tp ^ gsw));
  const uint32_t fo1 = (uint32_t)((16 * g + tq + 8 * (1 ^ gsw)) * 16 + 8 * (tp ^ 1 ^ gsw));
  const int iota = 4 * i16 + g;
  constexpr int64_t tile_bytes = 8 * 1024;
  char* const xw = &s_x[wave][0];
  const int nblk = (nt + PB - 1) / PB;
  // thread t's share of every block: tile t >> 6, individual t & 63 (also its LDS sum entries)
  const int jt = threadIdx.x >> 6, ind = threadIdx.x & 63;
  int gb = 0;  // running block count (the parity of the s_o buffer)
  for (int r = 0; r < passes; ++r) {
    const int bi = NW * r + wave;
    const int bw = bi < nbr ? __builtin_amdgcn_readfirstlane(blist[loff + bi]) : -1;
    const bool act_w = bw >= 0;  // wave-uniform: the last pass's waves may have no branch
    const int b = act_w ? bw : __builtin_amdgcn_readfirstlane(blist[loff]);
    const BranchDev& bd = st.br[b];
    const float* th = st.theta + bd.p_off;
    for (int t = lane; t < NL * 20; t += 64) {
      const int l = t / 20, rr = t - l * 20;
      float v = 0.f;
      if (rr < 16) {
        const int j = rr >> 2, k = rr & 3;
        if (l >= 1 && j < bd.win[l] && k < bd.widths[l]) v = th[bd.woff[l] + k * bd.win[l] + j];
      } else {
        const int k = rr - 16;
        if (l == 0 && k < bd.widths[0]) v = st.fc[b].c0[k];
        if (l >= 1 && l < NH && k < bd.widths[l]) v = th[bd.boff[l] + k];
      }
      s_hw[wave][l][rr] = v;
    }
    float zscale = st.fc[b].scale[g];
    v4i Areg[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) Areg[c] = *reinterpret_cast<const v4i*>(st.dig + bd.dig_off + ((int64_t)c * 64 + lane) * 16);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // (the ring is empty between passes)
    asm volatile("" : "+v"(zscale));
    v4i rowsum64 = v4i{0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < 8; ++c) rowsum64 = fx_rowsum64_acc(Areg[c], rowsum64);
    float uWm[NL][4][4], uB[NH][4];
#pragma unroll
    for (int l = 0; l < NL; ++l) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          uWm[l][j][k] = (l >= 1 && (l < NL - 1 || k == 0)) ? sgpr_f(s_hw[wave][l][4 * j + k]) : 0.f;
      if (l < NH)
#pragma unroll
        for (int k = 0; k < 4; ++k) uB[l][k] = sgpr_f(s_hw[wave][l][16 + k]);
    }
    const char* xsrc = reinterpret_cast<const char*>(st.xu2) + bd.x_off + lane * 16;
    const bool pad_row = 64 * 7 + 16 * (lane >> 4) + (((lane & 15) - 8 * ((lane >> 4) & 1)) & 15) >= bd.m;
    const int nu = act_w ? 2 * nt : 0;
    auto issue_unit = [&](int u) {
      const int64_t tt = tb + (u >> 1);
      char* dst = xw + (u % NU) * 4096;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int cc = 4 * (u & 1) + c;
        if (cc == 7 && pad_row) continue;  // lane 0 never pads: the wave's instruction always issues
        glds16(xsrc + tt * tile_bytes + cc * 1024, dst + c * 1024);
      }
    };
    auto head_out = [&](v4i (&facc)[4]) -> float {
      fx_fwd_fields(facc);
      float z0 = zscale * comb4(facc[0]), z1 = (0.25f * zscale) * comb4(facc[1]);
      float z2 = (0.0625f * zscale) * comb4(facc[2]), z3 = (0.015625f * zscale) * comb4(facc[3]);
      swap32(z0, z2);
      swap32(z1, z3);
      swap16(z0, z1);
      swap16(z2, z3);
      float a[4];
      a[0] = act_h_t<ACT>(z0 + uB[0][0]);
      a[1] = act_h_t<ACT>(z1 + uB[0][1]);
      a[2] = act_h_t<ACT>(z2 + uB[0][2]);
      a[3] = act_h_t<ACT>(z3 + uB[0][3]);
#pragma unroll
      for (int l = 1; l < NH; ++l) {
        float an[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float sacc = uB[l][k];
#pragma unroll
          for (int j = 0; j < 4; ++j) sacc = fmaf(a[j], uWm[l][j][k], sacc);
          an[k] = act_h_t<ACT>(sacc);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) a[k] = an[k];
      }
      float out = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) out = fmaf(a[j], uWm[NL - 1][j][0], out);
      return out;
    };
    for (int u = 0; u < NU && u < nu; ++u) issue_unit(u);
    for (int blk = 0; blk < nblk; ++blk, ++gb) {
      const int k0 = blk * PB;
      float obuf[PB];
#pragma unroll
      for (int j = 0; j < PB; ++j) obuf[j] = 0.f;
      if (act_w) {
#pragma unroll
        for (int j = 0; j < PB; ++j) {
          const int k = k0 + j;
          if (k >= nt) continue;  // (not break: a break makes obuf a dynamically indexed array)
          v4i facc[4] = {v4i{0, 0, 0, 0}, v4i{0, 0, 0, 0}, v4i{0, 0, 0, 0}, rowsum64};
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int u = 2 * k + h;
            const int last = u + NU - 1 < nu - 1 ? u + NU - 1 : nu - 1;
            vm_wait_n(4 * (last - u));  // this wave issues nothing but the ring's pieces in the loop
            const char* xs = xw + (u % NU) * 4096;
            v4u Xq[2];
#pragma unroll
            for (int c = 0; c < 2; ++c) Xq[c] = (v4u)lds_tr8_pair(xs + c * 1024 + fo0, xs + c * 1024 + fo1);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const v4u Xc = Xq[c % 2];
              if (c + 2 < 4) Xq[c % 2] = (v4u)lds_tr8_pair(xs + (c + 2) * 1024 + fo0, xs + (c + 2) * 1024 + fo1);
              fx_fwd_chunk(Areg[4 * h + c], Xc, facc);
              __builtin_amdgcn_sched_barrier(0);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (u + NU < nu) issue_unit(u + NU);
          }
          __builtin_amdgcn_sched_barrier(0);
          obuf[j] = head_out(facc);
        }
      }
      // the block's outputs -> LDS (asm stores: no compiler drain of the DMA in front of them)
      float (*const so)[64] = s_o[gb & 1][wave];
#pragma unroll
      for (int j = 0; j < PB; ++j) lds_st_f32(&so[j][iota], obuf[j]);
      LDS_BARRIER();
      // thread t: tile jt of the block over the 8 waves in wave order, into the item's sum in pass order
      if (k0 + jt < nt) {
        float sacc = s_o[gb & 1][0][jt][ind];
#pragma unroll
        for (int w = 1; w < NW; ++w) sacc += s_o[gb & 1][w][jt][ind];
        float* a = &s_acc[k0 + jt][ind];
        lds_st_f32(a, r == 0 ? sacc : *a + sacc);
      }
    }
  }
  // the item's row: every thread stores the entries it accumulated (tile 8 blk + jt, individual ind)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  float* const grow = gsum + (int64_t)itp->row * n;
  for (int blk = 0; blk < nblk; ++blk) {
    const int k = blk * PB + jt;
    const int64_t row = 64 * (int64_t)(tb + k) + ind;
    if (k < nt && row < n) grow[row] = s_acc[k][ind];
  }
}

template <int NL>
static void launch_gsum_nl(const DevState& st, const NetGroupItem* items, int32_t nitems, const int32_t* blist,
                           int act, float* gsum, hipStream_t s) {
  const dim3 grid((unsigned)nitems), block(64 * 8);
  switch (act) {
    case 0: hipLaunchKernelGGL((k_forward_gsum<NL, 0>), grid, block, 0, s, st, items, blist, gsum); break;
    case 1: hipLaunchKernelGGL((k_forward_gsum<NL, 1>), grid, block, 0, s, st, items, blist, gsum); break;
    case 2: hipLaunchKernelGGL((k_forward_gsum<NL, 2>), grid, block, 0, s, st, items, blist, gsum); break;
    case 3: hipLaunchKernelGGL((k_forward_gsum<NL, 3>), grid, block, 0, s, st, items, blist, gsum); break;
    default: hipLaunchKernelGGL((k_forward_gsum<NL, 4>), grid, block, 0, s, st, items, blist, gsum); break;
  }
}

int forward_gsum_max_tiles() { return GS_TMAX; }

void launch_forward_gsum(const DevState& st, const NetGroupItem* items, int32_t nitems, const int32_t* blist,
                         int32_t L, int32_t act, float* gsum, hipStream_t s) {
  if (nitems <= 0) return;
  if (L == 2) launch_gsum_nl<2>(st, items, nitems, blist, act, gsum, s);
  if (L == 3) launch_gsum_nl<3>(st, items, nitems, blist, act, gsum, s);
  if (L == 4) launch_gsum_nl<4>(st, items, nitems, blist, act, gsum, s);
}

// ===========================================================================
// "fxl": the fx scheme for branches of 9 .. 64 marker chunks (m_b <= 4096, e.g.
// BASELINE config C2's 2 000-SNP branches).
//
// An fx wave keeps the int32 dW0 digit sums of ALL its branch's markers in
// registers (128 VGPRs at 8 chunks), so fx stops at 512 markers.  Here a
// workgroup of NW = ceil(chunks / 8) waves processes ONE 64-individual tile at a
// time and wave w owns a fixed block of <= 8 chunks for the whole item:
//   * forward: each wave's partial Z0 over its block (exact int32, one f32
//     conversion), published through LDS (double-buffered, one barrier per
//     tile) and summed in a fixed wave order -- identical in every wave;
//   * head + delta0 digits: in every wave (the same values, no second barrier);
//   * backward: dW0 digit sums of the wave's own block, in registers across all
//     tiles of the item, written straight to the partial slab at the end.
// The genotype block of the next tile streams into the wave's second LDS slot
// during the forward (LDS-DMA, counted vmcnt), as in fx.  The LDS holds the two
// tile slots, the delta0 digit image and the Z0 exchange (19 KiB per wave: two
// 4-wave workgroups per CU), so the W0/sigma digit operand is read from L2 into
// registers two chunks ahead with counted loads instead of an LDS image.
// ===========================================================================
#define FXL_MAXW 8
// k_fused_grad_fxh (below)
#define FXH_CPW 5   // chunks per compute wave (at most)
#define FXH_MAXC 7  // compute waves (+ the head wave: 8 waves)
#define FXH_NSL 4   // genotype slots per compute wave
#ifndef FXL_PD
#define FXL_PD 8  // backward genotype-window prefetch depth
#endif
// fxh compute waves without the per-window / per-chunk scheduling barriers (round 6, kbench at C2,
// three alternating reps: 0.0921 -> 0.0888 ms per launch; either alone 0.0899 / ~0.092; profiles/r06_fx_knobs.txt)
#ifndef FXH_SBB
#define FXH_SBB 0  // a scheduling barrier after each backward window (1: the round-5 schedule)
#endif
#ifndef FXH_SBF
#define FXH_SBF 0  // a scheduling barrier after each forward chunk (1: the round-5 schedule)
#endif
#ifndef FXL_DPRE
#define FXL_DPRE 31  // backward window after which the next tile's first digit loads issue (earlier: spills)
#endif

// one global_load_dwordx4 outside the compiler's wait model (counted by hand)
__device__ __forceinline__ v4i ld_counted(const char* p) {
  v4i d;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(d) : "v"(p) : "memory");
  return d;
}
// wait until at most k vector-memory ops are outstanding, and only then let d be used
__device__ __forceinline__ void vm_wait_tie(int k, v4i& d) {
  switch (k) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" : "+v"(d)::"memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" : "+v"(d)::"memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" : "+v"(d)::"memory"); break;
    default: asm volatile("s_waitcnt vmcnt(3)" : "+v"(d)::"memory"); break;
  }
}

int fxl_lds_bytes(int nw, int nl, int cpw) {
  const int ns = 8 + (nl - 2) * 20;
  return nw * (2 * cpw * 1024 + 4 * FX_DROW + 2 * 64 * 16) + 2 * 64 * 4 + nl * 20 * 4 + ns * 4;
}

// CPW: chunks per wave.  8 (branches of 33 .. 64 chunks): the wave's W0 digit
// operand is read from L2 two chunks ahead of its MFMAs, every tile.  4 (<= 32
// chunks, e.g. C2's 2 000 markers on 8 waves): the wave's four digit operands stay
// in registers for the whole item (16 VGPRs; its dW0 digit sums take 64): no digit
// traffic and no digit-load latency in the tile loop, half the per-wave work per
// tile at the same 8 waves per CU.
template <int NL, int ACT, int FULL, int CPW>
__global__ void __launch_bounds__(64 * FXL_MAXW, 1)
    k_fused_grad_fxl(DevState st, const GradItem* __restrict__ items, int write_pred) {
  // Counted digit loads only where the kernel fits in 256 VGPRs without spills
  // (every wave 8 chunks, <= 3 layers: C2's shape before CPW = 4): a spill of a
  // register whose load is still in flight would store garbage.  Elsewhere the
  // digit loads are ordinary loads under the compiler's own (conservative) waits.
  constexpr bool RES = CPW == 4;  // digit operands resident in registers
  constexpr bool CNT = FULL && NL <= 3 && !RES;
  constexpr int NWIN = 4 * CPW;   // 16-marker windows per wave
  constexpr int NH = NL - 1;
  constexpr int NS = 8 + (NH - 1) * 20;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int NW = __builtin_amdgcn_readfirstlane(blockDim.x >> 6);
  constexpr int SLOT = CPW * 1024;
  char* const s_x = lds;                                                    // [NW][2][SLOT]
  char* const s_dig = s_x + NW * 2 * SLOT;                                  // [NW][4 * FX_DROW]
  v4f* const s_xch = reinterpret_cast<v4f*>(s_dig + NW * 4 * FX_DROW);      // [2][NW][64]
  float* const s_y = reinterpret_cast<float*>(s_xch + 2 * NW * 64);         // [2][64]
  float* const s_hw = s_y + 128;                                            // [NL][20]
  float* const s_hs = s_hw + NL * 20;                                       // [NS]

  const GradItem it = items[blockIdx.x];
  const int b = it.branch;
  const BranchDev& bd = st.br[b];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int nch = bd.nchunks;
  const int cpw = FULL ? CPW : (nch + NW - 1) / NW;
  const int c0 = wave * cpw;
  const int cw = FULL ? CPW : (nch - c0 < cpw ? nch - c0 : cpw);  // >= 1 (NW = ceil(nch / CPW))
  const int64_t n = st.n;
  const int tb = it.frag_begin >> 2, te = (it.frag_end + 3) >> 2;

  const float* th = st.theta + bd.p_off;
  for (int t = threadIdx.x; t < NL * 20; t += 64 * NW) {
    const int l = t / 20, r = t - l * 20;
    float v = 0.f;
    if (r < 16) {
      const int j = r >> 2, k = r & 3;
      if (l >= 1 && j < bd.win[l] && k < bd.widths[l]) v = th[bd.woff[l] + k * bd.win[l] + j];
    } else {
      const int k = r - 16;
      if (l == 0 && k < bd.widths[0]) v = st.fc[b].c0[k];
      if (l >= 1 && l < NH && k < bd.widths[l]) v = th[bd.boff[l] + k];
    }
    s_hw[t] = v;
  }
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 1, tp = lane & 1;
  float zscale = st.fc[b].scale[g];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("" : "+v"(zscale));
  __syncthreads();
  float uW[NL][4][4], uB[NH][4];  // head weights in scalar registers (as fx)
#pragma unroll
  for (int l = 0; l < NL; ++l) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        uW[l][j][k] = (l >= 1 && (l < NL - 1 || k == 0)) ? sgpr_f(s_hw[l * 20 + 4 * j + k]) : 0.f;
    if (l < NH)
#pragma unroll
      for (int k = 0; k < 4; ++k) uB[l][k] = sgpr_f(s_hw[l * 20 + 16 + k]);
  }

  const int gsw = g & 1;
  const uint32_t fo0 = (uint32_t)((16 * g + tq + 8 * gsw) * 16 + 8 * (tp ^ gsw));
  const uint32_t fo1 = (uint32_t)((16 * g + tq + 8 * (1 ^ gsw)) * 16 + 8 * (tp ^ 1 ^ gsw));
  const int pe = i16, po = (i16 + 8) & 15;
  const uint32_t boe = (uint32_t)(pe * 16 + 4 * (2 * ((g >> 1) ^ (pe >> 3)) + (g & 1)));
  const uint32_t boo = (uint32_t)(po * 16 + 4 * (2 * ((g >> 1) ^ (po >> 3)) + (g & 1)));
  const int iota = 4 * i16 + g;
  char* const sd = s_dig + wave * 4 * FX_DROW;
  char* const sd_w = sd + (i16 >> 2) * FX_DROW + (4 * g + (i16 & 3)) * 16;
  const char* const sd_r = sd + g * FX_DROW + tq * 16 + 8 * tp;
  const float* ybr = st.y + bd.y_off;
  float* predb = st.pred + bd.y_off;
  const int64_t tile_bytes = (int64_t)nch * 1024;
  const char* xsrc = reinterpret_cast<const char*>(st.xu2) + bd.x_off + (int64_t)c0 * 1024 + lane * 16;
  const char* dsrc = reinterpret_cast<const char*>(st.dig) + bd.dig_off + (int64_t)c0 * 1024 + lane * 16;
  char* const xslot0 = s_x + wave * 2 * SLOT;

  auto issue_chunk = [&](int tt, int sl, int c) {
    glds16(xsrc + (int64_t)tt * tile_bytes + c * 1024, xslot0 + sl * SLOT + c * 1024);
  };
  auto issue_y = [&](int tt, int sl) {  // wave 0 streams the tile's targets for every wave
    if (wave != 0) return;
    const int64_t row = 64 * (int64_t)tt + iota;
    glds4(ybr + (row < n ? row : n - 1), s_y + sl * 64);
  };

  v4i acc[NWIN];
#pragma unroll
  for (int u = 0; u < NWIN; ++u) acc[u] = v4i{0, 0, 0, 0};
  int R[4] = {0, 0, 0, 0};
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

  int tt = tb, sl = 0, xb = 0;
  auto ldig = [&](int off) -> v4i {
    if constexpr (CNT) return ld_counted(dsrc + off);
    return *reinterpret_cast<const v4i*>(dsrc + off);
  };
  v4i Dres[RES ? CPW : 1];  // RES: the wave's digit operands for the whole item
  if constexpr (RES) {
#pragma unroll
    for (int c = 0; c < CPW; ++c) Dres[c] = (FULL || c < cw) ? ldig(c * 1024) : v4i{0, 0, 0, 0};
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int c = 0; c < CPW; ++c) asm volatile("" : "+v"(Dres[c]));  // landed: no compiler waits in the loop
  }
  // field 3 stored as code - 1: z3 = (s / 64) comb4(C3 - C2) + s comb4(sum_k A) over the
  // wave's block (the float form: fxl's partials are f32 anyway, and an int32 start value
  // would take 4 more VGPRs in the counted 8-chunk waves)
  float zrow;
  {
    v4i rs = v4i{0, 0, 0, 0};
    if constexpr (RES) {
#pragma unroll
      for (int c = 0; c < CPW; ++c)
        if (FULL || c < cw) rs = fx_rowsum64_acc(Dres[c], rs);
    } else {
      for (int c = 0; c < cw; ++c) rs = fx_rowsum64_acc(*reinterpret_cast<const v4i*>(dsrc + c * 1024), rs);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    zrow = (0.015625f * zscale) * comb4(rs);
    asm volatile("" : "+v"(zrow));
  }
  if (tt < te) {
    for (int c = 0; c < cw; ++c) issue_chunk(tt, 0, c);
    issue_y(tt, 0);
  }
  v4i Dn0 = Dres[0], Dn1 = Dres[0];
  if constexpr (!RES) {
    Dn0 = ldig(0);
    Dn1 = Dn0;
    if (FULL || cw > 1) Dn1 = ldig(1024);
  }
  for (; tt < te; ++tt, sl ^= 1, xb ^= 1) {
    const bool more = tt + 1 < te;
    // this tile's genotype block (and targets) have landed; the two digit loads may fly
    if constexpr (RES)
      vm_wait(0);
    else
      vm_wait((FULL || cw > 1) ? 2 : 1);
    const char* xs = xslot0 + sl * SLOT;

    // ---- forward: partial Z0 over this wave's block ----
    v4i facc[4] = {v4i{0, 0, 0, 0}, v4i{0, 0, 0, 0}, v4i{0, 0, 0, 0}, v4i{0, 0, 0, 0}};
    {
      v4i Dg[CPW];
      if constexpr (RES) {
#pragma unroll
        for (int c = 0; c < CPW; ++c) Dg[c] = Dres[c];
      } else {
        Dg[0] = Dn0;
        Dg[1] = Dn1;
      }
      v4u Xc = (v4u)lds_tr8_pair(xs + fo0, xs + fo1);
#pragma unroll
      for (int c = 0; c < CPW; ++c) {
        if (!FULL && c >= cw) continue;
        v4u Xn = Xc;
        if (c + 1 < CPW && (FULL || c + 1 < cw))
          Xn = (v4u)lds_tr8_pair(xs + (c + 1) * 1024 + fo0, xs + (c + 1) * 1024 + fo1);
        if constexpr (CNT) {
          // loads younger than digit load c (issue order below: D(c+2) then
          // piece c per chunk, the pieces issued on every tile so the count is a
          // compile-time constant -- a runtime count would need a branch, and the
          // compiler copies the tied register ahead of the wait on one side)
          constexpr int young_c[8] = {1, 2, 3, 3, 3, 3, 3, 2};
          vm_wait_tie(young_c[c], Dg[c]);
        }
        if (!RES && c + 2 < CPW && (FULL || c + 2 < cw)) Dg[c + 2] = ldig((c + 2) * 1024);
        if (more)
          issue_chunk(tt + 1, sl ^ 1, c);
        else if (CNT)  // last tile: a harmless L2-resident DMA keeps the counts fixed
          glds16(dsrc + c * 1024, xslot0 + (sl ^ 1) * SLOT + c * 1024);
        fx_fwd_chunk(Dg[c], Xc, facc);
        __builtin_amdgcn_sched_barrier(0);
        Xc = Xn;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    fx_fwd_fields(facc);  // F3 = 64 S3 - 64 sum_k A: zrow adds the latter back
    float z0 = zscale * comb4(facc[0]), z1 = (0.25f * zscale) * comb4(facc[1]);
    float z2 = (0.0625f * zscale) * comb4(facc[2]), z3 = fmaf(0.015625f * zscale, comb4(facc[3]), zrow);
    swap32(z0, z2);
    swap32(z1, z3);
    swap16(z0, z1);
    swap16(z2, z3);
    // ---- Z0 exchange: every wave sums the NW partials in wave order ----
    v4f* xw = s_xch + (xb * NW) * 64;
    lds_st_v4f(xw + wave * 64 + lane, v4f{z0, z1, z2, z3});
    LDS_BARRIER();
    {
      v4f zs = xw[lane];
      for (int w = 1; w < NW; ++w) zs += xw[w * 64 + lane];
      z0 = zs[0];
      z1 = zs[1];
      z2 = zs[2];
      z3 = zs[3];
    }

    // ---- head: one individual per lane (every wave, identical values) ----
    const int64_t row = 64 * (int64_t)tt + iota;
    const bool valid = row < n;
    const float yv = s_y[sl * 64 + lane];
    if (more) issue_y(tt + 1, sl ^ 1);
    float d[4];
    {
      const auto& Wh = uW;
      const auto& Bh = uB;
      float z[NH][4], a[NH][4];
      z[0][0] = z0 + Bh[0][0];
      z[0][1] = z1 + Bh[0][1];
      z[0][2] = z2 + Bh[0][2];
      z[0][3] = z3 + Bh[0][3];
#pragma unroll
      for (int k = 0; k < 4; ++k) a[0][k] = act_h_t<ACT>(z[0][k]);
#pragma unroll
      for (int l = 1; l < NH; ++l) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float s = Bh[l][k];
#pragma unroll
          for (int j = 0; j < 4; ++j) s = fmaf(a[l - 1][j], Wh[l][j][k], s);
          z[l][k] = s;
          a[l][k] = act_h_t<ACT>(s);
        }
      }
      float out = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) out = fmaf(a[NH - 1][j], Wh[NL - 1][j][0], out);
      const float e = valid ? out - yv : 0.f;
      if (write_pred && valid && wave == 0) predb[row] = out;
      rss += (double)e * (double)e;
      float err[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dWo[j] = fmaf(a[NH - 1][j], e, dWo[j]);
        err[j] = e * Wh[NL - 1][j][0];
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
              sj = fmaf(dl[k], Wh[l][j][k], sj);
            }
            err[j] = sj;
          }
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) d[k] = dl[k];
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // ---- delta0 -> signed digits at the running per-column scale (as fx) ----
    int dl[4] = {0, 0, 0, 0};
    bool grow = false;
    {
      bool lane_need = false;  // one ballot for the four columns (no compare -> branch chain)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int ek = (int)((fbits(d[k]) >> 23) & 0xFFu);
        lane_need |= ek > (R[k] ? R[k] : 5);
      }
      if (__builtin_amdgcn_ballot_w64(lane_need) != 0) {
        const uint32_t e01 = wave_max_u16x2(((fbits(d[0]) >> 23) & 0xFFu) | (((fbits(d[1]) >> 23) & 0xFFu) << 16));
        const uint32_t e23 = wave_max_u16x2(((fbits(d[2]) >> 23) & 0xFFu) | (((fbits(d[3]) >> 23) & 0xFFu) << 16));
        const int E[4] = {(int)(e01 & 0xFFFFu), (int)(e01 >> 16), (int)(e23 & 0xFFFFu), (int)(e23 >> 16)};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (E[k] >= 6 && (R[k] == 0 || E[k] > R[k])) {
            if (R[k] != 0) {
              dl[k] = E[k] + 2 - R[k];
              grow = true;
            }
            R[k] = E[k] + 2;
          }
        }
      }
    }
    if (grow) {
      const int sh = g == 0 ? dl[0] : g == 1 ? dl[1] : g == 2 ? dl[2] : dl[3];
#pragma unroll
      for (int u = 0; u < NWIN; ++u)
        if (FULL || u < 4 * cw) acc[u] = shr_digits(acc[u], sh);
    }
    v4u w;
    const int kslot_sh = g == 1 ? 2 : g == 2 ? 4 : 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = digits4_fx(d[k], 153 - kslot_sh - (R[k] ? R[k] : 255));
    *reinterpret_cast<v4u*>(sd_w) = w;
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(0);

    // ---- backward: dW0 digit sums of this wave's block += G^T delta0 ----
    const v4i A = lds_tr8_pair(sd_r, sd_r + 8 * 16);
    {
      constexpr int PD = FXL_PD < NWIN ? FXL_PD : NWIN;
      uint32_t wq[PD];
#pragma unroll
      for (int u = 0; u < PD; ++u)
        wq[u] = (FULL || u < 4 * cw) ? *reinterpret_cast<const uint32_t*>(xs + 256 * u + ((u & 1) ? boo : boe)) : 0u;
      // field 3 (stored as code - 1) decoded: ((x >> 6) + 1) & 3 per byte (fields 0-2 hold
      // codes <= 2, so the +1 never carries out of a byte)
      auto unpack = [](uint32_t wv) -> v4i {
        return v4i{(int)(wv & 0x03030303u), (int)(wv & 0x0C0C0C0Cu), (int)(wv & 0x30303030u),
                   (int)(((wv >> 6) + 0x01010101u) & 0x03030303u)};
      };
      v4i Bn = unpack(wq[0]), Bn2 = unpack(wq[1]);  // two windows ahead of their MFMA (as in fx)
#pragma unroll
      for (int u = 0; u < NWIN; ++u) {
        if (!FULL && u >= 4 * cw) continue;
        const v4i Bv = Bn;
        Bn = Bn2;
        if (u + 2 < NWIN && (FULL || u + 2 < 4 * cw)) Bn2 = unpack(wq[(u + 2) % PD]);
        if (u + PD < NWIN && (FULL || u + PD < 4 * cw))
          wq[u % PD] = *reinterpret_cast<const uint32_t*>(xs + 256 * (u + PD) + (((u + PD) & 1) ? boo : boe));
        acc[u] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, Bv, acc[u], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        // the next tile's first two digit operands, half a backward ahead of their use
        if (!RES && u == FXL_DPRE && more) {
          Dn0 = ldig(0);
          if (FULL || cw > 1) Dn1 = ldig(1024);
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- epilogue ----
  float* part = st.part + it.part_at;
  float db0[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) db0[k] = wave_sum(db[0][k]);
  if (wave == 0) {  // head statistics (identical in every wave)
    const double rs = wave_sum_d(rss);
    float hs[NS];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      hs[k] = db0[k];
      hs[4 + k] = wave_sum(dWo[k]);
    }
#pragma unroll
    for (int l = 1; l < NH; ++l)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        hs[8 + (l - 1) * 20 + k] = wave_sum(db[l][k]);
#pragma unroll
        for (int j = 0; j < 4; ++j) hs[8 + (l - 1) * 20 + 4 + 4 * j + k] = wave_sum(dW[l - 1][j][k]);
      }
    if (lane == 0) {
#pragma unroll
      for (int q = 0; q < NS; ++q) s_hs[q] = hs[q];
      st.rss_part[it.rss_at] = rs;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane < NS) {
      const float v = s_hs[lane];
      const int q = lane;
      if (q < 4) {
        if (q < bd.widths[0]) part[bd.boff[0] + q] = v;
      } else if (q < 8) {
        const int j = q - 4;
        if (j < bd.win[NL - 1]) part[bd.woff[NL - 1] + j] = v;
      } else {
        const int l = 1 + (q - 8) / 20, r = (q - 8) % 20;
        if (r < 4) {
          if (r < bd.widths[l]) part[bd.boff[l] + r] = v;
        } else {
          const int j = (r - 4) >> 2, k = (r - 4) & 3;
          if (j < bd.win[l] && k < bd.widths[l]) part[bd.woff[l] + k * bd.win[l] + j] = v;
        }
      }
    }
  }
  {  // this wave's markers: dW0 = (G^T delta0 - mu sum delta0) / sigma
    const int Rl = g == 0 ? R[0] : g == 1 ? R[1] : g == 2 ? R[2] : R[3];
    const float dbc = g == 0 ? db0[0] : g == 1 ? db0[1] : g == 2 ? db0[2] : db0[3];
    const int m = bd.m;
#pragma unroll
    for (int u = 0; u < NWIN; ++u) {
      if (!FULL && u >= 4 * cw) continue;
      const int mk = 16 * (4 * c0 + u) + i16;
      if (mk < m && g < bd.widths[0]) {
        const float s = Rl ? __builtin_amdgcn_ldexpf(comb4_exact(acc[u]), Rl - 153) : 0.f;
        const float mu = st.mu[bd.mk_off + mk], sg = st.sigma[bd.mk_off + mk];
        part[bd.woff[0] + g * m + mk] = sg > 0.f ? (s - mu * dbc) / sg : 0.f;
      }
    }
  }
}

template <int NL, int FULL, int CPW>
static void launch_fxl_nl(const DevState& st, const GradItem* items, int32_t nitems, int act, int nw, int wp,
                          hipStream_t s) {
  const dim3 grid((unsigned)nitems), block(64 * nw);
  const size_t shm = (size_t)fxl_lds_bytes(nw, NL, CPW);
#define FXL_GO(A)                                                                                      \
  do {                                                                                                 \
    static bool attr_ = false;                                                                         \
    if (!attr_) {                                                                                      \
      (void)hipFuncSetAttribute((const void*)k_fused_grad_fxl<NL, A, FULL, CPW>,                       \
                                hipFuncAttributeMaxDynamicSharedMemorySize, fxl_lds_bytes(FXL_MAXW, 4, CPW)); \
      attr_ = true;                                                                                    \
    }                                                                                                  \
    hipLaunchKernelGGL((k_fused_grad_fxl<NL, A, FULL, CPW>), grid, block, shm, s, st, items, wp);      \
  } while (0)
  switch (act) {
    case 0: FXL_GO(0); break;
    case 1: FXL_GO(1); break;
    case 2: FXL_GO(2); break;
    case 3: FXL_GO(3); break;
    default: FXL_GO(4); break;
  }
#undef FXL_GO
}

int fxl_cpw(int nchunks) {
  static const int force = getenv("BANN_FXL_CPW") ? atoi(getenv("BANN_FXL_CPW")) : 0;  // 8: the old scheme (A/B)
  return (nchunks <= 4 * FXL_MAXW && force != 8) ? 4 : 8;
}

// nw waves per workgroup (= ceil(chunks / cpw) of every branch of the launch);
// full: every branch has exactly cpw * nw chunks
bool fxh_takes(int nw, int cpw, int head);
template <int NL>
static void launch_fxh_nl(const DevState& st, const GradItem* items, int32_t nitems, int act, int nc, int wp,
                          int slot_kib, hipStream_t s);
void launch_fused_grad_fxl(const DevState& st, const GradItem* items, int32_t nitems, int32_t L, int32_t act,
                           int32_t nw, int32_t cpw, int full, int write_pred, int head, hipStream_t s) {
  if (nitems <= 0 || nw < 1 || nw > FXL_MAXW || (cpw != 4 && cpw != 8)) return;
  if (fxh_takes(nw, cpw, head) && L >= 2 && L <= 4) {  // the head-wave kernel: ceil(4 nw / 5) compute waves
    const int nc = (4 * nw + FXH_CPW - 1) / FXH_CPW;
    if (L == 2) launch_fxh_nl<2>(st, items, nitems, act, nc, write_pred, FXH_CPW, s);
    if (L == 3) launch_fxh_nl<3>(st, items, nitems, act, nc, write_pred, FXH_CPW, s);
    if (L == 4) launch_fxh_nl<4>(st, items, nitems, act, nc, write_pred, FXH_CPW, s);
    return;
  }
  switch (L * 4 + (full ? 2 : 0) + (cpw == 4 ? 1 : 0)) {
    case 8: launch_fxl_nl<2, 0, 8>(st, items, nitems, act, nw, write_pred, s); break;
    case 9: launch_fxl_nl<2, 0, 4>(st, items, nitems, act, nw, write_pred, s); break;
    case 10: launch_fxl_nl<2, 1, 8>(st, items, nitems, act, nw, write_pred, s); break;
    case 11: launch_fxl_nl<2, 1, 4>(st, items, nitems, act, nw, write_pred, s); break;
    case 12: launch_fxl_nl<3, 0, 8>(st, items, nitems, act, nw, write_pred, s); break;
    case 13: launch_fxl_nl<3, 0, 4>(st, items, nitems, act, nw, write_pred, s); break;
    case 14: launch_fxl_nl<3, 1, 8>(st, items, nitems, act, nw, write_pred, s); break;
    case 15: launch_fxl_nl<3, 1, 4>(st, items, nitems, act, nw, write_pred, s); break;
    case 16: launch_fxl_nl<4, 0, 8>(st, items, nitems, act, nw, write_pred, s); break;
    case 17: launch_fxl_nl<4, 0, 4>(st, items, nitems, act, nw, write_pred, s); break;
    case 18: launch_fxl_nl<4, 1, 8>(st, items, nitems, act, nw, write_pred, s); break;
    case 19: launch_fxl_nl<4, 1, 4>(st, items, nitems, act, nw, write_pred, s); break;
    default: break;
  }
}

// ===========================================================================
// k_fused_grad_fxh: fxl's one-tile-at-a-time scheme with the head in ONE wave.
//
// fxl repeats the head (hidden / summary / output layers, e, rss, delta0 and
// its digits) in every wave of the workgroup: at C2 (32 chunks, 8 waves) that
// is 8 x ~300 VALU per tile against 8 x 160 for the 2-bit unpack.  Here wave 0
// is the HEAD wave and waves 1 .. NC are COMPUTE waves owning <= 5 chunks each
// (C2: 7 waves of 5,5,5,5,4,4,4), software-pipelined two tiles deep with ONE
// workgroup barrier per phase p:
//   compute waves: backward of tile p - 2 (its delta0 digits published by the
//                  head wave in phase p - 1), then the LDS-DMA of tile
//                  p + NSL - 2 into the slot just freed, then the forward of
//                  tile p -> partial Z0 (f32, the per-column scale applied)
//                  into the exchange slot p % 2;
//   head wave:     the fixed-order sum of the NC partials of tile p - 1, the
//                  transpose to one individual per lane, the head, the delta0
//                  digits at the running per-column scale -> digit image
//                  (p - 1) % 2, with the scale shifts for the compute waves'
//                  digit sums.
// A tile stays resident in its compute waves' slots from its forward (phase
// p) to its backward (p + 2): NSL = 4 slots per wave (one tile two phases
// ahead in flight), 157 KiB of LDS at NC = 7: one workgroup per CU, two waves
// per SIMD, the head wave sharing its SIMD with one compute wave.
// Arithmetic per tile is fxl's (the same digits, int32 digit sums, head in
// f32); the Z0 partials are summed in compute-wave order, so the bits differ
// from fxl only through the partition of the chunks over waves.
// ===========================================================================

// slot_kib: the largest chunk count of a compute wave (one KiB per chunk and slot)
int fxh_lds_bytes(int nc, int nl, int slot_kib) {
  const int ns = 8 + (nl - 2) * 20;
  return nc * FXH_NSL * slot_kib * 1024 + 2 * nc * 64 * 16 + 2 * 4 * FX_DROW + 3 * 64 * 4 + 16 * 4 + nl * 20 * 4 +
         ns * 4 + 4 * 4;
}

template <int NL, int ACT>
__global__ void __launch_bounds__(64 * (FXH_MAXC + 1), 1)
    k_fused_grad_fxh(DevState st, const GradItem* __restrict__ items, int write_pred, int slot_kib) {
  constexpr int NH = NL - 1;
  constexpr int NS = 8 + (NH - 1) * 20;
  constexpr int NSL = FXH_NSL;
  const int SLOT = __builtin_amdgcn_readfirstlane(slot_kib) * 1024;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int NC = __builtin_amdgcn_readfirstlane((int)(blockDim.x >> 6) - 1);
  char* const s_x = lds;                                                // [NC][NSL][SLOT]
  v4f* const s_zx = reinterpret_cast<v4f*>(s_x + NC * NSL * SLOT);      // [2][NC][64]
  char* const s_d = reinterpret_cast<char*>(s_zx + 2 * NC * 64);        // [2][4 * FX_DROW]
  float* const s_y = reinterpret_cast<float*>(s_d + 2 * 4 * FX_DROW);   // [3][64]
  int* const s_sc = reinterpret_cast<int*>(s_y + 3 * 64);               // [2][8]: shift[4], R[4]
  float* const s_hw = reinterpret_cast<float*>(s_sc + 16);              // [NL][20]
  float* const s_hs = s_hw + NL * 20;                                   // [NS]
  float* const s_db0 = s_hs + NS;                                       // [4]

  const GradItem it = items[blockIdx.x];
  const int b = it.branch;
  const BranchDev& bd = st.br[b];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int64_t n = st.n;
  const int tb = it.frag_begin >> 2, te = (it.frag_end + 3) >> 2;
  const int T = te > tb ? te - tb : 0;
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 1, tp = lane & 1;
  float* const part = st.part + it.part_at;

  if (wave == 0) {
    // ================= head wave =================
    const float* th = st.theta + bd.p_off;
    for (int t = lane; t < NL * 20; t += 64) {
      const int l = t / 20, r = t - l * 20;
      float v = 0.f;
      if (r < 16) {
        const int j = r >> 2, k = r & 3;
        if (l >= 1 && j < bd.win[l] && k < bd.widths[l]) v = th[bd.woff[l] + k * bd.win[l] + j];
      } else {
        const int k = r - 16;
        if (l == 0 && k < bd.widths[0]) v = st.fc[b].c0[k];
        if (l >= 1 && l < NH && k < bd.widths[l]) v = th[bd.boff[l] + k];
      }
      s_hw[t] = v;
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    float uW[NL][4][4], uB[NH][4];
#pragma unroll
    for (int l = 0; l < NL; ++l) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          uW[l][j][k] = (l >= 1 && (l < NL - 1 || k == 0)) ? sgpr_f(s_hw[l * 20 + 4 * j + k]) : 0.f;
      if (l < NH)
#pragma unroll
        for (int k = 0; k < 4; ++k) uB[l][k] = sgpr_f(s_hw[l * 20 + 16 + k]);
    }
    const int iota = 4 * i16 + g;
    // the tile's targets -- or, in network mode, the network's output error (as fx)
    const bool net_err = st.nete != nullptr;
    const float* ybr = net_err ? st.nete : st.y + bd.y_off;
    float* predb = st.pred + bd.y_off;
    auto issue_y = [&](int k) {
      const int64_t row = 64 * (int64_t)(tb + k) + iota;
      glds4(ybr + (row < n ? row : n - 1), s_y + (k % 3) * 64);
    };
    if (T > 0) issue_y(0);
    if (T > 1) issue_y(1);
    const int wp = write_pred != 0;
    const int kslot_sh = 2 * g;  // K-group g's genotype field in place (x 4^g): digits pre-divided
    int R[4] = {0, 0, 0, 0};
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
    for (int p = 0; p < T + 2; ++p) {
      if (p >= 1 && p <= T) {
        const int k = p - 1;
        // y(k) has landed: younger are store(k - 2), y(k + 1), store(k - 1)
        vm_wait_n(wp * (k >= 2) + (k + 1 < T) + wp * (k >= 1));
        __builtin_amdgcn_s_setprio(1);
        // the NC partials in compute-wave order; FXH_MAXC loads issued together (past NC
        // they re-read the last partial, not added)
        const v4f* xz = s_zx + (k & 1) * NC * 64 + lane;
        v4f zp[FXH_MAXC];
#pragma unroll
        for (int w = 0; w < FXH_MAXC; ++w) zp[w] = xz[(w < NC ? w : NC - 1) * 64];
        v4f zs = zp[0];
#pragma unroll
        for (int w = 1; w < FXH_MAXC; ++w)
          if (w < NC) zs += zp[w];
        float z0 = zs[0], z1 = zs[1], z2 = zs[2], z3 = zs[3];
        swap32(z0, z2);
        swap32(z1, z3);
        swap16(z0, z1);
        swap16(z2, z3);
        const int64_t row = 64 * (int64_t)(tb + k) + iota;
        const bool valid = row < n;
        const float yv = s_y[(k % 3) * 64 + lane];
        if (k + 2 < T) issue_y(k + 2);  // slot (k + 2) % 3 = (k - 1) % 3, read in the previous phase
        float d[4];
        {
          float z[NH][4], a[NH][4];
          z[0][0] = z0 + uB[0][0];
          z[0][1] = z1 + uB[0][1];
          z[0][2] = z2 + uB[0][2];
          z[0][3] = z3 + uB[0][3];
#pragma unroll
          for (int q = 0; q < 4; ++q) a[0][q] = act_h_t<ACT>(z[0][q]);
#pragma unroll
          for (int l = 1; l < NH; ++l) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              float s = uB[l][q];
#pragma unroll
              for (int j = 0; j < 4; ++j) s = fmaf(a[l - 1][j], uW[l][j][q], s);
              z[l][q] = s;
              a[l][q] = act_h_t<ACT>(s);
            }
          }
          float out = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) out = fmaf(a[NH - 1][j], uW[NL - 1][j][0], out);
          const float e = valid ? (net_err ? yv : out - yv) : 0.f;
          rss += (double)e * (double)e;
          float err[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            dWo[j] = fmaf(a[NH - 1][j], e, dWo[j]);
            err[j] = e * uW[NL - 1][j][0];
          }
#pragma unroll
          for (int l = NH - 1; l >= 0; --l) {
            float dl[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              dl[q] = act_dh_t<ACT>(z[l][q], a[l][q]) * err[q];
              db[l][q] += dl[q];
            }
            if (l >= 1) {
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                float sj = 0.f;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                  dW[l - 1][j][q] = fmaf(a[l - 1][j], dl[q], dW[l - 1][j][q]);
                  sj = fmaf(dl[q], uW[l][j][q], sj);
                }
                err[j] = sj;
              }
            } else {
#pragma unroll
              for (int q = 0; q < 4; ++q) d[q] = dl[q];
            }
          }
          if (wp && valid) predb[row] = out;
        }
        // delta0 -> signed digits at the running per-column scale (fxl's rule)
        int sh[4] = {0, 0, 0, 0};
        {
          bool lane_need = false;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int eq = (int)((fbits(d[q]) >> 23) & 0xFFu);
            lane_need |= eq > (R[q] ? R[q] : 5);
          }
          if (__builtin_amdgcn_ballot_w64(lane_need) != 0) {
            const uint32_t e01 =
                wave_max_u16x2(((fbits(d[0]) >> 23) & 0xFFu) | (((fbits(d[1]) >> 23) & 0xFFu) << 16));
            const uint32_t e23 =
                wave_max_u16x2(((fbits(d[2]) >> 23) & 0xFFu) | (((fbits(d[3]) >> 23) & 0xFFu) << 16));
            const int E[4] = {(int)(e01 & 0xFFFFu), (int)(e01 >> 16), (int)(e23 & 0xFFFFu), (int)(e23 >> 16)};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              if (E[q] >= 6 && (R[q] == 0 || E[q] > R[q])) {
                if (R[q] != 0) sh[q] = E[q] + 2 - R[q];
                R[q] = E[q] + 2;
              }
            }
          }
        }
        v4u w;
#pragma unroll
        for (int q = 0; q < 4; ++q) w[q] = digits4_fx(d[q], 153 - kslot_sh - (R[q] ? R[q] : 255));
        char* const sd = s_d + (k & 1) * 4 * FX_DROW;
        *reinterpret_cast<v4u*>(sd + (i16 >> 2) * FX_DROW + (4 * g + (i16 & 3)) * 16) = w;
        if (lane == 0) {
          *reinterpret_cast<v4i*>(s_sc + (k & 1) * 8) = v4i{sh[0], sh[1], sh[2], sh[3]};
          *reinterpret_cast<v4i*>(s_sc + (k & 1) * 8 + 4) = v4i{R[0], R[1], R[2], R[3]};
        }
        __builtin_amdgcn_s_setprio(0);
      }
      LDS_BARRIER();
    }
    // head statistics -> the partial slab; sum delta0 per column for the compute waves
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const double rs = wave_sum_d(rss);
    float hs[NS];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      hs[k] = wave_sum(db[0][k]);
      hs[4 + k] = wave_sum(dWo[k]);
    }
#pragma unroll
    for (int l = 1; l < NH; ++l)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        hs[8 + (l - 1) * 20 + k] = wave_sum(db[l][k]);
#pragma unroll
        for (int j = 0; j < 4; ++j) hs[8 + (l - 1) * 20 + 4 + 4 * j + k] = wave_sum(dW[l - 1][j][k]);
      }
    if (lane == 0) {
#pragma unroll
      for (int q = 0; q < NS; ++q) s_hs[q] = hs[q];
#pragma unroll
      for (int k = 0; k < 4; ++k) s_db0[k] = hs[k];
      st.rss_part[it.rss_at] = rs;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane < NS) {
      const float v = s_hs[lane];
      const int q = lane;
      if (q < 4) {
        if (q < bd.widths[0]) part[bd.boff[0] + q] = v;
      } else if (q < 8) {
        const int j = q - 4;
        if (j < bd.win[NL - 1]) part[bd.woff[NL - 1] + j] = v;
      } else {
        const int l = 1 + (q - 8) / 20, r = (q - 8) % 20;
        if (r < 4) {
          if (r < bd.widths[l]) part[bd.boff[l] + r] = v;
        } else {
          const int j = (r - 4) >> 2, k = (r - 4) & 3;
          if (j < bd.win[l] && k < bd.widths[l]) part[bd.woff[l] + k * bd.win[l] + j] = v;
        }
      }
    }
    LDS_BARRIER();
    return;
  }

  // ================= compute waves =================
  const int cwi = wave - 1;
  const int nch = bd.nchunks;
  const int cbase = nch / NC, crem = nch - cbase * NC;
  const int c0 = cwi * cbase + (cwi < crem ? cwi : crem);
  const int cw = cbase + (cwi < crem ? 1 : 0);  // 1 .. CPW chunks of this wave
  float zscale = st.fc[b].scale[g];
  const uint32_t gsw = g & 1;
  const uint32_t fo0 = (uint32_t)((16 * g + tq + 8 * gsw) * 16 + 8 * (tp ^ gsw));
  const uint32_t fo1 = (uint32_t)((16 * g + tq + 8 * (1 ^ gsw)) * 16 + 8 * (tp ^ 1 ^ gsw));
  const int pe = i16, po = (i16 + 8) & 15;
  const uint32_t boe = (uint32_t)(pe * 16 + 4 * (2 * ((g >> 1) ^ (pe >> 3)) + (g & 1)));
  const uint32_t boo = (uint32_t)(po * 16 + 4 * (2 * ((g >> 1) ^ (po >> 3)) + (g & 1)));
  const int64_t tile_bytes = (int64_t)nch * 1024;
  const char* xsrc = reinterpret_cast<const char*>(st.xu2) + bd.x_off + (int64_t)c0 * 1024 + lane * 16;
  const char* dsrc = reinterpret_cast<const char*>(st.dig) + bd.dig_off + (int64_t)c0 * 1024 + lane * 16;
  char* const xslot0 = s_x + cwi * NSL * SLOT;
  const char* const sd_r0 = s_d + g * FX_DROW + tq * 16 + 8 * tp;
  // the chunk count as a compile-time constant (4 or 5 for every group fxh_takes: nch in
  // (4 (nw - 1), 4 nw], NC = ceil(4 nw / 5)): no per-chunk / per-window guards, so each
  // phase is one basic block the compiler schedules across (guards collapse the LDS
  // prefetch distance to one window)
  auto run = [&](auto cw_const) {
    constexpr int CW = decltype(cw_const)::value, NWC = 4 * CW;
    auto issue_tile = [&](int k) {
      const int sl = k % NSL;
#pragma unroll
      for (int c = 0; c < CW; ++c)
        glds16(xsrc + (int64_t)(tb + k) * tile_bytes + c * 1024, xslot0 + sl * SLOT + c * 1024);
    };
    v4i Dres[CW];
#pragma unroll
    for (int c = 0; c < CW; ++c) Dres[c] = *reinterpret_cast<const v4i*>(dsrc + c * 1024);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int c = 0; c < CW; ++c) asm volatile("" : "+v"(Dres[c]));
    asm volatile("" : "+v"(zscale));
    v4i rowsum64 = v4i{0, 0, 0, 0};  // facc[3]'s start (field 3 stored as code - 1)
#pragma unroll
    for (int c = 0; c < CW; ++c) rowsum64 = fx_rowsum64_acc(Dres[c], rowsum64);
    for (int k = 0; k < NSL && k < T; ++k) issue_tile(k);  // every slot filled; tile k + NSL refills slot k in B(k)
    v4i acc[NWC];
#pragma unroll
    for (int u = 0; u < NWC; ++u) acc[u] = v4i{0, 0, 0, 0};
    v4i acc3 = v4i{0, 0, 0, 0};  // field 3's -1: 64 sum over K-group 3 of the digits, every marker
    int Rg = 0;  // the running delta0 scale of this lane's column (published by the head wave)

    for (int p = 0; p < T + 2; ++p) {
      // ---- backward of tile p - 2: dW0 digit sums of this wave's chunks += G^T delta0 ----
      if (p >= 2) {
        const int k = p - 2;
        const int* sc = s_sc + (k & 1) * 8;
        const int sh = sc[g];
        Rg = sc[4 + g];
        if (__builtin_amdgcn_ballot_w64(sh != 0) != 0) {
#pragma unroll
          for (int u = 0; u < NWC; ++u) acc[u] = shr_digits(acc[u], sh);
          acc3 = shr_digits(acc3, sh);
        }
        const char* sd_r = sd_r0 + (k & 1) * 4 * FX_DROW;
        const v4i A = lds_tr8_pair(sd_r, sd_r + 8 * 16);
        acc3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, FX_ONES3, acc3, 0, 0, 0);
        const char* xs = xslot0 + (k % NSL) * SLOT;
        const bool refill = k + NSL < T;  // tile k + NSL into this slot, chunk by chunk
        const char* rsrc = xsrc + (int64_t)(tb + k + NSL) * tile_bytes;
        constexpr int PD = FXL_PD < NWC ? FXL_PD : NWC;
        uint32_t wq[PD];
#pragma unroll
        for (int u = 0; u < PD; ++u) wq[u] = *reinterpret_cast<const uint32_t*>(xs + 256 * u + ((u & 1) ? boo : boe));
        auto unpack = [](uint32_t wv) -> v4i { return fx_bwd_unpack(wv); };
        v4i Bn = unpack(wq[0]), Bn2 = unpack(wq[1]);
#pragma unroll
        for (int u = 0; u < NWC; ++u) {
          const v4i Bv = Bn;
          Bn = Bn2;
          if (u + 2 < NWC) Bn2 = unpack(wq[(u + 2) % PD]);
          if (u + PD < NWC)
            wq[u % PD] = *reinterpret_cast<const uint32_t*>(xs + 256 * (u + PD) + (((u + PD) & 1) ? boo : boe));
          acc[u] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, Bv, acc[u], 0, 0, 0);
          // chunk u >> 2's last window (u | 3) was unpacked at u = 4c + 1: its LDS bytes are free
          if ((u & 3) == 1) {
            asm volatile("" ::"v"(Bn2));
            if (refill) glds16(rsrc + (u >> 2) * 1024, xslot0 + (k % NSL) * SLOT + (u >> 2) * 1024);
          }
          if (FXH_SBB) __builtin_amdgcn_sched_barrier(0);
        }
      }
      // ---- forward of tile p: partial Z0 over this wave's chunks -> exchange slot p % 2 ----
      if (p < T) {
        // pieces younger than tile p's: tiles p + 1 .. min(max(p + NSL - 2, NSL - 1), T - 1) (the
        // prologue's NSL tiles, then one refill per backward, tile p + NSL - 2 in phase p)
        const int hi = p + NSL - 2 > NSL - 1 ? p + NSL - 2 : NSL - 1;
        vm_wait_n(CW * ((hi < T - 1 ? hi : T - 1) - p));
        const char* xs = xslot0 + (p % NSL) * SLOT;
        v4i facc[4] = {v4i{0, 0, 0, 0}, v4i{0, 0, 0, 0}, v4i{0, 0, 0, 0}, rowsum64};
        __builtin_amdgcn_s_setprio(1);
        v4u Xc = (v4u)lds_tr8_pair(xs + fo0, xs + fo1);
#pragma unroll
        for (int c = 0; c < CW; ++c) {
          v4u Xn = Xc;
          if (c + 1 < CW) Xn = (v4u)lds_tr8_pair(xs + (c + 1) * 1024 + fo0, xs + (c + 1) * 1024 + fo1);
          fx_fwd_chunk(Dres[c], Xc, facc);
          if (FXH_SBF) __builtin_amdgcn_sched_barrier(0);
          Xc = Xn;
        }
        fx_fwd_fields(facc);
        const float z0 = zscale * comb4(facc[0]), z1 = (0.25f * zscale) * comb4(facc[1]);
        const float z2 = (0.0625f * zscale) * comb4(facc[2]), z3 = (0.015625f * zscale) * comb4(facc[3]);
        lds_st_v4f(s_zx + ((p & 1) * NC + cwi) * 64 + lane, v4f{z0, z1, z2, z3});
        __builtin_amdgcn_s_setprio(0);
      }
      LDS_BARRIER();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    LDS_BARRIER();  // the head wave's delta0 column sums
    {  // this wave's markers: dW0 = (G^T delta0 - mu sum delta0) / sigma
      const float dbc = s_db0[g];
      const int m = bd.m;
#pragma unroll
      for (int u = 0; u < NWC; ++u) {
        const int mk = 16 * (4 * c0 + u) + i16;
        if (mk < m && g < bd.widths[0]) {
          const float s = Rg ? __builtin_amdgcn_ldexpf(comb4_exact2(acc[u], acc3), Rg - 153) : 0.f;
          const float mu = st.mu[bd.mk_off + mk], sg = st.sigma[bd.mk_off + mk];
          part[bd.woff[0] + g * m + mk] = sg > 0.f ? (s - mu * dbc) / sg : 0.f;
        }
      }
    }
  };
  if (cw == 5)
    run(std::integral_constant<int, 5>{});
  else
    run(std::integral_constant<int, 4>{});
}

template <int NL>
static void launch_fxh_nl(const DevState& st, const GradItem* items, int32_t nitems, int act, int nc, int wp,
                          int slot_kib, hipStream_t s) {
  const dim3 grid((unsigned)nitems), block(64 * (nc + 1));
  const size_t shm = (size_t)fxh_lds_bytes(nc, NL, slot_kib);
#define FXH_GO(A)                                                                                       \
  do {                                                                                                  \
    static bool attr_ = false;                                                                          \
    if (!attr_) {                                                                                       \
      (void)hipFuncSetAttribute((const void*)k_fused_grad_fxh<NL, A>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                fxh_lds_bytes(FXH_MAXC, 4, FXH_CPW));                                   \
      attr_ = true;                                                                                     \
    }                                                                                                   \
    hipLaunchKernelGGL((k_fused_grad_fxh<NL, A>), grid, block, shm, s, st, items, wp, slot_kib);        \
  } while (0)
  switch (act) {
    case 0: FXH_GO(0); break;
    case 1: FXH_GO(1); break;
    case 2: FXH_GO(2); break;
    case 3: FXH_GO(3); break;
    default: FXH_GO(4); break;
  }
#undef FXH_GO
}

// the head-wave kernel for fxl groups of 4-chunk waves with >= 5 waves (17 .. 32
// chunks); head = the context's choice (bann_ctx::fxl_head, read once at context
// creation: BANN_FXL_HEAD=0 keeps fxl for A/B), part of the launch group and its graph key
bool fxh_takes(int nw, int cpw, int head) { return head && cpw == 4 && nw >= 5 && nw <= 8; }
