// kernels_fi.hip — forward-only pass of the fx-shaped branches (every width <= 4,
// m_b <= 512) over an INDIVIDUAL-major 2-bit image: forward_feed
// (branch_sampler.rs:743-782) to the output neuron, f_b(theta) of every
// individual, for the network-joint sampler's per-step forward and the
// prediction paths.
//
// Why a second image.  The gradient kernel (kernels_fx.hip) needs the genotype
// block in both orientations (forward: K = markers, backward: K = individuals)
// and gets them from one marker-major tile image through LDS (transposing
// ds_read_b64_tr_b8 for the forward).  A forward alone needs one orientation
// only, so with the block stored individual-major the MFMA B operand is what a
// plain coalesced global_load_dwordx4 returns: no LDS-DMA, no LDS reads, no
// transposes -- the pass is a register stream of 2-bit codes into the i8 MFMA.
// The image costs the same bytes again (6.4 GB at C3 beside 288 GB of HBM).
//
// Image ("fi"), per branch: [frag = 16 individuals][segment s = 256 markers]
// [lane = 16 g + i][16 B]: lane (g, i) holds individual 16 frag + i, byte q =
// markers 256 s + 64 g + 4 q + p as 2-bit codes at bits 2p (p = 0..3).  One
// 64-individual tile = 4 frags x nseg KiB, contiguous.
//
// MFMA (v_mfma_i32_16x16x64_i8, one per segment and field p): B[k = 16 g + q]
// [n = i] = field p of the lane's byte q -- kept in place (x 4^p; field 3 shifted
// to x 16), one int32 accumulator per field; A[m][16 g + q] = W0/sigma digit m
// (m = 4 column + digit, the digit image of kernels_update.hip) of marker
// 256 s + 64 g + 4 q + p, gathered once per branch into registers.
//
// Work split: the tiles of every item of the launch group form one index space,
// cut into equal contiguous ranges, one per wave of a grid sized to the GPU's
// residency: every wave streams the same number of tiles (no tail round), and
// reloads its branch constants when its range crosses into the next item.
#include <stdlib.h>

#include <algorithm>

#include "activations.h"
#include "bann_internal.h"
#include "kernel_util.h"

#define FI_WAVES 4
#define FI_MAXSEG 2  // m_b <= 512
#ifndef FI_NT
#define FI_NT 1  // non-temporal loads: the image is read once per pass
#endif

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float fi_comb4(v4i d) {  // sum_d D_d 2^(-7 d)
  return (float)d[0] + (float)d[1] * 0x1p-7f + (float)d[2] * 0x1p-14f + (float)d[3] * 0x1p-21f;
}
__device__ __forceinline__ void fi_swap32(float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b),
                                                  false, false);
  a = __builtin_bit_cast(float, (unsigned)r[0]);
  b = __builtin_bit_cast(float, (unsigned)r[1]);
}
__device__ __forceinline__ void fi_swap16(float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b),
                                                  false, false);
  a = __builtin_bit_cast(float, (unsigned)r[0]);
  b = __builtin_bit_cast(float, (unsigned)r[1]);
}
__device__ __forceinline__ float fi_uni(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}

// tiles of a work item (64-individual tiles, frag ranges on tile boundaries)
__device__ __forceinline__ int32_t fi_tiles(const GradItem& it) { return ((it.frag_end + 3) >> 2) - (it.frag_begin >> 2); }

template <int NL>
struct FiBranch {  // the constants of the branch a wave is streaming
  v4i A[FI_MAXSEG][4];
  float zs;           // W0/sigma digit scale of this lane's column, / 16 (the field weights)
  float W[NL][4][4];  // head weights W_l[j][k], l >= 1 (wave-uniform)
  float B[NL][4];     // c0 (l = 0), b_l
  int nseg;
  const char* x;      // this lane's 16 B of frag 0, segment 0
  float* pred;
};

template <int NL>
__device__ __forceinline__ void fi_load_branch(const DevState& st, int b, int lane, FiBranch<NL>& c) {
  const BranchDev& bd = st.br[b];
  const int g = lane >> 4, m = lane & 15;
  const int nch = bd.nchunks;
  c.nseg = (nch + 3) >> 2;
  const uint8_t* dig = st.dig + bd.dig_off;
#pragma unroll
  for (int s = 0; s < FI_MAXSEG; ++s) {
    // rows R_qq = digit row m of markers 256 s + 64 g + 16 qq + (0..15): chunk 4 s + g, window qq
    v4i R[4];
#pragma unroll
    for (int qq = 0; qq < 4; ++qq)
      R[qq] = (4 * s + g < nch) ? *reinterpret_cast<const v4i*>(dig + ((int64_t)(4 * s + g) * 64 + 16 * qq + m) * 16)
                                : v4i{0, 0, 0, 0};
    // A_sp byte q = 4 qq + r  <-  R_qq byte 4 r + p  (marker 16 qq + 4 r + p of the window)
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      v4i a;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        uint32_t d = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) d |= (((uint32_t)R[qq][r] >> (8 * p)) & 0xFFu) << (8 * r);
        a[qq] = (int)d;
      }
      c.A[s][p] = a;
    }
  }
  c.zs = st.fc[b].scale[g] * 0.0625f;
  const float* th = st.theta + bd.p_off;
#pragma unroll
  for (int l = 0; l < NL; ++l) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float v = 0.f;
        if (l >= 1 && (l < NL - 1 || k == 0) && j < bd.win[l] && k < bd.widths[l]) v = th[bd.woff[l] + k * bd.win[l] + j];
        c.W[l][j][k] = fi_uni(v);
      }
    if (l < NL - 1)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float v = 0.f;
        if (k < bd.widths[l]) v = l == 0 ? st.fc[b].c0[k] : th[bd.boff[l] + k];
        c.B[l][k] = fi_uni(v);
      }
  }
  c.x = reinterpret_cast<const char*>(st.xi) + bd.xi_off + lane * 16;
  c.pred = st.pred + bd.y_off;
}

template <int NSEG>
__device__ __forceinline__ void fi_load_tile(const char* x, int nseg, int64_t tt, v4u (&X)[4][NSEG]) {
  const char* p = x + tt * (int64_t)(4 * nseg * 1024);
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int s = 0; s < NSEG; ++s)
      X[f][s] = (s < nseg) ? (FI_NT ? __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p + (int64_t)(f * nseg + s) * 1024))
                                    : *reinterpret_cast<const v4u*>(p + (int64_t)(f * nseg + s) * 1024))
                           : v4u{0u, 0u, 0u, 0u};
}

template <int NL, int ACT, int NSEG>
__device__ __forceinline__ void fi_tile(const FiBranch<NL>& c, const v4u (&X)[4][NSEG], int64_t tt, int lane,
                                        int64_t n) {
  constexpr int NH = NL - 1;
  float z[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    v4i acc[4] = {v4i{0, 0, 0, 0}, v4i{0, 0, 0, 0}, v4i{0, 0, 0, 0}, v4i{0, 0, 0, 0}};
#pragma unroll
    for (int s = 0; s < NSEG; ++s) {
      if (s >= c.nseg) break;
      const v4u x = X[f][s];
      acc[0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(c.A[s][0], (v4i)(x & 0x03030303u), acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(c.A[s][1], (v4i)(x & 0x0C0C0C0Cu), acc[1], 0, 0, 0);
      acc[2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(c.A[s][2], (v4i)(x & 0x30303030u), acc[2], 0, 0, 0);
      acc[3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(c.A[s][3], (v4i)((x >> 2u) & 0x30303030u), acc[3], 0, 0, 0);
    }
    // value x 16 = 16 acc0 + 4 acc1 + acc2 + acc3, per digit, exact in int32
    const v4i D = acc[0] * 16 + acc[1] * 4 + acc[2] + acc[3];
    z[f] = c.zs * fi_comb4(D);  // lane (g, i): column g of individual 16 f + i
  }
  // transpose (frag, lane group) -> (column, lane group): lane L = individual L of the tile
  fi_swap32(z[0], z[2]);
  fi_swap32(z[1], z[3]);
  fi_swap16(z[0], z[1]);
  fi_swap16(z[2], z[3]);
  float a[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) a[k] = act_h_t<ACT>(z[k] + c.B[0][k]);
#pragma unroll
  for (int l = 1; l < NH; ++l) {
    float an[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float s = c.B[l][k];
#pragma unroll
      for (int j = 0; j < 4; ++j) s = fmaf(a[j], c.W[l][j][k], s);
      an[k] = act_h_t<ACT>(s);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] = an[k];
  }
  float out = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) out = fmaf(a[j], c.W[NL - 1][j][0], out);
  const int64_t row = 64 * tt + lane;
  if (row < n) c.pred[row] = out;
}

// a wave's position in its tile range: item, tile within the branch, the item's
// end tile, the branch and its fi image base (wave-uniform)
struct FiPos {
  int item;
  int b;
  int nseg;
  int64_t tt, tend;
  const char* x;
};

__device__ __forceinline__ void fi_pos_item(const DevState& st, const GradItem* items, int item, FiPos& p) {
  const GradItem it = items[item];
  const BranchDev& bd = st.br[it.branch];
  p.item = item;
  p.b = it.branch;
  p.tt = it.frag_begin >> 2;
  p.tend = (it.frag_end + 3) >> 2;
  p.nseg = (bd.nchunks + 3) >> 2;
  p.x = reinterpret_cast<const char*>(st.xi) + bd.xi_off;
}
__device__ __forceinline__ void fi_advance(const DevState& st, const GradItem* items, FiPos& p) {
  if (p.tt + 1 < p.tend) ++p.tt;
  else fi_pos_item(st, items, p.item + 1, p);
}

// The stream runs one tile ahead: two register buffers, the loop unrolled twice
// so each buffer keeps its registers (no copies); 3 waves per SIMD (two tiles
// ahead in three buffers at 2 waves per SIMD measured slower: 1.33 vs 1.21 ms at
// C3).
template <int NL, int ACT, int NSEG>
__global__ void __launch_bounds__(64 * FI_WAVES, NL <= 3 ? 3 : 2) k_forward_fi(DevState st, const GradItem* __restrict__ items,
                                                                 int nitems) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int64_t n = st.n;
  const int64_t T = (int64_t)items[nitems - 1].tile0 + fi_tiles(items[nitems - 1]);
  const int64_t TW = (int64_t)gridDim.x * FI_WAVES, W = (int64_t)blockIdx.x * FI_WAVES + wave;
  const int64_t t0 = T * W / TW, t1 = T * (W + 1) / TW;
  if (t0 >= t1) return;
  int lo = 0, hi = nitems - 1;  // the item holding tile t0
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (items[mid].tile0 <= t0) lo = mid;
    else hi = mid - 1;
  }
  FiPos P0, P1;
  fi_pos_item(st, items, lo, P0);
  P0.tt += t0 - items[lo].tile0;
  P1 = P0;
  v4u X0[4][NSEG], X1[4][NSEG];
  fi_load_tile<NSEG>(P0.x + lane * 16, P0.nseg, P0.tt, X0);
  FiBranch<NL> c;
  int cb = -1;
  // compute tile t from (Xc, Pc); first issue tile t + 1 into (Xl, Pl)
  auto step = [&](int64_t t, v4u (&Xc)[4][NSEG], const FiPos& Pc, v4u (&Xl)[4][NSEG], FiPos& Pl) {
    if (t + 1 < t1) {
      Pl = Pc;
      fi_advance(st, items, Pl);
      fi_load_tile<NSEG>(Pl.x + lane * 16, Pl.nseg, Pl.tt, Xl);
    }
    if (Pc.b != cb) {  // rare: the range crosses into another branch
      fi_load_branch<NL>(st, Pc.b, lane, c);
      cb = Pc.b;
    }
    fi_tile<NL, ACT, NSEG>(c, Xc, Pc.tt, lane, n);
  };
  for (int64_t t = t0; t < t1; t += 2) {
    step(t, X0, P0, X1, P1);
    if (t + 1 < t1) step(t + 1, X1, P1, X0, P0);
  }
}

template <int NL, int NSEG>
static void launch_fi_nl(const DevState& st, const GradItem* items, int32_t nitems, int act, int grid,
                         hipStream_t s) {
  const dim3 g((unsigned)grid), block(64 * FI_WAVES);
  switch (act) {
    case 0: hipLaunchKernelGGL((k_forward_fi<NL, 0, NSEG>), g, block, 0, s, st, items, nitems); break;
    case 1: hipLaunchKernelGGL((k_forward_fi<NL, 1, NSEG>), g, block, 0, s, st, items, nitems); break;
    case 2: hipLaunchKernelGGL((k_forward_fi<NL, 2, NSEG>), g, block, 0, s, st, items, nitems); break;
    case 3: hipLaunchKernelGGL((k_forward_fi<NL, 3, NSEG>), g, block, 0, s, st, items, nitems); break;
    default: hipLaunchKernelGGL((k_forward_fi<NL, 4, NSEG>), g, block, 0, s, st, items, nitems); break;
  }
}

// items: one fx launch group (every branch has an fi image), tile0 = the prefix
// of the items' tile counts; max_seg: the group's largest segment count
void launch_forward_fi(const DevState& st, const GradItem* items, int32_t nitems, int64_t total_tiles, int32_t L,
                       int32_t act, int32_t max_seg, int32_t cus, hipStream_t s) {
  if (nitems <= 0 || total_tiles <= 0) return;
  const int64_t waves = (int64_t)cus * 4 * (int64_t)(getenv("BANN_FI_WAVES_PER_SIMD") ? atoi(getenv("BANN_FI_WAVES_PER_SIMD")) : 3);
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(waves, total_tiles) / FI_WAVES);
  switch (L * 2 + (max_seg > 1 ? 1 : 0)) {
    case 4: launch_fi_nl<2, 1>(st, items, nitems, act, grid, s); break;
    case 5: launch_fi_nl<2, 2>(st, items, nitems, act, grid, s); break;
    case 6: launch_fi_nl<3, 1>(st, items, nitems, act, grid, s); break;
    case 7: launch_fi_nl<3, 2>(st, items, nitems, act, grid, s); break;
    case 8: launch_fi_nl<4, 1>(st, items, nitems, act, grid, s); break;
    case 9: launch_fi_nl<4, 2>(st, items, nitems, act, grid, s); break;
    default: break;
  }
}

// ---------------------------------------------------------------------------
// the fi image from the raw variant-major image (kernels_data.hip layout: row =
// marker, byte i >> 2 holds individuals 4 (i >> 2) .. + 3 at bits 2 (i & 3)).
// One workgroup per (job = branch segment, 64-individual tile): the 256 marker
// rows' 16 bytes of the tile through LDS, then each thread writes 4 dwords:
// dword r of lane (g, i) of frag f = 16 markers 64 g + 16 r + kk of individual
// 16 f + i, code at bit 2 kk.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_pack_fi(const uint8_t* __restrict__ raw, int64_t rowb,
                                                 const PackJob* __restrict__ jobs, const int32_t* __restrict__ idx,
                                                 int64_t ntile, uint8_t* __restrict__ dst) {
  __shared__ uint4 s_rows[256];
  const PackJob jb = jobs[blockIdx.x];
  const int64_t t = blockIdx.y;
  const int r = threadIdx.x;
  uint4 v = make_uint4(0, 0, 0, 0);
  if (r < jb.rows) v = *reinterpret_cast<const uint4*>(raw + (int64_t)idx[jb.idx_off + r] * rowb + 16 * t);
  s_rows[r] = v;
  __syncthreads();
  const uint8_t* rb = reinterpret_cast<const uint8_t*>(s_rows);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int e = threadIdx.x + 256 * k;  // output dword: frag f, lane, dword rr
    const int f = e >> 8, lane = (e >> 2) & 63, rr = e & 3;
    const int g = lane >> 4, i = lane & 15;
    const int ind = 16 * f + i;  // individual within the tile
    uint32_t d = 0;
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const int mk = 64 * g + 16 * rr + kk;
      d |= (uint32_t)((rb[mk * 16 + (ind >> 2)] >> (2 * (ind & 3))) & 3u) << (2 * kk);
    }
    *reinterpret_cast<uint32_t*>(dst + jb.dst + (4 * t + f) * jb.tile_stride + lane * 16 + 4 * rr) = d;
  }
}

// jobs: dst = byte offset of segment s in frag 0 of the branch's fi image,
// tile_stride = bytes per FRAG (nseg KiB), idx_off / rows: the segment's markers
void launch_pack_fi(const uint8_t* raw, int64_t rowb, const PackJob* jobs, int32_t njobs, const int32_t* idx,
                    int64_t ntile, uint8_t* dst, hipStream_t s) {
  if (njobs <= 0 || ntile <= 0) return;
  hipLaunchKernelGGL(k_pack_fi, dim3((unsigned)njobs, (unsigned)ntile), dim3(256), 0, s, raw, rowb, jobs, idx, ntile,
                     dst);
}
