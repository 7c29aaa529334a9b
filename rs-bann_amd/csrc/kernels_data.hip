// kernels_data.hip — genotype ingestion on the device.
//
// Replaces the host-side path of the reference that decodes the PLINK .bed and
// re-uploads a dense standardized f32 block for every branch on every Gibbs
// sweep (net.rs:265 -> genotypes.rs:44-48 -> bed.rs:325-355).  Here the cohort
// lives on the device ONCE, as a 2-bit variant-major image -- the .bed payload
// layout with the codes replaced by the genotype values:
//
//   raw[j][q]  (row j = marker, rowb = ceil(n / 64) * 16 bytes per row)
//   byte q holds individuals 4q .. 4q+3, individual 4q+p at bits 2p;
//   rows padded with zeros to whole 64-individual tiles
//
// (6.3 GB at C3 where an int8 matrix would take 25 GB).  Every ingestion path
// streams into it through a bounded staging buffer: int8 genotypes, the .bed
// payload (code LUT, bed_lookup_tables.rs:4) or the synthetic cohort; column
// statistics come from the 2-bit image; and finalize packs all branches' tile
// images (u2t layout, kernels_fx.hip) in ONE batched launch: a 64-individual
// tile row of a marker is 16 bytes of its raw row, so the pack is a gather of
// 16-byte pieces, transposed through LDS so that both the reads (128 B per
// marker and 8 tiles) and the writes (1 KiB per chunk and tile) are contiguous.
#include "bann_internal.h"
#include "rng.h"

// ---------------------------------------------------------------------------
// synthetic cohort: g_ij ~ Binomial(2, p_j), p_j ~ U(0.01, 0.5); zero-variance
// markers redrawn (bed.rs:136-188 semantics).  One workgroup per marker, one
// byte (4 individuals, two Philox draws) per thread and step.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_synthetic(uint8_t* __restrict__ raw, int64_t rowb, float* __restrict__ mu,
                                                   float* __restrict__ sigma, int64_t n, int64_t M,
                                                   uint64_t seed) {
  __shared__ int64_t red[2][4];
  __shared__ int done;
  const int64_t j = blockIdx.x;
  if (j >= M) return;
  uint8_t* row = raw + j * rowb;
  for (uint32_t attempt = 0;; ++attempt) {
    u32x4 pb = philox_bits(seed, 0xA11E1Eull + ((uint64_t)attempt << 40), (uint64_t)j);
    const float p = 0.01f + 0.49f * u01(pb.x);
    int64_t s1 = 0, s2 = 0;
    const uint64_t stream = ((uint64_t)j << 8) | attempt;
    for (int64_t q = threadIdx.x; q < rowb; q += blockDim.x) {
      uint32_t byte = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // individuals 4q + 2h, 4q + 2h + 1: one Philox call, two Bernoulli(p) each
        const int64_t i = 4 * q + 2 * h;
        if (i >= n) break;
        const u32x4 r = philox_bits(seed, stream, (uint64_t)(2 * q + h));
        const int v0 = (u01(r.x) < p) + (u01(r.y) < p);
        const int v1 = i + 1 < n ? (u01(r.z) < p) + (u01(r.w) < p) : 0;
        byte |= (uint32_t)(v0 | (v1 << 2)) << (4 * h);
        s1 += v0 + v1;
        s2 += v0 * v0 + v1 * v1;
      }
      row[q] = (uint8_t)byte;
    }
    for (int o = 32; o > 0; o >>= 1) {
      s1 += __shfl_xor(s1, o);
      s2 += __shfl_xor(s2, o);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
      red[0][w] = s1;
      red[1][w] = s2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t t1 = 0, t2 = 0;
      for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
        t1 += red[0][k];
        t2 += red[1][k];
      }
      const double m = (double)t1 / (double)n;
      const double var = (double)t2 / (double)n - m * m;
      done = (var > 0.0 || n == 1 || attempt >= 64) ? 1 : 0;
      if (done) {
        mu[j] = (float)m;
        sigma[j] = (float)sqrt(var > 0.0 ? var : 0.0);
      }
    }
    __syncthreads();
    if (done) return;
    __syncthreads();
  }
}

void launch_synthetic_genotypes(uint8_t* raw, int64_t rowb, float* mu, float* sigma, int64_t n, int64_t M,
                                uint64_t seed, hipStream_t s) {
  if (M <= 0) return;
  hipLaunchKernelGGL(k_synthetic, dim3((unsigned)M), dim3(256), 0, s, raw, rowb, mu, sigma, n, M, seed);
}

// ---------------------------------------------------------------------------
// int8 genotypes [m][n] (a staging block of markers) -> raw rows; flag |= any
// value outside 0..3
// ---------------------------------------------------------------------------
__global__ void k_i8_to_raw(const int8_t* __restrict__ g, int64_t n, int64_t m, uint8_t* __restrict__ raw,
                            int64_t rowb, int32_t* __restrict__ flag) {
  const int64_t total = rowb * m;
  int bad = 0;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = t / rowb, q = t - j * rowb;
    uint32_t byte = 0;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int64_t i = 4 * q + p;
      if (i < n) {
        const uint32_t v = (uint32_t)(uint8_t)g[j * n + i];
        bad |= v > 3u;
        byte |= (v & 3u) << (2 * p);
      }
    }
    raw[t] = (uint8_t)byte;
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

void launch_i8_to_raw(const int8_t* g, int64_t n, int64_t m, uint8_t* raw, int64_t rowb, int32_t* flag,
                      hipStream_t s) {
  const int64_t total = rowb * m;
  if (total <= 0) return;
  const int64_t blocks = (total + 255) / 256;
  hipLaunchKernelGGL(k_i8_to_raw, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(256), 0, s, g, n, m, raw,
                     rowb, flag);
}

// ---------------------------------------------------------------------------
// .bed payload rows (ceil(n/4) bytes per marker, first individual in the lowest
// bits, bed.rs:378-389) -> raw rows: every 2-bit code through the LUT of
// bed_lookup_tables.rs:4 (00 -> 2, 01 -> 0 (missing), 10 -> 1, 11 -> 0); the
// codes past n in the last byte and the row padding become 0
// ---------------------------------------------------------------------------
__global__ void k_bed_to_raw(const uint8_t* __restrict__ pl, int64_t n, int64_t m, uint8_t* __restrict__ raw,
                             int64_t rowb) {
  const int64_t bpc = (n + 3) / 4;
  const int64_t total = rowb * m;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = t / rowb, q = t - j * rowb;
    uint32_t out = 0;
    if (q < bpc) {
      const uint32_t code = pl[j * bpc + q];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const uint32_t c = (code >> (2 * p)) & 3u;
        const uint32_t v = c == 0u ? 2u : (c == 2u ? 1u : 0u);
        if (4 * q + p < n) out |= v << (2 * p);
      }
    }
    raw[t] = (uint8_t)out;
  }
}

void launch_bed_to_raw(const uint8_t* payload, int64_t n, int64_t m, uint8_t* raw, int64_t rowb, hipStream_t s) {
  const int64_t total = rowb * m;
  if (total <= 0) return;
  const int64_t blocks = (total + 255) / 256;
  hipLaunchKernelGGL(k_bed_to_raw, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(256), 0, s, payload, n,
                     m, raw, rowb);
}

// ---------------------------------------------------------------------------
// column statistics (bed.rs:231-242): mean and population std, from exact
// integer sums over the 2-bit rows (more accurate than the reference's
// sequential f32 sums).  One workgroup per marker; the two bit planes of a
// 32-bit word give sum f = lo + 2 hi and sum f^2 = lo + 4 hi + 4 (lo and hi).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_col_stats(const uint8_t* __restrict__ raw, int64_t rowb,
                                                   float* __restrict__ mu, float* __restrict__ sigma, int64_t n) {
  __shared__ int64_t red[2][4];
  const int64_t j = blockIdx.x;
  const uint32_t* row = reinterpret_cast<const uint32_t*>(raw + j * rowb);  // rowb is a multiple of 16
  int64_t s1 = 0, s2 = 0;
  for (int64_t w = threadIdx.x; w < rowb / 4; w += blockDim.x) {
    const uint32_t v = row[w];
    const uint32_t lo = v & 0x55555555u, hi = (v >> 1) & 0x55555555u;
    const int c_lo = __builtin_popcount(lo), c_hi = __builtin_popcount(hi), c_both = __builtin_popcount(lo & hi);
    s1 += c_lo + 2 * c_hi;
    s2 += c_lo + 4 * c_hi + 4 * c_both;
  }
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s1;
    red[1][threadIdx.x >> 6] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t1 = 0, t2 = 0;
    for (int k = 0; k < 4; ++k) {
      t1 += red[0][k];
      t2 += red[1][k];
    }
    const double m = (double)t1 / (double)n;
    const double var = (double)t2 / (double)n - m * m;
    mu[j] = (float)m;
    sigma[j] = (float)sqrt(var > 0.0 ? var : 0.0);
  }
}

void launch_col_stats(const uint8_t* raw, int64_t rowb, float* mu, float* sigma, int64_t n, int64_t M,
                      hipStream_t s) {
  if (M <= 0) return;
  hipLaunchKernelGGL(k_col_stats, dim3((unsigned)M), dim3(256), 0, s, raw, rowb, mu, sigma, n);
}

// ---------------------------------------------------------------------------
// raw rows of markers idx[0..m) -> int8 [m][n] (bann_genotypes_download)
// ---------------------------------------------------------------------------
__global__ void k_unpack(const uint8_t* __restrict__ raw, int64_t rowb, const int32_t* __restrict__ idx, int32_t m,
                         int64_t n, int8_t* __restrict__ out) {
  const int64_t total = (int64_t)m * n;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = t / n, i = t - j * n;
    out[t] = (int8_t)((raw[(int64_t)idx[j] * rowb + (i >> 2)] >> (2 * (i & 3))) & 3u);
  }
}

void launch_unpack_markers(const uint8_t* raw, int64_t rowb, const int32_t* snp_idx, int32_t m, int64_t n,
                           int8_t* out, hipStream_t s) {
  const int64_t total = (int64_t)m * n;
  if (total <= 0) return;
  const int64_t blocks = (total + 255) / 256;
  hipLaunchKernelGGL(k_unpack, dim3((unsigned)(blocks < 16384 ? blocks : 16384)), dim3(256), 0, s, raw, rowb, snp_idx,
                     m, n, out);
}

// ---------------------------------------------------------------------------
// batched pack of every branch's tile image (u2t layout, kernels_fx.hip header):
// tile t of marker row r of a branch = bytes [16 t, 16 t + 16) of raw row idx[r]
// (zeros for the rows that pad m up to whole chunks).  One workgroup per
// (chunk job, 8 tiles): 64 rows x 8 tiles of 16 B, read 128 B per row, written
// 1 KiB per tile, through LDS.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_pack_tiles(const uint8_t* __restrict__ raw, int64_t rowb,
                                                    const PackJob* __restrict__ jobs, const int32_t* __restrict__ idx,
                                                    int64_t ntile, uint8_t* __restrict__ dst) {
  __shared__ uint4 s[8][64];
  const PackJob jb = jobs[blockIdx.x];
  const int64_t t0 = (int64_t)blockIdx.y * 8;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int e = threadIdx.x + 256 * k;
    const int r = e >> 3, tt = e & 7;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r < jb.rows && t0 + tt < ntile)
      v = *reinterpret_cast<const uint4*>(raw + (int64_t)idx[jb.idx_off + r] * rowb + 16 * (t0 + tt));
    s[tt][r] = v;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int e = threadIdx.x + 256 * k;
    const int tt = e >> 6, r = e & 63;
    if (t0 + tt >= ntile) continue;
    // row r of the chunk sits in window w = r >> 4 at position ((r & 15) + 8 (w & 1)) & 15,
    // its two 8-byte halves swapped at positions >= 8 (the parity of w is the global one: 4 windows per chunk)
    const int w = r >> 4, P = ((r & 15) + 8 * (w & 1)) & 15;
    uint4 v = s[tt][r];
    if (jb.f3m1) {  // field 3 as code - 1 (codes <= 2: 0 -> 11, 1 -> 00, 2 -> 01; padding rows too)
      auto f3 = [](uint32_t x) { return (x & 0x3F3F3F3Fu) | (((((x >> 6) & 0x03030303u) + 0x03030303u) & 0x03030303u) << 6); };
      v = make_uint4(f3(v.x), f3(v.y), f3(v.z), f3(v.w));
    }
    if (P >= 8) v = make_uint4(v.z, v.w, v.x, v.y);
    *reinterpret_cast<uint4*>(dst + jb.dst + (t0 + tt) * jb.tile_stride + (16 * w + P) * 16) = v;
  }
}

void launch_pack_tiles(const uint8_t* raw, int64_t rowb, const PackJob* jobs, int32_t njobs, const int32_t* idx,
                       int64_t ntile, uint8_t* dst, hipStream_t s) {
  if (njobs <= 0 || ntile <= 0) return;
  hipLaunchKernelGGL(k_pack_tiles, dim3((unsigned)njobs, (unsigned)((ntile + 7) / 8)), dim3(256), 0, s, raw, rowb,
                     jobs, idx, ntile, dst);
}

__global__ void k_gather_stats(const float* mu, const float* sigma, const int32_t* idx, int32_t m, float* mu_b,
                               float* sig_b) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < m) {
    mu_b[t] = mu[idx[t]];
    sig_b[t] = sigma[idx[t]];
  }
}

void launch_gather_stats(const float* mu, const float* sigma, const int32_t* snp_idx, int32_t m, float* mu_b,
                         float* sig_b, hipStream_t s) {
  if (m <= 0) return;
  hipLaunchKernelGGL(k_gather_stats, dim3((m + 255) / 256), dim3(256), 0, s, mu, sigma, snp_idx, m, mu_b, sig_b);
}
