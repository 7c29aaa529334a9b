// kernels_data.hip — genotype ingestion on the device.
//
// Replaces the host-side path of the reference that decodes the PLINK .bed and
// re-uploads a dense standardized f32 block for every branch on every Gibbs
// sweep (net.rs:265 -> genotypes.rs:44-48 -> bed.rs:325-355).  Here genotypes
// are uploaded ONCE as int8 (1 byte per genotype instead of 4), column
// statistics are reduced on the device, and each branch's marker block is
// packed into the fragment-major layout streamed by the gradient kernel:
//
//   packed[b] : [frag f][chunk c][lane l][16 bytes]
//   lane l <-> individual 16 f + (l & 15), markers 64 c + 16 (l >> 4) + 0..15
//
// i.e. one 1 KiB wave-load per (16 individuals x 64 markers), which is exactly
// the B operand of v_mfma_i32_16x16x64_i8 (lane l holds B[k=16(l>>4)+j][n=l&15]).
#include "bann_internal.h"
#include "rng.h"

// ---------------------------------------------------------------------------
// synthetic cohort: g_ij ~ Binomial(2, p_j), p_j ~ U(0.01, 0.5); zero-variance
// markers redrawn (bed.rs:136-188 semantics).  One workgroup per marker.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_synthetic(int8_t* __restrict__ g, float* __restrict__ mu,
                                                   float* __restrict__ sigma, int64_t n, int64_t M,
                                                   uint64_t seed) {
  __shared__ int64_t red[2][4];
  __shared__ int done;
  const int64_t j = blockIdx.x;
  if (j >= M) return;
  int8_t* col = g + j * n;
  for (uint32_t attempt = 0;; ++attempt) {
    u32x4 pb = philox_bits(seed, 0xA11E1Eull + ((uint64_t)attempt << 40), (uint64_t)j);
    const float p = 0.01f + 0.49f * u01(pb.x);
    int64_t s1 = 0, s2 = 0;
    const uint64_t stream = ((uint64_t)j << 8) | attempt;
    for (int64_t i4 = threadIdx.x; i4 * 2 < n; i4 += blockDim.x) {
      u32x4 r = philox_bits(seed, stream, (uint64_t)i4);
      // two individuals per philox call, two Bernoulli(p) draws each
      const int v0 = (u01(r.x) < p) + (u01(r.y) < p);
      const int v1 = (u01(r.z) < p) + (u01(r.w) < p);
      const int64_t i = 2 * i4;
      col[i] = (int8_t)v0;
      s1 += v0;
      s2 += v0 * v0;
      if (i + 1 < n) {
        col[i + 1] = (int8_t)v1;
        s1 += v1;
        s2 += v1 * v1;
      }
    }
    // block reduction of the exact integer sums
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

void launch_synthetic_genotypes(int8_t* g, float* mu, float* sigma, int64_t n, int64_t M, uint64_t seed,
                                hipStream_t s) {
  if (M <= 0) return;
  hipLaunchKernelGGL(k_synthetic, dim3((unsigned)M), dim3(256), 0, s, g, mu, sigma, n, M, seed);
}

// ---------------------------------------------------------------------------
// .bed decode: 2-bit codes, first individual in the lowest bits (bed.rs:378-389),
// code -> genotype LUT of bed_lookup_tables.rs:4: 00->2, 01->0, 10->1, 11->0.
// ---------------------------------------------------------------------------
__constant__ int8_t c_bed_lut[4] = {2, 0, 1, 0};
__global__ void k_decode_bed_lut(const uint8_t* __restrict__ payload, int8_t* __restrict__ g, int64_t n,
                                 int64_t M) {
  const int64_t bpc = (n + 3) / 4;
  const int64_t total = bpc * M;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = t / bpc, q = t - j * bpc;
    const uint32_t byte = payload[t];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i = 4 * q + k;
      if (i < n) g[j * n + i] = c_bed_lut[(byte >> (2 * k)) & 3u];
    }
  }
}

void launch_decode_bed(const uint8_t* payload, int8_t* g, int64_t n, int64_t M, hipStream_t s) {
  const int64_t total = ((n + 3) / 4) * M;
  if (total <= 0) return;
  const int64_t blocks = (total + 255) / 256;
  hipLaunchKernelGGL(k_decode_bed_lut, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(256), 0, s, payload,
                     g, n, M);
}

// ---------------------------------------------------------------------------
// column statistics (bed.rs:231-242): mean and population std, from exact
// integer sums (more accurate than the reference's sequential f32 sums).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_col_stats(const int8_t* __restrict__ g, float* __restrict__ mu,
                                                   float* __restrict__ sigma, int64_t n) {
  __shared__ int64_t red[2][4];
  const int64_t j = blockIdx.x;
  const int8_t* col = g + j * n;
  int64_t s1 = 0, s2 = 0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const int v = col[i];
    s1 += v;
    s2 += v * v;
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

void launch_col_stats(const int8_t* g, float* mu, float* sigma, int64_t n, int64_t M, hipStream_t s) {
  if (M <= 0) return;
  hipLaunchKernelGGL(k_col_stats, dim3((unsigned)M), dim3(256), 0, s, g, mu, sigma, n);
}

__global__ void k_check_2bit(const int8_t* __restrict__ g, int64_t count, int32_t* __restrict__ flag) {
  int bad = 0;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < count; t += (int64_t)gridDim.x * blockDim.x)
    bad |= (uint32_t)(uint8_t)g[t] > 3u;
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

void launch_check_2bit(const int8_t* g, int64_t count, int32_t* flag, hipStream_t s) {
  if (count <= 0) return;
  const int64_t blocks = (count + 255) / 256;
  hipLaunchKernelGGL(k_check_2bit, dim3((unsigned)(blocks < 16384 ? blocks : 16384)), dim3(256), 0, s, g, count,
                     flag);
}

__global__ void k_unpack(const int8_t* __restrict__ g, const int32_t* __restrict__ idx, int32_t m, int64_t n,
                         int8_t* __restrict__ out) {
  const int64_t total = (int64_t)m * n;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = t / n, i = t - j * n;
    out[t] = g[(int64_t)idx[j] * n + i];
  }
}

void launch_unpack_markers(const int8_t* g, const int32_t* snp_idx, int32_t m, int64_t n, int8_t* out,
                           hipStream_t s) {
  const int64_t total = (int64_t)m * n;
  if (total <= 0) return;
  const int64_t blocks = (total + 255) / 256;
  hipLaunchKernelGGL(k_unpack, dim3((unsigned)(blocks < 16384 ? blocks : 16384)), dim3(256), 0, s, g, snp_idx, m, n,
                     out);
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
