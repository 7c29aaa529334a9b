// kernels_update.hip — fused leapfrog update (one workgroup per branch).
//
// One launch per leapfrog step replaces, for every branch at once, the
// reference sequence (branch_sampler.rs:1239-1285):
//   log_density_gradient_wrt_weights / _biases  (prior terms, ridge_ard.rs:196-219,
//       ridge_base.rs:175-184, lasso_ard.rs:196-218, lasso_base.rs:175-185,
//       std_normal_branch.rs:160-169, branch_sampler.rs:322-331)
//   momentum.half_step                          (momentum.rs:121-136)
//   neg_hamiltonian = log_density - K(p)         (878-883, 72-78, momentum.rs:149-158)
//   early rejection |dH| > max                    (1264-1279)
//   U-turn diagnostic net_movement                (551-592, 1281-1284)
//   momentum.half_step + params.full_step         (params.rs:728-738)
// with every scalar kept on the device (no host syncs; the reference does ~9
// per step and branch).  The first half step of step k+1 is fused with the
// second half step of step k.  Partial sums from the gradient kernels are
// combined here in a fixed order (deterministic).
#include <math.h>

#include "bann_internal.h"
#include "rng.h"

#define UPD_THREADS 256

__device__ double block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double t = 0.0;
  for (int k = 0; k < UPD_THREADS / 64; ++k) t += red[k];
  return t;
}

__device__ float block_max(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float t = red[0];
  for (int k = 1; k < UPD_THREADS / 64; ++k) t = fmaxf(t, red[k]);
  return t;
}

// Recompute the fused-path constants of branch b from theta: per column k of
// W0 the power-of-two scale s_k, the four signed 7-bit digits of
// (W0_jk / sigma_j) / s_k in the MFMA A-operand layout, and c0_k.
__device__ void refresh_fused_const(const DevState& st, int b, const BranchDev& bd, double* redd, float* redf) {
  const float* W0 = st.theta + bd.p_off + bd.woff[0];
  const float* b0 = st.theta + bd.p_off + bd.boff[0];
  const float* mu = st.mu + bd.mk_off;
  const float* sg = st.sigma + bd.mk_off;
  const int m = bd.m, w0 = bd.widths[0];
  const int NB = bd.fused == 2 ? 8 : 1;  // column blocks of 4 in the digit image (wide kernel: 8)
  uint8_t* dig = const_cast<uint8_t*>(st.dig) + bd.dig_off;
  for (int k = 0; k < w0; ++k) {
    float mx = 0.f;
    double cs = 0.0;
    for (int j = threadIdx.x; j < m; j += UPD_THREADS) {
      const float wp = sg[j] > 0.f ? W0[k * m + j] / sg[j] : 0.f;
      mx = fmaxf(mx, fabsf(wp));
      cs += (double)mu[j] * (double)wp;
    }
    mx = block_max(mx, redf);
    cs = block_sum(cs, redd);
    // s = 2^e with max/s <= 127
    float s = 1.f;
    if (mx > 0.f) {
      int e;
      frexpf(mx / 127.f, &e);
      s = ldexpf(1.f, e);
    }
    if (threadIdx.x == 0) {
      st.fc[b].scale[k] = s;
      st.fc[b].c0[k] = (float)((double)b0[k] - cs);
    }
    const double inv = 1.0 / (double)s;
    for (int j = threadIdx.x; j < m; j += UPD_THREADS) {
      const float wp = sg[j] > 0.f ? W0[k * m + j] / sg[j] : 0.f;
      double v = (double)wp * inv;  // |v| <= 127, exact (power-of-two scale)
      int8_t q[4];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const double r = rint(v);
        q[d] = (int8_t)r;
        v = (v - r) * 128.0;
      }
      const int c = j >> 6, grp = (j & 63) >> 4, jj = j & 15;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int lane = 16 * grp + 4 * (k & 3) + d;
        dig[(((int64_t)c * NB + (k >> 2)) * 64 + lane) * 16 + jj] = (uint8_t)q[d];
      }
    }
  }
}

__global__ void __launch_bounds__(UPD_THREADS) k_update(DevState st, const int32_t* __restrict__ blist, int mode,
                                                        int step) {
  __shared__ double redd[UPD_THREADS / 64];
  __shared__ float redf[UPD_THREADS / 64];
  const int b = blist[blockIdx.x];
  const BranchDev bd = st.br[b];
  const int P = bd.P;
  const int64_t base = bd.p_off;
  if ((mode == MODE_STEP || mode == MODE_LAST) && st.status[b] != ST_RUNNING) return;

  // ---- rss and the log-density gradient (fixed-order split reduction) ----
  double rss = 0.0;
  for (int s = 0; s < bd.nsplits; ++s) rss += st.rss_part[(int64_t)b * st.max_splits + s];
  const float le = st.eprec[b];
  const bool lasso = (bd.prior == 2 || bd.prior == 3);
  double ldp = 0.0;
  for (int i = threadIdx.x; i < P; i += UPD_THREADS) {
    float d = 0.f;
    for (int s = 0; s < bd.nsplits; ++s) d += st.part[bd.part_off + (int64_t)s * P + i];
    const float th = st.theta[base + i];
    const float lm = st.lam[base + i];
    const float sgn = th > 0.f ? 1.f : (th < 0.f ? -1.f : 0.f);  // af_helpers.rs:53-58
    const float reg = lasso ? lm * sgn : lm * th;
    st.grad[base + i] = -(le * d + reg);
    const float ll = st.lamld[base + i];
    ldp -= lasso ? (double)ll * fabs((double)th) : 0.5 * (double)ll * (double)th * (double)th;
  }
  ldp = block_sum(ldp, redd);
  const double ld = ldp - (double)le * rss / 2.0;  // + log_density_wrt_rss (100-102)

  if (mode == MODE_GRAD) {
    if (threadIdx.x == 0) {
      st.ld_out[b] = ld;
      st.rss_out[b] = rss;
    }
    return;
  }
  __syncthreads();  // grad visible block-wide

  const int stride = st.lint + 1;
  if (mode == MODE_INIT) {
    double kin = 0.0;
    for (int i = threadIdx.x; i < P; i += UPD_THREADS) {
      const float p = st.mom[base + i];
      kin += (double)p * (double)p;
    }
    kin = 0.5 * block_sum(kin, redd);
    if (threadIdx.x == 0) {
      const double h = ld - kin;
      st.h0[b] = h;
      st.htrace[(int64_t)b * stride] = h;
      st.status[b] = ST_RUNNING;
      st.uturn[b] = -1;
      st.rss_out[b] = rss;
      st.ld_out[b] = ld;
    }
    for (int i = threadIdx.x; i < P; i += UPD_THREADS) {
      const float e = st.eps[base + i];
      const float th = st.theta[base + i];
      st.theta0[base + i] = th;
      const float p = st.mom[base + i] + 0.5f * e * st.grad[base + i];
      st.mom[base + i] = p;
      st.theta[base + i] = th + e * p;
    }
  } else {
    // second half step of this leapfrog step, then -H (1249-1253)
    double kin = 0.0;
    for (int i = threadIdx.x; i < P; i += UPD_THREADS) {
      const float p = st.mom[base + i] + st.eps[base + i] * 0.5f * st.grad[base + i];
      st.mom[base + i] = p;
      kin += (double)p * (double)p;
    }
    kin = 0.5 * block_sum(kin, redd);
    const double h = ld - kin;
    const double h0 = st.h0[b];
    const bool diverged = fabs(h - h0) > (double)st.max_dh;
    if (threadIdx.x == 0) st.htrace[(int64_t)b * stride + step] = h;
    if (diverged) {  // RejectedEarly: restore the initial params (1277-1278)
      for (int i = threadIdx.x; i < P; i += UPD_THREADS) st.theta[base + i] = st.theta0[base + i];
      if (threadIdx.x == 0) st.status[b] = ST_REJECTED_EARLY;
    } else {
      // U-turn diagnostic (1281-1284): sum (theta - theta0) . p < 0
      double nm = 0.0;
      for (int i = threadIdx.x; i < P; i += UPD_THREADS)
        nm += ((double)st.theta[base + i] - (double)st.theta0[base + i]) * (double)st.mom[base + i];
      nm = block_sum(nm, redd);
      if (threadIdx.x == 0 && nm < 0.0 && st.uturn[b] < 0) st.uturn[b] = step - 1;
      if (mode == MODE_STEP) {
        for (int i = threadIdx.x; i < P; i += UPD_THREADS) {
          const float e = st.eps[base + i];
          const float p = st.mom[base + i] + 0.5f * e * st.grad[base + i];
          st.mom[base + i] = p;
          st.theta[base + i] += e * p;
        }
      } else {  // MODE_LAST: Metropolis decision (accept_or_reject_hmc_state, 928-962)
        const double log_acc = h - h0;
        const double acc_p = log_acc >= 0.0 ? 1.0 : exp(log_acc);
        const bool accept = (double)st.uacc[b] < acc_p;
        if (!accept)
          for (int i = threadIdx.x; i < P; i += UPD_THREADS) st.theta[base + i] = st.theta0[base + i];
        if (threadIdx.x == 0) {
          st.status[b] = accept ? ST_ACCEPTED : ST_REJECTED;
          st.ld_out[b] = ld;
          st.rss_out[b] = rss;
        }
      }
    }
  }
  if (bd.fused) {
    __syncthreads();
    __threadfence_block();
    refresh_fused_const(st, b, bd, redd, redf);
  }
}

void launch_update(const DevState& st, const int32_t* branches, int32_t nb, int32_t mode, int32_t step,
                   hipStream_t s) {
  if (nb <= 0) return;
  hipLaunchKernelGGL(k_update, dim3(nb), dim3(UPD_THREADS), 0, s, st, branches, mode, step);
}

__global__ void __launch_bounds__(UPD_THREADS) k_fused_const(DevState st, const int32_t* __restrict__ blist) {
  __shared__ double redd[UPD_THREADS / 64];
  __shared__ float redf[UPD_THREADS / 64];
  const int b = blist[blockIdx.x];
  const BranchDev bd = st.br[b];
  if (bd.fused) refresh_fused_const(st, b, bd, redd, redf);
}

void launch_fused_const(const DevState& st, const int32_t* branches, int32_t nb, hipStream_t s) {
  if (nb <= 0) return;
  hipLaunchKernelGGL(k_fused_const, dim3(nb), dim3(UPD_THREADS), 0, s, st, branches);
}

// momentum ~ N(0, 1) (sample_momentum, branch_sampler.rs:594-609): Box-Muller on Philox
__global__ void k_sample_momentum(DevState st, const int32_t* __restrict__ blist, uint64_t seed) {
  const int b = blist[blockIdx.y];
  const BranchDev bd = st.br[b];
  const int i2 = blockIdx.x * blockDim.x + threadIdx.x;  // pair index
  if (2 * i2 >= bd.P) return;
  const u32x4 r = philox_bits(seed, 0x3011E47ull + (uint64_t)b, (uint64_t)i2);
  const float u1 = u01_open(r.x), u2 = u01(r.y);
  const float rad = sqrtf(-2.f * logf(u1));
  float sn, cs;
  sincosf(6.283185307179586f * u2, &sn, &cs);
  st.mom[bd.p_off + 2 * i2] = rad * cs;
  if (2 * i2 + 1 < bd.P) st.mom[bd.p_off + 2 * i2 + 1] = rad * sn;
}

void launch_sample_momentum(const DevState& st, const int32_t* branches, int32_t nb, int32_t max_p, uint64_t seed,
                            hipStream_t s) {
  if (nb <= 0 || max_p <= 0) return;
  const int pairs = (max_p + 1) / 2;
  hipLaunchKernelGGL(k_sample_momentum, dim3((pairs + 255) / 256, nb), dim3(256), 0, s, st, branches, seed);
}

// residual change of a finished trajectory (net.rs:292-300): accepted branches
// replace their previous prediction by f(theta_L); rejected ones leave it.
// Two passes, deterministic: RD_GROUPS branch slices each sum their accepted
// branches into a partial row (4 individuals per thread, the q loop unrolled so
// several pred/pred0 loads are in flight), then the rows are added in order.
constexpr int RD_GROUPS = 16;
__global__ void __launch_bounds__(256) k_residual_delta_part(DevState st, const int32_t* __restrict__ blist, int nb,
                                                             float* __restrict__ part) {
  const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i0 >= st.n) return;
  const int g = blockIdx.y;
  const int q0 = (int)((int64_t)nb * g / RD_GROUPS), q1 = (int)((int64_t)nb * (g + 1) / RD_GROUPS);
  const bool full = i0 + 4 <= st.n && (st.n & 3) == 0;  // float4 path needs 16-byte aligned rows
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll 4
  for (int q = q0; q < q1; ++q) {
    const int b = blist[q];
    if (st.status[b] != ST_ACCEPTED) continue;
    const int64_t o = (int64_t)b * st.n + i0;
    if (full) {
      const float4 p = *reinterpret_cast<const float4*>(st.pred + o);
      const float4 r = *reinterpret_cast<const float4*>(st.pred0 + o);
      a0 += p.x - r.x;
      a1 += p.y - r.y;
      a2 += p.z - r.z;
      a3 += p.w - r.w;
    } else {
      a0 += st.pred[o] - st.pred0[o];
      if (i0 + 1 < st.n) a1 += st.pred[o + 1] - st.pred0[o + 1];
      if (i0 + 2 < st.n) a2 += st.pred[o + 2] - st.pred0[o + 2];
      if (i0 + 3 < st.n) a3 += st.pred[o + 3] - st.pred0[o + 3];
    }
  }
  float* row = part + (int64_t)g * st.n + i0;
  row[0] = a0;
  if (i0 + 1 < st.n) row[1] = a1;
  if (i0 + 2 < st.n) row[2] = a2;
  if (i0 + 3 < st.n) row[3] = a3;
}

__global__ void k_residual_delta_sum(const float* __restrict__ part, int64_t n, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float acc = 0.f;
#pragma unroll
  for (int g = 0; g < RD_GROUPS; ++g) acc += part[(int64_t)g * n + i];
  out[i] = acc;
}

int64_t residual_delta_scratch_floats(int64_t n) { return (int64_t)RD_GROUPS * n; }

void launch_residual_delta(const DevState& st, const int32_t* branches, int32_t nb, float* scratch, float* out,
                           hipStream_t s) {
  const unsigned gx = (unsigned)((st.n + 1023) / 1024);
  hipLaunchKernelGGL(k_residual_delta_part, dim3(gx, RD_GROUPS), dim3(256), 0, s, st, branches, nb, scratch);
  hipLaunchKernelGGL(k_residual_delta_sum, dim3((unsigned)((st.n + 255) / 256)), dim3(256), 0, s, scratch, st.n, out);
}

// pred0 <- pred for the listed branches (trajectory start), one launch
__global__ void __launch_bounds__(256) k_snapshot_pred(DevState st, const int32_t* __restrict__ blist) {
  const int b = blist[blockIdx.y];
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const int64_t o = (int64_t)b * st.n + i;
  if (i + 4 <= st.n && (st.n & 3) == 0) {
    *reinterpret_cast<float4*>(st.pred0 + o) = *reinterpret_cast<const float4*>(st.pred + o);
  } else {
    for (int k = 0; k < 4 && i + k < st.n; ++k) st.pred0[o + k] = st.pred[o + k];
  }
}

void launch_snapshot_pred(const DevState& st, const int32_t* branches, int32_t nb, hipStream_t s) {
  if (nb <= 0) return;
  hipLaunchKernelGGL(k_snapshot_pred, dim3((unsigned)((st.n + 1023) / 1024), (unsigned)nb), dim3(256), 0, s, st,
                     branches);
}

// step sizes on the device (uniform 706-732; izmailov: see step_bases in
// bann_api.hip): eps = c, or |base| * (base > 0 ? c : 1) / L, rounded once to f32
__global__ void __launch_bounds__(256) k_step_sizes(DevState st, const double* __restrict__ base,
                                                    const int32_t* __restrict__ blist, int izmailov, float c, int L) {
  const int b = blist[blockIdx.y];
  const BranchDev bd = st.br[b];
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= bd.P) return;
  float e = c;
  if (izmailov) {
    const double v = base[bd.p_off + i];
    e = (float)(v > 0.0 ? (double)c * v / (double)L : -v / (double)L);
  }
  st.eps[bd.p_off + i] = e;
}

void launch_step_sizes(const DevState& st, const double* base, const int32_t* branches, int32_t nb, int32_t max_p,
                       int izmailov, float c, int32_t L, hipStream_t s) {
  if (nb <= 0 || max_p <= 0) return;
  hipLaunchKernelGGL(k_step_sizes, dim3((unsigned)((max_p + 255) / 256), (unsigned)nb), dim3(256), 0, s, st, base,
                     branches, izmailov, c, L);
}
