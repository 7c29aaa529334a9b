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
#include <stdlib.h>

#include <algorithm>

#include "bann_internal.h"
#include "rng.h"

#define UPD_THREADS 256   // small-branch limits P <= UPD_CAP x 256 = 2048, m <= 512 (C3 / C4); k_fused_const
#define UPD_THREADS_S 512  // the small-branch update kernel
#define UPD_THREADS_L 1024  // large branches (C2: P = 8028, m = 2000; wide / generic)

// Recompute the fused-path constants of branch b from theta: per column k of
// W0 the power-of-two scale s_k, the four signed 7-bit digits of
// (W0_jk / sigma_j) / s_k in the MFMA A-operand layout, and c0_k.
template <int NT>
__device__ void refresh_fused_const(const DevState& st, int b, const BranchDev& bd) {
  __shared__ float s_mx[4][NT / 64];
  __shared__ double s_cs[4][NT / 64];
  const float* W0 = st.theta + bd.p_off + bd.woff[0];
  const float* b0 = st.theta + bd.p_off + bd.boff[0];
  const float* mu = st.mu + bd.mk_off;
  const float* sg = st.sigma + bd.mk_off;
  const int m = bd.m, w0 = bd.widths[0];
  const int NB = bd.fused == 2 ? 8 : 1;  // column blocks of 4 in the digit image (wide kernel: 8)
  uint8_t* dig = const_cast<uint8_t*>(st.dig) + bd.dig_off;
  const int wv = threadIdx.x >> 6;
  // four columns per pass: their max |W0/sigma| and mu . (W0/sigma) in one
  // combined reduction (one barrier pair per four columns)
  for (int k0 = 0; k0 < w0; k0 += 4) {
    const int nk = w0 - k0 < 4 ? w0 - k0 : 4;
    float mx[4] = {0.f, 0.f, 0.f, 0.f};
    double cs[4] = {0.0, 0.0, 0.0, 0.0};
    for (int j = threadIdx.x; j < m; j += NT) {
      const float sj = sg[j];
      const double mj = (double)mu[j];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (q < nk) {
          const float wp = sj > 0.f ? W0[(k0 + q) * m + j] / sj : 0.f;
          mx[q] = fmaxf(mx[q], fabsf(wp));
          cs[q] += mj * (double)wp;
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        mx[q] = fmaxf(mx[q], __shfl_xor(mx[q], o));
        cs[q] += __shfl_xor(cs[q], o);
      }
    __syncthreads();
    if ((threadIdx.x & 63) == 0)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        s_mx[q][wv] = mx[q];
        s_cs[q][wv] = cs[q];
      }
    __syncthreads();
    double inv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float M = s_mx[q][0];
      double C = s_cs[q][0];
      for (int w = 1; w < NT / 64; ++w) {
        M = fmaxf(M, s_mx[q][w]);
        C += s_cs[q][w];
      }
      // s = 2^e with max/s <= 127
      float sc = 1.f;
      if (M > 0.f) {
        int e;
        frexpf(M / 127.f, &e);
        sc = ldexpf(1.f, e);
      }
      inv[q] = 1.0 / (double)sc;
      if (threadIdx.x == 0 && q < nk) {
        st.fc[b].scale[k0 + q] = sc;
        st.fc[b].c0[k0 + q] = (float)((double)b0[k0 + q] - C);
      }
    }
    for (int j = threadIdx.x; j < m; j += NT) {
      const float sj = sg[j];
      const int c = j >> 6, grp = (j & 63) >> 4, jj = j & 15;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (q >= nk) continue;
        const int k = k0 + q;
        const float wp = sj > 0.f ? W0[k * m + j] / sj : 0.f;
        double v = (double)wp * inv[q];  // |v| <= 127, exact (power-of-two scale)
        int8_t dq[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const double r = rint(v);
          dq[d] = (int8_t)r;
          v = (v - r) * 128.0;
        }
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const int lane = 16 * grp + 4 * (k & 3) + d;
          dig[(((int64_t)c * NB + (k >> 2)) * 64 + lane) * 16 + jj] = (uint8_t)dq[d];
        }
      }
    }
  }
}

#include "update_core.h"

// Per leapfrog step: ONE pass over the parameters computes the prior gradient,
// the half-stepped momentum and every scalar of the step (log prior, kinetic
// energy, U-turn dot product), with one combined workgroup reduction; a second
// pass applies the position step (or the restore).  (The first version had a
// reduction per scalar and re-read each array per phase: ~40 us per launch,
// 18 % of a step at 125 branches per GPU.)  MODE_PROFILE repeats STEP's work
// without changing the chain (bann_profile_session).
template <int NT, int MPT>
#ifndef UPD_WPE
#define UPD_WPE 8  // A/B builds: -DUPD_WPE=1 leaves the register budget to the compiler
#endif
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT == 512 ? UPD_WPE : 1)))  // 512: <= 64 VGPRs, four per CU (C3: 1000 in one round)
    k_update(DevState st, const int32_t* __restrict__ blist, int mode, int step) {
  __shared__ double redd[4 * (NT / 64)];
  const int b = blist[blockIdx.x];
  const BranchDev bd = st.br[b];
  const int P = bd.P;
  const int64_t base = bd.p_off;
  const bool prof = mode == MODE_PROFILE;
  if (prof) mode = MODE_STEP;
  if (mode == MODE_RESTORE) {  // back to theta_0 (a rejected network trajectory)
    for (int i = threadIdx.x; i < P; i += NT) st.theta[base + i] = st.theta0[base + i];
    if (bd.fused) {
      __syncthreads();
      refresh_fused_const<NT>(st, b, bd);
    }
    return;
  }
  if ((((bd.fused == 1 || bd.fused == 3) && bd.widths[0] <= 4) || (bd.fused == 2 && bd.widths[0] <= 32)) &&
      P <= upd_cap<NT>() * NT && bd.m <= MPT * NT) {
    __shared__ float s_th[upd_cap<NT>() * NT];
    update_small<NT, MPT>(st, b, bd, mode, prof, step, redd, s_th);  // checks the status itself
    return;
  }
  if (!prof && (mode == MODE_STEP || mode == MODE_LAST) && st.status[b] != ST_RUNNING) return;

  // ---- rss (fixed-order split reduction) ----
  double rss = 0.0;
  for (int s = 0; s < bd.nsplits; ++s) rss += st.rss_part[(int64_t)b * st.max_splits + s];
  const float le = st.netmode ? st.net_le : st.eprec[b];  // network mode: the network error precision
  const bool lasso = (bd.prior == 2 || bd.prior == 3);
  // sums[0] = log prior (ridge_ard.rs:171-194 and the other priors), sums[1] =
  // sum p^2 (momentum.rs:149-158; INIT: the drawn momentum, else the
  // half-stepped one), sums[2] = sum (theta - theta0) . p (551-592)
  double sums[3] = {0.0, 0.0, 0.0};
  for (int i = threadIdx.x; i < P; i += NT) {
    float d = 0.f;
    for (int s = 0; s < bd.nsplits; ++s) d += st.part[bd.part_off + (int64_t)s * P + i];
    const float th = st.theta[base + i];
    const float lm = st.lam[base + i];
    const float sgn = th > 0.f ? 1.f : (th < 0.f ? -1.f : 0.f);  // af_helpers.rs:53-58
    const float reg = lasso ? lm * sgn : lm * th;
    const float gr = -(le * d + reg);  // log_density_gradient (branch_sampler.rs:380-391)
    st.grad[base + i] = gr;
    const float ll = st.lamld[base + i];
    sums[0] -= lasso ? (double)ll * fabs((double)th) : 0.5 * (double)ll * (double)th * (double)th;
    if (mode == MODE_INIT) {
      const float p = st.mom[base + i];
      sums[1] += (double)p * (double)p;
    } else if (mode != MODE_GRAD) {  // second half step of this leapfrog step (momentum.rs:121-136)
      const float p = st.mom[base + i] + st.eps[base + i] * 0.5f * gr;
      if (!prof) st.mom[base + i] = p;
      sums[1] += (double)p * (double)p;
      sums[2] += ((double)th - (double)st.theta0[base + i]) * (double)p;
    }
  }
  if (mode == MODE_GRAD) {
    double v1[1] = {sums[0]};
    block_sum_n<NT, 1>(v1, redd);
    if (threadIdx.x == 0) {
      st.ld_out[b] = v1[0] - (double)le * rss / 2.0;
      st.rss_out[b] = rss;
    }
    return;
  }
  block_sum_n<NT, 3>(sums, redd);
  // + log_density_wrt_rss (100-102); network mode: the rss term is added once for the network by the host
  const double ld = sums[0] - (st.netmode ? 0.0 : (double)le * rss / 2.0);
  const double h = ld - 0.5 * sums[1];                   // -H = log density - K (878-883)
  const int stride = st.lint + 1;
  if (mode == MODE_INIT) {
    if (threadIdx.x == 0) {
      st.h0[b] = h;
      st.htrace[(int64_t)b * stride] = h;
      st.status[b] = ST_RUNNING;
      st.uturn[b] = -1;
      st.rss_out[b] = rss;
      st.ld_out[b] = ld;
    }
    for (int i = threadIdx.x; i < P; i += NT) {  // first half step + full position step
      const float e = st.eps[base + i];
      const float th = st.theta[base + i];
      st.theta0[base + i] = th;
      const float p = st.mom[base + i] + 0.5f * e * st.grad[base + i];
      st.mom[base + i] = p;
      st.theta[base + i] = th + e * p;
    }
  } else {
    const double h0 = st.h0[b];
    const bool diverged = !prof && !st.netmode && fabs(h - h0) > (double)st.max_dh;
    if (!prof && threadIdx.x == 0) st.htrace[(int64_t)b * stride + step] = h;
    if (diverged) {  // RejectedEarly: restore the initial params (1264-1279)
      for (int i = threadIdx.x; i < P; i += NT) st.theta[base + i] = st.theta0[base + i];
      if (threadIdx.x == 0) st.status[b] = ST_REJECTED_EARLY;
    } else {
      // U-turn diagnostic (1281-1284)
      if (!prof && threadIdx.x == 0 && sums[2] < 0.0 && st.uturn[b] < 0) st.uturn[b] = step - 1;
      if (mode == MODE_STEP) {  // next step's first half step + position step (params.rs:728-738)
        for (int i = threadIdx.x; i < P; i += NT) {
          const float e = st.eps[base + i];
          const float g = st.grad[base + i];
          const float p = (prof ? st.mom[base + i] + st.eps[base + i] * 0.5f * g : st.mom[base + i]) + 0.5f * e * g;
          if (prof) {
            st.grad[base + i] = st.theta[base + i] + e * p;  // same traffic, chain unchanged
          } else {
            st.mom[base + i] = p;
            st.theta[base + i] += e * p;
          }
        }
      } else if (st.netmode) {  // MODE_LAST, network mode: the host decides for the network
        if (threadIdx.x == 0) {
          st.ld_out[b] = ld;
          st.rss_out[b] = rss;
        }
      } else {  // MODE_LAST: Metropolis decision (accept_or_reject_hmc_state, 928-962)
        const double log_acc = h - h0;
        const double acc_p = log_acc >= 0.0 ? 1.0 : exp(log_acc);
        const bool accept = (double)st.uacc[b] < acc_p;
        if (!accept)
          for (int i = threadIdx.x; i < P; i += NT) st.theta[base + i] = st.theta0[base + i];
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
    refresh_fused_const<NT>(st, b, bd);
  }
}

// small: branches with P <= 2048 and m <= 512 (512 threads: more loads in flight per branch
// than 256, N = 8 shard 0.0163 -> 0.0129 ms, C3 unchanged); large: the rest (1024 threads)
void launch_update(const DevState& st, const int32_t* branches, int32_t nb, int32_t mode, int32_t step,
                   hipStream_t s, int large) {
  if (nb <= 0) return;
  if (large)
    hipLaunchKernelGGL((k_update<UPD_THREADS_L, 4>), dim3(nb), dim3(UPD_THREADS_L), 0, s, st, branches, mode, step);
  else  // one block size for every launch: the reductions' order, hence every bit, does not depend on nb
    hipLaunchKernelGGL((k_update<UPD_THREADS_S, 1>), dim3(nb), dim3(UPD_THREADS_S), 0, s, st, branches, mode, step);
}

bool update_is_large(const BranchDev& d) { return d.P > UPD_CAP * UPD_THREADS || d.m > 2 * UPD_THREADS; }

__global__ void __launch_bounds__(UPD_THREADS) k_fused_const(DevState st, const int32_t* __restrict__ blist) {
  const int b = blist[blockIdx.x];
  const BranchDev bd = st.br[b];
  if (bd.fused) refresh_fused_const<UPD_THREADS>(st, b, bd);
}

void launch_fused_const(const DevState& st, const int32_t* branches, int32_t nb, hipStream_t s) {
  if (nb <= 0) return;
  hipLaunchKernelGGL(k_fused_const, dim3(nb), dim3(UPD_THREADS), 0, s, st, branches);
}

// solo-mode fold (build_plan): the nslab partial slabs a solo plan wrote for a
// branch, summed into the branch's slab 0; its other slabs and rss partials
// zeroed, so k_update's fixed-order split reduction sees the same sum.
// grid (parameter blocks of 32, jobs), 256 threads: thread (lane q of 8, param
// p) adds slabs q, q + 8, ... in order (its loads independent, all in flight),
// then lane 0 adds the 8 partials in q order -- a fixed order, one round of
// memory latency instead of nslab / 16 (the single-branch step of the
// sequential driver: 15 -> ~4 us)
__global__ void __launch_bounds__(256) k_fold_solo(DevState st, const FoldJob* __restrict__ jobs) {
  __shared__ float s_part[FOLD_Q][32];
  const FoldJob j = jobs[blockIdx.y];
  const BranchDev& bd = st.br[j.branch];
  const int P = bd.P;
  float* dst = st.part + bd.part_off;
  const int q = threadIdx.x >> 5, pl = threadIdx.x & 31;
  const int i = blockIdx.x * 32 + pl;
  s_part[q][pl] = i < P ? fold_solo_param(st.part + j.part, P, j.nslab, i, q) : 0.f;
  __syncthreads();
  if (q == 0 && i < P) {
    float t = s_part[0][pl];
#pragma unroll
    for (int k = 1; k < FOLD_Q; ++k) t += s_part[k][pl];
    dst[i] = t;
    for (int s = 1; s < bd.nsplits; ++s) dst[(int64_t)s * P + i] = 0.f;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) fold_solo_rss(st, j, bd);
}

void launch_fold_solo(const DevState& st, const FoldJob* jobs, int32_t njobs, int32_t max_p, hipStream_t s) {
  if (njobs > 0) hipLaunchKernelGGL(k_fold_solo, dim3((max_p + 31) / 32, njobs), dim3(256), 0, s, st, jobs);
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

// Metropolis uniforms, one per branch (accept_or_reject_hmc_state's ThreadRng
// draw, branch_sampler.rs:546-548): Philox, independent of the momentum stream
__global__ void k_uniforms(DevState st, const int32_t* __restrict__ blist, int nb, uint64_t seed) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nb) return;
  const int b = blist[i];
  st.uacc[b] = u01(philox_bits(seed, 0xACCE97ull, (uint64_t)b).x);
}

void launch_uniforms(const DevState& st, const int32_t* branches, int32_t nb, uint64_t seed, hipStream_t s) {
  if (nb <= 0) return;
  hipLaunchKernelGGL(k_uniforms, dim3((nb + 255) / 256), dim3(256), 0, s, st, branches, nb, seed);
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

// network mode (bann_network_hmc_step): out[i] = sum over the listed branches of
// pred[b][i].  Two passes as the residual change: RD_GROUPS branch slices sum
// their rows (4 individuals per thread, loads unrolled), then the slices are
// added in order (deterministic).  (One thread per individual looping over all
// 1000 branches: 0.42 ms, latency-bound on 196 workgroups.)
__global__ void __launch_bounds__(256) k_net_sum_part(DevState st, const int32_t* __restrict__ blist, int nb,
                                                      float* __restrict__ part) {
  const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i0 >= st.n) return;
  const int g = blockIdx.y;
  const int q0 = (int)((int64_t)nb * g / RD_GROUPS), q1 = (int)((int64_t)nb * (g + 1) / RD_GROUPS);
  const bool full = i0 + 4 <= st.n && (st.n & 3) == 0;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll 8
  for (int q = q0; q < q1; ++q) {
    const int64_t o = (int64_t)blist[q] * st.n + i0;
    if (full) {
      const float4 p = *reinterpret_cast<const float4*>(st.pred + o);
      a0 += p.x;
      a1 += p.y;
      a2 += p.z;
      a3 += p.w;
    } else {
      a0 += st.pred[o];
      if (i0 + 1 < st.n) a1 += st.pred[o + 1];
      if (i0 + 2 < st.n) a2 += st.pred[o + 2];
      if (i0 + 3 < st.n) a3 += st.pred[o + 3];
    }
  }
  float* row = part + (int64_t)g * st.n + i0;
  row[0] = a0;
  if (i0 + 1 < st.n) row[1] = a1;
  if (i0 + 2 < st.n) row[2] = a2;
  if (i0 + 3 < st.n) row[3] = a3;
}

void launch_net_sum(const DevState& st, const int32_t* branches, int32_t nb, float* out, float* scratch,
                    hipStream_t s) {
  const unsigned gx = (unsigned)((st.n + 1023) / 1024);
  hipLaunchKernelGGL(k_net_sum_part, dim3(gx, RD_GROUPS), dim3(256), 0, s, st, branches, nb, scratch);
  hipLaunchKernelGGL(k_residual_delta_sum, dim3((unsigned)((st.n + 255) / 256)), dim3(256), 0, s, scratch, st.n, out);
}

// the same over contiguous rows (group sums of k_forward_gsum): RD_GROUPS row slices, then in order
__global__ void __launch_bounds__(256) k_net_sum_rows_part(const float* __restrict__ rows, int nrows, int64_t n,
                                                           float* __restrict__ part) {
  const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i0 >= n) return;
  const int g = blockIdx.y;
  const int q0 = (int)((int64_t)nrows * g / RD_GROUPS), q1 = (int)((int64_t)nrows * (g + 1) / RD_GROUPS);
  const bool full = i0 + 4 <= n && (n & 3) == 0;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll 8
  for (int q = q0; q < q1; ++q) {
    const int64_t o = (int64_t)q * n + i0;
    if (full) {
      const float4 p = *reinterpret_cast<const float4*>(rows + o);
      a0 += p.x;
      a1 += p.y;
      a2 += p.z;
      a3 += p.w;
    } else {
      a0 += rows[o];
      if (i0 + 1 < n) a1 += rows[o + 1];
      if (i0 + 2 < n) a2 += rows[o + 2];
      if (i0 + 3 < n) a3 += rows[o + 3];
    }
  }
  float* row = part + (int64_t)g * n + i0;
  row[0] = a0;
  if (i0 + 1 < n) row[1] = a1;
  if (i0 + 2 < n) row[2] = a2;
  if (i0 + 3 < n) row[3] = a3;
}

void launch_net_sum_rows(const DevState& st, const float* rows, int32_t nrows, float* out, float* scratch,
                         hipStream_t s) {
  const unsigned gx = (unsigned)((st.n + 1023) / 1024);
  hipLaunchKernelGGL(k_net_sum_rows_part, dim3(gx, RD_GROUPS), dim3(256), 0, s, rows, nrows, st.n, scratch);
  hipLaunchKernelGGL(k_residual_delta_sum, dim3((unsigned)((st.n + 255) / 256)), dim3(256), 0, s, scratch, st.n, out);
}

// e = sum f + bias - y (the network's output error, every branch's output
// gradient), in place of the sum; each branch's target becomes y_b = f_b - e so
// that the per-branch gradient kernels see e as their error; rss = sum e^2
// (per-block partials, then a fixed-order sum: deterministic)
#define NET_BLK 1024
__global__ void __launch_bounds__(NET_BLK) k_net_err(int64_t n, float* __restrict__ sum_e, const float* __restrict__ y,
                                                     float bias, double* __restrict__ part) {
  __shared__ double red[NET_BLK / 64];
  const int64_t i = (int64_t)blockIdx.x * NET_BLK + threadIdx.x;
  double acc = 0.0;
  if (i < n) {
    const float e = sum_e[i] + bias - y[i];
    sum_e[i] = e;
    acc = (double)e * (double)e;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < NET_BLK / 64; ++w) t += red[w];
    part[blockIdx.x] = t;
  }
}

__global__ void k_net_rss(const double* __restrict__ part, int nparts, double* __restrict__ rss_out) {
  if (threadIdx.x != 0) return;
  double t = 0.0;
  for (int k = 0; k < nparts; ++k) t += part[k];
  *rss_out = t;
}

__global__ void __launch_bounds__(256) k_net_targets(DevState st, const int32_t* __restrict__ blist,
                                                     const float* __restrict__ e) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= st.n) return;
  const int64_t o = (int64_t)blist[blockIdx.y] * st.n + i;
  st.y[o] = st.pred[o] - e[i];
}

int64_t net_scratch_doubles(int64_t n) { return (n + NET_BLK - 1) / NET_BLK; }

void launch_net_targets(const DevState& st, const int32_t* branches, int32_t nb, float* sum_e, const float* y,
                        float bias, double* part, double* rss_out, hipStream_t s) {
  const int nparts = (int)((st.n + NET_BLK - 1) / NET_BLK);
  if (y) {  // y = null: sum_e already holds e, only the targets are written
    hipLaunchKernelGGL(k_net_err, dim3(nparts), dim3(NET_BLK), 0, s, st.n, sum_e, y, bias, part);
    hipLaunchKernelGGL(k_net_rss, dim3(1), dim3(64), 0, s, part, nparts, rss_out);
  }
  if (nb > 0)
    hipLaunchKernelGGL(k_net_targets, dim3((unsigned)((st.n + 255) / 256), (unsigned)nb), dim3(256), 0, s, st,
                       branches, sum_e);
}

// pred <- pred0 for the listed branches that were not accepted (session end)
__global__ void __launch_bounds__(256) k_restore_pred(DevState st, const int32_t* __restrict__ blist) {
  const int b = blist[blockIdx.y];
  if (st.status[b] == ST_ACCEPTED) return;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (int64_t r = i; r < st.n; r += (int64_t)gridDim.x * 256) st.pred[(int64_t)b * st.n + r] = st.pred0[(int64_t)b * st.n + r];
}

void launch_restore_pred(const DevState& st, const int32_t* branches, int32_t nb, hipStream_t s) {
  if (nb <= 0) return;
  const int64_t blocks = std::min<int64_t>((st.n + 255) / 256, 64);
  hipLaunchKernelGGL(k_restore_pred, dim3((unsigned)blocks, (unsigned)nb), dim3(256), 0, s, st, branches);
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

// ===========================================================================
// joint HMC update: hmc_step_joint (branch_sampler.rs:1070-1178) samples the
// parameters AND the precisions.  Per branch and leapfrog step (one workgroup):
//   * per-precision statistics S_q of the current theta: sum theta^2 (ridge) or
//     sum |theta| (lasso) over each precision's group -- an ARD row (one thread,
//     fixed order), a whole layer or a bias vector (fixed-order block sums);
//   * log_density_gradient_joint (406-422): the parameter gradient with the
//     precisions taken from the coordinates phi (l2-regularised biases,
//     333-344), the precision gradients (ridge_ard.rs:221-250, lasso_ard.rs,
//     ridge_base.rs, lasso_base.rs; bias precisions 346-367, error precision
//     369-378);
//   * the joint -H (log_density_joint 292-305 with the output-weight term of the
//     other branches, minus K over both momenta, momentum.rs:78-101), early
//     rejection on it, and the Metropolis test of accept_or_reject_hmc_state
//     (928-962), whose final -H uses the NON-joint log_density (72-78) -- a
//     reference quirk kept for parity;
//   * momentum half steps and the position steps of both coordinate sets
//     (params.rs:344-355, 728-738).
// ===========================================================================
#define UPD_J 256

// (shape, scale) of layer l: NetworkPrecisionHyperparameters::layer_prior_hyperparams (params.rs:146-163)
__device__ __forceinline__ void hyper_of(const DevState& st, int l, int L, double& k, double& s) {
  const int c = l == L - 1 ? 2 : (l == L - 2 ? 1 : 0);
  k = (double)st.hyper[2 * c];
  s = (double)st.hyper[2 * c + 1];
}

__global__ void __launch_bounds__(UPD_J) k_update_joint(DevState st, const int32_t* __restrict__ blist, int mode,
                                                        int step) {
  __shared__ double s_S[BANN_JOINT_MAXQ];
  __shared__ double redd[4 * (UPD_J / 64)];
  const int b = blist[blockIdx.x];
  const BranchDev bd = st.br[b];
  const int P = bd.P, nq = bd.nq, L = bd.L, t = threadIdx.x;
  const int64_t base = bd.p_off, qb = bd.q_off;
  if ((mode == MODE_STEP || mode == MODE_LAST) && st.status[b] != ST_RUNNING) return;
  const bool lasso = bd.prior == 2 || bd.prior == 3;
  const bool ard = bd.prior == 0 || bd.prior == 2;
  double rss = 0.0;
  for (int s = 0; s < bd.nsplits; ++s) rss += st.rss_part[(int64_t)b * st.max_splits + s];
  float* phi = st.phi + qb;
  const float le = phi[nq - 1];
  const double n = (double)st.n;

  // ---- S_q at the current theta ----
  for (int q = t; q < nq; q += UPD_J) s_S[q] = 0.0;
  __syncthreads();
  for (int l = 0; l < L; ++l) {
    const int wi = bd.win[l], wo = bd.widths[l];
    const float* W = st.theta + base + bd.woff[l];
    if (ard && l < L - 1) {  // one precision per input row, tiled over the columns (ridge_ard.rs:36-37)
      for (int j = t; j < wi; j += UPD_J) {
        double a = 0.0;
        for (int k = 0; k < wo; ++k) {
          const double w = (double)W[k * wi + j];
          a += lasso ? fabs(w) : w * w;
        }
        s_S[bd.qoff[l] + j] = a;
      }
    } else {
      double a[1] = {0.0};
      for (int i = t; i < wi * wo; i += UPD_J) {
        const double w = (double)W[i];
        a[0] += lasso ? fabs(w) : w * w;
      }
      block_sum_n<UPD_J, 1>(a, redd);
      if (t == 0) s_S[bd.qoff[l]] = a[0];
    }
  }
  for (int l = 0; l < L - 1; ++l) {  // bias precisions: l2 (sum_of_squares, 346-367)
    const float* B = st.theta + base + bd.boff[l];
    double a[1] = {0.0};
    for (int i = t; i < bd.widths[l]; i += UPD_J) a[0] += (double)B[i] * (double)B[i];
    block_sum_n<UPD_J, 1>(a, redd);
    if (t == 0) s_S[bd.qbias + l] = a[0];
  }
  __syncthreads();

  // sums[0]: joint log density (every term is attached to one precision),
  // sums[1]: sum p^2 over both momenta, sums[2]: non-joint weight prior
  double sums[3] = {0.0, 0.0, 0.0};
  for (int i = t; i < P; i += UPD_J) {
    float d = 0.f;
    for (int s = 0; s < bd.nsplits; ++s) d += st.part[bd.part_off + (int64_t)s * P + i];
    const float th = st.theta[base + i];
    const float lm = phi[st.pidx[base + i]];
    float reg;
    if (i >= bd.boff[0])
      reg = lm * th;  // log_density_gradient_wrt_biases_l2 (333-344)
    else
      reg = lasso ? lm * (th > 0.f ? 1.f : (th < 0.f ? -1.f : 0.f)) : lm * th;
    const float gr = -(le * d + reg);
    st.grad[base + i] = gr;
    float p = st.mom[base + i];
    if (mode == MODE_STEP || mode == MODE_LAST) {  // second half step of this leapfrog step (momentum.rs:30-63)
      p = p + st.eps[base + i] * 0.5f * gr;
      st.mom[base + i] = p;
    }
    sums[1] += (double)p * (double)p;
  }
  for (int q = t; q < nq; q += UPD_J) {
    const double lam = (double)phi[q], S = s_S[q];
    double k, s, g, ldj, ldn = 0.0;
    if (q == nq - 1) {  // error precision (log_density_joint_wrt_rss 240-257, gradient 369-378)
      hyper_of(st, L - 1, L, k, s);
      g = (2.0 * k + n - 2.0) / (2.0 * lam) - 1.0 / s - rss / 2.0;
      ldj = (k + (n - 2.0) / 2.0) * log(lam) - lam * (rss / 2.0 + 1.0 / s);
    } else if (q >= bd.qbias) {  // bias precision (260-279, 346-367)
      const int l = q - bd.qbias;
      hyper_of(st, l, L, k, s);
      const double nv = (double)bd.widths[l];
      g = (2.0 * k + (nv - 2.0)) / (2.0 * lam) - 1.0 / s - S / 2.0;
      ldj = -lam * (S / 2.0 + 1.0 / s) + (k + (nv - 2.0) / 2.0) * log(lam);
    } else {
      int l = 0;
      while (l + 1 < L && bd.qoff[l + 1] <= q) ++l;
      hyper_of(st, l, L, k, s);
      if (l == L - 1) {  // output layer: the other branches' summary stat joins (ridge_ard.rs:150-169, 236-248)
        const double rs = (double)st.ows[2 * b], np_ = (double)st.ows[2 * b + 1];
        if (lasso) {
          g = (k + np_ - 1.0) / lam - 1.0 / s - (S + rs);
          ldj = -((S + rs) + 1.0 / s) * lam + (k + np_ - 1.0) * log(lam);
        } else {
          g = (2.0 * k + np_ - 2.0) / (2.0 * lam) - 1.0 / s - (S + rs) / 2.0;
          ldj = -(0.5 * (S + rs) + 1.0 / s) * lam + (k + (np_ - 2.0) / 2.0) * log(lam);
        }
      } else if (ard) {  // per input row: the gradient counts the rows (precisions.elements(), quirk), the density the columns
        const double nr = (double)bd.win[l], nc = (double)bd.widths[l];
        if (lasso) {
          g = (k + nr - 1.0) / lam - 1.0 / s - S;
          ldj = -(S + 1.0 / s) * lam + (k + nc - 1.0) * log(lam);
        } else {
          g = (2.0 * k + nr - 2.0) / (2.0 * lam) - 1.0 / s - S / 2.0;
          ldj = -(S / 2.0 + 1.0 / s) * lam + (k + (nc - 2.0) / 2.0) * log(lam);
        }
      } else {  // base priors: one precision per layer
        const double sz = (double)bd.win[l] * (double)bd.widths[l];
        if (lasso) {
          g = (k + sz - 1.0) / lam - 1.0 / s - S;
          ldj = -(S + 1.0 / s) * lam + (k + sz - 1.0) * log(lam);
        } else {
          g = (2.0 * k + sz - 2.0) / (2.0 * lam) - 1.0 / s - S / 2.0;
          ldj = -(S / 2.0 + 1.0 / s) * lam + (k + (sz - 2.0) / 2.0) * log(lam);
        }
      }
      ldn = -lam * (lasso ? S : S / 2.0);  // non-joint log_density_wrt_weights (ridge_ard.rs:171-194 etc.)
    }
    const float gq = (float)g;
    st.gphi[qb + q] = gq;
    float p = st.mphi[qb + q];
    if (mode == MODE_STEP || mode == MODE_LAST) {
      p = p + st.ephi[qb + q] * 0.5f * gq;
      st.mphi[qb + q] = p;
    }
    sums[0] += ldj;
    sums[1] += (double)p * (double)p;
    sums[2] += ldn;
  }
  block_sum_n<UPD_J, 3>(sums, redd);
  const double ldj = sums[0];
  const double ldn = sums[2] - (double)le * rss / 2.0;
  const double h = ldj - 0.5 * sums[1];
  if (mode == MODE_GRAD) {  // bann_log_density_gradient_joint: gradients, joint log density and rss only
    if (t == 0) {
      st.ld_out[b] = ldj;
      st.rss_out[b] = rss;
    }
    return;
  }
  const int stride = st.lint + 1;
  int act = 0;  // 0: (half step +) position step, 1: restore theta0 / phi0, 2: keep
  if (mode == MODE_INIT) {
    if (t == 0) {
      st.h0[b] = h;
      st.htrace[(int64_t)b * stride] = h;
      st.status[b] = ST_RUNNING;
      st.uturn[b] = -1;
      st.rss_out[b] = rss;
      st.ld_out[b] = ldn;
    }
  } else {
    const double h0 = st.h0[b];
    if (t == 0) st.htrace[(int64_t)b * stride + step] = h;
    if (fabs(h - h0) > (double)st.max_dh) {  // RejectedEarly (1138-1158); NaN never exceeds
      act = 1;
      if (t == 0) st.status[b] = ST_REJECTED_EARLY;
    } else if (mode == MODE_LAST) {  // accept_or_reject_hmc_state: the final -H is NON-joint (943)
      const double log_acc = (ldn - 0.5 * sums[1]) - h0;
      const double acc_p = log_acc >= 0.0 ? 1.0 : exp(log_acc);
      const bool accept = (double)st.uacc[b] < acc_p;
      act = accept ? 2 : 1;
      if (t == 0) {
        st.status[b] = accept ? ST_ACCEPTED : ST_REJECTED;
        st.ld_out[b] = ldn;
        st.rss_out[b] = rss;
      }
    }
  }
  if (act == 0) {
    for (int i = t; i < P; i += UPD_J) {
      const float e = st.eps[base + i], th = st.theta[base + i];
      const float p = st.mom[base + i] + 0.5f * e * st.grad[base + i];
      st.mom[base + i] = p;
      if (mode == MODE_INIT) st.theta0[base + i] = th;
      st.theta[base + i] = th + e * p;
    }
    for (int q = t; q < nq; q += UPD_J) {
      const float e = st.ephi[qb + q], v = phi[q];
      const float p = st.mphi[qb + q] + 0.5f * e * st.gphi[qb + q];
      st.mphi[qb + q] = p;
      if (mode == MODE_INIT) st.phi0[qb + q] = v;
      phi[q] = v + e * p;
    }
  } else if (act == 1) {
    for (int i = t; i < P; i += UPD_J) st.theta[base + i] = st.theta0[base + i];
    for (int q = t; q < nq; q += UPD_J) phi[q] = st.phi0[qb + q];
  }
  if (bd.fused && act != 2) {
    __syncthreads();
    refresh_fused_const<UPD_J>(st, b, bd);
  }
}

void launch_update_joint(const DevState& st, const int32_t* branches, int32_t nb, int32_t mode, int32_t step,
                         hipStream_t s) {
  if (nb <= 0) return;
  hipLaunchKernelGGL(k_update_joint, dim3(nb), dim3(UPD_J), 0, s, st, branches, mode, step);
}

// N(0, 1) momenta of the precision coordinates (sample_joint_momentum, 611-645)
__global__ void k_sample_momentum_phi(DevState st, const int32_t* __restrict__ blist, uint64_t seed) {
  const int b = blist[blockIdx.y];
  const BranchDev bd = st.br[b];
  const int i2 = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i2 >= bd.nq) return;
  const u32x4 r = philox_bits(seed, 0x7A0E100ull + (uint64_t)b, (uint64_t)i2);
  const float rad = sqrtf(-2.f * logf(u01_open(r.x)));
  float sn, cs;
  sincosf(6.283185307179586f * u01(r.y), &sn, &cs);
  st.mphi[bd.q_off + 2 * i2] = rad * cs;
  if (2 * i2 + 1 < bd.nq) st.mphi[bd.q_off + 2 * i2 + 1] = rad * sn;
}

void launch_sample_momentum_joint(const DevState& st, const int32_t* branches, int32_t nb, int32_t max_q,
                                  uint64_t seed, hipStream_t s) {
  if (nb <= 0 || max_q <= 0) return;
  const int pairs = (max_q + 1) / 2;
  hipLaunchKernelGGL(k_sample_momentum_phi, dim3((pairs + 255) / 256, nb), dim3(256), 0, s, st, branches, seed);
}

// ---- common-mode step sizes of the network-joint state (bann_network_hmc_step) ----
// With Izmailov steps eps_p the joint leapfrog's stiffest direction is the common mode: every
// branch shifting the network output together (u = 1/sqrt(n)); its eigenvalue of E H E is
// lambda_e ||E J^T u||^2 = lambda_e / n sum_p a_p^2 with a_p = eps_p |g_p|, g = J^T 1 (the
// gradient of sum_i F_i, one gradient launch with output error 1) -- B times one branch's for B
// aligned branches.  Water-filling: d_p = min(1, t / a_p) with the largest t such that
// sum_p min(a_p, t)^2 <= T = tau^2 n / lambda_e, so the mode sits at omega eps = tau while
// the parameters that do not drive it keep their steps.  t is chosen among candidates
// t_k^2 = T 2^(-k/2) from a histogram of r_p = a_p^2 / T (integer counts and fixed-point sums:
// deterministic), summed over branches and ranks.
// bin 0: r >= 1; bin j (1 <= j < CM_NC - 1): 2^(-j/2) <= r < 2^(-(j-1)/2); last bin: smaller
// fixed-point unit of the r sums: bins >= 1 hold r < 1, so a u64 bin sum cannot wrap below 2^32
// parameters (bann_dist.hip refuses more than 2^31 per rank)
#define CM_FIX ((double)(1ull << CM_FIX_LOG2))
__device__ __forceinline__ int cm_bin(float r) {
  if (!(r < 1.f)) return 0;
  if (!(r > 0.f)) return CM_NC - 1;
  const int j = (int)floorf(-2.f * __log2f(r)) + 1;
  return j < 1 ? 1 : (j > CM_NC - 1 ? CM_NC - 1 : j);
}

// one workgroup per branch: a_p (into st.grad, scratch before the trajectory's first update) and
// the branch's histogram part[b][0..CM_NC) counts, part[b][CM_NC..2 CM_NC) fixed-point r sums
__global__ void __launch_bounds__(256) k_cm_hist(DevState st, const int32_t* __restrict__ blist, float inv_T,
                                                 unsigned long long* __restrict__ part) {
  __shared__ unsigned long long h[2 * CM_NC];
  const int bi = blockIdx.x;
  const int b = blist[bi];
  const BranchDev bd = st.br[b];
  const int P = bd.P;
  for (int k = threadIdx.x; k < 2 * CM_NC; k += 256) h[k] = 0ull;
  __syncthreads();
  for (int i = threadIdx.x; i < P; i += 256) {
    float g = 0.f;
    for (int s = 0; s < bd.nsplits; ++s) g += st.part[bd.part_off + (int64_t)s * P + i];  // k_update's order
    const float a = st.eps[bd.p_off + i] * fabsf(g);
    st.grad[bd.p_off + i] = a;
    const float r = a * a * inv_T;
    const int k = cm_bin(r);
    atomicAdd(&h[k], 1ull);
    if (k >= 1) atomicAdd(&h[CM_NC + k], (unsigned long long)((double)r * CM_FIX));
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 2 * CM_NC; k += 256) part[(int64_t)bi * 2 * CM_NC + k] = h[k];
}

__global__ void __launch_bounds__(2 * CM_NC) k_cm_sum(const unsigned long long* __restrict__ part, int nb,
                                                      unsigned long long* __restrict__ out) {
  unsigned long long v = 0ull;
  for (int b = 0; b < nb; ++b) v += part[(int64_t)b * 2 * CM_NC + threadIdx.x];
  out[threadIdx.x] = v;
}

// eps_p *= min(1, t / a_p)
// eps_p *= min(1, t / a_p) (a_p = eps_p |g_p|, left in grad by k_cm_hist); the factor is kept
// per parameter (scale) for the frozen form of the rule
__global__ void __launch_bounds__(256) k_cm_apply(DevState st, const int32_t* __restrict__ blist, float t,
                                                  float* __restrict__ scale) {
  const int b = blist[blockIdx.y];
  const BranchDev bd = st.br[b];
  for (int i = blockIdx.x * 256 + threadIdx.x; i < bd.P; i += gridDim.x * 256) {
    const float a = st.grad[bd.p_off + i];
    const float f = a > t ? t / a : 1.f;
    if (a > t) st.eps[bd.p_off + i] *= f;
    scale[bd.p_off + i] = f;
  }
}
// the frozen rule: eps_p *= the factor of the last adapted trajectory (state-independent steps)
__global__ void __launch_bounds__(256) k_cm_rescale(DevState st, const int32_t* __restrict__ blist,
                                                    const float* __restrict__ scale) {
  const int b = blist[blockIdx.y];
  const BranchDev bd = st.br[b];
  for (int i = blockIdx.x * 256 + threadIdx.x; i < bd.P; i += gridDim.x * 256) {
    const float f = scale[bd.p_off + i];
    if (f < 1.f) st.eps[bd.p_off + i] *= f;
  }
}

__global__ void __launch_bounds__(256) k_fill_f32(float* __restrict__ p, float v, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = v;
}
void launch_fill_f32(float* p, float v, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(k_fill_f32, dim3(g), dim3(256), 0, s, p, v, n);
}

void launch_cm_hist(const DevState& st, const int32_t* branches, int32_t nb, float inv_T, unsigned long long* part,
                    unsigned long long* out, hipStream_t s) {
  if (nb <= 0) return;
  hipLaunchKernelGGL(k_cm_hist, dim3(nb), dim3(256), 0, s, st, branches, inv_T, part);
  hipLaunchKernelGGL(k_cm_sum, dim3(1), dim3(2 * CM_NC), 0, s, part, nb, out);
}

void launch_cm_apply(const DevState& st, const int32_t* branches, int32_t nb, int32_t max_p, float t, float* scale,
                     hipStream_t s) {
  if (nb <= 0) return;
  const unsigned gx = (unsigned)std::min<int64_t>((max_p + 255) / 256, 16);
  hipLaunchKernelGGL(k_cm_apply, dim3(gx, (unsigned)nb), dim3(256), 0, s, st, branches, t, scale);
}
void launch_cm_rescale(const DevState& st, const int32_t* branches, int32_t nb, int32_t max_p, const float* scale,
                       hipStream_t s) {
  if (nb <= 0) return;
  const unsigned gx = (unsigned)std::min<int64_t>((max_p + 255) / 256, 16);
  hipLaunchKernelGGL(k_cm_rescale, dim3(gx, (unsigned)nb), dim3(256), 0, s, st, branches, scale);
}
