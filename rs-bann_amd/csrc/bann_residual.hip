// bann_residual.hip — the network residual on the device (include/bann.h,
// "residual bookkeeping"): the bookkeeping Net::train does between branch
// updates (net.rs:158-171 initialize_stats, 279-300 the partial-residual target
// and its update, 319-332 the output bias) and the target rebuild of a packed
// sweep, without n-float host round trips.
//
// The reference keeps the residual as a device Array (net.rs:221) and updates
// it with ArrayFire element-wise ops; here the context owns one n-float device
// residual and every update is one launch.  Reductions (sum, sum of squares)
// are two-pass and fixed-order: deterministic.
#include <math.h>

#include <algorithm>
#include <vector>

#include "ctx_internal.h"

#define RES_BLK 256
#define RES_PER 4  // elements per thread

// out[b][i] = r[i] + pred[b][i] for every listed branch (net.rs:279-280: the
// branch is fitted to the residual plus its own prediction)
__global__ void __launch_bounds__(RES_BLK) k_targets_from_residual(DevState st, const int32_t* __restrict__ blist,
                                                                   int b1, const float* __restrict__ r) {
  const int b = blist ? blist[blockIdx.y] : b1;  // one branch: by value (no list upload, no host wait)
  const int64_t i = ((int64_t)blockIdx.x * RES_BLK + threadIdx.x) * 4;
  const int64_t o = (int64_t)b * st.n + i;
  if (i + 4 <= st.n && (st.n & 3) == 0) {
    const float4 p = *reinterpret_cast<const float4*>(st.pred + o);
    const float4 q = *reinterpret_cast<const float4*>(r + i);
    *reinterpret_cast<float4*>(st.y + o) = make_float4(q.x + p.x, q.y + p.y, q.z + p.z, q.w + p.w);
  } else {
    for (int k = 0; k < 4 && i + k < st.n; ++k) st.y[o + k] = r[i + k] + st.pred[o + k];
  }
}

// residual update + block partials of (sum, sum of squares):
//   op 0: r = r + add                        (output bias, net.rs:321 / 332)
//   op 1: r = y_b - pred_b                   (net.rs:295 / 299: the target minus the branch's
//                                             final prediction; a rejected branch's pred is f(theta_0))
//   op 2: r = (y - add) - sum_b pred_b        (initialize_stats, net.rs:158-171, branches in order)
//   op 3: r unchanged (statistics only)
//   op 4: r = (y_b - pred_b) + add            (op 1 then op 0 in one pass: the sequential
//                                             driver's residual update and output-bias shift;
//                                             the statistics of both states, four values)
// The statistics come out of the same launch: every block writes its (sum, sum of
// squares) partial, the last block to arrive (an agent-scope counter, reset by it)
// adds the partials in block order -- the order of the former second launch,
// k_residual_stats -- and writes the pair to out (device) and out_host (the mapped
// pinned result the host reads after the stream synchronises: no copy launch).
__global__ void __launch_bounds__(RES_BLK) k_residual_op(DevState st, float* __restrict__ r, int op, int b,
                                                         const float* __restrict__ y, float add,
                                                         const int32_t* __restrict__ blist, int nb,
                                                         double* __restrict__ part, unsigned* __restrict__ cnt,
                                                         double* __restrict__ out, double* __restrict__ out_host) {
  __shared__ double s_s[RES_BLK / 64], s_q[RES_BLK / 64], s_s2[RES_BLK / 64], s_q2[RES_BLK / 64];
  __shared__ int s_last;
  double s = 0.0, q = 0.0, s2 = 0.0, q2 = 0.0;
  const int64_t base = (int64_t)blockIdx.x * RES_BLK * RES_PER + threadIdx.x;
#pragma unroll
  for (int k = 0; k < RES_PER; ++k) {
    const int64_t i = base + (int64_t)k * RES_BLK;
    if (i >= st.n) break;
    float v;
    if (op == 0) {
      v = r[i] + add;
    } else if (op == 1 || op == 4) {
      const int64_t o = (int64_t)b * st.n + i;
      v = st.y[o] - st.pred[o];
    } else if (op == 2) {
      v = y[i] - add;
      for (int j = 0; j < nb; ++j) v -= st.pred[(int64_t)blist[j] * st.n + i];
    } else {
      v = r[i];
    }
    s += (double)v;
    q += (double)v * (double)v;
    if (op == 4) {
      v = v + add;
      s2 += (double)v;
      q2 += (double)v * (double)v;
    }
    if (op != 3) r[i] = v;
  }
  const int NV = op == 4 ? 4 : 2;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o);
    q += __shfl_xor(q, o);
    s2 += __shfl_xor(s2, o);
    q2 += __shfl_xor(q2, o);
  }
  if ((threadIdx.x & 63) == 0) {
    s_s[threadIdx.x >> 6] = s;
    s_q[threadIdx.x >> 6] = q;
    s_s2[threadIdx.x >> 6] = s2;
    s_q2[threadIdx.x >> 6] = q2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double ts = 0.0, tq = 0.0, ts2 = 0.0, tq2 = 0.0;
    for (int w = 0; w < RES_BLK / 64; ++w) {
      ts += s_s[w];
      tq += s_q[w];
      ts2 += s_s2[w];
      tq2 += s_q2[w];
    }
    part[NV * blockIdx.x] = ts;
    part[NV * blockIdx.x + 1] = tq;
    if (NV == 4) {
      part[NV * blockIdx.x + 2] = ts2;
      part[NV * blockIdx.x + 3] = tq2;
    }
    __threadfence();  // release the partial before counting in
    s_last = atomicAdd(cnt, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last || threadIdx.x >= 64) return;
  __threadfence();  // acquire every block's partial
  const int nblk = (int)gridDim.x;
  double ts = 0.0, tq = 0.0, ts2 = 0.0, tq2 = 0.0;
  for (int k = threadIdx.x; k < nblk; k += 64) {
    ts += part[NV * k];
    tq += part[NV * k + 1];
    if (NV == 4) {
      ts2 += part[NV * k + 2];
      tq2 += part[NV * k + 3];
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ts += __shfl_xor(ts, o);
    tq += __shfl_xor(tq, o);
    ts2 += __shfl_xor(ts2, o);
    tq2 += __shfl_xor(tq2, o);
  }
  if (threadIdx.x == 0) {
    out[0] = ts;
    out[1] = tq;
    out[2] = ts2;
    out[3] = tq2;
    if (out_host) {
      out_host[0] = ts;
      out_host[1] = tq;
      out_host[2] = ts2;
      out_host[3] = tq2;
    }
    *cnt = 0u;  // the next launch counts from zero (stream order)
  }
}

// r -= d (the residual change of a trajectory, summed over the ranks)
__global__ void __launch_bounds__(RES_BLK) k_residual_sub(float* __restrict__ r, const float* __restrict__ d, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * RES_BLK + threadIdx.x;
  if (i < n) r[i] -= d[i];
}

void launch_residual_sub(float* r, const float* d, int64_t n, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_residual_sub, dim3((unsigned)((n + RES_BLK - 1) / RES_BLK)), dim3(RES_BLK), 0, s, r, d, n);
}

static int64_t res_blocks(int64_t n) { return (n + RES_BLK * RES_PER - 1) / (RES_BLK * RES_PER); }

// lazily allocated: the residual, its reduction scratch and a pinned result pair
static int ensure_residual(bann_ctx* ctx) {
  if (!ctx || !ctx->finalized) return fail(ctx, BANN_E_STATE, "not finalized");
  if (!ctx->d_res) {
    CK(dalloc(&ctx->d_res, ctx->n));
    CK(hipMemsetAsync(ctx->d_res, 0, ctx->n * sizeof(float), ctx->stream));
    // block partials (up to four per block), the result (four), the counter
    CK(dalloc(&ctx->d_res_part, 4 * res_blocks(ctx->n) + 8));
    CK(hipMemsetAsync(ctx->d_res_part, 0, (4 * res_blocks(ctx->n) + 8) * sizeof(double), ctx->stream));
    CK(hipHostMalloc((void**)&ctx->h_res_stat, 4 * sizeof(double), hipHostMallocDefault));
    CK(hipHostGetDevicePointer((void**)&ctx->d_res_stat_host, ctx->h_res_stat, 0));
  }
  return BANN_OK;
}

// predictions of the listed branches current (pred_b = f_b(theta_b)): one packed
// launch over the branches whose prediction row is stale
int ensure_predictions(bann_ctx* ctx, const int32_t* branches, int32_t nb) {
  std::vector<int32_t> stale;
  for (int i = 0; i < nb; ++i)
    if (!ctx->pred_ok[branches[i]]) stale.push_back(branches[i]);
  if (stale.empty()) return BANN_OK;
  Plan p;
  int rc = build_plan(ctx, stale.data(), (int32_t)stale.size(), p, false);
  if (rc) return rc;
  return run_forward(ctx, p);
}

// defer: the statistics are written to the pinned h_res_stat but not waited for (the
// caller synchronises the stream later: hmc_step_tail)
static int residual_op(bann_ctx* ctx, int op, int b, const float* d_y, float add, const int32_t* d_list, int nb,
                       double* sum, double* sumsq, double* after = nullptr, bool defer = false) {
  const int64_t nblk = res_blocks(ctx->n);
  const bool want = sum || sumsq || after || defer;
  hipLaunchKernelGGL(k_residual_op, dim3((unsigned)nblk), dim3(RES_BLK), 0, ctx->stream, ctx->st, ctx->d_res, op, b,
                     d_y, add, d_list, nb, ctx->d_res_part,
                     reinterpret_cast<unsigned*>(ctx->d_res_part + 4 * nblk + 4), ctx->d_res_part + 4 * nblk,
                     want ? ctx->d_res_stat_host : nullptr);
  CK(hipGetLastError());
  if (want && !defer) {
    CK(hipStreamSynchronize(ctx->stream));
    if (sum) *sum = ctx->h_res_stat[0];
    if (sumsq) *sumsq = ctx->h_res_stat[1];
    if (after) {
      after[0] = ctx->h_res_stat[2];
      after[1] = ctx->h_res_stat[3];
    }
  }
  return BANN_OK;
}

static bool session_free(bann_ctx* ctx) { return !ctx->lf_active; }

extern "C" int bann_residual_set(bann_ctx* ctx, const float* r) {
  int rc = ensure_residual(ctx);
  if (rc) return rc;
  if (!r) return fail(ctx, BANN_E_ARG, "null residual");
  CK(hipMemcpyAsync(ctx->d_res, r, ctx->n * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  return BANN_OK;
}

extern "C" int bann_residual_get(bann_ctx* ctx, float* r) {
  int rc = ensure_residual(ctx);
  if (rc) return rc;
  if (!r) return fail(ctx, BANN_E_ARG, "null output");
  CK(hipMemcpyAsync(r, ctx->d_res, ctx->n * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  return BANN_OK;
}

extern "C" int bann_residual_device(bann_ctx* ctx, float** out) {
  int rc = ensure_residual(ctx);
  if (rc) return rc;
  if (!out) return fail(ctx, BANN_E_ARG, "null output");
  *out = ctx->d_res;
  return BANN_OK;
}

extern "C" int bann_residual_stats(bann_ctx* ctx, double* sum, double* sumsq) {
  int rc = ensure_residual(ctx);
  if (rc) return rc;
  return residual_op(ctx, 3, 0, nullptr, 0.f, nullptr, 0, sum, sumsq);
}

extern "C" int bann_residual_shift(bann_ctx* ctx, float add, double* sum, double* sumsq) {
  int rc = ensure_residual(ctx);
  if (rc) return rc;
  return residual_op(ctx, 0, 0, nullptr, add, nullptr, 0, sum, sumsq);
}

extern "C" int bann_residual_init(bann_ctx* ctx, const float* y, float bias, double* sum, double* sumsq) {
  int rc = ensure_residual(ctx);
  if (rc) return rc;
  if (!y) return fail(ctx, BANN_E_ARG, "null phenotype");
  if (!session_free(ctx)) return fail(ctx, BANN_E_STATE, "a leapfrog session is active");
  const int32_t nb = (int32_t)ctx->br.size();
  std::vector<int32_t> all(nb);
  for (int b = 0; b < nb; ++b) all[b] = b;
  rc = ensure_predictions(ctx, all.data(), nb);
  if (rc) return rc;
  // y staged through the residual-change scratch (n floats)
  CK(hipMemcpyAsync(ctx->d_delta, y, ctx->n * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
  CK(hipMemcpyAsync(ctx->d_list_scr, all.data(), nb * sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream));
  rc = residual_op(ctx, 2, 0, ctx->d_delta, bias, ctx->d_list_scr, nb, sum, sumsq);
  if (rc) return rc;
  CK(hipStreamSynchronize(ctx->stream));  // `all` goes out of scope
  return BANN_OK;
}

extern "C" int bann_rebuild_targets(bann_ctx* ctx, const int32_t* branches, int32_t nb, const float* residual_device) {
  if (!ctx || !ctx->finalized) return fail(ctx, BANN_E_STATE, "not finalized");
  if (!branches || nb <= 0 || nb > (int32_t)ctx->br.size()) return fail(ctx, BANN_E_ARG, "bad branch list");
  if (!session_free(ctx)) return fail(ctx, BANN_E_STATE, "a leapfrog session is active");
  for (int i = 0; i < nb; ++i)
    if (branches[i] < 0 || branches[i] >= (int32_t)ctx->br.size()) return fail(ctx, BANN_E_SHAPE, "branch index");
  const float* r = residual_device;
  if (!r) {
    int rc = ensure_residual(ctx);
    if (rc) return rc;
    r = ctx->d_res;
  }
  int rc = ensure_predictions(ctx, branches, nb);
  if (rc) return rc;
  // the branch list: the leapfrog session's persistent list when it is the same set
  const int32_t* d_list = nullptr;
  if (nb == 1) {  // one branch (the sequential driver): by value
    hipLaunchKernelGGL(k_targets_from_residual, dim3((unsigned)((ctx->n + 4 * RES_BLK - 1) / (4 * RES_BLK)), 1u),
                       dim3(RES_BLK), 0, ctx->stream, ctx->st, nullptr, branches[0], r);
    CK(hipGetLastError());
    return BANN_OK;
  }
  if (ctx->lf.owns && ctx->lf.all.size() == (size_t)nb && std::equal(branches, branches + nb, ctx->lf.all.begin())) {
    d_list = ctx->lf.d_all;
  } else {
    CK(hipMemcpyAsync(ctx->d_list_scr, branches, nb * sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream));
    d_list = ctx->d_list_scr;
  }
  hipLaunchKernelGGL(k_targets_from_residual, dim3((unsigned)((ctx->n + 4 * RES_BLK - 1) / (4 * RES_BLK)), (unsigned)nb),
                     dim3(RES_BLK), 0, ctx->stream, ctx->st, d_list, 0, r);
  CK(hipGetLastError());
  if (d_list == ctx->d_list_scr) CK(hipStreamSynchronize(ctx->stream));  // host list copied
  return BANN_OK;
}

extern "C" int bann_residual_to_target(bann_ctx* ctx, int32_t b) { return bann_rebuild_targets(ctx, &b, 1, nullptr); }

extern "C" int bann_residual_from_target(bann_ctx* ctx, int32_t b, double* sum, double* sumsq) {
  int rc = ensure_residual(ctx);
  if (rc) return rc;
  if (!check_branch(ctx, b)) return fail(ctx, BANN_E_ARG, "bad branch");
  if (!session_free(ctx)) return fail(ctx, BANN_E_STATE, "a leapfrog session is active");
  rc = ensure_predictions(ctx, &b, 1);
  if (rc) return rc;
  return residual_op(ctx, 1, b, nullptr, 0.f, nullptr, 0, sum, sumsq);
}

// the sequential driver's residual update (net.rs:292-300) and the output-bias shift that
// follows it (net.rs:319-321) in one launch: residual = (y_b - f_b) + add; stats of the
// residual before (sum, sum of squares) and after the shift -- the bits of
// bann_residual_from_target followed by bann_residual_shift(add)
// the same residual op launched without a wait: its statistics (sum, sum of squares
// before and after the shift) are in ctx->h_res_stat once the stream has drained
int residual_from_target_shift_launch(bann_ctx* ctx, int32_t b, float add) {
  int rc = ensure_residual(ctx);
  if (rc) return rc;
  if (!check_branch(ctx, b)) return fail(ctx, BANN_E_ARG, "bad branch");
  if (!session_free(ctx)) return fail(ctx, BANN_E_STATE, "a leapfrog session is active");
  rc = ensure_predictions(ctx, &b, 1);
  if (rc) return rc;
  return residual_op(ctx, 4, b, nullptr, add, nullptr, 0, nullptr, nullptr, nullptr, true);
}

int residual_from_target_shift(bann_ctx* ctx, int32_t b, float add, double* sum, double* sumsq, double* sum_after,
                               double* sumsq_after) {
  int rc = ensure_residual(ctx);
  if (rc) return rc;
  if (!check_branch(ctx, b)) return fail(ctx, BANN_E_ARG, "bad branch");
  if (!session_free(ctx)) return fail(ctx, BANN_E_STATE, "a leapfrog session is active");
  rc = ensure_predictions(ctx, &b, 1);
  if (rc) return rc;
  double aft[2] = {0.0, 0.0};
  rc = residual_op(ctx, 4, b, nullptr, add, nullptr, 0, sum, sumsq, aft);
  if (rc) return rc;
  if (sum_after) *sum_after = aft[0];
  if (sumsq_after) *sumsq_after = aft[1];
  return BANN_OK;
}
