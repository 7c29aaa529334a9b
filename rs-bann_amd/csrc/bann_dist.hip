// bann_dist.hip — multi-GPU entry points of include/bann.h: branch shards (one
// process per GPU), the context's communicator (RCCL over xGMI, or a caller
// all-reduce), the residual exchange of a leapfrog session, and the
// network-joint HMC trajectory with its per-step all-reduce of the summed
// branch outputs (north_star: "an RCCL all-reduce over xGMI only
// for the summary-layer output and its gradient").
//
// The reference is single-device: Net::train (net.rs:251-334) visits the
// branches one after another against a residual it refreshes in between.  The
// branch-sharded equivalents here are (a) leapfrog sessions per rank with the
// residual change exchanged per trajectory (the sweep bookkeeping of
// net.rs:292-300 over ranks) and (b) one HMC state over all branches of all
// ranks (network mode).
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <random>
#include <vector>

#include <rccl/rccl.h>

#include "ctx_internal.h"

void comm_destroy(bann_ctx* ctx) {
  if (ctx->nccl) (void)ncclCommDestroy((ncclComm_t)ctx->nccl);
  ctx->nccl = nullptr;
  ctx->comm_kind = 0;
}

extern "C" int bann_shard_branches(const int32_t* marker_counts, int32_t nbranches, int32_t world,
                                   int32_t* starts_out) {
  if (!marker_counts || !starts_out || nbranches <= 0 || world <= 0 || world > nbranches) return BANN_E_ARG;
  std::vector<int64_t> csum(nbranches + 1, 0);
  for (int b = 0; b < nbranches; ++b) {
    if (marker_counts[b] <= 0) return BANN_E_ARG;
    csum[b + 1] = csum[b] + marker_counts[b];
  }
  starts_out[0] = 0;
  for (int r = 1; r < world; ++r) {
    // first branch whose prefix reaches r/world of the markers, leaving every
    // rank at least one branch on either side
    const double target = (double)csum[nbranches] * r / world;
    int c = (int)(std::lower_bound(csum.begin(), csum.end(), (int64_t)ceil(target)) - csum.begin());
    c = std::max(c, starts_out[r - 1] + 1);
    c = std::min(c, nbranches - (world - r));
    starts_out[r] = c;
  }
  starts_out[world] = nbranches;
  return BANN_OK;
}

extern "C" int bann_comm_unique_id(uint8_t* id_out) {
  if (!id_out) return BANN_E_ARG;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return BANN_E_HIP;
  static_assert(sizeof(id) == 128, "RCCL unique id size");
  memcpy(id_out, &id, sizeof(id));
  return BANN_OK;
}

extern "C" int bann_ctx_comm_init(bann_ctx* ctx, const uint8_t* id, int32_t nranks, int32_t rank) {
  if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks) return BANN_E_ARG;
  comm_destroy(ctx);
  CK(hipSetDevice(ctx->device));
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclComm_t comm;
  const ncclResult_t r = ncclCommInitRank(&comm, nranks, uid, rank);
  if (r != ncclSuccess) return fail(ctx, BANN_E_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  ctx->nccl = comm;
  ctx->comm_kind = 1;
  ctx->nranks = nranks;
  ctx->rank = rank;
  return BANN_OK;
}

extern "C" int bann_comm_info(const bann_ctx* ctx, int32_t* kind, int32_t* nranks, int32_t* rank,
                               int32_t* backend_ranks) {
  if (!ctx) return BANN_E_ARG;
  int32_t count = ctx->comm_kind == 0 ? 1 : ctx->nranks;
  if (ctx->comm_kind == 1) {  // RCCL's own view of the communicator
    int c = 0;
    if (ncclCommCount((ncclComm_t)ctx->nccl, &c) != ncclSuccess) return BANN_E_HIP;
    count = c;
  }
  if (kind) *kind = ctx->comm_kind;
  if (nranks) *nranks = ctx->comm_kind == 0 ? 1 : ctx->nranks;
  if (rank) *rank = ctx->comm_kind == 0 ? 0 : ctx->rank;
  if (backend_ranks) *backend_ranks = count;
  return BANN_OK;
}

extern "C" int bann_ctx_comm_callback(bann_ctx* ctx, bann_allreduce_fn fn, void* user, int32_t nranks, int32_t rank) {
  if (!ctx || !fn || nranks < 1 || rank < 0 || rank >= nranks) return BANN_E_ARG;
  comm_destroy(ctx);
  ctx->ar_fn = fn;
  ctx->ar_user = user;
  ctx->comm_kind = 2;
  ctx->nranks = nranks;
  ctx->rank = rank;
  return BANN_OK;
}

extern "C" int bann_residual_update_host(bann_allreduce_fn fn, void* user, float* local_delta, float* residual,
                                         int64_t n) {
  if (!local_delta || !residual || n < 0) return BANN_E_ARG;
  if (fn && fn(user, local_delta, n, 0) != 0) return BANN_E_HIP;
  for (int64_t i = 0; i < n; ++i) residual[i] -= local_delta[i];  // net.rs:292-300
  return BANN_OK;
}

// in-place sum over the ranks of n floats in a DEVICE buffer (on the context stream)
static int allreduce_device_f32(bann_ctx* ctx, float* d, int64_t n) {
  if (ctx->comm_kind == 1) {
    const ncclResult_t r = ncclAllReduce(d, d, (size_t)n, ncclFloat32, ncclSum, (ncclComm_t)ctx->nccl, ctx->stream);
    if (r != ncclSuccess) return fail(ctx, BANN_E_HIP, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
  } else if (ctx->comm_kind == 2) {
    std::vector<float> h(n);
    CK(hipMemcpyAsync(h.data(), d, n * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    CK(hipStreamSynchronize(ctx->stream));
    if (ctx->ar_fn(ctx->ar_user, h.data(), n, 0) != 0) return fail(ctx, BANN_E_HIP, "all-reduce callback failed");
    CK(hipMemcpyAsync(d, h.data(), n * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
    CK(hipStreamSynchronize(ctx->stream));
  }
  return BANN_OK;
}

// in-place sum over the ranks of n doubles in a HOST buffer (RCCL: through a
// context-owned device buffer, grown geometrically, not allocated per call)
static int allreduce_host_f64(bann_ctx* ctx, double* h, int64_t n) {
  if (ctx->comm_kind == 1) {
    if (ctx->ar64_cap < n) {
      dfree(ctx->d_ar64);
      ctx->d_ar64 = nullptr;
      const int64_t cap = std::max<int64_t>(n, 2 * ctx->ar64_cap);
      CK(dalloc(&ctx->d_ar64, cap));
      ctx->ar64_cap = cap;
    }
    double* d = ctx->d_ar64;
    CK(hipMemcpyAsync(d, h, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    const ncclResult_t r = ncclAllReduce(d, d, (size_t)n, ncclFloat64, ncclSum, (ncclComm_t)ctx->nccl, ctx->stream);
    if (r != ncclSuccess) return fail(ctx, BANN_E_HIP, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
    CK(hipMemcpyAsync(h, d, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    CK(hipStreamSynchronize(ctx->stream));
  } else if (ctx->comm_kind == 2) {
    if (ctx->ar_fn(ctx->ar_user, h, n, 1) != 0) return fail(ctx, BANN_E_HIP, "all-reduce callback failed");
  }
  return BANN_OK;
}

extern "C" int bann_exchange_residual(bann_ctx* ctx, float* residual_host) {
  if (!ctx || !residual_host) return BANN_E_ARG;
  if (ctx->lf.all.empty() || ctx->lf_active) return fail(ctx, BANN_E_STATE, "call after bann_leapfrog_end");
  launch_residual_delta(ctx->st, ctx->lf.d_all, (int32_t)ctx->lf.all.size(), ctx->d_delta_part, ctx->d_delta,
                        ctx->stream);
  CK(hipGetLastError());
  if (ctx->comm_kind == 1) {  // sum over the ranks on the device (RCCL over xGMI), one copy back
    int rc = allreduce_device_f32(ctx, ctx->d_delta, ctx->n);
    if (rc) return rc;
  }
  CK(hipMemcpyAsync(ctx->h_delta, ctx->d_delta, ctx->n * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  const bann_allreduce_fn fn = ctx->comm_kind == 2 ? ctx->ar_fn : nullptr;
  const int rc = bann_residual_update_host(fn, ctx->ar_user, ctx->h_delta, residual_host, ctx->n);
  return rc ? fail(ctx, rc, "residual exchange failed") : BANN_OK;
}

// d_res -= sum over ranks of the last session's residual change, on the device
// (net.rs:292-300 over ranks; with RCCL no host copy at all)
extern "C" int bann_exchange_residual_device(bann_ctx* ctx) {
  if (!ctx) return BANN_E_ARG;
  if (ctx->lf.all.empty() || ctx->lf_active) return fail(ctx, BANN_E_STATE, "call after bann_leapfrog_end");
  float* res = nullptr;
  int rc = bann_residual_device(ctx, &res);
  if (rc) return rc;
  launch_residual_delta(ctx->st, ctx->lf.d_all, (int32_t)ctx->lf.all.size(), ctx->d_delta_part, ctx->d_delta,
                        ctx->stream);
  CK(hipGetLastError());
  rc = allreduce_device_f32(ctx, ctx->d_delta, ctx->n);
  if (rc) return rc;
  launch_residual_sub(res, ctx->d_delta, ctx->n, ctx->stream);
  CK(hipGetLastError());
  return BANN_OK;
}

extern "C" int bann_set_network_step_rule(bann_ctx* ctx, int32_t common_mode, float tau) {
  if (!ctx) return BANN_E_ARG;
  if (common_mode < 0 || common_mode > 3)
    return fail(ctx, BANN_E_ARG, "common_mode: 0 off, 1 adapt every trajectory, 2 frozen, 3 auto");
  if (common_mode && !(tau > 0.f)) return fail(ctx, BANN_E_ARG, "tau must be positive");
  if ((common_mode == 1 || common_mode == 3) && ctx->cm_tau != tau) ctx->cm_have_scale = false;
  if (common_mode == 3) ctx->cm_adapted = 0;  // auto: adapt afresh, then freeze
  ctx->cm_rule = common_mode;
  ctx->cm_tau = tau;
  return BANN_OK;
}

extern "C" int bann_set_network_adapt_trajectories(bann_ctx* ctx, int32_t k) {
  if (!ctx) return BANN_E_ARG;
  if (k < 1) return fail(ctx, BANN_E_ARG, "at least one adapting trajectory");
  ctx->cm_adapt_total = k;
  ctx->cm_adapted = 0;
  return BANN_OK;
}

extern "C" int bann_network_step_rule_state(const bann_ctx* ctx, int32_t* mode, int32_t* adapted, int32_t* frozen) {
  if (!ctx) return BANN_E_ARG;
  if (mode) *mode = ctx->cm_rule;
  if (adapted) *adapted = ctx->cm_adapted;
  // the next trajectory takes the stored factors without recomputing them
  const bool fz = ctx->cm_have_scale &&
                  (ctx->cm_rule == 2 || (ctx->cm_rule == 3 && ctx->cm_adapted >= ctx->cm_adapt_total));
  if (frozen) *frozen = fz ? 1 : 0;
  return BANN_OK;
}

// the network sampler's buffers (bann_finalize): the error / sum n-vectors, the rss
// trace, the common-mode rule's factors, ones and histograms.  Nothing is allocated
// or uploaded synchronously inside bann_network_hmc_step (but a longer L grows the
// rss trace once).
int net_buffers_init(bann_ctx* ctx) {
  const int64_t n = ctx->n;
  if (!ctx->d_netsum) {
    CK(dalloc(&ctx->d_netsum, n));
    CK(dalloc(&ctx->d_nety, n));
    CK(dalloc(&ctx->d_netpart, net_scratch_doubles(n)));
  }
  if (ctx->netrss_cap < 129) {
    dfree(ctx->d_netrss);
    ctx->d_netrss = nullptr;
    CK(dalloc(&ctx->d_netrss, 129));
    ctx->netrss_cap = 129;
  }
  if (!ctx->d_cm_scale && !ctx->br.empty()) {
    const BranchHost& last = ctx->br.back();
    CK(dalloc(&ctx->d_cm_scale, last.dev.p_off + last.P));
  }
  if (!ctx->d_gsum && ctx->net_gsum) {  // one row per (at least) 8 fx branches of 8 chunks and one (L, act)
    std::vector<std::pair<int64_t, int32_t>> cls;  // ((L, act), count)
    for (const auto& h : ctx->br)
      if (h.dev.fused == 1 && h.dev.nchunks == 8) {
        const int64_t key = (int64_t)h.L * 64 + h.act;
        bool found = false;
        for (auto& c : cls)
          if (c.first == key) ++c.second, found = true;
        if (!found) cls.push_back({key, 1});
      }
    int64_t rows = 0;
    for (const auto& c : cls) rows += (c.second + 7) / 8;
    if (rows > 0) {
      CK(dalloc(&ctx->d_gsum, rows * n));
      ctx->gsum_cap = (int32_t)rows;
    }
  }
  if (!ctx->d_ones) {
    CK(dalloc(&ctx->d_ones, n));
    launch_fill_f32(ctx->d_ones, 1.f, n, ctx->stream);
    CK(hipGetLastError());
    CK(dalloc(&ctx->d_cm, ((int64_t)ctx->br.size() + 1) * 2 * CM_NC));
  }
  return BANN_OK;
}

extern "C" int bann_network_info(const bann_ctx* ctx, int32_t* group_rows) {
  if (!ctx) return BANN_E_ARG;
  if (group_rows) *group_rows = ctx->lf.nsum_built ? ctx->lf.nsum_rows : -1;
  return BANN_OK;
}

extern "C" int bann_network_step_rule_info(const bann_ctx* ctx, double* out4) {
  if (!ctx || !out4) return BANN_E_ARG;
  for (int k = 0; k < 4; ++k) out4[k] = ctx->cm_info[k];
  return BANN_OK;
}

// k_forward_gsum's work items for a persistent network plan: usable when every branch of the
// plan is an fx branch of exactly 8 chunks (the full8 groups), L <= 4.  An item takes up to
// 8 R of a launch group's branches (plan order) over one range of T <= forward_gsum_max_tiles()
// tiles, and writes one row; (R, number of ranges) minimise rounds (one workgroup per CU) x
// R x (T + 2), ties going to the larger R (fewer rows).  BANN_NET_GSUM_R forces R (tests).
int build_net_groups(bann_ctx* ctx, Plan& p) {
  p.nsum_built = true;
  p.nsum_rows = 0;
  if (!ctx->d_gsum || !p.gx.empty() || p.groups.empty()) return BANN_OK;
  for (const auto& g : p.groups)
    if (g.kind != 1 || !g.full || g.L < 2 || g.L > 4) return BANN_OK;
  const int64_t ntile = ((int64_t)ctx->nfrag + BANN_TILE_FRAGS - 1) / BANN_TILE_FRAGS;
  const int64_t tmax = forward_gsum_max_tiles();
  const int64_t slots = ctx->cus;
  int force_r = 0;
  if (const char* e = getenv("BANN_NET_GSUM_R")) force_r = std::max(1, atoi(e));
  int32_t row = 0;
  for (auto& g : p.groups) {
    std::vector<int32_t> brs;
    for (const auto& it : g.items)
      if (brs.empty() || brs.back() != it.branch) brs.push_back(it.branch);
    const int64_t nb = (int64_t)brs.size();
    int64_t best = -1, r_best = 1, k_best = 1;
    for (int64_t R = 1; R <= 32; ++R) {
      if (force_r && R != force_r) continue;
      const int64_t ng = (nb + 8 * R - 1) / (8 * R);
      for (int64_t k = (ntile + tmax - 1) / tmax; k <= std::min<int64_t>(ntile, 512); ++k) {
        const int64_t T = (ntile + k - 1) / k;
        const int64_t cost = ((ng * k + slots - 1) / slots) * R * (T + 2);
        if (best < 0 || cost <= best) best = cost, r_best = R, k_best = k;
      }
    }
    const int64_t per = 8 * r_best, ng = (nb + per - 1) / per;
    if (row + ng > ctx->gsum_cap) {  // cannot happen: the cap counts every 8-chunk fx branch in 8s
      p.nsum_rows = 0;
      return BANN_OK;
    }
    g.nitems.clear();
    for (int64_t gi = 0; gi < ng; ++gi)
      for (int64_t s = 0; s < k_best; ++s) {
        NetGroupItem it{};
        it.list_off = (int32_t)(gi * per);
        it.nbr = (int32_t)std::min<int64_t>(per, nb - gi * per);
        it.tile_begin = (int32_t)(ntile * s / k_best);
        it.tile_end = (int32_t)(ntile * (s + 1) / k_best);
        it.row = row + (int32_t)gi;
        if (it.tile_end > it.tile_begin) g.nitems.push_back(it);
      }
    row += (int32_t)ng;
    g.nlist = brs;
    dfree(g.d_nitems);
    dfree(g.d_nlist);
    g.d_nitems = nullptr;
    g.d_nlist = nullptr;
    CK(dalloc(&g.d_nitems, (int64_t)g.nitems.size()));
    CK(dalloc(&g.d_nlist, (int64_t)g.nlist.size()));
    CK(hipMemcpyAsync(g.d_nitems, g.nitems.data(), g.nitems.size() * sizeof(NetGroupItem), hipMemcpyHostToDevice,
                      ctx->stream));
    CK(hipMemcpyAsync(g.d_nlist, g.nlist.data(), g.nlist.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                      ctx->stream));
  }
  CK(hipStreamSynchronize(ctx->stream));  // keep the copies off the timed trajectory
  p.nsum_rows = row;
  return BANN_OK;
}

namespace {
// the group-sum forward of a plan with build_net_groups items (network mode)
void run_forward_gsum(bann_ctx* ctx, const Plan& p) {
  for (const auto& g : p.groups)
    launch_forward_gsum(ctx->st, g.d_nitems, (int32_t)g.nitems.size(), g.d_nlist, g.L, g.act, ctx->d_gsum,
                        ctx->stream);
}

// the common-mode rule (bann.h bann_set_network_step_rule; kernels_update.hip k_cm_*): one gradient
// launch with output error 1 gives g = J^T 1 of every local branch, the histogram of
// r_p = (eps_p g_p)^2 / T is summed over branches and ranks, and eps_p *= min(1, t / (eps_p |g_p|))
// with the largest candidate t^2 = T 2^(-k/2) whose sum_p min(eps_p |g_p|, t)^2 <= T = tau^2 n / lambda_e
int common_mode_steps(bann_ctx* ctx, const Plan& p, bool fx_only, float lambda_e) {
  const int64_t n = ctx->n;
  const int32_t nb = (int32_t)p.all.size();
  int rc = net_buffers_init(ctx);  // no-op after bann_finalize
  if (rc) return rc;
  const bool frozen = ctx->cm_have_scale &&
                      (ctx->cm_rule == 2 || (ctx->cm_rule == 3 && ctx->cm_adapted >= ctx->cm_adapt_total));
  if (frozen) {  // the adapted factors, no gradient launch: step sizes independent of theta_0
    launch_cm_rescale(ctx->st, p.d_all, nb, p.max_p, ctx->d_cm_scale, ctx->stream);
    CK(hipGetLastError());
    return BANN_OK;
  }
  if (ctx->total_p > (int64_t(1) << 31))  // the per-bin u64 fixed-point r sums (k_cm_hist, CM_FIX)
    return fail(ctx, BANN_E_SHAPE, "common-mode rule: more than 2^31 parameters on one rank");
  if (ctx->cm_rule == 3) ++ctx->cm_adapted;
  if (!fx_only) {  // every branch's target f_b - 1 (the prediction rows at theta_0 first)
    int rc = run_forward(ctx, p);
    if (rc) return rc;
    launch_net_targets(ctx->st, p.d_all, nb, ctx->d_ones, nullptr, 0.f, nullptr, nullptr, ctx->stream);
  }
  ctx->st.nete = fx_only ? ctx->d_ones : nullptr;
  rc = run_grad(ctx, p, 0);
  ctx->st.nete = fx_only ? ctx->d_netsum : nullptr;
  if (rc) return rc;
  const double T = (double)ctx->cm_tau * ctx->cm_tau * (double)n / (double)lambda_e;
  unsigned long long* d_out = ctx->d_cm + (int64_t)ctx->br.size() * 2 * CM_NC;
  launch_cm_hist(ctx->st, p.d_all, nb, (float)(1.0 / T), ctx->d_cm, d_out, ctx->stream);
  CK(hipGetLastError());
  unsigned long long hist[2 * CM_NC];
  CK(hipMemcpyAsync(hist, d_out, sizeof(hist), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  std::vector<double> h(2 * CM_NC);
  for (int k = 0; k < 2 * CM_NC; ++k) h[k] = (double)hist[k];
  rc = allreduce_host_f64(ctx, h.data(), 2 * CM_NC);  // over ranks: every rank picks the same t
  if (rc) return rc;
  // f_k / T = 2^(-k/2) #{r >= 2^(-k/2)} + sum_{r < 2^(-k/2)} r, in bins (bin j >= 1 holds
  // 2^(-j/2) <= r < 2^(-(j-1)/2); its r sum in units of 2^-CM_FIX_LOG2)
  std::vector<double> tail(CM_NC + 1, 0.0);  // tail[k] = sum of r over bins > k
  for (int k = CM_NC - 1; k >= 1; --k) tail[k - 1] = tail[k] + std::ldexp(h[CM_NC + k], -CM_FIX_LOG2);
  double total = 0.0;
  for (int k = 0; k < CM_NC; ++k) total += h[k];
  double cnt = 0.0;
  int kst = -1;
  if (h[0] > 0.0 || tail[0] > 1.0) {
    kst = CM_NC - 1;
    for (int k = 0; k < CM_NC; ++k) {
      cnt += h[k];
      if (k >= 1 && std::pow(2.0, -0.5 * k) * cnt + tail[k] <= 1.0) {
        kst = k;
        break;
      }
    }
  }
  if (kst < 0) {  // the common mode is already below tau: steps unchanged
    launch_cm_apply(ctx->st, p.d_all, nb, p.max_p, INFINITY, ctx->d_cm_scale, ctx->stream);  // factors 1
    CK(hipGetLastError());
    ctx->cm_have_scale = true;
    ctx->cm_info[0] = INFINITY;
    ctx->cm_info[1] = ctx->cm_info[2] = tail[0] * ctx->cm_tau * ctx->cm_tau;
    ctx->cm_info[3] = 0.0;
    return BANN_OK;
  }
  double scaled = 0.0;
  for (int k = 0; k <= kst; ++k) scaled += h[k];
  const double t = std::sqrt(T * std::pow(2.0, -0.5 * kst));
  launch_cm_apply(ctx->st, p.d_all, nb, p.max_p, (float)t, ctx->d_cm_scale, ctx->stream);
  CK(hipGetLastError());
  ctx->cm_have_scale = true;
  ctx->cm_info[0] = t;
  ctx->cm_info[1] = h[0] > 0.0 ? INFINITY : tail[0] * ctx->cm_tau * ctx->cm_tau;  // (omega eps)^2 of the mode
  ctx->cm_info[2] = (std::pow(2.0, -0.5 * kst) * scaled + tail[kst]) * ctx->cm_tau * ctx->cm_tau;
  ctx->cm_info[3] = total > 0.0 ? scaled / total : 0.0;
  return BANN_OK;
}
}  // namespace

extern "C" int bann_network_hmc_step(bann_ctx* ctx, const float* y, float bias, float lambda_e, int32_t L,
                                     float max_dh, int32_t step_mode, float factor, const float* eps,
                                     const float* momentum, uint64_t seed, const float* u, int32_t* status_out,
                                     double* h_trace_out, double* rss_out) {
  if (!ctx || !ctx->finalized) return fail(ctx, BANN_E_STATE, "not finalized");
  if (!y || L < 1) return fail(ctx, BANN_E_ARG, "null targets or L < 1");
  if (ctx->lf_active) return fail(ctx, BANN_E_STATE, "a leapfrog session is active");
  if (step_mode != BANN_STEP_IZMAILOV && step_mode != BANN_STEP_UNIFORM && step_mode != BANN_STEP_STD_SCALED &&
      step_mode != BANN_STEP_INJECTED)
    return fail(ctx, BANN_E_ARG, "network mode: Izmailov, uniform, StdScaled or injected step sizes");
  const int64_t n = ctx->n;
  const int32_t nb = (int32_t)ctx->br.size();
  {
    int rc0 = net_buffers_init(ctx);  // allocated at bann_finalize: a no-op here
    if (rc0) return rc0;
  }
  if (ctx->netrss_cap < L + 1) {
    dfree(ctx->d_netrss);
    ctx->d_netrss = nullptr;
    CK(dalloc(&ctx->d_netrss, L + 1));
    ctx->netrss_cap = L + 1;
  }
  std::vector<int32_t> all(nb);
  for (int b = 0; b < nb; ++b) all[b] = b;
  // every local branch, packed (the persistent plan of the leapfrog sessions is reused)
  if (!(ctx->lf.owns && ctx->lf.all == all)) {
    int rc = build_plan(ctx, all.data(), nb, ctx->lf, true);
    if (rc) return rc;
  }
  if (!ctx->lf.nsum_built) {
    int rc0 = build_net_groups(ctx, ctx->lf);
    if (rc0) return rc0;
  }
  const Plan& p = ctx->lf;
  int rc = traj_prepare(ctx, p, L, max_dh, step_mode, factor, eps, momentum, seed, nullptr);
  if (rc) return rc;
  CK(hipMemcpyAsync(ctx->d_nety, y, n * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
  ctx->st.netmode = 1;
  ctx->st.net_le = lambda_e;
  // fx-only plans: the gradient kernel reads e itself (DevState::nete), no per-branch targets
  bool fx_only = p.gx.empty();
  for (const auto& g : p.groups) fx_only = fx_only && g.kind == 1;
  if (const char* e = getenv("BANN_NET_ERR"))  // 0: per-branch targets for every kind (diagnostics)
    fx_only = fx_only && atoi(e) != 0;
  ctx->st.nete = fx_only ? ctx->d_netsum : nullptr;
  // group sums (k_forward_gsum): every step's forward but the last writes one row per group of
  // four branches instead of every branch's outputs -- the step needs only their sum, and the
  // per-gradient kernels read e (fx_only).  Step 0 too when every prediction row is already
  // f_b(theta_0) (the snapshot into pred0 below copies them); the last step's forward writes
  // the per-branch rows the final targets and the residual need.
  const bool gsum = fx_only && p.nsum_rows > 0;
  bool rows_current = true;
  for (int32_t b : p.all) rows_current = rows_current && ctx->pred_ok[b];
  // f_b at the current theta -> sum over branches and ranks -> e -> targets y_b = f_b - e -> gradients
  // (launch timing, when enabled: forward, all-reduce, gradient and update spans)
  auto forward_and_targets = [&](int k) -> int {
    tm_mark_follow(ctx, TM_FWD0);  // the previous step's update end
    const bool grp = gsum && k < L && (k > 0 || rows_current);
    if (grp) {
      run_forward_gsum(ctx, p);
      CK(hipGetLastError());
    } else {
      int r = run_forward(ctx, p);  // forward-only: the outputs the all-reduce needs
      if (r) return r;
    }
    tm_mark(ctx, TM_FWD1);
    if (grp)
      launch_net_sum_rows(ctx->st, ctx->d_gsum, p.nsum_rows, ctx->d_netsum, ctx->d_delta_part, ctx->stream);
    else
      launch_net_sum(ctx->st, p.d_all, nb, ctx->d_netsum, ctx->d_delta_part, ctx->stream);
    tm_mark(ctx, TM_AR0);
    int r = allreduce_device_f32(ctx, ctx->d_netsum, n);
    if (r) return r;
    tm_mark(ctx, TM_AR1);
    launch_net_targets(ctx->st, p.d_all, fx_only ? 0 : nb, ctx->d_netsum, ctx->d_nety, bias, ctx->d_netpart,
                       ctx->d_netrss + k, ctx->stream);
    tm_mark(ctx, TM_GRAD0);
    r = run_grad(ctx, p, 0);
    tm_mark(ctx, TM_GRAD1);
    return r;
  };
  if (ctx->cm_rule && step_mode != BANN_STEP_INJECTED && lambda_e > 0.f) {
    rc = common_mode_steps(ctx, p, fx_only, lambda_e);
    if (rc) {
      ctx->st.netmode = 0;
      ctx->st.nete = nullptr;
      return rc;
    }
  }
  rc = forward_and_targets(0);
  if (!rc) {
    launch_snapshot_pred(ctx->st, p.d_all, nb, ctx->stream);
    run_update(ctx, p, MODE_INIT, 0);
    tm_mark(ctx, TM_UPD1);
    for (int k = 1; k <= L && !rc; ++k) {
      rc = forward_and_targets(k);
      if (!rc) run_update(ctx, p, k < L ? MODE_STEP : MODE_LAST, k);
      tm_mark(ctx, TM_UPD1);
    }
  }
  ctx->st.netmode = 0;
  ctx->st.nete = nullptr;
  if (rc) {
    ctx->tm_marks.clear();
    return rc;
  }
  CK(hipGetLastError());
  // network -H per step: sum over local branches (list order) and ranks, plus the rss term once.
  // The Metropolis uniform rides along as entry L + 1: rank 0's draw (or the
  // injected u), zero elsewhere, so every rank decides with the same u.
  std::vector<double> tr((size_t)nb * ctx->htrace_cap), rss(L + 1), H(L + 2, 0.0);
  CK(hipMemcpyAsync(tr.data(), ctx->d_htrace, tr.size() * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipMemcpyAsync(rss.data(), ctx->d_netrss, (L + 1) * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  rc = tm_resolve(ctx);
  if (rc) return rc;
  for (int k = 0; k <= L; ++k)
    for (int b = 0; b < nb; ++b) H[k] += tr[(size_t)b * ctx->htrace_cap + k];
  if (ctx->rank == 0) {
    if (u) {
      H[L + 1] = (double)*u;
    } else {  // accept_or_reject_hmc_state's ThreadRng draw (branch_sampler.rs:546-548), from the seed
      std::mt19937_64 g(seed ^ 0x9E3779B97F4A7C15ull);
      H[L + 1] = std::uniform_real_distribution<double>(0.0, 1.0)(g);
    }
  }
  rc = allreduce_host_f64(ctx, H.data(), L + 2);
  if (rc) return rc;
  const double u_net = H[L + 1];
  for (int k = 0; k <= L; ++k) H[k] -= (double)lambda_e * rss[k] / 2.0;  // log_density_wrt_rss (100-102), once
  int status = BANN_ACCEPTED;
  for (int k = 1; k <= L; ++k)
    if (fabs(H[k] - H[0]) > (double)max_dh) {  // early rejection (1264-1279)
      status = BANN_REJECTED_EARLY;
      break;
    }
  if (status == BANN_ACCEPTED) {  // one Metropolis decision for the network (928-962)
    const double log_acc = H[L] - H[0];
    const double acc_p = log_acc >= 0.0 ? 1.0 : exp(log_acc);
    status = u_net < acc_p ? BANN_ACCEPTED : BANN_REJECTED;
  }
  std::vector<int32_t> st(nb, status);
  CK(hipMemcpyAsync(ctx->d_status, st.data(), nb * sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream));
  if (status != BANN_ACCEPTED) {  // every local branch back to theta_0, predictions to f(theta_0)
    run_update(ctx, p, MODE_RESTORE, 0);
    launch_restore_pred(ctx->st, p.d_all, nb, ctx->stream);
    // e at theta_0 (the step-L error of the netsum buffer belongs to theta_L): the
    // restored outputs summed over branches and ranks, no genotype pass
    launch_net_sum(ctx->st, p.d_all, nb, ctx->d_netsum, ctx->d_delta_part, ctx->stream);
    rc = allreduce_device_f32(ctx, ctx->d_netsum, n);
    if (rc) return rc;
    launch_net_targets(ctx->st, p.d_all, 0, ctx->d_netsum, ctx->d_nety, bias, ctx->d_netpart, ctx->d_netrss + L,
                       ctx->stream);
  }
  // the final state's Gibbs targets and residual: y_b = f_b - e = y - bias - sum_{c != b} f_c
  // for every local branch (net.rs:279-280) and the context's device residual
  // y - bias - sum_b f_b = -e, so a branch sampler or bann_rebuild_targets that follows sees
  // the network where this trajectory left it
  launch_net_targets(ctx->st, p.d_all, nb, ctx->d_netsum, nullptr, 0.f, nullptr, nullptr, ctx->stream);
  {
    float* res = nullptr;
    rc = bann_residual_device(ctx, &res);
    if (rc) return rc;
    CK(hipMemsetAsync(res, 0, n * sizeof(float), ctx->stream));
    launch_residual_sub(res, ctx->d_netsum, n, ctx->stream);
  }
  mark_predictions(ctx, p, true);
  CK(hipGetLastError());
  double rss_final = rss[L];
  if (status != BANN_ACCEPTED)  // theta_0's rss, recomputed into d_netrss[L] after the restore above
    CK(hipMemcpyAsync(&rss_final, ctx->d_netrss + L, sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  if (status_out) *status_out = status;
  if (h_trace_out) std::copy(H.begin(), H.begin() + L + 1, h_trace_out);  // H[L + 1] is the shared uniform
  if (rss_out) *rss_out = rss_final;
  return BANN_OK;
}
