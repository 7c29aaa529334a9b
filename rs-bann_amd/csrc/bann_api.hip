// bann_api.hip — C ABI of include/bann.h: context, genotype ingestion, branch
// registry, per-branch BranchSampler math, and the packed HMC driver.
//
// Host-side counterpart of the reference's per-branch orchestration:
//   B::from_cfg / to_cfg          branch_struct.rs:12-29, branch_sampler.rs:155-171
//   hmc_step                       branch_sampler.rs:1192-1299
//   izmailov / uniform / random step sizes (ridge_ard.rs:70-117, ...)
// The device work is in kernels_{data,grad,update}.hip.
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "ctx_internal.h"

#define BANN_VERSION "rs-bann_amd 0.1.0 (gfx950, HIP)"

void comm_destroy(bann_ctx* ctx);  // bann_dist.hip

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------
void free_plan(Plan& p) {
  if (p.owns) {
    dfree(p.d_all);
    dfree(p.d_gx);
    dfree(p.d_gxpre);
    dfree(p.d_fold);
    for (auto& g : p.groups) {
      dfree(g.d_items);
      dfree(g.d_nitems);
      dfree(g.d_nlist);
    }
  }
  p = Plan{};
}

void clear_graphs(bann_ctx* ctx);

void refresh_state(bann_ctx* ctx) {
  clear_graphs(ctx);  // captured kernel arguments hold the old state
  DevState& s = ctx->st;
  s.br = ctx->d_br;
  s.xu2 = ctx->d_xu2;
  s.xi = ctx->d_xi;
  s.dig = ctx->d_dig;
  s.fc = ctx->d_fc;
  s.mu = ctx->d_mub;
  s.sigma = ctx->d_sigb;
  s.theta = ctx->d_theta;
  s.mom = ctx->d_mom;
  s.eps = ctx->d_eps;
  s.theta0 = ctx->d_theta0;
  s.lam = ctx->d_lam;
  s.lamld = ctx->d_lamld;
  s.grad = ctx->d_grad;
  s.part = ctx->d_part;
  s.rss_part = ctx->d_rss_part;
  s.y = ctx->d_y;
  s.pred = ctx->d_pred;
  s.pred0 = ctx->d_pred0;
  s.scr = ctx->d_scr;
  s.dbg = ctx->d_dbg;
  s.eprec = ctx->d_eprec;
  s.h0 = ctx->d_h0;
  s.htrace = ctx->d_htrace;
  s.ld_out = ctx->d_ld;
  s.rss_out = ctx->d_rss;
  s.status = ctx->d_status;
  s.uturn = ctx->d_uturn;
  s.uacc = ctx->d_u;
  s.n = ctx->n;
  s.nfrag = ctx->nfrag;
  s.max_splits = ctx->max_splits;
  s.lint = ctx->htrace_cap - 1;
  s.phi = ctx->d_phi;
  s.phi0 = ctx->d_phi0;
  s.mphi = ctx->d_mphi;
  s.ephi = ctx->d_ephi;
  s.gphi = ctx->d_gphi;
  s.pidx = ctx->d_pidx;
  s.ows = ctx->d_ows;
}

bool check_branch(const bann_ctx* ctx, int32_t b) {
  return ctx && ctx->finalized && b >= 0 && b < (int32_t)ctx->br.size();
}

// expanded per-parameter precision multipliers and the error precision
static void expand_precisions(const BranchHost& h, std::vector<float>& lam, std::vector<float>& lamld,
                              float& eprec) {
  const BranchDev& d = h.dev;
  lam.assign(h.P, 0.f);
  lamld.assign(h.P, 0.f);
  const bool ard = (h.prior == BANN_RIDGE_ARD || h.prior == BANN_LASSO_ARD);
  int pi = 0;
  for (int l = 0; l < h.L; ++l) {
    const int wi = d.win[l], wo = d.widths[l];
    for (int k = 0; k < wo; ++k)
      for (int j = 0; j < wi; ++j) {
        float v;
        if (h.prior == BANN_STD_NORMAL)
          v = 1.f;
        else if (ard && l < h.L - 1)
          v = h.prec[pi + j];
        else
          v = h.prec[pi];
        lam[d.woff[l] + k * wi + j] = v;
        lamld[d.woff[l] + k * wi + j] = v;
      }
    pi += (ard && l < h.L - 1) ? wi : 1;
  }
  if (h.prior == BANN_STD_NORMAL)  // std_normal_branch.rs:149-158: l2 bias term in log_density only
    for (int l = 0; l < h.L - 1; ++l)
      for (int k = 0; k < d.widths[l]; ++k) lamld[d.boff[l] + k] = 1.f;
  eprec = h.prec.back();
}

// random step sizes (branch_sampler.rs:654-681): U(0,1) * P^(-1/4) * c, drawn on
// the host; uniform (706-732) and Izmailov (ridge_ard.rs:70-117, ridge_base.rs:
// 83-114, lasso_ard.rs:77-117, lasso_base.rs:83-114, std_normal_branch.rs:83-114)
// are formed on the device from step_bases below.
static void host_random_step_sizes(const BranchHost& h, float c, std::mt19937_64& rng, std::vector<float>& eps) {
  eps.assign(h.P, c);
  std::uniform_real_distribution<float> U(0.f, 1.f);
  const float f = powf((float)h.P, -0.25f) * c;
  for (auto& e : eps) e = U(rng) * f;
}

// StdScaled step sizes (dispatched at branch_sampler.rs:1213) for the Base priors:
// ridge_base.rs:52-82, lasso_base.rs:53-82, std_normal_branch.rs:51-80 -- in f32 as the
// reference: weights c * (1 / lambda_l).sqrt() (host scalar), biases
// c * (1 / sqrt(lambda_b)) (the lasso form 1 * c * (1 / sqrt) rounds identically).
// The ARD priors return empty vectors (ridge_ard.rs:56-68, lasso_ard.rs:62-74): refused.
static bool host_std_scaled_step_sizes(const BranchHost& h, float c, std::vector<float>& eps) {
  if (h.prior == BANN_RIDGE_ARD || h.prior == BANN_LASSO_ARD) return false;
  const BranchDev& d = h.dev;
  eps.assign(h.P, 0.f);
  for (int l = 0; l < h.L; ++l) {
    const volatile float inv = 1.f / h.prec[l];
    const float e = c * sqrtf(inv);
    const int cnt = d.win[l] * d.widths[l];
    for (int k = 0; k < cnt; ++k) eps[d.woff[l] + k] = e;
  }
  for (int l = 0; l < h.L - 1; ++l) {
    const volatile float rs = 1.f / sqrtf(h.prec[h.L + l]);
    const float e = c * rs;
    for (int k = 0; k < d.widths[l]; ++k) eps[d.boff[l] + k] = e;
  }
  return true;
}

// per-parameter Izmailov step base, so the device can form eps = base * c / L
// for any factor c and trajectory length L without a host round trip:
// ridge / bias terms pi / (2 sqrt(lam)), lasso 1 / (4 lam); negative = the
// factor c does not apply (std_normal weights and biases).  eps = base * c / L
// reproduces the reference's c * pi / (2 sqrt(lam) L) and c / (4 lam L).
static void step_bases(const BranchHost& h, std::vector<double>& out) {
  const BranchDev& d = h.dev;
  out.assign(h.P, 0.0);
  const bool ard = (h.prior == BANN_RIDGE_ARD || h.prior == BANN_LASSO_ARD);
  const bool lasso = (h.prior == BANN_LASSO_ARD || h.prior == BANN_LASSO_BASE);
  const bool stdn = h.prior == BANN_STD_NORMAL;
  const double PI = 3.14159265358979323846;
  int pi = 0;
  for (int l = 0; l < h.L; ++l) {
    const int wi = d.win[l], wo = d.widths[l];
    for (int k = 0; k < wo; ++k)
      for (int j = 0; j < wi; ++j) {
        const double lam = (ard && l < h.L - 1) ? h.prec[pi + j] : h.prec[pi];
        double e;
        if (stdn)
          e = -PI / (2.0 * sqrt(lam));
        else if (lasso)
          e = 1.0 / (4.0 * lam);
        else
          e = PI / (2.0 * sqrt(lam));
        out[d.woff[l] + k * wi + j] = e;
      }
    pi += (ard && l < h.L - 1) ? wi : 1;
  }
  for (int l = 0; l < h.L - 1; ++l) {
    const double lb = h.prec[pi + l];
    const double e = PI / (2.0 * sqrt(lb));
    for (int k = 0; k < d.widths[l]; ++k) out[d.boff[l] + k] = stdn ? -e : e;
  }
}

int build_plan(bann_ctx* ctx, const int32_t* branches, int32_t nb, Plan& p, bool persistent) {
  free_plan(p);
  const int32_t nbr = (int32_t)ctx->br.size();
  if (nb > nbr) return fail(ctx, BANN_E_ARG, "branch list longer than the branch set");
  std::vector<char> seen(nbr, 0);
  for (int i = 0; i < nb; ++i) {
    const int b = branches[i];
    if (b < 0 || b >= nbr) return fail(ctx, BANN_E_SHAPE, "branch index out of range");
    if (seen[b]) return fail(ctx, BANN_E_ARG, "duplicate branch in list");
    seen[b] = 1;
  }
  p.all.assign(branches, branches + nb);
  std::vector<int32_t> lists(p.all);
  for (int i = 0; i < nb; ++i)
    if (!update_is_large(ctx->br[branches[i]].dev)) lists.push_back(branches[i]);
  p.n_small = (int32_t)lists.size() - nb;
  for (int i = 0; i < nb; ++i)
    if (update_is_large(ctx->br[branches[i]].dev)) lists.push_back(branches[i]);
  p.n_large = nb - p.n_small;
  const int64_t nfrag = ctx->nfrag, ntile = (nfrag + BANN_TILE_FRAGS - 1) / BANN_TILE_FRAGS;
  // solo mode: too few work items to fill the GPU -> every fused branch re-split
  // into its solo_items items, partials into the solo region, folded afterwards
  bool solo = false;
  {
    int64_t items = 0, need = 0, need_rss = 0;
    for (int i = 0; i < nb; ++i) {
      const BranchHost& h = ctx->br[branches[i]];
      if (!h.dev.fused) continue;
      items += h.dev.nsplits;
      need += (int64_t)h.solo_items * h.P;
      need_rss += h.solo_items;
    }
    solo = items > 0 && items < ctx->solo_threshold && need <= ctx->solo_part_cap && need_rss <= ctx->solo_rss_cap;
  }
  int64_t solo_part = ctx->part_total, solo_rss = (int64_t)nbr * ctx->max_splits;
  for (int i = 0; i < nb; ++i) {
    const int b = branches[i];
    const BranchHost& h = ctx->br[b];
    const BranchDev& d = h.dev;
    p.max_p = std::max(p.max_p, h.P);
    if (!d.fused) {
      p.gx.push_back(b);
      continue;
    }
    LaunchGroup key;
    key.kind = d.fused;
    key.act = h.act;
    if (d.fused == 1) {  // fx: (L, act, exactly 8 chunks)
      key.L = h.L;
      key.full = d.nchunks == 8;
    } else if (d.fused == 3) {  // fxl: (L, act, chunks per wave, waves, every wave full)
      key.L = h.L;
      key.cpw = fxl_cpw(d.nchunks);
      key.nw = (d.nchunks + key.cpw - 1) / key.cpw;
      key.head = ctx->fxl_head ? 1 : 0;
      key.full = d.nchunks == key.cpw * key.nw;
    } else if (d.fused == 2) {  // wx: (act, marker chunks: the plane kernel is compiled per chunk count)
      key.nw = d.nchunks;
    }
    LaunchGroup* grp = nullptr;
    for (auto& g : p.groups)
      if (g.kind == key.kind && g.L == key.L && g.act == key.act && g.nw == key.nw && g.full == key.full &&
          g.cpw == key.cpw)
        grp = &g;
    if (!grp) {
      p.groups.push_back(key);
      grp = &p.groups.back();
    }
    const int spi = 1;  // partial slabs per work item
    const int ns = solo ? h.solo_items : d.nsplits;
    if (grp->items.empty()) grp->fi = true;
    if (d.fused == 1) {
      grp->fi = grp->fi && d.xi_off >= 0;
      grp->max_seg = std::max(grp->max_seg, (d.nchunks + 3) / 4);
    }
    for (int s = 0; s < ns; ++s) {  // splits on tile (4-fragment) boundaries
      GradItem it{};
      it.branch = b;
      it.split = s;
      it.frag_begin = (int32_t)(BANN_TILE_FRAGS * (ntile * s / ns));
      it.frag_end = (int32_t)std::min<int64_t>(nfrag, BANN_TILE_FRAGS * (ntile * (s + 1) / ns));
      it.tile0 = (int32_t)grp->tiles;
      grp->tiles += ((it.frag_end + 3) >> 2) - (it.frag_begin >> 2);
      it.part_at = solo ? solo_part + (int64_t)s * spi * h.P : d.part_off + (int64_t)s * spi * h.P;
      it.rss_at = solo ? solo_rss + (int64_t)s * spi : (int64_t)b * ctx->max_splits + (int64_t)s * spi;
      it.fold_ix = solo ? (int32_t)p.fold.size() : -1;  // this branch's job, pushed below
      grp->items.push_back(it);
    }
    if (solo) {
      p.fold.push_back(FoldJob{b, ns * spi, solo_part, solo_rss});
      solo_part += (int64_t)ns * spi * h.P;
      solo_rss += (int64_t)ns * spi;
    }
  }
  {  // the fused update (kernels_fx.hip tail): fx branches only, the small update, one round of items
    int64_t items = 0;
    bool ok = p.gx.empty() && ctx->d_upd_cnt != nullptr && ctx->fuse_update_mode > 0;
    bool single = true;  // every branch one split: its one workgroup updates it
    for (const auto& g : p.groups) {
      ok = ok && g.kind == 1;
      items += (int64_t)g.items.size();
    }
    for (int i = 0; i < nb && ok; ++i) {
      const BranchHost& h = ctx->br[branches[i]];
      ok = h.P <= 2048 && h.m <= 512 && !update_is_large(h.dev);
      single = single && h.dev.nsplits == 1;
    }
    // solo plans: the last arriving workgroup folds the branch's slabs, then updates it
    p.fuse_update = ok && items > 0 && (solo || single || items <= 2ll * ctx->cus);
  }
  // gx branches: grouped by scratch group, one tile prefix array per GEMM phase
  std::stable_sort(p.gx.begin(), p.gx.end(),
                   [&](int32_t a, int32_t b) { return ctx->br[a].gx_group < ctx->br[b].gx_group; });
  for (size_t i = 0; i < p.gx.size();) {
    size_t j = i;
    GxGroup g;
    int32_t maxL = 2;
    while (j < p.gx.size() && ctx->br[p.gx[j]].gx_group == ctx->br[p.gx[i]].gx_group) {
      maxL = std::max(maxL, ctx->br[p.gx[j]].L);
      g.max_splits = std::max(g.max_splits, ctx->br[p.gx[j]].dev.nsplits);
      ++j;
    }
    g.first = (int32_t)i;
    g.count = (int32_t)(j - i);
    std::vector<std::pair<int, int>> order;  // (phase, layer) in launch order
    order.push_back({GX_FWD0, 0});
    for (int l = 1; l < maxL - 1; ++l) order.push_back({GX_FWD, l});
    order.push_back({GX_HEAD, 0});
    for (int l = maxL - 2; l >= 1; --l) order.push_back({GX_BWD, l});
    for (int l = maxL - 2; l >= 1; --l) order.push_back({GX_GRAD, l});
    order.push_back({GX_GRAD0, 0});
    for (auto& o : order) {
      GxPhase ph;
      ph.ph = o.first;
      ph.l = o.second;
      if (ph.ph != GX_HEAD) {
        ph.pre_off = (int32_t)p.gx_pre.size();
        int64_t tot = 0;
        p.gx_pre.push_back(0);
        for (size_t k = i; k < j; ++k) {
          tot += gx_tiles(ctx->br[p.gx[k]].dev, ph.ph, ph.l, ctx->nfrag);
          if (tot >= (1ll << 30)) return fail(ctx, BANN_E_SHAPE, "gx phase has too many tiles for one launch");
          p.gx_pre.push_back((int32_t)tot);
        }
        ph.total = (int32_t)tot;
        if (tot == 0) continue;
      }
      g.phases.push_back(ph);
    }
    p.gxg.push_back(std::move(g));
    i = j;
  }
  if (persistent) {
    p.owns = true;
    CK(dalloc(&p.d_all, 2 * nb));
    CK(dalloc(&p.d_gx, (int64_t)p.gx.size()));
    CK(dalloc(&p.d_gxpre, (int64_t)p.gx_pre.size()));
    CK(dalloc(&p.d_fold, (int64_t)p.fold.size()));
    if (!p.fold.empty())
      CK(hipMemcpyAsync(p.d_fold, p.fold.data(), p.fold.size() * sizeof(FoldJob), hipMemcpyHostToDevice,
                        ctx->stream));
    CK(hipMemcpyAsync(p.d_all, lists.data(), 2 * nb * sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream));
    if (!p.gx.empty()) {
      CK(hipMemcpyAsync(p.d_gx, p.gx.data(), p.gx.size() * sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream));
      CK(hipMemcpyAsync(p.d_gxpre, p.gx_pre.data(), p.gx_pre.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                        ctx->stream));
    }
    for (auto& g : p.groups) {
      CK(dalloc(&g.d_items, (int64_t)g.items.size()));
      CK(hipMemcpyAsync(g.d_items, g.items.data(), g.items.size() * sizeof(GradItem), hipMemcpyHostToDevice,
                        ctx->stream));
    }
  } else {
    p.owns = false;
    p.d_all = ctx->d_list_scr;
    p.d_gx = ctx->d_gen_scr;
    p.d_gxpre = ctx->d_gxpre_scr;
    p.d_fold = ctx->d_fold_scr;
    if ((int64_t)p.gx_pre.size() > ctx->gxpre_cap) return fail(ctx, BANN_E_STATE, "gx plan scratch overflow");
    if (ctx->plan_ev_pending) CK(hipEventSynchronize(ctx->ev_plan));  // the last plan's copy has read the stage
    char* hs = ctx->h_plan_stage;
    std::memcpy(hs, lists.data(), 2 * nb * sizeof(int32_t));
    int64_t end = 2 * (int64_t)nb * (int64_t)sizeof(int32_t);
    if (!p.fold.empty()) {
      std::memcpy(hs + ctx->plan_off_fold, p.fold.data(), p.fold.size() * sizeof(FoldJob));
      end = ctx->plan_off_fold + (int64_t)(p.fold.size() * sizeof(FoldJob));
    }
    if (!p.gx.empty()) {
      CK(hipMemcpyAsync(p.d_gx, p.gx.data(), p.gx.size() * sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream));
      CK(hipMemcpyAsync(p.d_gxpre, p.gx_pre.data(), p.gx_pre.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                        ctx->stream));
    }
    int64_t off = 0;
    for (auto& g : p.groups) {
      if (off + (int64_t)g.items.size() > ctx->items_cap) return fail(ctx, BANN_E_STATE, "work-item scratch overflow");
      g.d_items = ctx->d_items_scr + off;
      std::memcpy(hs + ctx->plan_off_items + off * (int64_t)sizeof(GradItem), g.items.data(),
                  g.items.size() * sizeof(GradItem));
      off += (int64_t)g.items.size();
    }
    if (off > 0) end = ctx->plan_off_items + off * (int64_t)sizeof(GradItem);
    CK(hipMemcpyAsync(ctx->d_plan_scr, hs, (size_t)end, hipMemcpyHostToDevice, ctx->stream));
    CK(hipEventRecord(ctx->ev_plan, ctx->stream));
    ctx->plan_ev_pending = true;
  }
  return BANN_OK;
}

// gradient (partials) of every branch in the plan at the current theta.
// write_pred: 0 = no predictions (the layered path writes them anyway), 1 = the
// predictions f_b(theta) into pred, 2 = into pred0 (a trajectory's start: the
// restore copy and the residual change read them there)
// upd_mode >= 0 (a plan with fuse_update): the leapfrog update of that mode and
// step runs in the fx launch's tail -- the caller launches no update (run_grad_update)
int run_grad(bann_ctx* ctx, const Plan& p, int write_pred, int upd_mode, int upd_step) {
  DevState s = ctx->st;
  if (write_pred == 2) s.pred = ctx->d_pred0;
  const int wp = write_pred != 0;
  int32_t* cnt = upd_mode >= 0 ? ctx->d_upd_cnt : nullptr;
  // a fused solo plan folds in the gradient launch's tail (kernels_fx.hip), not in k_fold_solo
  const FoldJob* fo = (cnt && !p.fold.empty()) ? p.d_fold : nullptr;
  for (const auto& g : p.groups) {
    const int32_t ni = (int32_t)g.items.size();
    if (g.kind == 2)
      launch_fused_grad_wx(s, g.d_items, ni, g.act, ctx->wide_bf16 ? 1 : (wx_exact() ? 0 : 2), g.nw, wp, ctx->stream);
    else if (g.kind == 3)
      launch_fused_grad_fxl(s, g.d_items, ni, g.L, g.act, g.nw, g.cpw, g.full, wp, g.head, ctx->stream);
    else
      launch_fused_grad_fx(s, g.d_items, ni, g.L, g.act, g.full, wp, upd_mode, upd_step, cnt, fo, ctx->stream);
  }
  if (!p.fold.empty() && !fo) launch_fold_solo(s, p.d_fold, (int32_t)p.fold.size(), p.max_p, ctx->stream);
  // gx branches: scratch group by scratch group (the groups reuse one scratch)
  for (const auto& g : p.gxg) {
    const int32_t* bl = p.d_gx + g.first;
    launch_gx_prep(s, bl, g.count, ctx->stream);
    for (const auto& ph : g.phases) {
      if (ph.ph == GX_HEAD)
        launch_gx_head(s, bl, g.count, g.max_splits, ctx->stream);
      else
        launch_gx_gemm(s, ph.ph, ph.l, bl, p.d_gxpre + ph.pre_off, g.count, ph.total, ctx->stream);
    }
  }
  CK(hipGetLastError());
  if (write_pred == 1) mark_predictions(ctx, p, true);
  return BANN_OK;
}

// predictions f_b(theta) of every branch in the plan: fx groups through the
// forward-only kernel (no target, no backward), every other path through its
// gradient launch with predictions (their partial slabs are scratch here)
int run_forward(bann_ctx* ctx, const Plan& p) {
  const DevState& s = ctx->st;
  for (const auto& g : p.groups) {
    const int32_t ni = (int32_t)g.items.size();
    if (g.kind == 2)
      launch_fused_grad_wx(s, g.d_items, ni, g.act, ctx->wide_bf16 ? 1 : (wx_exact() ? 0 : 2), g.nw, 1, ctx->stream);
    else if (g.kind == 3)
      launch_fused_grad_fxl(s, g.d_items, ni, g.L, g.act, g.nw, g.cpw, g.full, 1, g.head, ctx->stream);
    else if (g.fi)
      launch_forward_fi(s, g.d_items, ni, g.tiles, g.L, g.act, g.max_seg, ctx->cus, ctx->stream);
    else
      launch_forward_fx(s, g.d_items, ni, g.L, g.act, g.full, ctx->stream);
  }
  for (const auto& g : p.gxg) {
    const int32_t* bl = p.d_gx + g.first;
    launch_gx_prep(s, bl, g.count, ctx->stream);
    for (const auto& ph : g.phases) {
      if (ph.ph == GX_HEAD) {
        launch_gx_head(s, bl, g.count, g.max_splits, ctx->stream);
        break;  // the head writes the predictions; the backward phases are not needed
      }
      launch_gx_gemm(s, ph.ph, ph.l, bl, p.d_gxpre + ph.pre_off, g.count, ph.total, ctx->stream);
    }
  }
  CK(hipGetLastError());
  mark_predictions(ctx, p, true);
  return BANN_OK;
}

void mark_predictions(bann_ctx* ctx, const Plan& p, bool current) {
  for (int32_t b : p.all) ctx->pred_ok[b] = current;
}

// the fused leapfrog update of every branch in the plan (small and large kernels)
void run_update(bann_ctx* ctx, const Plan& p, int32_t mode, int32_t step) {
  const int32_t nb = (int32_t)p.all.size();
  if (mode != MODE_GRAD && mode != MODE_PROFILE) mark_predictions(ctx, p, false);  // theta moves
  launch_update(ctx->st, p.d_all + nb, p.n_small, mode, step, ctx->stream, 0);
  launch_update(ctx->st, p.d_all + nb + p.n_small, p.n_large, mode, step, ctx->stream, 1);
}

int ensure_htrace(bann_ctx* ctx, int32_t L) {
  if (L + 1 <= ctx->htrace_cap) return BANN_OK;
  const int32_t cap = std::max({L + 1, 2 * ctx->htrace_cap, 129});  // grow geometrically: no realloc per trajectory
  dfree(ctx->d_htrace);
  ctx->d_htrace = nullptr;
  CK(dalloc(&ctx->d_htrace, (int64_t)ctx->br.size() * cap));
  ctx->htrace_cap = cap;
  refresh_state(ctx);
  return BANN_OK;
}

// ---------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------
extern "C" const char* bann_version(void) { return BANN_VERSION; }

extern "C" int bann_ctx_create(int device, bann_ctx** out) {
  if (!out) return BANN_E_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return BANN_E_HIP;
  if (device < 0 || device >= ndev) return BANN_E_ARG;
  bann_ctx* ctx = new bann_ctx();
  ctx->device = device;
  if (const char* e = getenv("BANN_HMC_GRAPH")) ctx->graph_replay = atoi(e) != 0;
  if (const char* e = getenv("BANN_FXL_HEAD")) ctx->fxl_head = atoi(e) != 0;
  if (const char* e = getenv("BANN_NET_GSUM")) ctx->net_gsum = atoi(e) != 0;
  if (const char* e = getenv("BANN_FUSE_UPDATE")) ctx->fuse_update_mode = atoi(e) != 0 ? 1 : 0;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return BANN_E_HIP;
  }
  *out = ctx;
  return BANN_OK;
}

extern "C" int bann_ctx_destroy(bann_ctx* ctx) {
  if (!ctx) return BANN_OK;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  if (ctx->d_dbg) {  // diagnostic build: per-phase cycle sums of the fused kernel
    unsigned long long h[16] = {};
    (void)hipMemcpy(h, ctx->d_dbg, sizeof(h), hipMemcpyDeviceToHost);
    fprintf(stderr, "BANN_STAMPS tiles=%llu cycles/tile:", h[15]);
    for (int i = 0; i < 8; ++i) fprintf(stderr, " p%d=%.0f", i, h[15] ? (double)h[i] / (double)h[15] : 0.0);
    fprintf(stderr, "\n");
    (void)hipFree(ctx->d_dbg);
  }
  free_plan(ctx->lf);
  void* bufs[] = {ctx->d_g, ctx->d_mu, ctx->d_sigma, ctx->d_br, ctx->d_xu2, ctx->d_xi, ctx->d_dig, ctx->d_fc, ctx->d_mub,
                  ctx->d_sigb, ctx->d_theta, ctx->d_mom, ctx->d_eps, ctx->d_theta0, ctx->d_lam, ctx->d_lamld,
                  ctx->d_grad, ctx->d_part, ctx->d_rss_part, ctx->d_y, ctx->d_pred, ctx->d_pred0, ctx->d_scr, ctx->d_eprec,
                  ctx->d_u, ctx->d_h0, ctx->d_htrace, ctx->d_ld, ctx->d_rss, ctx->d_status, ctx->d_uturn,
                  ctx->d_plan_scr, ctx->d_gen_scr, ctx->d_gxpre_scr, ctx->d_delta, ctx->d_delta_part, ctx->d_stepbase,
                  ctx->d_phi, ctx->d_phi0, ctx->d_mphi, ctx->d_ephi, ctx->d_gphi, ctx->d_pidx, ctx->d_ows,
                  ctx->d_netsum, ctx->d_nety, ctx->d_netrss, ctx->d_netpart, ctx->d_ar64, ctx->d_res, ctx->d_upd_cnt,
                  ctx->d_res_part, ctx->d_ones, ctx->d_cm, ctx->d_cm_scale, ctx->d_gsum};
  for (hipEvent_t e : ctx->tm_pool) (void)hipEventDestroy(e);
  clear_graphs(ctx);
  comm_destroy(ctx);
  for (void* p : bufs) dfree(p);
  if (ctx->h_status) (void)hipHostFree(ctx->h_status);
  if (ctx->h_par_stage) (void)hipHostFree(ctx->h_par_stage);
  if (ctx->h_delta) (void)hipHostFree(ctx->h_delta);
  if (ctx->h_res_stat) (void)hipHostFree(ctx->h_res_stat);
  if (ctx->plan_ev_pending && ctx->ev_plan) (void)hipEventSynchronize(ctx->ev_plan);
  if (ctx->u_ev_pending && ctx->ev_u) (void)hipEventSynchronize(ctx->ev_u);
  if (ctx->h_u_stage) (void)hipHostFree(ctx->h_u_stage);
  if (ctx->ev_u) (void)hipEventDestroy(ctx->ev_u);
  if (ctx->h_plan_stage) (void)hipHostFree(ctx->h_plan_stage);
  if (ctx->ev_plan) (void)hipEventDestroy(ctx->ev_plan);
  if (ctx->prec_ev_pending && ctx->ev_prec) (void)hipEventSynchronize(ctx->ev_prec);
  if (ctx->h_prec_stage) (void)hipHostFree(ctx->h_prec_stage);
  if (ctx->d_prec_stage) (void)hipFree(ctx->d_prec_stage);
  if (ctx->ev_prec) (void)hipEventDestroy(ctx->ev_prec);
  (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return BANN_OK;
}

extern "C" const char* bann_last_error(const bann_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

extern "C" int bann_synchronize(bann_ctx* ctx) {
  if (!ctx) return BANN_E_ARG;
  CK(hipStreamSynchronize(ctx->stream));
  return BANN_OK;
}

// ---------------------------------------------------------------------------
// genotypes
// ---------------------------------------------------------------------------
int alloc_genotypes(bann_ctx* ctx, int64_t n, int64_t M) {
  if (ctx->finalized) return fail(ctx, BANN_E_STATE, "genotypes must be set before bann_finalize");
  if (n <= 0 || M <= 0) return fail(ctx, BANN_E_SHAPE, "n and num_markers must be positive");
  CK(hipSetDevice(ctx->device));
  dfree(ctx->d_g);
  dfree(ctx->d_mu);
  dfree(ctx->d_sigma);
  ctx->d_g = nullptr;
  ctx->d_mu = ctx->d_sigma = nullptr;
  ctx->n = n;
  ctx->M = M;
  ctx->rowb = (n + 63) / 64 * 16;
  CK(dalloc(&ctx->d_g, ctx->rowb * M));
  CK(dalloc(&ctx->d_mu, M));
  CK(dalloc(&ctx->d_sigma, M));
  return BANN_OK;
}

// markers per staged block: ~256 MiB of host input per copy
int64_t stage_markers(int64_t bytes_per_marker, int64_t M) {
  return std::max<int64_t>(1, std::min<int64_t>(M, (int64_t(256) << 20) / std::max<int64_t>(1, bytes_per_marker)));
}

extern "C" int bann_genotypes_upload(bann_ctx* ctx, const int8_t* g, int64_t n, int64_t num_markers) {
  if (!ctx || !g) return BANN_E_ARG;
  int rc = alloc_genotypes(ctx, n, num_markers);
  if (rc) return rc;
  // int8 [M][n] streamed through a bounded staging block, packed to 2 bits on the device
  const int64_t blk = stage_markers(n, num_markers);
  int8_t* d_st = nullptr;
  int32_t* d_flag = nullptr;
  int32_t flag = 0;
  CK(dalloc(&d_st, blk * n));
  CK(dalloc(&d_flag, 1));
  CK(hipMemsetAsync(d_flag, 0, sizeof(int32_t), ctx->stream));
  for (int64_t j0 = 0; j0 < num_markers; j0 += blk) {
    const int64_t m = std::min(blk, num_markers - j0);
    CK(hipMemcpyAsync(d_st, g + j0 * n, (size_t)(m * n), hipMemcpyHostToDevice, ctx->stream));
    launch_i8_to_raw(d_st, n, m, ctx->d_g + j0 * ctx->rowb, ctx->rowb, d_flag, ctx->stream);
    CK(hipGetLastError());
  }
  launch_col_stats(ctx->d_g, ctx->rowb, ctx->d_mu, ctx->d_sigma, n, num_markers, ctx->stream);
  CK(hipMemcpyAsync(&flag, d_flag, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  dfree(d_st);
  dfree(d_flag);
  if (flag) return fail(ctx, BANN_E_ARG, "genotypes must be 2-bit codes in 0..3 (.bed semantics)");
  return BANN_OK;
}

extern "C" int bann_genotypes_upload_bed(bann_ctx* ctx, const uint8_t* payload, int64_t n, int64_t num_markers) {
  if (!ctx || !payload) return BANN_E_ARG;
  int rc = alloc_genotypes(ctx, n, num_markers);
  if (rc) return rc;
  // payload rows streamed through a bounded staging block, decoded into the 2-bit image
  const int64_t bpc = (n + 3) / 4;
  const int64_t blk = stage_markers(bpc, num_markers);
  uint8_t* d_st = nullptr;
  CK(dalloc(&d_st, blk * bpc));
  for (int64_t j0 = 0; j0 < num_markers; j0 += blk) {
    const int64_t m = std::min(blk, num_markers - j0);
    CK(hipMemcpyAsync(d_st, payload + j0 * bpc, (size_t)(m * bpc), hipMemcpyHostToDevice, ctx->stream));
    launch_bed_to_raw(d_st, n, m, ctx->d_g + j0 * ctx->rowb, ctx->rowb, ctx->stream);
    CK(hipGetLastError());
  }
  launch_col_stats(ctx->d_g, ctx->rowb, ctx->d_mu, ctx->d_sigma, n, num_markers, ctx->stream);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(ctx->stream));
  dfree(d_st);
  return BANN_OK;
}

extern "C" int bann_genotypes_synthetic(bann_ctx* ctx, int64_t n, int64_t num_markers, uint64_t seed) {
  if (!ctx) return BANN_E_ARG;
  int rc = alloc_genotypes(ctx, n, num_markers);
  if (rc) return rc;
  launch_synthetic_genotypes(ctx->d_g, ctx->rowb, ctx->d_mu, ctx->d_sigma, n, num_markers, seed, ctx->stream);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(ctx->stream));
  return BANN_OK;
}

extern "C" int bann_genotypes_stats(bann_ctx* ctx, float* mu, float* sigma) {
  if (!ctx || !ctx->d_mu) return fail(ctx, BANN_E_STATE, "no genotypes");
  if (mu) CK(hipMemcpy(mu, ctx->d_mu, ctx->M * sizeof(float), hipMemcpyDeviceToHost));
  if (sigma) CK(hipMemcpy(sigma, ctx->d_sigma, ctx->M * sizeof(float), hipMemcpyDeviceToHost));
  return BANN_OK;
}

extern "C" int bann_genotypes_set_stats(bann_ctx* ctx, const float* mu, const float* sigma) {
  if (!ctx || !mu || !sigma) return BANN_E_ARG;
  if (!ctx->d_mu) return fail(ctx, BANN_E_STATE, "no genotypes");
  if (ctx->finalized) return fail(ctx, BANN_E_STATE, "statistics are folded at bann_finalize; set them before");
  CK(hipMemcpy(ctx->d_mu, mu, ctx->M * sizeof(float), hipMemcpyHostToDevice));
  CK(hipMemcpy(ctx->d_sigma, sigma, ctx->M * sizeof(float), hipMemcpyHostToDevice));
  return BANN_OK;
}

extern "C" int bann_genotypes_download(bann_ctx* ctx, const int32_t* snp_idx, int32_t m, int8_t* g_out) {
  if (!ctx || !snp_idx || !g_out || m <= 0) return BANN_E_ARG;
  if (!ctx->d_g) return fail(ctx, BANN_E_STATE, "raw genotypes not resident (freed at finalize?)");
  for (int i = 0; i < m; ++i)
    if (snp_idx[i] < 0 || snp_idx[i] >= ctx->M) return fail(ctx, BANN_E_SHAPE, "marker index out of range");
  int32_t* d_idx = nullptr;
  int8_t* d_out = nullptr;
  CK(dalloc(&d_idx, m));
  CK(dalloc(&d_out, (int64_t)m * ctx->n));
  CK(hipMemcpyAsync(d_idx, snp_idx, m * sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream));
  launch_unpack_markers(ctx->d_g, ctx->rowb, d_idx, m, ctx->n, d_out, ctx->stream);
  CK(hipMemcpyAsync(g_out, d_out, (size_t)m * ctx->n, hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  dfree(d_idx);
  dfree(d_out);
  return BANN_OK;
}

// ---------------------------------------------------------------------------
// branches
// ---------------------------------------------------------------------------
extern "C" int bann_branch_add(bann_ctx* ctx, const int32_t* snp_idx, int32_t m, const int32_t* layer_widths,
                               int32_t num_layers, int32_t activation, int32_t prior) {
  if (!ctx || !snp_idx || !layer_widths) return BANN_E_ARG;
  if (ctx->finalized) return fail(ctx, BANN_E_STATE, "branch set is fixed after bann_finalize");
  if (m <= 0) return fail(ctx, BANN_E_SHAPE, "a branch needs at least one marker");
  if (num_layers < 2 || num_layers > BANN_MAXL)
    return fail(ctx, BANN_E_SHAPE, "num_layers must be in [2, 8] (summary + output at least)");
  if (layer_widths[num_layers - 1] != 1) return fail(ctx, BANN_E_SHAPE, "output layer width must be 1");
  if (activation < 0 || activation > 4) return fail(ctx, BANN_E_ARG, "unknown activation");
  if (prior < 0 || prior > 4) return fail(ctx, BANN_E_ARG, "unknown prior");
  BranchHost h;
  h.snp_idx.assign(snp_idx, snp_idx + m);
  h.widths.assign(layer_widths, layer_widths + num_layers);
  for (int l = 0; l < num_layers; ++l)
    if (h.widths[l] <= 0) return fail(ctx, BANN_E_SHAPE, "layer widths must be positive");
  for (int i = 0; i < m; ++i)
    if (snp_idx[i] < 0 || (ctx->M > 0 && snp_idx[i] >= ctx->M))
      return fail(ctx, BANN_E_SHAPE, "marker index out of range");
  h.m = m;
  h.L = num_layers;
  h.act = activation;
  h.prior = prior;
  BranchDev& d = h.dev;
  d.m = m;
  d.L = num_layers;
  d.act = activation;
  d.prior = prior;
  int off = 0;
  for (int l = 0; l < num_layers; ++l) {
    d.widths[l] = h.widths[l];
    d.win[l] = l == 0 ? m : h.widths[l - 1];
    d.woff[l] = off;
    off += d.win[l] * d.widths[l];
  }
  for (int l = 0; l < num_layers - 1; ++l) {
    d.boff[l] = off;
    off += d.widths[l];
  }
  d.P = h.P = off;
  const bool ard = (prior == BANN_RIDGE_ARD || prior == BANN_LASSO_ARD);
  int np = 0;
  for (int l = 0; l < num_layers; ++l) np += (ard && l < num_layers - 1) ? d.win[l] : 1;
  h.nprec = np + (num_layers - 1) + 1;
  h.prec.assign(h.nprec, 1.f);
  ctx->br.push_back(std::move(h));
  return (int)ctx->br.size() - 1;
}

extern "C" int bann_num_branches(const bann_ctx* ctx) { return ctx ? (int)ctx->br.size() : BANN_E_ARG; }
extern "C" int64_t bann_num_params(const bann_ctx* ctx, int32_t b) {
  if (!ctx || b < 0 || b >= (int32_t)ctx->br.size()) return BANN_E_ARG;
  return ctx->br[b].P;
}
extern "C" int64_t bann_num_precisions(const bann_ctx* ctx, int32_t b) {
  if (!ctx || b < 0 || b >= (int32_t)ctx->br.size()) return BANN_E_ARG;
  return ctx->br[b].nprec;
}
extern "C" int bann_branch_info(const bann_ctx* ctx, int32_t b, int32_t* m, int32_t* num_layers, int32_t* widths_out,
                                int32_t widths_cap, int32_t* activation, int32_t* prior) {
  if (!ctx || b < 0 || b >= (int32_t)ctx->br.size()) return BANN_E_ARG;
  const BranchHost& h = ctx->br[b];
  if (m) *m = h.m;
  if (num_layers) *num_layers = h.L;
  if (widths_out)
    for (int l = 0; l < h.L && l < widths_cap; ++l) widths_out[l] = h.widths[l];
  if (activation) *activation = h.act;
  if (prior) *prior = h.prior;
  return BANN_OK;
}
extern "C" int bann_branch_kernel_path(const bann_ctx* ctx, int32_t b) {
  if (!check_branch(ctx, b)) return BANN_E_ARG;
  return ctx->br[b].dev.fused;
}
extern "C" const char* bann_fused_kernel_name(void) { return "k_fused_grad_fx"; }

extern "C" int bann_set_hidden_gemm_bf16(bann_ctx* ctx, int32_t enabled) {
  if (!ctx) return BANN_E_ARG;
  ctx->wide_bf16 = enabled != 0;
  std::fill(ctx->pred_ok.begin(), ctx->pred_ok.end(), 0);  // wide-branch predictions change with the GEMM precision
  return BANN_OK;
}
extern "C" int bann_set_fused_enabled(bann_ctx* ctx, int32_t enabled) {
  if (!ctx) return BANN_E_ARG;
  if (ctx->finalized) return fail(ctx, BANN_E_STATE, "set before bann_finalize");
  ctx->fused_enabled = enabled != 0;
  return BANN_OK;
}
extern "C" int bann_set_graph_replay(bann_ctx* ctx, int32_t enabled) {
  if (!ctx) return BANN_E_ARG;
  ctx->graph_replay = enabled != 0;
  return BANN_OK;
}
extern "C" int bann_get_graph_replay(const bann_ctx* ctx) { return ctx ? (ctx->graph_replay ? 1 : 0) : BANN_E_ARG; }
extern "C" int64_t bann_packed_genotype_bytes(const bann_ctx* ctx) { return ctx ? ctx->packed_bytes : 0; }

extern "C" int bann_finalize(bann_ctx* ctx, int32_t free_raw) {
  if (!ctx) return BANN_E_ARG;
  if (ctx->finalized) return fail(ctx, BANN_E_STATE, "already finalized");
  if (!ctx->d_g) return fail(ctx, BANN_E_STATE, "no genotypes uploaded");
  if (ctx->br.empty()) return fail(ctx, BANN_E_STATE, "no branches");
  CK(hipSetDevice(ctx->device));
  const int64_t n = ctx->n;
  ctx->nfrag = (int32_t)((n + 15) / 16);
  // kernel path per branch: fx (widths <= 4, <= 8 chunks), fxl (widths <= 4,
  // 9..64 chunks), wx (one hidden layer up to 32 x 32, m <= 128), else gx (layered MFMA GEMMs)
  int64_t total_frags = 0;
  for (auto& h : ctx->br) {
    for (int i = 0; i < h.m; ++i)
      if (h.snp_idx[i] >= ctx->M) return fail(ctx, BANN_E_SHAPE, "marker index out of range");
    BranchDev& d = h.dev;
    d.nchunks = (h.m + BANN_CHUNK - 1) / BANN_CHUNK;
    bool narrow = ctx->fused_enabled && h.L >= 2 && h.L <= 4;
    for (int l = 0; l < h.L; ++l) narrow = narrow && h.widths[l] <= BANN_FUSED_MAXW;
    d.fused = 0;
    if (narrow && d.nchunks <= BANN_FX_MAXCH)
      d.fused = 1;
    else if (narrow && d.nchunks <= BANN_FXL_MAXCH)
      d.fused = 3;
    else if (ctx->fused_enabled && h.L == 3 && d.nchunks <= BANN_WIDE_MAXCH && h.widths[0] <= BANN_WIDE_MAXW &&
             h.widths[1] <= BANN_WIDE_MAXW)
      d.fused = 2;
    if (d.fused) total_frags += ctx->nfrag;
  }
  int64_t target_items = 1024;  // wx (and fx with BANN_TARGET_ITEMS / BANN_MIN_FRAGS): ~target work items
  if (const char* e = getenv("BANN_TARGET_ITEMS")) target_items = std::max<int64_t>(1, atoll(e));
  int64_t min_frags = 64;  // >= 16 tiles per work item amortises the per-item prologue/epilogue
  if (const char* e = getenv("BANN_MIN_FRAGS")) min_frags = std::max<int64_t>(1, atoll(e));
  const int64_t frags_per_item =
      std::max<int64_t>(min_frags, (total_frags + target_items - 1) / std::max<int64_t>(1, target_items));
  const int64_t ntile = (ctx->nfrag + BANN_TILE_FRAGS - 1) / BANN_TILE_FRAGS;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess || cus <= 0)
    cus = 256;
  ctx->cus = cus;
  // Splits: whole rounds of resident workgroups.  All items of a packed launch
  // are equally long, so a launch costs ceil(items / slots) rounds of (per-item
  // prologue/epilogue + tiles per wave); choose the split count minimising that
  // (e.g. 125 fx branches on one GPU of an 8-GPU shard: 4 splits = 500 items in
  // one round, where a 1024-item target gave 9 splits = 1125 items in 3 partly
  // empty rounds).  Lower bound: <= BANN_MAX_TILES_PER_WAVE tiles per wave, so
  // the int32 dW0 digit sums cannot overflow.
  auto best_splits = [&](int64_t nbr, int64_t slots, int64_t tiles_per_split_wave_div) -> int32_t {
    const int64_t min_sp = (ntile + tiles_per_split_wave_div * BANN_MAX_TILES_PER_WAVE - 1) /
                           (tiles_per_split_wave_div * BANN_MAX_TILES_PER_WAVE);
    int32_t best_sp = (int32_t)std::max<int64_t>(1, min_sp);
    double best = -1.0;
    for (int64_t sp = std::max<int64_t>(1, min_sp); nbr > 0 && sp <= std::max<int64_t>(64, min_sp); ++sp) {
      if (sp > min_sp && tiles_per_split_wave_div * sp > ntile) break;
      const int64_t rounds = (nbr * sp + slots - 1) / slots;
      const int64_t per_wave = (ntile + tiles_per_split_wave_div * sp - 1) / (tiles_per_split_wave_div * sp);
      const double cost = (double)rounds * (2.0 + (double)per_wave);  // ~2 tiles of prologue + epilogue
      if (best < 0.0 || cost < best) best = cost, best_sp = (int32_t)sp;
    }
    return best_sp;
  };
  const bool env_split = getenv("BANN_TARGET_ITEMS") || getenv("BANN_MIN_FRAGS");
  int64_t nfx = 0, nfxl[2][9] = {};  // fxl branches by (chunks per wave 4?, waves)
  auto fxl_key = [](int nch, int& c4, int& nw) {
    const int cpw = fxl_cpw(nch);
    c4 = cpw == 4;
    nw = (nch + cpw - 1) / cpw;
  };
  for (auto& h : ctx->br) {
    if (h.dev.fused == 1) ++nfx;
    if (h.dev.fused == 3) {
      int c4, nw;
      fxl_key(h.dev.nchunks, c4, nw);
      ++nfxl[c4][nw];
    }
  }
  const int32_t fx_splits = best_splits(nfx, 2 * (int64_t)cus, 4);  // fx: 2 workgroups of 4 waves per CU, tiles interleaved
  int64_t nwx = 0;
  for (auto& h : ctx->br) nwx += h.dev.fused == 2;
  // wx: 4 two-wave workgroups per CU, a tile at a time (exact f32 MFMA); wx3: 2
  // four-wave workgroups per CU, two tiles at a time
  const int32_t wx_splits = wx_exact() ? best_splits(nwx, 4 * (int64_t)cus, 1) : best_splits(nwx, 2 * (int64_t)cus, 2);
  int32_t fxl_splits[2][9] = {};
  for (int c4 = 0; c4 < 2; ++c4)
    for (int nw = 1; nw <= 8; ++nw) {  // fxl: all waves of a workgroup on one tile; LDS- and VGPR-limited residency
      const int64_t per_cu =
          std::max<int64_t>(1, std::min<int64_t>(163840 / fxl_lds_bytes(nw, 4, c4 ? 4 : 8), 8 / nw));
      fxl_splits[c4][nw] = best_splits(nfxl[c4][nw], per_cu * cus, 1);
    }
  int64_t q_off = 0;
  // forward-only fi images (kernels_fi.hip) for the fx branches with BANN_FWD_FI=1; by default
  // the LDS forward (k_forward_fx): inside the network trajectory, interleaved with the
  // gradient launches, it measured faster (2.573 vs 2.660 ms per step, r4c/r4d), and it
  // needs no second 2-bit image
  const bool fi_on = getenv("BANN_FWD_FI") && atoi(getenv("BANN_FWD_FI")) != 0;
  int64_t xi_off = 0;
  int64_t x2_off = 0, dig_off = 0, p_off = 0, mk_off = 0, part_off = 0, scr_off = 0, items = 0;
  // gx scratch groups: branches in index order until the budget (BANN_GX_SCRATCH_MB,
  // default a quarter of the free device memory, at most 64 GiB) is full; every
  // group reuses the same device scratch.  Fewer, larger groups fill the GPU better
  // (c3def: 8 GiB = 40 branches per group 335 ms per evaluation, 32 GiB 321 ms)
  const int64_t gx_rows = ntile * 64;
  int64_t gx_budget = 8192ll << 18;  // floats
  {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess && fr > 0)
      gx_budget = std::max<int64_t>(gx_budget, std::min<int64_t>((int64_t)(fr / 4) / 4, 65536ll << 18));
  }
  if (const char* e = getenv("BANN_GX_SCRATCH_MB")) gx_budget = std::max<int64_t>(1, atoll(e)) << 18;
  int64_t gx_cur = 0, n_gx = 0;
  int32_t gx_ngroups = 0;
  int32_t max_splits = 1;
  for (size_t b = 0; b < ctx->br.size(); ++b) {
    BranchHost& h = ctx->br[b];
    BranchDev& d = h.dev;
    d.x_off = x2_off;  // byte offset of the branch's 2-bit tile image: [tile][chunk][1 KiB]
    x2_off += ntile * d.nchunks * 1024;
    d.xi_off = -1;  // fx branches: the individual-major image of the forward-only pass, [frag][segment][1 KiB]
    if (d.fused == 1 && fi_on) {
      d.xi_off = xi_off;
      xi_off += 4 * ntile * ((d.nchunks + 3) / 4) * 1024;
    }
    d.dig_off = dig_off;
    if (d.fused) dig_off += (int64_t)d.nchunks * 1024 * (d.fused == 2 ? 8 : 1);
    d.p_off = p_off;
    p_off += h.P;
    {  // precision coordinates in precision_vec order (params.rs:272-289)
      const bool ard = (h.prior == BANN_RIDGE_ARD || h.prior == BANN_LASSO_ARD);
      int qo = 0;
      for (int l = 0; l < h.L; ++l) {
        d.qoff[l] = qo;
        qo += (ard && l < h.L - 1) ? d.win[l] : 1;
      }
      d.qbias = qo;
      d.nq = qo + (h.L - 1) + 1;
      d.q_off = q_off;
      q_off += d.nq;
    }
    d.mk_off = mk_off;
    mk_off += h.m;
    d.y_off = (int64_t)b * n;
    // gx: row splits of ~64 tiles (4096 individuals) for the K = n gradient GEMMs
    d.nsplits = d.fused ? (int32_t)std::max<int64_t>(1, (ctx->nfrag + frags_per_item - 1) / frags_per_item)
                        : (int32_t)((ntile + 63) / 64);
    if (d.fused == 1 && !env_split) d.nsplits = fx_splits;
    if (d.fused == 3) {
      int c4, nw;
      fxl_key(d.nchunks, c4, nw);
      d.nsplits = fxl_splits[c4][nw];
    }
    if (d.fused == 2) d.nsplits = wx_splits;
    if (d.fused == 1)  // overflow guard also under the env overrides
      d.nsplits = std::max<int32_t>(d.nsplits, (int32_t)((ntile + 4 * BANN_MAX_TILES_PER_WAVE - 1) /
                                                         (4 * BANN_MAX_TILES_PER_WAVE)));
    d.nsplits = (int32_t)std::max<int64_t>(1, std::min<int64_t>(d.nsplits, ntile));
    if (d.fused) items += d.nsplits;
    max_splits = std::max(max_splits, d.nsplits);
    d.part_off = part_off;
    part_off += (int64_t)d.nsplits * h.P;
    if (!d.fused) {  // gx scratch (kernels_gx.hip): padded weights, biases, A_l and H_l per layer
      if (d.widths[h.L - 2] > GX_HEAD_MAXW) return fail(ctx, BANN_E_SHAPE, "summary layer wider than 4096");
      auto r4 = [](int64_t v) { return (v + 3) & ~3ll; };
      int64_t o = 0;
      for (int l = 0; l < h.L; ++l) {
        d.gx_wld[l] = (int32_t)r4(d.win[l]);
        d.gx_w[l] = (int32_t)o;
        o += (int64_t)d.widths[l] * d.gx_wld[l];
      }
      for (int l = 0; l < h.L - 1; ++l) {
        d.gx_b[l] = (int32_t)o;
        o += r4(d.widths[l]);
      }
      d.gx_w0p = (int32_t)o;  // 3 x w0 x 64 nchunks bf16
      o += r4((3ll * d.widths[0] * 64 * d.nchunks + 1) / 2);
      for (int l = 1; l < h.L - 1; ++l) {  // 3 x w_l x r32(win_l) bf16
        d.gx_wp[l] = (int32_t)o;
        o += r4((3ll * d.widths[l] * ((d.win[l] + 31) & ~31) + 1) / 2);
      }
      d.gx_dwo = (int32_t)o;
      o += 2 * ntile * r4(d.widths[h.L - 2]);
      d.gx_rss = (int32_t)o;
      o += r4(2 * ntile);
      d.gx_op = (int32_t)o;
      o += 2 * ((d.widths[h.L - 2] + 63) / 64) * gx_rows;
      d.gx_e = (int32_t)o;
      o += gx_rows;
      d.gx_wps = (int32_t)o;
      if (h.L >= 3) o += r4((3ll * d.widths[h.L - 2] * ((d.win[h.L - 2] + 31) & ~31) + 1) / 2);
      for (int l = 0; l < h.L - 1; ++l) {
        d.gx_ld[l] = (int32_t)r4(d.widths[l]);
        d.gx_a[l] = (int32_t)o;
        o += gx_rows * d.gx_ld[l];
        d.gx_h[l] = (int32_t)o;
        o += gx_rows * d.gx_ld[l];
        if (o >= (1ll << 31)) return fail(ctx, BANN_E_SHAPE, "gx scratch of one branch exceeds 2^31 floats");
      }
      if (gx_cur > 0 && gx_cur + o > gx_budget) {  // a new scratch group
        ++gx_ngroups;
        gx_cur = 0;
      }
      h.gx_group = gx_ngroups;
      d.scr_off = gx_cur;
      gx_cur += o;
      scr_off = std::max(scr_off, gx_cur);
      ++n_gx;
    }
  }
  ctx->max_splits = max_splits;
  // solo mode (build_plan): ~one tile per wave for a branch alone on the GPU
  // (BANN_SOLO_TPW: more tiles per wave, fewer slabs to fold)
  int64_t solo_tpw = 1;
  if (const char* e = getenv("BANN_SOLO_TPW")) solo_tpw = std::max(1, atoi(e));
  int64_t max_p_fused = 0;
  for (auto& h : ctx->br) {
    const BranchDev& d = h.dev;
    if (!d.fused) continue;
    max_p_fused = std::max<int64_t>(max_p_fused, h.P);
    // fx: 4 waves on their own tiles, solo_tpw tiles each; fxl / wx: a tile at a time
    const int64_t per_item = d.fused == 1 ? 4 * solo_tpw : 1;
    h.solo_items = (int32_t)std::max<int64_t>(d.nsplits,
                                              std::min<int64_t>(2 * cus, (ntile + per_item - 1) / per_item));
  }
  ctx->solo_threshold = cus;
  if (const char* e = getenv("BANN_SOLO")) ctx->solo_threshold = atoi(e) ? cus : 0;  // 0: never re-split
  ctx->solo_rss_cap = 8ll * cus;
  ctx->solo_part_cap = ctx->solo_rss_cap * max_p_fused;
  ctx->part_total = part_off;
  ctx->packed_bytes = x2_off;
  ctx->total_p = p_off;
  ctx->total_q = q_off;
  const int64_t nb = (int64_t)ctx->br.size();
  CK(dalloc(&ctx->d_xu2, x2_off));
  ctx->xi_bytes = xi_off;
  if (xi_off > 0) CK(dalloc(&ctx->d_xi, xi_off));
  CK(dalloc(&ctx->d_dig, dig_off));
  CK(hipMemsetAsync(ctx->d_dig, 0, (size_t)std::max<int64_t>(dig_off, 1), ctx->stream));
  CK(dalloc(&ctx->d_fc, nb));
  CK(hipMemsetAsync(ctx->d_fc, 0, nb * sizeof(FusedConst), ctx->stream));
  CK(dalloc(&ctx->d_mub, mk_off));
  CK(dalloc(&ctx->d_sigb, mk_off));
  float** pbufs[] = {&ctx->d_theta, &ctx->d_mom, &ctx->d_eps, &ctx->d_theta0, &ctx->d_lam, &ctx->d_lamld,
                     &ctx->d_grad};
  for (float** pb : pbufs) {
    CK(dalloc(pb, p_off));
    CK(hipMemsetAsync(*pb, 0, p_off * sizeof(float), ctx->stream));
  }
  CK(dalloc(&ctx->d_stepbase, p_off));
  for (float** qb : {&ctx->d_phi, &ctx->d_phi0, &ctx->d_mphi, &ctx->d_ephi, &ctx->d_gphi}) CK(dalloc(qb, q_off));
  CK(dalloc(&ctx->d_ows, 2 * (int64_t)ctx->br.size()));
  {  // parameter -> precision index (within the branch), for the joint update
    std::vector<int32_t> pidx(p_off);
    for (auto& h : ctx->br) {
      const BranchDev& d = h.dev;
      const bool ard = (h.prior == BANN_RIDGE_ARD || h.prior == BANN_LASSO_ARD);
      for (int l = 0; l < h.L; ++l)
        for (int k = 0; k < d.widths[l]; ++k)
          for (int j = 0; j < d.win[l]; ++j)
            pidx[d.p_off + d.woff[l] + (int64_t)k * d.win[l] + j] = d.qoff[l] + ((ard && l < h.L - 1) ? j : 0);
      for (int l = 0; l < h.L - 1; ++l)
        for (int k = 0; k < d.widths[l]; ++k) pidx[d.p_off + d.boff[l] + k] = d.qbias + l;
    }
    CK(dalloc(&ctx->d_pidx, p_off));
    CK(hipMemcpy(ctx->d_pidx, pidx.data(), p_off * sizeof(int32_t), hipMemcpyHostToDevice));
  }
  CK(dalloc(&ctx->d_part, part_off + ctx->solo_part_cap));
  CK(hipMemsetAsync(ctx->d_part, 0, part_off * sizeof(float), ctx->stream));
  CK(dalloc(&ctx->d_rss_part, nb * max_splits + ctx->solo_rss_cap));
  CK(hipMemsetAsync(ctx->d_rss_part, 0, nb * max_splits * sizeof(double), ctx->stream));
  CK(dalloc(&ctx->d_y, nb * n));
  CK(hipMemsetAsync(ctx->d_y, 0, nb * n * sizeof(float), ctx->stream));
  CK(dalloc(&ctx->d_pred, nb * n));
  CK(hipMemsetAsync(ctx->d_pred, 0, nb * n * sizeof(float), ctx->stream));
  CK(dalloc(&ctx->d_pred0, nb * n));
  CK(dalloc(&ctx->d_delta, n));
  CK(dalloc(&ctx->d_delta_part, residual_delta_scratch_floats(n)));
  CK(hipHostMalloc((void**)&ctx->h_status, nb * sizeof(int32_t), hipHostMallocDefault));
  {
    int64_t max_p = 1;
    for (const auto& h : ctx->br) max_p = std::max<int64_t>(max_p, h.P);
    CK(hipHostMalloc((void**)&ctx->h_par_stage, max_p * sizeof(float), hipHostMallocDefault));
  }
  CK(hipHostMalloc((void**)&ctx->h_delta, n * sizeof(float), hipHostMallocDefault));
  CK(hipMemsetAsync(ctx->d_pred0, 0, nb * n * sizeof(float), ctx->stream));
  CK(dalloc(&ctx->d_scr, scr_off));
  CK(dalloc(&ctx->d_eprec, nb));
  CK(dalloc(&ctx->d_upd_cnt, nb));
  CK(hipMemsetAsync(ctx->d_upd_cnt, 0, nb * sizeof(int32_t), ctx->stream));
  CK(dalloc(&ctx->d_u, nb));
  CK(dalloc(&ctx->d_h0, nb));
  CK(dalloc(&ctx->d_ld, nb));
  CK(dalloc(&ctx->d_rss, nb));
  CK(dalloc(&ctx->d_status, nb));
  CK(dalloc(&ctx->d_uturn, nb));
  CK(dalloc(&ctx->d_gen_scr, nb));
  ctx->gxpre_cap = (int64_t)(3 * BANN_MAXL) * (n_gx + gx_ngroups + 2);
  CK(dalloc(&ctx->d_gxpre_scr, ctx->gxpre_cap));
  ctx->items_cap = items + ctx->solo_rss_cap;  // a solo plan has <= solo_rss_cap items
  {  // a per-call plan's branch lists, fold jobs and work items: one device block, filled by
     // ONE copy from a pinned stage (build_plan; was three copies per bann_hmc_step call)
    auto al = [](int64_t v) { return (v + 255) & ~(int64_t)255; };
    ctx->plan_off_fold = al(2 * (int64_t)nb * (int64_t)sizeof(int32_t));
    ctx->plan_off_items = ctx->plan_off_fold + al((int64_t)nb * (int64_t)sizeof(FoldJob));
    ctx->plan_scr_bytes = ctx->plan_off_items + ctx->items_cap * (int64_t)sizeof(GradItem);
    CK(hipMalloc((void**)&ctx->d_plan_scr, (size_t)ctx->plan_scr_bytes));
    CK(hipHostMalloc((void**)&ctx->h_plan_stage, (size_t)ctx->plan_scr_bytes, hipHostMallocDefault));
    CK(hipEventCreateWithFlags(&ctx->ev_plan, hipEventDisableTiming));
    ctx->d_list_scr = reinterpret_cast<int32_t*>(ctx->d_plan_scr);
    ctx->d_fold_scr = reinterpret_cast<FoldJob*>(ctx->d_plan_scr + ctx->plan_off_fold);
    ctx->d_items_scr = reinterpret_cast<GradItem*>(ctx->d_plan_scr + ctx->plan_off_items);
  }
  // every branch's tile image in ONE batched pack launch (no per-branch sync), the
  // marker statistics in one gather, the precision-derived arrays in one copy each
  std::vector<int32_t> allidx;
  allidx.reserve(mk_off);
  std::vector<PackJob> jobs;
  for (auto& h : ctx->br) {
    const int32_t base = (int32_t)allidx.size();
    allidx.insert(allidx.end(), h.snp_idx.begin(), h.snp_idx.end());
    for (int c = 0; c < h.dev.nchunks; ++c)
      jobs.push_back(PackJob{h.dev.x_off + 1024ll * c, 1024ll * h.dev.nchunks, base + 64 * c,
                             std::min(64, h.m - 64 * c), tile_f3m1(h.dev.fused) ? 1 : 0});
  }
  int32_t* d_idx = nullptr;
  PackJob* d_jobs = nullptr;
  CK(dalloc(&d_idx, (int64_t)allidx.size()));
  CK(dalloc(&d_jobs, (int64_t)jobs.size()));
  CK(hipMemcpyAsync(d_idx, allidx.data(), allidx.size() * sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream));
  CK(hipMemcpyAsync(d_jobs, jobs.data(), jobs.size() * sizeof(PackJob), hipMemcpyHostToDevice, ctx->stream));
  launch_pack_tiles(ctx->d_g, ctx->rowb, d_jobs, (int32_t)jobs.size(), d_idx, ntile, ctx->d_xu2, ctx->stream);
  PackJob* d_fijobs = nullptr;
  if (ctx->d_xi) {  // the fi images: one job per (branch, 256-marker segment)
    std::vector<PackJob> fj;
    int32_t base = 0;
    for (auto& h : ctx->br) {
      const int nseg = (h.dev.nchunks + 3) / 4;
      if (h.dev.xi_off >= 0)
        for (int sg = 0; sg < nseg; ++sg)
          fj.push_back(PackJob{h.dev.xi_off + 1024ll * sg, 1024ll * nseg, base + 256 * sg,
                               std::min(256, h.m - 256 * sg)});
      base += h.m;
    }
    CK(dalloc(&d_fijobs, (int64_t)fj.size()));
    CK(hipMemcpyAsync(d_fijobs, fj.data(), fj.size() * sizeof(PackJob), hipMemcpyHostToDevice, ctx->stream));
    launch_pack_fi(ctx->d_g, ctx->rowb, d_fijobs, (int32_t)fj.size(), d_idx, ntile, ctx->d_xi, ctx->stream);
    CK(hipStreamSynchronize(ctx->stream));  // fj goes out of scope
  }
  launch_gather_stats(ctx->d_mu, ctx->d_sigma, d_idx, (int32_t)allidx.size(), ctx->d_mub, ctx->d_sigb, ctx->stream);
  CK(hipGetLastError());
  std::vector<BranchDev> descs;
  std::vector<float> lam_all(p_off), lamld_all(p_off), eprec(nb, 1.f), lam, lamld;
  std::vector<double> sbase_all(p_off), sbase;
  for (size_t b = 0; b < ctx->br.size(); ++b) {
    BranchHost& h = ctx->br[b];
    descs.push_back(h.dev);
    float ep = 1.f;
    expand_precisions(h, lam, lamld, ep);
    eprec[b] = ep;
    step_bases(h, sbase);
    std::copy(lam.begin(), lam.end(), lam_all.begin() + h.dev.p_off);
    std::copy(lamld.begin(), lamld.end(), lamld_all.begin() + h.dev.p_off);
    std::copy(sbase.begin(), sbase.end(), sbase_all.begin() + h.dev.p_off);
  }
  CK(hipMemcpyAsync(ctx->d_lam, lam_all.data(), p_off * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
  CK(hipMemcpyAsync(ctx->d_lamld, lamld_all.data(), p_off * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
  CK(hipMemcpyAsync(ctx->d_stepbase, sbase_all.data(), p_off * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));  // host vectors go out of scope
  dfree(d_idx);
  dfree(d_jobs);
  dfree(d_fijobs);
  CK(dalloc(&ctx->d_br, nb));
  CK(hipMemcpyAsync(ctx->d_br, descs.data(), nb * sizeof(BranchDev), hipMemcpyHostToDevice, ctx->stream));
  CK(hipMemcpyAsync(ctx->d_eprec, eprec.data(), nb * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
  if (getenv("BANN_STAMPS")) {
    CK(hipMalloc((void**)&ctx->d_dbg, 16 * sizeof(unsigned long long)));
    CK(hipMemsetAsync(ctx->d_dbg, 0, 16 * sizeof(unsigned long long), ctx->stream));
  }
  ctx->finalized = true;
  ctx->pred_ok.assign(ctx->br.size(), 0);
  int rc = ensure_htrace(ctx, 1);
  if (rc) return rc;
  rc = net_buffers_init(ctx);  // the network sampler allocates nothing inside its trajectories
  if (rc) return rc;
  refresh_state(ctx);
  CK(hipStreamSynchronize(ctx->stream));
  if (free_raw) {
    dfree(ctx->d_g);
    ctx->d_g = nullptr;
  }
  return BANN_OK;
}

extern "C" int bann_branch_set_params(bann_ctx* ctx, int32_t b, const float* param_vec) {
  if (!check_branch(ctx, b) || !param_vec) return fail(ctx, BANN_E_ARG, "bad branch or null params");
  if (ctx->lf_active) return fail(ctx, BANN_E_STATE, "a leapfrog session is active");
  const BranchHost& h = ctx->br[b];
  CK(hipMemcpyAsync(ctx->d_theta + h.dev.p_off, param_vec, h.P * sizeof(float), hipMemcpyHostToDevice,
                    ctx->stream));
  int32_t bb = b;
  CK(hipMemcpyAsync(ctx->d_list_scr, &bb, sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream));
  launch_fused_const(ctx->st, ctx->d_list_scr, 1, ctx->stream);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(ctx->stream));
  ctx->pred_ok[b] = 0;
  return BANN_OK;
}

extern "C" int bann_branch_get_params(bann_ctx* ctx, int32_t b, float* out) {
  if (!check_branch(ctx, b) || !out) return fail(ctx, BANN_E_ARG, "bad branch or null output");
  const BranchHost& h = ctx->br[b];
  CK(hipMemcpyAsync(out, ctx->d_theta + h.dev.p_off, h.P * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  return BANN_OK;
}

// device copies derived from the host precision vector h.prec: per-parameter
// prior multipliers, error precision, Izmailov step bases
// the staged arrays of upload_precisions -> their device homes (one launch)
__global__ void k_scatter_prec(const char* __restrict__ stage, int P, float* __restrict__ lam,
                               float* __restrict__ lamld, double* __restrict__ sbase, float* __restrict__ ep) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const double* sb = reinterpret_cast<const double*>(stage);
  const float* l = reinterpret_cast<const float*>(stage + 8 * (size_t)P);
  if (i < P) {
    sbase[i] = sb[i];
    lam[i] = l[i];
    lamld[i] = l[P + i];
  }
  if (i == 0) *ep = l[2 * P];
}

// One branch's precision-derived device arrays (prior multipliers, error precision,
// Izmailov step bases): staged in pinned memory as [sbase (f64) | lam | lamld | ep], one
// H2D copy and one scatter launch, no host wait -- the sequential driver does this once
// per branch update (it was four copies and a stream synchronisation).  The staging
// buffer is reused after the previous upload's copy has completed (event).
static int upload_precisions(bann_ctx* ctx, int32_t b) {
  const BranchHost& h = ctx->br[b];
  std::vector<float> lam, lamld;
  float ep = 1.f;
  expand_precisions(h, lam, lamld, ep);
  std::vector<double> sbase;
  step_bases(h, sbase);
  const size_t bytes = 16 * (size_t)h.P + 16;
  if (bytes > ctx->prec_stage_cap) {
    if (ctx->prec_ev_pending) CK(hipEventSynchronize(ctx->ev_prec));
    if (ctx->h_prec_stage) (void)hipHostFree(ctx->h_prec_stage);
    if (ctx->d_prec_stage) (void)hipFree(ctx->d_prec_stage);
    ctx->h_prec_stage = nullptr;
    ctx->d_prec_stage = nullptr;
    ctx->prec_stage_cap = 0;
    size_t cap = bytes;
    for (const auto& o : ctx->br) cap = std::max(cap, 16 * (size_t)o.P + 16);
    CK(hipHostMalloc((void**)&ctx->h_prec_stage, cap, hipHostMallocDefault));
    CK(hipMalloc((void**)&ctx->d_prec_stage, cap));
    if (!ctx->ev_prec) CK(hipEventCreateWithFlags(&ctx->ev_prec, hipEventDisableTiming));
    ctx->prec_stage_cap = cap;
    ctx->prec_ev_pending = false;
  }
  if (ctx->prec_ev_pending) CK(hipEventSynchronize(ctx->ev_prec));  // the last upload's copy has read the stage
  char* st = ctx->h_prec_stage;
  std::memcpy(st, sbase.data(), 8 * (size_t)h.P);
  std::memcpy(st + 8 * (size_t)h.P, lam.data(), 4 * (size_t)h.P);
  std::memcpy(st + 12 * (size_t)h.P, lamld.data(), 4 * (size_t)h.P);
  std::memcpy(st + 16 * (size_t)h.P, &ep, sizeof(float));
  CK(hipMemcpyAsync(ctx->d_prec_stage, st, bytes, hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(k_scatter_prec, dim3((unsigned)((h.P + 255) / 256)), dim3(256), 0, ctx->stream, ctx->d_prec_stage,
                     (int)h.P, ctx->d_lam + h.dev.p_off, ctx->d_lamld + h.dev.p_off, ctx->d_stepbase + h.dev.p_off,
                     ctx->d_eprec + b);
  CK(hipGetLastError());
  CK(hipEventRecord(ctx->ev_prec, ctx->stream));
  ctx->prec_ev_pending = true;
  return BANN_OK;
}

extern "C" int bann_branch_set_precisions(bann_ctx* ctx, int32_t b, const float* prec) {
  if (!check_branch(ctx, b) || !prec) return fail(ctx, BANN_E_ARG, "bad branch or null precisions");
  if (ctx->lf_active) return fail(ctx, BANN_E_STATE, "a leapfrog session is active");
  ctx->br[b].prec.assign(prec, prec + ctx->br[b].nprec);
  return upload_precisions(ctx, b);
}

extern "C" int bann_branch_set_output_stats(bann_ctx* ctx, int32_t b, float reg_sum_others, float num_params) {
  if (!check_branch(ctx, b)) return fail(ctx, BANN_E_ARG, "bad branch");
  ctx->br[b].ows_reg_sum = reg_sum_others;
  ctx->br[b].ows_num = num_params;
  return BANN_OK;
}

extern "C" int bann_branch_get_step_sizes(bann_ctx* ctx, int32_t b, float* out) {
  if (!check_branch(ctx, b) || !out) return fail(ctx, BANN_E_ARG, "bad branch or null output");
  const BranchHost& h = ctx->br[b];
  CK(hipMemcpyAsync(out, ctx->d_eps + h.dev.p_off, h.P * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  return BANN_OK;
}

extern "C" int bann_branch_get_precisions(bann_ctx* ctx, int32_t b, float* out) {
  if (!check_branch(ctx, b) || !out) return fail(ctx, BANN_E_ARG, "bad branch or null output");
  std::copy(ctx->br[b].prec.begin(), ctx->br[b].prec.end(), out);
  return BANN_OK;
}

extern "C" int bann_branch_set_target(bann_ctx* ctx, int32_t b, const float* y) {
  if (!check_branch(ctx, b) || !y) return fail(ctx, BANN_E_ARG, "bad branch or null target");
  if (ctx->lf_active) return fail(ctx, BANN_E_STATE, "a leapfrog session is active");
  CK(hipMemcpyAsync(ctx->d_y + (int64_t)b * ctx->n, y, ctx->n * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  return BANN_OK;
}

extern "C" int bann_set_target_all(bann_ctx* ctx, const float* y) {
  if (!ctx || !ctx->finalized || !y) return fail(ctx, BANN_E_ARG, "not finalized or null target");
  if (ctx->lf_active) return fail(ctx, BANN_E_STATE, "a leapfrog session is active");
  for (size_t b = 0; b < ctx->br.size(); ++b)
    CK(hipMemcpyAsync(ctx->d_y + (int64_t)b * ctx->n, y, ctx->n * sizeof(float), hipMemcpyHostToDevice,
                      ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  return BANN_OK;
}

// ---------------------------------------------------------------------------
// per-branch math
// ---------------------------------------------------------------------------
static int eval_branch(bann_ctx* ctx, int32_t b, int write_pred) {
  Plan p;
  int rc = build_plan(ctx, &b, 1, p, false);
  if (rc) return rc;
  rc = run_grad(ctx, p, write_pred);
  if (rc) return rc;
  run_update(ctx, p, MODE_GRAD, 0);
  CK(hipGetLastError());
  return BANN_OK;
}

extern "C" int bann_predict(bann_ctx* ctx, int32_t b, float* pred_out) {
  if (!check_branch(ctx, b) || !pred_out) return fail(ctx, BANN_E_ARG, "bad branch or null output");
  if (ctx->lf_active) return fail(ctx, BANN_E_STATE, "a leapfrog session is active");
  int rc = ensure_predictions(ctx, &b, 1);
  if (rc) return rc;
  CK(hipMemcpyAsync(pred_out, ctx->d_pred + (int64_t)b * ctx->n, ctx->n * sizeof(float), hipMemcpyDeviceToHost,
                    ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  return BANN_OK;
}

extern "C" int bann_predict_many(bann_ctx* ctx, const int32_t* branches, int32_t nb, float* pred_out) {
  if (!ctx || !branches || nb <= 0 || !pred_out) return fail(ctx, BANN_E_ARG, "bad branch list or null output");
  if (!ctx->finalized) return fail(ctx, BANN_E_STATE, "call bann_finalize first");
  if (ctx->lf_active) return fail(ctx, BANN_E_STATE, "a leapfrog session is active");
  Plan p;
  int rc = build_plan(ctx, branches, nb, p, false);
  if (rc) return rc;
  rc = run_forward(ctx, p);  // one packed forward launch per kernel group
  if (rc) return rc;
  for (int32_t i = 0; i < nb; ++i)
    CK(hipMemcpyAsync(pred_out + (int64_t)i * ctx->n, ctx->d_pred + (int64_t)branches[i] * ctx->n,
                      ctx->n * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  return BANN_OK;
}

extern "C" int bann_rss(bann_ctx* ctx, int32_t b, double* rss_out) {
  if (!check_branch(ctx, b) || !rss_out) return fail(ctx, BANN_E_ARG, "bad branch or null output");
  int rc = eval_branch(ctx, b, 0);
  if (rc) return rc;
  CK(hipMemcpyAsync(rss_out, ctx->d_rss + b, sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  return BANN_OK;
}

extern "C" int bann_log_density_gradient(bann_ctx* ctx, int32_t b, float* grad_out, double* rss_out) {
  if (!check_branch(ctx, b) || !grad_out) return fail(ctx, BANN_E_ARG, "bad branch or null output");
  int rc = eval_branch(ctx, b, 0);
  if (rc) return rc;
  const BranchHost& h = ctx->br[b];
  CK(hipMemcpyAsync(grad_out, ctx->d_grad + h.dev.p_off, h.P * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
  if (rss_out) CK(hipMemcpyAsync(rss_out, ctx->d_rss + b, sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  return BANN_OK;
}

// Net::gradient (net.rs:520-527): the log-density gradients of several branches
// against their current targets from one packed gradient launch
extern "C" int bann_log_density_gradient_many(bann_ctx* ctx, const int32_t* branches, int32_t nb, float* grad_out,
                                              double* rss_out) {
  if (!ctx || !branches || nb <= 0 || !grad_out) return fail(ctx, BANN_E_ARG, "bad branch list or null output");
  if (!ctx->finalized) return fail(ctx, BANN_E_STATE, "call bann_finalize first");
  if (ctx->lf_active) return fail(ctx, BANN_E_STATE, "a leapfrog session is active");
  for (int i = 0; i < nb; ++i) {
    if (!check_branch(ctx, branches[i])) return fail(ctx, BANN_E_ARG, "bad branch");
    for (int k = 0; k < i; ++k)
      if (branches[i] == branches[k]) return fail(ctx, BANN_E_ARG, "duplicate branch in list");
  }
  Plan p;
  int rc = build_plan(ctx, branches, nb, p, false);
  if (rc) return rc;
  rc = run_grad(ctx, p, 0);
  if (rc) return rc;
  run_update(ctx, p, MODE_GRAD, 0);
  CK(hipGetLastError());
  int64_t off = 0;
  for (int i = 0; i < nb; ++i) {
    const BranchHost& h = ctx->br[branches[i]];
    CK(hipMemcpyAsync(grad_out + off, ctx->d_grad + h.dev.p_off, h.P * sizeof(float), hipMemcpyDeviceToHost,
                      ctx->stream));
    if (rss_out) CK(hipMemcpyAsync(rss_out + i, ctx->d_rss + branches[i], sizeof(double), hipMemcpyDeviceToHost,
                                   ctx->stream));
    off += h.P;
  }
  CK(hipStreamSynchronize(ctx->stream));
  return BANN_OK;
}

// log_density_gradient_joint (branch_sampler.rs:406-422) at the branch's current
// parameters and precisions: [params | precisions], the joint log density
// (log_density_joint 292-305) and the rss; k_update_joint in MODE_GRAD
extern "C" int bann_log_density_gradient_joint(bann_ctx* ctx, int32_t b, const float* hyper, float* grad_out,
                                               double* rss_out, double* log_density_out) {
  if (!check_branch(ctx, b) || !hyper || !grad_out) return fail(ctx, BANN_E_ARG, "bad branch or null pointer");
  if (ctx->lf_active) return fail(ctx, BANN_E_STATE, "a leapfrog session is active");
  const BranchHost& h = ctx->br[b];
  if (h.prior == BANN_STD_NORMAL)
    return fail(ctx, BANN_E_ARG, "std_normal has no joint density (std_normal_branch.rs:119-131)");
  if (h.dev.nq > BANN_JOINT_MAXQ) return fail(ctx, BANN_E_SHAPE, "too many precisions for the joint update");
  for (int k = 0; k < 6; ++k) ctx->st.hyper[k] = hyper[k];
  const float ows[2] = {h.ows_reg_sum, h.ows_num >= 0.f ? h.ows_num : (float)h.widths[h.L - 2]};
  CK(hipMemcpyAsync(ctx->d_phi + h.dev.q_off, h.prec.data(), h.dev.nq * sizeof(float), hipMemcpyHostToDevice,
                    ctx->stream));
  CK(hipMemcpyAsync(ctx->d_ows + 2 * b, ows, 2 * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
  Plan p;
  int rc = build_plan(ctx, &b, 1, p, false);
  if (rc) return rc;
  rc = run_grad(ctx, p, 0);
  if (rc) return rc;
  launch_update_joint(ctx->st, p.d_all, 1, MODE_GRAD, 0, ctx->stream);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(grad_out, ctx->d_grad + h.dev.p_off, h.P * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipMemcpyAsync(grad_out + h.P, ctx->d_gphi + h.dev.q_off, h.dev.nq * sizeof(float), hipMemcpyDeviceToHost,
                    ctx->stream));
  double r[2] = {0.0, 0.0};
  CK(hipMemcpyAsync(&r[0], ctx->d_rss + b, sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipMemcpyAsync(&r[1], ctx->d_ld + b, sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  if (rss_out) *rss_out = r[0];
  if (log_density_out) *log_density_out = r[1];
  return BANN_OK;
}

// forward_feed (branch_sampler.rs:743-782) with every layer kept, for
// Net::activations (net.rs:509-518): kernels_feed.hip, scratch per call
extern "C" int bann_forward_feed(bann_ctx* ctx, int32_t b, float* pre_out, float* act_out) {
  if (!check_branch(ctx, b) || !act_out) return fail(ctx, BANN_E_ARG, "bad branch or null output");
  if (ctx->lf_active) return fail(ctx, BANN_E_STATE, "a leapfrog session is active");
  const BranchHost& h = ctx->br[b];
  int64_t wa = 0, wp = 0;
  for (int l = 0; l < h.L; ++l) {
    wa += h.widths[l];
    if (l < h.L - 1) wp += h.widths[l];
  }
  const int64_t n = ctx->n;
  float *d_act = nullptr, *d_pre = nullptr;
  CK(dalloc(&d_act, wa * n));
  if (pre_out && dalloc(&d_pre, wp * n) != hipSuccess) {
    dfree(d_act);
    return fail(ctx, BANN_E_OOM, "forward_feed scratch");
  }
  launch_forward_feed(ctx->st, b, h.dev, d_pre, d_act, ctx->stream);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(act_out, d_act, wa * n * sizeof(float), hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess && pre_out)
    e = hipMemcpyAsync(pre_out, d_pre, wp * n * sizeof(float), hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  dfree(d_act);
  dfree(d_pre);
  CK(e);
  return BANN_OK;
}

namespace {
// device scratch of the effect-size chain, sized for the largest listed branch
struct EffectScratch {
  float *pre = nullptr, *act = nullptr, *ea = nullptr, *eb = nullptr, *full = nullptr, *pop = nullptr;
  double* s = nullptr;
  ~EffectScratch() {
    dfree(pre);
    dfree(act);
    dfree(ea);
    dfree(eb);
    dfree(full);
    dfree(pop);
    dfree(s);
  }
  hipError_t alloc(const bann_ctx* ctx, const int32_t* branches, int32_t nb, bool want_full) {
    int64_t wp = 1, wa = 1, we = 1, wm = 1, w0 = 1;
    for (int32_t i = 0; i < nb; ++i) {
      const BranchHost& h = ctx->br[branches[i]];
      int64_t p = 0, a = 0;
      for (int l = 0; l < h.L; ++l) {
        a += h.widths[l];
        if (l < h.L - 1) p += h.widths[l];
        if (l >= 1) we = std::max<int64_t>(we, h.dev.win[l]);
      }
      wp = std::max(wp, p);
      wa = std::max(wa, a);
      wm = std::max<int64_t>(wm, h.m);
      w0 = std::max<int64_t>(w0, h.widths[0]);
    }
    const int64_t n = ctx->n;
    hipError_t e = dalloc(&pre, wp * n);
    if (e == hipSuccess) e = dalloc(&act, wa * n);
    if (e == hipSuccess) e = dalloc(&ea, we * n);
    if (e == hipSuccess) e = dalloc(&eb, we * n);
    if (e == hipSuccess) e = want_full ? dalloc(&full, wm * n) : dalloc(&pop, wm);
    if (e == hipSuccess) e = dalloc(&s, w0);
    return e;
  }
};
}  // namespace

// BranchSampler::effect_sizes (branch_sampler.rs:784-811): forward_feed + the
// output-seeded backward chain (kernels_feed.hip), the n x m matrix to the host
extern "C" int bann_effect_sizes(bann_ctx* ctx, int32_t b, float* out) {
  if (!check_branch(ctx, b) || !out) return fail(ctx, BANN_E_ARG, "bad branch or null output");
  if (ctx->lf_active) return fail(ctx, BANN_E_STATE, "a leapfrog session is active");
  const BranchHost& h = ctx->br[b];
  EffectScratch sc;
  if (sc.alloc(ctx, &b, 1, true) != hipSuccess) return fail(ctx, BANN_E_OOM, "effect_sizes scratch");
  launch_forward_feed(ctx->st, b, h.dev, sc.pre, sc.act, ctx->stream);
  launch_effect_sizes(ctx->st, b, h.dev, sc.pre, sc.act, sc.ea, sc.eb, sc.full, nullptr, nullptr, ctx->stream);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(out, sc.full, (int64_t)h.m * ctx->n * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  return BANN_OK;
}

// Net::population_effect_sizes' per-branch column means (net.rs:529-543)
extern "C" int bann_population_effect_sizes(bann_ctx* ctx, const int32_t* branches, int32_t nb, float* out) {
  if (!ctx || !branches || nb <= 0 || !out) return fail(ctx, BANN_E_ARG, "null pointer or empty branch list");
  if (ctx->lf_active) return fail(ctx, BANN_E_STATE, "a leapfrog session is active");
  for (int32_t i = 0; i < nb; ++i)
    if (!check_branch(ctx, branches[i])) return fail(ctx, BANN_E_ARG, "bad branch index");
  EffectScratch sc;
  if (sc.alloc(ctx, branches, nb, false) != hipSuccess) return fail(ctx, BANN_E_OOM, "population_effect_sizes scratch");
  int64_t at = 0;
  for (int32_t i = 0; i < nb; ++i) {
    const BranchHost& h = ctx->br[branches[i]];
    launch_forward_feed(ctx->st, branches[i], h.dev, sc.pre, sc.act, ctx->stream);
    launch_effect_sizes(ctx->st, branches[i], h.dev, sc.pre, sc.act, sc.ea, sc.eb, nullptr, sc.s, sc.pop,
                        ctx->stream);
    CK(hipGetLastError());
    CK(hipMemcpyAsync(out + at, sc.pop, (int64_t)h.m * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    at += h.m;
  }
  CK(hipStreamSynchronize(ctx->stream));
  return BANN_OK;
}

// host evaluation of log_density at the current parameters (branch_sampler.rs:72-78)
static int host_log_density(bann_ctx* ctx, int32_t b, double rss, double* out) {
  const BranchHost& h = ctx->br[b];
  std::vector<float> th(h.P), lam, lamld;
  CK(hipMemcpyAsync(th.data(), ctx->d_theta + h.dev.p_off, h.P * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  float ep = 1.f;
  expand_precisions(h, lam, lamld, ep);
  const bool lasso = (h.prior == BANN_LASSO_ARD || h.prior == BANN_LASSO_BASE);
  double ld = 0.0;
  for (int i = 0; i < h.P; ++i)
    ld -= lasso ? (double)lamld[i] * fabs((double)th[i]) : 0.5 * (double)lamld[i] * (double)th[i] * (double)th[i];
  *out = ld - (double)ep * rss / 2.0;
  return BANN_OK;
}

extern "C" int bann_log_density(bann_ctx* ctx, int32_t b, double rss, double* out) {
  if (!check_branch(ctx, b) || !out) return fail(ctx, BANN_E_ARG, "bad branch or null output");
  return host_log_density(ctx, b, rss, out);
}

extern "C" int bann_neg_hamiltonian(bann_ctx* ctx, int32_t b, const float* momentum, double* out) {
  if (!check_branch(ctx, b) || !momentum || !out) return fail(ctx, BANN_E_ARG, "bad branch or null pointer");
  double rss = 0.0;
  int rc = bann_rss(ctx, b, &rss);
  if (rc) return rc;
  double ld = 0.0;
  rc = host_log_density(ctx, b, rss, &ld);
  if (rc) return rc;
  double k = 0.0;
  for (int64_t i = 0; i < ctx->br[b].P; ++i) k += (double)momentum[i] * (double)momentum[i];
  *out = ld - 0.5 * k;
  return BANN_OK;
}

// ---------------------------------------------------------------------------
// HMC
// ---------------------------------------------------------------------------
int traj_prepare(bann_ctx* ctx, const Plan& p, int32_t L, float max_dh, int32_t step_mode, float factor,
                        const float* eps, const float* momentum, uint64_t seed, const float* u) {
  int rc = ensure_htrace(ctx, L);
  if (rc) return rc;
  ctx->st.max_dh = max_dh;
  ctx->st.lint = ctx->htrace_cap - 1;
  std::mt19937_64 rng(seed ^ 0x5DEECE66Dull);
  std::vector<float> e;
  int64_t off = 0;
  const bool device_eps = step_mode == BANN_STEP_UNIFORM || step_mode == BANN_STEP_IZMAILOV;
  if (device_eps) {
    launch_step_sizes(ctx->st, ctx->d_stepbase, p.d_all, (int32_t)p.all.size(), p.max_p,
                      step_mode == BANN_STEP_UNIFORM ? 0 : 1, factor, L, ctx->stream);
    CK(hipGetLastError());
  }
  for (int32_t b : p.all) {
    const BranchHost& h = ctx->br[b];
    if (device_eps) {
      // formed on the device above
    } else if (step_mode == BANN_STEP_INJECTED) {
      if (!eps) return fail(ctx, BANN_E_ARG, "injected step sizes need eps");
      CK(hipMemcpyAsync(ctx->d_eps + h.dev.p_off, eps + off, h.P * sizeof(float), hipMemcpyHostToDevice,
                        ctx->stream));
    } else if (step_mode == BANN_STEP_STD_SCALED) {
      if (!host_std_scaled_step_sizes(h, factor, e))
        return fail(ctx, BANN_E_ARG,
                    "StdScaled step sizes are empty for the ARD priors in the reference (ridge_ard.rs:56-68, "
                    "lasso_ard.rs:62-74; hmc_step would index-panic): use Izmailov, uniform or random");
      CK(hipMemcpyAsync(ctx->d_eps + h.dev.p_off, e.data(), h.P * sizeof(float), hipMemcpyHostToDevice,
                        ctx->stream));
      CK(hipStreamSynchronize(ctx->stream));  // e is reused for the next branch
    } else {
      if (step_mode != BANN_STEP_RANDOM) return fail(ctx, BANN_E_ARG, "unknown step size mode");
      host_random_step_sizes(h, factor, rng, e);
      CK(hipMemcpyAsync(ctx->d_eps + h.dev.p_off, e.data(), h.P * sizeof(float), hipMemcpyHostToDevice,
                        ctx->stream));
    }
    if (momentum)
      CK(hipMemcpyAsync(ctx->d_mom + h.dev.p_off, momentum + off, h.P * sizeof(float), hipMemcpyHostToDevice,
                        ctx->stream));
    off += h.P;
  }
  if (!momentum) {
    launch_sample_momentum(ctx->st, p.d_all, (int32_t)p.all.size(), p.max_p, seed, ctx->stream);
    CK(hipGetLastError());
  }
  bool host_data = momentum || (!device_eps);
  if (u) {  // injected acceptance uniforms (parity runs; the sequential driver's host draws)
    // staged in pinned memory that outlives the copy: no host wait here (the stage is
    // reused once the previous call's copy has completed)
    if (!ctx->h_u_stage) {
      CK(hipHostMalloc((void**)&ctx->h_u_stage, ctx->br.size() * sizeof(float), hipHostMallocDefault));
      CK(hipEventCreateWithFlags(&ctx->ev_u, hipEventDisableTiming));
      std::fill(ctx->h_u_stage, ctx->h_u_stage + ctx->br.size(), 0.f);
    }
    if (ctx->u_ev_pending) CK(hipEventSynchronize(ctx->ev_u));
    for (size_t i = 0; i < p.all.size(); ++i) ctx->h_u_stage[p.all[i]] = u[i];
    CK(hipMemcpyAsync(ctx->d_u, ctx->h_u_stage, ctx->br.size() * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
    CK(hipEventRecord(ctx->ev_u, ctx->stream));
    ctx->u_ev_pending = true;
    CK(hipMemsetAsync(ctx->d_htrace, 0xFF, ctx->br.size() * ctx->htrace_cap * sizeof(double), ctx->stream));
    if (host_data) CK(hipStreamSynchronize(ctx->stream));  // host step sizes / momenta copied
    return BANN_OK;
  }
  // acceptance uniforms u ~ U(0,1) per branch (branch_sampler.rs:546-548) on the device
  launch_uniforms(ctx->st, p.d_all, (int32_t)p.all.size(), seed, ctx->stream);
  CK(hipMemsetAsync(ctx->d_htrace, 0xFF, ctx->br.size() * ctx->htrace_cap * sizeof(double), ctx->stream));
  // device-only trajectory start (leapfrog sessions): no host round trip; host
  // vectors (random / injected step sizes, injected momenta) must outlive their copies
  if (host_data) CK(hipStreamSynchronize(ctx->stream));
  return BANN_OK;
}

// per-branch outputs of a finished bann_hmc_step (the stream has drained)
static int hmc_outputs(bann_ctx* ctx, const int32_t* branches, int32_t nb, int32_t L, int32_t* status_out,
                       double* h_trace_out, int32_t* uturn_out, double* log_density_out) {
  const int stride = ctx->htrace_cap;
  for (int i = 0; i < nb; ++i) {
    const int b = branches[i];
    if (status_out) CK(hipMemcpy(status_out + i, ctx->d_status + b, sizeof(int32_t), hipMemcpyDeviceToHost));
    if (uturn_out) CK(hipMemcpy(uturn_out + i, ctx->d_uturn + b, sizeof(int32_t), hipMemcpyDeviceToHost));
    if (log_density_out) CK(hipMemcpy(log_density_out + i, ctx->d_ld + b, sizeof(double), hipMemcpyDeviceToHost));
    if (h_trace_out)
      CK(hipMemcpy(h_trace_out + (int64_t)i * (L + 1), ctx->d_htrace + (int64_t)b * stride, (L + 1) * sizeof(double),
                   hipMemcpyDeviceToHost));
  }
  return BANN_OK;
}

// ---- graph replay of a trajectory's launch sequence (bann_hmc_step) ----
// The sequential driver runs one small trajectory after another (one branch,
// L steps of gradient + update launches): the host's launch overhead, not the
// GPU, paces it.  The sequence of a plan shape is captured once into a HIP
// graph and replayed; the plan's device arrays live in the context's scratch
// buffers (fixed addresses), so one graph serves every branch of the same shape.
// The key holds everything the captured kernel arguments depend on.
static std::string traj_graph_key(const bann_ctx* ctx, const Plan& p, int32_t L) {
  std::string k;
  auto put = [&](int64_t v) { k.append(reinterpret_cast<const char*>(&v), sizeof(v)); };
  put(L);
  put(ctx->wide_bf16);
  put((int64_t)p.all.size());
  put(p.n_small);
  put(p.n_large);
  put(p.max_p);
  put(p.fuse_update);
  put((int64_t)p.fold.size());
  put((int64_t)(intptr_t)p.d_all);
  put((int64_t)(intptr_t)p.d_fold);
  put((int64_t)(intptr_t)p.d_gx);
  put((int64_t)(intptr_t)p.d_gxpre);
  for (const auto& g : p.groups) {
    put(g.kind), put(g.L), put(g.act), put(g.nw), put(g.cpw), put(g.full), put(g.head);  // cpw, head: fxl's kernel
    put((int64_t)g.items.size());
    put((int64_t)(intptr_t)g.d_items);
  }
  for (const auto& g : p.gxg) {
    put(g.first), put(g.count), put(g.max_splits);
    for (const auto& ph : g.phases) put(ph.ph), put(ph.l), put(ph.total), put(ph.pre_off);
  }
  k.append(reinterpret_cast<const char*>(&ctx->st), sizeof(DevState));  // the kernels' by-value state
  return k;
}

void clear_graphs(bann_ctx* ctx) {
  for (auto& e : ctx->graphs) (void)hipGraphExecDestroy(e.second);
  ctx->graphs.clear();
}

// the launches of one trajectory after traj_prepare: initial gradient (f(theta_0) -> pred0),
// INIT update, L x (gradient, update), restore of the rejected branches' predictions
// one leapfrog step's launches: gradient + update, or the gradient launch alone with
// the update in its tail (a fuse_update plan)
static int traj_step(bann_ctx* ctx, const Plan& p, int write_pred, int mode, int step) {
  if (p.fuse_update) {
    mark_predictions(ctx, p, false);
    return run_grad(ctx, p, write_pred, mode, step);
  }
  const int rc = run_grad(ctx, p, write_pred);
  if (rc) return rc;
  run_update(ctx, p, mode, step);
  return BANN_OK;
}

static int traj_launches(bann_ctx* ctx, const Plan& p, int32_t L) {
  int rc = traj_step(ctx, p, 2, MODE_INIT, 0);
  if (rc) return rc;
  for (int k = 1; k <= L; ++k) {
    rc = traj_step(ctx, p, k == L ? 1 : 0, k < L ? MODE_STEP : MODE_LAST, k);
    if (rc) return rc;
  }
  launch_restore_pred(ctx->st, p.d_all, (int32_t)p.all.size(), ctx->stream);
  CK(hipGetLastError());
  return BANN_OK;
}

// trajectory recording: the -H trace of every recorded branch after the stream
// has drained; an early rejection leaves the later entries unwritten (NaN) and
// ends the recorded steps there (branch_sampler.rs:1264-1279)
static int rec_finish(bann_ctx* ctx, const int32_t* branches, int32_t nb, int32_t L) {
  const int stride = ctx->htrace_cap;
  for (int i = 0; i < nb; ++i) {
    auto& R = ctx->rec[branches[i]];
    R.h.assign(L + 1, 0.0);
    CK(hipMemcpy(R.h.data(), ctx->d_htrace + (int64_t)branches[i] * stride, (L + 1) * sizeof(double),
                 hipMemcpyDeviceToHost));
    int steps = 0;
    while (steps < L && R.h[steps + 1] == R.h[steps + 1]) ++steps;
    R.steps = steps;
    R.h.resize(steps + 1);
  }
  return BANN_OK;
}

static int traj_replay(bann_ctx* ctx, const Plan& p, int32_t L) {
  const std::string key = traj_graph_key(ctx, p, L);
  hipGraphExec_t exec = nullptr;
  for (auto& e : ctx->graphs)
    if (e.first == key) exec = e.second;
  if (!exec) {
    if (ctx->graphs.size() >= 16) clear_graphs(ctx);
    CK(hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeRelaxed));
    const int rc = traj_launches(ctx, p, L);
    hipGraph_t g = nullptr;
    const hipError_t ee = hipStreamEndCapture(ctx->stream, &g);
    if (rc) {
      if (g) (void)hipGraphDestroy(g);
      return rc;
    }
    CK(ee);
    const hipError_t ei = hipGraphInstantiate(&exec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    CK(ei);
    ctx->graphs.push_back({key, exec});
  }
  CK(hipGraphLaunch(exec, ctx->stream));
  mark_predictions(ctx, p, true);
  return BANN_OK;
}

extern "C" int bann_hmc_step(bann_ctx* ctx, const int32_t* branches, int32_t nb, int32_t L, float max_dh,
                             int32_t step_mode, float factor, const float* eps, const float* momentum, uint64_t seed,
                             const float* u, int32_t* status_out, double* h_trace_out, int32_t* uturn_out,
                             double* log_density_out) {
  if (!ctx || !ctx->finalized) return fail(ctx, BANN_E_STATE, "not finalized");
  if (!branches || nb <= 0 || L < 0) return fail(ctx, BANN_E_ARG, "bad branch list or L");
  if (ctx->lf_active) return fail(ctx, BANN_E_STATE, "a leapfrog session is active");
  for (int i = 0; i < nb; ++i)
    for (int k = 0; k < i; ++k)
      if (branches[i] == branches[k]) return fail(ctx, BANN_E_ARG, "duplicate branch in list");
  Plan p;
  int rc = build_plan(ctx, branches, nb, p, false);
  if (rc) return rc;
  rc = traj_prepare(ctx, p, std::max(L, 1), max_dh, step_mode, factor, eps, momentum, seed, u);
  if (rc) return rc;
  if (L >= 1 && !ctx->rec_on) {  // the whole launch sequence, as one graph launch or launch by launch
    if (ctx->graph_replay) {
      rc = traj_replay(ctx, p, L);
    } else {
      rc = traj_launches(ctx, p, L);
      mark_predictions(ctx, p, true);
    }
    if (rc) return rc;
    CK(hipStreamSynchronize(ctx->stream));
    return hmc_outputs(ctx, branches, nb, L, status_out, h_trace_out, uturn_out, log_density_out);
  }
  rc = run_grad(ctx, p, L == 0 ? 1 : 2);  // f(theta_0) -> pred0 (restore copy of a rejected branch)
  if (rc) return rc;
  if (L == 0) {  // empty leapfrog loop: accept_or_reject at the initial state accepts
    run_update(ctx, p, MODE_GRAD, 0);
    CK(hipGetLastError());
    CK(hipStreamSynchronize(ctx->stream));
    for (int i = 0; i < nb; ++i) {
      if (status_out) status_out[i] = BANN_ACCEPTED;
      if (uturn_out) uturn_out[i] = -1;
    }
    if (log_density_out)
      for (int i = 0; i < nb; ++i)
        CK(hipMemcpy(log_density_out + i, ctx->d_ld + branches[i], sizeof(double), hipMemcpyDeviceToHost));
    return BANN_OK;
  }
  run_update(ctx, p, MODE_INIT, 0);
  if (ctx->rec_on) {  // params[k-1] = theta_k (after the k-th position step), ldg[k-1] = its gradient
    ctx->rec.resize(ctx->br.size());
    for (int i = 0; i < nb; ++i) {
      auto& R = ctx->rec[branches[i]];
      R.q = 0;
      R.prec.clear();
      R.params.assign((size_t)L * ctx->br[branches[i]].P, 0.f);
      R.ldg.assign((size_t)L * ctx->br[branches[i]].P, 0.f);
    }
  }
  for (int k = 1; k <= L; ++k) {
    rc = run_grad(ctx, p, k == L ? 1 : 0);
    if (rc) return rc;
    if (ctx->rec_on)
      for (int i = 0; i < nb; ++i) {
        const BranchHost& h = ctx->br[branches[i]];
        CK(hipMemcpyAsync(ctx->rec[branches[i]].params.data() + (size_t)(k - 1) * h.P, ctx->d_theta + h.dev.p_off,
                          h.P * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
      }
    run_update(ctx, p, k < L ? MODE_STEP : MODE_LAST, k);
    if (ctx->rec_on)
      for (int i = 0; i < nb; ++i) {
        const BranchHost& h = ctx->br[branches[i]];
        CK(hipMemcpyAsync(ctx->rec[branches[i]].ldg.data() + (size_t)(k - 1) * h.P, ctx->d_grad + h.dev.p_off,
                          h.P * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
      }
  }
  // rejected branches are back at theta_0: their prediction rows go back to f(theta_0)
  launch_restore_pred(ctx->st, p.d_all, nb, ctx->stream);
  mark_predictions(ctx, p, true);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(ctx->stream));
  if (ctx->rec_on) {
    const int rc2 = rec_finish(ctx, branches, nb, L);
    if (rc2) return rc2;
  }
  return hmc_outputs(ctx, branches, nb, L, status_out, h_trace_out, uturn_out, log_density_out);
}

// The sequential driver's branch-update tail in ONE host wait (bann_net.cpp update_branch;
// net.rs:286-300): bann_hmc_step's trajectory for branch b, then -- stream-ordered, not
// waited for -- residual_from_target_shift's residual op (residual = target - f_b(final) +
// add) and the copies of the trajectory status and the final parameters into pinned
// stages: one stream synchronisation instead of three waits and two synchronous copies
// (profiles/r06_seq_api.txt).  The same launches in the same order as bann_hmc_step +
// bann_branch_get_params + residual_from_target_shift, hence the same bits.  stats: sum
// and sum of squares of the residual before and after the shift.  A recording context and
// L = 0 take those three calls as they are.
int hmc_step_tail(bann_ctx* ctx, int32_t b, int32_t L, float max_dh, int32_t step_mode, float factor, const float* eps,
                  const float* momentum, uint64_t seed, const float* u, float add, int32_t* status_out,
                  float* params_out, double* stats) {
  if (!ctx || !ctx->finalized) return fail(ctx, BANN_E_STATE, "not finalized");
  if (!status_out || !params_out || !stats) return fail(ctx, BANN_E_ARG, "null output");
  if (L < 1 || ctx->rec_on) {
    int rc = bann_hmc_step(ctx, &b, 1, L, max_dh, step_mode, factor, eps, momentum, seed, u, status_out, nullptr,
                           nullptr, nullptr);
    if (rc) return rc;
    rc = bann_branch_get_params(ctx, b, params_out);
    if (rc) return rc;
    return residual_from_target_shift(ctx, b, add, &stats[0], &stats[1], &stats[2], &stats[3]);
  }
  if (!check_branch(ctx, b)) return fail(ctx, BANN_E_ARG, "bad branch");
  if (ctx->lf_active) return fail(ctx, BANN_E_STATE, "a leapfrog session is active");
  Plan p;
  int rc = build_plan(ctx, &b, 1, p, false);
  if (rc) return rc;
  rc = traj_prepare(ctx, p, L, max_dh, step_mode, factor, eps, momentum, seed, u);
  if (rc) return rc;
  if (ctx->graph_replay) {
    rc = traj_replay(ctx, p, L);
  } else {
    rc = traj_launches(ctx, p, L);
    mark_predictions(ctx, p, true);
  }
  if (rc) return rc;
  rc = residual_from_target_shift_launch(ctx, b, add);
  if (rc) return rc;
  const BranchHost& h = ctx->br[b];
  CK(hipMemcpyAsync(ctx->h_status + b, ctx->d_status + b, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipMemcpyAsync(ctx->h_par_stage, ctx->d_theta + h.dev.p_off, h.P * sizeof(float), hipMemcpyDeviceToHost,
                    ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  *status_out = ctx->h_status[b];
  std::memcpy(params_out, ctx->h_par_stage, h.P * sizeof(float));
  for (int k = 0; k < 4; ++k) stats[k] = ctx->h_res_stat[k];
  return BANN_OK;
}

// hmc_step_joint (branch_sampler.rs:1070-1178): parameters AND precisions
extern "C" int bann_hmc_step_joint(bann_ctx* ctx, const int32_t* branches, int32_t nb, int32_t L, float max_dh,
                                   int32_t step_mode, float factor, const float* eps, const float* momentum,
                                   uint64_t seed, const float* u, const float* hyper, int32_t* status_out,
                                   double* h_trace_out, double* log_density_out) {
  if (!ctx || !ctx->finalized) return fail(ctx, BANN_E_STATE, "not finalized");
  if (!branches || nb <= 0 || L < 1 || !hyper) return fail(ctx, BANN_E_ARG, "bad branch list, L or hyperparameters");
  if (ctx->lf_active) return fail(ctx, BANN_E_STATE, "a leapfrog session is active");
  if (step_mode == BANN_STEP_INJECTED && !eps) return fail(ctx, BANN_E_ARG, "injected step sizes need eps");
  Plan p;
  int rc = build_plan(ctx, branches, nb, p, false);
  if (rc) return rc;
  int32_t max_q = 0;
  for (int i = 0; i < nb; ++i) {
    const BranchHost& h = ctx->br[branches[i]];
    if (h.prior == BANN_STD_NORMAL)
      return fail(ctx, BANN_E_ARG, "std_normal has no joint density (std_normal_branch.rs:119-131)");
    if (h.dev.nq > BANN_JOINT_MAXQ) return fail(ctx, BANN_E_SHAPE, "too many precisions for the joint update");
    max_q = std::max(max_q, h.dev.nq);
  }
  rc = ensure_htrace(ctx, L);
  if (rc) return rc;
  for (int k = 0; k < 6; ++k) ctx->st.hyper[k] = hyper[k];
  ctx->st.max_dh = max_dh;
  ctx->st.lint = ctx->htrace_cap - 1;
  // host staging: precision coordinates, output-weight stats, step sizes, momenta, uniforms
  std::vector<float> ows(2 * ctx->br.size(), 0.f), ep, mo, uu(ctx->br.size(), 0.f);
  std::mt19937_64 rng(seed ^ 0x5DEECE66Dull);
  std::uniform_real_distribution<float> U(0.f, 1.f);
  int64_t off = 0;
  for (int i = 0; i < nb; ++i) {
    const int b = branches[i];
    const BranchHost& h = ctx->br[b];
    const int P = h.P, Q = h.dev.nq;
    CK(hipMemcpyAsync(ctx->d_phi + h.dev.q_off, h.prec.data(), Q * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
    ows[2 * b] = h.ows_reg_sum;
    ows[2 * b + 1] = h.ows_num >= 0.f ? h.ows_num : (float)h.widths[h.L - 2];
    if (step_mode == BANN_STEP_INJECTED) {
      ep.assign(eps + off, eps + off + P + Q);
    } else {  // random_step_sizes (654-704): U(0,1) (P + Q)^-1/4 c -- the joint sampler's only mode (1092-1101)
      ep.resize(P + Q);
      const float f = powf((float)(P + Q), -0.25f) * factor;
      for (auto& e : ep) e = U(rng) * f;
    }
    CK(hipMemcpyAsync(ctx->d_eps + h.dev.p_off, ep.data(), P * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
    CK(hipMemcpyAsync(ctx->d_ephi + h.dev.q_off, ep.data() + P, Q * sizeof(float), hipMemcpyHostToDevice,
                      ctx->stream));
    if (momentum) {
      CK(hipMemcpyAsync(ctx->d_mom + h.dev.p_off, momentum + off, P * sizeof(float), hipMemcpyHostToDevice,
                        ctx->stream));
      CK(hipMemcpyAsync(ctx->d_mphi + h.dev.q_off, momentum + off + P, Q * sizeof(float), hipMemcpyHostToDevice,
                        ctx->stream));
    }
    uu[b] = u ? u[i] : U(rng);
    off += P + Q;
    CK(hipStreamSynchronize(ctx->stream));  // ep is reused
  }
  CK(hipMemcpyAsync(ctx->d_ows, ows.data(), ows.size() * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
  CK(hipMemcpyAsync(ctx->d_u, uu.data(), uu.size() * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
  if (!momentum) {
    launch_sample_momentum(ctx->st, p.d_all, nb, p.max_p, seed, ctx->stream);
    launch_sample_momentum_joint(ctx->st, p.d_all, nb, max_q, seed, ctx->stream);
  }
  CK(hipMemsetAsync(ctx->d_htrace, 0xFF, ctx->br.size() * ctx->htrace_cap * sizeof(double), ctx->stream));
  mark_predictions(ctx, p, false);  // theta moves (launch_update_joint does not go through run_update)
  if (ctx->rec_on) {  // the joint Trajectory (1126-1135): params, precisions, joint ldg [params | precisions], -H
    ctx->rec.resize(ctx->br.size());
    for (int i = 0; i < nb; ++i) {
      auto& R = ctx->rec[branches[i]];
      const BranchHost& h = ctx->br[branches[i]];
      R.q = h.dev.nq;
      R.params.assign((size_t)L * h.P, 0.f);
      R.prec.assign((size_t)L * R.q, 0.f);
      R.ldg.assign((size_t)L * (h.P + R.q), 0.f);
    }
  }
  rc = run_grad(ctx, p, 2);  // f(theta_0) -> pred0
  if (rc) return rc;
  launch_update_joint(ctx->st, p.d_all, nb, MODE_INIT, 0, ctx->stream);
  for (int k = 1; k <= L; ++k) {
    rc = run_grad(ctx, p, k == L ? 1 : 0);
    if (rc) return rc;
    if (ctx->rec_on)  // (theta_k, phi_k) after the k-th position step
      for (int i = 0; i < nb; ++i) {
        const BranchHost& h = ctx->br[branches[i]];
        auto& R = ctx->rec[branches[i]];
        CK(hipMemcpyAsync(R.params.data() + (size_t)(k - 1) * h.P, ctx->d_theta + h.dev.p_off, h.P * sizeof(float),
                          hipMemcpyDeviceToHost, ctx->stream));
        CK(hipMemcpyAsync(R.prec.data() + (size_t)(k - 1) * R.q, ctx->d_phi + h.dev.q_off, R.q * sizeof(float),
                          hipMemcpyDeviceToHost, ctx->stream));
      }
    launch_update_joint(ctx->st, p.d_all, nb, k < L ? MODE_STEP : MODE_LAST, k, ctx->stream);
    if (ctx->rec_on)  // the joint log-density gradient there
      for (int i = 0; i < nb; ++i) {
        const BranchHost& h = ctx->br[branches[i]];
        auto& R = ctx->rec[branches[i]];
        float* row = R.ldg.data() + (size_t)(k - 1) * (h.P + R.q);
        CK(hipMemcpyAsync(row, ctx->d_grad + h.dev.p_off, h.P * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
        CK(hipMemcpyAsync(row + h.P, ctx->d_gphi + h.dev.q_off, R.q * sizeof(float), hipMemcpyDeviceToHost,
                          ctx->stream));
      }
  }
  launch_restore_pred(ctx->st, p.d_all, nb, ctx->stream);  // rejected: predictions back to f(theta_0)
  mark_predictions(ctx, p, true);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(ctx->stream));
  if (ctx->rec_on) {
    rc = rec_finish(ctx, branches, nb, L);
    if (rc) return rc;
  }
  const int stride = ctx->htrace_cap;
  for (int i = 0; i < nb; ++i) {
    const int b = branches[i];
    BranchHost& h = ctx->br[b];
    if (status_out) CK(hipMemcpy(status_out + i, ctx->d_status + b, sizeof(int32_t), hipMemcpyDeviceToHost));
    if (log_density_out) CK(hipMemcpy(log_density_out + i, ctx->d_ld + b, sizeof(double), hipMemcpyDeviceToHost));
    if (h_trace_out)
      CK(hipMemcpy(h_trace_out + (int64_t)i * (L + 1), ctx->d_htrace + (int64_t)b * stride, (L + 1) * sizeof(double),
                   hipMemcpyDeviceToHost));
    // the sampled precisions become the branch's precisions (host copy and derived device arrays)
    CK(hipMemcpy(h.prec.data(), ctx->d_phi + h.dev.q_off, h.dev.nq * sizeof(float), hipMemcpyDeviceToHost));
    rc = upload_precisions(ctx, b);
    if (rc) return rc;
  }
  return BANN_OK;
}

extern "C" int bann_set_trajectory_recording(bann_ctx* ctx, int32_t enabled) {
  if (!ctx) return BANN_E_ARG;
  ctx->rec_on = enabled != 0;
  return BANN_OK;
}

extern "C" int bann_branch_get_trajectory(bann_ctx* ctx, int32_t b, int32_t cap, int32_t* steps, float* params,
                                          float* ldg, double* hamiltonian) {
  if (!check_branch(ctx, b)) return fail(ctx, BANN_E_ARG, "bad branch");
  if (b >= (int32_t)ctx->rec.size() || ctx->rec[b].h.empty()) return fail(ctx, BANN_E_STATE, "no recorded trajectory");
  const auto& R = ctx->rec[b];
  if (R.q) return fail(ctx, BANN_E_STATE, "the last recorded trajectory is joint (bann_branch_get_trajectory_joint)");
  const int64_t P = ctx->br[b].P;
  const int32_t k = std::min(cap, R.steps);
  if (steps) *steps = R.steps;
  if (params) std::copy(R.params.begin(), R.params.begin() + k * P, params);
  if (ldg) std::copy(R.ldg.begin(), R.ldg.begin() + k * P, ldg);
  if (hamiltonian) std::copy(R.h.begin(), R.h.begin() + k + 1, hamiltonian);
  return BANN_OK;
}

extern "C" int bann_branch_get_trajectory_joint(bann_ctx* ctx, int32_t b, int32_t cap, int32_t* steps, float* params,
                                                float* precisions, float* ldg, double* hamiltonian) {
  if (!check_branch(ctx, b)) return fail(ctx, BANN_E_ARG, "bad branch");
  if (b >= (int32_t)ctx->rec.size() || ctx->rec[b].h.empty()) return fail(ctx, BANN_E_STATE, "no recorded trajectory");
  const auto& R = ctx->rec[b];
  if (!R.q) return fail(ctx, BANN_E_STATE, "the last recorded trajectory is not joint (bann_branch_get_trajectory)");
  const int64_t P = ctx->br[b].P, Q = R.q;
  const int32_t k = std::min(cap, R.steps);
  if (steps) *steps = R.steps;
  if (params) std::copy(R.params.begin(), R.params.begin() + k * P, params);
  if (precisions) std::copy(R.prec.begin(), R.prec.begin() + k * Q, precisions);
  if (ldg) std::copy(R.ldg.begin(), R.ldg.begin() + k * (P + Q), ldg);
  if (hamiltonian) std::copy(R.h.begin(), R.h.begin() + k + 1, hamiltonian);
  return BANN_OK;
}

// ---- in-trajectory launch timing (bann_set_launch_timing) ----
// an event at every launch boundary: TM_GRAD0 before a gradient launch, TM_GRAD1
// between the gradient and the update launch, TM_UPD1 after the update; network
// mode adds TM_FWD0/1 around the forward launch and TM_AR0/1 around the all-reduce
void tm_mark(bann_ctx* ctx, int32_t kind) {
  if (!ctx->tm_on) return;
  // the next unused event of the pool (a follow mark reuses its predecessor's event)
  const size_t k = ctx->tm_marks.empty() ? 0 : (size_t)ctx->tm_marks.back().first + 1;
  if (k == ctx->tm_pool.size()) {
    hipEvent_t e;
    // timing only (resolved after a stream synchronisation): no system-scope fence on
    // record -- with it every mark wrote back and invalidated the caches between two
    // launches (the N = 8 shard's line: 4 477 vs 4 656 steps/s with marks vs without)
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return;  // best effort: no sample
    ctx->tm_pool.push_back(e);
  }
  if (hipEventRecord(ctx->tm_pool[k], ctx->stream) != hipSuccess) return;
  ctx->tm_marks.push_back({(int32_t)k, kind});
}

// after the stream has drained: elapsed time of every (start, end) pair of marks
// a mark that starts where the previous mark (an update's end) left off, with nothing
// enqueued in between: the same event, no second record on the stream
void tm_mark_follow(bann_ctx* ctx, int32_t kind) {
  if (!ctx->tm_on) return;
  if (!ctx->tm_marks.empty() && ctx->tm_marks.back().second == TM_UPD1) {
    ctx->tm_marks.push_back({ctx->tm_marks.back().first, kind});
    return;
  }
  tm_mark(ctx, kind);
}

int tm_resolve(bann_ctx* ctx) {
  for (size_t i = 0; i + 1 < ctx->tm_marks.size(); ++i) {
    const auto a = ctx->tm_marks[i], b = ctx->tm_marks[i + 1];
    double* acc = nullptr;
    int32_t* cnt = nullptr;
    if (a.second == TM_GRAD0 && b.second == TM_GRAD1) acc = &ctx->tm_grad_ms, cnt = &ctx->tm_grad_n;
    else if (a.second == TM_GRAD1 && b.second == TM_UPD1) acc = &ctx->tm_upd_ms, cnt = &ctx->tm_upd_n;
    else if (a.second == TM_FWD0 && b.second == TM_FWD1) acc = &ctx->tm_fwd_ms, cnt = &ctx->tm_fwd_n;
    else if (a.second == TM_AR0 && b.second == TM_AR1) acc = &ctx->tm_ar_ms, cnt = &ctx->tm_ar_n;
    if (!acc) continue;
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, ctx->tm_pool[a.first], ctx->tm_pool[b.first]));
    *acc += ms;
    ++*cnt;
  }
  ctx->tm_marks.clear();
  return BANN_OK;
}

extern "C" int bann_set_launch_timing(bann_ctx* ctx, int32_t enabled) {
  if (!ctx) return BANN_E_ARG;
  if (ctx->lf_active) return fail(ctx, BANN_E_STATE, "a leapfrog session is active");
  ctx->tm_on = enabled != 0;
  ctx->tm_marks.clear();
  return BANN_OK;
}

extern "C" int bann_launch_timing(bann_ctx* ctx, float* grad_ms, float* update_ms, int32_t* grad_launches,
                                  int32_t reset) {
  if (!ctx) return BANN_E_ARG;
  if (grad_ms) *grad_ms = ctx->tm_grad_n ? (float)(ctx->tm_grad_ms / ctx->tm_grad_n) : 0.f;
  if (update_ms) *update_ms = ctx->tm_upd_n ? (float)(ctx->tm_upd_ms / ctx->tm_upd_n) : 0.f;
  if (grad_launches) *grad_launches = ctx->tm_grad_n;
  if (reset) {
    ctx->tm_grad_ms = ctx->tm_upd_ms = 0.0;
    ctx->tm_grad_n = ctx->tm_upd_n = 0;
  }
  return BANN_OK;
}

extern "C" int bann_network_timing(bann_ctx* ctx, float* forward_ms, float* allreduce_ms, int32_t* allreduces,
                                   int32_t reset) {
  if (!ctx) return BANN_E_ARG;
  if (forward_ms) *forward_ms = ctx->tm_fwd_n ? (float)(ctx->tm_fwd_ms / ctx->tm_fwd_n) : 0.f;
  if (allreduce_ms) *allreduce_ms = ctx->tm_ar_n ? (float)(ctx->tm_ar_ms / ctx->tm_ar_n) : 0.f;
  if (allreduces) *allreduces = ctx->tm_ar_n;
  if (reset) {
    ctx->tm_fwd_ms = ctx->tm_ar_ms = 0.0;
    ctx->tm_fwd_n = ctx->tm_ar_n = 0;
  }
  return BANN_OK;
}

extern "C" int64_t bann_ctx_num_individuals(const bann_ctx* ctx) { return ctx ? ctx->n : BANN_E_ARG; }

// one leapfrog step of a session: the gradient launch and the update (fused into
// the gradient launch's tail for a fuse_update plan; launch timing then books
// both on the gradient)
static int grad_update(bann_ctx* ctx, const Plan& p, int write_pred, int mode, int step) {
  if (p.fuse_update) {
    mark_predictions(ctx, p, false);  // theta moves
    int rc = run_grad(ctx, p, write_pred, mode, step);
    tm_mark(ctx, TM_GRAD1);
    return rc;
  }
  int rc = run_grad(ctx, p, write_pred);
  if (rc) return rc;
  tm_mark(ctx, TM_GRAD1);
  run_update(ctx, p, mode, step);
  return BANN_OK;
}

extern "C" int bann_leapfrog_begin(bann_ctx* ctx, const int32_t* branches, int32_t nb, int32_t L, float max_dh,
                                   int32_t step_mode, float factor, uint64_t seed) {
  if (!ctx || !ctx->finalized) return fail(ctx, BANN_E_STATE, "not finalized");
  if (ctx->lf_active) return fail(ctx, BANN_E_STATE, "a leapfrog session is already active (call bann_leapfrog_end)");
  if (!branches || nb <= 0 || L < 1) return fail(ctx, BANN_E_ARG, "bad branch list or L");
  int rc = BANN_OK;
  // the packed launch plan of a branch set is reused across trajectories (a sweep
  // runs the same set every time); rebuild only when the set changes
  if (!(ctx->lf.owns && ctx->lf.all.size() == (size_t)nb && std::equal(branches, branches + nb, ctx->lf.all.begin()))) {
    rc = build_plan(ctx, branches, nb, ctx->lf, true);
    if (rc) return rc;
  }
  rc = traj_prepare(ctx, ctx->lf, L, max_dh, step_mode, factor, nullptr, nullptr, seed, nullptr);
  if (rc) return rc;
  tm_mark(ctx, TM_GRAD0);
  rc = grad_update(ctx, ctx->lf, 2, MODE_INIT, 0);  // f(theta_0) straight into pred0 (the restore copy and the residual change)
  if (rc) return rc;
  tm_mark(ctx, TM_UPD1);
  CK(hipGetLastError());
  ctx->lf_active = true;
  ctx->lf_L = L;
  ctx->lf_step = 0;
  return BANN_OK;
}

extern "C" int bann_leapfrog_steps(bann_ctx* ctx, int32_t k) {
  if (!ctx || !ctx->lf_active) return fail(ctx, BANN_E_STATE, "no leapfrog session");
  if (k < 0 || ctx->lf_step + k > ctx->lf_L) return fail(ctx, BANN_E_ARG, "steps beyond the trajectory length");
  for (int i = 0; i < k; ++i) {
    const int step = ++ctx->lf_step;
    // the previous step's end -- within this call only: between calls the caller may
    // have enqueued work of its own, so a call's first step records a fresh mark
    if (i == 0)
      tm_mark(ctx, TM_GRAD0);
    else
      tm_mark_follow(ctx, TM_GRAD0);
    int rc = grad_update(ctx, ctx->lf, step == ctx->lf_L ? 1 : 0, step < ctx->lf_L ? MODE_STEP : MODE_LAST, step);
    if (rc) return rc;
    tm_mark(ctx, TM_UPD1);
  }
  CK(hipGetLastError());
  return BANN_OK;
}

extern "C" int bann_leapfrog_end(bann_ctx* ctx, int32_t* status_out, int32_t* num_accepted) {
  if (!ctx || !ctx->lf_active) return fail(ctx, BANN_E_STATE, "no leapfrog session");
  if (ctx->lf_step != ctx->lf_L) {
    int rc = bann_leapfrog_steps(ctx, ctx->lf_L - ctx->lf_step);
    if (rc) return rc;
  }
  // rejected branches were restored to theta_0: their prediction rows go back to f(theta_0)
  launch_restore_pred(ctx->st, ctx->lf.d_all, (int32_t)ctx->lf.all.size(), ctx->stream);
  mark_predictions(ctx, ctx->lf, true);
  CK(hipMemcpyAsync(ctx->h_status, ctx->d_status, ctx->br.size() * sizeof(int32_t), hipMemcpyDeviceToHost,
                    ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  {
    int rc = tm_resolve(ctx);
    if (rc) return rc;
  }
  const int32_t* st = ctx->h_status;
  int acc = 0;
  for (size_t i = 0; i < ctx->lf.all.size(); ++i) {
    const int s = st[ctx->lf.all[i]];
    if (status_out) status_out[i] = s;
    acc += s == BANN_ACCEPTED;
  }
  if (num_accepted) *num_accepted = acc;
  ctx->lf_active = false;
  return BANN_OK;
}

extern "C" int bann_leapfrog_residual_delta_device(bann_ctx* ctx, float* out_device) {
  if (!ctx || !out_device) return BANN_E_ARG;
  if (ctx->lf.all.empty() || ctx->lf_active) return fail(ctx, BANN_E_STATE, "call after bann_leapfrog_end");
  launch_residual_delta(ctx->st, ctx->lf.d_all, (int32_t)ctx->lf.all.size(), ctx->d_delta_part, out_device,
                        ctx->stream);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(ctx->stream));
  return BANN_OK;
}

extern "C" int bann_leapfrog_residual_delta(bann_ctx* ctx, float* out_host) {
  if (!ctx || !out_host) return BANN_E_ARG;
  if (ctx->lf.all.empty() || ctx->lf_active) return fail(ctx, BANN_E_STATE, "call after bann_leapfrog_end");
  launch_residual_delta(ctx->st, ctx->lf.d_all, (int32_t)ctx->lf.all.size(), ctx->d_delta_part, ctx->d_delta,
                        ctx->stream);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(ctx->h_delta, ctx->d_delta, ctx->n * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  memcpy(out_host, ctx->h_delta, ctx->n * sizeof(float));
  return BANN_OK;
}

extern "C" int bann_leapfrog_predictions_device(bann_ctx* ctx, float** out) {
  if (!ctx || !out) return BANN_E_ARG;
  if (ctx->lf_active) return fail(ctx, BANN_E_STATE, "predictions are current after bann_leapfrog_end");
  *out = ctx->d_pred;
  return BANN_OK;
}

extern "C" int bann_profile_session(bann_ctx* ctx, int32_t iters, float* grad_ms, float* update_ms) {
  if (!ctx || !ctx->lf_active) return fail(ctx, BANN_E_STATE, "no leapfrog session");
  if (iters <= 0) return fail(ctx, BANN_E_ARG, "iters must be positive");
  hipEvent_t e0, e1, e2;
  CK(hipEventCreateWithFlags(&e0, hipEventDisableSystemFence));  // timing only
  CK(hipEventCreateWithFlags(&e1, hipEventDisableSystemFence));
  CK(hipEventCreateWithFlags(&e2, hipEventDisableSystemFence));
  CK(hipEventRecord(e0, ctx->stream));
  for (int i = 0; i < iters; ++i) {
    int rc = run_grad(ctx, ctx->lf, 0);
    if (rc) return rc;
  }
  CK(hipEventRecord(e1, ctx->stream));
  for (int i = 0; i < iters; ++i) run_update(ctx, ctx->lf, MODE_PROFILE, 1);
  CK(hipEventRecord(e2, ctx->stream));
  CK(hipEventSynchronize(e2));
  float t01 = 0.f, t12 = 0.f;
  CK(hipEventElapsedTime(&t01, e0, e1));
  CK(hipEventElapsedTime(&t12, e1, e2));
  if (grad_ms) *grad_ms = t01 / iters;
  if (update_ms) *update_ms = t12 / iters;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipEventDestroy(e2);
  return BANN_OK;
}
