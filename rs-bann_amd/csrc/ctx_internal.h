// ctx_internal.h — the bann_ctx context and the host helpers shared by the C-ABI
// translation units (bann_api.hip: single-GPU API; bann_dist.hip: multi-GPU).
#pragma once
#include <hip/hip_runtime.h>

#include <random>
#include <string>
#include <vector>

#include "../../include/bann.h"
#include "bann_internal.h"

struct BranchHost {
  std::vector<int32_t> snp_idx;
  std::vector<int32_t> widths;
  int32_t m = 0, L = 0, act = 0, prior = 0;
  int32_t P = 0, nprec = 0;
  std::vector<float> prec;  // precision_vec order
  float ows_reg_sum = 0.f;  // output-weight summary stat of the OTHER branches (joint HMC)
  float ows_num = -1.f;     // output-weight count of the network (< 0: this branch's own)
  int32_t gx_group = -1;    // gx path: scratch group (branches of one group share no scratch)
  int32_t solo_items = 1;   // fused path: work items of the branch in a solo-mode plan (~1 tile per wave)
  BranchDev dev{};
};

// one packed gradient launch: every work item of one kernel instantiation
struct LaunchGroup {
  int32_t kind = 0;  // BranchDev::fused of its branches: 1 fx, 3 fxl, 2 wx
  int32_t L = 0, act = 0, nw = 1, full = 0;
  int32_t cpw = 8;      // fxl: marker chunks per wave (fxl_cpw)
  int32_t head = 0;     // fxl: the head-wave kernel fxh where its shape allows (bann_ctx::fxl_head)
  int64_t tiles = 0;    // fx: the items' 64-individual tiles (the fi forward's index space, GradItem::tile0)
  int32_t max_seg = 1;  // fx: the largest 256-marker segment count of its branches
  bool fi = false;      // fx: every branch has an individual-major fi image (kernels_fi.hip)
  std::vector<GradItem> items;
  GradItem* d_items = nullptr;
  // network mode, fx groups of 8-chunk branches: k_forward_gsum's group items (build_net_groups)
  std::vector<NetGroupItem> nitems;
  NetGroupItem* d_nitems = nullptr;
  std::vector<int32_t> nlist;  // the items' branch lists
  int32_t* d_nlist = nullptr;
};

// gx path (kernels_gx.hip): the GEMM phases of one scratch group, each over a
// tile-count prefix array of the group's branches
struct GxPhase {
  int32_t ph = 0, l = 0, total = 0, pre_off = 0;
};
struct GxGroup {
  int32_t first = 0, count = 0, max_splits = 1;  // branches p.gx[first .. first + count)
  std::vector<GxPhase> phases;                    // in launch order; GX_HEAD marks the head kernel
};

struct Plan {
  std::vector<int32_t> all, gx;
  int32_t n_small = 0, n_large = 0;  // update kernels: d_all[nb .. nb+n_small) small, then n_large large
  std::vector<LaunchGroup> groups;
  std::vector<GxGroup> gxg;
  std::vector<int32_t> gx_pre;       // concatenated tile prefix arrays of the gx phases
  std::vector<FoldJob> fold;         // solo mode: per fused branch, its solo slabs -> its slab 0
  FoldJob* d_fold = nullptr;
  int32_t max_p = 0;
  int32_t* d_all = nullptr;
  int32_t* d_gx = nullptr;
  int32_t* d_gxpre = nullptr;
  bool owns = false;
  // every branch fx-shaped with the small update (P <= 2048, m <= 512), one round of
  // work items, no solo re-split: the leapfrog session runs the update in the
  // gradient launch's tail (kernels_fx.hip, BANN_FUSE_UPDATE=0: separate launches)
  bool fuse_update = false;
  // network mode: the forward writes group sums (k_forward_gsum) into nsum_rows rows of
  // bann_ctx::d_gsum (build_net_groups; nsum_built: tried, nsum_rows > 0: usable)
  bool nsum_built = false;
  int32_t nsum_rows = 0;
};

struct bann_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  // genotypes
  int64_t n = 0, M = 0;
  uint8_t* d_g = nullptr;  // 2-bit variant-major genotype image (kernels_data.hip), rowb bytes per marker
  int64_t rowb = 0;
  float* d_mu = nullptr;
  float* d_sigma = nullptr;
  // branches
  std::vector<BranchHost> br;
  bool finalized = false;
  bool fused_enabled = true;
  bool wide_bf16 = false;
  bool fxl_head = true;    // fxl groups of 17..32 chunks on the head-wave kernel (BANN_FXL_HEAD=0 at creation: off)  // wx kernel: hidden GEMMs on bf16 MFMA (opt-in, reduced precision)
  int32_t nfrag = 0, max_splits = 1;
  int64_t packed_bytes = 0, total_p = 0;
  // device buffers
  BranchDev* d_br = nullptr;
  uint8_t* d_xu2 = nullptr;  // 2-bit genotype tile images of every branch (u2t, kernels_fx.hip)
  uint8_t* d_xi = nullptr;   // individual-major 2-bit images of the fx branches (kernels_fi.hip; BANN_FWD_FI=0: none)
  int64_t xi_bytes = 0;
  int32_t cus = 256;
  int32_t* d_upd_cnt = nullptr;  // per-branch arrival counters of the fused update (zero between launches)
  // the update in the gradient launch's tail (BANN_FUSE_UPDATE=1; same bits either way):
  // one-split plans (the branch's one workgroup), one-round multi-split plans and solo
  // plans (the last arriving workgroup; solo: it folds the branch's slabs first).  Off
  // by default: measured slower everywhere (r4c: C3 747.7 vs 752.9 steps/s, N = 8 shard
  // 4 269 vs 4 531, sequential driver 6.5 vs 21.9 -- one workgroup adding 49 slabs)
  int fuse_update_mode = 0;
  uint8_t* d_dig = nullptr;
  FusedConst* d_fc = nullptr;
  float *d_mub = nullptr, *d_sigb = nullptr;
  float *d_theta = nullptr, *d_mom = nullptr, *d_eps = nullptr, *d_theta0 = nullptr, *d_lam = nullptr,
        *d_lamld = nullptr, *d_grad = nullptr, *d_part = nullptr;
  double* d_rss_part = nullptr;
  float* d_pred0 = nullptr;
  double* d_stepbase = nullptr;  // per-parameter Izmailov step base (sign: factor applies)
  float *d_phi = nullptr, *d_phi0 = nullptr, *d_mphi = nullptr, *d_ephi = nullptr, *d_gphi = nullptr;  // joint HMC
  int32_t* d_pidx = nullptr;
  float* d_ows = nullptr;
  int64_t total_q = 0;
  float* d_delta = nullptr;       // n floats: residual change of the last trajectory (host-copy variant)
  float* d_delta_part = nullptr;  // per-branch-slice partial rows of the residual change
  int32_t* h_status = nullptr;    // pinned host mirrors (trajectory status, residual change)
  float* h_par_stage = nullptr;   // pinned: one branch's parameters (hmc_step_tail), max P floats
  float* h_delta = nullptr;
  float *d_y = nullptr, *d_pred = nullptr, *d_scr = nullptr, *d_eprec = nullptr, *d_u = nullptr;
  double *d_h0 = nullptr, *d_htrace = nullptr, *d_ld = nullptr, *d_rss = nullptr;
  int32_t *d_status = nullptr, *d_uturn = nullptr;
  int32_t htrace_cap = 0;  // L+1 capacity of d_htrace rows
  // scratch plan buffers (per-call plans)
  int32_t* d_list_scr = nullptr;
  int32_t* d_gen_scr = nullptr;   // gx branch list of a per-call plan
  int32_t* d_gxpre_scr = nullptr; // its tile prefix arrays (gxpre_cap ints)
  int64_t gxpre_cap = 0;
  FoldJob* d_fold_scr = nullptr;   // fold jobs of a per-call plan (one per branch)
  // solo mode: a plan whose fused branches give too few work items to fill the
  // GPU (e.g. the sequential driver's one-branch trajectories) re-splits them
  // into solo_items each, writing into the solo region after the branch slabs
  int64_t part_total = 0, solo_part_cap = 0, solo_rss_cap = 0;
  int32_t solo_threshold = 256;    // normal work items below which a plan goes solo
  GradItem* d_items_scr = nullptr;
  unsigned long long* d_dbg = nullptr;  // BANN_STAMPS diagnostics
  int64_t items_cap = 0;
  // multi-GPU: one rank per GPU (bann_dist.hip)
  int32_t comm_kind = 0;  // 0 none, 1 RCCL, 2 caller all-reduce callback
  int32_t nranks = 1, rank = 0;
  void* nccl = nullptr;   // ncclComm_t
  bann_allreduce_fn ar_fn = nullptr;
  void* ar_user = nullptr;
  float* d_gsum = nullptr;     // network mode: per-group output sums of the fx branches (gsum_cap rows of n)
  int32_t gsum_cap = 0;
  bool net_gsum = true;        // BANN_NET_GSUM=0 at creation: per-branch output rows in every step (A/B)
  float* d_netsum = nullptr;   // network mode: n-vector sum of the local branch outputs, then the error e
  float* d_nety = nullptr;     // network mode: the targets y
  double* d_netrss = nullptr;  // network mode: global rss per leapfrog step (netrss_cap entries)
  double* d_netpart = nullptr; // network mode: rss block partials
  int32_t netrss_cap = 0;
  // network mode: the common-mode step-size rule (bann_set_network_step_rule)
  // 0 off, 1 adapt before every trajectory (diagnostic: state-dependent proposals), 2 frozen,
  // 3 auto (default): adapt on the first cm_adapt_total trajectories, then frozen
  int32_t cm_rule = 3;
  int32_t cm_adapt_total = 1, cm_adapted = 0;  // auto mode: adapting trajectories asked / done
  float* d_cm_scale = nullptr;    // the last adapted per-parameter step factors
  bool cm_have_scale = false;
  float cm_tau = 1.0f;
  float* d_ones = nullptr;                 // n ones: the output error of the common-mode gradient launch
  unsigned long long* d_cm = nullptr;      // per-branch histograms (nbranch x 2 CM_NC), then their sum
  double cm_info[4] = {0.0, 0.0, 0.0, 0.0};  // last trajectory: threshold t, bound before / after (omega eps)^2, scaled fraction
  double* d_ar64 = nullptr;    // RCCL all-reduce of host f64 vectors (the network -H trace): reused device buffer
  int64_t ar64_cap = 0;
  // the network residual on the device (bann_residual.hip): n floats, reduction scratch, pinned (sum, sum sq)
  float* d_res = nullptr;
  double* d_res_part = nullptr;
  double* h_res_stat = nullptr;
  double* d_res_stat_host = nullptr;  // the same pinned pair, as the kernels address it
  char* h_prec_stage = nullptr;  // upload_precisions: pinned staging of one branch's precision arrays
  char* d_prec_stage = nullptr;
  size_t prec_stage_cap = 0;
  hipEvent_t ev_prec = nullptr;  // the staging copy of the last upload
  bool prec_ev_pending = false;
  char* d_plan_scr = nullptr;    // one block: d_list_scr | d_fold_scr | d_items_scr (build_plan)
  char* h_plan_stage = nullptr;  // its pinned stage (one copy per per-call plan)
  int64_t plan_scr_bytes = 0, plan_off_fold = 0, plan_off_items = 0;
  hipEvent_t ev_plan = nullptr;
  bool plan_ev_pending = false;
  float* h_u_stage = nullptr;    // traj_prepare: injected acceptance uniforms, pinned
  hipEvent_t ev_u = nullptr;
  bool u_ev_pending = false;
  // pred_ok[b]: the prediction row of branch b is f_b(theta_b) at the current parameters
  std::vector<char> pred_ok;
  // in-trajectory launch timing (bann_set_launch_timing): HIP events around every
  // gradient and update launch of the leapfrog sessions, resolved at bann_leapfrog_end
  bool tm_on = false;
  std::vector<hipEvent_t> tm_pool;
  // (event index, kind): TM_* below; a sample is the span between a kind and its successor kind
  std::vector<std::pair<int32_t, int32_t>> tm_marks;
  double tm_grad_ms = 0.0, tm_upd_ms = 0.0, tm_fwd_ms = 0.0, tm_ar_ms = 0.0;
  int32_t tm_grad_n = 0, tm_upd_n = 0, tm_fwd_n = 0, tm_ar_n = 0;
  // trajectory recording (mcmc_cfg.trajectories, trajectory.rs): per branch of the last bann_hmc_step
  bool rec_on = false;
  struct Rec {
    int32_t steps = 0;
    int32_t q = 0;                   // joint trajectory: precisions per step (0: parameters only)
    std::vector<float> params, ldg;  // [L][P], [L][P + q]
    std::vector<float> prec;         // [L][q]
    std::vector<double> h;           // [L + 1]
  };
  std::vector<Rec> rec;  // indexed by branch
  // captured launch sequences of bann_hmc_step, keyed by plan shape, L and the by-value state
  bool graph_replay = false;  // BANN_HMC_GRAPH=1: replay captured graphs (+5 % sequential; rocprofv3 crashes on them)
  std::vector<std::pair<std::string, hipGraphExec_t>> graphs;
  // leapfrog session
  Plan lf;
  bool lf_active = false;
  int32_t lf_L = 0, lf_step = 0;
  DevState st{};
};


inline int fail(bann_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define CK(call)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (call);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail(ctx, e_ == hipErrorOutOfMemory ? BANN_E_OOM : BANN_E_HIP,              \
                  std::string(#call) + ": " + hipGetErrorString(e_));                     \
  } while (0)

template <typename T>
inline hipError_t dalloc(T** p, int64_t count) {
  *p = nullptr;
  if (count <= 0) count = 1;
  return hipMalloc((void**)p, (size_t)count * sizeof(T));
}

inline void dfree(void* p) {
  if (p) (void)hipFree(p);
}

// implemented in bann_api.hip
void refresh_state(bann_ctx* ctx);
bool check_branch(const bann_ctx* ctx, int32_t b);
int build_plan(bann_ctx* ctx, const int32_t* branches, int32_t nb, Plan& p, bool persistent);
void free_plan(Plan& p);
int run_grad(bann_ctx* ctx, const Plan& p, int write_pred, int upd_mode = -1, int upd_step = 0);
int run_forward(bann_ctx* ctx, const Plan& p);  // predictions only
void run_update(bann_ctx* ctx, const Plan& p, int32_t mode, int32_t step);
int ensure_htrace(bann_ctx* ctx, int32_t L);
int alloc_genotypes(bann_ctx* ctx, int64_t n, int64_t M);   // the 2-bit genotype image of n x M
int64_t stage_markers(int64_t bytes_per_marker, int64_t M);  // markers per ~256 MiB staging block
int ensure_predictions(bann_ctx* ctx, const int32_t* branches, int32_t nb);  // bann_residual.hip
void launch_residual_sub(float* r, const float* d, int64_t n, hipStream_t s);
void mark_predictions(bann_ctx* ctx, const Plan& p, bool current);
int traj_prepare(bann_ctx* ctx, const Plan& p, int32_t L, float max_dh, int32_t step_mode, float factor,
                 const float* eps, const float* momentum, uint64_t seed, const float* u);
// in-trajectory launch timing (bann_set_launch_timing): event marks on the context stream
enum { TM_GRAD0 = 0, TM_GRAD1 = 1, TM_UPD1 = 2, TM_AR0 = 3, TM_AR1 = 4, TM_FWD0 = 5, TM_FWD1 = 6 };
void tm_mark(bann_ctx* ctx, int32_t kind);
void tm_mark_follow(bann_ctx* ctx, int32_t kind);
int tm_resolve(bann_ctx* ctx);  // after the stream has drained
// bann_dist.hip: the network sampler's device buffers, allocated once at bann_finalize
// (no allocation or synchronous upload inside a collective trajectory)
// the sequential driver's branch-update tail (bann_api.hip / bann_residual.hip)
int residual_from_target_shift(bann_ctx* ctx, int32_t b, float add, double* sum, double* sumsq, double* sum_after,
                               double* sumsq_after);
int residual_from_target_shift_launch(bann_ctx* ctx, int32_t b, float add);
int hmc_step_tail(bann_ctx* ctx, int32_t b, int32_t L, float max_dh, int32_t step_mode, float factor, const float* eps,
                  const float* momentum, uint64_t seed, const float* u, float add, int32_t* status_out,
                  float* params_out, double* stats);
int net_buffers_init(bann_ctx* ctx);
// network mode: k_forward_gsum's items for a persistent fx-only plan of 8-chunk branches
int build_net_groups(bann_ctx* ctx, Plan& p);
