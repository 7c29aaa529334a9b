// bann_internal.h — device-visible descriptors and launcher declarations shared
// by the HIP kernels (kernels_*.hip) and the C-ABI implementation (bann_api.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define BANN_MAXL 8          // max layers per branch (hidden + summary + output)
#define BANN_FUSED_MAXW 4    // fused kernels (fx, fxl): every layer width <= 4
#define BANN_WIDE_MAXW 32    // wide fused kernel (wx): one hidden layer, W, S <= 32
#define BANN_WIDE_MAXCH 2    // wide fused kernel: m_b <= 128
#define BANN_FX_MAXCH 8      // fx: <= 8 marker chunks of 64 (m_b <= 512), one wave per tile
#define BANN_FXL_MAXCH 64    // fxl: <= 64 chunks (m_b <= 4096), one wave per <= 8-chunk block
#define BANN_MAX_TILES_PER_WAVE 4096  // int32 dW0 digit sums: < 2^31 / (4.4e5 per tile: 16 K slots x 255 x (2 + 8 + 32 + 64))
#define BANN_CHUNK 64        // markers per chunk (one 16x16x64 i8 MFMA K-step)
#define BANN_FRAG 16         // individuals per fragment (MFMA N)
#define BANN_TILE_FRAGS 4    // fragments per fused-kernel tile (64 individuals)

enum { MODE_GRAD = 0, MODE_INIT = 1, MODE_STEP = 2, MODE_LAST = 3, MODE_PROFILE = 4, MODE_RESTORE = 5 };
enum { ST_RUNNING = -1, ST_ACCEPTED = 0, ST_REJECTED = 1, ST_REJECTED_EARLY = 2 };

// Per-branch descriptor (device resident, one per branch).
struct BranchDev {
  int64_t x_off;      // byte offset of the packed genotype block
  int64_t p_off;      // offset into the params-sized arrays (theta, p, eps, ...)
  int64_t mk_off;     // offset into per-branch marker arrays (mu/sigma gathered), m entries
  int64_t part_off;   // float offset into the partial-gradient slabs: nsplits x P
  int64_t dig_off;    // byte offset of the MFMA A-operand digits [nchunks][64][16]
  int64_t y_off;      // offset of the target / prediction vectors (b * n)
  int64_t scr_off;    // gx path: float offset of the branch's scratch within its scratch group
  int64_t xi_off;     // byte offset of the individual-major fi image (kernels_fi.hip), -1 if none
  int32_t m;          // markers in the branch
  int32_t nchunks;    // ceil(m / 64)
  int32_t L;          // number of layers (weight matrices)
  int32_t act;        // bann_activation
  int32_t prior;      // bann_prior
  int32_t P;          // num params
  int32_t nsplits;    // row splits (partial slabs)
  int32_t fused;      // kernel path: 1 = fx, 3 = fxl (widths <= 4), 2 = wide (wx), 0 = gx (layered MFMA GEMMs)
  int32_t widths[BANN_MAXL];  // out width of each layer (last = 1)
  int32_t win[BANN_MAXL];     // in width of each layer (win[0] = m)
  int32_t woff[BANN_MAXL];    // param_vec offset of W_l
  int32_t boff[BANN_MAXL];    // param_vec offset of b_l (l < L-1)
  // gx path scratch (kernels_gx.hip), float offsets from scr_off, every one a multiple of 4
  int32_t gx_w[BANN_MAXL];    // Wp_l: W_l as [out][gx_wld[l]] rows (layer 0: W0 / sigma)
  int32_t gx_wld[BANN_MAXL];  //   its row stride: win_l rounded up to 4
  int32_t gx_b[BANN_MAXL];    // b_l (layer 0: c0 = b0 - mu^T W0 / sigma), l < L-1
  int32_t gx_a[BANN_MAXL];    // A_l = h(Z_l): [rows][gx_ld[l]], l < L-1
  int32_t gx_h[BANN_MAXL];    // H_l = h'(Z_l), overwritten by delta_l in the backward
  int32_t gx_ld[BANN_MAXL];   //   row stride: w_l rounded up to 4
  int32_t gx_dwo;             // head: f64 dW_out partials [tile][S]
  int32_t gx_rss;             // head: f64 rss partials [tile]
  int32_t gx_op;              // FWD of the summary layer: f32 partial outputs A_s w_out [2 ceil(S/64)][rows]
  int32_t gx_e;               // head: the output error e = out - y [rows] (0 past n)
  int32_t gx_wps;             // Wp_s (s = L-2 >= 1) with row k scaled by w_out[k], as three bf16 planes like gx_wp (lazy head BWD_s)
  int32_t gx_w0p;             // W0 / sigma as three bf16 planes [3][w0][64 nchunks] (masked layer on bf16 MFMA)
  int32_t gx_wp[BANN_MAXL];   // Wp_l, 1 <= l < L-1, as three bf16 planes [3][w_l][win_l rounded up to 32] (hidden GEMMs)
  // precision coordinates (precision_vec order, params.rs:272-289) for joint HMC
  int64_t q_off;              // offset into the per-precision arrays (phi, ...)
  int32_t nq;                 // num precisions
  int32_t qoff[BANN_MAXL];    // first weight precision of layer l
  int32_t qbias;              // first bias precision (L-1 of them), then the error precision
};

// One work item of the fused gradient kernel: a contiguous fragment range of one
// branch, and where its partial gradient slab(s) and rss partial(s) go: the
// branch's own slabs (part_off + split P) or, for plans too small to fill the
// GPU, the "solo" region after them (folded into the branch's slabs by
// launch_fold_solo).  wx items own 4 consecutive slabs / rss entries (one per wave).
struct GradItem {
  int32_t branch;
  int32_t split;
  int32_t frag_begin;
  int32_t frag_end;
  int64_t part_at;  // float offset in DevState::part of the item's (first) slab
  int64_t rss_at;   // index in DevState::rss_part of its (first) rss partial
  int32_t tile0;    // forward-only fi pass: the group's tiles before this item (its index space)
  int32_t fold_ix;  // solo plans: index of the branch's FoldJob in the plan's fold list (else -1)
};
// network-mode forward with per-group output sums (k_forward_gsum): nbr fx branches (the
// plan's branch list from list_off), 8 per pass, over one tile range, summed into row `row`
struct NetGroupItem {
  int32_t list_off;
  int32_t nbr;
  int32_t tile_begin;
  int32_t tile_end;
  int32_t row;
  int32_t pad[3];
};
// solo-mode fold: a branch's ns slabs at part[part] / rss_part[rss] -> its slab 0
struct FoldJob {
  int32_t branch;
  int32_t nslab;
  int64_t part;
  int64_t rss;
};

// Per-branch derived constants of the fused path (rewritten after every position update).
struct FusedConst {
  float scale[BANN_WIDE_MAXW];  // power-of-two scale of the W0/sigma digits per column
  float c0[BANN_WIDE_MAXW];     // b0_k - sum_j mu_j W0_jk / sigma_j
};

struct DevState {
  const BranchDev* br;    // [nbranch]
  const uint8_t* xu2;     // 2-bit genotype tile images of every branch ([tile][chunk][1 KiB], kernels_fx.hip)
  const uint8_t* xi;      // individual-major 2-bit images of the fx branches (kernels_fi.hip), or null
  const uint8_t* dig;     // digits
  FusedConst* fc;         // [nbranch]
  const float* mu;        // gathered per-branch marker means  [sum m]
  const float* sigma;     // gathered per-branch marker stds
  float* theta;           // [sum P]
  float* mom;             // momentum
  float* eps;             // step sizes
  float* theta0;          // trajectory start
  float* lam;             // per-parameter gradient precision multiplier
  float* lamld;           // per-parameter log-density multiplier
  float* grad;            // scratch: log density gradient
  float* part;            // partial d(rss/2) slabs
  double* rss_part;       // [nbranch][max splits]
  float* y;               // targets [nbranch][n]
  float* pred;            // predictions [nbranch][n]
  float* pred0;           // predictions at the trajectory start
  float* scr;             // gx-path scratch (one scratch group's worth)
  float* eprec;           // error precision per branch
  double* h0;             // initial -H per branch
  double* htrace;         // [nbranch][Lint+1]
  double* ld_out;         // log density per branch (last evaluation)
  double* rss_out;        // rss per branch (last evaluation)
  int32_t* status;        // per-branch trajectory status
  int32_t* uturn;         // first U-turn step
  float* uacc;            // acceptance uniforms per branch
  int64_t n;              // individuals
  int32_t nfrag;          // ceil(n / 16)
  int32_t max_splits;
  int32_t lint;           // trajectory length L (for the trace stride)
  float max_dh;
  unsigned long long* dbg;  // diagnostic phase stamps (BANN_STAMPS=1 with a BANN_ABLATE=16 build), else null
  // joint HMC (precisions as coordinates, branch_sampler.rs:1070-1178)
  float* phi;             // precision coordinates [sum nq]
  float* phi0;            // trajectory start
  float* mphi;            // their momenta
  float* ephi;            // their step sizes
  float* gphi;            // their log-density gradient
  const int32_t* pidx;    // [sum P]: precision index (within the branch) of every parameter
  const float* ows;       // [nbranch][2]: output-weight summary stat of the OTHER branches (reg_sum), and
                          //   the network's output-weight count (OutputWeightSummaryStats, params.rs:404-465)
  int32_t netmode;        // network-joint HMC: no per-branch rss term / decisions in k_update
  const float* nete;      // network mode: the network's output error e = sum f + bias - y [n], read by the
                          //   fx gradient kernel as every branch's error (no per-branch targets); else null
  float net_le;           // its error precision (every branch's)
  float hyper[6];         // NetworkPrecisionHyperparameters: (shape, scale) dense, summary, output (params.rs:134-142)
};

// ---- launchers (defined in the kernel translation units) ----
// one chunk (64 marker rows) of one branch's tile image: batched pack (kernels_data.hip)
struct PackJob {
  int64_t dst;          // byte offset of the chunk in tile 0 of the branch's image (x_off + 1024 c)
  int64_t tile_stride;  // bytes per tile of the branch's image (1024 nchunks)
  int32_t idx_off;      // first of the chunk's rows in the concatenated marker-index list
  int32_t rows;         // valid rows (markers) of the chunk, <= 64; the rest are zero padding
  int32_t f3m1;         // tile images only: field 3 (bits 6-7) stored as code - 1 (fx / fxl / fxh branches)
};
// the fx / fxl / fxh kernels read their tile images with field 3 stored as code - 1
// (kernels_fx.hip header); the wide and layered kernels read plain codes
__host__ __device__ inline bool tile_f3m1(int fused) { return fused == 1 || fused == 3; }
// genotype image: 2-bit variant-major rows of rowb = ceil(n/64)*16 bytes (kernels_data.hip header)
void launch_synthetic_genotypes(uint8_t* raw, int64_t rowb, float* mu, float* sigma, int64_t n, int64_t M,
                                uint64_t seed, hipStream_t s);
void launch_i8_to_raw(const int8_t* g, int64_t n, int64_t m, uint8_t* raw, int64_t rowb, int32_t* flag,
                      hipStream_t s);
void launch_bed_to_raw(const uint8_t* payload, int64_t n, int64_t m, uint8_t* raw, int64_t rowb, hipStream_t s);
void launch_col_stats(const uint8_t* raw, int64_t rowb, float* mu, float* sigma, int64_t n, int64_t M,
                      hipStream_t s);
void launch_unpack_markers(const uint8_t* raw, int64_t rowb, const int32_t* snp_idx, int32_t m, int64_t n,
                           int8_t* out, hipStream_t s);
void launch_pack_tiles(const uint8_t* raw, int64_t rowb, const PackJob* jobs, int32_t njobs, const int32_t* idx,
                       int64_t ntile, uint8_t* dst, hipStream_t s);
void launch_gather_stats(const float* mu, const float* sigma, const int32_t* snp_idx, int32_t m, float* mu_b,
                         float* sig_b, hipStream_t s);

// gx: the layered MFMA path (kernels_gx.hip)
enum { GX_FWD0 = 0, GX_FWD = 1, GX_BWD = 2, GX_GRAD = 3, GX_GRAD0 = 4, GX_HEAD = 5 };
int64_t gx_tiles(const BranchDev& d, int ph, int l, int32_t nfrag);
void launch_gx_prep(const DevState& st, const int32_t* blist, int nb, hipStream_t s);
void launch_gx_head(const DevState& st, const int32_t* blist, int nb, int max_splits, hipStream_t s);
void launch_gx_gemm(const DevState& st, int ph, int l, const int32_t* blist, const int32_t* prefix, int nb,
                    int total, hipStream_t s);
#define GX_HEAD_MAXW 4096   // widest summary layer of a gx branch
void launch_fold_solo(const DevState& st, const FoldJob* jobs, int32_t njobs, int32_t max_p, hipStream_t s);
void launch_update(const DevState& st, const int32_t* branches, int32_t nb, int32_t mode, int32_t step,
                   hipStream_t s, int large);
bool update_is_large(const BranchDev& d);  // served by the 1024-thread update kernel
void launch_fused_const(const DevState& st, const int32_t* branches, int32_t nb, hipStream_t s);
void launch_sample_momentum(const DevState& st, const int32_t* branches, int32_t nb, int32_t max_p, uint64_t seed,
                            hipStream_t s);
void launch_update_joint(const DevState& st, const int32_t* branches, int32_t nb, int32_t mode, int32_t step,
                         hipStream_t s);
void launch_sample_momentum_joint(const DevState& st, const int32_t* branches, int32_t nb, int32_t max_q,
                                  uint64_t seed, hipStream_t s);
#define BANN_JOINT_MAXQ 4608  // joint HMC: precisions per branch (ARD: m + hidden widths + L)
// scratch: residual_delta_scratch_floats(n)
void launch_net_sum(const DevState& st, const int32_t* branches, int32_t nb, float* out, float* scratch,
                    hipStream_t s);
// out[i] = sum over rows r < nrows of rows[r n + i] (contiguous rows, e.g. the group sums of
// k_forward_gsum): the same two-pass fixed-order sum; scratch: residual_delta_scratch_floats(n)
void launch_net_sum_rows(const DevState& st, const float* rows, int32_t nrows, float* out, float* scratch,
                         hipStream_t s);
// network-mode forward of fx branches of 8 chunks, one row per item (kernels_fx.hip); blist:
// the items' branch lists; at most forward_gsum_max_tiles() tiles per item
void launch_forward_gsum(const DevState& st, const NetGroupItem* items, int32_t nitems, const int32_t* blist,
                         int32_t L, int32_t act, float* gsum, hipStream_t s);
int forward_gsum_max_tiles();
// sum_e: in = sum over ranks of the branch outputs, out = the error e; part: net_scratch_doubles(n);
// y = null: sum_e already holds e and only the nb branch targets y_b = f_b - e are written
void launch_net_targets(const DevState& st, const int32_t* branches, int32_t nb, float* sum_e, const float* y,
                        float bias, double* part, double* rss_out, hipStream_t s);
int64_t net_scratch_doubles(int64_t n);
// common-mode step sizes of the network-joint state (kernels_update.hip): per branch the common-mode
// gains a_p = eps_p |g_p| (g: the branch's partial slabs after a gradient launch with output error 1)
// into st.grad and a histogram of a_p^2 / T (part: nb x 2 CM_NC, out: 2 CM_NC = counts, then
// fixed-point sums in units of 2^-32: no wrap below 2^32 parameters per bin); then eps_p *= min(1, t / a_p)
#define CM_NC 96
#define CM_FIX_LOG2 32
void launch_fill_f32(float* p, float v, int64_t n, hipStream_t s);
void launch_cm_hist(const DevState& st, const int32_t* branches, int32_t nb, float inv_T, unsigned long long* part,
                    unsigned long long* out, hipStream_t s);
void launch_cm_apply(const DevState& st, const int32_t* branches, int32_t nb, int32_t max_p, float t, float* scale,
                     hipStream_t s);
void launch_cm_rescale(const DevState& st, const int32_t* branches, int32_t nb, int32_t max_p, const float* scale,
                       hipStream_t s);
void launch_uniforms(const DevState& st, const int32_t* branches, int32_t nb, uint64_t seed, hipStream_t s);
// mode 0 exact f32 MFMA, 1 bf16 MFMA, 2 f32-accurate bf16 planes (kernels_wx.hip)
void launch_fused_grad_wx(const DevState& st, const GradItem* items, int32_t nitems, int32_t act, int mode,
                          int nch, int write_pred, hipStream_t s);
bool wx_exact();
// upd_cnt != null: the fused leapfrog update (mode, step) in the tail -- the last workgroup of
// each branch updates it (update_core.h); upd_cnt = one zeroed arrival counter per branch
void launch_fused_grad_fx(const DevState& st, const GradItem* items, int32_t nitems, int32_t L, int32_t act,
                          int full8, int write_pred, int upd_mode, int upd_step, int32_t* upd_cnt,
                          const FoldJob* folds, hipStream_t s);
// forward-only fx pass (predictions into st.pred, no target / backward / partials)
void launch_forward_fx(const DevState& st, const GradItem* items, int32_t nitems, int32_t L, int32_t act, int full8,
                       hipStream_t s);
// forward-only fx pass over the individual-major fi images (kernels_fi.hip)
void launch_forward_fi(const DevState& st, const GradItem* items, int32_t nitems, int64_t total_tiles, int32_t L,
                       int32_t act, int32_t max_seg, int32_t cus, hipStream_t s);
void launch_pack_fi(const uint8_t* raw, int64_t rowb, const PackJob* jobs, int32_t njobs, const int32_t* idx,
                    int64_t ntile, uint8_t* dst, hipStream_t s);
void launch_fused_grad_fxl(const DevState& st, const GradItem* items, int32_t nitems, int32_t L, int32_t act,
                           int32_t nw, int32_t cpw, int full, int write_pred, int head, hipStream_t s);
int fxl_lds_bytes(int nw, int nl, int cpw);
int fxl_cpw(int nchunks);  // marker chunks per fxl wave: 4 up to 32 chunks, else 8
void launch_step_sizes(const DevState& st, const double* base, const int32_t* branches, int32_t nb, int32_t max_p,
                       int izmailov, float c, int32_t L, hipStream_t s);
void launch_restore_pred(const DevState& st, const int32_t* branches, int32_t nb, hipStream_t s);
void launch_snapshot_pred(const DevState& st, const int32_t* branches, int32_t nb, hipStream_t s);
int64_t residual_delta_scratch_floats(int64_t n);
// forward_feed with every layer (kernels_feed.hip): pre [sum_{l<L-1} w_l][n] (may be null), act [sum_l w_l][n]
void launch_forward_feed(const DevState& st, int b, const BranchDev& bd, float* pre, float* act, hipStream_t s);
// effect_sizes over forward_feed's layers: ea / eb two [max w_l][n] buffers; full [m][n] and / or
// pop [m] (column means, s: w_0 doubles of scratch); either may be null
void launch_effect_sizes(const DevState& st, int b, const BranchDev& bd, const float* pre, const float* act,
                         float* ea, float* eb, float* full, double* s, float* pop, hipStream_t strm);
void launch_residual_delta(const DevState& st, const int32_t* branches, int32_t nb, float* scratch, float* out,
                           hipStream_t s);
