/*
 * bann.h — C ABI of the MI355X-native branch-network HMC hot path.
 *
 * Drop-in boundary for the per-branch math of medical-genomics-group/rs-bann
 * (Rust + ArrayFire).  The reference has no FFI: its hot path sits behind the
 * Rust traits BranchSampler (src/net/branch/branch_sampler.rs:32-1300) and
 * BranchStruct (src/net/branch/branch_struct.rs:119-141) and reaches the device
 * through ArrayFire calls.  Each entry point below names the reference item it
 * replaces (file:line).  A Rust binding is sketched in INTEGRATION.md.
 *
 * Conventions
 *  - Every function returns BANN_OK (0) or a negative bann_status; the message
 *    of the last failure is available from bann_last_error().
 *  - Pointers are HOST pointers unless the name ends in _device.  They are read
 *    or written synchronously inside the call and never retained.
 *  - Parameter vectors use the reference param_vec order (params.rs:700-715):
 *    all weights layer by layer, each (in x out) matrix column-major
 *    (element (j,k) at k*in + j), then all biases.  num_params(b) floats.
 *  - Precision vectors use the BranchPrecisions::param_vec order
 *    (params.rs:272-289): weight precisions layer by layer (ARD priors: one per
 *    input node for layers 0..L-2 and one for the output layer; base priors and
 *    std-normal: one per layer), then the L-1 bias precisions, then the error
 *    precision.  num_precisions(b) floats.
 *  - A context owns one HIP device, one stream and all device buffers.  It is
 *    not thread-safe; use one context per GPU (one process per GPU for
 *    multi-GPU runs).
 */
#ifndef BANN_H
#define BANN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bann_ctx bann_ctx;

typedef enum {
  BANN_OK = 0,
  BANN_E_HIP = -1,    /* HIP runtime error (no device, launch failure, ...) */
  BANN_E_SHAPE = -2,  /* inconsistent sizes / indices                        */
  BANN_E_OOM = -3,    /* device allocation failed                            */
  BANN_E_STATE = -4,  /* call order violated (e.g. compute before finalize)  */
  BANN_E_ARG = -5     /* invalid argument value                              */
} bann_status;

/* activation_functions.rs:6-12 (same discriminants) */
typedef enum { BANN_TANH = 0, BANN_RELU = 1, BANN_LEAKY_RELU = 2, BANN_SILU = 3, BANN_IDENTITY = 4 } bann_activation;

/* one code per BranchSampler impl (model_type.rs:6-13) */
typedef enum {
  BANN_RIDGE_ARD = 0,   /* ridge_ard.rs   */
  BANN_RIDGE_BASE = 1,  /* ridge_base.rs  */
  BANN_LASSO_ARD = 2,   /* lasso_ard.rs   */
  BANN_LASSO_BASE = 3,  /* lasso_base.rs  */
  BANN_STD_NORMAL = 4   /* std_normal_branch.rs */
} bann_prior;

/* HMCStepResult (branch_sampler.rs:1310-1314) */
typedef enum { BANN_ACCEPTED = 0, BANN_REJECTED = 1, BANN_REJECTED_EARLY = 2 } bann_hmc_status;

/* StepSizeMode (mcmc_cfg.rs:264-270); INJECTED = caller supplies eps.
 * STD_SCALED (branch_sampler.rs:1213): eps = c * sqrt(1 / lambda_l) per weight layer and
 * c * (1 / sqrt(lambda_b)) per bias layer in f32 (ridge_base.rs:52-82, lasso_base.rs:53-82,
 * std_normal_branch.rs:51-80).  The ARD priors return EMPTY step-size vectors there
 * (ridge_ard.rs:56-68, lasso_ard.rs:62-74: hmc_step would index-panic), so it is refused
 * (BANN_E_ARG) for a branch with an ARD prior.  Joint HMC falls back to random step sizes
 * as the reference does (branch_sampler.rs:1092-1101). */
typedef enum {
  BANN_STEP_UNIFORM = 0,
  BANN_STEP_RANDOM = 1,
  BANN_STEP_STD_SCALED = 2,
  BANN_STEP_IZMAILOV = 3,
  BANN_STEP_INJECTED = 100
} bann_step_mode;

/* ---------------- context ---------------- */
int bann_ctx_create(int device, bann_ctx** out);
int bann_ctx_destroy(bann_ctx* ctx);
const char* bann_last_error(const bann_ctx* ctx);
/* library build/version string; callable without a device */
const char* bann_version(void);

/* ---------------- genotypes: replaces GroupedGenotypes / BedVM ----------------
 * genotypes.rs:7-12,44-48 (x_group_af), bed.rs:193-245 (from_file + column
 * stats), bed.rs:325-355 (get_submatrix_af_standardized).  The cohort stays
 * resident on the device as a 2-bit variant-major image (the .bed payload's
 * information content), packed at bann_finalize into per-branch 2-bit tile
 * images; standardization (g - mu)/sigma with the population std
 * (bed.rs:231-242) is folded into the first-layer weights. */

/* g: variant-major int8 genotypes g[j*n + i] in {0,1,2}; mu/sigma computed on device */
int bann_genotypes_upload(bann_ctx* ctx, const int8_t* g, int64_t n, int64_t num_markers);
/* payload: variant-major .bed bytes without the 3-byte signature (bed.rs:100-116),
 * ceil(n/4) bytes per marker; decoded on the device with the 2-bit LUT of
 * bed_lookup_tables.rs:4 (00->2, 01->0, 10->1, 11->0) */
int bann_genotypes_upload_bed(bann_ctx* ctx, const uint8_t* payload, int64_t n, int64_t num_markers);
/* synthetic cohort generated on the device: g_ij ~ Binomial(2, p_j),
 * p_j ~ U(0.01, 0.5) (bed.rs:136-188 semantics; counter-based RNG, not the
 * reference's ChaCha stream).  Zero-variance markers are redrawn. */
int bann_genotypes_synthetic(bann_ctx* ctx, int64_t n, int64_t num_markers, uint64_t seed);
int bann_genotypes_stats(bann_ctx* ctx, float* mu, float* sigma);
/* override the standardization constants (e.g. statistics of a reference
 * cohort, or mu = 0, sigma = 1 for pre-standardized / raw inputs); before finalize */
int bann_genotypes_set_stats(bann_ctx* ctx, const float* mu, const float* sigma);
/* copy genotypes of markers snp_idx[0..m) back to the host as g[j*n + i] */
int bann_genotypes_download(bann_ctx* ctx, const int32_t* snp_idx, int32_t m, int8_t* g_out);

/* BedVM::from_file (bed.rs:193-245): stem.bed (3-byte signature checked;
 * variant-major only, as the reference) with the dims of stem.dims or the line
 * counts of stem.fam / stem.bim, streamed from the file into the device image
 * in bounded blocks */
int bann_genotypes_load_bed(bann_ctx* ctx, const char* stem);

/* ---------------- files on either side of the path (host only, no device) ---------------- */
/* BedDims (io/dims.rs:15-34): stem.dims "n M", else the .fam / .bim line counts */
int bann_bed_dims(const char* stem, int64_t* n_out, int64_t* num_markers_out);
/* ExternalGrouping::from_file (group/external.rs:15-60): two columns
 * "marker_ix group_ix" (0-based, groups 0..G-1), as CSR: offsets[G+1],
 * markers[num_entries] in file order.  Call with offsets/markers NULL for the sizes. */
int bann_grouping_read(const char* path, int32_t* num_groups, int64_t* num_entries, int64_t* offsets,
                       int32_t* markers);
/* UniformGrouping::new (group/uniform.rs:11-23): group g = markers [g*size, (g+1)*size) */
int bann_grouping_uniform(int32_t num_groups, int32_t group_size, int64_t* offsets, int32_t* markers);
/* Phenotypes::from_file / to_file (data/phenotypes.rs:28-36): bincode Vec<f32>
 * (u64 length + values, little endian).  bann_phen_read with y_out NULL gives n. */
int bann_phen_read(const char* path, int64_t* n_out, float* y_out);
int bann_phen_write(const char* path, const float* y, int64_t n);

/* ---------------- branches: replaces BranchCfg -> B::from_cfg ----------------
 * branch_struct.rs:12-29 (from_cfg), branch_cfg.rs:185-193 (BranchCfg). */

/* Adds a branch over markers snp_idx[0..m) (groups may overlap, external.rs).
 * layer_widths: hidden..., summary, 1 (params.rs:470); num_layers >= 2.
 * Returns the branch index (>= 0) or a negative bann_status. */
int bann_branch_add(bann_ctx* ctx, const int32_t* snp_idx, int32_t m, const int32_t* layer_widths,
                    int32_t num_layers, int32_t activation, int32_t prior);
/* packs every branch's genotype block into the device layout; after this the
 * branch set is fixed.  free_raw != 0 releases the full genotype matrix. */
int bann_finalize(bann_ctx* ctx, int32_t free_raw);
int bann_num_branches(const bann_ctx* ctx);
int64_t bann_num_params(const bann_ctx* ctx, int32_t b);
int64_t bann_num_precisions(const bann_ctx* ctx, int32_t b);
/* shape of branch b (the BranchCfg header fields, branch_cfg.rs:8-16):
 * markers, number of layers, layer widths (min(num_layers, widths_cap)
 * entries), activation (bann_activation) and prior (bann_prior); any output
 * may be NULL.  Callable before finalize and without compute. */
int bann_branch_info(const bann_ctx* ctx, int32_t b, int32_t* m, int32_t* num_layers, int32_t* widths_out,
                     int32_t widths_cap, int32_t* activation, int32_t* prior);

/* BranchParams::from_host / load_param_vec (params.rs:634-698) */
int bann_branch_set_params(bann_ctx* ctx, int32_t b, const float* param_vec);
/* BranchParams::to_host / param_vec (params.rs:663-715) */
int bann_branch_get_params(bann_ctx* ctx, int32_t b, float* param_vec_out);
/* BranchPrecisions::from_host (params.rs:248-262) */
int bann_branch_set_precisions(bann_ctx* ctx, int32_t b, const float* precision_vec);
int bann_branch_get_precisions(bann_ctx* ctx, int32_t b, float* precision_vec_out);
/* step sizes of branch b used by the last trajectory (hmc_step / leapfrog_begin),
 * param_vec order (izmailov_step_sizes ridge_ard.rs:70-117 etc.) */
int bann_branch_get_step_sizes(bann_ctx* ctx, int32_t b, float* out);
/* target y_b (n floats) the branch is fitted to: the partial residual
 * residual + f_b(theta) of net.rs:279-280 */
int bann_branch_set_target(bann_ctx* ctx, int32_t b, const float* y);
int bann_set_target_all(bann_ctx* ctx, const float* y);

/* ---------------- per-branch math: replaces the BranchSampler methods ---------------- */
/* predict (branch_sampler.rs:915-918, forward_feed 743-782): pred_out[n] */
int bann_predict(bann_ctx* ctx, int32_t b, float* pred_out);
/* predictions of several branches from ONE packed gradient launch (the
 * per-branch loop of net.rs:272-282 when the residual is rebuilt); pred_out is
 * nb x n, row i = branch branches[i]. */
int bann_predict_many(bann_ctx* ctx, const int32_t* branches, int32_t nb, float* pred_out);
/* rss (branch_sampler.rs:905-909) against the branch target */
int bann_rss(bann_ctx* ctx, int32_t b, double* rss_out);
/* log_density_gradient (branch_sampler.rs:380-391: backpropagate 813-875 +
 * the prior's log_density_gradient_wrt_weights, e.g. ridge_ard.rs:196-219, and
 * log_density_gradient_wrt_biases 322-331); grad_out in param_vec order.
 * rss_out (optional) receives the rss at the same parameters (823-828). */
int bann_log_density_gradient(bann_ctx* ctx, int32_t b, float* grad_out, double* rss_out);
/* the same for several branches from ONE packed gradient launch, each against
 * its own current target (Net::gradient, net.rs:520-527, sets every target to
 * the phenotype first): grad_out = the branches' param_vec gradients
 * concatenated in list order, rss_out[nb] (may be NULL) */
int bann_log_density_gradient_many(bann_ctx* ctx, const int32_t* branches, int32_t nb, float* grad_out,
                                   double* rss_out);
/* log_density_gradient_joint (branch_sampler.rs:406-422) at the branch's current
 * parameters and precision vector: grad_out[P + Q] = [params | precisions]
 * (ridge_ard.rs:221-250 etc.), the rss and the joint log density
 * (log_density_joint, 292-305; the output-weight stat of bann_branch_set_output_stats).
 * hyper: 6 floats as bann_hmc_step_joint.  rss_out / log_density_out may be NULL. */
int bann_log_density_gradient_joint(bann_ctx* ctx, int32_t b, const float* hyper, float* grad_out, double* rss_out,
                                    double* log_density_out);
/* forward_feed (branch_sampler.rs:743-782) keeping every layer, for
 * Net::activations (net.rs:509-518): act_out = the activations of layer 0, 1,
 * ..., L-1 (the last one is the output), each [w_l][n] column-major (element
 * (i, k) at k n + i), sum_l w_l n floats; pre_out (may be NULL) = the
 * pre-activations of the hidden and summary layers (the output's equals its
 * activation and is not repeated), sum_{l<L-1} w_l n floats. */
int bann_forward_feed(bann_ctx* ctx, int32_t b, float* pre_out, float* act_out);
/* BranchSampler::effect_sizes (branch_sampler.rs:784-811): the n x m matrix of
 * branch b at its current parameters, column-major (element (i, j) at j n + i).
 * As the reference: the backward chain is seeded with the branch output times
 * W_out^T (792-797), not with the error (so entry (i, j) is out_i d out_i / d x_ij),
 * and no absolute value is taken (the doc comment says "absolute values"; the
 * code does not). */
int bann_effect_sizes(bann_ctx* ctx, int32_t b, float* out);
/* the per-branch part of Net::population_effect_sizes (net.rs:529-543): for
 * each listed branch the column means sum_i effect_sizes(i, j) / n, m_b floats
 * per branch, concatenated in list order.  The sum over individuals is taken
 * through the layer-0 deltas (sum_j W0(j,k) sum_i delta0(i,k)), in f64. */
int bann_population_effect_sizes(bann_ctx* ctx, const int32_t* branches, int32_t nb, float* out);
/* log_density (branch_sampler.rs:72-78; std_normal_branch.rs:149-158) at the
 * current parameters and the given rss */
int bann_log_density(bann_ctx* ctx, int32_t b, double rss, double* out);
/* neg_hamiltonian (branch_sampler.rs:878-883) with momentum p (param_vec order) */
int bann_neg_hamiltonian(bann_ctx* ctx, int32_t b, const float* momentum, double* out);

/* ---------------- HMC: replaces hmc_step (branch_sampler.rs:1192-1299) ----------------
 * Runs one HMC trajectory of L leapfrog steps for each branch in
 * branches[0..nb), all branches packed into one grad launch + one update
 * launch per leapfrog step.  Branches are independent (each against its own
 * target).  RNG draws may be injected for parity (SURVEY §0 caveat 3):
 *   step_mode == BANN_STEP_INJECTED: eps = concatenated per-branch step-size
 *       vectors (param_vec order); otherwise eps may be NULL and the sizes are
 *       computed on the device (izmailov_step_sizes, ridge_ard.rs:70-117 etc.;
 *       uniform 706-732) with factor step_factor.
 *   momentum: concatenated p0 (param_vec order), or NULL to sample N(0,1) on
 *       the device from seed.
 *   u: one acceptance uniform per branch (branch_sampler.rs:546-548).
 * Outputs (each may be NULL): status_out[nb] (bann_hmc_status),
 * h_trace_out[nb*(L+1)] (-H after each step; entry 0 = initial; a branch that
 * was rejected early stops updating its trace), uturn_out[nb] (first step with
 * net_movement < 0, 551-592, or -1), log_density_out[nb] (accepted state).
 * Rejected / early-rejected branches are restored to their initial params. */
int bann_hmc_step(bann_ctx* ctx, const int32_t* branches, int32_t nb, int32_t L, float max_hamiltonian_error,
                  int32_t step_mode, float step_factor, const float* eps, const float* momentum, uint64_t seed,
                  const float* u, int32_t* status_out, double* h_trace_out, int32_t* uturn_out,
                  double* log_density_out);

/* trajectory recording (MCMCCfg::trajectories, trajectory.rs:1-43,
 * branch_sampler.rs:1253-1289): while enabled, bann_hmc_step keeps per listed
 * branch the parameters after every position step, the log-density gradient
 * there and the -H trace (host copies after every launch: a debugging aid) */
int bann_set_trajectory_recording(bann_ctx* ctx, int32_t enabled);
/* the last recorded trajectory of branch b: steps taken (an early rejection
 * stops it), params[steps][P] and ldg[steps][P] in param_vec order,
 * hamiltonian[steps + 1]; at most cap steps are copied; outputs may be NULL */
int bann_branch_get_trajectory(bann_ctx* ctx, int32_t b, int32_t cap, int32_t* steps, float* params, float* ldg,
                               double* hamiltonian);
/* the same for a trajectory recorded by bann_hmc_step_joint (the joint
 * Trajectory of branch_sampler.rs:1126-1135): per step the parameters [P], the
 * precisions [Q] (precision_vec order) and the joint log-density gradient
 * [P + Q] (params | precisions); hamiltonian = the joint -H trace.  Each call
 * refuses the other kind of recording (BANN_E_STATE). */
int bann_branch_get_trajectory_joint(bann_ctx* ctx, int32_t b, int32_t cap, int32_t* steps, float* params,
                                     float* precisions, float* ldg, double* hamiltonian);

/* ---------------- joint HMC: replaces hmc_step_joint (branch_sampler.rs:1070-1178) ----------------
 * One trajectory per listed branch over its parameters AND its precisions
 * (ridge / lasso priors; std_normal has no joint density and is refused),
 * packed like bann_hmc_step.  The precisions start from the branch's precision
 * vector and the sampled ones become its precisions (bann_branch_get_precisions).
 *   hyper: 6 floats, NetworkPrecisionHyperparameters (params.rs:134-142):
 *       dense (shape, scale), summary (shape, scale), output (shape, scale)
 *   step_mode == BANN_STEP_INJECTED: eps = per branch [num_params | num_precisions]
 *       step sizes; any other mode: random step sizes U(0,1) (P+Q)^-1/4 factor
 *       drawn from seed (the reference joint sampler falls back to random for
 *       every mode, 1092-1101)
 *   momentum: per branch [num_params | num_precisions], or NULL (device N(0,1))
 *   u: acceptance uniform per branch, or NULL (drawn from seed)
 * The early-rejection test uses the joint -H; the final Metropolis test uses the
 * NON-joint log_density against the joint initial -H, as accept_or_reject_hmc_state
 * (928-962) does.  log_density_out: the non-joint log density of the final
 * state.  L >= 1. */
int bann_hmc_step_joint(bann_ctx* ctx, const int32_t* branches, int32_t nb, int32_t L, float max_hamiltonian_error,
                        int32_t step_mode, float step_factor, const float* eps, const float* momentum, uint64_t seed,
                        const float* u, const float* hyper, int32_t* status_out, double* h_trace_out,
                        double* log_density_out);
/* OutputWeightSummaryStats of branch b (params.rs:404-465) for the joint density
 * of the output layer: the reg sum of the OTHER branches' output weights and the
 * network's output-weight count (default 0 and the branch's own count). */
int bann_branch_set_output_stats(bann_ctx* ctx, int32_t b, float reg_sum_others, float num_params);

/* ---------------- benchmark / production leapfrog stepping ----------------
 * Device-resident trajectory state for a fixed branch set: begin samples the
 * momenta on the device and evaluates the initial gradient and -H; each
 * leapfrog step is one packed gradient launch + one fused update launch with
 * no host synchronisation; end performs the final half step, the Metropolis
 * decision (uniforms from seed) and restores rejected branches. */
int bann_leapfrog_begin(bann_ctx* ctx, const int32_t* branches, int32_t nb, int32_t L, float max_hamiltonian_error,
                        int32_t step_mode, float step_factor, uint64_t seed);
int bann_leapfrog_steps(bann_ctx* ctx, int32_t k);
int bann_leapfrog_end(bann_ctx* ctx, int32_t* status_out, int32_t* num_accepted);
/* device pointer to the branch predictions f_b(theta_L) written by the last
 * leapfrog step (indexed by branch id: pred[b*n + i]), for the residual update. */
int bann_leapfrog_predictions_device(bann_ctx* ctx, float** out);
/* residual change of the finished trajectory, written to a DEVICE buffer of n
 * floats: out[i] = sum over the session's accepted branches of
 * f_b(theta_L)[i] - f_b(theta_0)[i]  (net.rs:279-300 bookkeeping: the caller
 * does residual -= out, after an all-reduce over GPUs when branches are sharded) */
int bann_leapfrog_residual_delta_device(bann_ctx* ctx, float* out_device);
/* same, copied to a HOST buffer of n floats (device scratch owned by the context) */
int bann_leapfrog_residual_delta(bann_ctx* ctx, float* out_host);
int bann_synchronize(bann_ctx* ctx);
/* in-trajectory launch timing: while enabled, every gradient and update launch
 * of a leapfrog session (bann_leapfrog_begin / _steps) is bracketed by HIP
 * events on the context's stream; bann_leapfrog_end accumulates their elapsed
 * times.  bann_launch_timing returns the average milliseconds per gradient and
 * per update launch and the number of gradient launches since the last reset.
 * (Set outside a session.) */
int bann_set_launch_timing(bann_ctx* ctx, int32_t enabled);
int bann_launch_timing(bann_ctx* ctx, float* grad_ms, float* update_ms, int32_t* grad_launches, int32_t reset);
/* the same timing inside bann_network_hmc_step (whose gradient and update
 * launches also count in bann_launch_timing): average milliseconds of the
 * forward-only launch and of the per-step all-reduce of the summed branch
 * outputs (RCCL, or the callback's host round trip), and the all-reduce count */
int bann_network_timing(bann_ctx* ctx, float* forward_ms, float* allreduce_ms, int32_t* allreduces, int32_t reset);
/* individuals n of the context's cohort */
int64_t bann_ctx_num_individuals(const bann_ctx* ctx);
/* measurement hook: times `iters` packed gradient launches and `iters` update
 * launches (gradient-only mode, no state change) of the active leapfrog
 * session's branch set with HIP events on the context's stream; returns the
 * average milliseconds per launch of each. */
int bann_profile_session(bann_ctx* ctx, int32_t iters, float* grad_ms, float* update_ms);

/* ---------------- the network residual on the device ----------------
 * Net::train keeps the residual y - bias - sum_b f_b as a device Array and
 * updates it between branch updates (net.rs:158-171, 221, 279-300, 319-332).
 * The context owns one n-float device residual; every operation below is one
 * launch on the device (no n-float host copy).  Where a branch's prediction row
 * is needed and is not current (params set since the last forward pass), the
 * call first runs one packed forward launch over those branches.  sum / sumsq
 * (each may be NULL; both NULL = no host synchronisation) receive the sum and
 * the sum of squares of the residual after the operation, reduced in a fixed
 * order (deterministic). */
int bann_residual_set(bann_ctx* ctx, const float* residual);  /* host -> device residual */
int bann_residual_get(bann_ctx* ctx, float* residual_out);    /* device residual -> host */
int bann_residual_device(bann_ctx* ctx, float** out);         /* its device pointer (n floats) */
/* initialize_stats (net.rs:158-171): residual = (y - bias) - f_0 - f_1 - ... (branch order, f32) */
int bann_residual_init(bann_ctx* ctx, const float* y, float bias, double* sum, double* sumsq);
int bann_residual_stats(bann_ctx* ctx, double* sum, double* sumsq);
/* residual += add (the output bias: net.rs:321, 332) */
int bann_residual_shift(bann_ctx* ctx, float add, double* sum, double* sumsq);
/* net.rs:279-280: target y_b = residual + f_b(theta_b) */
int bann_residual_to_target(bann_ctx* ctx, int32_t b);
/* net.rs:292-300: residual = y_b - f_b(theta_b) after the branch's trajectory
 * (accepted: f_b(theta_L), i.e. residual -= y_pred; rejected: f_b(theta_0), i.e.
 * residual -= prev_pred) */
int bann_residual_from_target(bann_ctx* ctx, int32_t b, double* sum, double* sumsq);
/* targets of a packed sweep in one launch: y_b = r + f_b(theta_b) for every listed
 * branch, r = residual_device (n floats on the device) or NULL for the
 * context's own residual */
int bann_rebuild_targets(bann_ctx* ctx, const int32_t* branches, int32_t nb, const float* residual_device);

/* ---------------- multi-GPU: branch shards, one process (rank) per GPU ----------------
 * Branches share no weights: a rank owns a contiguous branch
 * range and only its markers' genotypes.  The context's communicator carries
 * the two exchanges of the path: the per-trajectory residual change of a
 * leapfrog session (the sweep bookkeeping of net.rs:292-300, over ranks) and,
 * in network-joint HMC, the per-step sum of the branch outputs.  The reference
 * is single-device (no collectives); these entry points have no counterpart. */

/* in-place sum over ranks of count values (dtype 0 = f32, 1 = f64) in a HOST
 * buffer, e.g. MPI_Allreduce or a gloo all_reduce; returns 0 on success */
typedef int (*bann_allreduce_fn)(void* user, void* host_buf, int64_t count, int32_t dtype);

/* contiguous branch ranges with ~equal marker totals: rank r owns
 * [starts_out[r], starts_out[r+1]); starts_out has world+1 entries; world must
 * not exceed nbranches (every rank owns a branch).  Host only. */
int bann_shard_branches(const int32_t* marker_counts, int32_t nbranches, int32_t world, int32_t* starts_out);
/* RCCL (xGMI) communicator: rank 0 calls bann_comm_unique_id, every rank gets
 * the 128 bytes out of band, then all ranks call bann_ctx_comm_init together */
int bann_comm_unique_id(uint8_t* id_out);
int bann_ctx_comm_init(bann_ctx* ctx, const uint8_t* id, int32_t nranks, int32_t rank);
/* a caller-provided all-reduce on host buffers instead of RCCL */
int bann_ctx_comm_callback(bann_ctx* ctx, bann_allreduce_fn fn, void* user, int32_t nranks, int32_t rank);
/* the context's communicator: kind 0 none, 1 RCCL, 2 callback; its rank count
 * and rank; backend_ranks = the rank count RCCL itself reports (ncclCommCount)
 * for kind 1, else nranks.  Outputs may be NULL. */
int bann_comm_info(const bann_ctx* ctx, int32_t* kind, int32_t* nranks, int32_t* rank, int32_t* backend_ranks);
/* residual bookkeeping over ranks on the host: local_delta is summed over the
 * ranks in place, then residual[i] -= local_delta[i].  The exchange step of
 * bann_exchange_residual for a callback communicator.  Host only. */
int bann_residual_update_host(bann_allreduce_fn fn, void* user, float* local_delta, float* residual, int64_t n);
/* after bann_leapfrog_end: residual_host[i] -= (sum over ranks of each rank's
 * bann_leapfrog_residual_delta)[i]; collective over the ranks */
int bann_exchange_residual(bann_ctx* ctx, float* residual_host);
/* the same on the context's device residual (bann_residual_*): with RCCL the
 * change is summed over the ranks on the device, no host copy; collective */
int bann_exchange_residual_device(bann_ctx* ctx);
/* network-joint HMC trajectory (SURVEY 8(e) packed-joint mode): the parameters
 * of every branch of every rank form ONE HMC state for
 *   -U = -lambda_e/2 ||sum_b f_b + bias - y||^2 + sum_b log prior_b(theta_b)
 * Per leapfrog step: a forward launch over the local branches, ONE all-reduce
 * of the n-vector sum of their outputs, e = sum f + bias - y as every branch's
 * output error (the summary output and its gradient), a gradient launch and
 * the update.  -H is summed over the ranks; early rejection and the Metropolis
 * test decide for the whole network, identically on every rank.  Collective.
 *   y: n targets on the host (identical on every rank); step_mode: Izmailov or
 *   uniform (device step sizes from the local precisions) or INJECTED (eps:
 *   the local branches' step sizes, concatenated in branch order); momentum:
 *   concatenated p0 of the local branches or NULL (device N(0,1) from seed; a
 *   rank-distinct stream is the caller's choice of seed); u: the Metropolis
 *   uniform (injected, parity runs) or NULL: drawn on rank 0 from seed and
 *   shared with every rank through the -H all-reduce, so all ranks decide alike.
 * Per step the first pass over the genotypes is forward-only (the outputs the
 * all-reduce needs); the gradient pass follows once e is known.
 * Outputs (may be NULL): status, h_trace[L+1], rss of the final state (theta_L
 * if accepted, theta_0 otherwise).  On
 * return (accepted: theta_L, otherwise theta_0) every local branch's target is
 * its Gibbs target y_b = f_b - e = y - bias - sum_{c != b} f_c over all ranks
 * (net.rs:279-280), and the context's device residual is y - bias - sum_b f_b. */
int bann_network_hmc_step(bann_ctx* ctx, const float* y, float bias, float lambda_e, int32_t L,
                          float max_hamiltonian_error, int32_t step_mode, float step_factor, const float* eps,
                          const float* momentum, uint64_t seed, const float* u, int32_t* status_out,
                          double* h_trace_out, double* rss_out);
/* Step sizes of the network-joint state (no reference counterpart: the network
 * sampler is this library's).  With per-branch Izmailov / uniform
 * steps the joint leapfrog's stiffest direction is the common mode -- every branch
 * shifting the network output together -- whose curvature grows with the number
 * of branches B (B aligned branches: B times one branch's).  Adapting: one extra
 * gradient launch with output error 1 gives g = J^T 1 (the gradient of sum_i F_i)
 * and every step size becomes eps_p min(1, t / (eps_p |g_p|)) with the largest t
 * (within 2^(1/4)) such that lambda_e / n sum_p min(eps_p |g_p|, t)^2 <= tau^2: the
 * common mode runs at omega eps <= tau while the parameters that do not drive it
 * keep their steps.  Summed over the ranks (collective); not applied to injected
 * step sizes.  Frozen: the per-parameter factors of the last adapted trajectory are
 * applied again without recomputing g -- step sizes that do not depend on the
 * trajectory's start, as HMC's reversibility asks.
 *   common_mode = 3 (DEFAULT, tau = 1): auto -- the first K trajectories adapt
 *     (K = 1 unless bann_set_network_adapt_trajectories says otherwise; burn-in),
 *     every later one is frozen.  Setting mode 3 again restarts the adaptation.
 *   common_mode = 2: frozen (adapts once if nothing was adapted yet).
 *   common_mode = 1: adapt before EVERY trajectory -- the proposal then depends on
 *     theta_0 and detailed balance does not hold: a diagnostic, not a sampler.
 *   common_mode = 0: off (plain per-branch steps). */
int bann_set_network_step_rule(bann_ctx* ctx, int32_t common_mode, float tau);
/* auto mode (3): the number K >= 1 of adapting trajectories before the factors freeze;
 * restarts the adaptation */
int bann_set_network_adapt_trajectories(bann_ctx* ctx, int32_t k);
/* the rule's state: mode, adapting trajectories done in auto mode, and whether the NEXT
 * trajectory applies frozen factors (1) or adapts / runs without the rule (0) */
int bann_network_step_rule_state(const bann_ctx* ctx, int32_t* mode, int32_t* adapted, int32_t* frozen);
/* the network sampler's forward: the group-sum rows of its plan (k_forward_gsum: every
 * branch an fx branch of 8 chunks -- each step's forward but the last writes one row per
 * group of four branches), 0 = per-branch output rows, -1 = no network trajectory yet */
int bann_network_info(const bann_ctx* ctx, int32_t* group_rows);
/* the last network trajectory's rule: [threshold t (inf: no step changed),
 * (omega eps)^2 of the common mode before (inf when some single parameter alone
 * exceeded tau) and after, the fraction of parameters whose step was reduced] */
int bann_network_step_rule_info(const bann_ctx* ctx, double* out4);

/* ---------------- introspection for tests / profiling ---------------- */
/* which gradient kernel serves branch b: 1 = fx fused single-pass kernel (every
 * width <= 4, m <= 512), 3 = fxl (every width <= 4, 512 < m <= 4096: one wave
 * per 512-marker block), 2 = wide fused kernel (one hidden layer, W, S <= 32,
 * m <= 128: masked layer on i8 MFMA, hidden GEMMs on f32 or bf16 MFMA),
 * 0 = the layered gx path (any depth / widths: batched MFMA GEMMs per layer) */
int bann_branch_kernel_path(const bann_ctx* ctx, int32_t b);
/* name of the fused gradient kernel family used for branches of <= 512 markers */
const char* bann_fused_kernel_name(void);
/* wide kernel: run the hidden-layer GEMMs (forward, error propagation, dW1) on
 * the bf16 MFMA with bf16-rounded operands (1) instead of at f32 accuracy (0,
 * default: each f32 operand as three bf16 planes, six plane products per
 * product on the bf16 MFMA; BANN_WX_EXACT=1 selects the f32 MFMA instead).
 * BASELINE config C5's "bf16 hidden GEMM on MFMA vs fp32": bf16 operand
 * rounding (~1e-3 relative on gradients; not parity-exact).  Any time. */
int bann_set_hidden_gemm_bf16(bann_ctx* ctx, int32_t enabled);
/* replay a trajectory's whole launch sequence as one captured HIP graph in
 * bann_hmc_step (1) or launch kernel by kernel (0; default, or BANN_HMC_GRAPH);
 * the same launches, the same bits.  Trajectory recording always launches. */
int bann_set_graph_replay(bann_ctx* ctx, int32_t enabled);
/* the current graph-replay setting (0 / 1), or a negative status */
int bann_get_graph_replay(const bann_ctx* ctx);
/* force every branch onto the layered gx path (0) or allow the fused kernels (1) */
int bann_set_fused_enabled(bann_ctx* ctx, int32_t enabled);
/* bytes of packed genotype data read per full gradient evaluation of all branches */
int64_t bann_packed_genotype_bytes(const bann_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* BANN_H */
