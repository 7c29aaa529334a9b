/*
 * bann_net.h — C ABI of the sequential network driver: Net<B>::train over the
 * HIP branch kernels of bann.h, and the Net<B> model file.
 *
 * Replaces (medical-genomics-group/rs-bann):
 *   Net::train             src/net/net.rs:201-358 (HMC path: per sweep, branches
 *                          in shuffled order, each against the residual refreshed
 *                          after the previous one -- the reference's Gibbs order)
 *   initialize_stats       src/net/net.rs:158-171
 *   OutputBias             src/net/net.rs:29-72
 *   LogPosteriorDensity    src/net/log_posterior_density.rs:18-68
 *   TrainingStats          src/net/train_stats.rs:24-88
 *   GlobalParams           src/net/params.rs:13-63
 *   Net::to_file/from_file src/net/net.rs:107-115 (bincode 1.3 legacy encoding of
 *                          the Net<B> struct)
 *
 * The per-branch math (predict, the HMC trajectory, step sizes) and the
 * residual bookkeeping (the context's device residual, bann.h "the network
 * residual on the device": net.rs keeps it as a device Array too) run on the
 * device through bann.h; the Gibbs precision draws, the output bias and the log
 * posterior density -- scalars -- stay on the host, as in the reference
 * (north_star: "the Gibbs hyperparameter sweep stays on the host").  Same
 * conventions as bann.h: int status codes, host pointers read or written inside
 * the call and never retained.
 */
#ifndef BANN_NET_H
#define BANN_NET_H

#include <stdint.h>

#include "bann.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bann_net bann_net;

/* NetworkPrecisionHyperparameters (params.rs:134-142): Gamma (shape, scale) of
 * the precision priors of the dense, summary and output layers.  The reference
 * default is vague: shape 0.001, scale 1000 (params.rs:119-124). */
typedef struct {
  float dense_shape, dense_scale;
  float summary_shape, summary_scale;
  float output_shape, output_scale;
} bann_precision_hyperparams;

/* The MCMCCfg fields (mcmc_cfg.rs:181-204) Net::train reads on its HMC path.
 * Defaults (MCMCCfgBuilder::default, mcmc_cfg.rs:34-56): factor 1, max error 10,
 * L 100, Izmailov, chain 100, burn_in chain-1, precisions sampled, ML bias,
 * no joint HMC. */
typedef struct {
  float hmc_step_size_factor;
  float hmc_max_hamiltonian_error;
  int32_t hmc_integration_length;
  int32_t hmc_step_size_mode; /* bann_step_mode: BANN_STEP_IZMAILOV, BANN_STEP_UNIFORM, BANN_STEP_RANDOM or
                                 BANN_STEP_STD_SCALED (StepSizeMode, mcmc_cfg.rs:264-270); StdScaled is
                                 refused for ARD-prior branches, whose reference step sizes are empty
                                 (ridge_ard.rs:56-68, lasso_ard.rs:62-74); joint HMC uses random sizes */
  int32_t chain_length;
  int32_t burn_in;
  int32_t fixed_param_precisions;
  int32_t sampled_output_bias;
  int32_t trace;         /* outdir/trace: the BranchCfgs as a JSON line after init and every sweep (net.rs:241-244, 350-353) */
  int32_t trajectories;  /* outdir/traj: one JSON Trajectory line per HMC step (trajectory.rs, branch_sampler.rs:1196-1289) */
  int32_t joint_hmc;     /* MCMCCfg::joint_hmc: hmc_step_joint over params and precisions, no Gibbs draws
                            (net.rs:270-290; random step sizes, branch_sampler.rs:1092-1101) */
  int32_t gradient_descent;        /* MCMCCfg::gradient_descent (takes precedence, net.rs:282-290):
                                      BranchSampler::gradient_descent (branch_sampler.rs:964-1002), L ascent
                                      steps with a doubling / halving rss line search from the step size
                                      factor; Gibbs draws as HMC; always accepted; no trajectories */
  int32_t gradient_descent_joint;  /* MCMCCfg::gradient_descent_joint: gradient_descent_joint (1019-1066), L
                                      ascent steps of params and precisions at the step size factor, no Gibbs
                                      draws; rejected if the error precision ends <= 0 */
  int32_t effect_sizes;  /* MCMCCfg::effect_sizes (mcmc_cfg.rs:29): after burn-in, every branch update
                            writes outdir/effect_sizes/<chain_ix>_<branch_ix>, the n x m effect_sizes
                            of the branch as CSV (net.rs:307-315, 458-465, 571-587) */
} bann_mcmc_cfg;

/* Host random source for the driver's draws (the reference's ThreadRng,
 * net.rs:218 and branch rng_mut()).  A NULL member selects the built-in
 * generator (mt19937_64 seeded at bann_net_create).  Tests install hooks that
 * replay the oracle's stream.  Draw order per branch update: error precision
 * (1 gamma); unless fixed precisions, per layer l < L-1 the weight precisions
 * (one gamma per input node for ARD priors, else one) then the bias precision
 * (1 gamma), then the output-layer precision (1 gamma); the momentum (P
 * normals, param_vec order -- only while a normal hook is installed: without
 * one the momentum is drawn on the device, as the reference's ArrayFire randn
 * does, from one 64-bit seed of the built-in generator); the acceptance uniform (1 uniform); then, with
 * sampled output bias, 1 gamma + 1 normal.  Random step sizes: P uniforms
 * (param_vec order) before the momentum.  Joint HMC instead: no Gibbs draws;
 * P + Q uniforms (step sizes, [param_vec | precision_vec]), P + Q normals
 * (momentum), the acceptance uniform.  Each sweep of bann_net_train starts
 * with the branch shuffle: nb-1 uniforms (Fisher-Yates, i = nb-1 .. 1,
 * j = floor(u (i+1))); bann_net_train_single_branch draws no shuffle. */
typedef struct {
  void* user;
  double (*uniform)(void* user);
  double (*normal)(void* user);
  double (*gamma)(void* user, double shape, double scale);
} bann_rng_hooks;

/* Summary of TrainingStats + the current global state. */
typedef struct {
  uint64_t num_samples, num_accepted, num_early_rejected;
  int32_t num_records;    /* entries of mse_train / lpd recorded so far */
  float mse_train_last;   /* sum(residual^2) / n at the last record (net.rs:597-610) */
  float lpd_last;         /* LogPosteriorDensity::lpd at the last record */
  float output_bias;      /* OutputBias::bias */
  float error_precision;  /* GlobalParams::error_precision */
  float output_layer_precision;
  float output_reg_sum;   /* GlobalParams::output_weight_summary_stats.reg_sum */
} bann_train_summary;

/* A network over every branch of a finalized context.  Global state follows
 * BlockNetCfg::build_net (architectures.rs:187-237): error precision 2,
 * output-layer precision = branch 0's current output precision, the output
 * weight summary statistic summed over branches (sum of squares for ridge
 * priors, sum of abs for lasso), OutputBias {2, 1, 0}.  The context's branch
 * params / precisions are the initial BranchCfgs.  std-normal branches are
 * rejected with BANN_E_ARG: the reference panics in Net::train for them
 * (log_posterior_density.rs:55 -> std_normal_branch.rs:129 unimplemented!). */
int bann_net_create(bann_ctx* ctx, const bann_precision_hyperparams* hp, uint64_t seed, bann_net** out);
int bann_net_destroy(bann_net* net);
int bann_net_set_rng_hooks(bann_net* net, const bann_rng_hooks* hooks);
/* override GlobalParams / OutputBias (e.g. to continue a loaded chain) */
int bann_net_set_global(bann_net* net, float error_precision, float output_layer_precision, float output_bias,
                        float output_bias_precision);
/* test data of record_perf (net.rs:597-610: mse_test = rss / n_test): a
 * context over the test cohort with the same branches (count, markers, layer
 * widths) and targets y_test[n_test]; the driver copies its current
 * parameters there at every record.  NULL detaches (mse_test: None). */
int bann_net_set_test_data(bann_net* net, bann_ctx* test_ctx, const float* y_test, int64_t n_test);
/* the recorded mse_test series (min(cap, records) entries); 0 entries without test data */
int bann_net_records_test(const bann_net* net, float* mse_test, int32_t cap);
/* Net::train (net.rs:201-358) on the phenotype y[n].  outdir (may be NULL):
 * models/<chain_ix>.bin after burn-in (net.rs:338-342, 565-569) and
 * training_stats (JSON, train_stats.rs:83-87). */
int bann_net_train(bann_net* net, const float* y, int64_t n, const bann_mcmc_cfg* cfg, const char* outdir);
/* Net::train_single_branch (net.rs:360-507): branch 0 only, one HMC update per
 * chain iteration, record_perf / model file / trace after every update */
int bann_net_train_single_branch(bann_net* net, const float* y, int64_t n, const bann_mcmc_cfg* cfg,
                                 const char* outdir);
/* Net::perturb (net.rs:187-199, params.rs:219-233, 602-614): add params_by to
 * every weight and bias and / or precisions_by to every precision of every
 * branch (has_* = 0: that part untouched), e.g. to restart a loaded chain */
int bann_net_perturb(bann_net* net, int32_t has_params, float params_by, int32_t has_precisions,
                     float precisions_by);
/* Net::predict (net.rs:545-559): y_hat[i] = bias + sum_b f_b (f32, branch order)
 * on the cohort of ctx, a context with the net's branches (count, markers, layer
 * widths) -- e.g. a test cohort -- or NULL for the net's own context.  The net's
 * current parameters are loaded into ctx first. */
int bann_net_predict(bann_net* net, bann_ctx* ctx, float* y_hat_out);
/* Net::rss / Net::mse (net.rs:637-646) on the cohort of ctx (NULL: the net's own)
 * against y[n]: sum (y - y_hat)^2 with y_hat of bann_net_predict; mse = rss / n */
int bann_net_rss(bann_net* net, bann_ctx* ctx, const float* y, int64_t n, double* rss_out);
/* Net::gradient (net.rs:520-527): every branch's log_density_gradient against
 * the phenotype y[n] itself (not the residual), at the net's parameters and
 * precisions, one packed launch; grad_out = the branches' param_vecs
 * concatenated in branch order.  ctx: a context with the net's branches or NULL
 * (the net's own, whose branch targets this overwrites). */
int bann_net_gradient(bann_net* net, bann_ctx* ctx, const float* y, int64_t n, float* grad_out);
/* Net::branch_r2s (net.rs:648-656, r2 = 1 - rss(x_b, y) / sum y^2,
 * branch_sampler.rs:911-913) for every branch against y[n]; ctx as above */
int bann_net_branch_r2s(bann_net* net, bann_ctx* ctx, const float* y, int64_t n, float* r2_out);
/* Net::activations (net.rs:509-518) of branch b: forward_feed's activations of
 * every layer at the net's parameters (bann_forward_feed layout); ctx as above */
int bann_net_activations(bann_net* net, bann_ctx* ctx, int32_t b, float* act_out);
/* Net::population_effect_sizes (net.rs:529-543): per branch, in branch order, the
 * mean over the individuals of ctx's cohort of effect_sizes (branch_sampler.rs:784-811)
 * at the net's parameters: sum_b m_b floats; ctx as above */
int bann_net_population_effect_sizes(bann_net* net, bann_ctx* ctx, float* out);
int bann_net_summary(const bann_net* net, bann_train_summary* out);
/* the recorded mse_train / lpd series (TrainingStats::mse_train / lpd);
 * writes min(cap, num_records) entries of each (either may be NULL) */
int bann_net_records(const bann_net* net, float* mse_train, float* lpd, int32_t cap);
/* the residual y - bias - sum_b f_b after the last branch update (n floats,
 * copied from the context's device residual) */
int bann_net_residual(const bann_net* net, float* out);
/* Net::to_file (net.rs:112-115): bincode Net<B> of the current state */
int bann_net_save(const bann_net* net, const char* path);
/* Net::from_file (net.rs:107-110): read a bincode Net<B> whose branches match
 * the context's (count, markers, layer widths); loads params / precisions into
 * the context and the global state, output bias, stats and LPD into the net. */
int bann_net_load(bann_net* net, const char* path);
const char* bann_net_last_error(const bann_net* net);

#ifdef __cplusplus
}
#endif
#endif /* BANN_NET_H */
