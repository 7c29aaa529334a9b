// bann_net.cpp — host side of the sequential network driver (include/bann_net.h):
// Net<B>::train over the HIP branch kernels of bann.h, the Gibbs precision
// draws, the output bias, the log posterior density, TrainingStats and the
// bincode Net<B> model file.
//
// Host C++ only.  Every per-branch computation (predict, the HMC trajectory with
// its device step sizes and gradients) and the residual bookkeeping (the
// context's device residual) go through the bann.h entry points; what stays
// here is what the reference also keeps on the host between branch updates:
// Gamma/Normal draws from host RNG and scalar log-density terms (net.rs:201-358).
#include <sys/stat.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/bann_net.h"

#define BANN_NET_MAXL 64  // layer widths read back per branch (bann_branch_info)

// bann_residual.hip (library-internal): bann_residual_from_target + bann_residual_shift(add) in one launch
int residual_from_target_shift(bann_ctx* ctx, int32_t b, float add, double* sum, double* sumsq, double* sum_after,
                               double* sumsq_after);
// bann_api.hip (library-internal): bann_hmc_step + bann_branch_get_params + residual_from_target_shift
// for one branch with one host wait (stats: sum, sum of squares before / after the shift)
int hmc_step_tail(bann_ctx* ctx, int32_t b, int32_t L, float max_dh, int32_t step_mode, float factor, const float* eps,
                  const float* momentum, uint64_t seed, const float* u, float add, int32_t* status_out,
                  float* params_out, double* stats);

namespace {

enum { P_RIDGE_ARD = 0, P_RIDGE_BASE = 1, P_LASSO_ARD = 2, P_LASSO_BASE = 3, P_STD_NORMAL = 4 };
bool is_ard(int prior) { return prior == P_RIDGE_ARD || prior == P_LASSO_ARD; }
bool is_lasso(int prior) { return prior == P_LASSO_ARD || prior == P_LASSO_BASE; }

// One branch: the BranchCfg (branch_cfg.rs:8-16) held on the host between
// updates, with the offsets of its layers in the param / precision vectors.
struct Branch {
  int m = 0, L = 0, act = 0, prior = 0;
  std::vector<int> widths, win;        // out / in width of layer l
  std::vector<int64_t> woff, boff;     // param_vec offsets of W_l (in x out, col-major) and b_l
  std::vector<int64_t> wpoff, wpn;     // precision_vec offset / count of layer l's weight precisions
  int64_t bpoff = 0, epoff = 0;        // first bias precision, the error precision
  int64_t P = 0, NP = 0, num_weights = 0;
  std::vector<float> params, prec;     // BranchParamsHost / BranchPrecisionsHost as flat vectors
  float ows_reg_sum = 0.f;             // BranchParamsHost::output_weight_summary_stats
  uint64_t ows_num = 0;

  int64_t out_prec_ix() const { return wpoff[L - 1]; }
  // summary_stat_fn_host of the output weights (ridge_ard.rs:39-41, lasso_ard.rs:45-47)
  double out_stat() const {
    const float* w = params.data() + woff[L - 1];
    double s = 0.0;
    for (int j = 0; j < win[L - 1]; ++j) s += is_lasso(prior) ? std::fabs((double)w[j]) : (double)w[j] * w[j];
    return s;
  }
};

struct Writer {  // bincode 1.3 legacy config: fixint, little-endian
  std::vector<uint8_t> b;
  void raw(const void* p, size_t k) { b.insert(b.end(), (const uint8_t*)p, (const uint8_t*)p + k); }
  void u8(uint8_t v) { raw(&v, 1); }
  void u32(uint32_t v) { raw(&v, 4); }
  void u64(uint64_t v) { raw(&v, 8); }
  void f32(float v) { raw(&v, 4); }
  void vf32(const float* p, size_t k) {
    u64(k);
    raw(p, 4 * k);
  }
  void vu64(const std::vector<int>& v) {
    u64(v.size());
    for (int x : v) u64((uint64_t)x);
  }
};

struct Reader {
  const uint8_t* p;
  size_t n, pos = 0;
  bool ok = true;
  void raw(void* d, size_t k) {
    if (!ok || pos + k > n) {
      ok = false;
      std::memset(d, 0, k);
      return;
    }
    std::memcpy(d, p + pos, k);
    pos += k;
  }
  uint8_t u8() {
    uint8_t v;
    raw(&v, 1);
    return v;
  }
  uint32_t u32() {
    uint32_t v;
    raw(&v, 4);
    return v;
  }
  uint64_t u64() {
    uint64_t v;
    raw(&v, 8);
    return v;
  }
  float f32() {
    float v;
    raw(&v, 4);
    return v;
  }
  std::vector<float> vf32() {
    const uint64_t k = u64();
    if (!ok || k > (n - pos) / 4) {
      ok = false;
      return {};
    }
    std::vector<float> v(k);
    raw(v.data(), 4 * k);
    return v;
  }
  std::vector<uint64_t> vu64() {
    const uint64_t k = u64();
    if (!ok || k > (n - pos) / 8) {
      ok = false;
      return {};
    }
    std::vector<uint64_t> v(k);
    for (auto& x : v) x = u64();
    return v;
  }
};

}  // namespace

struct bann_net {
  bann_ctx* ctx = nullptr;
  bann_precision_hyperparams hp{};
  std::mt19937_64 gen;
  bann_rng_hooks hooks{};
  std::string err;
  std::vector<Branch> br;
  int64_t n = 0;
  double rss_cur = 0.0;  // sum of squares of the context's device residual after the last operation
  // GlobalParams (params.rs:13-18)
  float g_eprec = 2.f, g_oprec = 0.05f, g_reg_sum = 0.f;
  uint64_t g_num = 0;
  // OutputBias (net.rs:29-36); build_net's initial value (architectures.rs:224-228)
  float ob_eprec = 2.f, ob_prec = 1.f, ob_bias = 0.f;
  // TrainingStats (train_stats.rs:24-32)
  uint64_t ns = 0, nacc = 0, nearly = 0;
  std::vector<float> mse, lpd;
  // LogPosteriorDensity (log_posterior_density.rs:9-16)
  float lpd_rss = -INFINITY, lpd_outw = -INFINITY;
  std::vector<float> lpd_local;
  // test data of record_perf (net.rs:597-610)
  bann_ctx* test_ctx = nullptr;
  std::vector<float> y_test, mse_test;
};

namespace {

int fail(bann_net* t, int code, const std::string& msg) {
  if (t) t->err = msg;
  return code;
}
#define CKB(call)                                                                                   \
  do {                                                                                              \
    const int rc_ = (call);                                                                         \
    if (rc_ < 0) return fail(t, rc_, std::string(#call) + ": " + bann_last_error(t->ctx));         \
  } while (0)

double draw_uniform(bann_net* t) {
  if (t->hooks.uniform) return t->hooks.uniform(t->hooks.user);
  return std::uniform_real_distribution<double>(0.0, 1.0)(t->gen);
}
double draw_normal(bann_net* t) {
  if (t->hooks.normal) return t->hooks.normal(t->hooks.user);
  return std::normal_distribution<double>(0.0, 1.0)(t->gen);
}
double draw_gamma(bann_net* t, double shape, double scale) {
  if (t->hooks.gamma) return t->hooks.gamma(t->hooks.user, shape, scale);
  return std::gamma_distribution<double>(shape, scale)(t->gen);
}

// NetworkPrecisionHyperparameters::layer_prior_hyperparams (params.rs:146-163)
void layer_hp(const bann_net* t, int l, int L, double& shape, double& scale) {
  if (l == L - 1) {
    shape = t->hp.output_shape;
    scale = t->hp.output_scale;
  } else if (l == L - 2) {
    shape = t->hp.summary_shape;
    scale = t->hp.summary_scale;
  } else {
    shape = t->hp.dense_shape;
    scale = t->hp.dense_scale;
  }
}

// gibbs_steps.rs:76-94 / 113-129 (ridge) and 25-57 (lasso): Gamma posterior draws
double ridge_posterior(bann_net* t, double shape, double scale, double sum_sq, double num) {
  return draw_gamma(t, shape + num / 2.0, 2.0 * scale / (2.0 + scale * sum_sq));
}
double lasso_posterior(bann_net* t, double shape, double scale, double sum_abs, double num) {
  return draw_gamma(t, shape + num, scale / (1.0 + scale * sum_abs));
}

double sum_sq(const float* v, int64_t k) {
  double s = 0.0;
  for (int64_t i = 0; i < k; ++i) s += (double)v[i] * v[i];
  return s;
}
double sum_abs(const float* v, int64_t k) {
  double s = 0.0;
  for (int64_t i = 0; i < k; ++i) s += std::fabs((double)v[i]);
  return s;
}

// BranchCfg::update_global_params (branch_cfg.rs:59-63)
void cfg_update_global(bann_net* t, Branch& B) {
  B.prec[B.epoff] = t->g_eprec;
  B.prec[B.out_prec_ix()] = t->g_oprec;
  B.ows_reg_sum = t->g_reg_sum;
  B.ows_num = t->g_num;
}

// sample_prior_precisions: ridge_ard.rs:271-301, lasso_ard.rs:271-298,
// ridge_base.rs / lasso_base.rs (whole-layer draws); biases always ridge.
void sample_prior_precisions(bann_net* t, Branch& B) {
  for (int l = 0; l < B.L - 1; ++l) {
    double shape, scale;
    layer_hp(t, l, B.L, shape, scale);
    const float* W = B.params.data() + B.woff[l];
    const int in = B.win[l], out = B.widths[l];
    if (is_ard(B.prior)) {
      for (int j = 0; j < in; ++j) {  // one precision per input node (row of W_l)
        double s = 0.0;
        for (int k = 0; k < out; ++k) {
          const double w = W[(int64_t)k * in + j];
          s += B.prior == P_LASSO_ARD ? std::fabs(w) : w * w;
        }
        B.prec[B.wpoff[l] + j] = (float)(B.prior == P_LASSO_ARD ? draw_gamma(t, out + shape, scale / (1.0 + scale * s))
                                                                : draw_gamma(t, out / 2.0 + shape,
                                                                             2.0 * scale / (2.0 + scale * s)));
      }
    } else if (B.prior == P_LASSO_BASE) {
      B.prec[B.wpoff[l]] = (float)lasso_posterior(t, shape, scale, sum_abs(W, (int64_t)in * out), (double)in * out);
    } else {
      B.prec[B.wpoff[l]] = (float)ridge_posterior(t, shape, scale, sum_sq(W, (int64_t)in * out), (double)in * out);
    }
    const float* b = B.params.data() + B.boff[l];
    B.prec[B.bpoff + l] = (float)ridge_posterior(t, shape, scale, sum_sq(b, out), out);
  }
}

// log_density_joint_wrt_biases (branch_sampler.rs:260-279) + _wrt_local_weights
// (ridge_ard.rs:119-148, ridge_base.rs:119-137, lasso_ard.rs:119-149, lasso_base.rs:119-137)
double ld_joint_local(const bann_net* t, const Branch& B) {
  double ld = 0.0;
  for (int l = 0; l < B.L - 1; ++l) {
    double shape, scale;
    layer_hp(t, l, B.L, shape, scale);
    const float* b = B.params.data() + B.boff[l];
    const double lb = B.prec[B.bpoff + l];
    ld -= lb * (sum_sq(b, B.widths[l]) / 2.0 + 1.0 / scale);
    ld += (shape + (B.widths[l] - 2.0) / 2.0) * std::log(lb);
    const float* W = B.params.data() + B.woff[l];
    const int in = B.win[l], out = B.widths[l];
    if (is_ard(B.prior)) {
      for (int j = 0; j < in; ++j) {
        const double lam = B.prec[B.wpoff[l] + j];
        double s = 0.0;
        for (int k = 0; k < out; ++k) {
          const double w = W[(int64_t)k * in + j];
          s += B.prior == P_LASSO_ARD ? std::fabs(w) : w * w;
        }
        if (B.prior == P_RIDGE_ARD) {
          ld -= (s / 2.0 + 1.0 / scale) * lam;
          ld += (shape + (out - 2.0) / 2.0) * std::log(lam);
        } else {
          ld -= (s + 1.0 / scale) * lam;
          ld += (shape + out - 1.0) * std::log(lam);
        }
      }
    } else {
      const double lam = B.prec[B.wpoff[l]];
      const double k = (double)in * out;
      if (B.prior == P_RIDGE_BASE) {
        ld -= (sum_sq(W, (int64_t)k) / 2.0 + 1.0 / scale) * lam;
        ld += (shape + (k - 2.0) / 2.0) * std::log(lam);
      } else {
        ld -= (sum_abs(W, (int64_t)k) + 1.0 / scale) * lam;
        ld += (shape + k - 1.0) * std::log(lam);
      }
    }
  }
  return ld;
}

// log_density_joint_wrt_output_weights (ridge_ard.rs:150-169, lasso_ard.rs:153-172;
// base priors identical): global statistic = own + the other branches' (`others`)
double ld_joint_out(const bann_net* t, const Branch& B, double others) {
  double shape, scale;
  layer_hp(t, B.L - 1, B.L, shape, scale);
  const double lam = B.prec[B.out_prec_ix()];
  const double num = (double)B.ows_num;
  if (is_lasso(B.prior)) return -((B.out_stat() + others) + 1.0 / scale) * lam + (shape + num - 1.0) * std::log(lam);
  return -(0.5 * (B.out_stat() + others) + 1.0 / scale) * lam + (shape + (num - 2.0) / 2.0) * std::log(lam);
}

// LogPosteriorDensity::update_from_branch (log_posterior_density.rs:27-61);
// the rss of the device residual comes from the residual operation before it
void update_lpd(bann_net* t, int b, double others) {
  const Branch& B = t->br[b];
  t->lpd_local[b] = (float)ld_joint_local(t, B);
  t->lpd_outw = (float)ld_joint_out(t, B, others);
  const double rss = t->rss_cur;
  const double le = B.prec[B.epoff];
  t->lpd_rss = (float)(std::log(le) * (t->hp.output_shape + (t->n - 2.0) / 2.0) -
                       le * (rss / 2.0 + 1.0 / t->hp.output_scale));
}

// Net::record_perf (net.rs:597-610); with test data: Net::mse (644-646) = rss / n
// of the network prediction sum_b f_b + bias on the test cohort
int record_perf(bann_net* t) {
  double l = (double)t->lpd_rss + t->lpd_outw;
  for (float v : t->lpd_local) l += v;
  t->lpd.push_back((float)l);
  t->mse.push_back((float)(t->rss_cur / (double)t->n));
  if (t->test_ctx) {
    const int nb = (int)t->br.size();
    const int64_t nt = (int64_t)t->y_test.size();
    std::vector<int32_t> all(nb);
    for (int b = 0; b < nb; ++b) {
      all[b] = b;
      const int rc = bann_branch_set_params(t->test_ctx, b, t->br[b].params.data());
      if (rc < 0) return fail(t, rc, std::string("test context: ") + bann_last_error(t->test_ctx));
    }
    std::vector<float> preds((size_t)nb * nt);
    const int rc = bann_predict_many(t->test_ctx, all.data(), nb, preds.data());
    if (rc < 0) return fail(t, rc, std::string("test context: ") + bann_last_error(t->test_ctx));
    double rss = 0.0;
    for (int64_t i = 0; i < nt; ++i) {
      double f = t->ob_bias;
      for (int b = 0; b < nb; ++b) f += preds[(size_t)b * nt + i];
      const double r = (double)t->y_test[i] - f;
      rss += r * r;
    }
    t->mse_test.push_back((float)(rss / (double)nt));
  }
  return BANN_OK;
}

// serde_json of a float (non-finite values have no JSON form: serde writes null)
void jf(std::string& o, double v) {
  char buf[32];
  if (std::isfinite(v))
    std::snprintf(buf, sizeof(buf), "%.9g", v);
  else
    std::snprintf(buf, sizeof(buf), "null");
  o += buf;
}
void jvec(std::string& o, const float* p, int64_t k) {
  o += '[';
  for (int64_t i = 0; i < k; ++i) {
    if (i) o += ',';
    jf(o, p[i]);
  }
  o += ']';
}
void jvec_u(std::string& o, const std::vector<int>& v) {
  o += '[';
  for (size_t i = 0; i < v.size(); ++i) o += (i ? "," : "") + std::to_string(v[i]);
  o += ']';
}

// the branch_cfgs as serde_json (BranchCfg, branch_cfg.rs:7-16 and params.rs:192-199, 468-476)
std::string trace_line(const bann_net* t) {
  static const char* acts[] = {"Tanh", "ReLU", "LeakyReLU", "SiLU", "Identity"};
  std::string o = "[";
  for (size_t bi = 0; bi < t->br.size(); ++bi) {
    const Branch& B = t->br[bi];
    if (bi) o += ',';
    o += "{\"num_params\":" + std::to_string(B.P) + ",\"num_weights\":" + std::to_string(B.num_weights) +
         ",\"num_markers\":" + std::to_string(B.m) + ",\"layer_widths\":";
    jvec_u(o, B.widths);
    o += ",\"params\":{\"weights\":[";
    for (int l = 0; l < B.L; ++l) {
      if (l) o += ',';
      jvec(o, B.params.data() + B.woff[l], (int64_t)B.win[l] * B.widths[l]);
    }
    o += "],\"biases\":[";
    for (int l = 0; l < B.L - 1; ++l) {
      if (l) o += ',';
      jvec(o, B.params.data() + B.boff[l], B.widths[l]);
    }
    o += "],\"layer_widths\":";
    jvec_u(o, B.widths);
    o += ",\"num_markers\":" + std::to_string(B.m) + ",\"output_weight_summary_stats\":{\"reg_sum\":";
    jf(o, B.ows_reg_sum);
    o += ",\"num_params\":" + std::to_string(B.ows_num) + "}},\"precisions\":{\"weight_precisions\":[";
    for (int l = 0; l < B.L; ++l) {
      if (l) o += ',';
      jvec(o, B.prec.data() + B.wpoff[l], B.wpn[l]);
    }
    o += "],\"bias_precisions\":[";
    for (int l = 0; l < B.L - 1; ++l) {
      if (l) o += ',';
      jvec(o, B.prec.data() + B.bpoff + l, 1);
    }
    o += "],\"error_precision\":";
    jvec(o, B.prec.data() + B.epoff, 1);
    o += "},\"activation_function\":\"" + std::string(acts[B.act]) + "\"}";
  }
  return o + "]\n";
}

// one Trajectory (trajectory.rs:3-11) of the last hmc_step of branch b as serde_json
// one Trajectory JSON line (trajectory.rs:1-43): hmc_step records params, ldg and
// -H (branch_sampler.rs:1253-1289), hmc_step_joint also the precisions and the
// joint ldg [params | precisions] (1126-1135)
int traj_line(bann_net* t, int b, bool joint, std::string& o) {
  const Branch& B = t->br[b];
  const int64_t Q = joint ? B.NP : 0, G = B.P + Q;
  int32_t steps = 0;
  if (joint)
    CKB(bann_branch_get_trajectory_joint(t->ctx, b, 0, &steps, nullptr, nullptr, nullptr, nullptr));
  else
    CKB(bann_branch_get_trajectory(t->ctx, b, 0, &steps, nullptr, nullptr, nullptr));
  std::vector<float> pr((size_t)steps * B.P), pq((size_t)steps * Q), lg((size_t)steps * G);
  std::vector<double> h(steps + 1);
  if (joint)
    CKB(bann_branch_get_trajectory_joint(t->ctx, b, steps, &steps, pr.data(), pq.data(), lg.data(), h.data()));
  else
    CKB(bann_branch_get_trajectory(t->ctx, b, steps, &steps, pr.data(), lg.data(), h.data()));
  auto rows = [&](const std::vector<float>& v, int64_t w) {
    for (int k = 0; k < steps; ++k) {
      if (k) o += ',';
      jvec(o, v.data() + (size_t)k * w, w);
    }
  };
  o = "{\"params\":[";
  rows(pr, B.P);
  o += "],\"precisions\":[";
  if (joint) rows(pq, Q);
  o += "],\"ldg\":[";
  rows(lg, G);
  o += "],\"num_ldg\":[],\"hamiltonian\":[";
  for (int k = 0; k <= steps; ++k) {
    if (k) o += ',';
    jf(o, (float)h[k]);
  }
  o += "]}\n";
  return BANN_OK;
}

int append_text(bann_net* t, const std::string& path, const std::string& text) {
  FILE* f = std::fopen(path.c_str(), "a");
  if (!f) return fail(t, BANN_E_ARG, "cannot open " + path);
  const bool ok = std::fwrite(text.data(), 1, text.size(), f) == text.size();
  return (std::fclose(f) == 0 && ok) ? BANN_OK : fail(t, BANN_E_ARG, "short write to " + path);
}

// Rust's Display of an f32 (f32::to_string, as net.rs:584 writes the effect
// sizes): the shortest decimal that reads back to the same f32 (the closest of
// them if several), printed positionally -- no exponent, no trailing ".0"
// ("1", "0.1", "0.0000001", "100000000000000000000"), "-0", "NaN", "inf".
void rust_f32(std::string& o, float v) {
  if (std::isnan(v)) {
    o += "NaN";
    return;
  }
  if (std::signbit(v)) o += '-';
  const float a = std::fabs(v);
  if (std::isinf(a)) {
    o += "inf";
    return;
  }
  if (a == 0.f) {
    o += '0';
    return;
  }
  char buf[48];
  std::string dig;
  int e10 = 0;
  for (int p = 0; p < 9; ++p) {  // p + 1 significant digits; 9 always round-trip
    std::snprintf(buf, sizeof(buf), "%.*e", p, (double)a);
    char* ep = std::strchr(buf, 'e');
    std::string d(buf, ep);
    const int ex = std::atoi(ep + 1);
    d.erase(std::remove(d.begin(), d.end(), '.'), d.end());
    auto reads_back = [&](const std::string& s) {
      std::snprintf(buf, sizeof(buf), "%s.%se%d", s.substr(0, 1).c_str(), s.substr(1).c_str(), ex);
      return std::strtof(buf, nullptr) == a;
    };
    if (reads_back(d)) {
      dig = d;
      e10 = ex;
      break;
    }
    // the correctly rounded p+1 digits miss, a neighbour of the same length may not
    // (asymmetric rounding intervals at powers of two): take the closer one that reads back
    std::string best;
    double bd = 0.0;
    for (int s = -1; s <= 1; s += 2) {
      long long q = std::atoll(d.c_str()) + s;
      std::string c = std::to_string(q);
      if ((int)c.size() != p + 1) continue;
      if (reads_back(c)) {
        std::snprintf(buf, sizeof(buf), "%s.%se%d", c.substr(0, 1).c_str(), c.substr(1).c_str(), ex);
        const double dist = std::fabs(std::strtod(buf, nullptr) - (double)a);
        if (best.empty() || dist < bd) {
          best = c;
          bd = dist;
        }
      }
    }
    if (!best.empty()) {
      dig = best;
      e10 = ex;
      break;
    }
  }
  while (dig.size() > 1 && dig.back() == '0') dig.pop_back();
  const int k = (int)dig.size(), pt = e10 + 1;  // value = 0.dig x 10^pt
  if (pt <= 0) {
    o += "0.";
    o.append((size_t)(-pt), '0');
    o += dig;
  } else if (pt < k) {
    o += dig.substr(0, pt);
    o += '.';
    o += dig.substr(pt);
  } else {
    o += dig;
    o.append((size_t)(pt - k), '0');
  }
}

bool mkdir_p(const std::string& d) {
  if (d.empty()) return true;
  std::string cur;
  for (size_t i = 0; i < d.size(); ++i) {
    cur += d[i];
    if ((d[i] == '/' || i + 1 == d.size()) && cur != "/") {
      if (mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return false;
    }
  }
  return true;
}

// Net::save_effect_sizes (net.rs:571-587): effect_sizes of branch b (n x m, the
// device chain of bann_effect_sizes) as CSV at dir/effect_sizes/<chain_ix>_<b>:
// one row per individual, one field per marker (transpose + chunks(m) of the
// column-major matrix), csv::Writer defaults (',' and "\n", numbers unquoted)
int save_effect_sizes(bann_net* t, int b, int chain_ix, const std::string& dir) {
  const Branch& B = t->br[b];
  const int64_t n = t->n, m = B.m;
  std::vector<float> e((size_t)n * m);
  CKB(bann_effect_sizes(t->ctx, b, e.data()));
  const std::string path = dir + "/effect_sizes/" + std::to_string(chain_ix) + "_" + std::to_string(b);
  FILE* f = std::fopen(path.c_str(), "w");
  if (!f) return fail(t, BANN_E_ARG, "cannot open " + path);
  std::string row;
  bool ok = true;
  for (int64_t i = 0; i < n && ok; ++i) {
    row.clear();
    for (int64_t j = 0; j < m; ++j) {
      if (j) row += ',';
      rust_f32(row, e[(size_t)j * n + i]);
    }
    row += '\n';
    ok = std::fwrite(row.data(), 1, row.size(), f) == row.size();
  }
  return (std::fclose(f) == 0 && ok) ? BANN_OK : fail(t, BANN_E_ARG, "short write to " + path);
}

Writer serialize(const bann_net* t) {
  Writer w;
  const auto& hp = t->hp;  // NetworkPrecisionHyperparameters (params.rs:134-142)
  w.f32(hp.dense_shape);
  w.f32(hp.dense_scale);
  w.f32(hp.summary_shape);
  w.f32(hp.summary_scale);
  w.f32(hp.output_shape);
  w.f32(hp.output_scale);
  w.u64(t->br.size());  // num_branches
  w.u64(t->br.size());  // branch_cfgs: Vec<BranchCfg>
  for (const Branch& B : t->br) {
    w.u64(B.P);
    w.u64(B.num_weights);
    w.u64(B.m);
    w.vu64(B.widths);
    // BranchParamsHost (params.rs:468-476)
    w.u64(B.L);
    for (int l = 0; l < B.L; ++l) w.vf32(B.params.data() + B.woff[l], (size_t)B.win[l] * B.widths[l]);
    w.u64(B.L - 1);
    for (int l = 0; l < B.L - 1; ++l) w.vf32(B.params.data() + B.boff[l], B.widths[l]);
    w.vu64(B.widths);
    w.u64(B.m);
    w.f32(B.ows_reg_sum);
    w.u64(B.ows_num);
    // BranchPrecisionsHost (params.rs:192-199)
    w.u64(B.L);
    for (int l = 0; l < B.L; ++l) w.vf32(B.prec.data() + B.wpoff[l], B.wpn[l]);
    w.u64(B.L - 1);
    for (int l = 0; l < B.L - 1; ++l) w.vf32(B.prec.data() + B.bpoff + l, 1);
    w.vf32(B.prec.data() + B.epoff, 1);
    w.u32((uint32_t)B.act);  // ActivationFunction (activation_functions.rs:6-12)
  }
  w.f32(t->ob_eprec);  // OutputBias
  w.f32(t->ob_prec);
  w.f32(t->ob_bias);
  w.u64(t->ns);  // TrainingStats
  w.u64(t->nacc);
  w.u64(t->nearly);
  w.vf32(t->mse.data(), t->mse.size());
  if (t->test_ctx) {  // mse_test: Option<Vec<f32>>
    w.u8(1);
    w.vf32(t->mse_test.data(), t->mse_test.size());
  } else {
    w.u8(0);
  }
  w.vf32(t->lpd.data(), t->lpd.size());
  w.f32(t->lpd_rss);  // LogPosteriorDensity
  w.f32(t->lpd_outw);
  w.vf32(t->lpd_local.data(), t->lpd_local.size());
  w.f32(t->g_eprec);  // GlobalParams
  w.f32(t->g_oprec);
  w.f32(t->g_reg_sum);
  w.u64(t->g_num);
  return w;  // branch_type: PhantomData, 0 bytes
}

int write_file(bann_net* t, const std::string& path) {
  const Writer w = serialize(t);
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return fail(t, BANN_E_ARG, "cannot open " + path + " for writing");
  const size_t k = std::fwrite(w.b.data(), 1, w.b.size(), f);
  const int rc = std::fclose(f);
  if (k != w.b.size() || rc != 0) return fail(t, BANN_E_ARG, "short write to " + path);
  return BANN_OK;
}

int write_training_stats(bann_net* t, const std::string& dir) {  // train_stats.rs:83-87 (serde_json)
  const std::string path = dir + "/training_stats";
  FILE* f = std::fopen(path.c_str(), "w");
  if (!f) return fail(t, BANN_E_ARG, "cannot open " + path);
  std::fprintf(f, "{\"num_samples\":%llu,\"num_accepted\":%llu,\"num_early_rejected\":%llu,\"mse_train\":[",
               (unsigned long long)t->ns, (unsigned long long)t->nacc, (unsigned long long)t->nearly);
  for (size_t i = 0; i < t->mse.size(); ++i) std::fprintf(f, i ? ",%.9g" : "%.9g", t->mse[i]);
  if (t->test_ctx) {
    std::fprintf(f, "],\"mse_test\":[");
    for (size_t i = 0; i < t->mse_test.size(); ++i) std::fprintf(f, i ? ",%.9g" : "%.9g", t->mse_test[i]);
    std::fprintf(f, "],\"lpd\":[");
  } else {
    std::fprintf(f, "],\"mse_test\":null,\"lpd\":[");
  }
  for (size_t i = 0; i < t->lpd.size(); ++i) std::fprintf(f, i ? ",%.9g" : "%.9g", t->lpd[i]);
  std::fprintf(f, "]}");
  std::fclose(f);
  return BANN_OK;
}

}  // namespace

extern "C" int bann_net_create(bann_ctx* ctx, const bann_precision_hyperparams* hp, uint64_t seed, bann_net** out) {
  if (!ctx || !out) return BANN_E_ARG;
  *out = nullptr;
  const int nb = bann_num_branches(ctx);
  if (nb <= 0) return BANN_E_STATE;
  bann_net* t = new bann_net();
  t->ctx = ctx;
  t->gen.seed(seed);
  if (hp) t->hp = *hp;
  else t->hp = bann_precision_hyperparams{0.001f, 1000.f, 0.001f, 1000.f, 0.001f, 1000.f};  // vague (params.rs:119-124)
  t->br.resize(nb);
  t->lpd_local.assign(nb, -INFINITY);
  for (int b = 0; b < nb; ++b) {
    Branch& B = t->br[b];
    int w[64];
    int rc = bann_branch_info(ctx, b, &B.m, &B.L, w, 64, &B.act, &B.prior);
    if (rc < 0 || B.L < 2 || B.L > 64) {
      delete t;
      return rc < 0 ? rc : BANN_E_SHAPE;
    }
    if (B.prior == P_STD_NORMAL) {  // Net::train panics for StdNormalBranch (net.rs:167 -> std_normal_branch.rs:129)
      delete t;
      return BANN_E_ARG;
    }
    B.widths.assign(w, w + B.L);
    B.win.resize(B.L);
    B.woff.resize(B.L);
    B.boff.resize(B.L - 1);
    B.wpoff.resize(B.L);
    B.wpn.resize(B.L);
    int64_t o = 0, po = 0;
    for (int l = 0; l < B.L; ++l) {
      B.win[l] = l == 0 ? B.m : B.widths[l - 1];
      B.woff[l] = o;
      o += (int64_t)B.win[l] * B.widths[l];
      B.wpoff[l] = po;
      B.wpn[l] = is_ard(B.prior) && l < B.L - 1 ? B.win[l] : 1;
      po += B.wpn[l];
    }
    B.num_weights = o;
    for (int l = 0; l < B.L - 1; ++l) {
      B.boff[l] = o;
      o += B.widths[l];
    }
    B.P = o;
    B.bpoff = po;
    B.epoff = po + B.L - 1;
    B.NP = B.epoff + 1;
    if (B.P != bann_num_params(ctx, b) || B.NP != bann_num_precisions(ctx, b)) {
      delete t;
      return BANN_E_SHAPE;
    }
    B.params.resize(B.P);
    B.prec.resize(B.NP);
    if ((rc = bann_branch_get_params(ctx, b, B.params.data())) < 0 ||
        (rc = bann_branch_get_precisions(ctx, b, B.prec.data())) < 0) {
      delete t;
      return rc;
    }
  }
  // BlockNetCfg::build_net (architectures.rs:187-237): summed output-weight
  // statistic and count, error precision 2, one output-layer precision
  double reg = 0.0;
  for (const Branch& B : t->br) {
    reg += B.out_stat();
    t->g_num += (uint64_t)B.win[B.L - 1];
  }
  t->g_reg_sum = (float)reg;
  t->g_oprec = t->br[0].prec[t->br[0].out_prec_ix()];
  *out = t;
  return BANN_OK;
}

extern "C" int bann_net_destroy(bann_net* t) {
  delete t;
  return BANN_OK;
}

extern "C" const char* bann_net_last_error(const bann_net* t) { return t ? t->err.c_str() : "null net"; }

extern "C" int bann_net_set_rng_hooks(bann_net* t, const bann_rng_hooks* hooks) {
  if (!t) return BANN_E_ARG;
  t->hooks = hooks ? *hooks : bann_rng_hooks{};
  return BANN_OK;
}

extern "C" int bann_net_set_global(bann_net* t, float error_precision, float output_layer_precision, float output_bias,
                                   float output_bias_precision) {
  if (!t) return BANN_E_ARG;
  if (!(error_precision > 0.f) || !(output_layer_precision > 0.f) || !(output_bias_precision > 0.f))
    return fail(t, BANN_E_ARG, "precisions must be positive");
  t->g_eprec = t->ob_eprec = error_precision;
  t->g_oprec = output_layer_precision;
  t->ob_bias = output_bias;
  t->ob_prec = output_bias_precision;
  return BANN_OK;
}

namespace {

// the per-trajectory draws of one branch update (order: include/bann_net.h)
struct Draws {
  std::vector<float> eps, mom;
  float u = 0.f;
};

// BranchParams::descend_gradient (params.rs:740-749; 357-367 for the precisions):
// v += step * g in f32, the ArrayFire op order (the product rounds first)
void descend(std::vector<float>& v, const float* g, float step) {
  for (size_t i = 0; i < v.size(); ++i) {
    const float d = step * g[i];
    v[i] = v[i] + d;
  }
}

// BranchSampler::gradient_descent (branch_sampler.rs:964-1002): L ascent steps
// on the log density, each with a doubling / halving line search over rss
// probes (probe_gradient_step, 1004-1016); always Accepted.  Every probe and
// gradient runs on the device (bann_rss / bann_log_density_gradient); the
// parameter vector moves on the host, in f32 as the reference.
int gradient_descent(bann_net* t, int b, const bann_mcmc_cfg* cfg, int32_t& status) {
  Branch& B = t->br[b];
  std::vector<float> th(B.P), g(B.P), probe(B.P);
  CKB(bann_branch_get_params(t->ctx, b, th.data()));
  CKB(bann_log_density_gradient(t->ctx, b, g.data(), nullptr));
  auto probe_rss = [&](float step, double& r) -> int {
    probe = th;
    descend(probe, g.data(), step);
    CKB(bann_branch_set_params(t->ctx, b, probe.data()));
    CKB(bann_rss(t->ctx, b, &r));
    return BANN_OK;
  };
  for (int k = 0; k < cfg->hmc_integration_length; ++k) {
    float step = cfg->hmc_step_size_factor;
    double prev = 0.0, twice = 0.0, curr = 0.0;
    int rc = probe_rss(step, prev);
    if (!rc) rc = probe_rss(2.f * step, twice);
    if (rc) return rc;
    const float f = twice < prev ? 2.f : 0.5f;
    step *= f;
    if ((rc = probe_rss(step, curr))) return rc;
    // terminates: halving reaches step * g == 0 (rss == prev), doubling inf / NaN
    for (int guard = 0; curr < prev && guard < 4096; ++guard) {
      prev = curr;
      step *= f;
      if ((rc = probe_rss(step, curr))) return rc;
    }
    step /= f;
    descend(th, g.data(), step);
    CKB(bann_branch_set_params(t->ctx, b, th.data()));
    CKB(bann_log_density_gradient(t->ctx, b, g.data(), nullptr));
  }
  status = BANN_ACCEPTED;
  return BANN_OK;
}

// BranchSampler::gradient_descent_joint (branch_sampler.rs:1019-1066): L ascent
// steps of the parameters and the precisions along the joint log-density
// gradient at the fixed step size factor; Rejected (state restored) if the error
// precision ends <= 0, else Accepted.
int gradient_descent_joint(bann_net* t, int b, const bann_mcmc_cfg* cfg, double others, int32_t& status) {
  Branch& B = t->br[b];
  const float hyper[6] = {t->hp.dense_shape, t->hp.dense_scale, t->hp.summary_shape,
                          t->hp.summary_scale, t->hp.output_shape, t->hp.output_scale};
  CKB(bann_branch_set_output_stats(t->ctx, b, (float)others, (float)t->g_num));
  std::vector<float> th(B.P), pr = B.prec, g(B.P + B.NP);
  CKB(bann_branch_get_params(t->ctx, b, th.data()));
  const std::vector<float> th0 = th, pr0 = pr;
  CKB(bann_log_density_gradient_joint(t->ctx, b, hyper, g.data(), nullptr, nullptr));
  for (int k = 0; k < cfg->hmc_integration_length; ++k) {
    descend(th, g.data(), cfg->hmc_step_size_factor);
    descend(pr, g.data() + B.P, cfg->hmc_step_size_factor);
    CKB(bann_branch_set_params(t->ctx, b, th.data()));
    CKB(bann_branch_set_precisions(t->ctx, b, pr.data()));
    CKB(bann_log_density_gradient_joint(t->ctx, b, hyper, g.data(), nullptr, nullptr));
  }
  status = BANN_ACCEPTED;
  if (!(pr[B.epoff] > 0.f)) {  // scalar_to_host(error_precision) <= 0.0 (1058-1062)
    CKB(bann_branch_set_params(t->ctx, b, th0.data()));
    CKB(bann_branch_set_precisions(t->ctx, b, pr0.data()));
    status = BANN_REJECTED;
  }
  return BANN_OK;
}

// one branch update of Net::train / train_single_branch (net.rs:261-332): Gibbs
// draws (unless joint), target = residual + f_b, the HMC trajectory on the
// device, the residual bookkeeping on the device, global params, output bias
int update_branch(bann_net* t, int b, const bann_mcmc_cfg* cfg, bool traj, const std::string& dir, Draws& dr,
                  int chain_ix) {
  Branch& B = t->br[b];
  const int64_t n = t->n;
  const double kout = t->hp.output_shape, sout = t->hp.output_scale;
  // cfg.update_global_params (net.rs:261-262).  train_single_branch applies it
  // AFTER from_cfg (net.rs:416-418), i.e. the branch runs on its cfg's values --
  // which are the globals too: initialize_stats (net.rs:158-166) applied them to
  // every cfg before the first iteration, and every later cfg is to_cfg of the
  // branch whose values became the globals (update_from_branch_cfg, 447-449)
  cfg_update_global(t, B);
  const double others = B.ows_reg_sum - B.out_stat();  // from_cfg (branch_struct.rs:26)
  // net.rs:270-277: no Gibbs draws for the joint samplers; the step (282-290):
  // gradient descent, joint gradient descent, joint HMC, else HMC
  const bool gd = cfg->gradient_descent != 0, gdj = !gd && cfg->gradient_descent_joint != 0;
  const bool joint = cfg->joint_hmc != 0 && !gd && !gdj;
  if (!(cfg->gradient_descent_joint || cfg->joint_hmc)) {
    // sample_error_precision (branch_sampler.rs:190-202): output-layer hyperparameters
    B.prec[B.epoff] = (float)ridge_posterior(t, kout, sout, t->rss_cur, (double)n);
    if (!cfg->fixed_param_precisions) {  // sample_param_precisions (173-188)
      sample_prior_precisions(t, B);
      const double total = others + B.out_stat();  // add_output_weight_summary_stat_to_global
      B.prec[B.out_prec_ix()] = (float)(is_lasso(B.prior) ? lasso_posterior(t, kout, sout, total, (double)B.ows_num)
                                                          : ridge_posterior(t, kout, sout, total, (double)B.ows_num));
    }
  }
  CKB(bann_branch_set_precisions(t->ctx, b, B.prec.data()));
  CKB(bann_residual_to_target(t->ctx, b));  // net.rs:279-280: fitted to residual + its own prediction
  int32_t status = 0;
  bool tail = false;  // hmc_step_tail ran: the parameters and the residual statistics are in already
  double tail_stats[4] = {0.0, 0.0, 0.0, 0.0};
  if (gd) {
    int rc = gradient_descent(t, b, cfg, status);
    if (rc) return rc;
  } else if (gdj) {
    int rc = gradient_descent_joint(t, b, cfg, others, status);
    if (rc) return rc;
    CKB(bann_branch_get_precisions(t->ctx, b, B.prec.data()));  // to_cfg
  } else if (joint) {  // hmc_step_joint (branch_sampler.rs:1070-1178): random step sizes over [params | precisions]
    const int64_t PQ = B.P + B.NP;
    const float f = std::pow((float)PQ, -0.25f) * cfg->hmc_step_size_factor;  // random_step_sizes (654-662)
    dr.eps.resize(PQ);
    for (auto& e : dr.eps) e = (float)draw_uniform(t) * f;
    dr.mom.resize(PQ);
    for (auto& p : dr.mom) p = (float)draw_normal(t);
    dr.u = (float)draw_uniform(t);
    CKB(bann_branch_set_output_stats(t->ctx, b, (float)others, (float)t->g_num));
    const float hyper[6] = {t->hp.dense_shape, t->hp.dense_scale, t->hp.summary_shape,
                            t->hp.summary_scale, t->hp.output_shape, t->hp.output_scale};
    CKB(bann_hmc_step_joint(t->ctx, &b, 1, cfg->hmc_integration_length, cfg->hmc_max_hamiltonian_error,
                            BANN_STEP_INJECTED, cfg->hmc_step_size_factor, dr.eps.data(), dr.mom.data(), 0, &dr.u,
                            hyper, &status, nullptr, nullptr));
    CKB(bann_branch_get_precisions(t->ctx, b, B.prec.data()));  // to_cfg: the sampled precisions
  } else {
    const float* eps = nullptr;
    int32_t mode = cfg->hmc_step_size_mode;
    if (mode == BANN_STEP_RANDOM) {  // random_step_sizes (654-681): U(0,1) P^-1/4 c, param_vec order
      const float f = std::pow((float)B.P, -0.25f) * cfg->hmc_step_size_factor;
      dr.eps.resize(B.P);
      for (auto& e : dr.eps) e = (float)draw_uniform(t) * f;
      eps = dr.eps.data();
      mode = BANN_STEP_INJECTED;
    }
    // sample_momentum (branch_sampler.rs:594-609) draws on the device in the reference
    // (ArrayFire randn): so does the driver unless the caller replays a host stream
    // (RNG hooks, the parity tests) -- then P normals from the hook, uploaded
    const bool dev_mom = !t->hooks.normal;
    uint64_t mseed = 0;
    if (dev_mom) {
      mseed = t->gen();
    } else {
      dr.mom.resize(B.P);
      for (auto& p : dr.mom) p = (float)draw_normal(t);
    }
    dr.u = (float)draw_uniform(t);
    if (!traj) {  // the trajectory, get_params and the residual op below in one host wait
      CKB(hmc_step_tail(t->ctx, b, cfg->hmc_integration_length, cfg->hmc_max_hamiltonian_error, mode,
                        cfg->hmc_step_size_factor, eps, dev_mom ? nullptr : dr.mom.data(), mseed, &dr.u,
                        t->ob_bias, &status, B.params.data(), tail_stats));
      tail = true;
    } else {
      CKB(bann_hmc_step(t->ctx, &b, 1, cfg->hmc_integration_length, cfg->hmc_max_hamiltonian_error, mode,
                        cfg->hmc_step_size_factor, eps, dev_mom ? nullptr : dr.mom.data(), mseed, &dr.u, &status,
                        nullptr, nullptr, nullptr));
    }
  }
  if (traj && !gd && !gdj) {  // trajectories file opened in append mode (branch_sampler.rs:1199-1207)
    std::string line;
    int rc = traj_line(t, b, joint, line);
    if (!rc) rc = append_text(t, dir + "/traj", line);
    if (rc) return rc;
  }
  ++t->ns;  // TrainingStats::add_hmc_step_result (train_stats.rs:46-53)
  if (status == BANN_ACCEPTED) ++t->nacc;
  if (status == BANN_REJECTED_EARLY) ++t->nearly;
  // net.rs:292-300: residual = target - f_b(final) (accepted: y_pred; rejected: prev_pred),
  // and the output-bias shift of net.rs:321 (residual += bias) in the same launch: nothing
  // between the two touches the residual (sr_bias: its sum after the shift)
  double sr = 0.0, sr_bias = 0.0;
  if (tail) {
    sr = tail_stats[0];
    t->rss_cur = tail_stats[1];
    sr_bias = tail_stats[2];
  } else {
    CKB(bann_branch_get_params(t->ctx, b, B.params.data()));
    CKB(residual_from_target_shift(t->ctx, b, t->ob_bias, &sr, &t->rss_cur, &sr_bias, nullptr));
  }
  if (status == BANN_ACCEPTED) update_lpd(t, b, others);
  // to_cfg + GlobalParams::update_from_branch_cfg (net.rs:303-305, params.rs:41-56)
  B.ows_reg_sum = (float)(others + B.out_stat());
  if (!(B.prec[B.epoff] >= 0.f) || !(B.prec[B.out_prec_ix()] >= 0.f) || !(B.ows_reg_sum >= 0.f))
    return fail(t, BANN_E_STATE, "invalid global parameter after branch update (params.rs:42-54)");
  t->g_eprec = B.prec[B.epoff];
  t->g_oprec = B.prec[B.out_prec_ix()];
  t->g_reg_sum = B.ows_reg_sum;
  // net.rs:307-315 / 458-465: the branch's effect sizes after burn-in
  if (cfg->effect_sizes && chain_ix >= cfg->burn_in && !dir.empty()) {
    const int rc = save_effect_sizes(t, b, chain_ix, dir);
    if (rc) return rc;
  }
  // output bias (net.rs:319-332): residual += bias, draw, residual -= bias
  t->ob_eprec = t->g_eprec;
  sr = sr_bias;  // residual += bias happened with the residual update above
  if (cfg->sampled_output_bias) {
    // sample_prior_precision passes the prior SHAPE as the scale (net.rs:61-66)
    const double bsq = (double)t->ob_bias * t->ob_bias;
    t->ob_prec = (float)draw_gamma(t, kout + 0.5, 2.0 * kout / (2.0 + kout * bsq));
    const double den = (double)n * t->ob_eprec + t->ob_prec;  // sample_bias (47-53)
    t->ob_bias = (float)(t->ob_eprec / den * sr + std::sqrt(1.0 / den) * draw_normal(t));
  } else {
    t->ob_bias = (float)(sr / (double)n);  // set_to_maximum_likelihood (43-45)
  }
  CKB(bann_residual_shift(t->ctx, -t->ob_bias, nullptr, &t->rss_cur));
  return BANN_OK;
}

// checks + initialize_stats (net.rs:158-171) + the first record / trace / model (net.rs:232-249)
int train_begin(bann_net* t, const float* y, int64_t n, const bann_mcmc_cfg* cfg, const std::string& dir,
                bool& trace, bool& traj) {
  if (cfg->hmc_integration_length < 1 || cfg->chain_length < 0 || cfg->burn_in < 0)
    return fail(t, BANN_E_ARG, "bad MCMC configuration");
  const int32_t m = cfg->hmc_step_size_mode;
  if (!cfg->joint_hmc && m != BANN_STEP_IZMAILOV && m != BANN_STEP_UNIFORM && m != BANN_STEP_RANDOM &&
      m != BANN_STEP_STD_SCALED)
    return fail(t, BANN_E_ARG, "step size mode: Izmailov, uniform, random or StdScaled");
  // StdScaled returns empty step sizes for the ARD priors (ridge_ard.rs:56-68, lasso_ard.rs:62-74):
  // the reference's hmc_step would index-panic on the first half step; joint HMC uses random
  // sizes instead (branch_sampler.rs:1092-1101)
  if (!cfg->joint_hmc && !cfg->gradient_descent && !cfg->gradient_descent_joint && m == BANN_STEP_STD_SCALED)
    for (const auto& B : t->br)
      if (is_ard(B.prior))
        return fail(t, BANN_E_ARG,
                    "StdScaled step sizes are empty for the ARD priors in the reference (ridge_ard.rs:56-68, "
                    "lasso_ard.rs:62-74): use Izmailov, uniform or random");
  if (n != bann_ctx_num_individuals(t->ctx)) return fail(t, BANN_E_SHAPE, "phenotype length differs from the cohort");
  t->n = n;
  // net.rs:208-211: the models and effect-size directories
  if (!dir.empty() && (!mkdir_p(dir + "/models") || !mkdir_p(dir + "/effect_sizes")))
    return fail(t, BANN_E_ARG, "cannot create the output directories under " + dir);
  // initialize_stats: residual = y - bias - sum_b f_b on the device (one packed forward for stale rows)
  for (auto& B : t->br) cfg_update_global(t, B);
  CKB(bann_residual_init(t->ctx, y, t->ob_bias, nullptr, &t->rss_cur));
  for (int b = 0; b < (int)t->br.size(); ++b) {
    const Branch& B = t->br[b];
    update_lpd(t, b, B.ows_reg_sum - B.out_stat());
  }
  int rc = record_perf(t);
  if (rc) return rc;
  trace = cfg->trace && !dir.empty();
  traj = cfg->trajectories && !dir.empty();
  if (trace) {  // File::create (net.rs:213-215): a fresh trace, the initial cfgs first (241-244)
    std::remove((dir + "/trace").c_str());
    rc = append_text(t, dir + "/trace", trace_line(t));
    if (rc) return rc;
  }
  CKB(bann_set_trajectory_recording(t->ctx, traj ? 1 : 0));
  if (!dir.empty() && cfg->burn_in == 0) return write_file(t, dir + "/models/0.bin");
  return BANN_OK;
}

// record_perf, trace line, model file after a sweep (net.rs:336-353)
int train_record(bann_net* t, int chain_ix, const bann_mcmc_cfg* cfg, const std::string& dir, bool trace) {
  int rc = record_perf(t);
  if (rc) return rc;
  if (trace && (rc = append_text(t, dir + "/trace", trace_line(t)))) return rc;
  if (!dir.empty() && chain_ix >= cfg->burn_in) return write_file(t, dir + "/models/" + std::to_string(chain_ix) + ".bin");
  return BANN_OK;
}

}  // namespace

namespace {
// the driver's one-branch trajectories are launch-latency-bound: replay each as one
// captured HIP graph (bann_set_graph_replay) unless BANN_HMC_GRAPH=0; the
// context's previous setting is restored after training
struct GraphReplayScope {
  bann_ctx* ctx;
  int32_t prev;
  explicit GraphReplayScope(bann_ctx* c) : ctx(c), prev(bann_get_graph_replay(c)) {
    const char* e = std::getenv("BANN_HMC_GRAPH");
    (void)bann_set_graph_replay(ctx, !e || std::atoi(e) != 0);
  }
  ~GraphReplayScope() { (void)bann_set_graph_replay(ctx, prev); }
};
}  // namespace

extern "C" int bann_net_train(bann_net* t, const float* y, int64_t n, const bann_mcmc_cfg* cfg, const char* outdir) {
  if (!t || !y || !cfg) return BANN_E_ARG;
  const std::string dir = outdir ? outdir : "";
  bool trace = false, traj = false;
  GraphReplayScope graphs(t->ctx);
  int rc = train_begin(t, y, n, cfg, dir, trace, traj);
  if (rc) return rc;
  const int nb = (int)t->br.size();
  std::vector<int> order(nb);
  for (int b = 0; b < nb; ++b) order[b] = b;
  Draws dr;
  for (int chain_ix = 1; chain_ix <= cfg->chain_length; ++chain_ix) {
    for (int i = nb - 1; i >= 1; --i) {  // branch_ixs.shuffle (net.rs:257)
      const int j = std::min(i, (int)std::floor(draw_uniform(t) * (i + 1)));
      std::swap(order[i], order[j]);
    }
    for (int b : order)
      if ((rc = update_branch(t, b, cfg, traj, dir, dr, chain_ix))) return rc;
    if ((rc = train_record(t, chain_ix, cfg, dir, trace))) return rc;
  }
  CKB(bann_set_trajectory_recording(t->ctx, 0));
  if (!dir.empty()) return write_training_stats(t, dir);
  return BANN_OK;
}

extern "C" int bann_net_train_single_branch(bann_net* t, const float* y, int64_t n, const bann_mcmc_cfg* cfg,
                                            const char* outdir) {
  if (!t || !y || !cfg) return BANN_E_ARG;
  const std::string dir = outdir ? outdir : "";
  bool trace = false, traj = false;
  GraphReplayScope graphs(t->ctx);
  int rc = train_begin(t, y, n, cfg, dir, trace, traj);
  if (rc) return rc;
  Draws dr;
  for (int chain_ix = 1; chain_ix <= cfg->chain_length; ++chain_ix) {  // net.rs:412-502: branch 0 every time
    if ((rc = update_branch(t, 0, cfg, traj, dir, dr, chain_ix))) return rc;
    if ((rc = train_record(t, chain_ix, cfg, dir, trace))) return rc;
  }
  CKB(bann_set_trajectory_recording(t->ctx, 0));
  if (!dir.empty()) return write_training_stats(t, dir);
  return BANN_OK;
}

extern "C" int bann_net_perturb(bann_net* t, int32_t has_params, float params_by, int32_t has_precisions,
                                float precisions_by) {
  if (!t) return BANN_E_ARG;
  if (!has_params && !has_precisions) return BANN_OK;
  for (int b = 0; b < (int)t->br.size(); ++b) {  // BranchCfg::perturb_params / perturb_precisions
    Branch& B = t->br[b];
    if (has_params) {
      for (auto& v : B.params) v += params_by;
      CKB(bann_branch_set_params(t->ctx, b, B.params.data()));
    }
    if (has_precisions) {
      for (auto& v : B.prec) v += precisions_by;
      CKB(bann_branch_set_precisions(t->ctx, b, B.prec.data()));
    }
  }
  return BANN_OK;
}

extern "C" int bann_net_predict(bann_net* t, bann_ctx* ctx, float* y_hat) {
  if (!t || !y_hat) return BANN_E_ARG;
  bann_ctx* c = ctx ? ctx : t->ctx;
  const int nb = (int)t->br.size();
  if (bann_num_branches(c) != nb) return fail(t, BANN_E_SHAPE, "context branch count differs from the net");
  for (int b = 0; b < nb; ++b) {
    int32_t m = 0, L = 0, w[BANN_NET_MAXL] = {0};
    if (bann_branch_info(c, b, &m, &L, w, BANN_NET_MAXL, nullptr, nullptr) != BANN_OK || m != t->br[b].m ||
        L != t->br[b].L || L > BANN_NET_MAXL || !std::equal(w, w + L, t->br[b].widths.begin()))
      return fail(t, BANN_E_SHAPE, "context branches differ from the net's");
  }
  const int64_t nt = bann_ctx_num_individuals(c);
  if (nt <= 0) return fail(t, BANN_E_STATE, "context has no cohort");
  std::vector<int32_t> all(nb);
  for (int b = 0; b < nb; ++b) {
    all[b] = b;
    if (c != t->ctx) {
      const int rc = bann_branch_set_params(c, b, t->br[b].params.data());
      if (rc < 0) return fail(t, rc, std::string("predict context: ") + bann_last_error(c));
    }
  }
  std::vector<float> preds((size_t)nb * nt);
  const int rc = bann_predict_many(c, all.data(), nb, preds.data());
  if (rc < 0) return fail(t, rc, std::string("predict: ") + bann_last_error(c));
  for (int64_t i = 0; i < nt; ++i) {  // y_hat = 0 + bias, then += f_b in branch order (f32, net.rs:546-557)
    float v = 0.f + t->ob_bias;
    for (int b = 0; b < nb; ++b) v += preds[(size_t)b * nt + i];
    y_hat[i] = v;
  }
  return BANN_OK;
}

namespace {
// B::from_cfg on another context (or the net's own): the context must hold the
// net's branches; its parameters (another context only) and precisions are
// loaded from the BranchCfgs
int load_cfgs(bann_net* t, bann_ctx* c, int64_t n) {
  const int nb = (int)t->br.size();
  if (bann_num_branches(c) != nb) return fail(t, BANN_E_SHAPE, "context branch count differs from the net");
  if (n != bann_ctx_num_individuals(c)) return fail(t, BANN_E_SHAPE, "y length differs from the context's cohort");
  for (int b = 0; b < nb; ++b) {
    int32_t m = 0, L = 0, w[BANN_NET_MAXL] = {0};
    if (bann_branch_info(c, b, &m, &L, w, BANN_NET_MAXL, nullptr, nullptr) != BANN_OK || m != t->br[b].m ||
        L != t->br[b].L || L > BANN_NET_MAXL || !std::equal(w, w + L, t->br[b].widths.begin()))
      return fail(t, BANN_E_SHAPE, "context branches differ from the net's");
    int rc = c != t->ctx ? bann_branch_set_params(c, b, t->br[b].params.data()) : BANN_OK;
    if (!rc) rc = bann_branch_set_precisions(c, b, t->br[b].prec.data());
    if (rc < 0) return fail(t, rc, std::string("loading the branch cfgs: ") + bann_last_error(c));
  }
  return BANN_OK;
}
}  // namespace

extern "C" int bann_net_rss(bann_net* t, bann_ctx* ctx, const float* y, int64_t n, double* rss_out) {
  if (!t || !y || !rss_out) return BANN_E_ARG;
  bann_ctx* c = ctx ? ctx : t->ctx;
  if (n != bann_ctx_num_individuals(c)) return fail(t, BANN_E_SHAPE, "y length differs from the context's cohort");
  std::vector<float> yh(n);
  const int rc = bann_net_predict(t, ctx, yh.data());
  if (rc) return rc;
  double s = 0.0;
  for (int64_t i = 0; i < n; ++i) {  // residual = y - y_hat (f32), sum_of_squares
    const float r = y[i] - yh[i];
    s += (double)r * r;
  }
  *rss_out = s;
  return BANN_OK;
}

extern "C" int bann_net_gradient(bann_net* t, bann_ctx* ctx, const float* y, int64_t n, float* grad_out) {
  if (!t || !y || !grad_out) return BANN_E_ARG;
  bann_ctx* c = ctx ? ctx : t->ctx;
  int rc = load_cfgs(t, c, n);
  if (rc) return rc;
  const int nb = (int)t->br.size();
  std::vector<int32_t> all(nb);
  for (int b = 0; b < nb; ++b) all[b] = b;
  rc = bann_set_target_all(c, y);
  if (!rc) rc = bann_log_density_gradient_many(c, all.data(), nb, grad_out, nullptr);
  return rc < 0 ? fail(t, rc, std::string("gradient: ") + bann_last_error(c)) : BANN_OK;
}

extern "C" int bann_net_branch_r2s(bann_net* t, bann_ctx* ctx, const float* y, int64_t n, float* r2_out) {
  if (!t || !y || !r2_out) return BANN_E_ARG;
  bann_ctx* c = ctx ? ctx : t->ctx;
  int rc = load_cfgs(t, c, n);
  if (rc) return rc;
  const int nb = (int)t->br.size();
  std::vector<int32_t> all(nb);
  int64_t ptot = 0;
  for (int b = 0; b < nb; ++b) {
    all[b] = b;
    ptot += t->br[b].P;
  }
  std::vector<float> g(ptot);
  std::vector<double> rss(nb);
  rc = bann_set_target_all(c, y);
  if (!rc) rc = bann_log_density_gradient_many(c, all.data(), nb, g.data(), rss.data());
  if (rc < 0) return fail(t, rc, std::string("branch_r2s: ") + bann_last_error(c));
  double yy = 0.0;
  for (int64_t i = 0; i < n; ++i) yy += (double)y[i] * y[i];
  for (int b = 0; b < nb; ++b) r2_out[b] = 1.f - (float)rss[b] / (float)yy;  // r2 (branch_sampler.rs:911-913)
  return BANN_OK;
}

extern "C" int bann_net_activations(bann_net* t, bann_ctx* ctx, int32_t b, float* act_out) {
  if (!t || !act_out || b < 0 || b >= (int)t->br.size()) return BANN_E_ARG;
  bann_ctx* c = ctx ? ctx : t->ctx;
  int rc = load_cfgs(t, c, bann_ctx_num_individuals(c));
  if (rc) return rc;
  rc = bann_forward_feed(c, b, nullptr, act_out);
  return rc < 0 ? fail(t, rc, std::string("activations: ") + bann_last_error(c)) : BANN_OK;
}

extern "C" int bann_net_population_effect_sizes(bann_net* t, bann_ctx* ctx, float* out) {
  if (!t || !out) return BANN_E_ARG;
  bann_ctx* c = ctx ? ctx : t->ctx;
  int rc = load_cfgs(t, c, bann_ctx_num_individuals(c));
  if (rc) return rc;
  const int nb = (int)t->br.size();
  std::vector<int32_t> all(nb);
  for (int b = 0; b < nb; ++b) all[b] = b;
  rc = bann_population_effect_sizes(c, all.data(), nb, out);
  return rc < 0 ? fail(t, rc, std::string("population_effect_sizes: ") + bann_last_error(c)) : BANN_OK;
}

extern "C" int bann_net_set_test_data(bann_net* t, bann_ctx* test_ctx, const float* y_test, int64_t n_test) {
  if (!t) return BANN_E_ARG;
  if (!test_ctx) {
    t->test_ctx = nullptr;
    t->y_test.clear();
    return BANN_OK;
  }
  if (!y_test || n_test <= 0) return fail(t, BANN_E_ARG, "null or empty test targets");
  if (n_test != bann_ctx_num_individuals(test_ctx))
    return fail(t, BANN_E_SHAPE, "n_test differs from the test context's cohort size");
  if (bann_num_branches(test_ctx) != (int)t->br.size()) return fail(t, BANN_E_SHAPE, "test context branch count");
  for (int b = 0; b < (int)t->br.size(); ++b) {
    int32_t m = 0, L = 0, w[BANN_NET_MAXL] = {0};
    if (bann_branch_info(test_ctx, b, &m, &L, w, BANN_NET_MAXL, nullptr, nullptr) != BANN_OK || m != t->br[b].m ||
        L != t->br[b].L || L > BANN_NET_MAXL || !std::equal(w, w + L, t->br[b].widths.begin()))
      return fail(t, BANN_E_SHAPE, "test context branches differ from the training branches");
  }
  t->test_ctx = test_ctx;
  t->y_test.assign(y_test, y_test + n_test);
  return BANN_OK;
}

extern "C" int bann_net_records_test(const bann_net* t, float* mse_test, int32_t cap) {
  if (!t) return BANN_E_ARG;
  const int32_t k = std::min<int32_t>(cap, (int32_t)t->mse_test.size());
  if (mse_test) std::copy(t->mse_test.begin(), t->mse_test.begin() + k, mse_test);
  return (int)t->mse_test.size();
}

extern "C" int bann_net_summary(const bann_net* t, bann_train_summary* out) {
  if (!t || !out) return BANN_E_ARG;
  out->num_samples = t->ns;
  out->num_accepted = t->nacc;
  out->num_early_rejected = t->nearly;
  out->num_records = (int32_t)t->mse.size();
  out->mse_train_last = t->mse.empty() ? NAN : t->mse.back();
  out->lpd_last = t->lpd.empty() ? NAN : t->lpd.back();
  out->output_bias = t->ob_bias;
  out->error_precision = t->g_eprec;
  out->output_layer_precision = t->g_oprec;
  out->output_reg_sum = t->g_reg_sum;
  return BANN_OK;
}

extern "C" int bann_net_records(const bann_net* t, float* mse_train, float* lpd, int32_t cap) {
  if (!t || cap < 0) return BANN_E_ARG;
  const int32_t k = std::min<int32_t>(cap, (int32_t)t->mse.size());
  for (int32_t i = 0; i < k; ++i) {
    if (mse_train) mse_train[i] = t->mse[i];
    if (lpd) lpd[i] = t->lpd[i];
  }
  return k;
}

extern "C" int bann_net_residual(const bann_net* t, float* out) {
  if (!t || !out) return BANN_E_ARG;
  if (t->n == 0) return BANN_E_STATE;
  const int rc = bann_residual_get(t->ctx, out);
  return rc < 0 ? rc : BANN_OK;
}

extern "C" int bann_net_save(const bann_net* t, const char* path) {
  if (!t || !path) return BANN_E_ARG;
  return write_file(const_cast<bann_net*>(t), path);
}

extern "C" int bann_net_load(bann_net* t, const char* path) {
  if (!t || !path) return BANN_E_ARG;
  FILE* f = std::fopen(path, "rb");
  if (!f) return fail(t, BANN_E_ARG, std::string("cannot open ") + path);
  std::vector<uint8_t> buf;
  uint8_t chunk[1 << 16];
  size_t k;
  while ((k = std::fread(chunk, 1, sizeof(chunk), f)) > 0) buf.insert(buf.end(), chunk, chunk + k);
  std::fclose(f);
  Reader r{buf.data(), buf.size()};
  bann_precision_hyperparams hp;
  hp.dense_shape = r.f32();
  hp.dense_scale = r.f32();
  hp.summary_shape = r.f32();
  hp.summary_scale = r.f32();
  hp.output_shape = r.f32();
  hp.output_scale = r.f32();
  const uint64_t nb = r.u64();
  if (!r.ok || nb != t->br.size() || r.u64() != nb) return fail(t, BANN_E_SHAPE, "branch count differs from the context");
  std::vector<Branch> br = t->br;
  for (Branch& B : br) {
    const uint64_t P = r.u64(), nw = r.u64(), m = r.u64();
    const auto lw = r.vu64();
    if (!r.ok || P != (uint64_t)B.P || nw != (uint64_t)B.num_weights || m != (uint64_t)B.m || lw.size() != (size_t)B.L)
      return fail(t, BANN_E_SHAPE, "branch shape differs from the context");
    for (int l = 0; l < B.L; ++l)
      if (lw[l] != (uint64_t)B.widths[l]) return fail(t, BANN_E_SHAPE, "layer widths differ from the context");
    if (r.u64() != (uint64_t)B.L) return fail(t, BANN_E_SHAPE, "weights: layer count");
    for (int l = 0; l < B.L; ++l) {
      const auto v = r.vf32();
      if (v.size() != (size_t)B.win[l] * B.widths[l]) return fail(t, BANN_E_SHAPE, "weights: layer size");
      std::copy(v.begin(), v.end(), B.params.begin() + B.woff[l]);
    }
    if (r.u64() != (uint64_t)(B.L - 1)) return fail(t, BANN_E_SHAPE, "biases: layer count");
    for (int l = 0; l < B.L - 1; ++l) {
      const auto v = r.vf32();
      if (v.size() != (size_t)B.widths[l]) return fail(t, BANN_E_SHAPE, "biases: layer size");
      std::copy(v.begin(), v.end(), B.params.begin() + B.boff[l]);
    }
    r.vu64();  // layer_widths (again) and num_markers inside BranchParamsHost
    r.u64();
    B.ows_reg_sum = r.f32();
    B.ows_num = r.u64();
    if (r.u64() != (uint64_t)B.L) return fail(t, BANN_E_SHAPE, "weight precisions: layer count");
    for (int l = 0; l < B.L; ++l) {
      const auto v = r.vf32();
      if (v.size() != (size_t)B.wpn[l]) return fail(t, BANN_E_SHAPE, "weight precisions: size (prior differs?)");
      std::copy(v.begin(), v.end(), B.prec.begin() + B.wpoff[l]);
    }
    if (r.u64() != (uint64_t)(B.L - 1)) return fail(t, BANN_E_SHAPE, "bias precisions: layer count");
    for (int l = 0; l < B.L - 1; ++l) {
      const auto v = r.vf32();
      if (v.size() != 1) return fail(t, BANN_E_SHAPE, "bias precisions: size");
      B.prec[B.bpoff + l] = v[0];
    }
    const auto ep = r.vf32();
    if (ep.size() != 1) return fail(t, BANN_E_SHAPE, "error precision: size");
    B.prec[B.epoff] = ep[0];
    if ((int)r.u32() != B.act) return fail(t, BANN_E_SHAPE, "activation differs from the context");
  }
  const float ob_e = r.f32(), ob_p = r.f32(), ob_b = r.f32();
  const uint64_t ns = r.u64(), na = r.u64(), ne = r.u64();
  const auto mse = r.vf32();
  if (r.u8() != 0) r.vf32();  // mse_test
  const auto lpd = r.vf32();
  const float l_rss = r.f32(), l_out = r.f32();
  const auto l_loc = r.vf32();
  const float ge = r.f32(), go = r.f32(), gr = r.f32();
  const uint64_t gn = r.u64();
  if (!r.ok || r.pos != r.n || l_loc.size() != nb) return fail(t, BANN_E_SHAPE, "truncated or malformed model file");
  for (size_t b = 0; b < br.size(); ++b) {
    CKB(bann_branch_set_params(t->ctx, (int32_t)b, br[b].params.data()));
    CKB(bann_branch_set_precisions(t->ctx, (int32_t)b, br[b].prec.data()));
  }
  t->br = std::move(br);
  t->hp = hp;
  t->ob_eprec = ob_e;
  t->ob_prec = ob_p;
  t->ob_bias = ob_b;
  t->ns = ns;
  t->nacc = na;
  t->nearly = ne;
  t->mse = mse;
  t->lpd = lpd;
  t->lpd_rss = l_rss;
  t->lpd_outw = l_out;
  t->lpd_local = l_loc;
  t->g_eprec = ge;
  t->g_oprec = go;
  t->g_reg_sum = gr;
  t->g_num = gn;
  return BANN_OK;
}
