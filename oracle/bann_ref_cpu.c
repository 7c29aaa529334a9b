/*
 * bann_ref_cpu.c — CPU restatement of the reference's per-branch HMC leapfrog
 * step, in the reference's op order, for the bench.py cpu_baseline leg.
 *
 * TEST / MEASUREMENT INFRASTRUCTURE ONLY: never linked into the product.
 *
 * The reference (Rust + ArrayFire, CPU backend) cannot be built here (no
 * cargo/rustc, no ArrayFire).  This file restates what its CPU backend executes
 * per leapfrog step and branch (branch_sampler.rs:1239-1285), f32 throughout:
 *   momentum.half_step (momentum.rs:121-136), params.full_step (params.rs:728-738),
 *   log_density_gradient -> backpropagate (branch_sampler.rs:813-875):
 *       forward_feed (743-782): Z0 = X W0 + b0, A = tanh, Z1 = A0 W1 + b1, out = A1 w
 *       e = out - y, rss, dW_out, error back-propagation, dW0 = X^T delta0
 *   RidgeARD prior gradient (ridge_ard.rs:196-219),
 *   momentum.half_step,
 *   neg_hamiltonian (878-883): a SECOND full forward over X (rss, 905-909),
 *       log density (ridge_ard.rs:171-194) and K(p) (momentum.rs:149-158).
 * The dense standardized f32 block X_b (bed.rs:325-355) is materialized once per
 * branch (the reference does it once per branch per Gibbs sweep, net.rs:265).
 * X is read three times per step, as in the reference.  OpenMP over rows/markers
 * stands in for ArrayFire-CPU's threaded BLAS.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static uint64_t sm64(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static float unif(uint64_t* s) { return (float)((sm64(s) >> 40) * (1.0 / 16777216.0)); }
static float gauss(uint64_t* s) {
  float u1 = unif(s) + 1e-7f, u2 = unif(s);
  return sqrtf(-2.f * logf(u1)) * cosf(6.2831853f * u2);
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

typedef struct {
  int64_t n;
  int m, W, S;
  float *X;                    /* n x m column-major standardized */
  float *W0, *b0, *W1, *b1, *wo;  /* params */
  float *y;
} Branch;

/* forward_feed: returns rss; fills Z0,A0 (n x W col-major), Z1,A1 (n x S), out */
static double forward(const Branch* B, float* Z0, float* A0, float* Z1, float* A1, float* out) {
  const int64_t n = B->n;
  const int m = B->m, W = B->W, S = B->S;
  /* Z0 = X W0 (sgemm n x m x W), column axpy form, parallel over row blocks */
#pragma omp parallel for schedule(static)
  for (int64_t i0 = 0; i0 < n; i0 += 1024) {
    const int64_t i1 = i0 + 1024 < n ? i0 + 1024 : n;
    for (int k = 0; k < W; ++k) {
      float* z = Z0 + (int64_t)k * n;
      for (int64_t i = i0; i < i1; ++i) z[i] = 0.f;
      for (int j = 0; j < m; ++j) {
        const float w = B->W0[k * m + j];
        const float* x = B->X + (int64_t)j * n;
        for (int64_t i = i0; i < i1; ++i) z[i] += x[i] * w;
      }
      for (int64_t i = i0; i < i1; ++i) {  /* + tile(b0), tanh */
        z[i] += B->b0[k];
        A0[(int64_t)k * n + i] = tanhf(z[i]);
      }
    }
  }
  double rss = 0.0;
#pragma omp parallel for reduction(+ : rss) schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    float o = 0.f;
    for (int k = 0; k < S; ++k) {
      float s = B->b1[k];
      for (int j = 0; j < W; ++j) s += A0[(int64_t)j * n + i] * B->W1[k * W + j];
      Z1[(int64_t)k * n + i] = s;
      const float a = tanhf(s);
      A1[(int64_t)k * n + i] = a;
      o += a * B->wo[k];
    }
    out[i] = o;
    const float e = o - B->y[i];
    rss += (double)(e * e);
  }
  return rss;
}

/* one leapfrog step of hmc_step; g holds the gradient at entry and exit */
static double leapfrog_step(Branch* B, float* p, float* g, const float* eps, const float* lam, float le, float* Z0,
                            float* A0, float* Z1, float* A1, float* out, float* D0, int P) {
  const int64_t n = B->n;
  const int m = B->m, W = B->W, S = B->S;
  float* th = B->W0; /* params are contiguous: W0, W1, wo, b0, b1 */
  for (int i = 0; i < P; ++i) p[i] += 0.5f * eps[i] * g[i];  /* half_step */
  for (int i = 0; i < P; ++i) th[i] += eps[i] * p[i];         /* full_step */
  /* backpropagate */
  forward(B, Z0, A0, Z1, A1, out);
  float* dW0 = g;
  float* dW1 = g + m * W;
  float* dwo = dW1 + W * S;
  float* db0 = dwo + S;
  float* db1 = db0 + W;
  for (int i = 0; i < P; ++i) g[i] = 0.f;
#pragma omp parallel
  {
    float* l_dW1 = (float*)malloc(sizeof(float) * ((size_t)W * S + 2 * S + 2 * W));
    float *l_dwo = l_dW1 + W * S, *l_db0 = l_dwo + S, *l_db1 = l_db0 + W, *err0 = l_db1 + S;
    memset(l_dW1, 0, sizeof(float) * W * S);
    memset(l_dwo, 0, sizeof(float) * S);
    memset(l_db0, 0, sizeof(float) * W);
    memset(l_db1, 0, sizeof(float) * S);
#pragma omp for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      const float e = out[i] - B->y[i];
      for (int j = 0; j < W; ++j) err0[j] = 0.f;
      for (int k = 0; k < S; ++k) {
        const float a1 = A1[(int64_t)k * n + i];
        l_dwo[k] += a1 * e;
        const float d1 = (1.f - a1 * a1) * (e * B->wo[k]);
        l_db1[k] += d1;
        for (int j = 0; j < W; ++j) {
          l_dW1[k * W + j] += A0[(int64_t)j * n + i] * d1;
          err0[j] += d1 * B->W1[k * W + j];
        }
      }
      for (int j = 0; j < W; ++j) {
        const float a0 = A0[(int64_t)j * n + i];
        const float d0 = (1.f - a0 * a0) * err0[j];
        D0[(int64_t)j * n + i] = d0;
        l_db0[j] += d0;
      }
    }
#pragma omp critical
    {
      for (int q = 0; q < W * S; ++q) dW1[q] += l_dW1[q];
      for (int q = 0; q < S; ++q) dwo[q] += l_dwo[q];
      for (int q = 0; q < W; ++q) db0[q] += l_db0[q];
      for (int q = 0; q < S; ++q) db1[q] += l_db1[q];
    }
    free(l_dW1);
  }
  /* dW0 = (delta0^T X)^T : second pass over X */
#pragma omp parallel for schedule(static)
  for (int j = 0; j < m; ++j) {
    const float* x = B->X + (int64_t)j * n;
    for (int k = 0; k < W; ++k) {
      const float* d = D0 + (int64_t)k * n;
      float s = 0.f;
      for (int64_t i = 0; i < n; ++i) s += x[i] * d[i];
      dW0[k * m + j] = s;
    }
  }
  /* ridge ARD prior gradient: -(le * d_rss + lam * theta) */
  for (int i = 0; i < P; ++i) g[i] = -(le * g[i] + lam[i] * th[i]);
  for (int i = 0; i < P; ++i) p[i] += 0.5f * eps[i] * g[i];  /* half_step */
  /* neg_hamiltonian: third pass over X */
  const double rss = forward(B, Z0, A0, Z1, A1, out);
  double ld = -(double)le * rss / 2.0, k = 0.0;
  for (int i = 0; i < m * W + W * S + S; ++i) ld -= 0.5 * lam[i] * th[i] * th[i];
  for (int i = 0; i < P; ++i) k += 0.5 * (double)p[i] * p[i];
  return ld - k;
}

/*
 * Times `nsteps` leapfrog steps for each of `nbranch` synthetic branches of the
 * given shape (D = 1 hidden layer of width W, summary width S, tanh, RidgeARD).
 * Returns the wall seconds spent in the leapfrog steps; *setup_s receives the
 * time spent materializing the standardized f32 blocks; *checksum a value that
 * depends on every result (keeps the work live).
 */
double bann_ref_cpu_bench(int64_t n, int m, int W, int S, int nbranch, int nsteps, uint64_t seed, int threads,
                          double* setup_s, double* checksum) {
  if (threads > 0) omp_set_num_threads(threads);
  const int P = m * W + W * S + S + W + S;
  Branch B;
  B.n = n;
  B.m = m;
  B.W = W;
  B.S = S;
  B.X = (float*)malloc(sizeof(float) * n * m);
  float* theta = (float*)malloc(sizeof(float) * P);
  B.W0 = theta;
  B.W1 = theta + m * W;
  B.wo = B.W1 + W * S;
  B.b0 = B.wo + S;
  B.b1 = B.b0 + W;
  B.y = (float*)malloc(sizeof(float) * n);
  float *Z0 = malloc(sizeof(float) * n * W), *A0 = malloc(sizeof(float) * n * W), *D0 = malloc(sizeof(float) * n * W);
  float *Z1 = malloc(sizeof(float) * n * S), *A1 = malloc(sizeof(float) * n * S), *out = malloc(sizeof(float) * n);
  float *p = malloc(sizeof(float) * P), *g = malloc(sizeof(float) * P), *eps = malloc(sizeof(float) * P),
        *lam = malloc(sizeof(float) * P);
  int8_t* geno = (int8_t*)malloc((size_t)n * m);
  double t_steps = 0.0, t_setup = 0.0, cs = 0.0;
  uint64_t s = seed;
  for (int b = 0; b < nbranch; ++b) {
    /* synthetic genotypes of the branch (Binomial(2, p), p ~ U(0.01, 0.5)) */
    for (int j = 0; j < m; ++j) {
      const float pj = 0.01f + 0.49f * unif(&s);
      uint64_t sj = sm64(&s);
      for (int64_t i = 0; i < n; ++i) geno[(int64_t)j * n + i] = (unif(&sj) < pj) + (unif(&sj) < pj);
    }
    for (int i = 0; i < P; ++i) {
      theta[i] = i < m * W + W * S + S ? gauss(&s) / sqrtf((float)m) : 0.f;
      p[i] = gauss(&s);
      lam[i] = i < m * W + W * S + S ? 1.f : 0.f;
      eps[i] = 1e-3f;
    }
    for (int64_t i = 0; i < n; ++i) B.y[i] = gauss(&s);
    /* x_branch_af: standardized f32 block (bed.rs:325-355) */
    double t0 = now_s();
#pragma omp parallel for schedule(static)
    for (int j = 0; j < m; ++j) {
      const int8_t* gc = geno + (int64_t)j * n;
      double s1 = 0.0, s2 = 0.0;
      for (int64_t i = 0; i < n; ++i) {
        s1 += gc[i];
        s2 += gc[i] * gc[i];
      }
      const float mu = (float)(s1 / n);
      float sd = (float)sqrt(fmax(s2 / n - (s1 / n) * (s1 / n), 1e-12));
      float* x = B.X + (int64_t)j * n;
      for (int64_t i = 0; i < n; ++i) x[i] = ((float)gc[i] - mu) / sd;
    }
    double t1 = now_s();
    t_setup += t1 - t0;
    /* initial gradient (hmc_step 1232-1236) is trajectory start: not timed */
    forward(&B, Z0, A0, Z1, A1, out);
    for (int i = 0; i < P; ++i) g[i] = 0.f;
    double t2 = now_s();
    for (int st = 0; st < nsteps; ++st)
      cs += leapfrog_step(&B, p, g, eps, lam, 2.f, Z0, A0, Z1, A1, out, D0, P);
    t_steps += now_s() - t2;
  }
  for (int i = 0; i < P; ++i) cs += theta[i];
  free(B.X); free(theta); free(B.y); free(Z0); free(A0); free(D0); free(Z1); free(A1); free(out);
  free(p); free(g); free(eps); free(lam); free(geno);
  if (setup_s) *setup_s = t_setup;
  if (checksum) *checksum = cs;
  return t_steps;
}
