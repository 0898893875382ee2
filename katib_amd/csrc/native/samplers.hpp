// Native search samplers - the C++ counterparts of the goptuna (Go) suggestion
// service (reference pkg/suggestion/v1beta1/goptuna/*, library
// github.com/c-bata/goptuna v0.8.0) plus the TPE/multivariate-TPE core used by
// the hyperopt- and optuna-compatible services.
//
//   SobolEngine : Joe-Kuo direction numbers (table supplied by the caller),
//                 Gray-code generation, 30-bit output identical to an
//                 unscrambled scipy.stats.qmc.Sobol sequence.
//   CmaEs       : (mu/mu_w, lambda)-CMA-ES with active (negative-weight)
//                 covariance update, bound repair by resampling then clipping,
//                 IPOP/BIPOP restart support (tutorial: Hansen 2016).
//   tpe_sample  : Parzen-estimator TPE (univariate, hyperopt-style adaptive
//                 bandwidths) and multivariate TPE (joint kernels, optuna-style
//                 Scott bandwidth), EI maximisation over n_ei_candidates draws.
// All are deterministic for a given seed.
#pragma once
#include <cstdint>
#include <random>
#include <string>
#include <vector>

namespace katib {

class SobolEngine {
 public:
  // poly: Joe-Kuo polynomial integers (incl. leading/trailing 1 bits), vinit: rows of m_i
  SobolEngine(int dim, const std::vector<int64_t>& poly, const std::vector<std::vector<int64_t>>& vinit);
  // point with index `idx` (0-based; idx 0 is the origin)
  std::vector<double> point(uint64_t idx) const;
  std::vector<std::vector<double>> points(uint64_t start, uint64_t n) const;
  int dim() const { return dim_; }

 private:
  static const int kBits = 30;
  int dim_;
  std::vector<std::vector<uint32_t>> v_;  // [dim][bit]
};

struct CmaState {
  std::vector<double> mean;
  double sigma;
  int generation;
  int popsize;
};

class CmaEs {
 public:
  CmaEs(const std::vector<double>& mean, double sigma, const std::vector<double>& lower,
        const std::vector<double>& upper, uint64_t seed, int popsize = 0);
  std::vector<double> ask();
  // exactly `popsize` (x, f) pairs of the current generation; minimisation
  void tell(const std::vector<std::vector<double>>& xs, const std::vector<double>& fs);
  bool should_stop() const;
  int popsize() const { return lambda_; }
  int generation() const { return gen_; }
  int dim() const { return n_; }
  double sigma() const { return sigma_; }
  std::vector<double> mean() const { return m_; }
  std::vector<std::vector<double>> cov() const { return C_; }

 private:
  void init_params();
  void eigen();
  std::vector<double> sample_unbounded();
  bool in_bounds(const std::vector<double>& x) const;

  int n_, lambda_, mu_, gen_ = 0;
  std::vector<double> w_;
  double mueff_, cc_, cs_, c1_, cmu_, damps_, chin_;
  std::vector<double> m_, pc_, ps_, lo_, hi_;
  double sigma_;
  std::vector<std::vector<double>> C_, B_;
  std::vector<double> D_;
  bool eigen_dirty_ = true;
  std::mt19937_64 rng_;
  std::normal_distribution<double> normal_{0.0, 1.0};
  std::vector<double> fhist_;
  double tolx_, tolfun_ = 1e-12, tolconditioncov_ = 1e14;
};

struct TpeDim {
  int kind = 0;  // 0 = numeric (already in internal, possibly log, space), 1 = categorical
  double low = 0, high = 1;
  double q = 0;  // quantisation step in internal space (0 = continuous)
  int n_choices = 0;
};

struct TpeSettings {
  double gamma = 0.25;
  int gamma_mode = 0;         // 0: hyperopt ceil(gamma*sqrt(n)); 1: optuna min(ceil(gamma*n), 25)
  double prior_weight = 1.0;
  int n_ei_candidates = 24;
  bool multivariate = false;
  bool consider_magic_clip = true;
  int linear_forgetting = 25;
};

// xs: n observations (internal coords, categorical as index), losses: lower is better.
// Returns the chosen point (internal coords).
std::vector<double> tpe_sample(const std::vector<TpeDim>& dims, const std::vector<std::vector<double>>& xs,
                               const std::vector<double>& losses, const TpeSettings& s, uint64_t seed);

void jacobi_eigen(std::vector<std::vector<double>> A, std::vector<double>& evals,
                  std::vector<std::vector<double>>& evecs);

}  // namespace katib
