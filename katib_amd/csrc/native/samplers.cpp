#include "samplers.hpp"

#include <algorithm>
#include <cmath>
#include <limits>
#include <numeric>
#include <stdexcept>

namespace katib {

// ============================================================================== Sobol
SobolEngine::SobolEngine(int dim, const std::vector<int64_t>& poly, const std::vector<std::vector<int64_t>>& vinit)
    : dim_(dim), v_(dim, std::vector<uint32_t>(kBits, 0)) {
  if (dim < 1) throw std::invalid_argument("sobol dim must be >= 1");
  if (static_cast<size_t>(dim) > poly.size() || static_cast<size_t>(dim) > vinit.size())
    throw std::invalid_argument("not enough direction numbers for requested dimension");
  // unshifted direction integers m_k, then shift into the top bits
  for (int d = 0; d < dim; ++d) {
    std::vector<uint64_t> m(kBits, 1);
    if (d > 0) {
      int64_t p = poly[d];
      int s = 0;
      while ((p >> (s + 1)) != 0) ++s;  // degree = bit_length - 1
      for (int k = 0; k < s && k < kBits; ++k) m[k] = static_cast<uint64_t>(vinit[d][k]);
      for (int j = s; j < kBits; ++j) {
        uint64_t nv = m[j - s];
        // m_j = m_{j-s} xor (2^s m_{j-s}) xor sum_{k=1}^{s-1} a_k 2^k m_{j-k}
        nv ^= m[j - s] << s;
        for (int k = 1; k < s; ++k) {
          int a = static_cast<int>((p >> (s - k)) & 1);
          if (a) nv ^= m[j - k] << k;
        }
        m[j] = nv;
      }
    }
    for (int j = 0; j < kBits; ++j) v_[d][j] = static_cast<uint32_t>(m[j] << (kBits - j - 1));
  }
}

std::vector<double> SobolEngine::point(uint64_t idx) const {
  // x_idx = XOR of v_j over set bits of gray(idx)
  uint64_t g = idx ^ (idx >> 1);
  std::vector<double> out(dim_);
  const double scale = 1.0 / static_cast<double>(1u << kBits);
  for (int d = 0; d < dim_; ++d) {
    uint32_t x = 0;
    uint64_t gg = g;
    for (int j = 0; gg && j < kBits; ++j, gg >>= 1)
      if (gg & 1) x ^= v_[d][j];
    out[d] = x * scale;
  }
  return out;
}

std::vector<std::vector<double>> SobolEngine::points(uint64_t start, uint64_t n) const {
  std::vector<std::vector<double>> out;
  out.reserve(n);
  for (uint64_t i = 0; i < n; ++i) out.push_back(point(start + i));
  return out;
}

// ============================================================================== eigen
void jacobi_eigen(std::vector<std::vector<double>> A, std::vector<double>& evals,
                  std::vector<std::vector<double>>& V) {
  const int n = static_cast<int>(A.size());
  V.assign(n, std::vector<double>(n, 0.0));
  for (int i = 0; i < n; ++i) V[i][i] = 1.0;
  for (int sweep = 0; sweep < 100; ++sweep) {
    double off = 0;
    for (int i = 0; i < n; ++i)
      for (int j = i + 1; j < n; ++j) off += A[i][j] * A[i][j];
    if (off < 1e-30) break;
    for (int p = 0; p < n; ++p) {
      for (int q = p + 1; q < n; ++q) {
        if (std::fabs(A[p][q]) < 1e-300) continue;
        double theta = (A[q][q] - A[p][p]) / (2 * A[p][q]);
        double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1));
        double c = 1 / std::sqrt(t * t + 1), s = t * c;
        for (int k = 0; k < n; ++k) {
          double akp = A[k][p], akq = A[k][q];
          A[k][p] = c * akp - s * akq;
          A[k][q] = s * akp + c * akq;
        }
        for (int k = 0; k < n; ++k) {
          double apk = A[p][k], aqk = A[q][k];
          A[p][k] = c * apk - s * aqk;
          A[q][k] = s * apk + c * aqk;
        }
        for (int k = 0; k < n; ++k) {
          double vkp = V[k][p], vkq = V[k][q];
          V[k][p] = c * vkp - s * vkq;
          V[k][q] = s * vkp + c * vkq;
        }
      }
    }
  }
  evals.resize(n);
  for (int i = 0; i < n; ++i) evals[i] = A[i][i];
}

// ============================================================================== CMA-ES
CmaEs::CmaEs(const std::vector<double>& mean, double sigma, const std::vector<double>& lower,
             const std::vector<double>& upper, uint64_t seed, int popsize)
    : n_(static_cast<int>(mean.size())), m_(mean), lo_(lower), hi_(upper), sigma_(sigma), rng_(seed) {
  if (n_ < 1) throw std::invalid_argument("CMA-ES needs >= 1 dimension");
  if (sigma <= 0) throw std::invalid_argument("sigma must be > 0");
  lambda_ = popsize > 0 ? popsize : 4 + static_cast<int>(std::floor(3 * std::log(static_cast<double>(n_))));
  if (lambda_ < 2) lambda_ = 2;
  tolx_ = 1e-12 * sigma;
  init_params();
}

void CmaEs::init_params() {
  const double n = n_;
  mu_ = lambda_ / 2;
  std::vector<double> wp(lambda_);
  for (int i = 0; i < lambda_; ++i) wp[i] = std::log((lambda_ + 1) / 2.0) - std::log(i + 1.0);
  double sp = 0, sp2 = 0, sn = 0, sn2 = 0;
  for (int i = 0; i < mu_; ++i) {
    sp += wp[i];
    sp2 += wp[i] * wp[i];
  }
  for (int i = mu_; i < lambda_; ++i) {
    sn += wp[i];
    sn2 += wp[i] * wp[i];
  }
  mueff_ = sp * sp / sp2;
  double mueff_minus = sn2 > 0 ? sn * sn / sn2 : 0;
  const double alpha_cov = 2;
  c1_ = alpha_cov / ((n + 1.3) * (n + 1.3) + mueff_);
  cmu_ = std::min(1 - c1_, alpha_cov * (mueff_ - 2 + 1 / mueff_) / ((n + 2) * (n + 2) + alpha_cov * mueff_ / 2));
  double alpha_mu_minus = 1 + c1_ / cmu_;
  double alpha_mueff_minus = 1 + 2 * mueff_minus / (mueff_ + 2);
  double alpha_posdef_minus = (1 - c1_ - cmu_) / (n * cmu_);
  double min_alpha = std::min(alpha_mu_minus, std::min(alpha_mueff_minus, alpha_posdef_minus));
  double sum_pos = 0, sum_neg = 0;
  for (double w : wp) (w >= 0 ? sum_pos : sum_neg) += std::fabs(w);
  w_.resize(lambda_);
  for (int i = 0; i < lambda_; ++i)
    w_[i] = wp[i] >= 0 ? wp[i] / sum_pos : min_alpha * wp[i] / (sum_neg > 0 ? sum_neg : 1);
  cs_ = (mueff_ + 2) / (n + mueff_ + 5);
  damps_ = 1 + 2 * std::max(0.0, std::sqrt((mueff_ - 1) / (n + 1)) - 1) + cs_;
  cc_ = (4 + mueff_ / n) / (n + 4 + 2 * mueff_ / n);
  chin_ = std::sqrt(n) * (1 - 1 / (4 * n) + 1 / (21 * n * n));
  pc_.assign(n_, 0);
  ps_.assign(n_, 0);
  C_.assign(n_, std::vector<double>(n_, 0));
  for (int i = 0; i < n_; ++i) C_[i][i] = 1;
  eigen_dirty_ = true;
}

void CmaEs::eigen() {
  if (!eigen_dirty_) return;
  // symmetrise, decompose, floor tiny eigenvalues (numerical repair as in the cmaes library)
  for (int i = 0; i < n_; ++i)
    for (int j = i + 1; j < n_; ++j) C_[i][j] = C_[j][i] = 0.5 * (C_[i][j] + C_[j][i]);
  std::vector<double> ev;
  jacobi_eigen(C_, ev, B_);
  D_.resize(n_);
  bool fix = false;
  for (int i = 0; i < n_; ++i) {
    if (ev[i] < 0) {
      ev[i] = 1e-14;
      fix = true;
    }
    D_[i] = std::sqrt(ev[i]);
  }
  if (fix) {
    for (int i = 0; i < n_; ++i)
      for (int j = 0; j < n_; ++j) {
        double s = 0;
        for (int k = 0; k < n_; ++k) s += B_[i][k] * ev[k] * B_[j][k];
        C_[i][j] = s;
      }
  }
  eigen_dirty_ = false;
}

std::vector<double> CmaEs::sample_unbounded() {
  eigen();
  std::vector<double> z(n_), y(n_, 0), x(n_);
  for (int i = 0; i < n_; ++i) z[i] = normal_(rng_) * D_[i];
  for (int i = 0; i < n_; ++i) {
    double s = 0;
    for (int k = 0; k < n_; ++k) s += B_[i][k] * z[k];
    y[i] = s;
  }
  for (int i = 0; i < n_; ++i) x[i] = m_[i] + sigma_ * y[i];
  return x;
}

bool CmaEs::in_bounds(const std::vector<double>& x) const {
  for (int i = 0; i < n_; ++i) {
    if (!lo_.empty() && x[i] < lo_[i]) return false;
    if (!hi_.empty() && x[i] > hi_[i]) return false;
  }
  return true;
}

std::vector<double> CmaEs::ask() {
  for (int t = 0; t < 100; ++t) {
    std::vector<double> x = sample_unbounded();
    if (in_bounds(x)) return x;
  }
  std::vector<double> x = sample_unbounded();
  for (int i = 0; i < n_; ++i) {
    if (!lo_.empty()) x[i] = std::max(x[i], lo_[i]);
    if (!hi_.empty()) x[i] = std::min(x[i], hi_[i]);
  }
  return x;
}

void CmaEs::tell(const std::vector<std::vector<double>>& xs, const std::vector<double>& fs) {
  if (static_cast<int>(xs.size()) != lambda_ || fs.size() != xs.size())
    throw std::invalid_argument("tell() needs exactly popsize solutions");
  eigen();
  gen_++;
  std::vector<int> idx(lambda_);
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return fs[a] < fs[b]; });
  for (int i = 0; i < lambda_; ++i) fhist_.push_back(fs[idx[i]]);
  size_t keep = static_cast<size_t>(10 + std::ceil(30.0 * n_ / lambda_)) * lambda_;
  if (fhist_.size() > keep) fhist_.erase(fhist_.begin(), fhist_.end() - keep);

  std::vector<std::vector<double>> y(lambda_, std::vector<double>(n_));
  for (int i = 0; i < lambda_; ++i)
    for (int d = 0; d < n_; ++d) y[i][d] = (xs[idx[i]][d] - m_[d]) / sigma_;
  std::vector<double> yw(n_, 0);
  for (int i = 0; i < mu_; ++i)
    for (int d = 0; d < n_; ++d) yw[d] += w_[i] * y[i][d];
  for (int d = 0; d < n_; ++d) m_[d] += sigma_ * yw[d];  // c_m = 1

  // C^{-1/2} = B D^-1 B^T
  auto cinvsqrt = [&](const std::vector<double>& v) {
    std::vector<double> t(n_, 0), o(n_, 0);
    for (int k = 0; k < n_; ++k) {
      double s = 0;
      for (int i = 0; i < n_; ++i) s += B_[i][k] * v[i];
      t[k] = s / D_[k];
    }
    for (int i = 0; i < n_; ++i) {
      double s = 0;
      for (int k = 0; k < n_; ++k) s += B_[i][k] * t[k];
      o[i] = s;
    }
    return o;
  };
  std::vector<double> cy = cinvsqrt(yw);
  double a = std::sqrt(cs_ * (2 - cs_) * mueff_);
  double psn = 0;
  for (int d = 0; d < n_; ++d) {
    ps_[d] = (1 - cs_) * ps_[d] + a * cy[d];
    psn += ps_[d] * ps_[d];
  }
  psn = std::sqrt(psn);
  sigma_ *= std::exp((cs_ / damps_) * (psn / chin_ - 1));
  sigma_ = std::min(sigma_, 1e32);
  double hs_thr = (1.4 + 2.0 / (n_ + 1)) * chin_;
  double hsig = psn / std::sqrt(1 - std::pow(1 - cs_, 2.0 * (gen_ + 1))) < hs_thr ? 1.0 : 0.0;
  double b = std::sqrt(cc_ * (2 - cc_) * mueff_);
  for (int d = 0; d < n_; ++d) pc_[d] = (1 - cc_) * pc_[d] + hsig * b * yw[d];
  std::vector<double> wo(lambda_);
  for (int i = 0; i < lambda_; ++i) {
    if (w_[i] >= 0) {
      wo[i] = w_[i];
    } else {
      std::vector<double> c = cinvsqrt(y[i]);
      double nn = 0;
      for (double v : c) nn += v * v;
      wo[i] = w_[i] * n_ / (nn + 1e-300);
    }
  }
  double delta_h = (1 - hsig) * cc_ * (2 - cc_);
  double sumw = std::accumulate(w_.begin(), w_.end(), 0.0);
  double base = 1 + c1_ * delta_h - c1_ - cmu_ * sumw;
  for (int i = 0; i < n_; ++i) {
    for (int j = 0; j <= i; ++j) {
      double rmu = 0;
      for (int k = 0; k < lambda_; ++k) rmu += wo[k] * y[k][i] * y[k][j];
      double v = base * C_[i][j] + c1_ * pc_[i] * pc_[j] + cmu_ * rmu;
      C_[i][j] = C_[j][i] = v;
    }
  }
  eigen_dirty_ = true;
}

bool CmaEs::should_stop() const {
  // tolfun: fitness range of recent generations
  if (!fhist_.empty() && static_cast<int>(fhist_.size()) >= lambda_ * 10) {
    auto mm = std::minmax_element(fhist_.begin(), fhist_.end());
    if (*mm.second - *mm.first < tolfun_) return true;
  }
  // tolx: all axes tiny
  bool small = true;
  for (int i = 0; i < n_; ++i) {
    if (sigma_ * std::sqrt(std::fabs(C_[i][i])) >= tolx_ || sigma_ * std::fabs(pc_[i]) >= tolx_) {
      small = false;
      break;
    }
  }
  if (small) return true;
  // condition number of C
  double dmin = std::numeric_limits<double>::max(), dmax = 0;
  for (int i = 0; i < n_; ++i) {
    dmin = std::min(dmin, std::fabs(C_[i][i]));
    dmax = std::max(dmax, std::fabs(C_[i][i]));
  }
  if (dmin > 0 && dmax / dmin > tolconditioncov_) return true;
  return false;
}

// ============================================================================== TPE
namespace {

const double kEps = 1e-12;
const double kLogSqrt2Pi = 0.5 * std::log(2 * M_PI);

inline double norm_cdf(double x) { return 0.5 * std::erfc(-x / std::sqrt(2.0)); }

struct Gmm {
  std::vector<double> w, mu, sigma;
  double low, high, q;
  double logZ = 0;  // log of truncated mass
  void finalize() {
    double z = 0;
    for (size_t k = 0; k < w.size(); ++k)
      z += w[k] * (norm_cdf((high - mu[k]) / sigma[k]) - norm_cdf((low - mu[k]) / sigma[k]));
    logZ = std::log(std::max(z, kEps));
  }
  double sample(std::mt19937_64& rng) const {
    std::discrete_distribution<int> pick(w.begin(), w.end());
    std::normal_distribution<double> nd(0, 1);
    for (int t = 0; t < 1000; ++t) {
      int k = pick(rng);
      double x = mu[k] + sigma[k] * nd(rng);
      if (x >= low && x <= high) return quantize(x);
    }
    std::uniform_real_distribution<double> u(low, high);
    return quantize(u(rng));
  }
  double quantize(double x) const {
    if (q <= 0) return x;
    double r = low + std::round((x - low) / q) * q;
    return std::min(std::max(r, low), high);
  }
  double logpdf(double x) const {
    double acc = 0;
    if (q > 0) {
      double lb = std::max(x - q / 2, low), ub = std::min(x + q / 2, high);
      for (size_t k = 0; k < w.size(); ++k)
        acc += w[k] * (norm_cdf((ub - mu[k]) / sigma[k]) - norm_cdf((lb - mu[k]) / sigma[k]));
      return std::log(std::max(acc, kEps)) - logZ;
    }
    double mx = -std::numeric_limits<double>::infinity();
    std::vector<double> t(w.size());
    for (size_t k = 0; k < w.size(); ++k) {
      double z = (x - mu[k]) / sigma[k];
      t[k] = std::log(std::max(w[k], kEps)) - 0.5 * z * z - std::log(sigma[k]) - kLogSqrt2Pi;
      mx = std::max(mx, t[k]);
    }
    double s = 0;
    for (double v : t) s += std::exp(v - mx);
    return mx + std::log(s) - logZ;
  }
};

std::vector<double> forgetting_weights(size_t n, int lf) {
  std::vector<double> w(n, 1.0);
  if (lf <= 0 || n <= static_cast<size_t>(lf)) return w;
  size_t nramp = n - lf;
  for (size_t i = 0; i < nramp; ++i)
    w[i] = nramp == 1 ? 1.0 / n : (1.0 / n) + (1.0 - 1.0 / n) * i / (nramp - 1);
  return w;
}

// hyperopt.tpe.adaptive_parzen_normal
Gmm parzen(const std::vector<double>& obs, const TpeDim& d, const TpeSettings& s) {
  Gmm g;
  g.low = d.low;
  g.high = d.high;
  g.q = d.q;
  double prior_mu = 0.5 * (d.low + d.high), prior_sigma = std::max(d.high - d.low, kEps);
  if (obs.empty()) {
    g.w = {1.0};
    g.mu = {prior_mu};
    g.sigma = {prior_sigma};
  } else if (obs.size() == 1) {
    if (prior_mu < obs[0]) {
      g.mu = {prior_mu, obs[0]};
      g.sigma = {prior_sigma, prior_sigma * 0.5};
      g.w = {s.prior_weight, 1.0};
    } else {
      g.mu = {obs[0], prior_mu};
      g.sigma = {prior_sigma * 0.5, prior_sigma};
      g.w = {1.0, s.prior_weight};
    }
  } else {
    std::vector<size_t> order(obs.size());
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return obs[a] < obs[b]; });
    std::vector<double> sorted;
    for (size_t i : order) sorted.push_back(obs[i]);
    size_t pos = std::lower_bound(sorted.begin(), sorted.end(), prior_mu) - sorted.begin();
    std::vector<double> fw = forgetting_weights(obs.size(), s.linear_forgetting);
    std::vector<double> sw;
    for (size_t i : order) sw.push_back(fw[i]);
    sorted.insert(sorted.begin() + pos, prior_mu);
    sw.insert(sw.begin() + pos, s.prior_weight);
    size_t m = sorted.size();
    std::vector<double> sig(m);
    for (size_t i = 1; i + 1 < m; ++i) sig[i] = std::max(sorted[i] - sorted[i - 1], sorted[i + 1] - sorted[i]);
    sig[0] = sorted[1] - sorted[0];
    sig[m - 1] = sorted[m - 1] - sorted[m - 2];
    sig[pos] = prior_sigma;
    g.mu = sorted;
    g.sigma = sig;
    g.w = sw;
  }
  double maxs = prior_sigma;
  double mins = s.consider_magic_clip ? prior_sigma / std::min(100.0, 1.0 + g.mu.size()) : kEps;
  for (auto& v : g.sigma) v = std::min(std::max(v, mins), maxs);
  double tw = std::accumulate(g.w.begin(), g.w.end(), 0.0);
  for (auto& v : g.w) v /= tw;
  g.finalize();
  return g;
}

std::vector<double> cat_dist(const std::vector<double>& obs, int n, double prior_weight) {
  std::vector<double> p(n, prior_weight);
  for (double v : obs) {
    int c = static_cast<int>(std::llround(v));
    if (c >= 0 && c < n) p[c] += 1.0;
  }
  double t = std::accumulate(p.begin(), p.end(), 0.0);
  for (auto& v : p) v /= t;
  return p;
}

size_t n_below(size_t n, const TpeSettings& s) {
  double v = s.gamma_mode == 0 ? std::ceil(s.gamma * std::sqrt(static_cast<double>(n)))
                               : std::min(std::ceil(s.gamma * n), 25.0);
  size_t k = static_cast<size_t>(v);
  if (k < 1 && n > 0) k = 1;
  return std::min(k, n);
}

double logsumexp(const std::vector<double>& v) {
  double mx = -std::numeric_limits<double>::infinity();
  for (double x : v) mx = std::max(mx, x);
  if (!std::isfinite(mx)) return mx;
  double s = 0;
  for (double x : v) s += std::exp(x - mx);
  return mx + std::log(s);
}

// Joint-kernel Parzen estimator for multivariate TPE.
struct JointKde {
  const std::vector<TpeDim>* dims;
  std::vector<std::vector<double>> centers;  // per kernel
  std::vector<double> logw;
  std::vector<double> bw;  // per numeric dim
  double prior_weight;
  void build(const std::vector<TpeDim>& ds, const std::vector<std::vector<double>>& obs, double pw) {
    dims = &ds;
    prior_weight = pw;
    size_t D = ds.size(), n = obs.size();
    centers = obs;
    std::vector<double> prior(D);
    for (size_t d = 0; d < D; ++d) prior[d] = ds[d].kind == 1 ? -1 : 0.5 * (ds[d].low + ds[d].high);
    centers.push_back(prior);  // prior kernel (categorical -1 == uniform)
    logw.assign(n + 1, std::log(1.0));
    logw[n] = std::log(std::max(pw, kEps));
    double tot = logsumexp(logw);
    for (auto& v : logw) v -= tot;
    bw.assign(D, 1);
    double nn = std::max<double>(1, n);
    for (size_t d = 0; d < D; ++d) {
      double range = std::max(ds[d].high - ds[d].low, kEps);
      bw[d] = std::max(0.2 * std::pow(nn, -1.0 / (D + 4)) * range, range / std::min(100.0, 1.0 + nn));
    }
  }
  double dim_logpdf(size_t k, size_t d, double x) const {
    const TpeDim& td = (*dims)[d];
    double c = centers[k][d];
    if (td.kind == 1) {
      int n = std::max(1, td.n_choices);
      if (c < 0) return -std::log(static_cast<double>(n));
      // peaked categorical kernel
      double p_same = (1.0 + 1.0 / n) / (1.0 + 1.0), p_other = (1.0 / n) / 2.0;
      return std::log(static_cast<int>(std::llround(x)) == static_cast<int>(std::llround(c)) ? p_same : p_other);
    }
    if (k == centers.size() - 1) return -std::log(std::max(td.high - td.low, kEps));  // uniform prior
    double s = bw[d];
    double z = (x - c) / s;
    double mass = norm_cdf((td.high - c) / s) - norm_cdf((td.low - c) / s);
    return -0.5 * z * z - std::log(s) - kLogSqrt2Pi - std::log(std::max(mass, kEps));
  }
  double logpdf(const std::vector<double>& x) const {
    std::vector<double> t(centers.size());
    for (size_t k = 0; k < centers.size(); ++k) {
      double v = logw[k];
      for (size_t d = 0; d < x.size(); ++d) v += dim_logpdf(k, d, x[d]);
      t[k] = v;
    }
    return logsumexp(t);
  }
  std::vector<double> sample(std::mt19937_64& rng) const {
    std::vector<double> w;
    for (double lw : logw) w.push_back(std::exp(lw));
    std::discrete_distribution<size_t> pick(w.begin(), w.end());
    size_t k = pick(rng);
    std::vector<double> x(dims->size());
    std::normal_distribution<double> nd(0, 1);
    for (size_t d = 0; d < dims->size(); ++d) {
      const TpeDim& td = (*dims)[d];
      double c = centers[k][d];
      if (td.kind == 1) {
        int n = std::max(1, td.n_choices);
        std::uniform_int_distribution<int> ui(0, n - 1);
        if (c < 0) {
          x[d] = ui(rng);
        } else {
          std::uniform_real_distribution<double> u(0, 1);
          double p_same = (1.0 + 1.0 / n) / 2.0;
          x[d] = u(rng) < p_same ? std::llround(c) : ui(rng);
        }
        continue;
      }
      double v;
      if (k == centers.size() - 1) {
        std::uniform_real_distribution<double> u(td.low, td.high);
        v = u(rng);
      } else {
        v = c;
        for (int t = 0; t < 1000; ++t) {
          v = c + bw[d] * nd(rng);
          if (v >= td.low && v <= td.high) break;
        }
        v = std::min(std::max(v, td.low), td.high);
      }
      if (td.q > 0) v = std::min(std::max(td.low + std::round((v - td.low) / td.q) * td.q, td.low), td.high);
      x[d] = v;
    }
    return x;
  }
};

}  // namespace

std::vector<double> tpe_sample(const std::vector<TpeDim>& dims, const std::vector<std::vector<double>>& xs,
                               const std::vector<double>& losses, const TpeSettings& s, uint64_t seed) {
  std::mt19937_64 rng(seed);
  const size_t n = xs.size(), D = dims.size();
  std::vector<size_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return losses[a] < losses[b]; });
  size_t nb = n_below(n, s);
  std::vector<char> is_below(n, 0);
  for (size_t i = 0; i < nb; ++i) is_below[order[i]] = 1;
  // chronological order within each group (for linear forgetting)
  std::vector<std::vector<double>> below, above;
  for (size_t i = 0; i < n; ++i) (is_below[i] ? below : above).push_back(xs[i]);
  std::vector<double> out(D, 0);
  const int ncand = std::max(1, s.n_ei_candidates);

  if (s.multivariate) {
    JointKde lk, gk;
    lk.build(dims, below, s.prior_weight);
    gk.build(dims, above, s.prior_weight);
    double best = -std::numeric_limits<double>::infinity();
    for (int c = 0; c < ncand; ++c) {
      std::vector<double> x = lk.sample(rng);
      double score = lk.logpdf(x) - gk.logpdf(x);
      if (score > best) {
        best = score;
        out = x;
      }
    }
    return out;
  }
  for (size_t d = 0; d < D; ++d) {
    std::vector<double> ob, oa;
    for (const auto& x : below) ob.push_back(x[d]);
    for (const auto& x : above) oa.push_back(x[d]);
    if (dims[d].kind == 1) {
      int nc = std::max(1, dims[d].n_choices);
      std::vector<double> pb = cat_dist(ob, nc, s.prior_weight), pa = cat_dist(oa, nc, s.prior_weight);
      std::discrete_distribution<int> pick(pb.begin(), pb.end());
      double best = -std::numeric_limits<double>::infinity();
      int bi = 0;
      for (int c = 0; c < ncand; ++c) {
        int k = pick(rng);
        double score = std::log(pb[k]) - std::log(pa[k]);
        if (score > best) {
          best = score;
          bi = k;
        }
      }
      out[d] = bi;
      continue;
    }
    Gmm gb = parzen(ob, dims[d], s), ga = parzen(oa, dims[d], s);
    double best = -std::numeric_limits<double>::infinity();
    double bx = gb.mu.empty() ? dims[d].low : gb.mu[0];
    for (int c = 0; c < ncand; ++c) {
      double x = gb.sample(rng);
      double score = gb.logpdf(x) - ga.logpdf(x);
      if (score > best) {
        best = score;
        bx = x;
      }
    }
    out[d] = bx;
  }
  return out;
}

}  // namespace katib
