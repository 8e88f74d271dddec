// Objectives (gradient/hessian, init score, output transform) and metrics.
//
// Objective list = the reference's documented set (LightGBMRegressor.scala
// :25-36 regression family; LightGBMClassifier binary/multiclass; LightGBMRanker
// lambdarank). The per-row formulas are SML_HD so the HIP gradient kernel (K2)
// evaluates exactly the same expressions as the host path.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "config.h"
#include "dataset.h"
#include "split_math.h"

namespace sml {

enum ObjKind : int {
  kObjBinary = 0, kObjMulticlass, kObjMulticlassOVA, kObjRegression, kObjL1, kObjHuber, kObjFair,
  kObjPoisson, kObjQuantile, kObjMape, kObjGamma, kObjTweedie, kObjCrossEntropy, kObjLambdarank,
  kObjCustom
};

struct ObjParams {
  int kind;
  int num_class;
  double sigmoid;
  double alpha;
  double fair_c;
  double poisson_max_delta_step;
  double tweedie_rho;
  double pos_weight, neg_weight;  // binary label weights (is_unbalance / scale_pos_weight)
};

// Single-output per-row gradient. `w` is the sample weight (1 if none).
SML_HD void PointGradient(const ObjParams& p, double s, double y, double w, float* g, float* h) {
  double gg = 0, hh = 1;
  switch (p.kind) {
    case kObjBinary:
    case kObjMulticlassOVA: {
      const double lab = y > 0 ? 1.0 : -1.0;
      const double lw = y > 0 ? p.pos_weight : p.neg_weight;
      const double resp = -lab * p.sigmoid / (1.0 + exp(lab * p.sigmoid * s));
      const double ar = fabs(resp);
      gg = resp * lw;
      hh = ar * (p.sigmoid - ar) * lw;
      break;
    }
    case kObjCrossEntropy: {
      const double z = 1.0 / (1.0 + exp(-s));
      gg = z - y; hh = z * (1.0 - z);
      break;
    }
    case kObjRegression: gg = s - y; hh = 1; break;
    case kObjL1: { const double d = s - y; gg = d > 0 ? 1.0 : (d < 0 ? -1.0 : 0.0); hh = 1; break; }
    case kObjHuber: {
      const double d = s - y;
      gg = fabs(d) <= p.alpha ? d : (d > 0 ? p.alpha : -p.alpha); hh = 1;
      break;
    }
    case kObjFair: {
      const double x = s - y, c = p.fair_c;
      gg = c * x / (fabs(x) + c); hh = c * c / ((fabs(x) + c) * (fabs(x) + c));
      break;
    }
    case kObjPoisson: {
      const double e = exp(s);
      gg = e - y; hh = exp(s + p.poisson_max_delta_step);
      break;
    }
    case kObjQuantile: {
      const double d = s - y;
      gg = d >= 0 ? (1.0 - p.alpha) : -p.alpha; hh = 1;
      break;
    }
    case kObjMape: {
      const double d = s - y;
      const double lw = 1.0 / (fabs(y) > 1.0 ? fabs(y) : 1.0);
      gg = (d > 0 ? 1.0 : (d < 0 ? -1.0 : 0.0)) * lw; hh = 1;
      break;
    }
    case kObjGamma: {
      const double e = exp(-s);
      gg = 1.0 - y * e; hh = y * e;
      break;
    }
    case kObjTweedie: {
      const double rho = p.tweedie_rho;
      const double e1 = exp((1.0 - rho) * s), e2 = exp((2.0 - rho) * s);
      gg = -y * e1 + e2; hh = -y * (1.0 - rho) * e1 + (2.0 - rho) * e2;
      break;
    }
    default: break;
  }
  *g = static_cast<float>(gg * w);
  *h = static_cast<float>(hh * w);
}

class Objective {
 public:
  explicit Objective(const Config& cfg);
  void Init(const Dataset& data);
  void Init(const float* label, const float* weight, int64_t n, const std::vector<int32_t>& qb);
  // score layout: class-major, score[k * n + i]
  void GetGradients(const double* score, float* g, float* h) const;
  // the start score over every rank's rows (comm: the data-parallel group, or nullptr)
  double BoostFromScore(int class_id, class Comm* comm = nullptr) const;
  void ConvertOutput(const double* raw, double* out) const;  // one row, num_out values
  int NumModelPerIteration() const { return num_tree_per_iter_; }
  bool NeedRenewTreeOutput() const { return p_.kind == kObjL1 || p_.kind == kObjQuantile || p_.kind == kObjMape; }
  // Renewed leaf output (percentile of residuals of the rows in the leaf).
  double RenewLeafOutput(const double* score, const int64_t* rows, int64_t cnt) const;
  std::string ToString() const;
  const ObjParams& params() const { return p_; }
  std::string name() const { return name_; }
  std::string DefaultMetric() const;
  static std::string Canonical(const std::string& name);
  // lambdarank tables (the HIP gradient kernel uploads them once)
  const std::vector<int32_t>& query_boundaries() const { return qb_; }
  const std::vector<double>& inv_max_dcg() const { return inv_max_dcg_; }
  const std::vector<double>& label_gain() const { return label_gain_; }
  const float* labels() const { return label_; }
  int64_t num_rows() const { return n_; }
  int max_position() const { return max_position_; }
  bool lambdarank_norm() const { return lambdarank_norm_; }

 private:
  void LambdarankGradients(const double* score, float* g, float* h) const;
  std::string name_;
  ObjParams p_{};
  int num_tree_per_iter_ = 1;
  const float* label_ = nullptr;
  const float* weight_ = nullptr;
  int64_t n_ = 0;
  std::vector<int32_t> qb_;
  std::vector<double> label_gain_;
  std::vector<double> inv_max_dcg_;
  int max_position_ = 20;
  bool lambdarank_norm_ = true;
  bool boost_from_average_ = true;
  bool unbalance_ = false;
};

// Metrics (K11). score layout class-major like above; returns one value.
double EvalMetric(const std::string& name, const Objective& obj, const double* score,
                  const float* label, const float* weight, int64_t n, int num_class,
                  const std::vector<int32_t>& qb, const std::vector<double>& label_gain);
bool MetricHigherBetter(const std::string& name);

}  // namespace sml
