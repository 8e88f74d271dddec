// K11 for validation sets: the binned validation matrix, its scores, labels, weights and query
// boundaries live in HBM next to the training state. Every new tree is applied to the validation
// scores by a device traversal over the bins (the tree itself is a ~1 KB upload), and the metrics
// (auc / logloss / error / l1 / l2 / rmse / multi_logloss / multi_error / ndcg@k / map@k) reduce where
// the scores are: the host reads one double per metric, never the n x K score matrix. The reference
// evaluates validation data inside LightGBM's native booster every iteration for early stopping
// (lightgbm/.../TrainUtils.scala:137-169, LightGBMBooster.scala:300-314).
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "dataset.h"
#include "objective.h"
#include "tree.h"

namespace sml {

// how a tree's output `o` (leaf value of the row) is folded into a validation score `v`
enum ValidOp : int {
  kValidAdd = 0,      // v += p * o
  kValidAddSub = 1,   // v += o - p           (first iteration: the tree carries the init bias p)
  kValidRfAvg = 2,    // v = p == 0 ? o : (v * p + o) / (p + 1)   (random forest running mean, p = trees so far)
  kValidDart = 3,     // v += o - o / p       (DART renormalisation of a dropped tree, p = factor)
  kValidConst = 4,    // v += p               (tree ignored)
};

// host reference of the fold (booster.cpp uses it for host-resident validation sets)
inline double ValidFold(double v, double o, int op, double p) {
  switch (op) {
    case kValidAdd: return v + p * o;
    case kValidAddSub: return v + (o - p);
    case kValidRfAvg: return p == 0.0 ? o : (v * p + o) / (p + 1.0);
    case kValidDart: return v + (o - o / p);
    default: return v + p;
  }
}

class DeviceValidSet {
 public:
  // `scores` is class-major (K x n). Bins come from the dataset's HBM copy when it has one on this
  // device, else from its host bins (uploaded once).
  DeviceValidSet(const Dataset& vd, const std::vector<double>& scores, int K, const std::vector<double>& label_gain,
                 int device, void* stream);
  ~DeviceValidSet();
  void ApplyTree(const Tree& t, int k, int op, double p);
  void GetScores(std::vector<double>* out);
  bool Eval(const std::string& name, const ObjParams& p, int num_class, double* out);

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

// metric_gpu.hip: every device metric, on class-major device scores (qb / gain only for ndcg / map)
struct DeviceMetricInputs {
  const double* score = nullptr;
  const float* label = nullptr;
  const float* weight = nullptr;
  int64_t n = 0;
  int num_class = 1;
  const int32_t* qb = nullptr;  // device query boundaries (nq + 1)
  int nq = 0;
  const double* gain = nullptr;  // device label gains
  int ngain = 0;
};
bool DeviceEvalMetricFull(const std::string& name, const ObjParams& p, const DeviceMetricInputs& in, void* stream,
                          double* out);

}  // namespace sml
