// Boosting driver + model (native components N2/N4 of SURVEY §2.3).
//
// API mirrors the C-API surface the reference calls through SWIG
// (lightgbm/.../booster/LightGBMBooster.scala: BoosterCreate 241, Merge 256,
// AddValidData 264, UpdateOneIter 359, UpdateOneIterCustom 384, GetEval 303,
// SaveModelToString 276, DumpModel 481, PredictFor* 520-557,
// FeatureImportance 504, ResetParameter 320).
#pragma once
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <random>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "backend.h"
#include "comm.h"
#include "config.h"
#include "dataset.h"
#include "objective.h"
#include "tree.h"

namespace sml {

enum PredictType { kPredictRaw = 0, kPredictNormal = 1, kPredictLeaf = 2, kPredictContrib = 3 };

// What Booster::DetachTraining takes out of a fitted booster: freed by whoever holds it (Free() / destructor),
// e.g. on a background thread, while the booster keeps serving predictions.
struct DetachedTraining {
  std::unique_ptr<TrainBackend> backend;
  std::shared_ptr<Dataset> train;
  std::vector<std::shared_ptr<Dataset>> valid;
  std::vector<std::unique_ptr<Objective>> valid_objectives;
  std::vector<std::vector<double>> valid_scores;
  void Free() {
    static const bool prof = std::getenv("SML_RELEASE_PROF") != nullptr;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    const auto t0 = now();
    if (backend) backend->Synchronize();
    const auto t1 = now();
    backend.reset();
    const auto t2 = now();
    train.reset();
    const auto t3 = now();
    valid.clear();
    valid_objectives.clear();
    valid_scores.clear();
    if (prof && (t3 - t0) > std::chrono::microseconds(50))
      std::fprintf(stderr, "release: sync %.3f backend %.3f train %.3f valid %.3f ms\n", ms(t0, t1), ms(t1, t2),
                   ms(t2, t3), ms(t3, now()));
  }
  ~DetachedTraining() { Free(); }
};

class Booster {
 public:
  Booster() = default;
  // training constructor
  Booster(std::shared_ptr<Dataset> train, const std::string& params, Comm* comm = nullptr);
  static std::unique_ptr<Booster> FromModelString(const std::string& model);

  void AddValidData(std::shared_ptr<Dataset> valid, const std::string& name);
  bool ValidOnDevice(int i) const { return valid_dev_.at(i) != 0; }
  void MergeFrom(const Booster& other);       // continue training from `other`
  void ResetParameter(const std::string& params);
  // One boosting iteration. Custom gradients (class-major n*K) if non-null.
  // Returns true when no tree could be grown (training finished).
  bool TrainOneIter(const float* grad = nullptr, const float* hess = nullptr);
  void RollbackOneIter();
  // metric values of data set `idx` (0 = train, 1.. = valid)
  std::vector<std::pair<std::string, double>> Eval(int idx, bool device = true);
  std::vector<std::string> EvalNames() const;
  void GetTrainScores(std::vector<double>* s);
  void GetPredictForValid(int idx, std::vector<double>* s) const;

  // model
  std::string SaveModelToString(int start_iteration, int num_iteration, int importance_type) const;
  std::string DumpModel(int start_iteration, int num_iteration) const;
  void Predict(const double* X, int64_t nrows, int ncols, int predict_type, int start_iteration,
               int num_iteration, double* out) const;
  int PredictOutputSize(int predict_type, int start_iteration, int num_iteration) const;
  std::vector<double> FeatureImportance(int num_iteration, int importance_type) const;
  // raw scores (n x K, row-major) -> transformed outputs (sigmoid/softmax/exp)
  void ConvertOutputs(const double* raw, int64_t n, double* out) const;
  const std::vector<Tree>& trees() const { return trees_; }
  bool average_output() const { return average_output_; }
  std::pair<int, int> TreeRangePublic(int s, int n) const { return TreeRange(s, n); }

  int NumClasses() const { return num_class_; }
  int NumModelPerIteration() const { return num_tree_per_iter_; }
  int NumFeatures() const { return max_feature_idx_ + 1; }
  int NumTotalModel() const { return static_cast<int>(trees_.size()); }
  int CurrentIteration() const { return static_cast<int>(trees_.size()) / std::max(1, num_tree_per_iter_); }
  const std::vector<std::string>& FeatureNames() const { return feature_names_; }
  const Config& config() const { return cfg_; }
  // the backend that trained this booster (kept after ReleaseTraining)
  std::string BackendName() const { return backend_ ? backend_->Name() : (released_ ? released_backend_ : "none"); }
  TrainStats* stats() { return backend_ ? &backend_->stats : nullptr; }
  void Synchronize() { if (backend_) backend_->Synchronize(); }
  // gradients / hessians of the last iteration (class-major n*K; after GOSS rescaling)
  void GetGradients(std::vector<float>* g, std::vector<float>* h) { Backend()->GetGradients(g, h); }
  // Keep only the first `num_iteration` iterations (early stopping).
  void Truncate(int num_iteration);
  // Free everything only training needs (backend with its device buffers, datasets, validation state); the
  // trees, objective and feature metadata stay, so prediction / model text / importance keep working and
  // training calls raise. A fitted model's booster is released off the fit's critical path.
  void ReleaseTraining();
  // the same, but the released state is handed back instead of freed here (quick: pointer moves only)
  std::unique_ptr<DetachedTraining> DetachTraining();
  bool training_released() const { return released_; }
  const Objective* objective() const { return objective_.get(); }

 private:
  void InitTraining();
  void Bagging(int iter);
  void Goss();
  std::vector<char> SampleFeatures();
  void PredictRaw(const double* x, int start_tree, int end_tree, double* out) const;
  std::pair<int, int> TreeRange(int start_iteration, int num_iteration) const;

  Config cfg_;
  std::string params_str_;
  std::shared_ptr<Dataset> train_;
  std::vector<std::shared_ptr<Dataset>> valid_;
  std::vector<std::string> valid_names_;
  std::vector<std::vector<double>> valid_scores_;  // host-resident sets only (empty when on the device)
  std::vector<char> valid_dev_;                    // the backend holds set vi's bins and scores
  // fold tree t into validation set vi's class-k scores (ValidOp), on the device or the host
  void ValidApply(size_t vi, const Tree& t, int k, int op, double p);
  std::unique_ptr<Objective> objective_;
  std::vector<std::unique_ptr<Objective>> valid_objectives_;
  std::unique_ptr<TrainBackend> backend_;
  Comm* comm_ = nullptr;
  std::vector<Tree> trees_;
  std::vector<double> init_scores_;   // per class, folded into the first tree(s)
  bool boosted_first_ = false;
  int num_class_ = 1;
  int num_tree_per_iter_ = 1;
  int max_feature_idx_ = 0;
  int label_index_ = 0;
  bool average_output_ = false;
  std::string objective_str_;
  std::vector<std::string> feature_names_;
  std::vector<std::string> feature_infos_;
  std::string loaded_parameters_;
  int iter_ = 0;
  std::mt19937 bag_rng_, feat_rng_, drop_rng_;
  bool bagged_ = false;
  std::vector<int32_t> bag_rows_;
  // rf: per-class running sums of tree outputs are kept as scores/iter count
  int rf_trees_ = 0;
  bool released_ = false;
  std::string released_backend_;
  TrainBackend* Backend() const {
    if (!backend_) throw std::runtime_error(released_ ? "booster training state was released" : "booster has no backend");
    return backend_.get();
  }
};

}  // namespace sml
