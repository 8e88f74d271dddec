// Batched tree-ensemble inference on the MI355X (K9 in SURVEY §2.4).
// The reference scores one row per UDF call through
// LGBM_BoosterPredictForMatSingle (lightgbm/.../booster/LightGBMBooster.scala
// :539-557); here a whole partition is scored by one kernel launch with the
// ensemble packed once into device memory.
#pragma once
#include <cstdint>
#include <memory>

namespace sml {

class Booster;

class GpuPredictor {
 public:
  GpuPredictor(const Booster& b, int start_iteration, int num_iteration, int device);
  ~GpuPredictor();
  int NumOutputs() const { return num_out_; }
  int NumTrees() const { return num_trees_; }
  void Predict(const double* X, int64_t n, int ncols, bool normal, double* out);
  // raw scores of float32 (f32) or float64 rows, one chunked upload + traversal pass (n x NumOutputs)
  void PredictRaw(const void* X, bool f32, int64_t n, int ncols, double* out);
  void PredictLeaf(const double* X, int64_t n, int ncols, int32_t* out);
  // TreeSHAP contributions, layout of Booster::Predict(kPredictContrib);
  // false if a path has more unique features than a wave64 holds
  bool PredictContrib(const double* X, int64_t n, int ncols, double* out);

 private:
  struct Impl;
  bool BuildShap();
  std::unique_ptr<Impl> impl_;
  const Booster* booster_;
  int num_out_ = 1, num_trees_ = 0;
};

}  // namespace sml
