// Training backends: where histograms, split search, row partitioning and
// score updates run. The CPU backend is the oracle / no-GPU path (SURVEY §7.0
// D4); the HIP backend keeps the binned matrix, gradients, scores and the
// whole leaf-wise growth loop resident on the MI355X.
#pragma once
#include <algorithm>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "comm.h"
#include "config.h"
#include "dataset.h"
#include "objective.h"
#include "sampling.h"
#include "split_math.h"
#include "tree.h"

namespace sml {

struct TrainStats {
  double hist_ms = 0, split_ms = 0, partition_ms = 0, grad_ms = 0, score_ms = 0, comm_ms = 0;
  int64_t comm_calls = 0;  // device histogram allreduces issued
  int64_t comm_dyn_calls = 0;   // of which sized on the device (only the round's expansions travel)
  double comm_bytes_max = 0;    // host-side upper bound of the histogram bytes reduced
  int64_t comm_dev_bytes = 0;   // bytes this rank pushed through the device-driven transport (P2P)
  // device-side (hipEvent) time of whole tree growths and score updates; device memory in use after Init
  double device_tree_ms = 0, device_score_ms = 0, device_mem_mb = 0;
  int64_t trees = 0;
};

class TrainBackend {
 public:
  virtual ~TrainBackend() = default;
  virtual std::string Name() const = 0;
  virtual void Init(const Dataset* data, const Config& cfg, int num_tree_per_iter) = 0;
  virtual void SetScores(const std::vector<double>& s) = 0;  // class-major n*K
  // score[k][i] = per_class[k] for every row (boost-from-average start); backends fill in place
  virtual void FillScores(const std::vector<double>& per_class, int64_t n) {
    std::vector<double> s(static_cast<size_t>(n) * per_class.size());
    for (size_t k = 0; k < per_class.size(); ++k) std::fill(s.begin() + k * n, s.begin() + (k + 1) * n, per_class[k]);
    SetScores(s);
  }
  virtual void GetScores(std::vector<double>* s) = 0;
  virtual void AddBias(int k, double b) = 0;
  virtual void ScaleScore(int k, double s) = 0;
  virtual void ComputeGradients(const Objective& obj) = 0;
  virtual void SetGradients(const float* g, const float* h) = 0;  // class-major n*K
  virtual void GetGradients(std::vector<float>* g, std::vector<float>* h) = 0;
  // Restrict training rows (bagging/GOSS). nullptr = all rows.
  virtual void SetBag(const std::vector<int32_t>* rows) = 0;
  // Draw the bag (and apply GOSS gradient scaling) where the gradients live.
  // Returns false when the backend leaves sampling to the host.
  virtual bool SampleRows(const RowSampleSpec& spec) { (void)spec; return false; }
  // Training-metric value computed where the scores live (K11); false = host path.
  virtual bool EvalOnDevice(const std::string& name, const Objective& obj, double* out) {
    (void)name; (void)obj; (void)out;
    return false;
  }
  // K11 validation sets: the backend may keep a validation set's bins and scores where its own scores
  // live (true: it now owns the scores, `scores` = the class-major start values); false = host-resident.
  virtual bool AddValidSet(int vi, const Dataset& vd, const std::vector<double>& scores, const Config& cfg) {
    (void)vi; (void)vd; (void)scores; (void)cfg;
    return false;
  }
  // fold tree `t` (class k) into a backend-owned validation set's scores (ValidOp in valid_gpu.h)
  virtual void ValidApplyTree(int vi, const Tree& t, int k, int op, double p) {
    (void)vi; (void)t; (void)k; (void)op; (void)p;
    throw std::logic_error("backend holds no validation sets");
  }
  virtual void GetValidScores(int vi, std::vector<double>* s) {
    (void)vi; (void)s;
    throw std::logic_error("backend holds no validation sets");
  }
  virtual bool EvalValidOnDevice(int vi, const std::string& name, const Objective& obj, double* out) {
    (void)vi; (void)name; (void)obj; (void)out;
    return false;
  }
  virtual Tree TrainTree(int k, const std::vector<char>& feature_mask) = 0;
  // Grow a tree and, when the backend can, apply score[k] += shrink * tree(row) right behind the
  // growth on the device (no host round trip between them); *updated tells the caller whether
  // it still has to call UpdateScore(t, k, 1.0) with the returned (unshrunk) tree shrunk by `shrink`.
  virtual Tree TrainTreeAndUpdateScore(int k, const std::vector<char>& feature_mask, double shrink, bool* updated) {
    (void)shrink;
    *updated = false;
    return TrainTree(k, feature_mask);
  }
  // score[k] += scale * tree(row) for every training row
  virtual void UpdateScore(const Tree& t, int k, double scale) = 0;
  // Leaf index of every training row for `t` (renew / DART helpers).
  virtual void PredictLeafIndex(const Tree& t, std::vector<int32_t>* leaf) = 0;
  virtual void Synchronize() {}
  void SetComm(Comm* c) { comm_ = c; }
  Comm* comm() const { return comm_; }
  TrainStats stats;

 protected:
  Comm* comm_ = nullptr;
};

std::unique_ptr<TrainBackend> MakeCpuBackend();
// Defined in the HIP translation unit; returns nullptr if no device.
std::unique_ptr<TrainBackend> MakeGpuBackend(int device_id);
bool GpuAvailable();
// metric_gpu.hip: auc / binary_logloss / binary_error / l2 / rmse / l1 on device scores
bool DeviceEvalMetric(const std::string& name, const ObjParams& p, const double* score, const float* label,
                      const float* weight, int64_t n, void* stream, double* out);

// Host reference of the split search (K5): best split of one feature given its
// histogram. Used by the CPU backend and by tests that compare the device.
void FindBestSplitFeature(const double* hg, const double* hh, int nb, const BinMapper& m,
                          int feature_inner, double sum_g, double sum_h, int64_t cnt,
                          const SplitParams& sp, SplitResult* best, const MonoCtx* mc = nullptr);
SplitParams MakeSplitParams(const Config& cfg);
// features each node samples under feature_fraction_bynode (0 = every allowed feature)
int BynodeK(const Config& cfg, const std::vector<char>& allowed);

}  // namespace sml
