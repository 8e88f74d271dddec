// Device-resident hashed linear learner (K12/K13 of SURVEY §2.4): the weight
// table (2^b x {w, G, N}) lives in HBM, mini-batches of CSR examples are learned
// by one wave per example with VW's adaptive / normalized / invariant update as
// hogwild atomics on the touched weights (batch 1 = the sequential learner),
// --oaa runs one wave per class, and touched blocks are averaged across GPUs with
// RCCL at sync points (C4: the reference's spanning-tree AllReduce at endPass).
#pragma once
#include <array>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace smlvw {

struct GpuSgdConfig {
  int bits = 18;
  float lr = 0.5f;
  float power_t = 0.5f;
  float initial_t = 0.f;
  float l2 = 0.f;
  float l1 = 0.f;
  float tau = 0.5f;      // quantile loss
  int loss = 0;          // 0 squared, 1 logistic, 2 hinge, 3 quantile
  bool adaptive = true;  // VW's default update: adaptive + normalized + invariant
  bool normalized = true;
  bool invariant = true;
  int oaa = 0;           // one-against-all classes (0: scalar learner)
  int csoaa = 0;         // cost-sensitive one-against-all classes (0: off)
  int cb = -1;           // contextual bandit with action-dependent features: -1 off, 0 mtr, 1 dr, 2 ips
  int cats = 0;          // --cats_pdf / --cats K discretized actions (0: off): the filter tree of K leaves
  float cats_min = 0.f, cats_max = 1.f, cats_bw = 1.f;  // --min_value / --max_value / --bandwidth
  bool cb_explore = false;
  float epsilon = 0.05f;
};

// Namespace blocks of a partition for the device featurization (GpuSgd::StagePlan): one CSR per feature
// column, already hashed; `group` = the namespace (blocks sharing it are concatenated per row), `level` 1 =
// indexed through the plan's row_map (contextual-bandit action rows reading their example's shared block).
struct HostBlock {
  const int64_t* ip;
  const uint32_t* idx;
  const float* val;
  int64_t rows;
  int level;
  int group;
};

struct FeatPlan {
  std::vector<HostBlock> blocks;
  int ngroups = 0;
  std::vector<std::array<int, 3>> inter;  // namespace groups; [2] = -1 for a pair
  bool constant = true;
  const int64_t* row_map = nullptr;       // n entries (level-1 blocks)
};

class GpuSgd {
 public:
  GpuSgd(const GpuSgdConfig& cfg, int device);
  ~GpuSgd();
  // indices are pre-hashed feature ids (masked on device); labels in the loss's convention (logistic:
  // -1/+1; oaa: 1-based class). Returns the progressive predictions (oaa: predicted class).
  void Learn(const int64_t* indptr, const uint32_t* indices, const float* values, const float* labels,
             const float* weights, int64_t n, int batch, float* preds_out);
  void Predict(const int64_t* indptr, const uint32_t* indices, const float* values, int64_t n, float* out);
  // device-resident pass data (multi-pass / multi-segment training reads it from HBM): Stage uploads once,
  // LearnStaged learns rows [r0, r1) of it in order
  void Stage(const int64_t* indptr, const uint32_t* indices, const float* values, const float* labels,
             const float* weights, int64_t n);
  void LearnStaged(int64_t r0, int64_t r1, int batch, float* preds_out);
  // Device featurization: the plan's namespace blocks -> the staged example CSR (interactions and the
  // constant expanded on the device). Then optionally the per-example label extras of the reductions:
  // csoaa (class, cost) lists, or the CB multi-line structure (rows of the plan = action rows).
  // learn_r1 > 0: rows [0, learn_r1) are also learned (batch examples per launch) while the pass stages -
  // the blocks go up in chunks on the copy stream and each chunk is expanded and learned as soon as it has
  // landed (LearnStaged(0, learn_r1, batch) after a plain StagePlan, without the serial upload before it)
  void StagePlan(const FeatPlan& plan, int64_t n, const float* labels, const float* weights, int64_t learn_r1 = 0,
                 int batch = 1);
  void StageCosts(const int64_t* cptr, const int32_t* cls, const float* cost, int64_t n);
  void StageCb(const int64_t* aip, const int32_t* chosen, const float* cost, const float* prob, int64_t n_examples);
  // CATS labels of the staged rows (action, cost, logged pdf; has = 0: no label, prediction only)
  void StageCats(const float* action, const float* cost, const float* pdf, const uint8_t* has, int64_t n);
  // predictions of every staged row (scalar: clamped score; oaa / csoaa: 1-based class; cb: action scores,
  // plus the greedy action per example in *best)
  void PredictStaged(float* out, float* best);
  int64_t staged_rows() const { return staged_rows_; }
  int64_t staged_examples() const { return staged_n_; }
  void CbStats(double* ips_num, double* snips_den, double* examples) const;
  // weighted average over ranks of the blocks touched since the last sync (RCCL on the learner's stream)
  // timeout_ms > 0 bounds each collective's settling (a dead peer): past it the call throws
  void AllReduceAverage(void* nccl_comm_handle, int world, double timeout_ms = 0);
  uint64_t NumWeights() const;
  // the table's nonzero components as (stride-4 index, value) - the host model format's records
  void ExportNonzeros(std::vector<uint64_t>* idx, std::vector<float>* val) const;
  // the same records in the host model's byte layout: CountNonzeros() sizes the export, WriteRecords(dst)
  // fills 12 * count bytes at dst (u64 stride-4 index + f32 value each, slot order)
  int64_t CountNonzeros() const;
  void WriteRecords(char* dst) const;
  // final export (a fit's last use of the learner): WriteRecords also zeroes every exported component in place,
  // so at destruction the table goes to the process's clean-table cache and the next learner of that size
  // skips its 16 GiB memset (2^30); the learner refuses further learning / import / syncs afterwards
  void SetFinalExport(bool on) { final_export_ = on; }
  bool retired() const { return retired_; }
  void ImportNonzeros(const std::vector<uint64_t>& idx, const std::vector<float>& val);
  void GlobalState(double* t, double* total_weight, double* sum_norm_x) const;
  void SetGlobalState(double t, double total_weight, double sum_norm_x);
  double examples() const { return examples_; }
  double sum_loss() const { return sum_loss_; }
  double min_label() const { return min_label_; }
  double max_label() const { return max_label_; }
  void SetLabelRange(double lo, double hi) { min_label_ = lo; max_label_ = hi; }
  int64_t last_sync_bytes() const { return last_sync_bytes_; }
  int64_t last_sync_blocks() const { return last_sync_blocks_; }
  void* weights_device();
  void* stream();

 private:
  void Launch(int64_t b0, int64_t b1, bool learn, bool have_weights);
  // end of the launch starting at row b0 of the range [r0, r1) being learned (warm-up sizes, then `batch`)
  int64_t NextLaunch(int64_t b0, int64_t r0, int64_t r1, int batch) const;
  struct Impl;
  std::unique_ptr<Impl> impl_;
  GpuSgdConfig cfg_;
  double examples_ = 0, sum_loss_ = 0;
  double min_label_ = 0, max_label_ = 0;
  int64_t last_sync_bytes_ = 0, last_sync_blocks_ = 0;
  std::vector<float> staged_labels_;
  bool clamp_const_ = false;  // the learning launches clamp to the fixed [min_label_, max_label_] (logistic)
  int64_t staged_n_ = 0;       // examples
  int64_t staged_rows_ = 0;    // CSR rows (= examples, or action rows under cb)
  bool staged_weights_ = false;
  bool staged_costs_ = false;
  int64_t max_actions_ = 0;
  std::vector<float> cats_cost_;   // staged CATS costs / label flags: the host builds each example's
  std::vector<uint8_t> cats_has_;  // control-variate baseline (a running mean over the labelled examples)
  double cats_cost_sum_ = 0, cats_cost_n_ = 0;
  mutable std::vector<int64_t> export_base_;  // per-4096-slot record offsets of the last CountNonzeros()
  mutable int64_t export_count_ = 0;
  mutable uint32_t* export_reg_ = nullptr;  // one-scan export: per-block record regions + counts (device)
  mutable int32_t* export_cnt_ = nullptr;
  bool final_export_ = false;
  mutable bool retired_ = false;
  void CheckLive() const;
  void ExpandToStage(const FeatPlan& plan, int64_t n, int64_t learn_r1 = 0, int batch = 1);
  // per-row clamp bounds + loss reset before learning rows [r0, r1); loss read-back (and predictions) after
  void PrepLearn(int64_t r0, int64_t r1);
  void FinishLearn(int64_t r0, int64_t r1, float* preds_out);
};

bool VwGpuAvailable();
// the pinned stager refuses a null source / destination (host-only; no HIP call is reached)
bool StagerRejectsNull();
// value pieces the shared stager sent as a device fill of 1.0f instead of their bytes (since process start)
int64_t StagerUnitPieces();
// K13: murmur3_32(bytes[offsets[i]:offsets[i+1]], seed) & mask for every i, on the device
void MurmurBatchGpu(const uint8_t* bytes, int64_t nbytes, const int64_t* offsets, int64_t n, uint32_t seed,
                    uint32_t mask, uint32_t* out);

}  // namespace smlvw
