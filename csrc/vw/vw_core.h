// Hashed online linear learning with Vowpal Wabbit semantics (native
// components N5/N7 of SURVEY.md §2.3). Replaces the reference's vw-jni
// (VowpalWabbitNative / VowpalWabbitExample / VowpalWabbitMurmur, called from
// vw/.../VowpalWabbitBaseSpark.scala:143-184, VowpalWabbitContextualBandit
// .scala:209-264, VowpalWabbitGeneric.scala:47,113).
//
// What is implemented: murmur3 feature hashing (VW's hashstring), the VW text
// example format, quadratic/cubic interactions, constant feature, the default
// adaptive + normalized + invariant ("safe") gradient update and the --sgd /
// --adaptive / --normalized / --invariant variants, l1/l2, power_t /
// initial_t, squared/logistic/hinge/quantile losses, --link logistic, the
// reductions used by the reference's tests (binary, --oaa [--probabilities],
// --csoaa, --cb_adf / --cb_explore_adf with epsilon-greedy and ips/mtr/dr),
// multi-pass replay, model averaging (endPass allreduce / mergeModels), a
// binary model format and --readable_model.
#pragma once
#include <array>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace smlvw {

uint32_t Murmur3(const void* key, size_t len, uint32_t seed);
// VW hashstring: all-digit strings hash to value + seed, others murmur3.
uint32_t HashString(const std::string& s, uint32_t seed);
uint32_t HashFeatureName(const std::string& s, uint32_t ns_hash);

constexpr uint32_t kConstantHash = 11650396u;
constexpr unsigned char kConstantNamespace = 128;
constexpr uint64_t kFnvPrime = 16777619u;

struct Feature {
  float x;
  uint64_t idx;
};

struct Namespace {
  unsigned char ns = ' ';
  std::vector<Feature> f;
};

struct Label {
  // CATS label "ca action:cost:pdf_value"
  bool cats_has = false;
  float cats_action = 0.f, cats_cost = 0.f, cats_pdf = 1.f;
  float label = 0.f;          // simple label (FLT_MAX = none)
  float weight = 1.f;         // importance
  float initial = 0.f;
  bool has_label = false;
  int multiclass = 0;         // 1-based (oaa)
  std::vector<std::pair<int, float>> costs;  // (class, cost) csoaa
  // contextual bandit (per action example): chosen action cost/prob
  bool cb_shared = false;
  bool cb_has = false;
  int cb_action = 0;
  float cb_cost = 0.f, cb_prob = 1.f;
};

struct Example {
  std::vector<Namespace> ns;
  Label l;
  std::string tag;
  // predictions
  float pred = 0.f;
  std::vector<float> scores;                // oaa/csoaa/cb scores
  std::vector<std::pair<int, float>> action_probs;  // cb_explore: (action 0-based, prob)
  // CATS (continuous actions): the smoothed policy's density as (left, right, value) segments (--cats_pdf),
  // or a sampled action with its density (--cats)
  std::vector<std::array<float, 3>> pdf_segments;
  float cats_action = 0.f, cats_pdf_value = 0.f;
  float loss = 0.f;
  Namespace& Get(unsigned char c);
};

struct Stats {
  int64_t examples = 0;
  double weighted_examples = 0, weighted_labels = 0, sum_loss = 0;
  double total_features = 0;
  int64_t passes = 0;
  double min_label = 0, max_label = 0;
  // contextual bandit online estimates (ips/snips)
  double cb_ips_num = 0, cb_snips_den = 0;
};

class VW {
 public:
  explicit VW(const std::string& args, const std::string* model_bytes = nullptr);
  ~VW();
  // single-line examples
  void Learn(Example& ex);
  void Predict(Example& ex);
  // multi-line (ADF: shared example first if cb_shared)
  void LearnMulti(std::vector<Example>& exs);
  void PredictMulti(std::vector<Example>& exs);
  // text format
  Example ParseLine(const std::string& line) const;
  void EndPass();
  void PerformRemainingPasses();
  std::string SaveModel() const;
  std::string ReadableModel() const;
  const Stats& stats() const { return stats_; }
  Stats& mutable_stats() { return stats_; }
  const std::string& args() const { return args_str_; }
  std::string OutputPredictionType() const;
  uint64_t NumWeights() const { return weights_.size(); }
  float* weights() { return weights_.data(); }
  uint32_t stride() const { return stride_; }
  int num_bits() const { return bits_; }
  uint32_t HashSeed() const { return hash_seed_; }
  // model averaging: w = sum over models / n (mergeModels / endPass allreduce)
  static std::unique_ptr<VW> Merge(const std::vector<const VW*>& models);
  // parse and validate a command line without allocating the weight table (GPU learner set-up)
  static std::map<std::string, std::string> DescribeArgs(const std::string& args);
  // parse text examples with a command line's hashing / ngram settings, without a weight table (the GPU
  // learner's text ingest)
  static std::vector<Example> ParseLines(const std::string& args, const std::vector<std::string>& lines);
  void SetAllReduce(std::function<void(float*, size_t)> fn) { allreduce_ = std::move(fn); }
  int world_size = 1;

 private:
  VW() = default;  // DescribeArgs: parse only
  void ParseArgs(const std::string& args);
  void LoadModel(const std::string& bytes);
  // linear core over (interaction-expanded) features of one example with a
  // learner offset (oaa class / csoaa class).
  float Dot(const Example& ex, uint64_t offset) const;
  void Update(const Example& ex, uint64_t offset, float pred, float label, float importance);
  template <class F> void ForEachFeature(const Example& ex, F&& fn) const;
  float Loss(float pred, float label) const;
  float FirstDeriv(float pred, float label) const;
  float FinalizePred(float raw) const;
  void CbLearn(std::vector<Example>& exs, bool learn);
  // CATS: continuous actions over [min_value, max_value] discretised into cats_k_ centroids, a binary tree of
  // linear node scorers picks one, the policy is that centroid's bandwidth window (prob 1 - epsilon) plus a
  // uniform epsilon over the range
  int CatsPredictLeaf(const Example& ex) const;
  void CatsSegments(int leaf, Example* ex) const;
  void CatsLearn(Example& ex);
  uint64_t CatsNodeOffset(int node) const { return static_cast<uint64_t>(node + 1) * 2654435761ull; }

  std::string args_str_;
  int bits_ = 18;
  uint64_t mask_ = 0;
  uint32_t stride_ = 4;   // w, adaptive G, normalizer N, spare
  uint32_t hash_seed_ = 0;
  float lr_ = 0.5f, power_t_ = 0.5f, initial_t_ = 0.f, l1_ = 0.f, l2_ = 0.f;
  bool adaptive_ = true, normalized_ = true, invariant_ = true;
  bool constant_ = true;
  std::string loss_ = "squared";
  float quantile_tau_ = 0.5f;
  bool link_logistic_ = false;
  std::vector<std::string> interactions_;
  std::vector<unsigned char> ignore_;
  int oaa_ = 0, csoaa_ = 0;
  bool probabilities_ = false;
  bool cb_adf_ = false, cb_explore_ = false;
  std::string cb_type_ = "mtr";
  float epsilon_ = 0.05f;
  int passes_ = 1;
  bool testonly_ = false;
  bool holdout_off_ = true;
  int ngram_ = 0;
  std::array<int, 256> ngram_ns_{};  // per-namespace "--ngram aN"
  int cats_k_ = 0;             // --cats_pdf K / --cats K: discrete centroids
  bool cats_sample_ = false;   // --cats: emit a sampled action (action_pdf_value) instead of the pdf
  float bandwidth_ = -1.f, min_value_ = 0.f, max_value_ = -1.f;
  bool epsilon_set_ = false;
  int cats_depth_ = 0;
  uint64_t cats_draws_ = 0;
  double cats_cost_sum_ = 0, cats_cost_n_ = 0;  // control-variate baseline of the CATS cost estimates
  std::vector<float> weights_;
  double t_ = 0;                    // weighted examples seen (power_t schedule)
  double total_weight_ = 0, sum_norm_x_ = 0;
  Stats stats_;
  std::vector<Example> cache_;      // multi-pass replay
  std::vector<std::vector<Example>> cache_multi_;
  bool caching_ = false;
  std::function<void(float*, size_t)> allreduce_;
  mutable std::vector<float> spare_;  // per-feature rate decay scratch
};

}  // namespace smlvw
