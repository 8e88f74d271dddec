#include "booster.h"
#include "valid_gpu.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <map>
#include <numeric>
#include <sstream>
#include <stdexcept>

namespace sml {

namespace {
// Re-express a tree loaded from text (real thresholds) in the bin space of `ref`
// so it can update binned training scores (continued training / merge).
void MapTreeToBins(Tree* t, const DatasetReference& ref) {
  for (int node = 0; node < t->num_leaves - 1; ++node) {
    int f = t->split_feature[node];
    int inner = (f >= 0 && f < static_cast<int>(ref.real_to_inner.size())) ? ref.real_to_inner[f] : -1;
    t->split_feature_inner[node] = inner < 0 ? 0 : inner;
    if (inner < 0) continue;
    const BinMapper& m = ref.mappers[f];
    if (t->decision_type[node] & 1) {
      // categorical: bin bitset from value bitset
      int ci = static_cast<int>(t->threshold[node]);
      std::vector<uint32_t> bb(8, 0);
      for (int b = 0; b < static_cast<int>(m.bin2cat.size()); ++b) {
        int c = m.bin2cat[b];
        int s = t->cat_boundaries[ci], e = t->cat_boundaries[ci + 1];
        if (c / 32 < e - s && ((t->cat_threshold[s + c / 32] >> (c % 32)) & 1u)) bb[b / 32] |= 1u << (b % 32);
      }
      t->threshold_in_bin[node] = static_cast<uint32_t>(t->cat_boundaries_inner.size() - 1);
      t->cat_threshold_inner.insert(t->cat_threshold_inner.end(), bb.begin(), bb.end());
      t->cat_boundaries_inner.push_back(static_cast<int>(t->cat_threshold_inner.size()));
    } else {
      double v = t->threshold[node];
      uint32_t tb = 0;
      const int nb = static_cast<int>(m.upper_bounds.size());
      // largest bin whose upper bound <= v  (bin <= tb  <=>  value <= v)
      int lo = -1;
      for (int b = 0; b < nb; ++b) if (m.upper_bounds[b] <= v + 1e-12 * std::fabs(v)) lo = b;
      tb = lo < 0 ? 0 : static_cast<uint32_t>(lo);
      if (lo < 0) {
        // every value is > v: make the comparison always false except missing
        tb = 0;
      }
      t->threshold_in_bin[node] = tb;
    }
  }
}

std::unique_ptr<Objective> MakeConverter(const std::string& objective_str) {
  Config c = Config::Parse("objective=" + objective_str.substr(0, objective_str.find(' ')));
  std::stringstream ss(objective_str);
  std::string tok;
  ss >> tok;
  while (ss >> tok) {
    auto colon = tok.find(':');
    if (colon != std::string::npos) c.Set(tok.substr(0, colon), tok.substr(colon + 1));
  }
  if (c.objective == "custom" || c.objective == "none" || c.objective == "lambdarank") c.objective = "regression";
  return std::unique_ptr<Objective>(new Objective(c));
}

std::string Trim(const std::string& s) {
  size_t b = s.find_first_not_of(" \t\r\n");
  if (b == std::string::npos) return "";
  size_t e = s.find_last_not_of(" \t\r\n");
  return s.substr(b, e - b + 1);
}
}  // namespace

Booster::Booster(std::shared_ptr<Dataset> train, const std::string& params, Comm* comm)
    : train_(std::move(train)), comm_(comm) {
  params_str_ = params;
  cfg_ = Config::Parse(params);
  InitTraining();
}

void Booster::InitTraining() {
  // SML_GBDT_INIT_TIMING=1: the phases of the booster construction on stderr (profiling runs)
  const bool timing = std::getenv("SML_GBDT_INIT_TIMING") != nullptr;
  auto tick = std::chrono::steady_clock::now();
  auto mark = [&](const char* what) {
    if (!timing) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[booster init] %-22s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(now - tick).count());
    tick = now;
  };
  train_->FinalizeLabel();
  objective_.reset(new Objective(cfg_));
  objective_->Init(*train_);
  mark("objective init");
  num_tree_per_iter_ = objective_->NumModelPerIteration();
  num_class_ = cfg_.IsClassification() && cfg_.objective != "binary" ? cfg_.num_class : 1;
  objective_str_ = objective_->ToString();
  max_feature_idx_ = train_->ref.num_total_features - 1;
  feature_names_ = train_->ref.feature_names;
  feature_infos_.clear();
  for (const auto& m : train_->ref.mappers) feature_infos_.push_back(m.FeatureInfo());
  average_output_ = cfg_.boosting == "rf";
  bool want_gpu = cfg_.device_type == "gpu" || cfg_.device_type == "cuda" || cfg_.device_type == "rocm";
  if (want_gpu && GpuAvailable()) backend_ = MakeGpuBackend(cfg_.gpu_device_id);
  if (!backend_) backend_ = MakeCpuBackend();
  if (comm_) backend_->SetComm(comm_);
  mark("backend create");
  backend_->Init(train_.get(), cfg_, num_tree_per_iter_);
  mark("backend init");
  const int64_t n = train_->num_data;
  const int K = num_tree_per_iter_;
  init_scores_.assign(K, 0.0);
  if (!train_->init_score.empty()) {
    if (static_cast<int64_t>(train_->init_score.size()) != n * K)
      throw std::runtime_error("init_score has wrong size");
    backend_->SetScores(train_->init_score);
  } else {
    if (cfg_.boost_from_average && objective_->params().kind != kObjLambdarank &&
        objective_->params().kind != kObjCustom) {
      for (int k = 0; k < K; ++k) {
        init_scores_[k] = objective_->BoostFromScore(k, comm_);
      }
    }
    mark("boost from score");
    backend_->FillScores(init_scores_, n);  // constant start scores, written where the scores live
    mark("fill scores");
  }
  bag_rng_.seed(cfg_.bagging_seed);
  feat_rng_.seed(cfg_.feature_fraction_seed);
  drop_rng_.seed(cfg_.drop_seed);
  iter_ = 0;
}

void Booster::AddValidData(std::shared_ptr<Dataset> valid, const std::string& name) {
  const int K = num_tree_per_iter_;
  valid->FinalizeLabel();
  std::vector<double> s(static_cast<size_t>(valid->num_data) * K, 0.0);
  if (!valid->init_score.empty()) s = valid->init_score;
  else for (int k = 0; k < K; ++k) for (int64_t i = 0; i < valid->num_data; ++i) s[k * valid->num_data + i] += (trees_.empty() ? init_scores_[k] : 0.0);
  const size_t vi = valid_.size();
  // K11: with a device backend the set's bins and scores stay in HBM (no host bins needed)
  const bool on_dev = backend_ && backend_->AddValidSet(static_cast<int>(vi), *valid, s, cfg_);
  if (!on_dev) valid->EnsureHostBins();
  std::unique_ptr<Objective> vo(new Objective(cfg_));
  vo->Init(*valid);
  valid_objectives_.push_back(std::move(vo));
  valid_.push_back(std::move(valid));
  valid_names_.push_back(name);
  valid_dev_.push_back(on_dev ? 1 : 0);
  valid_scores_.push_back(on_dev ? std::vector<double>() : std::move(s));
  // existing trees
  for (size_t t = 0; t < trees_.size(); ++t) ValidApply(vi, trees_[t], static_cast<int>(t % K), kValidAdd, 1.0);
}

void Booster::ValidApply(size_t vi, const Tree& t, int k, int op, double p) {
  if (valid_dev_[vi]) {
    backend_->ValidApplyTree(static_cast<int>(vi), t, k, op, p);
    return;
  }
  auto& vd = valid_[vi];
  double* vs = valid_scores_[vi].data() + static_cast<size_t>(k) * vd->num_data;
  if (op == kValidConst) {
    for (int64_t i = 0; i < vd->num_data; ++i) vs[i] = ValidFold(vs[i], 0.0, op, p);
    return;
  }
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < vd->num_data; ++i) {
    const double o = t.leaf_value[t.GetLeafByBins(&vd->bins[i * vd->row_stride], vd->ref.mappers, vd->ref.used_features)];
    vs[i] = ValidFold(vs[i], o, op, p);
  }
}

void Booster::MergeFrom(const Booster& other) {
  if (!train_) { trees_.insert(trees_.begin(), other.trees_.begin(), other.trees_.end()); return; }
  const int K = num_tree_per_iter_;
  if (other.num_tree_per_iter_ != K) throw std::runtime_error("cannot merge models with different class counts");
  // Continued training: remove the boost-from-average offset, add the old trees.
  for (int k = 0; k < K; ++k) if (init_scores_[k] != 0.0) backend_->AddBias(k, -init_scores_[k]);
  for (size_t vi = 0; vi < valid_.size(); ++vi)
    for (int k = 0; k < K; ++k) ValidApply(vi, Tree(), k, kValidConst, -init_scores_[k]);
  init_scores_.assign(K, 0.0);
  std::vector<Tree> old = other.trees_;
  for (size_t t = 0; t < old.size(); ++t) {
    MapTreeToBins(&old[t], train_->ref);
    const int k = static_cast<int>(t % K);
    const double scale = other.average_output_ ? 1.0 / std::max(1, other.CurrentIteration()) : 1.0;
    backend_->UpdateScore(old[t], k, scale);
    for (size_t vi = 0; vi < valid_.size(); ++vi) ValidApply(vi, old[t], k, kValidAdd, scale);
  }
  trees_.insert(trees_.begin(), old.begin(), old.end());
  boosted_first_ = true;
}

void Booster::ResetParameter(const std::string& params) {
  std::stringstream ss(params);
  std::string tok;
  while (ss >> tok) {
    auto eq = tok.find('=');
    if (eq == std::string::npos) continue;
    cfg_.Set(tok.substr(0, eq), tok.substr(eq + 1));
  }
}

void Booster::Bagging(int iter) {
  const int64_t n = train_->num_data;
  const bool balanced = cfg_.pos_bagging_fraction < 1.0 || cfg_.neg_bagging_fraction < 1.0;
  const bool need = cfg_.bagging_freq > 0 && (cfg_.bagging_fraction < 1.0 || balanced);
  if (!need) { if (bagged_) { backend_->SetBag(nullptr); bagged_ = false; } return; }
  if (iter % cfg_.bagging_freq != 0) return;
  RowSampleSpec spec;
  spec.kind = kSampleBagging;
  spec.seed = static_cast<uint64_t>(cfg_.bagging_seed);
  spec.iter = iter;
  spec.fraction = cfg_.bagging_fraction;
  spec.pos_fraction = cfg_.pos_bagging_fraction;
  spec.neg_fraction = cfg_.neg_bagging_fraction;
  spec.balanced = balanced;
  // leaf renewal (l1 / quantile / mape) needs the bag on the host
  if (!objective_->NeedRenewTreeOutput() && backend_->SampleRows(spec)) {
    bag_rows_.clear();
    bagged_ = true;
    return;
  }
  bag_rows_.clear();
  bag_rows_.reserve(static_cast<size_t>(n * cfg_.bagging_fraction) + 16);
  for (int64_t i = 0; i < n; ++i) {
    double frac = cfg_.bagging_fraction;
    if (balanced) frac = train_->label[i] > 0 ? cfg_.pos_bagging_fraction : cfg_.neg_bagging_fraction;
    if (RowUniform(spec.seed, iter, i) < frac) bag_rows_.push_back(static_cast<int32_t>(i));
  }
  backend_->SetBag(&bag_rows_);
  bagged_ = true;
}

void Booster::Goss() {
  const int K = num_tree_per_iter_;
  const int64_t n = train_->num_data;
  RowSampleSpec spec;
  spec.kind = kSampleGoss;
  spec.seed = static_cast<uint64_t>(cfg_.bagging_seed);
  spec.iter = iter_;
  spec.top_k = std::max<int64_t>(1, static_cast<int64_t>(n * cfg_.top_rate));
  const int64_t other_k = std::max<int64_t>(1, static_cast<int64_t>(n * cfg_.other_rate));
  spec.other_mult = static_cast<double>(n - spec.top_k) / other_k;
  spec.other_prob = static_cast<double>(other_k) / std::max<int64_t>(1, n - spec.top_k);
  if (!objective_->NeedRenewTreeOutput() && backend_->SampleRows(spec)) {
    bag_rows_.clear();
    bagged_ = true;
    return;
  }
  std::vector<float> g, h;
  backend_->GetGradients(&g, &h);
  // |g*h| summed over classes in float: the device computes the same value
  std::vector<float> a(n, 0.f);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    float s = 0.f;
    for (int k = 0; k < K; ++k) s += std::fabs(g[k * n + i] * h[k * n + i]);
    a[i] = s;
  }
  std::vector<float> tmp = a;
  std::nth_element(tmp.begin(), tmp.begin() + (spec.top_k - 1), tmp.end(), std::greater<float>());
  const float thr = tmp[spec.top_k - 1];
  const float mult = static_cast<float>(spec.other_mult);
  bag_rows_.clear();
  for (int64_t i = 0; i < n; ++i) {
    if (a[i] >= thr) { bag_rows_.push_back(static_cast<int32_t>(i)); continue; }
    if (RowUniform(spec.seed, iter_, i) < spec.other_prob) {
      bag_rows_.push_back(static_cast<int32_t>(i));
      for (int k = 0; k < K; ++k) { g[k * n + i] *= mult; h[k * n + i] *= mult; }
    }
  }
  backend_->SetGradients(g.data(), h.data());
  backend_->SetBag(&bag_rows_);
  bagged_ = true;
}

std::vector<char> Booster::SampleFeatures() {
  const int F = train_->ref.num_inner();
  std::vector<char> m(F, 1);
  if (cfg_.feature_fraction >= 1.0 || F == 0) return m;
  int keep = std::max(1, static_cast<int>(std::ceil(F * cfg_.feature_fraction - 1e-9)));
  std::vector<int> idx(F);
  std::iota(idx.begin(), idx.end(), 0);
  std::shuffle(idx.begin(), idx.end(), feat_rng_);
  std::fill(m.begin(), m.end(), 0);
  for (int i = 0; i < keep; ++i) m[idx[i]] = 1;
  return m;
}

bool Booster::TrainOneIter(const float* grad, const float* hess) {
  if (!train_) throw std::runtime_error("booster has no training data");
  const int K = num_tree_per_iter_;
  const int64_t n = train_->num_data;
  const bool is_rf = cfg_.boosting == "rf";
  const bool is_dart = cfg_.boosting == "dart";
  const bool is_goss = cfg_.boosting == "goss";
  // ---- DART: drop trees before computing gradients
  std::vector<int> drop_iters;
  if (is_dart && CurrentIteration() > 0) {
    std::uniform_real_distribution<double> U(0.0, 1.0);
    if (U(drop_rng_) >= cfg_.skip_drop) {
      const int ni = CurrentIteration();
      for (int i = 0; i < ni; ++i) if (U(drop_rng_) < cfg_.drop_rate) drop_iters.push_back(i);
      if (drop_iters.empty() && ni > 0) drop_iters.push_back(std::uniform_int_distribution<int>(0, ni - 1)(drop_rng_));
      std::shuffle(drop_iters.begin(), drop_iters.end(), drop_rng_);
      if (cfg_.max_drop > 0 && static_cast<int>(drop_iters.size()) > cfg_.max_drop) drop_iters.resize(cfg_.max_drop);
      std::sort(drop_iters.begin(), drop_iters.end());
      for (int it : drop_iters) for (int k = 0; k < K; ++k) backend_->UpdateScore(trees_[it * K + k], k, -1.0);
    }
  }
  // ---- gradients
  if (grad && hess) {
    backend_->SetGradients(grad, hess);
  } else if (!is_rf || iter_ == 0) {
    backend_->ComputeGradients(*objective_);
  }
  // ---- row sampling
  if (is_goss && iter_ >= static_cast<int>(1.0 / cfg_.learning_rate)) {
    Goss();
  } else if (!is_goss) {
    Bagging(iter_);
  }
  // ---- grow one tree per class
  bool any_split = false;
  std::vector<Tree> new_trees;
  // plain boosting: the backend may apply the shrunk tree to the scores right behind its growth
  const bool device_update = !is_rf && !is_dart && !objective_->NeedRenewTreeOutput();
  std::vector<char> updated(K, 0);
  for (int k = 0; k < K; ++k) {
    std::vector<char> fmask = SampleFeatures();
    bool upd = false;
    Tree t = device_update ? backend_->TrainTreeAndUpdateScore(k, fmask, cfg_.learning_rate, &upd)
                           : backend_->TrainTree(k, fmask);
    updated[k] = upd ? 1 : 0;
    if (t.num_leaves > 1) {
      any_split = true;
      if (objective_->NeedRenewTreeOutput()) {
        std::vector<int32_t> leaf;
        backend_->PredictLeafIndex(t, &leaf);
        std::vector<double> sc;
        backend_->GetScores(&sc);
        std::vector<std::vector<int64_t>> rows(t.num_leaves);
        if (bagged_) { for (int32_t r : bag_rows_) rows[leaf[r]].push_back(r); }
        else for (int64_t i = 0; i < n; ++i) rows[leaf[i]].push_back(i);
        for (int l = 0; l < t.num_leaves; ++l)
          if (!rows[l].empty()) t.leaf_value[l] = objective_->RenewLeafOutput(sc.data() + k * n, rows[l].data(), static_cast<int64_t>(rows[l].size()));
      }
      double shrink = cfg_.learning_rate;
      if (is_rf) shrink = 1.0;
      if (is_dart) {
        const double nd = static_cast<double>(drop_iters.size());
        shrink = cfg_.xgboost_dart_mode ? cfg_.learning_rate / (cfg_.learning_rate + nd) : cfg_.learning_rate / (1.0 + nd);
      }
      t.Shrink(shrink);
    } else {
      // constant tree (LightGBM keeps the init score in it on the first iteration)
      t.leaf_value[0] = 0.0;
    }
    new_trees.push_back(std::move(t));
  }
  if (!any_split && CurrentIteration() > 0) {
    // undo DART drops
    for (int it : drop_iters) for (int k = 0; k < K; ++k) backend_->UpdateScore(trees_[it * K + k], k, 1.0);
    return true;
  }
  for (int k = 0; k < K; ++k) {
    Tree& t = new_trees[k];
    if (is_rf) {
      // running average of tree outputs: score = (score*c + tree)/(c+1), trees carry the init bias
      const double c = static_cast<double>(CurrentIteration());
      t.AddBias(init_scores_[k]);
      backend_->ScaleScore(k, c / (c + 1.0));
      backend_->UpdateScore(t, k, 1.0 / (c + 1.0));
    } else {
      if (!updated[k]) backend_->UpdateScore(t, k, 1.0);
      if (!boosted_first_ && CurrentIteration() == 0) t.AddBias(init_scores_[k]);
    }
  }
  // DART: normalise dropped trees
  if (is_dart && !drop_iters.empty()) {
    const double nd = static_cast<double>(drop_iters.size());
    const double factor = cfg_.xgboost_dart_mode ? nd / (nd + cfg_.learning_rate) : nd / (nd + 1.0);
    for (int it : drop_iters) {
      for (int k = 0; k < K; ++k) {
        Tree& old = trees_[it * K + k];
        old.Shrink(factor);
        backend_->UpdateScore(old, k, 1.0);
        // valid scores: old contribution was unscaled; remove (1-factor) of it
        for (size_t vi = 0; vi < valid_.size(); ++vi) ValidApply(vi, old, k, kValidDart, factor);
      }
    }
  }
  // validation scores
  const int citer = CurrentIteration();
  for (size_t vi = 0; vi < valid_.size(); ++vi) {
    for (int k = 0; k < K; ++k) {
      const Tree& t = new_trees[k];
      if (is_rf) {
        ValidApply(vi, t, k, kValidRfAvg, static_cast<double>(citer));
      } else {
        const bool first_bias = !boosted_first_ && citer == 0;  // valid scores already carry the init bias
        ValidApply(vi, t, k, kValidAddSub, first_bias ? init_scores_[k] : 0.0);
      }
    }
  }
  for (auto& t : new_trees) trees_.push_back(std::move(t));
  ++iter_;
  backend_->stats.trees += K;
  return false;
}

void Booster::RollbackOneIter() {
  const int K = num_tree_per_iter_;
  if (static_cast<int>(trees_.size()) < K) return;
  for (int k = K - 1; k >= 0; --k) {
    Tree& t = trees_[trees_.size() - K + k];
    if (train_) backend_->UpdateScore(t, k, -1.0);
  }
  trees_.resize(trees_.size() - K);
  --iter_;
}

void Booster::ReleaseTraining() { DetachTraining()->Free(); }

std::unique_ptr<DetachedTraining> Booster::DetachTraining() {
  auto d = std::make_unique<DetachedTraining>();
  if (train_) loaded_parameters_ = cfg_.ToParametersSection();  // the model text's parameters section
  if (backend_) released_backend_ = backend_->Name();
  d->backend = std::move(backend_);
  d->train = std::move(train_);
  d->valid = std::move(valid_);
  d->valid_objectives = std::move(valid_objectives_);
  d->valid_scores = std::move(valid_scores_);
  backend_.reset();
  train_.reset();
  valid_.clear();
  valid_objectives_.clear();
  valid_scores_.clear();
  valid_dev_.clear();
  bag_rows_.clear();
  bag_rows_.shrink_to_fit();
  released_ = true;
  return d;
}

void Booster::Truncate(int num_iteration) {
  const size_t keep = static_cast<size_t>(std::max(0, num_iteration)) * num_tree_per_iter_;
  if (keep < trees_.size()) trees_.resize(keep);
}

std::vector<std::string> Booster::EvalNames() const {
  std::vector<std::string> names;
  auto ms = cfg_.Metrics();
  if (ms.empty() && objective_) ms.push_back(objective_->DefaultMetric());
  for (auto& m : ms) {
    if (m == "None" || m == "none" || m == "null" || m == "na" || m.empty()) continue;
    std::string mm = m;
    if (mm == "binary") mm = "binary_logloss";
    if (mm == "multiclass" || mm == "softmax") mm = "multi_logloss";
    if (mm == "regression" || mm == "mean_squared_error" || mm == "mse" || mm == "regression_l2") mm = "l2";
    if (mm == "regression_l1" || mm == "mean_absolute_error" || mm == "mae") mm = "l1";
    if (mm == "root_mean_squared_error" || mm == "l2_root") mm = "rmse";
    if (mm == "lambdarank") mm = "ndcg";
    if ((mm == "ndcg" || mm == "map") && mm.find('@') == std::string::npos) {
      for (int k : cfg_.eval_at) names.push_back(mm + "@" + std::to_string(k));
    } else {
      names.push_back(mm);
    }
  }
  return names;
}

std::vector<std::pair<std::string, double>> Booster::Eval(int idx, bool device) {
  Backend();  // raises once the training state was released
  std::vector<std::pair<std::string, double>> out;
  const Dataset* d;
  const Objective* obj;
  std::vector<double> train_scores;
  const double* scores;
  if (idx == 0) {
    d = train_.get(); obj = objective_.get();
    scores = nullptr;  // fetched from the backend only if a metric has no device implementation
  } else {
    d = valid_[idx - 1].get(); obj = valid_objectives_[idx - 1].get();
    scores = valid_dev_[idx - 1] ? nullptr : valid_scores_[idx - 1].data();
  }
  for (const auto& name : EvalNames()) {
    double dv = 0.0;
    const bool on_dev = device && (idx == 0 ? backend_->EvalOnDevice(name, *obj, &dv)
                                            : valid_dev_[idx - 1] && backend_->EvalValidOnDevice(idx - 1, name, *obj, &dv));
    if (on_dev) {
      out.emplace_back(name, dv);
      continue;
    }
    if (!scores) {  // a metric without a device implementation: one score copy for the remaining metrics
      if (idx == 0) backend_->GetScores(&train_scores);
      else backend_->GetValidScores(idx - 1, &train_scores);
      scores = train_scores.data();
    }
    double v = EvalMetric(name, *obj, scores, d->label.data(), d->weight.empty() ? nullptr : d->weight.data(),
                          d->num_data, num_class_, d->query_boundaries, cfg_.label_gain);
    out.emplace_back(name, v);
  }
  return out;
}

void Booster::GetTrainScores(std::vector<double>* s) { Backend()->GetScores(s); }
void Booster::GetPredictForValid(int idx, std::vector<double>* s) const {
  if (valid_dev_.at(idx)) backend_->GetValidScores(idx, s);
  else *s = valid_scores_.at(idx);
}

std::pair<int, int> Booster::TreeRange(int start_iteration, int num_iteration) const {
  const int K = num_tree_per_iter_;
  const int total_iter = static_cast<int>(trees_.size()) / K;
  int s = std::max(0, std::min(start_iteration, total_iter));
  int e = num_iteration > 0 ? std::min(total_iter, s + num_iteration) : total_iter;
  return {s * K, e * K};
}

void Booster::PredictRaw(const double* x, int st, int et, double* out) const {
  const int K = num_tree_per_iter_;
  for (int k = 0; k < K; ++k) out[k] = 0.0;
  for (int t = st; t < et; ++t) out[t % K] += trees_[t].Predict(x);
  if (average_output_ && et > st) {
    const int ni = (et - st) / K;
    for (int k = 0; k < K; ++k) out[k] /= ni;
  }
}

int Booster::PredictOutputSize(int type, int start_iteration, int num_iteration) const {
  auto r = TreeRange(start_iteration, num_iteration);
  if (type == kPredictLeaf) return r.second - r.first;
  if (type == kPredictContrib) return (max_feature_idx_ + 2) * num_tree_per_iter_;
  return num_tree_per_iter_;
}

void Booster::Predict(const double* X, int64_t nrows, int ncols, int type, int start_iteration,
                      int num_iteration, double* out) const {
  auto r = TreeRange(start_iteration, num_iteration);
  const int K = num_tree_per_iter_;
  const int nf = max_feature_idx_ + 1;
  const int osz = PredictOutputSize(type, start_iteration, num_iteration);
  std::unique_ptr<Objective> conv;
  if (type == kPredictNormal) conv = MakeConverter(objective_str_);
  // small batches (serving) stay on the calling thread: waking an OpenMP team
  // costs more than scoring a handful of rows
#pragma omp parallel if (nrows * (r.second - r.first) >= 4096)
  {
    std::vector<double> row(std::max(nf, ncols) + 1, 0.0), raw(K);
#pragma omp for schedule(static)
    for (int64_t i = 0; i < nrows; ++i) {
      std::fill(row.begin(), row.end(), 0.0);
      std::memcpy(row.data(), X + i * ncols, sizeof(double) * std::min(ncols, static_cast<int>(row.size())));
      double* o = out + i * osz;
      if (type == kPredictLeaf) {
        for (int t = r.first; t < r.second; ++t) o[t - r.first] = trees_[t].GetLeaf(row.data());
      } else if (type == kPredictContrib) {
        std::fill(o, o + osz, 0.0);
        for (int t = r.first; t < r.second; ++t) trees_[t].TreeSHAP(row.data(), o + (t % K) * (nf + 1), nf);
        if (average_output_ && r.second > r.first) {
          const int ni = (r.second - r.first) / K;
          for (int j = 0; j < osz; ++j) o[j] /= ni;
        }
      } else {
        PredictRaw(row.data(), r.first, r.second, raw.data());
        if (type == kPredictNormal) conv->ConvertOutput(raw.data(), o);
        else for (int k = 0; k < K; ++k) o[k] = raw[k];
      }
    }
  }
}

void Booster::ConvertOutputs(const double* raw, int64_t n, double* out) const {
  auto conv = MakeConverter(objective_str_);
  const int K = num_tree_per_iter_;
#pragma omp parallel for schedule(static) if (n >= 16384)
  for (int64_t i = 0; i < n; ++i) conv->ConvertOutput(raw + i * K, out + i * K);
}

std::vector<double> Booster::FeatureImportance(int num_iteration, int importance_type) const {
  std::vector<double> imp(max_feature_idx_ + 1, 0.0);
  auto r = TreeRange(0, num_iteration);
  for (int t = r.first; t < r.second; ++t) {
    const Tree& tr = trees_[t];
    for (int node = 0; node < tr.num_leaves - 1; ++node) {
      if (tr.split_gain[node] <= 0 && importance_type == 1) continue;
      int f = tr.split_feature[node];
      if (f < 0 || f > max_feature_idx_) continue;
      imp[f] += importance_type == 0 ? 1.0 : tr.split_gain[node];
    }
  }
  return imp;
}

std::string Booster::SaveModelToString(int start_iteration, int num_iteration, int importance_type) const {
  std::ostringstream o;
  o << "tree\n";
  o << "version=v3\n";
  o << "num_class=" << num_class_ << "\n";
  o << "num_tree_per_iteration=" << num_tree_per_iter_ << "\n";
  o << "label_index=" << label_index_ << "\n";
  o << "max_feature_idx=" << max_feature_idx_ << "\n";
  o << "objective=" << objective_str_ << "\n";
  if (average_output_) o << "average_output\n";
  o << "feature_names=";
  for (size_t i = 0; i < feature_names_.size(); ++i) o << (i ? " " : "") << feature_names_[i];
  o << "\nfeature_infos=";
  for (size_t i = 0; i < feature_infos_.size(); ++i) o << (i ? " " : "") << feature_infos_[i];
  o << "\n";
  auto r = TreeRange(start_iteration, num_iteration);
  // the trees' text blocks are independent: one per thread (a 100-tree model took ~5 ms serially, inside
  // every timed fit that returns the model text)
  std::vector<std::string> blocks(static_cast<size_t>(std::max(0, r.second - r.first)));
#pragma omp parallel for schedule(dynamic, 4) if (blocks.size() > 8)
  for (int t = r.first; t < r.second; ++t) blocks[t - r.first] = trees_[t].ToString(t - r.first);
  o << "tree_sizes=";
  for (size_t i = 0; i < blocks.size(); ++i) o << (i ? " " : "") << blocks[i].size();
  o << "\n\n";
  for (auto& b : blocks) o << b;
  o << "end of trees\n\n";
  auto imp = FeatureImportance(num_iteration > 0 ? r.second / num_tree_per_iter_ : 0, importance_type);
  std::vector<std::pair<double, int>> pairs;
  for (size_t i = 0; i < imp.size(); ++i) if (imp[i] > 0) pairs.emplace_back(imp[i], static_cast<int>(i));
  std::stable_sort(pairs.begin(), pairs.end(), [](auto& a, auto& b) { return a.first > b.first; });
  o << "feature_importances:\n";
  for (auto& p : pairs) {
    o << (p.second < static_cast<int>(feature_names_.size()) ? feature_names_[p.second] : "Column_" + std::to_string(p.second))
      << "=";
    if (importance_type == 0) o << static_cast<long long>(p.first); else o << p.first;
    o << "\n";
  }
  o << "\nparameters:\n";
  o << (train_ ? cfg_.ToParametersSection() : loaded_parameters_);
  o << "end of parameters\n\npandas_categorical:null\n";
  return o.str();
}

std::string Booster::DumpModel(int start_iteration, int num_iteration) const {
  std::ostringstream o;
  o << "{\"name\":\"tree\",\"version\":\"v3\",\"num_class\":" << num_class_
    << ",\"num_tree_per_iteration\":" << num_tree_per_iter_ << ",\"label_index\":" << label_index_
    << ",\"max_feature_idx\":" << max_feature_idx_ << ",\"objective\":\"" << objective_str_ << "\""
    << ",\"average_output\":" << (average_output_ ? "true" : "false") << ",\"feature_names\":[";
  for (size_t i = 0; i < feature_names_.size(); ++i) o << (i ? "," : "") << "\"" << feature_names_[i] << "\"";
  o << "],\"tree_info\":[";
  auto r = TreeRange(start_iteration, num_iteration);
  for (int t = r.first; t < r.second; ++t) o << (t > r.first ? "," : "") << trees_[t].ToJSON(t - r.first);
  o << "]}";
  return o.str();
}

std::unique_ptr<Booster> Booster::FromModelString(const std::string& model) {
  std::unique_ptr<Booster> b(new Booster());
  std::istringstream is(model);
  std::string line;
  std::map<std::string, std::string> header;
  // header until first Tree=
  std::vector<std::string> lines;
  while (std::getline(is, line)) lines.push_back(line);
  size_t i = 0;
  for (; i < lines.size(); ++i) {
    std::string l = Trim(lines[i]);
    if (l.rfind("Tree=", 0) == 0) break;
    if (l == "average_output") { b->average_output_ = true; continue; }
    auto eq = l.find('=');
    if (eq != std::string::npos) header[l.substr(0, eq)] = l.substr(eq + 1);
  }
  if (!header.count("num_tree_per_iteration") && !header.count("num_class"))
    throw std::runtime_error("model string is not a LightGBM text model");
  b->num_class_ = header.count("num_class") ? std::stoi(header["num_class"]) : 1;
  b->num_tree_per_iter_ = header.count("num_tree_per_iteration") ? std::stoi(header["num_tree_per_iteration"]) : b->num_class_;
  b->label_index_ = header.count("label_index") ? std::stoi(header["label_index"]) : 0;
  b->max_feature_idx_ = header.count("max_feature_idx") ? std::stoi(header["max_feature_idx"]) : 0;
  if (b->max_feature_idx_ < 0 || b->max_feature_idx_ > (1 << 28)) throw std::runtime_error("model string: bad max_feature_idx");
  if (b->num_class_ < 1 || b->num_tree_per_iter_ < 1 || b->num_class_ > (1 << 16) || b->num_tree_per_iter_ > (1 << 16))
    throw std::runtime_error("model string: bad num_class / num_tree_per_iteration");
  b->objective_str_ = header.count("objective") ? header["objective"] : "regression";
  {
    std::istringstream fs(header["feature_names"]);
    std::string tok;
    while (fs >> tok) b->feature_names_.push_back(tok);
    std::istringstream fi(header["feature_infos"]);
    while (fi >> tok) b->feature_infos_.push_back(tok);
  }
  // trees
  std::string block;
  bool in_tree = false, saw_tree = false, saw_end = false;
  for (; i < lines.size(); ++i) {
    std::string l = Trim(lines[i]);
    if (l.rfind("Tree=", 0) == 0) saw_tree = true;
    if (l == "end of trees") saw_end = true;
    if (l.rfind("Tree=", 0) == 0 || l == "end of trees") {
      if (in_tree) {
        Tree t = Tree::FromString(block);
        for (int n = 0; n + 1 < t.num_leaves; ++n)
          if (t.split_feature[n] > b->max_feature_idx_)
            throw std::runtime_error("malformed tree in model string: split_feature " +
                                     std::to_string(t.split_feature[n]) + " > max_feature_idx " +
                                     std::to_string(b->max_feature_idx_));
        b->trees_.push_back(std::move(t));
      }
      block.clear();
      in_tree = l.rfind("Tree=", 0) == 0;
      if (l == "end of trees") { ++i; break; }
      continue;
    }
    if (in_tree) { block += l; block += "\n"; }
  }
  if (saw_tree && !saw_end) throw std::runtime_error("model string is truncated: no 'end of trees' after the trees");
  // parameters section
  std::ostringstream params;
  bool in_params = false;
  std::string cfg_str;
  for (; i < lines.size(); ++i) {
    std::string l = Trim(lines[i]);
    if (l == "parameters:") { in_params = true; continue; }
    if (l == "end of parameters") break;
    if (in_params && l.size() > 2 && l.front() == '[') {
      params << l << "\n";
      auto colon = l.find(':');
      if (colon != std::string::npos) {
        std::string k = Trim(l.substr(1, colon - 1)), v = Trim(l.substr(colon + 1, l.size() - colon - 2));
        if (!v.empty() && v.find(' ') == std::string::npos) cfg_str += k + "=" + v + " ";
      }
    }
  }
  b->loaded_parameters_ = params.str();
  b->cfg_ = Config::Parse(cfg_str);
  {
    std::string on = b->objective_str_.substr(0, b->objective_str_.find(' '));
    b->cfg_.objective = on;
  }
  b->params_str_ = cfg_str;
  return b;
}

}  // namespace sml
