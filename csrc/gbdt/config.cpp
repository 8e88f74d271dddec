#include "config.h"

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <sstream>
#include <stdexcept>

namespace sml {
namespace {

std::string Trim(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e && std::isspace(static_cast<unsigned char>(s[b]))) ++b;
  while (e > b && std::isspace(static_cast<unsigned char>(s[e - 1]))) --e;
  return s.substr(b, e - b);
}

bool ParseBool(const std::string& v) {
  std::string l = v;
  std::transform(l.begin(), l.end(), l.begin(), ::tolower);
  return l == "true" || l == "1" || l == "+" || l == "yes";
}

template <class T>
std::vector<T> ParseList(const std::string& v) {
  std::vector<T> out;
  std::string tok;
  std::stringstream ss(v);
  while (std::getline(ss, tok, ',')) {
    tok = Trim(tok);
    if (tok.empty()) continue;
    out.push_back(static_cast<T>(std::stod(tok)));
  }
  return out;
}

// alias -> canonical name (subset of LightGBM's alias table that users pass)
const std::map<std::string, std::string>& Aliases() {
  static const std::map<std::string, std::string> m = {
      {"objective_type", "objective"}, {"app", "objective"}, {"application", "objective"},
      {"loss", "objective"}, {"boosting_type", "boosting"}, {"boost", "boosting"},
      {"num_iteration", "num_iterations"}, {"n_iter", "num_iterations"},
      {"num_tree", "num_iterations"}, {"num_trees", "num_iterations"},
      {"num_round", "num_iterations"}, {"num_rounds", "num_iterations"},
      {"num_boost_round", "num_iterations"}, {"n_estimators", "num_iterations"},
      {"shrinkage_rate", "learning_rate"}, {"eta", "learning_rate"},
      {"num_leaf", "num_leaves"}, {"max_leaves", "num_leaves"}, {"max_leaf", "num_leaves"},
      {"min_data_per_leaf", "min_data_in_leaf"}, {"min_data", "min_data_in_leaf"},
      {"min_child_samples", "min_data_in_leaf"},
      {"min_sum_hessian_per_leaf", "min_sum_hessian_in_leaf"},
      {"min_sum_hessian", "min_sum_hessian_in_leaf"}, {"min_hessian", "min_sum_hessian_in_leaf"},
      {"min_child_weight", "min_sum_hessian_in_leaf"},
      {"reg_alpha", "lambda_l1"}, {"l1_regularization", "lambda_l1"},
      {"reg_lambda", "lambda_l2"}, {"lambda", "lambda_l2"}, {"l2_regularization", "lambda_l2"},
      {"min_split_gain", "min_gain_to_split"}, {"max_tree_output", "max_delta_step"},
      {"max_leaf_output", "max_delta_step"}, {"num_classes", "num_class"},
      {"unbalance", "is_unbalance"}, {"unbalanced_sets", "is_unbalance"},
      {"sub_row", "bagging_fraction"}, {"subsample", "bagging_fraction"},
      {"bagging", "bagging_fraction"}, {"subsample_freq", "bagging_freq"},
      {"bagging_fraction_seed", "bagging_seed"}, {"sub_feature", "feature_fraction"},
      {"colsample_bytree", "feature_fraction"}, {"colsample_bynode", "feature_fraction_bynode"},
      {"sub_feature_bynode", "feature_fraction_bynode"},
      {"max_bins", "max_bin"}, {"subsample_for_bin", "bin_construct_sample_cnt"},
      {"data_seed", "data_random_seed"}, {"cat_feature", "categorical_feature"},
      {"categorical_column", "categorical_feature"}, {"cat_column", "categorical_feature"},
      {"is_sparse", "is_enable_sparse"}, {"enable_sparse", "is_enable_sparse"},
      {"random_seed", "seed"}, {"random_state", "seed"}, {"num_thread", "num_threads"},
      {"nthread", "num_threads"}, {"nthreads", "num_threads"}, {"n_jobs", "num_threads"},
      {"early_stopping_rounds", "early_stopping_round"}, {"early_stopping", "early_stopping_round"},
      {"n_iter_no_change", "early_stopping_round"}, {"metrics", "metric"},
      {"metric_types", "metric"}, {"ndcg_eval_at", "eval_at"}, {"ndcg_at", "eval_at"},
      {"map_eval_at", "eval_at"}, {"map_at", "eval_at"}, {"num_machine", "num_machines"},
      {"tree", "tree_learner"}, {"tree_type", "tree_learner"}, {"tree_learner_type", "tree_learner"},
      {"device", "device_type"}, {"verbose", "verbosity"}, {"mc", "monotone_constraints"},
      {"monotone_constraint", "monotone_constraints"}, {"top_k", "top_k"}, {"topk", "top_k"},
      {"monotone_constraining_method", "monotone_constraints_method"}, {"mc_method", "monotone_constraints_method"},
      {"monotone_splits_penalty", "monotone_penalty"}, {"ms_penalty", "monotone_penalty"},
      {"mc_penalty", "monotone_penalty"},
  };
  return m;
}

}  // namespace

void Config::Set(const std::string& key_in, const std::string& value_in) {
  std::string key = Trim(key_in), v = Trim(value_in);
  auto it = Aliases().find(key);
  if (it != Aliases().end()) key = it->second;
  raw.emplace_back(key, v);
  auto I = [&] { return std::atoi(v.c_str()); };
  auto D = [&] { return std::atof(v.c_str()); };
  auto B = [&] { return ParseBool(v); };
  if (key == "objective") {
    objective = v;
    // "binary sigmoid:1" style (model text) is tolerated
    auto sp = objective.find(' ');
    if (sp != std::string::npos) objective = objective.substr(0, sp);
  } else if (key == "boosting") boosting = v;
  else if (key == "metric") metric_str = v;
  else if (key == "device_type") device_type = v;
  else if (key == "num_iterations") num_iterations = I();
  else if (key == "learning_rate") learning_rate = D();
  else if (key == "num_leaves") num_leaves = I();
  else if (key == "max_depth") max_depth = I();
  else if (key == "min_data_in_leaf") min_data_in_leaf = I();
  else if (key == "min_sum_hessian_in_leaf") min_sum_hessian_in_leaf = D();
  else if (key == "lambda_l1") lambda_l1 = D();
  else if (key == "lambda_l2") lambda_l2 = D();
  else if (key == "min_gain_to_split") min_gain_to_split = D();
  else if (key == "max_delta_step") max_delta_step = D();
  else if (key == "num_class") num_class = I();
  else if (key == "is_unbalance") is_unbalance = B();
  else if (key == "scale_pos_weight") scale_pos_weight = D();
  else if (key == "sigmoid") sigmoid = D();
  else if (key == "boost_from_average") boost_from_average = B();
  else if (key == "alpha") alpha = D();
  else if (key == "fair_c") fair_c = D();
  else if (key == "poisson_max_delta_step") poisson_max_delta_step = D();
  else if (key == "tweedie_variance_power") tweedie_variance_power = D();
  else if (key == "bagging_fraction") bagging_fraction = D();
  else if (key == "pos_bagging_fraction") pos_bagging_fraction = D();
  else if (key == "neg_bagging_fraction") neg_bagging_fraction = D();
  else if (key == "bagging_freq") bagging_freq = I();
  else if (key == "bagging_seed") bagging_seed = I();
  else if (key == "feature_fraction") feature_fraction = D();
  else if (key == "feature_fraction_bynode") feature_fraction_bynode = D();
  else if (key == "feature_fraction_seed") feature_fraction_seed = I();
  else if (key == "top_rate") top_rate = D();
  else if (key == "other_rate") other_rate = D();
  else if (key == "drop_rate") drop_rate = D();
  else if (key == "max_drop") max_drop = I();
  else if (key == "skip_drop") skip_drop = D();
  else if (key == "xgboost_dart_mode") xgboost_dart_mode = B();
  else if (key == "uniform_drop") uniform_drop = B();
  else if (key == "drop_seed") drop_seed = I();
  else if (key == "max_bin") max_bin = I();
  else if (key == "min_data_in_bin") min_data_in_bin = I();
  else if (key == "bin_construct_sample_cnt") bin_construct_sample_cnt = I();
  else if (key == "data_random_seed") data_random_seed = I();
  else if (key == "use_missing") use_missing = B();
  else if (key == "zero_as_missing") zero_as_missing = B();
  else if (key == "is_enable_sparse") is_enable_sparse = B();
  else if (key == "categorical_feature") categorical_feature = ParseList<int>(v);
  else if (key == "max_bin_by_feature") max_bin_by_feature = ParseList<int>(v);
  else if (key == "max_cat_threshold") max_cat_threshold = I();
  else if (key == "cat_l2") cat_l2 = D();
  else if (key == "cat_smooth") cat_smooth = D();
  else if (key == "max_cat_to_onehot") max_cat_to_onehot = I();
  else if (key == "min_data_per_group") min_data_per_group = I();
  else if (key == "monotone_constraints") monotone_constraints = ParseList<int>(v);
  else if (key == "monotone_constraints_method") monotone_constraints_method = v;
  else if (key == "monotone_penalty") monotone_penalty = D();
  else if (key == "label_gain") label_gain = ParseList<double>(v);
  else if (key == "eval_at") eval_at = ParseList<int>(v);
  else if (key == "max_position" || key == "lambdarank_truncation_level") max_position = I();
  else if (key == "lambdarank_norm") lambdarank_norm = B();
  else if (key == "seed") { seed = I(); seed_set = true; }
  else if (key == "deterministic") deterministic = B();
  else if (key == "num_threads") num_threads = I();
  else if (key == "verbosity") verbosity = I();
  else if (key == "early_stopping_round") early_stopping_round = I();
  else if (key == "improvement_tolerance") improvement_tolerance = D();
  else if (key == "extra_seed") extra_seed = I();
  else if (key == "objective_seed") objective_seed = I();
  else if (key == "num_machines") num_machines = I();
  else if (key == "tree_learner") {
    tree_learner = v;
    if (v == "voting_parallel") tree_learner = "voting";
    else if (v == "data_parallel") tree_learner = "data";
    else if (v == "feature_parallel") tree_learner = "feature";
  }
  else if (key == "top_k") top_k = I();
  else if (key == "time_out") time_out = I();
  else if (key == "gpu_device_id") gpu_device_id = I();
  else if (key == "use_quantized_grad") use_quantized_grad = B();
  // unknown keys are kept in `raw` (echoed in the model) and otherwise ignored,
  // like LightGBM's "Unknown parameter" warning.
}

Config Config::Parse(const std::string& s) {
  Config c;
  std::stringstream ss(s);
  std::string tok;
  std::map<std::string, bool> seen;
  // First occurrence wins: the reference puts passThroughArgs first and skips
  // later duplicates (ParamsStringBuilder.scala:54-71).
  while (ss >> tok) {
    auto eq = tok.find('=');
    if (eq == std::string::npos) continue;
    std::string k = Trim(tok.substr(0, eq));
    auto it = Aliases().find(k);
    std::string canon = it == Aliases().end() ? k : it->second;
    if (seen[canon]) continue;
    seen[canon] = true;
    c.Set(k, tok.substr(eq + 1));
  }
  if (c.seed_set) {
    // LightGBM derives the other seeds from `seed` when it is given.
    uint32_t s0 = static_cast<uint32_t>(c.seed);
    auto next = [&s0]() { s0 = s0 * 214013u + 2531011u; return static_cast<int>((s0 >> 16) & 0x7FFF); };
    if (!seen["data_random_seed"]) c.data_random_seed = next();
    if (!seen["bagging_seed"]) c.bagging_seed = next();
    if (!seen["drop_seed"]) c.drop_seed = next();
    if (!seen["feature_fraction_seed"]) c.feature_fraction_seed = next();
    if (!seen["objective_seed"]) c.objective_seed = next();
    if (!seen["extra_seed"]) c.extra_seed = next();
  }
  if (c.objective == "multiclass" || c.objective == "softmax" || c.objective == "multiclassova" ||
      c.objective == "multiclass_ova" || c.objective == "ova" || c.objective == "ovr") {
    if (c.objective == "softmax") c.objective = "multiclass";
    if (c.objective != "multiclass") c.objective = "multiclassova";
  } else {
    if (c.objective == "regression_l2" || c.objective == "l2" || c.objective == "mean_squared_error" ||
        c.objective == "mse" || c.objective == "l2_root" || c.objective == "root_mean_squared_error" ||
        c.objective == "rmse")
      c.objective = "regression";
    if (c.objective == "l1" || c.objective == "mean_absolute_error" || c.objective == "mae")
      c.objective = "regression_l1";
    if (c.objective == "xentropy") c.objective = "cross_entropy";
    if (c.objective == "mean_absolute_percentage_error") c.objective = "mape";
  }
  if (c.boosting == "random_forest") c.boosting = "rf";
  if (c.label_gain.empty()) {
    for (int i = 0; i < 31; ++i) c.label_gain.push_back(static_cast<double>((1u << i) - 1));
  }
  if (c.eval_at.empty()) c.eval_at = {1, 2, 3, 4, 5};
  if (c.max_bin > 255) c.max_bin = 255;  // bins are stored as uint8 on device
  return c;
}

std::vector<std::string> Config::Metrics() const {
  std::vector<std::string> out;
  std::string tok;
  std::stringstream ss(metric_str);
  while (std::getline(ss, tok, ',')) {
    tok = Trim(tok);
    if (!tok.empty()) out.push_back(tok);
  }
  return out;
}

bool Config::IsClassification() const {
  return objective == "binary" || objective == "multiclass" || objective == "multiclassova";
}

int Config::NumTreePerIteration() const {
  return (objective == "multiclass" || objective == "multiclassova") ? num_class : 1;
}

std::string Config::ToParametersSection() const {
  std::ostringstream o;
  auto b = [](bool x) { return x ? 1 : 0; };
  auto lst = [](const auto& v) {
    std::ostringstream s;
    for (size_t i = 0; i < v.size(); ++i) s << (i ? "," : "") << v[i];
    return s.str();
  };
  o << "[boosting: " << boosting << "]\n";
  o << "[objective: " << objective << "]\n";
  o << "[metric: " << metric_str << "]\n";
  o << "[tree_learner: " << tree_learner << "]\n";
  o << "[device_type: " << device_type << "]\n";
  o << "[num_iterations: " << num_iterations << "]\n";
  o << "[learning_rate: " << learning_rate << "]\n";
  o << "[num_leaves: " << num_leaves << "]\n";
  o << "[num_threads: " << num_threads << "]\n";
  o << "[deterministic: " << b(deterministic) << "]\n";
  o << "[max_depth: " << max_depth << "]\n";
  o << "[min_data_in_leaf: " << min_data_in_leaf << "]\n";
  o << "[min_sum_hessian_in_leaf: " << min_sum_hessian_in_leaf << "]\n";
  o << "[bagging_fraction: " << bagging_fraction << "]\n";
  o << "[pos_bagging_fraction: " << pos_bagging_fraction << "]\n";
  o << "[neg_bagging_fraction: " << neg_bagging_fraction << "]\n";
  o << "[bagging_freq: " << bagging_freq << "]\n";
  o << "[bagging_seed: " << bagging_seed << "]\n";
  o << "[feature_fraction: " << feature_fraction << "]\n";
  o << "[feature_fraction_bynode: " << feature_fraction_bynode << "]\n";
  o << "[feature_fraction_seed: " << feature_fraction_seed << "]\n";
  o << "[early_stopping_round: " << early_stopping_round << "]\n";
  o << "[max_delta_step: " << max_delta_step << "]\n";
  o << "[lambda_l1: " << lambda_l1 << "]\n";
  o << "[lambda_l2: " << lambda_l2 << "]\n";
  o << "[min_gain_to_split: " << min_gain_to_split << "]\n";
  o << "[drop_rate: " << drop_rate << "]\n";
  o << "[max_drop: " << max_drop << "]\n";
  o << "[skip_drop: " << skip_drop << "]\n";
  o << "[xgboost_dart_mode: " << b(xgboost_dart_mode) << "]\n";
  o << "[uniform_drop: " << b(uniform_drop) << "]\n";
  o << "[drop_seed: " << drop_seed << "]\n";
  o << "[top_rate: " << top_rate << "]\n";
  o << "[other_rate: " << other_rate << "]\n";
  o << "[min_data_per_group: " << min_data_per_group << "]\n";
  o << "[max_cat_threshold: " << max_cat_threshold << "]\n";
  o << "[cat_l2: " << cat_l2 << "]\n";
  o << "[cat_smooth: " << cat_smooth << "]\n";
  o << "[max_cat_to_onehot: " << max_cat_to_onehot << "]\n";
  o << "[top_k: " << top_k << "]\n";
  o << "[monotone_constraints: " << lst(monotone_constraints) << "]\n";
  o << "[monotone_constraints_method: " << monotone_constraints_method << "]\n";
  o << "[monotone_penalty: " << monotone_penalty << "]\n";
  o << "[max_bin: " << max_bin << "]\n";
  o << "[max_bin_by_feature: " << lst(max_bin_by_feature) << "]\n";
  o << "[min_data_in_bin: " << min_data_in_bin << "]\n";
  o << "[bin_construct_sample_cnt: " << bin_construct_sample_cnt << "]\n";
  o << "[data_random_seed: " << data_random_seed << "]\n";
  o << "[is_enable_sparse: " << b(is_enable_sparse) << "]\n";
  o << "[use_missing: " << b(use_missing) << "]\n";
  o << "[zero_as_missing: " << b(zero_as_missing) << "]\n";
  o << "[categorical_feature: " << lst(categorical_feature) << "]\n";
  o << "[num_class: " << num_class << "]\n";
  o << "[is_unbalance: " << b(is_unbalance) << "]\n";
  o << "[scale_pos_weight: " << scale_pos_weight << "]\n";
  o << "[sigmoid: " << sigmoid << "]\n";
  o << "[boost_from_average: " << b(boost_from_average) << "]\n";
  o << "[alpha: " << alpha << "]\n";
  o << "[fair_c: " << fair_c << "]\n";
  o << "[poisson_max_delta_step: " << poisson_max_delta_step << "]\n";
  o << "[tweedie_variance_power: " << tweedie_variance_power << "]\n";
  o << "[max_position: " << max_position << "]\n";
  o << "[lambdarank_norm: " << b(lambdarank_norm) << "]\n";
  o << "[label_gain: " << lst(label_gain) << "]\n";
  o << "[eval_at: " << lst(eval_at) << "]\n";
  o << "[num_machines: " << num_machines << "]\n";
  o << "[gpu_device_id: " << gpu_device_id << "]\n";
  o << "[use_quantized_grad: " << b(use_quantized_grad) << "]\n";
  // anything else the user passed through (unknown to us) is echoed verbatim
  static const char* known[] = {
      "boosting", "objective", "metric", "tree_learner", "device_type", "num_iterations",
      "learning_rate", "num_leaves", "num_threads", "deterministic", "max_depth",
      "min_data_in_leaf", "min_sum_hessian_in_leaf", "bagging_fraction", "pos_bagging_fraction",
      "neg_bagging_fraction", "bagging_freq", "bagging_seed", "feature_fraction",
      "feature_fraction_bynode", "feature_fraction_seed", "early_stopping_round", "max_delta_step",
      "lambda_l1", "lambda_l2", "min_gain_to_split", "drop_rate", "max_drop", "skip_drop",
      "xgboost_dart_mode", "uniform_drop", "drop_seed", "top_rate", "other_rate",
      "min_data_per_group", "max_cat_threshold", "cat_l2", "cat_smooth", "max_cat_to_onehot",
      "top_k", "monotone_constraints", "monotone_constraints_method", "monotone_penalty", "max_bin", "max_bin_by_feature", "min_data_in_bin",
      "bin_construct_sample_cnt", "data_random_seed", "is_enable_sparse", "use_missing",
      "zero_as_missing", "categorical_feature", "num_class", "is_unbalance", "scale_pos_weight",
      "sigmoid", "boost_from_average", "alpha", "fair_c", "poisson_max_delta_step",
      "tweedie_variance_power", "max_position", "lambdarank_norm", "label_gain", "eval_at",
      "num_machines", "gpu_device_id", "use_quantized_grad", "time_out"};
  for (const auto& kv : raw) {
    bool k = false;
    for (const char* n : known) if (kv.first == n) { k = true; break; }
    if (!k) o << "[" << kv.first << ": " << kv.second << "]\n";
  }
  return o.str();
}

}  // namespace sml
