// Training/prediction configuration for the native GBDT engine.
//
// The engine is configured the same way the reference configures its native
// booster: a whitespace separated "key=value" string (see reference
// lightgbm/.../params/BaseTrainParams.scala:25-40, which builds that string, and
// ParamsStringBuilder semantics in core/.../utils/ParamsStringBuilder.scala).
// Keys and aliases follow LightGBM's documented parameter names so a user's
// passThroughArgs keep working.
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace sml {

struct Config {
  // core
  std::string objective = "regression";
  std::string boosting = "gbdt";  // gbdt | rf | dart | goss
  std::string metric_str;         // comma separated
  std::string device_type = "gpu";  // gpu | cpu
  int num_iterations = 100;
  double learning_rate = 0.1;
  int num_leaves = 31;
  int max_depth = -1;
  int min_data_in_leaf = 20;
  double min_sum_hessian_in_leaf = 1e-3;
  double lambda_l1 = 0.0;
  double lambda_l2 = 0.0;
  double min_gain_to_split = 0.0;
  double max_delta_step = 0.0;
  int num_class = 1;
  bool is_unbalance = false;
  double scale_pos_weight = 1.0;
  double sigmoid = 1.0;
  bool boost_from_average = true;
  double alpha = 0.9;                 // huber / quantile
  double fair_c = 1.0;
  double poisson_max_delta_step = 0.7;
  double tweedie_variance_power = 1.5;
  // sampling
  double bagging_fraction = 1.0;
  double pos_bagging_fraction = 1.0;
  double neg_bagging_fraction = 1.0;
  int bagging_freq = 0;
  int bagging_seed = 3;
  double feature_fraction = 1.0;
  double feature_fraction_bynode = 1.0;
  int feature_fraction_seed = 2;
  double top_rate = 0.2;    // goss
  double other_rate = 0.1;  // goss
  // dart
  double drop_rate = 0.1;
  int max_drop = 50;
  double skip_drop = 0.5;
  bool xgboost_dart_mode = false;
  bool uniform_drop = false;
  int drop_seed = 4;
  // dataset
  int max_bin = 255;
  int min_data_in_bin = 3;
  int bin_construct_sample_cnt = 200000;
  int data_random_seed = 1;
  bool use_missing = true;
  bool zero_as_missing = false;
  bool is_enable_sparse = true;
  std::vector<int> categorical_feature;
  std::vector<int> max_bin_by_feature;
  // categorical
  int max_cat_threshold = 32;
  double cat_l2 = 10.0;
  double cat_smooth = 10.0;
  int max_cat_to_onehot = 4;
  int min_data_per_group = 100;
  // constraints
  std::vector<int> monotone_constraints;
  std::string monotone_constraints_method = "basic";  // basic (intermediate/advanced run as basic)
  double monotone_penalty = 0.0;
  // ranking
  std::vector<double> label_gain;
  std::vector<int> eval_at;
  int max_position = 20;
  bool lambdarank_norm = true;
  // misc
  int seed = 0;
  bool seed_set = false;
  bool deterministic = false;
  int num_threads = 0;
  int verbosity = -1;
  int early_stopping_round = 0;
  double improvement_tolerance = 0.0;
  int extra_seed = 6;
  int objective_seed = 5;
  // distributed
  int num_machines = 1;
  std::string tree_learner = "serial";
  int top_k = 20;
  int time_out = 120;  // minutes a collective may block before the job fails (LightGBM `time_out`)
  // gpu
  int gpu_device_id = -1;
  bool use_quantized_grad = false;

  // every key/value pair seen (in order), so the model text can echo them
  std::vector<std::pair<std::string, std::string>> raw;

  static Config Parse(const std::string& s);
  void Set(const std::string& key, const std::string& value);
  std::vector<std::string> Metrics() const;
  // LightGBM-style "[key: value]" lines for the model's parameters section.
  std::string ToParametersSection() const;
  bool IsClassification() const;
  int NumTreePerIteration() const;
};

}  // namespace sml
