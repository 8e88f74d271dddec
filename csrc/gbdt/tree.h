// Decision tree in LightGBM's array layout (internal nodes 0..L-2, a negative
// child c means leaf ~c). The text form is LightGBM's v3 "Tree=" block, which
// the reference round-trips through saveNativeModel / loadNativeModelFromString
// (lightgbm/.../booster/LightGBMBooster.scala:272-278,458-467).
#pragma once
#include <cmath>
#include <cstdint>
#include <string>
#include <vector>

#include "dataset.h"

namespace sml {

// decision_type bit layout (LightGBM): bit0 categorical, bit1 default_left,
// bits 2-3 missing type.
inline int8_t MakeDecisionType(bool categorical, bool default_left, int missing_type) {
  return static_cast<int8_t>((categorical ? 1 : 0) | (default_left ? 2 : 0) | ((missing_type & 3) << 2));
}

struct Tree {
  int max_leaves = 0;
  int num_leaves = 1;
  int num_cat = 0;
  double shrinkage = 1.0;
  std::vector<int> split_feature_inner, split_feature;
  std::vector<double> split_gain, threshold;
  std::vector<uint32_t> threshold_in_bin;
  std::vector<int8_t> decision_type;
  std::vector<int> left_child, right_child;
  std::vector<double> leaf_value, leaf_weight;
  std::vector<int64_t> leaf_count;
  std::vector<double> internal_value, internal_weight;
  std::vector<int64_t> internal_count;
  std::vector<int> leaf_parent, leaf_depth;
  std::vector<int> cat_boundaries{0};
  std::vector<uint32_t> cat_threshold;        // bitsets over category values
  std::vector<int> cat_boundaries_inner{0};
  std::vector<uint32_t> cat_threshold_inner;  // bitsets over bins

  explicit Tree(int max_leaves_ = 1);
  // Split `leaf` numerically. Returns the index of the new (right) leaf.
  int Split(int leaf, int feat_inner, int feat_real, uint32_t thr_bin, double thr_value,
            bool default_left, int missing_type, double left_value, double right_value,
            int64_t left_cnt, int64_t right_cnt, double left_weight, double right_weight, double gain);
  int SplitCategorical(int leaf, int feat_inner, int feat_real, const std::vector<uint32_t>& bin_bitset,
                       const std::vector<uint32_t>& value_bitset, double left_value, double right_value,
                       int64_t left_cnt, int64_t right_cnt, double left_weight, double right_weight,
                       double gain);
  void Shrink(double rate);
  void AddBias(double bias);
  void SetLeafValue(int leaf, double v) { leaf_value[leaf] = v; }

  // value-domain traversal (prediction on raw features)
  int GetLeaf(const double* x) const;
  int GetLeafSparse(const int32_t* idx, const double* val, int nnz, std::vector<double>* buf) const;
  double Predict(const double* x) const { return num_leaves > 1 ? leaf_value[GetLeaf(x)] : leaf_value[0]; }
  // bin-domain traversal (training-time score updates)
  int GetLeafByBins(const uint8_t* row, const std::vector<BinMapper>& mappers,
                    const std::vector<int>& used) const;

  int NumericalDecision(double fval, int node) const;
  int CategoricalDecision(double fval, int node) const;
  void TreeSHAP(const double* x, double* phi, int num_features) const;
  double ExpectedValue() const;
  int MaxDepth() const;

  std::string ToString(int index) const;
  static Tree FromString(const std::string& block);
  std::string ToJSON(int index) const;
};

}  // namespace sml
