// Row sampling for bagging and GOSS (K8 of SURVEY.md §2.4).
//
// The reference's booster draws bagging / GOSS subsets inside lib_lightgbm
// (bagging_fraction / bagging_freq / pos|neg_bagging_fraction, GOSS top_rate /
// other_rate; lightgbm/.../params/LightGBMParams.scala:218-224,302-324). Here
// the random draw of row i at iteration t is a counter-based hash of
// (seed, t, i): no RNG state has to be carried per row, the HIP backend can
// sample on the device in one pass, and the CPU and HIP backends draw exactly
// the same rows for the same seed.
#pragma once
#include <cstdint>

#include "split_math.h"

namespace sml {

SML_HD uint64_t SplitMix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// uniform double in [0, 1) for (seed, iteration, row)
SML_HD double RowUniform(uint64_t seed, int iter, int64_t row) {
  const uint64_t s = SplitMix64(seed ^ (0xD1B54A32D192ED03ull * static_cast<uint64_t>(iter + 1)));
  return static_cast<double>(SplitMix64(s + static_cast<uint64_t>(row)) >> 11) * (1.0 / 9007199254740992.0);
}

// feature_fraction_bynode: is feature f among the k sampled for node `node`
// of tree `tree`? Every allowed feature gets a hash key; the k smallest win.
// Pure function of (seed, tree, node, f), so host and device agree and each
// split-search block decides for its own feature without a shared shuffle.
SML_HD uint64_t NodeFeatureKey(uint64_t seed, int tree, int node, int f) {
  return SplitMix64(SplitMix64(seed ^ (0x9E3779B97F4A7C15ull * static_cast<uint64_t>(tree + 1))) ^
                    (0xC2B2AE3D27D4EB4Full * static_cast<uint64_t>(node + 1)) ^ static_cast<uint64_t>(f));
}

SML_HD bool NodeFeatureSelected(uint64_t seed, int tree, int node, int f, const int8_t* allowed, int F, int k) {
  const uint64_t key = NodeFeatureKey(seed, tree, node, f);
  int rank = 0;
  for (int g = 0; g < F; ++g) {
    if (g == f || !allowed[g]) continue;
    const uint64_t kg = NodeFeatureKey(seed, tree, node, g);
    rank += (kg < key) || (kg == key && g < f);
  }
  return rank < k;
}

enum RowSampleKind : int { kSampleBagging = 1, kSampleGoss = 2 };

struct RowSampleSpec {
  int kind = 0;
  uint64_t seed = 0;
  int iter = 0;
  // bagging: keep row with probability fraction (pos/neg_fraction by label when balanced)
  double fraction = 1.0, pos_fraction = 1.0, neg_fraction = 1.0;
  bool balanced = false;
  // GOSS: keep the top_k rows by sum_k |g*h| (float), then the rest with
  // probability other_prob, their gradients scaled by other_mult
  int64_t top_k = 0;
  double other_prob = 0.0, other_mult = 1.0;
};

}  // namespace sml
