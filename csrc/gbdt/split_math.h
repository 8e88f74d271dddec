// Split-gain / leaf-output formulas shared by the CPU learner and the HIP
// split-search kernel (K5 in SURVEY.md §2.4). Semantics follow LightGBM's
// FeatureHistogram: L1 soft-threshold, L2 shrink, max_delta_step clamp, and
// data counts estimated from hessian sums (cnt_factor = n / sum_hessian).
#pragma once
#include <cmath>
#include <cstdint>

#if defined(__HIPCC__)
#define SML_HD __host__ __device__ __forceinline__
#else
#define SML_HD inline
#endif

namespace sml {

// Round half to even (the default FP rounding mode, what rint / nearbyint return) without a libm call:
// |x| + 2^52 lands where doubles are spaced 1 apart, so the FPU's addition rounds it (SSE2 double; the pair is
// not folded without -ffast-math); |x| >= 2^52 is integral already. Used where a quantised value per row is
// computed on the host (fixed-point histograms and label sums).
inline double RintFast(double x) {
  constexpr double kTwo52 = 4503599627370496.0;
  const double a = std::fabs(x);
  if (!(a < kTwo52)) return x;  // integral already (or nan / inf)
  return std::copysign((a + kTwo52) - kTwo52, x);
}

constexpr double kEpsilon = 1e-15;

struct SplitParams {
  double lambda_l1, lambda_l2, max_delta_step, min_gain_to_split, min_sum_hessian;
  int min_data_in_leaf;
  int num_leaves, max_depth;
  // categorical
  double cat_l2, cat_smooth;
  int max_cat_threshold, max_cat_to_onehot, min_data_per_group;
  // monotone constraints (LightGBM "basic" method): any feature constrained
  int has_mono;
  double monotone_penalty;
  // feature_fraction_bynode: each node samples bynode_k of the tree's allowed
  // features (bynode_k == 0: off); tree_seq numbers the trees of the run
  int bynode_k, tree_seq;
  unsigned long long bynode_seed;
};

// Output bounds of the leaf being split and the monotone direction of the
// candidate feature (+1 increasing, -1 decreasing, 0 none). LightGBM's basic
// method (BasicLeafConstraints): child outputs are clamped into the leaf's
// [lo, hi], a split whose clamped outputs violate the direction is rejected,
// and the gain is evaluated at the clamped outputs.
struct MonoCtx {
  double lo, hi;
  int mono;
};

SML_HD double ThresholdL1(double s, double l1) {
  double reg = fabs(s) - l1;
  if (reg < 0) reg = 0;
  return (s > 0 ? 1.0 : (s < 0 ? -1.0 : 0.0)) * reg;
}

SML_HD double LeafOutput(double g, double h, double l1, double l2, double max_delta_step) {
  double out = -ThresholdL1(g, l1) / (h + l2);
  if (max_delta_step > 0 && fabs(out) > max_delta_step) out = (out > 0 ? 1.0 : -1.0) * max_delta_step;
  return out;
}

SML_HD double LeafGainGivenOutput(double g, double h, double l1, double l2, double out) {
  const double sg = ThresholdL1(g, l1);
  return -(2.0 * sg * out + (h + l2) * out * out);
}

SML_HD double LeafGain(double g, double h, double l1, double l2, double max_delta_step) {
  if (max_delta_step <= 0) {
    const double sg = ThresholdL1(g, l1);
    return sg * sg / (h + l2);
  }
  return LeafGainGivenOutput(g, h, l1, l2, LeafOutput(g, h, l1, l2, max_delta_step));
}

// Gain of a candidate split (before subtracting the parent's gain) and the two
// leaf outputs; false if a monotone constraint rejects it. mc == nullptr is the
// unconstrained path (bitwise the historical formulas).
SML_HD bool EvalSplit(double gl, double hl, double gr, double hr, double l1, double l2, double max_delta_step,
                      const MonoCtx* mc, double* gain, double* lout, double* rout) {
  double lo = LeafOutput(gl, hl, l1, l2, max_delta_step);
  double ro = LeafOutput(gr, hr, l1, l2, max_delta_step);
  if (mc == nullptr) {
    *gain = LeafGain(gl, hl, l1, l2, max_delta_step) + LeafGain(gr, hr, l1, l2, max_delta_step);
  } else {
    lo = lo < mc->lo ? mc->lo : (lo > mc->hi ? mc->hi : lo);
    ro = ro < mc->lo ? mc->lo : (ro > mc->hi ? mc->hi : ro);
    if ((mc->mono > 0 && lo > ro) || (mc->mono < 0 && lo < ro)) return false;
    *gain = LeafGainGivenOutput(gl, hl, l1, l2, lo) + LeafGainGivenOutput(gr, hr, l1, l2, ro);
  }
  *lout = lo;
  *rout = ro;
  return true;
}

// LightGBM's monotone_penalty: monotone splits in the first levels are damped
// (LeafConstraintsBase::ComputeMonotoneSplitGainPenalty).
SML_HD double MonotonePenaltyFactor(int depth, double penalty) {
  if (penalty >= depth + 1.0) return kEpsilon;
  if (penalty <= 1.0) return 1.0 - penalty / pow(2.0, depth) + kEpsilon;
  return 1.0 - pow(2.0, penalty - 1.0 - depth) + kEpsilon;
}

SML_HD int64_t EstimateCount(double h, double cnt_factor) {
  return static_cast<int64_t>(h * cnt_factor + 0.5);
}

// Best split of one leaf (host-side result record; the device kernel writes
// the same fields into a POD of identical layout).
struct SplitResult {
  double gain;         // split gain minus parent gain (LightGBM's "split_gain")
  double left_g, left_h, right_g, right_h;
  double left_out, right_out;
  int64_t left_cnt, right_cnt;
  int feature;         // inner feature index, -1 = no split
  uint32_t threshold;  // bin threshold (numerical) or number of categories (categorical)
  int default_left;
  int is_cat;
  uint32_t cat_bits[8];  // categorical: bins that go left (256 bins max)
};

SML_HD bool SplitBetter(double gain_a, int feat_a, uint32_t thr_a, double gain_b, int feat_b, uint32_t thr_b) {
  // deterministic ordering: larger gain, then smaller feature, then smaller threshold
  if (gain_a != gain_b) return gain_a > gain_b;
  if (feat_a != feat_b) return feat_a < feat_b;
  return thr_a < thr_b;
}

}  // namespace sml
