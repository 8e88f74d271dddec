// K11: training-metric evaluation on the device (reference: LGBM_BoosterGetEval,
// lightgbm/.../booster/LightGBMBooster.scala:300-314, called per iteration when
// isProvideTrainingMetric is set, TrainUtils.scala:137-169).
//
// The training scores already live in HBM; the host path would copy n doubles
// back and sort them on the CPU every iteration (~1 s at 11M rows). Here:
//   auc        radix sort (score desc, hipCUB) -> per-distinct-score positive /
//              negative weight sums (reduce-by-key) -> exclusive scan of the
//              positives -> sum_g NEG_g * (POS_before_g + POS_g / 2)
//              = the host's trapezoid over tied groups (objective.cpp AUC)
//   binary_logloss / binary_error (binary objective) and l2 / rmse / l1 / mae
//   (identity-output objectives): one fused transform-reduce
// hipCUB is used only for the generic sort / scan / reduce-by-key.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "hip_common.h"
#include "objective.h"

namespace sml {
namespace {

constexpr int kThreads = 256;

__global__ void iota_kernel(int32_t* v, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    v[i] = static_cast<int32_t>(i);
}

// per sorted position: positive / negative weight
__global__ void posneg_kernel(const int32_t* __restrict__ order, const float* __restrict__ label,
                              const float* __restrict__ weight, int64_t n, double* __restrict__ pos,
                              double* __restrict__ neg) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
    const int32_t i = order[k];
    const double w = weight ? weight[i] : 1.0;
    const bool y = label[i] > 0;
    pos[k] = y ? w : 0.0;
    neg[k] = y ? 0.0 : w;
  }
}

__global__ void area_terms_kernel(const double* __restrict__ gpos, const double* __restrict__ gneg,
                                  const double* __restrict__ pos_before, const int* __restrict__ ngroups,
                                  double* __restrict__ terms) {
  const int g_n = *ngroups;
  for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < g_n; g += gridDim.x * blockDim.x)
    terms[g] = gneg[g] * (pos_before[g] + 0.5 * gpos[g]);
}

struct PointLoss {
  int kind;  // 0 logloss, 1 error, 2 squared, 3 absolute
  double sigmoid;
  const double* score;
  const float* label;
  const float* weight;
  __device__ double2 operator()(int64_t i) const {
    const double w = weight ? weight[i] : 1.0;
    const double s = score[i];
    double v;
    if (kind <= 1) {
      const double pr = 1.0 / (1.0 + exp(-sigmoid * s));
      const bool y = label[i] > 0;
      if (kind == 0) {
        const double p = fmin(fmax(pr, kEpsilon), 1.0 - kEpsilon);
        v = y ? -log(p) : -log(1.0 - p);
      } else {
        v = ((pr > 0.5) != y) ? 1.0 : 0.0;
      }
    } else {
      const double d = s - label[i];
      v = kind == 2 ? d * d : fabs(d);
    }
    return make_double2(v * w, w);
  }
};

__global__ void point_loss_kernel(PointLoss f, int64_t n, double2* __restrict__ partial) {
  double a = 0.0, b = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double2 v = f(i);
    a += v.x;
    b += v.y;
  }
  using BR = hipcub::BlockReduce<double, kThreads>;
  __shared__ typename BR::TempStorage ta, tb;
  a = BR(ta).Sum(a);
  b = BR(tb).Sum(b);
  if (threadIdx.x == 0) partial[blockIdx.x] = make_double2(a, b);
}

int Grid(int64_t n) { return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(2048, (n + kThreads - 1) / kThreads))); }

double DeviceAUC(const double* score, const float* label, const float* weight, int64_t n, hipStream_t s) {
  DevBuf<double> keys_out, pos, neg, gkeys, gpos, gneg, pbefore, terms, total;
  DevBuf<int32_t> idx_in, idx_out;
  DevBuf<int> ngroups;
  keys_out.alloc(n); pos.alloc(n); neg.alloc(n); gkeys.alloc(n); gpos.alloc(n); gneg.alloc(n);
  pbefore.alloc(n); terms.alloc(n); total.alloc(4);
  idx_in.alloc(n); idx_out.alloc(n); ngroups.alloc(1);
  hipLaunchKernelGGL(iota_kernel, dim3(Grid(n)), dim3(kThreads), 0, s, idx_in.get(), n);
  size_t tmp_bytes = 0, t;
  const int nn = static_cast<int>(n);
  SML_HIP_CHECK(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, t, score, keys_out.get(), idx_in.get(),
                                                             idx_out.get(), nn, 0, 64, s));
  tmp_bytes = std::max(tmp_bytes, t);
  hipcub::Sum sum;
  SML_HIP_CHECK(hipcub::DeviceReduce::ReduceByKey(nullptr, t, keys_out.get(), gkeys.get(), pos.get(), gpos.get(),
                                                  ngroups.get(), sum, nn, s));
  tmp_bytes = std::max(tmp_bytes, t);
  SML_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, t, gpos.get(), pbefore.get(), nn, s));
  tmp_bytes = std::max(tmp_bytes, t);
  SML_HIP_CHECK(hipcub::DeviceReduce::Sum(nullptr, t, terms.get(), total.get(), nn, s));
  tmp_bytes = std::max(tmp_bytes, t);
  DevBuf<uint8_t> tmp;
  tmp.alloc(std::max<size_t>(1, tmp_bytes));
  t = tmp_bytes;
  SML_HIP_CHECK(hipcub::DeviceRadixSort::SortPairsDescending(tmp.get(), t, score, keys_out.get(), idx_in.get(),
                                                             idx_out.get(), nn, 0, 64, s));
  hipLaunchKernelGGL(posneg_kernel, dim3(Grid(n)), dim3(kThreads), 0, s, idx_out.get(), label, weight, n, pos.get(),
                     neg.get());
  t = tmp_bytes;
  SML_HIP_CHECK(hipcub::DeviceReduce::ReduceByKey(tmp.get(), t, keys_out.get(), gkeys.get(), pos.get(), gpos.get(),
                                                  ngroups.get(), sum, nn, s));
  t = tmp_bytes;
  SML_HIP_CHECK(hipcub::DeviceReduce::ReduceByKey(tmp.get(), t, keys_out.get(), gkeys.get(), neg.get(), gneg.get(),
                                                  ngroups.get(), sum, nn, s));
  // positives before each group (groups past ngroups are unused: zero them first)
  SML_HIP_CHECK(hipMemsetAsync(terms.get(), 0, sizeof(double) * n, s));
  t = tmp_bytes;
  SML_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp.get(), t, gpos.get(), pbefore.get(), nn, s));
  hipLaunchKernelGGL(area_terms_kernel, dim3(Grid(n)), dim3(kThreads), 0, s, gpos.get(), gneg.get(), pbefore.get(),
                     ngroups.get(), terms.get());
  t = tmp_bytes;
  SML_HIP_CHECK(hipcub::DeviceReduce::Sum(tmp.get(), t, terms.get(), total.get(), nn, s));
  t = tmp_bytes;
  SML_HIP_CHECK(hipcub::DeviceReduce::Sum(tmp.get(), t, pos.get(), total.get() + 1, nn, s));
  t = tmp_bytes;
  SML_HIP_CHECK(hipcub::DeviceReduce::Sum(tmp.get(), t, neg.get(), total.get() + 2, nn, s));
  double h[3];
  SML_HIP_CHECK(hipMemcpyAsync(h, total.get(), 3 * sizeof(double), hipMemcpyDeviceToHost, s));
  SML_HIP_CHECK(hipStreamSynchronize(s));
  if (h[1] == 0 || h[2] == 0) return 1.0;
  return h[0] / (h[1] * h[2]);
}

}  // namespace

bool DeviceEvalMetric(const std::string& name, const ObjParams& p, const double* score, const float* label,
                      const float* weight, int64_t n, void* stream, double* out) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (n <= 0 || n >= (int64_t(1) << 31)) return false;
  if (name == "auc") {
    *out = DeviceAUC(score, label, weight, n, s);
    return true;
  }
  int kind = -1;
  if ((name == "binary_logloss" || name == "binary_error") && p.kind == kObjBinary) kind = name == "binary_logloss" ? 0 : 1;
  const bool identity = p.kind == kObjRegression || p.kind == kObjL1 || p.kind == kObjHuber || p.kind == kObjFair ||
                        p.kind == kObjQuantile || p.kind == kObjMape;
  if (identity && (name == "l2" || name == "mse" || name == "rmse" || name == "l2_root" || name == "regression"))
    kind = 2;
  if (identity && (name == "l1" || name == "mae")) kind = 3;
  if (kind < 0) return false;
  PointLoss f{kind, p.sigmoid, score, label, weight};
  const int grid = Grid(n);
  DevBuf<double2> partial;
  partial.alloc(grid);
  hipLaunchKernelGGL(point_loss_kernel, dim3(grid), dim3(kThreads), 0, s, f, n, partial.get());
  SML_HIP_CHECK(hipGetLastError());
  std::vector<double2> h(grid);
  SML_HIP_CHECK(hipMemcpyAsync(h.data(), partial.get(), sizeof(double2) * grid, hipMemcpyDeviceToHost, s));
  SML_HIP_CHECK(hipStreamSynchronize(s));
  double a = 0, b = 0;
  for (const auto& v : h) { a += v.x; b += v.y; }
  double r = b > 0 ? a / b : 0.0;
  if (name == "rmse" || name == "l2_root") r = std::sqrt(r);
  *out = r;
  return true;
}

}  // namespace sml
