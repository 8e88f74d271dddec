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
//   multi_logloss / multi_error@k (softmax multiclass): the same reduce, one row's K class-major scores
//   per thread
//   ndcg@k / map@k: one wave64 per query; the top-k documents are selected k times by a wave arg-max
//   over (score desc, index asc) strictly after the previous pick - the order of the host's stable
//   sort, with no per-query scratch - and DCG / IDCG / AP accumulate in the host's order
// hipCUB is used only for the generic sort / scan / reduce-by-key.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "hip_common.h"
#include "objective.h"
#include "valid_gpu.h"

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

struct MultiLoss {
  int kind;  // 0 multi_logloss, 1 multi_error (top_k)
  int K, top_k;
  int64_t n;
  const double* score;
  const float* label;
  const float* weight;
  __device__ double2 operator()(int64_t i) const {
    const double w = weight ? weight[i] : 1.0;
    const int y = static_cast<int>(label[i]);
    double mx = score[i];
    for (int k = 1; k < K; ++k) mx = fmax(mx, score[k * n + i]);
    double s = 0.0;
    for (int k = 0; k < K; ++k) s += exp(score[k * n + i] - mx);
    const double py = exp(score[y * n + i] - mx) / s;
    double v;
    if (kind == 0) {
      v = -log(fmax(py, kEpsilon));
    } else {
      int rank = 0;
      for (int k = 0; k < K; ++k) rank += (exp(score[k * n + i] - mx) / s) > py;
      v = rank >= top_k ? 1.0 : 0.0;
    }
    return make_double2(v * w, w);
  }
};

template <class F>
__global__ void reduce_kernel(F f, int64_t n, double2* __restrict__ partial) {
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

// wave arg-max of (key desc, index asc); every lane returns the winner's index (-1: none)
__device__ __forceinline__ int WaveArgMax(double key, int idx) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double ok = __shfl_xor(key, off, 64);
    const int oi = __shfl_xor(idx, off, 64);
    if (oi >= 0 && (idx < 0 || ok > key || (ok == key && oi < idx))) { key = ok; idx = oi; }
  }
  return idx;
}

// one wave per query (grid-stride): ndcg@k (is_map 0) or map@k (1) of the query into per_query[q]
__global__ __launch_bounds__(64) void rank_metric_kernel(const double* __restrict__ score, const float* __restrict__ label,
                                                         const int32_t* __restrict__ qb, int nq, int k, int is_map,
                                                         const double* __restrict__ gain, int ngain,
                                                         double* __restrict__ per_query) {
  const int lane = threadIdx.x;
  for (int q = blockIdx.x; q < nq; q += gridDim.x) {
    const int b = qb[q], cnt = qb[q + 1] - qb[q];
    const int kk = min(k, cnt);
    auto gain_of = [&](float l) {
      const size_t li = static_cast<size_t>(static_cast<int>(l));  // the host's size_t clamp of an int label
      return gain[li < static_cast<size_t>(ngain - 1) ? li : static_cast<size_t>(ngain - 1)];
    };
    // picks strictly after (ps, pi) in (score desc, index asc) order
    double ps = INFINITY, ls = INFINITY;
    int pi = -1, li_prev = -1;
    double dcg = 0.0, idcg = 0.0, hits = 0.0, ap = 0.0;
    int npos = 0;
    if (is_map) {
      int c = 0;
      for (int j = lane; j < cnt; j += 64) c += label[b + j] > 0.5f;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
      npos = c;
    }
    for (int i = 0; i < kk; ++i) {
      double bk = -INFINITY;
      int bi = -1;
      for (int j = lane; j < cnt; j += 64) {
        const double s = score[b + j];
        const bool after = s < ps || (s == ps && j > pi);
        if (after && (bi < 0 || s > bk)) { bk = s; bi = j; }  // j ascends per lane: ties keep the lowest
      }
      const int w = WaveArgMax(bk, bi);
      if (w < 0) break;  // NaN scores are never picked (the host's order is undefined for them too)
      ps = score[b + w];
      pi = w;
      const float lw = label[b + w];
      if (is_map) {
        if (lw > 0.5f) { hits += 1.0; ap += hits / (i + 1.0); }
      } else {
        dcg += gain_of(lw) / log2(2.0 + i);
        // ideal order: labels desc (ties by index: the gains are equal either way)
        double lk = -INFINITY;
        int lj = -1;
        for (int j = lane; j < cnt; j += 64) {
          const double l = static_cast<double>(static_cast<int>(label[b + j]));
          const bool after = l < ls || (l == ls && j > li_prev);
          if (after && (lj < 0 || l > lk)) { lk = l; lj = j; }
        }
        const int wl = WaveArgMax(lk, lj);
        if (wl < 0) break;
        ls = static_cast<double>(static_cast<int>(label[b + wl]));
        li_prev = wl;
        idcg += gain_of(label[b + wl]) / log2(2.0 + i);
      }
    }
    if (lane == 0) {
      if (is_map) per_query[q] = npos > 0 ? ap / min(k, npos) : 1.0;
      else per_query[q] = idcg > 0 ? dcg / idcg : 1.0;
    }
  }
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

template <class F>
double ReduceRatio(F f, int64_t n, hipStream_t s) {
  const int grid = Grid(n);
  DevBuf<double2> partial;
  partial.alloc(grid);
  hipLaunchKernelGGL(reduce_kernel<F>, dim3(grid), dim3(kThreads), 0, s, f, n, partial.get());
  SML_HIP_CHECK(hipGetLastError());
  std::vector<double2> h(grid);
  SML_HIP_CHECK(hipMemcpyAsync(h.data(), partial.get(), sizeof(double2) * grid, hipMemcpyDeviceToHost, s));
  SML_HIP_CHECK(hipStreamSynchronize(s));
  double a = 0, b = 0;
  for (const auto& v : h) { a += v.x; b += v.y; }
  return b > 0 ? a / b : 0.0;
}

double DeviceRankMetric(const DeviceMetricInputs& in, int k, bool is_map, hipStream_t s) {
  if (in.nq <= 0) return 0.0;
  DevBuf<double> per_q, total;
  per_q.alloc(in.nq);
  total.alloc(1);
  const int grid = std::min(in.nq, 65536);
  hipLaunchKernelGGL(rank_metric_kernel, dim3(grid), dim3(64), 0, s, in.score, in.label, in.qb, in.nq, k,
                     is_map ? 1 : 0, in.gain, in.ngain, per_q.get());
  SML_HIP_CHECK(hipGetLastError());
  size_t t = 0;
  SML_HIP_CHECK(hipcub::DeviceReduce::Sum(nullptr, t, per_q.get(), total.get(), in.nq, s));
  DevBuf<uint8_t> tmp;
  tmp.alloc(std::max<size_t>(1, t));
  SML_HIP_CHECK(hipcub::DeviceReduce::Sum(tmp.get(), t, per_q.get(), total.get(), in.nq, s));
  double h = 0;
  SML_HIP_CHECK(hipMemcpyAsync(&h, total.get(), sizeof(double), hipMemcpyDeviceToHost, s));
  SML_HIP_CHECK(hipStreamSynchronize(s));
  return h / in.nq;
}

}  // namespace

bool DeviceEvalMetricFull(const std::string& name_in, const ObjParams& p, const DeviceMetricInputs& in, void* stream,
                          double* out) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t n = in.n;
  if (n <= 0 || n >= (int64_t(1) << 31)) return false;
  std::string name = name_in;
  int at = -1;
  const auto pos = name.find('@');
  if (pos != std::string::npos) {
    try { at = std::stoi(name.substr(pos + 1)); } catch (...) { return false; }
    name = name.substr(0, pos);
  }
  if (name == "ndcg" || name == "map") {
    if (!in.qb || in.nq <= 0 || (name == "ndcg" && (!in.gain || in.ngain <= 0))) return false;
    *out = DeviceRankMetric(in, at > 0 ? at : 5, name == "map", s);
    return true;
  }
  if (name == "multi_logloss" || name == "multi_error") {
    if (p.kind != kObjMulticlass || in.num_class < 2) return false;
    MultiLoss f{name == "multi_logloss" ? 0 : 1, in.num_class, at > 0 ? at : 1, n, in.score, in.label, in.weight};
    *out = ReduceRatio(f, n, s);
    return true;
  }
  if (at > 0 || in.num_class != 1) return false;
  if (name == "auc") {
    *out = DeviceAUC(in.score, in.label, in.weight, n, s);
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
  double r = ReduceRatio(PointLoss{kind, p.sigmoid, in.score, in.label, in.weight}, n, s);
  if (name == "rmse" || name == "l2_root") r = std::sqrt(r);
  *out = r;
  return true;
}

bool DeviceEvalMetric(const std::string& name, const ObjParams& p, const double* score, const float* label,
                      const float* weight, int64_t n, void* stream, double* out) {
  DeviceMetricInputs in;
  in.score = score; in.label = label; in.weight = weight; in.n = n;
  return DeviceEvalMetricFull(name, p, in, stream, out);
}

}  // namespace sml
