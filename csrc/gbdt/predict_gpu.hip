// K9: batched ensemble traversal. One thread scores one row; a block first
// stages its tile of rows in LDS (coalesced 16-B loads) so the per-node feature
// reads of every tree hit LDS instead of strided global memory.
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <vector>

#include "booster.h"
#include "hip_common.h"
#include "predictor.h"

namespace sml {
namespace {

constexpr int kPredThreads = 128;
constexpr int kMaxStagedCols = 64;  // 128 rows * 64 cols * 8 B = 64 KiB

struct PackedEnsemble {
  const int32_t* node_off;   // per tree
  const int32_t* leaf_off;   // per tree
  const int32_t* num_leaves; // per tree
  const int32_t* feat;
  const double* thr;
  const int32_t* flags;      // bit0 cat, bit1 default_left, bits2-3 missing
  const int32_t* left;
  const int32_t* right;
  const int32_t* cat_off;    // per node: offset into cat_words
  const int32_t* cat_len;    // per node: number of words
  const uint32_t* cat_words;
  const double* lval;
  int num_trees;
  int K;
};

__device__ __forceinline__ int TraverseTree(const PackedEnsemble& e, int t, const double* row, int ncols) {
  if (e.num_leaves[t] <= 1) return 0;
  const int no = e.node_off[t];
  int node = 0;
  const int nl = e.num_leaves[t];
  for (int guard = 0; node >= 0 && guard < nl; ++guard) {
    const int gi = no + node;
    const int f = e.feat[gi];
    double x = f < ncols ? row[f] : 0.0;
    const int fl = e.flags[gi];
    if (fl & 1) {
      int iv = isnan(x) ? -1 : static_cast<int>(x);
      bool left = false;
      if (iv >= 0) {
        const int w = iv >> 5;
        if (w < e.cat_len[gi]) left = (e.cat_words[e.cat_off[gi] + w] >> (iv & 31)) & 1u;
      }
      node = left ? e.left[gi] : e.right[gi];
    } else {
      const int mt = (fl >> 2) & 3;
      if (isnan(x) && mt != kMissingNaN) x = 0.0;
      if ((mt == kMissingZero && fabs(x) <= kZeroThreshold) || (mt == kMissingNaN && isnan(x))) {
        node = (fl & 2) ? e.left[gi] : e.right[gi];
      } else {
        node = x <= e.thr[gi] ? e.left[gi] : e.right[gi];
      }
    }
  }
  return node < 0 ? ~node : 0;
}

template <bool LEAF>
__global__ __launch_bounds__(kPredThreads) void predict_kernel(PackedEnsemble e, const double* __restrict__ X,
                                                              int64_t n, int ncols, double* __restrict__ out,
                                                              int32_t* __restrict__ leaf_out, double avg_div) {
  __shared__ double tile[kPredThreads * kMaxStagedCols];
  const int64_t row0 = static_cast<int64_t>(blockIdx.x) * kPredThreads;
  const int rows = static_cast<int>(min<int64_t>(kPredThreads, n - row0));
  const bool staged = ncols <= kMaxStagedCols;
  if (staged) {
    const int total = rows * ncols;
    const double* src = X + row0 * ncols;
    for (int i = threadIdx.x; i < total; i += kPredThreads) tile[i] = src[i];
    __syncthreads();
  }
  const int r = threadIdx.x;
  if (r >= rows) return;
  const double* row = staged ? tile + r * ncols : X + (row0 + r) * ncols;
  const int64_t gi = row0 + r;
  if (LEAF) {
    for (int t = 0; t < e.num_trees; ++t) leaf_out[gi * e.num_trees + t] = TraverseTree(e, t, row, ncols);
    return;
  }
  double acc[16];
  const int K = e.K;
  for (int k = 0; k < K && k < 16; ++k) acc[k] = 0.0;
  for (int t = 0; t < e.num_trees; ++t) {
    const int leaf = TraverseTree(e, t, row, ncols);
    const double v = e.lval[e.leaf_off[t] + leaf];
    const int k = t % K;
    if (k < 16) acc[k] += v;
  }
  for (int k = 0; k < K && k < 16; ++k) out[gi * K + k] = acc[k] / avg_div;
}

}  // namespace

struct GpuPredictor::Impl {
  DevBuf<int32_t> ints;
  DevBuf<double> dbls;
  DevBuf<uint32_t> cats;
  DevBuf<double> x, o;
  DevBuf<int32_t> lo;
  PackedEnsemble e{};
  hipStream_t stream = nullptr;
  double avg_div = 1.0;
  ~Impl() { if (stream) { (void)hipStreamSynchronize(stream); (void)hipStreamDestroy(stream); } }
};

GpuPredictor::GpuPredictor(const Booster& b, int start_iteration, int num_iteration, int device)
    : impl_(new Impl()), booster_(&b) {
  if (device >= 0) SML_HIP_CHECK(hipSetDevice(device));
  SML_HIP_CHECK(hipStreamCreateWithFlags(&impl_->stream, hipStreamNonBlocking));
  auto range = b.TreeRangePublic(start_iteration, num_iteration);
  const auto& trees = b.trees();
  const int K = b.NumModelPerIteration();
  if (K > 16) throw std::runtime_error("GPU predictor supports up to 16 outputs per iteration");
  num_out_ = K;
  num_trees_ = range.second - range.first;
  std::vector<int32_t> node_off, leaf_off, nleaves, feat, flags, left, right, cat_off, cat_len;
  std::vector<double> thr, lval;
  std::vector<uint32_t> cw;
  for (int t = range.first; t < range.second; ++t) {
    const Tree& tr = trees[t];
    node_off.push_back(static_cast<int32_t>(feat.size()));
    leaf_off.push_back(static_cast<int32_t>(lval.size()));
    nleaves.push_back(tr.num_leaves);
    for (int node = 0; node < tr.num_leaves - 1; ++node) {
      feat.push_back(tr.split_feature[node]);
      thr.push_back(tr.threshold[node]);
      flags.push_back(static_cast<int32_t>(tr.decision_type[node]) & 0xF);
      left.push_back(tr.left_child[node]);
      right.push_back(tr.right_child[node]);
      if (tr.decision_type[node] & 1) {
        int ci = static_cast<int>(tr.threshold[node]);
        int s = tr.cat_boundaries[ci], e2 = tr.cat_boundaries[ci + 1];
        cat_off.push_back(static_cast<int32_t>(cw.size()));
        cat_len.push_back(e2 - s);
        for (int w = s; w < e2; ++w) cw.push_back(tr.cat_threshold[w]);
      } else {
        cat_off.push_back(0);
        cat_len.push_back(0);
      }
    }
    for (int l = 0; l < tr.num_leaves; ++l) lval.push_back(tr.leaf_value[l]);
  }
  if (feat.empty()) { feat.push_back(0); thr.push_back(0); flags.push_back(0); left.push_back(0); right.push_back(0); cat_off.push_back(0); cat_len.push_back(0); }
  if (cw.empty()) cw.push_back(0);
  if (lval.empty()) lval.push_back(0);
  const int T = std::max(1, num_trees_);
  node_off.resize(T, 0); leaf_off.resize(T, 0); nleaves.resize(T, 1);
  const size_t NN = feat.size();
  std::vector<int32_t> ints;
  ints.insert(ints.end(), node_off.begin(), node_off.end());
  ints.insert(ints.end(), leaf_off.begin(), leaf_off.end());
  ints.insert(ints.end(), nleaves.begin(), nleaves.end());
  ints.insert(ints.end(), feat.begin(), feat.end());
  ints.insert(ints.end(), flags.begin(), flags.end());
  ints.insert(ints.end(), left.begin(), left.end());
  ints.insert(ints.end(), right.begin(), right.end());
  ints.insert(ints.end(), cat_off.begin(), cat_off.end());
  ints.insert(ints.end(), cat_len.begin(), cat_len.end());
  std::vector<double> dbls = thr;
  dbls.insert(dbls.end(), lval.begin(), lval.end());
  impl_->ints.alloc(ints.size());
  impl_->dbls.alloc(dbls.size());
  impl_->cats.alloc(cw.size());
  SML_HIP_CHECK(hipMemcpy(impl_->ints.get(), ints.data(), ints.size() * 4, hipMemcpyHostToDevice));
  SML_HIP_CHECK(hipMemcpy(impl_->dbls.get(), dbls.data(), dbls.size() * 8, hipMemcpyHostToDevice));
  SML_HIP_CHECK(hipMemcpy(impl_->cats.get(), cw.data(), cw.size() * 4, hipMemcpyHostToDevice));
  int32_t* p = impl_->ints.get();
  PackedEnsemble& e = impl_->e;
  e.node_off = p; p += T;
  e.leaf_off = p; p += T;
  e.num_leaves = p; p += T;
  e.feat = p; p += NN;
  e.flags = p; p += NN;
  e.left = p; p += NN;
  e.right = p; p += NN;
  e.cat_off = p; p += NN;
  e.cat_len = p; p += NN;
  e.thr = impl_->dbls.get();
  e.lval = impl_->dbls.get() + NN;
  e.cat_words = impl_->cats.get();
  e.num_trees = num_trees_;
  e.K = K;
  impl_->avg_div = (b.average_output() && num_trees_ > 0) ? static_cast<double>(num_trees_ / K) : 1.0;
}

GpuPredictor::~GpuPredictor() = default;

void GpuPredictor::Predict(const double* X, int64_t n, int ncols, bool normal, double* out) {
  if (n <= 0) return;
  impl_->x.alloc(static_cast<size_t>(n) * ncols);
  impl_->o.alloc(static_cast<size_t>(n) * num_out_);
  hipStream_t s = impl_->stream;
  SML_HIP_CHECK(hipMemcpyAsync(impl_->x.get(), X, sizeof(double) * n * ncols, hipMemcpyHostToDevice, s));
  const int grid = static_cast<int>((n + kPredThreads - 1) / kPredThreads);
  hipLaunchKernelGGL(predict_kernel<false>, dim3(grid), dim3(kPredThreads), 0, s, impl_->e, impl_->x.get(), n, ncols,
                     impl_->o.get(), static_cast<int32_t*>(nullptr), impl_->avg_div);
  SML_HIP_CHECK(hipGetLastError());
  SML_HIP_CHECK(hipMemcpyAsync(out, impl_->o.get(), sizeof(double) * n * num_out_, hipMemcpyDeviceToHost, s));
  SML_HIP_CHECK(hipStreamSynchronize(s));
  if (normal) {
    std::vector<double> raw(out, out + n * num_out_);
    booster_->ConvertOutputs(raw.data(), n, out);
  }
}

void GpuPredictor::PredictLeaf(const double* X, int64_t n, int ncols, int32_t* out) {
  if (n <= 0 || num_trees_ == 0) return;
  impl_->x.alloc(static_cast<size_t>(n) * ncols);
  impl_->lo.alloc(static_cast<size_t>(n) * num_trees_);
  hipStream_t s = impl_->stream;
  SML_HIP_CHECK(hipMemcpyAsync(impl_->x.get(), X, sizeof(double) * n * ncols, hipMemcpyHostToDevice, s));
  const int grid = static_cast<int>((n + kPredThreads - 1) / kPredThreads);
  hipLaunchKernelGGL(predict_kernel<true>, dim3(grid), dim3(kPredThreads), 0, s, impl_->e, impl_->x.get(), n, ncols,
                     static_cast<double*>(nullptr), impl_->lo.get(), 1.0);
  SML_HIP_CHECK(hipGetLastError());
  SML_HIP_CHECK(hipMemcpyAsync(out, impl_->lo.get(), sizeof(int32_t) * n * num_trees_, hipMemcpyDeviceToHost, s));
  SML_HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace sml
