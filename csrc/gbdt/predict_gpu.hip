// K9: batched ensemble traversal. One thread scores one row; a block first
// stages its tile of rows in LDS (coalesced 16-B loads) so the per-node feature
// reads of every tree hit LDS instead of strided global memory.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <vector>

#include "booster.h"
#include "dataset.h"
#include "hip_common.h"
#include "trace.h"
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

// child reached from internal node gi (global index) for feature vector `row`
template <typename T>
__device__ __forceinline__ int NodeNext(const PackedEnsemble& e, int gi, const T* row, int ncols) {
  const int f = e.feat[gi];
  double x = f < ncols ? static_cast<double>(row[f]) : 0.0;
  const int fl = e.flags[gi];
  if (fl & 1) {
    int iv = isnan(x) ? -1 : static_cast<int>(x);
    bool left = false;
    if (iv >= 0) {
      const int w = iv >> 5;
      if (w < e.cat_len[gi]) left = (e.cat_words[e.cat_off[gi] + w] >> (iv & 31)) & 1u;
    }
    return left ? e.left[gi] : e.right[gi];
  }
  const int mt = (fl >> 2) & 3;
  if (isnan(x) && mt != kMissingNaN) x = 0.0;
  if ((mt == kMissingZero && fabs(x) <= kZeroThreshold) || (mt == kMissingNaN && isnan(x)))
    return (fl & 2) ? e.left[gi] : e.right[gi];
  return x <= e.thr[gi] ? e.left[gi] : e.right[gi];
}

template <typename T>
__device__ __forceinline__ int TraverseTree(const PackedEnsemble& e, int t, const T* row, int ncols) {
  if (e.num_leaves[t] <= 1) return 0;
  const int no = e.node_off[t];
  int node = 0;
  const int nl = e.num_leaves[t];
  for (int guard = 0; node >= 0 && guard < nl; ++guard) node = NodeNext(e, no + node, row, ncols);
  return node < 0 ? ~node : 0;
}

// T = double or float: float32 feature rows are scored as they are (a float converts to double exactly, so the
// threshold comparisons are those of the float64 path) - half the bytes over PCIe and in LDS.
template <bool LEAF, typename T = double>
__global__ __launch_bounds__(kPredThreads) void predict_kernel(PackedEnsemble e, const T* __restrict__ X,
                                                              int64_t n, int ncols, double* __restrict__ out,
                                                              int32_t* __restrict__ leaf_out, double avg_div) {
  __shared__ T tile[kPredThreads * kMaxStagedCols];
  const int64_t row0 = static_cast<int64_t>(blockIdx.x) * kPredThreads;
  const int rows = static_cast<int>(min<int64_t>(kPredThreads, n - row0));
  const bool staged = ncols <= kMaxStagedCols;
  if (staged) {
    const int total = rows * ncols;
    const T* src = X + row0 * ncols;
    for (int i = threadIdx.x; i < total; i += kPredThreads) tile[i] = src[i];
    __syncthreads();
  }
  const int r = threadIdx.x;
  if (r >= rows) return;
  const T* row = staged ? tile + r * ncols : X + (row0 + r) * ncols;
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


// ---------------------------------------------------------------------------
// K10: path-dependent TreeSHAP on the GPU (reference: featuresShap,
// lightgbm/.../booster/LightGBMBooster.scala:418-427 -> LGBM contrib predict).
//
// Lundberg's recursion visits every root->leaf path; at a leaf the SHAP
// contribution only depends on that path's UNIQUE features, each with
//   zero_fraction = product of cover ratios of its nodes on the path and
//   one_fraction  = 1 if the row follows the path at all of its nodes, else 0.
// So the recursion is flattened on the host into leaf paths, and the paths are
// bin-packed into wave64s, one lane per path element (lane 0 of a path is the
// root element). EXTEND is then a lane shift (one shuffle per depth step) and
// each lane computes its own UNWOUND sum with broadcasts of the path weights:
// O(depth) shuffles per (row, path) instead of O(depth^2) scalar work.
// A block owns a tile of rows: row values and the phi accumulators live in LDS
// and every wave of the block strides over the path bins.
struct ShapLanes {
  const int32_t* feat;     // -1 root element / unused lane -2
  const double* zf;        // zero fraction
  const int32_t* cond_off; // this element's (node, expected child) list
  const int32_t* cond_cnt;
  const int32_t* elem;     // element index within its path (0 = root)
  const int32_t* m;        // number of unique features of the path
  const int32_t* k;        // output class of the path's tree
  const double* lval;      // leaf value of the path
  const int32_t* cond_gi;
  const int32_t* cond_child;
  const int32_t* bin_maxm; // per bin: max m over its paths
  int num_bins;
};

constexpr int kShapThreads = 256;

template <bool LDS_ACC>
__global__ __launch_bounds__(kShapThreads) void shap_kernel(PackedEnsemble e, ShapLanes L, const double* __restrict__ X,
                                                            int64_t n, int ncols, int rows_per_block, int stage_cols,
                                                            int nf1, double* __restrict__ out) {
  const int phi_stride = nf1 * e.K;
  extern __shared__ double smem[];
  __shared__ double inv[72];
  const int64_t row0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int R = static_cast<int>(min<int64_t>(rows_per_block, n - row0));
  double* phi = smem;                                             // [rows_per_block][phi_stride] (LDS_ACC)
  double* rows = smem + (LDS_ACC ? rows_per_block * phi_stride : 0);  // [rows_per_block][ncols] when staged
  for (int i = threadIdx.x; i < 72; i += kShapThreads) inv[i] = i ? 1.0 / i : 0.0;
  if (LDS_ACC)
    for (int i = threadIdx.x; i < rows_per_block * phi_stride; i += kShapThreads) phi[i] = 0.0;
  if (stage_cols)
    for (int i = threadIdx.x; i < R * ncols; i += kShapThreads) rows[i] = X[row0 * ncols + i];
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  for (int b = wave; b < L.num_bins; b += kShapThreads / 64) {
    const int li = b * 64 + lane;
    const int feat = L.feat[li];
    const bool used = feat >= -1;
    const int el = used ? L.elem[li] : 0;
    const int m = used ? L.m[li] : 0;
    const int base = lane - el;  // lane of this path's root element
    const double zf = used ? L.zf[li] : 1.0;
    const double izf = zf != 0.0 ? 1.0 / zf : 0.0;
    const int coff = used ? L.cond_off[li] : 0, ccnt = used ? L.cond_cnt[li] : 0;
    const int kk = used ? L.k[li] : 0;
    const double lv = used ? L.lval[li] : 0.0;
    const int maxm = L.bin_maxm[b];
    for (int r = 0; r < R; ++r) {
      const double* row = stage_cols ? rows + r * ncols : X + (row0 + r) * ncols;
      // one fraction: does the row follow the path at every node of this feature?
      double of = 1.0;
      for (int c = 0; c < ccnt; ++c)
        if (NodeNext(e, L.cond_gi[coff + c], row, ncols) != L.cond_child[coff + c]) of = 0.0;
      // EXTEND with elements 1..m (element 0, the root, starts the path with weight 1)
      double w = (el == 0) ? 1.0 : 0.0;
      for (int d = 1; d <= maxm; ++d) {
        const int src_d = min(base + d, 63);
        const double zf_d = __shfl(zf, src_d, 64);
        const double of_d = __shfl(of, src_d, 64);
        const double wprev = __shfl(w, max(lane - 1, 0), 64);
        if (used && d <= m && el <= d) {
          const double a = inv[d + 1];
          w = zf_d * w * (d - el) * a + (el > 0 ? of_d * wprev * el * a : 0.0);
        }
      }
      // UNWOUND sum for this lane's element, then its contribution
      double next = __shfl(w, min(base + m, 63), 64);
      double total = 0.0;
      for (int j = maxm - 1; j >= 0; --j) {
        const double wj = __shfl(w, min(base + max(j, 0), 63), 64);
        if (used && el > 0 && j < m) {
          if (of != 0.0) {
            const double tmp = next * (m + 1) * inv[j + 1];
            total += tmp;
            next = wj - tmp * zf * (m - j) * inv[m + 1];
          } else if (zf != 0.0) {
            total += wj * izf * (m + 1) * inv[m - j];
          }
        }
      }
      if (used && el > 0) {
        const double contrib = total * (of - zf) * lv;
        if (LDS_ACC)
          atomicAdd(&phi[r * phi_stride + kk * nf1 + feat], contrib);
        else
          atomicAdd(&out[(row0 + r) * phi_stride + kk * nf1 + feat], contrib);
      }
    }
  }
  if (LDS_ACC) {
    __syncthreads();
    for (int i = threadIdx.x; i < R * phi_stride; i += kShapThreads) out[row0 * phi_stride + i] += phi[i];
  }
}

}  // namespace

struct GpuPredictor::Impl {
  DevBuf<int32_t> ints;
  DevBuf<double> dbls;
  DevBuf<uint32_t> cats;
  DevBuf<double> x, o;
  DevBuf<int32_t> lo;
  PackedEnsemble e{};
  // TreeSHAP tables (built on first use)
  bool shap_ready = false, shap_ok = false;
  DevBuf<int32_t> s_ints;
  DevBuf<double> s_dbls;
  ShapLanes sl{};
  std::vector<double> bias;  // per class: sum of tree expected values
  int t0 = 0, t1 = 0;
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
  impl_->t0 = range.first;
  impl_->t1 = range.second;
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
  TraceRange tr("sml::Predict");
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

// One device pass over a batch in its own dtype: rows go to HBM through the pinned multi-threaded staging
// pipeline (UploadPinned) in chunks, chunk c+1's upload overlapping chunk c's traversal, and the raw scores
// come back once; the transformed outputs (probabilities) are derived from them on the host
// (Booster::ConvertOutputs), so a transform never runs the ensemble twice.
void GpuPredictor::PredictRaw(const void* X, bool f32, int64_t n, int ncols, double* out) {
  TraceRange tr("sml::PredictRaw");
  if (n <= 0) return;
  const size_t esz = f32 ? 4 : 8;
  const int64_t chunk = std::max<int64_t>(kPredThreads, (static_cast<int64_t>(256) << 20) / std::max<int64_t>(1, ncols * esz));
  const int64_t rows_buf = std::min<int64_t>(n, chunk);
  impl_->x.alloc((2 * static_cast<size_t>(rows_buf) * ncols * esz + sizeof(double) - 1) / sizeof(double));  // 2 chunk buffers
  impl_->o.alloc(static_cast<size_t>(n) * num_out_);
  hipStream_t s = impl_->stream;
  char* xb[2] = {reinterpret_cast<char*>(impl_->x.get()),
                 reinterpret_cast<char*>(impl_->x.get()) + static_cast<size_t>(rows_buf) * ncols * esz};
  hipEvent_t done[2] = {nullptr, nullptr};
  for (auto& e : done) SML_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  bool used[2] = {false, false};
  try {
    int k = 0;
    for (int64_t r0 = 0; r0 < n; r0 += chunk, k ^= 1) {
      const int64_t m = std::min(chunk, n - r0);
      if (used[k]) SML_HIP_CHECK(hipEventSynchronize(done[k]));  // the traversal that read this buffer finished
      UploadPinned(static_cast<const char*>(X) + static_cast<size_t>(r0) * ncols * esz, xb[k],
                   static_cast<size_t>(m) * ncols * esz);
      const int grid = static_cast<int>((m + kPredThreads - 1) / kPredThreads);
      if (f32)
        hipLaunchKernelGGL((predict_kernel<false, float>), dim3(grid), dim3(kPredThreads), 0, s, impl_->e,
                           reinterpret_cast<const float*>(xb[k]), m, ncols, impl_->o.get() + r0 * num_out_,
                           static_cast<int32_t*>(nullptr), impl_->avg_div);
      else
        hipLaunchKernelGGL((predict_kernel<false, double>), dim3(grid), dim3(kPredThreads), 0, s, impl_->e,
                           reinterpret_cast<const double*>(xb[k]), m, ncols, impl_->o.get() + r0 * num_out_,
                           static_cast<int32_t*>(nullptr), impl_->avg_div);
      SML_HIP_CHECK(hipGetLastError());
      SML_HIP_CHECK(hipEventRecord(done[k], s));
      used[k] = true;
    }
    SML_HIP_CHECK(hipMemcpyAsync(out, impl_->o.get(), sizeof(double) * n * num_out_, hipMemcpyDeviceToHost, s));
    SML_HIP_CHECK(hipStreamSynchronize(s));
  } catch (...) {
    (void)hipStreamSynchronize(s);
    for (auto& e : done) (void)hipEventDestroy(e);
    throw;
  }
  for (auto& e : done) (void)hipEventDestroy(e);
}

void GpuPredictor::PredictLeaf(const double* X, int64_t n, int ncols, int32_t* out) {
  TraceRange tr("sml::PredictLeaf");
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


namespace {
struct ShapLane {
  int feat = -2;
  double zf = 1.0;
  int coff = 0, ccnt = 0, elem = 0, m = 0, k = 0;
  double lval = 0.0;
};

double NodeCount(const Tree& t, int c) {
  return c >= 0 ? static_cast<double>(t.internal_count[c]) : static_cast<double>(t.leaf_count[~c]);
}

// flatten one tree into leaf paths of unique-feature elements
void CollectPaths(const Tree& t, int node_base, int k, std::vector<std::pair<int, int>>* stack,
                  int node, std::vector<std::vector<ShapLane>>* paths, std::vector<int32_t>* cgi,
                  std::vector<int32_t>* cchild) {
  for (int side = 0; side < 2; ++side) {
    const int child = side ? t.right_child[node] : t.left_child[node];
    stack->push_back({node, child});
    if (child >= 0) {
      CollectPaths(t, node_base, k, stack, child, paths, cgi, cchild);
    } else {
      std::vector<ShapLane> p(1);
      p[0].feat = -1;
      std::vector<int> order;  // unique features in first-occurrence order
      std::vector<std::vector<std::pair<int, int>>> conds;
      for (const auto& nc : *stack) {
        const int f = t.split_feature[nc.first];
        size_t j = 0;
        while (j < order.size() && order[j] != f) ++j;
        if (j == order.size()) {
          order.push_back(f);
          conds.emplace_back();
          p.emplace_back();
          p.back().feat = f;
        }
        const double w = NodeCount(t, nc.first);
        p[j + 1].zf *= w > 0 ? NodeCount(t, nc.second) / w : 0.0;
        conds[j].push_back({node_base + nc.first, nc.second});
      }
      const int m = static_cast<int>(order.size());
      for (int j = 0; j <= m; ++j) {
        p[j].elem = j;
        p[j].m = m;
        p[j].k = k;
        p[j].lval = t.leaf_value[~child];
        if (j > 0) {
          p[j].coff = static_cast<int>(cgi->size());
          p[j].ccnt = static_cast<int>(conds[j - 1].size());
          for (const auto& c : conds[j - 1]) {
            cgi->push_back(c.first);
            cchild->push_back(c.second);
          }
        }
      }
      paths->push_back(std::move(p));
    }
    stack->pop_back();
  }
}
}  // namespace

bool GpuPredictor::BuildShap() {
  Impl& I = *impl_;
  I.shap_ready = true;
  const auto& trees = booster_->trees();
  const int K = num_out_;
  I.bias.assign(K, 0.0);
  std::vector<std::vector<ShapLane>> paths;
  std::vector<int32_t> cgi, cchild;
  std::vector<std::pair<int, int>> stack;
  int node_base = 0;
  for (int t = I.t0; t < I.t1; ++t) {
    const Tree& tr = trees[t];
    I.bias[t % K] += tr.ExpectedValue();
    if (tr.num_leaves > 1) CollectPaths(tr, node_base, t % K, &stack, 0, &paths, &cgi, &cchild);
    node_base += std::max(0, tr.num_leaves - 1);
  }
  for (const auto& p : paths)
    if (p.size() > 64) return I.shap_ok = false;  // > 63 unique features on one path: host fallback
  // bin-pack paths into wave64s (best fit, longest first)
  std::vector<int> idx(paths.size());
  for (size_t i = 0; i < idx.size(); ++i) idx[i] = static_cast<int>(i);
  std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return paths[a].size() > paths[b].size(); });
  std::vector<std::vector<int>> by_room(65);  // bins indexed by remaining lanes
  std::vector<int> fill;                      // lanes used per bin
  std::vector<std::vector<int>> bins;
  for (int pi : idx) {
    const int len = static_cast<int>(paths[pi].size());
    int bin = -1;
    for (int room = len; room <= 64 && bin < 0; ++room)
      if (!by_room[room].empty()) { bin = by_room[room].back(); by_room[room].pop_back(); }
    if (bin < 0) { bin = static_cast<int>(bins.size()); bins.emplace_back(); fill.push_back(0); }
    bins[bin].push_back(pi);
    fill[bin] += len;
    by_room[64 - fill[bin]].push_back(bin);
  }
  const int nb = static_cast<int>(bins.size());
  const size_t NL = static_cast<size_t>(std::max(1, nb)) * 64;
  std::vector<int32_t> feat(NL, -2), coff(NL, 0), ccnt(NL, 0), elem(NL, 0), mm(NL, 0), kk(NL, 0), bmax(std::max(1, nb), 0);
  std::vector<double> zf(NL, 1.0), lv(NL, 0.0);
  for (int b = 0; b < nb; ++b) {
    int lane = 0;
    for (int pi : bins[b]) {
      for (const ShapLane& l : paths[pi]) {
        const size_t i = static_cast<size_t>(b) * 64 + lane++;
        feat[i] = l.feat; zf[i] = l.zf; coff[i] = l.coff; ccnt[i] = l.ccnt; elem[i] = l.elem; mm[i] = l.m;
        kk[i] = l.k; lv[i] = l.lval;
      }
      bmax[b] = std::max<int32_t>(bmax[b], static_cast<int32_t>(paths[pi].size()) - 1);
    }
  }
  if (cgi.empty()) { cgi.push_back(0); cchild.push_back(0); }
  std::vector<int32_t> ints;
  for (auto* v : {&feat, &coff, &ccnt, &elem, &mm, &kk}) ints.insert(ints.end(), v->begin(), v->end());
  const size_t C = cgi.size();
  ints.insert(ints.end(), cgi.begin(), cgi.end());
  ints.insert(ints.end(), cchild.begin(), cchild.end());
  ints.insert(ints.end(), bmax.begin(), bmax.end());
  std::vector<double> dbls = zf;
  dbls.insert(dbls.end(), lv.begin(), lv.end());
  I.s_ints.alloc(ints.size());
  I.s_dbls.alloc(dbls.size());
  SML_HIP_CHECK(hipMemcpy(I.s_ints.get(), ints.data(), ints.size() * 4, hipMemcpyHostToDevice));
  SML_HIP_CHECK(hipMemcpy(I.s_dbls.get(), dbls.data(), dbls.size() * 8, hipMemcpyHostToDevice));
  int32_t* p = I.s_ints.get();
  ShapLanes& S = I.sl;
  S.feat = p; p += NL;
  S.cond_off = p; p += NL;
  S.cond_cnt = p; p += NL;
  S.elem = p; p += NL;
  S.m = p; p += NL;
  S.k = p; p += NL;
  S.cond_gi = p; p += C;
  S.cond_child = p; p += C;
  S.bin_maxm = p;
  S.zf = I.s_dbls.get();
  S.lval = I.s_dbls.get() + NL;
  S.num_bins = nb;
  return I.shap_ok = true;
}

bool GpuPredictor::PredictContrib(const double* X, int64_t n, int ncols, double* out) {
  TraceRange tr("sml::PredictContrib");
  if (!impl_->shap_ready) BuildShap();
  if (!impl_->shap_ok) return false;
  Impl& I = *impl_;
  const int K = num_out_;
  const int nf1 = booster_->NumFeatures() + 1;
  const int64_t osz = static_cast<int64_t>(nf1) * K;
  if (n <= 0) return true;
  I.x.alloc(static_cast<size_t>(n) * ncols);
  I.o.alloc(static_cast<size_t>(n) * osz);
  hipStream_t s = I.stream;
  SML_HIP_CHECK(hipMemcpyAsync(I.x.get(), X, sizeof(double) * n * ncols, hipMemcpyHostToDevice, s));
  SML_HIP_CHECK(hipMemsetAsync(I.o.get(), 0, sizeof(double) * n * osz, s));
  if (I.sl.num_bins > 0) {
    int R = 16;
    while (R > 2 && static_cast<int64_t>(R) * osz * 8 > 48 * 1024) R >>= 1;
    const bool lds_acc = static_cast<int64_t>(R) * osz * 8 <= 48 * 1024;
    const int stage = static_cast<int64_t>(R) * ncols * 8 <= 16 * 1024 ? 1 : 0;
    const size_t lds = sizeof(double) * ((lds_acc ? R * osz : 0) + (stage ? R * ncols : 0));
    const int grid = static_cast<int>((n + R - 1) / R);
    if (lds_acc)
      hipLaunchKernelGGL(shap_kernel<true>, dim3(grid), dim3(kShapThreads), lds, s, I.e, I.sl, I.x.get(), n, ncols,
                         R, stage, nf1, I.o.get());
    else
      hipLaunchKernelGGL(shap_kernel<false>, dim3(grid), dim3(kShapThreads), lds, s, I.e, I.sl, I.x.get(), n, ncols,
                         R, stage, nf1, I.o.get());
    SML_HIP_CHECK(hipGetLastError());
  }
  SML_HIP_CHECK(hipMemcpyAsync(out, I.o.get(), sizeof(double) * n * osz, hipMemcpyDeviceToHost, s));
  SML_HIP_CHECK(hipStreamSynchronize(s));
  const double div = I.avg_div;
  for (int64_t i = 0; i < n; ++i) {
    double* o = out + i * osz;
    for (int k = 0; k < K; ++k) o[k * nf1 + nf1 - 1] += I.bias[k];
    if (div != 1.0)
      for (int64_t j = 0; j < osz; ++j) o[j] /= div;
  }
  return true;
}

}  // namespace sml
