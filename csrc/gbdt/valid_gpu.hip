// K11 validation sets on the device (see valid_gpu.h). The tree traversal mirrors Tree::GetLeafByBins
// (tree.cpp) on the row-major bin matrix: numerical nodes compare the bin with the threshold bin after
// the missing-value routing (zero bin / NaN bin -> default side), categorical nodes test the bin in the
// node's bitset. One thread per row; the tree (~30 nodes) stays in L1/L2 for the whole launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>

#include "hip_common.h"
#include "valid_gpu.h"

namespace sml {
namespace {

struct DNode {
  int32_t fi;       // inner feature (byte offset in the row)
  uint32_t thr;     // threshold bin (numerical) / unused (categorical)
  int32_t left, right;
  int32_t dt;       // decision type: bit0 categorical, bit1 default left, bits2-3 missing type
  int32_t a, b;     // numerical: default bin, NaN bin; categorical: bitset word range [a, b)
  int32_t pad;
};

__global__ void valid_tree_kernel(const uint8_t* __restrict__ bins, int stride, int64_t n,
                                  const DNode* __restrict__ nodes, int num_leaves, const double* __restrict__ leaf,
                                  const uint32_t* __restrict__ cat_words, int op, double p, double* __restrict__ v) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    int node = 0;
    if (num_leaves > 1) {
      const uint8_t* row = bins + i * stride;
      while (node >= 0) {
        const DNode d = nodes[node];
        const uint32_t bin = row[d.fi];
        bool go_left;
        if (d.dt & 1) {
          const uint32_t word = bin >> 5;
          go_left = static_cast<int32_t>(word) < d.b - d.a && ((cat_words[d.a + word] >> (bin & 31)) & 1u);
        } else {
          const int missing = (d.dt >> 2) & 3;
          if ((missing == kMissingZero && bin == static_cast<uint32_t>(d.a)) ||
              (missing == kMissingNaN && bin == static_cast<uint32_t>(d.b)))
            go_left = (d.dt & 2) != 0;
          else
            go_left = bin <= d.thr;
        }
        node = go_left ? d.left : d.right;
      }
      node = ~node;
    }
    const double o = leaf[node];
    double x = v[i];
    switch (op) {
      case kValidAdd: x = x + p * o; break;
      case kValidAddSub: x = x + (o - p); break;
      case kValidRfAvg: x = p == 0.0 ? o : (x * p + o) / (p + 1.0); break;
      case kValidDart: x = x + (o - o / p); break;
      default: x = x + p;
    }
    v[i] = x;
  }
}

int GridFor(int64_t n) { return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(8192, (n + 255) / 256))); }

}  // namespace

struct DeviceValidSet::Impl {
  hipStream_t stream = nullptr;
  int64_t n = 0;
  int K = 1, stride = 0;
  std::shared_ptr<DeviceBins> dev_bins;  // the dataset's own HBM copy, when it has one here
  DevBuf<uint8_t> bins;                  // else an upload of its host bins
  const uint8_t* bins_ptr = nullptr;
  DevBuf<double> score, gain;
  DevBuf<float> label, weight;
  DevBuf<int32_t> qb;
  int nq = 0, ngain = 0;
  bool weighted = false;
  // per-tree staging: nodes | leaf values | categorical words, one H2D copy from pinned memory
  DevBuf<uint8_t> tree;
  uint8_t* pinned = nullptr;
  size_t pinned_cap = 0;
  hipEvent_t copied = nullptr;
  std::vector<int> default_bin, nan_bin;  // per inner feature
};

DeviceValidSet::DeviceValidSet(const Dataset& vd, const std::vector<double>& scores, int K,
                               const std::vector<double>& label_gain, int device, void* stream)
    : impl_(new Impl()) {
  Impl& m = *impl_;
  m.stream = static_cast<hipStream_t>(stream);
  m.n = vd.num_data;
  m.K = K;
  m.stride = vd.row_stride;
  const size_t nb = static_cast<size_t>(m.n) * m.stride;
  if (vd.dev_valid && vd.dev && vd.dev->device == device && vd.dev->rows) {
    m.dev_bins = vd.dev;
    m.bins_ptr = vd.dev->rows;
  } else {
    vd.EnsureHostBins();
    m.bins.alloc(std::max<size_t>(1, nb));
    if (nb) SML_HIP_CHECK(hipMemcpyAsync(m.bins.get(), vd.bins.data(), nb, hipMemcpyHostToDevice, m.stream));
    m.bins_ptr = m.bins.get();
  }
  if (scores.size() != static_cast<size_t>(m.n) * K) throw std::runtime_error("validation scores have the wrong size");
  m.score.alloc(std::max<size_t>(1, scores.size()));
  m.label.alloc(std::max<int64_t>(1, m.n));
  if (!scores.empty())
    SML_HIP_CHECK(hipMemcpyAsync(m.score.get(), scores.data(), sizeof(double) * scores.size(), hipMemcpyHostToDevice,
                                 m.stream));
  if (m.n)
    SML_HIP_CHECK(hipMemcpyAsync(m.label.get(), vd.label.data(), sizeof(float) * m.n, hipMemcpyHostToDevice, m.stream));
  if (!vd.weight.empty()) {
    m.weighted = true;
    m.weight.alloc(m.n);
    SML_HIP_CHECK(hipMemcpyAsync(m.weight.get(), vd.weight.data(), sizeof(float) * m.n, hipMemcpyHostToDevice, m.stream));
  }
  if (vd.query_boundaries.size() >= 2) {
    m.nq = static_cast<int>(vd.query_boundaries.size()) - 1;
    m.qb.alloc(vd.query_boundaries.size());
    SML_HIP_CHECK(hipMemcpyAsync(m.qb.get(), vd.query_boundaries.data(), sizeof(int32_t) * vd.query_boundaries.size(),
                                 hipMemcpyHostToDevice, m.stream));
  }
  if (!label_gain.empty()) {
    m.ngain = static_cast<int>(label_gain.size());
    m.gain.alloc(label_gain.size());
    SML_HIP_CHECK(hipMemcpyAsync(m.gain.get(), label_gain.data(), sizeof(double) * label_gain.size(),
                                 hipMemcpyHostToDevice, m.stream));
  }
  const int F = vd.ref.num_inner();
  m.default_bin.resize(F);
  m.nan_bin.resize(F);
  for (int f = 0; f < F; ++f) {
    const BinMapper& bm = vd.ref.mappers[vd.ref.used_features[f]];
    m.default_bin[f] = bm.default_bin;
    m.nan_bin[f] = bm.num_bin - 1;
  }
  SML_HIP_CHECK(hipEventCreateWithFlags(&m.copied, hipEventDisableTiming));
  // the host vectors above are only guaranteed read once the stream has passed the copies
  SML_HIP_CHECK(hipStreamSynchronize(m.stream));
}

DeviceValidSet::~DeviceValidSet() {
  if (!impl_) return;
  (void)hipStreamSynchronize(impl_->stream);
  if (impl_->pinned) (void)hipHostFree(impl_->pinned);
  if (impl_->copied) (void)hipEventDestroy(impl_->copied);
}

void DeviceValidSet::ApplyTree(const Tree& t, int k, int op, double p) {
  Impl& m = *impl_;
  if (m.n == 0) return;
  if (k < 0 || k >= m.K) throw std::runtime_error("validation tree class out of range");
  const int L = std::max(1, t.num_leaves);
  const int nn = L - 1;
  const size_t cat_words = t.cat_threshold_inner.size();
  const size_t node_bytes = sizeof(DNode) * nn, leaf_off = (node_bytes + 7) / 8 * 8;
  const size_t cat_off = leaf_off + sizeof(double) * L;
  const size_t bytes = cat_off + sizeof(uint32_t) * std::max<size_t>(1, cat_words);
  if (m.pinned) SML_HIP_CHECK(hipEventSynchronize(m.copied));  // the previous tree's copy has left the buffer
  if (bytes > m.pinned_cap) {
    if (m.pinned) SML_HIP_CHECK(hipHostFree(m.pinned));
    m.pinned_cap = std::max<size_t>(bytes, 4096);
    SML_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&m.pinned), m.pinned_cap, hipHostMallocDefault));
  }
  DNode* nodes = reinterpret_cast<DNode*>(m.pinned);
  const int F = static_cast<int>(m.default_bin.size());
  for (int i = 0; i < nn; ++i) {
    DNode& d = nodes[i];
    d.fi = t.split_feature_inner[i];
    if (d.fi < 0 || d.fi >= F || d.fi >= m.stride) throw std::runtime_error("validation tree feature out of range");
    d.thr = t.threshold_in_bin[i];
    d.left = t.left_child[i];
    d.right = t.right_child[i];
    d.dt = t.decision_type[i];
    if (d.dt & 1) {
      const int ci = static_cast<int>(t.threshold_in_bin[i]);
      d.a = t.cat_boundaries_inner[ci];
      d.b = t.cat_boundaries_inner[ci + 1];
    } else {
      d.a = m.default_bin[d.fi];
      d.b = m.nan_bin[d.fi];
    }
    d.pad = 0;
  }
  std::copy(t.leaf_value.begin(), t.leaf_value.begin() + L, reinterpret_cast<double*>(m.pinned + leaf_off));
  if (cat_words) std::copy(t.cat_threshold_inner.begin(), t.cat_threshold_inner.end(),
                           reinterpret_cast<uint32_t*>(m.pinned + cat_off));
  m.tree.alloc(bytes);
  SML_HIP_CHECK(hipMemcpyAsync(m.tree.get(), m.pinned, bytes, hipMemcpyHostToDevice, m.stream));
  SML_HIP_CHECK(hipEventRecord(m.copied, m.stream));
  const uint8_t* tb = m.tree.get();
  hipLaunchKernelGGL(valid_tree_kernel, dim3(GridFor(m.n)), dim3(256), 0, m.stream, m.bins_ptr, m.stride, m.n,
                     reinterpret_cast<const DNode*>(tb), t.num_leaves, reinterpret_cast<const double*>(tb + leaf_off),
                     reinterpret_cast<const uint32_t*>(tb + cat_off), op, p, m.score.get() + static_cast<size_t>(k) * m.n);
  SML_HIP_CHECK(hipGetLastError());
}

void DeviceValidSet::GetScores(std::vector<double>* out) {
  Impl& m = *impl_;
  out->resize(static_cast<size_t>(m.n) * m.K);
  if (!out->empty())
    SML_HIP_CHECK(hipMemcpyAsync(out->data(), m.score.get(), sizeof(double) * out->size(), hipMemcpyDeviceToHost,
                                 m.stream));
  SML_HIP_CHECK(hipStreamSynchronize(m.stream));
}

bool DeviceValidSet::Eval(const std::string& name, const ObjParams& p, int num_class, double* out) {
  Impl& m = *impl_;
  DeviceMetricInputs in;
  in.score = m.score.get();
  in.label = m.label.get();
  in.weight = m.weighted ? m.weight.get() : nullptr;
  in.n = m.n;
  in.num_class = num_class;
  in.qb = m.nq > 0 ? m.qb.get() : nullptr;
  in.nq = m.nq;
  in.gain = m.ngain > 0 ? m.gain.get() : nullptr;
  in.ngain = m.ngain;
  return DeviceEvalMetricFull(name, p, in, m.stream, out);
}

}  // namespace sml
