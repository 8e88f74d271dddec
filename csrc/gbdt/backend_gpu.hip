// HIP/CDNA4 training backend: the whole leaf-wise tree growth runs on the
// MI355X with the binned matrix, gradients, scores and row partitions resident
// in HBM. Kernels:
//   K2 gradients      grad_kernel           one thread per row, fused objective
//   K3 histogram      hist_kernel           LDS-privatised per-block histograms
//                                           (ds_add_f32), fixed-order slab reduce
//   K4 subtraction    find_split_kernel     larger child = parent - smaller
//   K5 split search   find_split_kernel     one block per (feature, child), bins
//                                           on lanes, fp64 prefix scan
//   K6 partition      part_count/scatter    stable 2-pass partition, wave ballots
//   K7 score update   score_kernel          tree traversal on bins
// The host enqueues a fixed kernel sequence per split; which leaf is split,
// its row range and the split itself live in device memory, so a tree is built
// without any host round trip (the tree is read back once at the end).
// Data-parallel training inserts an RCCL allreduce of the smaller child's
// histogram between the slab reduce and the split search (C2 over xGMI).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <numeric>
#include <vector>

#include "backend.h"
#include "hip_common.h"

namespace sml {
namespace {

constexpr int kBinsPerFeature = 256;
constexpr int kHistThreads = 512;
constexpr int kFeatPerGroup = 32;          // 8 dwords of bins per block
constexpr int kHistStride = 257;           // padded LDS row (bank spread)
constexpr int kMaxHistBlocks = 512;        // = resident capacity at 2 blocks/CU
constexpr int kMinRowsPerHistBlock = 2048;
constexpr int kReduceSplit = 8;
constexpr int kPartThreads = 512;
constexpr int kMaxPartBlocks = 1024;
constexpr int kMinRowsPerPartBlock = 4096;

struct DLeaf {
  int32_t begin, count, buf, depth;  // local row segment; buf: -1 physical, 0/1 ping-pong
  int64_t gcount;                    // global rows
  double sum_g, sum_h;
  int32_t slot, pad;
};

struct DState {
  int32_t num_leaves, done, split_leaf, new_leaf;
  int32_t small_leaf, large_leaf, parent_slot, max_leaves;
  int32_t phase;  // 0 = root, 1 = children
  // segment of the leaf being partitioned and the partition result
  int32_t pbegin, pcount, pbuf, ptotal;
  int32_t pad;
};

// Row segment of the leaf whose histogram is built next (root or smaller child).
__device__ __forceinline__ DLeaf HistSeg(const DState* st, const DLeaf* leaves) {
  if (st->phase == 0) return leaves[0];
  DLeaf L;
  const int ob = st->pbuf == 0 ? 1 : 0;
  L.buf = ob;
  if (st->small_leaf == st->split_leaf) { L.begin = st->pbegin; L.count = st->ptotal; }
  else { L.begin = st->pbegin + st->ptotal; L.count = st->pcount - st->ptotal; }
  return L;
}

struct DTree {  // device tree arrays (capacity L)
  int32_t* feat;        // L-1
  uint32_t* thr;        // L-1
  int32_t* dleft;       // L-1
  int32_t* is_cat;      // L-1
  uint32_t* cat_bits;   // (L-1)*8
  int32_t* left;        // L-1
  int32_t* right;       // L-1
  double* gain;         // L-1
  double* ival;         // L-1
  double* iweight;      // L-1
  int64_t* icount;      // L-1
  double* lval;         // L
  double* lweight;      // L
  int64_t* lcount;      // L
  int32_t* lparent;     // L
  int32_t* ldepth;      // L
};

struct FeatMeta {
  const int32_t* num_bin;
  const int32_t* missing;
  const int32_t* default_bin;
  const int32_t* is_cat;
  const int8_t* mask;
};

__device__ __forceinline__ bool DeviceGoesLeft(uint32_t b, int nb, int mt, int dbin, int is_cat,
                                               uint32_t thr, int dleft, const uint32_t* cat_bits) {
  if (is_cat) return (cat_bits[b >> 5] >> (b & 31)) & 1u;
  if ((mt == kMissingZero && b == static_cast<uint32_t>(dbin)) ||
      (mt == kMissingNaN && b == static_cast<uint32_t>(nb - 1)))
    return dleft != 0;
  return b <= thr;
}

// ---------------------------------------------------------------- K2
__global__ void grad_kernel(ObjParams p, const double* __restrict__ score, const float* __restrict__ label,
                            const float* __restrict__ weight, float* __restrict__ g, float* __restrict__ h,
                            int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double w = weight ? weight[i] : 1.0;
    if (p.kind == kObjMulticlass) {
      const int K = p.num_class;
      double mx = -1e300;
      for (int k = 0; k < K; ++k) mx = fmax(mx, score[k * n + i]);
      double s = 0;
      for (int k = 0; k < K; ++k) s += exp(score[k * n + i] - mx);
      const int y = static_cast<int>(label[i]);
      const double factor = K / (K - 1.0);
      for (int k = 0; k < K; ++k) {
        const double pk = exp(score[k * n + i] - mx) / s;
        g[k * n + i] = static_cast<float>(((k == y) ? pk - 1.0 : pk) * w);
        h[k * n + i] = static_cast<float>(factor * pk * (1.0 - pk) * w);
      }
    } else if (p.kind == kObjMulticlassOVA) {
      for (int k = 0; k < p.num_class; ++k) {
        const double y = static_cast<int>(label[i]) == k ? 1.0 : 0.0;
        PointGradient(p, score[k * n + i], y, w, &g[k * n + i], &h[k * n + i]);
      }
    } else {
      PointGradient(p, score[i], label[i], w, &g[i], &h[i]);
    }
  }
}

// ---------------------------------------------------------------- root init
__global__ void root_init_kernel(DState* st, DLeaf* leaves, int32_t count, int buf, int max_leaves) {
  if (threadIdx.x == 0) {
    st->num_leaves = 1; st->done = 0; st->split_leaf = 0; st->new_leaf = -1;
    st->small_leaf = 0; st->large_leaf = -1; st->parent_slot = -1; st->max_leaves = max_leaves;
    st->phase = 0;
    DLeaf l{};
    l.begin = 0; l.count = count; l.buf = buf; l.depth = 0; l.gcount = count; l.slot = 0;
    leaves[0] = l;
  }
}

__global__ void gather_bag_kernel(const int32_t* __restrict__ rows, int32_t n, const float* __restrict__ g,
                                  const float* __restrict__ h, int32_t* __restrict__ perm,
                                  float2* __restrict__ ogh) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    int r = rows[i];
    perm[i] = r;
    ogh[i] = make_float2(g[r], h[r]);
  }
}

// ---------------------------------------------------------------- K3
// One block = one contiguous chunk of the leaf's row segment x one group of 32
// features. A thread owns whole rows: the 32 bins of its feature group are two
// dwordx4 loads (rows are padded to 16 B), the gradient pair one float2 load
// from the ordered copy (or the physical arrays for an unpartitioned root).
// kHistUnroll rows are fetched before any is accumulated so every wave keeps
// several gathers in flight (the loop is latency-bound otherwise); the adds go
// to LDS-privatised histograms with ds_add_f32, one row per lane, so the lanes
// of a wave hit the same feature at random bins (bank = (feature + bin) % 32
// thanks to the 257-float row pitch).
constexpr int kHistUnroll = 4;

// Accumulation modes (selected per backend, SML_HIST_MODE overrides):
//  0: two ds_add_f32 per (row, feature)
//  1: fixed point, g and h packed in one 64-bit word -> one ds_add_u64; h >= 0
//     lives in the low 32 bits (never carries), g in the high 32 (two's
//     complement wraps exactly). Integer adds are order independent, so the
//     histogram is bitwise deterministic.
//  2: fixed point, two ds_add_u32
// Fixed-point scales are chosen per launch from the block's row count and the
// tree's max |g|, max h so no block sum can overflow (>= 16 bits per value at
// the root, ~20 bits for typical leaves).
__device__ __forceinline__ uint32_t word_of(const uint4& b, int j) {
  return j < 4 ? b.x : (j < 8 ? b.y : (j < 12 ? b.z : b.w));
}

template <int MODE>
__device__ __forceinline__ void hist_add(void* lds, int j, uint32_t bin, float2 v, int32_t gq, uint32_t hq,
                                         unsigned long long packed) {
  if (MODE == 0) {
    float* shg = static_cast<float*>(lds);
    float* shh = shg + kFeatPerGroup * kHistStride;
    atomicAdd(&shg[j * kHistStride + bin], v.x);
    atomicAdd(&shh[j * kHistStride + bin], v.y);
  } else if (MODE == 1) {
    unsigned long long* sh = static_cast<unsigned long long*>(lds);
    atomicAdd(&sh[j * kHistStride + bin], packed);
  } else {
    uint32_t* shg = static_cast<uint32_t*>(lds);
    uint32_t* shh = shg + kFeatPerGroup * kHistStride;
    atomicAdd(&shg[j * kHistStride + bin], static_cast<uint32_t>(gq));
    atomicAdd(&shh[j * kHistStride + bin], hq);
  }
}

template <int MODE>
__device__ __forceinline__ void hist_accumulate(void* lds, const uint4& b0, const uint4& b1, float2 v, int Fg,
                                                float sg, float sh) {
  int32_t gq = 0;
  uint32_t hq = 0;
  unsigned long long packed = 0;
  if (MODE != 0) {
    gq = __float2int_rn(v.x * sg);
    hq = static_cast<uint32_t>(__float2uint_rn(fmaxf(v.y, 0.f) * sh));
    packed = (static_cast<unsigned long long>(static_cast<uint32_t>(gq)) << 32) | hq;
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    if (j < Fg) hist_add<MODE>(lds, j, (word_of(b0, j) >> (8 * (j & 3))) & 255u, v, gq, hq, packed);
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    if (j + 16 < Fg) hist_add<MODE>(lds, j + 16, (word_of(b1, j) >> (8 * (j & 3))) & 255u, v, gq, hq, packed);
  }
}

template <int MODE>
__global__ __launch_bounds__(kHistThreads) void hist_kernel(
    const DState* __restrict__ st, const DLeaf* __restrict__ leaves, const uint4* __restrict__ bins4,
    int W4, int F, const int32_t* __restrict__ perm0, const int32_t* __restrict__ perm1,
    const float2* __restrict__ ogh0, const float2* __restrict__ ogh1, const float* __restrict__ g,
    const float* __restrict__ h, const float* __restrict__ ghmax, float2* __restrict__ slab) {
  if (st->done) return;
  const DLeaf L = HistSeg(st, leaves);
  const int count = L.count;
  const int nb_active = max(1, min(kMaxHistBlocks, ceil_div_i(count, kMinRowsPerHistBlock)));
  if (static_cast<int>(blockIdx.x) >= nb_active) return;
  constexpr int kWordBytes = MODE == 1 ? 8 : 4;
  constexpr int kArrays = MODE == 1 ? 1 : 2;
  __shared__ __attribute__((aligned(16))) unsigned char lds_raw[kArrays * kFeatPerGroup * kHistStride * kWordBytes];
  void* lds = lds_raw;
  const int tid = threadIdx.x;
  {
    uint32_t* z = reinterpret_cast<uint32_t*>(lds_raw);
    for (int i = tid; i < kArrays * kFeatPerGroup * kHistStride * kWordBytes / 4; i += kHistThreads) z[i] = 0u;
  }
  __syncthreads();
  const int grp = blockIdx.y;
  const int Fg = min(kFeatPerGroup, F - grp * kFeatPerGroup);
  const int col = grp * 2;            // first uint4 of this group in a row
  const bool two = Fg > 16;
  const int chunk = ceil_div_i(count, nb_active);
  const int p0 = L.begin + blockIdx.x * chunk;
  const int p1 = min(L.begin + count, p0 + chunk);
  // fixed-point scales (unused in MODE 0)
  float sg = 0.f, shs = 0.f;
  if (MODE != 0) {
    const float gmax = fmaxf(ghmax[0], 1e-30f), hmax = fmaxf(ghmax[1], 1e-30f);
    const float rows = static_cast<float>(max(1, chunk));
    sg = 2.0e9f / (rows * gmax);
    shs = (MODE == 1 ? 4.0e9f : 2.0e9f) / (rows * hmax);
  }
  const int32_t* __restrict__ perm = L.buf == 0 ? perm0 : perm1;
  const float2* __restrict__ ogh = L.buf == 0 ? ogh0 : ogh1;
  const bool phys = L.buf < 0;
  for (int base = p0 + tid; base < p1; base += kHistThreads * kHistUnroll) {
    int r[kHistUnroll];
    bool ok[kHistUnroll];
#pragma unroll
    for (int u = 0; u < kHistUnroll; ++u) {
      const int pos = base + u * kHistThreads;
      ok[u] = pos < p1;
      r[u] = ok[u] ? (phys ? pos : perm[pos]) : 0;
    }
    uint4 b0[kHistUnroll], b1[kHistUnroll];
    float2 v[kHistUnroll];
#pragma unroll
    for (int u = 0; u < kHistUnroll; ++u) {
      const int pos = base + u * kHistThreads;
      const size_t rb = static_cast<size_t>(r[u]) * W4 + col;
      b0[u] = bins4[rb];
      b1[u] = two ? bins4[rb + 1] : make_uint4(0, 0, 0, 0);
      v[u] = phys ? make_float2(g[r[u]], h[r[u]]) : (ok[u] ? ogh[pos] : make_float2(0.f, 0.f));
    }
#pragma unroll
    for (int u = 0; u < kHistUnroll; ++u)
      if (ok[u]) hist_accumulate<MODE>(lds, b0[u], b1[u], v[u], Fg, sg, shs);
  }
  __syncthreads();
  float2* out = slab + static_cast<size_t>(blockIdx.x) * F * kBinsPerFeature;
  for (int i = tid; i < Fg * kBinsPerFeature; i += kHistThreads) {
    const int f = i >> 8, b = i & 255;
    float2 o;
    if (MODE == 0) {
      const float* shg = reinterpret_cast<const float*>(lds_raw);
      o = make_float2(shg[f * kHistStride + b], shg[kFeatPerGroup * kHistStride + f * kHistStride + b]);
    } else if (MODE == 1) {
      const unsigned long long w = reinterpret_cast<const unsigned long long*>(lds_raw)[f * kHistStride + b];
      o = make_float2(static_cast<float>(static_cast<double>(static_cast<int32_t>(w >> 32)) / sg),
                      static_cast<float>(static_cast<double>(static_cast<uint32_t>(w)) / shs));
    } else {
      const uint32_t* shg = reinterpret_cast<const uint32_t*>(lds_raw);
      o = make_float2(static_cast<float>(static_cast<double>(static_cast<int32_t>(shg[f * kHistStride + b])) / sg),
                      static_cast<float>(static_cast<double>(shg[kFeatPerGroup * kHistStride + f * kHistStride + b]) / shs));
    }
    out[(grp * kFeatPerGroup + f) * kBinsPerFeature + b] = o;
  }
}

// max |g|, max h of one class (fixed-point scales of the histogram kernel)
__global__ void ghmax_kernel(const float* __restrict__ g, const float* __restrict__ h, int64_t n,
                             unsigned int* __restrict__ out_bits) {
  float mg = 0.f, mh = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    mg = fmaxf(mg, fabsf(g[i]));
    mh = fmaxf(mh, fabsf(h[i]));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) { mg = fmaxf(mg, __shfl_xor(mg, off, 64)); mh = fmaxf(mh, __shfl_xor(mh, off, 64)); }
  if ((threadIdx.x & 63) == 0) {
    // non-negative floats order like their bit patterns
    atomicMax(&out_bits[0], __float_as_uint(mg));
    atomicMax(&out_bits[1], __float_as_uint(mh));
  }
}

// Fixed-order reduction of the per-block slabs: part[y][e] = sum over blocks
// y, y+S, ... (deterministic). The last element of part[0] carries the leaf's
// local row count so one allreduce also yields the global count.
__global__ void hist_reduce_kernel(const DState* __restrict__ st, const DLeaf* __restrict__ leaves,
                                   const float2* __restrict__ slab, int E, double2* __restrict__ part,
                                   double* __restrict__ count_slot) {
  if (st->done) return;
  const int count = HistSeg(st, leaves).count;
  const int nb_active = max(1, min(kMaxHistBlocks, ceil_div_i(count, kMinRowsPerHistBlock)));
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.y;
  if (e < E) {
    double sg = 0, sh = 0;
    for (int b = y; b < nb_active; b += kReduceSplit) {
      const float2 v = slab[static_cast<size_t>(b) * E + e];
      sg += v.x; sh += v.y;
    }
    part[static_cast<size_t>(y) * E + e] = make_double2(sg, sh);
  }
  if (e == 0 && y == 0) *count_slot = static_cast<double>(count);
}

// Data-parallel only: part[0] += part[1..S-1], parts zeroed, count stored in
// the double right after part[0] so one collective moves everything.
__global__ void fold_parts_kernel(double2* __restrict__ part, int E, const double* __restrict__ count_slot) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < E) {
    double2 acc = part[e];
    for (int y = 1; y < kReduceSplit; ++y) {
      const double2 v = part[static_cast<size_t>(y) * E + e];
      acc.x += v.x; acc.y += v.y;
      part[static_cast<size_t>(y) * E + e] = make_double2(0.0, 0.0);
    }
    part[e] = acc;
  }
  if (e == 0) reinterpret_cast<double*>(part + E)[0] = *count_slot;
}

__global__ void unfold_count_kernel(double2* __restrict__ part, int E, double* __restrict__ count_slot) {
  if (threadIdx.x == 0) {
    double* p = reinterpret_cast<double*>(part + E);
    *count_slot = p[0];
    p[0] = 0.0;
    p[1] = 0.0;
  }
}

// ---------------------------------------------------------------- K4 + K5
struct Cand {
  double gain;
  int thr;
  int dl;
};

__device__ __forceinline__ bool CandBetter(const Cand& a, const Cand& b) {
  if (a.gain != b.gain) return a.gain > b.gain;
  if (a.thr != b.thr) return a.thr < b.thr;
  return a.dl < b.dl;
}

__device__ void CategoricalSearch(const double* hg, const double* hh, int nb, int fi, double G, double H,
                                  int64_t cnt, const SplitParams& sp, SplitResult* best, int* idx) {
  // serial port of the host search (one thread): bins are <= 256
  const double cnt_factor = cnt / fmax(H, kEpsilon);
  const int other = nb - 1;
  const double l2 = sp.lambda_l2 + sp.cat_l2;
  const double cat_parent = LeafGain(G, H, sp.lambda_l1, l2, sp.max_delta_step);
  auto try_set = [&](int nleft, const int* left_bins, double gl, double hl) {
    const double gr = G - gl, hr = H - hl;
    const int64_t cl = EstimateCount(hl, cnt_factor), cr = cnt - cl;
    if (cl < sp.min_data_in_leaf || cr < sp.min_data_in_leaf) return;
    if (hl < sp.min_sum_hessian || hr < sp.min_sum_hessian) return;
    if (nleft > 1 && (cl < sp.min_data_per_group || cr < sp.min_data_per_group)) return;
    const double gain = LeafGain(gl, hl, sp.lambda_l1, l2, sp.max_delta_step) +
                        LeafGain(gr, hr, sp.lambda_l1, l2, sp.max_delta_step);
    const double shift = cat_parent + sp.min_gain_to_split;
    if (!(gain > shift)) return;
    const double sg = gain - shift;
    if (best->feature >= 0 && !SplitBetter(sg, fi, static_cast<uint32_t>(nleft), best->gain, best->feature, best->threshold)) return;
    best->gain = sg; best->feature = fi; best->threshold = static_cast<uint32_t>(nleft);
    best->default_left = 0; best->is_cat = 1;
    for (int w = 0; w < 8; ++w) best->cat_bits[w] = 0;
    for (int k = 0; k < nleft; ++k) best->cat_bits[left_bins[k] >> 5] |= 1u << (left_bins[k] & 31);
    best->left_g = gl; best->left_h = hl; best->right_g = gr; best->right_h = hr;
    best->left_cnt = cl; best->right_cnt = cr;
    best->left_out = LeafOutput(gl, hl, sp.lambda_l1, l2, sp.max_delta_step);
    best->right_out = LeafOutput(gr, hr, sp.lambda_l1, l2, sp.max_delta_step);
  };
  if (nb <= sp.max_cat_to_onehot + 1) {
    for (int b = 0; b < other; ++b) { int lb = b; try_set(1, &lb, hg[b], hh[b]); }
    return;
  }
  int m = 0;
  for (int b = 0; b < other; ++b)
    if (EstimateCount(hh[b], cnt_factor) >= sp.cat_smooth) idx[m++] = b;
  // stable insertion sort by g/(h+smooth)
  for (int i = 1; i < m; ++i) {
    int v = idx[i];
    double key = hg[v] / (hh[v] + sp.cat_smooth);
    int j = i - 1;
    while (j >= 0 && hg[idx[j]] / (hh[idx[j]] + sp.cat_smooth) > key) { idx[j + 1] = idx[j]; --j; }
    idx[j + 1] = v;
  }
  const int maxk = min(sp.max_cat_threshold, (m + 1) / 2);
  int left[256];
  for (int dir = 0; dir < 2; ++dir) {
    double gl = 0, hl = 0;
    for (int k = 0; k < m && k < maxk; ++k) {
      int b = dir == 0 ? idx[k] : idx[m - 1 - k];
      left[k] = b;
      gl += hg[b]; hl += hh[b];
      try_set(k + 1, left, gl, hl);
    }
  }
}

// grid: (F, nchild). Block = 256 threads, thread = bin.
__global__ __launch_bounds__(256) void find_split_kernel(
    DState* __restrict__ st, DLeaf* __restrict__ leaves, const double2* __restrict__ part, int E,
    const double* __restrict__ count_slot, double2* __restrict__ hist_pool, FeatMeta fm, SplitParams sp,
    SplitResult* __restrict__ fbest, int F) {
  if (st->done) return;
  const int f = blockIdx.x;
  const int child = blockIdx.y;  // 0 = small (or root), 1 = large
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const bool root = st->phase == 0;
  if (root && child == 1) return;
  const int leaf_id = root ? 0 : (child == 0 ? st->small_leaf : st->large_leaf);
  const int e = f * kBinsPerFeature + tid;
  // reduce the partial sums (fixed order) -> small histogram
  double2 sm = make_double2(0, 0);
#pragma unroll
  for (int y = 0; y < kReduceSplit; ++y) {
    const double2 v = part[static_cast<size_t>(y) * E + e];
    sm.x += v.x; sm.y += v.y;
  }
  double2 mine;
  if (root || child == 0) {
    mine = sm;
  } else {
    const double2 par = hist_pool[static_cast<size_t>(st->parent_slot) * E + e];
    mine = make_double2(par.x - sm.x, par.y - sm.y);
  }
  const DLeaf Lf = leaves[leaf_id];
  hist_pool[static_cast<size_t>(Lf.slot) * E + e] = mine;
  __shared__ double sg_[256], shh_[256];
  __shared__ double wtot_g[4], wtot_h[4];
  __shared__ Cand wbest[4];
  __shared__ int idxbuf[256];
  sg_[tid] = mine.x;
  shh_[tid] = mine.y;
  const int nb = fm.num_bin[f];
  const int mt = fm.missing[f];
  const int dbin = fm.default_bin[f];
  // leaf totals: from this feature's histogram (root) or the split record
  double G, H;
  int64_t cnt;
  {
    // total over bins (for the root and as a consistent parent sum)
    double tg = tid < nb ? mine.x : 0.0, th = tid < nb ? mine.y : 0.0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) { tg += __shfl_xor(tg, off, 64); th += __shfl_xor(th, off, 64); }
    if (lane == 0) { wtot_g[wid] = tg; wtot_h[wid] = th; }
    __syncthreads();
    G = wtot_g[0] + wtot_g[1] + wtot_g[2] + wtot_g[3];
    H = wtot_h[0] + wtot_h[1] + wtot_h[2] + wtot_h[3];
  }
  if (root) {
    cnt = static_cast<int64_t>(*count_slot);
    if (f == 0 && tid == 0) {
      leaves[0].sum_g = G; leaves[0].sum_h = H; leaves[0].gcount = cnt;
    }
  } else {
    const int64_t small_cnt = static_cast<int64_t>(*count_slot);
    cnt = child == 0 ? small_cnt : (Lf.gcount - small_cnt);  // Lf.gcount of large holds the parent count (set by choose)
    G = Lf.sum_g; H = Lf.sum_h;
  }
  SplitResult* out = fbest + child * F + f;
  const bool eligible = fm.mask[f] && nb > 1 && cnt >= 2 * static_cast<int64_t>(sp.min_data_in_leaf) &&
                        (sp.max_depth <= 0 || Lf.depth < sp.max_depth);
  if (!eligible) {
    if (tid == 0) { out->feature = -1; out->gain = -INFINITY; }
    return;
  }
  if (fm.is_cat[f]) {
    if (tid == 0) {
      SplitResult best;
      best.feature = -1; best.gain = -INFINITY;
      CategoricalSearch(sg_, shh_, nb, f, G, H, cnt, sp, &best, idxbuf);
      *out = best;
    }
    return;
  }
  const int nan_bin = mt == kMissingNaN ? nb - 1 : -1;
  const int zero_bin = mt == kMissingZero ? dbin : -1;
  const double mg = nan_bin >= 0 ? sg_[nan_bin] : (zero_bin >= 0 ? sg_[zero_bin] : 0.0);
  const double mh = nan_bin >= 0 ? shh_[nan_bin] : (zero_bin >= 0 ? shh_[zero_bin] : 0.0);
  const int last = nan_bin >= 0 ? nb - 2 : nb - 1;
  // inclusive prefix over ordered bins (zero bin excluded for Zero missing)
  double vg = (tid < nb && tid != zero_bin && tid != nan_bin) ? mine.x : 0.0;
  double vh = (tid < nb && tid != zero_bin && tid != nan_bin) ? mine.y : 0.0;
  vg = wave_incl_scan(vg, lane);
  vh = wave_incl_scan(vh, lane);
  __shared__ double wsum_g[4], wsum_h[4];
  if (lane == 63) { wsum_g[wid] = vg; wsum_h[wid] = vh; }
  __syncthreads();
  for (int w = 0; w < wid; ++w) { vg += wsum_g[w]; vh += wsum_h[w]; }
  __shared__ double pref_g[256], pref_h[256];
  pref_g[tid] = vg;
  pref_h[tid] = vh;
  const double cnt_factor = cnt / fmax(H, kEpsilon);
  const double parent_gain = LeafGain(G, H, sp.lambda_l1, sp.lambda_l2, sp.max_delta_step);
  const double shift = parent_gain + sp.min_gain_to_split;
  Cand best{-INFINITY, 1 << 30, 1 << 30};
  if (tid < last) {
    auto consider = [&](double gl, double hl, int dl) {
      const double gr = G - gl, hr = H - hl;
      const int64_t cl = EstimateCount(hl, cnt_factor), cr = cnt - cl;
      if (cl < sp.min_data_in_leaf || cr < sp.min_data_in_leaf) return;
      if (hl < sp.min_sum_hessian || hr < sp.min_sum_hessian) return;
      const double gain = LeafGain(gl, hl, sp.lambda_l1, sp.lambda_l2, sp.max_delta_step) +
                          LeafGain(gr, hr, sp.lambda_l1, sp.lambda_l2, sp.max_delta_step);
      if (!(gain > shift)) return;
      Cand c{gain - shift, tid, dl};
      if (CandBetter(c, best)) best = c;
    };
    if (mt == kMissingNone) consider(vg, vh, 1);
    else { consider(vg, vh, 0); consider(vg + mg, vh + mh, 1); }
  }
  // block argmax
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    Cand o;
    o.gain = __shfl_xor(best.gain, off, 64);
    o.thr = __shfl_xor(best.thr, off, 64);
    o.dl = __shfl_xor(best.dl, off, 64);
    if (CandBetter(o, best)) best = o;
  }
  if (lane == 0) wbest[wid] = best;
  __syncthreads();
  if (tid == 0) {
    Cand b = wbest[0];
    for (int w = 1; w < 4; ++w) if (CandBetter(wbest[w], b)) b = wbest[w];
    SplitResult r;
    if (b.gain == -INFINITY) {
      r.feature = -1; r.gain = -INFINITY;
    } else {
      // the winning prefix, exactly as the candidate saw it
      double gl = pref_g[b.thr], hl = pref_h[b.thr];
      if (mt != kMissingNone && b.dl) { gl += mg; hl += mh; }
      const double gr = G - gl, hr = H - hl;
      r.feature = f; r.gain = b.gain; r.threshold = static_cast<uint32_t>(b.thr); r.default_left = b.dl;
      r.is_cat = 0;
      r.left_g = gl; r.left_h = hl; r.right_g = gr; r.right_h = hr;
      r.left_cnt = EstimateCount(hl, cnt_factor); r.right_cnt = cnt - r.left_cnt;
      r.left_out = LeafOutput(gl, hl, sp.lambda_l1, sp.lambda_l2, sp.max_delta_step);
      r.right_out = LeafOutput(gr, hr, sp.lambda_l1, sp.lambda_l2, sp.max_delta_step);
      for (int w = 0; w < 8; ++w) r.cat_bits[w] = 0;
    }
    *out = r;
  }
}

// ---------------------------------------------------------------- choose + tree bookkeeping
// One block. Wave c reduces the per-feature results of new leaf c (lanes
// stride over features), all threads then reduce the leaves' best gains, and
// thread 0 records the chosen split in the device tree and sets up the
// partition of that leaf. Every global read on the serial path is independent
// so the bookkeeping costs a few memory latencies, not one per leaf/feature.
struct KeyG {
  double gain;
  int a, b;  // tie-breakers (smaller wins)
};

__device__ __forceinline__ bool KeyBetter(const KeyG& x, const KeyG& y) {
  if (x.gain != y.gain) return x.gain > y.gain;
  if (x.a != y.a) return x.a < y.a;
  return x.b < y.b;
}

__device__ __forceinline__ KeyG WaveArgmax(KeyG k) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    KeyG o;
    o.gain = __shfl_xor(k.gain, off, 64);
    o.a = __shfl_xor(k.a, off, 64);
    o.b = __shfl_xor(k.b, off, 64);
    if (KeyBetter(o, k)) k = o;
  }
  return k;
}

__global__ __launch_bounds__(256) void choose_kernel(DState* __restrict__ st, DLeaf* __restrict__ leaves,
                                                     SplitResult* __restrict__ lbest, double* __restrict__ lgain,
                                                     const SplitResult* __restrict__ fbest, int F, DTree t,
                                                     const double* __restrict__ count_slot) {
  if (st->done) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  __shared__ int sh_best_f[2];
  __shared__ KeyG wk[4];
  const bool root = st->phase == 0;
  const int nchild = root ? 1 : 2;
  const int small_leaf = st->small_leaf, large_leaf = st->large_leaf;
  if (wid < nchild) {
    KeyG k{-INFINITY, 1 << 30, 1 << 30};
    for (int f = lane; f < F; f += 64) {
      const SplitResult& r = fbest[wid * F + f];
      if (r.feature < 0) continue;
      KeyG c{r.gain, r.feature, static_cast<int>(r.threshold)};
      if (KeyBetter(c, k)) { k = c; k.b = (static_cast<int>(r.threshold) & 0xFFFF) | (f << 16); }
    }
    k = WaveArgmax(k);
    if (lane == 0) sh_best_f[wid] = k.gain == -INFINITY ? -1 : (k.b >> 16);
  }
  __syncthreads();
  if (tid == 0) {
    if (root) {
      const int bi = sh_best_f[0];
      if (bi >= 0) { lbest[0] = fbest[bi]; lgain[0] = fbest[bi].gain; }
      else { lbest[0].feature = -1; lbest[0].gain = -INFINITY; lgain[0] = -INFINITY; }
      t.lval[0] = 0.0;
      t.lcount[0] = leaves[0].gcount;
      t.lweight[0] = leaves[0].sum_h;
      t.lparent[0] = -1;
      t.ldepth[0] = 0;
    } else {
      const int64_t small_cnt = static_cast<int64_t>(*count_slot);
      const int64_t parent_cnt = leaves[large_leaf].gcount;  // stored by the previous choose
      const int ob = st->pbuf == 0 ? 1 : 0;
      DLeaf& Lc = leaves[st->split_leaf];
      DLeaf& Rc = leaves[st->new_leaf];
      Lc.begin = st->pbegin; Lc.count = st->ptotal; Lc.buf = ob;
      Rc.begin = st->pbegin + st->ptotal; Rc.count = st->pcount - st->ptotal; Rc.buf = ob;
      leaves[small_leaf].gcount = small_cnt;
      leaves[large_leaf].gcount = parent_cnt - small_cnt;
      t.lcount[small_leaf] = small_cnt;
      t.lcount[large_leaf] = parent_cnt - small_cnt;
      for (int c = 0; c < 2; ++c) {
        const int leaf = c == 0 ? small_leaf : large_leaf;
        const int bi = sh_best_f[c];
        if (bi >= 0) { lbest[leaf] = fbest[c * F + bi]; lgain[leaf] = fbest[c * F + bi].gain; }
        else { lbest[leaf].feature = -1; lbest[leaf].gain = -INFINITY; lgain[leaf] = -INFINITY; }
      }
    }
  }
  __syncthreads();
  const int nl = st->num_leaves;
  if (nl >= st->max_leaves) {
    if (tid == 0) st->done = 1;
    return;
  }
  // argmax over leaves (ties -> smaller leaf id)
  KeyG k{-INFINITY, 1 << 30, 0};
  for (int i = tid; i < nl; i += 256) {
    const double gi = lgain[i];
    KeyG c{gi, i, 0};
    if (gi > -INFINITY && KeyBetter(c, k)) k = c;
  }
  k = WaveArgmax(k);
  if (lane == 0) wk[wid] = k;
  __syncthreads();
  if (tid != 0) return;
  KeyG best = wk[0];
  for (int w = 1; w < 4; ++w) if (KeyBetter(wk[w], best)) best = wk[w];
  const int bl = best.gain == -INFINITY ? -1 : best.a;
  if (bl < 0 || !(best.gain > 0.0)) { st->done = 1; return; }
  const SplitResult sr = lbest[bl];
  const int node = nl - 1;
  const int parent = t.lparent[bl];
  if (parent >= 0) {
    if (t.left[parent] == ~bl) t.left[parent] = node; else t.right[parent] = node;
  }
  t.feat[node] = sr.feature;
  t.thr[node] = sr.threshold;
  t.dleft[node] = sr.default_left;
  t.is_cat[node] = sr.is_cat;
  for (int w = 0; w < 8; ++w) t.cat_bits[node * 8 + w] = sr.cat_bits[w];
  t.left[node] = ~bl;
  t.right[node] = ~nl;
  t.gain[node] = sr.gain;
  t.ival[node] = t.lval[bl];
  t.iweight[node] = sr.left_h + sr.right_h;
  t.icount[node] = leaves[bl].gcount;
  t.lparent[bl] = node; t.lparent[nl] = node;
  t.lval[bl] = sr.left_out; t.lval[nl] = sr.right_out;
  t.lweight[bl] = sr.left_h; t.lweight[nl] = sr.right_h;
  t.lcount[bl] = sr.left_cnt; t.lcount[nl] = sr.right_cnt;
  const int depth = t.ldepth[bl] + 1;
  t.ldepth[bl] = depth; t.ldepth[nl] = depth;
  const DLeaf P = leaves[bl];
  DLeaf Lc = P, Rc = P;
  Lc.depth = depth; Rc.depth = depth;
  Lc.sum_g = sr.left_g; Lc.sum_h = sr.left_h;
  Rc.sum_g = sr.right_g; Rc.sum_h = sr.right_h;
  const bool left_small = sr.left_cnt <= sr.right_cnt;
  st->parent_slot = P.slot;
  Lc.slot = 2 * node + 1;
  Rc.slot = 2 * node + 2;
  // the large child's gcount temporarily holds the parent's global count
  if (left_small) { Rc.gcount = P.gcount; } else { Lc.gcount = P.gcount; }
  leaves[bl] = Lc;
  leaves[nl] = Rc;
  lgain[bl] = -INFINITY;
  lgain[nl] = -INFINITY;
  st->pbegin = P.begin; st->pcount = P.count; st->pbuf = P.buf; st->ptotal = 0;
  st->split_leaf = bl;
  st->new_leaf = nl;
  st->small_leaf = left_small ? bl : nl;
  st->large_leaf = left_small ? nl : bl;
  st->num_leaves = nl + 1;
  st->phase = 1;
}

// ---------------------------------------------------------------- K6
// Decisions read the column-major copy: the lanes of a wave touch one byte
// column (contiguous for the physical root, increasing for partitioned leaves)
// instead of one 32-B row each.
__device__ __forceinline__ bool RowGoesLeft(const uint8_t* cbins, int64_t n, int r, const SplitResult& sr, FeatMeta fm) {
  const int f = sr.feature;
  const uint32_t b = cbins[static_cast<size_t>(f) * n + r];
  return DeviceGoesLeft(b, fm.num_bin[f], fm.missing[f], fm.default_bin[f], sr.is_cat, sr.threshold,
                        sr.default_left, sr.cat_bits);
}

__global__ __launch_bounds__(kPartThreads) void part_count_kernel(
    const DState* __restrict__ st, const DLeaf* __restrict__ leaves, const SplitResult* __restrict__ lbest,
    const uint8_t* __restrict__ cbins, int64_t n, const int32_t* __restrict__ perm0,
    const int32_t* __restrict__ perm1, FeatMeta fm, int32_t* __restrict__ counts) {
  if (st->done) return;
  DLeaf P;
  P.begin = st->pbegin; P.count = st->pcount; P.buf = st->pbuf;
  const SplitResult sr = lbest[st->split_leaf];
  const int nbp = max(1, min(kMaxPartBlocks, ceil_div_i(P.count, kMinRowsPerPartBlock)));
  if (static_cast<int>(blockIdx.x) >= nbp) return;
  const int chunk = ceil_div_i(P.count, nbp);
  const int p0 = P.begin + blockIdx.x * chunk;
  const int p1 = min(P.begin + P.count, p0 + chunk);
  const int32_t* perm = P.buf == 0 ? perm0 : perm1;
  int c = 0;
  for (int p = p0 + threadIdx.x; p < p1; p += kPartThreads) {
    const int r = P.buf < 0 ? p : perm[p];
    c += RowGoesLeft(cbins, n, r, sr, fm) ? 1 : 0;
  }
  __shared__ int sc[kPartThreads / 64];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
  if ((threadIdx.x & 63) == 0) sc[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < kPartThreads / 64; ++w) t += sc[w];
    counts[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(kPartThreads) void part_scatter_kernel(
    DState* __restrict__ st, const DLeaf* __restrict__ leaves, const SplitResult* __restrict__ lbest,
    const uint8_t* __restrict__ cbins, int64_t n, const int32_t* __restrict__ perm0, const int32_t* __restrict__ perm1,
    const float2* __restrict__ ogh0, const float2* __restrict__ ogh1, int32_t* __restrict__ wperm0,
    int32_t* __restrict__ wperm1, float2* __restrict__ wogh0, float2* __restrict__ wogh1,
    const float* __restrict__ g, const float* __restrict__ h, FeatMeta fm, const int32_t* __restrict__ counts) {
  if (st->done) return;
  const int sl = st->split_leaf;
  DLeaf P;
  P.begin = st->pbegin; P.count = st->pcount; P.buf = st->pbuf;
  const SplitResult sr = lbest[sl];
  const int nbp = max(1, min(kMaxPartBlocks, ceil_div_i(P.count, kMinRowsPerPartBlock)));
  if (static_cast<int>(blockIdx.x) >= nbp) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  __shared__ int red[2][kPartThreads / 64];
  __shared__ int wl[kPartThreads / 64];
  // prefix of left counts before this block + total
  int before = 0, total = 0;
  for (int j = tid; j < nbp; j += kPartThreads) {
    const int c = counts[j];
    total += c;
    if (j < static_cast<int>(blockIdx.x)) before += c;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    before += __shfl_xor(before, off, 64);
    total += __shfl_xor(total, off, 64);
  }
  if (lane == 0) { red[0][wid] = before; red[1][wid] = total; }
  __syncthreads();
  before = 0; total = 0;
  for (int w = 0; w < kPartThreads / 64; ++w) { before += red[0][w]; total += red[1][w]; }
  const int chunk = ceil_div_i(P.count, nbp);
  const int p0 = P.begin + blockIdx.x * chunk;
  const int p1 = min(P.begin + P.count, p0 + chunk);
  const int ob = P.buf == 0 ? 1 : 0;
  const int32_t* perm = P.buf == 0 ? perm0 : perm1;
  const float2* ogh = P.buf == 0 ? ogh0 : ogh1;
  int32_t* operm = ob == 0 ? wperm0 : wperm1;
  float2* oogh = ob == 0 ? wogh0 : wogh1;
  int left_base = P.begin + before;
  int right_base = P.begin + total + ((p0 - P.begin) - before);
  for (int tile = p0; tile < p1; tile += kPartThreads) {
    const int p = tile + tid;
    const bool valid = p < p1;
    int r = 0;
    float2 v = make_float2(0.f, 0.f);
    bool left = false;
    if (valid) {
      if (P.buf < 0) { r = p; v = make_float2(g[r], h[r]); }
      else { r = perm[p]; v = ogh[p]; }
      left = RowGoesLeft(cbins, n, r, sr, fm);
    }
    const unsigned long long bl = __ballot(valid && left);
    const unsigned long long bv = __ballot(valid);
    const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int rl = __popcll(bl & below);
    const int rv = __popcll(bv & below);
    if (lane == 0) wl[wid] = __popcll(bl);
    __syncthreads();
    int wbefore_l = 0, tile_l = 0;
    for (int w = 0; w < kPartThreads / 64; ++w) {
      if (w < wid) wbefore_l += wl[w];
      tile_l += wl[w];
    }
    const int wbase_total = wid * 64;  // valid elements are contiguous from tile start
    if (valid) {
      int dst;
      if (left) dst = left_base + wbefore_l + rl;
      else dst = right_base + (wbase_total - wbefore_l) + (rv - rl);
      operm[dst] = r;
      oogh[dst] = v;
    }
    const int tile_valid = min(kPartThreads, p1 - tile);
    left_base += tile_l;
    right_base += tile_valid - tile_l;
    __syncthreads();
  }
  if (blockIdx.x == 0 && tid == 0) st->ptotal = total;  // children segments: finalised by choose
}

// ---------------------------------------------------------------- K7
// Node = one int4 {feature | missing<<16 | default_left<<18 | is_cat<<19,
// threshold bin, left, right}: a single 16-B load per level; bins come from the
// column-major copy so a wave's loads of one level are coalesced.
struct DevTreeView {
  const int4* nodes;
  const uint32_t* cat_bits;  // 8 words per node
  const double* lval;
  int num_leaves;
};

__global__ void score_kernel(DevTreeView tv, const uint8_t* __restrict__ cbins, int64_t n, FeatMeta fm,
                             double scale, double* __restrict__ score, int32_t* __restrict__ leaf_out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int node = 0;
    if (tv.num_leaves > 1) {
      for (int guard = 0; node >= 0 && guard < tv.num_leaves; ++guard) {
        const int4 nd = tv.nodes[node];
        const int f = nd.x & 0xFFFF;
        const int mt = (nd.x >> 16) & 3, dl = (nd.x >> 18) & 1, ic = (nd.x >> 19) & 1;
        const uint32_t b = cbins[static_cast<size_t>(f) * n + i];
        const bool left = DeviceGoesLeft(b, fm.num_bin[f], mt, fm.default_bin[f], ic, static_cast<uint32_t>(nd.y), dl,
                                         tv.cat_bits + node * 8);
        node = left ? nd.z : nd.w;
      }
      node = node < 0 ? ~node : 0;  // a malformed tree cannot loop forever
    }
    if (score) score[i] += scale * tv.lval[node];
    if (leaf_out) leaf_out[i] = node;
  }
}

// row-major -> column-major bin copy (once per dataset)
__global__ void transpose_bins_kernel(const uint8_t* __restrict__ bins, int S, int F, int64_t n,
                                      uint8_t* __restrict__ cbins) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* row = bins + i * S;
    for (int f = 0; f < F; ++f) cbins[static_cast<size_t>(f) * n + i] = row[f];
  }
}

__global__ void axpby_kernel(double* __restrict__ s, int64_t n, double a, double b) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    s[i] = a * s[i] + b;
}

// ---------------------------------------------------------------- backend
class GpuBackend : public TrainBackend {
 public:
  explicit GpuBackend(int dev) : dev_(dev) {}
  ~GpuBackend() override {
    if (stream_) { (void)hipStreamSynchronize(stream_); (void)hipStreamDestroy(stream_); }
    if (pinned_) (void)hipHostFree(pinned_);
  }
  std::string Name() const override { return "hip"; }

  void Init(const Dataset* d, const Config& cfg, int K) override {
    data_ = d; cfg_ = cfg; K_ = K; n_ = d->num_data;
    if (n_ >= (int64_t(1) << 31)) throw std::runtime_error("GPU backend: more than 2^31 rows per device");
    if (cfg.num_leaves > 4096) throw std::runtime_error("GPU backend: num_leaves > 4096");
    if (dev_ >= 0) SML_HIP_CHECK(hipSetDevice(dev_));
    SML_HIP_CHECK(hipGetDevice(&dev_));
    SML_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    sp_ = MakeSplitParams(cfg);
    hist_mode_ = 1;  // packed fixed point (deterministic); SML_HIST_MODE=0 selects float atomics
    if (const char* e = std::getenv("SML_HIST_MODE")) hist_mode_ = std::atoi(e);
    ghmax_.alloc(2);
    F_ = d->ref.num_inner();
    S_ = d->row_stride;
    W_ = S_ / 4;
    E_ = F_ * kBinsPerFeature;
    L_ = std::max(2, cfg.num_leaves);
    FG_ = (F_ + kFeatPerGroup - 1) / kFeatPerGroup;
    bins_.alloc(static_cast<size_t>(n_) * S_);
    SML_HIP_CHECK(hipMemcpyAsync(bins_.get(), d->bins.data(), static_cast<size_t>(n_) * S_, hipMemcpyHostToDevice, stream_));
    cbins_.alloc(static_cast<size_t>(n_) * std::max(1, F_));
    hipLaunchKernelGGL(transpose_bins_kernel, dim3(GridFor(n_)), dim3(256), 0, stream_, bins_.get(), S_, F_, n_,
                       cbins_.get());
    SML_HIP_CHECK(hipGetLastError());
    label_.alloc(n_);
    SML_HIP_CHECK(hipMemcpyAsync(label_.get(), d->label.data(), sizeof(float) * n_, hipMemcpyHostToDevice, stream_));
    if (!d->weight.empty()) {
      weight_.alloc(n_);
      SML_HIP_CHECK(hipMemcpyAsync(weight_.get(), d->weight.data(), sizeof(float) * n_, hipMemcpyHostToDevice, stream_));
    }
    score_.alloc(static_cast<size_t>(n_) * K);
    g_.alloc(static_cast<size_t>(n_) * K);
    h_.alloc(static_cast<size_t>(n_) * K);
    for (int b = 0; b < 2; ++b) { perm_[b].alloc(n_); ogh_[b].alloc(n_); }
    slab_.alloc(static_cast<size_t>(kMaxHistBlocks) * E_);
    part_.alloc(static_cast<size_t>(kReduceSplit) * E_);
    hist_pool_.alloc(static_cast<size_t>(2 * L_ + 2) * E_);
    count_slot_.alloc(1);
    fbest_.alloc(2 * F_);
    lbest_.alloc(L_);
    lgain_.alloc(L_);
    leaves_.alloc(L_);
    state_.alloc(1);
    counts_.alloc(kMaxPartBlocks);
    // feature meta
    std::vector<int32_t> nb(F_), mt(F_), db(F_), ic(F_);
    for (int f = 0; f < F_; ++f) {
      const BinMapper& m = d->ref.mappers[d->ref.used_features[f]];
      nb[f] = m.num_bin; mt[f] = m.missing_type; db[f] = m.default_bin; ic[f] = m.is_categorical ? 1 : 0;
    }
    meta_i_.alloc(4 * F_);
    SML_HIP_CHECK(hipMemcpy(meta_i_.get(), nb.data(), sizeof(int32_t) * F_, hipMemcpyHostToDevice));
    SML_HIP_CHECK(hipMemcpy(meta_i_.get() + F_, mt.data(), sizeof(int32_t) * F_, hipMemcpyHostToDevice));
    SML_HIP_CHECK(hipMemcpy(meta_i_.get() + 2 * F_, db.data(), sizeof(int32_t) * F_, hipMemcpyHostToDevice));
    SML_HIP_CHECK(hipMemcpy(meta_i_.get() + 3 * F_, ic.data(), sizeof(int32_t) * F_, hipMemcpyHostToDevice));
    mask_.alloc(F_);
    fm_.num_bin = meta_i_.get(); fm_.missing = meta_i_.get() + F_; fm_.default_bin = meta_i_.get() + 2 * F_;
    fm_.is_cat = meta_i_.get() + 3 * F_; fm_.mask = mask_.get();
    // device tree
    const int NI = L_ - 1;
    tree_i_.alloc(static_cast<size_t>(NI) * 6 + L_ * 2);
    tree_u_.alloc(static_cast<size_t>(NI) * 9);
    tree_d_.alloc(static_cast<size_t>(NI) * 3 + L_ * 2);
    tree_l_.alloc(static_cast<size_t>(NI) + L_);
    int32_t* ti = tree_i_.get();
    dt_.feat = ti; dt_.dleft = ti + NI; dt_.is_cat = ti + 2 * NI; dt_.left = ti + 3 * NI; dt_.right = ti + 4 * NI;
    dt_.lparent = ti + 6 * NI; dt_.ldepth = ti + 6 * NI + L_;
    flags_ = ti + 5 * NI;
    dt_.thr = tree_u_.get(); dt_.cat_bits = tree_u_.get() + NI;
    double* td = tree_d_.get();
    dt_.gain = td; dt_.ival = td + NI; dt_.iweight = td + 2 * NI; dt_.lval = td + 3 * NI; dt_.lweight = td + 3 * NI + L_;
    dt_.icount = tree_l_.get(); dt_.lcount = tree_l_.get() + NI;
    // score-update tree (uploaded from host trees)
    up_nodes_.alloc(static_cast<size_t>(NI) + 1);
    up_u_.alloc(static_cast<size_t>(NI) * 8 + 8);
    up_d_.alloc(L_ + 4);
    leaf_idx_.alloc(n_);
    SML_HIP_CHECK(hipHostMalloc(&pinned_, kPinnedBytes, hipHostMallocDefault));
    SML_HIP_CHECK(hipStreamSynchronize(stream_));
  }

  void SetScores(const std::vector<double>& s) override {
    SML_HIP_CHECK(hipMemcpyAsync(score_.get(), s.data(), sizeof(double) * s.size(), hipMemcpyHostToDevice, stream_));
    SML_HIP_CHECK(hipStreamSynchronize(stream_));
  }
  void GetScores(std::vector<double>* s) override {
    s->resize(static_cast<size_t>(n_) * K_);
    SML_HIP_CHECK(hipMemcpyAsync(s->data(), score_.get(), sizeof(double) * s->size(), hipMemcpyDeviceToHost, stream_));
    SML_HIP_CHECK(hipStreamSynchronize(stream_));
  }
  void AddBias(int k, double b) override {
    hipLaunchKernelGGL(axpby_kernel, dim3(GridFor(n_)), dim3(256), 0, stream_, score_.get() + k * n_, n_, 1.0, b);
    SML_HIP_CHECK(hipGetLastError());
  }
  void ScaleScore(int k, double sc) override {
    hipLaunchKernelGGL(axpby_kernel, dim3(GridFor(n_)), dim3(256), 0, stream_, score_.get() + k * n_, n_, sc, 0.0);
    SML_HIP_CHECK(hipGetLastError());
  }
  void ComputeGradients(const Objective& obj) override {
    const ObjParams& p = obj.params();
    if (p.kind == kObjLambdarank || p.kind == kObjCustom) {
      // ranking gradients are computed per query on the host (v1)
      std::vector<double> sc;
      GetScores(&sc);
      std::vector<float> g(static_cast<size_t>(n_) * K_), h(g.size());
      obj.GetGradients(sc.data(), g.data(), h.data());
      SetGradients(g.data(), h.data());
      return;
    }
    auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(grad_kernel, dim3(GridFor(n_)), dim3(256), 0, stream_, p, score_.get(), label_.get(),
                       weight_.get(), g_.get(), h_.get(), n_);
    SML_HIP_CHECK(hipGetLastError());
    stats.grad_ms += Ms(t0);
  }
  void SetGradients(const float* g, const float* h) override {
    SML_HIP_CHECK(hipMemcpyAsync(g_.get(), g, sizeof(float) * n_ * K_, hipMemcpyHostToDevice, stream_));
    SML_HIP_CHECK(hipMemcpyAsync(h_.get(), h, sizeof(float) * n_ * K_, hipMemcpyHostToDevice, stream_));
    SML_HIP_CHECK(hipStreamSynchronize(stream_));
  }
  void GetGradients(std::vector<float>* g, std::vector<float>* h) override {
    g->resize(static_cast<size_t>(n_) * K_); h->resize(g->size());
    SML_HIP_CHECK(hipMemcpyAsync(g->data(), g_.get(), sizeof(float) * g->size(), hipMemcpyDeviceToHost, stream_));
    SML_HIP_CHECK(hipMemcpyAsync(h->data(), h_.get(), sizeof(float) * h->size(), hipMemcpyDeviceToHost, stream_));
    SML_HIP_CHECK(hipStreamSynchronize(stream_));
  }
  void SetBag(const std::vector<int32_t>* rows) override {
    if (!rows) { bag_n_ = -1; return; }
    bag_n_ = static_cast<int32_t>(rows->size());
    bag_.alloc(std::max<size_t>(1, rows->size()));
    SML_HIP_CHECK(hipMemcpyAsync(bag_.get(), rows->data(), sizeof(int32_t) * rows->size(), hipMemcpyHostToDevice, stream_));
    SML_HIP_CHECK(hipStreamSynchronize(stream_));
  }

  void Synchronize() override { SML_HIP_CHECK(hipStreamSynchronize(stream_)); }

  Tree TrainTree(int k, const std::vector<char>& fmask_in) override {
    std::vector<int8_t> fmask(F_, 1);
    for (int f = 0; f < F_ && f < static_cast<int>(fmask_in.size()); ++f) fmask[f] = fmask_in[f] ? 1 : 0;
    SML_HIP_CHECK(hipMemcpyAsync(mask_.get(), fmask.data(), F_, hipMemcpyHostToDevice, stream_));
    const float* g = g_.get() + static_cast<size_t>(k) * n_;
    const float* h = h_.get() + static_cast<size_t>(k) * n_;
    int32_t root_count = static_cast<int32_t>(n_);
    int root_buf = -1;
    if (bag_n_ >= 0) {
      root_count = bag_n_;
      root_buf = 0;
      hipLaunchKernelGGL(gather_bag_kernel, dim3(GridFor(std::max(1, bag_n_))), dim3(256), 0, stream_, bag_.get(), bag_n_,
                         g, h, perm_[0].get(), ogh_[0].get());
      SML_HIP_CHECK(hipGetLastError());
    }
    if (hist_mode_ != 0) {
      SML_HIP_CHECK(hipMemsetAsync(ghmax_.get(), 0, 2 * sizeof(unsigned int), stream_));
      hipLaunchKernelGGL(ghmax_kernel, dim3(GridFor(n_) < 2048 ? GridFor(n_) : 2048), dim3(256), 0, stream_, g, h, n_,
                         ghmax_.get());
      SML_HIP_CHECK(hipGetLastError());
    }
    hipLaunchKernelGGL(root_init_kernel, dim3(1), dim3(64), 0, stream_, state_.get(), leaves_.get(), root_count, root_buf, L_);
    SML_HIP_CHECK(hipGetLastError());
    // root histogram + split search
    EnqueueHistogram(g, h);
    EnqueueFindChoose();
    for (int s = 1; s < L_; ++s) {
      // partition the chosen leaf, histogram its smaller child, search both
      hipLaunchKernelGGL(part_count_kernel, dim3(kMaxPartBlocks), dim3(kPartThreads), 0, stream_, state_.get(),
                         leaves_.get(), lbest_.get(), cbins_.get(), n_, perm_[0].get(), perm_[1].get(), fm_, counts_.get());
      SML_HIP_CHECK(hipGetLastError());
      hipLaunchKernelGGL(part_scatter_kernel, dim3(kMaxPartBlocks), dim3(kPartThreads), 0, stream_, state_.get(),
                         leaves_.get(), lbest_.get(), cbins_.get(), n_, perm_[0].get(), perm_[1].get(), ogh_[0].get(),
                         ogh_[1].get(), perm_[0].get(), perm_[1].get(), ogh_[0].get(), ogh_[1].get(), g, h, fm_,
                         counts_.get());
      SML_HIP_CHECK(hipGetLastError());
      EnqueueHistogram(g, h);
      EnqueueFindChoose();
    }
    // read the tree back (one transfer, one sync)
    Tree t = ReadTree();
    return t;
  }

  void UpdateScore(const Tree& t, int k, double scale) override {
    DevTreeView tv = UploadTree(t);
    hipLaunchKernelGGL(score_kernel, dim3(GridFor(n_)), dim3(256), 0, stream_, tv, cbins_.get(), n_, fm_, scale,
                       score_.get() + static_cast<size_t>(k) * n_, static_cast<int32_t*>(nullptr));
    SML_HIP_CHECK(hipGetLastError());
  }

  void PredictLeafIndex(const Tree& t, std::vector<int32_t>* leaf) override {
    DevTreeView tv = UploadTree(t);
    hipLaunchKernelGGL(score_kernel, dim3(GridFor(n_)), dim3(256), 0, stream_, tv, cbins_.get(), n_, fm_, 0.0,
                       static_cast<double*>(nullptr), leaf_idx_.get());
    SML_HIP_CHECK(hipGetLastError());
    leaf->resize(n_);
    SML_HIP_CHECK(hipMemcpyAsync(leaf->data(), leaf_idx_.get(), sizeof(int32_t) * n_, hipMemcpyDeviceToHost, stream_));
    SML_HIP_CHECK(hipStreamSynchronize(stream_));
  }

 private:
  static double Ms(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  static int GridFor(int64_t n) {
    int64_t b = (n + 255) / 256;
    return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(b, 8192)));
  }

  void EnqueueHistogram(const float* g, const float* h) {
    auto launch = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(kMaxHistBlocks, FG_), dim3(kHistThreads), 0, stream_, state_.get(), leaves_.get(),
                         reinterpret_cast<const uint4*>(bins_.get()), S_ / 16, F_, perm_[0].get(), perm_[1].get(),
                         ogh_[0].get(), ogh_[1].get(), g, h, reinterpret_cast<const float*>(ghmax_.get()), slab_.get());
    };
    if (hist_mode_ == 1) launch(hist_kernel<1>);
    else if (hist_mode_ == 2) launch(hist_kernel<2>);
    else launch(hist_kernel<0>);
    SML_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(hist_reduce_kernel, dim3((E_ + 255) / 256, kReduceSplit), dim3(256), 0, stream_, state_.get(),
                       leaves_.get(), slab_.get(), E_, part_.get(), count_slot_.get());
    SML_HIP_CHECK(hipGetLastError());
    if (comm_ && comm_->world() > 1) {
      // fold the partial sums into part[0] (and the row count next to it), then
      // one allreduce of E*2+1 doubles over RCCL
      hipLaunchKernelGGL(fold_parts_kernel, dim3((E_ + 255) / 256), dim3(256), 0, stream_, part_.get(), E_,
                         count_slot_.get());
      SML_HIP_CHECK(hipGetLastError());
      auto t0 = std::chrono::steady_clock::now();
      comm_->AllReduceDeviceF64(reinterpret_cast<double*>(part_.get()), static_cast<int64_t>(E_) * 2 + 1, stream_);
      stats.comm_ms += Ms(t0);
      hipLaunchKernelGGL(unfold_count_kernel, dim3(1), dim3(64), 0, stream_, part_.get(), E_, count_slot_.get());
      SML_HIP_CHECK(hipGetLastError());
    }
  }

  void EnqueueFindChoose() {
    hipLaunchKernelGGL(find_split_kernel, dim3(F_, 2), dim3(256), 0, stream_, state_.get(), leaves_.get(), part_.get(),
                       E_, count_slot_.get(), hist_pool_.get(), fm_, sp_, fbest_.get(), F_);
    SML_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(choose_kernel, dim3(1), dim3(256), 0, stream_, state_.get(), leaves_.get(), lbest_.get(),
                       lgain_.get(), fbest_.get(), F_, dt_, count_slot_.get());
    SML_HIP_CHECK(hipGetLastError());
  }

  Tree ReadTree() {
    const int NI = L_ - 1;
    DState st;
    SML_HIP_CHECK(hipMemcpyAsync(&st, state_.get(), sizeof(DState), hipMemcpyDeviceToHost, stream_));
    std::vector<int32_t> ti(tree_i_.n);
    std::vector<uint32_t> tu(tree_u_.n);
    std::vector<double> td(tree_d_.n);
    std::vector<int64_t> tl(tree_l_.n);
    SML_HIP_CHECK(hipMemcpyAsync(ti.data(), tree_i_.get(), sizeof(int32_t) * ti.size(), hipMemcpyDeviceToHost, stream_));
    SML_HIP_CHECK(hipMemcpyAsync(tu.data(), tree_u_.get(), sizeof(uint32_t) * tu.size(), hipMemcpyDeviceToHost, stream_));
    SML_HIP_CHECK(hipMemcpyAsync(td.data(), tree_d_.get(), sizeof(double) * td.size(), hipMemcpyDeviceToHost, stream_));
    SML_HIP_CHECK(hipMemcpyAsync(tl.data(), tree_l_.get(), sizeof(int64_t) * tl.size(), hipMemcpyDeviceToHost, stream_));
    SML_HIP_CHECK(hipStreamSynchronize(stream_));
    const int nl = st.num_leaves;
    Tree t(L_);
    t.num_leaves = nl;
    const auto& ref = data_->ref;
    // leaf 0 of a stump: LeafOutput of the root
    for (int node = 0; node < nl - 1; ++node) {
      const int fi = ti[node];
      const int fr = ref.used_features[fi];
      const BinMapper& m = ref.mappers[fr];
      t.split_feature_inner[node] = fi;
      t.split_feature[node] = fr;
      t.split_gain[node] = td[node];
      t.left_child[node] = ti[3 * NI + node];
      t.right_child[node] = ti[4 * NI + node];
      t.internal_value[node] = td[NI + node];
      t.internal_weight[node] = td[2 * NI + node];
      t.internal_count[node] = tl[node];
      const bool is_cat = ti[2 * NI + node] != 0;
      if (is_cat) {
        std::vector<uint32_t> binbits(8), valbits;
        int maxcat = 0;
        for (int w = 0; w < 8; ++w) binbits[w] = tu[NI + node * 8 + w];
        for (int b = 0; b < m.num_bin - 1; ++b) if ((binbits[b / 32] >> (b % 32)) & 1u) maxcat = std::max(maxcat, m.bin2cat[b]);
        valbits.assign(maxcat / 32 + 1, 0);
        for (int b = 0; b < m.num_bin - 1; ++b)
          if ((binbits[b / 32] >> (b % 32)) & 1u) valbits[m.bin2cat[b] / 32] |= 1u << (m.bin2cat[b] % 32);
        t.threshold_in_bin[node] = static_cast<uint32_t>(t.num_cat);
        t.threshold[node] = static_cast<double>(t.num_cat);
        t.decision_type[node] = MakeDecisionType(true, false, kMissingNaN);
        t.cat_threshold.insert(t.cat_threshold.end(), valbits.begin(), valbits.end());
        t.cat_boundaries.push_back(static_cast<int>(t.cat_threshold.size()));
        t.cat_threshold_inner.insert(t.cat_threshold_inner.end(), binbits.begin(), binbits.end());
        t.cat_boundaries_inner.push_back(static_cast<int>(t.cat_threshold_inner.size()));
        ++t.num_cat;
      } else {
        const uint32_t thr = tu[node];
        t.threshold_in_bin[node] = thr;
        t.threshold[node] = m.BinToValue(thr);
        t.decision_type[node] = MakeDecisionType(false, ti[NI + node] != 0, m.missing_type);
      }
    }
    for (int l = 0; l < nl; ++l) {
      t.leaf_value[l] = td[3 * NI + l];
      t.leaf_weight[l] = td[3 * NI + L_ + l];
      t.leaf_count[l] = tl[NI + l];
      t.leaf_parent[l] = ti[6 * NI + l];
      t.leaf_depth[l] = ti[6 * NI + L_ + l];
    }
    if (nl == 1) t.leaf_value[0] = 0.0;
    return t;
  }

  DevTreeView UploadTree(const Tree& t) {
    const int NI = std::max(1, t.num_leaves - 1);
    const size_t need_n = static_cast<size_t>(NI), need_u = static_cast<size_t>(NI) * 8, need_d = t.num_leaves;
    if (need_n > up_nodes_.n) up_nodes_.alloc(need_n);
    if (need_u > up_u_.n) up_u_.alloc(need_u);
    if (need_d > up_d_.n) up_d_.alloc(need_d);
    const size_t bytes = need_n * 16 + need_u * 4 + need_d * 8;
    if (bytes > kPinnedBytes) throw std::runtime_error("tree too large for staging buffer");
    SML_HIP_CHECK(hipStreamSynchronize(stream_));  // pinned buffer reuse
    int4* pn = static_cast<int4*>(pinned_);
    uint32_t* pu = reinterpret_cast<uint32_t*>(pn + need_n);
    double* pd = reinterpret_cast<double*>(pu + need_u);
    for (int node = 0; node < t.num_leaves - 1; ++node) {
      const int8_t dt = t.decision_type[node];
      const int mt = (dt >> 2) & 3, dl = (dt >> 1) & 1, ic = dt & 1;
      pn[node] = make_int4(t.split_feature_inner[node] | (mt << 16) | (dl << 18) | (ic << 19),
                           static_cast<int>(t.threshold_in_bin[node]), t.left_child[node], t.right_child[node]);
      for (int w = 0; w < 8; ++w) pu[node * 8 + w] = 0;
      if (ic) {
        int ci = static_cast<int>(t.threshold_in_bin[node]);
        int s0 = t.cat_boundaries_inner[ci], e0 = t.cat_boundaries_inner[ci + 1];
        for (int w = 0; w < 8 && s0 + w < e0; ++w) pu[node * 8 + w] = t.cat_threshold_inner[s0 + w];
      }
    }
    for (int l = 0; l < t.num_leaves; ++l) pd[l] = t.leaf_value[l];
    SML_HIP_CHECK(hipMemcpyAsync(up_nodes_.get(), pn, need_n * 16, hipMemcpyHostToDevice, stream_));
    SML_HIP_CHECK(hipMemcpyAsync(up_u_.get(), pu, need_u * 4, hipMemcpyHostToDevice, stream_));
    SML_HIP_CHECK(hipMemcpyAsync(up_d_.get(), pd, need_d * 8, hipMemcpyHostToDevice, stream_));
    DevTreeView tv;
    tv.nodes = up_nodes_.get(); tv.cat_bits = up_u_.get(); tv.lval = up_d_.get(); tv.num_leaves = t.num_leaves;
    return tv;
  }

  static constexpr size_t kPinnedBytes = 4 << 20;
  int dev_ = -1;
  hipStream_t stream_ = nullptr;
  const Dataset* data_ = nullptr;
  Config cfg_;
  SplitParams sp_{};
  int K_ = 1, F_ = 0, S_ = 4, W_ = 1, E_ = 0, L_ = 2, FG_ = 1;
  int64_t n_ = 0;
  int32_t bag_n_ = -1;
  DevBuf<uint8_t> bins_, cbins_;
  DevBuf<float> label_, weight_, g_, h_;
  DevBuf<double> score_;
  DevBuf<int32_t> perm_[2];
  DevBuf<float2> ogh_[2];
  DevBuf<float2> slab_;
  DevBuf<double2> part_, hist_pool_;
  DevBuf<double> count_slot_, lgain_;
  DevBuf<SplitResult> fbest_, lbest_;
  DevBuf<DLeaf> leaves_;
  DevBuf<DState> state_;
  DevBuf<int32_t> counts_, meta_i_, bag_;
  DevBuf<int8_t> mask_;
  DevBuf<unsigned int> ghmax_;
  int hist_mode_ = 1;
  DevBuf<int32_t> tree_i_;
  DevBuf<uint32_t> tree_u_;
  DevBuf<double> tree_d_;
  DevBuf<int64_t> tree_l_;
  DevBuf<int4> up_nodes_;
  DevBuf<uint32_t> up_u_;
  DevBuf<double> up_d_;
  DevBuf<int32_t> leaf_idx_;
  int32_t* flags_ = nullptr;
  DTree dt_{};
  FeatMeta fm_{};
  void* pinned_ = nullptr;
};

}  // namespace

bool GpuAvailable() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) { (void)hipGetLastError(); return false; }
  return n > 0;
}

std::unique_ptr<TrainBackend> MakeGpuBackend(int device_id) {
  if (!GpuAvailable()) return nullptr;
  return std::unique_ptr<TrainBackend>(new GpuBackend(device_id));
}

}  // namespace sml
