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
// features. Rows' bins are fetched as dwords (4 features), gradients as float2
// from the ordered copy (or the physical arrays for an unpartitioned root).
__global__ __launch_bounds__(kHistThreads) void hist_kernel(
    const DState* __restrict__ st, const DLeaf* __restrict__ leaves, const uint32_t* __restrict__ bins,
    int W, int F, const int32_t* __restrict__ perm0, const int32_t* __restrict__ perm1,
    const float2* __restrict__ ogh0, const float2* __restrict__ ogh1, const float* __restrict__ g,
    const float* __restrict__ h, float2* __restrict__ slab) {
  if (st->done) return;
  const DLeaf L = HistSeg(st, leaves);
  const int count = L.count;
  const int nb_active = max(1, min(kMaxHistBlocks, ceil_div_i(count, kMinRowsPerHistBlock)));
  if (static_cast<int>(blockIdx.x) >= nb_active) return;
  __shared__ float sh[2 * kFeatPerGroup * kHistStride];
  const int tid = threadIdx.x;
  for (int i = tid; i < 2 * kFeatPerGroup * kHistStride; i += kHistThreads) sh[i] = 0.f;
  __syncthreads();
  const int grp = blockIdx.y;
  const int Wg = min(kFeatPerGroup / 4, W - grp * (kFeatPerGroup / 4));
  const int Fg = min(kFeatPerGroup, F - grp * kFeatPerGroup);
  const int chunk = ceil_div_i(count, nb_active);
  const int p0 = L.begin + blockIdx.x * chunk;
  const int p1 = min(L.begin + count, p0 + chunk);
  const int32_t* perm = L.buf == 0 ? perm0 : perm1;
  const float2* ogh = L.buf == 0 ? ogh0 : ogh1;
  const bool phys = L.buf < 0;
  if (p1 > p0) {
    const int items = (p1 - p0) * Wg;
    for (int it = tid; it < items; it += kHistThreads) {
      const int q = it / Wg;
      const int w = it - q * Wg;
      const int pos = p0 + q;
      int r;
      float2 v;
      if (phys) { r = pos; v = make_float2(g[r], h[r]); }
      else { r = perm[pos]; v = ogh[pos]; }
      const uint32_t b4 = bins[static_cast<size_t>(r) * W + grp * (kFeatPerGroup / 4) + w];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int f = w * 4 + j;
        if (f < Fg) {
          const uint32_t b = (b4 >> (8 * j)) & 255u;
          atomicAdd(&sh[f * kHistStride + b], v.x);
          atomicAdd(&sh[kFeatPerGroup * kHistStride + f * kHistStride + b], v.y);
        }
      }
    }
  }
  __syncthreads();
  float2* out = slab + static_cast<size_t>(blockIdx.x) * F * kBinsPerFeature;
  for (int i = tid; i < Fg * kBinsPerFeature; i += kHistThreads) {
    const int f = i >> 8, b = i & 255;
    out[(grp * kFeatPerGroup + f) * kBinsPerFeature + b] =
        make_float2(sh[f * kHistStride + b], sh[kFeatPerGroup * kHistStride + f * kHistStride + b]);
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
      // recompute the winning prefix (serial, cheap) for exact sums
      double gl = 0, hl = 0;
      for (int t = 0; t <= b.thr; ++t) if (t != zero_bin && t != nan_bin) { gl += sg_[t]; hl += shh_[t]; }
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
// One block. Reduces the per-feature results of the new leaves, then picks the
// next leaf to split (max gain), records the split in the device tree and sets
// up the partition of that leaf.
__global__ __launch_bounds__(256) void choose_kernel(DState* __restrict__ st, DLeaf* __restrict__ leaves,
                                                     SplitResult* __restrict__ lbest,
                                                     const SplitResult* __restrict__ fbest, int F, DTree t,
                                                     const int32_t* __restrict__ feat_missing,
                                                     const double* __restrict__ count_slot) {
  if (st->done) return;
  const int tid = threadIdx.x;
  __shared__ int sh_best_child[2];
  const bool root = st->phase == 0;
  const int nchild = root ? 1 : 2;
  // per-child argmax over features (thread 0/1 serially; F is small)
  if (tid < nchild) {
    int bi = -1;
    for (int f = 0; f < F; ++f) {
      const SplitResult& r = fbest[tid * F + f];
      if (r.feature < 0) continue;
      if (bi < 0 || SplitBetter(r.gain, r.feature, r.threshold, fbest[tid * F + bi].gain, fbest[tid * F + bi].feature,
                                fbest[tid * F + bi].threshold))
        bi = f;
    }
    sh_best_child[tid] = bi;
  }
  __syncthreads();
  if (tid != 0) return;
  // store leaf bests + global counts
  if (root) {
    const int bi = sh_best_child[0];
    if (bi >= 0) lbest[0] = fbest[bi]; else { lbest[0].feature = -1; lbest[0].gain = -INFINITY; }
    t.lval[0] = 0.0;
    t.lcount[0] = leaves[0].gcount;
    t.lweight[0] = leaves[0].sum_h;
    t.lparent[0] = -1;
    t.ldepth[0] = 0;
  } else {
    const int64_t small_cnt = static_cast<int64_t>(*count_slot);
    const int s = st->small_leaf, l = st->large_leaf;
    const int64_t parent_cnt = leaves[l].gcount;  // choose stored parent count here
    {
      const int ob = st->pbuf == 0 ? 1 : 0;
      DLeaf& Lc = leaves[st->split_leaf];
      DLeaf& Rc = leaves[st->new_leaf];
      Lc.begin = st->pbegin; Lc.count = st->ptotal; Lc.buf = ob;
      Rc.begin = st->pbegin + st->ptotal; Rc.count = st->pcount - st->ptotal; Rc.buf = ob;
    }
    leaves[s].gcount = small_cnt;
    leaves[l].gcount = parent_cnt - small_cnt;
    t.lcount[s] = leaves[s].gcount;
    t.lcount[l] = leaves[l].gcount;
    for (int c = 0; c < 2; ++c) {
      const int leaf = c == 0 ? s : l;
      const int bi = sh_best_child[c];
      if (bi >= 0) lbest[leaf] = fbest[c * F + bi]; else { lbest[leaf].feature = -1; lbest[leaf].gain = -INFINITY; }
    }
  }
  // pick the next leaf
  const int nl = st->num_leaves;
  if (nl >= st->max_leaves) { st->done = 1; return; }
  int bl = -1;
  for (int i = 0; i < nl; ++i) {
    if (lbest[i].feature < 0) continue;
    if (bl < 0 || lbest[i].gain > lbest[bl].gain) bl = i;
  }
  if (bl < 0 || !(lbest[bl].gain > 0.0)) { st->done = 1; return; }
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
  // leaf records for the children (segments are filled by the partition)
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
  st->pbegin = P.begin; st->pcount = P.count; st->pbuf = P.buf; st->ptotal = 0;
  st->split_leaf = bl;
  st->new_leaf = nl;
  st->small_leaf = left_small ? bl : nl;
  st->large_leaf = left_small ? nl : bl;
  st->num_leaves = nl + 1;
  st->phase = 1;
  (void)feat_missing;
}

// ---------------------------------------------------------------- K6
__device__ __forceinline__ bool RowGoesLeft(const uint8_t* bins8, int S, int r, const SplitResult& sr, FeatMeta fm) {
  const int f = sr.feature;
  const uint32_t b = bins8[static_cast<size_t>(r) * S + f];
  return DeviceGoesLeft(b, fm.num_bin[f], fm.missing[f], fm.default_bin[f], sr.is_cat, sr.threshold,
                        sr.default_left, sr.cat_bits);
}

__global__ __launch_bounds__(kPartThreads) void part_count_kernel(
    const DState* __restrict__ st, const DLeaf* __restrict__ leaves, const SplitResult* __restrict__ lbest,
    const uint8_t* __restrict__ bins8, int S, const int32_t* __restrict__ perm0,
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
    c += RowGoesLeft(bins8, S, r, sr, fm) ? 1 : 0;
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
    const uint8_t* __restrict__ bins8, int S, const int32_t* __restrict__ perm0, const int32_t* __restrict__ perm1,
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
      left = RowGoesLeft(bins8, S, r, sr, fm);
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
struct DevTreeView {
  const int32_t* feat;
  const uint32_t* thr;
  const int32_t* flags;  // bit0 cat, bit1 default_left, bits2-3 missing
  const int32_t* left;
  const int32_t* right;
  const uint32_t* cat_bits;  // 8 words per node
  const double* lval;
  int num_leaves;
};

__global__ void score_kernel(DevTreeView tv, const uint8_t* __restrict__ bins8, int S, int64_t n,
                             FeatMeta fm, double scale, double* __restrict__ score, int32_t* __restrict__ leaf_out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int node = 0;
    if (tv.num_leaves > 1) {
      const uint8_t* row = bins8 + i * S;
      for (int guard = 0; node >= 0 && guard < tv.num_leaves; ++guard) {
        const int f = tv.feat[node];
        const int fl = tv.flags[node];
        const bool left = DeviceGoesLeft(row[f], fm.num_bin[f], (fl >> 2) & 3, fm.default_bin[f], fl & 1,
                                         tv.thr[node], (fl >> 1) & 1, tv.cat_bits + node * 8);
        node = left ? tv.left[node] : tv.right[node];
      }
      node = node < 0 ? ~node : 0;  // a malformed tree cannot loop forever
    }
    if (score) score[i] += scale * tv.lval[node];
    if (leaf_out) leaf_out[i] = node;
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
    F_ = d->ref.num_inner();
    S_ = d->row_stride;
    W_ = S_ / 4;
    E_ = F_ * kBinsPerFeature;
    L_ = std::max(2, cfg.num_leaves);
    FG_ = (F_ + kFeatPerGroup - 1) / kFeatPerGroup;
    bins_.alloc(static_cast<size_t>(n_) * S_);
    SML_HIP_CHECK(hipMemcpyAsync(bins_.get(), d->bins.data(), static_cast<size_t>(n_) * S_, hipMemcpyHostToDevice, stream_));
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
    up_i_.alloc(static_cast<size_t>(NI) * 4 + 4);
    up_u_.alloc(static_cast<size_t>(NI) * 9 + 4);
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
    hipLaunchKernelGGL(root_init_kernel, dim3(1), dim3(64), 0, stream_, state_.get(), leaves_.get(), root_count, root_buf, L_);
    SML_HIP_CHECK(hipGetLastError());
    // root histogram + split search
    EnqueueHistogram(g, h);
    EnqueueFindChoose();
    for (int s = 1; s < L_; ++s) {
      // partition the chosen leaf, histogram its smaller child, search both
      hipLaunchKernelGGL(part_count_kernel, dim3(kMaxPartBlocks), dim3(kPartThreads), 0, stream_, state_.get(),
                         leaves_.get(), lbest_.get(), bins_.get(), S_, perm_[0].get(), perm_[1].get(), fm_, counts_.get());
      SML_HIP_CHECK(hipGetLastError());
      hipLaunchKernelGGL(part_scatter_kernel, dim3(kMaxPartBlocks), dim3(kPartThreads), 0, stream_, state_.get(),
                         leaves_.get(), lbest_.get(), bins_.get(), S_, perm_[0].get(), perm_[1].get(), ogh_[0].get(),
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
    hipLaunchKernelGGL(score_kernel, dim3(GridFor(n_)), dim3(256), 0, stream_, tv, bins_.get(), S_, n_, fm_, scale,
                       score_.get() + static_cast<size_t>(k) * n_, static_cast<int32_t*>(nullptr));
    SML_HIP_CHECK(hipGetLastError());
  }

  void PredictLeafIndex(const Tree& t, std::vector<int32_t>* leaf) override {
    DevTreeView tv = UploadTree(t);
    hipLaunchKernelGGL(score_kernel, dim3(GridFor(n_)), dim3(256), 0, stream_, tv, bins_.get(), S_, n_, fm_, 0.0,
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
    hipLaunchKernelGGL(hist_kernel, dim3(kMaxHistBlocks, FG_), dim3(kHistThreads), 0, stream_, state_.get(),
                       leaves_.get(), reinterpret_cast<const uint32_t*>(bins_.get()), W_, F_, perm_[0].get(),
                       perm_[1].get(), ogh_[0].get(), ogh_[1].get(), g, h, slab_.get());
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
                       fbest_.get(), F_, dt_, fm_.missing, count_slot_.get());
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
    const size_t need_i = static_cast<size_t>(NI) * 4, need_u = static_cast<size_t>(NI) * 9, need_d = t.num_leaves;
    if (need_i > up_i_.n) up_i_.alloc(need_i);
    if (need_u > up_u_.n) up_u_.alloc(need_u);
    if (need_d > up_d_.n) up_d_.alloc(need_d);
    // stage everything in the pinned buffer, then 3 async copies
    const size_t bytes = need_i * 4 + need_u * 4 + need_d * 8;
    if (bytes > kPinnedBytes) throw std::runtime_error("tree too large for staging buffer");
    SML_HIP_CHECK(hipStreamSynchronize(stream_));  // pinned buffer reuse
    int32_t* pi = static_cast<int32_t*>(pinned_);
    uint32_t* pu = reinterpret_cast<uint32_t*>(pi + need_i);
    double* pd = reinterpret_cast<double*>(pu + need_u + (need_u & 1));
    for (int node = 0; node < t.num_leaves - 1; ++node) {
      pi[node] = t.split_feature_inner[node];
      pi[NI + node] = static_cast<int32_t>(t.decision_type[node]);
      pi[2 * NI + node] = t.left_child[node];
      pi[3 * NI + node] = t.right_child[node];
      pu[node] = t.threshold_in_bin[node];
      for (int w = 0; w < 8; ++w) pu[NI + node * 8 + w] = 0;
      if (t.decision_type[node] & 1) {
        int ci = static_cast<int>(t.threshold_in_bin[node]);
        int s = t.cat_boundaries_inner[ci], e = t.cat_boundaries_inner[ci + 1];
        for (int w = 0; w < 8 && s + w < e; ++w) pu[NI + node * 8 + w] = t.cat_threshold_inner[s + w];
      }
    }
    for (int l = 0; l < t.num_leaves; ++l) pd[l] = t.leaf_value[l];
    SML_HIP_CHECK(hipMemcpyAsync(up_i_.get(), pi, need_i * 4, hipMemcpyHostToDevice, stream_));
    SML_HIP_CHECK(hipMemcpyAsync(up_u_.get(), pu, need_u * 4, hipMemcpyHostToDevice, stream_));
    SML_HIP_CHECK(hipMemcpyAsync(up_d_.get(), pd, need_d * 8, hipMemcpyHostToDevice, stream_));
    DevTreeView tv;
    tv.feat = up_i_.get(); tv.flags = up_i_.get() + NI; tv.left = up_i_.get() + 2 * NI; tv.right = up_i_.get() + 3 * NI;
    tv.thr = up_u_.get(); tv.cat_bits = up_u_.get() + NI; tv.lval = up_d_.get(); tv.num_leaves = t.num_leaves;
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
  DevBuf<uint8_t> bins_;
  DevBuf<float> label_, weight_, g_, h_;
  DevBuf<double> score_;
  DevBuf<int32_t> perm_[2];
  DevBuf<float2> ogh_[2];
  DevBuf<float2> slab_;
  DevBuf<double2> part_, hist_pool_;
  DevBuf<double> count_slot_;
  DevBuf<SplitResult> fbest_, lbest_;
  DevBuf<DLeaf> leaves_;
  DevBuf<DState> state_;
  DevBuf<int32_t> counts_, meta_i_, bag_;
  DevBuf<int8_t> mask_;
  DevBuf<int32_t> tree_i_;
  DevBuf<uint32_t> tree_u_;
  DevBuf<double> tree_d_;
  DevBuf<int64_t> tree_l_;
  DevBuf<int32_t> up_i_;
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
