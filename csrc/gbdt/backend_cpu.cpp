// CPU training backend: OpenMP histogram construction + host split search.
// It is the numerical oracle for the HIP kernels and the runtime for hosts
// without an MI355X (BASELINE config 1, "local[2] CPU plumbing").
#include <emmintrin.h>
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <numeric>
#include <stdexcept>

#include "backend.h"

#ifdef _OPENMP
#include <omp.h>
#endif

namespace sml {

int BynodeK(const Config& c, const std::vector<char>& allowed) {
  if (c.feature_fraction_bynode >= 1.0) return 0;
  int n = 0;
  for (char a : allowed) n += a ? 1 : 0;
  return std::max(1, static_cast<int>(std::ceil(n * c.feature_fraction_bynode - 1e-9)));
}

SplitParams MakeSplitParams(const Config& c) {
  SplitParams p;
  p.lambda_l1 = c.lambda_l1; p.lambda_l2 = c.lambda_l2; p.max_delta_step = c.max_delta_step;
  p.min_gain_to_split = c.min_gain_to_split; p.min_sum_hessian = c.min_sum_hessian_in_leaf;
  p.min_data_in_leaf = c.min_data_in_leaf; p.num_leaves = c.num_leaves; p.max_depth = c.max_depth;
  p.cat_l2 = c.cat_l2; p.cat_smooth = c.cat_smooth; p.max_cat_threshold = c.max_cat_threshold;
  p.max_cat_to_onehot = c.max_cat_to_onehot; p.min_data_per_group = c.min_data_per_group;
  p.has_mono = 0;
  for (int m : c.monotone_constraints) if (m != 0) p.has_mono = 1;
  p.monotone_penalty = c.monotone_penalty;
  p.bynode_k = 0;  // set per tree by the backends
  p.tree_seq = 0;
  p.bynode_seed = static_cast<unsigned long long>(c.feature_fraction_seed) * 0x2545F4914F6CDD1Dull + 17ull;
  return p;
}

static void ConsiderSplit(double gl, double hl, double gr, double hr, int64_t cl, int64_t cr,
                          double parent_gain, const SplitParams& sp, double l2, int feature,
                          uint32_t thr, int default_left, SplitResult* best, const MonoCtx* mc) {
  if (cl < sp.min_data_in_leaf || cr < sp.min_data_in_leaf) return;
  if (hl < sp.min_sum_hessian || hr < sp.min_sum_hessian) return;
  double gain, lout, rout;
  if (!EvalSplit(gl, hl, gr, hr, sp.lambda_l1, l2, sp.max_delta_step, mc, &gain, &lout, &rout)) return;
  const double shift = parent_gain + sp.min_gain_to_split;
  if (!(gain > shift)) return;
  const double sg = gain - shift;
  if (best->feature >= 0 && !SplitBetter(sg, feature, thr, best->gain, best->feature, best->threshold)) return;
  best->gain = sg;
  best->feature = feature;
  best->threshold = thr;
  best->default_left = default_left;
  best->is_cat = 0;
  best->left_g = gl; best->left_h = hl; best->right_g = gr; best->right_h = hr;
  best->left_cnt = cl; best->right_cnt = cr;
  best->left_out = lout;
  best->right_out = rout;
}

void FindBestSplitFeature(const double* hg, const double* hh, int nb, const BinMapper& m,
                          int fi, double G, double H, int64_t cnt, const SplitParams& sp,
                          SplitResult* best, const MonoCtx* mc) {
  const double cnt_factor = cnt / std::max(H, kEpsilon);
  const double parent_gain = LeafGain(G, H, sp.lambda_l1, sp.lambda_l2, sp.max_delta_step);
  if (m.is_categorical) {
    // one-vs-rest for few categories, otherwise sorted-by-ratio prefix search
    const int other = nb - 1;
    const double l2 = sp.lambda_l2 + sp.cat_l2;
    const double cat_parent = LeafGain(G, H, sp.lambda_l1, l2, sp.max_delta_step);
    SplitResult local = *best;
    bool found = false;
    // categorical splits are clamped into the leaf's bounds but carry no direction
    MonoCtx cat_mc{0.0, 0.0, 0};
    if (mc) cat_mc = MonoCtx{mc->lo, mc->hi, 0};
    const MonoCtx* cmc = mc ? &cat_mc : nullptr;
    auto try_set = [&](const std::vector<int>& left_bins, double gl, double hl) {
      const double gr = G - gl, hr = H - hl;
      const int64_t cl = EstimateCount(hl, cnt_factor), cr = cnt - cl;
      if (cl < sp.min_data_in_leaf || cr < sp.min_data_in_leaf) return;
      if (hl < sp.min_sum_hessian || hr < sp.min_sum_hessian) return;
      if (static_cast<int>(left_bins.size()) > 1 && (cl < sp.min_data_per_group || cr < sp.min_data_per_group)) return;
      double gain, lout, rout;
      if (!EvalSplit(gl, hl, gr, hr, sp.lambda_l1, l2, sp.max_delta_step, cmc, &gain, &lout, &rout)) return;
      const double shift = cat_parent + sp.min_gain_to_split;
      if (!(gain > shift)) return;
      const double sg = gain - shift;
      if (local.feature >= 0 && !SplitBetter(sg, fi, static_cast<uint32_t>(left_bins.size()), local.gain, local.feature, local.threshold)) return;
      local.gain = sg; local.feature = fi; local.threshold = static_cast<uint32_t>(left_bins.size());
      local.default_left = 0; local.is_cat = 1;
      std::memset(local.cat_bits, 0, sizeof(local.cat_bits));
      for (int b : left_bins) local.cat_bits[b / 32] |= 1u << (b % 32);
      local.left_g = gl; local.left_h = hl; local.right_g = gr; local.right_h = hr;
      local.left_cnt = cl; local.right_cnt = cr;
      local.left_out = lout;
      local.right_out = rout;
      found = true;
    };
    if (nb <= sp.max_cat_to_onehot + 1) {
      for (int b = 0; b < other; ++b) try_set({b}, hg[b], hh[b]);
    } else {
      std::vector<int> idx;
      for (int b = 0; b < other; ++b)
        if (EstimateCount(hh[b], cnt_factor) >= sp.cat_smooth) idx.push_back(b);
      std::stable_sort(idx.begin(), idx.end(), [&](int a, int c) {
        return hg[a] / (hh[a] + sp.cat_smooth) < hg[c] / (hh[c] + sp.cat_smooth);
      });
      const int maxk = std::min<int>(sp.max_cat_threshold, (static_cast<int>(idx.size()) + 1) / 2);
      for (int dir = 0; dir < 2; ++dir) {
        std::vector<int> left;
        double gl = 0, hl = 0;
        for (int k = 0; k < static_cast<int>(idx.size()) && k < maxk; ++k) {
          int b = dir == 0 ? idx[k] : idx[idx.size() - 1 - k];
          left.push_back(b);
          gl += hg[b]; hl += hh[b];
          try_set(left, gl, hl);
        }
      }
    }
    if (found) *best = local;
    return;
  }
  const int mt = m.missing_type;
  const int nan_bin = (mt == kMissingNaN) ? nb - 1 : -1;
  const int zero_bin = (mt == kMissingZero) ? m.default_bin : -1;
  double mg = 0, mh = 0;  // missing bin sums
  if (nan_bin >= 0) { mg = hg[nan_bin]; mh = hh[nan_bin]; }
  if (zero_bin >= 0) { mg = hg[zero_bin]; mh = hh[zero_bin]; }
  const int last = (nan_bin >= 0) ? nb - 2 : nb - 1;  // last ordered bin
  double gl = 0, hl = 0;
  for (int t = 0; t < last; ++t) {
    if (t != zero_bin) { gl += hg[t]; hl += hh[t]; }
    if (mt == kMissingNone) {
      const int64_t cl = EstimateCount(hl, cnt_factor);
      ConsiderSplit(gl, hl, G - gl, H - hl, cl, cnt - cl, parent_gain, sp, sp.lambda_l2, fi, t, 1, best, mc);
    } else {
      // missing -> right
      {
        const int64_t cl = EstimateCount(hl, cnt_factor);
        ConsiderSplit(gl, hl, G - gl, H - hl, cl, cnt - cl, parent_gain, sp, sp.lambda_l2, fi, t, 0, best, mc);
      }
      // missing -> left
      {
        const double g2 = gl + mg, h2 = hl + mh;
        const int64_t cl = EstimateCount(h2, cnt_factor);
        ConsiderSplit(g2, h2, G - g2, H - h2, cl, cnt - cl, parent_gain, sp, sp.lambda_l2, fi, t, 1, best, mc);
      }
    }
  }
}

namespace {

using Clock = std::chrono::steady_clock;
inline double Ms(Clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
}

struct ScoreTimer {
  explicit ScoreTimer(double* acc) : acc_(acc), t0_(Clock::now()) {}
  ~ScoreTimer() { *acc_ += Ms(t0_); }
  double* acc_;
  Clock::time_point t0_;
};

struct LeafInfo {
  int64_t begin = 0, count = 0;  // local row range
  int64_t gcount = 0;            // global row count (all ranks)
  double sum_g = 0, sum_h = 0;
  int depth = 0;
  int slot = 0;  // node id for feature_fraction_bynode: root 0, children of internal node i: 2i+1, 2i+2
  double lo = -std::numeric_limits<double>::infinity();  // monotone output bounds
  double hi = std::numeric_limits<double>::infinity();
  SplitResult best;
  bool has_best = false;
};

class CpuBackend : public TrainBackend {
 public:
  std::string Name() const override { return "cpu"; }
  void Init(const Dataset* d, const Config& cfg, int K) override {
    d->EnsureHostBins();  // the host learner reads the host bin matrix
    data_ = d; cfg_ = cfg; K_ = K; n_ = d->num_data;
    if (n_ > static_cast<int64_t>(UINT32_MAX))
      throw std::runtime_error("the CPU learner indexes rows with 32 bits (at most 4294967295 rows per partition); "
                               "use more partitions or deviceType=gpu");
    sp_ = MakeSplitParams(cfg);
    score_.assign(static_cast<size_t>(n_) * K, 0.0);
    g_.assign(static_cast<size_t>(n_) * K, 0.f);
    h_.assign(static_cast<size_t>(n_) * K, 0.f);
    F_ = d->ref.num_inner();
    mono_.assign(F_, 0);
    for (int f = 0; f < F_; ++f) {
      const int col = d->ref.used_features[f];
      if (col < static_cast<int>(cfg.monotone_constraints.size())) mono_[f] = cfg.monotone_constraints[col];
    }
    if (const char* e = std::getenv("SML_CPU_HIST_FPS")) feats_per_slice_ = std::max(1, std::atoi(e));
    nthreads_ = 1;
#ifdef _OPENMP
    nthreads_ = cfg.num_threads > 0 ? cfg.num_threads : omp_get_max_threads();
#endif
    // column-major copy of the bins for the partition: deciding a split reads ONE byte per row, and from
    // the row-major matrix that byte costs a whole cache line per row (32-B rows)
    const int64_t rs = d->row_stride;
    colbins_.resize(static_cast<size_t>(F_) * n_);
    const uint8_t* rb = d->bins.data();
    uint8_t* cb = colbins_.data();
    const int64_t blk = 4096;
#pragma omp parallel for schedule(static) num_threads(nthreads_)
    for (int64_t b0 = 0; b0 < n_; b0 += blk) {
      const int64_t b1 = std::min<int64_t>(n_, b0 + blk);
      for (int f = 0; f < F_; ++f) {
        uint8_t* dst = cb + static_cast<size_t>(f) * n_;
        for (int64_t r = b0; r < b1; ++r) dst[r] = rb[r * rs + f];
      }
    }
  }
  void SetScores(const std::vector<double>& s) override { score_ = s; }
  void GetScores(std::vector<double>* s) override { *s = score_; }
  void AddBias(int k, double b) override {
    for (int64_t i = 0; i < n_; ++i) score_[k * n_ + i] += b;
  }
  void ScaleScore(int k, double sc) override {
    for (int64_t i = 0; i < n_; ++i) score_[k * n_ + i] *= sc;
  }
  void ComputeGradients(const Objective& obj) override {
    const auto t0 = Clock::now();
    obj.GetGradients(score_.data(), g_.data(), h_.data());
    stats.grad_ms += Ms(t0);
  }
  void SetGradients(const float* g, const float* h) override {
    std::memcpy(g_.data(), g, sizeof(float) * g_.size());
    std::memcpy(h_.data(), h, sizeof(float) * h_.size());
  }
  void GetGradients(std::vector<float>* g, std::vector<float>* h) override { *g = g_; *h = h_; }
  void SetBag(const std::vector<int32_t>* rows) override {
    if (rows) { bag_ = *rows; use_bag_ = true; } else { bag_.clear(); use_bag_ = false; }
  }

  // Histogram of one leaf in 64-bit fixed point (the device engine's K3 representation): the leaf's (g, h)
  // are quantised once into a contiguous ordered buffer of int64 pairs with the tree's GLOBAL scale (the
  // global row count bound and the global max |g| / max h, see TreeScale), then the threads split the work
  // into row groups x feature slices, each adding into its row group's int64 table, and the tables are summed.
  // Integer sums are associative: the histogram is bitwise independent of threads, row order and - summed
  // over ranks as int64 - of how the rows are partitioned, so an N-rank model is the 1-rank model. The
  // returned fp64 histogram is the int64 sums x 2^-e. `tot` (optional) receives the leaf's exact (g, h) sums.
  void BuildHist(int k, const LeafInfo& leaf, const std::vector<char>& fmask, std::vector<double>* hist,
                 bool reduce = true, int64_t* tot = nullptr) {
    const auto t0 = Clock::now();
    const int stride = 256 * 2;
    const size_t hsz = static_cast<size_t>(F_) * stride;
    hist->assign(hsz, 0.0);
    const float* g = g_.data() + static_cast<size_t>(k) * n_;
    const float* h = h_.data() + static_cast<size_t>(k) * n_;
    const int64_t cnt = leaf.count;
    std::vector<int> feats;
    for (int f = 0; f < F_; ++f) if (fmask[f]) feats.push_back(f);
    const int nf = static_cast<int>(feats.size());
    const int* fl = feats.data();
    const int64_t rs = data_->row_stride;
    const uint8_t* bins = data_->bins.data();
    const uint32_t* idx = idx_.data() + leaf.begin;
    const int nt = std::max<int>(1, std::min<int64_t>(nthreads_, cnt / 2048 + 1));
    if (static_cast<int64_t>(ogh_.size()) < 2 * cnt) ogh_.resize(2 * cnt);
    int64_t* og = ogh_.data();
    const double sg = scale_g_, sh = scale_h_;
    int64_t tg = 0, th = 0;
#pragma omp parallel for num_threads(nt) schedule(static) reduction(+ : tg, th)
    for (int64_t p = 0; p < cnt; ++p) {
      const int64_t r = idx[p];
      const int64_t qg = static_cast<int64_t>(RintFast(static_cast<double>(g[r]) * sg));
      const int64_t qh = static_cast<int64_t>(RintFast(static_cast<double>(std::max(h[r], 0.f)) * sh));
      og[2 * p] = qg;
      og[2 * p + 1] = qh;
      tg += qg;
      th += qh;
    }
    // row groups x feature slices; one row group unless there are fewer features than threads
    // up to feats_per_slice_ features per thread: the rows are split into row groups (each random row of a
    // child leaf gathered by one thread per slice), with per-row-group tables summed afterwards.
    // The tables are accumulated at a padded feature pitch (kPitch = 512 + 8 words): at the natural 4 KiB
    // pitch the same bin of every feature shares its low 12 address bits, and a row whose features sit in
    // the same (e.g. the most common) bin makes every load look like it aliases the previous feature's store
    // (4K aliasing): 3.5x slower per update on skewed bins (hb2 microbench, 28 features, 60 % in one bin).
    constexpr int kPitch = stride + 8;
    const size_t psz = static_cast<size_t>(F_) * kPitch;
    const int fps = std::max(1, feats_per_slice_);
    const int fs = std::max(1, std::min(nt, (nf + fps - 1) / fps));
    const int rg = std::max(1, nt / fs);
    if (static_cast<int>(hloc_.size()) < rg) hloc_.resize(rg);
    for (int gi = 0; gi < rg; ++gi) if (hloc_[gi].size() < psz) hloc_[gi].resize(psz);
#pragma omp parallel for num_threads(fs * rg) schedule(static, 1) collapse(2)
    for (int gi = 0; gi < rg; ++gi) {
      for (int si = 0; si < fs; ++si) {
        int64_t* dst = hloc_[gi].data();
        const int fa = nf * si / fs, fb = nf * (si + 1) / fs;
        for (int j = fa; j < fb; ++j) std::fill(dst + fl[j] * kPitch, dst + fl[j] * kPitch + stride, int64_t{0});
        const int64_t pa = cnt * gi / rg, pb = cnt * (gi + 1) / rg;
        // one 16-B (g, h) integer add per feature (SSE2: one load, add and store instead of two of each)
        for (int64_t p = pa; p < pb; ++p) {
          if (p + 24 < pb) __builtin_prefetch(bins + idx[p + 24] * rs);  // random rows of a child leaf
          const uint8_t* row = bins + idx[p] * rs;
          const __m128i gh = _mm_loadu_si128(reinterpret_cast<const __m128i*>(og + 2 * p));
          // four features per step, loads ahead of stores: the four cells are in different features' tables
          // (never the same address), so the loads need not wait for the stores (2.2x per update, hb3)
          int j = fa;
          for (; j + 4 <= fb; j += 4) {
            __m128i* c0 = reinterpret_cast<__m128i*>(dst + fl[j] * kPitch + row[fl[j]] * 2);
            __m128i* c1 = reinterpret_cast<__m128i*>(dst + fl[j + 1] * kPitch + row[fl[j + 1]] * 2);
            __m128i* c2 = reinterpret_cast<__m128i*>(dst + fl[j + 2] * kPitch + row[fl[j + 2]] * 2);
            __m128i* c3 = reinterpret_cast<__m128i*>(dst + fl[j + 3] * kPitch + row[fl[j + 3]] * 2);
            const __m128i a0 = _mm_load_si128(c0), a1 = _mm_load_si128(c1), a2 = _mm_load_si128(c2),
                          a3 = _mm_load_si128(c3);
            _mm_store_si128(c0, _mm_add_epi64(a0, gh));
            _mm_store_si128(c1, _mm_add_epi64(a1, gh));
            _mm_store_si128(c2, _mm_add_epi64(a2, gh));
            _mm_store_si128(c3, _mm_add_epi64(a3, gh));
          }
          for (; j < fb; ++j) {
            __m128i* c = reinterpret_cast<__m128i*>(dst + fl[j] * kPitch + row[fl[j]] * 2);
            _mm_store_si128(c, _mm_add_epi64(_mm_load_si128(c), gh));
          }
        }
      }
    }
    // int64 histogram (+ the leaf's exact sums and row count): summed tables, then over ranks
    std::vector<int64_t>& acc = hsum_;
    acc.assign(hsz + 3, 0);
#pragma omp parallel for num_threads(std::max(1, std::min(nt, nf))) schedule(static)
    for (int j = 0; j < nf; ++j) {
      int64_t* o = acc.data() + fl[j] * stride;
      std::memcpy(o, hloc_[0].data() + fl[j] * kPitch, sizeof(int64_t) * stride);
      for (int gi = 1; gi < rg; ++gi) {
        const int64_t* src = hloc_[gi].data() + fl[j] * kPitch;
        for (int b = 0; b < stride; ++b) o[b] += src[b];
      }
    }
    acc[hsz] = tg;
    acc[hsz + 1] = th;
    acc[hsz + 2] = leaf.count;
    stats.hist_ms += Ms(t0);
    if (reduce && comm_ && comm_->world() > 1) {
      const auto tc = Clock::now();
      comm_->AllReduceHostI64(acc.data(), static_cast<int64_t>(acc.size()));
      last_gcount_ = acc[hsz + 2];
      stats.comm_ms += Ms(tc);
      ++stats.comm_calls;
    } else {
      last_gcount_ = leaf.count;
    }
    double* out = hist->data();
    for (int j = 0; j < nf; ++j) {
      const int64_t* a = acc.data() + fl[j] * stride;
      double* o = out + fl[j] * stride;
      for (int b = 0; b < stride; b += 2) {
        o[b] = static_cast<double>(a[b]) * inv_g_;
        o[b + 1] = static_cast<double>(a[b + 1]) * inv_h_;
      }
    }
    if (tot) { tot[0] = acc[hsz]; tot[1] = acc[hsz + 1]; tot[2] = acc[hsz + 2]; }
  }

  // The tree's fixed-point scale (the device engine's HistScaleV): 2^e with e the largest exponent such that
  // scale_n * max * 2^e <= 2^62, from the global row count and the global max |g| / max h of class k.
  void TreeScale(int k) {
    if (scale_n_ == 0) {
      double c = static_cast<double>(n_);
      if (comm_ && comm_->world() > 1) comm_->AllReduceHost(&c, 1);
      scale_n_ = static_cast<int64_t>(c);
    }
    const float* g = g_.data() + static_cast<size_t>(k) * n_;
    const float* h = h_.data() + static_cast<size_t>(k) * n_;
    float mg = 0.f, mh = 0.f;
#pragma omp parallel for num_threads(nthreads_) reduction(max : mg, mh)
    for (int64_t i = 0; i < n_; ++i) {
      mg = std::max(mg, std::fabs(g[i]));
      mh = std::max(mh, std::fabs(h[i]));
    }
    double m[2] = {mg, mh};
    if (comm_ && comm_->world() > 1) comm_->AllReduceHostMax(m, 2);
    auto ex = [&](double vmax) {
      const double r = 4.611686018427387904e18 / (static_cast<double>(std::max<int64_t>(1, scale_n_)) *
                                                  std::max(static_cast<double>(static_cast<float>(vmax)), 1e-300));
      return std::max(-1000, std::min(1000, std::ilogb(r)));
    };
    const int eg = ex(m[0]), eh = ex(m[1]);
    scale_g_ = std::ldexp(1.0, eg); inv_g_ = std::ldexp(1.0, -eg);
    scale_h_ = std::ldexp(1.0, eh); inv_h_ = std::ldexp(1.0, -eh);
  }

  // Stable partition of idx_[begin, begin + count) by `left(r)`: every thread flags and counts its chunk,
  // an exclusive scan of the per-thread counts gives each chunk its output offsets on both sides, then the
  // chunks scatter into the scratch buffer in parallel, which is copied back. Returns the left count.
  template <typename Pred>
  int64_t ParallelPartition(int64_t begin, int64_t count, Pred left, const uint8_t* pf, int64_t pf_stride) {
    const int nt = std::max<int>(1, std::min<int64_t>(nthreads_, count / 4096 + 1));
    if (static_cast<int64_t>(part_tmp_.size()) < count) part_tmp_.resize(count);
    if (static_cast<int64_t>(part_flag_.size()) < count) part_flag_.resize(count);
    std::vector<int64_t> nleft(nt + 1, 0);
    uint32_t* idx = idx_.data() + begin;
    uint8_t* flag = part_flag_.data();
#pragma omp parallel num_threads(nt)
    {
#ifdef _OPENMP
      const int t = omp_get_thread_num();
#else
      const int t = 0;
#endif
      const int64_t b = count * t / nt, e = count * (t + 1) / nt;
      int64_t c = 0;
      for (int64_t p = b; p < e; ++p) {
        if (p + 24 < e) __builtin_prefetch(pf + idx[p + 24] * pf_stride);
        const uint8_t l = left(idx[p]) ? 1 : 0;
        flag[p] = l;
        c += l;
      }
      nleft[t + 1] = c;
#pragma omp barrier
#pragma omp single
      for (int i = 0; i < nt; ++i) nleft[i + 1] += nleft[i];
      const int64_t total_left = nleft[nt];
      int64_t lo = nleft[t], ro = total_left + (b - nleft[t]);
      uint32_t* tmp = part_tmp_.data();
      for (int64_t p = b; p < e; ++p) {
        if (flag[p]) tmp[lo++] = idx[p]; else tmp[ro++] = idx[p];
      }
#pragma omp barrier
      std::memcpy(idx + b, tmp + b, sizeof(uint32_t) * (e - b));
    }
    return nleft[nt];
  }

  void FindBest(const std::vector<double>& hist, LeafInfo* leaf, const std::vector<char>& fmask) {
    const auto t0 = Clock::now();
    std::vector<SplitResult> per;
    PerFeatureBest(hist, *leaf, fmask, &per);
    stats.split_ms += Ms(t0);
    SplitResult best{};
    best.feature = -1;
    best.gain = -std::numeric_limits<double>::infinity();
    for (int f = 0; f < F_; ++f) {
      if (per[f].feature < 0) continue;
      if (best.feature < 0 || SplitBetter(per[f].gain, per[f].feature, per[f].threshold, best.gain, best.feature, best.threshold))
        best = per[f];
    }
    leaf->best = best;
    leaf->has_best = best.feature >= 0;
  }

  // Voting-parallel split search (PV-Tree; reference parallelism=voting_parallel, topK,
  // LightGBMParams.scala:25-35, C3 in SURVEY §2.5). Histograms stay local; every rank
  // votes for its top_k features per leaf by LOCAL gain, one allreduce sums the votes
  // (and the smaller child's row count), and only the 2*top_k most-voted features'
  // histograms of each leaf are summed across ranks before the global split search.
  void VotingFind(const std::vector<LeafInfo*>& ls, const std::vector<const std::vector<double>*>& lh,
                  const std::vector<char>& fmask, int64_t parent_gcount) {
    const int C = static_cast<int>(ls.size());
    const int topk = std::max(1, cfg_.top_k);
    std::vector<double> msg(static_cast<size_t>(2 * C * F_) + 1, 0.0);
    std::vector<SplitResult> per;
    for (int c = 0; c < C; ++c) {
      LeafInfo loc = *ls[c];
      double G = 0, H = 0;
      int f0 = 0;
      while (f0 < F_ && !fmask[f0]) ++f0;
      if (f0 < F_)
        for (int b = 0; b < 256; ++b) { G += (*lh[c])[f0 * 512 + b * 2]; H += (*lh[c])[f0 * 512 + b * 2 + 1]; }
      loc.sum_g = G; loc.sum_h = H; loc.gcount = loc.count;
      // local search with per-machine data limits (LightGBM scales min_data / min_hessian by 1/#machines)
      const SplitParams keep = sp_;
      sp_.min_data_in_leaf = std::max(1, sp_.min_data_in_leaf / comm_->world());
      sp_.min_sum_hessian /= comm_->world();
      PerFeatureBest(*lh[c], loc, fmask, &per);
      sp_ = keep;
      std::vector<int> order;
      for (int f = 0; f < F_; ++f) if (per[f].feature >= 0) order.push_back(f);
      std::sort(order.begin(), order.end(), [&](int a, int b) {
        return SplitBetter(per[a].gain, a, 0, per[b].gain, b, 0);
      });
      for (int i = 0; i < static_cast<int>(order.size()) && i < topk; ++i) {
        msg[c * F_ + order[i]] = 1.0;
        msg[(C + c) * F_ + order[i]] = per[order[i]].gain;
      }
    }
    if (C == 2) msg.back() = static_cast<double>(ls[0]->count);  // ls[0] = smaller child
    comm_->AllReduceHost(msg.data(), static_cast<int64_t>(msg.size()));
    if (C == 2) {
      ls[0]->gcount = static_cast<int64_t>(msg.back());
      ls[1]->gcount = parent_gcount - ls[0]->gcount;
    }
    std::vector<std::vector<int>> sel(C);
    std::vector<double> compact;
    for (int c = 0; c < C; ++c) {
      std::vector<int> cand;
      for (int f = 0; f < F_; ++f) if (msg[c * F_ + f] > 0) cand.push_back(f);
      std::sort(cand.begin(), cand.end(), [&](int a, int b) {
        const double va = msg[c * F_ + a], vb = msg[c * F_ + b];
        if (va != vb) return va > vb;
        const double ga = msg[(C + c) * F_ + a], gb = msg[(C + c) * F_ + b];
        if (ga != gb) return ga > gb;
        return a < b;
      });
      // fewer voted features than slots: fill with unvoted allowed ones (so top_k >= #features == data-parallel)
      for (int f = 0; f < F_ && static_cast<int>(cand.size()) < 2 * topk; ++f)
        if (fmask[f] && msg[c * F_ + f] <= 0) cand.push_back(f);
      if (static_cast<int>(cand.size()) > 2 * topk) cand.resize(2 * topk);
      sel[c] = cand;
      for (int f : cand) compact.insert(compact.end(), lh[c]->begin() + f * 512, lh[c]->begin() + (f + 1) * 512);
    }
    if (!compact.empty()) comm_->AllReduceHost(compact.data(), static_cast<int64_t>(compact.size()));
    size_t off = 0;
    for (int c = 0; c < C; ++c) {
      std::vector<double> global(static_cast<size_t>(F_) * 512, 0.0);
      std::vector<char> mask(F_, 0);
      for (int f : sel[c]) {
        std::copy(compact.begin() + off, compact.begin() + off + 512, global.begin() + f * 512);
        off += 512;
        mask[f] = fmask[f];
      }
      FindBest(global, ls[c], mask);
    }
  }

  void PerFeatureBest(const std::vector<double>& hist, const LeafInfo& leaf_in, const std::vector<char>& fmask,
                      std::vector<SplitResult>* per_out) {
    std::vector<std::vector<SplitResult>*> outs{per_out};
    PerFeatureBestMulti({&hist}, {&leaf_in}, fmask, outs);
  }

  // per-feature best splits of several leaves in ONE parallel region over (leaf, feature) pairs
  void PerFeatureBestMulti(const std::vector<const std::vector<double>*>& hists,
                           const std::vector<const LeafInfo*>& lv, const std::vector<char>& fmask,
                           const std::vector<std::vector<SplitResult>*>& outs) {
    const int C = static_cast<int>(lv.size());
    std::vector<char> ok(C);
    for (int c = 0; c < C; ++c) {
      std::vector<SplitResult>& per = *outs[c];
      per.assign(F_, SplitResult{});
      for (auto& r : per) { r.feature = -1; r.gain = -std::numeric_limits<double>::infinity(); }
      ok[c] = lv[c]->gcount >= 2 * sp_.min_data_in_leaf && (sp_.max_depth <= 0 || lv[c]->depth < sp_.max_depth);
    }
    const int tasks = C * F_;
    const int nt = std::max(1, std::min(nthreads_, tasks / 4));
#pragma omp parallel for schedule(dynamic, 2) num_threads(nt)
    for (int task = 0; task < tasks; ++task) {
      const int c = task / F_, f = task % F_;
      if (!ok[c] || !fmask[f]) continue;
      const LeafInfo* leaf = lv[c];
      if (sp_.bynode_k > 0 &&
          !NodeFeatureSelected(sp_.bynode_seed, sp_.tree_seq, leaf->slot, f,
                               reinterpret_cast<const int8_t*>(fmask.data()), F_, sp_.bynode_k))
        continue;
      double tg[256], th[256];
      const std::vector<double>& hist = *hists[c];
      SplitResult& out = (*outs[c])[f];
      const BinMapper& m = data_->ref.mappers[data_->ref.used_features[f]];
      for (int b = 0; b < m.num_bin; ++b) { tg[b] = hist[f * 512 + b * 2]; th[b] = hist[f * 512 + b * 2 + 1]; }
      const MonoCtx mc{leaf->lo, leaf->hi, mono_[f]};
      FindBestSplitFeature(tg, th, m.num_bin, m, f, leaf->sum_g, leaf->sum_h, leaf->gcount, sp_, &out,
                           sp_.has_mono ? &mc : nullptr);
      if (sp_.has_mono && mono_[f] != 0 && sp_.monotone_penalty > 0 && out.feature >= 0)
        out.gain *= MonotonePenaltyFactor(leaf->depth, sp_.monotone_penalty);
    }
  }

  // best split of several leaves (FindBest per leaf, one parallel region)
  void FindBestMulti(const std::vector<const std::vector<double>*>& hists, const std::vector<LeafInfo*>& ls,
                     const std::vector<char>& fmask) {
    const auto t0 = Clock::now();
    const int C = static_cast<int>(ls.size());
    std::vector<std::vector<SplitResult>> per(C);
    std::vector<std::vector<SplitResult>*> outs;
    std::vector<const LeafInfo*> lv;
    for (int c = 0; c < C; ++c) { outs.push_back(&per[c]); lv.push_back(ls[c]); }
    PerFeatureBestMulti(hists, lv, fmask, outs);
    for (int c = 0; c < C; ++c) {
      SplitResult best{};
      best.feature = -1;
      best.gain = -std::numeric_limits<double>::infinity();
      for (int f = 0; f < F_; ++f) {
        if (per[c][f].feature < 0) continue;
        if (best.feature < 0 ||
            SplitBetter(per[c][f].gain, per[c][f].feature, per[c][f].threshold, best.gain, best.feature, best.threshold))
          best = per[c][f];
      }
      ls[c]->best = best;
      ls[c]->has_best = best.feature >= 0;
    }
    stats.split_ms += Ms(t0);
  }

  bool GoesLeft(const SplitResult& s, const uint8_t* row) const {
    const uint32_t b = row[s.feature];
    if (s.is_cat) return (s.cat_bits[b / 32] >> (b % 32)) & 1u;
    const BinMapper& m = data_->ref.mappers[data_->ref.used_features[s.feature]];
    if ((m.missing_type == kMissingZero && b == static_cast<uint32_t>(m.default_bin)) ||
        (m.missing_type == kMissingNaN && b == static_cast<uint32_t>(m.num_bin - 1)))
      return s.default_left != 0;
    return b <= s.threshold;
  }

  Tree TrainTree(int k, const std::vector<char>& fmask_in) override {
    std::vector<char> fmask = fmask_in;
    if (static_cast<int>(fmask.size()) != F_) fmask.assign(F_, 1);
    sp_.tree_seq = tree_seq_++;
    sp_.bynode_k = BynodeK(cfg_, fmask);
    const int L = std::max(2, cfg_.num_leaves);
    Tree tree(L);
    // root
    if (use_bag_) { idx_.assign(bag_.begin(), bag_.end()); }
    else { idx_.resize(n_); std::iota(idx_.begin(), idx_.end(), 0u); }
    std::vector<LeafInfo> leaves(L);
    std::vector<std::vector<double>> hists(L);
    const float* g = g_.data() + static_cast<size_t>(k) * n_;
    const float* h = h_.data() + static_cast<size_t>(k) * n_;
    leaves[0].begin = 0; leaves[0].count = static_cast<int64_t>(idx_.size());
    TreeScale(k);
    const bool voting = cfg_.tree_learner == "voting" && comm_ && comm_->world() > 1;
    // root totals: the exact int64 sums of the quantised (g, h) (global: summed with the histogram, or on
    // their own when voting keeps the histograms local)
    int64_t tot[3];
    BuildHist(k, leaves[0], fmask, &hists[0], !voting, tot);
    if (voting) comm_->AllReduceHostI64(tot, 3);
    const double G = static_cast<double>(tot[0]) * inv_g_, H = static_cast<double>(tot[1]) * inv_h_;
    leaves[0].gcount = tot[2];
    leaves[0].sum_g = G; leaves[0].sum_h = H;
    tree.leaf_value[0] = LeafOutput(G, H, sp_.lambda_l1, sp_.lambda_l2, sp_.max_delta_step);
    tree.leaf_count[0] = leaves[0].gcount;
    tree.leaf_weight[0] = H;
    if (voting) VotingFind({&leaves[0]}, {&hists[0]}, fmask, leaves[0].gcount);
    else FindBest(hists[0], &leaves[0], fmask);
    for (int s = 1; s < L; ++s) {
      int bl = -1;
      for (int l = 0; l < tree.num_leaves; ++l) {
        if (!leaves[l].has_best) continue;
        if (bl < 0 || leaves[l].best.gain > leaves[bl].best.gain) bl = l;
      }
      if (bl < 0 || leaves[bl].best.gain <= 0) break;
      const SplitResult sr = leaves[bl].best;
      LeafInfo& P = leaves[bl];
      // stable partition of the leaf's rows
      const auto tp = Clock::now();
      const uint8_t* col = colbins_.data() + static_cast<size_t>(sr.feature) * n_;  // the split feature's column
      const int64_t rs = 1;
      const BinMapper& pm = data_->ref.mappers[data_->ref.used_features[sr.feature]];
      const uint32_t miss_bin = pm.missing_type == kMissingZero ? static_cast<uint32_t>(pm.default_bin)
                                : (pm.missing_type == kMissingNaN ? static_cast<uint32_t>(pm.num_bin - 1) : 256u);
      const bool dleft = sr.default_left != 0;
      const uint32_t thr = sr.threshold;
      int64_t nl;
      if (sr.is_cat) {
        nl = ParallelPartition(P.begin, P.count, [&](int64_t r) {
          const uint32_t b = col[r * rs];
          return ((sr.cat_bits[b / 32] >> (b % 32)) & 1u) != 0;
        }, col, rs);
      } else {
        nl = ParallelPartition(P.begin, P.count, [&](int64_t r) {
          const uint32_t b = col[r * rs];
          return b == miss_bin ? dleft : b <= thr;
        }, col, rs);
      }
      stats.partition_ms += Ms(tp);
      const int fr = data_->ref.used_features[sr.feature];
      const BinMapper& m = data_->ref.mappers[fr];
      int right;
      if (sr.is_cat) {
        std::vector<uint32_t> binbits(8, 0), valbits;
        int maxcat = 0;
        for (int b = 0; b < m.num_bin - 1; ++b)
          if ((sr.cat_bits[b / 32] >> (b % 32)) & 1u) { binbits[b / 32] |= 1u << (b % 32); maxcat = std::max(maxcat, m.bin2cat[b]); }
        valbits.assign(maxcat / 32 + 1, 0);
        for (int b = 0; b < m.num_bin - 1; ++b)
          if ((sr.cat_bits[b / 32] >> (b % 32)) & 1u) valbits[m.bin2cat[b] / 32] |= 1u << (m.bin2cat[b] % 32);
        right = tree.SplitCategorical(bl, sr.feature, fr, binbits, valbits, sr.left_out, sr.right_out,
                                      sr.left_cnt, sr.right_cnt, sr.left_h, sr.right_h, sr.gain);
      } else {
        right = tree.Split(bl, sr.feature, fr, sr.threshold, m.BinToValue(sr.threshold), sr.default_left != 0,
                           m.missing_type, sr.left_out, sr.right_out, sr.left_cnt, sr.right_cnt, sr.left_h, sr.right_h, sr.gain);
      }
      LeafInfo& Lf = leaves[bl];
      LeafInfo& R = leaves[right];
      const int depth = P.depth + 1;
      R.begin = P.begin + nl; R.count = P.count - nl; R.sum_g = sr.right_g; R.sum_h = sr.right_h; R.depth = depth;
      Lf.count = nl; Lf.sum_g = sr.left_g; Lf.sum_h = sr.left_h; Lf.depth = depth;
      // children inherit the parent's output bounds; a monotone split also
      // separates them at the midpoint of the two outputs (basic method)
      R.lo = Lf.lo; R.hi = Lf.hi;
      const int inode = tree.num_leaves - 2;
      Lf.slot = 2 * inode + 1;
      R.slot = 2 * inode + 2;
      const int mdir = sr.is_cat ? 0 : mono_[sr.feature];
      if (mdir != 0) {
        const double mid = (sr.left_out + sr.right_out) / 2.0;
        if (mdir < 0) { Lf.lo = std::max(Lf.lo, mid); R.hi = std::min(R.hi, mid); }
        else { Lf.hi = std::min(Lf.hi, mid); R.lo = std::max(R.lo, mid); }
      }
      // smaller child (by the globally consistent estimate) gets a fresh
      // histogram, the larger = parent - smaller
      const int64_t pg = P.gcount;
      const bool left_small = sr.left_cnt <= sr.right_cnt;
      int small = left_small ? bl : right, large = left_small ? right : bl;
      std::vector<double> parent = std::move(hists[bl]);
      BuildHist(k, leaves[small], fmask, &hists[small], !voting);
      hists[large].resize(parent.size());
      for (size_t i = 0; i < parent.size(); ++i) hists[large][i] = parent[i] - hists[small][i];
      if (voting) {
        VotingFind({&leaves[small], &leaves[large]}, {&hists[small], &hists[large]}, fmask, pg);
      } else {
        leaves[small].gcount = last_gcount_;
        leaves[large].gcount = pg - last_gcount_;
        FindBestMulti({&hists[bl], &hists[right]}, {&leaves[bl], &leaves[right]}, fmask);
      }
    }
    // exact (global) leaf counts; each leaf's row segment is kept for the score update
    seg_.resize(tree.num_leaves);
    for (int l = 0; l < tree.num_leaves; ++l) {
      tree.leaf_count[l] = leaves[l].gcount;
      seg_[l] = {leaves[l].begin, leaves[l].count};
    }
    return tree;
  }

  // Without bagging every row sits in exactly one leaf's segment of idx_ after the growth, so the new
  // tree's shrunk output is added per segment instead of walking the tree for every row (LightGBM's
  // score updater does the same with its data partition).
  Tree TrainTreeAndUpdateScore(int k, const std::vector<char>& feature_mask, double shrink, bool* updated) override {
    Tree t = TrainTree(k, feature_mask);
    *updated = false;
    if (use_bag_ || t.num_leaves <= 1) return t;
    const auto t0 = Clock::now();
    double* s = score_.data() + static_cast<size_t>(k) * n_;
    const uint32_t* idx = idx_.data();
    for (int l = 0; l < t.num_leaves; ++l) {
      const double v = t.leaf_value[l] * shrink;
      const int64_t b = seg_[l].first, e = b + seg_[l].second;
#pragma omp parallel for schedule(static) num_threads(std::max<int>(1, std::min<int64_t>(nthreads_, (e - b) / 16384 + 1)))
      for (int64_t p = b; p < e; ++p) s[idx[p]] += v;
    }
    stats.score_ms += Ms(t0);
    *updated = true;
    return t;
  }

  void UpdateScore(const Tree& t, int k, double scale) override {
    const ScoreTimer timer(&stats.score_ms);
    double* s = score_.data() + static_cast<size_t>(k) * n_;
    if (t.num_leaves <= 1) {
      for (int64_t i = 0; i < n_; ++i) s[i] += scale * t.leaf_value[0];
      return;
    }
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n_; ++i) {
      int l = t.GetLeafByBins(&data_->bins[i * data_->row_stride], data_->ref.mappers, data_->ref.used_features);
      s[i] += scale * t.leaf_value[l];
    }
  }

  void PredictLeafIndex(const Tree& t, std::vector<int32_t>* leaf) override {
    leaf->resize(n_);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n_; ++i)
      (*leaf)[i] = t.GetLeafByBins(&data_->bins[i * data_->row_stride], data_->ref.mappers, data_->ref.used_features);
  }

 private:
  const Dataset* data_ = nullptr;
  Config cfg_;
  SplitParams sp_{};
  int K_ = 1, F_ = 0, nthreads_ = 1;
  int64_t n_ = 0;
  std::vector<double> score_;
  std::vector<float> g_, h_;
  std::vector<uint32_t> idx_;  // row indices, grouped by leaf (32-bit: half the bytes the partition moves)
  std::vector<std::pair<int64_t, int64_t>> seg_;  // (begin, count) in idx_ of each leaf of the last tree
  std::vector<std::vector<int64_t>> hloc_;        // per-thread int64 histogram tables (BuildHist)
  std::vector<int64_t> hsum_;                     // summed int64 histogram + leaf sums + count (BuildHist)
  int64_t scale_n_ = 0;                           // global row count (the histogram scale's count bound)
  double scale_g_ = 1, scale_h_ = 1, inv_g_ = 1, inv_h_ = 1;  // this tree's fixed-point scales
  int feats_per_slice_ = 32;  // SML_CPU_HIST_FPS (A/B at 1M x 28, 8 threads: 28 -> 2.47 s, 14 -> 2.70, 7 -> 2.99, 1 -> 3.35)
  std::vector<int64_t> ogh_;                      // the leaf's quantised (g, h) in row order (BuildHist)
  std::vector<uint32_t> part_tmp_;                // partition scratch
  std::vector<uint8_t> colbins_;                  // bins, column-major (partition decisions)
  std::vector<uint8_t> part_flag_;
  std::vector<int32_t> bag_;
  bool use_bag_ = false;
  int64_t last_gcount_ = 0;
  std::vector<int> mono_;  // monotone direction per inner feature
  int tree_seq_ = 0;
};

}  // namespace

std::unique_ptr<TrainBackend> MakeCpuBackend() { return std::unique_ptr<TrainBackend>(new CpuBackend()); }

}  // namespace sml
