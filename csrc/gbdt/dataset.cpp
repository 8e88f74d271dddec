#include "dataset.h"

#include <algorithm>
#include <cstring>
#include <mutex>
#include <numeric>
#include <random>
#include <sstream>
#include <stdexcept>

#ifdef _OPENMP
#include <omp.h>
#else
static inline int omp_get_max_threads() { return 1; }
static inline int omp_get_thread_num() { return 0; }
static inline int omp_get_num_threads() { return 1; }
#endif

namespace sml {
namespace {

constexpr double kInf = std::numeric_limits<double>::infinity();

// Greedy equal-frequency binning over sorted distinct values.
// Returns upper bounds (last one +inf). A value with at least `mean` samples
// keeps a bin of its own; bin edges sit halfway between neighbouring values.
std::vector<double> GreedyBins(const std::vector<double>& vals, const std::vector<int64_t>& cnts,
                               int max_bin, int64_t total, int min_data_in_bin) {
  std::vector<double> ub;
  const int n = static_cast<int>(vals.size());
  if (n == 0 || max_bin <= 0) { ub.push_back(kInf); return ub; }
  if (n <= max_bin) {
    int64_t cur = 0;
    for (int i = 0; i < n - 1; ++i) {
      cur += cnts[i];
      if (cur >= min_data_in_bin) {
        ub.push_back((vals[i] + vals[i + 1]) / 2.0);
        cur = 0;
      }
    }
    ub.push_back(kInf);
    return ub;
  }
  if (min_data_in_bin > 0) {
    max_bin = static_cast<int>(std::min<int64_t>(max_bin, std::max<int64_t>(1, total / min_data_in_bin)));
  }
  double mean = static_cast<double>(total) / max_bin;
  // values that are "big" get a private bin; recompute the mean for the rest
  std::vector<char> big(n, 0);
  int64_t rest_cnt = total;
  int rest_bins = max_bin;
  for (int i = 0; i < n; ++i) {
    if (cnts[i] >= mean) { big[i] = 1; rest_cnt -= cnts[i]; --rest_bins; }
  }
  mean = rest_bins > 0 ? static_cast<double>(rest_cnt) / rest_bins : static_cast<double>(rest_cnt);
  std::vector<int> upper_idx;  // last value index of each bin
  int64_t cur = 0;
  int bins_used = 0;
  for (int i = 0; i < n - 1; ++i) {
    cur += cnts[i];
    bool cut = big[i] || big[i + 1] || cur >= mean;
    if (cut && cur >= min_data_in_bin) {
      upper_idx.push_back(i);
      ++bins_used;
      cur = 0;
      if (bins_used >= max_bin - 1) break;
    }
  }
  for (int i : upper_idx) ub.push_back((vals[i] + vals[i + 1]) / 2.0);
  ub.push_back(kInf);
  return ub;
}

// Ascending sort of NaN-free doubles: LSD radix over the order-preserving uint64 image of the bits,
// 11-bit digits, skipping digits every key shares (float32-origin samples have 29 zero low mantissa
// bits, so 3 of the 6 passes vanish). ~10x std::sort on the 200k-row bin sample; same order except
// that -0.0 sorts before +0.0 (both are counted as the zero bin by the caller).
// LSD radix sort of doubles (order-preserving key map), 8-bit digits: 256 buckets stay in L1, and a
// digit every key shares is skipped - float32-origin samples have 29 zero mantissa bits, so 3 of the 8
// passes drop out.
void SortDoubles(std::vector<double>* v) {
  const size_t n = v->size();
  if (n < 2048) { std::sort(v->begin(), v->end()); return; }
  std::vector<uint64_t> a(n), b(n);
  uint64_t all_or = 0, all_and = ~uint64_t(0);
  for (size_t i = 0; i < n; ++i) {
    uint64_t u;
    std::memcpy(&u, &(*v)[i], 8);
    a[i] = (u >> 63) ? ~u : (u | (uint64_t(1) << 63));
    all_or |= a[i];
    all_and &= a[i];
  }
  const uint64_t varying = all_or ^ all_and;  // bits that differ between some keys
  uint32_t cnt[256];
  for (int shift = 0; shift < 64; shift += 8) {
    if (((varying >> shift) & 0xFFu) == 0) continue;  // every key has this digit
    std::memset(cnt, 0, sizeof(cnt));
    for (size_t i = 0; i < n; ++i) ++cnt[(a[i] >> shift) & 0xFFu];
    uint32_t run = 0;
    for (int d = 0; d < 256; ++d) { const uint32_t c = cnt[d]; cnt[d] = run; run += c; }
    for (size_t i = 0; i < n; ++i) b[cnt[(a[i] >> shift) & 0xFFu]++] = a[i];
    a.swap(b);
  }
  for (size_t i = 0; i < n; ++i) {
    const uint64_t k = a[i];
    const uint64_t u = (k >> 63) ? (k & ~(uint64_t(1) << 63)) : ~k;
    std::memcpy(&(*v)[i], &u, 8);
  }
}

}  // namespace

void BinMapper::FindBin(std::vector<double> values, size_t total_sample_cnt, int max_bin,
                        int min_data_in_bin, bool categorical, bool use_missing,
                        bool zero_as_missing) {
  is_categorical = categorical;
  upper_bounds.clear();
  bin2cat.clear();
  cat2bin.clear();
  // split off NaNs
  size_t na_cnt = 0;
  {
    size_t w = 0;
    for (double v : values) {
      if (std::isnan(v)) ++na_cnt; else values[w++] = v;
    }
    values.resize(w);
  }
  int64_t zero_cnt = static_cast<int64_t>(total_sample_cnt) - static_cast<int64_t>(values.size()) -
                     static_cast<int64_t>(na_cnt);
  if (zero_cnt < 0) zero_cnt = 0;
  SortDoubles(&values);
  // distinct values + counts, zeros merged into one 0.0 entry
  std::vector<double> dv;
  std::vector<int64_t> dc;
  for (double v : values) {
    if (std::fabs(v) <= kZeroThreshold) { ++zero_cnt; continue; }
    if (!dv.empty() && v == dv.back()) ++dc.back(); else { dv.push_back(v); dc.push_back(1); }
  }
  if (zero_cnt > 0) {
    auto pos = std::lower_bound(dv.begin(), dv.end(), 0.0) - dv.begin();
    dv.insert(dv.begin() + pos, 0.0);
    dc.insert(dc.begin() + pos, zero_cnt);
  }
  min_val = dv.empty() ? 0.0 : dv.front();
  max_val = dv.empty() ? 0.0 : dv.back();

  if (categorical) {
    // categories sorted by frequency, keep up to max_bin-1 of them covering
    // 99% of the data; everything else (and NaN / negatives) -> "other" bin.
    std::vector<std::pair<int64_t, int>> cc;
    for (size_t i = 0; i < dv.size(); ++i) {
      if (dv[i] < 0) continue;
      cc.emplace_back(dc[i], static_cast<int>(dv[i]));
    }
    std::stable_sort(cc.begin(), cc.end(), [](auto& a, auto& b) { return a.first > b.first; });
    int64_t tot = 0;
    for (auto& p : cc) tot += p.first;
    int64_t acc = 0;
    for (auto& p : cc) {
      if (static_cast<int>(bin2cat.size()) >= max_bin - 1) break;
      if (acc >= 0.99 * tot && bin2cat.size() > 0) break;
      cat2bin[p.second] = static_cast<int>(bin2cat.size());
      bin2cat.push_back(p.second);
      acc += p.first;
    }
    num_bin = static_cast<int>(bin2cat.size()) + 1;  // + "other"
    missing_type = kMissingNaN;
    default_bin = cat2bin.count(0) ? cat2bin[0] : num_bin - 1;
    is_trivial = bin2cat.size() <= 1 && (cc.size() <= 1);
    return;
  }

  if (!use_missing) missing_type = kMissingNone;
  else if (zero_as_missing) missing_type = kMissingZero;
  else missing_type = na_cnt > 0 ? kMissingNaN : kMissingNone;

  int eff_max_bin = missing_type == kMissingNaN ? max_bin - 1 : max_bin;
  // zero gets a bin of its own: bin negatives and positives separately
  std::vector<double> nv, pv;
  std::vector<int64_t> nc, pc;
  int64_t zc = 0;
  for (size_t i = 0; i < dv.size(); ++i) {
    if (dv[i] < -kZeroThreshold) { nv.push_back(dv[i]); nc.push_back(dc[i]); }
    else if (dv[i] > kZeroThreshold) { pv.push_back(dv[i]); pc.push_back(dc[i]); }
    else zc += dc[i];
  }
  int64_t ncnt = std::accumulate(nc.begin(), nc.end(), int64_t(0));
  int64_t pcnt = std::accumulate(pc.begin(), pc.end(), int64_t(0));
  int64_t nz = ncnt + pcnt;
  int left_max = 0;
  if (!nv.empty()) {
    left_max = static_cast<int>(static_cast<double>(ncnt) / std::max<int64_t>(1, nz) * (eff_max_bin - 1));
    left_max = std::max(1, left_max);
  }
  std::vector<double> ub;
  if (!nv.empty()) {
    auto lb = GreedyBins(nv, nc, left_max, ncnt, min_data_in_bin);
    lb.back() = -kZeroThreshold;
    ub.insert(ub.end(), lb.begin(), lb.end());
  }
  int right_max = eff_max_bin - 1 - static_cast<int>(ub.size());
  if (!pv.empty() && right_max > 0) {
    ub.push_back(kZeroThreshold);
    auto rb = GreedyBins(pv, pc, right_max, pcnt, min_data_in_bin);
    ub.insert(ub.end(), rb.begin(), rb.end());
  } else {
    ub.push_back(kInf);
  }
  (void)zc;
  upper_bounds = ub;
  num_bin = static_cast<int>(upper_bounds.size()) + (missing_type == kMissingNaN ? 1 : 0);
  default_bin = static_cast<int>(ValueToBin(0.0));
  is_trivial = num_bin <= 1 || (dv.size() <= 1 && missing_type != kMissingNaN);
  if (num_bin > 256) throw std::runtime_error("more than 256 bins per feature is not supported");
}

std::string BinMapper::FeatureInfo() const {
  if (is_trivial) return "none";
  std::ostringstream o;
  o.precision(17);
  if (is_categorical) {
    for (size_t i = 0; i < bin2cat.size(); ++i) o << (i ? ":" : "") << bin2cat[i];
    return o.str();
  }
  o << "[" << min_val << ":" << max_val << "]";
  return o.str();
}

namespace {
template <class T> void Put(std::string* s, const T& v) { s->append(reinterpret_cast<const char*>(&v), sizeof(T)); }
template <class T> const char* Get(const char* p, T* v) { std::memcpy(v, p, sizeof(T)); return p + sizeof(T); }
}  // namespace

void BinMapper::Serialize(std::string* out) const {
  Put(out, num_bin); Put(out, missing_type); Put(out, static_cast<int>(is_categorical));
  Put(out, static_cast<int>(is_trivial)); Put(out, default_bin); Put(out, min_val); Put(out, max_val);
  Put(out, static_cast<int>(upper_bounds.size()));
  for (double d : upper_bounds) Put(out, d);
  Put(out, static_cast<int>(bin2cat.size()));
  for (int c : bin2cat) Put(out, c);
}

const char* BinMapper::Deserialize(const char* p) {
  int cat, triv, n;
  p = Get(p, &num_bin); p = Get(p, &missing_type); p = Get(p, &cat); p = Get(p, &triv);
  p = Get(p, &default_bin); p = Get(p, &min_val); p = Get(p, &max_val);
  is_categorical = cat != 0; is_trivial = triv != 0;
  p = Get(p, &n); upper_bounds.resize(n);
  for (int i = 0; i < n; ++i) p = Get(p, &upper_bounds[i]);
  p = Get(p, &n); bin2cat.resize(n); cat2bin.clear();
  for (int i = 0; i < n; ++i) { p = Get(p, &bin2cat[i]); cat2bin[bin2cat[i]] = i; }
  return p;
}

std::string DatasetReference::Serialize() const {
  std::string s = "SMLREF01";
  Put(&s, num_total_features);
  for (const auto& m : mappers) m.Serialize(&s);
  Put(&s, static_cast<int>(feature_names.size()));
  for (const auto& n : feature_names) { Put(&s, static_cast<int>(n.size())); s.append(n); }
  return s;
}

DatasetReference DatasetReference::Deserialize(const std::string& bytes) {
  if (bytes.size() < 12 || bytes.compare(0, 8, "SMLREF01") != 0)
    throw std::runtime_error("invalid serialized reference dataset");
  DatasetReference r;
  const char* p = bytes.data() + 8;
  p = Get(p, &r.num_total_features);
  r.mappers.resize(r.num_total_features);
  for (auto& m : r.mappers) p = m.Deserialize(p);
  int nn; p = Get(p, &nn);
  for (int i = 0; i < nn; ++i) {
    int l; p = Get(p, &l); r.feature_names.emplace_back(p, p + l); p += l;
  }
  r.real_to_inner.assign(r.num_total_features, -1);
  for (int f = 0; f < r.num_total_features; ++f) {
    if (!r.mappers[f].is_trivial) { r.real_to_inner[f] = static_cast<int>(r.used_features.size()); r.used_features.push_back(f); }
  }
  return r;
}

DatasetReference DatasetReference::FromSampledColumns(const std::vector<std::vector<double>>& cols,
                                                      int64_t total_sample_cnt, const Config& cfg,
                                                      const std::vector<std::string>& names) {
  DatasetReference r;
  r.num_total_features = static_cast<int>(cols.size());
  r.mappers.resize(cols.size());
  std::vector<char> is_cat(cols.size(), 0);
  for (int c : cfg.categorical_feature) if (c >= 0 && c < static_cast<int>(cols.size())) is_cat[c] = 1;
#pragma omp parallel for schedule(dynamic)
  for (int f = 0; f < static_cast<int>(cols.size()); ++f) {
    int mb = cfg.max_bin;
    if (f < static_cast<int>(cfg.max_bin_by_feature.size())) mb = std::min(255, cfg.max_bin_by_feature[f]);
    r.mappers[f].FindBin(cols[f], static_cast<size_t>(total_sample_cnt), mb, cfg.min_data_in_bin,
                         is_cat[f] != 0, cfg.use_missing, cfg.zero_as_missing);
  }
  r.real_to_inner.assign(cols.size(), -1);
  for (int f = 0; f < r.num_total_features; ++f) {
    if (!r.mappers[f].is_trivial) { r.real_to_inner[f] = static_cast<int>(r.used_features.size()); r.used_features.push_back(f); }
  }
  r.feature_names = names;
  if (r.feature_names.size() != cols.size()) {
    r.feature_names.clear();
    for (size_t i = 0; i < cols.size(); ++i) r.feature_names.push_back("Column_" + std::to_string(i));
  }
  return r;
}

namespace {
// sampled rows (row-major) -> per-feature columns of the values that are not (near) zero, one pass over
// the rows per thread block of features: the sample is read in row order (no 28-way strided re-reads)
template <class T>
std::vector<std::vector<double>> SampleColumns(const T* sample, int64_t n_sample, int num_cols) {
  std::vector<std::vector<double>> cols(num_cols);
  const int nt = std::max(1, std::min(omp_get_max_threads(), num_cols));
#pragma omp parallel num_threads(nt)
  {
    const int t = omp_get_thread_num(), T_ = omp_get_num_threads();
    const int f0 = static_cast<int>(static_cast<int64_t>(num_cols) * t / T_);
    const int f1 = static_cast<int>(static_cast<int64_t>(num_cols) * (t + 1) / T_);
    for (int f = f0; f < f1; ++f) cols[f].reserve(static_cast<size_t>(n_sample));
    for (int64_t i = 0; i < n_sample; ++i) {
      const T* row = sample + i * num_cols;
      for (int f = f0; f < f1; ++f) {
        const double v = static_cast<double>(row[f]);
        if (std::isnan(v) || std::fabs(v) > kZeroThreshold) cols[f].push_back(v);
      }
    }
  }
  return cols;
}
}  // namespace

DatasetReference DatasetReference::FromSample(const double* sample, int64_t n_sample, int num_cols,
                                              int64_t total_rows, const Config& cfg,
                                              const std::vector<std::string>& names) {
  (void)total_rows;
  return FromSampledColumns(SampleColumns(sample, n_sample, num_cols), n_sample, cfg, names);
}

DatasetReference DatasetReference::FromSampleF32(const float* sample, int64_t n_sample, int num_cols,
                                                 int64_t total_rows, const Config& cfg,
                                                 const std::vector<std::string>& names) {
  (void)total_rows;
  return FromSampledColumns(SampleColumns(sample, n_sample, num_cols), n_sample, cfg, names);
}

std::vector<int64_t> SampleRowIndices(int64_t n, int64_t k, uint64_t seed) {
  // Floyd's algorithm over a bitmap: k distinct rows of [0, n) uniformly at random in O(k) draws, then the
  // bitmap scan returns them sorted (sequential reads of the sampled rows). splitmix64 stream of `seed`.
  std::vector<int64_t> out;
  if (n <= 0 || k <= 0) return out;
  if (k >= n) {
    out.resize(n);
    for (int64_t i = 0; i < n; ++i) out[i] = i;
    return out;
  }
  std::vector<uint64_t> bits(static_cast<size_t>((n + 63) / 64), 0);
  uint64_t x = seed * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
  auto next = [&x]() {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  };
  for (int64_t j = n - k; j < n; ++j) {
    // uniform in [0, j] (128-bit multiply: no modulo bias worth measuring at these sizes)
    const int64_t t = static_cast<int64_t>((static_cast<unsigned __int128>(next()) * static_cast<uint64_t>(j + 1)) >> 64);
    const int64_t pick = (bits[t >> 6] >> (t & 63)) & 1ull ? j : t;
    bits[pick >> 6] |= 1ull << (pick & 63);
  }
  out.reserve(static_cast<size_t>(k));
  for (size_t w = 0; w < bits.size(); ++w) {
    uint64_t m = bits[w];
    while (m) {
      out.push_back(static_cast<int64_t>(w * 64 + __builtin_ctzll(m)));
      m &= m - 1;
    }
  }
  return out;
}

void Dataset::Init(const DatasetReference& r, int64_t n) {
  ref = r;
  num_data = n;
  row_stride = r.row_stride();
  // no bin storage yet: host pushes allocate the host matrix, device pushes the HBM one
  bins.clear();
  host_valid = false;
  dev.reset();
  dev_valid = false;
  label.resize(static_cast<size_t>(n));  // default-initialised: SetLabel or FinalizeLabel writes it
  label_set = false;
}

bool GroupRuns(const int64_t* a, int64_t n, std::vector<int64_t>* starts) {
  starts->clear();
  if (n <= 0) return true;
  // one pass over the column in parallel chunks (12.5M ids: ~8 ms as two numpy passes), then the run ids
  const int nt = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(omp_get_max_threads(), n >> 16)));
  std::vector<std::vector<int64_t>> part(nt);
#pragma omp parallel for schedule(static) num_threads(nt)
  for (int t = 0; t < nt; ++t) {
    const int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
    auto& v = part[t];
    for (int64_t i = std::max<int64_t>(lo, 1); i < hi; ++i)
      if (a[i] != a[i - 1]) v.push_back(i);
  }
  size_t total = 1;
  for (auto& v : part) total += v.size();
  starts->reserve(total);
  starts->push_back(0);
  for (auto& v : part) starts->insert(starts->end(), v.begin(), v.end());
  // grouped iff the run ids are distinct: monotone run ids (the usual layout) are, otherwise sort and look
  const size_t r = starts->size();
  bool inc = true, dec = true;
  for (size_t k = 1; k < r && (inc || dec); ++k) {
    const int64_t x = a[(*starts)[k - 1]], y = a[(*starts)[k]];
    inc &= x < y;
    dec &= x > y;
  }
  if (inc || dec) return true;
  std::vector<int64_t> ids(r);
  for (size_t k = 0; k < r; ++k) ids[k] = a[(*starts)[k]];
  std::sort(ids.begin(), ids.end());
  return std::adjacent_find(ids.begin(), ids.end()) == ids.end();
}

void Dataset::SetLabel(const float* y, int64_t n) {
  if (n != num_data) throw std::runtime_error("label size mismatch");
  label.resize(static_cast<size_t>(n));
  float* dst = label.data();
  if (n >= (int64_t(1) << 20)) {  // 11M labels: ~4 ms on one thread
    const int nt = std::min<int>(8, omp_get_max_threads());
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int t = 0; t < nt; ++t) {
      const int64_t a = n * t / nt, b = n * (t + 1) / nt;
      std::memcpy(dst + a, y + a, sizeof(float) * (b - a));
    }
  } else {
    std::copy(y, y + n, dst);
  }
  label_set = true;
}

void Dataset::FinalizeLabel() {
  if (label_set) return;
  std::fill(label.begin(), label.end(), 0.f);
  label_set = true;
}

std::vector<uint8_t> Dataset::DefaultRow() const {
  std::vector<uint8_t> zrow(row_stride, 0);
  for (int i = 0; i < ref.num_inner(); ++i) zrow[i] = static_cast<uint8_t>(ref.mappers[ref.used_features[i]].default_bin);
  return zrow;
}

namespace {
std::mutex& BinsMutex() {
  static std::mutex m;
  return m;
}
}  // namespace


namespace {
// Bin-encode dense rows: blocks of 8 rows, one column at a time, the 8 searches of a column interleaved
template <class T>
void PushDenseRows(const DatasetReference& ref, const T* rows, int64_t nrows, int num_cols, uint8_t* out,
                   int64_t row_stride) {
  const int ni = ref.num_inner();
  constexpr int R = 8;
  const int64_t nblk = (nrows + R - 1) / R;
#pragma omp parallel for schedule(static)
  for (int64_t blk = 0; blk < nblk; ++blk) {
    const int64_t i0 = blk * R;
    const int rows_here = static_cast<int>(std::min<int64_t>(R, nrows - i0));
    uint8_t* dst = out + i0 * row_stride;
    const T* src = rows + i0 * num_cols;
    for (int k = 0; k < ni; ++k) {
      const int f = ref.used_features[k];
      const BinMapper& m = ref.mappers[f];
      if (f >= num_cols) {
        for (int r = 0; r < rows_here; ++r) dst[r * row_stride + k] = static_cast<uint8_t>(m.default_bin);
      } else if (rows_here == R) {
        m.ValueToBinN<R>(src + f, num_cols, dst + k, row_stride);
      } else {
        for (int r = 0; r < rows_here; ++r)
          dst[r * row_stride + k] = static_cast<uint8_t>(m.ValueToBin(static_cast<double>(src[r * num_cols + f])));
      }
    }
  }
}
}  // namespace

void Dataset::EnsureHostBins() const {
  std::lock_guard<std::mutex> lk(BinsMutex());
  if (host_valid) return;
  bins.resize(static_cast<size_t>(num_data) * row_stride);
  if (dev && dev_valid) {
    DatasetDownloadBins(*this, bins.data());
  } else {
    // rows that are never pushed hold every feature's zero bin
    const std::vector<uint8_t> zrow = DefaultRow();
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < num_data; ++i) std::memcpy(&bins[i * row_stride], zrow.data(), row_stride);
  }
  host_valid = true;
}

// Host pushes run concurrently at disjoint offsets (one thread per partition, StreamingPartitionTask.scala:
// 220-231): the shared state they touch - materialising the host matrix, invalidating the device copy -
// changes under the bins mutex; the row writes themselves are disjoint.
void Dataset::BeginHostPush() {
  EnsureHostBins();
  std::lock_guard<std::mutex> lk(BinsMutex());
  dev_valid = false;  // the device copy (if any) no longer has every row
}

void Dataset::PushDense(const double* rows, int64_t nrows, int num_cols, int64_t start) {
  BeginHostPush();
  PushDenseRows(ref, rows, nrows, num_cols, &bins[start * row_stride], row_stride);
}

void Dataset::PushDenseF32(const float* rows, int64_t nrows, int num_cols, int64_t start) {
  BeginHostPush();
  PushDenseRows(ref, rows, nrows, num_cols, &bins[start * row_stride], row_stride);
}

void Dataset::PushCSR(const int64_t* indptr, const int32_t* indices, const double* values,
                      int64_t nrows, int64_t start) {
  BeginHostPush();
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < nrows; ++i) {
    uint8_t* dst = &bins[(start + i) * row_stride];
    for (int64_t p = indptr[i]; p < indptr[i + 1]; ++p) {
      int f = indices[p];
      if (f < 0 || f >= ref.num_total_features) continue;
      int k = ref.real_to_inner[f];
      if (k < 0) continue;
      dst[k] = static_cast<uint8_t>(ref.mappers[f].ValueToBin(values[p]));
    }
  }
}

void Dataset::SetQueryFromGroupSizes(const std::vector<int32_t>& sizes) {
  query_boundaries.assign(1, 0);
  for (int32_t s : sizes) query_boundaries.push_back(query_boundaries.back() + s);
}

}  // namespace sml
