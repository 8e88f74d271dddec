// Binned training dataset (native component N1 of SURVEY.md §2.3).
//
// Reference behaviour being reproduced: the reference builds LightGBM bin
// mappers from a driver-side row sample (lightgbm/.../dataset/
// ReferenceDatasetUtils.scala:14-71, LGBM_DatasetCreateFromSampledColumn),
// serialises them to bytes (":52") and lets every executor push rows into a
// Dataset initialised from that reference (":73-97", StreamingPartitionTask
// .scala:202-277). Here the bin matrix is a row-major uint8 array padded to a
// multiple of 4 features, so a HIP kernel can fetch 4 feature bins per dword
// and a gathered row (leaf index lists) is one contiguous 4*k byte segment.
#pragma once
#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <limits>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "config.h"
#include "host_pool.h"

namespace sml {

constexpr double kZeroThreshold = 1e-35;
enum MissingType : int { kMissingNone = 0, kMissingZero = 1, kMissingNaN = 2 };

struct BinMapper {
  int num_bin = 1;
  int missing_type = kMissingNone;
  bool is_categorical = false;
  bool is_trivial = true;
  int default_bin = 0;   // bin that holds 0.0
  double min_val = 0.0, max_val = 0.0;
  std::vector<double> upper_bounds;  // numerical: one per non-NaN bin, last = +inf
  std::vector<int> bin2cat;          // categorical: bin -> category value
  std::unordered_map<int, int> cat2bin;

  // values: sampled feature values (zeros may be omitted: total_sample_cnt
  // counts them implicitly, exactly like LightGBM's sampled-column API).
  void FindBin(std::vector<double> values, size_t total_sample_cnt, int max_bin,
               int min_data_in_bin, bool categorical, bool use_missing, bool zero_as_missing);
  inline uint32_t ValueToBin(double v) const {
    if (is_categorical) {
      if (std::isnan(v) || v < 0) return static_cast<uint32_t>(num_bin - 1);
      auto it = cat2bin.find(static_cast<int>(v));
      return it == cat2bin.end() ? static_cast<uint32_t>(num_bin - 1) : static_cast<uint32_t>(it->second);
    }
    if (std::isnan(v)) {
      if (missing_type == kMissingNaN) return static_cast<uint32_t>(num_bin - 1);
      v = 0.0;
    }
    // smallest i with v <= upper_bounds[i] (the last bound is +inf): a branchless lower bound - the halving
    // step is a conditional move, so a row of random values costs no branch mispredictions (the branchy
    // search mispredicted about half of its ~8 steps per value)
    // (index arithmetic, not a pointer select: g++ turns the select back into a branch; 16.5 vs 66 ns per
    // value over 255 normal-distributed bounds)
    const double* b = upper_bounds.data();
    size_t base = 0, n = upper_bounds.size();
    while (n > 1) {
      const size_t half = n >> 1;
      base += static_cast<size_t>(b[base + half - 1] < v) * half;
      n -= half;
    }
    return static_cast<uint32_t>(base + static_cast<size_t>(b[base] < v));
  }
  // ValueToBin of R values of this column at once (v[r * vs] -> o[r * os]): the R searches are interleaved
  // step by step, so their dependent load chains overlap (8 rows: 8.6 vs 17 ns per value, vb3 microbench)
  template <int R, class T>
  inline void ValueToBinN(const T* v, int64_t vs, uint8_t* o, int64_t os) const {
    if (is_categorical) {
      for (int r = 0; r < R; ++r) o[r * os] = static_cast<uint8_t>(ValueToBin(static_cast<double>(v[r * vs])));
      return;
    }
    double x[R];
    size_t base[R];
    for (int r = 0; r < R; ++r) {
      const double d = static_cast<double>(v[r * vs]);
      x[r] = std::isnan(d) ? 0.0 : d;
      base[r] = 0;
    }
    const double* b = upper_bounds.data();
    size_t n = upper_bounds.size();
    while (n > 1) {
      const size_t half = n >> 1;
      for (int r = 0; r < R; ++r) base[r] += static_cast<size_t>(b[base[r] + half - 1] < x[r]) * half;
      n -= half;
    }
    for (int r = 0; r < R; ++r) {
      const uint32_t bin = static_cast<uint32_t>(base[r] + static_cast<size_t>(b[base[r]] < x[r]));
      o[r * os] = static_cast<uint8_t>(missing_type == kMissingNaN && std::isnan(static_cast<double>(v[r * vs]))
                                           ? static_cast<uint32_t>(num_bin - 1) : bin);
    }
  }
  double BinToValue(uint32_t bin) const {  // split threshold for "bin <= t"
    return upper_bounds[bin];
  }
  std::string FeatureInfo() const;
  void Serialize(std::string* out) const;
  const char* Deserialize(const char* p);
};

// Bin boundaries for all columns: what the reference calls the "reference
// dataset" (serialisable, broadcast to executors).
struct DatasetReference {
  int num_total_features = 0;
  std::vector<BinMapper> mappers;          // one per column
  std::vector<int> used_features;          // inner index -> column index
  std::vector<int> real_to_inner;          // column -> inner (or -1)
  std::vector<std::string> feature_names;
  std::string Serialize() const;
  static DatasetReference Deserialize(const std::string& bytes);
  // Build from a row-major sample (n_sample x num_cols) of doubles.
  static DatasetReference FromSample(const double* sample, int64_t n_sample, int num_cols,
                                     int64_t total_rows, const Config& cfg,
                                     const std::vector<std::string>& names);
  static DatasetReference FromSampleF32(const float* sample, int64_t n_sample, int num_cols, int64_t total_rows,
                                        const Config& cfg, const std::vector<std::string>& names);
  // Build from a column-wise sample with explicit non-zero values per column
  // (LGBM_DatasetCreateFromSampledColumn semantics).
  static DatasetReference FromSampledColumns(const std::vector<std::vector<double>>& cols,
                                             int64_t total_sample_cnt, const Config& cfg,
                                             const std::vector<std::string>& names);
  int num_inner() const { return static_cast<int>(used_features.size()); }
  // rows are padded to 16 bytes so the HIP histogram kernel fetches 16
  // feature bins per dwordx4 load
  int row_stride() const { return std::max(16, ((num_inner() + 15) / 16) * 16); }
};

// Row-major bin matrix resident in HBM (num_data x row_stride bytes), written by the K1 device encoder
// and adopted by the HIP training backend without a host round trip (bin_encode.hip).
struct DeviceBins {
  int device = -1;
  uint8_t* rows = nullptr;
  size_t granted = 0;
  ~DeviceBins();
};

struct Dataset {
  DatasetReference ref;
  int64_t num_data = 0;
  int row_stride = 4;                 // bytes per row in `bins`
  // Host copy of the bin matrix (num_data * row_stride). Datasets built by the device encoder keep their
  // bins only in HBM (`dev`); the host copy is materialised on first use by a host consumer (CPU backend,
  // validation scoring, get_bins) - call EnsureHostBins() before touching `bins`.
  mutable std::vector<uint8_t> bins;
  mutable bool host_valid = false;    // `bins` holds every pushed row
  std::shared_ptr<DeviceBins> dev;    // device copy, current when dev_valid
  bool dev_valid = false;
  // per-row vectors on the host block pool (host_pool.h): a repeated fit reuses the previous fit's blocks
  PooledVector<float> label;          // num_data entries; zeros unless set (see FinalizeLabel)
  PooledVector<float> weight;         // empty = unweighted
  std::vector<double> init_score;     // empty or num_data * num_tree_per_iteration
  // Init leaves the labels unwritten (the caller's set_label overwrites them all - one pass over a 44 MB
  // vector instead of two); consumers call FinalizeLabel, which zero-fills labels nobody set
  bool label_set = false;
  void SetLabel(const float* y, int64_t n);
  void FinalizeLabel();
  std::vector<int32_t> query_boundaries;  // ranking: size num_queries+1

  void Init(const DatasetReference& r, int64_t n);
  // host bins: download the device copy, or allocate rows filled with every feature's zero bin
  void EnsureHostBins() const;
  std::vector<uint8_t> DefaultRow() const;
  // Push a block of dense rows (row-major, num_cols doubles each) at `start`.
  void PushDense(const double* rows, int64_t nrows, int num_cols, int64_t start);
  void PushDenseF32(const float* rows, int64_t nrows, int num_cols, int64_t start);
  // Push CSR rows at `start` (indptr has nrows+1 entries).
  void PushCSR(const int64_t* indptr, const int32_t* indices, const double* values,
               int64_t nrows, int64_t start);
  void SetQueryFromGroupSizes(const std::vector<int32_t>& sizes);
  // host bins materialised and the device copy invalidated (thread-safe; called by every host push)
  void BeginHostPush();
  inline uint8_t Bin(int64_t row, int inner) const { return bins[row * row_stride + inner]; }
};

// K1 on the device (bin_encode.hip): same bins as PushDense / PushDenseF32; the rows stay in HBM.
void DatasetPushDenseDevice(Dataset* d, const double* rows, int64_t nrows, int num_cols, int64_t start, int device);
void DatasetPushDenseDeviceF32(Dataset* d, const float* rows, int64_t nrows, int num_cols, int64_t start, int device);
// Raw dense rows (float32 / float64, row-major) uploaded to HBM on a background thread, so the caller can
// sample rows and build bin boundaries while the copy runs; DatasetPushDeviceRows then bin-encodes them
// in place (no second transfer). Keeps `owner` (e.g. the numpy array) alive until the copy is done.
struct DeviceRows {
  DeviceRows(const void* host, int64_t nrows, int ncols, int elem_bytes, int device);
  ~DeviceRows();
  DeviceRows(const DeviceRows&) = delete;
  DeviceRows& operator=(const DeviceRows&) = delete;
  void Wait();  // copy finished (raises if it failed)
  int64_t nrows;
  int ncols, elem_bytes, device;
  void* ptr = nullptr;
  size_t granted = 0;
  std::thread worker;
  std::string error;
  // upload progress, for an encode that follows the copy chunk by chunk: chunk_ev[i] (a hipEvent_t) completes
  // when the first chunk_end[i] bytes are in HBM; `finished` once no more chunks come (done or failed)
  std::mutex mu;
  std::condition_variable cv;
  std::vector<void*> chunk_ev;
  std::vector<size_t> chunk_end;
  bool finished = false;
};
void DatasetPushDeviceRows(Dataset* d, DeviceRows* src, int64_t start);
// host (pageable) -> device copy through pinned staging buffers filled by parallel CPU threads (bin_encode.hip)
// `progress`: optional - each chunk's completion event is published there as the copy is queued
void UploadPinned(const char* host, char* dev, size_t bytes, DeviceRows* progress = nullptr);

// device -> host copy of a device-resident bin matrix (bin_encode.hip)
void DatasetDownloadBins(const Dataset& d, uint8_t* host);

// Runs of equal ids in a query-group column (LightGBMRanker): *starts gets the first row of every run (in
// row order); returns true when no id starts two runs (the rows are grouped, no reorder needed). Parallel scan.
bool GroupRuns(const int64_t* ids, int64_t n, std::vector<int64_t>* starts);

// k distinct row indices of [0, n), sorted, drawn from the seed (bin-boundary sampling, K1's host side)
std::vector<int64_t> SampleRowIndices(int64_t n, int64_t k, uint64_t seed);

}  // namespace sml
