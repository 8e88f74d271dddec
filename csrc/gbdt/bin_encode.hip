// K1: bin encoding on the MI355X (reference call sites
// LGBM_DatasetPushRowsWithMetadata, lightgbm/.../StreamingPartitionTask.scala
// :202-236, whose bin lookup runs inside lib_lightgbm on the executor's CPU).
//
// Raw feature rows are streamed to the device in chunks; one thread encodes
// four features of one row (one dword of the row-major bin matrix) with a
// binary search over that feature's upper bounds held in LDS, using the same
// double comparisons as BinMapper::ValueToBin, so the result is bit-identical
// with the host path. Categorical features use a dense category->bin table.
// The bins stay in HBM (Dataset::dev): the HIP training backend adopts them
// without a host round trip, and a host copy is only materialised when a host
// consumer asks for it (Dataset::EnsureHostBins). The raw rows stream up in
// chunks whose copies overlap the previous chunk's encode.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <vector>

#include "dataset.h"
#include "hip_common.h"
#include "trace.h"

namespace sml {
namespace {

constexpr int kEncThreads = 256;
constexpr int kMaxCatTable = 1 << 16;  // dense category table cap per feature

struct EncMeta {
  const int32_t* col;        // inner feature -> source column
  const int32_t* bound_off;  // inner feature -> offset into bounds
  const int32_t* nbound;     // number of upper bounds
  const int32_t* flags;      // bit0 categorical, bit1 NaN-missing
  const int32_t* num_bin;
  const int32_t* default_bin;
  const int32_t* cat_off;  // categorical: offset into the category table (or -1)
  const int32_t* cat_len;
  const double* bounds;
  const float* fbounds;  // each bound rounded down to a float (float32 inputs)
  const uint16_t* cat_table;
  int F;       // inner features
  int stride;  // bytes per row in the bin matrix
  int total_bounds;
};

// Per-feature metadata staged in LDS next to the bounds (the value loop reads it per element).
struct FeatLds {
  int col, off, nbound, flags, num_bin, default_bin, cat_off, cat_len;
};

// Bounds are compared in the input's precision: for float32 rows every double upper bound is replaced by
// the largest float not above it (Encoder::fbounds_), and for a float v, v <= b (double) <=> v <= that
// float - no float lies between them - so the bins are bit-identical with BinMapper::ValueToBin's double
// comparisons while the bounds take half the LDS (more resident blocks per CU).
template <class T, class B>
__device__ __forceinline__ uint32_t EncodeOne(const EncMeta& m, const B* sb, const FeatLds& fm, T raw) {
  const int nb = fm.num_bin;
  if (fm.flags & 1) {
    const double v = static_cast<double>(raw);
    if (isnan(v) || v < 0) return static_cast<uint32_t>(nb - 1);
    const int c = static_cast<int>(v);
    if (fm.cat_off < 0 || c >= fm.cat_len) return static_cast<uint32_t>(nb - 1);
    const uint16_t b = m.cat_table[fm.cat_off + c];
    return b == 0xFFFFu ? static_cast<uint32_t>(nb - 1) : b;
  }
  B v = static_cast<B>(raw);
  if (isnan(v)) {
    if (fm.flags & 2) return static_cast<uint32_t>(nb - 1);
    v = B(0);
  }
  const B* ub = sb + fm.off;
  // first index with v <= ub[i] among the first nbound - 1 bounds, else nbound - 1
  int base = 0, len = fm.nbound - 1;
  while (len > 0) {
    const int half = len >> 1;
    if (ub[base + half] < v) { base += half + 1; len -= half + 1; } else { len = half; }
  }
  return static_cast<uint32_t>(base);
}

template <class T>
__global__ __launch_bounds__(kEncThreads) void encode_kernel(EncMeta m, const T* __restrict__ X, int64_t nrows,
                                                             int ncols, uint32_t* __restrict__ out) {
  using B = T;  // bounds in the input's precision (float rows: the round-down float bounds)
  extern __shared__ double s_dyn[];
  B* sb = reinterpret_cast<B*>(s_dyn);
  FeatLds* sf = reinterpret_cast<FeatLds*>(sb + ((m.total_bounds + 1) & ~1));
  const B* gb = sizeof(B) == 4 ? reinterpret_cast<const B*>(m.fbounds) : reinterpret_cast<const B*>(m.bounds);
  for (int i = threadIdx.x; i < m.total_bounds; i += kEncThreads) sb[i] = gb[i];
  for (int f = threadIdx.x; f < m.F; f += kEncThreads)
    sf[f] = FeatLds{m.col[f], m.bound_off[f], m.nbound[f], m.flags[f], m.num_bin[f], m.default_bin[f], m.cat_off[f],
                    m.cat_len[f]};
  __syncthreads();
  const int words = m.stride / 4;
  const int64_t total = nrows * words;
  for (int64_t t = blockIdx.x * (int64_t)kEncThreads + threadIdx.x; t < total; t += (int64_t)gridDim.x * kEncThreads) {
    const int64_t r = t / words;
    const int w = static_cast<int>(t - r * words);
    uint32_t packed = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int f = w * 4 + j;
      uint32_t b = 0;
      if (f < m.F) {
        const FeatLds fm = sf[f];
        b = fm.col < ncols ? EncodeOne<T, B>(m, sb, fm, X[r * ncols + fm.col]) : static_cast<uint32_t>(fm.default_bin);
      }
      packed |= (b & 255u) << (8 * j);
    }
    out[t] = packed;
  }
}

template <class T>
size_t EncodeLds(const EncMeta& m) {
  return sizeof(T) * static_cast<size_t>((m.total_bounds + 1) & ~1) + sizeof(FeatLds) * static_cast<size_t>(std::max(1, m.F));
}

// Device copies of the bin mappers of one reference.
class Encoder {
 public:
  Encoder(const DatasetReference& ref, int stride) {
    const int F = ref.num_inner();
    std::vector<int32_t> col(F), off(F), nbd(F), fl(F), nb(F), db(F), coff(F, -1), clen(F, 0);
    std::vector<double> bounds;
    std::vector<uint16_t> cats;
    for (int f = 0; f < F; ++f) {
      const BinMapper& bm = ref.mappers[ref.used_features[f]];
      col[f] = ref.used_features[f];
      off[f] = static_cast<int32_t>(bounds.size());
      nbd[f] = static_cast<int32_t>(bm.upper_bounds.size());
      bounds.insert(bounds.end(), bm.upper_bounds.begin(), bm.upper_bounds.end());
      fl[f] = (bm.is_categorical ? 1 : 0) | (bm.missing_type == kMissingNaN ? 2 : 0);
      nb[f] = bm.num_bin;
      db[f] = bm.default_bin;
      if (bm.is_categorical) {
        int maxc = -1;
        for (const auto& kv : bm.cat2bin) maxc = std::max(maxc, kv.first);
        if (maxc >= kMaxCatTable) throw std::runtime_error("device bin encode: category value too large");
        coff[f] = static_cast<int32_t>(cats.size());
        clen[f] = maxc + 1;
        cats.resize(cats.size() + static_cast<size_t>(maxc + 1), 0xFFFFu);
        for (const auto& kv : bm.cat2bin)
          if (kv.first >= 0) cats[coff[f] + kv.first] = static_cast<uint16_t>(kv.second);
      }
    }
    if (bounds.size() * sizeof(double) + sizeof(FeatLds) * static_cast<size_t>(F) + 8 > 64 * 1024)
      throw std::runtime_error("device bin encode: bin bounds exceed the LDS budget");
    ints_.alloc(8 * static_cast<size_t>(std::max(1, F)));
    auto up = [&](int k, const std::vector<int32_t>& v) {
      if (F) SML_HIP_CHECK(hipMemcpy(ints_.get() + k * F, v.data(), sizeof(int32_t) * F, hipMemcpyHostToDevice));
    };
    up(0, col); up(1, off); up(2, nbd); up(3, fl); up(4, nb); up(5, db); up(6, coff); up(7, clen);
    bounds_.alloc(std::max<size_t>(1, bounds.size()));
    if (!bounds.empty())
      SML_HIP_CHECK(hipMemcpy(bounds_.get(), bounds.data(), sizeof(double) * bounds.size(), hipMemcpyHostToDevice));
    std::vector<float> fb(bounds.size());
    for (size_t i = 0; i < bounds.size(); ++i) {
      float x = static_cast<float>(bounds[i]);
      if (static_cast<double>(x) > bounds[i]) x = std::nextafter(x, -INFINITY);
      fb[i] = x;
    }
    fbounds_.alloc(std::max<size_t>(1, fb.size()));
    if (!fb.empty())
      SML_HIP_CHECK(hipMemcpy(fbounds_.get(), fb.data(), sizeof(float) * fb.size(), hipMemcpyHostToDevice));
    cats_.alloc(std::max<size_t>(1, cats.size()));
    if (!cats.empty())
      SML_HIP_CHECK(hipMemcpy(cats_.get(), cats.data(), sizeof(uint16_t) * cats.size(), hipMemcpyHostToDevice));
    int32_t* p = ints_.get();
    m_.col = p; m_.bound_off = p + F; m_.nbound = p + 2 * F; m_.flags = p + 3 * F; m_.num_bin = p + 4 * F;
    m_.default_bin = p + 5 * F; m_.cat_off = p + 6 * F; m_.cat_len = p + 7 * F;
    m_.bounds = bounds_.get(); m_.fbounds = fbounds_.get(); m_.cat_table = cats_.get();
    m_.F = F; m_.stride = stride; m_.total_bounds = static_cast<int>(bounds.size());
  }

  // Encode `nrows` raw rows into the device bin matrix at `dev_out` (row-major). The raw input streams
  // up in ~64 MB chunks through two staging buffers: chunk c+1's host->device copy (copy stream) overlaps
  // chunk c's encode (kernel stream); event pairs order slot reuse.
  template <class T>
  void Encode(const T* rows, int64_t nrows, int ncols, uint8_t* dev_out, hipStream_t ks, hipStream_t cs) {
    if (nrows <= 0) return;
    const int64_t chunk = std::max<int64_t>(1, (64ll << 20) / (static_cast<int64_t>(std::max(1, ncols)) * sizeof(T)));
    const int64_t cap = std::min(chunk, nrows);
    for (int b = 0; b < 2; ++b) in_[b].alloc(static_cast<size_t>(cap) * ncols * sizeof(T));
    const size_t lds = EncodeLds<T>(m_);
    int c = 0;
    for (int64_t r0 = 0; r0 < nrows; r0 += chunk, ++c) {
      const int slot = c & 1;
      const int64_t nr = std::min(chunk, nrows - r0);
      if (c >= 2) SML_HIP_CHECK(hipStreamWaitEvent(cs, done_[slot], 0));
      SML_HIP_CHECK(hipMemcpyAsync(in_[slot].get(), rows + r0 * ncols, static_cast<size_t>(nr) * ncols * sizeof(T),
                                   hipMemcpyHostToDevice, cs));
      SML_HIP_CHECK(hipEventRecord(copied_[slot], cs));
      SML_HIP_CHECK(hipStreamWaitEvent(ks, copied_[slot], 0));
      const int64_t words = nr * (m_.stride / 4);
      const int grid =
          static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(4096, (words + kEncThreads - 1) / kEncThreads)));
      hipLaunchKernelGGL(encode_kernel<T>, dim3(grid), dim3(kEncThreads), lds, ks, m_,
                         reinterpret_cast<const T*>(in_[slot].get()), nr, ncols,
                         reinterpret_cast<uint32_t*>(dev_out + r0 * m_.stride));
      SML_HIP_CHECK(hipGetLastError());
      SML_HIP_CHECK(hipEventRecord(done_[slot], ks));
    }
    SML_HIP_CHECK(hipStreamSynchronize(ks));
  }

  // Encode rows already resident in HBM (DeviceRows): one launch over all rows.
  template <class T>
  void EncodeResident(const T* dev_rows, int64_t nrows, int ncols, uint8_t* dev_out, hipStream_t ks,
                      bool sync = true) {
    if (nrows <= 0) return;
    const size_t lds = EncodeLds<T>(m_);
    const int64_t words = nrows * (m_.stride / 4);
    const int grid = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(8192, (words + kEncThreads - 1) / kEncThreads)));
    hipLaunchKernelGGL(encode_kernel<T>, dim3(grid), dim3(kEncThreads), lds, ks, m_, dev_rows, nrows, ncols,
                       reinterpret_cast<uint32_t*>(dev_out));
    SML_HIP_CHECK(hipGetLastError());
    if (sync) SML_HIP_CHECK(hipStreamSynchronize(ks));
  }

  Encoder(const Encoder&) = delete;
  Encoder& operator=(const Encoder&) = delete;
  ~Encoder() {
    for (hipEvent_t e : copied_) if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : done_) if (e) (void)hipEventDestroy(e);
  }
  void MakeEvents() {
    for (hipEvent_t& e : copied_) SML_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (hipEvent_t& e : done_) SML_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }

 private:
  EncMeta m_{};
  DevBuf<int32_t> ints_;
  DevBuf<double> bounds_;
  DevBuf<float> fbounds_;
  DevBuf<uint16_t> cats_;
  DevBuf<uint8_t> in_[2];
  hipEvent_t copied_[2] = {nullptr, nullptr}, done_[2] = {nullptr, nullptr};
};

// every row = the dataset's default row (each feature's zero bin)
__global__ void fill_rows_kernel(uint4* __restrict__ out, int64_t nrows, int w4, uint4 a, uint4 b) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nrows * w4; t += (int64_t)gridDim.x * blockDim.x)
    out[t] = (t % w4) == 0 ? a : b;
}

std::mutex& DevBinsMutex() {
  static std::mutex m;
  return m;
}

// The HBM bin matrix of `d` on `device`, current for every row pushed so far (uploads the host copy or
// fills default rows the first time).
void EnsureDeviceBins(Dataset* d, int device, hipStream_t s) {
  TraceRange tr("sml::EnsureDeviceBins");
  std::lock_guard<std::mutex> lk(DevBinsMutex());
  if (d->dev && d->dev->device != device) { d->dev.reset(); d->dev_valid = false; }
  if (!d->dev) {
    auto db = std::make_shared<DeviceBins>();
    db->device = device;
    db->rows = static_cast<uint8_t*>(DevPoolAlloc(std::max<size_t>(16, static_cast<size_t>(d->num_data) * d->row_stride),
                                                  &db->granted));
    d->dev = db;
    d->dev_valid = false;
  }
  if (d->dev_valid) return;
  if (d->host_valid) {
    SML_HIP_CHECK(hipMemcpyAsync(d->dev->rows, d->bins.data(), static_cast<size_t>(d->num_data) * d->row_stride,
                                 hipMemcpyHostToDevice, s));
  } else if (d->num_data > 0) {
    if (d->row_stride % 16 != 0 || d->row_stride > 32 * 16) throw std::runtime_error("device bins: row stride");
    const std::vector<uint8_t> z = d->DefaultRow();
    // rows are 16 or 32 bytes for <= 32 features; wider rows repeat the fill per 16-byte word
    const int w4 = d->row_stride / 16;
    if (w4 > 2) {
      std::vector<uint8_t> all(static_cast<size_t>(d->num_data) * d->row_stride);
      for (int64_t i = 0; i < d->num_data; ++i) std::memcpy(&all[i * d->row_stride], z.data(), d->row_stride);
      SML_HIP_CHECK(hipMemcpyAsync(d->dev->rows, all.data(), all.size(), hipMemcpyHostToDevice, s));
      SML_HIP_CHECK(hipStreamSynchronize(s));
    } else {
      uint4 a, b = make_uint4(0, 0, 0, 0);
      std::memcpy(&a, z.data(), 16);
      if (w4 == 2) std::memcpy(&b, z.data() + 16, 16);
      else b = a;
      const int64_t words = d->num_data * w4;
      const int grid = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(8192, (words + 255) / 256)));
      hipLaunchKernelGGL(fill_rows_kernel, dim3(grid), dim3(256), 0, s, reinterpret_cast<uint4*>(d->dev->rows),
                         d->num_data, w4, a, b);
      SML_HIP_CHECK(hipGetLastError());
    }
  }
  SML_HIP_CHECK(hipStreamSynchronize(s));
  d->dev_valid = true;
}

template <class T>
void PushDenseDeviceImpl(Dataset* d, const T* rows, int64_t nrows, int num_cols, int64_t start, int device) {
  TraceRange tr("sml::PushRowsEncode");
  if (start < 0 || start + nrows > d->num_data) throw std::runtime_error("push_dense_gpu out of range");
  if (d->row_stride % 4 != 0) throw std::runtime_error("device bin encode needs a 4-byte aligned row stride");
  if (device >= 0) SML_HIP_CHECK(hipSetDevice(device));
  SML_HIP_CHECK(hipGetDevice(&device));
  hipStream_t ks = nullptr, cs = nullptr;
  SML_HIP_CHECK(hipStreamCreateWithFlags(&ks, hipStreamNonBlocking));
  try {
    SML_HIP_CHECK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    EnsureDeviceBins(d, device, ks);
    uint8_t* dst = d->dev->rows + static_cast<size_t>(start) * d->row_stride;
    {
      Encoder enc(d->ref, d->row_stride);
      enc.MakeEvents();
      enc.Encode(rows, nrows, num_cols, dst, ks, cs);
    }
    // a host copy that already exists stays complete: mirror the pushed rows
    if (d->host_valid)
      SML_HIP_CHECK(hipMemcpy(d->bins.data() + static_cast<size_t>(start) * d->row_stride, dst,
                              static_cast<size_t>(nrows) * d->row_stride, hipMemcpyDeviceToHost));
  } catch (...) {
    (void)hipStreamDestroy(ks);
    if (cs) (void)hipStreamDestroy(cs);
    throw;
  }
  SML_HIP_CHECK(hipStreamDestroy(ks));
  SML_HIP_CHECK(hipStreamDestroy(cs));
}

template <class T>
void PushResidentImpl(Dataset* d, DeviceRows* src, int64_t start) {
  TraceRange tr("sml::EncodeResidentRows");
  const int64_t nrows = src->nrows;
  if (start < 0 || start + nrows > d->num_data) throw std::runtime_error("push_device_rows out of range");
  if (d->row_stride % 4 != 0) throw std::runtime_error("device bin encode needs a 4-byte aligned row stride");
  SML_HIP_CHECK(hipSetDevice(src->device));
  hipStream_t ks = nullptr;
  SML_HIP_CHECK(hipStreamCreateWithFlags(&ks, hipStreamNonBlocking));
  try {
    EnsureDeviceBins(d, src->device, ks);
    uint8_t* dst = d->dev->rows + static_cast<size_t>(start) * d->row_stride;
    {
      // the encode follows the upload: rows already in HBM are encoded at once, the rest chunk by chunk as
      // their copies land (a device-side wait on each chunk's event), so the bin matrix is ready ~one chunk
      // after the last byte arrives instead of one whole-matrix encode after the upload (r6)
      Encoder enc(d->ref, d->row_stride);
      const T* rows = static_cast<const T*>(src->ptr);
      const size_t row_bytes = static_cast<size_t>(src->ncols) * sizeof(T);
      int64_t r_done = 0;
      for (size_t c = 0;; ++c) {
        hipEvent_t e = nullptr;
        size_t end = 0;
        {
          std::unique_lock<std::mutex> lk(src->mu);
          src->cv.wait(lk, [&] { return src->chunk_ev.size() > c || src->finished; });
          if (src->chunk_ev.size() <= c) break;
          e = static_cast<hipEvent_t>(src->chunk_ev[c]);
          end = src->chunk_end[c];
        }
        const int64_t r_end = std::min<int64_t>(nrows, static_cast<int64_t>(end / row_bytes));
        if (r_end <= r_done) continue;
        SML_HIP_CHECK(hipStreamWaitEvent(ks, e, 0));
        enc.EncodeResident(rows + r_done * src->ncols, r_end - r_done, src->ncols, dst + r_done * d->row_stride, ks,
                           false);
        r_done = r_end;
      }
      src->Wait();  // the copy thread is done (raises if it failed)
      enc.EncodeResident(rows + r_done * src->ncols, nrows - r_done, src->ncols, dst + r_done * d->row_stride, ks,
                         false);
      SML_HIP_CHECK(hipStreamSynchronize(ks));
    }
    if (d->host_valid)
      SML_HIP_CHECK(hipMemcpy(d->bins.data() + static_cast<size_t>(start) * d->row_stride, dst,
                              static_cast<size_t>(nrows) * d->row_stride, hipMemcpyDeviceToHost));
  } catch (...) {
    (void)hipStreamDestroy(ks);
    throw;
  }
  SML_HIP_CHECK(hipStreamDestroy(ks));
}

}  // namespace

// ---------------------------------------------------------------- pinned upload
// Host -> HBM copy of a pageable buffer at DMA speed: the runtime's pageable path stages through one
// CPU memcpy thread (~25 GB/s measured for the 1.2 GB bench matrix). Here kStageBufs pinned staging
// buffers (allocated once per process) are filled by kCopyThreads CPU threads in parallel and drained
// by the copy engine on one stream, so the CPU copy of chunk k+1 overlaps the DMA of chunk k.
namespace {
constexpr int kStageBufs = 4;
constexpr size_t kStageBytes = 32ull << 20;

struct StagePool {
  std::mutex mu;
  char* buf[kStageBufs] = {};
  ~StagePool() {
    for (char* b : buf) if (b) (void)hipHostFree(b);
  }
};
StagePool& Stage() {
  static StagePool p;
  return p;
}

int CopyThreads() {
  int n = 8;
  if (const char* e = std::getenv("SML_UPLOAD_THREADS")) n = std::atoi(e);
  const unsigned hw = std::thread::hardware_concurrency();
  return std::max(1, std::min<int>(n, hw ? static_cast<int>(hw) : 1));
}

void ParallelCopy(char* dst, const char* src, size_t bytes, int threads) {
  if (threads <= 1 || bytes < (4u << 20)) {
    std::memcpy(dst, src, bytes);
    return;
  }
  std::vector<std::thread> th;
  const size_t per = (bytes + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const size_t a = t * per, b = std::min(bytes, a + per);
    if (a >= b) break;
    th.emplace_back([=]() { std::memcpy(dst + a, src + a, b - a); });
  }
  for (auto& x : th) x.join();
}
}  // namespace

void UploadPinned(const char* host, char* dev, size_t bytes, DeviceRows* progress) {
  TraceRange tr("sml::UploadPinned");
  StagePool& sp = Stage();
  std::lock_guard<std::mutex> lk(sp.mu);  // one pinned pipeline at a time per process
  for (auto& b : sp.buf)
    if (!b) SML_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&b), kStageBytes, hipHostMallocDefault));
  hipStream_t s = nullptr;
  SML_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev[kStageBufs] = {};
  bool used[kStageBufs] = {};
  try {
    for (auto& e : ev) SML_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    const int threads = CopyThreads();
    int k = 0;
    for (size_t off = 0; off < bytes; off += kStageBytes, k = (k + 1) % kStageBufs) {
      const size_t n = std::min(kStageBytes, bytes - off);
      if (used[k]) SML_HIP_CHECK(hipEventSynchronize(ev[k]));  // the DMA that last read this buffer is done
      ParallelCopy(sp.buf[k], host + off, n, threads);
      SML_HIP_CHECK(hipMemcpyAsync(dev + off, sp.buf[k], n, hipMemcpyHostToDevice, s));
      SML_HIP_CHECK(hipEventRecord(ev[k], s));
      used[k] = true;
      if (progress) {  // the encode may start on these rows as soon as this copy lands
        hipEvent_t ce = nullptr;
        SML_HIP_CHECK(hipEventCreateWithFlags(&ce, hipEventDisableTiming));
        SML_HIP_CHECK(hipEventRecord(ce, s));
        std::lock_guard<std::mutex> g(progress->mu);
        progress->chunk_ev.push_back(ce);
        progress->chunk_end.push_back(off + n);
        progress->cv.notify_all();
      }
    }
    SML_HIP_CHECK(hipStreamSynchronize(s));
  } catch (...) {
    (void)hipStreamSynchronize(s);
    for (auto& e : ev) if (e) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(s);
    throw;
  }
  for (auto& e : ev) (void)hipEventDestroy(e);
  SML_HIP_CHECK(hipStreamDestroy(s));
}

// ---------------------------------------------------------------- DeviceRows
DeviceRows::DeviceRows(const void* host, int64_t nrows_, int ncols_, int elem_bytes_, int device_)
    : nrows(nrows_), ncols(ncols_), elem_bytes(elem_bytes_), device(device_) {
  if (elem_bytes != 4 && elem_bytes != 8) throw std::runtime_error("DeviceRows: float32 or float64 rows");
  if (device < 0) SML_HIP_CHECK(hipGetDevice(&device));
  SML_HIP_CHECK(hipSetDevice(device));
  const size_t bytes = static_cast<size_t>(nrows) * ncols * elem_bytes;
  ptr = DevPoolAlloc(std::max<size_t>(bytes, 16), &granted);
  // the copy runs on its own thread and stream so the caller (row sampling, bin boundaries) overlaps it
  worker = std::thread([this, host, bytes]() {
    try {
      SML_HIP_CHECK(hipSetDevice(device));
      UploadPinned(static_cast<const char*>(host), static_cast<char*>(ptr), bytes, this);
    } catch (const std::exception& e) {
      error = e.what();
    }
    std::lock_guard<std::mutex> g(mu);
    finished = true;
    cv.notify_all();
  });
}

void DeviceRows::Wait() {
  if (worker.joinable()) worker.join();
  if (!error.empty()) throw std::runtime_error("DeviceRows upload failed: " + error);
}

DeviceRows::~DeviceRows() {
  if (worker.joinable()) worker.join();
  for (void* e : chunk_ev) (void)hipEventDestroy(static_cast<hipEvent_t>(e));
  if (ptr) DevPoolFree(ptr, granted);
}

void DatasetPushDeviceRows(Dataset* d, DeviceRows* src, int64_t start) {
  if (src->elem_bytes == 4) PushResidentImpl<float>(d, src, start);
  else PushResidentImpl<double>(d, src, start);
}

void DatasetPushDenseDevice(Dataset* d, const double* rows, int64_t nrows, int num_cols, int64_t start, int device) {
  PushDenseDeviceImpl(d, rows, nrows, num_cols, start, device);
}

void DatasetPushDenseDeviceF32(Dataset* d, const float* rows, int64_t nrows, int num_cols, int64_t start,
                               int device) {
  PushDenseDeviceImpl(d, rows, nrows, num_cols, start, device);
}

void DatasetDownloadBins(const Dataset& d, uint8_t* host) {
  if (!d.dev || !d.dev_valid) throw std::runtime_error("dataset has no device bins");
  int cur = -1;
  SML_HIP_CHECK(hipGetDevice(&cur));
  if (cur != d.dev->device) SML_HIP_CHECK(hipSetDevice(d.dev->device));
  SML_HIP_CHECK(hipMemcpy(host, d.dev->rows, static_cast<size_t>(d.num_data) * d.row_stride, hipMemcpyDeviceToHost));
  if (cur != d.dev->device) SML_HIP_CHECK(hipSetDevice(cur));
}

DeviceBins::~DeviceBins() {
  if (rows) DevPoolFree(rows, granted);
}

}  // namespace sml
