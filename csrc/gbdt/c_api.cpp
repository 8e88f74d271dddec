// Plain C ABI of the GBDT engine (libsml_gbdt.so): the layer other languages bind to - the generated .NET
// P/Invoke wrapper (codegen.generate_dotnet) and anything with a C FFI. It plays the role lib_lightgbm's
// C API plays for the reference (the SWIG lightgbmlib calls in lightgbm/.../LightGBMUtils.scala,
// LightGBMBooster.scala: LGBM_DatasetCreateFromMat, LGBM_BoosterCreate, LGBM_BoosterUpdateOneIter,
// LGBM_BoosterPredictForMat, LGBM_BoosterSaveModelToString, LGBM_BoosterGetEval), over this engine's
// Dataset / Booster (CPU backend, or the HIP backend when device_type=gpu).
//
// Conventions: every function returns 0 on success and -1 on failure, with the message available from
// SML_GetLastError() (thread-local); handles are opaque pointers freed by the matching *Free function.
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "booster.h"
#include "config.h"
#include "dataset.h"

using namespace sml;

namespace {
thread_local std::string g_last_error;

template <class F>
int Guard(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    g_last_error = e.what();
  } catch (...) {
    g_last_error = "unknown error";
  }
  return -1;
}

struct DatasetHandle {
  std::shared_ptr<Dataset> d;
};

// rows as float64 (the engine's host binning / prediction input)
std::vector<double> AsF64(const void* data, int data_type, int64_t n) {
  std::vector<double> x(static_cast<size_t>(n));
  if (data_type == 0) {
    const float* p = static_cast<const float*>(data);
    for (int64_t i = 0; i < n; ++i) x[i] = p[i];
  } else if (data_type == 1) {
    std::memcpy(x.data(), data, sizeof(double) * static_cast<size_t>(n));
  } else {
    throw std::invalid_argument("data_type must be 0 (float32) or 1 (float64)");
  }
  return x;
}
}  // namespace

extern "C" {

const char* SML_GetLastError() { return g_last_error.c_str(); }

// Row-major dense matrix -> binned Dataset; bin boundaries from the first min(nrow, bin_construct_sample_cnt)
// rows (params as "key=value ..." like the reference's parameter strings), labels of every row.
int SML_DatasetCreateFromMat(const void* data, int data_type, int32_t nrow, int32_t ncol, const char* params,
                             const float* label, void** out) {
  return Guard([&] {
    if (!data || !label || !out || nrow <= 0 || ncol <= 0) throw std::invalid_argument("empty matrix or null pointer");
    const std::string p = params ? params : "";
    Config cfg = Config::Parse(p);
    std::vector<double> x = AsF64(data, data_type, static_cast<int64_t>(nrow) * ncol);
    const int64_t ns = std::min<int64_t>(nrow, std::max(1, cfg.bin_construct_sample_cnt));
    std::vector<std::string> names;
    for (int f = 0; f < ncol; ++f) names.push_back("Column_" + std::to_string(f));
    auto ref = DatasetReference::FromSample(x.data(), ns, ncol, nrow, cfg, names);
    auto h = std::make_unique<DatasetHandle>();
    h->d = std::make_shared<Dataset>();
    h->d->Init(ref, nrow);
    h->d->PushDense(x.data(), nrow, ncol, 0);
    h->d->SetLabel(label, nrow);
    *out = h.release();
  });
}

int SML_DatasetSetWeight(void* dataset, const float* weight, int32_t n) {
  return Guard([&] {
    auto* h = static_cast<DatasetHandle*>(dataset);
    if (!h || n != h->d->num_data) throw std::invalid_argument("weight length must equal the row count");
    h->d->weight.assign(weight, weight + n);
  });
}

int SML_DatasetGetNumData(void* dataset, int32_t* out) {
  return Guard([&] { *out = static_cast<int32_t>(static_cast<DatasetHandle*>(dataset)->d->num_data); });
}

int SML_DatasetFree(void* dataset) {
  return Guard([&] { delete static_cast<DatasetHandle*>(dataset); });
}

int SML_BoosterCreate(void* train, const char* params, void** out) {
  return Guard([&] {
    auto* h = static_cast<DatasetHandle*>(train);
    if (!h || !out) throw std::invalid_argument("null dataset or output handle");
    *out = new Booster(h->d, params ? params : "");
  });
}

int SML_BoosterAddValidData(void* booster, void* valid) {
  return Guard([&] {
    auto* b = static_cast<Booster*>(booster);
    auto* h = static_cast<DatasetHandle*>(valid);
    b->AddValidData(h->d, "valid");
  });
}

int SML_BoosterLoadModelFromString(const char* model, void** out) {
  return Guard([&] {
    if (!model || !out) throw std::invalid_argument("null model string or output handle");
    *out = Booster::FromModelString(model).release();
  });
}

int SML_BoosterFree(void* booster) {
  return Guard([&] { delete static_cast<Booster*>(booster); });
}

int SML_BoosterUpdateOneIter(void* booster, int* is_finished) {
  return Guard([&] {
    const bool done = static_cast<Booster*>(booster)->TrainOneIter();
    if (is_finished) *is_finished = done ? 1 : 0;
  });
}

int SML_BoosterGetCurrentIteration(void* booster, int* out) {
  return Guard([&] { *out = static_cast<Booster*>(booster)->CurrentIteration(); });
}

int SML_BoosterGetNumClasses(void* booster, int* out) {
  return Guard([&] { *out = static_cast<Booster*>(booster)->NumClasses(); });
}

// Metrics of data set data_idx (0 = train, 1.. = validation sets), in EvalNames order; *out_len = count.
// out_results holds buffer_len doubles; a call with a smaller buffer (or none) only reports the count, so a
// caller sized for a stale metric list (e.g. before ResetParameter changed the metrics) cannot overflow it.
int SML_BoosterGetEval(void* booster, int data_idx, int buffer_len, int* out_len, double* out_results) {
  return Guard([&] {
    auto ev = static_cast<Booster*>(booster)->Eval(data_idx);
    *out_len = static_cast<int>(ev.size());
    if (out_results && buffer_len >= *out_len)
      for (size_t i = 0; i < ev.size(); ++i) out_results[i] = ev[i].second;
  });
}

// predict_type: 0 raw, 1 normal, 2 leaf index, 3 contributions. *out_len = nrow * per-row output size
// (call with out_result == nullptr to size the buffer).
int SML_BoosterPredictForMat(void* booster, const void* data, int data_type, int32_t nrow, int32_t ncol,
                             int predict_type, int start_iteration, int num_iteration, int64_t* out_len,
                             double* out_result) {
  return Guard([&] {
    auto* b = static_cast<Booster*>(booster);
    const int per = b->PredictOutputSize(predict_type, start_iteration, num_iteration);
    *out_len = static_cast<int64_t>(nrow) * per;
    if (!out_result) return;
    std::vector<double> x = AsF64(data, data_type, static_cast<int64_t>(nrow) * ncol);
    b->Predict(x.data(), nrow, ncol, predict_type, start_iteration, num_iteration, out_result);
  });
}

// Model text into out_str (buffer_len bytes incl. the terminating NUL); *out_len = bytes needed. A call
// with a too-small buffer only reports the size.
int SML_BoosterSaveModelToString(void* booster, int start_iteration, int num_iteration, int64_t buffer_len,
                                 int64_t* out_len, char* out_str) {
  return Guard([&] {
    const std::string s = static_cast<Booster*>(booster)->SaveModelToString(start_iteration, num_iteration, 0);
    *out_len = static_cast<int64_t>(s.size()) + 1;
    if (out_str && buffer_len >= *out_len) std::memcpy(out_str, s.c_str(), s.size() + 1);
  });
}

}  // extern "C"
