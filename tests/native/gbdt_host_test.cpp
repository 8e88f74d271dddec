// Native host test of the GBDT engine for sanitizer builds (ASan + UBSan, TSan):
// dataset construction (dense + CSR), training for several objectives/boosting modes with the OpenMP CPU
// backend, model text round trip, prediction consistency, and the concurrent paths the Python layer drives
// from worker threads (disjoint-offset pushes into one Dataset - StreamingPartitionTask.scala:220-231 - and
// predictions from several threads on one Booster), which the TSan build checks with >= 4 threads.
// Exit code != 0 on any mismatch.
#include <cmath>
#include <cstdio>
#include <memory>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "booster.h"
#include "config.h"
#include "dataset.h"

using namespace sml;

static int failures = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                       \
    }                                                                   \
  } while (0)

static void run(const std::string& params, bool csr) {
  const int n = 4000, F = 7;
  std::mt19937 rng(7);
  std::normal_distribution<double> nd;
  std::vector<double> X(static_cast<size_t>(n) * F);
  std::vector<float> y(n);
  for (int i = 0; i < n; ++i) {
    for (int f = 0; f < F; ++f) X[i * F + f] = (f == 3 && i % 5 == 0) ? 0.0 : nd(rng);
    if (i % 97 == 0) X[i * F + 2] = NAN;
    const double s = X[i * F] + 0.5 * X[i * F + 1] * (std::isnan(X[i * F + 2]) ? 0.0 : X[i * F + 2]);
    y[i] = params.find("regression") != std::string::npos ? static_cast<float>(s) : (s > 0 ? 1.f : 0.f);
  }
  Config cfg = Config::Parse(params);
  std::vector<std::string> names;
  for (int f = 0; f < F; ++f) names.push_back("f" + std::to_string(f));
  auto ref = DatasetReference::FromSample(X.data(), n, F, n, cfg, names);
  auto ds = std::make_shared<Dataset>();
  ds->Init(ref, n);
  if (csr) {
    std::vector<int64_t> indptr(n + 1, 0);
    std::vector<int32_t> idx;
    std::vector<double> val;
    for (int i = 0; i < n; ++i) {
      for (int f = 0; f < F; ++f)
        if (X[i * F + f] != 0.0) { idx.push_back(f); val.push_back(X[i * F + f]); }
      indptr[i + 1] = static_cast<int64_t>(idx.size());
    }
    ds->PushCSR(indptr.data(), idx.data(), val.data(), n, 0);
  } else {
    ds->PushDense(X.data(), n, F, 0);
  }
  ds->SetLabel(y.data(), static_cast<int64_t>(y.size()));
  Booster b(ds, params);
  // a validation set (the first 1000 rows): its incrementally folded scores equal the model's raw predictions
  const int nv = 1000;
  auto vd = std::make_shared<Dataset>();
  vd->Init(ref, nv);
  vd->PushDense(X.data(), nv, F, 0);
  vd->SetLabel(y.data(), nv);
  b.AddValidData(vd, "valid_0");
  for (int it = 0; it < 15; ++it)
    if (b.TrainOneIter()) break;
  {
    std::vector<double> vs, raw(static_cast<size_t>(nv) * b.NumClasses());
    b.GetPredictForValid(0, &vs);
    b.Predict(X.data(), nv, F, kPredictRaw, 0, -1, raw.data());  // raw scores, row-major n x K
    const int K = b.NumClasses();
    CHECK(vs.size() == raw.size());
    for (int i = 0; i < nv && vs.size() == raw.size(); ++i)
      for (int k = 0; k < K; ++k) CHECK(std::fabs(vs[k * nv + i] - raw[i * K + k]) <= 1e-9 * (1 + std::fabs(raw[i * K + k])));
    for (const auto& kv : b.Eval(1)) CHECK(std::isfinite(kv.second));
  }
  std::vector<double> p1(static_cast<size_t>(n) * b.NumClasses());
  b.Predict(X.data(), n, F, 0, 0, -1, p1.data());
  const std::string model = b.SaveModelToString(0, -1, 0);
  auto b2 = Booster::FromModelString(model);
  std::vector<double> p2(p1.size());
  b2->Predict(X.data(), n, F, 0, 0, -1, p2.data());
  for (size_t i = 0; i < p1.size(); ++i) CHECK(std::fabs(p1[i] - p2[i]) <= 1e-12 * (1 + std::fabs(p1[i])));
  CHECK(b2->SaveModelToString(0, -1, 0) == model);
  std::vector<double> contrib(static_cast<size_t>(n) * (F + 1));
  if (b.NumClasses() == 1) {
    b.Predict(X.data(), n, F, 3, 0, -1, contrib.data());  // SHAP: sums to the raw score
    std::vector<double> raw(n);
    b.Predict(X.data(), n, F, 0, 0, -1, raw.data());  // kPredictRaw
    for (int i = 0; i < n; i += 101) {
      double s = 0;
      for (int f = 0; f <= F; ++f) s += contrib[i * (F + 1) + f];
      CHECK(std::fabs(s - raw[i]) < 1e-6 * (1 + std::fabs(raw[i])));
    }
  }
  std::printf("ok  %-70s csr=%d trees=%zu\n", params.c_str(), csr ? 1 : 0, b.trees().size());
}

// Truncated / corrupted model strings must be rejected with an exception (never read out of bounds or
// recurse without end): each mutation below breaks one invariant of a valid two-tree model.
static void malformed_models() {
  const int n = 500, F = 3;
  std::mt19937 rng(3);
  std::normal_distribution<double> nd;
  std::vector<double> X(static_cast<size_t>(n) * F);
  std::vector<float> y(n);
  for (int i = 0; i < n; ++i) {
    for (int f = 0; f < F; ++f) X[i * F + f] = nd(rng);
    y[i] = X[i * F] > 0 ? 1.f : 0.f;
  }
  const std::string params = "objective=binary num_leaves=4 min_data_in_leaf=5 device_type=cpu";
  Config cfg = Config::Parse(params);
  auto ref = DatasetReference::FromSample(X.data(), n, F, n, cfg, {"a", "b", "c"});
  auto ds = std::make_shared<Dataset>();
  ds->Init(ref, n);
  ds->PushDense(X.data(), n, F, 0);
  ds->SetLabel(y.data(), static_cast<int64_t>(y.size()));
  Booster b(ds, params);
  b.TrainOneIter();
  b.TrainOneIter();
  const std::string good = b.SaveModelToString(0, -1, 0);
  auto replace_line = [&](const std::string& key, const std::string& val) {
    std::string m = good;
    const size_t p = m.find("\n" + key + "=");
    if (p == std::string::npos) return std::string();
    const size_t e = m.find('\n', p + 1);
    return m.substr(0, p + 1) + key + "=" + val + m.substr(e);
  };
  const std::vector<std::pair<std::string, std::string>> bad = {
      {"left_child", "1 -2"},           // truncated array
      {"left_child", "5 -1 -3"},        // child index out of range
      {"left_child", "0 -1 -3"},        // cycle back to the root
      {"right_child", "-2 -2 -4"},      // one leaf reached twice, another never
      {"split_feature", "0 99 1"},      // feature beyond max_feature_idx
      {"leaf_value", "0.1"},            // too few leaf values
      {"num_leaves", "-3"},             // negative size
      {"decision_type", "1 1 1"},       // categorical split with no category sets
      {"threshold", "abc def ghi"},     // not numbers
  };
  int rejected = 0;
  for (const auto& kv : bad) {
    const std::string m = replace_line(kv.first, kv.second);
    if (m.empty()) { std::fprintf(stderr, "no %s line to mutate\n", kv.first.c_str()); ++failures; continue; }
    try {
      auto bb = Booster::FromModelString(m);
      std::vector<double> out(n);
      bb->Predict(X.data(), n, F, 0, 0, -1, out.data());
      std::fprintf(stderr, "malformed model accepted: %s=%s\n", kv.first.c_str(), kv.second.c_str());
      ++failures;
    } catch (const std::exception&) {
      ++rejected;
    }
  }
  // a truncated string (cut mid-tree) is rejected too
  try {
    auto bb = Booster::FromModelString(good.substr(0, good.find("leaf_value")));
    (void)bb;
    std::fprintf(stderr, "truncated model accepted\n");
    ++failures;
  } catch (const std::exception&) {
    ++rejected;
  }
  std::printf("ok  malformed model strings rejected: %d\n", rejected);
}

// Four threads push disjoint row blocks of one Dataset at once (dense f64, dense f32 and CSR pushes),
// then four threads predict disjoint row ranges of one trained Booster while OpenMP runs inside each call.
static void concurrent_push_and_predict() {
  const int n = 24000, F = 9, T = 4;
  std::mt19937 rng(11);
  std::normal_distribution<double> nd;
  std::vector<double> X(static_cast<size_t>(n) * F);
  std::vector<float> Xf(X.size());
  std::vector<float> y(n);
  for (int i = 0; i < n; ++i) {
    for (int f = 0; f < F; ++f) X[i * F + f] = (f == 4 && i % 3 == 0) ? 0.0 : nd(rng);
    y[i] = X[i * F] + X[i * F + 1] > 0 ? 1.f : 0.f;
  }
  for (size_t i = 0; i < X.size(); ++i) Xf[i] = static_cast<float>(X[i]);
  const std::string params = "objective=binary num_leaves=15 device_type=cpu num_threads=4";
  Config cfg = Config::Parse(params);
  std::vector<std::string> names;
  for (int f = 0; f < F; ++f) names.push_back("f" + std::to_string(f));
  auto ref = DatasetReference::FromSample(X.data(), n, F, n, cfg, names);
  auto serial = std::make_shared<Dataset>();
  serial->Init(ref, n);
  serial->PushDense(X.data(), n, F, 0);
  for (int mode = 0; mode < 3; ++mode) {
    auto ds = std::make_shared<Dataset>();
    ds->Init(ref, n);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) {
      th.emplace_back([&, t]() {
        const int64_t r0 = static_cast<int64_t>(n) * t / T, r1 = static_cast<int64_t>(n) * (t + 1) / T;
        const int64_t m = r1 - r0;
        if (mode == 0) {
          ds->PushDense(X.data() + r0 * F, m, F, r0);
        } else if (mode == 1) {
          ds->PushDenseF32(Xf.data() + r0 * F, m, F, r0);
        } else {
          std::vector<int64_t> ip(m + 1, 0);
          std::vector<int32_t> idx;
          std::vector<double> val;
          for (int64_t i = 0; i < m; ++i) {
            for (int f = 0; f < F; ++f)
              if (X[(r0 + i) * F + f] != 0.0) { idx.push_back(f); val.push_back(X[(r0 + i) * F + f]); }
            ip[i + 1] = static_cast<int64_t>(idx.size());
          }
          ds->PushCSR(ip.data(), idx.data(), val.data(), m, r0);
        }
      });
    }
    for (auto& t : th) t.join();
    if (mode != 1) CHECK(ds->bins == serial->bins);  // f32 rounding may move a bin edge: compare f64 pushes
    if (mode == 0) {
      ds->SetLabel(y.data(), static_cast<int64_t>(y.size()));
      Booster b(ds, params);
      for (int it = 0; it < 8; ++it) b.TrainOneIter();
      std::vector<double> ref_pred(n), par(n);
      b.Predict(X.data(), n, F, 0, 0, -1, ref_pred.data());
      std::vector<std::thread> pt;
      for (int t = 0; t < T; ++t) {
        pt.emplace_back([&, t]() {
          const int64_t r0 = static_cast<int64_t>(n) * t / T, r1 = static_cast<int64_t>(n) * (t + 1) / T;
          b.Predict(X.data() + r0 * F, r1 - r0, F, 0, 0, -1, par.data() + r0);
        });
      }
      for (auto& t : pt) t.join();
      for (int i = 0; i < n; ++i) CHECK(par[i] == ref_pred[i]);
    }
  }
  std::printf("ok  concurrent pushes (dense f64 / f32 / CSR) and predictions from %d threads\n", T);
}

int main() {
  concurrent_push_and_predict();
  malformed_models();
  run("objective=binary num_leaves=15 device_type=cpu", false);
  run("objective=binary num_leaves=15 device_type=cpu", true);
  run("objective=regression num_leaves=31 lambda_l2=1 device_type=cpu", false);
  run("objective=binary boosting=dart drop_rate=0.3 device_type=cpu", false);
  run("objective=binary boosting=goss device_type=cpu", false);
  run("objective=regression boosting=rf bagging_fraction=0.7 bagging_freq=1 device_type=cpu", false);
  run("objective=multiclass num_class=3 device_type=cpu", false);
  if (failures) {
    std::fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  std::printf("all native host tests passed\n");
  return 0;
}
