// pybind11 module `synapseml_amd._gbdt`: Python surface of the native GBDT
// engine (dataset / booster / collectives). Replaces the reference's SWIG
// lightgbmlib bindings (lightgbm/.../swig/SwigUtils.scala) with zero-copy
// numpy buffers instead of per-element setItem calls (SURVEY §3.1 hot loop 1).
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <memory>
#include <stdexcept>
#include <type_traits>

#include "backend.h"
#include "booster.h"
#include "comm.h"
#include "dataset.h"
#include "predictor.h"

namespace py = pybind11;
using namespace sml;

namespace {

using F64 = py::array_t<double, py::array::c_style | py::array::forcecast>;
using F32 = py::array_t<float, py::array::c_style | py::array::forcecast>;
using I32 = py::array_t<int32_t, py::array::c_style | py::array::forcecast>;
using I64 = py::array_t<int64_t, py::array::c_style | py::array::forcecast>;

struct PyDataset {
  std::shared_ptr<Dataset> d;
};

struct PyComm {
  std::shared_ptr<Comm> c;
};

struct PyDeviceRows {
  py::object keep;                // the host rows; released only after the copy thread has joined
  std::shared_ptr<DeviceRows> r;  // destroyed first (members go in reverse order): joins the copy
};

}  // namespace

PYBIND11_MODULE(_gbdt, m) {
  m.doc() = "MI355X-native gradient boosting engine (HIP kernels + RCCL)";
  m.def("gpu_available", &GpuAvailable);
  // a failed / timed-out collective: fit() re-raises it on every rank (never "early termination")
  py::register_exception<CommError>(m, "CommError", PyExc_RuntimeError);

  py::class_<DatasetReference, std::shared_ptr<DatasetReference>>(m, "DatasetReference")
      .def_static("from_sample",
                  [](py::array sample, int64_t total_rows, const std::string& params, std::vector<std::string> names) {
                    Config cfg = Config::Parse(params);
                    // float32 samples are binned as they are (no float64 copy of the sample)
                    if (py::isinstance<py::array_t<float>>(sample) && (sample.flags() & py::array::c_style)) {
                      auto f = py::cast<py::array_t<float, py::array::c_style>>(sample);
                      if (f.ndim() != 2) throw std::runtime_error("sample must be 2-D");
                      const float* p = f.data();
                      const int64_t n = f.shape(0);
                      const int c = static_cast<int>(f.shape(1));
                      py::gil_scoped_release rel;
                      return std::make_shared<DatasetReference>(DatasetReference::FromSampleF32(p, n, c, total_rows, cfg, names));
                    }
                    auto d = py::cast<F64>(sample);
                    auto b = d.request();
                    if (b.ndim != 2) throw std::runtime_error("sample must be 2-D");
                    py::gil_scoped_release rel;
                    return std::make_shared<DatasetReference>(DatasetReference::FromSample(
                        static_cast<const double*>(b.ptr), b.shape[0], static_cast<int>(b.shape[1]), total_rows, cfg, names));
                  })
      .def_static("from_sampled_columns",
                  [](std::vector<std::vector<double>> cols, int64_t total, const std::string& params,
                     std::vector<std::string> names) {
                    Config cfg = Config::Parse(params);
                    return std::make_shared<DatasetReference>(DatasetReference::FromSampledColumns(cols, total, cfg, names));
                  })
      .def("serialize", [](const DatasetReference& r) { return py::bytes(r.Serialize()); })
      .def_static("deserialize", [](py::bytes b) { return std::make_shared<DatasetReference>(DatasetReference::Deserialize(b)); })
      .def_property_readonly("num_total_features", [](const DatasetReference& r) { return r.num_total_features; })
      .def_property_readonly("num_used_features", [](const DatasetReference& r) { return r.num_inner(); })
      .def_property_readonly("feature_names", [](const DatasetReference& r) { return r.feature_names; })
      .def("feature_infos", [](const DatasetReference& r) {
        std::vector<std::string> v;
        for (auto& mm : r.mappers) v.push_back(mm.FeatureInfo());
        return v;
      })
      .def("num_bins", [](const DatasetReference& r) {
        std::vector<int> v;
        for (auto& mm : r.mappers) v.push_back(mm.num_bin);
        return v;
      })
      .def("upper_bounds", [](const DatasetReference& r, int f) { return r.mappers.at(f).upper_bounds; })
      .def("value_to_bin", [](const DatasetReference& r, int f, double v) { return r.mappers.at(f).ValueToBin(v); });

  m.def("group_runs", [](I64 ids) {
    std::vector<int64_t> starts;
    bool grouped;
    {
      py::gil_scoped_release rel;
      grouped = GroupRuns(ids.data(), ids.size(), &starts);
    }
    return py::make_tuple(py::array_t<int64_t>(starts.size(), starts.data()), grouped);
  }, "first row of every run of equal ids, and whether each id forms one run");

  // K1 input staging: the raw rows go up on a native thread while Python samples / builds bin boundaries
  m.def("sample_dense_rows",
        [](py::array X, int64_t count, uint64_t seed) -> py::array {
          // `count` distinct rows of a dense C-contiguous float32 / float64 matrix, in row order, gathered
          // in parallel (bin-boundary sampling; LightGBM's bin_construct_sample_cnt)
          auto run = [&](auto tag) -> py::array {
            using T = decltype(tag);
            auto a = py::cast<py::array_t<T, py::array::c_style>>(X);
            if (a.ndim() != 2) throw std::runtime_error("X must be 2-D");
            const int64_t n = a.shape(0), c = a.shape(1);
            std::vector<int64_t> idx;
            {
              py::gil_scoped_release rel;
              idx = SampleRowIndices(n, count, seed);
            }
            py::array_t<T> out({static_cast<int64_t>(idx.size()), c});
            T* o = out.mutable_data();
            const T* src = a.data();
            {
              py::gil_scoped_release rel;
              const int64_t k = static_cast<int64_t>(idx.size());
#pragma omp parallel for schedule(static)
              for (int64_t i = 0; i < k; ++i) std::memcpy(o + i * c, src + idx[i] * c, sizeof(T) * c);
            }
            return out;
          };
          if (py::isinstance<py::array_t<float>>(X)) return run(float{});
          return run(double{});
        },
        py::arg("X"), py::arg("count"), py::arg("seed"));
  py::class_<PyDeviceRows>(m, "DeviceRows")
      .def(py::init([](py::array X, int device) {
             auto b = X.request();
             if (b.ndim != 2) throw std::runtime_error("rows must be 2-D");
             const bool f32 = b.format == py::format_descriptor<float>::format();
             PyDeviceRows p;
             p.keep = f32 ? py::array(py::cast<F32>(X)) : py::array(py::cast<F64>(X));  // C-contiguous, kept alive
             auto ab = p.keep.cast<py::array>().request();
             p.r = std::make_shared<DeviceRows>(ab.ptr, ab.shape[0], static_cast<int>(ab.shape[1]), f32 ? 4 : 8, device);
             return p;
           }),
           py::arg("X"), py::arg("device") = -1)
      .def("wait", [](PyDeviceRows& p) { py::gil_scoped_release rel; p.r->Wait(); })
      .def_property_readonly("num_rows", [](const PyDeviceRows& p) { return p.r->nrows; });
  py::class_<PyDataset>(m, "Dataset")
      .def(py::init([](std::shared_ptr<DatasetReference> ref, int64_t n) {
        PyDataset p;
        p.d = std::make_shared<Dataset>();
        p.d->Init(*ref, n);
        return p;
      }))
      .def("push_dense",
           [](PyDataset& p, py::array X, int64_t start) {
             auto b = X.request();
             if (b.ndim != 2) throw std::runtime_error("rows must be 2-D");
             if (start < 0 || start + b.shape[0] > p.d->num_data) throw std::runtime_error("push_dense out of range");
             if (b.format == py::format_descriptor<float>::format()) {
               F32 a = py::cast<F32>(X);
               py::gil_scoped_release rel;
               p.d->PushDenseF32(a.data(), a.shape(0), static_cast<int>(a.shape(1)), start);
             } else {
               F64 a = py::cast<F64>(X);
               py::gil_scoped_release rel;
               p.d->PushDense(a.data(), a.shape(0), static_cast<int>(a.shape(1)), start);
             }
           })
      .def("push_dense_gpu",
           [](PyDataset& p, py::array X, int64_t start, int device) {
             auto b = X.request();
             if (b.ndim != 2) throw std::runtime_error("rows must be 2-D");
             if (start < 0 || start + b.shape[0] > p.d->num_data) throw std::runtime_error("push_dense_gpu out of range");
             if (b.format == py::format_descriptor<float>::format()) {
               F32 a = py::cast<F32>(X);
               py::gil_scoped_release rel;
               DatasetPushDenseDeviceF32(p.d.get(), a.data(), a.shape(0), static_cast<int>(a.shape(1)), start, device);
             } else {
               F64 a = py::cast<F64>(X);
               py::gil_scoped_release rel;
               DatasetPushDenseDevice(p.d.get(), a.data(), a.shape(0), static_cast<int>(a.shape(1)), start, device);
             }
           },
           py::arg("X"), py::arg("start"), py::arg("device") = -1,
           "K1: encode dense rows into bins on the MI355X (bit-identical with push_dense)")
      .def("push_device_rows",
           [](PyDataset& p, PyDeviceRows& rows, int64_t start) {
             py::gil_scoped_release rel;
             DatasetPushDeviceRows(p.d.get(), rows.r.get(), start);
           },
           py::arg("rows"), py::arg("start") = 0,
           "K1 on rows already uploaded by DeviceRows (waits for the upload, encodes in HBM)")
      .def_property_readonly("bins", [](PyDataset& p) {
        p.d->EnsureHostBins();
        return py::array_t<uint8_t>({p.d->num_data, static_cast<int64_t>(p.d->row_stride)}, p.d->bins.data());
      })
      .def_property_readonly("device_resident", [](const PyDataset& p) { return p.d->dev && p.d->dev_valid; })
      .def("push_csr",
           [](PyDataset& p, I64 indptr, I32 indices, F64 values, int64_t start) {
             const int64_t nrows = indptr.shape(0) - 1;
             if (start < 0 || start + nrows > p.d->num_data) throw std::runtime_error("push_csr out of range");
             py::gil_scoped_release rel;
             p.d->PushCSR(indptr.data(), indices.data(), values.data(), nrows, start);
           })
      .def("set_label", [](PyDataset& p, F32 y) {
        if (y.size() != p.d->num_data) throw std::runtime_error("label size mismatch");
        py::gil_scoped_release rel;
        p.d->SetLabel(y.data(), y.size());
      })
      .def("set_weight", [](PyDataset& p, F32 w) {
        if (w.size() != p.d->num_data) throw std::runtime_error("weight size mismatch");
        p.d->weight.assign(w.data(), w.data() + w.size());
      })
      .def("set_init_score", [](PyDataset& p, F64 s) { p.d->init_score.assign(s.data(), s.data() + s.size()); })
      .def("set_group", [](PyDataset& p, I32 sizes) {
        std::vector<int32_t> v(sizes.data(), sizes.data() + sizes.size());
        p.d->SetQueryFromGroupSizes(v);
      })
      .def_property_readonly("num_data", [](const PyDataset& p) { return p.d->num_data; })
      .def_property_readonly("num_features", [](const PyDataset& p) { return p.d->ref.num_total_features; })
      .def("get_label", [](const PyDataset& p) {
        p.d->FinalizeLabel();
        return py::array_t<float>(p.d->label.size(), p.d->label.data());
      })
      .def("get_bins", [](const PyDataset& p) {
        p.d->EnsureHostBins();
        return py::array_t<uint8_t>({p.d->num_data, static_cast<int64_t>(p.d->row_stride)}, p.d->bins.data());
      });

  py::class_<PyComm>(m, "Comm")
      .def_property_readonly("rank", [](const PyComm& c) { return c.c->rank(); })
      .def_property_readonly("world", [](const PyComm& c) { return c.c->world(); })
      .def_property_readonly("is_device", [](const PyComm& c) { return c.c->is_device(); })
      .def_property_readonly("aborted", [](const PyComm& c) { return c.c->aborted(); })
      .def("abort", [](PyComm& c) { c.c->Abort(); })
      .def("allreduce_host", [](PyComm& c, py::array_t<double> a) {
        auto b = a.request();
        c.c->AllReduceHost(static_cast<double*>(b.ptr), b.size);
      })
      .def("allreduce_host_i64", [](PyComm& c, py::array_t<int64_t> a) {
        auto b = a.request();
        c.c->AllReduceHostI64(static_cast<int64_t*>(b.ptr), b.size);
      });
  // fn(array) sums a float64 or int64 host array in place over the ranks (the Python control plane)
  m.def("host_comm", [](int rank, int world, py::function fn) {
    PyComm c;
    auto call = [fn](auto* buf, int64_t n) {
      using T = std::remove_pointer_t<decltype(buf)>;
      py::gil_scoped_acquire acq;
      py::array_t<T> a({n}, {static_cast<py::ssize_t>(sizeof(T))}, buf, py::none());
      try {
        fn(a);
      } catch (py::error_already_set& e) {  // gloo / TCP failure of the host collective (peer died, timeout)
        throw CommError(std::string("host allreduce failed: ") + e.what());
      }
    };
    c.c = std::make_shared<HostComm>(rank, world, [call](double* buf, int64_t n) { call(buf, n); },
                                     [call](int64_t* buf, int64_t n) { call(buf, n); });
    return c;
  });
  m.def("p2p_comm", [](PyComm& base, int device, int64_t cap_bytes, double timeout_ms) {
    PyComm c;
    std::string why;
    {
      py::gil_scoped_release rel;  // the base host allreduce may call back into Python
      c.c = NewP2pComm(base.c, device, cap_bytes, timeout_ms, &why);
    }
    return py::make_tuple(c, why.empty(), why);
  }, py::arg("base"), py::arg("device"), py::arg("cap_bytes") = 1 << 20, py::arg("timeout_ms") = 60000.0);
  m.def("comm_device_allreduce", [](PyComm& c, std::vector<double> x, int reps) {
    py::gil_scoped_release rel;
    return CommDeviceAllReduce(c.c.get(), x, reps);
  }, py::arg("comm"), py::arg("x"), py::arg("reps") = 1);
  m.def("comm_device_allreduce_us", [](PyComm& c, int64_t n, int iters) {
    py::gil_scoped_release rel;
    return CommDeviceAllReduceUs(c.c.get(), n, iters);
  });
  m.def("rccl_unique_id", []() { return py::bytes(RcclGetUniqueId()); });
  m.def("rccl_comm", [](py::bytes uid, int rank, int world, int device, double timeout_ms) {
    PyComm c;
    std::string id(uid);
    py::gil_scoped_release rel;
    c.c.reset(NewRcclComm(id, rank, world, device, timeout_ms));
    return c;
  }, py::arg("uid"), py::arg("rank"), py::arg("world"), py::arg("device"), py::arg("timeout_ms") = 120000.0);

  py::class_<Booster, std::shared_ptr<Booster>>(m, "Booster")
      .def(py::init([](PyDataset& d, const std::string& params, py::object comm) {
             Comm* c = nullptr;
             std::shared_ptr<Comm> keep;
             if (!comm.is_none()) { keep = comm.cast<PyComm&>().c; c = keep.get(); }
             py::gil_scoped_release rel;
             auto b = std::make_shared<Booster>(d.d, params, c);
             return b;
           }),
           py::arg("train"), py::arg("params"), py::arg("comm") = py::none(), py::keep_alive<1, 4>())
      .def_static("from_model_string", [](const std::string& s) { return std::shared_ptr<Booster>(Booster::FromModelString(s)); })
      .def("add_valid", [](Booster& b, PyDataset& d, const std::string& name) { b.AddValidData(d.d, name); })
      // objective output transform (sigmoid / softmax / exp ...) of raw scores, n x num_model_per_iteration
      .def("convert_outputs", [](const Booster& b, F64 raw) {
        const int64_t n = raw.ndim() == 2 ? raw.shape(0) : raw.size();
        py::array_t<double> out(std::vector<py::ssize_t>(raw.shape(), raw.shape() + raw.ndim()));
        double* o = out.mutable_data();
        const double* r = raw.data();
        {
          py::gil_scoped_release rel;
          b.ConvertOutputs(r, n, o);
        }
        return out;
      })
      .def("merge", &Booster::MergeFrom)
      .def("reset_parameter", &Booster::ResetParameter)
      .def("update",
           [](Booster& b, py::object g, py::object h) {
             if (g.is_none()) { py::gil_scoped_release rel; return b.TrainOneIter(); }
             F32 ga = py::cast<F32>(g), ha = py::cast<F32>(h);
             py::gil_scoped_release rel;
             return b.TrainOneIter(ga.data(), ha.data());
           },
           py::arg("grad") = py::none(), py::arg("hess") = py::none())
      .def("rollback_one_iter", &Booster::RollbackOneIter)
      .def("eval", &Booster::Eval, py::arg("idx"), py::arg("device") = true,
           "metrics of data set idx (0 = train); device=False forces the host reference path")
      .def("eval_names", &Booster::EvalNames)
      .def("truncate", &Booster::Truncate)
      .def("synchronize", [](Booster& b) { py::gil_scoped_release rel; b.Synchronize(); })
      .def("train_scores", [](Booster& b) {
        std::vector<double> s;
        b.GetTrainScores(&s);
        return py::array_t<double>(s.size(), s.data());
      })
      .def("valid_on_device", [](const Booster& b, int i) { return b.ValidOnDevice(i); })
      .def("valid_scores", [](const Booster& b, int i) {
        std::vector<double> s;
        b.GetPredictForValid(i, &s);
        return py::array_t<double>(s.size(), s.data());
      })
      .def("save_model_string", &Booster::SaveModelToString, py::arg("start_iteration") = 0,
           py::arg("num_iteration") = -1, py::arg("importance_type") = 0)
      .def("dump_model", &Booster::DumpModel, py::arg("start_iteration") = 0, py::arg("num_iteration") = -1)
      .def("predict",
           [](const Booster& b, F64 X, int type, int start, int num) {
             if (X.ndim() != 2) throw std::runtime_error("X must be 2-D");
             const int64_t n = X.shape(0);
             const int osz = b.PredictOutputSize(type, start, num);
             py::array_t<double> out({n, static_cast<int64_t>(osz)});
             double* o = out.mutable_data();
             const double* x = X.data();
             const int nc = static_cast<int>(X.shape(1));
             {
               py::gil_scoped_release rel;
               b.Predict(x, n, nc, type, start, num, o);
             }
             return out;
           },
           py::arg("X"), py::arg("predict_type") = 0, py::arg("start_iteration") = 0, py::arg("num_iteration") = -1)
      .def("feature_importance", &Booster::FeatureImportance, py::arg("num_iteration") = -1, py::arg("importance_type") = 0)
      .def_property_readonly("num_classes", &Booster::NumClasses)
      .def_property_readonly("num_model_per_iteration", &Booster::NumModelPerIteration)
      .def_property_readonly("num_features", &Booster::NumFeatures)
      .def_property_readonly("num_total_model", &Booster::NumTotalModel)
      .def_property_readonly("current_iteration", &Booster::CurrentIteration)
      .def_property_readonly("feature_names", &Booster::FeatureNames)
      .def_property_readonly("backend", &Booster::BackendName)
      .def("release_training", [](Booster& b) {
        auto d = b.DetachTraining();  // the booster's own state changes under the GIL
        py::gil_scoped_release rel;
        d->Free();
      })
      .def_property_readonly("training_released", &Booster::training_released)
      .def("gradients", [](Booster& b) {
        std::vector<float> g, h;
        {
          py::gil_scoped_release rel;
          b.GetGradients(&g, &h);
        }
        return py::make_tuple(py::array_t<float>(g.size(), g.data()), py::array_t<float>(h.size(), h.data()));
      })
      .def("stats", [](Booster& b) {
        py::dict d;
        {
          py::gil_scoped_release rel;
          b.Synchronize();  // device timings of work still in flight
        }
        TrainStats* s = b.stats();
        if (s) {
          d["grad_ms"] = s->grad_ms; d["hist_ms"] = s->hist_ms; d["split_ms"] = s->split_ms;
          d["partition_ms"] = s->partition_ms; d["score_ms"] = s->score_ms; d["comm_ms"] = s->comm_ms; d["comm_calls"] = s->comm_calls;
          d["comm_dyn_calls"] = s->comm_dyn_calls; d["comm_bytes_max"] = s->comm_bytes_max;
          d["comm_dev_bytes"] = s->comm_dev_bytes;
          d["trees"] = s->trees;
          d["device_tree_ms"] = s->device_tree_ms; d["device_score_ms"] = s->device_score_ms;
          d["device_mem_mb"] = s->device_mem_mb;
        }
        return d;
      });

  py::class_<GpuPredictor, std::shared_ptr<GpuPredictor>>(m, "GpuPredictor")
      .def(py::init([](const Booster& b, int start, int num, int device) {
             return std::make_shared<GpuPredictor>(b, start, num, device);
           }),
           py::arg("booster"), py::arg("start_iteration") = 0, py::arg("num_iteration") = -1, py::arg("device") = -1,
           py::keep_alive<1, 2>())
      .def("predict",
           [](GpuPredictor& p, F64 X, bool normal) {
             const int64_t n = X.shape(0);
             py::array_t<double> out({n, static_cast<int64_t>(p.NumOutputs())});
             double* o = out.mutable_data();
             const double* x = X.data();
             const int nc = static_cast<int>(X.shape(1));
             {
               py::gil_scoped_release rel;
               p.Predict(x, n, nc, normal, o);
             }
             return out;
           },
           py::arg("X"), py::arg("normal") = false)
      // raw scores of a float32 or float64 row-major batch in ONE device pass (chunked pinned upload overlapped
      // with the traversal); no dtype conversion of the input on the host
      .def("predict_raw",
           [](GpuPredictor& p, py::array X) {
             if (X.ndim() != 2) throw std::runtime_error("predict_raw: X must be 2-D");
             const bool f32 = X.dtype().is(py::dtype::of<float>());
             py::array Xc = f32 ? py::array(py::array_t<float, py::array::c_style | py::array::forcecast>(X))
                                : py::array(py::array_t<double, py::array::c_style | py::array::forcecast>(X));
             const int64_t n = Xc.shape(0);
             const int nc = static_cast<int>(Xc.shape(1));
             py::array_t<double> out({n, static_cast<int64_t>(p.NumOutputs())});
             double* o = out.mutable_data();
             const void* x = Xc.data();
             {
               py::gil_scoped_release rel;
               p.PredictRaw(x, f32, n, nc, o);
             }
             return out;
           },
           py::arg("X"))
      .def("predict_contrib", [](GpuPredictor& p, const Booster& b, F64 X) -> py::object {
        const int64_t n = X.shape(0);
        py::array_t<double> out({n, static_cast<int64_t>((b.NumFeatures() + 1) * p.NumOutputs())});
        double* o = out.mutable_data();
        const double* x = X.data();
        const int nc = static_cast<int>(X.shape(1));
        bool ok;
        {
          py::gil_scoped_release rel;
          ok = p.PredictContrib(x, n, nc, o);
        }
        if (!ok) return py::none();
        return out;
      })
      .def("predict_leaf", [](GpuPredictor& p, F64 X) {
        const int64_t n = X.shape(0);
        py::array_t<int32_t> out({n, static_cast<int64_t>(p.NumTrees())});
        int32_t* o = out.mutable_data();
        const double* x = X.data();
        const int nc = static_cast<int>(X.shape(1));
        {
          py::gil_scoped_release rel;
          p.PredictLeaf(x, n, nc, o);
        }
        return out;
      });
}
