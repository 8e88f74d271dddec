// pybind11 module `synapseml_amd._vw`: VW-style learner + hashing + GPU SGD.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <array>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <thread>
#include <memory>
#include <stdexcept>

#include "vw_core.h"
#include "vw_gpu.h"

namespace py = pybind11;
using namespace smlvw;

namespace {
using F32 = py::array_t<float, py::array::c_style | py::array::forcecast>;
using I64 = py::array_t<int64_t, py::array::c_style | py::array::forcecast>;
using U32 = py::array_t<uint32_t, py::array::c_style | py::array::forcecast>;
using I32 = py::array_t<int32_t, py::array::c_style | py::array::forcecast>;

// One namespace block of a batch: CSR over examples.
struct Block {
  unsigned char ns;
  I64 indptr;
  U32 idx;
  F32 val;
};

std::vector<Block> ToBlocks(py::list blocks) {
  std::vector<Block> out;
  for (auto item : blocks) {
    py::tuple t = item.cast<py::tuple>();
    std::string ns = t[0].cast<std::string>();
    out.push_back(Block{static_cast<unsigned char>(ns.empty() ? ' ' : ns[0]), py::cast<I64>(t[1]), py::cast<U32>(t[2]),
                        py::cast<F32>(t[3])});
  }
  return out;
}

void FillExample(Example* ex, const std::vector<Block>& blocks, int64_t row) {
  ex->ns.clear();
  for (const auto& b : blocks) {
    const int64_t s = b.indptr.data()[row], e = b.indptr.data()[row + 1];
    if (e <= s) continue;
    Namespace& n = ex->Get(b.ns);
    for (int64_t p = s; p < e; ++p) n.f.push_back(Feature{b.val.data()[p], b.idx.data()[p]});
  }
}

// RCCL communicator of the device learner's weight averaging. A collective that failed or timed out (a peer
// died) aborts it: ncclCommAbort unblocks kernels of pending collectives, and the broken group is never
// destroyed collectively (ncclCommDestroy on it could wait for the dead peer).
struct NcclHandle {
  ncclComm_t c = nullptr;
  int world = 1;
  double timeout_ms = 0;
  bool aborted = false;
  void Abort() {
    if (c && !aborted) (void)ncclCommAbort(c);
    aborted = true;
    c = nullptr;
  }
  ~NcclHandle() { if (c && !aborted) ncclCommDestroy(c); }
};
}  // namespace

PYBIND11_MODULE(_vw, m) {
  m.doc() = "Vowpal Wabbit-style hashed online learning (C++ core + HIP hogwild SGD)";
  m.def("murmur3", [](py::bytes b, uint32_t seed) {
    std::string s = b;
    return Murmur3(s.data(), s.size(), seed);
  });
  m.def("hash_string", [](const std::string& s, uint32_t seed) { return HashString(s, seed); });
  m.def("murmur_batch", [](const std::vector<std::string>& strs, uint32_t seed, const std::string& prefix) {
    py::array_t<uint32_t> out(strs.size());
    auto o = out.mutable_data();
    for (size_t i = 0; i < strs.size(); ++i) {
      std::string s = prefix + strs[i];
      o[i] = Murmur3(s.data(), s.size(), seed);
    }
    return out;
  }, py::arg("strings"), py::arg("seed"), py::arg("prefix") = "");
  // packed UTF-8 strings (Arrow layout: bytes + n+1 offsets) -> murmur3 & mask; K13 on the GPU when asked
  m.def("murmur_offsets", [](py::array_t<uint8_t, py::array::c_style> bytes, py::array_t<int64_t, py::array::c_style> offs,
                             uint32_t seed, uint32_t mask, bool device) {
    const int64_t n = static_cast<int64_t>(offs.size()) - 1;
    if (n < 0) throw std::runtime_error("murmur_offsets: offsets must hold n + 1 entries");
    const int64_t* o = offs.data();
    const int64_t nb = static_cast<int64_t>(bytes.size());
    for (int64_t i = 0; i < n; ++i)
      if (o[i] < 0 || o[i] > o[i + 1] || o[i + 1] > nb) throw std::runtime_error("murmur_offsets: bad offsets");
    py::array_t<uint32_t> out(std::max<int64_t>(n, 0));
    uint32_t* r = out.mutable_data();
    const uint8_t* b = bytes.data();
    {
      py::gil_scoped_release rel;
      if (device) {
        MurmurBatchGpu(b, nb, o, n, seed, mask, r);
      } else {
#pragma omp parallel for schedule(static) if (n > 4096)
        for (int64_t i = 0; i < n; ++i) r[i] = Murmur3(b + o[i], static_cast<size_t>(o[i + 1] - o[i]), seed) & mask;
      }
    }
    return out;
  }, py::arg("bytes"), py::arg("offsets"), py::arg("seed"), py::arg("mask") = 0xFFFFFFFFu, py::arg("device") = false);
  // Text examples -> the GPU learner's columnar form (VowpalWabbitGeneric, deviceType="gpu"). Single-line:
  // {"blocks": [(ns, indptr, idx, val)] over rows, "labels", "weights", "multiclass", "cptr", "ccls", "ccost"}.
  // Multi-line (blank-line separated ADF groups, optional "shared" first line): {"shared": blocks over
  // examples, "actions": blocks over action rows, "aip", "chosen" (0-based, -1 none), "cost", "prob"}.
  m.def("parse_blocks", [](const std::string& args, const std::vector<std::string>& lines, bool multiline) {
    std::vector<Example> exs;
    {
      py::gil_scoped_release rel;
      exs = VW::ParseLines(args, lines);
    }
    auto to_blocks = [](const std::vector<const Example*>& rows) {
      // namespace char -> CSR over the rows (chars in first-appearance order)
      std::vector<unsigned char> order;
      std::array<int, 256> slot;
      slot.fill(-1);
      for (const Example* e : rows)
        for (const auto& ns : e->ns)
          if (slot[ns.ns] < 0) { slot[ns.ns] = static_cast<int>(order.size()); order.push_back(ns.ns); }
      const size_t n = rows.size();
      py::list out;
      for (unsigned char c : order) {
        std::vector<int64_t> ip(n + 1, 0);
        std::vector<uint32_t> idx;
        std::vector<float> val;
        for (size_t r = 0; r < n; ++r) {
          for (const auto& ns : rows[r]->ns)
            if (ns.ns == c)
              for (const auto& f : ns.f) { idx.push_back(static_cast<uint32_t>(f.idx)); val.push_back(f.x); }
          ip[r + 1] = static_cast<int64_t>(idx.size());
        }
        out.append(py::make_tuple(std::string(1, static_cast<char>(c)), py::array_t<int64_t>(ip.size(), ip.data()),
                                  py::array_t<uint32_t>(idx.size(), idx.data()), py::array_t<float>(val.size(), val.data())));
      }
      return out;
    };
    py::dict d;
    if (!multiline) {
      std::vector<const Example*> rows;
      std::vector<float> lab, w;
      std::vector<uint8_t> has;
      std::vector<int32_t> mc, ccls;
      std::vector<int64_t> cptr{0};
      std::vector<float> ccost, cact, ccst, cpdf;
      std::vector<uint8_t> chas;
      for (const auto& e : exs) {
        rows.push_back(&e);
        lab.push_back(e.l.label);
        w.push_back(e.l.weight);
        cact.push_back(e.l.cats_action);
        ccst.push_back(e.l.cats_cost);
        cpdf.push_back(e.l.cats_pdf);
        chas.push_back(e.l.cats_has ? 1 : 0);
        has.push_back(e.l.has_label || e.l.multiclass > 0 || !e.l.costs.empty() ? 1 : 0);
        mc.push_back(e.l.multiclass);
        for (const auto& c : e.l.costs) { ccls.push_back(c.first); ccost.push_back(c.second); }
        cptr.push_back(static_cast<int64_t>(ccls.size()));
      }
      d["blocks"] = to_blocks(rows);
      d["labels"] = py::array_t<float>(lab.size(), lab.data());
      d["weights"] = py::array_t<float>(w.size(), w.data());
      d["has_label"] = py::array_t<uint8_t>(has.size(), has.data());
      d["multiclass"] = py::array_t<int32_t>(mc.size(), mc.data());
      d["cptr"] = py::array_t<int64_t>(cptr.size(), cptr.data());
      d["ccls"] = py::array_t<int32_t>(ccls.size(), ccls.data());
      d["ccost"] = py::array_t<float>(ccost.size(), ccost.data());
      d["cats_action"] = py::array_t<float>(cact.size(), cact.data());
      d["cats_cost"] = py::array_t<float>(ccst.size(), ccst.data());
      d["cats_pdf"] = py::array_t<float>(cpdf.size(), cpdf.data());
      d["cats_has"] = py::array_t<uint8_t>(chas.size(), chas.data());
      return d;
    }
    std::vector<const Example*> shared, actions;
    std::vector<int64_t> aip{0};
    std::vector<int32_t> chosen;
    std::vector<float> cost, prob;
    Example empty;
    size_t i = 0;
    while (i < lines.size()) {
      // skip separators, then take one group
      while (i < lines.size() && lines[i].find_first_not_of(" \t\r\n") == std::string::npos) ++i;
      if (i >= lines.size()) break;
      const Example* sh = &empty;
      if (exs[i].l.cb_shared) { sh = &exs[i]; ++i; }
      int ch = -1, a = 0;
      float c = 0.f, p = 1.f;
      while (i < lines.size() && lines[i].find_first_not_of(" \t\r\n") != std::string::npos) {
        if (exs[i].l.cb_has) { ch = a; c = exs[i].l.cb_cost; p = exs[i].l.cb_prob; }
        actions.push_back(&exs[i]);
        ++a;
        ++i;
      }
      shared.push_back(sh);
      aip.push_back(static_cast<int64_t>(actions.size()));
      chosen.push_back(ch);
      cost.push_back(c);
      prob.push_back(p);
    }
    d["shared"] = to_blocks(shared);
    d["actions"] = to_blocks(actions);
    d["aip"] = py::array_t<int64_t>(aip.size(), aip.data());
    d["chosen"] = py::array_t<int32_t>(chosen.size(), chosen.data());
    d["cost"] = py::array_t<float>(cost.size(), cost.data());
    d["prob"] = py::array_t<float>(prob.size(), prob.data());
    return d;
  }, py::arg("args"), py::arg("lines"), py::arg("multiline") = false);
  m.def("gpu_available", &VwGpuAvailable);
  m.def("describe_args", &VW::DescribeArgs, "parse + validate a VW command line (no weight table)");

  py::class_<VW, std::shared_ptr<VW>>(m, "VW")
      .def(py::init([](const std::string& args, py::object model) {
             if (model.is_none()) return std::make_shared<VW>(args);
             std::string b = model.cast<py::bytes>();
             return std::make_shared<VW>(args, &b);
           }),
           py::arg("args"), py::arg("model") = py::none())
      .def("learn_batch",
           [](VW& vw, py::list blocks, F32 labels, py::object weights, py::object multiclass, py::object costs,
              bool learn) {
             auto bl = ToBlocks(blocks);
             const int64_t n = labels.size();
             py::array_t<float> preds(n);
             float* pr = preds.mutable_data();
             const float* w = weights.is_none() ? nullptr : py::cast<F32>(weights).data();
             I32 mc = multiclass.is_none() ? I32() : py::cast<I32>(multiclass);
             std::vector<std::vector<std::pair<int, float>>> cs;
             if (!costs.is_none()) cs = costs.cast<std::vector<std::vector<std::pair<int, float>>>>();
             std::vector<std::vector<float>> scores;
             Example ex;
             {
               for (int64_t i = 0; i < n; ++i) {
                 FillExample(&ex, bl, i);
                 ex.l = Label();
                 ex.l.label = labels.data()[i];
                 ex.l.has_label = true;
                 ex.l.weight = w ? w[i] : 1.f;
                 if (!multiclass.is_none()) ex.l.multiclass = mc.data()[i];
                 if (!cs.empty()) ex.l.costs = cs[i];
                 if (learn) vw.Learn(ex); else vw.Predict(ex);
                 pr[i] = ex.pred;
                 if (!ex.scores.empty()) scores.push_back(ex.scores);
               }
             }
             return py::make_tuple(preds, scores);
           },
           py::arg("blocks"), py::arg("labels"), py::arg("weights") = py::none(), py::arg("multiclass") = py::none(),
           py::arg("costs") = py::none(), py::arg("learn") = true)
      .def("learn_cb",
           [](VW& vw, py::list shared_blocks, py::list action_blocks, I64 action_indptr, I32 chosen, F32 cost, F32 prob,
              bool learn) {
             // shared_blocks: CSR over rows; action_blocks: CSR over all actions;
             // action_indptr: row -> [first action, last action)
             auto sb = ToBlocks(shared_blocks);
             auto ab = ToBlocks(action_blocks);
             const int64_t n = action_indptr.size() - 1;
             py::list out;
             for (int64_t i = 0; i < n; ++i) {
               std::vector<Example> exs;
               Example sh;
               FillExample(&sh, sb, i);
               sh.l.cb_shared = true;
               exs.push_back(std::move(sh));
               const int64_t a0 = action_indptr.data()[i], a1 = action_indptr.data()[i + 1];
               for (int64_t a = a0; a < a1; ++a) {
                 Example ax;
                 FillExample(&ax, ab, a);
                 if (chosen.data()[i] - 1 == a - a0) {
                   ax.l.cb_has = true;
                   ax.l.cb_action = chosen.data()[i];
                   ax.l.cb_cost = cost.data()[i];
                   ax.l.cb_prob = prob.data()[i];
                 }
                 exs.push_back(std::move(ax));
               }
               if (learn) vw.LearnMulti(exs); else vw.PredictMulti(exs);
               py::list probs;
               if (exs.size() > 1)
                 for (auto& ap : exs[1].action_probs) probs.append(py::make_tuple(ap.first, ap.second));
               out.append(probs);
             }
             return out;
           },
           py::arg("shared_blocks"), py::arg("action_blocks"), py::arg("action_indptr"), py::arg("chosen"),
           py::arg("cost"), py::arg("prob"), py::arg("learn") = true)
      .def("learn_text",
           [](VW& vw, const std::vector<std::string>& lines, bool learn) {
             py::array_t<float> preds(lines.size());
             float* pr = preds.mutable_data();
             for (size_t i = 0; i < lines.size(); ++i) {
               Example ex = vw.ParseLine(lines[i]);
               if (learn) vw.Learn(ex); else vw.Predict(ex);
               pr[i] = ex.pred;
             }
             return preds;
           },
           py::arg("lines"), py::arg("learn") = true)
      .def("learn_text_multi",
           [](VW& vw, const std::vector<std::string>& lines, bool learn) {
             std::vector<Example> exs;
             for (auto& l : lines) exs.push_back(vw.ParseLine(l));
             if (learn) vw.LearnMulti(exs); else vw.PredictMulti(exs);
             py::list probs;
             size_t head = (!exs.empty() && exs[0].l.cb_shared) ? 1 : 0;
             if (exs.size() > head)
               for (auto& ap : exs[head].action_probs) probs.append(py::make_tuple(ap.first, ap.second));
             return probs;
           },
           py::arg("lines"), py::arg("learn") = true)
      // one record per line in the shape of the learner's prediction type (VowpalWabbitPrediction.scala:18-101):
      // scalar (prediction, confidence) | scalars [..] | multiclass int | action_scores / action_probs
      // [(action, value)] | pdf [(left, right, pdf_value)] | action_pdf_value (action, pdf_value)
      .def("predict_text_structured",
           [](VW& vw, const std::vector<std::string>& lines, bool learn) {
             const std::string type = vw.OutputPredictionType();
             py::list out;
             for (const auto& line : lines) {
               Example ex = vw.ParseLine(line);
               if (learn) vw.Learn(ex); else vw.Predict(ex);
               if (type == "prediction_type_t::pdf") {
                 py::list segs;
                 for (auto& sg : ex.pdf_segments) segs.append(py::make_tuple(sg[0], sg[1], sg[2]));
                 out.append(segs);
               } else if (type == "prediction_type_t::action_pdf_value") {
                 out.append(py::make_tuple(ex.cats_action, ex.cats_pdf_value));
               } else if (type == "prediction_type_t::multiclass") {
                 out.append(static_cast<int>(ex.pred));
               } else if (type == "prediction_type_t::scalars") {
                 out.append(ex.scores);
               } else if (type == "prediction_type_t::action_probs" || type == "prediction_type_t::action_scores") {
                 py::list l;
                 for (auto& ap : ex.action_probs) l.append(py::make_tuple(ap.first, ap.second));
                 out.append(l);
               } else {
                 out.append(py::make_tuple(ex.pred, 0.f));
               }
             }
             return py::make_tuple(type, out);
           },
           py::arg("lines"), py::arg("learn") = false)
      .def("end_pass", &VW::EndPass)
      .def("perform_remaining_passes", &VW::PerformRemainingPasses)
      .def("save_model", [](const VW& vw) { return py::bytes(vw.SaveModel()); })
      .def("readable_model", &VW::ReadableModel)
      .def("output_prediction_type", &VW::OutputPredictionType)
      .def_property_readonly("args", &VW::args)
      .def_property_readonly("num_bits", &VW::num_bits)
      .def_property_readonly("hash_seed", &VW::HashSeed)
      .def("set_allreduce",
           [](VW& vw, int world, std::function<void(py::array_t<float>)> fn) {
             vw.world_size = world;
             vw.SetAllReduce([fn](float* buf, size_t n) {
               py::gil_scoped_acquire acq;
               py::array_t<float> a({static_cast<py::ssize_t>(n)}, {sizeof(float)}, buf, py::none());
               fn(a);
             });
           })
      .def("stats", [](const VW& vw) {
        const Stats& s = vw.stats();
        py::dict d;
        d["numberOfExamplesPerPass"] = s.examples;
        d["weightedExampleSum"] = s.weighted_examples;
        d["weightedLabelSum"] = s.weighted_labels;
        d["averageLoss"] = s.weighted_examples > 0 ? s.sum_loss / s.weighted_examples : 0.0;
        d["bestConstant"] = s.weighted_examples > 0 ? s.weighted_labels / s.weighted_examples : 0.0;
        d["totalNumberOfFeatures"] = s.total_features;
        d["passes"] = s.passes;
        d["ipsEstimate"] = s.examples > 0 ? s.cb_ips_num / s.examples : 0.0;
        d["snipsEstimate"] = s.cb_snips_den > 0 ? s.cb_ips_num / s.cb_snips_den : 0.0;
        return d;
      })
      .def("weights", [](VW& vw) {
        const uint64_t n = vw.NumWeights() / vw.stride();
        py::array_t<float> out(n);
        float* o = out.mutable_data();
        for (uint64_t i = 0; i < n; ++i) o[i] = vw.weights()[i * vw.stride()];
        return out;
      });
  // import a linear table trained elsewhere (the GPU learner) into w[0] of each slot
  m.def("import_linear", [](VW& vw, F32 w, double examples, double weighted_labels, double sum_loss, double min_label,
                            double max_label) {
    const uint64_t n = vw.NumWeights() / vw.stride();
    if (static_cast<uint64_t>(w.size()) != n) throw std::runtime_error("import_linear: size mismatch");
    float* dst = vw.weights();
    const float* src = w.data();
    for (uint64_t i = 0; i < n; ++i) dst[i * vw.stride()] = src[i];
    auto& st = vw.mutable_stats();
    st.examples += static_cast<int64_t>(examples);
    st.weighted_examples += examples;
    st.weighted_labels += weighted_labels;
    st.sum_loss += sum_loss;
    st.min_label = std::min(st.min_label, min_label);
    st.max_label = std::max(st.max_label, max_label);
  });
  m.def("merge_models", [](std::vector<std::shared_ptr<VW>> ms) {
    std::vector<const VW*> v;
    for (auto& p : ms) v.push_back(p.get());
    return std::shared_ptr<VW>(VW::Merge(v));
  });

  m.def("_stager_rejects_null", &StagerRejectsNull);
  m.def("_stager_unit_pieces", &StagerUnitPieces);
  py::class_<NcclHandle, std::shared_ptr<NcclHandle>>(m, "NcclComm")
      .def("abort", &NcclHandle::Abort)
      .def_property_readonly("aborted", [](const NcclHandle& h) { return h.aborted; });
  m.def("nccl_unique_id", []() {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) throw std::runtime_error("ncclGetUniqueId failed");
    return py::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
  });
  // Non-blocking communicator init bounded by timeout_ms: a peer that fails before (or inside) the collective
  // init cannot leave this rank blocked; on timeout / error the half-built communicator is aborted.
  m.def("nccl_comm", [](py::bytes uid, int rank, int world, double timeout_ms) {
    std::string s = uid;
    if (s.size() != sizeof(ncclUniqueId)) throw std::runtime_error("bad ncclUniqueId size");
    ncclUniqueId id;
    std::memcpy(&id, s.data(), sizeof(id));
    auto h = std::make_shared<NcclHandle>();
    {
      py::gil_scoped_release rel;
      ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
      cfg.blocking = 0;
      ncclResult_t r = ncclCommInitRankConfig(&h->c, world, id, rank, &cfg);
      const auto t0 = std::chrono::steady_clock::now();
      while (r == ncclInProgress) {
        if (ncclCommGetAsyncError(h->c, &r) != ncclSuccess) r = ncclInternalError;
        if (r != ncclInProgress) break;
        if (timeout_ms > 0 &&
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() > timeout_ms) {
          r = ncclInternalError;
          break;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(50));
      }
      if (r != ncclSuccess) {
        if (h->c) (void)ncclCommAbort(h->c);
        h->c = nullptr;
        throw std::runtime_error(std::string("RCCL communicator init failed or timed out: ") + ncclGetErrorString(r));
      }
    }
    h->world = world;
    h->timeout_ms = timeout_ms;
    return h;
  }, py::arg("uid"), py::arg("rank"), py::arg("world"), py::arg("timeout_ms") = 120000.0);

  py::class_<GpuSgdConfig>(m, "GpuSgdConfig")
      .def(py::init<>())
      .def_readwrite("bits", &GpuSgdConfig::bits)
      .def_readwrite("lr", &GpuSgdConfig::lr)
      .def_readwrite("power_t", &GpuSgdConfig::power_t)
      .def_readwrite("initial_t", &GpuSgdConfig::initial_t)
      .def_readwrite("l2", &GpuSgdConfig::l2)
      .def_readwrite("l1", &GpuSgdConfig::l1)
      .def_readwrite("tau", &GpuSgdConfig::tau)
      .def_readwrite("loss", &GpuSgdConfig::loss)
      .def_readwrite("adaptive", &GpuSgdConfig::adaptive)
      .def_readwrite("normalized", &GpuSgdConfig::normalized)
      .def_readwrite("invariant", &GpuSgdConfig::invariant)
      .def_readwrite("oaa", &GpuSgdConfig::oaa)
      .def_readwrite("csoaa", &GpuSgdConfig::csoaa)
      .def_readwrite("cb", &GpuSgdConfig::cb)
      .def_readwrite("cb_explore", &GpuSgdConfig::cb_explore)
      .def_readwrite("epsilon", &GpuSgdConfig::epsilon)
      .def_readwrite("cats", &GpuSgdConfig::cats)
      .def_readwrite("cats_min", &GpuSgdConfig::cats_min)
      .def_readwrite("cats_max", &GpuSgdConfig::cats_max)
      .def_readwrite("cats_bw", &GpuSgdConfig::cats_bw);
  py::class_<GpuSgd, std::shared_ptr<GpuSgd>>(m, "GpuSgd")
      .def(py::init([](const GpuSgdConfig& c, int dev) { return std::make_shared<GpuSgd>(c, dev); }),
           py::arg("config"), py::arg("device") = -1)
      .def("learn",
           [](GpuSgd& g, I64 indptr, U32 idx, F32 val, F32 labels, py::object weights, int batch) {
             const int64_t n = indptr.size() - 1;
             py::array_t<float> preds(n);
             const float* w = weights.is_none() ? nullptr : py::cast<F32>(weights).data();
             float* pr = preds.mutable_data();
             {
               py::gil_scoped_release rel;
               g.Learn(indptr.data(), idx.data(), val.data(), labels.data(), w, n, batch, pr);
             }
             return preds;
           },
           py::arg("indptr"), py::arg("indices"), py::arg("values"), py::arg("labels"), py::arg("weights") = py::none(),
           py::arg("batch") = 1024)
      .def("stage",
           [](GpuSgd& g, I64 indptr, U32 idx, F32 val, F32 labels, py::object weights) {
             const int64_t n = indptr.size() - 1;
             if (labels.size() != n) throw std::runtime_error("labels must have one entry per row");
             F32 w;
             if (!weights.is_none()) {
               w = py::cast<F32>(weights);
               if (w.size() != n) throw std::runtime_error("weights must have one entry per row");
             }
             py::gil_scoped_release rel;
             g.Stage(indptr.data(), idx.data(), val.data(), labels.data(), weights.is_none() ? nullptr : w.data(), n);
           },
           py::arg("indptr"), py::arg("indices"), py::arg("values"), py::arg("labels"), py::arg("weights") = py::none())
      // device featurization: blocks = [(group, level, indptr, indices, values)], interactions = [(a, b, c)]
      // (namespace group ids, c = -1 for pairs), row_map (n int64) for level-1 blocks
      .def("stage_plan",
           [](GpuSgd& g, py::list blocks, int ngroups, py::list inter, bool constant, py::object row_map, int64_t n,
              py::object labels, py::object weights, int64_t learn_r1, int batch) {
             FeatPlan plan;
             std::vector<I64> keep_i;
             std::vector<U32> keep_u;
             std::vector<F32> keep_f;
             for (auto item : blocks) {
               auto t = item.cast<py::tuple>();
               HostBlock b;
               b.group = t[0].cast<int>();
               b.level = t[1].cast<int>();
               keep_i.push_back(t[2].cast<I64>());
               keep_u.push_back(t[3].cast<U32>());
               keep_f.push_back(t[4].cast<F32>());
               b.ip = keep_i.back().data();
               b.rows = keep_i.back().size() - 1;
               b.idx = keep_u.back().data();
               b.val = keep_f.back().data();
               if (keep_u.back().size() < static_cast<size_t>(b.ip[b.rows]) || keep_f.back().size() < static_cast<size_t>(b.ip[b.rows]))
                 throw std::runtime_error("block indices / values shorter than indptr says");
               plan.blocks.push_back(b);
             }
             plan.ngroups = ngroups;
             for (auto item : inter) {
               auto t = item.cast<py::tuple>();
               plan.inter.push_back({t[0].cast<int>(), t[1].cast<int>(), t.size() > 2 ? t[2].cast<int>() : -1});
             }
             plan.constant = constant;
             I64 rm;
             if (!row_map.is_none()) {
               rm = row_map.cast<I64>();
               if (rm.size() != n) throw std::runtime_error("row_map must have one entry per row");
               plan.row_map = rm.data();
             }
             F32 lab, w;
             if (!labels.is_none()) {
               lab = labels.cast<F32>();
               if (lab.size() != n) throw std::runtime_error("labels must have one entry per row");
             }
             if (!weights.is_none()) {
               w = weights.cast<F32>();
               if (w.size() != n) throw std::runtime_error("weights must have one entry per row");
             }
             std::vector<float> zeros;
             if (labels.is_none()) zeros.assign(static_cast<size_t>(std::max<int64_t>(0, n)), 0.f);
             py::gil_scoped_release rel;
             g.StagePlan(plan, n, labels.is_none() ? zeros.data() : lab.data(), weights.is_none() ? nullptr : w.data(),
                         learn_r1, batch);
           },
           py::arg("blocks"), py::arg("ngroups"), py::arg("interactions"), py::arg("constant"), py::arg("row_map"),
           py::arg("n"), py::arg("labels") = py::none(), py::arg("weights") = py::none(), py::arg("learn_r1") = 0,
           py::arg("batch") = 1)
      .def("stage_costs",
           [](GpuSgd& g, I64 cptr, py::array_t<int32_t, py::array::c_style | py::array::forcecast> cls, F32 cost) {
             const int64_t n = cptr.size() - 1;
             if (cls.size() < cptr.data()[n] || cost.size() < cptr.data()[n]) throw std::runtime_error("cost lists too short");
             py::gil_scoped_release rel;
             g.StageCosts(cptr.data(), cls.data(), cost.data(), n);
           })
      .def("stage_cats",
           [](GpuSgd& g, F32 action, F32 cost, F32 pdf, py::array_t<uint8_t, py::array::c_style | py::array::forcecast> has) {
             const int64_t n = has.size();
             if (action.size() != n || cost.size() != n || pdf.size() != n)
               throw std::runtime_error("action / cost / pdf / has need one entry per row");
             py::gil_scoped_release rel;
             g.StageCats(action.data(), cost.data(), pdf.data(), has.data(), n);
           })
      .def("stage_cb",
           [](GpuSgd& g, I64 aip, py::array_t<int32_t, py::array::c_style | py::array::forcecast> chosen, F32 cost,
              F32 prob) {
             const int64_t ne = aip.size() - 1;
             if (chosen.size() != ne || cost.size() != ne || prob.size() != ne)
               throw std::runtime_error("chosen / cost / prob need one entry per example");
             py::gil_scoped_release rel;
             g.StageCb(aip.data(), chosen.data(), cost.data(), prob.data(), ne);
           })
      .def("predict_staged",
           [](GpuSgd& g) {
             py::array_t<float> out(g.staged_rows());
             py::array_t<float> best(g.staged_examples());
             float* o = out.mutable_data();
             float* b = best.mutable_data();
             {
               py::gil_scoped_release rel;
               g.PredictStaged(o, b);
             }
             return py::make_tuple(out, best);
           })
      .def_property_readonly("cb_stats", [](const GpuSgd& g) {
        double a, b, c;
        g.CbStats(&a, &b, &c);
        return py::make_tuple(a, b, c);
      })
      .def("learn_staged",
           [](GpuSgd& g, int64_t r0, int64_t r1, int batch) {
             py::array_t<float> preds(std::max<int64_t>(0, r1 - r0));
             float* pr = preds.mutable_data();
             {
               py::gil_scoped_release rel;
               g.LearnStaged(r0, r1, batch, pr);
             }
             return preds;
           },
           py::arg("r0"), py::arg("r1"), py::arg("batch") = 1024)
      .def("predict",
           [](GpuSgd& g, I64 indptr, U32 idx, F32 val) {
             const int64_t n = indptr.size() - 1;
             py::array_t<float> out(n);
             float* o = out.mutable_data();
             {
               py::gil_scoped_release rel;
               g.Predict(indptr.data(), idx.data(), val.data(), n, o);
             }
             return out;
           })
      .def("allreduce_average", [](GpuSgd& g, std::shared_ptr<NcclHandle> h) {
        if (h->aborted) throw std::runtime_error("VW RCCL communicator was aborted by an earlier failure");
        py::gil_scoped_release rel;
        try {
          g.AllReduceAverage(h->c, h->world, h->timeout_ms);
        } catch (...) {
          h->Abort();
          throw;
        }
      })
      // model bytes in the host learner's format (vw_core.cpp VW::SaveModel), built from the device nonzeros
      .def("export_model", [](GpuSgd& g, const std::string& args, bool final) {
        g.SetFinalExport(final);
        int64_t m = 0;
        double t, tw, snx;
        {
          py::gil_scoped_release rel;
          m = g.CountNonzeros();
          g.GlobalState(&t, &tw, &snx);
        }
        std::string s = "SMLVW001";
        auto put = [&s](const auto& v) { s.append(reinterpret_cast<const char*>(&v), sizeof(v)); };
        put(static_cast<uint32_t>(args.size()));
        s += args;
        int32_t bits = 0;
        while ((1ull << bits) < g.NumWeights()) ++bits;
        put(bits);
        put(static_cast<uint32_t>(4));
        put(t); put(tw); put(snx);
        put(g.min_label()); put(g.max_label());
        put(static_cast<uint64_t>(m));
        // the (index, value) records go from the device straight into the bytes object (a 2^30-slot model
        // can hold ~1e8 nonzeros: no host vectors, no second copy)
        PyObject* out = PyBytes_FromStringAndSize(nullptr, static_cast<Py_ssize_t>(s.size() + 12 * static_cast<size_t>(m)));
        if (!out) throw py::error_already_set();
        char* dst = PyBytes_AS_STRING(out);
        std::memcpy(dst, s.data(), s.size());
        try {
          py::gil_scoped_release rel;
          g.WriteRecords(dst + s.size());
        } catch (...) {
          Py_DECREF(out);
          throw;
        }
        return py::reinterpret_steal<py::bytes>(out);
      }, py::arg("args"), py::arg("final") = false,
         "final=True: the fit's last use - the table is cleared as it is exported (reused clean by the next learner)")
      // warm start from model bytes of either learner (same format)
      .def("import_model", [](GpuSgd& g, const std::string& bytes) {
        if (bytes.size() < 12 || bytes.compare(0, 8, "SMLVW001") != 0) throw std::runtime_error("not a VW model");
        const char* p = bytes.data() + 8;
        const char* end = bytes.data() + bytes.size();
        auto need = [&p, end](size_t k) {
          if (static_cast<size_t>(end - p) < k) throw std::runtime_error("truncated VW model");
        };
        auto get = [&p, &need](auto* v) { need(sizeof(*v)); std::memcpy(v, p, sizeof(*v)); p += sizeof(*v); };
        uint32_t alen; get(&alen); need(alen); p += alen;
        int32_t bits; uint32_t stride; get(&bits); get(&stride);
        if (stride != 4 || (1ull << bits) != g.NumWeights()) throw std::runtime_error("model table geometry differs");
        double t, tw, snx, lo, hi; get(&t); get(&tw); get(&snx); get(&lo); get(&hi);
        uint64_t nz; get(&nz);
        if (nz > static_cast<uint64_t>(end - p) / 12) throw std::runtime_error("truncated VW model");
        std::vector<uint64_t> idx(nz);
        std::vector<float> val(nz);
        for (uint64_t i = 0; i < nz; ++i) { get(&idx[i]); get(&val[i]); }
        py::gil_scoped_release rel;
        g.ImportNonzeros(idx, val);
        g.SetGlobalState(t, tw, snx);
        g.SetLabelRange(lo, hi);
      })
      .def_property_readonly("num_weights", &GpuSgd::NumWeights)
      .def_property_readonly("last_sync_bytes", &GpuSgd::last_sync_bytes)
      .def_property_readonly("last_sync_blocks", &GpuSgd::last_sync_blocks)
      .def_property_readonly("examples", &GpuSgd::examples)
      .def_property_readonly("sum_loss", &GpuSgd::sum_loss);
}
