#include "vw_core.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cctype>
#include <cstring>
#include <sstream>
#include <stdexcept>

namespace smlvw {

// ----------------------------------------------------------------- hashing
static inline uint32_t Rotl32(uint32_t x, int8_t r) { return (x << r) | (x >> (32 - r)); }
static inline uint32_t Fmix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85ebca6b; h ^= h >> 13; h *= 0xc2b2ae35; h ^= h >> 16;
  return h;
}

uint32_t Murmur3(const void* key, size_t len, uint32_t seed) {
  const uint8_t* data = static_cast<const uint8_t*>(key);
  const size_t nblocks = len / 4;
  uint32_t h1 = seed;
  const uint32_t c1 = 0xcc9e2d51, c2 = 0x1b873593;
  for (size_t i = 0; i < nblocks; ++i) {
    uint32_t k1;
    std::memcpy(&k1, data + i * 4, 4);
    k1 *= c1; k1 = Rotl32(k1, 15); k1 *= c2;
    h1 ^= k1; h1 = Rotl32(h1, 13); h1 = h1 * 5 + 0xe6546b64;
  }
  const uint8_t* tail = data + nblocks * 4;
  uint32_t k1 = 0;
  switch (len & 3) {
    case 3: k1 ^= static_cast<uint32_t>(tail[2]) << 16; [[fallthrough]];
    case 2: k1 ^= static_cast<uint32_t>(tail[1]) << 8; [[fallthrough]];
    case 1: k1 ^= tail[0]; k1 *= c1; k1 = Rotl32(k1, 15); k1 *= c2; h1 ^= k1;
  }
  h1 ^= static_cast<uint32_t>(len);
  return Fmix32(h1);
}

uint32_t HashString(const std::string& s_in, uint32_t seed) {
  size_t b = 0, e = s_in.size();
  while (b < e && (s_in[b] == ' ' || s_in[b] == '\t')) ++b;
  while (e > b && (s_in[e - 1] == ' ' || s_in[e - 1] == '\t')) --e;
  uint64_t ret = 0;
  bool digits = e > b;
  for (size_t i = b; i < e; ++i) {
    char c = s_in[i];
    if (c >= '0' && c <= '9') ret = 10 * ret + static_cast<uint64_t>(c - '0');
    else { digits = false; break; }
  }
  if (digits) return static_cast<uint32_t>(ret + seed);
  return Murmur3(s_in.data() + b, e - b, seed);
}

uint32_t HashFeatureName(const std::string& s, uint32_t ns_hash) { return HashString(s, ns_hash); }

Namespace& Example::Get(unsigned char c) {
  for (auto& n : ns) if (n.ns == c) return n;
  ns.push_back(Namespace{c, {}});
  return ns.back();
}

// ----------------------------------------------------------------- args
namespace {
std::vector<std::string> Tokenize(const std::string& s) {
  std::vector<std::string> out;
  std::istringstream is(s);
  std::string t;
  while (is >> t) out.push_back(t);
  return out;
}
}  // namespace

void VW::ParseArgs(const std::string& args) {
  auto tok = Tokenize(args);
  bool any_update_flag = false, adaptive = false, normalized = false, invariant = false, sgd = false;
  for (size_t i = 0; i < tok.size(); ++i) {
    std::string k = tok[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= tok.size()) throw std::runtime_error("missing value for " + k);
      return tok[++i];
    };
    // "--key=value" form
    std::string inline_val;
    auto eq = k.find('=');
    bool has_inline = false;
    if (eq != std::string::npos && k.rfind("--", 0) == 0) { inline_val = k.substr(eq + 1); k = k.substr(0, eq); has_inline = true; }
    auto val = [&]() { return has_inline ? inline_val : next(); };
    // numeric values: the whole token must parse, and a bad one names its option
    auto ival = [&]() {
      const std::string v = val();
      try {
        size_t used = 0;
        const int x = std::stoi(v, &used);
        if (used == v.size()) return x;
      } catch (const std::exception&) {
      }
      throw std::runtime_error("VW option " + k + " expects an integer, got '" + v + "'");
    };
    auto fval = [&]() {
      const std::string v = val();
      try {
        size_t used = 0;
        const float x = std::stof(v, &used);
        if (used == v.size()) return x;
      } catch (const std::exception&) {
      }
      throw std::runtime_error("VW option " + k + " expects a number, got '" + v + "'");
    };
    if (k == "-b" || k == "--bit_precision") bits_ = ival();
    else if (k == "-l" || k == "--learning_rate") lr_ = fval();
    else if (k == "--power_t") power_t_ = fval();
    else if (k == "--initial_t") initial_t_ = fval();
    else if (k == "--l1") l1_ = fval();
    else if (k == "--l2") l2_ = fval();
    else if (k == "--hash_seed") hash_seed_ = static_cast<uint32_t>(std::stoul(val()));
    else if (k == "-q" || k == "--quadratic") interactions_.push_back(val());
    else if (k == "--cubic") interactions_.push_back(val());
    else if (k == "--interactions") interactions_.push_back(val());
    else if (k == "--ignore") { for (char c : val()) ignore_.push_back(static_cast<unsigned char>(c)); }
    else if (k == "--noconstant") constant_ = false;
    else if (k == "--loss_function") loss_ = val();
    else if (k == "--quantile_tau") quantile_tau_ = fval();
    else if (k == "--link") link_logistic_ = (val() == "logistic");
    else if (k == "--oaa") oaa_ = ival();
    else if (k == "--probabilities") probabilities_ = true;
    else if (k == "--csoaa") csoaa_ = ival();
    else if (k == "--cb_adf") cb_adf_ = true;
    else if (k == "--cb_explore_adf") { cb_adf_ = true; cb_explore_ = true; }
    else if (k == "--cb_type") cb_type_ = val();
    else if (k == "--epsilon") { epsilon_ = fval(); epsilon_set_ = true; }
    else if (k == "--passes") passes_ = ival();
    else if (k == "-t" || k == "--testonly") testonly_ = true;
    else if (k == "--holdout_off") holdout_off_ = true;
    else if (k == "--sgd") { sgd = true; any_update_flag = true; }
    else if (k == "--adaptive") { adaptive = true; any_update_flag = true; }
    else if (k == "--normalized") { normalized = true; any_update_flag = true; }
    else if (k == "--invariant") { invariant = true; any_update_flag = true; }
    else if (k == "--ngram") {
      // "--ngram N" (every namespace) or "--ngram aN" (namespace a only)
      const std::string v = has_inline ? inline_val : (i + 1 < tok.size() ? tok[i + 1] : std::string());
      if (!v.empty() && !std::isdigit(static_cast<unsigned char>(v[0]))) {
        val();
        int g = 0;
        try { size_t used = 0; g = std::stoi(v.substr(1), &used); if (used != v.size() - 1) g = 0; } catch (...) { g = 0; }
        if (g < 1) throw std::runtime_error("VW option --ngram expects N or <namespace>N, got '" + v + "'");
        ngram_ns_[static_cast<unsigned char>(v[0])] = g;
      } else {
        ngram_ = ival();
      }
    }
    else if (k == "--cats_pdf") { cats_k_ = ival(); cats_sample_ = false; }
    else if (k == "--cats") { cats_k_ = ival(); cats_sample_ = true; }
    else if (k == "--bandwidth") bandwidth_ = fval();
    else if (k == "--min_value") min_value_ = fval();
    else if (k == "--max_value") max_value_ = fval();
    else if (k == "--cache_file" || k == "--span_server" || k == "--span_server_port" || k == "--unique_id" ||
             k == "--total" || k == "--node" || k == "--random_seed" || k == "--readable_model" || k == "-f" ||
             k == "-i" || k == "--initial_regressor" || k == "--quantile_loss" || k == "--data" || k == "-d" ||
             k == "--final_regressor" || k == "--cb_force_legacy" || k == "--save_resume") {
      if (!has_inline && k != "--cb_force_legacy" && k != "--save_resume") next();
    } else if (k == "--quiet" || k == "--no_stdin" || k == "-k" || k == "--kill_cache" || k == "--audit" ||
               k == "--predict_only_model" || k == "--save_per_pass") {
      // front-end / IO flags without an effect on learning
    } else if (k == "--bfgs" || k == "--lda" || k == "--ksvm" || k == "--nn" || k == "--boosting" ||
               k == "--cb_explore" || k == "--cb" || k == "--ccb_explore_adf" || k == "--slates" || k == "--bootstrap" ||
               k == "--search" || k == "--lrq" || k == "--stage_poly" || k == "--active" || k == "--multilabel_oaa" ||
               k == "--ect" || k == "--log_multi" || k == "--recall_tree" || k == "--plt" || k == "--dsjson" ||
               k == "--json" || k == "--ftrl" || k == "--coin" || k == "--pistol" || k == "--OjaNewton" ||
               k == "--marginal" || k == "--explore_eval" || k == "--cbify" || k == "--warm_cb") {
      throw std::runtime_error("VW option " + k + " is not supported by this engine");
    } else {
      // a typo or an unknown reduction must not silently train a different model
      throw std::runtime_error("unrecognised VW option '" + tok[i] + "'");
    }
  }
  if (cats_k_ > 0) {
    if (cats_k_ < 2) throw std::runtime_error("--cats / --cats_pdf needs at least 2 discrete actions");
    if (!(max_value_ > min_value_)) throw std::runtime_error("CATS needs --min_value < --max_value");
    if (!(bandwidth_ > 0.f)) throw std::runtime_error("CATS needs --bandwidth > 0");
    cats_depth_ = 0;
    while ((1 << cats_depth_) < cats_k_) ++cats_depth_;
  }
  if (any_update_flag) {
    adaptive_ = adaptive; normalized_ = normalized; invariant_ = invariant;
    if (sgd) { adaptive_ = normalized_ = invariant_ = false; }
  }
  if (loss_ != "squared" && loss_ != "classic" && loss_ != "logistic" && loss_ != "hinge" && loss_ != "quantile")
    throw std::runtime_error("VW --loss_function " + loss_ + " is not supported (squared, classic, logistic, hinge, quantile)");
  if (bits_ < 1 || bits_ > 32) throw std::runtime_error("bit_precision must be in [1, 32]");
  mask_ = (bits_ >= 64) ? ~0ull : ((1ull << bits_) - 1);
  if (loss_ == "logistic") { stats_.min_label = -50; stats_.max_label = 50; }
}

std::map<std::string, std::string> VW::DescribeArgs(const std::string& args) {
  VW v;
  v.ParseArgs(args);
  std::map<std::string, std::string> d;
  auto f = [](double x) { std::ostringstream o; o.precision(9); o << x; return o.str(); };
  d["bits"] = std::to_string(v.bits_);
  d["learning_rate"] = f(v.lr_);
  d["power_t"] = f(v.power_t_);
  d["initial_t"] = f(v.initial_t_);
  d["l1"] = f(v.l1_);
  d["l2"] = f(v.l2_);
  d["loss_function"] = v.loss_;
  d["adaptive"] = v.adaptive_ ? "1" : "0";
  d["normalized"] = v.normalized_ ? "1" : "0";
  d["invariant"] = v.invariant_ ? "1" : "0";
  d["oaa"] = std::to_string(v.oaa_);
  d["csoaa"] = std::to_string(v.csoaa_);
  d["cb_adf"] = v.cb_adf_ ? "1" : "0";
  d["cats"] = std::to_string(v.cats_k_);
  d["min_value"] = f(v.min_value_);
  d["max_value"] = f(v.max_value_);
  d["bandwidth"] = f(v.bandwidth_);
  int ng = v.ngram_;
  for (int g : v.ngram_ns_) ng = std::max(ng, g);
  d["ngram"] = std::to_string(ng);
  d["ignore"] = std::string(v.ignore_.begin(), v.ignore_.end());
  d["link_logistic"] = v.link_logistic_ ? "1" : "0";
  d["probabilities"] = v.probabilities_ ? "1" : "0";
  d["constant"] = v.constant_ ? "1" : "0";
  d["hash_seed"] = std::to_string(v.hash_seed_);
  d["passes"] = std::to_string(v.passes_);
  d["cb_type"] = v.cb_type_;
  d["cb_explore"] = v.cb_explore_ ? "1" : "0";
  d["epsilon"] = f(v.epsilon_);
  d["loss_quantile_tau"] = f(v.quantile_tau_);
  std::string inter;
  for (const auto& q : v.interactions_) inter += (inter.empty() ? "" : ",") + q;
  d["interactions"] = inter;
  return d;
}

std::vector<Example> VW::ParseLines(const std::string& args, const std::vector<std::string>& lines) {
  VW v;
  v.ParseArgs(args);
  std::vector<Example> out;
  out.reserve(lines.size());
  for (const auto& l : lines) out.push_back(v.ParseLine(l));
  return out;
}

VW::VW(const std::string& args, const std::string* model_bytes) : args_str_(args) {
  ParseArgs(args);
  weights_.assign(static_cast<size_t>(mask_ + 1) * stride_, 0.f);
  if (model_bytes && !model_bytes->empty()) LoadModel(*model_bytes);
  caching_ = passes_ > 1;
}

VW::~VW() = default;

// ----------------------------------------------------------------- features
template <class F>
void VW::ForEachFeature(const Example& ex, F&& fn) const {
  auto ignored = [&](unsigned char c) { return std::find(ignore_.begin(), ignore_.end(), c) != ignore_.end(); };
  for (const auto& n : ex.ns) {
    if (ignored(n.ns)) continue;
    for (const auto& f : n.f) fn(f.idx, f.x);
  }
  // interactions (VW semantics): a ':' position is a wildcard over the namespaces present in the example
  // (constant namespace excluded), expanded to combinations with repetition - `-q ::` over {a,b,c} is aa ab
  // ac bb bc cc, each unordered namespace multiset once; adjacent positions naming the same namespace keep
  // only non-decreasing feature positions (no duplicate permutations of a self-interaction), as VW does
  // without --leave_duplicate_interactions. Hash: ((f1 * FNV) ^ f2) [* FNV ^ f3].
  if (interactions_.empty()) { if (constant_) fn(static_cast<uint64_t>(kConstantHash), 1.f); return; }
  const std::vector<Feature>* by_char[256] = {};
  unsigned char present[256];
  int npresent = 0;
  for (const auto& n : ex.ns) {
    if (n.ns == kConstantNamespace || ignored(n.ns) || n.f.empty()) continue;
    if (!by_char[n.ns]) present[npresent++] = n.ns;
    by_char[n.ns] = &n.f;
  }
  std::sort(present, present + npresent);
  auto pair = [&](unsigned char ca, unsigned char cb) {
    const auto* A = by_char[ca];
    const auto* B = by_char[cb];
    if (!A || !B) return;
    const bool same = ca == cb;
    for (size_t i = 0; i < A->size(); ++i) {
      const uint64_t h1 = (*A)[i].idx * kFnvPrime;
      const float x1 = (*A)[i].x;
      for (size_t j = same ? i : 0; j < B->size(); ++j) fn(h1 ^ (*B)[j].idx, x1 * (*B)[j].x);
    }
  };
  auto triple = [&](unsigned char c1, unsigned char c2, unsigned char c3) {
    const auto* A = by_char[c1];
    const auto* B = by_char[c2];
    const auto* C = by_char[c3];
    if (!A || !B || !C) return;
    const bool s12 = c1 == c2, s23 = c2 == c3;
    for (size_t i = 0; i < A->size(); ++i)
      for (size_t j = s12 ? i : 0; j < B->size(); ++j) {
        const uint64_t h12 = (((*A)[i].idx * kFnvPrime) ^ (*B)[j].idx) * kFnvPrime;
        const float x12 = (*A)[i].x * (*B)[j].x;
        for (size_t k = s23 ? j : 0; k < C->size(); ++k) fn(h12 ^ (*C)[k].idx, x12 * (*C)[k].x);
      }
  };
  for (const auto& inter : interactions_) {
    const size_t m = inter.size();
    if (m != 2 && m != 3) continue;
    bool wild = false;
    for (char c : inter) wild |= c == ':';
    if (!wild) {
      if (m == 2) pair(static_cast<unsigned char>(inter[0]), static_cast<unsigned char>(inter[1]));
      else triple(static_cast<unsigned char>(inter[0]), static_cast<unsigned char>(inter[1]),
                  static_cast<unsigned char>(inter[2]));
      continue;
    }
    // expand the wildcard positions over the present namespaces; keep each namespace multiset once (the
    // first expansion in sorted order, so `::` yields ab, never ba)
    std::vector<std::array<unsigned char, 3>> seen;
    std::array<int, 3> it{0, 0, 0};
    while (true) {
      std::array<unsigned char, 3> c{0, 0, 0};
      for (size_t q = 0; q < m; ++q)
        c[q] = inter[q] == ':' ? (npresent ? present[it[q]] : 0) : static_cast<unsigned char>(inter[q]);
      if (npresent) {
        std::array<unsigned char, 3> key = c;
        std::sort(key.begin(), key.begin() + m);
        if (std::find(seen.begin(), seen.end(), key) == seen.end()) {
          seen.push_back(key);
          if (m == 2) pair(c[0], c[1]); else triple(c[0], c[1], c[2]);
        }
      }
      // odometer over the wildcard positions (last position fastest)
      int q = static_cast<int>(m) - 1;
      for (; q >= 0; --q) {
        if (inter[q] != ':') continue;
        if (++it[q] < npresent) break;
        it[q] = 0;
      }
      if (q < 0 || !npresent) break;
    }
  }
  if (constant_) fn(static_cast<uint64_t>(kConstantHash), 1.f);
}

float VW::Dot(const Example& ex, uint64_t offset) const {
  float s = 0.f;
  ForEachFeature(ex, [&](uint64_t idx, float x) { s += weights_[((idx + offset) & mask_) * stride_] * x; });
  return s;
}

float VW::Loss(float p, float y) const {
  if (loss_ == "logistic") return std::log1p(std::exp(-y * p));
  if (loss_ == "hinge") return std::max(0.f, 1.f - y * p);
  if (loss_ == "quantile") { float e = y - p; return e > 0 ? quantile_tau_ * e : (quantile_tau_ - 1.f) * e; }
  return (p - y) * (p - y);
}

float VW::FirstDeriv(float p, float y) const {
  if (loss_ == "logistic") return -y / (1.f + std::exp(y * p));
  if (loss_ == "hinge") return (y * p < 1.f) ? -y : 0.f;
  if (loss_ == "quantile") return (y - p) > 0 ? -quantile_tau_ : (1.f - quantile_tau_);
  return 2.f * (p - y);
}

float VW::FinalizePred(float raw) const {
  float p = raw;
  if (std::isnan(p)) p = 0.f;
  p = std::min(std::max(p, static_cast<float>(stats_.min_label)), static_cast<float>(stats_.max_label));
  return p;
}

void VW::Update(const Example& ex, uint64_t offset, float pred, float label, float importance) {
  if (testonly_ || importance <= 0.f) return;
  // pass 1: adaptive / normalizer state and per-feature rate decay
  const float g = FirstDeriv(pred, label);
  const float grad_sq = g * g * importance;
  float pred_per_update = 0.f, norm_x = 0.f;
  spare_.clear();
  ForEachFeature(ex, [&](uint64_t idx, float x) {
    float* w = &weights_[((idx + offset) & mask_) * stride_];
    float x2 = x * x;
    if (x2 < FLT_MIN) { x2 = FLT_MIN; }
    if (adaptive_) w[1] += grad_sq * x2;
    if (normalized_) {
      const float ax = std::fabs(x);
      if (ax > w[2]) {
        if (w[2] > 0.f) { const float r = w[2] / ax; w[0] *= adaptive_ ? r : r * r; }
        w[2] = ax;
      }
      norm_x += x2 / (w[2] * w[2]);
    }
    float rate = 1.f;
    if (adaptive_) rate = w[1] > 0.f ? 1.f / std::sqrt(w[1]) : 0.f;
    if (normalized_) { const float inv = 1.f / w[2]; rate *= adaptive_ ? inv : inv * inv; }
    spare_.push_back(rate);
    pred_per_update += x2 * rate;
  });
  // global step size
  t_ += importance;
  total_weight_ += importance;
  sum_norm_x_ += importance * norm_x;
  double eta = lr_;
  if (normalized_ && sum_norm_x_ > 0) {
    // average feature-norm multiplier (sqrt under adaptive, as for the per-feature decay)
    const double avg_norm = total_weight_ / sum_norm_x_;
    eta *= adaptive_ ? std::sqrt(avg_norm) : avg_norm;
  }
  if (!adaptive_) eta *= std::pow(initial_t_ + t_, -static_cast<double>(power_t_));
  const float update_scale = static_cast<float>(eta) * importance;
  float update;
  if (invariant_) {
    // importance-aware ("safe") update of Karampatziakis & Langford
    const float ppu = std::max(pred_per_update, FLT_MIN);
    if (loss_ == "squared" || loss_ == "classic") {
      if (update_scale * ppu < 1e-6f) update = 2.f * (label - pred) * update_scale;
      else update = (label - pred) * (1.f - std::exp(-2.f * update_scale * ppu)) / ppu;
    } else if (loss_ == "logistic") {
      // first-order implicit step, bounded so the margin cannot overshoot
      const float step = label * update_scale / (1.f + std::exp(label * pred));
      update = std::abs(step * ppu) > 50.f ? std::copysign(50.f / ppu, step) : step;
    } else if (loss_ == "hinge") {
      // the step stops at the margin (VW's hingeloss::getUpdate)
      const float err = 1.f - label * pred;
      update = err <= 0.f ? 0.f : label * std::min(update_scale, err / ppu);
    } else {
      // quantile: the step stops at the label (VW's quantileloss::getUpdate)
      const float err = label - pred;
      update = err == 0.f ? 0.f
                          : (err > 0.f ? std::min(quantile_tau_ * update_scale, err / ppu)
                                       : std::max(-(1.f - quantile_tau_) * update_scale, err / ppu));
    }
  } else {
    update = -g * update_scale;
  }
  size_t k = 0;
  ForEachFeature(ex, [&](uint64_t idx, float x) {
    float* w = &weights_[((idx + offset) & mask_) * stride_];
    w[0] += update * x * spare_[k++];
    if (l2_ > 0.f) w[0] -= static_cast<float>(eta) * l2_ * w[0];
    if (l1_ > 0.f) {
      const float sh = static_cast<float>(eta) * l1_;
      w[0] = w[0] > sh ? w[0] - sh : (w[0] < -sh ? w[0] + sh : 0.f);
    }
  });
}

// ----------------------------------------------------------------- learners
// ----------------------------------------------------------------- CATS
int VW::CatsPredictLeaf(const Example& ex) const {
  int node = 0;
  const int leaves = 1 << cats_depth_;
  for (int d = 0; d < cats_depth_; ++d) {
    // right only when its subtree holds a real action (K need not be a power of two)
    const int right = 2 * node + 2;
    int first_leaf = right;
    while (first_leaf < leaves - 1) first_leaf = 2 * first_leaf + 1;
    const bool right_ok = first_leaf - (leaves - 1) < cats_k_;
    const float sc = Dot(ex, CatsNodeOffset(node));
    node = (sc > 0.f && right_ok) ? right : 2 * node + 1;
  }
  return node - (leaves - 1);
}

void VW::CatsSegments(int leaf, Example* ex) const {
  const float range = max_value_ - min_value_;
  const float unit = range / cats_k_;
  const float c = min_value_ + (leaf + 0.5f) * unit;
  const float lo = std::max(min_value_, c - bandwidth_), hi = std::min(max_value_, c + bandwidth_);
  const float eps = epsilon_set_ ? epsilon_ : 0.05f;
  const float base = eps / range;
  ex->pdf_segments.clear();
  if (lo > min_value_) ex->pdf_segments.push_back({min_value_, lo, base});
  ex->pdf_segments.push_back({lo, hi, (1.f - eps) / (hi - lo) + base});
  if (hi < max_value_) ex->pdf_segments.push_back({hi, max_value_, base});
  if (cats_sample_) {
    // deterministic draw (per-model counter): the window w.p. 1 - eps, else uniform over the range
    uint64_t z = (cats_draws_ + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    const double u1 = static_cast<double>(z >> 11) * (1.0 / 9007199254740992.0);
    const double u2 = static_cast<double>((z * 0x2545F4914F6CDD1Dull) >> 11) * (1.0 / 9007199254740992.0);
    const float a = u1 < 1.0 - eps ? static_cast<float>(lo + u2 * (hi - lo)) : static_cast<float>(min_value_ + u2 * range);
    ex->cats_action = a;
    ex->cats_pdf_value = (a >= lo && a <= hi) ? (1.f - eps) / (hi - lo) + base : base;
  }
}

void VW::CatsLearn(Example& ex) {
  stats_.examples += 1;
  stats_.weighted_examples += 1;
  const int leaf = CatsPredictLeaf(ex);
  CatsSegments(leaf, &ex);
  if (cats_sample_) ++cats_draws_;
  ex.pred = cats_sample_ ? ex.cats_action : min_value_ + (leaf + 0.5f) * (max_value_ - min_value_) / cats_k_;
  if (!ex.l.cats_has || testonly_) return;
  stats_.sum_loss += ex.l.cats_cost;
  // IPS estimate of each discrete action's smoothed cost with a control variate: a running mean cost b
  // (this example included) stands in for an unobserved action, a covered one gets
  // b + (c - b) / (|window_k| * p). Unbiased for every action, and a single cost carries signal (cheaper
  // than usual pulls the policy towards the windows that covered it, dearer pushes it away).
  cats_cost_sum_ += ex.l.cats_cost;
  cats_cost_n_ += 1.0;
  const float b = static_cast<float>(cats_cost_sum_ / cats_cost_n_);
  const int leaves = 1 << cats_depth_;
  const float unit = (max_value_ - min_value_) / cats_k_;
  const float p = std::max(ex.l.cats_pdf, 1e-12f);
  std::vector<float> win(2 * leaves - 1, b);
  std::vector<char> valid(2 * leaves - 1, 0);
  for (int k = 0; k < cats_k_; ++k) {
    const float c = min_value_ + (k + 0.5f) * unit;
    const float lo = std::max(min_value_, c - bandwidth_), hi = std::min(max_value_, c + bandwidth_);
    valid[leaves - 1 + k] = 1;
    if (ex.l.cats_action >= lo && ex.l.cats_action <= hi) win[leaves - 1 + k] = b + (ex.l.cats_cost - b) / ((hi - lo) * p);
  }
  // filter-tree update, bottom up: each node learns which child's tournament winner (the leaf its current
  // routing reaches) has the lower estimate, weighted by the difference
  for (int node = leaves - 2; node >= 0; --node) {
    const int l = 2 * node + 1, r = 2 * node + 2;
    valid[node] = valid[l] || valid[r];
    if (!valid[l] || !valid[r]) {
      win[node] = valid[l] ? win[l] : win[r];
      continue;
    }
    const float sc = Dot(ex, CatsNodeOffset(node));
    const float imp = std::fabs(win[l] - win[r]);
    if (imp > 0.f) Update(ex, CatsNodeOffset(node), sc, win[r] < win[l] ? 1.f : -1.f, imp);
    win[node] = sc > 0.f ? win[r] : win[l];
  }
}

void VW::Predict(Example& ex) {
  if (cats_k_ > 0) {
    const int leaf = CatsPredictLeaf(ex);
    CatsSegments(leaf, &ex);
    if (cats_sample_) ++cats_draws_;
    ex.pred = cats_sample_ ? ex.cats_action : min_value_ + (leaf + 0.5f) * (max_value_ - min_value_) / cats_k_;
    return;
  }
  if (oaa_ > 0 || csoaa_ > 0) {
    const int K = oaa_ > 0 ? oaa_ : csoaa_;
    ex.scores.assign(K, 0.f);
    for (int k = 0; k < K; ++k) ex.scores[k] = Dot(ex, static_cast<uint64_t>(k) * 1315423911ull);
    if (oaa_ > 0) {
      int best = static_cast<int>(std::max_element(ex.scores.begin(), ex.scores.end()) - ex.scores.begin());
      if (probabilities_) {
        double s = 0;
        for (auto& v : ex.scores) { v = 1.f / (1.f + std::exp(-v)); s += v; }
        for (auto& v : ex.scores) v = static_cast<float>(v / s);
      }
      ex.pred = static_cast<float>(best + 1);
    } else {
      int best = static_cast<int>(std::min_element(ex.scores.begin(), ex.scores.end()) - ex.scores.begin());
      ex.pred = static_cast<float>(best + 1);
    }
    return;
  }
  const float raw = Dot(ex, 0);
  float p = FinalizePred(raw);
  if (link_logistic_) p = 1.f / (1.f + std::exp(-p));
  ex.pred = p;
}

void VW::Learn(Example& ex) {
  if (caching_ && stats_.passes == 0) cache_.push_back(ex);
  if (cats_k_ > 0) { CatsLearn(ex); return; }
  const float w = ex.l.weight;
  stats_.examples += 1;
  stats_.weighted_examples += w;
  if (oaa_ > 0) {
    Predict(ex);
    const int K = oaa_;
    const int y = ex.l.multiclass;
    float loss = 0;
    for (int k = 0; k < K; ++k) {
      const uint64_t off = static_cast<uint64_t>(k) * 1315423911ull;
      const float raw = Dot(ex, off);
      const float lab = (k + 1 == y) ? 1.f : -1.f;
      loss += Loss(raw, lab);
      Update(ex, off, raw, lab, w);
    }
    ex.loss = (static_cast<int>(ex.pred) == y) ? 0.f : 1.f;
    stats_.sum_loss += ex.loss * w;
    (void)loss;
    return;
  }
  if (csoaa_ > 0) {
    Predict(ex);
    for (const auto& c : ex.l.costs) {
      const int k = c.first - 1;
      if (k < 0 || k >= csoaa_) continue;
      const uint64_t off = static_cast<uint64_t>(k) * 1315423911ull;
      const float raw = Dot(ex, off);
      Update(ex, off, raw, c.second, w);
    }
    float chosen_cost = 0;
    for (const auto& c : ex.l.costs) if (c.first == static_cast<int>(ex.pred)) chosen_cost = c.second;
    ex.loss = chosen_cost;
    stats_.sum_loss += chosen_cost * w;
    return;
  }
  const float y = ex.l.label;
  if (ex.l.has_label && loss_ != "logistic") {
    // like VW's shared_data: the prediction range starts at [0, 0] and grows
    stats_.min_label = std::min<double>(stats_.min_label, y);
    stats_.max_label = std::max<double>(stats_.max_label, y);
  }
  const float raw = Dot(ex, 0);
  const float pred = FinalizePred(raw);
  ex.pred = link_logistic_ ? 1.f / (1.f + std::exp(-pred)) : pred;
  if (!ex.l.has_label) return;
  stats_.weighted_labels += y * w;
  ex.loss = Loss(pred, y);
  stats_.sum_loss += ex.loss * w;
  Update(ex, 0, raw, y, w);
}

void VW::CbLearn(std::vector<Example>& exs, bool learn) {
  // exs: optional shared example (cb_shared) followed by one example per action
  size_t first = 0;
  const Example* shared = nullptr;
  if (!exs.empty() && exs[0].l.cb_shared) { shared = &exs[0]; first = 1; }
  const int A = static_cast<int>(exs.size() - first);
  if (A <= 0) return;
  auto merged = [&](const Example& a) {
    Example m = a;
    if (shared) for (const auto& n : shared->ns) { auto& dst = m.Get(n.ns); dst.f.insert(dst.f.end(), n.f.begin(), n.f.end()); }
    return m;
  };
  std::vector<Example> acts;
  acts.reserve(A);
  for (int a = 0; a < A; ++a) acts.push_back(merged(exs[first + a]));
  std::vector<float> scores(A);
  for (int a = 0; a < A; ++a) scores[a] = Dot(acts[a], 0);
  int best = static_cast<int>(std::min_element(scores.begin(), scores.end()) - scores.begin());
  // exploration distribution (epsilon greedy), chosen action first
  std::vector<std::pair<int, float>> probs;
  if (cb_explore_) {
    const float e = epsilon_ / A;
    probs.emplace_back(best, 1.f - epsilon_ + e);
    for (int a = 0; a < A; ++a) if (a != best) probs.emplace_back(a, e);
  } else {
    std::vector<int> order(A);
    for (int a = 0; a < A; ++a) order[a] = a;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return scores[x] < scores[y]; });
    for (int a : order) probs.emplace_back(a, scores[a]);
  }
  Example& head = exs[first];
  head.action_probs = probs;
  head.scores = scores;
  // logged label
  int logged = -1;
  float cost = 0, prob = 1;
  for (int a = 0; a < A; ++a)
    if (exs[first + a].l.cb_has) { logged = a; cost = exs[first + a].l.cb_cost; prob = std::max(exs[first + a].l.cb_prob, 1e-6f); }
  stats_.examples += 1;
  stats_.weighted_examples += 1;
  if (logged >= 0) {
    float p_pred = 0;
    for (auto& pp : probs) if (pp.first == logged) p_pred = cb_explore_ ? pp.second : (pp.first == best ? 1.f : 0.f);
    stats_.cb_ips_num += cost * p_pred / prob;
    stats_.cb_snips_den += p_pred / prob;
    stats_.sum_loss += cost * p_pred / prob;
  }
  if (!learn || logged < 0) return;
  if (cb_type_ == "mtr") {
    Update(acts[logged], 0, scores[logged], cost, 1.f / prob);
  } else if (cb_type_ == "dr") {
    for (int a = 0; a < A; ++a) {
      const float lab = scores[a] + (a == logged ? (cost - scores[a]) / prob : 0.f);
      Update(acts[a], 0, scores[a], lab, 1.f);
    }
  } else {  // ips
    for (int a = 0; a < A; ++a) Update(acts[a], 0, scores[a], a == logged ? cost / prob : 0.f, 1.f);
  }
}

void VW::LearnMulti(std::vector<Example>& exs) {
  if (caching_ && stats_.passes == 0) cache_multi_.push_back(exs);
  if (cb_adf_) { CbLearn(exs, true); return; }
  for (auto& e : exs) Learn(e);
}

void VW::PredictMulti(std::vector<Example>& exs) {
  if (cb_adf_) {
    const bool tl = testonly_;
    testonly_ = true;
    Stats keep = stats_;
    CbLearn(exs, false);
    stats_ = keep;
    testonly_ = tl;
    return;
  }
  for (auto& e : exs) Predict(e);
}

std::string VW::OutputPredictionType() const {
  if (cats_k_ > 0) return cats_sample_ ? "prediction_type_t::action_pdf_value" : "prediction_type_t::pdf";
  if (cb_explore_) return "prediction_type_t::action_probs";
  if (cb_adf_) return "prediction_type_t::action_scores";
  if (oaa_ > 0 && probabilities_) return "prediction_type_t::scalars";
  if (oaa_ > 0 || csoaa_ > 0) return "prediction_type_t::multiclass";
  return "prediction_type_t::scalar";
}

// ----------------------------------------------------------------- text format
Example VW::ParseLine(const std::string& line) const {
  Example ex;
  auto bar = line.find('|');
  std::string head = bar == std::string::npos ? line : line.substr(0, bar);
  std::istringstream hs(head);
  std::vector<std::string> ht;
  std::string t;
  while (hs >> t) ht.push_back(t);
  if (!ht.empty()) {
    if (ht[0] == "shared") {
      ex.l.cb_shared = true;
    } else if (ht[0] == "ca") {
      // CATS: "ca action:cost:pdf_value"
      if (ht.size() > 1) {
        const std::string& v = ht[1];
        auto c1 = v.find(':'), c2 = c1 == std::string::npos ? std::string::npos : v.find(':', c1 + 1);
        if (c1 == std::string::npos || c2 == std::string::npos)
          throw std::runtime_error("CATS label must be 'ca action:cost:pdf_value', got '" + v + "'");
        ex.l.cats_has = true;
        ex.l.cats_action = std::stof(v.substr(0, c1));
        ex.l.cats_cost = std::stof(v.substr(c1 + 1, c2 - c1 - 1));
        ex.l.cats_pdf = std::stof(v.substr(c2 + 1));
      }
    } else if (cb_adf_ && ht[0].find(':') != std::string::npos) {
      // action:cost:probability
      std::string s = ht[0];
      auto c1 = s.find(':'), c2 = s.find(':', c1 + 1);
      ex.l.cb_has = true;
      ex.l.cb_action = std::stoi(s.substr(0, c1));
      ex.l.cb_cost = std::stof(s.substr(c1 + 1, c2 - c1 - 1));
      ex.l.cb_prob = c2 == std::string::npos ? 1.f : std::stof(s.substr(c2 + 1));
    } else if (csoaa_ > 0) {
      for (const auto& c : ht) {
        auto colon = c.find(':');
        if (colon == std::string::npos) continue;
        ex.l.costs.emplace_back(std::stoi(c.substr(0, colon)), std::stof(c.substr(colon + 1)));
      }
    } else {
      try {
        float v = std::stof(ht[0]);
        ex.l.label = v;
        ex.l.has_label = true;
        ex.l.multiclass = static_cast<int>(v);
        if (ht.size() > 1 && ht[1][0] != '\'') ex.l.weight = std::stof(ht[1]);
      } catch (...) {
      }
      for (const auto& x : ht) if (!x.empty() && x[0] == '\'') ex.tag = x.substr(1);
    }
  }
  // namespaces
  size_t pos = bar;
  while (pos != std::string::npos) {
    size_t nxt = line.find('|', pos + 1);
    std::string seg = line.substr(pos + 1, nxt == std::string::npos ? std::string::npos : nxt - pos - 1);
    pos = nxt;
    std::istringstream ss(seg);
    std::string first;
    unsigned char ns_char = ' ';
    uint32_t ns_hash = hash_seed_;
    float ns_scale = 1.f;
    std::vector<std::string> toks;
    if (!seg.empty() && seg[0] != ' ' && seg[0] != '\t') {
      ss >> first;
      auto colon = first.find(':');
      std::string name = colon == std::string::npos ? first : first.substr(0, colon);
      if (colon != std::string::npos) ns_scale = std::stof(first.substr(colon + 1));
      ns_char = static_cast<unsigned char>(name[0]);
      ns_hash = HashString(name, hash_seed_);
    }
    while (ss >> t) toks.push_back(t);
    Namespace& n = ex.Get(ns_char);
    std::vector<std::pair<std::string, float>> words;
    for (const auto& w : toks) {
      auto colon = w.rfind(':');
      float v = 1.f;
      std::string name = w;
      if (colon != std::string::npos && colon > 0) {
        try { v = std::stof(w.substr(colon + 1)); name = w.substr(0, colon); } catch (...) { name = w; }
      }
      words.emplace_back(name, v * ns_scale);
      n.f.push_back(Feature{v * ns_scale, HashString(name, ns_hash)});
    }
    const int ngram = ngram_ns_[ns_char] ? ngram_ns_[ns_char] : ngram_;
    for (int g = 2; g <= ngram; ++g) {
      for (size_t i = 0; i + g <= words.size(); ++i) {
        std::string nm = words[i].first;
        for (int j = 1; j < g; ++j) nm += "^" + words[i + j].first;
        n.f.push_back(Feature{1.f * ns_scale, HashString(nm, ns_hash)});
      }
    }
  }
  return ex;
}

// ----------------------------------------------------------------- passes / sync
void VW::EndPass() {
  if (allreduce_ && world_size > 1) {
    allreduce_(weights_.data(), weights_.size());
    const float inv = 1.f / world_size;
    for (auto& w : weights_) w *= inv;
  }
  stats_.passes += 1;
}

void VW::PerformRemainingPasses() {
  caching_ = false;
  for (int p = 1; p < passes_; ++p) {
    EndPass();
    for (auto& e : cache_) { Example c = e; Learn(c); }
    for (auto& m : cache_multi_) { auto c = m; LearnMulti(c); }
  }
  if (passes_ > 1) EndPass();
}

// ----------------------------------------------------------------- model io
namespace {
template <class T> void Put(std::string* s, const T& v) { s->append(reinterpret_cast<const char*>(&v), sizeof(T)); }
// bounds-checked reader over model bytes: a truncated or corrupted model throws instead of reading past the end
struct Reader {
  const char* p;
  const char* end;
  void Need(size_t k) const {
    if (static_cast<size_t>(end - p) < k) throw std::runtime_error("truncated VW model");
  }
  template <class T> T Get() {
    Need(sizeof(T));
    T v;
    std::memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
};
}  // namespace

std::string VW::SaveModel() const {
  std::string s = "SMLVW001";
  Put(&s, static_cast<uint32_t>(args_str_.size()));
  s += args_str_;
  Put(&s, static_cast<int32_t>(bits_));
  Put(&s, stride_);
  Put(&s, t_); Put(&s, total_weight_); Put(&s, sum_norm_x_);
  Put(&s, stats_.min_label); Put(&s, stats_.max_label);
  uint64_t nz = 0;
  for (float w : weights_) if (w != 0.f) ++nz;
  Put(&s, nz);
  for (uint64_t i = 0; i < weights_.size(); ++i)
    if (weights_[i] != 0.f) { Put(&s, i); Put(&s, weights_[i]); }
  return s;
}

void VW::LoadModel(const std::string& bytes) {
  if (bytes.size() < 8 || bytes.compare(0, 8, "SMLVW001") != 0) throw std::runtime_error("not a VW model of this engine");
  Reader r{bytes.data() + 8, bytes.data() + bytes.size()};
  const uint32_t alen = r.Get<uint32_t>();
  r.Need(alen);
  r.p += alen;
  const int32_t bits = r.Get<int32_t>();
  const uint32_t stride = r.Get<uint32_t>();
  if (bits < 1 || bits > 32 || stride < 1 || stride > 64) throw std::runtime_error("corrupt VW model header");
  const double t = r.Get<double>(), tw = r.Get<double>(), snx = r.Get<double>();
  const double lo = r.Get<double>(), hi = r.Get<double>();
  const uint64_t nz = r.Get<uint64_t>();
  if (nz > static_cast<uint64_t>(r.end - r.p) / (sizeof(uint64_t) + sizeof(float))) throw std::runtime_error("truncated VW model");
  if (bits != bits_ || stride != stride_) {
    // the model defines the table geometry
    bits_ = bits;
    mask_ = (1ull << bits_) - 1;
    stride_ = stride;
    weights_.assign(static_cast<size_t>(mask_ + 1) * stride_, 0.f);
  } else {
    std::fill(weights_.begin(), weights_.end(), 0.f);
  }
  t_ = t; total_weight_ = tw; sum_norm_x_ = snx;
  stats_.min_label = lo; stats_.max_label = hi;
  for (uint64_t k = 0; k < nz; ++k) {
    const uint64_t i = r.Get<uint64_t>();
    const float v = r.Get<float>();
    if (i < weights_.size()) weights_[i] = v;
  }
}

std::string VW::ReadableModel() const {
  std::ostringstream o;
  o << "Version 9.3.0\nId \nMin label:" << stats_.min_label << "\nMax label:" << stats_.max_label
    << "\nbits:" << bits_ << "\nlda:0\n0 ngram:\n0 skip:\noptions: " << args_str_ << "\nChecksum: 0\n:0\n";
  for (uint64_t i = 0; i < weights_.size(); i += stride_)
    if (weights_[i] != 0.f) o << (i / stride_) << ":" << weights_[i] << "\n";
  return o.str();
}

std::unique_ptr<VW> VW::Merge(const std::vector<const VW*>& models) {
  if (models.empty()) throw std::runtime_error("no models to merge");
  std::unique_ptr<VW> out(new VW(models[0]->args_str_));
  if (out->weights_.size() != models[0]->weights_.size()) out->weights_.assign(models[0]->weights_.size(), 0.f);
  for (const VW* m : models) {
    if (m->weights_.size() != out->weights_.size()) throw std::runtime_error("cannot merge models of different size");
    for (size_t i = 0; i < m->weights_.size(); ++i) out->weights_[i] += m->weights_[i];
    out->t_ += m->t_;
    out->total_weight_ += m->total_weight_;
    out->sum_norm_x_ += m->sum_norm_x_;
    out->stats_.examples += m->stats_.examples;
    out->stats_.weighted_examples += m->stats_.weighted_examples;
    out->stats_.sum_loss += m->stats_.sum_loss;
    out->stats_.min_label = std::min(out->stats_.min_label, m->stats_.min_label);
    out->stats_.max_label = std::max(out->stats_.max_label, m->stats_.max_label);
  }
  const float inv = 1.f / models.size();
  for (auto& w : out->weights_) w *= inv;
  return out;
}

}  // namespace smlvw
