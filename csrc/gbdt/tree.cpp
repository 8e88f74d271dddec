#include "tree.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <limits>
#include <map>
#include <sstream>
#include <stdexcept>
#include <type_traits>

namespace sml {

Tree::Tree(int ml) : max_leaves(ml) {
  int ni = std::max(1, ml - 1);
  split_feature_inner.assign(ni, 0); split_feature.assign(ni, 0); split_gain.assign(ni, 0);
  threshold.assign(ni, 0); threshold_in_bin.assign(ni, 0); decision_type.assign(ni, 0);
  left_child.assign(ni, 0); right_child.assign(ni, 0);
  internal_value.assign(ni, 0); internal_weight.assign(ni, 0); internal_count.assign(ni, 0);
  leaf_value.assign(ml, 0); leaf_weight.assign(ml, 0); leaf_count.assign(ml, 0);
  leaf_parent.assign(ml, -1); leaf_depth.assign(ml, 0);
}

static int SplitCommon(Tree* t, int leaf, int feat_inner, int feat_real, double left_value,
                       double right_value, int64_t left_cnt, int64_t right_cnt,
                       double left_weight, double right_weight, double gain) {
  int node = t->num_leaves - 1;
  int parent = t->leaf_parent[leaf];
  if (parent >= 0) {
    if (t->left_child[parent] == ~leaf) t->left_child[parent] = node;
    else t->right_child[parent] = node;
  }
  t->split_feature_inner[node] = feat_inner;
  t->split_feature[node] = feat_real;
  t->split_gain[node] = gain;
  t->left_child[node] = ~leaf;
  t->right_child[node] = ~t->num_leaves;
  t->internal_value[node] = t->leaf_value[leaf];
  t->internal_weight[node] = left_weight + right_weight;
  t->internal_count[node] = left_cnt + right_cnt;
  int nl = t->num_leaves;
  t->leaf_parent[leaf] = node;
  t->leaf_parent[nl] = node;
  t->leaf_value[leaf] = std::isnan(left_value) ? 0.0 : left_value;
  t->leaf_value[nl] = std::isnan(right_value) ? 0.0 : right_value;
  t->leaf_weight[leaf] = left_weight; t->leaf_weight[nl] = right_weight;
  t->leaf_count[leaf] = left_cnt; t->leaf_count[nl] = right_cnt;
  t->leaf_depth[nl] = t->leaf_depth[leaf] + 1;
  t->leaf_depth[leaf] += 1;
  ++t->num_leaves;
  return nl;
}

int Tree::Split(int leaf, int feat_inner, int feat_real, uint32_t thr_bin, double thr_value,
                bool default_left, int missing_type, double left_value, double right_value,
                int64_t left_cnt, int64_t right_cnt, double left_weight, double right_weight,
                double gain) {
  int node = num_leaves - 1;
  threshold_in_bin[node] = thr_bin;
  threshold[node] = thr_value;
  decision_type[node] = MakeDecisionType(false, default_left, missing_type);
  return SplitCommon(this, leaf, feat_inner, feat_real, left_value, right_value, left_cnt, right_cnt,
                     left_weight, right_weight, gain);
}

int Tree::SplitCategorical(int leaf, int feat_inner, int feat_real,
                           const std::vector<uint32_t>& bin_bitset,
                           const std::vector<uint32_t>& value_bitset, double left_value,
                           double right_value, int64_t left_cnt, int64_t right_cnt,
                           double left_weight, double right_weight, double gain) {
  int node = num_leaves - 1;
  threshold_in_bin[node] = static_cast<uint32_t>(num_cat);
  threshold[node] = static_cast<double>(num_cat);
  decision_type[node] = MakeDecisionType(true, false, kMissingNaN);
  cat_threshold.insert(cat_threshold.end(), value_bitset.begin(), value_bitset.end());
  cat_boundaries.push_back(static_cast<int>(cat_threshold.size()));
  cat_threshold_inner.insert(cat_threshold_inner.end(), bin_bitset.begin(), bin_bitset.end());
  cat_boundaries_inner.push_back(static_cast<int>(cat_threshold_inner.size()));
  ++num_cat;
  return SplitCommon(this, leaf, feat_inner, feat_real, left_value, right_value, left_cnt, right_cnt,
                     left_weight, right_weight, gain);
}

void Tree::Shrink(double rate) {
  for (int i = 0; i < num_leaves; ++i) leaf_value[i] *= rate;
  for (int i = 0; i < num_leaves - 1; ++i) internal_value[i] *= rate;
  shrinkage *= rate;
}

void Tree::AddBias(double bias) {
  for (int i = 0; i < num_leaves; ++i) leaf_value[i] += bias;
  for (int i = 0; i < num_leaves - 1; ++i) internal_value[i] += bias;
}

static inline bool FindInBitset(const uint32_t* bits, int n, int pos) {
  int w = pos / 32;
  if (pos < 0 || w >= n) return false;
  return (bits[w] >> (pos % 32)) & 1u;
}

int Tree::NumericalDecision(double fval, int node) const {
  int8_t dt = decision_type[node];
  int missing = (dt >> 2) & 3;
  bool default_left = (dt & 2) != 0;
  if (std::isnan(fval) && missing != kMissingNaN) fval = 0.0;
  if ((missing == kMissingZero && std::fabs(fval) <= kZeroThreshold) ||
      (missing == kMissingNaN && std::isnan(fval))) {
    return default_left ? left_child[node] : right_child[node];
  }
  return fval <= threshold[node] ? left_child[node] : right_child[node];
}

int Tree::CategoricalDecision(double fval, int node) const {
  if (std::isnan(fval)) return right_child[node];
  int iv = static_cast<int>(fval);
  if (iv < 0) return right_child[node];
  int ci = static_cast<int>(threshold[node]);
  int b = cat_boundaries[ci], e = cat_boundaries[ci + 1];
  return FindInBitset(cat_threshold.data() + b, e - b, iv) ? left_child[node] : right_child[node];
}

int Tree::GetLeaf(const double* x) const {
  if (num_leaves <= 1) return 0;
  int node = 0;
  while (node >= 0) {
    double f = x[split_feature[node]];
    node = (decision_type[node] & 1) ? CategoricalDecision(f, node) : NumericalDecision(f, node);
  }
  return ~node;
}

int Tree::GetLeafSparse(const int32_t* idx, const double* val, int nnz, std::vector<double>* buf) const {
  (void)idx; (void)val; (void)nnz; (void)buf;
  return 0;  // callers densify first; kept for API symmetry
}

int Tree::GetLeafByBins(const uint8_t* row, const std::vector<BinMapper>& mappers,
                        const std::vector<int>& used) const {
  if (num_leaves <= 1) return 0;
  int node = 0;
  while (node >= 0) {
    int fi = split_feature_inner[node];
    uint32_t b = row[fi];
    int8_t dt = decision_type[node];
    if (dt & 1) {
      int ci = static_cast<int>(threshold_in_bin[node]);
      int s = cat_boundaries_inner[ci], e = cat_boundaries_inner[ci + 1];
      node = FindInBitset(cat_threshold_inner.data() + s, e - s, static_cast<int>(b)) ? left_child[node] : right_child[node];
    } else {
      const BinMapper& m = mappers[used[fi]];
      int missing = (dt >> 2) & 3;
      bool dl = (dt & 2) != 0;
      if ((missing == kMissingZero && b == static_cast<uint32_t>(m.default_bin)) ||
          (missing == kMissingNaN && b == static_cast<uint32_t>(m.num_bin - 1))) {
        node = dl ? left_child[node] : right_child[node];
      } else {
        node = b <= threshold_in_bin[node] ? left_child[node] : right_child[node];
      }
    }
  }
  return ~node;
}

double Tree::ExpectedValue() const {
  if (num_leaves == 1) return leaf_value[0];
  double total = static_cast<double>(internal_count[0]);
  if (total <= 0) return 0.0;
  double e = 0;
  for (int i = 0; i < num_leaves; ++i) e += leaf_count[i] / total * leaf_value[i];
  return e;
}

int Tree::MaxDepth() const {
  int d = 0;
  for (int i = 0; i < num_leaves; ++i) d = std::max(d, leaf_depth[i]);
  return d;
}

// ---------------------------------------------------------------------------
// Path-dependent TreeSHAP (Lundberg, Erion & Lee 2018), the algorithm behind
// the reference's featuresShap (LightGBMBooster.scala:418-427).
namespace {
struct PathElement {
  int feature_index;
  double zero_fraction, one_fraction, pweight;
};

void ExtendPath(PathElement* p, int d, double zf, double of, int fi) {
  p[d].feature_index = fi; p[d].zero_fraction = zf; p[d].one_fraction = of;
  p[d].pweight = d == 0 ? 1.0 : 0.0;
  for (int i = d - 1; i >= 0; --i) {
    p[i + 1].pweight += of * p[i].pweight * (i + 1) / static_cast<double>(d + 1);
    p[i].pweight = zf * p[i].pweight * (d - i) / static_cast<double>(d + 1);
  }
}

void UnwindPath(PathElement* p, int d, int pi) {
  const double of = p[pi].one_fraction, zf = p[pi].zero_fraction;
  double next = p[d].pweight;
  for (int i = d - 1; i >= 0; --i) {
    if (of != 0) {
      const double tmp = p[i].pweight;
      p[i].pweight = next * (d + 1) / static_cast<double>((i + 1) * of);
      next = tmp - p[i].pweight * zf * (d - i) / static_cast<double>(d + 1);
    } else {
      p[i].pweight = p[i].pweight * (d + 1) / static_cast<double>(zf * (d - i));
    }
  }
  for (int i = pi; i < d; ++i) {
    p[i].feature_index = p[i + 1].feature_index;
    p[i].zero_fraction = p[i + 1].zero_fraction;
    p[i].one_fraction = p[i + 1].one_fraction;
  }
}

double UnwoundPathSum(const PathElement* p, int d, int pi) {
  const double of = p[pi].one_fraction, zf = p[pi].zero_fraction;
  double next = p[d].pweight, total = 0;
  for (int i = d - 1; i >= 0; --i) {
    if (of != 0) {
      const double tmp = next * (d + 1) / static_cast<double>((i + 1) * of);
      total += tmp;
      next = p[i].pweight - tmp * zf * ((d - i) / static_cast<double>(d + 1));
    } else if (zf != 0) {
      total += (p[i].pweight / zf) / ((d - i) / static_cast<double>(d + 1));
    }
  }
  return total;
}

struct ShapCtx {
  const Tree* t;
  const double* x;
  double* phi;
};

double DataCount(const Tree* t, int node) {
  return node >= 0 ? static_cast<double>(t->internal_count[node]) : static_cast<double>(t->leaf_count[~node]);
}

void Recurse(const ShapCtx& c, int node, PathElement* parent_path, int d, double pzf, double pof, int pfi) {
  PathElement* path = parent_path + d + 1;
  std::copy(parent_path, parent_path + d + 1, path);
  ExtendPath(path, d, pzf, pof, pfi);
  const Tree* t = c.t;
  if (node < 0) {
    for (int i = 1; i <= d; ++i) {
      const double w = UnwoundPathSum(path, d, i);
      const PathElement& el = path[i];
      c.phi[el.feature_index] += w * (el.one_fraction - el.zero_fraction) * t->leaf_value[~node];
    }
    return;
  }
  double f = c.x[t->split_feature[node]];
  int hot = (t->decision_type[node] & 1) ? t->CategoricalDecision(f, node) : t->NumericalDecision(f, node);
  int cold = hot == t->left_child[node] ? t->right_child[node] : t->left_child[node];
  const double w = DataCount(t, node);
  const double hzf = w > 0 ? DataCount(t, hot) / w : 0.0;
  const double czf = w > 0 ? DataCount(t, cold) / w : 0.0;
  double izf = 1, iof = 1;
  int pi = 0;
  for (; pi <= d; ++pi) if (path[pi].feature_index == t->split_feature[node]) break;
  if (pi != d + 1) {
    izf = path[pi].zero_fraction;
    iof = path[pi].one_fraction;
    UnwindPath(path, d, pi);
    d -= 1;
  }
  Recurse(c, hot, path, d + 1, hzf * izf, iof, t->split_feature[node]);
  Recurse(c, cold, path, d + 1, czf * izf, 0, t->split_feature[node]);
}
}  // namespace

void Tree::TreeSHAP(const double* x, double* phi, int num_features) const {
  phi[num_features] += ExpectedValue();
  if (num_leaves <= 1) return;
  int md = MaxDepth() + 2;
  std::vector<PathElement> buf(static_cast<size_t>((md + 1) * (md + 2) / 2 + md + 8));
  ShapCtx c{this, x, phi};
  Recurse(c, 0, buf.data(), 0, 1, 1, -1);
}

// ---------------------------------------------------------------------------
namespace {
template <class T>
std::string Join(const std::vector<T>& v, int n) {
  std::ostringstream o;
  o.precision(17);
  for (int i = 0; i < n; ++i) { if (i) o << ' '; o << v[i]; }
  return o.str();
}
std::string JoinD(const std::vector<double>& v, int n) {
  std::string s;
  char buf[64];
  for (int i = 0; i < n; ++i) {
    double x = v[i];
    if (std::isinf(x)) x = x > 0 ? 1e300 : -1e300;
    std::snprintf(buf, sizeof(buf), "%.17g", x);
    if (i) s += ' ';
    s += buf;
  }
  return s;
}
std::string JoinI8(const std::vector<int8_t>& v, int n) {
  std::ostringstream o;
  for (int i = 0; i < n; ++i) { if (i) o << ' '; o << static_cast<int>(v[i]); }
  return o.str();
}
}  // namespace

std::string Tree::ToString(int index) const {
  std::ostringstream o;
  int ni = num_leaves - 1;
  o << "Tree=" << index << "\n";
  o << "num_leaves=" << num_leaves << "\n";
  o << "num_cat=" << num_cat << "\n";
  if (ni > 0) {
    o << "split_feature=" << Join(split_feature, ni) << "\n";
    o << "split_gain=" << JoinD(split_gain, ni) << "\n";
    o << "threshold=" << JoinD(threshold, ni) << "\n";
    o << "decision_type=" << JoinI8(decision_type, ni) << "\n";
    o << "left_child=" << Join(left_child, ni) << "\n";
    o << "right_child=" << Join(right_child, ni) << "\n";
  }
  o << "leaf_value=" << JoinD(leaf_value, num_leaves) << "\n";
  o << "leaf_weight=" << JoinD(leaf_weight, num_leaves) << "\n";
  o << "leaf_count=" << Join(leaf_count, num_leaves) << "\n";
  if (ni > 0) {
    o << "internal_value=" << JoinD(internal_value, ni) << "\n";
    o << "internal_weight=" << JoinD(internal_weight, ni) << "\n";
    o << "internal_count=" << Join(internal_count, ni) << "\n";
  }
  if (num_cat > 0) {
    o << "cat_boundaries=" << Join(cat_boundaries, num_cat + 1) << "\n";
    o << "cat_threshold=" << Join(cat_threshold, static_cast<int>(cat_threshold.size())) << "\n";
  }
  o << "is_linear=0\n";
  char buf[64];
  std::snprintf(buf, sizeof(buf), "%.17g", shrinkage);
  o << "shrinkage=" << buf << "\n\n\n";
  return o.str();
}

namespace {
template <class T>
std::vector<T> ParseVec(const std::string& s) {
  std::vector<T> out;
  std::istringstream is(s);
  std::string tok;
  while (is >> tok) {
    const double v = std::stod(tok);  // std::invalid_argument / out_of_range on junk
    if (std::is_integral<T>::value &&
        !(v >= static_cast<double>(std::numeric_limits<T>::lowest()) &&
          v <= static_cast<double>(std::numeric_limits<T>::max())))
      throw std::runtime_error("model string: integer field out of range: " + tok);
    out.push_back(static_cast<T>(v));
  }
  return out;
}

[[noreturn]] void BadTree(const std::string& what) { throw std::runtime_error("malformed tree in model string: " + what); }

// A required per-node / per-leaf array: present and at least `need` entries long.
template <class T>
std::vector<T> Field(std::map<std::string, std::string>& kv, const char* key, size_t need) {
  auto it = kv.find(key);
  if (it == kv.end()) BadTree(std::string("missing ") + key);
  std::vector<T> v = ParseVec<T>(it->second);
  if (v.size() < need)
    BadTree(std::string(key) + " has " + std::to_string(v.size()) + " entries, expected " + std::to_string(need));
  return v;
}
}  // namespace

// Model strings can come from users (loadNativeModelFromString, LightGBMBooster(model_str)), so every
// array length, child index and categorical boundary is checked and the node graph must be a tree
// rooted at node 0 that reaches every node and leaf exactly once; anything else throws instead of
// indexing out of bounds or recursing without end.
Tree Tree::FromString(const std::string& block) {
  std::map<std::string, std::string> kv;
  std::istringstream is(block);
  std::string line;
  while (std::getline(is, line)) {
    auto eq = line.find('=');
    if (eq == std::string::npos) continue;
    kv[line.substr(0, eq)] = line.substr(eq + 1);
  }
  if (!kv.count("num_leaves")) BadTree("missing num_leaves");
  const int nl = std::stoi(kv.at("num_leaves"));
  if (nl < 1 || nl > (1 << 24)) BadTree("num_leaves out of range: " + std::to_string(nl));
  Tree t(nl);
  t.num_leaves = nl;
  t.num_cat = kv.count("num_cat") ? std::stoi(kv["num_cat"]) : 0;
  if (t.num_cat < 0 || t.num_cat > nl) BadTree("num_cat out of range");
  const auto lv = Field<double>(kv, "leaf_value", static_cast<size_t>(nl));
  for (int i = 0; i < nl; ++i) t.leaf_value[i] = lv[i];
  if (kv.count("leaf_weight")) { auto v = ParseVec<double>(kv["leaf_weight"]); for (int i = 0; i < nl && i < (int)v.size(); ++i) t.leaf_weight[i] = v[i]; }
  if (kv.count("leaf_count")) { auto v = ParseVec<double>(kv["leaf_count"]); for (int i = 0; i < nl && i < (int)v.size(); ++i) t.leaf_count[i] = static_cast<int64_t>(v[i]); }
  if (nl > 1) {
    const size_t ni = static_cast<size_t>(nl - 1);
    const auto sf = Field<int>(kv, "split_feature", ni);
    const auto th = Field<double>(kv, "threshold", ni);
    const auto dt = Field<int>(kv, "decision_type", ni);
    const auto lc = Field<int>(kv, "left_child", ni);
    const auto rc = Field<int>(kv, "right_child", ni);
    const auto sg = kv.count("split_gain") ? ParseVec<double>(kv["split_gain"]) : std::vector<double>();
    for (int i = 0; i < nl - 1; ++i) {
      if (sf[i] < 0) BadTree("negative split_feature");
      if (dt[i] < 0 || dt[i] > 127) BadTree("decision_type out of range");
      for (int c : {lc[i], rc[i]}) {
        if (c >= 0 ? c >= nl - 1 : ~c >= nl) BadTree("child index out of range: " + std::to_string(c));
      }
      t.split_feature[i] = sf[i];
      t.split_feature_inner[i] = sf[i];
      t.split_gain[i] = i < (int)sg.size() ? sg[i] : 0;
      t.threshold[i] = th[i];
      t.decision_type[i] = static_cast<int8_t>(dt[i]);
      t.left_child[i] = lc[i];
      t.right_child[i] = rc[i];
    }
    if (kv.count("internal_value")) { auto v = ParseVec<double>(kv["internal_value"]); for (int i = 0; i < nl - 1 && i < (int)v.size(); ++i) t.internal_value[i] = v[i]; }
    if (kv.count("internal_weight")) { auto v = ParseVec<double>(kv["internal_weight"]); for (int i = 0; i < nl - 1 && i < (int)v.size(); ++i) t.internal_weight[i] = v[i]; }
    if (kv.count("internal_count")) { auto v = ParseVec<double>(kv["internal_count"]); for (int i = 0; i < nl - 1 && i < (int)v.size(); ++i) t.internal_count[i] = static_cast<int64_t>(v[i]); }
    // parents & depths: iterative walk; each node and leaf must be reached exactly once
    std::vector<char> seen_node(nl - 1, 0), seen_leaf(nl, 0);
    std::vector<std::pair<int, int>> stack{{0, 0}};
    seen_node[0] = 1;
    int reached_nodes = 1, reached_leaves = 0;
    while (!stack.empty()) {
      const auto [node, depth] = stack.back();
      stack.pop_back();
      for (int c : {t.left_child[node], t.right_child[node]}) {
        if (c < 0) {
          if (seen_leaf[~c]++) BadTree("leaf reached twice");
          ++reached_leaves;
          t.leaf_parent[~c] = node;
          t.leaf_depth[~c] = depth + 1;
        } else {
          if (seen_node[c]++) BadTree("node reached twice (cycle or shared subtree)");
          ++reached_nodes;
          stack.push_back({c, depth + 1});
        }
      }
    }
    if (reached_nodes != nl - 1 || reached_leaves != nl) BadTree("nodes or leaves unreachable from the root");
  }
  if (t.num_cat > 0) {
    t.cat_boundaries = Field<int>(kv, "cat_boundaries", static_cast<size_t>(t.num_cat) + 1);
    auto ct = kv.count("cat_threshold") ? ParseVec<double>(kv["cat_threshold"]) : std::vector<double>();
    t.cat_threshold.clear();
    for (double d : ct) {
      if (!(d >= 0 && d <= 4294967295.0)) BadTree("cat_threshold word out of range");
      t.cat_threshold.push_back(static_cast<uint32_t>(d));
    }
    if (t.cat_boundaries[0] != 0) BadTree("cat_boundaries must start at 0");
    for (int c = 0; c < t.num_cat; ++c)
      if (t.cat_boundaries[c + 1] < t.cat_boundaries[c]) BadTree("cat_boundaries not increasing");
    if (t.cat_boundaries[t.num_cat] > static_cast<int>(t.cat_threshold.size())) BadTree("cat_boundaries beyond cat_threshold");
  }
  for (int i = 0; i < nl - 1; ++i) {
    if (t.decision_type[i] & 1) {  // categorical: threshold is an index into cat_boundaries
      const double ci = t.threshold[i];
      if (!(ci >= 0 && ci < t.num_cat) || ci != std::floor(ci)) BadTree("categorical split without a category set");
    }
  }
  t.shrinkage = kv.count("shrinkage") ? std::stod(kv["shrinkage"]) : 1.0;
  return t;
}

std::string Tree::ToJSON(int index) const {
  std::ostringstream o;
  o.precision(17);
  std::function<void(int)> node_json = [&](int node) {
    if (node < 0) {
      int l = ~node;
      o << "{\"leaf_index\":" << l << ",\"leaf_value\":" << leaf_value[l]
        << ",\"leaf_weight\":" << leaf_weight[l] << ",\"leaf_count\":" << leaf_count[l] << "}";
      return;
    }
    int8_t dt = decision_type[node];
    o << "{\"split_index\":" << node << ",\"split_feature\":" << split_feature[node]
      << ",\"split_gain\":" << split_gain[node] << ",\"threshold\":" << threshold[node]
      << ",\"decision_type\":\"" << ((dt & 1) ? "==" : "<=") << "\",\"default_left\":"
      << (((dt & 2) != 0) ? "true" : "false") << ",\"missing_type\":\""
      << (((dt >> 2) & 3) == 0 ? "None" : (((dt >> 2) & 3) == 1 ? "Zero" : "NaN"))
      << "\",\"internal_value\":" << internal_value[node] << ",\"internal_weight\":"
      << internal_weight[node] << ",\"internal_count\":" << internal_count[node]
      << ",\"left_child\":";
    node_json(left_child[node]);
    o << ",\"right_child\":";
    node_json(right_child[node]);
    o << "}";
  };
  o << "{\"tree_index\":" << index << ",\"num_leaves\":" << num_leaves << ",\"num_cat\":" << num_cat
    << ",\"shrinkage\":" << shrinkage << ",\"tree_structure\":";
  if (num_leaves == 1) o << "{\"leaf_value\":" << leaf_value[0] << "}";
  else node_json(0);
  o << "}";
  return o.str();
}

}  // namespace sml
