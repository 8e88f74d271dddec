// Native host test of the VW learner core (vw_core.cpp) for the ASan + UBSan build: every reduction the
// core implements learns from text examples, models round-trip through SaveModel / load, truncated or
// corrupted model bytes and malformed command lines / example lines are rejected with exceptions (never
// an out-of-bounds read). Exit code != 0 on any mismatch.
#include <cmath>
#include <cstdio>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "vw_core.h"

using namespace smlvw;

static int failures = 0;
#define CHECK(c)                                                                   \
  do {                                                                             \
    if (!(c)) {                                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c);    \
      ++failures;                                                                  \
    }                                                                              \
  } while (0)

static std::vector<std::string> scalar_lines(int n, bool logistic, std::mt19937& rng) {
  std::normal_distribution<double> nd;
  std::vector<std::string> out;
  for (int i = 0; i < n; ++i) {
    const double a = nd(rng), b = nd(rng) * 30.0, c = nd(rng) * 1e-3;
    const double s = a - 0.05 * b + 200.0 * c;
    char buf[256];
    const double y = logistic ? (s > 0 ? 1.0 : -1.0) : s;
    std::snprintf(buf, sizeof(buf), "%g 1.0 'ex%d |x a:%g b:%g |y c:%g word%d", y, i, a, b, c, i % 7);
    out.push_back(buf);
  }
  return out;
}

static void roundtrip(VW& vw, const std::vector<std::string>& probe) {
  const std::string m = vw.SaveModel();
  VW back(vw.args(), &m);
  for (const auto& l : probe) {
    Example a = vw.ParseLine(l), b = back.ParseLine(l);
    vw.Predict(a);
    back.Predict(b);
    CHECK(a.pred == b.pred);
  }
  CHECK(back.SaveModel() == m);
  // every truncation of the model bytes is rejected (or loads a prefix-complete model), never read past
  int rejected = 0;
  for (size_t cut = 0; cut < m.size(); cut += std::max<size_t>(1, m.size() / 97)) {
    const std::string t = m.substr(0, cut);
    try {
      VW bad(vw.args(), &t);
      (void)bad;
    } catch (const std::exception&) {
      ++rejected;
    }
  }
  CHECK(rejected > 0);
}

static void scalar(const std::string& args, bool logistic) {
  std::mt19937 rng(5);
  auto lines = scalar_lines(3000, logistic, rng);
  VW vw(args);
  for (int pass = 0; pass < 2; ++pass)
    for (const auto& l : lines) {
      Example ex = vw.ParseLine(l);
      vw.Learn(ex);
    }
  CHECK(std::isfinite(vw.stats().sum_loss));
  CHECK(vw.stats().examples == 6000);
  roundtrip(vw, std::vector<std::string>(lines.begin(), lines.begin() + 50));
  std::printf("ok  %-60s loss=%.4f\n", args.c_str(), vw.stats().sum_loss / vw.stats().weighted_examples);
}

static void multiclass(const std::string& args, bool cost_sensitive) {
  std::mt19937 rng(9);
  std::uniform_int_distribution<int> cls(1, 3);
  VW vw(args);
  std::vector<std::string> lines;
  for (int i = 0; i < 2000; ++i) {
    const int c = cls(rng);
    char buf[128];
    if (cost_sensitive)
      std::snprintf(buf, sizeof(buf), "1:%d 2:%d 3:%d | f%d g", c == 1 ? 0 : 1, c == 2 ? 0 : 1, c == 3 ? 0 : 1, c);
    else
      std::snprintf(buf, sizeof(buf), "%d | f%d g", c, c);
    lines.push_back(buf);
  }
  for (const auto& l : lines) {
    Example ex = vw.ParseLine(l);
    vw.Learn(ex);
  }
  int right = 0;
  for (int c = 1; c <= 3; ++c) {
    Example ex = vw.ParseLine("| f" + std::to_string(c) + " g");
    vw.Predict(ex);
    right += static_cast<int>(ex.pred) == c;
  }
  CHECK(right == 3);
  roundtrip(vw, {"| f1 g", "| f2", "| f3 g"});
  std::printf("ok  %-60s\n", args.c_str());
}

static void bandit() {
  VW vw("--cb_explore_adf -q sa --epsilon 0.2");
  std::mt19937 rng(3);
  std::uniform_int_distribution<int> ctx(0, 2);
  for (int i = 0; i < 1500; ++i) {
    const int s = ctx(rng), a = static_cast<int>(rng() % 3);
    std::vector<Example> exs;
    exs.push_back(vw.ParseLine("shared |s c" + std::to_string(s)));
    for (int k = 0; k < 3; ++k) {
      std::string lab = k == a ? std::to_string(k) + ":" + (a == s ? "-1" : "0") + ":0.333 " : "";
      exs.push_back(vw.ParseLine(lab + "|a act" + std::to_string(k)));
    }
    vw.LearnMulti(exs);
  }
  std::vector<Example> q;
  q.push_back(vw.ParseLine("shared |s c1"));
  for (int k = 0; k < 3; ++k) q.push_back(vw.ParseLine("|a act" + std::to_string(k)));
  vw.PredictMulti(q);
  double tot = 0;
  // the distribution lands on the first action example (VW's convention for ADF predictions)
  for (const auto& ap : q[1].action_probs) tot += ap.second;
  CHECK(std::fabs(tot - 1.0) < 1e-5);
  CHECK(!q[1].action_probs.empty() && q[1].action_probs[0].first == 1);
  std::printf("ok  cb_explore_adf\n");
}

static void cats() {
  VW vw("--cats_pdf 4 --bandwidth 2500 --min_value 0 --max_value 20000");
  std::mt19937 rng(0);
  std::uniform_real_distribution<double> u(0, 20000);
  for (int i = 0; i < 2000; ++i) {
    const double a = u(rng);
    char buf[96];
    std::snprintf(buf, sizeof(buf), "ca %.2f:%g:%.8f | x", a, (a > 12000 && a < 18000) ? 0.0 : 1.0, 1.0 / 20000);
    Example ex = vw.ParseLine(buf);
    vw.Learn(ex);
  }
  Example ex = vw.ParseLine("| x");
  vw.Predict(ex);
  double mass = 0;
  for (const auto& s : ex.pdf_segments) mass += (s[1] - s[0]) * s[2];
  CHECK(std::fabs(mass - 1.0) < 1e-3);
  std::printf("ok  cats_pdf (%zu segments)\n", ex.pdf_segments.size());
}

static void malformed() {
  const std::vector<std::string> bad_args = {"--bogus", "-b", "-b 99", "--oaa", "--oaa x", "--cats 3",
                                             "--nn 10", "--loss_function nope", "-l"};
  int rejected = 0;
  for (const auto& a : bad_args) {
    try {
      VW v(a);
      std::fprintf(stderr, "accepted bad args: %s\n", a.c_str());
      ++failures;
    } catch (const std::exception&) {
      ++rejected;
    }
  }
  // odd example lines: parsed or rejected, never out of bounds
  VW vw("--csoaa 3");
  VW plain("-q ab --ngram 2");
  VW adf("--cb_explore_adf");
  const std::vector<std::string> lines = {"", "|", "||", "1", "1 |", "| :", "| a:", "| :3", "|a:x b", "| a:1e39",
                                          "1:2:3 | a", "1: | a", "'tag", "1 'tag |a b:nan", "ca 1:2 | x",
                                          "| " + std::string(3000, 'z'), "|\t\ta b", "1 2 3 4 | a"};
  int parsed = 0, thrown = 0;
  for (VW* v : {&vw, &plain, &adf}) {
    for (const auto& l : lines) {
      try {
        Example ex = v->ParseLine(l);
        if (v == &plain) v->Learn(ex);
        ++parsed;
      } catch (const std::exception&) {
        ++thrown;
      }
    }
  }
  std::printf("ok  malformed: %d bad arg lines rejected; %d odd lines parsed, %d rejected\n", rejected, parsed, thrown);
}

int main() {
  std::setvbuf(stdout, nullptr, _IONBF, 0);
  scalar("", false);
  scalar("--sgd", false);
  scalar("--loss_function logistic -q xy --l2 1e-6", true);
  scalar("--adaptive --invariant -l 0.2 --power_t 0.3 --l1 1e-7", false);
  scalar("--ngram x2 --ignore y", false);
  multiclass("--oaa 3", false);
  multiclass("--csoaa 3", true);
  bandit();
  cats();
  malformed();
  if (failures) {
    std::fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  std::printf("all native vw host tests passed\n");
  return 0;
}
