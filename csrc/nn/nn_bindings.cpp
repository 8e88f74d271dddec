// pybind11 module _nn: raw-pointer entry points (torch data_ptr + stream).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "nn_ops.h"

namespace py = pybind11;
using namespace smlnn;

template <class T>
static T* P(uintptr_t p) {
  return reinterpret_cast<T*>(p);
}

PYBIND11_MODULE(_nn, m) {
  m.doc() = "MI355X fused epilogue kernels for the ONNX executor";
  m.def("gpu_available", &NnGpuAvailable);
  m.def("affine_act", [](uintptr_t x, int64_t n, int C, int HW, int nhwc, uintptr_t scale, uintptr_t shift,
                         uintptr_t res, int act, float alpha, int dtype, uintptr_t y, uintptr_t stream) {
    AffineAct(P<const void>(x), n, C, HW, nhwc, P<const float>(scale), P<const float>(shift), P<const void>(res), act,
              alpha, dtype, P<void>(y), P<void>(stream));
  });
  m.def("add_affine_act", [](uintptr_t a, uintptr_t b, int64_t n, int C, int HW, int nhwc, uintptr_t scale,
                             uintptr_t shift, int act, int dtype, uintptr_t sum_out, uintptr_t act_out,
                             uintptr_t stream) {
    AddAffineAct(P<const void>(a), P<const void>(b), n, C, HW, nhwc, P<const float>(scale), P<const float>(shift), act,
                 dtype, P<void>(sum_out), P<void>(act_out), P<void>(stream));
  });
  m.def("gap_nhwc", [](uintptr_t x, int N, int HW, int C, int dtype, uintptr_t out, uintptr_t stream) {
    GapNhwc(P<const void>(x), N, HW, C, dtype, P<void>(out), P<void>(stream));
  });
  m.def("maxpool_nhwc", [](uintptr_t x, int N, int H, int W, int C, int kh, int kw, int sh, int sw, int ph, int pw,
                           int OH, int OW, int dtype, uintptr_t y, uintptr_t stream, uintptr_t shift, int relu) {
    MaxPoolNhwc(reinterpret_cast<const void*>(x), N, H, W, C, kh, kw, sh, sw, ph, pw, OH, OW, dtype,
                reinterpret_cast<void*>(y), reinterpret_cast<void*>(stream), reinterpret_cast<const float*>(shift), relu);
  }, pybind11::arg("x"), pybind11::arg("N"), pybind11::arg("H"), pybind11::arg("W"), pybind11::arg("C"),
     pybind11::arg("kh"), pybind11::arg("kw"), pybind11::arg("sh"), pybind11::arg("sw"), pybind11::arg("ph"),
     pybind11::arg("pw"), pybind11::arg("OH"), pybind11::arg("OW"), pybind11::arg("dtype"), pybind11::arg("y"),
     pybind11::arg("stream"), pybind11::arg("shift") = 0, pybind11::arg("relu") = 0);
  m.def("conv_supported", &ConvMfmaSupported);
  m.def("conv_mfma", [](uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t in_scale, uintptr_t in_shift,
                        uintptr_t bias, uintptr_t res, uintptr_t out_scale, uintptr_t out_shift, uintptr_t y2,
                        std::vector<int> g, int relu, int prologue_relu, int dtype, uintptr_t stream, int kernel,
                        int split_k, uintptr_t ws, uintptr_t ws_cnt) {
    if (g.size() != 15) throw std::invalid_argument("geometry: B,H,W,C,Cout,R,S,sh,sw,ph,pw,dh,dw,OH,OW");
    ConvArgs a{P<const void>(x), P<const void>(w), P<void>(y), P<const float>(in_scale), P<const float>(in_shift),
               P<const float>(bias), P<const void>(res), P<const float>(out_scale), P<const float>(out_shift),
               P<void>(y2), g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9], g[10], g[11], g[12], g[13],
               g[14], relu, prologue_relu, kernel, split_k, P<float>(ws), P<int>(ws_cnt)};
    const int rc = ConvMfma(a, dtype, P<void>(stream));
    if (rc != 0) throw std::runtime_error("conv_mfma failed (rc=" + std::to_string(rc) + ")");
  }, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("y"), pybind11::arg("in_scale"), pybind11::arg("in_shift"),
     pybind11::arg("bias"), pybind11::arg("res"), pybind11::arg("out_scale"), pybind11::arg("out_shift"),
     pybind11::arg("y2"), pybind11::arg("geom"), pybind11::arg("relu"), pybind11::arg("prologue_relu"),
     pybind11::arg("dtype"), pybind11::arg("stream"), pybind11::arg("kernel") = 0, pybind11::arg("split_k") = 1,
     pybind11::arg("ws") = 0, pybind11::arg("ws_cnt") = 0);
  // few-channel stem conv: w packed [Cout][160] (ops.conv.pack_stem_weight)
  // (in_scale / in_shift: optional per-input-channel affine (+ ReLU) applied to the im2col values, padding
  // taps stay 0 - the input BatchNormalization of an image model)
  m.def("stem_conv", [](uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t bias, uintptr_t res, std::vector<int> g,
                        int relu, int dtype, uintptr_t stream, uintptr_t in_scale, uintptr_t in_shift, int pro_relu,
                        int kp, int form) {
    if (g.size() != 15) throw std::invalid_argument("geometry: B,H,W,C,Cout,R,S,sh,sw,ph,pw,dh,dw,OH,OW");
    if ((in_scale == 0) != (in_shift == 0)) throw std::invalid_argument("in_scale and in_shift go together");
    ConvArgs a{P<const void>(x), P<const void>(w), P<void>(y), P<const float>(in_scale), P<const float>(in_shift),
               P<const float>(bias), P<const void>(res), nullptr, nullptr, nullptr, g[0], g[1], g[2], g[3], g[4], g[5],
               g[6], g[7], g[8], g[9], g[10], g[11], g[12], g[13], g[14], relu, pro_relu, 0};
    const int rc = StemConv(a, dtype, P<void>(stream), kp, form);
    if (rc != 0) throw std::runtime_error("stem_conv failed (rc=" + std::to_string(rc) + ")");
  }, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("y"), pybind11::arg("bias"), pybind11::arg("res"),
     pybind11::arg("geom"), pybind11::arg("relu"), pybind11::arg("dtype"), pybind11::arg("stream"),
     pybind11::arg("in_scale") = 0, pybind11::arg("in_shift") = 0, pybind11::arg("pro_relu") = 0,
     pybind11::arg("kp") = 160, pybind11::arg("form") = 0);
  // split-K plan of the default tile: (splits, workspace fp32 floats, int32 counters)
  m.def("conv_split_plan", [](std::vector<int> g, int dtype, bool has_prologue, int kernel) {
    if (g.size() != 15) throw std::invalid_argument("geometry: B,H,W,C,Cout,R,S,sh,sw,ph,pw,dh,dw,OH,OW");
    static const float dummy = 0.f;
    ConvArgs a{nullptr, nullptr, nullptr, has_prologue ? &dummy : nullptr, nullptr, nullptr, nullptr, nullptr,
               nullptr, nullptr, g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9], g[10], g[11], g[12], g[13],
               g[14], 0, 0, kernel};
    int64_t wsf = 0;
    int cnt = 0;
    const int sk = ConvSplitPlan(a, dtype, &wsf, &cnt);
    return pybind11::make_tuple(sk, wsf, cnt);
  }, pybind11::arg("geom"), pybind11::arg("dtype"), pybind11::arg("has_prologue"), pybind11::arg("kernel") = 0);
  // conv: [] or [H, W, C, R, S, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w, OH, OW] (implicit im2col A)
  m.def("gemm", [](uintptr_t a, uintptr_t b, uintptr_t c, int M, int N, int K, int batch, int64_t lda, int64_t ldb,
                   int64_t ldc, int64_t sa, int64_t sb, int64_t sc, int trans_a, int trans_b, float alpha, float beta,
                   uintptr_t bias, uintptr_t cmat, int64_t ldcm, int64_t scm, int act, int dtype, uintptr_t stream,
                   std::vector<int> conv, int64_t stride_bias) {
    GemmArgs g;
    if (!conv.empty()) {
      if (conv.size() != 13) throw std::invalid_argument("conv geometry: H,W,C,R,S,sh,sw,ph,pw,dh,dw,OH,OW");
      g.conv = 1;
      g.H = conv[0]; g.W = conv[1]; g.C = conv[2]; g.R = conv[3]; g.S = conv[4]; g.stride_h = conv[5];
      g.stride_w = conv[6]; g.pad_h = conv[7]; g.pad_w = conv[8]; g.dil_h = conv[9]; g.dil_w = conv[10];
      g.OH = conv[11]; g.OW = conv[12];
    }
    g.stride_bias = stride_bias;
    g.a = P<const void>(a); g.b = P<const void>(b); g.c = P<void>(c);
    g.M = M; g.N = N; g.K = K; g.batch = batch;
    g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.stride_a = sa; g.stride_b = sb; g.stride_c = sc;
    g.trans_a = trans_a; g.trans_b = trans_b; g.alpha = alpha; g.beta = beta;
    g.bias = P<const float>(bias); g.cmat = P<const void>(cmat); g.ldcm = ldcm; g.stride_cm = scm; g.act = act;
    const int rc = GemmMfma(g, dtype, P<void>(stream));
    if (rc != 0) throw std::runtime_error("gemm_mfma failed (rc=" + std::to_string(rc) + ")");
  }, pybind11::arg("a"), pybind11::arg("b"), pybind11::arg("c"), pybind11::arg("M"), pybind11::arg("N"),
     pybind11::arg("K"), pybind11::arg("batch"), pybind11::arg("lda"), pybind11::arg("ldb"), pybind11::arg("ldc"),
     pybind11::arg("sa"), pybind11::arg("sb"), pybind11::arg("sc"), pybind11::arg("trans_a"), pybind11::arg("trans_b"),
     pybind11::arg("alpha"), pybind11::arg("beta"), pybind11::arg("bias"), pybind11::arg("cmat"), pybind11::arg("ldcm"),
     pybind11::arg("scm"), pybind11::arg("act"), pybind11::arg("dtype"), pybind11::arg("stream"),
     pybind11::arg("conv") = std::vector<int>(), pybind11::arg("stride_bias") = 0);
  m.def("group_conv", [](uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t bias, uintptr_t res, std::vector<int> g,
                         int groups, int relu, int dtype, uintptr_t stream) {
    if (g.size() != 15) throw std::invalid_argument("geometry: B,H,W,C,Cout,R,S,sh,sw,ph,pw,dh,dw,OH,OW");
    GroupConvArgs a{P<const void>(x), P<const void>(w), P<void>(y), P<const float>(bias), P<const void>(res),
                    g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9], g[10], g[11], g[12], g[13], g[14],
                    groups, relu};
    const int rc = GroupConv(a, dtype, P<void>(stream));
    if (rc != 0) throw std::runtime_error("group_conv failed (rc=" + std::to_string(rc) + ")");
  });
  m.def("softmax_rows", [](uintptr_t x, int rows, int cols, uintptr_t y, uintptr_t amax, uintptr_t stream) {
    SoftmaxRows(P<const float>(x), rows, cols, P<float>(y), P<int64_t>(amax), P<void>(stream));
  });
}
