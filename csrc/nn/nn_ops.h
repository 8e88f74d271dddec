// Fused epilogue / post-processing kernels of the ONNX executor (module _nn).
// dtype: 0 fp32, 1 fp16, 2 bf16. act: 0 none, 1 relu, 2 leaky(alpha),
// 3 sigmoid, 4 clip(0, alpha). All pointers are device pointers.
#pragma once
#include <cstdint>

namespace smlnn {

bool NnGpuAvailable();
// y = act(x * scale[c] + shift[c] + res); scale/shift/res may be null; y may alias x.
void AffineAct(const void* x, int64_t n, int C, int HW, int nhwc, const float* scale, const float* shift,
               const void* res, int act, float alpha, int dtype, void* y, void* stream);
// sum = a + b; act_out = act(sum * scale[c] + shift[c]) (one pass, two outputs)
void AddAffineAct(const void* a, const void* b, int64_t n, int C, int HW, int nhwc, const float* scale,
                  const float* shift, int act, int dtype, void* sum_out, void* act_out, void* stream);
// NHWC max pool (symmetric pads, -inf padding, no dilation), C % 8 == 0
// shift (per channel, fp32, may be null) and relu: epilogue applied to the pooled maxima
void MaxPoolNhwc(const void* x, int N, int H, int W, int C, int kh, int kw, int sh, int sw, int ph, int pw, int OH,
                 int OW, int dtype, void* y, void* stream, const float* shift = nullptr, int relu = 0);
// NHWC global average pool -> fp32 [N, C]
void GapNhwc(const void* x, int N, int HW, int C, int dtype, void* out, void* stream);  // out: input dtype
// Implicit-GEMM MFMA convolution with fused prologue/epilogue (conv_mfma.hip).
struct ConvArgs {
  const void* x;           // NHWC [B, H, W, C]
  const void* w;           // [Cout][R][S][C]
  void* y;                 // NHWC [B, OH, OW, Cout]
  const float* in_scale;   // prologue affine per input channel (null: none)
  const float* in_shift;
  const float* bias;       // per output channel (null: none)
  const void* res;         // residual, same layout as y (null: none)
  const float* out_scale;  // second output y2 = relu(y * out_scale + out_shift) (null: none)
  const float* out_shift;
  void* y2;
  int B, H, W, C, Cout, R, S, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w, OH, OW;
  int relu;            // 0 none, 1 after bias (before the residual add), 2 after the residual add
  int prologue_relu;   // relu after the prologue affine
  int kernel = 0;      // 0 picks the tile by shape; BM*1000+BN forces one (64064, 128064, 64128,
                       // 128128, 256128, 128256)
  // split-K (ConvSplitPlan): split_k > 1 K ranges per output tile, fp32 partial tiles in ws, one arrival
  // counter per tile in ws_cnt (zeroed before the launch); the last arriving split sums and runs the epilogue
  int split_k = 1;
  float* ws = nullptr;
  int* ws_cnt = nullptr;
};
constexpr int kConvStem = 1;  // ConvArgs::kernel: the packed few-channel stem form (C = 4, R = S = 8)
bool ConvMfmaSupported(int C, int Cout, int groups, int dtype);
int ConvMfma(const ConvArgs& a, int dtype, void* stream);
// few-channel (C <= 4) stem conv, K = R * S * C <= 160, weights packed [Cout][160] zero-padded; f16 / bf16
// kp = packed K width: 160 (k = (r * S + s) * C + c) or 192 (C = 3, S * 3 <= 24: k = r * 24 + s * 3 + c)
// form: 0 auto (the row-staged kernel where it applies), 1 the 2-byte gather kernel, 2 row-staged only
int StemConv(const ConvArgs& a, int dtype, void* stream, int kp = 160, int form = 0);
// split-K plan of the tile ConvMfma would pick for a (kernel = 0 only): the number of K splits (1: none) and
// the workspace it needs (fp32 floats, int32 tile counters)
int ConvSplitPlan(const ConvArgs& a, int dtype, int64_t* ws_floats, int* counters);
// K17: batched GEMM with fused epilogue (gemm_mfma.hip), dtype 0 fp32 / 1 fp16 / 2 bf16:
//   C[b] = act(alpha * op(A[b]) * op(B[b]) + beta * (bias[n] | Cin[b]))
// op(A) is [M][K] (trans_a = 0, lda >= K) or A stored [K][M] (trans_a = 1, lda >= M);
// op(B) is [K][N] stored [K][N] (trans_b = 0, ldb >= N) or stored [N][K] (trans_b = 1, ldb >= K).
// Batch strides are in elements (0 = broadcast). Returns 0, or < 0 when the shape is not supported.
struct GemmArgs {
  const void* a = nullptr;
  const void* b = nullptr;
  void* c = nullptr;
  int M = 0, N = 0, K = 0, batch = 1;
  int64_t lda = 0, ldb = 0, ldc = 0;
  int64_t stride_a = 0, stride_b = 0, stride_c = 0;
  int trans_a = 0, trans_b = 0;
  float alpha = 1.f, beta = 1.f;
  const float* bias = nullptr;   // [N] (scaled by beta); batch z reads bias + z * stride_bias
  int64_t stride_bias = 0;
  const void* cmat = nullptr;    // [M][N] additive input, ldcm, batch stride stride_cm (scaled by beta)
  int64_t ldcm = 0, stride_cm = 0;
  int act = 0;                   // 0 none, 1 relu
  // conv = 1: A is the implicit im2col of an NHWC input (any channel count, the 3-channel stem included):
  // row m = (b, oh, ow) of [B, OH, OW], column k = (r, s, c) of [R, S, Cg]; the element is
  // a[((b * H + ih) * W + iw) * C + c] (+ batch stride: a group's channel offset), zero in the padding.
  // K must equal R * S * Cg; M = B * OH * OW; C is the input's pixel stride (all channels).
  int conv = 0;
  int H = 0, W = 0, C = 0, R = 1, S = 1, stride_h = 1, stride_w = 1, pad_h = 0, pad_w = 0, dil_h = 1, dil_w = 1;
  int OH = 0, OW = 0;
};
int GemmMfma(const GemmArgs& g, int dtype, void* stream);
// Direct grouped / depthwise NHWC convolution (conv_direct.hip): x [B,H,W,C], w [Cout][R][S][C/groups],
// y [B,OH,OW,Cout]; fp32 accumulation; y = conv + bias, relu (1: before the residual add, 2: after), + res.
struct GroupConvArgs {
  const void* x;
  const void* w;
  void* y;
  const float* bias;
  const void* res;
  int B, H, W, C, Cout, R, S, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w, OH, OW, groups, relu;
};
int GroupConv(const GroupConvArgs& a, int dtype, void* stream);
// fp32 row softmax (y may be null) and argmax (amax may be null)
void SoftmaxRows(const float* x, int rows, int cols, float* y, int64_t* amax, void* stream);

}  // namespace smlnn
