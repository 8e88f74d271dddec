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
void GapNhwc(const void* x, int N, int HW, int C, int dtype, float* out, void* stream);
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
};
constexpr int kConvStem = 1;  // ConvArgs::kernel: the packed few-channel stem form (C = 4, R = S = 8)
bool ConvMfmaSupported(int C, int Cout, int groups, int dtype);
int ConvMfma(const ConvArgs& a, int dtype, void* stream);
// fp32 row softmax (y may be null) and argmax (amax may be null)
void SoftmaxRows(const float* x, int rows, int cols, float* y, int64_t* amax, void* stream);

}  // namespace smlnn
