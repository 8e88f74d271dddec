// K17: batched GEMM on the CDNA4 matrix cores with a fused epilogue (module _nn; the ONNX executor's
// Gemm / MatMul / FC path - reference: deep-learning/.../onnx/ONNXModel.scala:36-106 runs every graph
// through ORT, whose FC / MatMul kernels this replaces).
//
//   C[b][m, n] = act( alpha * sum_k A[b][m, k] * B[b][k, n] + beta * (bias[n] | Cin[b][m, n]) )
//
// A is [M][K] (lda) or, transposed, [K][M]; B is [K][N] (ONNX MatMul) or, transposed, [N][K] (Gemm
// transB=1, FC weights). Batch strides of 0 broadcast an operand. Any M, N, K.
//
// Tiling: 256 threads = 4 waves in 2x2, block tile 64 x 64 x (128 bytes of K): BK = 32 f32 or 64
// f16/bf16 elements; wave tile 32 x 32 of 16x16 MFMAs - v_mfma_f32_16x16x4_f32 (exact f32: fp32 graphs
// keep ORT-level parity, gfx950 has no xf32) or v_mfma_f32_16x16x32_{f16,bf16} with fp32 accumulation.
// Operand tiles go through registers into a double-buffered LDS image with a 144-byte row pitch (the
// 16-lane ds_read_b128 fragment reads are conflict-free); the next tile's global loads are issued before
// the current tile's MFMAs. Each operand is staged one of three ways (template kMode):
//   0  K-contiguous rows, 16-B aligned: 16-B buffer loads, out-of-range chunks read as zero
//   1  K-contiguous rows, unaligned or K % (16 B) != 0: element loads along k, bounds-checked
//   2  transposed (row index contiguous): element loads along the row index (coalesced), bounds-checked
//   3  convolution gather (A only): the implicit im2col of an NHWC input - a thread owns one output pixel
//      (row) per tile, its window origin and tap validity are computed once, and it walks BK/4
//      consecutive k = (r, s, c) per tile (contiguous channels of one tap; zero in the padding)
// Blocks are remapped so each XCD owns a contiguous run of (m, n) tiles (its L2 serves the operand reuse).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "nn_ops.h"

namespace smlnn {
namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kBM = 64, kBN = 64;

template <class T>
struct GTile {
  static constexpr int BK = 128 / static_cast<int>(sizeof(T));  // K elements per tile (128 B per row)
  static constexpr int EPV = 16 / static_cast<int>(sizeof(T));  // elements per 16-B chunk
  static constexpr int LD = BK + 2 * EPV;  // LDS row pitch (+32 B: 160 B rows are bank-conflict-free for the
                                          // 16x16 fragment reads under gfx950's ds_read_b128 lane groups; 144 B is 2-way)
};

template <class T>
__device__ __forceinline__ float ToF(T v) { return static_cast<float>(v); }
template <class T>
__device__ __forceinline__ T FromF(float v) { return static_cast<T>(v); }

// One operand's 64 x BK tile: rows r (m for A, n for B) x k. `base` points at this batch's operand.
// kMode 0/1: element (r, k) at base[r * ld + k]; kMode 2: at base[k * ld + r].
template <class T, int kMode>
struct Operand {
  static constexpr int BK = GTile<T>::BK, EPV = GTile<T>::EPV;
  static constexpr int kVec = kBM * BK / EPV / kThreads;  // 16-B chunks per thread (2)
  static constexpr int kElem = kBM * BK / kThreads;       // elements per thread (8 f32 / 16 f16)
  const T* base;
  int64_t ld;
  int rows, K;  // valid extent of the operand (rows = M or N)
  __amdgpu_buffer_rsrc_t rsrc;

  struct Regs {
    uint4 v[kMode == 0 ? kVec : 1];
    T e[kMode == 0 ? 1 : kElem];
  };
  // mode 3 (conv gather): this thread's pixel
  bool row_ok = false;  // the pixel is < M
  int pix = 0;          // element offset of (b, ih0, iw0, 0) (may be negative: only read with valid taps)
  int ih0 = 0, iw0 = 0;
  int H = 0, W = 0, C = 0, S = 1, Cg = 1, dh = 1, dw = 1;

  __device__ void InitConv(const GemmArgs& g, int r0, int tid) {
    H = g.H; W = g.W; C = g.C; S = g.S; dh = g.dil_h; dw = g.dil_w;
    Cg = K / (g.R * g.S);
    const int m = r0 + (tid & (kBM - 1));
    row_ok = m < rows;
    if (row_ok) {
      const int ow = m % g.OW, t = m / g.OW;
      const int oh = t % g.OH, b = t / g.OH;
      ih0 = oh * g.stride_h - g.pad_h;
      iw0 = ow * g.stride_w - g.pad_w;
      pix = ((b * H + ih0) * W + iw0) * C;
    }
  }

  __device__ void Init(const T* b, int64_t ld_, int rows_, int K_) {
    base = b; ld = ld_; rows = rows_; K = K_;
    if constexpr (kMode == 0) {
      const int64_t bytes = (static_cast<int64_t>(rows - 1) * ld + K) * static_cast<int64_t>(sizeof(T));
      rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(b), 0, static_cast<int>(bytes), 0x00020000);
    }
  }

  __device__ __forceinline__ void Load(Regs& rg, int r0, int k0, int tid) const {
    if constexpr (kMode == 0) {
      // chunk q of the tile: row q / 8, 16-B chunk q % 8
#pragma unroll
      for (int i = 0; i < kVec; ++i) {
        const int q = tid + kThreads * i;
        const int r = r0 + (q >> 3), k = k0 + (q & 7) * EPV;
        const uint32_t off = (r < rows && k < K) ? static_cast<uint32_t>((r * ld + k) * static_cast<int64_t>(sizeof(T)))
                                                 : 0x80000000u;
        auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
        rg.v[i] = *reinterpret_cast<uint4*>(&v);
      }
    } else if constexpr (kMode == 1) {
#pragma unroll
      for (int i = 0; i < kElem; ++i) {
        const int q = tid + kThreads * i;
        const int r = r0 + q / BK, k = k0 + q % BK;
        rg.e[i] = (r < rows && k < K) ? base[r * ld + k] : FromF<T>(0.f);
      }
    } else if constexpr (kMode == 2) {
#pragma unroll
      for (int i = 0; i < kElem; ++i) {
        const int q = tid + kThreads * i;
        const int r = r0 + (q & (kBM - 1)), k = k0 + q / kBM;
        rg.e[i] = (r < rows && k < K) ? base[static_cast<int64_t>(k) * ld + r] : FromF<T>(0.f);
      }
    } else {
      // this thread's pixel, k = k0 + (tid / 64) * kElem ... + kElem - 1 as (tap r, s, channel c)
      int k = k0 + (tid >> 6) * kElem;
      int c = k % Cg, t = k / Cg;
      int s = t % S, r = t / S;
#pragma unroll
      for (int i = 0; i < kElem; ++i) {
        const int ih = ih0 + r * dh, iw = iw0 + s * dw;
        const bool ok = row_ok && k + i < K && ih >= 0 && ih < H && iw >= 0 && iw < W;
        rg.e[i] = ok ? base[pix + (r * dh * W + s * dw) * C + c] : FromF<T>(0.f);
        if (++c == Cg) {
          c = 0;
          if (++s == S) { s = 0; ++r; }
        }
      }
    }
  }

  __device__ __forceinline__ void Store(const Regs& rg, T* lds, int tid) const {
    constexpr int LD = GTile<T>::LD;
    if constexpr (kMode == 0) {
#pragma unroll
      for (int i = 0; i < kVec; ++i) {
        const int q = tid + kThreads * i;
        *reinterpret_cast<uint4*>(lds + (q >> 3) * LD + (q & 7) * EPV) = rg.v[i];
      }
    } else if constexpr (kMode == 1) {
#pragma unroll
      for (int i = 0; i < kElem; ++i) {
        const int q = tid + kThreads * i;
        lds[(q / BK) * LD + q % BK] = rg.e[i];
      }
    } else if constexpr (kMode == 2) {
#pragma unroll
      for (int i = 0; i < kElem; ++i) {
        const int q = tid + kThreads * i;
        lds[(q & (kBM - 1)) * LD + q / kBM] = rg.e[i];
      }
    } else {
      // one row, kElem consecutive k: whole 16-B chunks
      T* dst = lds + (tid & (kBM - 1)) * LD + (tid >> 6) * kElem;
#pragma unroll
      for (int i = 0; i < kElem; i += EPV) {
        uint4 v;
        __builtin_memcpy(&v, &rg.e[i], 16);
        *reinterpret_cast<uint4*>(dst + i) = v;
      }
    }
  }
};

template <class T, int kAM, int kBMd>
__global__ __launch_bounds__(kThreads) void gemm_mfma_kernel(GemmArgs g) {
  constexpr int BK = GTile<T>::BK, LD = GTile<T>::LD, EPV = GTile<T>::EPV;
  constexpr int WM = kBM / 2, WN = kBN / 2, TM = WM / 16, TN = WN / 16;
  __shared__ __attribute__((aligned(16))) T lds[2 * (kBM + kBN) * LD];
  T* As = lds;
  T* Bs = lds + 2 * kBM * LD;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int tiles_n = (g.N + kBN - 1) / kBN, tiles_m = (g.M + kBM - 1) / kBM;
  const int total = tiles_m * tiles_n;
  int bid = blockIdx.x;
  if ((total & 7) == 0) bid = (bid & 7) * (total >> 3) + (bid >> 3);  // XCD-contiguous tile runs
  const int tn = bid % tiles_n, tm = bid / tiles_n;
  const int m0 = tm * kBM, n0 = tn * kBN;
  const int bz = blockIdx.z;
  Operand<T, kAM> A;
  Operand<T, kBMd> B;
  A.Init(static_cast<const T*>(g.a) + bz * g.stride_a, g.lda, g.M, g.K);
  if constexpr (kAM == 3) A.InitConv(g, m0, tid);
  B.Init(static_cast<const T*>(g.b) + bz * g.stride_b, g.ldb, g.N, g.K);

  f4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const int wm0 = (wid >> 1) * WM, wn0 = (wid & 1) * WN;
  const int fr = lane & 15, fk = EPV * (lane >> 4);
  const int nk = (g.K + BK - 1) / BK;

  auto compute = [&](int buf) {
    if constexpr (sizeof(T) == 4) {
      // lane group lane >> 4 holds k = 4g..4g+3 of its A row and B column; MFMA c takes component c of both
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        f4 af[TM], bf[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[i] = *reinterpret_cast<const f4*>(As + (buf * kBM + wm0 + i * 16 + fr) * LD + ks * 16 + fk);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bf[j] = *reinterpret_cast<const f4*>(Bs + (buf * kBN + wn0 + j * 16 + fr) * LD + ks * 16 + fk);
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][c], bf[j][c], acc[i][j], 0, 0, 0);
      }
    } else {
      typedef typename std::conditional<std::is_same<T, _Float16>::value, h8, b8>::type V8;
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
        V8 af[TM], bf[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[i] = *reinterpret_cast<const V8*>(As + (buf * kBM + wm0 + i * 16 + fr) * LD + ks * 32 + fk);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bf[j] = *reinterpret_cast<const V8*>(Bs + (buf * kBN + wn0 + j * 16 + fr) * LD + ks * 32 + fk);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            if constexpr (std::is_same<T, _Float16>::value)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
            else
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
          }
      }
    }
  };

  typename Operand<T, kAM>::Regs ra;
  typename Operand<T, kBMd>::Regs rb;
  A.Load(ra, m0, 0, tid);
  B.Load(rb, n0, 0, tid);
  A.Store(ra, As, tid);
  B.Store(rb, Bs, tid);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) {
      A.Load(ra, m0, (kt + 1) * BK, tid);
      B.Load(rb, n0, (kt + 1) * BK, tid);
    }
    compute(buf);
    if (kt + 1 < nk) {
      A.Store(ra, As + (buf ^ 1) * kBM * LD, tid);
      B.Store(rb, Bs + (buf ^ 1) * kBN * LD, tid);
    }
    __syncthreads();
  }

  // epilogue: lane holds column n = n0 + wn0 + 16 j + (lane & 15) of rows 4 (lane >> 4) + r
  T* __restrict__ c = static_cast<T*>(g.c) + bz * g.stride_c;
  const T* __restrict__ cin = g.cmat ? static_cast<const T*>(g.cmat) + bz * g.stride_cm : nullptr;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn0 + j * 16 + fr;
    if (n >= g.N) continue;
    const float bn = g.bias ? g.beta * g.bias[bz * g.stride_bias + n] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm0 + i * 16 + 4 * (lane >> 4) + r;
        if (m >= g.M) continue;
        float v = g.alpha * acc[i][j][r] + bn;
        if (cin) v += g.beta * ToF(cin[m * g.ldcm + n]);
        if (g.act == 1) v = fmaxf(v, 0.f);
        c[m * g.ldc + n] = FromF<T>(v);
      }
  }
}

template <class T>
int LaunchGemm(const GemmArgs& g, hipStream_t st) {
  constexpr int EPV = GTile<T>::EPV;
  auto vec_ok = [](const void* p, int64_t ld, int K) {
    return reinterpret_cast<uintptr_t>(p) % 16 == 0 && ld % EPV == 0 && K % EPV == 0;
  };
  // buffer-resource extents are 32-bit: the vector path needs each batch's operand under 2 GB
  auto fits = [](int rows, int64_t ld, int K) {
    return (static_cast<int64_t>(rows) * ld + K) * static_cast<int64_t>(sizeof(T)) < (1ll << 31);
  };
  const int am = g.conv ? 3 : g.trans_a ? 2
                 : (vec_ok(g.a, g.lda, g.K) && (g.stride_a % EPV == 0) && fits(g.M, g.lda, g.K) ? 0 : 1);
  const int bm = !g.trans_b ? 2
                 : (vec_ok(g.b, g.ldb, g.K) && (g.stride_b % EPV == 0) && fits(g.N, g.ldb, g.K) ? 0 : 1);
  const int tiles = ((g.M + kBM - 1) / kBM) * ((g.N + kBN - 1) / kBN);
  const dim3 grid(tiles, 1, g.batch);
#define SML_GEMM_CASE(X, Y) \
  if (am == X && bm == Y) { hipLaunchKernelGGL((gemm_mfma_kernel<T, X, Y>), grid, dim3(kThreads), 0, st, g); return 0; }
  SML_GEMM_CASE(0, 0) SML_GEMM_CASE(0, 1) SML_GEMM_CASE(0, 2)
  SML_GEMM_CASE(1, 0) SML_GEMM_CASE(1, 1) SML_GEMM_CASE(1, 2)
  SML_GEMM_CASE(2, 0) SML_GEMM_CASE(2, 1) SML_GEMM_CASE(2, 2)
  SML_GEMM_CASE(3, 0) SML_GEMM_CASE(3, 1)
#undef SML_GEMM_CASE
  return -1;
}

}  // namespace

int GemmMfma(const GemmArgs& g, int dtype, void* stream) {
  if (g.M <= 0 || g.N <= 0 || g.batch <= 0) return 0;
  if (g.K < 0) return -2;
  if (static_cast<int64_t>(g.M) * g.ldc >= (1ll << 31) || static_cast<int64_t>(g.K) * g.M >= (1ll << 31) ||
      static_cast<int64_t>(g.K) * g.N >= (1ll << 31))
    if (!g.conv) return -5;  // 32-bit element indexing inside one batch
  if (g.conv) {
    if (g.R <= 0 || g.S <= 0 || g.K % (g.R * g.S) != 0 || g.OH <= 0 || g.OW <= 0 || g.trans_b != 1 ||
        g.M % (g.OH * g.OW) != 0)
      return -2;
    if (static_cast<int64_t>(g.M / (g.OH * g.OW)) * g.H * g.W * g.C >= (1ll << 31) ||
        static_cast<int64_t>(g.M) * g.ldc >= (1ll << 31) || static_cast<int64_t>(g.N) * g.ldb >= (1ll << 31))
      return -5;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  int rc = -1;
  if (dtype == 0) rc = LaunchGemm<float>(g, st);
  else if (dtype == 1) rc = LaunchGemm<_Float16>(g, st);
  else if (dtype == 2) rc = LaunchGemm<__bf16>(g, st);
  if (rc != 0) return rc;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace smlnn
