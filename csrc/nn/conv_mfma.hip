// Implicit-GEMM convolution on the CDNA4 matrix cores with fused prologue and
// epilogue (module _nn, used by the ONNX executor for NHWC fp32/fp16/bf16 graphs).
//
//   y[m, n]  = epi( sum_k pro(x_col[m, k]) * w[n, k] )
//   m = (b, oh, ow) output pixel, n = output channel, k = (r, s, c) tap x input
//   channel; x NHWC [B,H,W,C], w [Cout][R][S][C] (K contiguous), y NHWC.
//   pro(v) = relu(v * in_scale[c] + in_shift[c])   (pre-activation BN+ReLU;
//            padding taps stay 0, as in the unfused graph)
//   epi(v) = v + bias[n]; relu (relu=1); + res[m, n] (optional); relu (relu=2) -> y;
//            optional second output y2 = relu(y * out_scale[n] + out_shift[n])
//            (the next pre-activation block's input, written from registers).
//
// Tiling: 256 threads = 4 waves in 2x2, block tile BM x BN x 128 bytes of K
// (BK = 64 f16/bf16 or 32 f32 elements), wave tile (BM/2) x (BN/2) of 16x16x32
// f16/bf16 MFMAs, or of 16x16x4 f32 MFMAs (exact f32; gfx950 has no xf32), or - for f32 - of
// 16x16x32 bf16 MFMAs over operands split into 2 or 3 bf16 planes (kSplit: 3 or 6 products per
// pair; the 6-product form matches the exact f32 MFMA's error and is the fp32 graphs' default). A and B
// tiles are staged through registers (the prologue is applied there) into a
// double-buffered LDS image with a 160-byte row pitch (conflict-free ds_read_b128
// fragment reads; 144 B for the 32x32 forms); the next tile's global loads are issued before
// the current tile's MFMAs so HBM latency hides behind matrix work. Blocks are
// remapped so that each XCD owns a contiguous run of (m, n) tiles: the blocks
// that share an activation tile (all n for one m) sit on one XCD's L2.
// The f32 form reads one 16-B fragment per lane and operand (k = 4*(lane>>4)..+3)
// and issues four MFMAs from its components: A and B use the same k order, so
// the 16-k sum is the same set of products (k order within an fmaf chain).
// Requires C % BK == 0 (every ResNet conv but the 3-channel stem).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "nn_ops.h"

namespace smlnn {
namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int kBKBytes = 128;  // K extent of a tile row in bytes (8 16-B chunks)
constexpr int kThreads = 256;
// per element type: K elements per tile, elements per 16-B chunk (the LDS row pitch is set per kernel form)
template <class T>
struct Tile {
  static constexpr int BK = kBKBytes / static_cast<int>(sizeof(T));
  static constexpr int EPV = 16 / static_cast<int>(sizeof(T));
};

template <class T>
struct Vec;
template <>
struct Vec<_Float16> {
  typedef h8 type;
  static __device__ __forceinline__ f4 mfma(const h8& a, const h8& b, const f4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ f16v mfma32(const h8& a, const h8& b, const f16v& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};
template <>
struct Vec<__bf16> {
  typedef b8 type;
  static __device__ __forceinline__ f4 mfma(const b8& a, const b8& b, const f4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ f16v mfma32(const b8& a, const b8& b, const f16v& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};
template <>
struct Vec<float> {
  typedef f4 type;  // four consecutive k of one row: the operands of four 16x16x4 MFMAs
};

template <class T>
__device__ __forceinline__ float ToF(T v) {
  return static_cast<float>(v);
}
template <class T>
__device__ __forceinline__ T FromF(float v) {
  return static_cast<T>(v);
}

// Epilogue part 2, shared by the accumulator layouts: the wave's tile, staged in LDS (Ct, row pitch CL) as T
// after bias + ReLU, is read back in 16-B row chunks -> residual add, dual output, coalesced 16-B stores.
template <class T, int WM, int WN, int CL>
__device__ __forceinline__ void EpilogueStore(const ConvArgs& a, const T* Ct, int M, int m0, int n0, int wm0, int wn0,
                                              int lane) {
  T* __restrict__ y = static_cast<T*>(a.y);
  const T* __restrict__ res = static_cast<const T*>(a.res);
  T* __restrict__ y2 = static_cast<T*>(a.y2);
  const bool relu_post = a.relu == 2 && res != nullptr;
  constexpr int EPV = Tile<T>::EPV;
  constexpr int CPR = WN / EPV;
  constexpr int NIT = WM * CPR / 64;
  static_assert(64 % CPR == 0, "a lane keeps one channel chunk across the row iterations");
  // Every global load of the tile's epilogue (residual rows, second-output affine) is issued before the
  // first store: the plain per-row loop waited out one memory latency per row iteration (the compiler
  // cannot move a residual load above the previous row's output store), which memory-bound 1x1 layers
  // with a residual paid NIT times per tile.
  const int ch = lane % CPR;  // idx = it * 64 + lane: the chunk is the same in every iteration
  const int n = n0 + wn0 + ch * EPV;
  const bool n_ok = n < a.Cout;
  uint4 pv[NIT], rv[NIT];
  int64_t o[NIT];
  bool ok[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int row = (it * 64 + lane) / CPR;
    const int m = m0 + wm0 + row;
    ok[it] = m < M && n_ok;
    o[it] = static_cast<int64_t>(ok[it] ? m : 0) * a.Cout + (n_ok ? n : 0);
    pv[it] = *reinterpret_cast<const uint4*>(Ct + row * CL + ch * EPV);
    rv[it] = make_uint4(0, 0, 0, 0);
    if (res && ok[it]) rv[it] = *reinterpret_cast<const uint4*>(res + o[it]);
  }
  float os[EPV], ob[EPV];
  if (y2 && n_ok) {
#pragma unroll
    for (int e = 0; e < EPV; ++e) { os[e] = a.out_scale[n + e]; ob[e] = a.out_shift[n + e]; }
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    if (!ok[it]) continue;
    uint4 v = pv[it];
    if (res) {
      T* pe = reinterpret_cast<T*>(&v);
      const T* re = reinterpret_cast<const T*>(&rv[it]);
#pragma unroll
      for (int e = 0; e < EPV; ++e) {
        const float t = ToF(pe[e]) + ToF(re[e]);
        pe[e] = FromF<T>(relu_post ? fmaxf(t, 0.f) : t);
      }
    }
    *reinterpret_cast<uint4*>(y + o[it]) = v;
    if (y2) {
      uint4 qv;
      const T* pe = reinterpret_cast<const T*>(&v);
      T* qe = reinterpret_cast<T*>(&qv);
#pragma unroll
      for (int e = 0; e < EPV; ++e) qe[e] = FromF<T>(fmaxf(ToF(pe[e]) * os[e] + ob[e], 0.f));
      *reinterpret_cast<uint4*>(y2 + o[it]) = qv;
    }
  }
}

// Epilogue of the 32x32x16 MFMA layout (Cout % 8 == 0 only): lane holds column (lane & 31) of each 32x32
// block and rows 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3) in register r; bias + ReLU, staged through LDS.
template <class T, int WM, int WN, int kWN>
__device__ __forceinline__ void ConvEpilogue32(const ConvArgs& a, f16v (&acc)[WM / 32][WN / 32], T* lds, int M, int m0,
                                               int n0, int wid, int lane) {
  constexpr int TM = WM / 32, TN = WN / 32;
  const int wm0 = (wid / kWN) * WM, wn0 = (wid % kWN) * WN;
  const bool relu_pre = a.relu == 1 || (a.relu == 2 && a.res == nullptr);
  constexpr int CL = WN + 8;
  T* Ct = lds + wid * WM * CL;
  const int fc = lane & 31, fh = 4 * (lane >> 5);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn0 + j * 32 + fc;
    const float bn = (a.bias && n < a.Cout) ? a.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = acc[i][j][r] + bn;
        if (relu_pre) v = fmaxf(v, 0.f);
        Ct[(i * 32 + 8 * (r >> 2) + fh + (r & 3)) * CL + j * 32 + fc] = FromF<T>(v);
      }
  }
  __syncthreads();
  EpilogueStore<T, WM, WN, CL>(a, Ct, M, m0, n0, wm0, wn0, lane);
}

// Epilogue shared by the conv kernels: bias, ReLU, residual add and the optional second output,
// staged per wave through LDS (lds must hold 4 * (BM/2) * (BN/2 + 8) elements and be free).
template <class T, int WM, int WN, int kWN = 2>
__device__ __forceinline__ void ConvEpilogue(const ConvArgs& a, f4 (&acc)[WM / 16][WN / 16], T* lds, int M, int m0,
                                             int n0, int wid, int lane) {
  constexpr int TM = WM / 16, TN = WN / 16;
  const int wm0 = (wid / kWN) * WM, wn0 = (wid % kWN) * WN;
  const int fr = lane & 15;
  // epilogue part 1 (registers): lane holds column n = .. + (lane & 15), rows 4*(lane >> 4) + reg;
  // bias + ReLU in fp32, rounded to T (the unfused graph's conv output), staged per wave through LDS.
  T* __restrict__ y = static_cast<T*>(a.y);
  const T* __restrict__ res = static_cast<const T*>(a.res);
  T* __restrict__ y2 = static_cast<T*>(a.y2);
  // relu=1: before the residual add; relu=2: after it (identical without a residual)
  const bool relu_pre = a.relu == 1 || (a.relu == 2 && res == nullptr);
  const bool relu_post = a.relu == 2 && res != nullptr;
  if ((a.Cout & 7) == 0) {
    // staged row pitch (elements): 144 B for f16/bf16 (WN=64) and 16 B of padding for f32, so the
    // accumulator rows 4 apart that one 32-lane write group touches land on different banks
    constexpr int CL = WN + (sizeof(T) == 4 ? 4 : 8);
    T* Ct = lds + wid * WM * CL;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn0 + j * 16 + fr;
      const float bn = (a.bias && n < a.Cout) ? a.bias[n] : 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r] + bn;
          if (relu_pre) v = fmaxf(v, 0.f);
          Ct[(i * 16 + 4 * (lane >> 4) + r) * CL + j * 16 + fr] = FromF<T>(v);
        }
    }
    __syncthreads();
    EpilogueStore<T, WM, WN, CL>(a, Ct, M, m0, n0, wm0, wn0, lane);
    return;
  }
  // generic epilogue (Cout not a multiple of 8): element stores straight from the accumulators
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn0 + j * 16 + fr;
    if (n >= a.Cout) continue;
    const float bn = a.bias ? a.bias[n] : 0.f;
    const float os = a.out_scale ? a.out_scale[n] : 0.f, ob = a.out_scale ? a.out_shift[n] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm0 + i * 16 + 4 * (lane >> 4) + r;
        if (m >= M) continue;
        float v = acc[i][j][r] + bn;
        if (relu_pre) v = fmaxf(v, 0.f);
        const int64_t o = static_cast<int64_t>(m) * a.Cout + n;
        const T c = FromF<T>(v);
        const T vt = res ? FromF<T>(relu_post ? fmaxf(ToF(c) + ToF(res[o]), 0.f) : ToF(c) + ToF(res[o])) : c;
        y[o] = vt;
        if (y2) y2[o] = FromF<T>(fmaxf(ToF(vt) * os + ob, 0.f));
      }
    }
  }
}

// Split-K hand-off (after the K loop, LDS free): every split stores its fp32 partial tile (lane-natural
// layout, one coalesced 1-KiB store per accumulator and wave), publishes it (vmcnt(0), barrier, agent-scope
// release, then a relaxed agent-scope ticket add) and the split that draws the last ticket acquires, sums
// the partial tiles in split order (deterministic whatever the arrival order) and returns true to run the
// epilogue; the others return false.
template <class V, int TM, int TN, int kThr>
__device__ __forceinline__ bool SplitKReduce(const ConvArgs& a, V (&acc)[TM][TN], unsigned char* smem, int tile,
                                             int split, int SK, int tid) {
  constexpr int kTileF4 = kThr * TM * TN;  // accumulator vectors per partial tile
  V* mine = reinterpret_cast<V*>(a.ws) + (static_cast<int64_t>(tile) * SK + split) * kTileF4;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) mine[(i * TN + j) * kThr + tid] = acc[i][j];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(smem);
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int old = __hip_atomic_fetch_add(a.ws_cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = old == SK - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last ? 1 : 0;
  }
  __syncthreads();
  const bool last = *flag != 0;
  __syncthreads();  // the flag's LDS word is reused by the epilogue staging
  if (!last) return false;
  const V* base = reinterpret_cast<const V*>(a.ws) + static_cast<int64_t>(tile) * SK * kTileF4;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      V v = base[(i * TN + j) * kThr + tid];
      for (int s2 = 1; s2 < SK; ++s2) v += base[static_cast<int64_t>(s2) * kTileF4 + (i * TN + j) * kThr + tid];
      acc[i][j] = v;
    }
  return true;
}

// kThr = 256 (4 waves, 2x2) or 512 (8 waves, 4x2: the 256x128 / 128x256 tiles, one block per CU)
// kDepth 2: two register stages (tile kt+2's loads in flight during tile kt's MFMAs)
// kStem: a few-channel stem conv (the 3-channel ResNet stem, input padded to C = 4, weights packed to
// [Cout][8][8][4] with zero taps): a 16-B A chunk is two horizontally adjacent pixels (taps s, s+1 of row r),
// each read as its own 8-B buffer load (zero outside the image), a 64-wide K tile = two tap rows.
// kSplit (f32 only): 0 = exact f32 MFMAs; 2 / 3 = every f32 operand split into that many bf16 planes
// (x = x1 + x2 (+ x3), each the bf16 rounding of what the earlier planes left) and the product rebuilt from
// the 16x16x32 bf16 MFMAs of the plane pairs whose weight reaches the f32 rounding level: 3 products for 2
// planes (~16 significant bits per product), 6 for 3 planes (~24 bits, f32-class). One K tile (32 f32) is
// one 16x16x32 step per plane pair instead of eight 16x16x4 f32 MFMAs (1/16 of the bf16 rate on gfx950).
// kWPre (with kSplit): the weights arrive already split, a.w = [kSplit][Cout][R][S][C] bf16 planes (packed
// once per model by the executor): no split work for B at staging, 2 B per plane and element from HBM / L2.
// kWN: waves along N (2, or 1 for the Cout = 64 tiles whose 64x64 wave tiles halve the LDS fragment reads per
// MFMA against 32x32 ones: at 32x32 a wave issues one ds_read_b128 per 16-cycle MFMA, which is the LDS array's
// whole rate with a wave per SIMD)
// kM32 (f16 / bf16): 32x32x16 MFMAs (16 accumulators per lane per 32x32 block) instead of 16x16x32 - half the
// MFMA instructions for the same tile, the same LDS fragment bytes per MFMA FLOP
// kPersist: a grid of about one wave of resident blocks, each walking tiles q = blockIdx.x, + gridDim.x, ...;
// the next tile's first K-tile loads are issued before the current tile's epilogue, so the short-K layers
// (a 1x1 conv over 64-256 channels is one to four K tiles) keep HBM reads in flight behind their stores.
template <class T, int BM, int BN, bool kPro, int kThr = kThreads, int kDepth = 1, bool kStem = false, int kSplit = 0,
          bool kWPre = false, int kWN = 2, bool kM32 = false, bool kPersist = false>
__global__ __launch_bounds__(kThr) void conv_mfma_kernel(ConvArgs a) {
  typedef typename Vec<T>::type V8;
  constexpr int kBK = Tile<T>::BK, EPV = Tile<T>::EPV;
  // LDS row pitch: 160 B (32 B of padding) for the 16x16 fragment reads (row lane & 15, 16-B chunk lane >> 4):
  // under gfx950's ds_read_b128 lane groups ({0-3,12-15,20-27}, ...) a 144-B pitch puts two lanes of every
  // group on one bank (2-way, the ~32 % conflict cycles of the r2 PMC pass); 160 B is conflict-free. The
  // 32x32 fragments (row lane & 31, chunk lane >> 5) are conflict-free at 144 B and 2-way at 160 B.
  constexpr int kLd = kM32 ? kBK + EPV : kBK + 2 * EPV;
  constexpr int kWavesM = kThr / 64 / kWN;        // waves along M
  constexpr int WM = BM / kWavesM, WN = BN / kWN; // wave tile
  constexpr int TM = WM / 16, TN = WN / 16;     // 16x16 MFMA tiles per wave
  static_assert(!kM32 || (sizeof(T) == 2 && kSplit == 0 && !kStem && WM % 32 == 0 && WN % 32 == 0),
                "32x32x16 tiles: f16 / bf16, wave tiles in 32s");
  constexpr int TM32 = kM32 ? WM / 32 : 1, TN32 = kM32 ? WN / 32 : 1;  // 32x32 MFMA blocks per wave (kM32)
  constexpr int AR = BM * kBKBytes / 16 / kThr;  // 16-B A chunks per thread per tile
  constexpr int BR = BN * kBKBytes / 16 / kThr;  // 16-B B chunks per thread per tile
  constexpr int RS = kThr / 8;                  // tile rows covered by one pass of the block
  static_assert(kSplit == 0 || sizeof(T) == 4, "bf16 operand splitting is an f32 mode");
  // split planes: bf16 row pitch - 96 B is conflict-free for the 16x16 fragment reads (80 B is 2-way); the
  // 2-plane form keeps 80 B so that its 128x128 tile still fits two blocks per CU
  constexpr int kLdB = kSplit == 3 ? kBK + 16 : kBK + 8;
  constexpr int kOpBytes = kSplit ? 2 * kSplit * (BM + BN) * kLdB * 2 : 2 * (BM + BN) * kLd * static_cast<int>(sizeof(T));
  // the epilogue re-uses the operand buffers to stage each wave's tile
  constexpr int kEpiBytes = (kThr / 64) * WM * (WN + 8) * static_cast<int>(sizeof(T));
  static_assert(kSplit || kOpBytes >= kEpiBytes, "epilogue staging exceeds the LDS tile");
  __shared__ __attribute__((aligned(16))) unsigned char smem[kOpBytes > kEpiBytes ? kOpBytes : kEpiBytes];
  T* lds = reinterpret_cast<T*>(smem);
  T* As = lds;
  T* Bs = lds + 2 * BM * kLd;
  __bf16* Asb = reinterpret_cast<__bf16*>(smem);            // [plane][buf][BM][kLdB]
  __bf16* Bsb = Asb + 2 * (kSplit ? kSplit : 1) * BM * kLdB;  // [plane][buf][BN][kLdB]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int M = a.B * a.OH * a.OW;
  const int K = a.R * a.S * a.C;
  const int tiles_n = (a.Cout + BN - 1) / BN;
  const int tiles_m = (M + BM - 1) / BM;
  static_assert(!kPersist || (!kStem && kDepth == 1), "persistent form: register-staged, one stage");
  const int SK = (kStem || kPersist) ? 1 : a.split_k;  // K splits per tile (a tile's splits are adjacent block ids)
  const int total = tiles_m * tiles_n * SK;
  int split = 0, tile = 0, m0 = 0, n0 = 0;
  auto decode = [&](int q) {
    int bid = q;
    if ((total & 7) == 0) bid = (bid & 7) * (total >> 3) + (bid >> 3);  // XCD-contiguous tile runs
    split = bid % SK;
    bid /= SK;
    tile = bid;
    m0 = (bid / tiles_n) * BM;
    n0 = (bid % tiles_n) * BN;
  };
  int q = blockIdx.x;
  if (kPersist && q >= total) return;
  decode(q);

  // Operands are read through buffer resources: a lane whose tap falls in the padding (or whose row
  // is past M / channel past Cout) gets an out-of-range offset and the hardware returns zeros, so the
  // loads need no select and no branch. Per row the valid taps are a bit mask computed once; per
  // K tile a row costs one add, one bit test and one select (the tap / channel state is scalar).
  const int kc = tid & 7;  // 16-B chunk within the 64-wide k tile
  constexpr uint32_t kOob = 0x80000000u;
  int abase[AR];       // element offset of the row's window origin (tap 0, channel kc*8)
  uint64_t amask[AR];  // bit t: tap t = r*S + s is inside the input
  uint32_t boff[BR];   // byte offset of the thread's weight row chunk (out of range past Cout)
  constexpr int kWElem = kWPre ? 2 : static_cast<int>(sizeof(T));  // bytes per weight element (per plane)
  auto setup_rows = [&]() {
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int m = m0 + (tid >> 3) + RS * i;
    const int mm = m < M ? m : 0;
    const int ow = mm % a.OW, t2 = mm / a.OW;
    const int oh = t2 % a.OH, b = t2 / a.OH;
    const int ih0 = oh * a.stride_h - a.pad_h, iw0 = ow * a.stride_w - a.pad_w;
    abase[i] = ((b * a.H + ih0) * a.W + iw0) * a.C + (kStem ? 0 : kc * EPV);
    uint64_t mk = 0;
    if (m < M)
      for (int r = 0, t = 0; r < a.R; ++r)
        for (int s2 = 0; s2 < a.S; ++s2, ++t) {
          const int ih = ih0 + r * a.dil_h, iw = iw0 + s2 * a.dil_w;
          if (ih >= 0 && ih < a.H && iw >= 0 && iw < a.W) mk |= 1ull << t;
        }
    amask[i] = mk;
  }
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int n = n0 + (tid >> 3) + RS * i;
    boff[i] = n < a.Cout ? static_cast<uint32_t>((n * K + kc * EPV) * kWElem) : kOob;
  }
  };
  setup_rows();
  const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(a.x), 0, a.B * a.H * a.W * a.C * static_cast<int>(sizeof(T)), 0x00020000);
  const int wplane = a.Cout * K * kWElem;                             // bytes of one weight plane
  const __amdgpu_buffer_rsrc_t wres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(a.w), 0, wplane * (kWPre ? kSplit : 1), 0x00020000);
  constexpr bool pro = kPro;  // prologue affine present (a.in_scale != nullptr): a template
                              // parameter, so no runtime branch sits between loads and their use

  f4 acc[TM][TN];
  f16v acc32[TM32][TN32];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    if constexpr (kM32) {
#pragma unroll
      for (int i = 0; i < TM32; ++i)
#pragma unroll
        for (int j = 0; j < TN32; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc32[i][j][r] = 0.f;
    }
  };

  const int wm0 = (wid / kWN) * WM, wn0 = (wid % kWN) * WN;
  const int fr = lane & 15, fk = EPV * (lane >> 4);
  const int nk_all = K / kBK;
  const int kt0 = split * nk_all / SK;
  const int nk = (split + 1) * nk_all / SK - kt0;  // K tiles of this split

  auto compute = [&](int buf) {
    if constexpr (kSplit > 0) {
      // one 32-deep k step: lane group g = lane >> 4 holds k = 8g..8g+7 of its A row / B column per plane
      const int kb = 8 * (lane >> 4);
      b8 af[kSplit][TM], bf[kSplit][TN];
#pragma unroll
      for (int p = 0; p < kSplit; ++p) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[p][i] = *reinterpret_cast<const b8*>(Asb + ((p * 2 + buf) * BM + wm0 + i * 16 + fr) * kLdB + kb);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bf[p][j] = *reinterpret_cast<const b8*>(Bsb + ((p * 2 + buf) * BN + wn0 + j * 16 + fr) * kLdB + kb);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          // small terms first
          if constexpr (kSplit == 3) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[2][i], bf[0][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1][i], bf[1][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][i], bf[2][j], acc[i][j], 0, 0, 0);
          }
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1][i], bf[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][i], bf[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][i], bf[0][j], acc[i][j], 0, 0, 0);
        }
    } else if constexpr (sizeof(T) == 4) {
      // 16 k per step; lane group g = lane >> 4 holds k = 4g..4g+3 of its A row and B column, and MFMA c
      // takes component c of both: every (k, row, col) product is summed exactly once
#pragma unroll
      for (int ks = 0; ks < kBK / 16; ++ks) {
        f4 af[TM], bf[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[i] = *reinterpret_cast<const f4*>(As + (buf * BM + wm0 + i * 16 + fr) * kLd + ks * 16 + fk);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bf[j] = *reinterpret_cast<const f4*>(Bs + (buf * BN + wn0 + j * 16 + fr) * kLd + ks * 16 + fk);
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][c], bf[j][c], acc[i][j], 0, 0, 0);
      }
    } else if constexpr (kM32) {
      // 16 k per step; lane holds row / column (lane & 31), k = 8 * (lane >> 5) .. + 7 of the step
      const int f32r = lane & 31, f32k = 8 * (lane >> 5);
#pragma unroll
      for (int ks = 0; ks < kBK / 16; ++ks) {
        V8 af[TM32], bf[TN32];
#pragma unroll
        for (int i = 0; i < TM32; ++i)
          af[i] = *reinterpret_cast<const V8*>(As + (buf * BM + wm0 + i * 32 + f32r) * kLd + ks * 16 + f32k);
#pragma unroll
        for (int j = 0; j < TN32; ++j)
          bf[j] = *reinterpret_cast<const V8*>(Bs + (buf * BN + wn0 + j * 32 + f32r) * kLd + ks * 16 + f32k);
#pragma unroll
        for (int i = 0; i < TM32; ++i)
#pragma unroll
          for (int j = 0; j < TN32; ++j) acc32[i][j] = Vec<T>::mfma32(af[i], bf[j], acc32[i][j]);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < kBK / 32; ++ks) {
        V8 af[TM], bf[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[i] = *reinterpret_cast<const V8*>(As + (buf * BM + wm0 + i * 16 + fr) * kLd + ks * 32 + fk);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bf[j] = *reinterpret_cast<const V8*>(Bs + (buf * BN + wn0 + j * 16 + fr) * kLd + ks * 32 + fk);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = Vec<T>::mfma(af[i], bf[j], acc[i][j]);
      }
    }
  };

  // The global loads of tile kt+1 are issued before the MFMAs of tile kt and consumed (written to
  // LDS) after them. The prologue affine is applied at that LDS write, not at the load, so prologue
  // layers keep the same overlap (its per-channel scale/shift are loaded with the tile). (A two-stage
  // register pipeline - tile kt+2 in flight - measured 7 % slower: profiles/r2_onnx/README.)
  constexpr int NQ = EPV / 4;  // float4s of prologue scale (and of shift) per 16-B chunk
  struct Stage {
    uint4 a[AR], b[BR];
    uint2 bp[kWPre ? kSplit : 1][kWPre ? BR : 1];  // pre-split weight planes: 4 bf16 per plane and chunk
    f4 q[2 * NQ];
    unsigned okm;
  };
  // next tile to load: tap (lr, ls) = index lt, channel offset lc0, element offset of the tap toff
  int lt = 0, lr = 0, ls = 0, lc0 = 0, lk0 = 0, toff = 0, loaded = 0;
  auto reset_taps = [&]() {
    lt = lr = ls = lc0 = lk0 = toff = loaded = 0;
    if (kt0 > 0) {  // a later split starts inside the (tap, channel) walk
      lk0 = kt0 * kBK;
      lt = lk0 / a.C;
      lc0 = lk0 - lt * a.C;
      lr = lt / a.S;
      ls = lt - lr * a.S;
      toff = (lr * a.dil_h * a.W + ls * a.dil_w) * a.C;
    }
  };
  reset_taps();
  auto load_tile = [&](Stage& st) {
    st.okm = 0;
    if constexpr (kStem) {
      const int r = 2 * loaded + (kc >> 2), s0 = 2 * (kc & 3), t0 = r * 8 + s0;
      const int toff_s = (r * a.W + s0) * 4;  // element offset of tap (r, s0) from the window origin
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        const uint32_t o0 = (amask[i] >> t0) & 1ull ? static_cast<uint32_t>((abase[i] + toff_s) * 2) : kOob;
        const uint32_t o1 = (amask[i] >> (t0 + 1)) & 1ull ? static_cast<uint32_t>((abase[i] + toff_s + 4) * 2) : kOob;
        auto lo = __builtin_amdgcn_raw_buffer_load_b64(xres, o0, 0, 0);
        auto hi = __builtin_amdgcn_raw_buffer_load_b64(xres, o1, 0, 0);
        st.a[i] = make_uint4(lo[0], lo[1], hi[0], hi[1]);
      }
    } else {
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const bool ok = (amask[i] >> lt) & 1ull;
      st.okm |= ok ? (1u << i) : 0u;
      const uint32_t vo = ok ? static_cast<uint32_t>((abase[i] + toff) * static_cast<int>(sizeof(T))) : kOob;
      auto v = __builtin_amdgcn_raw_buffer_load_b128(xres, vo, lc0 * static_cast<int>(sizeof(T)), 0);
      st.a[i] = *reinterpret_cast<uint4*>(&v);
    }
    }
    if constexpr (pro) {
      const f4* scp = reinterpret_cast<const f4*>(a.in_scale + lc0 + kc * EPV);
      const f4* shp = reinterpret_cast<const f4*>(a.in_shift + lc0 + kc * EPV);
#pragma unroll
      for (int t = 0; t < NQ; ++t) {
        st.q[t] = scp[t];
        st.q[NQ + t] = shp[t];
      }
    }
    if constexpr (kWPre) {
#pragma unroll
      for (int p = 0; p < kSplit; ++p)
#pragma unroll
        for (int i = 0; i < BR; ++i) {
          auto v = __builtin_amdgcn_raw_buffer_load_b64(wres, boff[i] + static_cast<uint32_t>(p * wplane), lk0 * 2, 0);
          st.bp[p][i] = make_uint2(v[0], v[1]);
        }
    } else {
#pragma unroll
      for (int i = 0; i < BR; ++i) {
        auto v = __builtin_amdgcn_raw_buffer_load_b128(wres, boff[i], lk0 * static_cast<int>(sizeof(T)), 0);
        st.b[i] = *reinterpret_cast<uint4*>(&v);
      }
    }
    // advance to the next K tile (64 more channels, or the next tap)
    if (++loaded < nk) {
      lk0 += kBK;
      lc0 += kBK;
      if (lc0 == a.C) {
        lc0 = 0;
        ++lt;
        if (++ls == a.S) {
          ls = 0;
          ++lr;
        }
        toff = (lr * a.dil_h * a.W + ls * a.dil_w) * a.C;
      }
    }
  };
  // split planes: 4 f32 -> kSplit x 4 bf16 (8 B per plane), x_p = bf16(x - x_1 - ... - x_{p-1})
  auto store_split = [&](__bf16* base, int rows, int buf, int row, const uint4& v) {
    const float* e = reinterpret_cast<const float*>(&v);
    float r[4] = {e[0], e[1], e[2], e[3]};
#pragma unroll
    for (int p = 0; p < (kSplit ? kSplit : 1); ++p) {
      __bf16 q[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        q[t] = static_cast<__bf16>(r[t]);
        r[t] -= static_cast<float>(q[t]);
      }
      *reinterpret_cast<uint2*>(base + ((p * 2 + buf) * rows + row) * kLdB + kc * 4) = *reinterpret_cast<const uint2*>(q);
    }
  };
  auto store_tile = [&](int buf, const Stage& st) {
    if constexpr (kSplit > 0) {
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        uint4 v = st.a[i];
        if constexpr (pro) {
          float* e = reinterpret_cast<float*>(&v);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float t = e[j] * st.q[0][j] + st.q[NQ][j];
            e[j] = a.prologue_relu ? fmaxf(t, 0.f) : t;
          }
          const unsigned mk = 0u - ((st.okm >> i) & 1u);
          v.x &= mk; v.y &= mk; v.z &= mk; v.w &= mk;
        }
        store_split(Asb, BM, buf, (tid >> 3) + RS * i, v);
      }
      if constexpr (kWPre) {
#pragma unroll
        for (int p = 0; p < kSplit; ++p)
#pragma unroll
          for (int i = 0; i < BR; ++i)
            *reinterpret_cast<uint2*>(Bsb + ((p * 2 + buf) * BN + (tid >> 3) + RS * i) * kLdB + kc * 4) = st.bp[p][i];
      } else {
#pragma unroll
        for (int i = 0; i < BR; ++i) store_split(Bsb, BN, buf, (tid >> 3) + RS * i, st.b[i]);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      uint4 v = st.a[i];
      if constexpr (pro) {
        T* e = reinterpret_cast<T*>(&v);
#pragma unroll
        for (int j = 0; j < EPV; ++j) {
          const float t = ToF(e[j]) * st.q[j >> 2][j & 3] + st.q[NQ + (j >> 2)][j & 3];
          e[j] = FromF<T>(a.prologue_relu ? fmaxf(t, 0.f) : t);
        }
        const unsigned mk = 0u - ((st.okm >> i) & 1u);  // padding taps stay 0, as in the unfused graph
        v.x &= mk; v.y &= mk; v.z &= mk; v.w &= mk;
      }
      *reinterpret_cast<uint4*>(As + (buf * BM + (tid >> 3) + RS * i) * kLd + kc * EPV) = v;
    }
#pragma unroll
    for (int i = 0; i < BR; ++i)
      *reinterpret_cast<uint4*>(Bs + (buf * BN + (tid >> 3) + RS * i) * kLd + kc * EPV) = st.b[i];
  };
  Stage s0;
  load_tile(s0);
  for (;;) {  // one pass unless kPersist
  zero_acc();
  store_tile(0, s0);
  if constexpr (kDepth == 2) {
    Stage s1;
    if (nk > 1) load_tile(s1);
    __syncthreads();
    // step kt: tile kt+1 sits in `nxt`, tile kt+2 is loaded into `far` (whose tile was stored last step)
    auto step = [&](int kt, Stage& nxt, Stage& far) {
      if (kt + 2 < nk) load_tile(far);
      compute(kt & 1);
      if (kt + 1 < nk) store_tile((kt & 1) ^ 1, nxt);
      __syncthreads();
    };
    for (int kt = 0; kt < nk; kt += 2) {
      step(kt, s1, s0);
      if (kt + 1 < nk) step(kt + 1, s0, s1);
    }
  } else {
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < nk) load_tile(s0);
      compute(buf);
      if (kt + 1 < nk) store_tile(buf ^ 1, s0);
      __syncthreads();
    }
  }

  const int em0 = m0, en0 = n0;  // this tile's origin (the prefetch below moves to the next tile)
  int qn = total;
  if constexpr (kPersist) {
    qn = q + static_cast<int>(gridDim.x);
    if (qn < total) {  // next tile's first K-tile loads in flight behind this tile's epilogue
      decode(qn);
      setup_rows();
      reset_taps();
      load_tile(s0);
    }
  }
  if constexpr (kM32) {
    if (SK > 1 && !SplitKReduce<f16v, TM32, TN32, kThr>(a, acc32, smem, tile, split, SK, tid)) return;
    ConvEpilogue32<T, WM, WN, kWN>(a, acc32, lds, M, em0, en0, wid, lane);
  } else {
    if (SK > 1 && !SplitKReduce<f4, TM, TN, kThr>(a, acc, smem, tile, split, SK, tid)) return;
    ConvEpilogue<T, WM, WN, kWN>(a, acc, lds, M, em0, en0, wid, lane);
  }
  if (!kPersist || qn >= total) break;
  q = qn;
  __syncthreads();  // the epilogue's LDS staging is read before the next tile's operands land there
  }
}

// LDS-DMA form (f16 / bf16): the A and B tiles go global -> LDS with buffer_load ... lds
// (16 B per lane, one 1-KiB wave-instruction = 8 tile rows of 128 B), so staging takes no VGPRs and no
// ds_write (whose 13-cycle wave-instruction transfer, at ~79 B/clk/CU, is as long as the tile's fragment
// reads). A DMA lands lane-linear, so the rows are unpadded 128-B lines and the bank spread comes from an XOR
// swizzle applied on the SOURCE side: lane l of an 8-row piece loads chunk (l & 7) ^ row%8 of its row, i.e.
// chunk c of row r sits at slot c ^ (r & 7); the fragment reads apply the same XOR (conflict-free 16-lane
// ds_read_b128 groups). Out-of-range rows / padding taps load from an out-of-range buffer offset: zeros.
// Tile kt+1's DMAs are issued before tile kt's MFMAs; a vmcnt(0) + barrier per K tile retires them.
// kPro (1x1, unpadded layers only: no padding tap must stay 0): the pre-activation BN + ReLU of the input
// is applied to the A fragments as they leave LDS (each A element is read by the kWN waves of its row
// band); the tile's 64 channels of scale / shift ride the same DMA into a 2 x 2 KiB side buffer.
// 16 B per lane from a buffer resource straight into LDS at the wave-uniform dst (+ 16 * lane): the
// LDS-address-space builtin exists in the device pass only (the host pass just needs the kernel's stub)
__device__ __forceinline__ void DmaToLds16(__amdgpu_buffer_rsrc_t r, void* dst, uint32_t voff, uint32_t soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(dst), 16, voff, soff, 0, 0);
#endif
}

// (r5 pass 13 A/B, ResNet-50 b128 per layer: issuing the next tile's A pieces before k-step 0 and its B pieces
// before k-step 1 - with or without s_setprio around the MFMA groups - measured 2-10 % slower than issuing
// them all ahead of the tile's MFMAs, so the pieces stay together)
template <class T, int BM, int BN, int kThr, int kWN, bool kPro = false, int kNB = 2>
__global__ __launch_bounds__(kThr) void conv_glds_kernel(ConvArgs a) {
  typedef typename Vec<T>::type V8;
  static_assert(sizeof(T) == 2, "LDS-DMA conv is the f16 / bf16 form");
  constexpr int kBK = 64, EPV = 8;
  constexpr int NW = kThr / 64;
  constexpr int kWavesM = NW / kWN;
  constexpr int WM = BM / kWavesM, WN = BN / kWN;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int AI = BM / 8 / NW, BI = BN / 8 / NW;  // 8-row DMA pieces per wave and tile
  static_assert(AI * 8 * NW == BM && BI * 8 * NW == BN, "tile rows must split into 8-row pieces per wave");
  // kNB LDS buffers: 2 (tile kt + 1 lands while kt computes), 1 for a single-K-tile layer (the 1x1 layers on
  // 64 channels): half the LDS, twice the resident blocks to hide their memory-bound epilogue
  constexpr int kOpBytes = kNB * (BM + BN) * kBK * 2;
  constexpr int kProBytes = kPro ? 2 * 2 * 1024 : 0;  // [buf][scale | shift][256 floats]: one DMA each
  constexpr int kEpiBytes = NW * WM * (WN + 8) * 2;
  __shared__ __attribute__((aligned(16)))
  unsigned char smem[kOpBytes + kProBytes > kEpiBytes ? kOpBytes + kProBytes : kEpiBytes];
  T* lds = reinterpret_cast<T*>(smem);
  T* As = lds;                 // [buf][BM][64], swizzled chunks
  T* Bs = lds + kNB * BM * kBK;  // [buf][BN][64]
  float* Ps = reinterpret_cast<float*>(smem + kOpBytes);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int M = a.B * a.OH * a.OW;
  const int K = a.R * a.S * a.C;
  const int tiles_n = (a.Cout + BN - 1) / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int total = tiles_m * tiles_n;
  int bid = blockIdx.x;
  if ((total & 7) == 0) bid = (bid & 7) * (total >> 3) + (bid >> 3);  // XCD-contiguous tile runs
  const int tn = bid % tiles_n, tm = bid / tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const int prow = lane >> 3;                 // row within an 8-row piece (= row % 8)
  const int kcs = (lane & 7) ^ prow;          // the chunk this lane fetches (source-side swizzle)
  constexpr uint32_t kOob = 0x80000000u;
  int abase[AI];
  uint64_t amask[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int m = m0 + (wid * AI + i) * 8 + prow;
    const int mm = m < M ? m : 0;
    const int ow = mm % a.OW, t2 = mm / a.OW;
    const int oh = t2 % a.OH, b = t2 / a.OH;
    const int ih0 = oh * a.stride_h - a.pad_h, iw0 = ow * a.stride_w - a.pad_w;
    abase[i] = ((b * a.H + ih0) * a.W + iw0) * a.C + kcs * EPV;
    uint64_t mk = 0;
    if (m < M)
      for (int r = 0, t = 0; r < a.R; ++r)
        for (int s2 = 0; s2 < a.S; ++s2, ++t) {
          const int ih = ih0 + r * a.dil_h, iw = iw0 + s2 * a.dil_w;
          if (ih >= 0 && ih < a.H && iw >= 0 && iw < a.W) mk |= 1ull << t;
        }
    amask[i] = mk;
  }
  const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(a.x), 0, a.B * a.H * a.W * a.C * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t wres = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.w), 0, a.Cout * K * 2, 0x00020000);
  // prologue scale / shift (unused, and dropped by the compiler, without kPro)
  const __amdgpu_buffer_rsrc_t sres = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.in_scale), 0, a.C * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t hres = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.in_shift), 0, a.C * 4, 0x00020000);
  uint32_t boff[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int n = n0 + (wid * BI + i) * 8 + prow;
    boff[i] = n < a.Cout ? static_cast<uint32_t>((n * K + kcs * EPV) * 2) : kOob;
  }

  f4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  const int wm0 = (wid / kWN) * WM, wn0 = (wid % kWN) * WN;
  const int fr = lane & 15;
  const int nk = K / kBK;

  int lt = 0, lr = 0, ls = 0, lc0 = 0, lk0 = 0, toff = 0, loaded = 0;
  // DMA of the next K tile into LDS buffer `buf` (wave-uniform destination: 8 rows of 128 B per piece)
  auto dma_a = [&](int buf) {
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const bool ok = (amask[i] >> lt) & 1ull;
      const uint32_t vo = ok ? static_cast<uint32_t>((abase[i] + toff) * 2) : kOob;
      DmaToLds16(xres, As + (buf * BM + (wid * AI + i) * 8) * kBK, vo, lc0 * 2);
    }
  };
  auto dma_b = [&](int buf) {
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      DmaToLds16(wres, Bs + (buf * BN + (wid * BI + i) * 8) * kBK, boff[i], lk0 * 2);
    }
    if constexpr (kPro) {
      if (wid == 0) {  // lanes 0-15: the tile's 64 channels (1x1: channel = k); the rest land zeros
        const uint32_t po = lane < 16 ? static_cast<uint32_t>(lane * 16) : kOob;
        DmaToLds16(sres, Ps + buf * 512, po, lc0 * 4);
        DmaToLds16(hres, Ps + buf * 512 + 256, po, lc0 * 4);
      }
    }
  };
  auto advance = [&]() {
    if (++loaded < nk) {
      lk0 += kBK;
      lc0 += kBK;
      if (lc0 == a.C) {
        lc0 = 0;
        ++lt;
        if (++ls == a.S) {
          ls = 0;
          ++lr;
        }
        toff = (lr * a.dil_h * a.W + ls * a.dil_w) * a.C;
      }
    }
  };
  auto dma_tile = [&](int buf) {
    dma_a(buf);
    dma_b(buf);
    advance();
  };
  auto compute_ks = [&](int buf, int ks) {
    {
      const int c = ks * 4 + (lane >> 4);  // 16-B chunk of the lane's k range
      V8 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm0 + i * 16 + fr;
        af[i] = *reinterpret_cast<const V8*>(As + (buf * BM + r) * kBK + ((c ^ (r & 7)) * EPV));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn0 + j * 16 + fr;
        bf[j] = *reinterpret_cast<const V8*>(Bs + (buf * BN + r) * kBK + ((c ^ (r & 7)) * EPV));
      }
      if constexpr (kPro) {
        // channels c * 8 .. c * 8 + 7 of the tile (16 lanes share them: broadcast reads)
        const float4* ps = reinterpret_cast<const float4*>(Ps + buf * 512 + c * EPV);
        const float4 s0 = ps[0], s1 = ps[1], h0 = ps[64], h1 = ps[65];
        const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          T* e = reinterpret_cast<T*>(&af[i]);
#pragma unroll
          for (int j = 0; j < EPV; ++j) {
            const float t = ToF(e[j]) * sc[j] + sh[j];
            e[j] = FromF<T>(a.prologue_relu ? fmaxf(t, 0.f) : t);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = Vec<T>::mfma(af[i], bf[j], acc[i][j]);
    }
  };
  auto compute = [&](int buf) {
#pragma unroll
    for (int ks = 0; ks < kBK / 32; ++ks) compute_ks(buf, ks);
  };
  if constexpr (kNB == 3) {
    // Three buffers, two tiles in flight across the barrier: at step kt a wave retires only its own DMAs of
    // tile kt (counted vmcnt: the kPieces of tile kt + 1 may stay outstanding), the raw s_barrier then makes
    // every wave's tile kt visible AND proves every wave is past compute(kt - 1), so tile kt + 2 may land in
    // that buffer. No __syncthreads() in the loop: its fence would drain the DMA queue (vmcnt(0)).
    constexpr int kPieces = AI + BI;
    static_assert(!kPro, "the 3-buffer form has no prologue side buffer");
    dma_tile(0);
    if (nk > 1) dma_tile(1);
    int buf = 0;
    for (int kt = 0; kt < nk; ++kt) {
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(kPieces) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 2 < nk) dma_tile(buf == 0 ? 2 : buf - 1);
      compute(buf);
      buf = buf == 2 ? 0 : buf + 1;
    }
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();  // the epilogue's LDS staging overwrites the operand buffers
  } else {
    dma_tile(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < nk) dma_tile(buf ^ 1);
      compute(buf);
      __builtin_amdgcn_sched_barrier(0);  // keep the tile's MFMAs ahead of the DMA wait
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  ConvEpilogue<T, WM, WN, kWN>(a, acc, lds, M, m0, n0, wid, lane);
}

// persistent form: about one wave of resident blocks (occupancy x CUs), each walking tiles with the next
// tile's loads overlapped with the current epilogue
template <class T, int BM, int BN, int kThr>
void LaunchPersist(const ConvArgs& a, int M, hipStream_t st) {
  const int total = ((M + BM - 1) / BM) * ((a.Cout + BN - 1) / BN);
  auto kp = conv_mfma_kernel<T, BM, BN, true, kThr, 1, false, 0, false, 2, false, true>;
  auto kn = conv_mfma_kernel<T, BM, BN, false, kThr, 1, false, 0, false, 2, false, true>;
  auto resident = [](decltype(kp) k) {
    int dev = 0, ncu = 0, nb = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      ncu = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, kThr, 0) != hipSuccess || nb < 1) nb = 1;
    return nb * ncu;
  };
  static const int res_p = resident(kp), res_n = resident(kn);
  auto k = a.in_scale ? kp : kn;
  const int res = a.in_scale ? res_p : res_n;
  const int grid = total < res ? total : res;
  hipLaunchKernelGGL(k, dim3(grid), dim3(kThr), 0, st, a);
}

template <class T, int BM, int BN, int kThr, int kWN = 2>
void LaunchGlds(const ConvArgs& a, int M, hipStream_t st) {
  const int blocks = ((M + BM - 1) / BM) * ((a.Cout + BN - 1) / BN);
  static const bool single = [] {
    const char* e = std::getenv("SML_CONV_GLDS_SINGLE");
    return !e || std::atoi(e) != 0;
  }();
  // SML_CONV_GLDS_NB=2 / 3 forces a depth; unset: three buffers only for launches of at most one block per CU.
  // r5 passes 10 / 13, ResNet-50 b128 per layer: the 3-buffer form halves the resident 128x128 blocks (96 KB
  // of LDS), which costs every layer with more blocks than CUs 10-40 % (occupancy hid more than the pipeline
  // does; the 392-block 256 3x3 at 14x14: 39.6 -> 52-56 us), and wins where the grid is below one block per
  // CU anyway (the 196-block 512 3x3 at 7x7: 52.9 -> 46.7 us; 2048 -> 512 1x1: 27.9 -> 23.1 us)
  static const int nb = [] {
    const char* e = std::getenv("SML_CONV_GLDS_NB");
    return e ? std::atoi(e) : 0;
  }();
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return n;
  }();
  const bool deep = nb == 3 || (nb == 0 && blocks <= ncu);

  if (a.in_scale) hipLaunchKernelGGL((conv_glds_kernel<T, BM, BN, kThr, kWN, true>), dim3(blocks), dim3(kThr), 0, st, a);
  else if (deep && a.R * a.S * a.C >= 3 * 64)  // two K tiles in flight across the barrier
    hipLaunchKernelGGL((conv_glds_kernel<T, BM, BN, kThr, kWN, false, 3>), dim3(blocks), dim3(kThr), 0, st, a);
  else if (single && a.R * a.S * a.C == 64)  // one K tile: no second buffer to fill (SML_CONV_GLDS_SINGLE=0: off)
    hipLaunchKernelGGL((conv_glds_kernel<T, BM, BN, kThr, kWN, false, 1>), dim3(blocks), dim3(kThr), 0, st, a);
  else hipLaunchKernelGGL((conv_glds_kernel<T, BM, BN, kThr, kWN>), dim3(blocks), dim3(kThr), 0, st, a);
}

// the LDS-DMA form applies a prologue only where no padding tap exists (1x1, unpadded)
inline bool GldsProOk(const ConvArgs& a) {
  return !a.in_scale || (a.R == 1 && a.S == 1 && a.pad_h == 0 && a.pad_w == 0);
}

template <class T, int BM, int BN, int kThr = kThreads, int kSplit = 0, bool kWPre = false, int kWN = 2,
          bool kM32 = false>
void LaunchTile(const ConvArgs& a, int M, hipStream_t st) {
  const int blocks = ((M + BM - 1) / BM) * ((a.Cout + BN - 1) / BN) * a.split_k;
  // f32 64x64: two register stages when the K loop is long enough and there is no prologue (the prologue
  // variant drops to 3 waves/SIMD at depth 2); r2_convdepth A/B: 2615-2623 -> 2536-2541 us over the 14
  // shapes, the short-K layers (C=64/256 1x1) a little slower. SML_CONV_DEPTH=1/2 forces one.
  static const int depth = [] {
    const char* e = std::getenv("SML_CONV_DEPTH");
    return e ? std::atoi(e) : 0;
  }();
  if constexpr (sizeof(T) == 4 && BM == 64 && BN == 64) {
    const int nk = a.R * a.S * a.C / Tile<T>::BK;
    if (depth == 2 || (depth == 0 && !a.in_scale && nk > 8)) {
      auto k2 = a.in_scale ? conv_mfma_kernel<T, BM, BN, true, kThr, 2, false, kSplit, kWPre>
                           : conv_mfma_kernel<T, BM, BN, false, kThr, 2, false, kSplit, kWPre>;
      hipLaunchKernelGGL(k2, dim3(blocks), dim3(kThr), 0, st, a);
      return;
    }
  }
  auto k = a.in_scale ? conv_mfma_kernel<T, BM, BN, true, kThr, 1, false, kSplit, kWPre, kWN, kM32>
                      : conv_mfma_kernel<T, BM, BN, false, kThr, 1, false, kSplit, kWPre, kWN, kM32>;
  hipLaunchKernelGGL(k, dim3(blocks), dim3(kThr), 0, st, a);
}

int EnvTile() {
  static const int t = [] {
    const char* e = std::getenv("SML_CONV_TILE");
    if (!e) return 0;
    const int bm = std::atoi(e);
    const char* x = std::strchr(e, 'x');
    return x ? bm * 1000 + std::atoi(x + 1) : 0;
  }();
  return t;
}

bool EnvPersist() {
  static const bool p = [] {
    const char* e = std::getenv("SML_CONV_PERSIST");
    return e && std::atoi(e) != 0;
  }();
  return p;
}

// LDS-DMA staging is the default for the f16/bf16 layers without a prologue (r4 per-layer sweep over the 14
// ResNet-50 shapes: every shape but the 2048->512 1x1 at least as fast as register staging, -10 % in total);
// SML_CONV_GLDS=0 restores register staging
bool EnvGlds() {
  static const bool g = [] {
    const char* e = std::getenv("SML_CONV_GLDS");
    return !e || std::atoi(e) != 0;
  }();
  return g;
}

// SML_CONV_GLDS_PRO=1: the LDS-DMA form for the 1x1 prologue layers too (off: r4 pass 9, ResNet-50 fp16
// b128, the 20 prologue convs took 1112 us on it vs 1028 us register-staged - the affine at fragment read
// runs kWN times per element plus the scale / shift reads, against once per element at the register
// path's LDS write; session 39.7k vs 40.4k img/s)
bool EnvGldsPro() {
  static const bool g = [] {
    const char* e = std::getenv("SML_CONV_GLDS_PRO");
    return e && std::atoi(e) != 0;
  }();
  return g;
}

template <class T, int kSplit = 0, bool kWPre = false>
int Launch(const ConvArgs& a, hipStream_t st) {
  const int M = a.B * a.OH * a.OW;
  // SML_CONV_TILE=BMxBN forces one register-staged tile shape for the process (tuning sweeps);
  // ConvArgs::kernel forces a kernel per call (tests)
  const int env_tile = EnvTile();
  if (a.split_k > 1 && (a.kernel || env_tile || !a.ws || !a.ws_cnt)) return -6;  // split-K: planned tiles only
  switch (a.kernel ? a.kernel : env_tile) {
    case 64064: LaunchTile<T, 64, 64, kThreads, kSplit, kWPre>(a, M, st); return 0;
    case 128064: LaunchTile<T, 128, 64, kThreads, kSplit, kWPre>(a, M, st); return 0;
    case 64128: LaunchTile<T, 64, 128, kThreads, kSplit, kWPre>(a, M, st); return 0;
    case 128128: LaunchTile<T, 128, 128, kThreads, kSplit, kWPre>(a, M, st); return 0;
    case 128999: LaunchTile<T, 128, 128, 512, kSplit, kWPre>(a, M, st); return 0;  // 128x128, 8 waves (4x2, 32x64 each)
    case 64999: LaunchTile<T, 64, 64, 512, kSplit, kWPre>(a, M, st); return 0;     // 64x64, 8 waves (4x2, 16x32 each)
    case 128555:  // persistent forms (tile walk, next tile's loads behind the epilogue): 128x128 8 waves, 64x64
    case 64555:
      if constexpr (kSplit == 0 && sizeof(T) == 2) {
        if (a.split_k != 1) return -4;
        if ((a.kernel ? a.kernel : env_tile) == 128555) LaunchPersist<T, 128, 128, 512>(a, M, st);
        else LaunchPersist<T, 64, 64, 256>(a, M, st);
        return 0;
      }
      return -4;
    case 128932:  // 32x32x16 MFMA forms: 128x128 8 waves (32x64), 256x128 8 waves (64x64), 64x64 4 waves (32x32)
    case 256932:
    case 64932:
      if constexpr (sizeof(T) == 2 && kSplit == 0) {
        if (a.Cout & 7) return -4;
        const int code = a.kernel ? a.kernel : env_tile;
        if (code == 128932) LaunchTile<T, 128, 128, 512, 0, false, 2, true>(a, M, st);
        else if (code == 256932) LaunchTile<T, 256, 128, 512, 0, false, 2, true>(a, M, st);
        else LaunchTile<T, 64, 64, 256, 0, false, 2, true>(a, M, st);
        return 0;
      }
      return -4;
    case 128777:  // LDS-DMA forms (f16 / bf16 without prologue): 128x128 8 waves, 64x64 4 waves, 256x64 4 waves
    case 64777:
    case 256777:
      if constexpr (sizeof(T) == 2 && kSplit == 0) {
        if (!GldsProOk(a) || a.split_k != 1) return -4;
        const int code = a.kernel ? a.kernel : env_tile;
        if (code == 128777) LaunchGlds<T, 128, 128, 512>(a, M, st);
        else if (code == 64777) LaunchGlds<T, 64, 64, 256>(a, M, st);
        else LaunchGlds<T, 256, 64, 256, 1>(a, M, st);
        return 0;
      }
      return -4;
    case 256064:  // 256x64, 4 waves (4x1, 64x64 each)
    case 128164:  // 128x64, 2 waves (2x1, 64x64 each)
      if constexpr (sizeof(T) == 2 && kSplit == 0) {
        if ((a.kernel ? a.kernel : env_tile) == 256064) LaunchTile<T, 256, 64, 256, 0, false, 1>(a, M, st);
        else LaunchTile<T, 128, 64, 128, 0, false, 1>(a, M, st);
        return 0;
      }
      return -4;
    case 256128:
    case 128256:
      // 8-wave tiles: the f32 epilogue staging would not fit the operand LDS
      if constexpr (sizeof(T) == 2) {
        if ((a.kernel ? a.kernel : env_tile) == 256128) LaunchTile<T, 256, 128, 512>(a, M, st);
        else LaunchTile<T, 128, 256, 512>(a, M, st);
        return 0;
      }
      return -4;
    case 0: break;
    default: return -4;
  }
  // Tile choice (per-shape sweeps over the ResNet-50 bottleneck shapes at batch 128, r2 conv1 / r2_s3
  // logs): Cout <= 64 -> 64x64 (store-bound 1x1 layers want more blocks in flight).
  // f32: 64x64 on every shape (r2_fp32conv sweep: 2625 us over the 14 shapes vs 2865-3258 for the larger
  // tiles; 36 KB of LDS, four blocks per CU hide the per-tile barrier behind the 32-cycle MFMAs), with
  // 8 waves of 16x32 (r2_tile64w8: 2537 -> 2467 us)
  if constexpr (sizeof(T) == 4 && kSplit == 0) {
    LaunchTile<T, 64, 64, 512>(a, M, st);
    return 0;
  }
  // f32 on bf16 planes: the K loop is MFMA-light, so the larger tile's operand reuse wins except on the
  // Cout = 64 layers (r3 sweep, bf16x3, 14 shapes: 64x64 (4 waves) 1591 us, 128x128 8 waves 1391 us, this
  // rule ~1323 us; exact f32 2502 us)
  if constexpr (kSplit > 0) {
    if (a.Cout <= 64) LaunchTile<T, 64, 64, kThreads, kSplit, kWPre>(a, M, st);
    else LaunchTile<T, 128, 128, 512, kSplit, kWPre>(a, M, st);
    return 0;
  }
  // SML_CONV_PERSIST=1: the persistent forms for the short-K layers (<= 4 K tiles; A/B switch)
  if constexpr (sizeof(T) == 2) {
    if (EnvPersist() && a.split_k == 1 && a.R * a.S * a.C <= 4 * Tile<T>::BK) {
      if (a.Cout <= 64) LaunchPersist<T, 64, 64, 256>(a, M, st);
      else LaunchPersist<T, 128, 128, 512>(a, M, st);
      return 0;
    }
  }
  // the LDS-DMA staged forms for the layers without a prologue, and (SML_CONV_GLDS_PRO=1) for the 1x1
  // pre-activation layers with one (SML_CONV_GLDS=0: register staging for all)
  if constexpr (sizeof(T) == 2) {
    if (EnvGlds() && (!a.in_scale || (EnvGldsPro() && GldsProOk(a))) && a.split_k == 1) {
      if (a.Cout <= 64) LaunchGlds<T, 64, 64, 256>(a, M, st);
      else LaunchGlds<T, 128, 128, 512>(a, M, st);
      return 0;
    }
  }
  if (a.Cout <= 64) {
    LaunchTile<T, 64, 64>(a, M, st);
    return 0;
  }
  // f16/bf16, Cout > 64: 128x128 with 8 waves (4x2, 32x64 wave tiles, two blocks per CU): r2_s3 sweep
  // 632 us over the 14 shapes vs 687 us for the 4-wave 128x128 / 64x128 table
  if constexpr (sizeof(T) == 2) LaunchTile<T, 128, 128, 512>(a, M, st);
  return 0;
}

// ---------------------------------------------------------------- few-channel stem conv
// The image stem (7x7, stride 2, 3 input channels -> 64 at 224x224: K = 147) has no channel run to tile over:
// the generic implicit GEMM gathers its A operand 2 bytes at a time (403 us per ResNet-50 fp16 batch of 128,
// 10 % of the replay). Here a block takes 128 consecutive output pixels and builds their im2col rows in LDS
// from the input's contiguous runs - for one pixel and filter row r the S * C input values (7 pixels x 3
// channels = 42 B) are adjacent in NHWC - with K zero-padded to kKP = 160; the [64][160] weight tile (packed
// once, zero-padded) sits beside it. 4 waves x (32 pixels x 64 channels) of 16x16x32 MFMAs, then the shared
// LDS-staged bias / ReLU / residual epilogue. Row pitch 176 elements (352 B): conflict-free fragment reads.
constexpr int kStemKP = 160;              // padded K (5 MFMA k-steps)
constexpr int kStemLd = kStemKP + 16;     // LDS row pitch
constexpr int kStemBM = 128, kStemBN = 64;

template <class T, int C, bool kPro = false>
__global__ __launch_bounds__(256) void stem_conv_kernel(ConvArgs a) {
  typedef typename Vec<T>::type V8;
  constexpr int kOpElems = (kStemBM + kStemBN) * kStemLd;
  __shared__ __attribute__((aligned(16))) T lds[kOpElems];
  T* As = lds;                      // [128][176]: im2col rows
  T* Bs = lds + kStemBM * kStemLd;  // [64][176]: weights
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int M = a.B * a.OH * a.OW;
  const int m0 = blockIdx.x * kStemBM, n0 = blockIdx.y * kStemBN;
  const int S = a.S, R = a.R, run = S * C, K = R * run;
  const T* __restrict__ w = static_cast<const T*>(a.w);
  // weights: 64 rows x 160 (already zero-padded by the packer), 16-B chunks - all 5 per thread in flight
  // before the first LDS store (the row-staged form's measured fix: one memory latency, not five)
  {
    constexpr int kWIt = kStemBN * (kStemKP / 8) / 256;
    uint4 wv[kWIt];
#pragma unroll
    for (int i = 0; i < kWIt; ++i) {
      const int q = tid + i * 256;
      const int n = n0 + q / (kStemKP / 8);
      wv[i] = n < a.Cout ? *reinterpret_cast<const uint4*>(w + static_cast<int64_t>(n) * kStemKP + (q % (kStemKP / 8)) * 8)
                         : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < kWIt; ++i) {
      const int q = tid + i * 256;
      *reinterpret_cast<uint4*>(Bs + (q / (kStemKP / 8)) * kStemLd + (q % (kStemKP / 8)) * 8) = wv[i];
    }
  }
  // the padded K tail of every A row is zero (NaN-free with the zero weight tail): every 16-B chunk from the
  // last partial one to kKP (the im2col runs below overwrite the real part of that first chunk)
  {
    const int c0 = K / 8, nch = kStemKP / 8 - c0;
    for (int q = tid; q < kStemBM * nch; q += 256) {
      const int row = q / nch, ch = c0 + q % nch;
      *reinterpret_cast<uint4*>(As + row * kStemLd + ch * 8) = make_uint4(0, 0, 0, 0);
    }
  }
  __syncthreads();
  // im2col runs: (pixel, filter row) -> the S * C contiguous input values of that row. Every value is a 2-byte
  // buffer load whose offset is out of range for padding (the hardware returns 0): the up-to-32 loads of a run
  // are independent and issue back to back (C is a template parameter, so the (s, c) of each slot is static).
  // The kernel is bound by how many of these gathers are in flight (2 blocks per CU, 8 waves).
  const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(a.x), 0, a.B * a.H * a.W * C * static_cast<int>(sizeof(T)), 0x00020000);
  constexpr uint32_t kOob = 0x80000000u;
  constexpr int kSlots = 8 * C;  // S <= 8
  // a thread's (up to 4) runs are all in flight before any is written to LDS: ~4 x 8C loads per lane
  // outstanding instead of one run's (the one-run loop waited out a full load latency per run)
  constexpr int kRunsPerThread = (kStemBM * 8 + 255) / 256;  // R <= 8
  unsigned short v[kRunsPerThread][kSlots];
  int dsto[kRunsPerThread];
  uint32_t okm[kRunsPerThread];  // kPro: in-range slots (padding stays 0 after the affine)
  float psc[C], psh[C];
  if constexpr (kPro) {
#pragma unroll
    for (int c = 0; c < C; ++c) { psc[c] = a.in_scale[c]; psh[c] = a.in_shift[c]; }
  }
#pragma unroll
  for (int u = 0; u < kRunsPerThread; ++u) {
    const int q = tid + u * 256;
    const int ml = q / R, r = q - ml * R;
    const int m = m0 + ml;
    const bool live = q < kStemBM * R && m < M;
    dsto[u] = live ? ml * kStemLd + r * run : -1;
    const int mm = live ? m : 0;
    const int ow = mm % a.OW, t2 = mm / a.OW;
    const int oh = t2 % a.OH, b = t2 / a.OH;
    const int ih = oh * a.stride_h - a.pad_h + r * a.dil_h;
    const int iw0 = ow * a.stride_w - a.pad_w;
    const bool row_ok = live && ih >= 0 && ih < a.H;
    const int rowbase = (b * a.H + ih) * a.W;
    okm[u] = 0u;
#pragma unroll
    for (int e = 0; e < kSlots; ++e) {
      const int s2 = e / C, c = e % C;
      const int iw = iw0 + s2 * a.dil_w;
      const bool ok = row_ok && s2 < S && iw >= 0 && iw < a.W;
      okm[u] |= ok ? (1u << e) : 0u;
      const uint32_t off = ok ? static_cast<uint32_t>(((rowbase + iw) * C + c) * static_cast<int>(sizeof(T))) : kOob;
      v[u][e] = __builtin_amdgcn_raw_buffer_load_b16(xres, off, 0, 0);
    }
  }
#pragma unroll
  for (int u = 0; u < kRunsPerThread; ++u) {
    if (dsto[u] < 0) continue;
    T* dst = As + dsto[u];
#pragma unroll
    for (int e = 0; e < kSlots; ++e) {
      if (e >= run) continue;
      if constexpr (kPro) {
        const int c = e % C;
        const float t = ToF(__builtin_bit_cast(T, v[u][e])) * psc[c] + psh[c];
        dst[e] = (okm[u] >> e) & 1u ? FromF<T>(a.prologue_relu ? fmaxf(t, 0.f) : t) : FromF<T>(0.f);
      } else {
        dst[e] = __builtin_bit_cast(T, v[u][e]);
      }
    }
  }
  __syncthreads();
  // 4 waves along M: 32 pixels x 64 channels each
  constexpr int TM = 2, TN = 4;
  f4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const int wm0 = wid * 32, fr = lane & 15, fk = 8 * (lane >> 4);
#pragma unroll
  for (int ks = 0; ks < kStemKP / 32; ++ks) {
    V8 af[TM], bf[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const V8*>(As + (wm0 + i * 16 + fr) * kStemLd + ks * 32 + fk);
#pragma unroll
    for (int j = 0; j < TN; ++j) bf[j] = *reinterpret_cast<const V8*>(Bs + (j * 16 + fr) * kStemLd + ks * 32 + fk);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = Vec<T>::mfma(af[i], bf[j], acc[i][j]);
  }
  __syncthreads();  // the epilogue stages through the operand LDS
  ConvEpilogue<T, 32, 64, 1>(a, acc, lds, M, m0, n0, wid, lane);
}

// Row-staged form of the stem: one block per output row (OW <= 128 pixels, C = 3, dilation 1). The R input
// rows the block reads are staged once in LDS by coalesced 16-B loads (zero columns of padding either side,
// zero rows out of range), and the im2col runs are built from LDS. The 2-byte gather form moves every input
// value ~R * S / (sh * sw) = 12 times through the texture path, which runs at ~4 B per clock per CU for
// scattered accesses (r4 passes 10-11: TA 75 % busy, 33 cycles per 64-lane gather); here each value
// crosses it once per block and the replication happens in LDS. With kPro the input affine (+ ReLU) is
// applied once per staged value; padding stays 0. Weights and the K order are the gather form's
// ([Cout][160], k = (r * S + s) * 3 + c); M rows past OW are computed and not stored.
constexpr int kRowPad = 8;  // zero columns staged either side of an input row (pad_w <= 8)

template <class T, bool kPro>
__global__ __launch_bounds__(256) void stem_rowbuf_kernel(ConvArgs a) {
  typedef typename Vec<T>::type V8;
  constexpr int C = 3;
  __shared__ __attribute__((aligned(16))) T lds[(kStemBM + kStemBN) * kStemLd];
  extern __shared__ __attribute__((aligned(16))) unsigned char stem_dyn_smem[];
  T* rowbuf = reinterpret_cast<T*>(stem_dyn_smem);  // [R][(W + 16) * 3], dynamic LDS
  T* As = lds;
  T* Bs = lds + kStemBM * kStemLd;
  const int tid = threadIdx.x;
  const int orow = blockIdx.x;  // b * OH + oh
  const int oh = orow % a.OH, b = orow / a.OH;
  const int m0 = orow * a.OW, n0 = blockIdx.y * kStemBN;
  const int S = a.S, R = a.R, run = S * C, K = R * run;
  const int SP = (a.W + 2 * kRowPad) * C;  // slot pitch (halfs), a multiple of 8
  const int cps = SP / 8, d0 = kRowPad * C / 8, d1 = d0 + a.W * C / 8;  // data chunks [d0, d1) of a slot
  // every global load of the prologue is issued before the first LDS store: one memory latency, not one
  // per loop trip (weights: 1280 16-B chunks = 5 per thread; staged rows: <= 768 chunks = 3 per thread)
  constexpr int kWIt = kStemBN * (kStemKP / 8) / 256, kRIt = 3;
  const T* __restrict__ w = static_cast<const T*>(a.w);
  const T* __restrict__ x = static_cast<const T*>(a.x);
  float psc[C], psh[C];  // the input affine's 3 scale / shift pairs, in flight with the tiles below
  if constexpr (kPro) {
#pragma unroll
    for (int c = 0; c < C; ++c) { psc[c] = a.in_scale[c]; psh[c] = a.in_shift[c]; }
  }
  uint4 wv[kWIt], rv[kRIt];
#pragma unroll
  for (int i = 0; i < kWIt; ++i) {
    const int q = tid + i * 256;
    const int row = q / (kStemKP / 8), ch = q % (kStemKP / 8);
    const int n = n0 + row;
    wv[i] = n < a.Cout ? *reinterpret_cast<const uint4*>(w + static_cast<int64_t>(n) * kStemKP + ch * 8)
                       : make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < kRIt; ++i) {
    const int q = tid + i * 256;
    const int r = q / cps, j = q - r * cps;
    const int ih = oh * a.stride_h - a.pad_h + r;
    rv[i] = make_uint4(0, 0, 0, 0);
    if (q < R * cps && ih >= 0 && ih < a.H && j >= d0 && j < d1)
      rv[i] = *reinterpret_cast<const uint4*>(x + (static_cast<int64_t>(b) * a.H + ih) * a.W * C + (j - d0) * 8);
  }
  {
    const int c0 = K / 8, nch = kStemKP / 8 - c0;
    for (int q = tid; q < kStemBM * nch; q += 256) {
      const int row = q / nch, ch = c0 + q % nch;
      *reinterpret_cast<uint4*>(As + row * kStemLd + ch * 8) = make_uint4(0, 0, 0, 0);
    }
  }
#pragma unroll
  for (int i = 0; i < kWIt; ++i) {
    const int q = tid + i * 256;
    *reinterpret_cast<uint4*>(Bs + (q / (kStemKP / 8)) * kStemLd + (q % (kStemKP / 8)) * 8) = wv[i];
  }
#pragma unroll
  for (int i = 0; i < kRIt; ++i) {
    const int q = tid + i * 256;
    if (q >= R * cps) continue;
    const int r = q / cps, j = q - r * cps;
    uint4 v = rv[i];
    if constexpr (kPro) {  // the affine of real values only: padding columns / rows stay 0
      const int ih = oh * a.stride_h - a.pad_h + r;
      if (ih >= 0 && ih < a.H && j >= d0 && j < d1) {
        T* e = reinterpret_cast<T*>(&v);
        const int c0 = (j * 8) % C;  // channel of the chunk's first value (rows are C-aligned in the slot)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int c = (c0 + k) % C;
          const float t = ToF(e[k]) * psc[c] + psh[c];
          e[k] = FromF<T>(a.prologue_relu ? fmaxf(t, 0.f) : t);
        }
      }
    }
    *reinterpret_cast<uint4*>(rowbuf + r * SP + j * 8) = v;
  }
  __syncthreads();
  // im2col runs from LDS, a dword at a time: thread -> (filter row r, pixel ml), a wave = 64 pixels of one r.
  // The run's S * 3 halves start at any half (h0) and land at any half (dst): read 12 dwords from h0's dword,
  // shift by h0's parity (v_alignbyte), store as dwords shifted by dst's parity (wave-uniform: r * run).
  for (int q = tid; q < R * kStemBM; q += 256) {
    const int r = q >> 7, ml = q & (kStemBM - 1);
    if (ml >= a.OW) continue;
    const int h0 = r * SP + (ml * a.stride_w - a.pad_w + kRowPad) * C;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(rowbuf) + (h0 >> 1);
    uint32_t d[12], o[11];
#pragma unroll
    for (int k = 0; k < 12; ++k) d[k] = src[k];
    const uint32_t sb = static_cast<uint32_t>(h0 & 1) * 2u;
#pragma unroll
    for (int k = 0; k < 11; ++k) o[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sb);  // halves 2k, 2k + 1
    const int dst = ml * kStemLd + r * run;  // half index in As
    uint32_t* A32 = reinterpret_cast<uint32_t*>(As);
    unsigned short* A16 = reinterpret_cast<unsigned short*>(As);
    if ((dst & 1) == 0) {
#pragma unroll
      for (int k = 0; k < 11; ++k) {
        if (2 * k + 1 < run) A32[(dst >> 1) + k] = o[k];
        else if (2 * k < run) A16[dst + 2 * k] = static_cast<unsigned short>(o[k] & 0xFFFFu);
      }
    } else {
      A16[dst] = static_cast<unsigned short>(o[0] & 0xFFFFu);
#pragma unroll
      for (int k = 0; k < 10; ++k) {  // halves (2k + 1, 2k + 2)
        const uint32_t pr = __builtin_amdgcn_alignbyte(o[k + 1], o[k], 2u);
        if (2 * k + 2 < run) A32[((dst + 1) >> 1) + k] = pr;
        else if (2 * k + 1 < run) A16[dst + 2 * k + 1] = static_cast<unsigned short>(pr & 0xFFFFu);
      }
    }
  }
  __syncthreads();
  const int lane = tid & 63, wid = tid >> 6;
  constexpr int TM = 2, TN = 4;
  f4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const int wm0 = wid * 32, fr = lane & 15, fk = 8 * (lane >> 4);
#pragma unroll
  for (int ks = 0; ks < kStemKP / 32; ++ks) {
    V8 af[TM], bf[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const V8*>(As + (wm0 + i * 16 + fr) * kStemLd + ks * 32 + fk);
#pragma unroll
    for (int j = 0; j < TN; ++j) bf[j] = *reinterpret_cast<const V8*>(Bs + (j * 16 + fr) * kStemLd + ks * 32 + fk);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = Vec<T>::mfma(af[i], bf[j], acc[i][j]);
  }
  __syncthreads();
  ConvEpilogue<T, 32, 64, 1>(a, acc, lds, m0 + a.OW, m0, n0, wid, lane);  // rows past OW are not stored
}

// the row-staged form's shapes: 3 channels, one block per output row, 16-B aligned input rows, padding and
// dilation it stages, and its LDS (static operand tiles + R staged rows) within two blocks per CU
inline int RowbufLds(const ConvArgs& a) { return a.R * (a.W + 2 * kRowPad) * 3 * 2; }
inline bool RowbufOk(const ConvArgs& a) {
  return reinterpret_cast<uintptr_t>(a.x) % 16 == 0 && a.C == 3 && a.S * 3 <= 21 && a.OW <= kStemBM && a.dil_h == 1 && a.dil_w == 1 && a.pad_w <= kRowPad && a.R <= 8 && a.S <= 8 &&
         (a.W * 3 * 2) % 16 == 0 && (a.OW - 1) * a.stride_w - a.pad_w + a.S <= a.W + kRowPad &&
         RowbufLds(a) <= 12 * 1024;
}

// Row-run form of the stem (C = 3, S * C <= 24, R <= 8: the 7x7 RGB stem). The b16 gathers above keep the
// texture path busy ~33 cycles per 64-lane load (r4 pass 10 counters: TA 75 %, TD 84 % busy over the
// kernel, 105 load instructions per wave), so here every (pixel, filter row) run is fetched as the
// enclosing 64 aligned bytes (4 x 16-B buffer loads, 5x fewer instructions, 8x the bytes each) and
// shifted into place in registers (dword selects + v_alignbyte). K is packed per filter row to RP = 24
// (k = r * 24 + s * 3 + c, weights zero in slots s * 3 + c >= S * C), so each run lands as 3 aligned
// 16-B LDS stores; K = R * 24 padded to 192 (6 MFMA k-steps; the MFMAs are ~5 % of the kernel).
// Row pitch 208 elements (416 B: the 16 rows x 2 chunks of a b128 fragment group hit 16 distinct slots).
constexpr int kWideRP = 24, kWideKP = 192, kWideLd = kWideKP + 16;

template <class T, bool kPro>
__global__ __launch_bounds__(256) void stem_wide_kernel(ConvArgs a) {
  typedef typename Vec<T>::type V8;
  constexpr int C = 3;
  constexpr int kOpElems = (kStemBM + kStemBN) * kWideLd;
  __shared__ __attribute__((aligned(16))) T lds[kOpElems];
  T* As = lds;                      // [128][208]: im2col rows, run r at r * 24
  T* Bs = lds + kStemBM * kWideLd;  // [64][208]: weights
  const int tid = threadIdx.x;
  const int M = a.B * a.OH * a.OW;
  const int m0 = blockIdx.x * kStemBM, n0 = blockIdx.y * kStemBN;
  const int S = a.S, R = a.R, SC = S * C, K = R * kWideRP;
  const T* __restrict__ w = static_cast<const T*>(a.w);
  for (int q = tid; q < kStemBN * (kWideKP / 8); q += 256) {
    const int row = q / (kWideKP / 8), ch = q % (kWideKP / 8);
    const int n = n0 + row;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (n < a.Cout) v = *reinterpret_cast<const uint4*>(w + static_cast<int64_t>(n) * kWideKP + ch * 8);
    *reinterpret_cast<uint4*>(Bs + row * kWideLd + ch * 8) = v;
  }
  // K tail beyond R * 24 (whole 16-B chunks: 24 is a multiple of 8)
  {
    const int c0 = K / 8, nch = kWideKP / 8 - c0;
    for (int q = tid; q < kStemBM * nch; q += 256) {
      const int row = q / nch, ch = c0 + q % nch;
      *reinterpret_cast<uint4*>(As + row * kWideLd + ch * 8) = make_uint4(0, 0, 0, 0);
    }
  }
  // records rounded up to the 16-B chunk: a chunk holding the input's last bytes loads whole (the few bytes
  // past the end land in masked slots; the caching allocator's blocks are 512-B granular)
  const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(a.x), 0, (a.B * a.H * a.W * C * static_cast<int>(sizeof(T)) + 15) & ~15, 0x00020000);
  constexpr uint32_t kOob = 0x80000000u;
  float psc[C], psh[C];
  if constexpr (kPro) {
#pragma unroll
    for (int c = 0; c < C; ++c) { psc[c] = a.in_scale[c]; psh[c] = a.in_shift[c]; }
  }
  constexpr int kRuns = (kStemBM * 8 + 255) / 256;  // R <= 8
  uint32_t win[kRuns][16];
  int dsto[kRuns], iw0s[kRuns], shs[kRuns];
  bool rows_ok[kRuns];
#pragma unroll
  for (int u = 0; u < kRuns; ++u) {
    const int q = tid + u * 256;
    const int ml = q / R, r = q - ml * R;
    const int m = m0 + ml;
    const bool live = q < kStemBM * R && m < M;
    dsto[u] = live ? ml * kWideLd + r * kWideRP : -1;
    const int mm = live ? m : 0;
    const int ow = mm % a.OW, t2 = mm / a.OW;
    const int oh = t2 % a.OH, b = t2 / a.OH;
    const int ih = oh * a.stride_h - a.pad_h + r * a.dil_h;
    const int iw0 = ow * a.stride_w - a.pad_w;
    rows_ok[u] = live && ih >= 0 && ih < a.H;
    iw0s[u] = iw0;
    const int byte0 = (((b * a.H + ih) * a.W + iw0) * C) * static_cast<int>(sizeof(T));  // may be < 0 at the border
    const int base = byte0 & ~15;
    shs[u] = byte0 - base;  // 0..14, even
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int o = base + 16 * k;
      const uint32_t off = rows_ok[u] && o >= 0 ? static_cast<uint32_t>(o) : kOob;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(xres, off, 0, 0);
      win[u][4 * k] = v[0]; win[u][4 * k + 1] = v[1]; win[u][4 * k + 2] = v[2]; win[u][4 * k + 3] = v[3];
    }
  }
#pragma unroll
  for (int u = 0; u < kRuns; ++u) {
    if (dsto[u] < 0) continue;
    // shift the window left by shs bytes: dword rotation by shs >> 2 (two select levels), then 0 / 2 bytes
    const int dsh = shs[u] >> 2;
    const uint32_t sb = static_cast<uint32_t>(shs[u] & 3);
    uint32_t v1[15], v2[13], o[12];
#pragma unroll
    for (int k = 0; k < 15; ++k) v1[k] = (dsh & 1) ? win[u][k + 1] : win[u][k];
#pragma unroll
    for (int k = 0; k < 13; ++k) v2[k] = (dsh & 2) ? v1[k + 2] : v1[k];
#pragma unroll
    for (int i = 0; i < 12; ++i) o[i] = __builtin_amdgcn_alignbyte(v2[i + 1], v2[i], sb);
    // element e = s * 3 + c of the run: real iff e < S * C, the row is in range and 0 <= iw0 + s < W
    const int iw0 = iw0s[u];
    const bool rok = rows_ok[u];
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      uint32_t outw = 0;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int e = 2 * i + hh;
        const int iw = iw0 + e / C;
        const bool ok = rok && e < SC && iw >= 0 && iw < a.W;
        const uint32_t bits = (o[i] >> (16 * hh)) & 0xFFFFu;
        uint32_t val = ok ? bits : 0u;
        if constexpr (kPro) {
          const float t = ToF(__builtin_bit_cast(T, static_cast<unsigned short>(bits))) * psc[e % C] + psh[e % C];
          val = ok ? static_cast<uint32_t>(__builtin_bit_cast(unsigned short, FromF<T>(a.prologue_relu ? fmaxf(t, 0.f) : t))) : 0u;
        }
        outw |= val << (16 * hh);
      }
      o[i] = outw;
    }
    uint4* dst = reinterpret_cast<uint4*>(As + dsto[u]);
    dst[0] = make_uint4(o[0], o[1], o[2], o[3]);
    dst[1] = make_uint4(o[4], o[5], o[6], o[7]);
    dst[2] = make_uint4(o[8], o[9], o[10], o[11]);
  }
  __syncthreads();
  const int lane = tid & 63, wid = tid >> 6;
  constexpr int TM = 2, TN = 4;
  f4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const int wm0 = wid * 32, fr = lane & 15, fk = 8 * (lane >> 4);
#pragma unroll
  for (int ks = 0; ks < kWideKP / 32; ++ks) {
    V8 af[TM], bf[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const V8*>(As + (wm0 + i * 16 + fr) * kWideLd + ks * 32 + fk);
#pragma unroll
    for (int j = 0; j < TN; ++j) bf[j] = *reinterpret_cast<const V8*>(Bs + (j * 16 + fr) * kWideLd + ks * 32 + fk);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = Vec<T>::mfma(af[i], bf[j], acc[i][j]);
  }
  __syncthreads();
  ConvEpilogue<T, 32, 64, 1>(a, acc, lds, M, m0, n0, wid, lane);
}

// fp32 stem on bf16 planes (the fp32 graphs' bf16x3 / bf16x6 modes, kP = 2 / 3 planes, 3 / 6 products per
// pair as in the tiled kernel's kSplit): the row-staged form above with fp32 input rows. Each staged value is
// (affine'd, then) split once into kP RNE bf16 planes (x = x0 + x1 (+ x2) up to the last plane's rounding),
// the im2col rows of one plane at a time are built in LDS from that plane's rows, and the products (xp, wq)
// with p + q < kP are accumulated in fp32 by 16x16x32 bf16 MFMAs. The weight planes ([kP][Cout][160] bf16,
// split once per model) live in registers: waves split 2 (pixels) x 2 (channels), 64 x 32 per wave, so a
// wave's B fragments are loaded once per block. Replaces the generic exact-f32 gather GEMM for the 3-channel
// stem of an fp32 graph (r6 pass 25: 954 us per ResNet-50 batch of 256, plus the input affine's own pass).
// LDS: one A plane [128][176] bf16 (45 KB, the fp32 epilogue staging reuses it) + kP staged row planes.
template <int kP, bool kPro>
__global__ __launch_bounds__(256) void stem_f32_kernel(ConvArgs a) {
  typedef __bf16 bt;
  constexpr int C = 3, TM = 4, TN = 2, kKS = kStemKP / 32, kRIt = 8;
  __shared__ __attribute__((aligned(16))) bt As[kStemBM * kStemLd];
  extern __shared__ __attribute__((aligned(16))) unsigned char stem_f32_smem[];
  bt* rowbuf = reinterpret_cast<bt*>(stem_f32_smem);  // [kP][R][SP]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int orow = blockIdx.x;  // b * OH + oh
  const int oh = orow % a.OH, b = orow / a.OH;
  const int m0 = orow * a.OW, n0 = blockIdx.y * kStemBN;
  const int S = a.S, R = a.R, run = S * C, K = R * run;
  const int SP = (a.W + 2 * kRowPad) * C;  // plane row pitch (elements), a multiple of 4
  const int cps = SP / 4, d0 = kRowPad * C / 4, d1 = d0 + a.W * C / 4;  // 4-value chunks; data in [d0, d1)
  const int plane = R * SP;
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  // every global load first: the wave's weight fragments (kP planes x 5 k-steps x 2 channel tiles) and the
  // block's input rows (<= 8 float4 per thread), one memory latency for all of them
  const bt* __restrict__ w = static_cast<const bt*>(a.w);
  b8 bfr[kP][kKS][TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * 32 + j * 16 + fr;
#pragma unroll
    for (int q = 0; q < kP; ++q)
#pragma unroll
      for (int ks = 0; ks < kKS; ++ks) {
        if (n < a.Cout) {
          bfr[q][ks][j] = *reinterpret_cast<const b8*>(w + (static_cast<int64_t>(q) * a.Cout + n) * kStemKP + ks * 32 + fk);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) bfr[q][ks][j][e] = static_cast<bt>(0.f);
        }
      }
  }
  const float* __restrict__ x = static_cast<const float*>(a.x);
  float psc[C], psh[C];
  if constexpr (kPro) {
#pragma unroll
    for (int c = 0; c < C; ++c) { psc[c] = a.in_scale[c]; psh[c] = a.in_shift[c]; }
  }
  f4 rv[kRIt];
  bool rok[kRIt];
#pragma unroll
  for (int i = 0; i < kRIt; ++i) {
    const int q = tid + i * 256;
    const int r = q / cps, j = q - r * cps;
    const int ih = oh * a.stride_h - a.pad_h + r;
    rok[i] = q < R * cps && ih >= 0 && ih < a.H && j >= d0 && j < d1;
    rv[i] = f4{0.f, 0.f, 0.f, 0.f};
    if (rok[i]) rv[i] = *reinterpret_cast<const f4*>(x + (static_cast<int64_t>(b) * a.H + ih) * a.W * C + (j - d0) * 4);
  }
  {  // the padded K tail of every A row is zero in every plane (the im2col below writes only [0, K))
    const int c0 = K / 8, nch = kStemKP / 8 - c0;
    for (int q = tid; q < kStemBM * nch; q += 256) {
      const int row = q / nch, ch = c0 + q % nch;
      *reinterpret_cast<uint4*>(As + row * kStemLd + ch * 8) = make_uint4(0, 0, 0, 0);
    }
  }
  // stage: affine (real values only: padding stays 0), then the plane split, 8 B per plane and chunk
#pragma unroll
  for (int i = 0; i < kRIt; ++i) {
    const int q = tid + i * 256;
    if (q >= R * cps) continue;
    const int r = q / cps, j = q - r * cps;
    float v[4] = {rv[i][0], rv[i][1], rv[i][2], rv[i][3]};
    if constexpr (kPro) {
      if (rok[i]) {
        const int c0 = (j * 4) % C;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int c = (c0 + k) % C;
          const float t = v[k] * psc[c] + psh[c];
          v[k] = a.prologue_relu ? fmaxf(t, 0.f) : t;
        }
      }
    }
#pragma unroll
    for (int p = 0; p < kP; ++p) {
      bt h[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        h[k] = static_cast<bt>(v[k]);
        v[k] -= static_cast<float>(h[k]);
      }
      *reinterpret_cast<uint2*>(rowbuf + p * plane + r * SP + j * 4) = *reinterpret_cast<const uint2*>(h);
    }
  }
  __syncthreads();
  f4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int p = 0; p < kP; ++p) {
    // im2col rows of plane p from its staged rows (the f16 row-staged form's dword shifts)
    const bt* rb = rowbuf + p * plane;
    for (int q = tid; q < R * kStemBM; q += 256) {
      const int r = q >> 7, ml = q & (kStemBM - 1);
      if (ml >= a.OW) continue;
      const int h0 = r * SP + (ml * a.stride_w - a.pad_w + kRowPad) * C;
      const uint32_t* src = reinterpret_cast<const uint32_t*>(rb) + (h0 >> 1);
      uint32_t d[12], o[11];
#pragma unroll
      for (int k = 0; k < 12; ++k) d[k] = src[k];
      const uint32_t sb = static_cast<uint32_t>(h0 & 1) * 2u;
#pragma unroll
      for (int k = 0; k < 11; ++k) o[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sb);
      const int dst = ml * kStemLd + r * run;
      uint32_t* A32 = reinterpret_cast<uint32_t*>(As);
      unsigned short* A16 = reinterpret_cast<unsigned short*>(As);
      if ((dst & 1) == 0) {
#pragma unroll
        for (int k = 0; k < 11; ++k) {
          if (2 * k + 1 < run) A32[(dst >> 1) + k] = o[k];
          else if (2 * k < run) A16[dst + 2 * k] = static_cast<unsigned short>(o[k] & 0xFFFFu);
        }
      } else {
        A16[dst] = static_cast<unsigned short>(o[0] & 0xFFFFu);
#pragma unroll
        for (int k = 0; k < 10; ++k) {
          const uint32_t pr = __builtin_amdgcn_alignbyte(o[k + 1], o[k], 2u);
          if (2 * k + 2 < run) A32[((dst + 1) >> 1) + k] = pr;
          else if (2 * k + 1 < run) A16[dst + 2 * k + 1] = static_cast<unsigned short>(pr & 0xFFFFu);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < kKS; ++ks) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if ((wm * TM + i) * 16 >= a.OW) continue;  // wave-uniform: pixel tiles past the output row
        const b8 af = *reinterpret_cast<const b8*>(As + (wm * 64 + i * 16 + fr) * kStemLd + ks * 32 + fk);
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int q = 0; q < kP - p; ++q) acc[i][j] = Vec<bt>::mfma(af, bfr[q][ks][j], acc[i][j]);
      }
    }
    __syncthreads();  // the next plane's im2col (or the epilogue staging) overwrites As
  }
  ConvEpilogue<float, 64, 32, 2>(a, acc, reinterpret_cast<float*>(As), m0 + a.OW, m0, n0, wid, lane);
}

// Strip form of the stride-2 RGB stem (f16 / bf16 with one plane, fp32 on kP bf16 planes): a block walks
// kRingOut consecutive output rows of one image. The input rows live in an LDS ring of R + stride_h rows
// (per plane); an output row needs only its stride_h new input rows, loaded into registers while the previous
// row's MFMAs run and written to the ring slots that row no longer reads. No im2col buffer: with the row-run
// K order (k = r * 24 + s * 3 + c, weights zero in slots s * 3 + c >= S * 3) a fragment's 8 consecutive k are 8
// consecutive values of one staged row, and stride_w * 3 even with the row staged pad_w zero pixels in keeps
// every fragment's first value at an even slot offset: 4 aligned dword reads per fragment. The weight planes
// sit in registers for the whole strip (waves 2 pixels x 2 channels, 64 x 32 each), the epilogue stages
// through its own LDS area (the shared bias / ReLU / residual / 16-B store path).
constexpr int kRingOut = 8;  // output rows per block

template <class T, int kP, bool kPro>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kP > 2 ? 1 : 2, 2))) void stem_ring_kernel(ConvArgs a, int SP,
                                                                                         int nstrip) {
  typedef typename std::conditional<sizeof(T) == 4, __bf16, T>::type MT;  // MFMA operand type
  typedef typename Vec<MT>::type V8;
  constexpr int C = 3, TM = 4, TN = 2, kKS = kWideKP / 32, EPC = 16 / static_cast<int>(sizeof(T));
  constexpr int kEpiL = 32 + (sizeof(T) == 4 ? 4 : 8);  // ConvEpilogue<T, 64, 32, 2>'s staged row pitch
  constexpr int kItInit = 8, kItPre = 2;
  __shared__ __attribute__((aligned(16))) T epi[4 * 64 * kEpiL];
  extern __shared__ __attribute__((aligned(16))) unsigned char stem_ring_smem[];
  MT* ring = reinterpret_cast<MT*>(stem_ring_smem);  // [kP][NR][SP] (+ one slack row)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int b = blockIdx.x / nstrip, oh0 = (blockIdx.x - b * nstrip) * kRingOut;
  const int nout = min(kRingOut, a.OH - oh0);
  const int n0 = blockIdx.y * kStemBN;
  const int R = a.R, sh = a.stride_h, NR = R + sh, plane = NR * SP;
  const int cpr = a.W * C / EPC;  // 16-B input chunks per row
  const int d0 = a.pad_w * C;     // slot offset of the row's first value (the row is staged pad_w pixels in)
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  const MT* __restrict__ w = static_cast<const MT*>(a.w);
  V8 bfr[kP][kKS][TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * 32 + j * 16 + fr;
#pragma unroll
    for (int q = 0; q < kP; ++q)
#pragma unroll
      for (int ks = 0; ks < kKS; ++ks) {
        if (n < a.Cout) {
          bfr[q][ks][j] = *reinterpret_cast<const V8*>(w + (static_cast<int64_t>(q) * a.Cout + n) * kWideKP + ks * 32 + fk);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) bfr[q][ks][j][e] = static_cast<MT>(0.f);
        }
      }
  }
  float psc[C], psh[C];
  if constexpr (kPro) {
#pragma unroll
    for (int c = 0; c < C; ++c) { psc[c] = a.in_scale[c]; psh[c] = a.in_shift[c]; }
  }
  const T* __restrict__ x = static_cast<const T*>(a.x);
  const int64_t img = static_cast<int64_t>(b) * a.H;
  auto slot_of = [&](int ih) { return (ih + 16 * NR) % NR; };
  // one 16-B input chunk: row ih (zero outside the image), chunk j
  auto load = [&](int ih, int j) -> uint4 {
    if (ih < 0 || ih >= a.H) return make_uint4(0, 0, 0, 0);
    return *reinterpret_cast<const uint4*>(x + (img + ih) * a.W * C + j * EPC);
  };
  // affine (real rows only), plane split, and the chunk's values written at slot offset d0 + j * EPC: dword
  // stores from the first even offset, a 2-byte store at an odd end
  auto commit = [&](int ih, int j, uint4 raw) {
    float v[EPC];
    const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
    for (int k = 0; k < EPC; ++k) v[k] = ToF(e[k]);
    if constexpr (kPro) {
      if (ih >= 0 && ih < a.H) {
        const int c0 = (j * EPC) % C;
#pragma unroll
        for (int k = 0; k < EPC; ++k) {
          const int c = (c0 + k) % C;
          const float t = v[k] * psc[c] + psh[c];
          v[k] = a.prologue_relu ? fmaxf(t, 0.f) : t;
        }
      }
    }
    const int off = slot_of(ih) * SP + d0 + j * EPC;
#pragma unroll
    for (int p = 0; p < kP; ++p) {
      MT h[EPC];
#pragma unroll
      for (int k = 0; k < EPC; ++k) {
        h[k] = static_cast<MT>(v[k]);
        if constexpr (kP > 1) v[k] -= static_cast<float>(h[k]);
      }
      unsigned short* r16 = reinterpret_cast<unsigned short*>(ring + p * plane + off);
      const unsigned short* hs = reinterpret_cast<const unsigned short*>(h);
      if ((off & 1) == 0) {
#pragma unroll
        for (int k = 0; k < EPC; k += 2)
          *reinterpret_cast<uint32_t*>(r16 + k) = static_cast<uint32_t>(hs[k]) | (static_cast<uint32_t>(hs[k + 1]) << 16);
      } else {
        r16[0] = hs[0];
#pragma unroll
        for (int k = 1; k + 1 < EPC; k += 2)
          *reinterpret_cast<uint32_t*>(r16 + k) = static_cast<uint32_t>(hs[k]) | (static_cast<uint32_t>(hs[k + 1]) << 16);
        r16[EPC - 1] = hs[EPC - 1];
      }
    }
  };
  // the whole ring zero (padding columns stay zero for the strip), then the first output row's R input rows
  {
    uint32_t* r32 = reinterpret_cast<uint32_t*>(ring);
    const int nd = (kP * plane + SP) / 2;
    for (int q = tid; q < nd; q += 256) r32[q] = 0u;
  }
  __syncthreads();
  {
    const int ih0 = oh0 * sh - a.pad_h;
    uint4 rv[kItInit];
#pragma unroll
    for (int i = 0; i < kItInit; ++i) {
      const int q = tid + i * 256;
      rv[i] = q < R * cpr ? load(ih0 + q / cpr, q % cpr) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < kItInit; ++i) {
      const int q = tid + i * 256;
      if (q < R * cpr) commit(ih0 + q / cpr, q % cpr, rv[i]);
    }
  }
  // per lane: the filter row and slot offset of its 8 k of every k-step (rows >= R carry zero weights: read row
  // R - 1 instead of a slot being refilled)
  for (int k = 0; k < nout; ++k) {
    __syncthreads();  // this row's input rows staged; the previous epilogue's staging reads done
    const int oh = oh0 + k;
    const bool more = k + 1 < nout;
    const int ihn = oh * sh - a.pad_h + R;  // the next output row's new input rows: [ihn, ihn + sh)
    uint4 pv[kItPre];
#pragma unroll
    for (int i = 0; i < kItPre; ++i) {
      const int q = tid + i * 256;
      pv[i] = (more && q < sh * cpr) ? load(ihn + q / cpr, q % cpr) : make_uint4(0, 0, 0, 0);
    }
    f4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    const int ihb = oh * sh - a.pad_h;
#pragma unroll
    for (int ks = 0; ks < kKS; ++ks) {
      const int k0 = ks * 32 + fk;
      const int r = min(k0 / kWideRP, R - 1), jj = k0 % kWideRP;
      const int rowoff = slot_of(ihb + r) * SP + jj;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if ((wm * TM + i) * 16 >= a.OW) continue;  // wave-uniform: pixel tiles past the output row
        const int ow = wm * 64 + i * 16 + fr;
        const int e0 = rowoff + ow * a.stride_w * C;  // even: stride_w * 3 even, pad_w cancels
#pragma unroll
        for (int p = 0; p < kP; ++p) {
          const uint32_t* src = reinterpret_cast<const uint32_t*>(ring + p * plane + e0);
          uint4 u;
          u.x = src[0];
          u.y = src[1];
          u.z = src[2];
          u.w = src[3];
          const V8 af = __builtin_bit_cast(V8, u);
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int q = 0; q < kP - p; ++q) acc[i][j] = Vec<MT>::mfma(af, bfr[q][ks][j], acc[i][j]);
        }
      }
    }
    if (more) {  // slots of the rows output row oh - 1 read (done before the barrier above), not row oh's
#pragma unroll
      for (int i = 0; i < kItPre; ++i) {
        const int q = tid + i * 256;
        if (q < sh * cpr) commit(ihn + q / cpr, q % cpr, pv[i]);
      }
    }
    const int m0 = (b * a.OH + oh) * a.OW;
    ConvEpilogue<T, 64, 32, 2>(a, acc, epi, m0 + a.OW, m0, n0, wid, lane);
  }
}

// slot pitch (elements) of the strip form's ring: the staged row (pad_w zero pixels, the row, zeros) and
// the farthest 24-value run a stored output pixel reads, rounded up to 8 values
inline int RingSP(const ConvArgs& a) {
  const int data_end = (a.pad_w + a.W) * 3;
  const int run_end = ((a.OW - 1) * a.stride_w) * 3 + kWideRP;
  return (std::max(data_end, run_end) + 8 + 7) / 8 * 8;
}
inline int RingLds(const ConvArgs& a, int planes) { return (planes * (a.R + a.stride_h) + 1) * RingSP(a) * 2; }
inline bool RingOk(const ConvArgs& a, int planes, int esize) {
  const int epc = 16 / esize;
  return reinterpret_cast<uintptr_t>(a.x) % 16 == 0 && a.C == 3 && (a.stride_w % 2) == 0 && a.stride_w <= 4 &&
         a.S * 3 <= kWideRP &&
         a.R <= 8 && a.R >= 1 && a.stride_h >= 1 && a.stride_h <= 4 && a.OW <= kStemBM && a.OW > 0 && a.OH > 0 &&
         a.dil_h == 1 && a.dil_w == 1 && a.pad_w <= 8 && (a.W * 3) % epc == 0 &&
         a.R * (a.W * 3 / epc) <= 8 * 256 && a.stride_h * (a.W * 3 / epc) <= 2 * 256 &&
         RingLds(a, planes) <= 44 * 1024 && a.B > 0 && a.Cout >= 1 &&
         static_cast<int64_t>(a.B) * a.OH * a.OW * a.Cout < (1ll << 31) &&
         static_cast<int64_t>(a.B) * a.H * a.W * 3 < (1ll << 31);
}

inline int StemF32Lds(const ConvArgs& a, int planes) { return planes * a.R * (a.W + 2 * kRowPad) * 3 * 2; }
inline bool StemF32Ok(const ConvArgs& a, int planes) {
  return reinterpret_cast<uintptr_t>(a.x) % 16 == 0 && a.C == 3 && a.S * 3 <= 21 && a.R <= 8 && a.R * a.S * 3 <= kStemKP &&
         a.OW <= kStemBM && a.dil_h == 1 && a.dil_w == 1 && a.pad_w <= kRowPad && a.W % 4 == 0 &&
         (a.OW - 1) * a.stride_w - a.pad_w + a.S <= a.W + kRowPad && a.R * (a.W + 2 * kRowPad) * 3 / 4 <= 8 * 256 &&
         StemF32Lds(a, planes) <= 34 * 1024 && a.B > 0 && a.OH > 0 && a.Cout >= 1 &&
         static_cast<int64_t>(a.B) * a.OH * a.OW * a.Cout < (1ll << 31) && static_cast<int64_t>(a.B) * a.H * a.W * 3 < (1ll << 31);
}

}  // namespace

template <class T>
int LaunchStem(const ConvArgs& a, hipStream_t st) {
  const int M = a.B * a.OH * a.OW;
  const int blocks = ((M + 63) / 64) * ((a.Cout + 63) / 64);
  hipLaunchKernelGGL((conv_mfma_kernel<T, 64, 64, false, kThreads, 1, true>), dim3(blocks), dim3(kThreads), 0, st, a);
  return 0;
}

// few-channel stem: x NHWC with C <= 4, w packed [Cout][160] (k = (r * S + s) * C + c, zero-padded),
// R * S * C <= 160, f16 (dtype 1) / bf16 (2)
namespace {
template <class T, int kP>
void LaunchRing(const ConvArgs& a, hipStream_t st) {
  const int nstrip = (a.OH + kRingOut - 1) / kRingOut;
  const dim3 grid(a.B * nstrip, (a.Cout + kStemBN - 1) / kStemBN);
  const size_t dyn = static_cast<size_t>(RingLds(a, kP));
  const int SP = RingSP(a);
  if (a.in_scale) hipLaunchKernelGGL((stem_ring_kernel<T, kP, true>), grid, dim3(256), dyn, st, a, SP, nstrip);
  else hipLaunchKernelGGL((stem_ring_kernel<T, kP, false>), grid, dim3(256), dyn, st, a, SP, nstrip);
}
}  // namespace

int StemConv(const ConvArgs& a, int dtype, void* stream, int kp, int form) {
  hipStream_t rst = static_cast<hipStream_t>(stream);
  if ((dtype == 3 || dtype == 4) && kp == kWideKP) {  // fp32 strip form: weights [planes][Cout][192] bf16
    const int planes = dtype == 3 ? 2 : 3;
    if (form == 1 || !RingOk(a, planes, 4)) return -4;
    if (planes == 2) LaunchRing<float, 2>(a, rst);
    else LaunchRing<float, 3>(a, rst);
    return hipGetLastError() == hipSuccess ? 0 : -3;
  }
  // f16 / bf16 row-run weights: form 0 = the strip form where it applies, else the row-run kernel; 1 = the
  // row-run kernel only; 3 = the strip form only
  if ((dtype == 1 || dtype == 2) && kp == kWideKP && form != 1 && RingOk(a, 1, 2)) {
    if (dtype == 1) LaunchRing<_Float16, 1>(a, rst);
    else LaunchRing<__bf16, 1>(a, rst);
    return hipGetLastError() == hipSuccess ? 0 : -3;
  }
  if (form == 3) return -4;
  if (dtype == 3 || dtype == 4) {  // fp32 input, weights [planes][Cout][160] bf16 (ops.conv.pack_stem_weight_f32)
    const int planes = dtype == 3 ? 2 : 3;
    if (kp != kStemKP || form == 1) return -1;
    if (!StemF32Ok(a, planes)) return -4;
    const dim3 grid(a.B * a.OH, (a.Cout + kStemBN - 1) / kStemBN);
    const size_t dyn = static_cast<size_t>(StemF32Lds(a, planes));
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (planes == 2) {
      if (a.in_scale) hipLaunchKernelGGL((stem_f32_kernel<2, true>), grid, dim3(256), dyn, st, a);
      else hipLaunchKernelGGL((stem_f32_kernel<2, false>), grid, dim3(256), dyn, st, a);
    } else {
      if (a.in_scale) hipLaunchKernelGGL((stem_f32_kernel<3, true>), grid, dim3(256), dyn, st, a);
      else hipLaunchKernelGGL((stem_f32_kernel<3, false>), grid, dim3(256), dyn, st, a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -3;
  }
  if (kp == kWideKP) {  // row-run form: weights packed [Cout][192], k = r * 24 + s * 3 + c
    if ((dtype != 1 && dtype != 2) || a.C != 3 || a.S * 3 > kWideRP || a.R > 8 || a.Cout < 1 || a.OH <= 0 ||
        a.OW <= 0 || a.B <= 0)
      return -1;
    if (static_cast<int64_t>(a.B) * a.OH * a.OW >= (1ll << 31)) return -5;
    if (static_cast<int64_t>(a.B) * a.H * a.W * 3 * 2 >= (1ll << 31) - 64) return -5;
    const int M = a.B * a.OH * a.OW;
    const dim3 grid((M + kStemBM - 1) / kStemBM, (a.Cout + kStemBN - 1) / kStemBN);
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (dtype == 1) {
      if (a.in_scale) hipLaunchKernelGGL((stem_wide_kernel<_Float16, true>), grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((stem_wide_kernel<_Float16, false>), grid, dim3(256), 0, st, a);
    } else {
      if (a.in_scale) hipLaunchKernelGGL((stem_wide_kernel<__bf16, true>), grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((stem_wide_kernel<__bf16, false>), grid, dim3(256), 0, st, a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -3;
  }
  if (kp != kStemKP) return -1;
  // the row-staged form where it applies (form 0 = auto, 1 = 2-byte gathers, 2 = row-staged)
  if (form != 1 && RowbufOk(a) && (dtype == 1 || dtype == 2) && a.Cout >= 1 && a.B > 0 && a.OH > 0 &&
      static_cast<int64_t>(a.B) * a.OH * a.OW < (1ll << 31) && static_cast<int64_t>(a.B) * a.H * a.W * 3 < (1ll << 31)) {
    const dim3 grid(a.B * a.OH, (a.Cout + kStemBN - 1) / kStemBN);
    const size_t dyn = static_cast<size_t>(RowbufLds(a));
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (dtype == 1) {
      if (a.in_scale) hipLaunchKernelGGL((stem_rowbuf_kernel<_Float16, true>), grid, dim3(256), dyn, st, a);
      else hipLaunchKernelGGL((stem_rowbuf_kernel<_Float16, false>), grid, dim3(256), dyn, st, a);
    } else {
      if (a.in_scale) hipLaunchKernelGGL((stem_rowbuf_kernel<__bf16, true>), grid, dim3(256), dyn, st, a);
      else hipLaunchKernelGGL((stem_rowbuf_kernel<__bf16, false>), grid, dim3(256), dyn, st, a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -3;
  }
  if (form == 2) return -4;  // row-staged form forced on a shape it does not take
  if ((dtype != 1 && dtype != 2) || a.C < 1 || a.C > 4 || a.R * a.S * a.C > kStemKP || a.Cout < 1 ||
      a.OH <= 0 || a.OW <= 0 || a.B <= 0)
    return -1;
  if (static_cast<int64_t>(a.B) * a.OH * a.OW >= (1ll << 31)) return -5;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int M = a.B * a.OH * a.OW;
  const dim3 grid((M + kStemBM - 1) / kStemBM, (a.Cout + kStemBN - 1) / kStemBN);
  if (a.S > 8 || a.R > 8) return -1;  // <= 8 x 8 taps: at most 4 (pixel, row) runs per thread
  if (static_cast<int64_t>(a.B) * a.H * a.W * a.C * 2 >= (1ll << 31)) return -5;
  auto launch = [&](auto k) { hipLaunchKernelGGL(k, grid, dim3(256), 0, st, a); };
  auto by_c = [&](auto tag, auto pro) {
    using T = decltype(tag);
    constexpr bool P = decltype(pro)::value;
    switch (a.C) {
      case 1: launch(stem_conv_kernel<T, 1, P>); break;
      case 2: launch(stem_conv_kernel<T, 2, P>); break;
      case 3: launch(stem_conv_kernel<T, 3, P>); break;
      default: launch(stem_conv_kernel<T, 4, P>); break;
    }
  };
  if (dtype == 1) {
    if (a.in_scale) by_c(_Float16{}, std::true_type{});
    else by_c(_Float16{}, std::false_type{});
  } else {
    if (a.in_scale) by_c(__bf16{}, std::true_type{});
    else by_c(__bf16{}, std::false_type{});
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// dtype: 0 fp32 (exact f32 MFMAs), 1 fp16, 2 bf16, 3 fp32 on 2 bf16 planes (3 products), 4 fp32 on 3 bf16
// planes (6 products), 5 / 6 = 3 / 4 with the weights pre-split (w = [planes][Cout][R][S][C] bf16)
// (C must be a multiple of one tile's K: 32 f32 / 64 f16/bf16 channels)
bool ConvMfmaSupported(int C, int Cout, int groups, int dtype) {
  const bool f32 = dtype == 0 || dtype >= 3;
  const int bk = f32 ? Tile<float>::BK : Tile<_Float16>::BK;
  return groups == 1 && C > 0 && C % bk == 0 && Cout > 0 && dtype >= 0 && dtype <= 6;
}

// Split-K for the default tiles when the output has too few tiles to give every CU two blocks (the deep
// ResNet layers: 7x7 / 14x14 maps at batch 128 make 196-392 tiles of 128x128 for 256 CUs) and the K loop is
// long: up to 8 splits of >= 4 K tiles each, aiming at >= 512 blocks. SML_CONV_SPLITK=0 disables, =N forces N.
int ConvSplitPlan(const ConvArgs& a, int dtype, int64_t* ws_floats, int* counters) {
  *ws_floats = 0;
  *counters = 0;
  if (a.kernel != 0 || EnvTile() != 0 || dtype < 0 || dtype > 6 || !ConvMfmaSupported(a.C, a.Cout, 1, dtype)) return 1;
  const bool half = dtype == 1 || dtype == 2;
  if (half && EnvGlds() && !a.in_scale) return 1;
  if (half && EnvPersist() && a.R * a.S * a.C <= 4 * 64) return 1;
  int bm = 128, bn = 128;
  if (dtype == 0 || a.Cout <= 64) bm = bn = 64;
  const int M = a.B * a.OH * a.OW;
  const int64_t tiles = static_cast<int64_t>((M + bm - 1) / bm) * ((a.Cout + bn - 1) / bn);
  const int nk = a.R * a.S * a.C / (half ? 64 : 32);
  static const int env = [] {
    const char* e = std::getenv("SML_CONV_SPLITK");
    return e ? std::atoi(e) : -1;
  }();
  int sk = 1;
  if (env >= 0) {
    sk = std::max(1, std::min(env, nk));
  } else if (tiles < 512 && nk >= 8) {
    sk = static_cast<int>(std::min<int64_t>({(512 + tiles - 1) / tiles, nk / 4, 8}));
  }
  if (sk > 1) {
    *ws_floats = tiles * sk * bm * bn;
    *counters = static_cast<int>(tiles);
  }
  return std::max(sk, 1);
}

int ConvMfma(const ConvArgs& a, int dtype, void* stream) {
  if (a.split_k < 1) return -6;
  if (a.kernel == kConvStem) {  // packed few-channel stem: C = 4, 8 x 8 taps, f16/bf16, no prologue
    if (a.split_k != 1) return -6;
    if (a.C != 4 || a.R != 8 || a.S != 8 || (dtype != 1 && dtype != 2) || a.in_scale || a.dil_h != 1 || a.dil_w != 1)
      return -1;
    if (a.OH <= 0 || a.OW <= 0 || a.B <= 0) return -2;
    if (static_cast<int64_t>(a.B) * a.H * a.W * a.C * 2 >= (1ll << 31)) return -5;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int rc = dtype == 1 ? LaunchStem<_Float16>(a, st) : LaunchStem<__bf16>(a, st);
    if (rc != 0) return rc;
    return hipGetLastError() == hipSuccess ? 0 : -3;
  }
  if (!ConvMfmaSupported(a.C, a.Cout, 1, dtype)) return -1;
  if (a.OH <= 0 || a.OW <= 0 || a.B <= 0) return -2;
  // buffer-resource offsets are 32-bit and the per-row tap mask holds 64 taps
  const int64_t es = (dtype == 0 || dtype >= 3) ? 4 : 2;
  if (static_cast<int64_t>(a.B) * a.H * a.W * a.C * es >= (1ll << 31) ||
      static_cast<int64_t>(a.Cout) * a.R * a.S * a.C * es >= (1ll << 31) || a.R * a.S > 64)
    return -5;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int rc = dtype == 0 ? Launch<float>(a, st)
                 : dtype == 1 ? Launch<_Float16>(a, st)
                 : dtype == 2 ? Launch<__bf16>(a, st)
                 : dtype == 3 ? Launch<float, 2>(a, st)
                 : dtype == 4 ? Launch<float, 3>(a, st)
                 : dtype == 5 ? Launch<float, 2, true>(a, st)
                              : Launch<float, 3, true>(a, st);
  if (rc != 0) return rc;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace smlnn
