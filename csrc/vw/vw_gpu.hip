// K12: hogwild mini-batch hashed SGD on the MI355X. One wave64 per example:
// lanes stride over the example's features, gather w[h & mask], reduce the dot
// product with DPP shuffles, evaluate the loss derivative once per wave and
// scatter AdaGrad updates back with float atomics (conflicts are rare in a
// 2^b table, which is what makes hogwild converge like sequential SGD).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "vw_gpu.h"

#define VW_HIP_CHECK(e)                                                                          \
  do {                                                                                           \
    hipError_t _e = (e);                                                                         \
    if (_e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e)); \
  } while (0)

namespace smlvw {
namespace {

constexpr int kWavesPerBlock = 4;

// ---------------------------------------------------------------- K13
// VW murmur3_32 of many strings at once: one thread per string over a packed
// UTF-8 byte buffer with (n + 1) offsets (the Arrow string-column layout), the
// featurizer's namespace hash as the seed and the feature mask applied on the
// way out. Bytes are read individually (strings start at arbitrary offsets);
// lanes of a wave hash neighbouring strings, so the loads stay coalesced.
__device__ __forceinline__ uint32_t Rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

__global__ __launch_bounds__(256) void murmur_batch_kernel(const uint8_t* __restrict__ bytes,
                                                           const int64_t* __restrict__ offsets, int64_t n,
                                                           uint32_t seed, uint32_t mask, uint32_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const uint8_t* d = bytes + offsets[i];
    const int64_t len = offsets[i + 1] - offsets[i];
    const int64_t nb = len / 4;
    uint32_t h = seed;
    const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
    for (int64_t b = 0; b < nb; ++b) {
      uint32_t k = static_cast<uint32_t>(d[4 * b]) | (static_cast<uint32_t>(d[4 * b + 1]) << 8) |
                   (static_cast<uint32_t>(d[4 * b + 2]) << 16) | (static_cast<uint32_t>(d[4 * b + 3]) << 24);
      k *= c1; k = Rotl(k, 15); k *= c2;
      h ^= k; h = Rotl(h, 13); h = h * 5 + 0xe6546b64u;
    }
    const uint8_t* t = d + 4 * nb;
    uint32_t k = 0;
    switch (len & 3) {
      case 3: k ^= static_cast<uint32_t>(t[2]) << 16; [[fallthrough]];
      case 2: k ^= static_cast<uint32_t>(t[1]) << 8; [[fallthrough]];
      case 1: k ^= t[0]; k *= c1; k = Rotl(k, 15); k *= c2; h ^= k;
    }
    h ^= static_cast<uint32_t>(len);
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    out[i] = h & mask;
  }
}

// ---------------------------------------------------------------- K12
// Weight slot = float4 {w, G (adaptive sum of squared gradients), N (normalizer: max |x| seen), -}: the
// CPU learner's stride-4 layout, so the exported table loads into the host model unchanged. One wave per
// (example, learner offset): lanes stride over the features, the dot product is a wave reduction, and the
// update follows the sequential learner's Update() (vw_core.cpp) step for step - VW's default
// adaptive + normalized + invariant ("safe") update or any subset of it:
//   pass 1: G += g^2 x^2 (adaptive); N = max(N, |x|), w rescaled when N grows (normalized);
//           rate = G^-1/2 * N^-1 (or N^-2 without adaptive); sum_x2rate, sum_norm_x (wave sums)
//   global: t, total weight, sum of feature norms (fp64 atomics): eta = lr * sqrt(tw / snx) (normalized,
//           adaptive) * (initial_t + t)^-power_t (non-adaptive)
//   update: importance-invariant closed form (squared) / bounded implicit step (logistic), else -g eta
//   pass 2: w += update * x * rate (+ l2), and the slot's 16 K-slot block is marked dirty for the sync.
// Hogwild: examples of a mini-batch run concurrently on atomics (conflicts are rare in a 2^b table);
// batch = 1 is the exact sequential learner.
constexpr int kDirtyShift = 12;  // dirty-tracking granularity: 4096 slots (64 KB) per block

struct SgdArgs {
  const int64_t* indptr;
  const uint32_t* idx;
  const float* val;
  const float* lab;    // scalar label, or the 1-based class for oaa
  const float* wt;     // importance (null = 1)
  const float* lo;     // running label range (prediction clamp), per example
  const float* hi;
  int64_t n0, n1;
  float4* W;
  uint64_t mask;
  uint8_t* dirty;
  double* gs;          // [t, total weight, sum of feature norms]
  float lr, power_t, initial_t, l2;
  int loss;            // 0 squared, 1 logistic
  int adaptive, normalized, invariant;
  int K;               // oaa classes (0: scalar learner)
  float* preds;
  float* loss_acc;
  int learn;
};

__device__ __forceinline__ float WaveSum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ float Dot(const SgdArgs& a, int64_t b, int64_t en, uint64_t off, int lane) {
  float s = 0.f;
  for (int64_t p = b + lane; p < en; p += 64) s += a.W[(a.idx[p] + off) & a.mask].x * a.val[p];
  return WaveSum(s);
}

__device__ __forceinline__ float Rate(const SgdArgs& a, float G, float N) {
  float r = 1.f;
  if (a.adaptive) r = G > 0.f ? rsqrtf(G) : 0.f;
  if (a.normalized) {
    const float inv = 1.f / N;
    r *= a.adaptive ? inv : inv * inv;
  }
  return r;
}

// One Update() of the sequential learner for (example rows [b, en), offset) at raw prediction `raw`, in two
// halves around the learner's global state (t, total weight, sum of normalised |x|^2): the first pass
// updates the touched slots' G and N and returns the wave sums the learning rate needs; the caller then
// advances the global state (one device atomic per block in sgd_kernel) and the second pass applies the
// update to the weights.
// Lanes keep the rates of their first kRateCache features from the first pass for the second (the
// sequential learner's second pass sees exactly those G / N); longer rows re-read the slots beyond.
constexpr int kRateCache = 4;

struct UpdPrep {
  float g, ppu, norm_x;
  float rate[kRateCache];
};

__device__ UpdPrep UpdateFirstPass(const SgdArgs& a, int64_t b, int64_t en, uint64_t off, float raw, float y,
                                   float imp, int lane) {
  UpdPrep pr;
  float g;
  if (a.loss == 1) g = -y / (1.f + expf(y * raw));
  else g = 2.f * (raw - y);
  const float grad_sq = g * g * imp;
  float ppu = 0.f, norm_x = 0.f;
  int k = 0;
  for (int64_t p = b + lane; p < en; p += 64, ++k) {
    const uint64_t h = (a.idx[p] + off) & a.mask;
    float4* w = &a.W[h];
    const float x = a.val[p];
    float x2 = x * x;
    if (x2 < FLT_MIN) x2 = FLT_MIN;
    float G = 0.f, N = 1.f;
    // G and N come back from returning atomics: in a hogwild batch of examples sharing dense features, each
    // update must see the accumulators of the updates serialized before it (a plain load would hand every
    // concurrent example the same tiny G and a huge first-step rate - measured: AUC 0.65 instead of 0.998)
    if (a.adaptive) G = atomicAdd(&w->y, grad_sq * x2) + grad_sq * x2;
    if (a.normalized) {
      const float ax = fabsf(x);
      // N only grows: the float bits of non-negative values order like unsigned integers
      const float old = __uint_as_float(atomicMax(reinterpret_cast<unsigned int*>(&w->z), __float_as_uint(ax)));
      if (ax > old && old > 0.f) {
        const float r = old / ax;
        w->x *= a.adaptive ? r : r * r;  // hogwild rescale of this slot's weight
      }
      N = fmaxf(old, ax);
      norm_x += x2 / (N * N);
    }
    const float rt = Rate(a, G, N);
    if (k < kRateCache) pr.rate[k] = rt;
    ppu += x2 * rt;
  }
  pr.g = g;
  pr.ppu = WaveSum(ppu);
  pr.norm_x = WaveSum(norm_x);
  return pr;
}

// t, tw, snx: the global state including this update (what the sequential learner sees)
__device__ void UpdateSecondPass(const SgdArgs& a, int64_t b, int64_t en, uint64_t off, float raw, float y,
                                 float imp, int lane, const UpdPrep& pr, double t, double tw, double snx) {
  double eta = a.lr;
  if (a.normalized && snx > 0.0) {
    const double avg = tw / snx;
    eta *= a.adaptive ? sqrt(avg) : avg;
  }
  if (!a.adaptive) eta *= pow(static_cast<double>(a.initial_t) + t, -static_cast<double>(a.power_t));
  const float us = static_cast<float>(eta) * imp;
  float update;
  if (a.invariant) {
    const float pp = fmaxf(pr.ppu, FLT_MIN);
    if (a.loss == 0) {
      update = us * pp < 1e-6f ? 2.f * (y - raw) * us : (y - raw) * (1.f - expf(-2.f * us * pp)) / pp;
    } else {
      const float step = y * us / (1.f + expf(y * raw));
      update = fabsf(step * pp) > 50.f ? copysignf(50.f / pp, step) : step;
    }
  } else {
    update = -pr.g * us;
  }
  const float decay = static_cast<float>(eta) * a.l2;
  int k = 0;
  for (int64_t p = b + lane; p < en; p += 64, ++k) {
    const uint64_t h = (a.idx[p] + off) & a.mask;
    float4* w = &a.W[h];
    const float x = a.val[p];
    const float rate = k < kRateCache ? pr.rate[k] : Rate(a, a.adaptive ? w->y : 0.f, a.normalized ? w->z : 1.f);
    if (decay > 0.f) {
      const float nw = atomicAdd(&w->x, update * x * rate) + update * x * rate;
      atomicAdd(&w->x, -decay * nw);
    } else {
      atomicAdd(&w->x, update * x * rate);  // result unused: a non-returning atomic
    }
    a.dirty[h >> kDirtyShift] = 1;
  }
}

// whole update with its own global-state step (oaa: one per class update)
__device__ void UpdateWave(const SgdArgs& a, int64_t b, int64_t en, uint64_t off, float raw, float y, float imp,
                           int lane) {
  const UpdPrep pr = UpdateFirstPass(a, b, en, off, raw, y, imp, lane);
  double t = 0.0, tw = 0.0, snx = 0.0;
  if (lane == 0) {
    t = atomicAdd(&a.gs[0], static_cast<double>(imp)) + imp;
    tw = atomicAdd(&a.gs[1], static_cast<double>(imp)) + imp;
    const double dn = static_cast<double>(imp) * pr.norm_x;
    snx = atomicAdd(&a.gs[2], dn) + dn;
  }
  t = __shfl(t, 0, 64); tw = __shfl(tw, 0, 64); snx = __shfl(snx, 0, 64);
  UpdateSecondPass(a, b, en, off, raw, y, imp, lane, pr, t, tw, snx);
}

__device__ __forceinline__ float LossOf(int loss, float p, float y) {
  if (loss == 1) return log1pf(expf(-y * p));
  return (p - y) * (p - y);
}

// scalar learners: one wave per example, kSgdWaves examples per block. The global learner state advances
// with ONE device atomic per component per block (block sum; each wave takes its prefix), not one per
// example: every update's t / tw / snx still includes exactly the updates ordered before it, and a
// one-example launch (gpuBatchSize=1) is the sequential learner.
constexpr int kSgdWaves = 16;

__global__ __launch_bounds__(64 * kSgdWaves) void sgd_kernel(SgdArgs a) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t e = a.n0 + static_cast<int64_t>(blockIdx.x) * kSgdWaves + wid;
  __shared__ float wloss[kSgdWaves];
  __shared__ double s_imp[kSgdWaves], s_nx[kSgdWaves], s_base[3];
  const bool act = e < a.n1;
  int64_t b = 0, en = 0;
  float raw = 0.f, y = 0.f, imp = 0.f;
  if (lane == 0) wloss[wid] = 0.f;
  if (act) {
    b = a.indptr[e]; en = a.indptr[e + 1];
    raw = Dot(a, b, en, 0, lane);
    float p = isnan(raw) ? 0.f : raw;
    if (a.lo) p = fminf(fmaxf(p, a.lo[e]), a.hi[e]);  // the learner's running label range
    if (a.preds && lane == 0) a.preds[e] = p;
    if (a.learn) {
      y = a.lab[e];
      imp = a.wt ? a.wt[e] : 1.f;
      if (lane == 0) wloss[wid] = LossOf(a.loss, p, y) * imp;
    }
  }
  if (!a.learn) return;  // uniform over the launch
  const bool upd = act && imp > 0.f;
  UpdPrep pr{0.f, 0.f, 0.f};
  if (upd) pr = UpdateFirstPass(a, b, en, 0, raw, y, imp, lane);
  if (lane == 0) {
    s_imp[wid] = upd ? static_cast<double>(imp) : 0.0;
    s_nx[wid] = upd ? static_cast<double>(imp) * pr.norm_x : 0.0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double si = 0.0, sn = 0.0;
    float sl = 0.f;
    for (int w = 0; w < kSgdWaves; ++w) { si += s_imp[w]; sn += s_nx[w]; sl += wloss[w]; }
    s_base[0] = si > 0.0 ? atomicAdd(&a.gs[0], si) : 0.0;
    s_base[1] = si > 0.0 ? atomicAdd(&a.gs[1], si) : 0.0;
    s_base[2] = sn > 0.0 ? atomicAdd(&a.gs[2], sn) : 0.0;
    atomicAdd(a.loss_acc, sl);
  }
  __syncthreads();
  if (!upd) return;
  double pi = 0.0, pn = 0.0;
  for (int w = 0; w <= wid; ++w) { pi += s_imp[w]; pn += s_nx[w]; }
  UpdateSecondPass(a, b, en, 0, raw, y, imp, lane, pr, s_base[0] + pi, s_base[1] + pi, s_base[2] + pn);
}

// --oaa K: one block per example, wave c handles classes c, c + waves, ...: scores (predict), then the
// per-class binary updates (label +1 for the true class, -1 otherwise) at the class offsets
constexpr uint64_t kOaaOffset = 1315423911ull;
constexpr int kOaaMaxWaves = 8;

__global__ __launch_bounds__(64 * kOaaMaxWaves) void oaa_kernel(SgdArgs a) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int64_t e = a.n0 + blockIdx.x;
  if (e >= a.n1) return;
  extern __shared__ float scores[];
  const int64_t b = a.indptr[e], en = a.indptr[e + 1];
  for (int k = wid; k < a.K; k += nw) {
    const float s = Dot(a, b, en, static_cast<uint64_t>(k) * kOaaOffset, lane);
    if (lane == 0) scores[k] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int best = 0;
    for (int k = 1; k < a.K; ++k) if (scores[k] > scores[best]) best = k;
    if (a.preds) a.preds[e] = static_cast<float>(best + 1);
    if (a.learn) atomicAdd(a.loss_acc, (best + 1 == static_cast<int>(a.lab[e]) ? 0.f : 1.f) * (a.wt ? a.wt[e] : 1.f));
  }
  if (!a.learn) return;
  const float imp = a.wt ? a.wt[e] : 1.f;
  if (imp <= 0.f) return;
  const int y = static_cast<int>(a.lab[e]);
  for (int k = wid; k < a.K; k += nw) UpdateWave(a, b, en, static_cast<uint64_t>(k) * kOaaOffset, scores[k],
                                                 k + 1 == y ? 1.f : -1.f, imp, lane);
}

// Sync payload per slot: double {w G (adaptive) or w, G} + float N. The weighted sum goes in double: a
// float w * G underflows (and is flushed) for slots with a tiny gradient mass, which would zero their
// weight on the average even at world 1.
__global__ void pack_kernel(const float4* __restrict__ W, const int32_t* __restrict__ blocks, int64_t nblk,
                            uint64_t nw, int adaptive, double* __restrict__ sums, float* __restrict__ nmax) {
  constexpr int64_t B = int64_t(1) << kDirtyShift;
  const int64_t m = nblk * B;
  for (int64_t j = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; j < m;
       j += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const uint64_t slot = static_cast<uint64_t>(blocks[j >> kDirtyShift]) * B + (j & (B - 1));
    const float4 v = slot < nw ? W[slot] : make_float4(0.f, 0.f, 0.f, 0.f);
    sums[2 * j] = adaptive ? static_cast<double>(v.x) * v.y : static_cast<double>(v.x);
    sums[2 * j + 1] = v.y;
    nmax[j] = v.z;
  }
}

// VW's weighted averaging: with adaptive state w = sum(w G) / sum(G) (a slot no rank has gradient mass
// on was never updated and keeps its value), G = sum(G) / world; N = max(N); without adaptive
// w = sum(w) / world
__global__ void unpack_kernel(float4* __restrict__ W, const int32_t* __restrict__ blocks, int64_t nblk, uint64_t nw,
                              int adaptive, double inv_world, const double* __restrict__ sums,
                              const float* __restrict__ nmax) {
  constexpr int64_t B = int64_t(1) << kDirtyShift;
  const int64_t m = nblk * B;
  for (int64_t j = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; j < m;
       j += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const uint64_t slot = static_cast<uint64_t>(blocks[j >> kDirtyShift]) * B + (j & (B - 1));
    if (slot >= nw) continue;
    float4 v = W[slot];
    const double s0 = sums[2 * j], sg = sums[2 * j + 1];
    if (!adaptive) v.x = static_cast<float>(s0 * inv_world);
    else if (sg > 0.0) v.x = static_cast<float>(s0 / sg);
    v.y = static_cast<float>(sg * inv_world);
    v.z = nmax[j];
    W[slot] = v;
  }
}

__global__ void dirty_list_kernel(const uint8_t* __restrict__ dirty, int64_t nblk, const int32_t* __restrict__ pos,
                                  int32_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < nblk;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    if (dirty[i]) out[pos[i]] = static_cast<int32_t>(i);
}

// nonzero components of the table -> (stride-4 index, value) records (model export, no host table)
__global__ void count_nz_kernel(const float4* __restrict__ W, uint64_t nw, uint64_t per, int32_t* __restrict__ cnt) {
  const uint64_t s0 = static_cast<uint64_t>(blockIdx.x) * per, s1 = min(nw, s0 + per);
  int c = 0;
  for (uint64_t s = s0 + threadIdx.x; s < s1; s += blockDim.x) {
    const float4 v = W[s];
    c += (v.x != 0.f) + (v.y != 0.f) + (v.z != 0.f);
  }
  c = static_cast<int>(WaveSum(static_cast<float>(c)));
  __shared__ int ws[4];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ void write_nz_kernel(const float4* __restrict__ W, uint64_t nw, uint64_t per, const int64_t* __restrict__ base,
                                uint64_t* __restrict__ oidx, float* __restrict__ oval) {
  // one thread per block keeps the records in slot order (the host model's order) - blocks are small
  if (threadIdx.x != 0) return;
  const uint64_t s0 = static_cast<uint64_t>(blockIdx.x) * per, s1 = min(nw, s0 + per);
  int64_t o = base[blockIdx.x];
  for (uint64_t s = s0; s < s1; ++s) {
    const float4 v = W[s];
    if (v.x != 0.f) { oidx[o] = 4 * s; oval[o++] = v.x; }
    if (v.y != 0.f) { oidx[o] = 4 * s + 1; oval[o++] = v.y; }
    if (v.z != 0.f) { oidx[o] = 4 * s + 2; oval[o++] = v.z; }
  }
}

__global__ void scatter_kernel(float4* __restrict__ W, uint64_t nw, const uint64_t* __restrict__ idx,
                               const float* __restrict__ val, int64_t n) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const uint64_t s = idx[i] >> 2;
    const int c = static_cast<int>(idx[i] & 3);
    if (s < nw && c < 3) reinterpret_cast<float*>(&W[s])[c] = val[i];
  }
}

}  // namespace

// Host -> HBM copies of a pass's CSR through pinned staging buffers: the pageable path stages through one
// runtime memcpy thread (~25 GB/s, and a 2M x 64-nonzero pass is 1 GB); here kStage buffers are filled by
// kStageThreads CPU threads in parallel and drained by the copy engine, the CPU copy of piece k+1
// overlapping the DMA of piece k.
namespace {
constexpr int kStage = 4;
constexpr size_t kStageBytes = 32ull << 20;
constexpr int kStageThreads = 8;

// One per learner (its events are recorded on that learner's copy stream only), buffers allocated on first use.
struct Stager {
  std::mutex mu;
  char* buf[kStage] = {};
  hipEvent_t ev[kStage] = {};
  bool used[kStage] = {};
  int next = 0;
  ~Stager() {
    for (int k = 0; k < kStage; ++k) {
      if (ev[k]) { (void)hipEventSynchronize(ev[k]); (void)hipEventDestroy(ev[k]); }
      if (buf[k]) (void)hipHostFree(buf[k]);
    }
  }
  // queue `bytes` from pageable `src` to device `dst` on stream s (caller holds mu)
  void Copy(char* dst, const char* src, size_t bytes, hipStream_t s) {
    for (size_t off = 0; off < bytes; off += kStageBytes) {
      const int k = next;
      next = (next + 1) % kStage;
      if (!buf[k]) {
        VW_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&buf[k]), kStageBytes, hipHostMallocDefault));
        VW_HIP_CHECK(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
      }
      if (used[k]) VW_HIP_CHECK(hipEventSynchronize(ev[k]));
      const size_t n = std::min(kStageBytes, bytes - off);
      if (n < (1u << 20)) {
        std::memcpy(buf[k], src + off, n);  // small pieces: a thread team costs more than the copy
      } else {
        const size_t per = (n + kStageThreads - 1) / kStageThreads;
        std::vector<std::thread> th;
        for (int t = 0; t < kStageThreads && t * per < n; ++t) {
          const size_t a0 = t * per, a1 = std::min(n, a0 + per);
          th.emplace_back([=]() { std::memcpy(buf[k] + a0, src + off + a0, a1 - a0); });
        }
        for (auto& x : th) x.join();
      }
      VW_HIP_CHECK(hipMemcpyAsync(dst + off, buf[k], n, hipMemcpyHostToDevice, s));
      VW_HIP_CHECK(hipEventRecord(ev[k], s));
      used[k] = true;
    }
  }
};
}  // namespace

struct GpuSgd::Impl {
  hipStream_t stream = nullptr, copy_stream = nullptr;
  Stager stager;  // pinned host->device staging of pass data (copy_stream)
  std::vector<hipEvent_t> events;
  float4* W = nullptr;
  uint64_t nw = 0;
  uint8_t* dirty = nullptr;
  int64_t nblk = 0;
  double* gs = nullptr;
  int64_t* indptr = nullptr;
  uint32_t* idx = nullptr;
  float *val = nullptr, *lab = nullptr, *wt = nullptr, *lo = nullptr, *hi = nullptr, *pred = nullptr, *loss = nullptr;
  size_t cap_rows = 0, cap_nnz = 0;
  // sync scratch
  int32_t *pos = nullptr, *blocks = nullptr;
  double* sums = nullptr;
  float* nmax = nullptr;
  size_t cap_sync = 0;
  void Reserve(size_t rows, size_t nnz) {
    if (rows > cap_rows) {
      for (void* q : {static_cast<void*>(indptr), static_cast<void*>(lab), static_cast<void*>(wt), static_cast<void*>(lo),
                      static_cast<void*>(hi), static_cast<void*>(pred)})
        (void)hipFree(q);
      VW_HIP_CHECK(hipMalloc(&indptr, (rows + 1) * sizeof(int64_t)));
      VW_HIP_CHECK(hipMalloc(&lab, rows * sizeof(float)));
      VW_HIP_CHECK(hipMalloc(&wt, rows * sizeof(float)));
      VW_HIP_CHECK(hipMalloc(&lo, rows * sizeof(float)));
      VW_HIP_CHECK(hipMalloc(&hi, rows * sizeof(float)));
      VW_HIP_CHECK(hipMalloc(&pred, rows * sizeof(float)));
      cap_rows = rows;
    }
    if (nnz > cap_nnz) {
      (void)hipFree(idx); (void)hipFree(val);
      VW_HIP_CHECK(hipMalloc(&idx, std::max<size_t>(1, nnz) * sizeof(uint32_t)));
      VW_HIP_CHECK(hipMalloc(&val, std::max<size_t>(1, nnz) * sizeof(float)));
      cap_nnz = nnz;
    }
  }
  ~Impl() {
    if (stream) (void)hipStreamSynchronize(stream);
    if (copy_stream) (void)hipStreamSynchronize(copy_stream);
    for (hipEvent_t e : events) (void)hipEventDestroy(e);
    if (copy_stream) (void)hipStreamDestroy(copy_stream);
    for (void* q : {static_cast<void*>(W), static_cast<void*>(dirty), static_cast<void*>(gs),
                    static_cast<void*>(indptr), static_cast<void*>(idx), static_cast<void*>(val),
                    static_cast<void*>(lab), static_cast<void*>(wt), static_cast<void*>(lo), static_cast<void*>(hi),
                    static_cast<void*>(pred), static_cast<void*>(loss), static_cast<void*>(pos),
                    static_cast<void*>(blocks), static_cast<void*>(sums), static_cast<void*>(nmax)})
      (void)hipFree(q);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

void MurmurBatchGpu(const uint8_t* bytes, int64_t nbytes, const int64_t* offsets, int64_t n, uint32_t seed,
                    uint32_t mask, uint32_t* out) {
  if (n <= 0) return;
  hipStream_t st = nullptr;
  VW_HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  uint8_t* db = nullptr;
  int64_t* doff = nullptr;
  uint32_t* dout = nullptr;
  try {
    VW_HIP_CHECK(hipMallocAsync(reinterpret_cast<void**>(&db), static_cast<size_t>(std::max<int64_t>(1, nbytes)), st));
    VW_HIP_CHECK(hipMallocAsync(reinterpret_cast<void**>(&doff), sizeof(int64_t) * (n + 1), st));
    VW_HIP_CHECK(hipMallocAsync(reinterpret_cast<void**>(&dout), sizeof(uint32_t) * n, st));
    if (nbytes > 0) VW_HIP_CHECK(hipMemcpyAsync(db, bytes, nbytes, hipMemcpyHostToDevice, st));
    VW_HIP_CHECK(hipMemcpyAsync(doff, offsets, sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice, st));
    const int grid = static_cast<int>(std::min<int64_t>((n + 255) / 256, 65536));
    hipLaunchKernelGGL(murmur_batch_kernel, dim3(grid), dim3(256), 0, st, db, doff, n, seed, mask, dout);
    VW_HIP_CHECK(hipGetLastError());
    VW_HIP_CHECK(hipMemcpyAsync(out, dout, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, st));
    VW_HIP_CHECK(hipStreamSynchronize(st));
  } catch (...) {
    (void)hipStreamSynchronize(st);
    (void)hipFree(db); (void)hipFree(doff); (void)hipFree(dout);
    (void)hipStreamDestroy(st);
    throw;
  }
  (void)hipFreeAsync(db, st); (void)hipFreeAsync(doff, st); (void)hipFreeAsync(dout, st);
  (void)hipStreamSynchronize(st);
  (void)hipStreamDestroy(st);
}

bool VwGpuAvailable() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) { (void)hipGetLastError(); return false; }
  return n > 0;
}

GpuSgd::GpuSgd(const GpuSgdConfig& cfg, int device) : impl_(new Impl()), cfg_(cfg) {
  if (device >= 0) VW_HIP_CHECK(hipSetDevice(device));
  if (cfg.oaa > 256) throw std::runtime_error("GPU oaa supports at most 256 classes");
  VW_HIP_CHECK(hipStreamCreateWithFlags(&impl_->stream, hipStreamNonBlocking));
  VW_HIP_CHECK(hipStreamCreateWithFlags(&impl_->copy_stream, hipStreamNonBlocking));
  impl_->nw = 1ull << cfg.bits;
  VW_HIP_CHECK(hipMalloc(&impl_->W, impl_->nw * sizeof(float4)));
  VW_HIP_CHECK(hipMemsetAsync(impl_->W, 0, impl_->nw * sizeof(float4), impl_->stream));
  impl_->nblk = static_cast<int64_t>((impl_->nw + (1ull << kDirtyShift) - 1) >> kDirtyShift);
  VW_HIP_CHECK(hipMalloc(&impl_->dirty, impl_->nblk));
  VW_HIP_CHECK(hipMemsetAsync(impl_->dirty, 0, impl_->nblk, impl_->stream));
  VW_HIP_CHECK(hipMalloc(&impl_->gs, 3 * sizeof(double)));
  VW_HIP_CHECK(hipMemsetAsync(impl_->gs, 0, 3 * sizeof(double), impl_->stream));
  VW_HIP_CHECK(hipMalloc(&impl_->loss, sizeof(float)));
  VW_HIP_CHECK(hipMemsetAsync(impl_->loss, 0, sizeof(float), impl_->stream));
  VW_HIP_CHECK(hipStreamSynchronize(impl_->stream));
  if (cfg.loss == 1) { min_label_ = -50.0; max_label_ = 50.0; }
}

GpuSgd::~GpuSgd() = default;

namespace {
SgdArgs BaseArgs(const GpuSgdConfig& c) {
  SgdArgs a{};
  a.lr = c.lr; a.power_t = c.power_t; a.initial_t = c.initial_t; a.l2 = c.l2; a.loss = c.loss;
  a.adaptive = c.adaptive ? 1 : 0; a.normalized = c.normalized ? 1 : 0; a.invariant = c.invariant ? 1 : 0;
  a.K = c.oaa;
  return a;
}
}  // namespace

void GpuSgd::Launch(int64_t b0, int64_t b1, bool learn, bool have_weights) {
  SgdArgs a = BaseArgs(cfg_);
  a.indptr = impl_->indptr; a.idx = impl_->idx; a.val = impl_->val; a.lab = impl_->lab;
  a.wt = have_weights ? impl_->wt : nullptr;
  a.lo = (learn && cfg_.oaa == 0) ? impl_->lo : nullptr;
  a.hi = impl_->hi;
  a.n0 = b0; a.n1 = b1; a.W = impl_->W; a.mask = impl_->nw - 1; a.dirty = impl_->dirty; a.gs = impl_->gs;
  a.preds = impl_->pred; a.loss_acc = impl_->loss; a.learn = learn ? 1 : 0;
  if (cfg_.oaa > 0) {
    const int waves = std::min(cfg_.oaa, kOaaMaxWaves);
    hipLaunchKernelGGL(oaa_kernel, dim3(static_cast<unsigned>(b1 - b0)), dim3(64 * waves), sizeof(float) * cfg_.oaa,
                       impl_->stream, a);
  } else {
    const int grid = static_cast<int>((b1 - b0 + kSgdWaves - 1) / kSgdWaves);
    hipLaunchKernelGGL(sgd_kernel, dim3(grid), dim3(64 * kSgdWaves), 0, impl_->stream, a);
  }
  VW_HIP_CHECK(hipGetLastError());
}

void GpuSgd::Learn(const int64_t* indptr, const uint32_t* indices, const float* values, const float* labels,
                   const float* weights, int64_t n, int batch, float* preds_out) {
  if (n <= 0) return;
  const size_t nnz = static_cast<size_t>(indptr[n] - indptr[0]);
  impl_->Reserve(n, nnz);
  hipStream_t s = impl_->stream, cs = impl_->copy_stream;
  std::vector<int64_t> ip(indptr, indptr + n + 1);
  for (auto& v : ip) v -= indptr[0];
  // the sequential learner's running label range (squared loss: starts at [0, 0], grows with every label
  // before the example is predicted; logistic: fixed [-50, 50]) -> per-example clamp bounds
  std::vector<float> lo(n), hi(n);
  for (int64_t i = 0; i < n; ++i) {
    if (cfg_.loss != 1 && cfg_.oaa == 0) {
      min_label_ = std::min<double>(min_label_, labels[i]);
      max_label_ = std::max<double>(max_label_, labels[i]);
    }
    lo[i] = static_cast<float>(min_label_);
    hi[i] = static_cast<float>(max_label_);
  }
  VW_HIP_CHECK(hipMemcpyAsync(impl_->indptr, ip.data(), (n + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  VW_HIP_CHECK(hipMemcpyAsync(impl_->lab, labels, n * sizeof(float), hipMemcpyHostToDevice, s));
  VW_HIP_CHECK(hipMemcpyAsync(impl_->lo, lo.data(), n * sizeof(float), hipMemcpyHostToDevice, s));
  VW_HIP_CHECK(hipMemcpyAsync(impl_->hi, hi.data(), n * sizeof(float), hipMemcpyHostToDevice, s));
  if (weights) VW_HIP_CHECK(hipMemcpyAsync(impl_->wt, weights, n * sizeof(float), hipMemcpyHostToDevice, s));
  VW_HIP_CHECK(hipMemsetAsync(impl_->loss, 0, sizeof(float), s));
  batch = std::max(1, batch);
  // The pass's feature ids / values stream in chunks of 16 mini-batches: a native thread copies chunk
  // k+1 through the pinned stager on the copy stream while the device learns chunk k (the launch loop waits
  // on the host until a chunk's event is recorded, then on the device for the copy itself).
  const int64_t chunk_rows = static_cast<int64_t>(batch) * 16;
  const int64_t nchunks = (n + chunk_rows - 1) / chunk_rows;
  for (size_t i = impl_->events.size(); i < static_cast<size_t>(nchunks); ++i) {
    hipEvent_t e;
    VW_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    impl_->events.push_back(e);
  }
  std::mutex rmu;
  std::condition_variable rcv;
  int64_t recorded = 0;
  std::string upload_error;
  const int dev = [] { int d = 0; (void)hipGetDevice(&d); return d; }();
  std::thread uploader([&]() {
    try {
      VW_HIP_CHECK(hipSetDevice(dev));
      Stager& st = impl_->stager;
      std::lock_guard<std::mutex> lk(st.mu);
      for (int64_t c = 0; c < nchunks; ++c) {
        const int64_t r0 = c * chunk_rows, r1 = std::min<int64_t>(n, r0 + chunk_rows);
        const size_t p0 = static_cast<size_t>(ip[r0]), p1 = static_cast<size_t>(ip[r1]);
        if (p1 > p0) {
          st.Copy(reinterpret_cast<char*>(impl_->idx + p0), reinterpret_cast<const char*>(indices + indptr[0] + p0),
                  (p1 - p0) * sizeof(uint32_t), cs);
          st.Copy(reinterpret_cast<char*>(impl_->val + p0), reinterpret_cast<const char*>(values + indptr[0] + p0),
                  (p1 - p0) * sizeof(float), cs);
        }
        VW_HIP_CHECK(hipEventRecord(impl_->events[c], cs));
        std::lock_guard<std::mutex> g(rmu);
        recorded = c + 1;
        rcv.notify_all();
      }
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> g(rmu);
      upload_error = e.what();
      recorded = nchunks;  // release the launch loop; it rethrows
      rcv.notify_all();
    }
  });
  try {
    for (int64_t c = 0; c < nchunks; ++c) {
      {
        std::unique_lock<std::mutex> g(rmu);
        rcv.wait(g, [&] { return recorded > c; });
        if (!upload_error.empty()) break;
      }
      VW_HIP_CHECK(hipStreamWaitEvent(s, impl_->events[c], 0));
      const int64_t r0 = c * chunk_rows, r1 = std::min<int64_t>(n, r0 + chunk_rows);
      for (int64_t b0 = r0; b0 < r1; b0 += batch) Launch(b0, std::min<int64_t>(r1, b0 + batch), true, weights != nullptr);
    }
  } catch (...) {
    uploader.join();
    throw;
  }
  uploader.join();
  if (!upload_error.empty()) throw std::runtime_error("VW pass upload failed: " + upload_error);
  float l = 0;
  VW_HIP_CHECK(hipMemcpyAsync(&l, impl_->loss, sizeof(float), hipMemcpyDeviceToHost, s));
  if (preds_out) VW_HIP_CHECK(hipMemcpyAsync(preds_out, impl_->pred, n * sizeof(float), hipMemcpyDeviceToHost, s));
  VW_HIP_CHECK(hipStreamSynchronize(s));
  examples_ += n;
  sum_loss_ += l;
}

// Device-resident pass data (VW's cache for multi-pass training): the CSR, labels and weights are uploaded
// once; LearnStaged(r0, r1) then learns rows [r0, r1) from HBM - passes and sync segments re-read nothing
// over PCIe. Only the per-row label-range clamp bounds of the rows being learned move (8 B / row).
void GpuSgd::Stage(const int64_t* indptr, const uint32_t* indices, const float* values, const float* labels,
                   const float* weights, int64_t n) {
  if (n < 0) throw std::runtime_error("negative row count");
  const size_t nnz = static_cast<size_t>(n ? indptr[n] - indptr[0] : 0);
  impl_->Reserve(std::max<int64_t>(1, n), nnz);
  hipStream_t s = impl_->stream, cs = impl_->copy_stream;
  std::vector<int64_t> ip(indptr, indptr + n + 1);
  for (auto& v : ip) v -= indptr[0];
  VW_HIP_CHECK(hipMemcpyAsync(impl_->indptr, ip.data(), (n + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  if (n) {
    VW_HIP_CHECK(hipMemcpyAsync(impl_->lab, labels, n * sizeof(float), hipMemcpyHostToDevice, s));
    if (weights) VW_HIP_CHECK(hipMemcpyAsync(impl_->wt, weights, n * sizeof(float), hipMemcpyHostToDevice, s));
  }
  if (nnz) {
    Stager& st = impl_->stager;
    std::lock_guard<std::mutex> lk(st.mu);
    st.Copy(reinterpret_cast<char*>(impl_->idx), reinterpret_cast<const char*>(indices + indptr[0]),
            nnz * sizeof(uint32_t), cs);
    st.Copy(reinterpret_cast<char*>(impl_->val), reinterpret_cast<const char*>(values + indptr[0]), nnz * sizeof(float),
            cs);
    VW_HIP_CHECK(hipStreamSynchronize(cs));
  }
  VW_HIP_CHECK(hipStreamSynchronize(s));
  staged_labels_.assign(labels, labels + n);
  staged_n_ = n;
  staged_weights_ = weights != nullptr;
}

void GpuSgd::LearnStaged(int64_t r0, int64_t r1, int batch, float* preds_out) {
  if (r0 < 0 || r1 > staged_n_ || r0 > r1) throw std::runtime_error("LearnStaged: rows outside the staged set");
  if (r1 == r0) return;
  hipStream_t s = impl_->stream;
  const int64_t m = r1 - r0;
  std::vector<float> lo(m), hi(m);
  for (int64_t i = 0; i < m; ++i) {
    if (cfg_.loss != 1 && cfg_.oaa == 0) {
      min_label_ = std::min<double>(min_label_, staged_labels_[r0 + i]);
      max_label_ = std::max<double>(max_label_, staged_labels_[r0 + i]);
    }
    lo[i] = static_cast<float>(min_label_);
    hi[i] = static_cast<float>(max_label_);
  }
  VW_HIP_CHECK(hipMemcpyAsync(impl_->lo + r0, lo.data(), m * sizeof(float), hipMemcpyHostToDevice, s));
  VW_HIP_CHECK(hipMemcpyAsync(impl_->hi + r0, hi.data(), m * sizeof(float), hipMemcpyHostToDevice, s));
  VW_HIP_CHECK(hipMemsetAsync(impl_->loss, 0, sizeof(float), s));
  batch = std::max(1, batch);
  for (int64_t b0 = r0; b0 < r1; b0 += batch) Launch(b0, std::min<int64_t>(r1, b0 + batch), true, staged_weights_);
  float l = 0;
  VW_HIP_CHECK(hipMemcpyAsync(&l, impl_->loss, sizeof(float), hipMemcpyDeviceToHost, s));
  if (preds_out) VW_HIP_CHECK(hipMemcpyAsync(preds_out, impl_->pred + r0, m * sizeof(float), hipMemcpyDeviceToHost, s));
  VW_HIP_CHECK(hipStreamSynchronize(s));
  examples_ += m;
  sum_loss_ += l;
}

void GpuSgd::Predict(const int64_t* indptr, const uint32_t* indices, const float* values, int64_t n, float* out) {
  if (n <= 0) return;
  const size_t nnz = static_cast<size_t>(indptr[n] - indptr[0]);
  impl_->Reserve(n, nnz);
  hipStream_t s = impl_->stream;
  std::vector<int64_t> ip(indptr, indptr + n + 1);
  for (auto& v : ip) v -= indptr[0];
  std::vector<float> lo(n, static_cast<float>(min_label_)), hi(n, static_cast<float>(max_label_));
  VW_HIP_CHECK(hipMemcpyAsync(impl_->indptr, ip.data(), (n + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  VW_HIP_CHECK(hipMemcpyAsync(impl_->lo, lo.data(), n * sizeof(float), hipMemcpyHostToDevice, s));
  VW_HIP_CHECK(hipMemcpyAsync(impl_->hi, hi.data(), n * sizeof(float), hipMemcpyHostToDevice, s));
  if (nnz) {
    VW_HIP_CHECK(hipMemcpyAsync(impl_->idx, indices + indptr[0], nnz * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    VW_HIP_CHECK(hipMemcpyAsync(impl_->val, values + indptr[0], nnz * sizeof(float), hipMemcpyHostToDevice, s));
  }
  SgdArgs a = BaseArgs(cfg_);
  a.indptr = impl_->indptr; a.idx = impl_->idx; a.val = impl_->val;
  a.lo = cfg_.oaa == 0 ? impl_->lo : nullptr; a.hi = impl_->hi;
  a.n0 = 0; a.n1 = n; a.W = impl_->W; a.mask = impl_->nw - 1; a.dirty = impl_->dirty; a.gs = impl_->gs;
  a.preds = impl_->pred; a.loss_acc = impl_->loss; a.learn = 0;
  if (cfg_.oaa > 0) {
    const int waves = std::min(cfg_.oaa, kOaaMaxWaves);
    hipLaunchKernelGGL(oaa_kernel, dim3(static_cast<unsigned>(n)), dim3(64 * waves), sizeof(float) * cfg_.oaa, s, a);
  } else {
    hipLaunchKernelGGL(sgd_kernel, dim3(static_cast<unsigned>((n + kSgdWaves - 1) / kSgdWaves)), dim3(64 * kSgdWaves), 0,
                       s, a);
  }
  VW_HIP_CHECK(hipGetLastError());
  VW_HIP_CHECK(hipMemcpyAsync(out, impl_->pred, n * sizeof(float), hipMemcpyDeviceToHost, s));
  VW_HIP_CHECK(hipStreamSynchronize(s));
}

// Average the table over ranks: only the 64 KB blocks some rank touched since the last sync (the union
// of the dirty maps, one small max-allreduce) are packed, reduced (fp64 sums of {wG or w, G}, max of N) and
// unpacked with VW's weighted averaging - no host staging, and a sparse pass moves a fraction of the table.
void GpuSgd::AllReduceAverage(void* comm, int world) {
  if (world < 1 || !comm) return;  // a world-1 communicator still runs the collectives (one-GPU tests)
  hipStream_t s = impl_->stream;
  ncclComm_t c = static_cast<ncclComm_t>(comm);
  auto nccl = [](ncclResult_t r) {
    if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL allreduce failed: ") + ncclGetErrorString(r));
  };
  const int64_t nblk = impl_->nblk;
  nccl(ncclAllReduce(impl_->dirty, impl_->dirty, nblk, ncclUint8, ncclMax, c, s));
  // deterministic compaction (every rank packs the same blocks in the same order): host prefix over the map
  std::vector<uint8_t> hd(nblk);
  VW_HIP_CHECK(hipMemcpyAsync(hd.data(), impl_->dirty, nblk, hipMemcpyDeviceToHost, s));
  VW_HIP_CHECK(hipStreamSynchronize(s));
  std::vector<int32_t> list;
  for (int64_t i = 0; i < nblk; ++i) if (hd[i]) list.push_back(static_cast<int32_t>(i));
  const int64_t m = static_cast<int64_t>(list.size());
  last_sync_bytes_ = 0;
  if (m > 0) {
    const size_t slots = static_cast<size_t>(m) << kDirtyShift;
    if (slots > impl_->cap_sync) {
      (void)hipFree(impl_->blocks); (void)hipFree(impl_->sums); (void)hipFree(impl_->nmax);
      VW_HIP_CHECK(hipMalloc(&impl_->blocks, nblk * sizeof(int32_t)));
      VW_HIP_CHECK(hipMalloc(&impl_->sums, slots * 2 * sizeof(double)));
      VW_HIP_CHECK(hipMalloc(&impl_->nmax, slots * sizeof(float)));
      impl_->cap_sync = slots;
    }
    VW_HIP_CHECK(hipMemcpyAsync(impl_->blocks, list.data(), m * sizeof(int32_t), hipMemcpyHostToDevice, s));
    const int grid = static_cast<int>(std::min<size_t>(65536, (slots + 255) / 256));
    const int adaptive = cfg_.adaptive ? 1 : 0;
    hipLaunchKernelGGL(pack_kernel, dim3(grid), dim3(256), 0, s, impl_->W, impl_->blocks, m, impl_->nw, adaptive,
                       impl_->sums, impl_->nmax);
    VW_HIP_CHECK(hipGetLastError());
    nccl(ncclAllReduce(impl_->sums, impl_->sums, slots * 2, ncclDouble, ncclSum, c, s));
    nccl(ncclAllReduce(impl_->nmax, impl_->nmax, slots, ncclFloat, ncclMax, c, s));
    hipLaunchKernelGGL(unpack_kernel, dim3(grid), dim3(256), 0, s, impl_->W, impl_->blocks, m, impl_->nw, adaptive,
                       1.0 / world, impl_->sums, impl_->nmax);
    VW_HIP_CHECK(hipGetLastError());
    last_sync_bytes_ = static_cast<int64_t>(slots) * (2 * sizeof(double) + sizeof(float)) + nblk;
  }
  VW_HIP_CHECK(hipMemsetAsync(impl_->dirty, 0, nblk, s));
  VW_HIP_CHECK(hipStreamSynchronize(s));
  last_sync_blocks_ = m;
}

uint64_t GpuSgd::NumWeights() const { return impl_->nw; }

// Nonzero table components as (stride-4 index, value), compacted on the device: the host only ever holds
// the nonzeros (a 2^30-slot table never crosses PCIe whole)
void GpuSgd::ExportNonzeros(std::vector<uint64_t>* idx, std::vector<float>* val) const {
  hipStream_t s = impl_->stream;
  const uint64_t per = 4096;
  const int64_t nb = static_cast<int64_t>((impl_->nw + per - 1) / per);
  int32_t* cnt = nullptr;
  int64_t* base = nullptr;
  VW_HIP_CHECK(hipMalloc(&cnt, nb * sizeof(int32_t)));
  VW_HIP_CHECK(hipMalloc(&base, nb * sizeof(int64_t)));
  hipLaunchKernelGGL(count_nz_kernel, dim3(static_cast<unsigned>(nb)), dim3(256), 0, s, impl_->W, impl_->nw, per, cnt);
  std::vector<int32_t> hc(nb);
  VW_HIP_CHECK(hipMemcpyAsync(hc.data(), cnt, nb * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  VW_HIP_CHECK(hipStreamSynchronize(s));
  std::vector<int64_t> hb(nb);
  int64_t tot = 0;
  for (int64_t i = 0; i < nb; ++i) { hb[i] = tot; tot += hc[i]; }
  idx->resize(tot);
  val->resize(tot);
  if (tot > 0) {
    uint64_t* di = nullptr;
    float* dv = nullptr;
    VW_HIP_CHECK(hipMalloc(&di, tot * sizeof(uint64_t)));
    VW_HIP_CHECK(hipMalloc(&dv, tot * sizeof(float)));
    VW_HIP_CHECK(hipMemcpyAsync(base, hb.data(), nb * sizeof(int64_t), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(write_nz_kernel, dim3(static_cast<unsigned>(nb)), dim3(64), 0, s, impl_->W, impl_->nw, per, base,
                       di, dv);
    VW_HIP_CHECK(hipMemcpyAsync(idx->data(), di, tot * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    VW_HIP_CHECK(hipMemcpyAsync(val->data(), dv, tot * sizeof(float), hipMemcpyDeviceToHost, s));
    VW_HIP_CHECK(hipStreamSynchronize(s));
    (void)hipFree(di);
    (void)hipFree(dv);
  }
  (void)hipFree(cnt);
  (void)hipFree(base);
}

void GpuSgd::ImportNonzeros(const std::vector<uint64_t>& idx, const std::vector<float>& val) {
  hipStream_t s = impl_->stream;
  VW_HIP_CHECK(hipMemsetAsync(impl_->W, 0, impl_->nw * sizeof(float4), s));
  const int64_t n = static_cast<int64_t>(idx.size());
  if (n > 0) {
    uint64_t* di = nullptr;
    float* dv = nullptr;
    VW_HIP_CHECK(hipMalloc(&di, n * sizeof(uint64_t)));
    VW_HIP_CHECK(hipMalloc(&dv, n * sizeof(float)));
    VW_HIP_CHECK(hipMemcpyAsync(di, idx.data(), n * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    VW_HIP_CHECK(hipMemcpyAsync(dv, val.data(), n * sizeof(float), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(scatter_kernel, dim3(static_cast<unsigned>(std::min<int64_t>(65536, (n + 255) / 256))), dim3(256),
                       0, s, impl_->W, impl_->nw, di, dv, n);
    VW_HIP_CHECK(hipStreamSynchronize(s));
    (void)hipFree(di);
    (void)hipFree(dv);
  }
  VW_HIP_CHECK(hipStreamSynchronize(s));
}

void GpuSgd::GlobalState(double* t, double* total_weight, double* sum_norm_x) const {
  double h[3] = {0, 0, 0};
  VW_HIP_CHECK(hipMemcpy(h, impl_->gs, sizeof(h), hipMemcpyDeviceToHost));
  *t = h[0]; *total_weight = h[1]; *sum_norm_x = h[2];
}

void GpuSgd::SetGlobalState(double t, double total_weight, double sum_norm_x) {
  const double h[3] = {t, total_weight, sum_norm_x};
  VW_HIP_CHECK(hipMemcpy(impl_->gs, h, sizeof(h), hipMemcpyHostToDevice));
}

void* GpuSgd::weights_device() { return impl_->W; }
void* GpuSgd::stream() { return impl_->stream; }

}  // namespace smlvw
