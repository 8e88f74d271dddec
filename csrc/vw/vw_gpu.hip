// K12: hogwild mini-batch hashed SGD on the MI355X. One wave64 per example:
// lanes stride over the example's features, gather w[h & mask], reduce the dot
// product with DPP shuffles, evaluate the loss derivative once per wave and
// scatter AdaGrad updates back with float atomics (conflicts are rare in a
// 2^b table, which is what makes hogwild converge like sequential SGD).
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <chrono>
#include <cstdio>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "vw_gpu.h"
#include "../gbdt/hip_common.h"  // sml::DevPoolAlloc / DevPoolFree: the process-wide caching device allocator

#define VW_HIP_CHECK(e)                                                                          \
  do {                                                                                           \
    hipError_t _e = (e);                                                                         \
    if (_e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e)); \
  } while (0)

namespace smlvw {
namespace {

// The learner's large buffers (the 2^bits weight table - 16 GiB at b=30 -, the staged example rows and the
// featurization's temporary blocks) come from the caching pool: a fit frees them at its end and the next fit
// of the same shape gets them back without a hipMalloc / hipFree of gigabytes; the per-learner small buffers
// (touched-block flags, global state, loss) too (a hipFree per buffer at every learner's end). A table a final
// export cleared skips even its memset (CleanTables).
std::mutex g_pool_mu;
std::unordered_map<void*, size_t> g_pool_granted;

template <class T>
void PoolMalloc(T** p, size_t bytes) {
  size_t granted = 0;
  void* q = sml::DevPoolAlloc(std::max<size_t>(bytes, 16), &granted);
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_pool_granted[q] = granted;
  }
  *p = static_cast<T*>(q);
}

void PoolFree(void* p) {
  if (!p) return;
  size_t granted = 0;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    auto it = g_pool_granted.find(p);
    if (it == g_pool_granted.end()) {
      (void)hipFree(p);
      return;
    }
    granted = it->second;
    g_pool_granted.erase(it);
  }
  sml::DevPoolFree(p, granted);
}


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
constexpr int kDirtyShift = 12;  // sync granularity: 4096 slots (64 KB) per block
// Touch map (one byte per 256 slots, 4 MB at 2^30): the sync epoch in which a 4 KB sub-block was last written
// (0 = never). The sync derives its 64 KB "touched since the last sync" blocks from it (coarsen_kernel) and the
// export scans only the sub-blocks ever written (a 2M-example pass writes ~16 % of them: the 16 GiB export scan
// was ~3 ms of every fit). One byte per feature update as before (the old map was 64 KB-granular and cleared at
// every sync, so it could not serve the export).
constexpr int kTouchShift = 8;
constexpr int kTouchPerBlock = 1 << (kDirtyShift - kTouchShift);

struct SgdArgs {
  const int64_t* indptr;
  const uint32_t* idx;
  const float* val;
  const float* lab;    // scalar label, or the 1-based class for oaa
  const float* wt;     // importance (null = 1)
  const float* lo;     // running label range (prediction clamp), per example
  const float* hi;
  int clamp_const;     // lo == null: clamp to [clo, chi] (logistic: the fixed label range, no per-example arrays)
  float clo, chi;
  int64_t n0, n1;
  float4* W;
  uint64_t mask;
  uint8_t* dirty;      // the touch map (kTouchShift granularity; epoch of the last write)
  double* gs;          // [t, total weight, sum of feature norms]
  float lr, power_t, initial_t, l2, l1, tau;
  int loss;            // 0 squared, 1 logistic, 2 hinge, 3 quantile (tau)
  int adaptive, normalized, invariant;
  int K;               // oaa classes (0: scalar learner)
  float* preds;
  float* loss_acc;
  int learn;
  int hot_agg;         // block-aggregate the constant feature's slot (sgd_kernel; SML_VW_HOT_AGG=0 disables)
  int epoch;           // the current sync epoch (1..255) written into the touch map
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
  float hot_x2, hot_x, hot_ax;  // the example's occurrences of the block-aggregated slot: sum x^2, sum x, max |x|
};

// slot index meaning "no aggregated slot"
constexpr uint64_t kNoHot = ~0ull;
constexpr uint32_t kVwConstantHash = 11650396u;  // VW's constant feature (the featurizer writes it as kConstantIdx)

__device__ UpdPrep UpdateFirstPass(const SgdArgs& a, int64_t b, int64_t en, uint64_t off, float raw, float y,
                                   float imp, int lane, uint64_t hot = kNoHot) {
  UpdPrep pr;
  float hx2 = 0.f, hx = 0.f, hax = 0.f;
  float g;
  if (a.loss == 1) g = -y / (1.f + expf(y * raw));
  else if (a.loss == 2) g = (y * raw < 1.f) ? -y : 0.f;
  else if (a.loss == 3) g = (y - raw) > 0.f ? -a.tau : (1.f - a.tau);
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
    if (h == hot) {  // the block-aggregated slot (sgd_kernel): its G / N / weight updates are done per block
      hx2 += x2;
      hx += x;
      hax = fmaxf(hax, fabsf(x));
      continue;
    }
    float G = 0.f, N = 1.f;
    // G and N come back from returning atomics: in a hogwild batch of examples sharing dense features, each
    // update must see the accumulators of the updates serialized before it (a plain load would hand every
    // concurrent example the same tiny G and a huge first-step rate - measured: AUC 0.65 instead of 0.998)
    if (a.adaptive) G = atomicAdd(&w->y, grad_sq * x2) + grad_sq * x2;
    if (a.normalized) {
      const float ax = fabsf(x);
      // N only grows: the float bits of non-negative values order like unsigned integers. A plain load first:
      // once a slot's N covers |x| (the steady state: every later example of the slot) the atomicMax would be a
      // no-op, so it is issued only when this update may raise N - one returning atomic fewer per feature on the
      // hot slots (identical at batch 1; under hogwild N is read as of the load instead of the atomic)
      float old = w->z;
      if (ax > old) old = __uint_as_float(atomicMax(reinterpret_cast<unsigned int*>(&w->z), __float_as_uint(ax)));
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
  pr.hot_x2 = hot == kNoHot ? 0.f : WaveSum(hx2);
  pr.hot_x = hot == kNoHot ? 0.f : WaveSum(hx);
  if (hot != kNoHot) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) hax = fmaxf(hax, __shfl_xor(hax, o, 64));
  }
  pr.hot_ax = hax;
  return pr;
}

// t, tw, snx: the global state including this update (what the sequential learner sees)
__device__ float UpdateSecondPass(const SgdArgs& a, int64_t b, int64_t en, uint64_t off, float raw, float y,
                                  float imp, int lane, const UpdPrep& pr, double t, double tw, double snx,
                                  uint64_t hot = kNoHot) {
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
    } else if (a.loss == 1) {
      const float step = y * us / (1.f + expf(y * raw));
      update = fabsf(step * pp) > 50.f ? copysignf(50.f / pp, step) : step;
    } else if (a.loss == 2) {
      // hinge: the step stops at the margin (VW's hingeloss::getUpdate)
      const float err = 1.f - y * raw;
      update = err <= 0.f ? 0.f : y * fminf(us, err / pp);
    } else {
      // quantile: the step stops at the label (VW's quantileloss::getUpdate)
      const float err = y - raw;
      update = err == 0.f ? 0.f : (err > 0.f ? fminf(a.tau * us, err / pp) : fmaxf(-(1.f - a.tau) * us, err / pp));
    }
  } else {
    update = -pr.g * us;  // the plain gradient step
  }
  const float decay = static_cast<float>(eta) * a.l2;
  const float shrink = static_cast<float>(eta) * a.l1;
  int k = 0;
  for (int64_t p = b + lane; p < en; p += 64, ++k) {
    const uint64_t h = (a.idx[p] + off) & a.mask;
    if (h == hot) continue;  // applied per block by the caller
    float4* w = &a.W[h];
    const float x = a.val[p];
    const float rate = k < kRateCache ? pr.rate[k] : Rate(a, a.adaptive ? w->y : 0.f, a.normalized ? w->z : 1.f);
    if (decay > 0.f || shrink > 0.f) {
      // the host learner's order: w += update; w -= eta l2 w; soft-threshold by eta l1 (as corrections to the
      // value this update produced: exact at batch 1, hogwild otherwise)
      float nw = atomicAdd(&w->x, update * x * rate) + update * x * rate;
      float t = nw - decay * nw;
      if (shrink > 0.f) t = t > shrink ? t - shrink : (t < -shrink ? t + shrink : 0.f);
      atomicAdd(&w->x, t - nw);
    } else {
      atomicAdd(&w->x, update * x * rate);  // result unused: a non-returning atomic
    }
    // the touched-block flag: written only when still clear (most updates hit blocks already marked; a plain
    // byte load instead of a store that takes the line from the other XCDs' caches)
    uint8_t* dflag = a.dirty + (h >> kTouchShift);
    if (*dflag != static_cast<uint8_t>(a.epoch)) *dflag = static_cast<uint8_t>(a.epoch);
  }
  return update;
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

__device__ __forceinline__ float LossOf(int loss, float p, float y, float tau = 0.5f) {
  if (loss == 1) return log1pf(expf(-y * p));
  if (loss == 2) return fmaxf(0.f, 1.f - y * p);
  if (loss == 3) { const float e = y - p; return e > 0.f ? tau * e : (tau - 1.f) * e; }
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
    else if (a.clamp_const) p = fminf(fmaxf(p, a.clo), a.chi);
    if (a.preds && lane == 0) a.preds[e] = p;
    if (a.learn) {
      y = a.lab[e];
      imp = a.wt ? a.wt[e] : 1.f;
      if (lane == 0) wloss[wid] = LossOf(a.loss, p, y, a.tau) * imp;
    }
  }
  if (!a.learn) return;  // uniform over the launch
  const bool upd = act && imp > 0.f;
  // VW's constant feature is in every example: per-example returning atomics on its slot serialize every
  // example of a hogwild batch on one address (769 vs 303 us per 16384-example batch at 2^30, r4 trace). Its
  // G / N / weight updates are aggregated per block instead: one returning atomic for the block's G, each
  // example taking G_base + the inclusive prefix of the block's contributions in wave order (the serialized
  // order the per-example atomics would have produced, up to the order among the block's examples), one
  // atomicMax for N, one atomicAdd for the summed weight deltas. Not with l1 / l2 (their per-update
  // corrections need the running value).
  const uint64_t hot = (!a.hot_agg || a.l1 > 0.f || a.l2 > 0.f) ? kNoHot
                                                                 : (static_cast<uint64_t>(kVwConstantHash) & a.mask);
  __shared__ float s_hg[kSgdWaves], s_hax[kSgdWaves], s_hd[kSgdWaves], s_hot[2];
  UpdPrep pr{0.f, 0.f, 0.f};
  if (upd) pr = UpdateFirstPass(a, b, en, 0, raw, y, imp, lane, hot);
  float hot_rate = 0.f;
  if (hot != kNoHot) {
    if (lane == 0) {
      s_hg[wid] = upd ? pr.g * pr.g * imp * pr.hot_x2 : 0.f;
      s_hax[wid] = upd ? pr.hot_ax : 0.f;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      float tot = 0.f, mx = 0.f;
      for (int w = 0; w < kSgdWaves; ++w) { tot += s_hg[w]; mx = fmaxf(mx, s_hax[w]); }
      float gb = 0.f, nn = 1.f;
      if (mx > 0.f) {
        float4* wh = &a.W[hot];
        if (a.adaptive) gb = atomicAdd(&wh->y, tot);
        if (a.normalized) {
          const float old = __uint_as_float(atomicMax(reinterpret_cast<unsigned int*>(&wh->z), __float_as_uint(mx)));
          if (mx > old && old > 0.f) {
            const float r = old / mx;
            wh->x *= a.adaptive ? r : r * r;
          }
          nn = fmaxf(old, mx);
        }
      }
      s_hot[0] = gb;
      s_hot[1] = nn;
    }
    __syncthreads();
    if (upd && pr.hot_x2 > 0.f) {
      float pre = 0.f;
      for (int w = 0; w <= wid; ++w) pre += s_hg[w];
      const float N = s_hot[1];
      hot_rate = Rate(a, s_hot[0] + pre, N);
      pr.ppu += pr.hot_x2 * hot_rate;
      if (a.normalized) pr.norm_x += pr.hot_x2 / (N * N);
    }
  }
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
  float upd_scalar = 0.f;
  if (upd) {
    double pi = 0.0, pn = 0.0;
    for (int w = 0; w <= wid; ++w) { pi += s_imp[w]; pn += s_nx[w]; }
    upd_scalar = UpdateSecondPass(a, b, en, 0, raw, y, imp, lane, pr, s_base[0] + pi, s_base[1] + pi, s_base[2] + pn,
                                  hot);
  }
  if (hot != kNoHot) {  // the aggregated slot's weight: one atomic for the block's summed deltas
    if (lane == 0) s_hd[wid] = (upd && pr.hot_x2 > 0.f) ? upd_scalar * pr.hot_x * hot_rate : 0.f;
    __syncthreads();
    if (threadIdx.x == 0) {
      float d = 0.f, mx = 0.f;
      for (int w = 0; w < kSgdWaves; ++w) { d += s_hd[w]; mx = fmaxf(mx, s_hax[w]); }
      if (mx > 0.f) {
        atomicAdd(&a.W[hot].x, d);
        a.dirty[hot >> kTouchShift] = static_cast<uint8_t>(a.epoch);
      }
    }
  }
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

// ---------------------------------------------------------------- CATS (--cats_pdf / --cats)
// Continuous actions over [min, max] discretized into K centroids, a filter tree of 2^depth leaves whose
// internal nodes are binary learners at their own table offsets (vw_core.cpp CatsPredictLeaf / CatsLearn).
// One wave per example: the leaf its current routing reaches (the progressive prediction), then - labelled
// examples - the IPS estimate of every leaf's smoothed cost with the control-variate baseline (the running
// mean cost, from the host: `base`) and the bottom-up tournament, each node with both children real learning
// which child's winner is cheaper, weighted by the difference, in the host learner's node order.
struct CatsArgs {
  const float* act;
  const float* cost;
  const float* pdf;
  const float* base;
  const uint8_t* has;
  int k, depth;
  float vmin, vmax, bw;
};

__device__ __forceinline__ uint64_t CatsOff(int node) { return static_cast<uint64_t>(node + 1) * 2654435761ull; }

__global__ __launch_bounds__(64) void cats_kernel(SgdArgs a, CatsArgs c) {
  const int lane = threadIdx.x;
  const int64_t e = a.n0 + blockIdx.x;
  if (e >= a.n1) return;
  extern __shared__ float cats_lds[];  // win[2L - 1], then valid[2L - 1] (0 / 1)
  const int L = 1 << c.depth;
  float* win = cats_lds;
  float* valid = cats_lds + (2 * L - 1);
  const int64_t b = a.indptr[e], en = a.indptr[e + 1];
  if (a.preds) {
    int node = 0;
    for (int d = 0; d < c.depth; ++d) {
      // right only when its subtree holds a real action (K need not be a power of two)
      const int right = 2 * node + 2;
      int fl = right;
      while (fl < L - 1) fl = 2 * fl + 1;
      const bool right_ok = fl - (L - 1) < c.k;
      const float sc = Dot(a, b, en, CatsOff(node), lane);
      node = (sc > 0.f && right_ok) ? right : 2 * node + 1;
    }
    if (lane == 0) a.preds[e] = static_cast<float>(node - (L - 1));  // leaf: the host maps it to the pdf / action
  }
  if (!a.learn || !c.has[e]) return;
  const float bb = c.base[e];
  const float unit = (c.vmax - c.vmin) / c.k;
  const float p = fmaxf(c.pdf[e], 1e-12f);
  const float act = c.act[e], cost = c.cost[e];
  for (int i = lane; i < 2 * L - 1; i += 64) {
    win[i] = bb;
    valid[i] = 0.f;
  }
  __syncthreads();
  for (int k = lane; k < c.k; k += 64) {
    const float ctr = c.vmin + (k + 0.5f) * unit;
    const float lo = fmaxf(c.vmin, ctr - c.bw), hi = fminf(c.vmax, ctr + c.bw);
    valid[L - 1 + k] = 1.f;
    if (act >= lo && act <= hi) win[L - 1 + k] = bb + (cost - bb) / ((hi - lo) * p);
  }
  __syncthreads();
  if (lane == 0) atomicAdd(a.loss_acc, cost);
  for (int node = L - 2; node >= 0; --node) {
    const int l = 2 * node + 1, r = 2 * node + 2;
    const bool vl = valid[l] != 0.f, vr = valid[r] != 0.f;
    const float wl = win[l], wr = win[r];
    float wn;
    if (!vl || !vr) {
      wn = vl ? wl : wr;
    } else {
      const float sc = Dot(a, b, en, CatsOff(node), lane);
      const float imp = fabsf(wl - wr);
      if (imp > 0.f) UpdateWave(a, b, en, CatsOff(node), sc, wr < wl ? 1.f : -1.f, imp, lane);
      wn = sc > 0.f ? wr : wl;
    }
    __syncthreads();  // every lane has read the children before lane 0 writes the node
    if (lane == 0) {
      valid[node] = (vl || vr) ? 1.f : 0.f;
      win[node] = wn;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- device featurization
// The learner's example CSR is built on the device from the namespace blocks (one CSR per feature column,
// already hashed): base features of every namespace, then each interaction's crosses, then VW's constant.
// Namespaces are groups of up to kMaxGroupBlocks blocks (columns sharing a first letter, or a CB action's
// namespace plus the shared example's); a block is indexed by the row itself (level 0) or by row_map[row]
// (level 1: contextual-bandit action rows read their example's shared features). Interactions follow the
// host learner (vw_core.cpp ForEachFeature): (a * FNV) ^ b [* FNV ^ c] in 32 bits (the table mask keeps
// <= 32 bits, so the low words of the host's 64-bit products), a namespace crossed with itself keeps only
// non-decreasing feature positions. Pass 1 counts every row's features (closed forms), a device scan gives
// the row offsets, pass 2 writes them with one wave per row.
constexpr int kMaxGroups = 32;
constexpr int kMaxGroupBlocks = 4;
constexpr int kMaxInter = 64;
constexpr uint32_t kFnv = 16777619u;
constexpr uint32_t kConstantIdx = kVwConstantHash;

struct DevBlock {
  const int64_t* ip;
  const uint32_t* idx;
  const float* val;
  int level;
};

struct ExpandSpec {
  int ngroups, ninter, constant, pad;
  int gblocks[kMaxGroups];
  DevBlock blk[kMaxGroups][kMaxGroupBlocks];
  int inter[kMaxInter][3];
  const int64_t* row_map;
};

__device__ __forceinline__ int64_t GroupLen(const ExpandSpec& s, int g, int64_t r, int64_t rm) {
  int64_t l = 0;
  for (int k = 0; k < s.gblocks[g]; ++k) {
    const DevBlock& b = s.blk[g][k];
    const int64_t row = b.level ? rm : r;
    l += b.ip[row + 1] - b.ip[row];
  }
  return l;
}

__device__ __forceinline__ int64_t InterCount(const ExpandSpec& s, int q, const int64_t* len) {
  const int a = s.inter[q][0], b = s.inter[q][1], c = s.inter[q][2];
  const int64_t la = len[a], lb = len[b];
  if (c < 0) return a == b ? la * (la + 1) / 2 : la * lb;
  const int64_t lc = len[c];
  const bool s12 = a == b, s23 = b == c;
  if (s12 && s23) return la * (la + 1) * (la + 2) / 6;
  if (s12) return la * (la + 1) / 2 * lc;
  if (s23) return la * (lb * (lb + 1) / 2);
  return la * lb * lc;
}

__global__ __launch_bounds__(256) void expand_count_kernel(const ExpandSpec* __restrict__ sp, int64_t n,
                                                           int64_t* __restrict__ counts) {
  const ExpandSpec& s = *sp;
  for (int64_t r = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; r < n;
       r += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t rm = s.row_map ? s.row_map[r] : r;
    int64_t len[kMaxGroups];
    int64_t c = s.constant ? 1 : 0;
    for (int g = 0; g < s.ngroups; ++g) { len[g] = GroupLen(s, g, r, rm); c += len[g]; }
    for (int q = 0; q < s.ninter; ++q) c += InterCount(s, q, len);
    counts[r] = c;
  }
}

// one wave per row; the group's block extents of the row are staged per wave in LDS
constexpr int kExpandWaves = 4;

struct RowExt {
  int64_t st[kMaxGroupBlocks];
  int32_t len[kMaxGroupBlocks];
  int32_t tot;
};

__device__ __forceinline__ void GroupFeat(const ExpandSpec& s, const RowExt& e, int g, int i, uint32_t* h, float* x) {
  for (int k = 0; k < s.gblocks[g]; ++k) {
    if (i < e.len[k]) {
      const DevBlock& b = s.blk[g][k];
      *h = b.idx[e.st[k] + i];
      *x = b.val[e.st[k] + i];
      return;
    }
    i -= e.len[k];
  }
  *h = 0;
  *x = 0.f;
}

// rows [r0, r1) (the staging pipeline fills the pass chunk by chunk as its blocks arrive)
__global__ __launch_bounds__(64 * kExpandWaves) void expand_fill_kernel(const ExpandSpec* __restrict__ sp, int64_t r0,
                                                                         int64_t r1, const int64_t* __restrict__ indptr,
                                                                         uint32_t* __restrict__ oidx,
                                                                         float* __restrict__ oval) {
  const ExpandSpec& s = *sp;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __shared__ RowExt ext[kExpandWaves][kMaxGroups];
  for (int64_t r = r0 + blockIdx.x * static_cast<int64_t>(kExpandWaves) + wid; r < r1;
       r += static_cast<int64_t>(gridDim.x) * kExpandWaves) {
    const int64_t rm = s.row_map ? s.row_map[r] : r;
    RowExt* E = ext[wid];
    for (int g = lane; g < s.ngroups; g += 64) {
      int tot = 0;
      for (int k = 0; k < s.gblocks[g]; ++k) {
        const DevBlock& b = s.blk[g][k];
        const int64_t row = b.level ? rm : r;
        E[g].st[k] = b.ip[row];
        E[g].len[k] = static_cast<int32_t>(b.ip[row + 1] - b.ip[row]);
        tot += E[g].len[k];
      }
      E[g].tot = tot;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    int64_t pos = indptr[r];
    for (int g = 0; g < s.ngroups; ++g) {
      const int la = E[g].tot;
      for (int i = lane; i < la; i += 64) {
        uint32_t h;
        float x;
        GroupFeat(s, E[g], g, i, &h, &x);
        oidx[pos + i] = h;
        oval[pos + i] = x;
      }
      pos += la;
    }
    for (int q = 0; q < s.ninter; ++q) {
      const int a = s.inter[q][0], b = s.inter[q][1], c = s.inter[q][2];
      const int la = E[a].tot, lb = E[b].tot;
      if (c < 0) {
        const bool same = a == b;
        for (int i = 0; i < la; ++i) {
          uint32_t ha;
          float xa;
          GroupFeat(s, E[a], a, i, &ha, &xa);
          const uint32_t h1 = ha * kFnv;
          const int j0 = same ? i : 0;
          for (int j = j0 + lane; j < lb; j += 64) {
            uint32_t hb;
            float xb;
            GroupFeat(s, E[b], b, j, &hb, &xb);
            oidx[pos + (j - j0)] = h1 ^ hb;
            oval[pos + (j - j0)] = xa * xb;
          }
          pos += lb - j0;
        }
      } else {
        const int lc = E[c].tot;
        const bool s12 = a == b, s23 = b == c;
        for (int i = 0; i < la; ++i) {
          uint32_t ha;
          float xa;
          GroupFeat(s, E[a], a, i, &ha, &xa);
          for (int j = s12 ? i : 0; j < lb; ++j) {
            uint32_t hb;
            float xb;
            GroupFeat(s, E[b], b, j, &hb, &xb);
            const uint32_t h12 = ((ha * kFnv) ^ hb) * kFnv;
            const float x12 = xa * xb;
            const int k0 = s23 ? j : 0;
            for (int k = k0 + lane; k < lc; k += 64) {
              uint32_t hc;
              float xc;
              GroupFeat(s, E[c], c, k, &hc, &xc);
              oidx[pos + (k - k0)] = h12 ^ hc;
              oval[pos + (k - k0)] = x12 * xc;
            }
            pos += lc - k0;
          }
        }
      }
    }
    if (s.constant && lane == 0) {
      oidx[pos] = kConstantIdx;
      oval[pos] = 1.f;
    }
  }
}

// ---------------------------------------------------------------- --csoaa K
// One block per example: wave c scores classes c, c + waves, ... (class offsets as --oaa), the prediction is
// the class of smallest score (first on ties, std::min_element); wave 0 then applies the example's (class,
// cost) regressions one after another, as the host learner does (batch 1 = the sequential learner).
__global__ __launch_bounds__(64 * kOaaMaxWaves) void csoaa_kernel(SgdArgs a, const int64_t* __restrict__ cptr,
                                                                  const int32_t* __restrict__ ccls,
                                                                  const float* __restrict__ ccost) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int64_t e = a.n0 + blockIdx.x;
  if (e >= a.n1) return;
  extern __shared__ float scores[];
  __shared__ int s_best;
  const int64_t b = a.indptr[e], en = a.indptr[e + 1];
  for (int k = wid; k < a.K; k += nw) {
    const float sc = Dot(a, b, en, static_cast<uint64_t>(k) * kOaaOffset, lane);
    if (lane == 0) scores[k] = sc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int best = 0;
    for (int k = 1; k < a.K; ++k) if (scores[k] < scores[best]) best = k;
    s_best = best;
    if (a.preds) a.preds[e] = static_cast<float>(best + 1);
    if (a.learn && cptr) {
      float chosen = 0.f;
      for (int64_t p = cptr[e]; p < cptr[e + 1]; ++p) if (ccls[p] == best + 1) chosen = ccost[p];
      atomicAdd(a.loss_acc, chosen * (a.wt ? a.wt[e] : 1.f));
    }
  }
  if (!a.learn || !cptr || wid != 0) return;
  const float imp = a.wt ? a.wt[e] : 1.f;
  if (imp <= 0.f) return;
  for (int64_t p = cptr[e]; p < cptr[e + 1]; ++p) {
    const int k = ccls[p] - 1;
    if (k < 0 || k >= a.K) continue;
    UpdateWave(a, b, en, static_cast<uint64_t>(k) * kOaaOffset, scores[k], ccost[p], imp, lane);
  }
}

// ---------------------------------------------------------------- --cb_adf / --cb_explore_adf
// One block per multi-line example: its action rows [aip[e], aip[e+1]) (shared features merged in by the
// device featurization) are scored by the waves, the greedy action is the smallest score, the exploration
// distribution is epsilon-greedy; with a logged (action, cost, probability) the IPS / SNIPS sums advance and
// the update follows --cb_type: mtr (the logged action regressed on its cost with importance 1/p), dr (every
// action towards its doubly-robust target) or ips (every action towards cost/p on the logged one, 0 else),
// applied action after action by wave 0 as the host learner does.
struct CbArgs {
  const int64_t* aip;
  const int32_t* chosen;  // 0-based logged action or -1
  const float* cost;
  const float* prob;
  int cb_type;            // 0 mtr, 1 dr, 2 ips
  int explore;
  float epsilon;
  double* stats;          // [ips numerator, snips denominator, examples]
  float* best_out;        // per example: greedy action (0-based)
};

constexpr int kCbWaves = 8;

__global__ __launch_bounds__(64 * kCbWaves) void cb_kernel(SgdArgs a, CbArgs cb) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t e = a.n0 + blockIdx.x;
  if (e >= a.n1) return;
  extern __shared__ float scores[];
  __shared__ int s_best;
  const int64_t r0 = cb.aip[e], r1 = cb.aip[e + 1];
  const int A = static_cast<int>(r1 - r0);
  if (A <= 0) return;
  for (int k = wid; k < A; k += kCbWaves) {
    const float sc = Dot(a, a.indptr[r0 + k], a.indptr[r0 + k + 1], 0, lane);
    if (lane == 0) {
      scores[k] = sc;
      if (a.preds) a.preds[r0 + k] = sc;
    }
  }
  __syncthreads();
  const int logged = cb.chosen ? cb.chosen[e] : -1;
  if (threadIdx.x == 0) {
    int best = 0;
    for (int k = 1; k < A; ++k) if (scores[k] < scores[best]) best = k;
    s_best = best;
    if (cb.best_out) cb.best_out[e] = static_cast<float>(best);
    if (cb.stats && logged >= 0 && logged < A) {
      const float p = fmaxf(cb.prob[e], 1e-6f);
      const float ppred = cb.explore ? (logged == best ? 1.f - cb.epsilon + cb.epsilon / A : cb.epsilon / A)
                                     : (logged == best ? 1.f : 0.f);
      atomicAdd(&cb.stats[0], static_cast<double>(cb.cost[e] * ppred / p));
      atomicAdd(&cb.stats[1], static_cast<double>(ppred / p));
    }
    if (cb.stats) atomicAdd(&cb.stats[2], 1.0);
  }
  if (!a.learn || logged < 0 || logged >= A || wid != 0) return;
  const float p = fmaxf(cb.prob[e], 1e-6f), c = cb.cost[e];
  if (cb.cb_type == 0) {
    UpdateWave(a, a.indptr[r0 + logged], a.indptr[r0 + logged + 1], 0, scores[logged], c, 1.f / p, lane);
  } else {
    for (int k = 0; k < A; ++k) {
      const float lab = cb.cb_type == 1 ? scores[k] + (k == logged ? (c - scores[k]) / p : 0.f)
                                        : (k == logged ? c / p : 0.f);
      UpdateWave(a, a.indptr[r0 + k], a.indptr[r0 + k + 1], 0, scores[k], lab, 1.f, lane);
    }
  }
}

// Sync payload per slot: float {w G (adaptive) or w, G} + float N. A plain float w * G underflows for slots
// with a tiny gradient mass (G ~ 1e-44 after a few updates on a well-classified logistic example), which
// would zero their weight on the average even at world 1; both adaptive sums therefore carry G scaled by
// 2^32 (exact: a power of two), which keeps w G representable for any w above ~1e-10 (G down to the
// smallest denormal) and G up to ~8e28 finite, and leaves the ratio sum(w G) / sum(G) unchanged.
constexpr float kSyncScale = 4294967296.0f;              // 2^32
constexpr float kSyncUnscale = 2.3283064365386963e-10f;  // 2^-32
__global__ void pack_kernel(const float4* __restrict__ W, const int32_t* __restrict__ blocks, int64_t nblk,
                            uint64_t nw, int adaptive, float* __restrict__ sums, float* __restrict__ nmax) {
  constexpr int64_t B = int64_t(1) << kDirtyShift;
  const int64_t m = nblk * B;
  for (int64_t j = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; j < m;
       j += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const uint64_t slot = static_cast<uint64_t>(blocks[j >> kDirtyShift]) * B + (j & (B - 1));
    const float4 v = slot < nw ? W[slot] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float g = v.y * kSyncScale;
    sums[2 * j] = adaptive ? v.x * g : v.x;
    sums[2 * j + 1] = g;
    nmax[j] = v.z;
  }
}

// VW's weighted averaging: with adaptive state w = sum(w G) / sum(G) (a slot no rank has gradient mass
// on was never updated and keeps its value), G = sum(G) / world; N = max(N); without adaptive
// w = sum(w) / world. The sums are fp32, as VW's own allreduce of its float weight buffers (half the bytes
// of the fp64 sums earlier builds sent).
__global__ void unpack_kernel(float4* __restrict__ W, const int32_t* __restrict__ blocks, int64_t nblk, uint64_t nw,
                              int adaptive, float inv_world, const float* __restrict__ sums,
                              const float* __restrict__ nmax) {
  constexpr int64_t B = int64_t(1) << kDirtyShift;
  const int64_t m = nblk * B;
  for (int64_t j = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; j < m;
       j += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const uint64_t slot = static_cast<uint64_t>(blocks[j >> kDirtyShift]) * B + (j & (B - 1));
    if (slot >= nw) continue;
    float4 v = W[slot];
    const float s0 = sums[2 * j], sg = sums[2 * j + 1];
    if (!adaptive) v.x = s0 * inv_world;
    else if (sg > 0.f) v.x = s0 / sg;
    v.y = sg * kSyncUnscale * inv_world;
    v.z = nmax[j];
    W[slot] = v;
  }
}

// The same walk writing the host model's 12-byte records (u64 stride-4 index, f32 value; little-endian, so
// three dword stores) straight into one device buffer: the export then moves each byte across PCIe once,
// into the Python bytes object, with no per-field host vectors to interleave.
__global__ __launch_bounds__(64) void write_rec_kernel(const float4* __restrict__ W, uint64_t nw, uint64_t per,
                                                       const int64_t* __restrict__ base, uint32_t* __restrict__ rec) {
  const int lane = threadIdx.x & 63;
  const uint64_t s0 = static_cast<uint64_t>(blockIdx.x) * per, s1 = min(nw, s0 + per);
  int64_t o = base[blockIdx.x];
  for (uint64_t s = s0; s < s1; s += 64) {
    const uint64_t my = s + lane;
    const float4 v = my < s1 ? W[my] : make_float4(0.f, 0.f, 0.f, 0.f);
    const int c = (v.x != 0.f) + (v.y != 0.f) + (v.z != 0.f);
    int inc = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int t = __shfl_up(inc, off, 64);
      if (lane >= off) inc += t;
    }
    int64_t p = o + (inc - c);
    const float vals[3] = {v.x, v.y, v.z};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (vals[k] != 0.f) {
        const uint64_t ix = 4 * my + k;
        uint32_t* r = rec + 3 * p++;
        r[0] = static_cast<uint32_t>(ix);
        r[1] = static_cast<uint32_t>(ix >> 32);
        r[2] = __float_as_uint(vals[k]);
      }
    }
    o += __shfl(inc, 63, 64);
  }
}

// One-scan export: block b (one per `per` slots) writes its records into its own region of `cap` records
// (any order of blocks, slot order within one) and its count; a block past `cap` records stops writing and
// reports the count, and the host then takes the two-scan path. rec_compact_kernel packs the regions.
__global__ __launch_bounds__(64) void write_rec_region_kernel(const float4* __restrict__ W, uint64_t nw, uint64_t per,
                                                              int cap, uint32_t* __restrict__ reg,
                                                              int32_t* __restrict__ cnt,
                                                              const uint8_t* __restrict__ touch) {
  const int lane = threadIdx.x & 63;
  const uint64_t s0 = static_cast<uint64_t>(blockIdx.x) * per, s1 = min(nw, s0 + per);
  uint32_t* rec = reg + static_cast<uint64_t>(blockIdx.x) * cap * 3;
  int64_t o = 0;
  for (uint64_t s = s0; s < s1; s += 64) {
    // (touch map: a never-written 256-slot sub-block is all zeros - the 64 slots of this step lie in one)
    if (touch && touch[s >> kTouchShift] == 0) continue;
    const uint64_t my = s + lane;
    const float4 v = my < s1 ? W[my] : make_float4(0.f, 0.f, 0.f, 0.f);
    const int c = (v.x != 0.f) + (v.y != 0.f) + (v.z != 0.f);
    int inc = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int t = __shfl_up(inc, off, 64);
      if (lane >= off) inc += t;
    }
    int64_t p = o + (inc - c);
    const float vals[3] = {v.x, v.y, v.z};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (vals[k] != 0.f) {
        if (p < cap) {
          const uint64_t ix = 4 * my + k;
          uint32_t* r = rec + 3 * p;
          r[0] = static_cast<uint32_t>(ix);
          r[1] = static_cast<uint32_t>(ix >> 32);
          r[2] = __float_as_uint(vals[k]);
        }
        ++p;
      }
    }
    o += __shfl(inc, 63, 64);
  }
  if (lane == 0) cnt[blockIdx.x] = static_cast<int32_t>(o);
}

// final export: every exported component (record index = the component's float index in the table) back to 0
__global__ void clear_records_kernel(const uint32_t* __restrict__ rec, int64_t n, float* __restrict__ W) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const uint64_t ix = static_cast<uint64_t>(rec[3 * i]) | (static_cast<uint64_t>(rec[3 * i + 1]) << 32);
    W[ix] = 0.f;
  }
}

// region b's records -> out at base[b] (12-byte records as dwords)
__global__ __launch_bounds__(256) void rec_compact_kernel(const uint32_t* __restrict__ reg, int cap,
                                                          const int32_t* __restrict__ cnt,
                                                          const int64_t* __restrict__ base, int64_t nb,
                                                          uint32_t* __restrict__ out) {
  for (int64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const int n3 = cnt[b] * 3;
    const uint32_t* src = reg + static_cast<uint64_t>(b) * cap * 3;
    uint32_t* dst = out + base[b] * 3;
    for (int i = threadIdx.x; i < n3; i += blockDim.x) dst[i] = src[i];
  }
}

// sync: 64 KB block b was written this epoch if any of its 16 touch bytes holds the epoch
__global__ void coarsen_kernel(const uint8_t* __restrict__ touch, int64_t nblk, int epoch, uint8_t* __restrict__ coarse) {
  for (int64_t b = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; b < nblk;
       b += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const uint8_t* t = touch + b * kTouchPerBlock;
    uint8_t any = 0;
#pragma unroll
    for (int j = 0; j < kTouchPerBlock; ++j) any |= t[j] == static_cast<uint8_t>(epoch) ? 1 : 0;
    coarse[b] = any;
  }
}

// sync: the averaged blocks were written on every rank (a block another rank touched gets values here too)
__global__ void mark_blocks_kernel(const int32_t* __restrict__ blocks, int64_t m, int epoch, uint8_t* __restrict__ touch) {
  const int64_t n = m * kTouchPerBlock;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    touch[static_cast<int64_t>(blocks[i / kTouchPerBlock]) * kTouchPerBlock + i % kTouchPerBlock] =
        static_cast<uint8_t>(epoch);
}

// epoch wrap (255 syncs): every written sub-block back to epoch 1
__global__ void touch_renorm_kernel(uint8_t* __restrict__ touch, int64_t n) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    if (touch[i]) touch[i] = 1;
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

// one wave per block of `per` slots, 64 slots per step: a wave prefix sum of the step's nonzero counts gives
// every lane its output offset, so the records stay in slot order (the host model's order) while all lanes
// work (the one-thread-per-block form took 36 ms over a 2^30-slot table)
__global__ __launch_bounds__(64) void write_nz_kernel(const float4* __restrict__ W, uint64_t nw, uint64_t per,
                                                      const int64_t* __restrict__ base, uint64_t* __restrict__ oidx,
                                                      float* __restrict__ oval) {
  const int lane = threadIdx.x & 63;
  const uint64_t s0 = static_cast<uint64_t>(blockIdx.x) * per, s1 = min(nw, s0 + per);
  int64_t o = base[blockIdx.x];
  for (uint64_t s = s0; s < s1; s += 64) {
    const uint64_t my = s + lane;
    const float4 v = my < s1 ? W[my] : make_float4(0.f, 0.f, 0.f, 0.f);
    const int c = (v.x != 0.f) + (v.y != 0.f) + (v.z != 0.f);
    int inc = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int t = __shfl_up(inc, off, 64);
      if (lane >= off) inc += t;
    }
    int64_t p = o + (inc - c);
    if (v.x != 0.f) { oidx[p] = 4 * my; oval[p++] = v.x; }
    if (v.y != 0.f) { oidx[p] = 4 * my + 1; oval[p++] = v.y; }
    if (v.z != 0.f) { oidx[p] = 4 * my + 2; oval[p] = v.z; }
    o += __shfl(inc, 63, 64);
  }
}

__global__ void scatter_kernel(float4* __restrict__ W, uint64_t nw, uint8_t* __restrict__ touch, int epoch,
                               const uint64_t* __restrict__ idx,
                               const float* __restrict__ val, int64_t n) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const uint64_t s = idx[i] >> 2;
    const int c = static_cast<int>(idx[i] & 3);
    if (s < nw && c < 3) {
      reinterpret_cast<float*>(&W[s])[c] = val[i];
      touch[s >> kTouchShift] = static_cast<uint8_t>(epoch);
    }
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

// One per process (SharedStager), buffers allocated on first use: 4 x 32 MiB of pinned memory cost ~4 ms per
// hipHostMalloc, which a per-learner stager paid again on every fit (the first chunk of a pass waited
// ~17 ms for them, r5 pass 11 trace). Callers hold `mu` for a whole copy sequence; a buffer's event may
// have been recorded on another learner's copy stream, and waiting on it is still correct.
// A fixed team of kStageThreads - 1 helper threads (the caller is member 0) for the staging copies: a 32 MiB
// piece used to start and join 8 std::threads, ~32 pieces per 1 GiB pass.
class CopyTeam {
 public:
  CopyTeam() {
    for (int t = 1; t < kStageThreads; ++t) th_.emplace_back([this, t] { Loop(t); });
  }
  ~CopyTeam() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& x : th_) x.join();
  }
  // fn(t) for t in [0, kStageThreads), t = 0 on the calling thread; returns when all have run
  template <class F>
  void Run(F&& fn) {
    std::function<void(int)> job(std::forward<F>(fn));
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &job;
      pending_ = kStageThreads - 1;
      ++gen_;
    }
    cv_.notify_all();
    job(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  void Loop(int t) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        job = job_;
      }
      (*job)(t);
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, done_;
  std::vector<std::thread> th_;
  const std::function<void(int)>* job_ = nullptr;
  int pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

struct Stager {
  std::mutex mu;
  char* buf[kStage] = {};
  hipEvent_t ev[kStage] = {};
  bool used[kStage] = {};
  int next = 0;
  CopyTeam* team = nullptr;  // made on the first large copy
  int64_t unit_pieces = 0;   // value pieces sent as a device fill (all 1.0f), for the tests
  ~Stager() {
    for (int k = 0; k < kStage; ++k) {
      if (ev[k]) { (void)hipEventSynchronize(ev[k]); (void)hipEventDestroy(ev[k]); }
      if (buf[k]) (void)hipHostFree(buf[k]);
    }
    delete team;
  }
  CopyTeam& Team() {
    if (!team) team = new CopyTeam();
    return *team;
  }
  // true when every float of src[0, n) is 1.0f (bit pattern 0x3F800000); the team scans slices and stops at
  // the first other value (non-unit data: after a few cache lines)
  bool AllOnes(const float* src, size_t n) {
    auto scan = [](const float* p, size_t m) {
      const uint32_t* u = reinterpret_cast<const uint32_t*>(p);
      size_t i = 0;
      for (; i + 16 <= m; i += 16) {
        uint32_t x = 0;
        for (int j = 0; j < 16; ++j) x |= u[i + j] ^ 0x3F800000u;
        if (x) return false;
      }
      for (; i < m; ++i)
        if (u[i] != 0x3F800000u) return false;
      return true;
    };
    if (n == 0) return true;
    if (!scan(src, std::min<size_t>(n, 4096))) return false;  // the common non-unit case, on this thread
    if (n < (size_t(1) << 18)) return scan(src, n);
    std::atomic<bool> ok{true};
    const size_t per = (n + kStageThreads - 1) / kStageThreads;
    Team().Run([&](int t) {
      const size_t a0 = t * per, a1 = std::min(n, a0 + per);
      if (a0 < a1 && ok.load(std::memory_order_relaxed) && !scan(src + a0, a1 - a0)) ok = false;
    });
    return ok.load();
  }
  // queue `bytes` from pageable `src` to device `dst` on stream s (caller holds mu). unit_floats: the bytes are
  // float values that are very often all 1.0f (binary hashed features): such a piece crosses PCIe as a device
  // fill instead of its bytes.
  void Copy(char* dst, const char* src, size_t bytes, hipStream_t s, bool unit_floats = false) {
    if (bytes == 0) return;
    // a null source or destination is a caller bug (round 4: a device scratch buffer "copied" from a null host
    // pointer segfaulted the staging threads) - refuse it here instead of faulting in a memcpy thread
    if (!src || !dst) throw std::invalid_argument("Stager::Copy: null source or destination for a non-empty copy");
    if (unit_floats) {  // SML_VW_UNIT_FILL=0: always send the bytes (read per call: the tests A/B it)
      const char* e = std::getenv("SML_VW_UNIT_FILL");
      unit_floats = !(e && e[0] == '0');
    }
    if (unit_floats && bytes % sizeof(float) == 0 &&
        AllOnes(reinterpret_cast<const float*>(src), bytes / sizeof(float))) {
      VW_HIP_CHECK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(dst), 0x3F800000, bytes / sizeof(float), s));
      ++unit_pieces;
      return;
    }
    for (size_t off = 0; off < bytes; off += kStageBytes) {
      const int k = next;
      next = (next + 1) % kStage;
      if (!buf[k]) {
        VW_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&buf[k]), kStageBytes, hipHostMallocPortable));
        VW_HIP_CHECK(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
      }
      if (used[k]) VW_HIP_CHECK(hipEventSynchronize(ev[k]));
      const size_t n = std::min(kStageBytes, bytes - off);
      if (n < (1u << 20)) {
        std::memcpy(buf[k], src + off, n);  // small pieces: a thread team costs more than the copy
      } else {
        const size_t per = (n + kStageThreads - 1) / kStageThreads;
        char* b = buf[k];
        const char* from = src + off;
        Team().Run([=](int t) {
          const size_t a0 = t * per, a1 = std::min(n, a0 + per);
          if (a0 < a1) std::memcpy(b + a0, from + a0, a1 - a0);
        });
      }
      VW_HIP_CHECK(hipMemcpyAsync(dst + off, buf[k], n, hipMemcpyHostToDevice, s));
      VW_HIP_CHECK(hipEventRecord(ev[k], s));
      used[k] = true;
    }
  }
};
}  // namespace

static Stager& SharedStager() {
  static Stager* st = new Stager();  // never destroyed: pinned buffers live for the process
  return *st;
}

int64_t StagerUnitPieces() {
  Stager& st = SharedStager();
  std::lock_guard<std::mutex> lk(st.mu);
  return st.unit_pieces;
}

// Host-only check of the staging guard (it throws before any HIP call, so it runs without a GPU).
bool StagerRejectsNull() {
  Stager st;
  char d[16];
  try {
    st.Copy(d, nullptr, sizeof(d), nullptr);
  } catch (const std::invalid_argument&) {
    return true;
  }
  return false;
}

// Tables a final export left all-zero (clear_records_kernel), per device: the next learner of the same size
// takes one instead of allocating and zeroing 16 GiB (a 2^30 table's memset was ~3 ms of every fit, and the
// staging's layout count waited behind it). One kept per device; never destroyed (teardown order).
struct CleanTables {
  std::mutex mu;
  std::unordered_map<int, std::pair<void*, size_t>> t;
  static CleanTables& Get() {
    static CleanTables* c = new CleanTables();
    return *c;
  }
  bool Take(int dev, size_t bytes, void** out) {
    std::lock_guard<std::mutex> lk(mu);
    auto it = t.find(dev);
    if (it == t.end() || it->second.second != bytes) return false;
    *out = it->second.first;
    t.erase(it);
    return true;
  }
  bool Give(int dev, void* p, size_t bytes) {
    std::lock_guard<std::mutex> lk(mu);
    if (t.count(dev)) return false;
    t[dev] = {p, bytes};
    return true;
  }
  // the learners' two streams, kept per device (create + destroy cost ~0.8 ms per learner)
  std::unordered_map<int, std::vector<hipStream_t>> streams;
  hipStream_t TakeStream(int dev) {
    {
      std::lock_guard<std::mutex> lk(mu);
      auto& v = streams[dev];
      if (!v.empty()) {
        hipStream_t s = v.back();
        v.pop_back();
        return s;
      }
    }
    hipStream_t s = nullptr;
    VW_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    return s;
  }
  void GiveStream(int dev, hipStream_t s) {
    {
      std::lock_guard<std::mutex> lk(mu);
      auto& v = streams[dev];
      if (v.size() < 4) {
        v.push_back(s);
        return;
      }
    }
    (void)hipStreamDestroy(s);
  }
};

struct GpuSgd::Impl {
  hipStream_t stream = nullptr, copy_stream = nullptr;
  int dev = 0;
  bool clean = false;  // W is all zeros again (a final export cleared it)
  Stager& stager = SharedStager();  // pinned host->device staging of pass data (on this learner's copy_stream)
  std::vector<hipEvent_t> events;
  hipEvent_t ev_ip = nullptr;  // ExpandToStage: the offsets' upload, ordered before the count kernel
  float4* W = nullptr;
  uint64_t nw = 0;
  uint8_t* dirty = nullptr;   // the touch map (nfine bytes)
  uint8_t* coarse = nullptr;  // sync: 64 KB blocks written this epoch (nblk bytes)
  int64_t nblk = 0, nfine = 0;
  int epoch = 1;
  double* gs = nullptr;
  int64_t* indptr = nullptr;
  uint32_t* idx = nullptr;
  float *val = nullptr, *lab = nullptr, *wt = nullptr, *lo = nullptr, *hi = nullptr, *pred = nullptr, *loss = nullptr;
  size_t cap_rows = 0, cap_nnz = 0;
  // reductions: csoaa (class, cost) lists; CB multi-line examples
  int64_t *cptr = nullptr, *aip = nullptr;
  int32_t *ccls = nullptr, *chosen = nullptr;
  float *ccost = nullptr, *cbcost = nullptr, *cbprob = nullptr, *best = nullptr;
  float *cats_act = nullptr, *cats_cost = nullptr, *cats_pdf = nullptr, *cats_base = nullptr;
  uint8_t* cats_has = nullptr;
  double* cbstats = nullptr;
  ExpandSpec* spec = nullptr;
  // sync scratch
  int32_t *pos = nullptr, *blocks = nullptr;
  float* sums = nullptr;  // per-slot (w or wG, G) sync sums, fp32 as VW's allreduce
  float* nmax = nullptr;
  size_t cap_sync = 0;
  void Reserve(size_t rows, size_t nnz) {
    if (rows > cap_rows) {
      for (void* q : {static_cast<void*>(indptr), static_cast<void*>(lab), static_cast<void*>(wt), static_cast<void*>(lo),
                      static_cast<void*>(hi), static_cast<void*>(pred)})
        PoolFree(q);
      PoolMalloc(&indptr, (rows + 1) * sizeof(int64_t));
      PoolMalloc(&lab, rows * sizeof(float));
      PoolMalloc(&wt, rows * sizeof(float));
      PoolMalloc(&lo, rows * sizeof(float));
      PoolMalloc(&hi, rows * sizeof(float));
      PoolMalloc(&pred, rows * sizeof(float));
      cap_rows = rows;
    }
    if (nnz > cap_nnz) {
      PoolFree(idx); PoolFree(val);
      PoolMalloc(&idx, std::max<size_t>(1, nnz) * sizeof(uint32_t));
      PoolMalloc(&val, std::max<size_t>(1, nnz) * sizeof(float));
      cap_nnz = nnz;
    }
  }
  ~Impl() {
    static const bool prof = std::getenv("SML_VW_LIFE_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    struct Done {
      bool on;
      std::chrono::steady_clock::time_point t0;
      ~Done() {
        if (on)
          std::fprintf(stderr, "[vw learner] destroy %.3f ms\n",
                       std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
      }
    } done{prof, t0};
    if (stream) (void)hipStreamSynchronize(stream);
    if (copy_stream) (void)hipStreamSynchronize(copy_stream);
    for (hipEvent_t e : events) (void)hipEventDestroy(e);
    if (ev_ip) (void)hipEventDestroy(ev_ip);
    if (copy_stream) CleanTables::Get().GiveStream(dev, copy_stream);
    for (void* q : {static_cast<void*>(cptr), static_cast<void*>(aip), static_cast<void*>(ccls),
                    static_cast<void*>(chosen), static_cast<void*>(ccost), static_cast<void*>(cbcost),
                    static_cast<void*>(cbprob), static_cast<void*>(best), static_cast<void*>(spec)})
      (void)hipFree(q);
    PoolFree(cbstats);
    for (void* q : {static_cast<void*>(cats_act), static_cast<void*>(cats_cost), static_cast<void*>(cats_pdf),
                    static_cast<void*>(cats_base), static_cast<void*>(cats_has)})
      PoolFree(q);
    if (W && clean && CleanTables::Get().Give(dev, W, nw * sizeof(float4))) W = nullptr;
    for (void* q : {static_cast<void*>(W), static_cast<void*>(indptr), static_cast<void*>(idx), static_cast<void*>(val),
                    static_cast<void*>(lab), static_cast<void*>(wt), static_cast<void*>(lo), static_cast<void*>(hi),
                    static_cast<void*>(pred)})
      PoolFree(q);
    PoolFree(dirty);
    PoolFree(coarse);
    PoolFree(gs);
    PoolFree(loss);
    for (void* q : {static_cast<void*>(pos), static_cast<void*>(blocks), static_cast<void*>(sums), static_cast<void*>(nmax)})
      (void)hipFree(q);
    if (stream) CleanTables::Get().GiveStream(dev, stream);
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
  static const bool prof = std::getenv("SML_VW_LIFE_TIMING") != nullptr;
  const auto t_start = std::chrono::steady_clock::now();
  if (device >= 0) VW_HIP_CHECK(hipSetDevice(device));
  if (cfg.oaa > 256) throw std::runtime_error("GPU oaa supports at most 256 classes");
  if (cfg.csoaa > 256) throw std::runtime_error("GPU csoaa supports at most 256 classes");
  if ((cfg.oaa > 0) + (cfg.csoaa > 0) + (cfg.cb >= 0) + (cfg.cats > 0) > 1) throw std::runtime_error("one reduction at a time");
  if (cfg.cats == 1 || cfg.cats > 4096) throw std::runtime_error("GPU CATS supports 2..4096 discrete actions");
  if (cfg.cats > 0 && !(cfg.cats_max > cfg.cats_min && cfg.cats_bw > 0.f))
    throw std::runtime_error("GPU CATS needs min_value < max_value and bandwidth > 0");
  VW_HIP_CHECK(hipGetDevice(&impl_->dev));
  impl_->stream = CleanTables::Get().TakeStream(impl_->dev);
  impl_->copy_stream = CleanTables::Get().TakeStream(impl_->dev);
  impl_->nw = 1ull << cfg.bits;
  void* clean = nullptr;
  if (std::getenv("SML_VW_CLEAN_TABLES") && std::atoi(std::getenv("SML_VW_CLEAN_TABLES")) == 0) {
    // (A/B: every learner zeroes its own table)
  } else if (CleanTables::Get().Take(impl_->dev, impl_->nw * sizeof(float4), &clean)) {
    impl_->W = static_cast<float4*>(clean);
  }
  if (!impl_->W) {
    PoolMalloc(&impl_->W, impl_->nw * sizeof(float4));
    VW_HIP_CHECK(hipMemsetAsync(impl_->W, 0, impl_->nw * sizeof(float4), impl_->stream));
  }
  impl_->nblk = static_cast<int64_t>((impl_->nw + (1ull << kDirtyShift) - 1) >> kDirtyShift);
  impl_->nfine = static_cast<int64_t>(impl_->nblk) * kTouchPerBlock;
  PoolMalloc(&impl_->dirty, impl_->nfine);
  VW_HIP_CHECK(hipMemsetAsync(impl_->dirty, 0, impl_->nfine, impl_->stream));
  PoolMalloc(&impl_->coarse, impl_->nblk);
  PoolMalloc(&impl_->gs, 3 * sizeof(double));
  VW_HIP_CHECK(hipMemsetAsync(impl_->gs, 0, 3 * sizeof(double), impl_->stream));
  PoolMalloc(&impl_->cbstats, 3 * sizeof(double));
  VW_HIP_CHECK(hipMemsetAsync(impl_->cbstats, 0, 3 * sizeof(double), impl_->stream));
  PoolMalloc(&impl_->loss, sizeof(float));
  VW_HIP_CHECK(hipMemsetAsync(impl_->loss, 0, sizeof(float), impl_->stream));
  // no wait here: every later use of the table is ordered behind the zeroing on this stream, and the
  // caller's host work (featurization, labels) overlaps the 16 GiB memset of a 2^30 table (~2.8 ms)
  if (cfg.loss == 1) { min_label_ = -50.0; max_label_ = 50.0; }
  if (prof)
    std::fprintf(stderr, "[vw learner] create %.3f ms\n",
                 std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count());
}

GpuSgd::~GpuSgd() {
  PoolFree(export_reg_);  // an export counted but never written
  PoolFree(export_cnt_);
}

namespace {
SgdArgs BaseArgs(const GpuSgdConfig& c) {
  SgdArgs a{};
  a.lr = c.lr; a.power_t = c.power_t; a.initial_t = c.initial_t; a.l2 = c.l2; a.l1 = c.l1; a.tau = c.tau;
  a.loss = c.loss;
  a.adaptive = c.adaptive ? 1 : 0; a.normalized = c.normalized ? 1 : 0; a.invariant = c.invariant ? 1 : 0;
  a.K = c.oaa > 0 ? c.oaa : c.csoaa;
  static const int hot_agg = [] {
    const char* e = std::getenv("SML_VW_HOT_AGG");
    return e ? std::atoi(e) : 1;
  }();
  a.hot_agg = hot_agg;
  return a;
}
}  // namespace

void GpuSgd::Launch(int64_t b0, int64_t b1, bool learn, bool have_weights) {
  CheckLive();
  SgdArgs a = BaseArgs(cfg_);
  a.indptr = impl_->indptr; a.idx = impl_->idx; a.val = impl_->val; a.lab = impl_->lab;
  a.wt = have_weights ? impl_->wt : nullptr;
  a.lo = (learn && cfg_.oaa == 0) ? impl_->lo : nullptr;
  a.hi = impl_->hi;
  if (learn && clamp_const_ && a.lo) {
    a.lo = nullptr;
    a.clamp_const = 1;
    a.clo = static_cast<float>(min_label_);
    a.chi = static_cast<float>(max_label_);
  }
  a.n0 = b0; a.n1 = b1; a.W = impl_->W; a.mask = impl_->nw - 1; a.dirty = impl_->dirty; a.epoch = impl_->epoch; a.gs = impl_->gs;
  a.preds = impl_->pred; a.loss_acc = impl_->loss; a.learn = learn ? 1 : 0;
  if (cfg_.cats > 0) {
    a.lo = nullptr;
    if (learn && !impl_->cats_has) throw std::runtime_error("CATS learning needs StageCats first");
    int depth = 0;
    while ((1 << depth) < cfg_.cats) ++depth;
    CatsArgs c{impl_->cats_act, impl_->cats_cost, impl_->cats_pdf, impl_->cats_base, impl_->cats_has, cfg_.cats, depth,
               cfg_.cats_min, cfg_.cats_max, cfg_.cats_bw};
    const size_t lds = sizeof(float) * 2 * (2 * (size_t(1) << depth) - 1);
    hipLaunchKernelGGL(cats_kernel, dim3(static_cast<unsigned>(b1 - b0)), dim3(64), lds, impl_->stream, a, c);
  } else if (cfg_.cb >= 0) {
    a.lo = nullptr;
    CbArgs cb{impl_->aip, impl_->chosen, impl_->cbcost, impl_->cbprob, cfg_.cb, cfg_.cb_explore ? 1 : 0, cfg_.epsilon,
              impl_->cbstats, impl_->best};
    // the widest example of the staged set sizes the score buffer
    hipLaunchKernelGGL(cb_kernel, dim3(static_cast<unsigned>(b1 - b0)), dim3(64 * kCbWaves),
                       sizeof(float) * std::max<int64_t>(1, max_actions_), impl_->stream, a, cb);
  } else if (cfg_.csoaa > 0) {
    a.lo = nullptr;
    const int waves = std::min(cfg_.csoaa, kOaaMaxWaves);
    hipLaunchKernelGGL(csoaa_kernel, dim3(static_cast<unsigned>(b1 - b0)), dim3(64 * waves), sizeof(float) * cfg_.csoaa,
                       impl_->stream, a, staged_costs_ ? impl_->cptr : nullptr, impl_->ccls, impl_->ccost);
  } else if (cfg_.oaa > 0) {
    const int waves = std::min(cfg_.oaa, kOaaMaxWaves);
    hipLaunchKernelGGL(oaa_kernel, dim3(static_cast<unsigned>(b1 - b0)), dim3(64 * waves), sizeof(float) * cfg_.oaa,
                       impl_->stream, a);
  } else {
    const int grid = static_cast<int>((b1 - b0 + kSgdWaves - 1) / kSgdWaves);
    hipLaunchKernelGGL(sgd_kernel, dim3(grid), dim3(64 * kSgdWaves), 0, impl_->stream, a);
  }
  VW_HIP_CHECK(hipGetLastError());
}

// Hogwild warm-up: the learner's first examples run in launches of 1, 1, 2, 4, ... examples (doubling up to
// `batch`), so the adaptive / normalized state (every slot's G and N, the global t / weight / norm sums) forms
// near-sequentially before wide concurrency. Without it, `batch` examples of a fresh table all take their large
// first-step rates at once: on dense features (every example updating the same slots) their summed steps
// overshoot, and 1-2 fits in 14 diverged at batch 64 / 256 (progressive loss 3-9, AUC 0.87-0.98; r5 passes
// 18-19). Launch sizes depend only on how many examples the learner has seen, so runs stay reproducible.
int64_t GpuSgd::NextLaunch(int64_t b0, int64_t r0, int64_t r1, int batch) const {
  const int64_t seen = static_cast<int64_t>(examples_) + (b0 - r0);
  int64_t bs = batch;
  if (seen < batch) {
    bs = 1;
    while (bs * 2 <= seen) bs *= 2;
  }
  return std::min<int64_t>(r1, b0 + bs);
}

void GpuSgd::Learn(const int64_t* indptr, const uint32_t* indices, const float* values, const float* labels,
                   const float* weights, int64_t n, int batch, float* preds_out) {
  CheckLive();
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
                  (p1 - p0) * sizeof(float), cs, /*unit_floats=*/true);
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
    // launches follow the unchunked boundary sequence (the warm-up's 1, 1, 2, 4, ... then `batch`): one that runs
    // past the chunk that has landed waits for the next chunk instead of being cut at the chunk boundary
    int64_t lb0 = 0;
    for (int64_t c = 0; c < nchunks; ++c) {
      {
        std::unique_lock<std::mutex> g(rmu);
        rcv.wait(g, [&] { return recorded > c; });
        if (!upload_error.empty()) break;
      }
      VW_HIP_CHECK(hipStreamWaitEvent(s, impl_->events[c], 0));
      const int64_t r1 = std::min<int64_t>(n, (c + 1) * chunk_rows);
      while (lb0 < r1) {
        const int64_t b1 = NextLaunch(lb0, 0, n, batch);
        if (b1 > r1) break;
        Launch(lb0, b1, true, weights != nullptr);
        lb0 = b1;
      }
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
  CheckLive();
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
            cs, /*unit_floats=*/true);
    VW_HIP_CHECK(hipStreamSynchronize(cs));
  }
  VW_HIP_CHECK(hipStreamSynchronize(s));
  staged_labels_.assign(labels, labels + n);
  staged_n_ = n;
  staged_rows_ = n;
  staged_weights_ = weights != nullptr;
  staged_costs_ = false;
}

void GpuSgd::PrepLearn(int64_t r0, int64_t r1) {
  hipStream_t s = impl_->stream;
  const int64_t m = r1 - r0;
  if (cfg_.cats > 0 && m > 0) {
    // CATS control variate: the running mean cost over the labelled examples so far, this one included (the
    // learner state carries across passes and segments, as the host learner's)
    if (static_cast<int64_t>(cats_has_.size()) < r1) throw std::runtime_error("CATS learning needs StageCats first");
    std::vector<float> base(m);
    for (int64_t i = 0; i < m; ++i) {
      if (cats_has_[r0 + i]) {
        cats_cost_sum_ += cats_cost_[r0 + i];
        cats_cost_n_ += 1.0;
      }
      base[i] = cats_cost_n_ > 0 ? static_cast<float>(cats_cost_sum_ / cats_cost_n_) : 0.f;
    }
    VW_HIP_CHECK(hipMemcpyAsync(impl_->cats_base + r0, base.data(), m * sizeof(float), hipMemcpyHostToDevice, s));
    VW_HIP_CHECK(hipStreamSynchronize(s));  // base is a local
  }
  const bool scalar = cfg_.oaa == 0 && cfg_.csoaa == 0 && cfg_.cb < 0 && cfg_.cats == 0;
  // logistic: the fixed [-50, 50] range, passed to the kernel as two scalars (per-example arrays cost a 16 MB
  // fill + pageable upload + stream wait ahead of the first learning launch: ~3 ms of a 45 ms fit, r5 pass 55)
  clamp_const_ = scalar && cfg_.loss == 1;
  if (scalar && m > 0 && !clamp_const_) {
    std::vector<float> lo(m), hi(m);
    for (int64_t i = 0; i < m; ++i) {
      min_label_ = std::min<double>(min_label_, staged_labels_[r0 + i]);
      max_label_ = std::max<double>(max_label_, staged_labels_[r0 + i]);
      lo[i] = static_cast<float>(min_label_);
      hi[i] = static_cast<float>(max_label_);
    }
    VW_HIP_CHECK(hipMemcpyAsync(impl_->lo + r0, lo.data(), m * sizeof(float), hipMemcpyHostToDevice, s));
    VW_HIP_CHECK(hipMemcpyAsync(impl_->hi + r0, hi.data(), m * sizeof(float), hipMemcpyHostToDevice, s));
    VW_HIP_CHECK(hipStreamSynchronize(s));  // lo / hi are locals: the copies must be done before they go
  }
  VW_HIP_CHECK(hipMemsetAsync(impl_->loss, 0, sizeof(float), s));
}

void GpuSgd::FinishLearn(int64_t r0, int64_t r1, float* preds_out) {
  hipStream_t s = impl_->stream;
  float l = 0;
  VW_HIP_CHECK(hipMemcpyAsync(&l, impl_->loss, sizeof(float), hipMemcpyDeviceToHost, s));
  if (preds_out && cfg_.cb < 0)
    VW_HIP_CHECK(hipMemcpyAsync(preds_out, impl_->pred + r0, (r1 - r0) * sizeof(float), hipMemcpyDeviceToHost, s));
  VW_HIP_CHECK(hipStreamSynchronize(s));
  examples_ += r1 - r0;
  sum_loss_ += l;
}

void GpuSgd::LearnStaged(int64_t r0, int64_t r1, int batch, float* preds_out) {
  CheckLive();
  if (r0 < 0 || r1 > staged_n_ || r0 > r1) throw std::runtime_error("LearnStaged: rows outside the staged set");
  if (r1 == r0) return;
  PrepLearn(r0, r1);
  batch = std::max(1, batch);
  for (int64_t b0 = r0, b1; b0 < r1; b0 = b1) {
    b1 = NextLaunch(b0, r0, r1, batch);
    Launch(b0, b1, true, staged_weights_);
  }
  FinishLearn(r0, r1, preds_out);
}

// ---- device featurization
void GpuSgd::ExpandToStage(const FeatPlan& plan, int64_t n, int64_t learn_r1, int batch) {
  if (plan.ngroups > kMaxGroups) throw std::runtime_error("device featurization: more than 32 namespaces");
  if (static_cast<int>(plan.inter.size()) > kMaxInter) throw std::runtime_error("device featurization: more than 64 interactions");
  hipStream_t s = impl_->stream, cs = impl_->copy_stream;
  ExpandSpec h{};
  h.ngroups = plan.ngroups;
  h.ninter = static_cast<int>(plan.inter.size());
  h.constant = plan.constant ? 1 : 0;
  for (int q = 0; q < h.ninter; ++q)
    for (int k = 0; k < 3; ++k) {
      const int g = plan.inter[q][k];
      if (g >= plan.ngroups || (k < 2 && g < 0)) throw std::runtime_error("device featurization: bad interaction");
      h.inter[q][k] = g;
    }
  std::vector<void*> tmp;
  auto dev_alloc = [&](size_t bytes) -> void* {  // freed at the end of the staging
    void* d = nullptr;
    PoolMalloc(&d, std::max<size_t>(bytes, 8));
    tmp.push_back(d);
    return d;
  };
  auto dev_copy = [&](const void* src, size_t bytes) -> void* {
    void* d = dev_alloc(bytes);
    if (bytes) impl_->stager.Copy(static_cast<char*>(d), static_cast<const char*>(src), bytes, cs);
    return d;
  };
  // Block feature ids / values are the pass's bulk (8 B per nonzero): they go up after the small per-row
  // arrays, in row chunks when learning rides along (a chunk's rows are expanded and learned while the next
  // chunk's bytes cross PCIe), else in one piece.
  struct Bulk {
    uint32_t* idx;
    float* val;
    const HostBlock* b;
  };
  std::vector<Bulk> bulk;
  const int64_t lr1 = std::min<int64_t>(std::max<int64_t>(0, learn_r1), n);
  batch = std::max(1, batch);
  // whole batches per chunk, >= 64k rows; the launches follow the unchunked LearnStaged's boundaries (a launch
  // that straddles a chunk boundary runs once the next chunk is expanded)
  // (SML_VW_STAGE_CHUNK_ROWS: another floor, read per call - the tests cut a small pass into many chunks)
  const char* ce = std::getenv("SML_VW_STAGE_CHUNK_ROWS");
  const int64_t floor_rows = ce && std::atoll(ce) > 0 ? std::atoll(ce) : 65536;
  const int64_t chunk_rows =
      lr1 > 0 ? std::max<int64_t>(1, (floor_rows + batch - 1) / batch) * batch : std::max<int64_t>(1, n);
  const int64_t nchunks = n > 0 ? (n + chunk_rows - 1) / chunk_rows : 0;
  try {
    {
      std::lock_guard<std::mutex> lk(impl_->stager.mu);
      for (const HostBlock& b : plan.blocks) {
        if (b.group < 0 || b.group >= plan.ngroups) throw std::runtime_error("device featurization: bad group");
        const int k = h.gblocks[b.group]++;
        if (k >= kMaxGroupBlocks) throw std::runtime_error("device featurization: more than 4 blocks in a namespace");
        if (b.level == 0 && b.rows != n) throw std::runtime_error("device featurization: block rows != examples");
        const int64_t nnz = b.ip[b.rows] - b.ip[0];
        DevBlock d;
        if (b.ip[0] == 0) {
          d.ip = static_cast<const int64_t*>(dev_copy(b.ip, (b.rows + 1) * sizeof(int64_t)));
        } else {  // a row slice of a larger CSR: rebase its offsets
          std::vector<int64_t> ip(b.ip, b.ip + b.rows + 1);
          for (auto& v : ip) v -= b.ip[0];
          d.ip = static_cast<const int64_t*>(dev_copy(ip.data(), ip.size() * sizeof(int64_t)));
        }
        auto* di = static_cast<uint32_t*>(dev_alloc(nnz * sizeof(uint32_t)));
        auto* dv = static_cast<float*>(dev_alloc(nnz * sizeof(float)));
        d.idx = di;
        d.val = dv;
        d.level = b.level;
        h.blk[b.group][k] = d;
        bulk.push_back({di, dv, &b});
      }
      if (plan.row_map) h.row_map = static_cast<const int64_t*>(dev_copy(plan.row_map, n * sizeof(int64_t)));
    }
    // the offsets (and row map) are ordered before the count kernel by an event, not a host wait, and the
    // bulk uploader starts now: its chunks cross PCIe while the table is zeroed and the layout is counted
    // (r5 pass 54: the host waits put ~8 ms between the fit's start and the first chunk)
    if (!impl_->ev_ip) VW_HIP_CHECK(hipEventCreateWithFlags(&impl_->ev_ip, hipEventDisableTiming));
    VW_HIP_CHECK(hipEventRecord(impl_->ev_ip, cs));
    VW_HIP_CHECK(hipStreamWaitEvent(s, impl_->ev_ip, 0));
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
          for (const Bulk& u : bulk) {
            const HostBlock& b = *u.b;
            // per-example blocks go up row range by row range; row-mapped (level 1) blocks whole, first
            int64_t p0, p1;
            if (b.level == 0) {
              p0 = b.ip[r0] - b.ip[0];
              p1 = b.ip[r1] - b.ip[0];
            } else if (c == 0) {
              p0 = 0;
              p1 = b.ip[b.rows] - b.ip[0];
            } else {
              continue;
            }
            if (p1 > p0) {
              st.Copy(reinterpret_cast<char*>(u.idx + p0), reinterpret_cast<const char*>(b.idx + b.ip[0] + p0),
                      (p1 - p0) * sizeof(uint32_t), cs);
              st.Copy(reinterpret_cast<char*>(u.val + p0), reinterpret_cast<const char*>(b.val + b.ip[0] + p0),
                      (p1 - p0) * sizeof(float), cs, /*unit_floats=*/true);
            }
          }
          VW_HIP_CHECK(hipEventRecord(impl_->events[c], cs));
          std::lock_guard<std::mutex> g(rmu);
          recorded = c + 1;
          rcv.notify_all();
        }
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> g(rmu);
        upload_error = e.what();
        recorded = nchunks;  // release the expand loop; it rethrows
        rcv.notify_all();
      }
    });
    try {
      if (!impl_->spec) VW_HIP_CHECK(hipMalloc(&impl_->spec, sizeof(ExpandSpec)));
      VW_HIP_CHECK(hipMemcpyAsync(impl_->spec, &h, sizeof(ExpandSpec), hipMemcpyHostToDevice, s));
      impl_->Reserve(std::max<int64_t>(1, n), impl_->cap_nnz);
      VW_HIP_CHECK(hipMemsetAsync(impl_->indptr, 0, sizeof(int64_t), s));
      if (n > 0) {  // row lengths need only the offsets: the whole pass's CSR layout before any bulk byte lands
        const int grid = static_cast<int>(std::min<int64_t>(65536, (n + 255) / 256));
        hipLaunchKernelGGL(expand_count_kernel, dim3(grid), dim3(256), 0, s, impl_->spec, n, impl_->indptr + 1);
        VW_HIP_CHECK(hipGetLastError());
        size_t tb = 0;
        VW_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(nullptr, tb, impl_->indptr + 1, impl_->indptr + 1, n, s));
        void* tbuf = dev_alloc(tb);  // the scan's temporary storage (no host source)
        VW_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(tbuf, tb, impl_->indptr + 1, impl_->indptr + 1, n, s));
      }
      int64_t nnz = 0;
      VW_HIP_CHECK(hipMemcpyAsync(&nnz, impl_->indptr + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
      VW_HIP_CHECK(hipStreamSynchronize(s));
      impl_->Reserve(std::max<int64_t>(1, n), static_cast<size_t>(nnz));
      if (lr1 > 0) PrepLearn(0, lr1);
      int64_t lb0 = 0;
      for (int64_t c = 0; c < nchunks; ++c) {
        {
          std::unique_lock<std::mutex> g(rmu);
          rcv.wait(g, [&] { return recorded > c; });
          if (!upload_error.empty()) break;
        }
        VW_HIP_CHECK(hipStreamWaitEvent(s, impl_->events[c], 0));
        const int64_t r0 = c * chunk_rows, r1 = std::min<int64_t>(n, r0 + chunk_rows);
        const int grid = static_cast<int>(std::min<int64_t>(65536, (r1 - r0 + kExpandWaves - 1) / kExpandWaves));
        hipLaunchKernelGGL(expand_fill_kernel, dim3(grid), dim3(64 * kExpandWaves), 0, s, impl_->spec, r0, r1,
                           impl_->indptr, impl_->idx, impl_->val);
        VW_HIP_CHECK(hipGetLastError());
        while (lb0 < std::min(r1, lr1)) {
          const int64_t b1 = NextLaunch(lb0, 0, lr1, batch);
          if (b1 > r1) break;
          Launch(lb0, b1, true, staged_weights_);
          lb0 = b1;
        }
      }
    } catch (...) {
      uploader.join();
      throw;
    }
    uploader.join();
    if (!upload_error.empty()) throw std::runtime_error("VW pass upload failed: " + upload_error);
    VW_HIP_CHECK(hipStreamSynchronize(s));
  } catch (...) {
    (void)hipStreamSynchronize(s);
    (void)hipStreamSynchronize(cs);
    for (void* q : tmp) PoolFree(q);
    throw;
  }
  for (void* q : tmp) PoolFree(q);
  staged_rows_ = n;
  if (lr1 > 0) FinishLearn(0, lr1, nullptr);
}

void GpuSgd::StagePlan(const FeatPlan& plan, int64_t n, const float* labels, const float* weights, int64_t learn_r1,
                       int batch) {
  CheckLive();
  if (n < 0) throw std::runtime_error("negative row count");
  hipStream_t s = impl_->stream;
  if (learn_r1 > 0 && (cfg_.cb >= 0 || cfg_.csoaa > 0 || cfg_.cats > 0))  // label extras staged after the plan
    throw std::runtime_error("StagePlan: learning while staging is for the scalar / oaa learners");
  // labels / weights first: a pipelined stage learns as the chunks land
  impl_->Reserve(std::max<int64_t>(1, n), impl_->cap_nnz);
  if (cfg_.cb < 0 && n) {
    // through the pinned stager on the copy stream: a pageable copy on the compute stream queued behind the
    // table's zeroing and held the host until it had run; ExpandToStage orders the copy stream before any
    // kernel that reads the labels (its offsets event)
    std::lock_guard<std::mutex> lk(impl_->stager.mu);
    impl_->stager.Copy(reinterpret_cast<char*>(impl_->lab), reinterpret_cast<const char*>(labels), n * sizeof(float),
                       impl_->copy_stream);
    if (weights)
      impl_->stager.Copy(reinterpret_cast<char*>(impl_->wt), reinterpret_cast<const char*>(weights),
                         n * sizeof(float), impl_->copy_stream);
    // the host copy feeds only the running label range of non-logistic scalar learners (PrepLearn); a logistic
    // learner clamps to fixed bounds, so its 8 MB per 2M-example pass is not copied (fresh pages every fit)
    const bool scalar = cfg_.oaa == 0 && cfg_.csoaa == 0 && cfg_.cb < 0 && cfg_.cats == 0;
    if (scalar && cfg_.loss == 1) staged_labels_.clear();
    else staged_labels_.assign(labels, labels + n);
    staged_n_ = n;
  }
  staged_weights_ = weights != nullptr;
  staged_costs_ = false;
  ExpandToStage(plan, n, learn_r1, batch);
  VW_HIP_CHECK(hipStreamSynchronize(s));
}

void GpuSgd::StageCosts(const int64_t* cptr, const int32_t* cls, const float* cost, int64_t n) {
  CheckLive();
  if (n != staged_n_) throw std::runtime_error("StageCosts: rows != staged examples");
  hipStream_t s = impl_->stream;
  const int64_t m = cptr[n] - cptr[0];
  std::vector<int64_t> ip(cptr, cptr + n + 1);
  for (auto& v : ip) v -= cptr[0];
  for (void* q : {static_cast<void*>(impl_->cptr), static_cast<void*>(impl_->ccls), static_cast<void*>(impl_->ccost)})
    (void)hipFree(q);
  VW_HIP_CHECK(hipMalloc(&impl_->cptr, (n + 1) * sizeof(int64_t)));
  VW_HIP_CHECK(hipMalloc(&impl_->ccls, std::max<int64_t>(1, m) * sizeof(int32_t)));
  VW_HIP_CHECK(hipMalloc(&impl_->ccost, std::max<int64_t>(1, m) * sizeof(float)));
  VW_HIP_CHECK(hipMemcpyAsync(impl_->cptr, ip.data(), (n + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  if (m) {
    VW_HIP_CHECK(hipMemcpyAsync(impl_->ccls, cls + cptr[0], m * sizeof(int32_t), hipMemcpyHostToDevice, s));
    VW_HIP_CHECK(hipMemcpyAsync(impl_->ccost, cost + cptr[0], m * sizeof(float), hipMemcpyHostToDevice, s));
  }
  VW_HIP_CHECK(hipStreamSynchronize(s));
  staged_costs_ = true;
}

void GpuSgd::StageCats(const float* action, const float* cost, const float* pdf, const uint8_t* has, int64_t n) {
  CheckLive();
  if (cfg_.cats <= 0) throw std::runtime_error("StageCats: the learner is not a CATS learner");
  if (n != staged_n_) throw std::runtime_error("StageCats: rows != staged examples");
  hipStream_t s = impl_->stream;
  for (void* q : {static_cast<void*>(impl_->cats_act), static_cast<void*>(impl_->cats_cost),
                  static_cast<void*>(impl_->cats_pdf), static_cast<void*>(impl_->cats_base),
                  static_cast<void*>(impl_->cats_has)})
    PoolFree(q);
  const size_t m = static_cast<size_t>(std::max<int64_t>(1, n));
  PoolMalloc(&impl_->cats_act, m * sizeof(float));
  PoolMalloc(&impl_->cats_cost, m * sizeof(float));
  PoolMalloc(&impl_->cats_pdf, m * sizeof(float));
  PoolMalloc(&impl_->cats_base, m * sizeof(float));
  PoolMalloc(&impl_->cats_has, m);
  if (n > 0) {
    VW_HIP_CHECK(hipMemcpyAsync(impl_->cats_act, action, n * sizeof(float), hipMemcpyHostToDevice, s));
    VW_HIP_CHECK(hipMemcpyAsync(impl_->cats_cost, cost, n * sizeof(float), hipMemcpyHostToDevice, s));
    VW_HIP_CHECK(hipMemcpyAsync(impl_->cats_pdf, pdf, n * sizeof(float), hipMemcpyHostToDevice, s));
    VW_HIP_CHECK(hipMemcpyAsync(impl_->cats_has, has, n, hipMemcpyHostToDevice, s));
  }
  cats_cost_.assign(cost, cost + n);
  cats_has_.assign(has, has + n);
  VW_HIP_CHECK(hipStreamSynchronize(s));
}

void GpuSgd::StageCb(const int64_t* aip, const int32_t* chosen, const float* cost, const float* prob, int64_t ne) {
  CheckLive();
  if (cfg_.cb < 0) throw std::runtime_error("StageCb on a learner without --cb_adf");
  if (aip[ne] - aip[0] != staged_rows_) throw std::runtime_error("StageCb: action rows != staged rows");
  hipStream_t s = impl_->stream;
  std::vector<int64_t> ip(aip, aip + ne + 1);
  for (auto& v : ip) v -= aip[0];
  max_actions_ = 0;
  for (int64_t e = 0; e < ne; ++e) max_actions_ = std::max(max_actions_, ip[e + 1] - ip[e]);
  if (max_actions_ > 4096) throw std::runtime_error("GPU cb_adf supports at most 4096 actions per example");
  for (void* q : {static_cast<void*>(impl_->aip), static_cast<void*>(impl_->chosen), static_cast<void*>(impl_->cbcost),
                  static_cast<void*>(impl_->cbprob), static_cast<void*>(impl_->best)})
    (void)hipFree(q);
  const size_t m = std::max<int64_t>(1, ne);
  VW_HIP_CHECK(hipMalloc(&impl_->aip, (ne + 1) * sizeof(int64_t)));
  VW_HIP_CHECK(hipMalloc(&impl_->chosen, m * sizeof(int32_t)));
  VW_HIP_CHECK(hipMalloc(&impl_->cbcost, m * sizeof(float)));
  VW_HIP_CHECK(hipMalloc(&impl_->cbprob, m * sizeof(float)));
  VW_HIP_CHECK(hipMalloc(&impl_->best, m * sizeof(float)));
  VW_HIP_CHECK(hipMemcpyAsync(impl_->aip, ip.data(), (ne + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  if (ne) {
    VW_HIP_CHECK(hipMemcpyAsync(impl_->chosen, chosen, ne * sizeof(int32_t), hipMemcpyHostToDevice, s));
    VW_HIP_CHECK(hipMemcpyAsync(impl_->cbcost, cost, ne * sizeof(float), hipMemcpyHostToDevice, s));
    VW_HIP_CHECK(hipMemcpyAsync(impl_->cbprob, prob, ne * sizeof(float), hipMemcpyHostToDevice, s));
  }
  VW_HIP_CHECK(hipStreamSynchronize(s));
  staged_n_ = ne;
  staged_labels_.assign(ne, 0.f);
  staged_weights_ = false;
}

void GpuSgd::PredictStaged(float* out, float* best) {
  CheckLive();
  hipStream_t s = impl_->stream;
  const int64_t ne = staged_n_;
  if (ne <= 0) return;
  const bool scalar = cfg_.oaa == 0 && cfg_.csoaa == 0 && cfg_.cb < 0 && cfg_.cats == 0;
  // the clamp bounds' host copies live until the stream is drained below: an async copy from pageable memory
  // may still be reading them after the call returns (these were block-scoped, freed under a pending copy:
  // intermittently garbage clamps and scores)
  std::vector<float> lo, hi;
  if (scalar) {
    lo.assign(ne, static_cast<float>(min_label_));
    hi.assign(ne, static_cast<float>(max_label_));
    VW_HIP_CHECK(hipMemcpyAsync(impl_->lo, lo.data(), ne * sizeof(float), hipMemcpyHostToDevice, s));
    VW_HIP_CHECK(hipMemcpyAsync(impl_->hi, hi.data(), ne * sizeof(float), hipMemcpyHostToDevice, s));
  }
  // prediction launches: the whole staged set at once (no updates, so no ordering to respect)
  SgdArgs a = BaseArgs(cfg_);
  a.indptr = impl_->indptr; a.idx = impl_->idx; a.val = impl_->val;
  a.lo = scalar ? impl_->lo : nullptr; a.hi = impl_->hi;
  a.n0 = 0; a.n1 = ne; a.W = impl_->W; a.mask = impl_->nw - 1; a.dirty = impl_->dirty; a.epoch = impl_->epoch; a.gs = impl_->gs;
  a.preds = impl_->pred; a.loss_acc = impl_->loss; a.learn = 0;
  if (cfg_.cats > 0) {
    int depth = 0;
    while ((1 << depth) < cfg_.cats) ++depth;
    CatsArgs c{nullptr, nullptr, nullptr, nullptr, nullptr, cfg_.cats, depth, cfg_.cats_min, cfg_.cats_max, cfg_.cats_bw};
    const size_t lds = sizeof(float) * 2 * (2 * (size_t(1) << depth) - 1);
    hipLaunchKernelGGL(cats_kernel, dim3(static_cast<unsigned>(ne)), dim3(64), lds, s, a, c);
  } else if (cfg_.cb >= 0) {
    CbArgs cb{impl_->aip, nullptr, impl_->cbcost, impl_->cbprob, cfg_.cb, cfg_.cb_explore ? 1 : 0, cfg_.epsilon, nullptr,
              impl_->best};
    hipLaunchKernelGGL(cb_kernel, dim3(static_cast<unsigned>(ne)), dim3(64 * kCbWaves),
                       sizeof(float) * std::max<int64_t>(1, max_actions_), s, a, cb);
  } else if (cfg_.csoaa > 0) {
    const int waves = std::min(cfg_.csoaa, kOaaMaxWaves);
    hipLaunchKernelGGL(csoaa_kernel, dim3(static_cast<unsigned>(ne)), dim3(64 * waves), sizeof(float) * cfg_.csoaa, s, a,
                       static_cast<const int64_t*>(nullptr), static_cast<const int32_t*>(nullptr),
                       static_cast<const float*>(nullptr));
  } else if (cfg_.oaa > 0) {
    const int waves = std::min(cfg_.oaa, kOaaMaxWaves);
    hipLaunchKernelGGL(oaa_kernel, dim3(static_cast<unsigned>(ne)), dim3(64 * waves), sizeof(float) * cfg_.oaa, s, a);
  } else {
    hipLaunchKernelGGL(sgd_kernel, dim3(static_cast<unsigned>((ne + kSgdWaves - 1) / kSgdWaves)), dim3(64 * kSgdWaves), 0,
                       s, a);
  }
  VW_HIP_CHECK(hipGetLastError());
  VW_HIP_CHECK(hipMemcpyAsync(out, impl_->pred, staged_rows_ * sizeof(float), hipMemcpyDeviceToHost, s));
  if (best && cfg_.cb >= 0) VW_HIP_CHECK(hipMemcpyAsync(best, impl_->best, ne * sizeof(float), hipMemcpyDeviceToHost, s));
  VW_HIP_CHECK(hipStreamSynchronize(s));
}

void GpuSgd::CbStats(double* ips_num, double* snips_den, double* examples) const {
  double h[3] = {0, 0, 0};
  VW_HIP_CHECK(hipMemcpyAsync(h, impl_->cbstats, sizeof(h), hipMemcpyDeviceToHost, impl_->stream));
  VW_HIP_CHECK(hipStreamSynchronize(impl_->stream));
  *ips_num = h[0]; *snips_den = h[1]; *examples = h[2];
}

void GpuSgd::Predict(const int64_t* indptr, const uint32_t* indices, const float* values, int64_t n, float* out) {
  CheckLive();
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
  a.n0 = 0; a.n1 = n; a.W = impl_->W; a.mask = impl_->nw - 1; a.dirty = impl_->dirty; a.epoch = impl_->epoch; a.gs = impl_->gs;
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
void GpuSgd::AllReduceAverage(void* comm, int world, double timeout_ms) {
  CheckLive();
  if (world < 1 || !comm) return;  // a world-1 communicator still runs the collectives (one-GPU tests)
  hipStream_t s = impl_->stream;
  ncclComm_t c = static_cast<ncclComm_t>(comm);
  // the communicator is non-blocking (bounded init): an enqueue may answer ncclInProgress (the lazy peer
  // connection of a first collective), and the next call must wait for the state to settle - bounded by
  // timeout_ms, so a peer that died cannot leave this rank spinning (the caller then aborts the communicator)
  auto nccl = [c, timeout_ms](ncclResult_t r) {
    const auto t0 = std::chrono::steady_clock::now();
    while (r == ncclInProgress) {
      if (ncclCommGetAsyncError(c, &r) != ncclSuccess) r = ncclInternalError;
      if (r != ncclInProgress) break;
      if (timeout_ms > 0 &&
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() > timeout_ms)
        throw std::runtime_error("RCCL allreduce did not settle within " + std::to_string(timeout_ms) +
                                 " ms (a peer rank failed)");
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL allreduce failed: ") + ncclGetErrorString(r));
  };
  const int64_t nblk = impl_->nblk;
  hipLaunchKernelGGL(coarsen_kernel, dim3(static_cast<unsigned>(std::min<int64_t>(65536, (nblk + 255) / 256))), dim3(256),
                     0, s, impl_->dirty, nblk, impl_->epoch, impl_->coarse);
  VW_HIP_CHECK(hipGetLastError());
  nccl(ncclAllReduce(impl_->coarse, impl_->coarse, nblk, ncclUint8, ncclMax, c, s));
  // deterministic compaction (every rank packs the same blocks in the same order): host prefix over the map
  std::vector<uint8_t> hd(nblk);
  VW_HIP_CHECK(hipMemcpyAsync(hd.data(), impl_->coarse, nblk, hipMemcpyDeviceToHost, s));
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
      VW_HIP_CHECK(hipMalloc(&impl_->sums, slots * 2 * sizeof(float)));
      VW_HIP_CHECK(hipMalloc(&impl_->nmax, slots * sizeof(float)));
      impl_->cap_sync = slots;
    }
    VW_HIP_CHECK(hipMemcpyAsync(impl_->blocks, list.data(), m * sizeof(int32_t), hipMemcpyHostToDevice, s));
    const int grid = static_cast<int>(std::min<size_t>(65536, (slots + 255) / 256));
    const int adaptive = cfg_.adaptive ? 1 : 0;
    hipLaunchKernelGGL(pack_kernel, dim3(grid), dim3(256), 0, s, impl_->W, impl_->blocks, m, impl_->nw, adaptive,
                       impl_->sums, impl_->nmax);
    VW_HIP_CHECK(hipGetLastError());
    nccl(ncclAllReduce(impl_->sums, impl_->sums, slots * 2, ncclFloat, ncclSum, c, s));
    nccl(ncclAllReduce(impl_->nmax, impl_->nmax, slots, ncclFloat, ncclMax, c, s));
    hipLaunchKernelGGL(unpack_kernel, dim3(grid), dim3(256), 0, s, impl_->W, impl_->blocks, m, impl_->nw, adaptive,
                       1.0f / world, impl_->sums, impl_->nmax);
    VW_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(mark_blocks_kernel, dim3(static_cast<unsigned>(std::min<int64_t>(65536, (m * kTouchPerBlock + 255) / 256))),
                       dim3(256), 0, s, impl_->blocks, m, impl_->epoch, impl_->dirty);
    VW_HIP_CHECK(hipGetLastError());
    last_sync_bytes_ = static_cast<int64_t>(slots) * (2 * sizeof(float) + sizeof(float)) + nblk;
  }
  // the next epoch (the touch map keeps every write for the export; 255 epochs fit a byte)
  if (impl_->epoch >= 255) {
    hipLaunchKernelGGL(touch_renorm_kernel, dim3(static_cast<unsigned>(std::min<int64_t>(65536, (impl_->nfine + 255) / 256))),
                       dim3(256), 0, s, impl_->dirty, impl_->nfine);
    VW_HIP_CHECK(hipGetLastError());
    impl_->epoch = 2;
  } else {
    ++impl_->epoch;
  }
  VW_HIP_CHECK(hipStreamSynchronize(s));
  last_sync_blocks_ = m;
}

uint64_t GpuSgd::NumWeights() const { return impl_->nw; }

// Nonzero table components as (stride-4 index, value), compacted on the device: the host only ever holds
// the nonzeros (a 2^30-slot table never crosses PCIe whole)
void GpuSgd::ExportNonzeros(std::vector<uint64_t>* idx, std::vector<float>* val) const {
  CheckLive();
  hipStream_t s = impl_->stream;
  const uint64_t per = 4096;
  const int64_t nb = static_cast<int64_t>((impl_->nw + per - 1) / per);
  int32_t* cnt = nullptr;
  int64_t* base = nullptr;
  PoolMalloc(&cnt, nb * sizeof(int32_t));  // caching pool: no hipMalloc / hipFree device syncs per export
  PoolMalloc(&base, nb * sizeof(int64_t));
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
    PoolMalloc(&di, tot * sizeof(uint64_t));
    PoolMalloc(&dv, tot * sizeof(float));
    VW_HIP_CHECK(hipMemcpyAsync(base, hb.data(), nb * sizeof(int64_t), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(write_nz_kernel, dim3(static_cast<unsigned>(nb)), dim3(64), 0, s, impl_->W, impl_->nw, per, base,
                       di, dv);
    VW_HIP_CHECK(hipMemcpyAsync(idx->data(), di, tot * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    VW_HIP_CHECK(hipMemcpyAsync(val->data(), dv, tot * sizeof(float), hipMemcpyDeviceToHost, s));
    VW_HIP_CHECK(hipStreamSynchronize(s));
    PoolFree(di);
    PoolFree(dv);
  }
  PoolFree(cnt);
  PoolFree(base);
}

// The export scans the table once when no 4096-slot block holds more than kRegionCap records (a hashed
// table's nonzeros spread evenly: ~8 per block for a 2M-example pass at 2^30), writing each block's records
// into its own region; a denser table (a small -b, a long training) takes the count scan + write scan.
constexpr int kRegionCap = 256;

// SML_VW_EXPORT_TIMING=1: per-phase export timings on stderr (profiling runs)
struct ExportClock {
  bool on;
  std::chrono::steady_clock::time_point t0;
  ExportClock() : on(std::getenv("SML_VW_EXPORT_TIMING") != nullptr), t0(std::chrono::steady_clock::now()) {}
  void mark(const char* what) {
    if (!on) return;
    const auto t1 = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[vw export] %-24s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t1 - t0).count());
    t0 = t1;
  }
};

int64_t GpuSgd::CountNonzeros() const {
  CheckLive();
  hipStream_t s = impl_->stream;
  const uint64_t per = 4096;
  const int64_t nb = static_cast<int64_t>((impl_->nw + per - 1) / per);
  int32_t* cnt = nullptr;
  PoolMalloc(&cnt, nb * sizeof(int32_t));
  ExportClock clk;
  const char* re = std::getenv("SML_VW_EXPORT_REGIONS");  // 0: the two-scan export (A/B, tests)
  const bool regions = !(re && std::atoi(re) == 0);
  if (regions) {
    PoolMalloc(&export_reg_, static_cast<size_t>(nb) * kRegionCap * 12);
    const char* sk = std::getenv("SML_VW_EXPORT_SKIP");  // 0: scan every sub-block (A/B, tests)
    const uint8_t* touch = (sk && std::atoi(sk) == 0) ? nullptr : impl_->dirty;
    hipLaunchKernelGGL(write_rec_region_kernel, dim3(static_cast<unsigned>(nb)), dim3(64), 0, s, impl_->W, impl_->nw,
                       per, kRegionCap, export_reg_, cnt, touch);
  } else {
    hipLaunchKernelGGL(count_nz_kernel, dim3(static_cast<unsigned>(nb)), dim3(256), 0, s, impl_->W, impl_->nw, per, cnt);
  }
  VW_HIP_CHECK(hipGetLastError());
  std::vector<int32_t> hc(nb);
  VW_HIP_CHECK(hipMemcpyAsync(hc.data(), cnt, nb * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  VW_HIP_CHECK(hipStreamSynchronize(s));
  clk.mark(regions ? "region scan + counts" : "count scan");
  export_base_.resize(nb);
  int64_t tot = 0;
  int32_t mx = 0;
  for (int64_t i = 0; i < nb; ++i) {
    export_base_[i] = tot;
    tot += hc[i];
    mx = std::max(mx, hc[i]);
  }
  if (regions && mx > kRegionCap) {  // too dense for the regions: the write scan runs in WriteRecords
    PoolFree(export_reg_);
    export_reg_ = nullptr;
  }
  if (export_reg_) {
    export_cnt_ = cnt;  // the region counts stay on the device for the compaction
  } else {
    PoolFree(cnt);
  }
  export_count_ = tot;
  clk.mark("host prefix");
  return tot;
}

void GpuSgd::CheckLive() const {
  if (retired_) throw std::runtime_error("GPU VW learner: its table was cleared by the final export");
}

void GpuSgd::WriteRecords(char* dst) const {
  const int64_t tot = export_count_;
  if (tot <= 0) {
    if (final_export_) {  // nothing nonzero: the table is clean as it is
      impl_->clean = true;
      retired_ = true;
    }
    PoolFree(export_reg_);
    PoolFree(export_cnt_);
    export_reg_ = nullptr;
    export_cnt_ = nullptr;
    return;
  }
  ExportClock clk;
  hipStream_t s = impl_->stream;
  const uint64_t per = 4096;
  const int64_t nb = static_cast<int64_t>(export_base_.size());
  int64_t* base = nullptr;
  uint32_t* rec = nullptr;
  PoolMalloc(&base, nb * sizeof(int64_t));
  PoolMalloc(&rec, static_cast<size_t>(tot) * 12);
  VW_HIP_CHECK(hipMemcpyAsync(base, export_base_.data(), nb * sizeof(int64_t), hipMemcpyHostToDevice, s));
  if (export_reg_) {
    const int grid = static_cast<int>(std::min<int64_t>(nb, 65536));
    hipLaunchKernelGGL(rec_compact_kernel, dim3(grid), dim3(256), 0, s, export_reg_, kRegionCap, export_cnt_, base, nb,
                       rec);
  } else {
    hipLaunchKernelGGL(write_rec_kernel, dim3(static_cast<unsigned>(nb)), dim3(64), 0, s, impl_->W, impl_->nw, per,
                       base, rec);
  }
  VW_HIP_CHECK(hipGetLastError());
  if (final_export_) {  // the records name every nonzero component: zero them behind the D2H copies below
    hipLaunchKernelGGL(clear_records_kernel, dim3(static_cast<unsigned>(std::min<int64_t>(65536, (tot + 255) / 256))),
                       dim3(256), 0, s, rec, tot, reinterpret_cast<float*>(impl_->W));
    VW_HIP_CHECK(hipGetLastError());
  }
  clk.mark("records queued");
  // device -> pinned ring (the shared stager's buffers) -> dst, the host copy of piece k overlapping the DMA
  // of piece k + 1 (a pageable D2H would bounce through the runtime's own staging at a fraction of the rate)
  Stager& st = impl_->stager;
  std::lock_guard<std::mutex> lk(st.mu);
  const size_t bytes = static_cast<size_t>(tot) * 12;
  const char* src = reinterpret_cast<const char*>(rec);
  struct Piece { int k; size_t off, n; };
  std::vector<Piece> inflight;
  auto drain_one = [&]() {
    const Piece pc = inflight.front();
    inflight.erase(inflight.begin());
    VW_HIP_CHECK(hipEventSynchronize(st.ev[pc.k]));
    const size_t per_t = (pc.n + kStageThreads - 1) / kStageThreads;
    const char* from = st.buf[pc.k];
    char* to = dst + pc.off;
    st.Team().Run([=](int t) {  // the stager's persistent copy team (the bytes object's pages fault in here)
      const size_t a0 = t * per_t, a1 = std::min(pc.n, a0 + per_t);
      if (a0 < a1) std::memcpy(to + a0, from + a0, a1 - a0);
    });
  };
  for (size_t off = 0; off < bytes; off += kStageBytes) {
    const int k = st.next;
    st.next = (st.next + 1) % kStage;
    if (!st.buf[k]) {
      VW_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&st.buf[k]), kStageBytes, hipHostMallocPortable));
      VW_HIP_CHECK(hipEventCreateWithFlags(&st.ev[k], hipEventDisableTiming));
    }
    if (st.used[k]) VW_HIP_CHECK(hipEventSynchronize(st.ev[k]));
    const size_t n = std::min(kStageBytes, bytes - off);
    VW_HIP_CHECK(hipMemcpyAsync(st.buf[k], src + off, n, hipMemcpyDeviceToHost, s));
    VW_HIP_CHECK(hipEventRecord(st.ev[k], s));
    st.used[k] = true;
    inflight.push_back({k, off, n});
    if (inflight.size() >= 2) drain_one();
  }
  while (!inflight.empty()) drain_one();
  VW_HIP_CHECK(hipStreamSynchronize(s));
  if (final_export_) {
    impl_->clean = true;
    retired_ = true;
  }
  clk.mark("d2h + host copy");
  PoolFree(base);
  PoolFree(rec);
  PoolFree(export_reg_);
  PoolFree(export_cnt_);
  export_reg_ = nullptr;
  export_cnt_ = nullptr;
  clk.mark("frees");
}

void GpuSgd::ImportNonzeros(const std::vector<uint64_t>& idx, const std::vector<float>& val) {
  CheckLive();
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
                       0, s, impl_->W, impl_->nw, impl_->dirty, impl_->epoch, di, dv, n);
    VW_HIP_CHECK(hipStreamSynchronize(s));
    (void)hipFree(di);
    (void)hipFree(dv);
  }
  VW_HIP_CHECK(hipStreamSynchronize(s));
}

void GpuSgd::GlobalState(double* t, double* total_weight, double* sum_norm_x) const {
  double h[3] = {0, 0, 0};
  VW_HIP_CHECK(hipMemcpyAsync(h, impl_->gs, sizeof(h), hipMemcpyDeviceToHost, impl_->stream));
  VW_HIP_CHECK(hipStreamSynchronize(impl_->stream));
  *t = h[0]; *total_weight = h[1]; *sum_norm_x = h[2];
}

// on the learner's (non-blocking) stream: a plain hipMemcpy runs on the null stream, which does not wait for
// the constructor's still-queued zeroing of gs on this stream and could be overwritten by it
void GpuSgd::SetGlobalState(double t, double total_weight, double sum_norm_x) {
  const double h[3] = {t, total_weight, sum_norm_x};
  VW_HIP_CHECK(hipMemcpyAsync(impl_->gs, h, sizeof(h), hipMemcpyHostToDevice, impl_->stream));
  VW_HIP_CHECK(hipStreamSynchronize(impl_->stream));
}

void* GpuSgd::weights_device() { return impl_->W; }
void* GpuSgd::stream() { return impl_->stream; }

}  // namespace smlvw
