// HIP/CDNA4 training backend: the whole leaf-wise tree growth runs on the
// MI355X with the binned matrix, gradients, scores and row partitions resident
// in HBM. Kernels:
//   K2 gradients      grad_kernel           one thread per row, fused objective
//                     lambdarank_kernel     one wave per query, pairwise lambdas
//   K8 sampling       goss_key/radix_*/     bagging + GOSS (exact radix top-k)
//                     sample_kernel         with ballot compaction
//   K3 histogram      hist_kernel           LDS-privatised per-block histograms
//                                           (packed u64 fixed point), exact slab reduce
//   K4 subtraction    find_split_kernel     larger child = parent - smaller
//   K5 split search   find_split_kernel     one block per (feature, child), bins
//                                           on lanes, fp64 prefix scan
//   K6 partition      part_kernel           single pass, wave ballots + tile cursors
//   K7 score update   score_kernel          tree traversal on bins
// The host enqueues a fixed kernel sequence per split; which leaf is split,
// its row range and the split itself live in device memory, so a tree is built
// without any host round trip (the tree is read back once at the end).
// Data-parallel training inserts an RCCL allreduce of the smaller child's
// histogram between the slab reduce and the split search (C2 over xGMI).
// tree_learner=voting (C3, PV-Tree) keeps the histograms local and reduces
// only the 2*top_k most-voted features of each new leaf (vote_kernel ..
// unpack_kernel): two small collectives per split instead of one full
// histogram. Over xGMI the full-histogram one-shot allreduce (~114 KB for 28
// features) is usually cheaper, so data_parallel stays the default; voting pays
// off for wide feature sets (thousands of features) or slower links.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <mutex>
#include <numeric>
#include <thread>
#include <unordered_map>
#include <vector>

#include <rocprofiler-sdk-roctx/roctx.h>
#include "trace.h"

#include "backend.h"
#include "comm.h"
#include "hip_common.h"
#include "valid_gpu.h"

namespace sml {
namespace {

constexpr int kBinsPerFeature = 256;
constexpr int kFeatPerGroup = 32;          // 8 dwords of bins per block
constexpr int kMaxHistBlocks = 256;        // = resident capacity: one 1024-thread, 128 KB-LDS block per CU
constexpr int kMinRowsPerHistBlockDefault = 1024;  // A/B: 1024 ~ 512 < 2048 < 4096
__constant__ int c_min_rows_per_hist_block = kMinRowsPerHistBlockDefault;
__constant__ int c_max_hist_blocks = kMaxHistBlocks;
// slab stores write through L2 (sc1) so the kernel boundary has less to write back before the
// reduce reads them from the other XCDs (A/B on MI355X: 1.952 -> 1.923 ms/iter); SML_SLAB_WT=0: plain
__constant__ int c_slab_wt = 1;
// SML_PART_WT=1: partition outputs (perm, ordered g/h) written through L2 (A/B: 1.96 -> 1.99 ms/iter, slower)
__constant__ int c_part_wt = 0;
__constant__ int c_part_pipe = 1;  // software-pipelined batched partition (SML_PART_PIPE=0: the plain tile loop)

constexpr int kPartThreads = 512;
constexpr int kMaxPartBlocks = 2048;
constexpr int kPartRowsDefault = 8;  // A/B on MI355X: 8 rows/thread beat 16 and 4 (profiles/README)

struct DLeaf {
  int32_t begin, count, buf, depth;  // local row segment; buf: -1 physical, 0/1 ping-pong
  int64_t gcount;                    // global rows
  double sum_g, sum_h;
  double lo, hi;  // monotone output bounds (basic method)
  int32_t slot, pad;
};

struct DState {
  int32_t num_leaves, done, split_leaf, new_leaf;
  int32_t small_leaf, large_leaf, parent_slot, max_leaves;
  int32_t phase;  // 0 = root, 1 = children
  // segment of the leaf being partitioned and the partition result
  int32_t pbegin, pcount, pbuf, pad;
  // tile cursor of the single-pass partition: left rows claimed so far in the
  // low 32 bits (filled from pbegin upwards), right rows in the high 32 bits
  // (filled from pbegin + pcount downwards). One 64-bit atomic per tile.
  unsigned long long cursor;
};

__device__ __forceinline__ int PTotal(const DState* st) { return static_cast<int>(st->cursor & 0xFFFFFFFFull); }

// Row segment of the leaf whose histogram is built next (root or smaller child).
__device__ __forceinline__ DLeaf HistSeg(const DState* st, const DLeaf* leaves) {
  if (st->phase == 0) return leaves[0];
  DLeaf L;
  const int ob = st->pbuf == 0 ? 1 : 0;
  L.buf = ob;
  const int lt = PTotal(st);
  if (st->small_leaf == st->split_leaf) { L.begin = st->pbegin; L.count = lt; }
  else { L.begin = st->pbegin + lt; L.count = st->pcount - lt; }
  return L;
}

struct DTree {  // device tree arrays (capacity L)
  int32_t* feat;        // L-1
  uint32_t* thr;        // L-1
  int32_t* dleft;       // L-1
  int32_t* is_cat;      // L-1
  uint32_t* cat_bits;   // (L-1)*8
  int32_t* left;        // L-1
  int32_t* right;       // L-1
  double* gain;         // L-1
  double* ival;         // L-1
  double* iweight;      // L-1
  int64_t* icount;      // L-1
  double* lval;         // L
  double* lweight;      // L
  int64_t* lcount;      // L
  int32_t* lparent;     // L
  int32_t* ldepth;      // L
  int4* lseg;           // L (batched growth, may be null): leaf li's node (w) and row segment (begin, count, buffer)
  double out_l1, out_l2, out_mds;  // leaf-output regularisation: the root's value (its internal value once split)
};

// the root's output as a leaf (LeafOutput of the root totals): the internal value node 0 gets when it splits,
// as the host learner (backend_cpu.cpp) sets tree.leaf_value[0] before growing
__device__ __forceinline__ double RootLeafOutput(const DTree& t, double g, double h) {
  return LeafOutput(g, h, t.out_l1, t.out_l2, t.out_mds);
}

struct FeatMeta {
  const int32_t* num_bin;
  const int32_t* missing;
  const int32_t* default_bin;
  const int32_t* is_cat;
  const int8_t* mask;
  const int8_t* mono;  // monotone direction per feature
};

__device__ __forceinline__ bool DeviceGoesLeft(uint32_t b, int nb, int mt, int dbin, int is_cat,
                                               uint32_t thr, int dleft, const uint32_t* cat_bits) {
  if (is_cat) return (cat_bits[b >> 5] >> (b & 31)) & 1u;
  if ((mt == kMissingZero && b == static_cast<uint32_t>(dbin)) ||
      (mt == kMissingNaN && b == static_cast<uint32_t>(nb - 1)))
    return dleft != 0;
  return b <= thr;
}

// Block max of (|g|, h) -> per-block partial (no atomics, no fences: a
// same-address device atomic or an agent-scope fence per block costs tens of
// ns each on this part, serialised); ghmax_final_kernel folds the partials.
__device__ void BlockMaxPartial(float mg, float mh, float* __restrict__ partial) {
  __shared__ float wg[16], wh[16];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) { mg = fmaxf(mg, __shfl_xor(mg, off, 64)); mh = fmaxf(mh, __shfl_xor(mh, off, 64)); }
  if (lane == 0) { wg[wid] = mg; wh[wid] = mh; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < nw; ++w) { mg = fmaxf(mg, wg[w]); mh = fmaxf(mh, wh[w]); }
    partial[2 * blockIdx.x] = mg;
    partial[2 * blockIdx.x + 1] = mh;
  }
}

__global__ __launch_bounds__(1024) void ghmax_final_kernel(const float* __restrict__ partial, int nblocks,
                                                           unsigned int* __restrict__ out_bits) {
  float mg = 0.f, mh = 0.f;
  for (int b = threadIdx.x; b < nblocks; b += blockDim.x) {
    mg = fmaxf(mg, partial[2 * b]);
    mh = fmaxf(mh, partial[2 * b + 1]);
  }
  __shared__ float wg[16], wh[16];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) { mg = fmaxf(mg, __shfl_xor(mg, off, 64)); mh = fmaxf(mh, __shfl_xor(mh, off, 64)); }
  if (lane == 0) { wg[wid] = mg; wh[wid] = mh; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < static_cast<int>(blockDim.x >> 6); ++w) { mg = fmaxf(mg, wg[w]); mh = fmaxf(mh, wh[w]); }
    out_bits[0] = __float_as_uint(mg);
    out_bits[1] = __float_as_uint(mh);
  }
}

// ---------------------------------------------------------------- K2
// Single-output objectives also produce max |g| / max h (the histogram's
// fixed-point scales) so no separate pass over g and h is needed.
__global__ __launch_bounds__(256) void grad_kernel(ObjParams p, const double* __restrict__ score,
                                                   const float* __restrict__ label, const float* __restrict__ weight,
                                                   float* __restrict__ g, float* __restrict__ h, int64_t n,
                                                   float* __restrict__ partial) {
  float mg = 0.f, mh = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double w = weight ? weight[i] : 1.0;
    if (p.kind == kObjMulticlass) {
      const int K = p.num_class;
      double mx = -1e300;
      for (int k = 0; k < K; ++k) mx = fmax(mx, score[k * n + i]);
      double s = 0;
      for (int k = 0; k < K; ++k) s += exp(score[k * n + i] - mx);
      const int y = static_cast<int>(label[i]);
      const double factor = K / (K - 1.0);
      for (int k = 0; k < K; ++k) {
        const double pk = exp(score[k * n + i] - mx) / s;
        g[k * n + i] = static_cast<float>(((k == y) ? pk - 1.0 : pk) * w);
        h[k * n + i] = static_cast<float>(factor * pk * (1.0 - pk) * w);
      }
    } else if (p.kind == kObjMulticlassOVA) {
      for (int k = 0; k < p.num_class; ++k) {
        const double y = static_cast<int>(label[i]) == k ? 1.0 : 0.0;
        PointGradient(p, score[k * n + i], y, w, &g[k * n + i], &h[k * n + i]);
      }
    } else {
      PointGradient(p, score[i], label[i], w, &g[i], &h[i]);
      mg = fmaxf(mg, fabsf(g[i]));
      mh = fmaxf(mh, fabsf(h[i]));
    }
  }
  if (partial) BlockMaxPartial(mg, mh, partial);
}

// ---------------------------------------------------------------- K2 (ranking)
// LambdaRank gradients, one wave64 workgroup per query (grid-stride over
// queries). A document's rank is the number of documents that score higher
// (ties broken by index = the host's stable sort); each lane then owns
// documents and accumulates the lambdas of every pair its document is part of,
// so there are no atomics and the result does not depend on scheduling. Pairs
// are kept exactly as in Objective::LambdarankGradients: different labels and
// min(rank) < max_position. Queries of up to kRankLds documents keep scores,
// labels and ranks in LDS and the lambdas in registers; longer ones stream
// them from global memory (ranks and unnormalised lambdas in scratch).
constexpr int kRankLds = 256;
constexpr int kRankPerLane = kRankLds / 64;

struct RankTables {
  float2* gh2;  // index-only partition: the interleaved (g, h) copy written alongside g / h (nullptr: off)
  const int32_t* qb;
  const double* inv_max_dcg;
  const double* gain;
  const double* disc;  // 1 / log2(2 + r) for r < kRankLds, computed once on the host (std::log2, as the
                       // host objective): each block copies 2 KB instead of evaluating 256 fp64 log2 + div
  int32_t* rank_scratch;
  double* lam_scratch;
  double* hes_scratch;
  const int32_t* order;  // register-path queries, largest first (longest-processing-time order), nreg of them
  int nq, ngain, max_position, norm;
  int gain_mono;  // label gains strictly increasing (the register kernel's kMono form)
  int nreg;
  int prof_phase;  // SML_RANK_PROF_PHASE (timing only, gradients wrong): 1 = identity ranks (no rank count)
  double sigma;
};
constexpr int kGainLds = 64;  // label gains staged in LDS by the register kernel (longer tables: global)

__device__ __forceinline__ double WaveSumD(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ float WaveSumF(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Full-wave sum on the DPP network (no LDS crossbar): xor-1 / xor-2 quad
// permutes, half-row and row mirrors give every row its sum, row_bcast:15 and
// row_bcast:31 fold the rows into lane 63, v_readlane broadcasts it. All 64
// lanes must be active. Measured on the lambdarank register path it was
// slower than WaveSumD (1.62 vs 1.46 ms per gradient call: the 64-bit value
// needs two DPP moves per step plus the readlanes), so it is not used there;
// see profiles/ranker_dpp_wavesum_experiment_r1.patch.
template <int kCtrl, int kRowMask>
__device__ __forceinline__ double DppD(double v) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(x), kCtrl, kRowMask, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(x >> 32), kCtrl, kRowMask, 0xF, false);
  return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}

__device__ __forceinline__ double WaveSumDpp(double v) {
  v += DppD<0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
  v += DppD<0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
  v += DppD<0x141, 0xF>(v);  // row_half_mirror
  v += DppD<0x140, 0xF>(v);  // row_mirror
  v += DppD<0x142, 0xA>(v);  // row_bcast:15 -> rows 1, 3
  v += DppD<0x143, 0xC>(v);  // row_bcast:31 -> rows 2, 3
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane(static_cast<int>(x), 63);
  const int hi = __builtin_amdgcn_readlane(static_cast<int>(x >> 32), 63);
  return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}

// lambda / hessian contribution of the pair (doc i, doc j) to doc i; disc(r)
// = 1/log2(2+r) comes from an LDS table for ranks below kRankLds
__device__ __forceinline__ double Discount(const double* s_disc, int r) {
  return r < kRankLds ? s_disc[r] : 1.0 / log2(2.0 + r);
}

__device__ __forceinline__ void PairLambda(const RankTables& t, const double* s_disc, double si, int li, int ri,
                                           double sj, int lj, int rj, double imd, bool use_norm, double* lam,
                                           double* hes, double* suml) {
  const bool i_high = li > lj;
  const int hr = i_high ? ri : rj, lr = i_high ? rj : ri;
  const unsigned lh = static_cast<unsigned>(i_high ? li : lj), ll = static_cast<unsigned>(i_high ? lj : li);
  const unsigned top = static_cast<unsigned>(t.ngain - 1);
  // The per-pair math runs in fp32 (FP64 divides / exp are ~20x the
  // instruction count and made the kernel FP64-issue bound); the lambdas are
  // accumulated in fp64 and end up as fp32 gradients, like the host path.
  const float gap = static_cast<float>(t.gain[min(lh, top)] - t.gain[min(ll, top)]);
  const float pd = fabsf(static_cast<float>(Discount(s_disc, hr) - Discount(s_disc, lr)));
  const float ds = static_cast<float>(i_high ? si - sj : sj - si);
  const float sig = static_cast<float>(t.sigma);
  float dn = gap * pd * static_cast<float>(imd);
  if (use_norm) dn = __fdividef(dn, 0.01f + fabsf(ds));
  float pl = __frcp_rn(1.0f + __expf(sig * ds));
  float ph = pl * (1.0f - pl);
  pl *= -sig * dn;
  ph *= sig * sig * dn;
  *lam += i_high ? pl : -pl;
  *hes += ph;
  *suml -= pl;  // each pair is visited from both ends: sum = -2 pl per pair
}

// Register-path pair terms (each document's label gain and rank discount looked up once, fp32, so the
// O(pairs) loop is ALU only) for the single visit of a (top, other) pair: c is the
// contribution to doc i's lambda (the partner's is exactly -c: the pair terms are symmetric in the
// two documents and only the sign follows the higher label), ph the hessian term of both, pl the
// term the normaliser sum takes from each end of the pair.
__device__ __forceinline__ void PairTermsPre(float sig, float imd, bool use_norm, double si, int li, float gi, float di,
                                             double sj, int lj, float gj, float dj, float* c, float* ph_out,
                                             float* pl_out) {
  const bool i_high = li > lj;
  const float gap = i_high ? gi - gj : gj - gi;
  const float pd = fabsf(di - dj);
  const float ds = static_cast<float>(i_high ? si - sj : sj - si);
  float dn = gap * pd * imd;
  if (use_norm) dn = __fdividef(dn, 0.01f + fabsf(ds));
  float pl = __frcp_rn(1.0f + __expf(sig * ds));
  float ph = pl * (1.0f - pl);
  pl *= -sig * dn;
  ph *= sig * sig * dn;
  *c = i_high ? pl : -pl;
  *ph_out = ph;
  *pl_out = pl;
}

// The register path's form of PairTermsPre, branch-free: the top document i (wave-uniform si / li / gi /
// di) against this lane's partner j. Both orientations of a difference are exact negations of one another
// (round-to-nearest is sign-symmetric), so ds and gap take one subtraction and a sign flip. No eligibility
// test: a same-label partner (the top document itself included) has gap = 0 and a padding lane imdv = 0,
// so dn = 0 zeroes all three terms (p stays finite for any ds, infinities included), exactly what skipping
// the pair adds to these sums. kMono (label gains strictly increasing - LightGBM's default 2^l - 1 table):
// i is the higher-labelled document iff gi > gj, so the flip is the sign bit of gi - gj and gap its
// magnitude (no label compare / select). The two quotients are hardware reciprocals (v_rcp_f32, 1 ulp)
// instead of IEEE divides (~11 VALU instructions each). sl2e = sigma * log2(e).
template <bool kMono>
__device__ __forceinline__ void PairTermsFast(float sig, float sl2e, float imdv, bool use_norm, double si, int li,
                                              float gi, float di, double sj, int lj, float gj, float dj, float* c,
                                              float* ph_out, float* pl_out) {
  const float dg = gi - gj;
  const unsigned flip = kMono ? (__float_as_uint(dg) & 0x80000000u) : (li > lj ? 0u : 0x80000000u);
  const float ds = __uint_as_float(__float_as_uint(static_cast<float>(si - sj)) ^ flip);
  const float gap = kMono ? fabsf(dg) : __uint_as_float(__float_as_uint(dg) ^ flip);
  const float pd = fabsf(di - dj);
  float dn = gap * pd * imdv;
  if (use_norm) dn *= __builtin_amdgcn_rcpf(0.01f + fabsf(ds));
  const float p = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(sl2e * ds));
  const float pl = p * (-sig * dn);
  *ph_out = p * (1.0f - p) * (sig * sig * dn);
  *pl_out = pl;
  *c = __uint_as_float(__float_as_uint(pl) ^ flip);
}

// All pairs of doc i: a doc ranked below max_position only pairs with the
// top max_position documents (s_top, by rank), a top document with every
// other document.
template <bool kSmall>
__device__ __forceinline__ void DocLambdas(const RankTables& t, const double* s_disc, const int* s_top, int ntop,
                                           const double* sc, const int* labs, const float* __restrict__ label,
                                           const int* rk, int b, int cnt, int i, double imd, bool use_norm,
                                           double* la, double* he, double* suml) {
  const double si = sc[i];
  const int li = kSmall ? labs[i] : static_cast<int>(label[b + i]);
  const int ri = rk[i];
  const bool scan_top = ri >= t.max_position && ntop >= 0;
  const int m = scan_top ? ntop : cnt;
  for (int q = 0; q < m; ++q) {
    const int j = scan_top ? s_top[q] : q;
    const int lj = kSmall ? labs[j] : static_cast<int>(label[b + j]);
    if (lj == li) continue;
    const int rj = rk[j];
    if (min(ri, rj) >= t.max_position) continue;
    PairLambda(t, s_disc, si, li, ri, sc[j], lj, rj, imd, use_norm, la, he, suml);
  }
}

template <bool kSmall>
__device__ void LambdarankQuery(const RankTables& t, int q, const double* __restrict__ score,
                                const float* __restrict__ label, const float* __restrict__ weight,
                                float* __restrict__ g, float* __restrict__ h, double* s_sc, int* s_lab, int* s_rk,
                                const double* s_disc, int* s_top, double* s_tlam, double* s_thes) {
  const int lane = threadIdx.x;
  const int b = t.qb[q], cnt = t.qb[q + 1] - b;
  const double* sc = kSmall ? s_sc : score + b;
  double mx = -INFINITY, mn = INFINITY;
  for (int i = lane; i < cnt; i += 64) {
    const double s = score[b + i];
    if (kSmall) { s_sc[i] = s; s_lab[i] = static_cast<int>(label[b + i]); }
    mx = fmax(mx, s);
    mn = fmin(mn, s);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mx = fmax(mx, __shfl_xor(mx, off, 64));
    mn = fmin(mn, __shfl_xor(mn, off, 64));
  }
  __syncthreads();
  int* rk = kSmall ? s_rk : t.rank_scratch + b;
  // ranks are a permutation of 0..cnt-1; the documents ranked above
  // max_position are listed by rank (s_top) when the list fits in LDS
  const int ntop = t.max_position <= kRankLds ? min(cnt, t.max_position) : -1;
  for (int i = lane; i < cnt; i += 64) {
    const double si = sc[i];
    int r = 0;
    for (int j = 0; j < cnt; ++j) {
      const double sj = sc[j];
      r += (sj > si) || (sj == si && j < i);
    }
    rk[i] = r;
    if (ntop >= 0 && r < ntop) s_top[r] = i;
  }
  __syncthreads();
  const double imd = t.inv_max_dcg[q];
  const bool use_norm = t.norm && mx != mn;
  double lam[kRankPerLane], hes[kRankPerLane];
  double suml = 0.0;
  if (ntop >= 0) {
    // (a) each top document's pairs with every other document: the wave
    //     spreads the partners over its lanes and reduces (no divergence)
    for (int r = 0; r < ntop; ++r) {
      const int i = s_top[r];
      const double si = sc[i];
      const int li = kSmall ? s_lab[i] : static_cast<int>(label[b + i]);
      double la = 0.0, he = 0.0;
      for (int j = lane; j < cnt; j += 64) {
        if (j == i) continue;
        const int lj = kSmall ? s_lab[j] : static_cast<int>(label[b + j]);
        if (lj == li) continue;
        PairLambda(t, s_disc, si, li, r, sc[j], lj, rk[j], imd, use_norm, &la, &he, &suml);
      }
      la = WaveSumD(la);
      he = WaveSumD(he);
      if (lane == 0) { s_tlam[r] = la; s_thes[r] = he; }
    }
    // (b) every other document pairs only with the ntop top documents
    for (int i0 = 0; i0 < cnt; i0 += 64 * kRankPerLane) {
#pragma unroll
      for (int u = 0; u < kRankPerLane; ++u) {
        const int i = i0 + u * 64 + lane;
        double la = 0.0, he = 0.0;
        if (i < cnt && rk[i] >= ntop) {
          const double si = sc[i];
          const int li = kSmall ? s_lab[i] : static_cast<int>(label[b + i]);
          const int ri = rk[i];
          for (int r = 0; r < ntop; ++r) {
            const int j = s_top[r];
            const int lj = kSmall ? s_lab[j] : static_cast<int>(label[b + j]);
            if (lj == li) continue;
            PairLambda(t, s_disc, si, li, ri, sc[j], lj, r, imd, use_norm, &la, &he, &suml);
          }
        }
        if (kSmall) {
          lam[u] = la;
          hes[u] = he;
        } else if (i < cnt) {
          t.lam_scratch[b + i] = la;
          t.hes_scratch[b + i] = he;
        }
      }
    }
    __syncthreads();  // s_tlam / s_thes visible to every lane
  } else {
    // max_position beyond the LDS top list: every document scans all partners
    for (int i0 = 0; i0 < cnt; i0 += 64 * kRankPerLane) {
#pragma unroll
      for (int u = 0; u < kRankPerLane; ++u) {
        const int i = i0 + u * 64 + lane;
        double la = 0.0, he = 0.0;
        if (i < cnt)
          DocLambdas<kSmall>(t, s_disc, s_top, -1, sc, s_lab, label, rk, b, cnt, i, imd, use_norm, &la, &he, &suml);
        if (kSmall) {
          lam[u] = la;
          hes[u] = he;
        } else if (i < cnt) {
          t.lam_scratch[b + i] = la;
          t.hes_scratch[b + i] = he;
        }
      }
    }
  }
  suml = WaveSumD(suml);
  const double nf = (t.norm && suml > 0) ? log2(1.0 + suml) / suml : 1.0;
  if (kSmall) {
#pragma unroll
    for (int u = 0; u < kRankPerLane; ++u) {
      const int i = u * 64 + lane;
      if (i < cnt) {
        const double w = weight ? weight[b + i] : 1.0;
        const int ri = rk[i];
        const bool top = ri < ntop;
        const float gv = static_cast<float>((top ? s_tlam[ri] : lam[u]) * nf * w);
        const float hv = static_cast<float>((top ? s_thes[ri] : hes[u]) * nf * w);
        g[b + i] = gv;
        h[b + i] = hv;
        if (t.gh2) t.gh2[b + i] = make_float2(gv, hv);
      }
    }
  } else {
    for (int i = lane; i < cnt; i += 64) {  // the same lane wrote lam/hes of i above
      const double w = weight ? weight[b + i] : 1.0;
      const int ri = rk[i];
      const bool top = ri < ntop;
      const float gv = static_cast<float>((top ? s_tlam[ri] : t.lam_scratch[b + i]) * nf * w);
      const float hv = static_cast<float>((top ? s_thes[ri] : t.hes_scratch[b + i]) * nf * w);
      g[b + i] = gv;
      h[b + i] = hv;
      if (t.gh2) t.gh2[b + i] = make_float2(gv, hv);
    }
  }
  __syncthreads();  // LDS reuse by the next query
}

__device__ __forceinline__ void WaveSync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ unsigned long long ReadLaneU64(unsigned long long v, int l) {
  const unsigned lo = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(v), l));
  const unsigned hi = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(v >> 32), l));
  return (static_cast<unsigned long long>(hi) << 32) | lo;
}

__device__ __forceinline__ double ReadLaneD(double v, int l) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane(static_cast<int>(x), l);
  const int hi = __builtin_amdgcn_readlane(static_cast<int>(x >> 32), l);
  return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}

// Register-resident form for the common case (<= kRankLds documents and a
// top list of <= 64): lane l owns documents l, l+64, ... (score, label, rank
// in registers); ranks come from comparing against every document broadcast
// with v_readlane (no memory in the O(cnt^2) loop); the top list lives in the
// lanes 0..ntop-1 and is broadcast the same way. Pairs: (a) every top
// document with every document, spread over the lanes and wave-reduced;
// (b) every other document with the top list, one lane per document.
// the top list's per-document values, staged by rank in LDS by their owning lanes (lane r of the wave reads
// rank r's; no second global load of the top documents' scores / labels)
struct RankTop {
  double sc[64];
  float gn[64];
  int lab[64];
};

template <int NU, bool kTR, bool kMono>  // documents per lane: cnt <= 64 * NU; kTR: transpose-reduced top sums
__device__ void LambdarankQueryRegs(const RankTables& t, int q, const double* __restrict__ score,
                                    const float* __restrict__ label, const float* __restrict__ weight,
                                    float* __restrict__ g, float* __restrict__ h, const double* s_disc,
                                    const float* s_gain, int* s_doc_of_rank, RankTop& top) {
  // one wave per query (its own kRankLds-entry rank -> doc map; wave-level syncs only)
  const int lane = threadIdx.x & 63;
  const int b = t.qb[q], cnt = t.qb[q + 1] - b;
  const int ntop = min(cnt, t.max_position);
  double sc[NU];
  int lab[NU], rk[NU];
  double mx = -INFINITY, mn = INFINITY;
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int i = u * 64 + lane;
    sc[u] = i < cnt ? score[b + i] : -INFINITY;
    lab[u] = i < cnt ? static_cast<int>(label[b + i]) : 0;
    rk[u] = 0;
    if (i < cnt) { mx = fmax(mx, sc[u]); mn = fmin(mn, sc[u]); }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mx = fmax(mx, __shfl_xor(mx, off, 64));
    mn = fmin(mn, __shfl_xor(mn, off, 64));
  }
  // ranks: number of documents scoring higher, ties by index (stable sort). First the strict count
  // #{j: sj > si} = #{j: sj >= next_up(si)} - one fp64 compare per pair and no per-partner index test; without
  // ties it IS the stable rank (a permutation), which the wave checks by scattering doc -> rank slot: a
  // shared slot means tied scores (every document of a query ties on the first iteration), and only then
  // the tie-aware count runs: rank(i) = #{j < i: sj >= si} + #{j > i: sj >= next_up(si)} (whether j < i is
  // static for documents in different lane slots (u != v) and jj < lane within one).
  double sup[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) sup[u] = nextafter(sc[u], INFINITY);
  // Partner scores: scalar loads through the constant address space (8 partners per s_load_dwordx16). r5 pass
  // 15 A/B on one box: 635 us per call, v_readlane pairs 727 us, broadcast reads of an LDS copy 635 us.
  const __attribute__((address_space(4))) double* sv =
      (const __attribute__((address_space(4))) double*)(score + b);
  auto count_ranks = [&](bool ties) {
#pragma unroll
    for (int v = 0; v < NU; ++v) {
      if (v * 64 >= cnt) break;
      const int jn = min(64, cnt - v * 64);
      if (!ties) {
        for (int jj = 0; jj < jn; ++jj) {
          const double sj = sv[v * 64 + jj];
#pragma unroll
          for (int u = 0; u < NU; ++u) rk[u] += sj >= sup[u] ? 1 : 0;
        }
      } else {
        for (int jj = 0; jj < jn; ++jj) {
          const double sj = sv[v * 64 + jj];
#pragma unroll
          for (int u = 0; u < NU; ++u) {
            if (u < v) rk[u] += sj >= sup[u] ? 1 : 0;         // every j of slot v is after i
            else if (u > v) rk[u] += sj >= sc[u] ? 1 : 0;     // every j of slot v is before i
            else rk[u] += sj >= (jj < lane ? sc[u] : sup[u]) ? 1 : 0;
          }
        }
      }
    }
  };
  auto scatter = [&]() {  // rank -> doc map (every document's slot)
#pragma unroll
    for (int u = 0; u < NU; ++u)
      if (u * 64 + lane < cnt) s_doc_of_rank[rk[u]] = u * 64 + lane;
    WaveSync();
  };
  if (t.prof_phase == 1) {
#pragma unroll
    for (int u = 0; u < NU; ++u) rk[u] = u * 64 + lane;
  } else {
    count_ranks(false);
  }
  scatter();
  bool clash = false;
#pragma unroll
  for (int u = 0; u < NU; ++u) clash |= u * 64 + lane < cnt && s_doc_of_rank[rk[u]] != u * 64 + lane;
  if (__builtin_amdgcn_ballot_w64(clash)) {  // tied scores: the exact, tie-aware ranks
    WaveSync();                               // every lane has read the map before it is rewritten
#pragma unroll
    for (int u = 0; u < NU; ++u) rk[u] = 0;
    count_ranks(true);
    scatter();
  }
  // per-document label gain (LDS table up to kGainLds labels) and rank discount (ranks < cnt <= kRankLds)
  const unsigned gtop = static_cast<unsigned>(t.ngain - 1);
  const bool gain_lds = t.ngain <= kGainLds;
  float gn[NU], dc[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const bool ok = u * 64 + lane < cnt;
    const unsigned gi = min(static_cast<unsigned>(lab[u]), gtop);
    gn[u] = ok ? (gain_lds ? s_gain[gi] : static_cast<float>(t.gain[gi])) : 0.f;
    dc[u] = ok ? static_cast<float>(s_disc[rk[u]]) : 0.f;
  }
  // top list: lane r holds the document of rank r (ranks are a permutation; the map is already written),
  // its score / label / gain staged by rank by the owning lane
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    if (u * 64 + lane < cnt && rk[u] < ntop) {
      top.sc[rk[u]] = sc[u];
      top.gn[rk[u]] = gn[u];
      top.lab[rk[u]] = lab[u];
    }
  }
  WaveSync();
  double tsc = 0.0;
  int tlab = 0, tdoc = 0;
  float tgn = 0.f;
  if (lane < ntop) {
    tdoc = s_doc_of_rank[lane];
    tsc = top.sc[lane];
    tlab = top.lab[lane];
    tgn = top.gn[lane];
  }
  WaveSync();  // the map and the top slots are read before the next query of this wave rewrites them
  const float tdc = static_cast<float>(s_disc[lane]);  // discount of rank `lane` (valid for lane < ntop)
  const float sig = static_cast<float>(t.sigma);
  const float sl2e = sig * 1.4426950408889634f;
  const float fimd = static_cast<float>(t.inv_max_dcg[q]);
  const bool use_norm = t.norm && mx != mn;
  // fp32 accumulators: a document sums at most max_position + cnt pair terms, each already fp32
  float lam[NU], hes[NU], ntf[NU], imdv[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    lam[u] = 0.f;
    hes[u] = 0.f;
    ntf[u] = u * 64 + lane < cnt && rk[u] >= ntop ? 1.f : 0.f;  // a non-top document mirrors its pair terms
    imdv[u] = u * 64 + lane < cnt ? fimd : 0.f;                  // padding lanes: dn = 0
  }
  float suml = 0.f;
  // Top document r against every document (partners on the lanes), each pair evaluated once: the
  // top document's terms are wave-reduced, a non-top partner (which pairs with the top list only) takes
  // the mirrored terms into its own registers in the same order of r as a separate pass over the top
  // list would (bitwise the same lambdas; that pass was ~18 % of the kernel's VALU work), and the
  // normaliser sum takes such a pair's term from both ends. Grouping four top documents so their wave
  // sums interleave measured no faster (1.44 vs 1.35 ms per call): not shuffle-latency bound.
  float top_la = 0.f, top_he = 0.f;  // lane r keeps the reduced lambdas of top document r
  // this lane's terms of top document r against its partners (and the partners' mirrored terms)
  auto top_terms = [&](int r, float* la_out, float* he_out) {
    const double si = ReadLaneD(tsc, r);
    const int li = kMono ? 0 : __builtin_amdgcn_readlane(tlab, r);
    const float gi = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tgn), r));
    const float dci = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tdc), r));
    float la = 0.f, he = 0.f;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      // branch-free: an ineligible pair adds signed zeros (bitwise a no-op on these sums), a top partner
      // takes no mirrored terms (ntf = 0: fma(-0, c, x) = x)
      float c, ph, pl;
      PairTermsFast<kMono>(sig, sl2e, imdv[u], use_norm, si, li, gi, dci, sc[u], lab[u], gn[u], dc[u], &c, &ph, &pl);
      la += c;
      he += ph;
      suml -= pl;
      lam[u] = fmaf(-ntf[u], c, lam[u]);
      hes[u] = fmaf(ntf[u], ph, hes[u]);
      suml = fmaf(-ntf[u], pl, suml);
    }
    *la_out = la;
    *he_out = he;
  };
  if constexpr (kTR) {
    // Eight top documents per round of cross-lane sums: their 16 partial sums are transpose-reduced (each
    // xor step keeps half of the values, 8 + 4 + 2 + 1 + 1 + 1 = 17 shuffles instead of 16 x 6). The shuffles
    // are ds_bpermute through the CU's one LDS pipe, which the 12 per top document saturated (4-wave blocks
    // measured slower, not faster). Same xor pairing as WaveSumF: every sum is bitwise the same.
    for (int r0 = 0; r0 < ntop; r0 += 8) {
      float v[16];
#pragma unroll
      for (int rr = 0; rr < 8; ++rr) {
        v[rr] = 0.f;
        v[8 + rr] = 0.f;
        if (r0 + rr < ntop) top_terms(r0 + rr, &v[rr], &v[8 + rr]);
      }
      const bool b5 = lane & 32, b4 = lane & 16, b3 = lane & 8, b2 = lane & 4;
      float a8[8], a4[4], a2[2];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float mine = b5 ? v[8 + k] : v[k], oth = b5 ? v[k] : v[8 + k];
        a8[k] = mine + __shfl_xor(oth, 32, 64);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float mine = b4 ? a8[4 + k] : a8[k], oth = b4 ? a8[k] : a8[4 + k];
        a4[k] = mine + __shfl_xor(oth, 16, 64);
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const float mine = b3 ? a4[2 + k] : a4[k], oth = b3 ? a4[k] : a4[2 + k];
        a2[k] = mine + __shfl_xor(oth, 8, 64);
      }
      float a1 = (b2 ? a2[1] : a2[0]) + __shfl_xor(b2 ? a2[0] : a2[1], 4, 64);
      a1 += __shfl_xor(a1, 2, 64);
      a1 += __shfl_xor(a1, 1, 64);
      // lane l now holds value (l >> 2): la of top document r0 + i at lane 4i, he at lane 32 + 4i
      const int rr = lane - r0;
      const float tla = __shfl(a1, (rr & 7) * 4, 64), the = __shfl(a1, 32 + (rr & 7) * 4, 64);
      if (rr >= 0 && rr < 8) { top_la = tla; top_he = the; }
    }
  } else {
    for (int r = 0; r < ntop; ++r) {
      float la, he;
      top_terms(r, &la, &he);
      la = WaveSumF(la);
      he = WaveSumF(he);
      if (lane == r) { top_la = la; top_he = he; }
    }
  }
  const double sumd = WaveSumF(suml);
  const double nf = (t.norm && sumd > 0) ? log2(1.0 + sumd) / sumd : 1.0;
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int i = u * 64 + lane;
    if (i < cnt && rk[u] >= ntop) {
      const double w = weight ? weight[b + i] : 1.0;
      const float gv = static_cast<float>(lam[u] * nf * w), hv = static_cast<float>(hes[u] * nf * w);
      g[b + i] = gv;
      h[b + i] = hv;
      if (t.gh2) t.gh2[b + i] = make_float2(gv, hv);
    }
  }
  if (lane < ntop) {
    const double w = weight ? weight[b + tdoc] : 1.0;
    const float gv = static_cast<float>(top_la * nf * w), hv = static_cast<float>(top_he * nf * w);
    g[b + tdoc] = gv;
    h[b + tdoc] = hv;
    if (t.gh2) t.gh2[b + tdoc] = make_float2(gv, hv);
  }
}

__device__ __forceinline__ bool RegsEligible(const RankTables& t, int cnt) {
  return cnt <= kRankLds && t.max_position <= 64;
}

// The common case on its own kernel: its LDS is the discount table and one 64-entry rank->doc map per
// wave (2 KB + 256 B per wave instead of the LDS path's 11.5 KB). kWaves independent waves per block, each
// walking its own queries (a CU holds at most 16 workgroups, so one-wave blocks cap residency at 4 waves
// per SIMD; kWaves = 4 lifts that, but measured slower - see rank_waves_).
// kSmall: the queries of <= 128 documents only (NU 1 / 2): without the NU 3 / 4 code paths the kernel needs
// fewer VGPRs, so more waves per SIMD hide the per-query latency chains; the host launches the > 128-document
// queries (the front of the largest-first order) on a kSmall = false launch first. [k0, k1) = the launch's
// slice of t.order.
template <int kWaves, bool kTR = true, bool kMono = true, bool kSmall = false>
__global__ __launch_bounds__(64 * kWaves, kSmall ? 5 : 4) void lambdarank_regs_kernel(
    RankTables t, const double* __restrict__ score, const float* __restrict__ label, const float* __restrict__ weight,
    float* __restrict__ g, float* __restrict__ h, int k0, int k1) {
  __shared__ double s_disc[kRankLds];
  __shared__ float s_gain[kGainLds];
  __shared__ int s_map[kWaves][kRankLds];
  __shared__ RankTop s_top[kWaves];
  for (int r = threadIdx.x; r < kRankLds; r += 64 * kWaves) s_disc[r] = t.disc[r];
  for (int r = threadIdx.x; r < kGainLds; r += 64 * kWaves) s_gain[r] = r < t.ngain ? static_cast<float>(t.gain[r]) : 0.f;
  __syncthreads();
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform to the compiler: q, b, cnt in SGPRs
  // documents per lane sized to the query: the pair loops run NU-wide, so a 100-document query
  // costs half of what the kRankLds-wide form would
  for (int k = k0 + blockIdx.x * kWaves + wid; k < k1; k += gridDim.x * kWaves) {
    const int q = t.order[k];
    const int cnt = t.qb[q + 1] - t.qb[q];
    if (cnt <= 0 || !RegsEligible(t, cnt)) continue;
    if (cnt <= 64) LambdarankQueryRegs<1, kTR, kMono>(t, q, score, label, weight, g, h, s_disc, s_gain, s_map[wid], s_top[wid]);
    else if (cnt <= 128) LambdarankQueryRegs<2, kTR, kMono>(t, q, score, label, weight, g, h, s_disc, s_gain, s_map[wid], s_top[wid]);
    else if constexpr (!kSmall) {
      if (cnt <= 192) LambdarankQueryRegs<3, kTR, kMono>(t, q, score, label, weight, g, h, s_disc, s_gain, s_map[wid], s_top[wid]);
      else LambdarankQueryRegs<kRankPerLane, kTR, kMono>(t, q, score, label, weight, g, h, s_disc, s_gain, s_map[wid], s_top[wid]);
    }
  }
}

__global__ __launch_bounds__(64) void lambdarank_kernel(RankTables t, const double* __restrict__ score,
                                                        const float* __restrict__ label,
                                                        const float* __restrict__ weight, float* __restrict__ g,
                                                        float* __restrict__ h) {
  __shared__ double s_sc[kRankLds];
  __shared__ double s_disc[kRankLds];
  __shared__ int s_lab[kRankLds];
  __shared__ int s_rk[kRankLds];
  __shared__ int s_top[kRankLds];
  __shared__ double s_tlam[kRankLds], s_thes[kRankLds];
  for (int r = threadIdx.x; r < kRankLds; r += 64) s_disc[r] = t.disc[r];
  __syncthreads();
  for (int q = blockIdx.x; q < t.nq; q += gridDim.x) {
    const int cnt = t.qb[q + 1] - t.qb[q];
    if (cnt <= 0 || RegsEligible(t, cnt)) continue;  // handled by lambdarank_regs_kernel
    if (cnt <= kRankLds) LambdarankQuery<true>(t, q, score, label, weight, g, h, s_sc, s_lab, s_rk, s_disc, s_top, s_tlam, s_thes);
    else LambdarankQuery<false>(t, q, score, label, weight, g, h, s_sc, s_lab, s_rk, s_disc, s_top, s_tlam, s_thes);
  }
}

// ---------------------------------------------------------------- K8
// Bagging / GOSS on the device. GOSS needs the top_k-th largest |g*h|: an
// exact 4-pass MSB radix select over the float bit patterns (non-negative
// floats order like their bits), one 256-bin LDS histogram per pass, the pick
// done by one thread, so the threshold never leaves the device. The sampling
// pass draws RowUniform (sampling.h, same value as the host), rescales the
// sampled small-gradient rows and compacts the kept rows with wave ballots and
// one atomic per block; the bag's row order is irrelevant (histogram sums are
// exact integers, K3).
struct SelectState {
  uint32_t prefix, mask;
  long long k;  // 1-based rank of the wanted key among keys matching prefix
  int count;    // rows kept by the sampling pass
  int pad;
};

__global__ __launch_bounds__(256) void goss_key_kernel(const float* __restrict__ g, const float* __restrict__ h,
                                                       int64_t n, int K, uint32_t* __restrict__ key) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < K; ++k) s += fabsf(g[k * n + i] * h[k * n + i]);
    key[i] = __float_as_uint(s);
  }
}

__global__ void select_init_kernel(SelectState* st, long long k) {
  if (threadIdx.x == 0) { st->prefix = 0u; st->mask = 0u; st->k = k; st->count = 0; }
}

__global__ __launch_bounds__(256) void radix_hist_kernel(const uint32_t* __restrict__ key, int64_t n,
                                                         const SelectState* __restrict__ st, int shift,
                                                         unsigned int* __restrict__ hist) {
  __shared__ unsigned int lh[256];
  lh[threadIdx.x] = 0u;
  __syncthreads();
  const uint32_t prefix = st->prefix, mask = st->mask;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t v = key[i];
    if ((v & mask) == prefix) atomicAdd(&lh[(v >> shift) & 255u], 1u);
  }
  __syncthreads();
  if (lh[threadIdx.x]) atomicAdd(&hist[threadIdx.x], lh[threadIdx.x]);
}

__global__ void radix_pick_kernel(SelectState* st, unsigned int* __restrict__ hist, int shift) {
  if (threadIdx.x != 0) return;
  long long cum = 0;
  const long long k = st->k;
  for (int d = 255; d >= 0; --d) {
    const long long c = hist[d];
    if (cum + c >= k) {
      st->prefix |= static_cast<uint32_t>(d) << shift;
      st->mask |= 255u << shift;
      st->k = k - cum;
      break;
    }
    cum += c;
  }
  for (int d = 0; d < 256; ++d) hist[d] = 0u;  // ready for the next pass
}

__global__ __launch_bounds__(256) void sample_kernel(RowSampleSpec sp, int64_t n, int K,
                                                     const uint32_t* __restrict__ key,
                                                     SelectState* __restrict__ st, const float* __restrict__ label,
                                                     float* __restrict__ g, float* __restrict__ h,
                                                     int32_t* __restrict__ bag) {
  __shared__ int wcnt[4];
  __shared__ int base;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t thr = sp.kind == kSampleGoss ? st->prefix : 0u;
  const float mult = static_cast<float>(sp.other_mult);
  const unsigned long long below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x; i0 < n; i0 += stride) {
    const int64_t i = i0 + threadIdx.x;
    bool keep = false;
    if (i < n) {
      if (sp.kind == kSampleBagging) {
        const double frac = sp.balanced ? (label[i] > 0 ? sp.pos_fraction : sp.neg_fraction) : sp.fraction;
        keep = RowUniform(sp.seed, sp.iter, i) < frac;
      } else if (key[i] >= thr) {
        keep = true;
      } else if (RowUniform(sp.seed, sp.iter, i) < sp.other_prob) {
        keep = true;
        for (int k = 0; k < K; ++k) { g[k * n + i] *= mult; h[k * n + i] *= mult; }
      }
    }
    const unsigned long long bl = __ballot(keep);
    if (lane == 0) wcnt[wid] = __popcll(bl);
    __syncthreads();
    if (threadIdx.x == 0) base = atomicAdd(&st->count, wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3]);
    __syncthreads();
    if (keep) {
      int off = base + __popcll(bl & below);
      for (int w = 0; w < wid; ++w) off += wcnt[w];
      bag[off] = static_cast<int32_t>(i);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- root init
// nparts > 0: also fold the per-block max |g| / max h partials of the pass that
// produced this tree's gradients into ghmax (what ghmax_final_kernel does, one
// launch fewer per tree).
__global__ __launch_bounds__(64) void root_init_kernel(DState* st, DLeaf* leaves, int32_t count, int buf,
                                                       int max_leaves, const float* __restrict__ partial, int nparts,
                                                       unsigned int* __restrict__ ghmax) {
  if (nparts > 0) {
    float mg = 0.f, mh = 0.f;
    for (int b = threadIdx.x; b < nparts; b += 64) {
      mg = fmaxf(mg, partial[2 * b]);
      mh = fmaxf(mh, partial[2 * b + 1]);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) { mg = fmaxf(mg, __shfl_xor(mg, off, 64)); mh = fmaxf(mh, __shfl_xor(mh, off, 64)); }
    if (threadIdx.x == 0) { ghmax[0] = __float_as_uint(mg); ghmax[1] = __float_as_uint(mh); }
  }
  if (threadIdx.x == 0) {
    st->num_leaves = 1; st->done = 0; st->split_leaf = 0; st->new_leaf = -1;
    st->small_leaf = 0; st->large_leaf = -1; st->parent_slot = -1; st->max_leaves = max_leaves;
    st->phase = 0; st->cursor = 0ull;
    DLeaf l{};
    l.begin = 0; l.count = count; l.buf = buf; l.depth = 0; l.gcount = count; l.slot = 0;
    l.lo = -INFINITY; l.hi = INFINITY;
    leaves[0] = l;
  }
}

__global__ void gather_bag_kernel(const int32_t* __restrict__ rows, int32_t n, const float* __restrict__ g,
                                  const float* __restrict__ h, int32_t* __restrict__ perm,
                                  float2* __restrict__ ogh) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    int r = rows[i];
    perm[i] = r;
    ogh[i] = make_float2(g[r], h[r]);
  }
}

// ---------------------------------------------------------------- K3
// One block = one contiguous chunk of the leaf's row segment x one group of 32
// features. A thread owns whole rows: the 32 bins of its feature group are two
// dwordx4 loads (rows are padded to 16 B), the gradient pair one float2 load
// from the ordered copy (or the physical arrays for an unpartitioned root).
// kHistUnroll rows are fetched before any is accumulated so every wave keeps
// several gathers in flight (the loop is latency-bound otherwise).
//
// Accumulation is 64-bit fixed point with g and h in separate LDS words: two
// ds_add_u64 per (row, feature) into 2 x 256 x 32 words (128 KB, one
// 1024-thread block per CU). Both scales are powers of two chosen per
// histogram from the leaf's row count and the tree's max |g| / max h so that
// the sum over ALL of the leaf's rows stays below 2^62 in magnitude: every
// per-block sum and the exact int64 cross-block reduction fit, the histogram
// is bitwise independent of row order and of the block decomposition, and the
// conversion back (x 2^-k) is exact up to one final int64 -> double rounding.
// Precision: one row's quantum is <= count * max / 2^61, i.e. <= 2^-37.6 of
// max |g| for the 11M-row root and <= 2^-50 for leaves under 2k rows; a bin of
// k rows carries ~sqrt(k) * quantum / 3.5 of rounding error - at or below the
// rounding of LightGBM's fp64 accumulation of fp32 gradients (~k * 2^-53 of
// the bin's sum) on populated bins. (Round 1-2 packed g | h as two 32-bit
// halves of one word: ~1e-5 of max |g| at the root; A/B in profiles/README.)
// A/B: 2 rows in flight per thread beat 4 and 8 (one 1024-thread block per CU: 1.93 / 1.97 / 2.04
// ms/iter; more rows in flight only queue more LDS atomics)
constexpr int kHistUnroll = 2;
constexpr int kHistBlockThreads = 1024;
constexpr int kHistWords = kFeatPerGroup * kBinsPerFeature;  // per plane (g or h), bin-major

__device__ __forceinline__ int HistBlocks(int count) {
  return max(1, min(c_max_hist_blocks, ceil_div_i(count, c_min_rows_per_hist_block)));
}

struct HScale {
  double g, h;    // 2^eg, 2^eh: quantisation scales
  double ig, ih;  // 2^-eg, 2^-eh: conversion back
};

// The fixed-point scale of every histogram of a tree is a function of GLOBAL quantities only: the bound
// `scale_n` = the training set's global row count (>= any leaf's global count, so every sum of the tree fits
// 2^62) and the global max |g| / max h (or the objective's a-priori bound). It does not depend on how the
// rows are spread over ranks, so per-rank int64 histograms summed over ranks are bitwise the 1-rank
// histogram: an N-rank model is the 1-rank model (VerifyLightGBMClassifierStream.scala:95-101).
__device__ __forceinline__ int ScaleExp(int64_t count, float vmax) {
  // largest e with count * vmax * 2^e <= 2^62
  const double r = 4.611686018427387904e18 / (static_cast<double>(max(int64_t{1}, count)) * fmax(static_cast<double>(vmax), 1e-300));
  return max(-1000, min(1000, ilogb(r)));
}

__device__ __forceinline__ HScale HistScaleV(int64_t scale_n, float gmax, float hmax) {
  const int eg = ScaleExp(scale_n, gmax), eh = ScaleExp(scale_n, hmax);
  return HScale{ldexp(1.0, eg), ldexp(1.0, eh), ldexp(1.0, -eg), ldexp(1.0, -eh)};
}

__device__ __forceinline__ HScale HistScale(int64_t scale_n, const float* ghmax) {
  return HistScaleV(scale_n, ghmax[0], ghmax[1]);
}

struct QGH {
  unsigned long long g, h;  // g two's complement (wraps exactly in unsigned adds)
};

__device__ __forceinline__ QGH QuantGH(float2 v, const HScale& s) {
  const long long gq = static_cast<long long>(__builtin_rint(static_cast<double>(v.x) * s.g));
  const unsigned long long hq =
      static_cast<unsigned long long>(__builtin_rint(static_cast<double>(fmaxf(v.y, 0.f)) * s.h));
  return QGH{static_cast<unsigned long long>(gq), hq};
}

// LDS histogram layout: bin-major, sh[b * kFPG + f] (kFPG = 16 or 32 feature slots per bin). A 64-bit LDS
// atomic is serviced in 4 groups of 16 contiguous lanes over 32 banks (an 8-B slot's bank pair = slot mod 16),
// so slot mod 16 = f mod 16 whatever the bin. Lane l walks its row's S features rotated by l & 15 (step j:
// feature (j + (l & 15)) mod S; 16 consecutive integers have distinct residues mod 16), so the 16 lanes of
// a group always add into 16 different bank pairs: conflict-free. (The round-1/2 [f][257] layout put the
// random bins of one feature on random bank pairs: ~3.5-way conflicts, 65 % of the LDS cycles in the PMC
// pass of profiles/r2_pmc.) The row is rotated once in registers (two dword-rotation selects + alignbyte),
// so every step extracts a fixed byte. Slots f >= Fg of a partial group collect the row's padding bytes
// (always < 256) and are never read.
// All-ones when bit `B` of x is set, else 0 (v_bfe_i32 x, B, 1). Kept opaque to the optimiser on purpose: a
// plain `cond ? a : b` over the row's dwords was turned into a dynamically indexed select - a 7-deep
// v_cmp / v_cndmask / s_nop chain per dword (~170 VALU per row in the root pass's ISA); with an opaque mask
// each select is one v_bfi_b32.
template <int B>
__device__ __forceinline__ uint32_t BitMask(uint32_t x) {
  uint32_t m;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(m) : "v"(x), "i"(B));
  return m;
}

__device__ __forceinline__ uint32_t SelBits(uint32_t m, uint32_t a, uint32_t b) { return (a & m) | (b & ~m); }

// The row rotated by `rot` bytes (0..S-1 lanes' residues): r byte j = row byte (j + rot) mod S, S = 4 * NW
template <int NW>
__device__ __forceinline__ void RotateRow(const uint4& b0, const uint4& b1, uint32_t rot, uint32_t* r) {
  const uint32_t w[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
  const uint32_t m1 = BitMask<2>(rot), m2 = BitMask<3>(rot);
  uint32_t v[NW], u[NW];
#pragma unroll
  for (int k = 0; k < NW; ++k) v[k] = SelBits(m1, w[(k + 1) % NW], w[k]);
#pragma unroll
  for (int k = 0; k < NW; ++k) u[k] = SelBits(m2, v[(k + 2) % NW], v[k]);
#pragma unroll
  for (int k = 0; k < NW; ++k) r[k] = __builtin_amdgcn_alignbyte(u[(k + 1) % NW], u[k], rot & 3u);
}

// Per-thread table for the 32-slot bin-major histogram (kFPG = 32, 8-B slots: byte address of slot (b, f) =
// b * 256 + f * 8): byte k of fo[q] = 8 * ((4q + k + rot) mod 32), the slot offset of step j = 4q + k. One
// v_perm_b32 per step then builds the LDS byte address from it and the rotated row's byte:
// perm(fo[q], r[q], 0x0C0C'k'(4+k)) = (row byte << 8) | fo byte.
__device__ __forceinline__ void SlotOffsets32(uint32_t rot, uint32_t* fo) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) x |= (((4u * q + k + rot) & 31u) * 8u) << (8 * k);
    fo[q] = x;
  }
}

// h plane base (bytes from the g plane) when every real feature of the group is below slot 28: the g plane's
// slots (bin 255, f 28..31) then coincide with the h plane's (bin 0, f 0..3) and are never written (padding
// bytes are 0, so padding slots only ever receive bin 0) nor read - and the h atomic's address fits the DS
// instruction's 16-bit offset (no add per step). Otherwise the planes are 64 KiB apart.
constexpr uint32_t kHPlaneTight = 65536u - 32u;
constexpr uint32_t kHPlaneApart = 65536u;

template <int S, int kFPG, uint32_t kHOff = kHPlaneApart>
__device__ __forceinline__ void hist_accumulate_rot(unsigned long long* shg, unsigned long long* shh,
                                                    const uint4& b0, const uint4& b1, const QGH& q, int rot,
                                                    const uint32_t* fo = nullptr) {
  static_assert(S == 16 || S == 32, "16 or 32 features per rotated row");
  static_assert(kFPG % 16 == 0 && S <= kFPG, "slots per bin");
  constexpr int NW = S / 4;
  uint32_t r[NW];
  RotateRow<NW>(b0, b1, static_cast<uint32_t>(rot), r);
  if constexpr (S == 32 && kFPG == 32) {
    // shg / shh are kHOff bytes apart (caller's layout); one perm per step gives the slot's byte address
    char* base = reinterpret_cast<char*>(shg);
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const uint32_t sel = 0x0C0C0000u | ((j & 3u) << 8) | (4u + (j & 3u));
      const uint32_t a = __builtin_amdgcn_perm(fo[j >> 2], r[j >> 2], sel);
      atomicAdd(reinterpret_cast<unsigned long long*>(base + a), q.g);
      atomicAdd(reinterpret_cast<unsigned long long*>(base + a + kHOff), q.h);
    }
  } else {
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const int f = (j + rot) & (S - 1);
      const int i = static_cast<int>((r[j >> 2] >> (8 * (j & 3))) & 255u) * kFPG + f;
      atomicAdd(&shg[i], q.g);
      atomicAdd(&shh[i], q.h);
    }
  }
}

// one slab element: (g, h) int64 pair; write-through (agent-scope relaxed stores = sc1) when c_slab_wt
__device__ __forceinline__ void SlabStore(ulonglong2* p, unsigned long long g, unsigned long long h) {
  if (c_slab_wt) {
    unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
    __hip_atomic_store(q, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 1, h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    *p = make_ulonglong2(g, h);
  }
}

// Block slab, bin-major over ALL features: element b * F + f (the LDS order of each group, so the copy
// reads LDS conflict-free and writes runs of Fg contiguous elements); hist_reduce_kernel transposes to the
// [f][b] histogram while summing.
template <int kFPG, int kThr>
__device__ __forceinline__ void SlabWrite(ulonglong2* out, const unsigned long long* shg, const unsigned long long* shh,
                                          int F, int f0, int Fg, int tid) {
  for (int i = tid; i < kFPG * kBinsPerFeature; i += kThr) {
    const int b = i / kFPG, fl = i % kFPG;
    if (fl < Fg) SlabStore(out + b * F + f0 + fl, shg[i], shh[i]);
  }
}

// One block's share of a leaf histogram: rows [begin, begin + count) of ping-pong buffer `buf` (-1 =
// physical rows) are cut into nb_active chunks; this block (chunk lb, feature group blockIdx.y) accumulates
// its chunk into LDS and writes its slab.
// kGH2: the index-only partition - the segment holds row ids only and each row's (g, h) is gathered from the
// interleaved physical copy `g` points to (float2 per row)
template <int kUnroll, int kFPG, bool kPipe = false, bool kTight = false, bool kGH2 = false>
__device__ __forceinline__ void HistBody(int begin, int count, int buf, int nb_active, int lb, const uint4* __restrict__ bins4,
                                         int W4, int F, const int32_t* __restrict__ perm0,
                                         const int32_t* __restrict__ perm1, const float2* __restrict__ ogh0,
                                         const float2* __restrict__ ogh1, const float* __restrict__ g,
                                         const float* __restrict__ h, const float* __restrict__ ghmax,
                                         ulonglong2* __restrict__ slab_out, int64_t scale_n) {
  constexpr int kWords = kFPG * kBinsPerFeature;
  // g plane at 0, h plane kHOff bytes above it (kTight: F <= 28, see kHPlaneTight)
  constexpr uint32_t kHOff = kFPG == 32 ? (kTight ? kHPlaneTight : kHPlaneApart) : kWords * 8u;
  constexpr int kShWords = static_cast<int>(kHOff / 8) + kWords;
  __shared__ unsigned long long sh[kShWords];
  unsigned long long* shg = sh;
  unsigned long long* shh = sh + kHOff / 8;
  const int tid = threadIdx.x;
  // the fixed-point scale's inputs load while the LDS histogram is zeroed (not after the barrier)
  const float gmax_g = ghmax[0], gmax_h = ghmax[1];
  for (int i = tid; i < kShWords; i += kHistBlockThreads) sh[i] = 0ull;
  uint32_t fo[8];
  if constexpr (kFPG == 32) SlotOffsets32(static_cast<uint32_t>(tid & 15), fo);
  __syncthreads();
  const int grp = blockIdx.y;
  const int Fg = min(kFPG, F - grp * kFPG);
  const int col = grp * (kFPG / 16);  // first uint4 of this group in a row
  const bool two = kFPG > 16 && Fg > 16;
  const int chunk = ceil_div_i(count, nb_active);
  const int p0 = begin + lb * chunk;
  const int p1 = min(begin + count, p0 + chunk);
  const HScale sc = HistScaleV(scale_n, gmax_g, gmax_h);
  const int32_t* __restrict__ perm = buf == 0 ? perm0 : perm1;
  const float2* __restrict__ ogh = buf == 0 ? ogh0 : ogh1;
  const float2* __restrict__ gh2 = reinterpret_cast<const float2*>(g);
  const bool phys = buf < 0;
  const int rot = tid & 15;
  static_assert(!(kPipe && kGH2), "the pipelined loop reads the ordered g / h copy");
  if constexpr (kPipe) {
    // Software pipeline, two stages deep: while the rows of step i go into the LDS histogram, the bins /
    // (g, h) of step i + 1 and the row ids of step i + 2 are in flight, so a wave's memory latency hides
    // behind its own atomics instead of only behind the other 15 waves' (the plain loop issues the next
    // loads only after the atomics). Positions past p1 load row 0 / position p0 and are never accumulated.
    constexpr int kStep = kHistBlockThreads * kUnroll;
    auto rows_at = [&](int base, int* r) {
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int pos = base + u * kHistBlockThreads;
        r[u] = pos < p1 ? (phys ? pos : perm[pos]) : 0;
      }
    };
    auto data_at = [&](int base, const int* r, uint4* b0, uint4* b1, float2* v) {
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int pos = base + u * kHistBlockThreads;
        const size_t rb = static_cast<size_t>(r[u]) * W4 + col;
        b0[u] = bins4[rb];
        b1[u] = two ? bins4[rb + 1] : make_uint4(0, 0, 0, 0);
        v[u] = phys ? make_float2(g[r[u]], h[r[u]]) : (pos < p1 ? ogh[pos] : make_float2(0.f, 0.f));
      }
    };
    int r1[kUnroll], r2[kUnroll];
    uint4 b0[kUnroll], b1[kUnroll];
    float2 v[kUnroll];
    int base = p0 + tid;
    rows_at(base, r1);
    data_at(base, r1, b0, b1, v);
    rows_at(base + kStep, r1);
    for (; base < p1; base += kStep) {
      rows_at(base + 2 * kStep, r2);
      uint4 n0[kUnroll], n1[kUnroll];
      float2 nv[kUnroll];
      data_at(base + kStep, r1, n0, n1, nv);
#pragma unroll
      for (int u = 0; u < kUnroll; ++u)
        if (base + u * kHistBlockThreads < p1) {
          if (kFPG > 16 && two) hist_accumulate_rot<(kFPG > 16 ? 32 : 16), kFPG, kHOff>(shg, shh, b0[u], b1[u], QuantGH(v[u], sc), rot, fo);
          else hist_accumulate_rot<16, kFPG>(shg, shh, b0[u], b1[u], QuantGH(v[u], sc), rot);
        }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) { b0[u] = n0[u]; b1[u] = n1[u]; v[u] = nv[u]; r1[u] = r2[u]; }
    }
    __syncthreads();
    SlabWrite<kFPG, kHistBlockThreads>(slab_out, shg, shh, F, grp * kFPG, Fg, tid);
    return;
  }
  for (int base = p0 + tid; base < p1; base += kHistBlockThreads * kUnroll) {
    // branch-free loads (positions past p1 read position p0, a valid row, and are never accumulated): a
    // guarded load is a branch, and the compiler waits out each one before the next row's
    int r[kUnroll], pq[kUnroll];
    bool ok[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int pos = base + u * kHistBlockThreads;
      ok[u] = pos < p1;
      pq[u] = ok[u] ? pos : p0;
      r[u] = phys ? pq[u] : perm[pq[u]];
    }
    uint4 b0[kUnroll], b1[kUnroll];
    float2 v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const size_t rb = static_cast<size_t>(r[u]) * W4 + col;
      b0[u] = bins4[rb];
      b1[u] = bins4[two ? rb + 1 : rb];
      if (!two) b1[u] = make_uint4(0, 0, 0, 0);
      v[u] = kGH2 ? gh2[r[u]] : (phys ? make_float2(g[r[u]], h[r[u]]) : ogh[pq[u]]);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u)
      if (ok[u]) {
        if (kFPG > 16 && two) hist_accumulate_rot<(kFPG > 16 ? 32 : 16), kFPG, kHOff>(shg, shh, b0[u], b1[u], QuantGH(v[u], sc), rot, fo);
        else hist_accumulate_rot<16, kFPG>(shg, shh, b0[u], b1[u], QuantGH(v[u], sc), rot);
      }
  }
  __syncthreads();
  SlabWrite<kFPG, kHistBlockThreads>(slab_out, shg, shh, F, grp * kFPG, Fg, tid);
}

// kFPG features per block (blockIdx.y = feature group): 32 = one 128 KB LDS histogram per CU; 16 halves
// the LDS (two blocks per CU) at the price of reading every row's perm / g / h once per group
template <int kUnroll, int kFPG, bool kPipe = false, bool kTight = false>
__global__ __launch_bounds__(kHistBlockThreads) void hist_kernel(
    const DState* __restrict__ st, const DLeaf* __restrict__ leaves, const uint4* __restrict__ bins4,
    int W4, int F, const int32_t* __restrict__ perm0, const int32_t* __restrict__ perm1,
    const float2* __restrict__ ogh0, const float2* __restrict__ ogh1, const float* __restrict__ g,
    const float* __restrict__ h, const float* __restrict__ ghmax, ulonglong2* __restrict__ slab, int64_t scale_n) {
  if (st->done) return;
  const DLeaf L = HistSeg(st, leaves);
  const int nb_active = HistBlocks(L.count);
  if (static_cast<int>(blockIdx.x) >= nb_active) return;
  HistBody<kUnroll, kFPG, kPipe, kTight>(L.begin, L.count, L.buf, nb_active, blockIdx.x, bins4, W4, F, perm0, perm1, ogh0, ogh1, g, h,
                          ghmax, slab + static_cast<size_t>(blockIdx.x) * F * kBinsPerFeature, scale_n);
}

// max |g|, max h of one class when the gradients did not come from grad_kernel
// (multiclass, host-provided, GOSS-rescaled).
constexpr int kGhmaxBlocks = 1024;

__global__ __launch_bounds__(256) void ghmax_kernel(const float* __restrict__ g, const float* __restrict__ h, int64_t n,
                                                    float* __restrict__ partial) {
  float mg = 0.f, mh = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    mg = fmaxf(mg, fabsf(g[i]));
    mh = fmaxf(mh, fabsf(h[i]));
  }
  BlockMaxPartial(mg, mh, partial);
}

// Exact reduction of the per-block integer slabs: block = 16 groups x 32
// elements; group y sums blocks y, y+16, ... in int64, the 16 partials are
// added in LDS and converted once with the histogram's scale. hist[E] (the
// slot after the histogram) carries the leaf's local row count so one
// data-parallel allreduce of 2E+2 doubles also yields the global count.
constexpr int kRedE = 32;
constexpr int kRedG = 16;

// i64_out (data-parallel): the int64 sums and the row count are written as int64 for the exact cross-rank
// allreduce; hist_convert_kernel then turns them into the fp64 histogram exactly as the 1-rank path does here.
__global__ __launch_bounds__(kRedE * kRedG) void hist_reduce_kernel(
    const DState* __restrict__ st, const DLeaf* __restrict__ leaves, const ulonglong2* __restrict__ slab, int E,
    const float* __restrict__ ghmax, double2* __restrict__ hist, int64_t scale_n, int i64_out) {
  if (st->done) return;
  const int count = HistSeg(st, leaves).count;
  const int nb_active = HistBlocks(count);
  const int tid = threadIdx.x, le = tid % kRedE, grp = tid / kRedE;
  const int e = blockIdx.x * kRedE + le;
  const bool valid = e < E;
  unsigned long long sg = 0, sh = 0;
  if (valid) {
#pragma unroll 8
    for (int b = grp; b < nb_active; b += kRedG) {
      const ulonglong2 v = slab[static_cast<size_t>(b) * E + e];
      sg += v.x;
      sh += v.y;
    }
  }
  __shared__ unsigned long long rg[kRedG][kRedE], rh[kRedG][kRedE];
  rg[grp][le] = sg;
  rh[grp][le] = sh;
  __syncthreads();
  if (grp == 0 && valid) {
    unsigned long long tg = 0, th = 0;
#pragma unroll
    for (int k = 0; k < kRedG; ++k) { tg += rg[k][le]; th += rh[k][le]; }
    const int F = E / kBinsPerFeature;  // slab element e = b * F + f -> histogram [f][b]
    const int bin = e / F, f = e - bin * F;
    if (i64_out) {
      reinterpret_cast<ulonglong2*>(hist)[f * kBinsPerFeature + bin] = make_ulonglong2(tg, th);
    } else {
      const HScale s = HistScale(scale_n, ghmax);
      hist[f * kBinsPerFeature + bin] = make_double2(static_cast<double>(static_cast<long long>(tg)) * s.ig,
                             static_cast<double>(static_cast<long long>(th)) * s.ih);
    }
  }
  if (blockIdx.x == 0 && tid == 0) {
    if (i64_out) reinterpret_cast<ulonglong2*>(hist)[E] = make_ulonglong2(static_cast<unsigned long long>(count), 0ull);
    else hist[E] = make_double2(static_cast<double>(count), 0.0);
  }
}

// Data-parallel histograms after the int64 allreduce: (E + 1) int64 pairs per histogram (blockIdx.y) -> fp64
// with the tree's global scale, the same conversion the 1-rank reduce applies; slot E = the global row count.
__global__ __launch_bounds__(256) void hist_convert_kernel(double2* __restrict__ part, int E, int64_t scale_n,
                                                           const float* __restrict__ ghmax) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e > E) return;
  double2* p = part + static_cast<size_t>(blockIdx.y) * (E + 1);
  const ulonglong2 v = reinterpret_cast<const ulonglong2*>(p)[e];
  if (e == E) {
    p[e] = make_double2(static_cast<double>(static_cast<long long>(v.x)), 0.0);
    return;
  }
  const HScale s = HistScale(scale_n, ghmax);
  p[e] = make_double2(static_cast<double>(static_cast<long long>(v.x)) * s.ig,
                      static_cast<double>(static_cast<long long>(v.y)) * s.ih);
}

// Global max |g| / max h over ranks (the histogram scale's inputs): every rank writes its maxima into its slot
// of a zeroed world-sized buffer, the buffer is sum-allreduced (exact: the other slots are zeros) and
// gh_slot_fold_kernel takes the max back into ghmax.
__global__ void gh_slot_fill_kernel(const unsigned int* __restrict__ ghmax, float* __restrict__ slots, int rank,
                                    int world) {
  for (int i = threadIdx.x; i < 2 * world; i += blockDim.x)
    slots[i] = (i >> 1) == rank ? __uint_as_float(ghmax[i & 1]) : 0.f;
}
__global__ void gh_slot_fold_kernel(const float* __restrict__ slots, int world, unsigned int* __restrict__ ghmax) {
  if (threadIdx.x < 2) {
    float m = 0.f;
    for (int q = 0; q < world; ++q) m = fmaxf(m, slots[2 * q + threadIdx.x]);
    ghmax[threadIdx.x] = __float_as_uint(m);
  }
}

// ---------------------------------------------------------------- K4 + K5
struct Cand {
  double gain;
  int thr;
  int dl;
};

__device__ __forceinline__ bool CandBetter(const Cand& a, const Cand& b) {
  if (a.gain != b.gain) return a.gain > b.gain;
  if (a.thr != b.thr) return a.thr < b.thr;
  return a.dl < b.dl;
}

// left: caller-provided buffer of 256 ints for the left-bin list (LDS in split_kernel, so the search
// needs no scratch)
__device__ void CategoricalSearchBuf(const double* hg, const double* hh, int nb, int fi, double G, double H,
                                     int64_t cnt, const SplitParams& sp, const MonoCtx* mc, SplitResult* best, int* idx,
                                     int* left) {
  // serial port of the host search (one thread): bins are <= 256
  const double cnt_factor = cnt / fmax(H, kEpsilon);
  const int other = nb - 1;
  const double l2 = sp.lambda_l2 + sp.cat_l2;
  const double cat_parent = LeafGain(G, H, sp.lambda_l1, l2, sp.max_delta_step);
  auto try_set = [&](int nleft, const int* left_bins, double gl, double hl) {
    const double gr = G - gl, hr = H - hl;
    const int64_t cl = EstimateCount(hl, cnt_factor), cr = cnt - cl;
    if (cl < sp.min_data_in_leaf || cr < sp.min_data_in_leaf) return;
    if (hl < sp.min_sum_hessian || hr < sp.min_sum_hessian) return;
    if (nleft > 1 && (cl < sp.min_data_per_group || cr < sp.min_data_per_group)) return;
    double gain, lout, rout;
    if (!EvalSplit(gl, hl, gr, hr, sp.lambda_l1, l2, sp.max_delta_step, mc, &gain, &lout, &rout)) return;
    const double shift = cat_parent + sp.min_gain_to_split;
    if (!(gain > shift)) return;
    const double sg = gain - shift;
    if (best->feature >= 0 && !SplitBetter(sg, fi, static_cast<uint32_t>(nleft), best->gain, best->feature, best->threshold)) return;
    best->gain = sg; best->feature = fi; best->threshold = static_cast<uint32_t>(nleft);
    best->default_left = 0; best->is_cat = 1;
    for (int w = 0; w < 8; ++w) best->cat_bits[w] = 0;
    for (int k = 0; k < nleft; ++k) best->cat_bits[left_bins[k] >> 5] |= 1u << (left_bins[k] & 31);
    best->left_g = gl; best->left_h = hl; best->right_g = gr; best->right_h = hr;
    best->left_cnt = cl; best->right_cnt = cr;
    best->left_out = lout;
    best->right_out = rout;
  };
  if (nb <= sp.max_cat_to_onehot + 1) {
    for (int b = 0; b < other; ++b) { int lb = b; try_set(1, &lb, hg[b], hh[b]); }
    return;
  }
  int m = 0;
  for (int b = 0; b < other; ++b)
    if (EstimateCount(hh[b], cnt_factor) >= sp.cat_smooth) idx[m++] = b;
  // stable insertion sort by g/(h+smooth)
  for (int i = 1; i < m; ++i) {
    int v = idx[i];
    double key = hg[v] / (hh[v] + sp.cat_smooth);
    int j = i - 1;
    while (j >= 0 && hg[idx[j]] / (hh[idx[j]] + sp.cat_smooth) > key) { idx[j + 1] = idx[j]; --j; }
    idx[j + 1] = v;
  }
  const int maxk = min(sp.max_cat_threshold, (m + 1) / 2);
  for (int dir = 0; dir < 2; ++dir) {
    double gl = 0, hl = 0;
    for (int k = 0; k < m && k < maxk; ++k) {
      int b = dir == 0 ? idx[k] : idx[m - 1 - k];
      left[k] = b;
      gl += hg[b]; hl += hh[b];
      try_set(k + 1, left, gl, hl);
    }
  }
}

__device__ void CategoricalSearch(const double* hg, const double* hh, int nb, int fi, double G, double H,
                                  int64_t cnt, const SplitParams& sp, const MonoCtx* mc, SplitResult* best, int* idx) {
  int left[256];
  CategoricalSearchBuf(hg, hh, nb, fi, G, H, cnt, sp, mc, best, idx, left);
}

// Search modes (tree_learner=voting runs 1 then 2 per split; everything else runs 0):
//   kFindFull   : `part` = the (globally reduced) smaller child / root histogram; the larger child is
//                 parent - smaller from the pool; both are stored in the pool
//   kFindLocal  : PV-Tree local pass - same histograms but LOCAL (not reduced), leaf totals and row counts
//                 local, min_data / min_hessian already divided by the world size in `sp`
//   kFindVoted  : PV-Tree global pass - `part` / `part1` = the globally reduced histograms of the voted
//                 features of the smaller / larger child (no pool access); only features with sel[child*F+f]
//                 are searched, leaf totals come from the split record (root: its own voted histogram)
enum FindMode { kFindFull = 0, kFindLocal = 1, kFindVoted = 2 };

__device__ void HistTotals(double2 mine, int nb, double* G, double* H);
__device__ void SearchFeatureBlock(double2 mine, double G, double H, int64_t cnt, int depth, int slot, double lo,
                                   double hi, int f, int F, const FeatMeta& fm, const SplitParams& sp, SplitResult* out,
                                   bool selected);

// Block (f, child): 256 threads, thread = bin.
__device__ void FindSplitBlock(
    DState* __restrict__ st, DLeaf* __restrict__ leaves, const double2* __restrict__ part, int E,
    const double* __restrict__ count_slot, double2* __restrict__ hist_pool, const FeatMeta& fm, const SplitParams& sp,
    SplitResult* __restrict__ fbest, int F, int mode, const double2* __restrict__ part1,
    const int8_t* __restrict__ sel, const int32_t* __restrict__ sel_first) {
  const int f = blockIdx.x;
  const int child = blockIdx.y;  // 0 = small (or root), 1 = large
  const int tid = threadIdx.x;
  const bool root = st->phase == 0;
  if (root && child == 1) return;
  const int leaf_id = root ? 0 : (child == 0 ? st->small_leaf : st->large_leaf);
  const int e = f * kBinsPerFeature + tid;
  double2 mine;
  if (mode == kFindVoted) {
    mine = (root || child == 0) ? part[e] : part1[e];
  } else {
    const double2 sm = part[e];  // smaller child's (or the root's) histogram
    if (root || child == 0) {
      mine = sm;
    } else {
      const double2 par = hist_pool[static_cast<size_t>(st->parent_slot) * E + e];
      mine = make_double2(par.x - sm.x, par.y - sm.y);
    }
  }
  const DLeaf Lf = leaves[leaf_id];
  if (mode != kFindVoted) hist_pool[static_cast<size_t>(Lf.slot) * E + e] = mine;
  // leaf totals: from this feature's histogram (root) or the split record
  double G, H;
  int64_t cnt;
  HistTotals(mine, fm.num_bin[f], &G, &H);
  if (root) {
    cnt = static_cast<int64_t>(*count_slot);
    const int writer = mode == kFindFull ? 0 : (mode == kFindVoted ? *sel_first : -1);
    if (f == writer && tid == 0) {
      leaves[0].sum_g = G; leaves[0].sum_h = H; leaves[0].gcount = cnt;
    }
  } else if (mode == kFindLocal) {
    // local totals (this feature's own histogram) and local row counts: the smaller child's from the slab
    // reduce's count slot, the larger's = the parent's local segment minus it
    const int64_t small_cnt = static_cast<int64_t>(*count_slot);
    cnt = child == 0 ? small_cnt : (static_cast<int64_t>(st->pcount) - small_cnt);
  } else {
    const int64_t small_cnt = static_cast<int64_t>(*count_slot);
    cnt = child == 0 ? small_cnt : (Lf.gcount - small_cnt);  // Lf.gcount of large holds the parent count (set by choose)
    G = Lf.sum_g; H = Lf.sum_h;
  }
  SearchFeatureBlock(mine, G, H, cnt, Lf.depth, Lf.slot, Lf.lo, Lf.hi, f, F, fm, sp, fbest + child * F + f,
                     mode != kFindVoted || sel[child * F + f]);
}

// Sum over the feature's bins of the block's histogram (thread = bin): the leaf totals at the root.
__device__ void HistTotals(double2 mine, int nb, double* G, double* H) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  __shared__ double wtot_g[4], wtot_h[4];
  double tg = tid < nb ? mine.x : 0.0, th = tid < nb ? mine.y : 0.0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) { tg += __shfl_xor(tg, off, 64); th += __shfl_xor(th, off, 64); }
  if (lane == 0) { wtot_g[wid] = tg; wtot_h[wid] = th; }
  __syncthreads();
  *G = wtot_g[0] + wtot_g[1] + wtot_g[2] + wtot_g[3];
  *H = wtot_h[0] + wtot_h[1] + wtot_h[2] + wtot_h[3];
}

// Best split of one (leaf, feature): 256 threads, thread = bin; `mine` = this thread's bin (g, h), G / H / cnt
// the leaf's totals, depth / slot / [lo, hi] its tree position and monotone bounds. Writes *out (feature -1,
// gain -inf when the feature cannot split the leaf).
__device__ void SearchFeatureBlock(double2 mine, double G, double H, int64_t cnt, int depth, int slot, double lo,
                                   double hi, int f, int F, const FeatMeta& fm, const SplitParams& sp, SplitResult* out,
                                   bool selected) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  __shared__ double sg_[256], shh_[256];
  __shared__ Cand wbest[4];
  __shared__ int idxbuf[256], leftbuf[256];
  __shared__ SplitResult s_cat_best;
  __shared__ MonoCtx s_mc;  // by pointer into EvalSplit / the categorical search: LDS, not scratch
  sg_[tid] = mine.x;
  shh_[tid] = mine.y;
  const int nb = fm.num_bin[f];
  const int mt = fm.missing[f];
  const int dbin = fm.default_bin[f];
  const bool eligible = fm.mask[f] && nb > 1 && selected &&
                        cnt >= 2 * static_cast<int64_t>(sp.min_data_in_leaf) &&
                        (sp.max_depth <= 0 || depth < sp.max_depth) &&
                        (sp.bynode_k <= 0 ||
                         NodeFeatureSelected(sp.bynode_seed, sp.tree_seq, slot, f, fm.mask, F, sp.bynode_k));
  if (!eligible) {
    if (tid == 0) { out->feature = -1; out->gain = -INFINITY; }
    return;
  }
  // monotone context of this (leaf, feature); categorical splits are clamped but carry no direction
  if (tid == 0) s_mc = MonoCtx{lo, hi, fm.is_cat[f] ? 0 : static_cast<int>(fm.mono[f])};
  __syncthreads();
  const MonoCtx* mcp = sp.has_mono ? &s_mc : nullptr;
  if (fm.is_cat[f]) {
    if (tid == 0) {
      SplitResult& best = s_cat_best;
      best.feature = -1; best.gain = -INFINITY;
      CategoricalSearchBuf(sg_, shh_, nb, f, G, H, cnt, sp, mcp, &best, idxbuf, leftbuf);
      const unsigned long long* src = reinterpret_cast<const unsigned long long*>(&best);
      unsigned long long* dst = reinterpret_cast<unsigned long long*>(out);
      for (int w = 0; w < static_cast<int>(sizeof(SplitResult) / 8); ++w) dst[w] = src[w];
    }
    return;
  }
  const int nan_bin = mt == kMissingNaN ? nb - 1 : -1;
  const int zero_bin = mt == kMissingZero ? dbin : -1;
  const double mg = nan_bin >= 0 ? sg_[nan_bin] : (zero_bin >= 0 ? sg_[zero_bin] : 0.0);
  const double mh = nan_bin >= 0 ? shh_[nan_bin] : (zero_bin >= 0 ? shh_[zero_bin] : 0.0);
  const int last = nan_bin >= 0 ? nb - 2 : nb - 1;
  // inclusive prefix over ordered bins (zero bin excluded for Zero missing)
  double vg = (tid < nb && tid != zero_bin && tid != nan_bin) ? mine.x : 0.0;
  double vh = (tid < nb && tid != zero_bin && tid != nan_bin) ? mine.y : 0.0;
  vg = wave_incl_scan(vg, lane);
  vh = wave_incl_scan(vh, lane);
  __shared__ double wsum_g[4], wsum_h[4];
  if (lane == 63) { wsum_g[wid] = vg; wsum_h[wid] = vh; }
  __syncthreads();
  for (int w = 0; w < wid; ++w) { vg += wsum_g[w]; vh += wsum_h[w]; }
  __shared__ double pref_g[256], pref_h[256];
  pref_g[tid] = vg;
  pref_h[tid] = vh;
  const double cnt_factor = cnt / fmax(H, kEpsilon);
  const double parent_gain = LeafGain(G, H, sp.lambda_l1, sp.lambda_l2, sp.max_delta_step);
  const double shift = parent_gain + sp.min_gain_to_split;
  Cand best{-INFINITY, 1 << 30, 1 << 30};
  if (tid < last) {
    auto consider = [&](double gl, double hl, int dl) {
      const double gr = G - gl, hr = H - hl;
      const int64_t cl = EstimateCount(hl, cnt_factor), cr = cnt - cl;
      if (cl < sp.min_data_in_leaf || cr < sp.min_data_in_leaf) return;
      if (hl < sp.min_sum_hessian || hr < sp.min_sum_hessian) return;
      double gain, lout, rout;
      if (!EvalSplit(gl, hl, gr, hr, sp.lambda_l1, sp.lambda_l2, sp.max_delta_step, mcp, &gain, &lout, &rout)) return;
      if (!(gain > shift)) return;
      Cand c{gain - shift, tid, dl};
      if (CandBetter(c, best)) best = c;
    };
    if (mt == kMissingNone) consider(vg, vh, 1);
    else { consider(vg, vh, 0); consider(vg + mg, vh + mh, 1); }
  }
  // block argmax
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    Cand o;
    o.gain = __shfl_xor(best.gain, off, 64);
    o.thr = __shfl_xor(best.thr, off, 64);
    o.dl = __shfl_xor(best.dl, off, 64);
    if (CandBetter(o, best)) best = o;
  }
  if (lane == 0) wbest[wid] = best;
  __syncthreads();
  if (tid == 0) {
    Cand b = wbest[0];
    for (int w = 1; w < 4; ++w) if (CandBetter(wbest[w], b)) b = wbest[w];
    SplitResult r;
    if (b.gain == -INFINITY) {
      r.feature = -1; r.gain = -INFINITY;
    } else {
      // the winning prefix, exactly as the candidate saw it
      double gl = pref_g[b.thr], hl = pref_h[b.thr];
      if (mt != kMissingNone && b.dl) { gl += mg; hl += mh; }
      const double gr = G - gl, hr = H - hl;
      r.feature = f; r.gain = b.gain; r.threshold = static_cast<uint32_t>(b.thr); r.default_left = b.dl;
      r.is_cat = 0;
      r.left_g = gl; r.left_h = hl; r.right_g = gr; r.right_h = hr;
      r.left_cnt = EstimateCount(hl, cnt_factor); r.right_cnt = cnt - r.left_cnt;
      double g2;
      (void)EvalSplit(gl, hl, gr, hr, sp.lambda_l1, sp.lambda_l2, sp.max_delta_step, mcp, &g2, &r.left_out, &r.right_out);
      if (mcp && mcp->mono != 0 && sp.monotone_penalty > 0) r.gain *= MonotonePenaltyFactor(depth, sp.monotone_penalty);
      for (int w = 0; w < 8; ++w) r.cat_bits[w] = 0;
    }
    *out = r;
  }
}

// ---------------------------------------------------------------- choose + tree bookkeeping
// One block. Wave c reduces the per-feature results of new leaf c (lanes
// stride over features), all threads then reduce the leaves' best gains, and
// thread 0 records the chosen split in the device tree and sets up the
// partition of that leaf. Every global read on the serial path is independent
// so the bookkeeping costs a few memory latencies, not one per leaf/feature.
struct KeyG {
  double gain;
  int a, b;  // tie-breakers (smaller wins)
};

__device__ __forceinline__ bool KeyBetter(const KeyG& x, const KeyG& y) {
  if (x.gain != y.gain) return x.gain > y.gain;
  if (x.a != y.a) return x.a < y.a;
  return x.b < y.b;
}

__device__ __forceinline__ KeyG WaveArgmax(KeyG k) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    KeyG o;
    o.gain = __shfl_xor(k.gain, off, 64);
    o.a = __shfl_xor(k.a, off, 64);
    o.b = __shfl_xor(k.b, off, 64);
    if (KeyBetter(o, k)) k = o;
  }
  return k;
}

__device__ void ChooseBlock(DState* __restrict__ st, DLeaf* __restrict__ leaves, SplitResult* __restrict__ lbest,
                            double* __restrict__ lgain, const SplitResult* __restrict__ fbest, int F, const DTree& t,
                            const double* __restrict__ count_slot, const int8_t* __restrict__ mono, int has_mono) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  __shared__ int sh_best_f[2];
  __shared__ KeyG wk[4];
  const bool root = st->phase == 0;
  const int nchild = root ? 1 : 2;
  const int small_leaf = st->small_leaf, large_leaf = st->large_leaf;
  if (wid < nchild) {
    KeyG k{-INFINITY, 1 << 30, 1 << 30};
    for (int f = lane; f < F; f += 64) {
      const SplitResult& r = fbest[wid * F + f];
      if (r.feature < 0) continue;
      KeyG c{r.gain, r.feature, static_cast<int>(r.threshold)};
      if (KeyBetter(c, k)) { k = c; k.b = (static_cast<int>(r.threshold) & 0xFFFF) | (f << 16); }
    }
    k = WaveArgmax(k);
    if (lane == 0) sh_best_f[wid] = k.gain == -INFINITY ? -1 : (k.b >> 16);
  }
  __syncthreads();
  if (tid == 0) {
    if (root) {
      const int bi = sh_best_f[0];
      if (bi >= 0) { lbest[0] = fbest[bi]; lgain[0] = fbest[bi].gain; }
      else { lbest[0].feature = -1; lbest[0].gain = -INFINITY; lgain[0] = -INFINITY; }
      t.lval[0] = RootLeafOutput(t, leaves[0].sum_g, leaves[0].sum_h);
      t.lcount[0] = leaves[0].gcount;
      t.lweight[0] = leaves[0].sum_h;
      t.lparent[0] = -1;
      t.ldepth[0] = 0;
    } else {
      const int64_t small_cnt = static_cast<int64_t>(*count_slot);
      const int64_t parent_cnt = leaves[large_leaf].gcount;  // stored by the previous choose
      const int ob = st->pbuf == 0 ? 1 : 0;
      DLeaf& Lc = leaves[st->split_leaf];
      DLeaf& Rc = leaves[st->new_leaf];
      const int lt = PTotal(st);
      Lc.begin = st->pbegin; Lc.count = lt; Lc.buf = ob;
      Rc.begin = st->pbegin + lt; Rc.count = st->pcount - lt; Rc.buf = ob;
      leaves[small_leaf].gcount = small_cnt;
      leaves[large_leaf].gcount = parent_cnt - small_cnt;
      t.lcount[small_leaf] = small_cnt;
      t.lcount[large_leaf] = parent_cnt - small_cnt;
      for (int c = 0; c < 2; ++c) {
        const int leaf = c == 0 ? small_leaf : large_leaf;
        const int bi = sh_best_f[c];
        if (bi >= 0) { lbest[leaf] = fbest[c * F + bi]; lgain[leaf] = fbest[c * F + bi].gain; }
        else { lbest[leaf].feature = -1; lbest[leaf].gain = -INFINITY; lgain[leaf] = -INFINITY; }
      }
    }
  }
  __syncthreads();
  const int nl = st->num_leaves;
  if (nl >= st->max_leaves) {
    if (tid == 0) st->done = 1;
    return;
  }
  // argmax over leaves (ties -> smaller leaf id)
  KeyG k{-INFINITY, 1 << 30, 0};
  for (int i = tid; i < nl; i += 256) {
    const double gi = lgain[i];
    KeyG c{gi, i, 0};
    if (gi > -INFINITY && KeyBetter(c, k)) k = c;
  }
  k = WaveArgmax(k);
  if (lane == 0) wk[wid] = k;
  __syncthreads();
  if (tid != 0) return;
  KeyG best = wk[0];
  for (int w = 1; w < 4; ++w) if (KeyBetter(wk[w], best)) best = wk[w];
  const int bl = best.gain == -INFINITY ? -1 : best.a;
  if (bl < 0 || !(best.gain > 0.0)) { st->done = 1; return; }
  const SplitResult sr = lbest[bl];
  const int node = nl - 1;
  const int parent = t.lparent[bl];
  if (parent >= 0) {
    if (t.left[parent] == ~bl) t.left[parent] = node; else t.right[parent] = node;
  }
  t.feat[node] = sr.feature;
  t.thr[node] = sr.threshold;
  t.dleft[node] = sr.default_left;
  t.is_cat[node] = sr.is_cat;
  for (int w = 0; w < 8; ++w) t.cat_bits[node * 8 + w] = sr.cat_bits[w];
  t.left[node] = ~bl;
  t.right[node] = ~nl;
  t.gain[node] = sr.gain;
  t.ival[node] = t.lval[bl];
  t.iweight[node] = sr.left_h + sr.right_h;
  t.icount[node] = leaves[bl].gcount;
  t.lparent[bl] = node; t.lparent[nl] = node;
  t.lval[bl] = sr.left_out; t.lval[nl] = sr.right_out;
  t.lweight[bl] = sr.left_h; t.lweight[nl] = sr.right_h;
  t.lcount[bl] = sr.left_cnt; t.lcount[nl] = sr.right_cnt;
  const int depth = t.ldepth[bl] + 1;
  t.ldepth[bl] = depth; t.ldepth[nl] = depth;
  const DLeaf P = leaves[bl];
  DLeaf Lc = P, Rc = P;
  Lc.depth = depth; Rc.depth = depth;
  Lc.sum_g = sr.left_g; Lc.sum_h = sr.left_h;
  Rc.sum_g = sr.right_g; Rc.sum_h = sr.right_h;
  // children inherit the parent's output bounds; a monotone split separates
  // them at the midpoint of the two outputs (basic method)
  const int mdir = (has_mono && !sr.is_cat) ? static_cast<int>(mono[sr.feature]) : 0;
  if (mdir != 0) {
    const double mid = (sr.left_out + sr.right_out) / 2.0;
    if (mdir < 0) { Lc.lo = fmax(Lc.lo, mid); Rc.hi = fmin(Rc.hi, mid); }
    else { Lc.hi = fmin(Lc.hi, mid); Rc.lo = fmax(Rc.lo, mid); }
  }
  const bool left_small = sr.left_cnt <= sr.right_cnt;
  st->parent_slot = P.slot;
  Lc.slot = 2 * node + 1;
  Rc.slot = 2 * node + 2;
  // the large child's gcount temporarily holds the parent's global count
  if (left_small) { Rc.gcount = P.gcount; } else { Lc.gcount = P.gcount; }
  leaves[bl] = Lc;
  leaves[nl] = Rc;
  lgain[bl] = -INFINITY;
  lgain[nl] = -INFINITY;
  st->pbegin = P.begin; st->pcount = P.count; st->pbuf = P.buf;
  st->cursor = 0ull;
  st->split_leaf = bl;
  st->new_leaf = nl;
  st->small_leaf = left_small ? bl : nl;
  st->large_leaf = left_small ? nl : bl;
  st->num_leaves = nl + 1;
  st->phase = 1;
}

__global__ __launch_bounds__(256) void find_split_kernel(
    DState* __restrict__ st, DLeaf* __restrict__ leaves, const double2* __restrict__ part, int E,
    const double* __restrict__ count_slot, double2* __restrict__ hist_pool, FeatMeta fm, SplitParams sp,
    SplitResult* __restrict__ fbest, int F, DState* __restrict__ st_next, int mode,
    const double2* __restrict__ part1, const int8_t* __restrict__ sel, const int32_t* __restrict__ sel_first) {
  // choose_part_kernel partitions on the next state version's cursor: zero it here (nothing reads it now)
  if (st_next && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) st_next->cursor = 0ull;
  if (st->done) return;
  FindSplitBlock(st, leaves, part, E, count_slot, hist_pool, fm, sp, fbest, F, mode, part1, sel, sel_first);
}

// ---------------------------------------------------------------- C3: PV-Tree voting on the device
// (reference parallelism=voting_parallel / topK, LightGBMParams.scala:25-35; the host backend's VotingFind
// in backend_cpu.cpp is the same algorithm on host buffers). Per split, after the LOCAL histograms and a local
// split search (kFindLocal):
//   vote_kernel     each rank votes for its top_k features of each new leaf by local gain
//   [allreduce]     votes + summed local gains + the smaller child's row count (4F+1 doubles)
//   select_kernel   per leaf the 2*top_k most-voted features (ties: summed gain, then feature id), filled with
//                   unvoted allowed features when fewer were voted
//   pack_kernel     the selected features' local histograms -> one compact buffer
//   [allreduce]     2 x 2*top_k x 256 bins x (g, h)
//   unpack_kernel   -> per-leaf global histograms of the selected features, then kFindVoted searches them
constexpr int kVoteMaxF = 8192;  // LDS flags of the vote / select kernels
constexpr int kVoteThreads = 1024;

struct VKey {
  double v, g;  // votes, summed gain (larger first)
  int f;        // feature (smaller first)
};

__device__ __forceinline__ bool VKeyBetter(const VKey& a, const VKey& b) {
  if (a.v != b.v) return a.v > b.v;
  if (a.g != b.g) return a.g > b.g;
  return a.f < b.f;
}

// block argmax of `k` (every thread of a kVoteThreads block calls it); returns the winner on every thread
__device__ VKey BlockArgmaxV(VKey k, VKey* s_w) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    VKey o;
    o.v = __shfl_xor(k.v, off, 64);
    o.g = __shfl_xor(k.g, off, 64);
    o.f = __shfl_xor(k.f, off, 64);
    if (VKeyBetter(o, k)) k = o;
  }
  if (lane == 0) s_w[wid] = k;
  __syncthreads();
  VKey b = s_w[0];
  for (int w = 1; w < kVoteThreads / 64; ++w) if (VKeyBetter(s_w[w], b)) b = s_w[w];
  __syncthreads();  // s_w is reused by the next call
  return b;
}

// top_k rounds of a block argmax over the local per-feature results (key: gain, then feature id = the host's
// SplitBetter order); vote layout [votes child 0 | votes child 1 | gains child 0 | gains child 1 | count]
__global__ __launch_bounds__(kVoteThreads) void vote_kernel(const DState* __restrict__ st,
                                                            const SplitResult* __restrict__ floc, int F, int topk,
                                                            const double* __restrict__ local_count,
                                                            double* __restrict__ vote) {
  __shared__ unsigned char chosen[2][kVoteMaxF];
  __shared__ VKey s_w[kVoteThreads / 64];
  const int tid = threadIdx.x;
  const bool done = st->done;
  const int C = st->phase == 0 ? 1 : 2;
  for (int c = 0; c < 2; ++c)
    for (int f = tid; f < F; f += kVoteThreads) chosen[c][f] = 0;
  __syncthreads();
  for (int c = 0; c < C && !done; ++c) {
    for (int r = 0; r < topk; ++r) {
      VKey k{-INFINITY, 0.0, 1 << 30};
      for (int f = tid; f < F; f += kVoteThreads) {
        const SplitResult& s = floc[c * F + f];
        if (s.feature < 0 || chosen[c][f]) continue;
        VKey o{s.gain, 0.0, f};
        if (VKeyBetter(o, k)) k = o;
      }
      const VKey b = BlockArgmaxV(k, s_w);
      if (b.v == -INFINITY) break;
      if (tid == 0) chosen[c][b.f] = 1;
      __syncthreads();
    }
  }
  // one writer per element
  for (int c = 0; c < 2; ++c)
    for (int f = tid; f < F; f += kVoteThreads) {
      const bool on = chosen[c][f] != 0;
      vote[c * F + f] = on ? 1.0 : 0.0;
      vote[(2 + c) * F + f] = on ? floc[c * F + f].gain : 0.0;
    }
  if (tid == 0) vote[4 * F] = *local_count;
}

// the summed votes -> per-leaf selection of up to K2 = min(2 top_k, F) features
__global__ __launch_bounds__(kVoteThreads) void select_kernel(const DState* __restrict__ st,
                                                              const double* __restrict__ vote, int F, int K2,
                                                              const int8_t* __restrict__ mask,
                                                              int32_t* __restrict__ sel_idx,
                                                              int32_t* __restrict__ sel_pos,
                                                              int8_t* __restrict__ sel_mask) {
  __shared__ int16_t rank[2][kVoteMaxF];
  __shared__ VKey s_w[kVoteThreads / 64];
  const int tid = threadIdx.x;
  const bool done = st->done;
  const int C = st->phase == 0 ? 1 : 2;
  for (int c = 0; c < 2; ++c)
    for (int f = tid; f < F; f += kVoteThreads) rank[c][f] = -1;
  __syncthreads();
  for (int c = 0; c < 2; ++c) {
    int r = 0;
    for (; c < C && !done && r < K2; ++r) {
      VKey k{-INFINITY, 0.0, 1 << 30};
      for (int f = tid; f < F; f += kVoteThreads) {
        const double v = vote[c * F + f];
        if (rank[c][f] >= 0 || !(v > 0.0 || mask[f])) continue;
        VKey o{v, v > 0.0 ? vote[(2 + c) * F + f] : 0.0, f};
        if (VKeyBetter(o, k)) k = o;
      }
      const VKey b = BlockArgmaxV(k, s_w);
      if (b.v == -INFINITY) break;
      if (tid == 0) { rank[c][b.f] = static_cast<int16_t>(r); sel_idx[c * K2 + r] = b.f; }
      __syncthreads();
    }
    for (int i = r + tid; i < K2; i += kVoteThreads) sel_idx[c * K2 + i] = -1;
  }
  __syncthreads();
  for (int c = 0; c < 2; ++c)
    for (int f = tid; f < F; f += kVoteThreads) {
      sel_pos[c * F + f] = rank[c][f];
      sel_mask[c * F + f] = rank[c][f] >= 0 ? 1 : 0;
    }
}

// block (i, c): the i-th selected feature of leaf c, its LOCAL histogram (stored in the pool by kFindLocal)
__global__ __launch_bounds__(256) void pack_kernel(const DState* __restrict__ st, const DLeaf* __restrict__ leaves,
                                                   const int32_t* __restrict__ sel_idx, int K2,
                                                   const double2* __restrict__ hist_pool, int E,
                                                   double2* __restrict__ compact) {
  const int i = blockIdx.x, c = blockIdx.y, tid = threadIdx.x;
  double2* dst = compact + (static_cast<size_t>(c) * K2 + i) * kBinsPerFeature + tid;
  const bool root = st->phase == 0;
  const int f = st->done ? -1 : sel_idx[c * K2 + i];
  if (f < 0 || (root && c == 1)) { *dst = make_double2(0.0, 0.0); return; }
  const int leaf_id = root ? 0 : (c == 0 ? st->small_leaf : st->large_leaf);
  *dst = hist_pool[static_cast<size_t>(leaves[leaf_id].slot) * E + f * kBinsPerFeature + tid];
}

// block (f, c): the reduced histogram of feature f of leaf c (zeros when f was not selected)
__global__ __launch_bounds__(256) void unpack_kernel(const DState* __restrict__ st, const int32_t* __restrict__ sel_pos,
                                                     int F, int K2, const double2* __restrict__ compact, int E,
                                                     double2* __restrict__ gh) {
  if (st->done) return;
  const int f = blockIdx.x, c = blockIdx.y, tid = threadIdx.x;
  const int p = sel_pos[c * F + f];
  gh[static_cast<size_t>(c) * E + f * kBinsPerFeature + tid] =
      p >= 0 ? compact[(static_cast<size_t>(c) * K2 + p) * kBinsPerFeature + tid] : make_double2(0.0, 0.0);
}

// The last split of a tree (single process): its children are never split, so their histograms and split
// searches are not needed; only their exact row counts are, and the partition just counted them (the
// split's estimated counts came from hessian sums). One thread replaces hist + reduce + find + choose.
__global__ void finalize_last_split_kernel(const DState* __restrict__ st, const DLeaf* __restrict__ leaves, DTree t) {
  if (threadIdx.x != 0 || st->done || st->phase == 0) return;
  const int lt = PTotal(st);
  const int64_t small_cnt = st->small_leaf == st->split_leaf ? lt : st->pcount - lt;
  const int64_t parent_cnt = leaves[st->large_leaf].gcount;  // the keeper left the parent's count there
  t.lcount[st->small_leaf] = small_cnt;
  t.lcount[st->large_leaf] = parent_cnt - small_cnt;
}

__global__ __launch_bounds__(256) void choose_kernel(DState* __restrict__ st, DLeaf* __restrict__ leaves,
                                                     SplitResult* __restrict__ lbest, double* __restrict__ lgain,
                                                     const SplitResult* __restrict__ fbest, int F, DTree t,
                                                     const double* __restrict__ count_slot,
                                                     const int8_t* __restrict__ mono, int has_mono) {
  if (st->done) return;
  ChooseBlock(st, leaves, lbest, lgain, fbest, F, t, count_slot, mono, has_mono);
}

// ---------------------------------------------------------------- K6
// Decisions read the column-major copy: the lanes of a wave touch one byte
// column (contiguous for the physical root, increasing for partitioned leaves)
// instead of one 32-B row each.
// The split the partition applies: scalars (wave-uniform, SGPRs) plus the
// category bitset staged in LDS. Copying the whole 120-byte SplitResult into
// a local made the compiler place it in scratch (cat_bits is indexed by a
// per-row bin): 128 B/lane of scratch on every partition launch.
struct PartSplit {
  int feature, nb, mt, dbin, is_cat, dleft;
  uint32_t thr;
};

__device__ __forceinline__ bool RowGoesLeft(const uint8_t* cbins, int64_t n, int r, const PartSplit& ps,
                                            const uint32_t* s_cat) {
  const uint32_t b = cbins[static_cast<size_t>(ps.feature) * n + r];
  return DeviceGoesLeft(b, ps.nb, ps.mt, ps.dbin, ps.is_cat, ps.thr, ps.dleft, s_cat);
}

// Single pass: a block takes tiles of kPartTile rows (kPartRows per thread,
// strided so every load is coalesced), keeps them in registers, counts the
// tile's left rows with wave ballots and claims its output ranges with one
// atomicAdd on the left cursor and one atomicSub on the right cursor, then
// writes the rows straight to their final slots. Row order inside a child
// depends on the order tiles claim their ranges; nothing downstream depends
// on it (histograms are exact integer sums, see K3).

// One tile of the single-pass partition of segment [pbegin, pbegin + pcount) of ping-pong buffer pbuf (-1 =
// physical rows) by split ps; claims its output ranges on *cursor (zeroed before the launch).
template <int kPartRows>
__device__ __forceinline__ void PartitionTile(
    const PartSplit& ps, const uint32_t* s_cat, int tile, int pbegin, int pcount, int pbuf, unsigned long long* cursor,
    const uint8_t* __restrict__ cbins, int64_t n, const int32_t* __restrict__ perm0,
    const int32_t* __restrict__ perm1, const float2* __restrict__ ogh0, const float2* __restrict__ ogh1,
    int32_t* __restrict__ wperm0, int32_t* __restrict__ wperm1, float2* __restrict__ wogh0,
    float2* __restrict__ wogh1, const float* __restrict__ g, const float* __restrict__ h) {
  constexpr int kPartTile = kPartThreads * kPartRows;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  constexpr int kWaves = kPartThreads / 64;
  __shared__ int wl[kPartRows][kWaves];
  __shared__ int bases[2];
  const int32_t* perm = pbuf == 0 ? perm0 : perm1;
  const float2* ogh = pbuf == 0 ? ogh0 : ogh1;
  int32_t* operm = pbuf == 0 ? wperm1 : wperm0;
  float2* oogh = pbuf == 0 ? wogh1 : wogh0;
  const unsigned long long below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  {
    const int t0 = pbegin + tile * kPartTile;
    const int tv = min(kPartTile, pbegin + pcount - t0);
    // Branch-free loads, every row of the tile in flight at once: rows past the segment read position t0
    // (always valid) and are masked afterwards. (Guarding each load with k < tv put every load in its own
    // branch, and the compiler waited out one memory latency per row - 8 serial bin-byte gathers per tile.)
    int r[kPartRows];
    float2 v[kPartRows];
    if (pbuf < 0) {
#pragma unroll
      for (int u = 0; u < kPartRows; ++u) {
        const int k = u * kPartThreads + tid;
        const int p = t0 + (k < tv ? k : 0);
        r[u] = p;
        v[u] = make_float2(g[p], h[p]);
      }
    } else {
#pragma unroll
      for (int u = 0; u < kPartRows; ++u) {
        const int k = u * kPartThreads + tid;
        const int p = t0 + (k < tv ? k : 0);
        r[u] = perm[p];
        v[u] = ogh[p];
      }
    }
    uint32_t bin[kPartRows];
    const uint8_t* __restrict__ col = cbins + static_cast<size_t>(ps.feature) * n;
#pragma unroll
    for (int u = 0; u < kPartRows; ++u) bin[u] = col[r[u]];
    int rl[kPartRows];
    unsigned lmask = 0;
#pragma unroll
    for (int u = 0; u < kPartRows; ++u) {
      const int k = u * kPartThreads + tid;
      const bool left = k < tv && DeviceGoesLeft(bin[u], ps.nb, ps.mt, ps.dbin, ps.is_cat, ps.thr, ps.dleft, s_cat);
      lmask |= left ? (1u << u) : 0u;
      const unsigned long long bl = __ballot(left);
      rl[u] = __popcll(bl & below);
      if (lane == 0) wl[u][wid] = __popcll(bl);
    }
    __syncthreads();
    if (tid == 0) {
      int tl = 0;
      for (int u = 0; u < kPartRows; ++u)
        for (int w = 0; w < kWaves; ++w) tl += wl[u][w];
      const int tr = tv - tl;
      const unsigned long long old =
          atomicAdd(cursor, static_cast<unsigned long long>(tl) | (static_cast<unsigned long long>(tr) << 32));
      bases[0] = pbegin + static_cast<int>(old & 0xFFFFFFFFull);
      bases[1] = pbegin + pcount - static_cast<int>(old >> 32) - tr;
    }
    __syncthreads();
    const int lb = bases[0], rb = bases[1];
    int run = 0;  // left rows in earlier row-groups of this tile
#pragma unroll
    for (int u = 0; u < kPartRows; ++u) {
      int wb = 0, ut = 0;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) {
        const int c = wl[u][w];
        wb += w < wid ? c : 0;
        ut += c;
      }
      const int k = u * kPartThreads + tid;
      if (k < tv) {
        const int lbefore = run + wb + rl[u];
        const int dst = (lmask >> u) & 1u ? lb + lbefore : rb + (k - lbefore);
        if (c_part_wt) {
          __hip_atomic_store(operm + dst, r[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(reinterpret_cast<unsigned long long*>(oogh + dst),
                             (static_cast<unsigned long long>(__float_as_uint(v[u].y)) << 32) | __float_as_uint(v[u].x),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          operm[dst] = r[u];
          oogh[dst] = v[u];
        }
      }
      run += ut;
    }
    __syncthreads();
  }
}

// Tile loop of the single-pass partition of one segment (blocks stride over its tiles).
template <int kPartRows>
__device__ __forceinline__ void PartitionTiles(
    const PartSplit& ps, const uint32_t* s_cat, int pbegin, int pcount, int pbuf, unsigned long long* cursor,
    const uint8_t* __restrict__ cbins, int64_t n, const int32_t* __restrict__ perm0,
    const int32_t* __restrict__ perm1, const float2* __restrict__ ogh0, const float2* __restrict__ ogh1,
    int32_t* __restrict__ wperm0, int32_t* __restrict__ wperm1, float2* __restrict__ wogh0,
    float2* __restrict__ wogh1, const float* __restrict__ g, const float* __restrict__ h) {
  constexpr int kPartTile = kPartThreads * kPartRows;
  const int ntiles = ceil_div_i(pcount, kPartTile);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x)
    PartitionTile<kPartRows>(ps, s_cat, tile, pbegin, pcount, pbuf, cursor, cbins, n, perm0, perm1, ogh0, ogh1, wperm0,
                             wperm1, wogh0, wogh1, g, h);
}

// ---------------------------------------------------------------- choose + K6, one launch
// The choose step (ChooseBlock) fused into the partition it decides: every
// block redundantly reduces the new children's per-feature records and the
// leaves' best gains (a few KB of L2-resident reads) to find the leaf to split
// and its split, then partitions its tiles; the LAST block (usually without
// tiles) alone writes the bookkeeping. That saves the 1-block choose launch
// per split. Nothing a block reads is written in the same launch except fields
// whose bytes do not change:
//  * the tree state is double-buffered: `sin` (read by all) -> `sout` (written
//    by the bookkeeping block; its cursor was zeroed by the preceding
//    find_split_kernel and only receives the partition's atomics here);
//  * lgain / lbest of the two new children are taken from fbest in registers
//    by every block; the bookkeeping block stores them for later launches and
//    does NOT mark the split leaf's gain -inf (the next launch replaces both
//    children's gains from fbest before any argmax reads them);
//  * leaves[bl] is rewritten with unchanged begin / count / buf (the only
//    fields the other blocks read).
template <int kPartRows>
__global__ __launch_bounds__(kPartThreads) void choose_part_kernel(
    const DState* __restrict__ sin, DState* __restrict__ sout, DLeaf* __restrict__ leaves,
    SplitResult* __restrict__ lbest, double* __restrict__ lgain, const SplitResult* __restrict__ fbest, int F,
    DTree t, const double* __restrict__ count_slot, const int8_t* __restrict__ mono, int has_mono,
    const uint8_t* __restrict__ cbins, int64_t n, const int32_t* __restrict__ perm0,
    const int32_t* __restrict__ perm1, const float2* __restrict__ ogh0, const float2* __restrict__ ogh1,
    int32_t* __restrict__ wperm0, int32_t* __restrict__ wperm1, float2* __restrict__ wogh0,
    float2* __restrict__ wogh1, const float* __restrict__ g, const float* __restrict__ h, FeatMeta fm) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  constexpr int kWaves = kPartThreads / 64;
  const bool keeper = blockIdx.x == gridDim.x - 1;  // writes the bookkeeping
  const DState S = *sin;
  if (S.done) {
    if (keeper && tid == 0) {
      DState o = S;
      o.cursor = 0ull;
      *sout = o;
    }
    return;
  }
  __shared__ int s_bf[2];
  __shared__ KeyG s_wk[kWaves];
  __shared__ uint32_t s_cat[8];
  const bool root = S.phase == 0;
  const int nchild = root ? 1 : 2;
  const int nl = S.num_leaves;
  // the leaves' stored gains do not depend on the children's records: load them first
  const double my_gain = tid < nl ? lgain[tid] : -INFINITY;
  if (wid < nchild) {
    KeyG k{-INFINITY, 1 << 30, 1 << 30};
    for (int f = lane; f < F; f += 64) {
      const SplitResult& r = fbest[wid * F + f];
      if (r.feature < 0) continue;
      KeyG c{r.gain, r.feature, static_cast<int>(r.threshold)};
      if (KeyBetter(c, k)) { k = c; k.b = (static_cast<int>(r.threshold) & 0xFFFF) | (f << 16); }
    }
    k = WaveArgmax(k);
    if (lane == 0) s_bf[wid] = k.gain == -INFINITY ? -1 : (k.b >> 16);
  }
  __syncthreads();
  const int bf0 = s_bf[0], bf1 = root ? -1 : s_bf[1];
  const double cg0 = bf0 >= 0 ? fbest[bf0].gain : -INFINITY;
  const double cg1 = bf1 >= 0 ? fbest[F + bf1].gain : -INFINITY;
  const int small_leaf = S.small_leaf, large_leaf = S.large_leaf;
  // argmax over leaves (ties -> smaller leaf id), the children's gains from registers
  KeyG k{-INFINITY, 1 << 30, 0};
  if (nl < S.max_leaves) {
    for (int i = tid; i < nl; i += kPartThreads) {
      const double gi = root ? cg0 : (i == small_leaf ? cg0 : (i == large_leaf ? cg1 : (i == tid ? my_gain : lgain[i])));
      KeyG c{gi, i, 0};
      if (gi > -INFINITY && KeyBetter(c, k)) k = c;
    }
  }
  k = WaveArgmax(k);
  if (lane == 0) s_wk[wid] = k;
  __syncthreads();
  KeyG best = s_wk[0];
  for (int w = 1; w < kWaves; ++w) if (KeyBetter(s_wk[w], best)) best = s_wk[w];
  const int bl = best.gain == -INFINITY ? -1 : best.a;
  const bool go = nl < S.max_leaves && bl >= 0 && best.gain > 0.0;
  // the chosen split and the segment of leaf bl
  const SplitResult* srp = nullptr;
  int pb = 0, pc = 0, pbuf = -1;
  if (go) {
    srp = (root || bl == small_leaf) ? fbest + bf0 : (bl == large_leaf ? fbest + F + bf1 : lbest + bl);
    if (!root && (bl == S.split_leaf || bl == S.new_leaf)) {
      const int lt = static_cast<int>(S.cursor & 0xFFFFFFFFull);
      pb = bl == S.split_leaf ? S.pbegin : S.pbegin + lt;
      pc = bl == S.split_leaf ? lt : S.pcount - lt;
      pbuf = S.pbuf == 0 ? 1 : 0;
    } else {
      pb = leaves[bl].begin; pc = leaves[bl].count; pbuf = leaves[bl].buf;
    }
  }
  if (keeper && tid == 0) {
    // children of the previous split (ChooseBlock's first half)
    if (root) {
      if (bf0 >= 0) { lbest[0] = fbest[bf0]; lgain[0] = cg0; }
      else { lbest[0].feature = -1; lbest[0].gain = -INFINITY; lgain[0] = -INFINITY; }
      t.lval[0] = RootLeafOutput(t, leaves[0].sum_g, leaves[0].sum_h);
      t.lcount[0] = leaves[0].gcount;
      t.lweight[0] = leaves[0].sum_h;
      t.lparent[0] = -1;
      t.ldepth[0] = 0;
    } else {
      const int64_t small_cnt = static_cast<int64_t>(*count_slot);
      const int64_t parent_cnt = leaves[large_leaf].gcount;  // stored by the previous choose
      const int lt = static_cast<int>(S.cursor & 0xFFFFFFFFull);
      const int ob = S.pbuf == 0 ? 1 : 0;
      DLeaf& Lc = leaves[S.split_leaf];
      DLeaf& Rc = leaves[S.new_leaf];
      Lc.begin = S.pbegin; Lc.count = lt; Lc.buf = ob;
      Rc.begin = S.pbegin + lt; Rc.count = S.pcount - lt; Rc.buf = ob;
      leaves[small_leaf].gcount = small_cnt;
      leaves[large_leaf].gcount = parent_cnt - small_cnt;
      t.lcount[small_leaf] = small_cnt;
      t.lcount[large_leaf] = parent_cnt - small_cnt;
      for (int c = 0; c < 2; ++c) {
        const int leaf = c == 0 ? small_leaf : large_leaf;
        const int bi = c == 0 ? bf0 : bf1;
        if (bi >= 0) { lbest[leaf] = fbest[c * F + bi]; lgain[leaf] = c == 0 ? cg0 : cg1; }
        else { lbest[leaf].feature = -1; lbest[leaf].gain = -INFINITY; lgain[leaf] = -INFINITY; }
      }
    }
    DState o = S;
    o.cursor = 0ull;
    if (!go) {
      o.done = 1;
      *sout = o;
    } else {
      // the split itself (ChooseBlock's second half, without the -inf gain marks)
      const SplitResult sr = *srp;
      const int node = nl - 1;
      const int parent = t.lparent[bl];
      if (parent >= 0) {
        if (t.left[parent] == ~bl) t.left[parent] = node; else t.right[parent] = node;
      }
      t.feat[node] = sr.feature;
      t.thr[node] = sr.threshold;
      t.dleft[node] = sr.default_left;
      t.is_cat[node] = sr.is_cat;
      for (int w = 0; w < 8; ++w) t.cat_bits[node * 8 + w] = sr.cat_bits[w];
      t.left[node] = ~bl;
      t.right[node] = ~nl;
      t.gain[node] = sr.gain;
      t.ival[node] = t.lval[bl];
      t.iweight[node] = sr.left_h + sr.right_h;
      t.icount[node] = leaves[bl].gcount;
      t.lparent[bl] = node; t.lparent[nl] = node;
      t.lval[bl] = sr.left_out; t.lval[nl] = sr.right_out;
      t.lweight[bl] = sr.left_h; t.lweight[nl] = sr.right_h;
      t.lcount[bl] = sr.left_cnt; t.lcount[nl] = sr.right_cnt;
      const int depth = t.ldepth[bl] + 1;
      t.ldepth[bl] = depth; t.ldepth[nl] = depth;
      const DLeaf P = leaves[bl];
      DLeaf Lc = P, Rc = P;
      Lc.depth = depth; Rc.depth = depth;
      Lc.sum_g = sr.left_g; Lc.sum_h = sr.left_h;
      Rc.sum_g = sr.right_g; Rc.sum_h = sr.right_h;
      const int mdir = (has_mono && !sr.is_cat) ? static_cast<int>(mono[sr.feature]) : 0;
      if (mdir != 0) {
        const double mid = (sr.left_out + sr.right_out) / 2.0;
        if (mdir < 0) { Lc.lo = fmax(Lc.lo, mid); Rc.hi = fmin(Rc.hi, mid); }
        else { Lc.hi = fmin(Lc.hi, mid); Rc.lo = fmax(Rc.lo, mid); }
      }
      const bool left_small = sr.left_cnt <= sr.right_cnt;
      Lc.slot = 2 * node + 1;
      Rc.slot = 2 * node + 2;
      if (left_small) { Rc.gcount = P.gcount; } else { Lc.gcount = P.gcount; }
      leaves[bl] = Lc;
      leaves[nl] = Rc;
      o.parent_slot = P.slot;
      o.pbegin = P.begin; o.pcount = P.count; o.pbuf = P.buf;
      o.split_leaf = bl;
      o.new_leaf = nl;
      o.small_leaf = left_small ? bl : nl;
      o.large_leaf = left_small ? nl : bl;
      o.num_leaves = nl + 1;
      o.phase = 1;
      // every field but the cursor (the other blocks are adding to it)
      sout->num_leaves = o.num_leaves; sout->done = 0; sout->split_leaf = o.split_leaf; sout->new_leaf = o.new_leaf;
      sout->small_leaf = o.small_leaf; sout->large_leaf = o.large_leaf; sout->parent_slot = o.parent_slot;
      sout->max_leaves = o.max_leaves; sout->phase = o.phase;
      sout->pbegin = o.pbegin; sout->pcount = o.pcount; sout->pbuf = o.pbuf;
    }
  }
  if (!go) return;
  constexpr int kPartTile = kPartThreads * kPartRows;
  if (static_cast<int>(blockIdx.x) >= ceil_div_i(pc, kPartTile)) return;
  PartSplit ps;
  ps.feature = srp->feature;
  ps.is_cat = srp->is_cat;
  ps.dleft = srp->default_left;
  ps.thr = srp->threshold;
  ps.nb = fm.num_bin[ps.feature];
  ps.mt = fm.missing[ps.feature];
  ps.dbin = fm.default_bin[ps.feature];
  if (tid < 8) s_cat[tid] = ps.is_cat ? srp->cat_bits[tid] : 0u;
  __syncthreads();
  PartitionTiles<kPartRows>(ps, s_cat, pb, pc, pbuf, &sout->cursor, cbins, n, perm0, perm1, ogh0, ogh1, wperm0,
                            wperm1, wogh0, wogh1, g, h);
}

// ---------------------------------------------------------------- batched speculative growth
// Leaf-wise growth splits the leaf of largest gain, one split at a time: ~4 dependent kernels per split, and
// at 31 leaves the per-split launch/latency chain was half of the iteration (profiles/README, round 3). The
// sequence of splits it makes is a pure function of the gains: in best-first order a node is split iff it is
// among the first B = num_leaves - 1 pops, and a node's gain never changes once its histogram exists. So
// splits can be computed AHEAD of their turn and the sequential order recovered afterwards:
//   bplan_kernel   replays the sequential best-first pops over the explored tree (nodes whose children's best
//                  splits are known). The first pop of an unexplored node u is exactly the next split the
//                  sequential learner would make; u and the next (spec_k - 1) unexplored nodes the replay
//                  would pop if u's children did not overtake them are expanded together this round.
//                  When the replay completes B pops (or runs out of positive gains) on explored nodes only,
//                  the tree is final: it is written in sequential node / leaf numbering, identical to the
//                  one-split-at-a-time result (expanded nodes that were never popped are simply leaves).
//   bpart_kernel   partitions all expansions of the round in one launch (tiles of every segment)
//   bhist_kernel   histograms of every expansion's smaller child (blocks shared out by row count)
//   breduce_kernel exact int64 slab reduce per expansion (+ one allreduce of all of them, data-parallel)
//   bfind_kernel   split search of both children of every expansion (larger = parent - smaller)
// Trees are bit-identical to the sequential growth (same histograms, same subtraction side, same tie
// breaks); the kernel count per tree drops from ~4 per split to ~5 per round, with ~B / spec_k rounds.
// The host keeps one round ahead of the device and stops when the plan of a round reports the tree final.
constexpr int kMaxSpec = 16;
constexpr int kBatchMaxLeaves = 256;
constexpr int kBatchMaxNodes = 1 + 2 * (2 * (kBatchMaxLeaves - 1) + kMaxSpec);

struct BNode {
  int32_t begin, count, buf, depth;  // local row segment
  int64_t gcount;                    // global rows
  double sum_g, sum_h, lo, hi;       // totals, monotone output bounds
  double out;                        // output as a leaf (the parent's left_out / right_out; root 0)
  int32_t c0, c1;                    // children (expanded) or -1
};

struct BExp {
  int32_t node, c0, c1, left_small;
  int32_t pbegin, pcount, pbuf, tile0;  // parent segment; first global partition tile of this expansion
  PartSplit ps;
  uint32_t cat[8];
  int64_t pgcount;  // the parent's global rows (the larger child's count = pgcount - the smaller's)
};

constexpr int kCurStride = 32;  // 8-byte words between two expansions' cursors (256 B)

struct BState {
  int32_t nexp, done, nnodes, expanded;
  int32_t spec_used, ntiles, cap_nodes, cap_exp;
  // expansion j's partition cursor is cursor[j * kCurStride]: each on its own 256-byte line, so the per-tile
  // claims of different expansions do not serialise on one cache line
  unsigned long long cursor[kMaxSpec * kCurStride];
  BExp exp[kMaxSpec];
  // the replay's committed prefix (every pop before the first unexplored one, which later rounds can only
  // confirm): the frontier at that point and the pops so far, so the next round resumes there instead of
  // replaying the whole tree again (the replay cost ~1 us per pop: 7.6 us at round 0, 36 us at round 29)
  int32_t rp_nf, rp_pops;
  int32_t rp_fnode[kBatchMaxLeaves + 1], rp_fli[kBatchMaxLeaves + 1];
  int32_t rp_pnode[kBatchMaxLeaves], rp_pli[kBatchMaxLeaves];
};

// Histogram block budget per expansion (the slab holds kMaxHistBlocks blocks): HistBlocks(count) each, scaled
// down proportionally (at least 1) when they do not fit. Deterministic in the counts, so bhist and breduce
// agree on it.
__device__ __forceinline__ void BatchHistAlloc(const int* cnt, int nexp, int* nb, int* off) {
  int tot = 0;
  for (int j = 0; j < nexp; ++j) { nb[j] = HistBlocks(cnt[j]); tot += nb[j]; }
  if (tot > c_max_hist_blocks) {
    const int spare = c_max_hist_blocks - nexp;
    int t2 = 0;
    for (int j = 0; j < nexp; ++j) { nb[j] = 1 + (nb[j] - 1) * spare / max(1, tot - nexp); t2 += nb[j]; }
  }
  int o = 0;
  for (int j = 0; j < nexp; ++j) { off[j] = o; o += nb[j]; }
}

__device__ __forceinline__ int BatchSmallCount(const BState* bs, int j) {
  const BExp& x = bs->exp[j];
  const int lt = static_cast<int>(bs->cursor[j * kCurStride] & 0xFFFFFFFFull);
  return x.left_small ? lt : x.pcount - lt;
}

constexpr int kPlanThreads = 1024;
constexpr int kPlanProfStride = 16;  // SML_BPLAN_PROF slots per round
constexpr int kPlanFm = 1024;  // features whose split metadata the plan stages in LDS

// round outcome for the host (coherent pinned memory, read after the plan's event): system-scope vector store
__device__ __forceinline__ void SetHostFlag(int* f, int v) {
  __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Wave-wide maximum of a 64-bit key: DPP exchanges inside each row of 16 lanes (quad swaps, half-row and row
// mirrors: VALU, no LDS round trip), then the four rows' maxima read into scalars. Every lane must be active.
template <int kCtrl>
__device__ __forceinline__ unsigned long long DppMaxU64(unsigned long long x) {
  const unsigned lo = static_cast<unsigned>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), kCtrl, 0xF, 0xF, false));
  const unsigned hi =
      static_cast<unsigned>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x >> 32), kCtrl, 0xF, 0xF, false));
  const unsigned long long y = (static_cast<unsigned long long>(hi) << 32) | lo;
  return y > x ? y : x;
}

// rows not in kRowMask keep x (the DPP write is masked off for them)
template <int kCtrl, int kRowMask>
__device__ __forceinline__ unsigned long long DppMaxRowsU64(unsigned long long x) {
  const int xl = static_cast<int>(x), xh = static_cast<int>(x >> 32);
  const unsigned lo = static_cast<unsigned>(__builtin_amdgcn_update_dpp(xl, xl, kCtrl, kRowMask, 0xF, false));
  const unsigned hi = static_cast<unsigned>(__builtin_amdgcn_update_dpp(xh, xh, kCtrl, kRowMask, 0xF, false));
  const unsigned long long y = (static_cast<unsigned long long>(hi) << 32) | lo;
  return y > x ? y : x;
}

__device__ __forceinline__ unsigned long long WaveMaxU64(unsigned long long x) {
  x = DppMaxU64<0xB1>(x);   // quad_perm [1,0,3,2]
  x = DppMaxU64<0x4E>(x);   // quad_perm [2,3,0,1]
  x = DppMaxU64<0x141>(x);  // row_half_mirror
  x = DppMaxU64<0x140>(x);  // row_mirror: every lane holds its row's maximum
  x = DppMaxRowsU64<0x142, 0xA>(x);  // row_bcast:15 -> rows 1, 3 fold in rows 0, 2
  x = DppMaxRowsU64<0x143, 0xC>(x);  // row_bcast:31 -> rows 2, 3 fold in row 1: lane 63 holds the maximum
  const unsigned lo = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(x), 63));
  const unsigned hi = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(x >> 32), 63));
  return (static_cast<unsigned long long>(hi) << 32) | lo;
}

__device__ __forceinline__ int WaveMinI32(int x) {
  x = min(x, __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false));
  x = min(x, __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false));
  x = min(x, __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, false));
  x = min(x, __builtin_amdgcn_update_dpp(0, x, 0x140, 0xF, 0xF, false));
  return min(min(__builtin_amdgcn_readlane(x, 0), __builtin_amdgcn_readlane(x, 16)),
             min(__builtin_amdgcn_readlane(x, 32), __builtin_amdgcn_readlane(x, 48)));
}

// a double's bits as an unsigned key with the same order (larger gain -> larger key; +0 -> 2^63)
__device__ __forceinline__ unsigned long long GainKey(double g) {
  const unsigned long long u = static_cast<unsigned long long>(__double_as_longlong(g));
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

// lane l's entry `s` of a per-lane register array, `s` wave-uniform: every slot is read with v_readlane and
// the scalar results selected (a select over the register array itself was turned back into an indexed
// scratch load for kSlots = 4)
template <int kSlots>
__device__ __forceinline__ int SlotReadLane(const int (&a)[kSlots], int s, int l) {
  int v = __builtin_amdgcn_readlane(a[0], l);
#pragma unroll
  for (int i = 1; i < kSlots; ++i) {
    const int x = __builtin_amdgcn_readlane(a[i], l);
    v = s == i ? x : v;
  }
  return v;
}

template <int kSlots>
__device__ __forceinline__ unsigned long long SlotReadLaneU64(const unsigned long long (&a)[kSlots], int s, int l) {
  unsigned long long v = ReadLaneU64(a[0], l);
#pragma unroll
  for (int i = 1; i < kSlots; ++i) {
    const unsigned long long x = ReadLaneU64(a[i], l);
    v = s == i ? x : v;
  }
  return v;
}

// kSlots: frontier entries per lane (entry e lives in lane e % 64, slot e / 64): 1 for num_leaves <= 64,
// 2 up to 128, 4 up to 256
template <int kSlots>
__global__ __launch_bounds__(kPlanThreads) void bplan_kernel(
    BState* __restrict__ bs, BNode* __restrict__ nodes, SplitResult* __restrict__ nbest,
    const SplitResult* __restrict__ fbest, int F, const double2* __restrict__ part, int E,
    const DLeaf* __restrict__ leaves, DState* __restrict__ st, DTree t, FeatMeta fm, const int8_t* __restrict__ mono,
    int has_mono, int first, int spec_k, int spec_max, int wide_div, int budget, int part_tile, int cap_nodes,
    int* __restrict__ host_flag, long long* __restrict__ prof) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  constexpr int kWaves = kPlanThreads / 64;
  // SML_BPLAN_PROF: thread 0 stamps the real-time clock at the phase boundaries (entry, absorbed, staged,
  // replayed, end) into prof[0..4]; prof[5] = pops replayed this round
  auto stamp = [&](int k) { if (prof != nullptr && tid == 0) prof[k] = static_cast<long long>(wall_clock64()); };
  stamp(0);
  __shared__ double s_gain[kBatchMaxNodes];
  __shared__ int s_c0[kBatchMaxNodes], s_c1[kBatchMaxNodes], s_pop[kBatchMaxNodes];
  __shared__ int p_node[kBatchMaxLeaves], p_li[kBatchMaxLeaves];
  __shared__ int ch_node[kMaxSpec];
  __shared__ long long s_cnt[kBatchMaxNodes];  // every node's global row count (the adaptive round width)
  __shared__ int s_rp[2], s_hdr[7];  // done, nnodes, nexp, cap_exp, expanded, spec_used, cap_nodes
  __shared__ int s_nb[kPlanFm], s_mt[kPlanFm], s_db[kPlanFm];
  // ---- phase 0: every load that does not depend on this round's header (done / nnodes / nexp) goes out
  // together - the header, the last round's expansion records and their children's per-feature best splits
  // (F <= 64 and 2 spec_k <= waves: one wave per child, lane f holding feature f's record in registers),
  // every node's gain and links up to the allocation's capacity, the committed replay prefix and the split
  // features' metadata - so the plan pays one memory round trip before the replay instead of four
  // (header -> records -> parent count / record copy -> node gains; r5 pass 22: absorb 3.0 + stage 1.9 us)
  // children go to waves 1.. (wave 0 replays right after the barrier; the others copy the winning records
  // into nbest after it, off the replay's path - the plan reads a child absorbed this round from fbest)
  // absorbing waves 1 .. kWaves - 1 take children cw and cw + kAbs (two each at 8 expansions per round)
  constexpr int kAbs = kWaves - 1;
  const bool fast = F <= 64 && spec_max <= kAbs;
  const int cw = wid - 1;  // fast path: this wave's first child
  __shared__ int s_src[kBatchMaxNodes];  // fbest record of a node absorbed this round (fast path), else -1
  int x_c0[2] = {0, 0}, x_c1[2] = {0, 0}, x_ls[2] = {0, 0}, x_pb[2] = {0, 0}, x_pc[2] = {0, 0};
  int x_buf[2] = {0, 0}, lt[2] = {0, 0};
  int64_t x_pg[2] = {0, 0}, small_cnt[2] = {0, 0};
  int rfeat[2] = {-1, -1};
  double rgain[2] = {-INFINITY, -INFINITY};
  auto load_exp = [&](int c, int q) {  // lane 0: child c's expansion record, cursor and smaller-child count
    const int j = c >> 1;
    const BExp& x = bs->exp[j];
    x_c0[q] = x.c0; x_c1[q] = x.c1; x_ls[q] = x.left_small;
    x_pb[q] = x.pbegin; x_pc[q] = x.pcount; x_buf[q] = x.pbuf; x_pg[q] = x.pgcount;
    lt[q] = static_cast<int>(bs->cursor[j * kCurStride] & 0xFFFFFFFFull);
    small_cnt[q] = static_cast<int64_t>(part[static_cast<size_t>(j) * (E + 1) + E].x);
  };
  if (first) {
    if (tid == 0) {
      const DLeaf R = leaves[0];
      BNode r;
      r.begin = R.begin; r.count = R.count; r.buf = R.buf; r.depth = 0;
      r.gcount = R.gcount; r.sum_g = R.sum_g; r.sum_h = R.sum_h; r.lo = -INFINITY; r.hi = INFINITY;
      r.out = RootLeafOutput(t, R.sum_g, R.sum_h); r.c0 = -1; r.c1 = -1;
      nodes[0] = r;
      bs->nexp = 0; bs->done = 0; bs->nnodes = 1; bs->expanded = 0; bs->spec_used = 0; bs->ntiles = 0;
      bs->cap_exp = 2 * budget + kMaxSpec;
      bs->cap_nodes = min(kBatchMaxNodes, 1 + 2 * bs->cap_exp);
      s_hdr[0] = 0; s_hdr[1] = 1; s_hdr[2] = 0;
      s_hdr[3] = 2 * budget + kMaxSpec; s_hdr[4] = 0; s_hdr[5] = 0;
      s_hdr[6] = min(kBatchMaxNodes, 1 + 2 * s_hdr[3]);
      s_c0[0] = -1; s_c1[0] = -1; s_pop[0] = -1; s_src[0] = -1;
      s_cnt[0] = R.gcount;
    }
    if (fast && cw == 0 && lane < F) { rfeat[0] = fbest[lane].feature; rgain[0] = fbest[lane].gain; }
  } else {
    if (tid == 0) {
      s_hdr[0] = bs->done; s_hdr[1] = bs->nnodes; s_hdr[2] = bs->nexp;
      s_hdr[3] = bs->cap_exp; s_hdr[4] = bs->expanded; s_hdr[5] = bs->spec_used; s_hdr[6] = bs->cap_nodes;
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c = cw + q * kAbs;
      if (fast && cw >= 0 && c < 2 * spec_max) {
        if (lane == 0) load_exp(c, q);
        if (lane < F) { rfeat[q] = fbest[c * F + lane].feature; rgain[q] = fbest[c * F + lane].gain; }
      }
    }
    for (int i = tid; i < cap_nodes; i += kPlanThreads) {
      const SplitResult& r = nbest[i];
      s_gain[i] = r.feature >= 0 ? r.gain : -INFINITY;
      s_c0[i] = nodes[i].c0;
      s_c1[i] = nodes[i].c1;
      s_cnt[i] = nodes[i].gcount;
      s_pop[i] = -1;
      s_src[i] = -1;
    }
  }
  const bool fm_lds = F <= kPlanFm;
  if (fm_lds)
    for (int f = tid; f < F; f += kPlanThreads) { s_nb[f] = fm.num_bin[f]; s_mt[f] = fm.missing[f]; s_db[f] = fm.default_bin[f]; }
  // the committed frontier (node, leaf index) goes straight into wave 0's registers
  int fn[kSlots], fl[kSlots];
#pragma unroll
  for (int q = 0; q < kSlots; ++q) { fn[q] = -1; fl[q] = 0; }
  if (!first) {
    if (tid == 0) { s_rp[0] = bs->rp_nf; s_rp[1] = bs->rp_pops; }
    // the prefix arrays are read whole-capacity-bounded by the stored counts after the barrier; loading
    // kBatchMaxLeaves entries regardless keeps this pass free of a dependent count load
    for (int i = tid; i < kBatchMaxLeaves; i += kPlanThreads) { p_node[i] = bs->rp_pnode[i]; p_li[i] = bs->rp_pli[i]; }
    if (wid == 0) {
#pragma unroll
      for (int q = 0; q < kSlots; ++q) { fn[q] = bs->rp_fnode[q * 64 + lane]; fl[q] = bs->rp_fli[q * 64 + lane]; }
    }
  } else if (lane == 0) {
    fn[0] = 0;  // the root, leaf 0
  }
  __syncthreads();
  if (s_hdr[0]) {
    if (tid == 0) { bs->nexp = 0; SetHostFlag(host_flag, 1); }
    return;
  }
  const int nnodes = s_hdr[1], nexp = s_hdr[2];
  // ---- absorb: the children of last round's expansions (first: the root) get their best splits, global
  // counts and row segments (ties: smaller feature); their gains go to the staged LDS table
  const int nchild = first ? 1 : 2 * nexp;
  auto child_id = [&](int c, int q) {
    const int small = x_ls[q] ? x_c0[q] : x_c1[q];
    return (c & 1) ? (small == x_c0[q] ? x_c1[q] : x_c0[q]) : small;
  };
  auto write_node = [&](int c, int id, int q) {
    BNode& nd = nodes[id];
    const bool is_left = id == x_c0[q];
    nd.begin = is_left ? x_pb[q] : x_pb[q] + lt[q];
    nd.count = is_left ? lt[q] : x_pc[q] - lt[q];
    nd.buf = x_buf[q] == 0 ? 1 : 0;
    nd.gcount = (c & 1) ? x_pg[q] - small_cnt[q] : small_cnt[q];
    s_cnt[id] = nd.gcount;
  };
  // fast path: the records this wave copies into nbest after the barrier
  int copy_src[2] = {-1, -1}, copy_id[2] = {0, 0};
  if (fast) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c = cw + q * kAbs;
      if (cw < 0 || c >= nchild) continue;
      // DPP argmax of the gain keys; equal gains -> the lowest lane = the smaller feature
      const bool valid = lane < F && rfeat[q] >= 0 && rgain[q] > -INFINITY;
      const unsigned long long key = valid ? GainKey(rgain[q]) : 0ull;
      const unsigned long long m = WaveMaxU64(key);
      const unsigned long long win = __ballot(valid && key == m);
      const int id = __builtin_amdgcn_readlane(first ? 0 : child_id(c, q), 0);  // x_* sit in lane 0
      if (lane == 0) {
        if (!first) write_node(c, id, q);
        if (m == 0) { nbest[id].feature = -1; nbest[id].gain = -INFINITY; s_gain[id] = -INFINITY; }
      }
      if (m != 0) {
        const int wl = static_cast<int>(__builtin_ctzll(win));
        if (lane == wl) { s_gain[id] = rgain[q]; s_src[id] = c * F + wl; }
        copy_src[q] = c * F + wl;
        copy_id[q] = id;
      }
    }
  } else {
    for (int c = wid; c < nchild; c += kWaves) {
      if (!first && lane == 0) load_exp(c, 0);
      KeyG k{-INFINITY, 1 << 30, 0};
      for (int f = lane; f < F; f += 64) {
        const SplitResult& r = fbest[c * F + f];
        if (r.feature < 0) continue;
        KeyG cand{r.gain, f, 0};
        if (KeyBetter(cand, k)) k = cand;
      }
      k = WaveArgmax(k);
      if (lane == 0) {
        const int id = first ? 0 : child_id(c, 0);
        if (!first) write_node(c, id, 0);
        if (k.gain == -INFINITY) {
          nbest[id].feature = -1;
          nbest[id].gain = -INFINITY;
        } else {
          nbest[id] = fbest[c * F + k.a];
        }
        s_gain[id] = k.gain;
      }
    }
  }
  stamp(1);
  __syncthreads();
  stamp(2);
  if (wid != 0) {
    static_assert(sizeof(SplitResult) % 4 == 0, "SplitResult copied as dwords");
#pragma unroll
    for (int q = 0; q < 2; ++q)
      if (copy_src[q] >= 0 && lane < static_cast<int>(sizeof(SplitResult) / 4))
        reinterpret_cast<uint32_t*>(nbest + copy_id[q])[lane] =
            reinterpret_cast<const uint32_t*>(fbest + copy_src[q])[lane];
    return;
  }
  // ---- replay of the sequential best-first growth (one wave), resumed at the committed prefix. The frontier
  // lives in registers (entry e: lane e % 64, slot e / 64) with each entry's gain and children, so a pop is
  // a DPP argmax + v_readlane of the winner and one broadcast LDS read of its children - no LDS round trip
  // for the frontier itself (the LDS-array replay cost ~1.1 us per pop, 8 us of a 15.6 us plan; r5 pass 22)
  int nf = 1, pops = 0, nch = 0;
  if (!first) {
    nf = s_rp[0];
    pops = s_rp[1];
    for (int i = lane; i < pops; i += 64) s_pop[p_node[i]] = i;
  }
  // fk: the entry's gain as an order-preserving key (GainKey), 0 for no candidate (-inf / NaN gain, or a slot
  // past the frontier), so the argmax needs no per-pop validity test
  unsigned long long fk[kSlots];
  int fc0[kSlots], fc1[kSlots];
  auto gkey = [](double g) { return g > -INFINITY ? GainKey(g) : 0ull; };
#pragma unroll
  for (int q = 0; q < kSlots; ++q) {
    const bool in = q * 64 + lane < nf;
    const int v = in && fn[q] >= 0 && fn[q] < nnodes ? fn[q] : 0;  // out-of-range ids are caught when popped
    fk[q] = in ? gkey(s_gain[v]) : 0ull;
    fc0[q] = s_c0[v];
    fc1[q] = s_c1[v];
  }
  const int committed = pops;
  WaveSync();
  const long long c_start = prof != nullptr ? static_cast<long long>(__builtin_amdgcn_s_memtime()) : 0;
  const int spec_room = max(1, min(spec_k, s_hdr[3] - s_hdr[4]));
  const bool may_spec = s_hdr[5] < budget && nnodes + 2 * spec_k <= s_hdr[6];
  // adaptive width: past spec_k, keep taking the replay's next unexplored nodes (up to spec_max) while the
  // round's expansions hold at most 1 / wide_div of the rows - late rounds are latency-bound (5-40 us per
  // kernel whatever their size), so a wider round costs little and saves whole rounds
  const int wide_room = max(1, min(spec_max, s_hdr[3] - s_hdr[4]));
  const bool may_wide = wide_div > 0 && may_spec && nnodes + 2 * spec_max <= s_hdr[6];
  const long long wide_rows = wide_div > 0 ? s_cnt[0] / wide_div : 0;
  long long srows = 0;
  constexpr int kFrontCap = kSlots * 64 < kBatchMaxLeaves ? kSlots * 64 : kBatchMaxLeaves;
  while (pops < budget) {
    // the sequential argmax: larger gain, then smaller leaf index (leaf indices are distinct)
    unsigned long long key = fk[0];
    int bli = fl[0], bsl = 0;
#pragma unroll
    for (int q = 1; q < kSlots; ++q) {
      const unsigned long long kq = fk[q];
      if (kq > key || (kq == key && fl[q] < bli)) { key = kq; bli = fl[q]; bsl = q; }
    }
    const unsigned long long m = WaveMaxU64(key);
    if (m <= 0x8000000000000000ull) break;  // no entry, or the best gain is not > 0
    const unsigned long long tied = __ballot(key == m);
    int w;
    if (__popcll(tied) == 1) {
      w = static_cast<int>(__builtin_ctzll(tied));
    } else {  // equal gains: the smallest leaf index among them
      const int mli = WaveMinI32(key == m ? bli : INT_MAX);
      w = static_cast<int>(__builtin_ctzll(__ballot(key == m && bli == mli)));
    }
    const int ws = __builtin_amdgcn_readlane(bsl, w);
    const int v = SlotReadLane(fn, ws, w);
    const int li = SlotReadLane(fl, ws, w);
    const int a = SlotReadLane(fc0, ws, w);
    const int b = SlotReadLane(fc1, ws, w);
    if (v < 0 || v >= nnodes || nf > kFrontCap - 1) {  // invariant broken: stop (host raises), never fault
      if (lane == 0) { bs->done = 1; bs->nexp = 0; SetHostFlag(host_flag, 2); }
      return;
    }
    const bool explored = a >= 0;
    if (!explored && nch == 0) {
      // the first unexplored pop: everything before it is final, so commit the frontier and the pops
#pragma unroll
      for (int q = 0; q < kSlots; ++q)
        if (q * 64 + lane < nf) { bs->rp_fnode[q * 64 + lane] = fn[q]; bs->rp_fli[q * 64 + lane] = fl[q]; }
      for (int i = committed + lane; i < pops; i += 64) { bs->rp_pnode[i] = p_node[i]; bs->rp_pli[i] = p_li[i]; }
      if (lane == 0) { bs->rp_nf = nf; bs->rp_pops = pops; }
    }
    if (explored) {
      // the popped entry becomes child a (it keeps the leaf index), child b is appended with leaf pops + 1
      const int ua = a < nnodes ? a : 0, ub = b >= 0 && b < nnodes ? b : 0;
      // both children's gain and links in one LDS round trip: lanes < 32 read a's, the others b's (lane-varying
      // addresses keep the three reads vector and in flight together; wave-uniform ones were scalarized and
      // read one after the other), then v_readlane from lanes 0 and 32
      const int ux = lane < 32 ? ua : ub;
      const double gx = s_gain[ux];
      const int cx0 = s_c0[ux], cx1 = s_c1[ux];
      const unsigned long long ka = gkey(ReadLaneD(gx, 0)), kb = gkey(ReadLaneD(gx, 32));
      const int a0 = __builtin_amdgcn_readlane(cx0, 0), a1 = __builtin_amdgcn_readlane(cx1, 0);
      const int b0 = __builtin_amdgcn_readlane(cx0, 32), b1 = __builtin_amdgcn_readlane(cx1, 32);
      const int nl = nf & 63, ns = nf >> 6;
#pragma unroll
      for (int q = 0; q < kSlots; ++q) {
        if (q == ws && lane == w) { fn[q] = a; fk[q] = ka; fc0[q] = a0; fc1[q] = a1; }
        if (q == ns && lane == nl) { fn[q] = b; fl[q] = pops + 1; fk[q] = kb; fc0[q] = b0; fc1[q] = b1; }
      }
      if (lane == 0) { p_node[pops] = v; p_li[pops] = li; s_pop[v] = pops; }
      ++nf;
    } else {
      // the popped entry is replaced by the last one
      const int ll = (nf - 1) & 63, ls = (nf - 1) >> 6;
      const int xn = SlotReadLane(fn, ls, ll);
      const int xl = SlotReadLane(fl, ls, ll);
      const unsigned long long xk = SlotReadLaneU64(fk, ls, ll);
      const int x0 = SlotReadLane(fc0, ls, ll);
      const int x1 = SlotReadLane(fc1, ls, ll);
#pragma unroll
      for (int q = 0; q < kSlots; ++q) {
        if (q == ws && lane == w) { fn[q] = xn; fl[q] = xl; fk[q] = xk; fc0[q] = x0; fc1[q] = x1; }
        if (q == ls && lane == ll) fk[q] = 0;  // after the move: the last slot leaves the frontier
      }
      if (lane == 0) ch_node[nch] = v;
      --nf;
      ++nch;
      srows += s_cnt[v];
      const bool wide = may_wide && nch < wide_room && srows <= wide_rows;
      if ((nch >= spec_room && !wide) || !may_spec) { ++pops; break; }
    }
    ++pops;
    WaveSync();
  }
  WaveSync();
  stamp(3);
  if (prof != nullptr && tid == 0) {
    prof[5] = pops - committed;
    prof[6] = static_cast<long long>(__builtin_amdgcn_s_memtime()) - c_start;  // shader clocks of the pop loop
  }
  if (nch == 0 && prof != nullptr) {
    // profiling: every expanded node (children allocated) and the ones the sequential order never popped
    long long er = 0, wr = 0;
    int ec = 0, wc = 0;
    for (int i = lane; i < nnodes; i += 64) {
      if (s_c0[i] < 0) continue;
      const int cnt = nodes[i].count;
      er += cnt; ++ec;
      if (s_pop[i] < 0) { wr += cnt; ++wc; }
    }
    for (int off = 32; off > 0; off >>= 1) {
      er += __shfl_xor(er, off, 64); wr += __shfl_xor(wr, off, 64);
      ec += __shfl_xor(ec, off, 64); wc += __shfl_xor(wc, off, 64);
    }
    if (lane == 0) { prof[7] = er; prof[8] = wr; prof[9] = ec; prof[10] = wc; }
  }
  if (nch == 0) {
    // ---- the tree is final: write it in sequential numbering. Pop i = internal node i; its left child
    // keeps the popped leaf's index, its right child gets leaf index i + 1.
    const int nl = pops + 1;
    for (int i = lane; i < pops; i += 64) {
      const int v = p_node[i];
      const SplitResult sr = nbest[v];
      const BNode P = nodes[v];
      const int a = s_c0[v], b = s_c1[v];
      t.feat[i] = sr.feature;
      t.thr[i] = sr.threshold;
      t.dleft[i] = sr.default_left;
      t.is_cat[i] = sr.is_cat;
      for (int w = 0; w < 8; ++w) t.cat_bits[i * 8 + w] = sr.cat_bits[w];
      t.left[i] = s_pop[a] >= 0 ? s_pop[a] : ~p_li[i];
      t.right[i] = s_pop[b] >= 0 ? s_pop[b] : ~(i + 1);
      t.gain[i] = sr.gain;
      t.ival[i] = P.out;
      t.iweight[i] = sr.left_h + sr.right_h;
      t.icount[i] = P.gcount;
    }
    // leaves: the final frontier (every entry is a node never popped) plus, for a stump, the root
#pragma unroll
    for (int q = 0; q < kSlots; ++q) {
      if (q * 64 + lane >= nf) continue;
      const int v = fn[q], li = fl[q];
      const BNode L = nodes[v];
      t.lval[li] = L.out;
      t.lweight[li] = L.sum_h;
      t.lcount[li] = L.gcount;
      t.ldepth[li] = L.depth;
      if (t.lseg) t.lseg[li] = make_int4(L.begin, L.count, L.buf, v);
    }
    // parent of each leaf: the pop that created it (leaf index li of a child of pop i: left = p_li[i], right = i+1)
    for (int i = lane; i < pops; i += 64) {
      const int v = p_node[i];
      if (s_pop[s_c0[v]] < 0) t.lparent[p_li[i]] = i;
      if (s_pop[s_c1[v]] < 0) t.lparent[i + 1] = i;
    }
    if (lane == 0) {
      if (pops == 0) t.lparent[0] = -1;
      st->num_leaves = nl;
      st->done = 1;
      bs->done = 1;
      bs->nexp = 0;
      SetHostFlag(host_flag, 1);
    }
    stamp(4);
    return;
  }
  // ---- plan this round's expansions: ch_node[0] is the sequential learner's next split, the rest are
  // speculative (counted against the waste budget spec_used < budget)
  const int base = nnodes;
  if (lane < nch) {
    const int j = lane, v = ch_node[j];
    const int src = s_src[v];  // absorbed this round: its record is still being copied into nbest
    const SplitResult sr = src >= 0 ? fbest[src] : nbest[v];
    const BNode P = nodes[v];
    const int a = base + 2 * j, b = a + 1;
    BNode L = P, R = P;
    L.depth = R.depth = P.depth + 1;
    L.sum_g = sr.left_g; L.sum_h = sr.left_h; L.out = sr.left_out;
    R.sum_g = sr.right_g; R.sum_h = sr.right_h; R.out = sr.right_out;
    L.c0 = L.c1 = R.c0 = R.c1 = -1;
    const int mdir = (has_mono && !sr.is_cat) ? static_cast<int>(mono[sr.feature]) : 0;
    if (mdir != 0) {
      const double mid = (sr.left_out + sr.right_out) / 2.0;
      if (mdir < 0) { L.lo = fmax(L.lo, mid); R.hi = fmin(R.hi, mid); }
      else { L.hi = fmin(L.hi, mid); R.lo = fmax(R.lo, mid); }
    }
    nodes[a] = L;
    nodes[b] = R;
    nodes[v].c0 = a;
    nodes[v].c1 = b;
    BExp x;
    x.node = v; x.c0 = a; x.c1 = b;
    x.left_small = sr.left_cnt <= sr.right_cnt ? 1 : 0;
    x.pbegin = P.begin; x.pcount = P.count; x.pbuf = P.buf; x.pgcount = P.gcount;
    x.ps.feature = sr.feature;
    x.ps.is_cat = sr.is_cat;
    x.ps.dleft = sr.default_left;
    x.ps.thr = sr.threshold;
    x.ps.nb = fm_lds ? s_nb[sr.feature] : fm.num_bin[sr.feature];
    x.ps.mt = fm_lds ? s_mt[sr.feature] : fm.missing[sr.feature];
    x.ps.dbin = fm_lds ? s_db[sr.feature] : fm.default_bin[sr.feature];
    for (int w = 0; w < 8; ++w) x.cat[w] = sr.is_cat ? sr.cat_bits[w] : 0u;
    // first global tile: prefix over the expansions' tile counts
    const int nt = (P.count + part_tile - 1) / part_tile;
    int pre = nt;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {
      const int o = __shfl_up(pre, off, 64);
      if (lane >= off) pre += o;
    }
    x.tile0 = pre - nt;
    bs->exp[j] = x;
    bs->cursor[j * kCurStride] = 0ull;
    if (j == nch - 1) bs->ntiles = pre;
  }
  if (lane == 0) {
    bs->nexp = nch;
    bs->nnodes = base + 2 * nch;
    bs->expanded = s_hdr[4] + nch;
    bs->spec_used = s_hdr[5] + nch - 1;
    SetHostFlag(host_flag, 0);
  }
  stamp(4);
}

// One tile's rows in registers (the software-pipelined batched partition below keeps two).
template <int kPartRows>
struct PartRegs {
  int r[kPartRows];
  float2 v[kPartRows];
  uint32_t bin[kPartRows];
};

// Issue the loads of a tile: row ids + (g, h) (physical or ordered), then the split feature's bins. Branch-free
// as PartitionTile's (rows past the segment read its first position and are masked later).
// kIdx: the index-only partition (row ids move, g / h stay in the interleaved physical copy bhist gathers from)
template <int kPartRows, bool kIdx = false>
__device__ __forceinline__ void PartLoad(PartRegs<kPartRows>& t, int feature, int t0, int tv, int pbuf,
                                         const uint8_t* __restrict__ cbins, int64_t n, const int32_t* __restrict__ perm0,
                                         const int32_t* __restrict__ perm1, const float2* __restrict__ ogh0,
                                         const float2* __restrict__ ogh1, const float* __restrict__ g,
                                         const float* __restrict__ h) {
  const int tid = threadIdx.x;
  if (pbuf < 0) {
#pragma unroll
    for (int u = 0; u < kPartRows; ++u) {
      const int k = u * kPartThreads + tid;
      const int p = t0 + (k < tv ? k : 0);
      t.r[u] = p;
      if (!kIdx) t.v[u] = make_float2(g[p], h[p]);
    }
  } else {
    const int32_t* perm = pbuf == 0 ? perm0 : perm1;
    const float2* ogh = pbuf == 0 ? ogh0 : ogh1;
#pragma unroll
    for (int u = 0; u < kPartRows; ++u) {
      const int k = u * kPartThreads + tid;
      const int p = t0 + (k < tv ? k : 0);
      t.r[u] = perm[p];
      if (!kIdx) t.v[u] = ogh[p];
    }
  }
  const uint8_t* __restrict__ col = cbins + static_cast<size_t>(feature) * n;
#pragma unroll
  for (int u = 0; u < kPartRows; ++u) t.bin[u] = col[t.r[u]];
}

// Batched partition with the tile loop software-pipelined: the next tile's row / gradient / bin loads are
// issued before this tile claims its output ranges (the block-wide ballot count -> one returning atomic on
// the expansion's cursor -> barrier), so their memory latency overlaps the atomic's round trip and the
// scatter instead of following it. Output order inside a child is still the claim order (histograms are
// exact integer sums: nothing downstream depends on it).
template <int kPartRows, bool kIdx = false>
__device__ __forceinline__ void BatchedPartitionPipelined(
    BState* __restrict__ bs, int nexp, int tlo, int ntiles, const int* s_tile0, const int* s_pb, const int* s_pc,
    const int* s_pbuf, const PartSplit* s_ps, const uint32_t (*s_cat)[8], const uint8_t* __restrict__ cbins, int64_t n,
    const int32_t* __restrict__ perm0, const int32_t* __restrict__ perm1, const float2* __restrict__ ogh0,
    const float2* __restrict__ ogh1, int32_t* __restrict__ wperm0, int32_t* __restrict__ wperm1,
    float2* __restrict__ wogh0, float2* __restrict__ wogh1, const float* __restrict__ g, const float* __restrict__ h) {
  constexpr int kPartTile = kPartThreads * kPartRows;
  constexpr int kWaves = kPartThreads / 64;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  __shared__ int wl[kPartRows][kWaves];
  __shared__ int bases[2];
  const unsigned long long below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  auto locate = [&](int tile, int* j, int* t0, int* tv) {
    int q = 0;
    while (q + 1 < nexp && s_tile0[q + 1] <= tile) ++q;
    *j = q;
    *t0 = s_pb[q] + (tile - s_tile0[q]) * kPartTile;
    *tv = min(kPartTile, s_pb[q] + s_pc[q] - *t0);
  };
  int tile = tlo + static_cast<int>(blockIdx.x);
  if (tile >= ntiles) return;
  PartRegs<kPartRows> cur, nxt;
  int j, t0, tv;
  locate(tile, &j, &t0, &tv);
  PartLoad<kPartRows, kIdx>(cur, s_ps[j].feature, t0, tv, s_pbuf[j], cbins, n, perm0, perm1, ogh0, ogh1, g, h);
  for (;;) {
    const PartSplit ps = s_ps[j];
    int rl[kPartRows];
    unsigned lmask = 0;
#pragma unroll
    for (int u = 0; u < kPartRows; ++u) {
      const int k = u * kPartThreads + tid;
      const bool left = k < tv && DeviceGoesLeft(cur.bin[u], ps.nb, ps.mt, ps.dbin, ps.is_cat, ps.thr, ps.dleft, s_cat[j]);
      lmask |= left ? (1u << u) : 0u;
      const unsigned long long bl = __ballot(left);
      rl[u] = __popcll(bl & below);
      if (lane == 0) wl[u][wid] = __popcll(bl);
    }
    __syncthreads();
    if (tid == 0) {
      int tl = 0;
      for (int u = 0; u < kPartRows; ++u)
        for (int w = 0; w < kWaves; ++w) tl += wl[u][w];
      const int tr = tv - tl;
      const unsigned long long old = atomicAdd(&bs->cursor[j * kCurStride], static_cast<unsigned long long>(tl) |
                                                                   (static_cast<unsigned long long>(tr) << 32));
      bases[0] = s_pb[j] + static_cast<int>(old & 0xFFFFFFFFull);
      bases[1] = s_pb[j] + s_pc[j] - static_cast<int>(old >> 32) - tr;
    }
    // the next tile's loads go out while thread 0's atomic is in flight
    const int ntile = tile + static_cast<int>(gridDim.x);
    int nj = j, nt0 = 0, ntv = 0;
    if (ntile < ntiles) {
      locate(ntile, &nj, &nt0, &ntv);
      PartLoad<kPartRows, kIdx>(nxt, s_ps[nj].feature, nt0, ntv, s_pbuf[nj], cbins, n, perm0, perm1, ogh0, ogh1, g, h);
    }
    __syncthreads();
    const int lb = bases[0], rb = bases[1];
    const int pbuf = s_pbuf[j];
    int32_t* operm = pbuf == 0 ? wperm1 : wperm0;
    float2* oogh = pbuf == 0 ? wogh1 : wogh0;
    int run = 0;
#pragma unroll
    for (int u = 0; u < kPartRows; ++u) {
      int wb = 0, ut = 0;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) {
        const int c = wl[u][w];
        wb += w < wid ? c : 0;
        ut += c;
      }
      const int k = u * kPartThreads + tid;
      if (k < tv) {
        const int lbefore = run + wb + rl[u];
        const int dst = (lmask >> u) & 1u ? lb + lbefore : rb + (k - lbefore);
        if (kIdx) {
          operm[dst] = cur.r[u];
        } else if (c_part_wt) {
          __hip_atomic_store(operm + dst, cur.r[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(reinterpret_cast<unsigned long long*>(oogh + dst),
                             (static_cast<unsigned long long>(__float_as_uint(cur.v[u].y)) << 32) |
                                 __float_as_uint(cur.v[u].x),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          operm[dst] = cur.r[u];
          oogh[dst] = cur.v[u];
        }
      }
      run += ut;
    }
    if (ntile >= ntiles) break;
    __syncthreads();  // wl / bases are rewritten by the next tile
    tile = ntile;
    j = nj;
    t0 = nt0;
    tv = ntv;
    cur = nxt;
  }
}

template <int kPartRows, bool kIdx = false>
__global__ __launch_bounds__(kPartThreads) void bpart_kernel(
    BState* __restrict__ bs, const uint8_t* __restrict__ cbins, int64_t n, const int32_t* __restrict__ perm0,
    const int32_t* __restrict__ perm1, const float2* __restrict__ ogh0, const float2* __restrict__ ogh1,
    int32_t* __restrict__ wperm0, int32_t* __restrict__ wperm1, float2* __restrict__ wogh0,
    float2* __restrict__ wogh1, const float* __restrict__ g, const float* __restrict__ h, int j0, int j1) {
  // expansions [j0, j1) of the round (the overlapped form partitions a round in two launches on two streams)
  const int nexp = bs->nexp;
  const int jb = min(j1, nexp);
  if (j0 >= jb) return;
  const int tlo = j0 == 0 ? 0 : bs->exp[j0].tile0;
  const int ntiles = jb < nexp ? bs->exp[jb].tile0 : bs->ntiles;
  if (tlo + static_cast<int>(blockIdx.x) >= ntiles) return;
  __shared__ int s_tile0[kMaxSpec], s_pb[kMaxSpec], s_pc[kMaxSpec], s_pbuf[kMaxSpec];
  __shared__ PartSplit s_ps[kMaxSpec];
  __shared__ uint32_t s_cat[kMaxSpec][8];
  const int tid = threadIdx.x;
  // every expansion's partition parameters staged once (the tile loop then starts its row loads without a
  // dependent read of the expansion record)
  if (tid < nexp) {
    const BExp& x = bs->exp[tid];
    s_tile0[tid] = x.tile0; s_pb[tid] = x.pbegin; s_pc[tid] = x.pcount; s_pbuf[tid] = x.pbuf; s_ps[tid] = x.ps;
  }
  if (tid < nexp * 8) s_cat[tid >> 3][tid & 7] = bs->exp[tid >> 3].cat[tid & 7];
  __syncthreads();
  if (kIdx || c_part_pipe) {  // the index-only partition has the pipelined form only
    BatchedPartitionPipelined<kPartRows, kIdx>(bs, nexp, tlo, ntiles, s_tile0, s_pb, s_pc, s_pbuf, s_ps, s_cat, cbins,
                                               n, perm0, perm1, ogh0, ogh1, wperm0, wperm1, wogh0, wogh1, g, h);
    return;
  }
  for (int tile = tlo + static_cast<int>(blockIdx.x); tile < ntiles; tile += gridDim.x) {
    int j = 0;
    while (j + 1 < nexp && s_tile0[j + 1] <= tile) ++j;
    const PartSplit ps = s_ps[j];
    PartitionTile<kPartRows>(ps, s_cat[j], tile - s_tile0[j], s_pb[j], s_pc[j], s_pbuf[j], &bs->cursor[j * kCurStride], cbins, n,
                             perm0, perm1, ogh0, ogh1, wperm0, wperm1, wogh0, wogh1, g, h);
  }
}

// kIdx: the index-only partition (row ids in the segments; `g` = the interleaved (g, h) copy, gathered per row)
template <int kUnroll, int kFPG, bool kPipe = false, bool kTight = false, bool kIdx = false>
__global__ __launch_bounds__(kHistBlockThreads) void bhist_kernel(
    const BState* __restrict__ bs, const uint4* __restrict__ bins4, int W4, int F, const int32_t* __restrict__ perm0,
    const int32_t* __restrict__ perm1, const float2* __restrict__ ogh0, const float2* __restrict__ ogh1,
    const float* __restrict__ g, const float* __restrict__ h, const float* __restrict__ ghmax,
    ulonglong2* __restrict__ slab, int64_t scale_n, int j0, int j1) {
  // expansions [j0, j1): their block budget (BatchHistAlloc over the subset) and slabs from `slab` on
  const int nexp = bs->nexp;
  const int jb = min(j1, nexp);
  if (j0 >= jb) return;
  const int m = jb - j0;
  __shared__ int s_cnt[kMaxSpec], s_nb[kMaxSpec], s_off[kMaxSpec];
  // the expansions' counts load in parallel (one thread each: one memory latency, not nexp in a row)
  if (threadIdx.x < m) s_cnt[threadIdx.x] = BatchSmallCount(bs, j0 + threadIdx.x);
  __syncthreads();
  if (threadIdx.x == 0) BatchHistAlloc(s_cnt, m, s_nb, s_off);
  __syncthreads();
  const int bx = blockIdx.x;
  int q = -1;
  for (int k = 0; k < m; ++k) if (bx >= s_off[k] && bx < s_off[k] + s_nb[k]) q = k;
  if (q < 0) return;
  const int j = j0 + q;
  const BExp& x = bs->exp[j];
  const int lt = static_cast<int>(bs->cursor[j * kCurStride] & 0xFFFFFFFFull);
  const int begin = x.left_small ? x.pbegin : x.pbegin + lt;
  HistBody<kUnroll, kFPG, kPipe, kTight, kIdx>(begin, s_cnt[q], x.pbuf == 0 ? 1 : 0, s_nb[q], bx - s_off[q], bins4, W4, F,
                                               perm0, perm1, ogh0, ogh1, g, h, ghmax,
                                               slab + static_cast<size_t>(bx) * F * kBinsPerFeature, scale_n);
}

// grid (ceil(E / kRedE), spec_k): block (x, j) reduces the slabs of expansion j into part[j * (E + 1) ..]
__global__ __launch_bounds__(kRedE * kRedG) void breduce_kernel(const BState* __restrict__ bs,
                                                                 const ulonglong2* __restrict__ slab, int E,
                                                                 const float* __restrict__ ghmax,
                                                                 double2* __restrict__ part, int64_t scale_n,
                                                                 int i64_out, int js) {
  const int nexp = bs->nexp;
  const float gmax_g = ghmax[0], gmax_h = ghmax[1];  // with the count: not a late dependent load
  const int j = blockIdx.y;
  if (j >= nexp) return;
  // js > 0: the round's histograms came from two launches, expansions [0, js) with slabs from block 0 and
  // [js, nexp) with slabs from block kMaxHistBlocks - each subset's own block budget
  const bool hi = js > 0 && j >= js;
  const int sj0 = hi ? js : 0, sj1 = js > 0 && !hi ? min(js, nexp) : nexp;
  const int m = sj1 - sj0;
  const int tid = threadIdx.x, le = tid % kRedE, grp = tid / kRedE;
  __shared__ int s_cnt[kMaxSpec], s_nb[kMaxSpec], s_off[kMaxSpec];
  if (tid < m) s_cnt[tid] = BatchSmallCount(bs, sj0 + tid);  // in parallel, as in bhist_kernel
  __syncthreads();
  if (tid == 0) BatchHistAlloc(s_cnt, m, s_nb, s_off);
  __syncthreads();
  const int count = s_cnt[j - sj0];
  const int nbj = s_nb[j - sj0], offj = s_off[j - sj0] + (hi ? kMaxHistBlocks : 0);
  const int e = blockIdx.x * kRedE + le;
  const bool valid = e < E;
  unsigned long long sg = 0, sh = 0;
  if (valid) {
    const ulonglong2* sl = slab + static_cast<size_t>(offj) * E;
#pragma unroll 8
    for (int b = grp; b < nbj; b += kRedG) {
      const ulonglong2 v = sl[static_cast<size_t>(b) * E + e];
      sg += v.x;
      sh += v.y;
    }
  }
  __shared__ unsigned long long rg[kRedG][kRedE], rh[kRedG][kRedE];
  rg[grp][le] = sg;
  rh[grp][le] = sh;
  __syncthreads();
  double2* out = part + static_cast<size_t>(j) * (E + 1);
  if (grp == 0 && valid) {
    unsigned long long tg = 0, th = 0;
#pragma unroll
    for (int k = 0; k < kRedG; ++k) { tg += rg[k][le]; th += rh[k][le]; }
    const int F = E / kBinsPerFeature;
    const int bin = e / F, f = e - bin * F;
    if (i64_out) {
      reinterpret_cast<ulonglong2*>(out)[f * kBinsPerFeature + bin] = make_ulonglong2(tg, th);
    } else {
      const HScale s = HistScaleV(scale_n, gmax_g, gmax_h);
      out[f * kBinsPerFeature + bin] = make_double2(static_cast<double>(static_cast<long long>(tg)) * s.ig,
                                                    static_cast<double>(static_cast<long long>(th)) * s.ih);
    }
  }
  if (blockIdx.x == 0 && tid == 0) {
    if (i64_out) reinterpret_cast<ulonglong2*>(out)[E] = make_ulonglong2(static_cast<unsigned long long>(count), 0ull);
    else out[E] = make_double2(static_cast<double>(count), 0.0);
  }
}

// grid (F, 2 * spec_k): block (f, 2j + c) searches feature f of expansion j's smaller (c = 0) or larger (c = 1)
// child; the larger child's histogram is the parent's minus the smaller's. Both go to the pool (slot = node id).
__global__ __launch_bounds__(256) void bfind_kernel(const BState* __restrict__ bs, const BNode* __restrict__ nodes,
                                                    const double2* __restrict__ part, int E,
                                                    double2* __restrict__ hist_pool, FeatMeta fm, SplitParams sp,
                                                    SplitResult* __restrict__ fbest, int F) {
  const int j = blockIdx.y >> 1, c = blockIdx.y & 1;
  const int f = blockIdx.x, tid = threadIdx.x;
  // the expansion record and this feature's reduced bins load together with the expansion count (all
  // within their buffers for any j < spec_k); the guard comes after, so the loads are not serialized behind it
  const int nexp = bs->nexp;
  const BExp x = bs->exp[j];
  const double2* pj = part + static_cast<size_t>(j) * (E + 1);
  const int e = f * kBinsPerFeature + tid;
  const double2 sm = pj[e];
  if (j >= nexp) return;
  const int small = x.left_small ? x.c0 : x.c1;
  const int child = c == 0 ? small : (small == x.c0 ? x.c1 : x.c0);
  double2 mine = sm;
  if (c == 1) {
    const double2 par = hist_pool[static_cast<size_t>(x.node) * E + e];
    mine = make_double2(par.x - sm.x, par.y - sm.y);
  }
  hist_pool[static_cast<size_t>(child) * E + e] = mine;
  const BNode nd = nodes[child];
  const int64_t small_cnt = static_cast<int64_t>(pj[E].x);
  const int64_t cnt = c == 0 ? small_cnt : x.pgcount - small_cnt;
  SearchFeatureBlock(mine, nd.sum_g, nd.sum_h, cnt, nd.depth, 0, nd.lo, nd.hi, f, F, fm, sp,
                     fbest + static_cast<size_t>(blockIdx.y) * F + f, true);
}

// ---------------------------------------------------------------- K7
// Node = one int4 {feature | missing<<16 | default_left<<18 | is_cat<<19 |
// missing_bin<<20, threshold bin, left, right}, staged in LDS. A thread loads
// its row's packed bins once (the row-major copy: two dwordx4 for up to 32
// features, coalesced across the wave) and walks the tree in registers, so a
// level costs a few ALU ops instead of a dependent, lane-divergent global
// load. kScoreRows rows per thread keep several row loads in flight. Rows
// with more than 32 features fall back to the column-major copy.
constexpr int kScoreRows = 2;
constexpr int kScoreThreads = 256;
// Nodes staged in LDS (trees up to 257 leaves; larger ones walk the global copy). 6 KB of LDS per block
// instead of 34 KB: the LDS no longer caps the streaming kernel at 4 blocks per CU.
constexpr int kScoreLdsNodes = 256;

struct DevTreeView {
  const int4* nodes;
  const uint32_t* cat_bits;  // 8 words per node
  const double* lval;
  int num_leaves;
};

constexpr int kPrepMaxNodes = 255;  // device-tree score updates: trees up to 256 leaves (nodes + values in LDS)

// The tree just grown, read where it was built (TrainTreeAndUpdateScore): nodes are encoded as
// UploadTree encodes them on the host, leaf values are lval * shrink (the host's Tree::Shrink).
struct DevTreeSrc {
  DTree t;
  const DState* st;  // final state version (num_leaves); nullptr: use the uploaded DevTreeView
  const int32_t* num_bin;
  const int32_t* missing;
  const int32_t* default_bin;
  double shrink;
};

__device__ __forceinline__ void StageDeviceTree(const DevTreeSrc& src, int num_leaves, int4* snodes, double* slval,
                                                int tid, int nthreads) {
  for (int i = tid; i < num_leaves - 1; i += nthreads) {
    const int f = src.t.feat[i], ic = src.t.is_cat[i] ? 1 : 0;
    const int mt = ic ? kMissingNaN : src.missing[f];
    const int dl = ic ? 0 : (src.t.dleft[i] ? 1 : 0);
    const int mbin = mt == kMissingNaN ? src.num_bin[f] - 1 : (mt == kMissingZero ? src.default_bin[f] : 0);
    snodes[i] = make_int4(f | (mt << 16) | (dl << 18) | (ic << 19) | (mbin << 20), static_cast<int>(src.t.thr[i]),
                          src.t.left[i], src.t.right[i]);
  }
  for (int i = tid; i < num_leaves; i += nthreads) slval[i] = src.t.lval[i] * src.shrink;
}

// Byte f (0..31) of a 32-byte row held in registers: one v_perm_b32 per dword pair picks byte f & 7 of that
// pair, and two levels of opaque-mask selects (bits 3 and 4 of f) pick the pair - 10 VALU, no VCC hazards
// (the nested ternary compiled to a 7-deep compare / cndmask / s_nop chain per tree-walk step).
__device__ __forceinline__ uint32_t ByteOfRow(const uint4& a, const uint4& b, int f) {
  const uint32_t sel = 0x0C0C0C00u | (static_cast<uint32_t>(f) & 7u);
  const uint32_t p0 = __builtin_amdgcn_perm(a.y, a.x, sel);
  const uint32_t p1 = __builtin_amdgcn_perm(a.w, a.z, sel);
  const uint32_t p2 = __builtin_amdgcn_perm(b.y, b.x, sel);
  const uint32_t p3 = __builtin_amdgcn_perm(b.w, b.z, sel);
  const uint32_t m3 = BitMask<3>(static_cast<uint32_t>(f)), m4 = BitMask<4>(static_cast<uint32_t>(f));
  return SelBits(m4, SelBits(m3, p3, p2), SelBits(m3, p1, p0));
}

// One tree-walk step. Numerical nodes are decided branch-free (the missing-bin test folded in with masks: a
// nested if / else if compiled to exec-mask juggling around every step); only categorical nodes, whose bitset
// lives in global memory, take a branch.
__device__ __forceinline__ int NodeStep(const int4& nd, uint32_t b, const uint32_t* cat_bits, int node) {
  const uint32_t x = static_cast<uint32_t>(nd.x);
  uint32_t left;
  if (__builtin_expect((x >> 19) & 1u, 0)) {
    const uint32_t* cb = cat_bits + node * 8;
    left = (cb[b >> 5] >> (b & 31)) & 1u;
  } else {
    const uint32_t miss = static_cast<uint32_t>(((x >> 16) & 3u) != kMissingNone) &
                          static_cast<uint32_t>(b == ((x >> 20) & 511u));
    const uint32_t le = static_cast<uint32_t>(b <= static_cast<uint32_t>(nd.y));
    left = (le & (miss ^ 1u)) | ((x >> 18) & miss);
  }
  return left ? nd.z : nd.w;
}

__global__ __launch_bounds__(kScoreThreads) void score_kernel(DevTreeView tv, DevTreeSrc src,
                                                              const uint4* __restrict__ bins4, int W4,
                                                              int F, const uint8_t* __restrict__ cbins, int64_t n,
                                                              double scale, double* __restrict__ score,
                                                              int32_t* __restrict__ leaf_out,
                                                              const uint8_t* __restrict__ row_leaf = nullptr) {
  __shared__ int4 snodes[kScoreLdsNodes];
  __shared__ double slv[kPrepMaxNodes + 1];
  if (src.st) {  // the tree just grown, straight from the device arrays (TrainTreeAndUpdateScore)
    tv.num_leaves = src.st->num_leaves;
    tv.cat_bits = src.t.cat_bits;
    tv.lval = slv;
    StageDeviceTree(src, tv.num_leaves, snodes, slv, threadIdx.x, kScoreThreads);
  }
  const int ni = tv.num_leaves - 1;
  const bool lds = ni <= kScoreLdsNodes;
  if (lds && !src.st)
    for (int i = threadIdx.x; i < ni; i += kScoreThreads) snodes[i] = tv.nodes[i];
  __syncthreads();
  const int4* nodes = lds ? snodes : tv.nodes;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kScoreThreads;
  const int64_t i0 = static_cast<int64_t>(blockIdx.x) * kScoreThreads + threadIdx.x;
  const bool packed = F <= 32;
  int leaf[kScoreRows];
  if (row_leaf) {  // every row's leaf from the scattered map (batched growth, no bag): no walk, no bin loads
#pragma unroll
    for (int u = 0; u < kScoreRows; ++u) {
      const int64_t i = i0 + u * stride;
      leaf[u] = i < n ? row_leaf[i] : 0;
    }
  } else if (packed) {
    uint4 ra[kScoreRows], rb[kScoreRows];
    if (ni > 0) {  // branch-free row loads (rows past n read row 0; their results are not stored)
#pragma unroll
      for (int u = 0; u < kScoreRows; ++u) {
        const int64_t i = i0 + u * stride;
        const int64_t iq = i < n ? i : 0;
        ra[u] = bins4[iq * W4];
        rb[u] = bins4[F > 16 ? iq * W4 + 1 : iq * W4];
        if (F <= 16) rb[u] = make_uint4(0, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int u = 0; u < kScoreRows; ++u) { ra[u] = make_uint4(0, 0, 0, 0); rb[u] = ra[u]; }
    }
#pragma unroll
    for (int u = 0; u < kScoreRows; ++u) {
      int node = ni > 0 ? 0 : ~0;
      for (int guard = 0; node >= 0 && guard < tv.num_leaves; ++guard) {
        const int4 nd = nodes[node];
        node = NodeStep(nd, ByteOfRow(ra[u], rb[u], nd.x & 0xFFFF), tv.cat_bits, node);
      }
      leaf[u] = ni > 0 ? ~node : 0;
    }
  } else {
#pragma unroll
    for (int u = 0; u < kScoreRows; ++u) {
      const int64_t i = i0 + u * stride;
      int node = (ni > 0 && i < n) ? 0 : ~0;
      for (int guard = 0; node >= 0 && guard < tv.num_leaves; ++guard) {
        const int4 nd = nodes[node];
        node = NodeStep(nd, cbins[static_cast<size_t>(nd.x & 0xFFFF) * n + i], tv.cat_bits, node);
      }
      leaf[u] = ni > 0 ? ~node : 0;
    }
  }
#pragma unroll
  for (int u = 0; u < kScoreRows; ++u) {
    const int64_t i = i0 + u * stride;
    if (i < n) {
      if (score) score[i] += scale * tv.lval[leaf[u]];
      if (leaf_out) leaf_out[i] = leaf[u];
    }
  }
}

// ---------------------------------------------------------------- K7 + K2 + root K3, one pass
// The score update of the tree just grown, the next iteration's gradients and
// the next tree's root histogram all walk every row in physical order and the
// first and last read the same 32-B bin row, so one kernel does all three:
// per row it walks the tree on the row's bins (nodes + leaf values staged in
// LDS), adds scale * leaf value to the score, evaluates the objective on the
// new score, stores g and h, and accumulates the 64-bit fixed-point (g, h) into
// the block's LDS histogram exactly as hist_kernel does for the root. The
// grid/chunk decomposition is hist_kernel's root decomposition (HistBlocks(n)
// blocks of ceil(n / blocks) contiguous rows), so hist_reduce_kernel reduces
// these slabs unchanged. The fixed-point scale cannot wait for this pass's
// max |g| / max h, so it comes from an a-priori bound of the objective
// (binary: sigmoid * label weight * max weight, h <= sigmoid^2 / 4 * ...;
// cross-entropy: |g| <= w, h <= w / 4) stored in `bound`; the pass still emits
// the block maxima of |g| and h, which the rest of the tree's histograms use.
// Replaces score_kernel + grad_kernel + the root hist_kernel (150 + 54 + 131
// us at 11M x 28 on MI355X, three full passes over rows).

// kGH2: the gradients go to one interleaved (g, h) array (`g`, float2 per row) for the index-only partition
template <int kUnroll, bool kPipe = false, bool kTight = false, bool kGH2 = false>
__global__ __launch_bounds__(kHistBlockThreads) void score_grad_hist_kernel(
    DevTreeView tv, DevTreeSrc src, const uint4* __restrict__ bins4, int W4, int F, int32_t n, double scale,
    double* __restrict__ score, ObjParams p, const float* __restrict__ label, const float* __restrict__ weight,
    float* __restrict__ g, float* __restrict__ h, const float* __restrict__ bound, float* __restrict__ partial,
    ulonglong2* __restrict__ slab, int64_t scale_n, const uint8_t* __restrict__ row_leaf) {
  constexpr int kThreads = kHistBlockThreads;
  const int nb_active = HistBlocks(n);
  if (static_cast<int>(blockIdx.x) >= nb_active) return;
  constexpr uint32_t kHOff = kTight ? kHPlaneTight : kHPlaneApart;  // h plane above the g plane (HistBody)
  constexpr int kShWords = static_cast<int>(kHOff / 8) + kHistWords;
  __shared__ unsigned long long sh[kShWords];
  unsigned long long* shg = sh;
  unsigned long long* shh = sh + kHOff / 8;
  __shared__ int4 snodes[kPrepMaxNodes];
  __shared__ double slval[kPrepMaxNodes + 1];
  const int tid = threadIdx.x;
  const int num_leaves = src.st ? src.st->num_leaves : tv.num_leaves;
  const int ni = num_leaves - 1;
  const uint32_t* cat_bits = src.st ? src.t.cat_bits : tv.cat_bits;
  for (int i = tid; i < kShWords; i += kThreads) sh[i] = 0ull;
  uint32_t fo[8];
  SlotOffsets32(static_cast<uint32_t>(tid & 15), fo);
  if (src.st) {
    StageDeviceTree(src, num_leaves, snodes, slval, tid, kThreads);
  } else {
    for (int i = tid; i < ni; i += kThreads) snodes[i] = tv.nodes[i];
    for (int i = tid; i < num_leaves; i += kThreads) slval[i] = tv.lval[i];
  }
  __syncthreads();
  const int chunk = ceil_div_i(n, nb_active);
  const int p0 = blockIdx.x * chunk;
  const int p1 = min(n, p0 + chunk);
  const HScale sc = HistScale(scale_n, bound);
  const bool two = F > 16;
  const int rot = tid & 15;
  float mg = 0.f, mh = 0.f;
  // one row of the pass: walk the tree, update the score, gradients, histogram
  // row_leaf (batched growth, no bagging): every row's leaf in the tree just grown, scattered from the final
  // leaves' row segments by leaf_scatter_kernel - no per-row walk (the walk was ~68 of this pass's 236 us at
  // 11M x 28: a divergent loop of dependent LDS node reads; r6 pass 23)
  auto row = [&](int i, const uint4& r0, const uint4& r1, double sv, float yv, float wv, int lf) {
    int li = lf;
    if (!row_leaf) {
      int node = ni > 0 ? 0 : ~0;
      for (int guard = 0; node >= 0 && guard < num_leaves; ++guard) {
        const int4 nd = snodes[node];
        node = NodeStep(nd, ByteOfRow(r0, r1, nd.x & 0xFFFF), cat_bits, node);
      }
      li = ni > 0 ? ~node : 0;
    }
    const double sn = sv + scale * slval[li];
    score[i] = sn;
    float gg, hh;
    PointGradient(p, sn, yv, wv, &gg, &hh);
    if (kGH2) {
      reinterpret_cast<float2*>(g)[i] = make_float2(gg, hh);
    } else {
      g[i] = gg;
      h[i] = hh;
    }
    mg = fmaxf(mg, fabsf(gg));
    mh = fmaxf(mh, fabsf(hh));
    hist_accumulate_rot<32, kFeatPerGroup, kHOff>(shg, shh, r0, r1, QuantGH(make_float2(gg, hh), sc), rot, fo);
  };
  if constexpr (kPipe) {
    // the next step's bins / score / label / weight are loaded before this step's rows are processed
    constexpr int kStep = kThreads * kUnroll;
    auto load = [&](int base, uint4* b0, uint4* b1, double* s, float* y, float* w, int* lf) {
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int i = base + u * kThreads;
        const bool ok = i < p1;
        const size_t rb = static_cast<size_t>(ok ? i : p0) * W4;
        b0[u] = bins4[rb];
        b1[u] = two ? bins4[rb + 1] : make_uint4(0, 0, 0, 0);
        s[u] = ok ? score[i] : 0.0;
        y[u] = ok ? label[i] : 0.f;
        w[u] = ok && weight ? weight[i] : 1.f;
        lf[u] = ok && row_leaf ? row_leaf[i] : 0;
      }
    };
    uint4 b0[kUnroll], b1[kUnroll];
    double s[kUnroll];
    float y[kUnroll], w[kUnroll];
    int lf[kUnroll];
    int base = p0 + tid;
    load(base, b0, b1, s, y, w, lf);
    for (; base < p1; base += kStep) {
      uint4 n0[kUnroll], n1[kUnroll];
      double ns[kUnroll];
      float ny[kUnroll], nw[kUnroll];
      int nl[kUnroll];
      load(base + kStep, n0, n1, ns, ny, nw, nl);
#pragma unroll
      for (int u = 0; u < kUnroll; ++u)
        if (base + u * kThreads < p1) row(base + u * kThreads, b0[u], b1[u], s[u], y[u], w[u], lf[u]);
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        b0[u] = n0[u]; b1[u] = n1[u]; s[u] = ns[u]; y[u] = ny[u]; w[u] = nw[u]; lf[u] = nl[u];
      }
    }
  }
  for (int base = kPipe ? p1 : p0 + tid; base < p1; base += kThreads * kUnroll) {
    uint4 b0[kUnroll], b1[kUnroll];
    double s[kUnroll];
    float y[kUnroll], w[kUnroll];
    int iq[kUnroll], lf[kUnroll];
    // branch-free loads: rows past p1 read row p0 and are skipped below (no guarded load to wait out)
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int i = base + u * kThreads;
      iq[u] = i < p1 ? i : p0;
      const size_t rb = static_cast<size_t>(iq[u]) * W4;
      b0[u] = bins4[rb];
      b1[u] = bins4[two ? rb + 1 : rb];
      if (!two) b1[u] = make_uint4(0, 0, 0, 0);
      s[u] = score[iq[u]];
      y[u] = label[iq[u]];
      w[u] = 1.f;
      lf[u] = row_leaf ? row_leaf[iq[u]] : 0;
    }
    if (weight) {
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) w[u] = weight[iq[u]];
    }
    // (stepping the kUnroll rows' tree walks together measured slower - 274.8 -> 281.9 us, r4 pass 18 - the
    // extra live state spills at this kernel's 128-VGPR cap)
    // all 32 slots (b1 = 0 when F <= 16: bin 0 of unused slots): one code path keeps this kernel unspilled
#pragma unroll
    for (int u = 0; u < kUnroll; ++u)
      if (base + u * kThreads < p1) row(base + u * kThreads, b0[u], b1[u], s[u], y[u], w[u], lf[u]);
  }
  BlockMaxPartial(mg, mh, partial);  // ends with a block barrier before thread 0 stores
  __syncthreads();
  SlabWrite<kFeatPerGroup, kThreads>(slab + static_cast<size_t>(blockIdx.x) * F * kBinsPerFeature, shg, shh, F, 0, F,
                                     tid);
}

// Every row's leaf in the tree batched growth just finished, for the fused score pass. A node's row segment is
// intact only while it has no descendants (a descendant's partition rewrites part of its range in the node's
// own buffer), and a final leaf may have some: the speculative continuation of a round's replay can pop an
// explored node and expand its children, and that node can still end up a leaf. The nodes never expanded
// are the finest partition - their segments tile [0, n) and are intact - so each of them is labelled with the
// final leaf it lies under (climbing parent links to the first node that is a final leaf), and the table is
// sorted by segment begin for leaf_scatter_kernel.
constexpr int kLeafTableThreads = 1024;
__global__ __launch_bounds__(kLeafTableThreads) void leaf_table_kernel(const BState* __restrict__ bs,
                                                                      const BNode* __restrict__ nodes,
                                                                      const DState* __restrict__ st,
                                                                      const int4* __restrict__ lseg,
                                                                      int4* __restrict__ rtab, int* __restrict__ rcount) {
  __shared__ int s_par[kBatchMaxNodes], s_lab[kBatchMaxNodes];
  __shared__ int4 s_ent[kBatchMaxNodes];
  __shared__ int s_m;
  const int tid = threadIdx.x;
  const int nn = min(bs->nnodes, kBatchMaxNodes);
  const int nl = min(st->num_leaves, kBatchMaxLeaves);
  if (tid == 0) s_m = 0;
  for (int x = tid; x < nn; x += kLeafTableThreads) { s_par[x] = -1; s_lab[x] = -1; }
  __syncthreads();
  for (int x = tid; x < nn; x += kLeafTableThreads) {
    const int c0 = nodes[x].c0, c1 = nodes[x].c1;
    if (c0 >= 0 && c0 < nn) s_par[c0] = x;
    if (c1 >= 0 && c1 < nn) s_par[c1] = x;
  }
  for (int li = tid; li < nl; li += kLeafTableThreads) {
    const int v = lseg[li].w;
    if (v >= 0 && v < nn) s_lab[v] = li;
  }
  __syncthreads();
  for (int y = tid; y < nn; y += kLeafTableThreads) {
    const BNode b = nodes[y];
    if (b.c0 >= 0 || b.count <= 0) continue;  // expanded, or no local rows
    int z = y, guard = 0;
    while (z >= 0 && s_lab[z] < 0 && guard++ < kBatchMaxNodes) z = s_par[z];
    if (z < 0 || s_lab[z] < 0) continue;  // (a subtree of no final leaf: not reachable for a finished tree)
    const int k = atomicAdd(&s_m, 1);
    s_ent[k] = make_int4(b.begin, b.count, b.buf, s_lab[z]);
  }
  __syncthreads();
  const int m = s_m;
  for (int k = tid; k < m; k += kLeafTableThreads) {  // rank by begin (distinct: the segments tile [0, n))
    const int bk = s_ent[k].x;
    int r = 0;
    for (int q = 0; q < m; ++q) r += s_ent[q].x < bk ? 1 : 0;
    rtab[r] = s_ent[k];
  }
  if (tid == 0) *rcount = m;
}

// row_leaf[perm[buf][k]] = label of the table segment holding position k (buf < 0: the root's physical order)
__global__ __launch_bounds__(256) void leaf_scatter_kernel(const int4* __restrict__ rtab, const int* __restrict__ rcount,
                                                           const int32_t* __restrict__ perm0,
                                                           const int32_t* __restrict__ perm1, int32_t n,
                                                           uint8_t* __restrict__ row_leaf) {
  __shared__ int s_beg[kBatchMaxNodes], s_buf[kBatchMaxNodes], s_lab[kBatchMaxNodes];
  const int m = min(*rcount, kBatchMaxNodes);
  for (int i = threadIdx.x; i < m; i += blockDim.x) {
    const int4 e = rtab[i];
    s_beg[i] = e.x;
    s_buf[i] = e.z;
    s_lab[i] = e.w;
  }
  __syncthreads();
  if (m == 0) return;
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
    int lo = 0, hi = m - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_beg[mid] <= k) lo = mid; else hi = mid - 1;
    }
    const int buf = s_buf[lo];
    const int row = buf < 0 ? k : (buf == 0 ? perm0[k] : perm1[k]);
    row_leaf[row] = static_cast<uint8_t>(s_lab[lo]);
  }
}

// (g, h) <-> the interleaved copy the index-only partition's histograms gather from
__global__ void pack_gh_kernel(const float* __restrict__ g, const float* __restrict__ h, int64_t n,
                               float2* __restrict__ gh) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    gh[i] = make_float2(g[i], h[i]);
}

__global__ void unpack_gh_kernel(const float2* __restrict__ gh, int64_t n, float* __restrict__ g,
                                 float* __restrict__ h) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float2 v = gh[i];
    g[i] = v.x;
    h[i] = v.y;
  }
}

// row-major -> column-major bin copy (once per dataset)
// Four rows per thread: each 16-byte chunk of the four rows is read as one dwordx4 per row and every feature of
// the chunk leaves as one dword (the four rows' bins) - a byte load + byte store per (row, feature) ran at
// ~1.1 TB/s (606 us at 11M x 28, r6 pass 24). n % 4 != 0 (dword stores misaligned) takes the byte form.
__global__ void transpose_bins_kernel(const uint8_t* __restrict__ bins, int S, int F, int64_t n,
                                      uint8_t* __restrict__ cbins) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if ((n & 3) != 0 || (S & 15) != 0) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
      const uint8_t* row = bins + i * S;
      for (int f = 0; f < F; ++f) cbins[static_cast<size_t>(f) * n + i] = row[f];
    }
    return;
  }
  const int64_t nq = n >> 2;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < nq; q += stride) {
    const int64_t i0 = q << 2;
    const uint4* r = reinterpret_cast<const uint4*>(bins + i0 * S);
    const int cs = S >> 4;  // 16-byte chunks per row
    for (int c = 0; c * 16 < F; ++c) {
      uint4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = r[k * cs + c];
      const uint32_t* w0 = reinterpret_cast<const uint32_t*>(&v[0]);
      const uint32_t* w1 = reinterpret_cast<const uint32_t*>(&v[1]);
      const uint32_t* w2 = reinterpret_cast<const uint32_t*>(&v[2]);
      const uint32_t* w3 = reinterpret_cast<const uint32_t*>(&v[3]);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int f = c * 16 + j;
        if (f >= F) break;
        const int d = j >> 2, sh = (j & 3) * 8;
        const uint32_t out = ((w0[d] >> sh) & 0xFFu) | (((w1[d] >> sh) & 0xFFu) << 8) |
                             (((w2[d] >> sh) & 0xFFu) << 16) | (((w3[d] >> sh) & 0xFFu) << 24);
        *reinterpret_cast<uint32_t*>(cbins + static_cast<size_t>(f) * n + i0) = out;
      }
    }
  }
}

__global__ void fill_f64_kernel(double* __restrict__ s, int64_t n, double v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) s[i] = v;
}

__global__ void axpby_kernel(double* __restrict__ s, int64_t n, double a, double b) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    s[i] = a * s[i] + b;
}

// ---------------------------------------------------------------- backend
// Per-device cache of the backend's runtime objects that cost milliseconds to make and free (the stream, the
// 4 MB pinned readback buffer, the mapped flag ring): a process that fits repeatedly hands them from one
// backend to the next (create + destroy measured at ~1.5 ms + ~1.8 ms per fit; r6 pass 15).
struct BackendObjects {
  std::mutex mu;
  std::unordered_map<int, std::vector<hipStream_t>> streams;
  std::unordered_map<int, std::vector<void*>> pinned, flags;
  static constexpr size_t kKeep = 4;  // per device and kind

  static BackendObjects& Get() {
    static BackendObjects* p = new BackendObjects();  // never destroyed (teardown order)
    return *p;
  }
  template <class T>
  bool Take(std::unordered_map<int, std::vector<T>>& m, int dev, T* out) {
    std::lock_guard<std::mutex> lk(mu);
    auto& v = m[dev];
    if (v.empty()) return false;
    *out = v.back();
    v.pop_back();
    return true;
  }
  template <class T>
  bool Give(std::unordered_map<int, std::vector<T>>& m, int dev, T x) {
    std::lock_guard<std::mutex> lk(mu);
    auto& v = m[dev];
    if (v.size() >= kKeep) return false;
    v.push_back(x);
    return true;
  }
};

class GpuBackend : public TrainBackend {
 public:
  explicit GpuBackend(int dev) : dev_(dev) {}
  ~GpuBackend() override {
    static const bool prof = std::getenv("SML_RELEASE_PROF") != nullptr;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    const auto t0 = now();
    BackendObjects& cache = BackendObjects::Get();
    vsets_.clear();  // they sync on stream_ before it goes
    const auto t1 = now();
    if (stream_) {
      const bool idle = hipStreamSynchronize(stream_) == hipSuccess;
      if (!idle || !cache.Give(cache.streams, dev_, stream_)) (void)hipStreamDestroy(stream_);
    }
    const auto t2 = now();
    for (hipEvent_t e : ev_) if (e) (void)hipEventDestroy(e);
    if (ev_copy_) (void)hipEventDestroy(ev_copy_);
    if (ev_sync_) (void)hipEventDestroy(ev_sync_);
    for (hipEvent_t e : comm_ev_) if (e) (void)hipEventDestroy(e);
    const auto t3 = now();
    if (pinned_ && !cache.Give(cache.pinned, dev_, pinned_)) (void)hipHostFree(pinned_);
    const auto t4 = now();
    for (hipEvent_t e : bev_) if (e) (void)hipEventDestroy(e);
    if (bflag_host_ && !cache.Give(cache.flags, dev_, static_cast<void*>(bflag_host_))) (void)hipHostFree(bflag_host_);
    if (prof)
      std::fprintf(stderr, "~GpuBackend: vsets %.3f stream %.3f events %.3f pinned %.3f bflag %.3f ms\n", ms(t0, t1),
                   ms(t1, t2), ms(t2, t3), ms(t3, t4), ms(t4, now()));
    if (bprof_) {
      if (bprof_n_ > 0) {  // wall_clock64 ticks at 100 MHz: 10 ns
        std::fprintf(stderr, "bplan phases (us/round over %lld rounds): absorb %.2f stage %.2f replay %.2f plan %.2f "
                     "pops/round %.2f pop-loop clocks/round %.0f\n", bprof_n_, bprof_sum_[0] / bprof_n_ * 1e-2,
                     bprof_sum_[1] / bprof_n_ * 1e-2, bprof_sum_[2] / bprof_n_ * 1e-2, bprof_sum_[3] / bprof_n_ * 1e-2,
                     bprof_sum_[4] / bprof_n_, bprof_sum_[5] / bprof_n_);
      }
      if (bprof_trees_ > 0) {
        const double t = static_cast<double>(bprof_trees_);
        std::fprintf(stderr, "bplan trees %lld: expansions/tree %.2f (never popped %.2f), partitioned rows/tree %.0f "
                     "(in never-popped nodes %.0f)\n", bprof_trees_, bprof_tree_[2] / t, bprof_tree_[3] / t,
                     bprof_tree_[0] / t, bprof_tree_[1] / t);
      }
      (void)hipFree(bprof_);
    }
  }
  std::string Name() const override { return "hip"; }

  void Init(const Dataset* d, const Config& cfg, int K) override {
    TraceRange tr("sml::BackendInit");
    data_ = d; cfg_ = cfg; K_ = K; n_ = d->num_data;
    if (n_ >= (int64_t(1) << 31)) throw std::runtime_error("GPU backend: more than 2^31 rows per device");
    if (cfg.num_leaves > 4096) throw std::runtime_error("GPU backend: num_leaves > 4096");
    if (dev_ >= 0) SML_HIP_CHECK(hipSetDevice(dev_));
    SML_HIP_CHECK(hipGetDevice(&dev_));
    if (!BackendObjects::Get().Take(BackendObjects::Get().streams, dev_, &stream_))
      SML_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    sp_ = MakeSplitParams(cfg);
    ghmax_.alloc(2);  // max |g|, max h (float bits)
    ghmax_partial_.alloc(2 * kGhmaxBlocks);
    F_ = d->ref.num_inner();
    S_ = d->row_stride;
    W_ = S_ / 4;
    E_ = F_ * kBinsPerFeature;
    L_ = std::max(2, cfg.num_leaves);
    FG_ = (F_ + kFeatPerGroup - 1) / kFeatPerGroup;
    if (d->dev && d->dev_valid && d->dev->device == dev_) {
      // K1 left the bin matrix in HBM on this device: adopt it (no host round trip)
      dev_bins_ = d->dev;
      bins_ptr_ = dev_bins_->rows;
    } else {
      d->EnsureHostBins();
      bins_.alloc(static_cast<size_t>(n_) * S_);
      SML_HIP_CHECK(hipMemcpyAsync(bins_.get(), d->bins.data(), static_cast<size_t>(n_) * S_, hipMemcpyHostToDevice, stream_));
      bins_ptr_ = bins_.get();
    }
    cbins_.alloc(static_cast<size_t>(n_) * std::max(1, F_));
    hipLaunchKernelGGL(transpose_bins_kernel, dim3(GridFor(n_)), dim3(256), 0, stream_, bins_ptr_, S_, F_, n_,
                       cbins_.get());
    SML_HIP_CHECK(hipGetLastError());
    label_.alloc(n_);
    SML_HIP_CHECK(hipMemcpyAsync(label_.get(), d->label.data(), sizeof(float) * n_, hipMemcpyHostToDevice, stream_));
    if (!d->weight.empty()) {
      weight_.alloc(n_);
      SML_HIP_CHECK(hipMemcpyAsync(weight_.get(), d->weight.data(), sizeof(float) * n_, hipMemcpyHostToDevice, stream_));
    }
    score_.alloc(static_cast<size_t>(n_) * K);
    g_.alloc(static_cast<size_t>(n_) * K);
    h_.alloc(static_cast<size_t>(n_) * K);
    for (int b = 0; b < 2; ++b) { perm_[b].alloc(n_); ogh_[b].alloc(n_); }
    slab_.alloc(static_cast<size_t>(kMaxHistBlocks) * E_);
    // batched speculative growth (bplan_kernel ..): one-split-at-a-time stays for voting, bynode sampling,
    // num_leaves > 256 and SML_GBDT_SPEC=0; SML_GBDT_SPEC=k sets the expansions per round (default 4)
    // 4 expansions per round: r4 A/B at 11M x 28 (profiles/r4/gbdt2): spec 2 231 ms / fit, 4 217 ms, 8 247 ms,
    // one-split growth 250 ms - wider rounds mostly add never-popped expansions (the rounds follow the
    // parent -> child dependency chain of the pops, ~15 per tree at 31 leaves)
    // more leaves, wider rounds: r5 pass 48 (11M x 28, ms per iteration at spec 4 / 8 / 16): 63 leaves 2.10 /
    // 2.16 / 2.84, 127 leaves 3.24 / 2.94 / 3.77, 255 leaves 5.28 / 4.39 / 4.48 (the per-round fixed cost -
    // plan, reduce, split search, launch gaps - over ~L / 3.8 rounds outweighs the extra speculation)
    spec_k_ = L_ > 64 ? 8 : 4;
    if (const char* e = std::getenv("SML_GBDT_SPEC")) spec_k_ = std::atoi(e);
    batch_ok_ = spec_k_ > 0 && L_ <= kBatchMaxLeaves && !(cfg.tree_learner == "voting" && comm_ && comm_->world() > 1);
    spec_k_ = std::max(1, std::min(kMaxSpec, spec_k_));
    // adaptive round width (bplan_kernel): rounds whose expansions hold <= 1 / wide_div of the rows may take up
    // to spec_max expansions (SML_GBDT_WIDE=<divisor>, 0 = fixed width; SML_GBDT_SPEC_MAX caps it; <= 15, the
    // plan's absorbing waves)
    wide_div_ = 0;
    if (const char* e = std::getenv("SML_GBDT_WIDE")) wide_div_ = std::max(0, std::atoi(e));
    spec_max_ = wide_div_ > 0 ? 2 * spec_k_ : spec_k_;
    if (const char* e = std::getenv("SML_GBDT_SPEC_MAX")) spec_max_ = std::atoi(e);
    spec_max_ = std::max(spec_k_, std::min(std::min(kMaxSpec, kPlanThreads / 64 - 1), spec_max_));
    if (const char* e = std::getenv("SML_GBDT_LOOKAHEAD")) blook_ = std::max(1, std::min(4, std::atoi(e)));
    const int cap_nodes = std::min(kBatchMaxNodes, 1 + 2 * (2 * (L_ - 1) + kMaxSpec));
    // histogram + (row count, 0) per expansion of a round
    part_.alloc(static_cast<size_t>(E_ + 1) * (batch_ok_ ? kMaxSpec : 1));
    hist_pool_.alloc(static_cast<size_t>(std::max(2 * L_ + 2, batch_ok_ ? cap_nodes : 0)) * E_);
    if (batch_ok_) {
      bstate_.alloc(1);
      bnodes_.alloc(cap_nodes);
      plan_cap_ = cap_nodes;
      nbest_.alloc(cap_nodes);
      if (void* f = nullptr; BackendObjects::Get().Take(BackendObjects::Get().flags, dev_, &f))
        bflag_host_ = static_cast<int*>(f);
      else
        SML_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&bflag_host_), sizeof(int) * kBRing,
                                    hipHostMallocMapped | hipHostMallocCoherent));
      SML_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&bflag_dev_), bflag_host_, 0));
      if (const char* e = std::getenv("SML_BPLAN_PROF"); e != nullptr && std::atoi(e) != 0) {
        const size_t nb = sizeof(long long) * kPlanProfStride * (cfg.num_leaves + 3);
        SML_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&bprof_), nb));
        SML_HIP_CHECK(hipMemset(bprof_, 0, nb));
      }
      for (hipEvent_t& e : bev_) SML_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      // index-only partition (bpart_kernel<.., true>): the batched partition moves row ids only (4 + 4 B per row
      // instead of 12 + 12 with the ordered g / h) and bhist gathers each row's (g, h) from one interleaved
      // physical copy (gh2_, written by the fused score / gradient pass or packed once per tree); one class, no
      // bagging. SML_GBDT_IDX=0: the ordered-gradient partition.
      idx_ok_ = K == 1;
      if (const char* e = std::getenv("SML_GBDT_IDX")) idx_ok_ = idx_ok_ && std::atoi(e) != 0;
      if (idx_ok_) gh2_.alloc(n_);
    }
    // launch-shape knobs for A/B runs (defaults are the measured best)
    if (const char* e = std::getenv("SML_PART_ROWS")) part_rows_ = std::atoi(e);
    if (part_rows_ != 4 && part_rows_ != 8 && part_rows_ != 16) part_rows_ = kPartRowsDefault;
    if (const char* e = std::getenv("SML_HIST_MIN_ROWS")) {
      const int v = std::max(256, std::atoi(e));
      SML_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_min_rows_per_hist_block), &v, sizeof(int)));
    }
    if (const char* e = std::getenv("SML_PART_WT")) {
      const int v = std::atoi(e) != 0 ? 1 : 0;
      SML_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_part_wt), &v, sizeof(int)));
    }
    if (const char* e = std::getenv("SML_PART_PIPE")) {
      const int v = std::atoi(e) != 0 ? 1 : 0;
      SML_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_part_pipe), &v, sizeof(int)));
    }
    if (const char* e = std::getenv("SML_SLAB_WT")) {
      const int v = std::atoi(e) != 0 ? 1 : 0;
      SML_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_slab_wt), &v, sizeof(int)));
    }
    if (const char* e = std::getenv("SML_SKIP_LAST_SPLIT")) skip_last_ = std::atoi(e) != 0;
    if (const char* e = std::getenv("SML_GBDT_COMM_WORLD1")) comm_world1_ = std::atoi(e) != 0;
    if (const char* e = std::getenv("SML_HIST_FPG")) hist_fpg_ = std::atoi(e) == 16 ? 16 : kFeatPerGroup;
    if (const char* e = std::getenv("SML_HIST_UNROLL")) hist_unroll4_ = std::atoi(e) == 4;
    if (const char* e = std::getenv("SML_GBDT_HIST_PIPE")) hist_pipe_ = std::atoi(e) != 0;
    if (const char* e = std::getenv("SML_GBDT_ROOT_PIPE")) root_pipe_ = std::atoi(e) != 0;
    // overlapped LDS planes (kHPlaneTight) need every group's features below slot 28
    tight_ = F_ <= 28;
    if (const char* e = std::getenv("SML_HIST_TIGHT")) tight_ = tight_ && std::atoi(e) != 0;
    if (const char* e = std::getenv("SML_RANK_WAVES")) rank_waves_ = std::atoi(e) == 4 ? 4 : 1;
    if (const char* e = std::getenv("SML_RANK_TREDUCE")) rank_treduce_ = std::atoi(e) != 0;
    if (const char* e = std::getenv("SML_RANK_SPLIT")) rank_split_ = std::atoi(e) != 0;
    if (const char* e = std::getenv("SML_RANK_SMALL_WAVES")) rank_small_waves_ = std::atoi(e) == 4 ? 4 : 1;
    voting_ = cfg.tree_learner == "voting" && Distributed();
    if (voting_) {
      if (F_ > kVoteMaxF) throw std::runtime_error("GPU voting_parallel: more than 8192 features");
      vote_k2_ = std::max(1, std::min(2 * std::max(1, cfg.top_k), F_));
      sp_local_ = sp_;
      sp_local_.min_data_in_leaf = std::max(1, sp_.min_data_in_leaf / comm_->world());
      sp_local_.min_sum_hessian = sp_.min_sum_hessian / comm_->world();
      floc_.alloc(2 * F_);
      vote_.alloc(4 * static_cast<size_t>(F_) + 1);
      sel_idx_.alloc(2 * static_cast<size_t>(vote_k2_));
      sel_pos_.alloc(2 * static_cast<size_t>(F_));
      sel_mask_.alloc(2 * static_cast<size_t>(F_));
      compact_.alloc(2 * static_cast<size_t>(vote_k2_) * kBinsPerFeature);
      gh_.alloc(2 * static_cast<size_t>(E_));
    }
    {
      const int64_t tile = static_cast<int64_t>(kPartThreads) * part_rows_;
      part_grid_ = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(kMaxPartBlocks, (n_ + tile - 1) / tile)));
      // choose_part_kernel: every block pays the choose prologue, so keep the grid within one resident
      // round (A/B on MI355X, 11M x 28: 2048 blocks 2.09-2.10 ms/iter, 1024 1.99-2.01, 768 1.97-2.01, 512 2.01-2.04)
      {
        int per_cu = 0, cus = 0;
        auto ck = part_rows_ == 16 ? choose_part_kernel<16> : (part_rows_ == 4 ? choose_part_kernel<4> : choose_part_kernel<8>);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ck, kPartThreads, 0) == hipSuccess &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev_) == hipSuccess && per_cu > 0 && cus > 0)
          part_grid_ = std::max(1, std::min(part_grid_, per_cu * cus));
        else
          (void)hipGetLastError();
      }
      if (const char* e = std::getenv("SML_PART_GRID")) part_grid_ = std::max(1, std::min(part_grid_, std::atoi(e)));
    }
    if (const char* e = std::getenv("SML_HIST_MIN_ROWS")) min_rows_hist_ = std::max(256, std::atoi(e));
    {
      // score_grad_hist_kernel: one class, every row in every tree (no bagging / GOSS / RF / DART
      // rescaling between the score update and the next gradients), <= 32 features, row-per-lane slabs
      const bool sampled = cfg.boosting != "gbdt" ||
                           (cfg.bagging_freq > 0 && (cfg.bagging_fraction < 1.0 || cfg.pos_bagging_fraction < 1.0 ||
                                                     cfg.neg_bagging_fraction < 1.0));
      const char* e = std::getenv("SML_PREP");
      prep_ok_ = K == 1 && !sampled && F_ > 0 &&
                 F_ <= kFeatPerGroup &&
                 L_ <= kPrepMaxNodes + 1 && !(e && std::atoi(e) == 0);
      wmax_ = 1.0;
      if (!d->weight.empty()) {
        wmax_ = 0.0;
        for (float w : d->weight) wmax_ = std::max(wmax_, static_cast<double>(std::fabs(w)));
      }
      ymax_ = -1.0;  // max |label|: computed when a cross-entropy prep pass first needs it
      ghbound_.alloc(2);
    }
    // global quantities of the histogram scale (HistScaleV): the row-count bound and the objective bound's
    // max |weight| are the same on every rank, so the fixed-point histograms do not depend on the partitioning
    scale_n_ = n_;
    comm_bytes0_ = comm_ ? comm_->DeviceBytes() : 0;  // the (cached) communicator's count so far
    if (comm_ && comm_->world() > 1) {
      double c = static_cast<double>(n_);
      comm_->AllReduceHost(&c, 1);
      scale_n_ = static_cast<int64_t>(c);
      comm_->AllReduceHostMax(&wmax_, 1);
    }
    fbest_.alloc(static_cast<size_t>(2) * F_ * (batch_ok_ ? kMaxSpec : 1));
    lbest_.alloc(L_);
    lgain_.alloc(L_);
    leaves_.alloc(L_);
    // feature meta
    std::vector<int32_t> nb(F_), mt(F_), db(F_), ic(F_);
    for (int f = 0; f < F_; ++f) {
      const BinMapper& m = d->ref.mappers[d->ref.used_features[f]];
      nb[f] = m.num_bin; mt[f] = m.missing_type; db[f] = m.default_bin; ic[f] = m.is_categorical ? 1 : 0;
    }
    meta_i_.alloc(4 * F_);
    SML_HIP_CHECK(hipMemcpy(meta_i_.get(), nb.data(), sizeof(int32_t) * F_, hipMemcpyHostToDevice));
    SML_HIP_CHECK(hipMemcpy(meta_i_.get() + F_, mt.data(), sizeof(int32_t) * F_, hipMemcpyHostToDevice));
    SML_HIP_CHECK(hipMemcpy(meta_i_.get() + 2 * F_, db.data(), sizeof(int32_t) * F_, hipMemcpyHostToDevice));
    SML_HIP_CHECK(hipMemcpy(meta_i_.get() + 3 * F_, ic.data(), sizeof(int32_t) * F_, hipMemcpyHostToDevice));
    mask_.alloc(F_);
    {
      std::vector<int8_t> mono(F_, 0);
      for (int f = 0; f < F_; ++f) {
        const int col = d->ref.used_features[f];
        if (col < static_cast<int>(cfg.monotone_constraints.size()))
          mono[f] = static_cast<int8_t>(cfg.monotone_constraints[col] > 0 ? 1 : (cfg.monotone_constraints[col] < 0 ? -1 : 0));
      }
      mono_.alloc(F_);
      SML_HIP_CHECK(hipMemcpy(mono_.get(), mono.data(), F_, hipMemcpyHostToDevice));
    }
    fm_.num_bin = meta_i_.get(); fm_.missing = meta_i_.get() + F_; fm_.default_bin = meta_i_.get() + 2 * F_;
    fm_.is_cat = meta_i_.get() + 3 * F_; fm_.mask = mask_.get(); fm_.mono = mono_.get();
    // device tree
    const int NI = L_ - 1;
    // DState + the device tree live in one allocation so a finished tree comes
    // back with a single D2H copy
    n_ti_ = static_cast<size_t>(NI) * 6 + L_ * 2;
    n_tu_ = static_cast<size_t>(NI) * 9;
    n_td_ = static_cast<size_t>(NI) * 3 + L_ * 2;
    n_tl_ = static_cast<size_t>(NI) + L_;
    off_td_ = (2 * sizeof(DState) + 63) / 64 * 64;  // two DState versions (choose_part_kernel) + tree
    off_tl_ = off_td_ + n_td_ * sizeof(double);
    off_ti_ = off_tl_ + n_tl_ * sizeof(int64_t);
    off_tu_ = off_ti_ + n_ti_ * sizeof(int32_t);
    blob_bytes_ = off_tu_ + n_tu_ * sizeof(uint32_t);
    if (blob_bytes_ > kPinnedBytes) throw std::runtime_error("GPU backend: tree too large for staging buffer");
    blob_.alloc(blob_bytes_);
    state_ = reinterpret_cast<DState*>(blob_.get());
    st_cur_ = state_;
    int32_t* ti = reinterpret_cast<int32_t*>(blob_.get() + off_ti_);
    dt_.feat = ti; dt_.dleft = ti + NI; dt_.is_cat = ti + 2 * NI; dt_.left = ti + 3 * NI; dt_.right = ti + 4 * NI;
    dt_.lparent = ti + 6 * NI; dt_.ldepth = ti + 6 * NI + L_;
    flags_ = ti + 5 * NI;
    uint32_t* tu = reinterpret_cast<uint32_t*>(blob_.get() + off_tu_);
    dt_.thr = tu; dt_.cat_bits = tu + NI;
    double* td = reinterpret_cast<double*>(blob_.get() + off_td_);
    dt_.gain = td; dt_.ival = td + NI; dt_.iweight = td + 2 * NI; dt_.lval = td + 3 * NI; dt_.lweight = td + 3 * NI + L_;
    int64_t* tl = reinterpret_cast<int64_t*>(blob_.get() + off_tl_);
    dt_.icount = tl; dt_.lcount = tl + NI;
    dt_.out_l1 = sp_.lambda_l1; dt_.out_l2 = sp_.lambda_l2; dt_.out_mds = sp_.max_delta_step;
    dt_.lseg = nullptr;
    if (batch_ok_ && L_ <= kBatchMaxLeaves && row_leaf_on_) {
      lseg_.alloc(L_);
      row_leaf_.alloc(n_);
      rtab_.alloc(kBatchMaxNodes + 1);  // the sorted segment table, then its length
      dt_.lseg = lseg_.get();
    }
    // score-update tree (uploaded from host trees)
    up_blob_.alloc(static_cast<size_t>(NI + 1) * (16 + 32) + static_cast<size_t>(L_ + 4) * 8);
    leaf_idx_.alloc(n_);
    if (!BackendObjects::Get().Take(BackendObjects::Get().pinned, dev_, &pinned_))
      SML_HIP_CHECK(hipHostMalloc(&pinned_, kPinnedBytes, hipHostMallocDefault));
    for (hipEvent_t& e : ev_) SML_HIP_CHECK(hipEventCreate(&e));
    SML_HIP_CHECK(hipEventCreateWithFlags(&ev_copy_, hipEventDisableTiming));
    SML_HIP_CHECK(hipEventCreateWithFlags(&ev_sync_, hipEventDisableTiming));
    SML_HIP_CHECK(hipStreamSynchronize(stream_));
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) stats.device_mem_mb = (total_b - free_b) / 1048576.0;
  }

  void SetScores(const std::vector<double>& s) override {
    prep_valid_ = root_ready_ = false;
    SML_HIP_CHECK(hipMemcpyAsync(score_.get(), s.data(), sizeof(double) * s.size(), hipMemcpyHostToDevice, stream_));
    SML_HIP_CHECK(hipStreamSynchronize(stream_));
  }
  void FillScores(const std::vector<double>& per_class, int64_t n) override {
    prep_valid_ = root_ready_ = false;
    for (size_t k = 0; k < per_class.size(); ++k) {
      hipLaunchKernelGGL(fill_f64_kernel, dim3(GridFor(n)), dim3(256), 0, stream_, score_.get() + k * n, n,
                         per_class[k]);
      SML_HIP_CHECK(hipGetLastError());
    }
  }
  void GetScores(std::vector<double>* s) override {
    s->resize(static_cast<size_t>(n_) * K_);
    SML_HIP_CHECK(hipMemcpyAsync(s->data(), score_.get(), sizeof(double) * s->size(), hipMemcpyDeviceToHost, stream_));
    SML_HIP_CHECK(hipStreamSynchronize(stream_));
  }
  void AddBias(int k, double b) override {
    prep_valid_ = root_ready_ = false;
    hipLaunchKernelGGL(axpby_kernel, dim3(GridFor(n_)), dim3(256), 0, stream_, score_.get() + k * n_, n_, 1.0, b);
    SML_HIP_CHECK(hipGetLastError());
  }
  void ScaleScore(int k, double sc) override {
    prep_valid_ = root_ready_ = false;
    hipLaunchKernelGGL(axpby_kernel, dim3(GridFor(n_)), dim3(256), 0, stream_, score_.get() + k * n_, n_, sc, 0.0);
    SML_HIP_CHECK(hipGetLastError());
  }
  void ComputeGradients(const Objective& obj) override {
    const ObjParams& p = obj.params();
    if (prep_valid_ && std::memcmp(&p, &prep_params_, sizeof(ObjParams)) == 0) {
      // score_grad_hist_kernel already evaluated this objective on the current scores and built the
      // next root histogram's slabs; its block maxima are folded into ghmax by root_init_kernel
      prep_valid_ = false;
      root_ready_ = true;
      ghmax_valid_ = true;
      pending_parts_ = prep_blocks_;
      return;
    }
    prep_valid_ = false;
    root_ready_ = false;
    gh2_valid_ = g_stale_ = false;  // g_ / h_ are rewritten below
    if (p.kind == kObjLambdarank && K_ == 1) {
      auto t0 = std::chrono::steady_clock::now();
      EnsureRankTables(obj);
      // index-only partition: the lambdarank kernels write the interleaved copy too (no pack pass per tree)
      rank_.gh2 = idx_ok_ && batch_ok_ ? gh2_.get() : nullptr;
      if (rank_.nq > 0) {
        gh2_valid_ = rank_.gh2 != nullptr;
        const int grid = std::min(rank_.nq, 65536);
        if (rank_regs_) {
          if (rank_waves_ == 1) {
            // the > 128-document queries (first in the largest-first order) on the full kernel, then the rest
            // on the NU <= 2 form (fewer VGPRs: more resident waves); SML_RANK_SPLIT=0: one launch
            const int k_split = rank_split_ ? rank_nbig_ : rank_.nreg;
            auto lk = rank_treduce_ ? (rank_.gain_mono ? lambdarank_regs_kernel<1, true, true>
                                                       : lambdarank_regs_kernel<1, true, false>)
                                    : (rank_.gain_mono ? lambdarank_regs_kernel<1, false, true>
                                                       : lambdarank_regs_kernel<1, false, false>);
            if (k_split > 0)
              hipLaunchKernelGGL(lk, dim3(std::min(k_split, 1 << 20)), dim3(64), 0, stream_, rank_, score_.get(),
                                 label_.get(), weight_.get(), g_.get(), h_.get(), 0, k_split);
            if (k_split < rank_.nreg) {
              const int nsmall = rank_.nreg - k_split;
              if (rank_small_waves_ == 4) {  // 4-wave blocks: past the per-CU workgroup cap of one-wave blocks
                auto ls = rank_.gain_mono ? lambdarank_regs_kernel<4, true, true, true>
                                          : lambdarank_regs_kernel<4, true, false, true>;
                hipLaunchKernelGGL(ls, dim3(std::min((nsmall + 3) / 4, 1 << 18)), dim3(256), 0, stream_, rank_,
                                   score_.get(), label_.get(), weight_.get(), g_.get(), h_.get(), k_split, rank_.nreg);
              } else {
                auto ls = rank_treduce_ ? (rank_.gain_mono ? lambdarank_regs_kernel<1, true, true, true>
                                                           : lambdarank_regs_kernel<1, true, false, true>)
                                        : (rank_.gain_mono ? lambdarank_regs_kernel<1, false, true, true>
                                                           : lambdarank_regs_kernel<1, false, false, true>);
                hipLaunchKernelGGL(ls, dim3(std::min(nsmall, 1 << 20)), dim3(64), 0, stream_, rank_, score_.get(),
                                   label_.get(), weight_.get(), g_.get(), h_.get(), k_split, rank_.nreg);
              }
            }
          } else {
            const int g4 = std::max(1, std::min((rank_.nreg + 3) / 4, 1 << 18));
            auto l4 = rank_.gain_mono ? lambdarank_regs_kernel<4, true, true> : lambdarank_regs_kernel<4, true, false>;
            hipLaunchKernelGGL(l4, dim3(g4), dim3(256), 0, stream_, rank_, score_.get(),
                               label_.get(), weight_.get(), g_.get(), h_.get(), 0, rank_.nreg);
          }
          SML_HIP_CHECK(hipGetLastError());
        }
        if (rank_lds_) {
          hipLaunchKernelGGL(lambdarank_kernel, dim3(grid), dim3(64), 0, stream_, rank_, score_.get(), label_.get(),
                             weight_.get(), g_.get(), h_.get());
          SML_HIP_CHECK(hipGetLastError());
        }
      }
      ghmax_valid_ = false;
      stats.grad_ms += Ms(t0);
      return;
    }
    if (p.kind == kObjLambdarank || p.kind == kObjCustom) {
      std::vector<double> sc;
      GetScores(&sc);
      std::vector<float> g(static_cast<size_t>(n_) * K_), h(g.size());
      obj.GetGradients(sc.data(), g.data(), h.data());
      SetGradients(g.data(), h.data());
      return;
    }
    auto t0 = std::chrono::steady_clock::now();
    const bool single = p.kind != kObjMulticlass && p.kind != kObjMulticlassOVA;
    const int grid = std::min(GridFor(n_), kGhmaxBlocks);
    hipLaunchKernelGGL(grad_kernel, dim3(grid), dim3(256), 0, stream_, p, score_.get(), label_.get(),
                       weight_.get(), g_.get(), h_.get(), n_, single ? ghmax_partial_.get() : static_cast<float*>(nullptr));
    SML_HIP_CHECK(hipGetLastError());
    if (single && K_ == 1) {
      pending_parts_ = grid;  // folded into ghmax by the next root_init_kernel
    } else if (single) {
      hipLaunchKernelGGL(ghmax_final_kernel, dim3(1), dim3(1024), 0, stream_, ghmax_partial_.get(), grid, ghmax_.get());
      SML_HIP_CHECK(hipGetLastError());
    }
    ghmax_valid_ = single && K_ == 1;
    ArmPrep(p);
    stats.grad_ms += Ms(t0);
  }
  void SetGradients(const float* g, const float* h) override {
    ghmax_valid_ = false;
    prep_valid_ = root_ready_ = false;
    gh2_valid_ = g_stale_ = false;
    pending_parts_ = 0;
    SML_HIP_CHECK(hipMemcpyAsync(g_.get(), g, sizeof(float) * n_ * K_, hipMemcpyHostToDevice, stream_));
    SML_HIP_CHECK(hipMemcpyAsync(h_.get(), h, sizeof(float) * n_ * K_, hipMemcpyHostToDevice, stream_));
    SML_HIP_CHECK(hipStreamSynchronize(stream_));
  }
  // g_ / h_ made current when the fused pass wrote only the interleaved copy
  void EnsureGH() {
    if (!g_stale_) return;
    hipLaunchKernelGGL(unpack_gh_kernel, dim3(GridFor(n_)), dim3(256), 0, stream_, gh2_.get(), n_, g_.get(), h_.get());
    SML_HIP_CHECK(hipGetLastError());
    g_stale_ = false;
  }
  void GetGradients(std::vector<float>* g, std::vector<float>* h) override {
    EnsureGH();
    g->resize(static_cast<size_t>(n_) * K_); h->resize(g->size());
    SML_HIP_CHECK(hipMemcpyAsync(g->data(), g_.get(), sizeof(float) * g->size(), hipMemcpyDeviceToHost, stream_));
    SML_HIP_CHECK(hipMemcpyAsync(h->data(), h_.get(), sizeof(float) * h->size(), hipMemcpyDeviceToHost, stream_));
    SML_HIP_CHECK(hipStreamSynchronize(stream_));
  }
  void SetBag(const std::vector<int32_t>* rows) override {
    if (!rows) { bag_n_ = -1; return; }
    bag_n_ = static_cast<int32_t>(rows->size());
    bag_.alloc(std::max<size_t>(1, rows->size()));
    SML_HIP_CHECK(hipMemcpyAsync(bag_.get(), rows->data(), sizeof(int32_t) * rows->size(), hipMemcpyHostToDevice, stream_));
    SML_HIP_CHECK(hipStreamSynchronize(stream_));
  }

  bool SampleRows(const RowSampleSpec& spec) override {
    if (spec.kind != kSampleBagging && spec.kind != kSampleGoss) return false;
    EnsureGH();
    gh2_valid_ = false;  // GOSS rescales g_ / h_
    roctxRangePushA("sml::SampleRows");
    bag_.alloc(static_cast<size_t>(std::max<int64_t>(1, n_)));
    sel_.alloc(1);
    const int grid = std::min(GridFor(n_), 2048);
    hipLaunchKernelGGL(select_init_kernel, dim3(1), dim3(64), 0, stream_, sel_.get(),
                       static_cast<long long>(spec.top_k));
    SML_HIP_CHECK(hipGetLastError());
    if (spec.kind == kSampleGoss) {
      sel_key_.alloc(static_cast<size_t>(std::max<int64_t>(1, n_)));
      sel_hist_.alloc(256);
      SML_HIP_CHECK(hipMemsetAsync(sel_hist_.get(), 0, 256 * sizeof(unsigned int), stream_));
      hipLaunchKernelGGL(goss_key_kernel, dim3(grid), dim3(256), 0, stream_, g_.get(), h_.get(), n_, K_,
                         sel_key_.get());
      SML_HIP_CHECK(hipGetLastError());
      for (int shift = 24; shift >= 0; shift -= 8) {
        hipLaunchKernelGGL(radix_hist_kernel, dim3(grid), dim3(256), 0, stream_, sel_key_.get(), n_, sel_.get(), shift,
                           sel_hist_.get());
        SML_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL(radix_pick_kernel, dim3(1), dim3(64), 0, stream_, sel_.get(), sel_hist_.get(), shift);
        SML_HIP_CHECK(hipGetLastError());
      }
    }
    hipLaunchKernelGGL(sample_kernel, dim3(grid), dim3(256), 0, stream_, spec, n_, K_,
                       spec.kind == kSampleGoss ? sel_key_.get() : static_cast<const uint32_t*>(nullptr), sel_.get(),
                       label_.get(), g_.get(), h_.get(), bag_.get());
    SML_HIP_CHECK(hipGetLastError());
    SelectState st{};
    SML_HIP_CHECK(hipMemcpyAsync(&st, sel_.get(), sizeof(SelectState), hipMemcpyDeviceToHost, stream_));
    SML_HIP_CHECK(hipStreamSynchronize(stream_));
    bag_n_ = st.count;
    if (spec.kind == kSampleGoss) ghmax_valid_ = false;  // gradients were rescaled
    roctxRangePop();
    return true;
  }

  bool EvalOnDevice(const std::string& name, const Objective& obj, double* out) override {
    TraceRange tr("sml::EvalTrain");
    DeviceMetricInputs in;
    in.score = score_.get(); in.label = label_.get(); in.weight = weight_.get(); in.n = n_; in.num_class = K_;
    const bool rank = name.rfind("ndcg", 0) == 0 || name.rfind("map", 0) == 0;
    if (rank) {
      if (obj.params().kind != kObjLambdarank) return false;  // the query tables come with the objective
      EnsureRankTables(obj);
      in.qb = rank_qb_.get(); in.nq = rank_.nq; in.gain = rank_gain_.get(); in.ngain = rank_.ngain;
    }
    return DeviceEvalMetricFull(name, obj.params(), in, stream_, out);
  }

  // K11: validation sets live in HBM; every tree is folded into their scores by a device traversal and
  // their metrics reduce on the device (valid_gpu.hip)
  bool AddValidSet(int vi, const Dataset& vd, const std::vector<double>& scores, const Config& cfg) override {
    TraceRange tr("sml::AddValidSet");
    if (vd.num_data >= (int64_t(1) << 31) || vd.row_stride < vd.ref.num_inner()) return false;
    if (static_cast<int>(vsets_.size()) <= vi) vsets_.resize(vi + 1);
    vsets_[vi].reset(new DeviceValidSet(vd, scores, K_, cfg.label_gain, dev_, stream_));
    return true;
  }
  DeviceValidSet& VSet(int vi) {
    if (vi < 0 || vi >= static_cast<int>(vsets_.size()) || !vsets_[vi]) throw std::logic_error("no device validation set");
    return *vsets_[vi];
  }
  void ValidApplyTree(int vi, const Tree& t, int k, int op, double p) override {
    TraceRange tr("sml::ValidApplyTree");
    VSet(vi).ApplyTree(t, k, op, p);
  }
  void GetValidScores(int vi, std::vector<double>* s) override { VSet(vi).GetScores(s); }
  bool EvalValidOnDevice(int vi, const std::string& name, const Objective& obj, double* out) override {
    TraceRange tr("sml::EvalValid");
    return VSet(vi).Eval(name, obj.params(), K_, out);
  }

  void Synchronize() override {
    if (Distributed()) {
      SML_HIP_CHECK(hipEventRecord(ev_sync_, stream_));
      WaitEvent(ev_sync_);
    }
    SML_HIP_CHECK(hipStreamSynchronize(stream_));
    AccountScoreTime();
    if (comm_) stats.comm_dev_bytes = comm_->DeviceBytes() - comm_bytes0_;  // this booster's share
  }

  Tree TrainTree(int k, const std::vector<char>& fmask_in) override {
    roctxRangePushA("sml::TrainTree");
    GrowTree(k, fmask_in);
    EnqueueTreeCopy();
    Tree t = FinishTree();
    AccountScoreTime();
    roctxRangePop();
    return t;
  }

  // Grow the tree and run the fused score / next-gradient / next-root-histogram pass on the device
  // tree right behind it: the host reads the tree back while that pass runs.
  Tree TrainTreeAndUpdateScore(int k, const std::vector<char>& fmask_in, double shrink, bool* updated) override {
    *updated = false;
    if (L_ > kPrepMaxNodes + 1) return TrainTree(k, fmask_in);
    roctxRangePushA("sml::TrainTreeAndUpdateScore");
    GrowTree(k, fmask_in);
    EnqueueTreeCopy();
    AccountScoreTime();  // the previous pass (done before this growth) frees the event pair
    DevTreeSrc src{dt_, state_ + final_v_, fm_.num_bin, fm_.missing, fm_.default_bin, shrink};
    // every row was partitioned (batched growth, no bag): its leaf comes from the finest segments' labels
    // (leaf_table_kernel + leaf_scatter_kernel), not a per-row tree walk
    const uint8_t* rl = nullptr;
    if (grew_batched_ && bag_n_ < 0 && dt_.lseg) {
      hipLaunchKernelGGL(leaf_table_kernel, dim3(1), dim3(kLeafTableThreads), 0, stream_, bstate_.get(),
                         bnodes_.get(), state_ + final_v_, dt_.lseg, rtab_.get(),
                         reinterpret_cast<int*>(rtab_.get() + kBatchMaxNodes));
      SML_HIP_CHECK(hipGetLastError());
      hipLaunchKernelGGL(leaf_scatter_kernel, dim3(std::min(GridFor(n_), 2048)), dim3(256), 0, stream_, rtab_.get(),
                         reinterpret_cast<const int*>(rtab_.get() + kBatchMaxNodes), perm_[0].get(), perm_[1].get(),
                         static_cast<int32_t>(n_), row_leaf_.get());
      SML_HIP_CHECK(hipGetLastError());
      rl = row_leaf_.get();
    }
    if (prep_armed_ && k == 0 && K_ == 1) {
      LaunchPrep(DevTreeView{}, src, 1.0, rl);
    } else {
      // any other objective: the plain score update, still without the host round trip
      prep_valid_ = root_ready_ = false;
      SML_HIP_CHECK(hipEventRecord(ev_[2], stream_));
      hipLaunchKernelGGL(score_kernel, dim3(ScoreGrid()), dim3(kScoreThreads), 0, stream_, DevTreeView{}, src,
                         reinterpret_cast<const uint4*>(bins_ptr_), S_ / 16, F_, cbins_.get(), n_, 1.0,
                         score_.get() + static_cast<size_t>(k) * n_, static_cast<int32_t*>(nullptr), rl);
      SML_HIP_CHECK(hipGetLastError());
      SML_HIP_CHECK(hipEventRecord(ev_[3], stream_));
      score_pending_ = true;
    }
    Tree t = FinishTree();
    *updated = true;
    roctxRangePop();
    return t;
  }

  void GrowTree(int k, const std::vector<char>& fmask_in) {
    SML_HIP_CHECK(hipEventRecord(ev_[0], stream_));
    grew_batched_ = false;
    std::vector<int8_t> fmask(F_, 1);
    for (int f = 0; f < F_ && f < static_cast<int>(fmask_in.size()); ++f) fmask[f] = fmask_in[f] ? 1 : 0;
    sp_.tree_seq = tree_seq_++;
    sp_.bynode_k = BynodeK(cfg_, std::vector<char>(fmask.begin(), fmask.end()));
    if (fmask != mask_host_) {  // one H2D copy fewer per tree when the feature mask is unchanged
      mask_host_ = fmask;
      SML_HIP_CHECK(hipMemcpyAsync(mask_.get(), mask_host_.data(), F_, hipMemcpyHostToDevice, stream_));
    }
    const float* g = g_.get() + static_cast<size_t>(k) * n_;
    const float* h = h_.get() + static_cast<size_t>(k) * n_;
    const bool root_prepared = root_ready_ && bag_n_ < 0 && k == 0;
    const bool idx = idx_ok_ && batch_ok_ && sp_.bynode_k <= 0 && !voting_ && bag_n_ < 0 && k == 0;
    if (!idx || !root_prepared) EnsureGH();  // the physical g / h are read below
    root_ready_ = false;
    int32_t root_count = static_cast<int32_t>(n_);
    int root_buf = -1;
    if (bag_n_ >= 0) {
      root_count = bag_n_;
      root_buf = 0;
      hipLaunchKernelGGL(gather_bag_kernel, dim3(GridFor(std::max(1, bag_n_))), dim3(256), 0, stream_, bag_.get(), bag_n_,
                         g, h, perm_[0].get(), ogh_[0].get());
      SML_HIP_CHECK(hipGetLastError());
    }
    if (!ghmax_valid_ || k != 0) {
      const int grid = std::min(GridFor(n_), kGhmaxBlocks);
      hipLaunchKernelGGL(ghmax_kernel, dim3(grid), dim3(256), 0, stream_, g, h, n_, ghmax_partial_.get());
      SML_HIP_CHECK(hipGetLastError());
      hipLaunchKernelGGL(ghmax_final_kernel, dim3(1), dim3(1024), 0, stream_, ghmax_partial_.get(), grid, ghmax_.get());
      SML_HIP_CHECK(hipGetLastError());
      pending_parts_ = 0;
    }
    st_cur_ = state_;
    st_next_ = state_ + 1;
    hipLaunchKernelGGL(root_init_kernel, dim3(1), dim3(64), 0, stream_, state_, leaves_.get(), root_count, root_buf, L_,
                       ghmax_partial_.get(), pending_parts_, ghmax_.get());
    SML_HIP_CHECK(hipGetLastError());
    pending_parts_ = 0;
    GlobalGhmax();
    // root histogram (slabs already built by score_grad_hist_kernel, or built here) + split search
    const float* root_scale = nullptr;
    if (root_prepared) {
      root_scale = reinterpret_cast<const float*>(ghbound_.get());
      EnqueueReduce(root_scale);
    } else {
      EnqueueHistogram(g, h);
    }
    EnqueueFindChoose(false);
    if (batch_ok_ && sp_.bynode_k <= 0 && !voting_) {
      if (idx && !gh2_valid_) {
        hipLaunchKernelGGL(pack_gh_kernel, dim3(GridFor(n_)), dim3(256), 0, stream_, g, h, n_, gh2_.get());
        SML_HIP_CHECK(hipGetLastError());
        gh2_valid_ = true;
      }
      GrowBatched(g, h, idx);
      grew_batched_ = true;
      final_v_ = 0;
      SML_HIP_CHECK(hipEventRecord(ev_[1], stream_));
      return;
    }
    for (int s = 1; s < L_; ++s) {
      // choose + partition the chosen leaf, histogram its smaller child, search both
      DState* sin = st_cur_;
      DState* sout = st_cur_ == state_ ? state_ + 1 : state_;
      auto ck = part_rows_ == 16 ? choose_part_kernel<16> : (part_rows_ == 4 ? choose_part_kernel<4> : choose_part_kernel<8>);
      hipLaunchKernelGGL(ck, dim3(part_grid_), dim3(kPartThreads), 0, stream_, sin, sout, leaves_.get(),
                         lbest_.get(), lgain_.get(), fbest_.get(), F_, dt_, CountSlot(), mono_.get(), sp_.has_mono,
                         cbins_.get(), n_, perm_[0].get(), perm_[1].get(), ogh_[0].get(), ogh_[1].get(),
                         perm_[0].get(), perm_[1].get(), ogh_[0].get(), ogh_[1].get(), g, h, fm_);
      SML_HIP_CHECK(hipGetLastError());
      st_cur_ = sout;
      st_next_ = sin;
      if (s == L_ - 1 && skip_last_ && !Distributed()) {
        hipLaunchKernelGGL(finalize_last_split_kernel, dim3(1), dim3(64), 0, stream_, st_cur_, leaves_.get(), dt_);
        SML_HIP_CHECK(hipGetLastError());
        break;
      }
      EnqueueHistogram(g, h);
      EnqueueFindChoose(s == L_ - 1);
    }
    final_v_ = st_cur_ == state_ ? 0 : 1;
    SML_HIP_CHECK(hipEventRecord(ev_[1], stream_));
  }

  // Rounds of the batched speculative growth (see bplan_kernel). The host stays blook_ rounds ahead: before
  // enqueueing round r it waits for the plan of round r - blook_ and stops once a plan reported the tree
  // final (the rounds already queued behind it are no-ops).
  void GrowBatched(const float* g, const float* h, bool idx) {
    TraceRange tr("sml::GrowBatched");
    const int budget = L_ - 1;
    const float* ghmax = reinterpret_cast<const float*>(ghmax_.get());
    const int part_tile = kPartThreads * part_rows_;
    const int max_rounds = budget + 2;
    auto bp = part_rows_ == 16 ? bpart_kernel<16> : (part_rows_ == 4 ? bpart_kernel<4> : bpart_kernel<8>);
    auto bh = hist_fpg_ == 16 ? bhist_kernel<kHistUnroll, 16>
              : (hist_unroll4_ ? (tight_ ? bhist_kernel<4, kFeatPerGroup, false, true> : bhist_kernel<4, kFeatPerGroup>)
                               : (hist_pipe_ ? (tight_ ? bhist_kernel<kHistUnroll, kFeatPerGroup, true, true>
                                                       : bhist_kernel<kHistUnroll, kFeatPerGroup, true>)
                                             : (tight_ ? bhist_kernel<kHistUnroll, kFeatPerGroup, false, true>
                                                       : bhist_kernel<kHistUnroll, kFeatPerGroup>)));
    // index-only partition: row ids in the segments, (g, h) gathered from gh2_
    auto bhi = hist_fpg_ == 16 ? bhist_kernel<kHistUnroll, 16, false, false, true>
                               : (tight_ ? bhist_kernel<kHistUnroll, kFeatPerGroup, false, true, true>
                                         : bhist_kernel<kHistUnroll, kFeatPerGroup, false, false, true>);
    auto bpi = part_rows_ == 16 ? bpart_kernel<16, true> : (part_rows_ == 4 ? bpart_kernel<4, true> : bpart_kernel<8, true>);
    const float* hg = idx ? reinterpret_cast<const float*>(gh2_.get()) : g;
    if (bprof_) SML_HIP_CHECK(hipMemsetAsync(bprof_, 0, sizeof(long long) * kPlanProfStride * (max_rounds + 1), stream_));
    int r = 0;
    for (; r <= max_rounds; ++r) {
      if (r >= blook_) {
        const int q = r - blook_;
        SpinEvent(bev_[q % kBRing]);
        const int fl = bflag_host_[q % kBRing];
        if (fl == 2) throw std::runtime_error("batched tree growth: device replay invariant violated");
        if (fl) break;
      }
      // frontier slots per lane: a tree of L leaves has at most L frontier entries
      auto plan = L_ <= 64 ? bplan_kernel<1> : (L_ <= 128 ? bplan_kernel<2> : bplan_kernel<4>);
      hipLaunchKernelGGL(plan, dim3(1), dim3(kPlanThreads), 0, stream_, bstate_.get(), bnodes_.get(),
                         nbest_.get(), fbest_.get(), F_, part_.get(), E_, leaves_.get(), state_, dt_, fm_, mono_.get(),
                         sp_.has_mono, r == 0 ? 1 : 0, spec_k_, spec_max_, wide_div_, budget, part_tile, plan_cap_,
                         bflag_dev_ + r % kBRing,
                         bprof_ ? bprof_ + kPlanProfStride * r : nullptr);
      SML_HIP_CHECK(hipGetLastError());
      SML_HIP_CHECK(hipEventRecord(bev_[r % kBRing], stream_));
      // partition + histograms of expansions [j0, j1) on stream st, slabs from block sb
      auto part_hist = [&](int j0, int j1, hipStream_t st, size_t sb) {
        hipLaunchKernelGGL(idx ? bpi : bp, dim3(part_grid_), dim3(kPartThreads), 0, st, bstate_.get(), cbins_.get(), n_,
                           perm_[0].get(), perm_[1].get(), ogh_[0].get(), ogh_[1].get(), perm_[0].get(), perm_[1].get(),
                           ogh_[0].get(), ogh_[1].get(), g, h, j0, j1);
        SML_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL(idx ? bhi : bh, dim3(kMaxHistBlocks, (F_ + hist_fpg_ - 1) / hist_fpg_), dim3(kHistBlockThreads),
                           0, st, bstate_.get(), reinterpret_cast<const uint4*>(bins_ptr_), S_ / 16, F_, perm_[0].get(),
                           perm_[1].get(), ogh_[0].get(), ogh_[1].get(), hg, h, ghmax, slab_.get() + sb * E_, scale_n_,
                           j0, j1);
        SML_HIP_CHECK(hipGetLastError());
      };
      // (a two-stream form - expansions [k, nexp) partitioned on a second stream while [0, k)'s histograms
      // build - measured 1.86-1.91 ms/iter against 1.51 on one stream: the cross-stream event waits of every
      // round cost more than the overlap gains; r6 pass 8)
      part_hist(0, kMaxSpec, stream_, 0);
      hipLaunchKernelGGL(breduce_kernel, dim3((E_ + kRedE - 1) / kRedE, spec_max_), dim3(kRedE * kRedG), 0, stream_,
                         bstate_.get(), slab_.get(), E_, ghmax, part_.get(), scale_n_, Distributed() ? 1 : 0, 0);
      SML_HIP_CHECK(hipGetLastError());
      // every expansion's smaller-child histogram + row count in ONE exact int64 collective per round
      if (Distributed()) ExactAllReduce(spec_max_, ghmax, &bstate_.get()->nexp);
      hipLaunchKernelGGL(bfind_kernel, dim3(F_, 2 * spec_max_), dim3(256), 0, stream_, bstate_.get(), bnodes_.get(),
                         part_.get(), E_, hist_pool_.get(), fm_, sp_, fbest_.get(), F_);
      SML_HIP_CHECK(hipGetLastError());
    }
    if (r > max_rounds) throw std::runtime_error("batched tree growth did not finish within num_leaves rounds");
    if (bprof_) {  // SML_BPLAN_PROF: the rounds' phase stamps (profiling only: a blocking copy per tree)
      std::vector<long long> p(kPlanProfStride * (max_rounds + 1));
      SML_HIP_CHECK(hipMemcpyAsync(p.data(), bprof_, p.size() * sizeof(long long), hipMemcpyDeviceToHost, stream_));
      SML_HIP_CHECK(hipStreamSynchronize(stream_));
      for (int q = 0; q < r; ++q) {
        const long long* s = p.data() + kPlanProfStride * q;
        if (s[9] > 0) {  // the final round: the tree's expansions and the ones never popped
          for (int k = 0; k < 4; ++k) bprof_tree_[k] += static_cast<double>(s[7 + k]);
          ++bprof_trees_;
        }
        if (s[4] == 0) continue;  // a round queued behind the final plan (it returned at entry)
        for (int k = 0; k < 4; ++k) bprof_sum_[k] += static_cast<double>(s[k + 1] - s[k]);
        bprof_sum_[4] += static_cast<double>(s[5]);
        bprof_sum_[5] += static_cast<double>(s[6]);
        ++bprof_n_;
      }
    }
  }

  // spin on an event (a blocking sync can sleep through the few microseconds the batched growth waits);
  // data-parallel runs poll the communicator and honour time_out like WaitEvent
  void SpinEvent(hipEvent_t ev) {
    if (Distributed()) { WaitEvent(ev); return; }
    for (;;) {
      const hipError_t q = hipEventQuery(ev);
      if (q == hipSuccess) return;
      if (q != hipErrorNotReady) SML_HIP_CHECK(q);
    }
  }

  // the finished tree (state + arrays: one allocation) -> pinned host memory, one transfer
  void EnqueueTreeCopy() {
    SML_HIP_CHECK(hipMemcpyAsync(pinned_, blob_.get(), blob_bytes_, hipMemcpyDeviceToHost, stream_));
    SML_HIP_CHECK(hipEventRecord(ev_copy_, stream_));
  }

  Tree FinishTree() {
    WaitEvent(ev_copy_);
    Tree t = ReadTree();
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, ev_[0], ev_[1]) == hipSuccess) stats.device_tree_ms += ms;
    for (int i = 0; i < comm_used_; ++i)
      if (hipEventElapsedTime(&ms, comm_ev_[2 * i], comm_ev_[2 * i + 1]) == hipSuccess) stats.comm_ms += ms;
    comm_used_ = 0;
    return t;
  }

  // Wait for `ev`. Data-parallel runs poll instead of blocking: a collective stuck on a dead peer never
  // completes, so while waiting the communicator's async error state is checked (CommError on failure)
  // and after cfg time_out minutes the communicator is aborted (its pending kernels return) and the wait
  // raises CommError - every rank fails instead of hanging (NetworkManager.scala:195-218).
  void WaitEvent(hipEvent_t ev) {
    if (!Distributed()) {
      SML_HIP_CHECK(hipEventSynchronize(ev));
      return;
    }
    const auto t0 = std::chrono::steady_clock::now();
    const double limit_s = 60.0 * std::max(1, cfg_.time_out);
    int spins = 0;
    for (;;) {
      const hipError_t q = hipEventQuery(ev);
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) SML_HIP_CHECK(q);
      comm_->Check();
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit_s) {
        comm_->Abort();
        throw CommError("collective did not complete within time_out=" + std::to_string(cfg_.time_out) +
                        " min (a peer rank died or diverged); communicator aborted");
      }
      if (++spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    comm_->Check();
  }

  void UpdateScore(const Tree& t, int k, double scale) override {
    roctxRangePushA("sml::UpdateScore");
    DevTreeView tv = UploadTree(t);
    SML_HIP_CHECK(hipEventRecord(ev_[2], stream_));
    prep_valid_ = root_ready_ = false;
    if (prep_armed_ && k == 0 && t.num_leaves <= kPrepMaxNodes + 1) {
      LaunchPrep(tv, DevTreeSrc{}, scale);  // score update + next gradients + next root histogram, one pass
    } else {
      hipLaunchKernelGGL(score_kernel, dim3(ScoreGrid()), dim3(kScoreThreads), 0, stream_, tv, DevTreeSrc{},
                         reinterpret_cast<const uint4*>(bins_ptr_), S_ / 16, F_, cbins_.get(), n_, scale,
                         score_.get() + static_cast<size_t>(k) * n_, static_cast<int32_t*>(nullptr));
      SML_HIP_CHECK(hipGetLastError());
    }
    SML_HIP_CHECK(hipEventRecord(ev_[3], stream_));
    score_pending_ = true;
    roctxRangePop();
  }

  void PredictLeafIndex(const Tree& t, std::vector<int32_t>* leaf) override {
    DevTreeView tv = UploadTree(t);
    hipLaunchKernelGGL(score_kernel, dim3(ScoreGrid()), dim3(kScoreThreads), 0, stream_, tv, DevTreeSrc{},
                       reinterpret_cast<const uint4*>(bins_ptr_), S_ / 16, F_, cbins_.get(), n_, 0.0,
                       static_cast<double*>(nullptr), leaf_idx_.get());
    SML_HIP_CHECK(hipGetLastError());
    leaf->resize(n_);
    SML_HIP_CHECK(hipMemcpyAsync(leaf->data(), leaf_idx_.get(), sizeof(int32_t) * n_, hipMemcpyDeviceToHost, stream_));
    SML_HIP_CHECK(hipStreamSynchronize(stream_));
  }

 private:
  static double Ms(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  int ScoreGrid() const {
    const int64_t per_block = static_cast<int64_t>(kScoreThreads) * kScoreRows;
    return static_cast<int>(std::max<int64_t>(1, (n_ + per_block - 1) / per_block));
  }
  static int GridFor(int64_t n) {
    int64_t b = (n + 255) / 256;
    return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(b, 8192)));
  }

  // the smaller child's (root's) GLOBAL row count: the allreduced histogram's extra slot, or under voting
  // the allreduced vote buffer's last slot
  const double* CountSlot() const {
    return voting_ ? vote_.get() + 4 * static_cast<size_t>(F_) : reinterpret_cast<const double*>(part_.get() + E_);
  }

  // device time of the last score update; call only after a stream sync
  // score update + next gradients + next root histogram in one pass (score_grad_hist_kernel) with
  // the uploaded host tree `tv` or, when src.st is set, the device tree just grown
  void LaunchPrep(const DevTreeView& tv, const DevTreeSrc& src, double scale, const uint8_t* row_leaf = nullptr) {
    if (src.st) SML_HIP_CHECK(hipEventRecord(ev_[2], stream_));
    // index-only partition: the pass writes the interleaved (g, h) copy instead of g_ / h_ (same bytes)
    const bool gh2 = idx_ok_ && batch_ok_;
    auto sgk = gh2 ? (root_pipe_ ? score_grad_hist_kernel<kHistUnroll, true, false, true>
                                 : (tight_ ? score_grad_hist_kernel<kHistUnroll, false, true, true>
                                           : score_grad_hist_kernel<kHistUnroll, false, false, true>))
                   : (root_pipe_ ? score_grad_hist_kernel<kHistUnroll, true>
                                 : (tight_ ? score_grad_hist_kernel<kHistUnroll, false, true> : score_grad_hist_kernel<kHistUnroll>));
    hipLaunchKernelGGL(sgk, dim3(kMaxHistBlocks), dim3(kHistBlockThreads), 0, stream_, tv, src,
                       reinterpret_cast<const uint4*>(bins_ptr_), S_ / 16, F_, static_cast<int32_t>(n_), scale,
                       score_.get(), prep_params_, label_.get(), weight_.get(),
                       gh2 ? reinterpret_cast<float*>(gh2_.get()) : g_.get(), h_.get(),
                       reinterpret_cast<const float*>(ghbound_.get()), ghmax_partial_.get(), slab_.get(), scale_n_,
                       row_leaf);
    SML_HIP_CHECK(hipGetLastError());
    gh2_valid_ = gh2;
    g_stale_ = gh2;
    if (src.st) {
      SML_HIP_CHECK(hipEventRecord(ev_[3], stream_));
      score_pending_ = true;
    }
    prep_valid_ = true;
    root_ready_ = false;
  }

  void AccountScoreTime() {
    if (!score_pending_) return;
    SML_HIP_CHECK(hipEventSynchronize(ev_[3]));
    float sms = 0.f;
    if (hipEventElapsedTime(&sms, ev_[2], ev_[3]) == hipSuccess) stats.device_score_ms += sms;
    score_pending_ = false;
  }

  // query boundaries, 1/maxDCG per query and the label gains for the
  // lambdarank kernel (uploaded once: they depend only on the dataset)
  void EnsureRankTables(const Objective& obj) {
    if (rank_ready_) return;
    const auto& qb = obj.query_boundaries();
    const auto& imd = obj.inv_max_dcg();
    const auto& gain = obj.label_gain();
    if (qb.size() < 2 || gain.empty()) throw std::runtime_error("lambdarank: missing query boundaries or label_gain");
    if (qb.back() > n_) throw std::runtime_error("lambdarank: query boundaries exceed the number of rows");
    rank_qb_.alloc(qb.size());
    rank_imd_.alloc(imd.size());
    rank_gain_.alloc(gain.size());
    SML_HIP_CHECK(hipMemcpy(rank_qb_.get(), qb.data(), sizeof(int32_t) * qb.size(), hipMemcpyHostToDevice));
    SML_HIP_CHECK(hipMemcpy(rank_imd_.get(), imd.data(), sizeof(double) * imd.size(), hipMemcpyHostToDevice));
    SML_HIP_CHECK(hipMemcpy(rank_gain_.get(), gain.data(), sizeof(double) * gain.size(), hipMemcpyHostToDevice));
    {
      std::vector<double> disc(kRankLds);
      for (int r = 0; r < kRankLds; ++r) disc[r] = 1.0 / std::log2(2.0 + r);
      rank_disc_.alloc(kRankLds);
      SML_HIP_CHECK(hipMemcpy(rank_disc_.get(), disc.data(), sizeof(double) * kRankLds, hipMemcpyHostToDevice));
    }
    int max_q = 0;
    rank_regs_ = rank_lds_ = false;
    const bool regs_pos = obj.max_position() <= 64;  // RegsEligible, host side: which kernels have work
    std::vector<int32_t> reg_q;
    for (size_t q = 0; q + 1 < qb.size(); ++q) {
      const int c = qb[q + 1] - qb[q];
      max_q = std::max(max_q, c);
      if (c <= 0) continue;
      if (regs_pos && c <= kRankLds) {
        rank_regs_ = true;
        reg_q.push_back(static_cast<int32_t>(q));
      } else {
        rank_lds_ = true;
      }
    }
    // the register kernel walks its queries largest first, one wave each (a query's cost grows with its
    // documents - NU lane slots of pair terms and ranks - and 20..180-document queries in index order left
    // a tail of long queries on a few waves)
    std::stable_sort(reg_q.begin(), reg_q.end(),
                     [&qb](int32_t a, int32_t b) { return qb[a + 1] - qb[a] > qb[b + 1] - qb[b]; });
    rank_nbig_ = 0;
    while (rank_nbig_ < static_cast<int>(reg_q.size()) && qb[reg_q[rank_nbig_] + 1] - qb[reg_q[rank_nbig_]] > 128)
      ++rank_nbig_;
    rank_order_.alloc(std::max<size_t>(1, reg_q.size()));
    if (!reg_q.empty())
      SML_HIP_CHECK(hipMemcpy(rank_order_.get(), reg_q.data(), sizeof(int32_t) * reg_q.size(), hipMemcpyHostToDevice));
    rank_ = RankTables{};
    rank_.order = rank_order_.get();
    rank_.nreg = static_cast<int>(reg_q.size());
    if (max_q > kRankLds) {  // long queries stream ranks / lambdas through global scratch
      rank_scratch_.alloc(n_);
      rank_lam_.alloc(n_);
      rank_hes_.alloc(n_);
      rank_.rank_scratch = rank_scratch_.get();
      rank_.lam_scratch = rank_lam_.get();
      rank_.hes_scratch = rank_hes_.get();
    }
    if (qb.back() < n_ || qb.front() > 0) {  // rows outside every query get zero gradients
      SML_HIP_CHECK(hipMemsetAsync(g_.get(), 0, sizeof(float) * n_, stream_));
      SML_HIP_CHECK(hipMemsetAsync(h_.get(), 0, sizeof(float) * n_, stream_));
    }
    rank_.qb = rank_qb_.get();
    rank_.inv_max_dcg = rank_imd_.get();
    rank_.gain = rank_gain_.get();
    rank_.disc = rank_disc_.get();
    rank_.nq = static_cast<int>(qb.size()) - 1;
    rank_.ngain = static_cast<int>(gain.size());
    rank_.max_position = obj.max_position();
    rank_.norm = obj.lambdarank_norm() ? 1 : 0;
    rank_.sigma = obj.params().sigmoid;
    // kMono: the higher label of a pair is the one with the larger gain - true when the gains (as the fp32
    // the kernel compares) strictly increase and no label is negative (a negative label clamps to the top gain)
    bool mono = true;
    for (size_t k = 0; k + 1 < gain.size(); ++k) mono &= static_cast<float>(gain[k + 1]) > static_cast<float>(gain[k]);
    if (mono && obj.labels()) {
      const float* lab = obj.labels();
      const int64_t nl = obj.num_rows();
      bool neg = false;
#pragma omp parallel for reduction(|| : neg) schedule(static)
      for (int64_t i = 0; i < nl; ++i) neg = neg || lab[i] < 0.f;
      mono = !neg;
    }
    const char* me = std::getenv("SML_RANK_MONO");  // 0: the label-compare form (A/B and tests), read per booster
    rank_.gain_mono = me && std::atoi(me) == 0 ? 0 : (mono ? 1 : 0);
    const char* pp = std::getenv("SML_RANK_PROF_PHASE");
    rank_.prof_phase = pp ? std::atoi(pp) : 0;
    rank_ready_ = true;
  }

  // Enable the fused score/gradient/root-histogram pass for objectives whose |g| and h have an
  // a-priori bound (the pass needs its fixed-point scale before it sees the gradients).
  void ArmPrep(const ObjParams& p) {
    prep_armed_ = false;
    if (!prep_ok_) return;
    double gb, hb;
    if (p.kind == kObjBinary) {
      const double lw = std::max(std::fabs(p.pos_weight), std::fabs(p.neg_weight));
      gb = std::fabs(p.sigmoid) * lw * wmax_;
      hb = p.sigmoid * p.sigmoid * 0.25 * lw * wmax_;
    } else if (p.kind == kObjCrossEntropy) {
      if (ymax_ < 0.0) {
        ymax_ = 0.0;
        for (float y : data_->label) ymax_ = std::max(ymax_, static_cast<double>(std::fabs(y)));
        if (comm_ && comm_->world() > 1) comm_->AllReduceHostMax(&ymax_, 1);
      }
      gb = (1.0 + ymax_) * wmax_;
      hb = 0.25 * wmax_;
    } else {
      return;
    }
    // float rounding of a gradient never exceeds the float rounding of its bound; 1e-4 of headroom
    const float nb[2] = {static_cast<float>(gb * 1.0001), static_cast<float>(hb * 1.0001)};
    if (nb[0] != bound_host_[0] || nb[1] != bound_host_[1]) {
      bound_host_[0] = nb[0];
      bound_host_[1] = nb[1];
      SML_HIP_CHECK(hipMemcpyAsync(ghbound_.get(), bound_host_, sizeof(bound_host_), hipMemcpyHostToDevice, stream_));
      SML_HIP_CHECK(hipStreamSynchronize(stream_));
    }
    prep_params_ = p;
    prep_blocks_ = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(kMaxHistBlocks, (n_ + min_rows_hist_ - 1) / min_rows_hist_)));
    prep_armed_ = true;
  }

  void EnqueueHistogram(const float* g, const float* h) {
    const float* ghmax = reinterpret_cast<const float*>(ghmax_.get());
    auto hk = hist_fpg_ == 16 ? hist_kernel<kHistUnroll, 16>
              : (hist_unroll4_ ? hist_kernel<4, kFeatPerGroup>
                               : (hist_pipe_ ? hist_kernel<kHistUnroll, kFeatPerGroup, true>
                                             : (tight_ ? hist_kernel<kHistUnroll, kFeatPerGroup, false, true>
                                                       : hist_kernel<kHistUnroll, kFeatPerGroup>)));
    hipLaunchKernelGGL(hk, dim3(kMaxHistBlocks, (F_ + hist_fpg_ - 1) / hist_fpg_), dim3(kHistBlockThreads), 0, stream_, st_cur_,
                       leaves_.get(), reinterpret_cast<const uint4*>(bins_ptr_), S_ / 16, F_, perm_[0].get(),
                       perm_[1].get(), ogh_[0].get(), ogh_[1].get(), g, h, ghmax, slab_.get(), scale_n_);
    SML_HIP_CHECK(hipGetLastError());
    EnqueueReduce(ghmax);
  }

  // slab reduce with the scale the slabs were built with (+ the data-parallel allreduce)
  void EnqueueReduce(const float* ghmax) {
    const bool exact = Distributed() && !voting_;
    hipLaunchKernelGGL(hist_reduce_kernel, dim3((E_ + kRedE - 1) / kRedE), dim3(kRedE * kRedG), 0, stream_, st_cur_,
                       leaves_.get(), slab_.get(), E_, ghmax, part_.get(), scale_n_, exact ? 1 : 0);
    SML_HIP_CHECK(hipGetLastError());
    // smaller child's histogram and its row count: one exact int64 allreduce of 2E+2 words over RCCL / P2P,
    // timed on the device (hipEvents around the collective on the engine stream). Voting keeps them local.
    if (exact) ExactAllReduce(1, ghmax);
  }

  // int64 histograms (+ counts) of `nh` histograms in part_ summed over ranks, then converted to fp64 with the
  // tree's global scale: bitwise the 1-rank histograms of the union of the partitions
  // `units` (device): the batched round's expansion count - only that many slots travel on a device-sized
  // transport; nullptr (root / one-split growth): all nh slots
  void ExactAllReduce(int nh, const float* ghmax, const int32_t* units = nullptr) {
    EnsureCommEvents();
    const bool timed = comm_used_ < static_cast<int>(comm_ev_.size()) / 2;
    if (timed) SML_HIP_CHECK(hipEventRecord(comm_ev_[2 * comm_used_], stream_));
    // batched growth: only the round's nexp expansions travel when the transport reads the count on the device
    // (the one-shot P2P kernel); host-sized collectives reduce all nh slots
    const int64_t per = static_cast<int64_t>(E_ + 1) * 2;
    if (units == nullptr)
      comm_->AllReduceDeviceI64(reinterpret_cast<int64_t*>(part_.get()), per * nh, stream_);
    else if (comm_->AllReduceDeviceI64Active(reinterpret_cast<int64_t*>(part_.get()), per * nh, units, per, stream_))
      stats.comm_dyn_calls += 1;
    stats.comm_bytes_max += static_cast<double>(per * nh * 8);
    if (timed) SML_HIP_CHECK(hipEventRecord(comm_ev_[2 * comm_used_ + 1], stream_));
    comm_used_ += timed ? 1 : 0;
    ++stats.comm_calls;
    hipLaunchKernelGGL(hist_convert_kernel, dim3((E_ + 1 + 255) / 256, nh), dim3(256), 0, stream_, part_.get(), E_,
                       scale_n_, ghmax);
    SML_HIP_CHECK(hipGetLastError());
  }

  // ghmax_ = max over ranks (data-parallel), on the stream: the scale of this tree's histograms
  void GlobalGhmax() {
    if (!Distributed() || comm_->world() <= 1) return;
    const int w = comm_->world();
    ghslot_.alloc(2 * w);
    hipLaunchKernelGGL(gh_slot_fill_kernel, dim3(1), dim3(64), 0, stream_, ghmax_.get(), ghslot_.get(), comm_->rank(), w);
    SML_HIP_CHECK(hipGetLastError());
    comm_->AllReduceDeviceF32(ghslot_.get(), 2 * w, stream_);
    hipLaunchKernelGGL(gh_slot_fold_kernel, dim3(1), dim3(64), 0, stream_, ghslot_.get(), w, ghmax_.get());
    SML_HIP_CHECK(hipGetLastError());
  }

  // SML_GBDT_COMM_WORLD1=1 (tests): a world-1 communicator runs the full data-parallel path (allreduce per
  // split, device comm timing, polling waits) so a one-GPU box executes it end to end
  bool Distributed() const { return comm_ && (comm_->world() > 1 || comm_world1_); }

  // one device allreduce on the engine stream, timed with a hipEvent pair while pairs are left
  void TimedAllReduce(double* buf, int64_t n) {
    EnsureCommEvents();
    const bool timed = comm_used_ < static_cast<int>(comm_ev_.size()) / 2;
    if (timed) SML_HIP_CHECK(hipEventRecord(comm_ev_[2 * comm_used_], stream_));
    comm_->AllReduceDeviceF64(buf, n, stream_);
    if (timed) SML_HIP_CHECK(hipEventRecord(comm_ev_[2 * comm_used_ + 1], stream_));
    comm_used_ += timed ? 1 : 0;
    ++stats.comm_calls;
  }

  // PV-Tree split search of the new leaves (see vote_kernel): local search, vote, allreduce of the votes,
  // selection, allreduce of only the selected features' histograms, global search of those
  void EnqueueVote() {
    const double* local_count = reinterpret_cast<const double*>(part_.get() + E_);
    hipLaunchKernelGGL(find_split_kernel, dim3(F_, 2), dim3(256), 0, stream_, st_cur_, leaves_.get(), part_.get(),
                       E_, local_count, hist_pool_.get(), fm_, sp_local_, floc_.get(), F_,
                       static_cast<DState*>(nullptr), static_cast<int>(kFindLocal),
                       static_cast<const double2*>(nullptr), static_cast<const int8_t*>(nullptr),
                       static_cast<const int32_t*>(nullptr));
    SML_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(vote_kernel, dim3(1), dim3(kVoteThreads), 0, stream_, st_cur_, floc_.get(), F_,
                       std::max(1, cfg_.top_k), local_count, vote_.get());
    SML_HIP_CHECK(hipGetLastError());
    TimedAllReduce(vote_.get(), 4 * static_cast<int64_t>(F_) + 1);
    hipLaunchKernelGGL(select_kernel, dim3(1), dim3(kVoteThreads), 0, stream_, st_cur_, vote_.get(), F_, vote_k2_,
                       mask_.get(), sel_idx_.get(), sel_pos_.get(), sel_mask_.get());
    SML_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(pack_kernel, dim3(vote_k2_, 2), dim3(256), 0, stream_, st_cur_, leaves_.get(), sel_idx_.get(),
                       vote_k2_, hist_pool_.get(), E_, compact_.get());
    SML_HIP_CHECK(hipGetLastError());
    TimedAllReduce(reinterpret_cast<double*>(compact_.get()), 2 * 2 * static_cast<int64_t>(vote_k2_) * kBinsPerFeature);
    hipLaunchKernelGGL(unpack_kernel, dim3(F_, 2), dim3(256), 0, stream_, st_cur_, sel_pos_.get(), F_, vote_k2_,
                       compact_.get(), E_, gh_.get());
    SML_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(find_split_kernel, dim3(F_, 2), dim3(256), 0, stream_, st_cur_, leaves_.get(), gh_.get(), E_,
                       CountSlot(), hist_pool_.get(), fm_, sp_, fbest_.get(), F_, st_next_,
                       static_cast<int>(kFindVoted), static_cast<const double2*>(gh_.get() + E_),
                       static_cast<const int8_t*>(sel_mask_.get()), static_cast<const int32_t*>(sel_idx_.get()));
    SML_HIP_CHECK(hipGetLastError());
  }

  // root (choose_now = false): choose_part_kernel does the choose step with the next partition
  void EnqueueFindChoose(bool choose_now) {
    // (A/B, round 3: folding this search into the slab reduce - the last of a feature's 8 reduce blocks
    // searching it after a device-scope release/acquire hand-off - ran 3.11 vs 2.14 ms/iter: the per-block
    // fences cost more than the launch they save)
    if (voting_) {
      EnqueueVote();
    } else {
      hipLaunchKernelGGL(find_split_kernel, dim3(F_, 2), dim3(256), 0, stream_, st_cur_, leaves_.get(), part_.get(),
                         E_, CountSlot(), hist_pool_.get(), fm_, sp_, fbest_.get(), F_, st_next_,
                         static_cast<int>(kFindFull), static_cast<const double2*>(nullptr),
                         static_cast<const int8_t*>(nullptr), static_cast<const int32_t*>(nullptr));
      SML_HIP_CHECK(hipGetLastError());
    }
    if (!choose_now) return;
    hipLaunchKernelGGL(choose_kernel, dim3(1), dim3(256), 0, stream_, st_cur_, leaves_.get(), lbest_.get(),
                       lgain_.get(), fbest_.get(), F_, dt_, CountSlot(), mono_.get(), sp_.has_mono);
    SML_HIP_CHECK(hipGetLastError());
  }

  // parse the tree copied by EnqueueTreeCopy (the caller has waited for the copy)
  Tree ReadTree() {
    const int NI = L_ - 1;
    if (comm_) comm_->Check();
    const uint8_t* hb = static_cast<const uint8_t*>(pinned_);
    DState st;
    std::memcpy(&st, hb + final_v_ * sizeof(DState), sizeof(DState));
    const int32_t* ti = reinterpret_cast<const int32_t*>(hb + off_ti_);
    const uint32_t* tu = reinterpret_cast<const uint32_t*>(hb + off_tu_);
    const double* td = reinterpret_cast<const double*>(hb + off_td_);
    const int64_t* tl = reinterpret_cast<const int64_t*>(hb + off_tl_);
    const int nl = st.num_leaves;
    Tree t(L_);
    t.num_leaves = nl;
    const auto& ref = data_->ref;
    // leaf 0 of a stump: LeafOutput of the root
    for (int node = 0; node < nl - 1; ++node) {
      const int fi = ti[node];
      const int fr = ref.used_features[fi];
      const BinMapper& m = ref.mappers[fr];
      t.split_feature_inner[node] = fi;
      t.split_feature[node] = fr;
      t.split_gain[node] = td[node];
      t.left_child[node] = ti[3 * NI + node];
      t.right_child[node] = ti[4 * NI + node];
      t.internal_value[node] = td[NI + node];
      t.internal_weight[node] = td[2 * NI + node];
      t.internal_count[node] = tl[node];
      const bool is_cat = ti[2 * NI + node] != 0;
      if (is_cat) {
        std::vector<uint32_t> binbits(8), valbits;
        int maxcat = 0;
        for (int w = 0; w < 8; ++w) binbits[w] = tu[NI + node * 8 + w];
        for (int b = 0; b < m.num_bin - 1; ++b) if ((binbits[b / 32] >> (b % 32)) & 1u) maxcat = std::max(maxcat, m.bin2cat[b]);
        valbits.assign(maxcat / 32 + 1, 0);
        for (int b = 0; b < m.num_bin - 1; ++b)
          if ((binbits[b / 32] >> (b % 32)) & 1u) valbits[m.bin2cat[b] / 32] |= 1u << (m.bin2cat[b] % 32);
        t.threshold_in_bin[node] = static_cast<uint32_t>(t.num_cat);
        t.threshold[node] = static_cast<double>(t.num_cat);
        t.decision_type[node] = MakeDecisionType(true, false, kMissingNaN);
        t.cat_threshold.insert(t.cat_threshold.end(), valbits.begin(), valbits.end());
        t.cat_boundaries.push_back(static_cast<int>(t.cat_threshold.size()));
        t.cat_threshold_inner.insert(t.cat_threshold_inner.end(), binbits.begin(), binbits.end());
        t.cat_boundaries_inner.push_back(static_cast<int>(t.cat_threshold_inner.size()));
        ++t.num_cat;
      } else {
        const uint32_t thr = tu[node];
        t.threshold_in_bin[node] = thr;
        t.threshold[node] = m.BinToValue(thr);
        t.decision_type[node] = MakeDecisionType(false, ti[NI + node] != 0, m.missing_type);
      }
    }
    for (int l = 0; l < nl; ++l) {
      t.leaf_value[l] = td[3 * NI + l];
      t.leaf_weight[l] = td[3 * NI + L_ + l];
      t.leaf_count[l] = tl[NI + l];
      t.leaf_parent[l] = ti[6 * NI + l];
      t.leaf_depth[l] = ti[6 * NI + L_ + l];
    }
    if (nl == 1) t.leaf_value[0] = 0.0;
    return t;
  }

  DevTreeView UploadTree(const Tree& t) {
    const int NI = std::max(1, t.num_leaves - 1);
    const size_t need_n = static_cast<size_t>(NI), need_u = static_cast<size_t>(NI) * 8, need_d = t.num_leaves;
    const size_t bytes = need_n * 16 + need_u * 4 + need_d * 8;
    if (bytes > kPinnedBytes) throw std::runtime_error("tree too large for staging buffer");
    SML_HIP_CHECK(hipStreamSynchronize(stream_));  // pinned buffer reuse
    int4* pn = static_cast<int4*>(pinned_);
    uint32_t* pu = reinterpret_cast<uint32_t*>(pn + need_n);
    double* pd = reinterpret_cast<double*>(pu + need_u);
    for (int node = 0; node < t.num_leaves - 1; ++node) {
      const int8_t dt = t.decision_type[node];
      const int mt = (dt >> 2) & 3, dl = (dt >> 1) & 1, ic = dt & 1;
      const BinMapper& m = data_->ref.mappers[data_->ref.used_features[t.split_feature_inner[node]]];
      const int mbin = mt == kMissingNaN ? m.num_bin - 1 : (mt == kMissingZero ? m.default_bin : 0);
      pn[node] = make_int4(t.split_feature_inner[node] | (mt << 16) | (dl << 18) | (ic << 19) | (mbin << 20),
                           static_cast<int>(t.threshold_in_bin[node]), t.left_child[node], t.right_child[node]);
      for (int w = 0; w < 8; ++w) pu[node * 8 + w] = 0;
      if (ic) {
        int ci = static_cast<int>(t.threshold_in_bin[node]);
        int s0 = t.cat_boundaries_inner[ci], e0 = t.cat_boundaries_inner[ci + 1];
        for (int w = 0; w < 8 && s0 + w < e0; ++w) pu[node * 8 + w] = t.cat_threshold_inner[s0 + w];
      }
    }
    for (int l = 0; l < t.num_leaves; ++l) pd[l] = t.leaf_value[l];
    // nodes | cat words | leaf values are contiguous in the pinned buffer: one H2D copy
    if (bytes > up_blob_.n) up_blob_.alloc(bytes);
    SML_HIP_CHECK(hipMemcpyAsync(up_blob_.get(), pinned_, bytes, hipMemcpyHostToDevice, stream_));
    DevTreeView tv;
    tv.nodes = reinterpret_cast<const int4*>(up_blob_.get());
    tv.cat_bits = reinterpret_cast<const uint32_t*>(up_blob_.get() + need_n * 16);
    tv.lval = reinterpret_cast<const double*>(up_blob_.get() + need_n * 16 + need_u * 4);
    tv.num_leaves = t.num_leaves;
    return tv;
  }

  static constexpr size_t kPinnedBytes = 4 << 20;
  hipEvent_t ev_[4] = {nullptr, nullptr, nullptr, nullptr};  // tree start/end, score start/end
  hipEvent_t ev_copy_ = nullptr;                               // tree copied to pinned memory
  bool score_pending_ = false;
  int dev_ = -1;
  hipStream_t stream_ = nullptr;
  const Dataset* data_ = nullptr;
  Config cfg_;
  SplitParams sp_{};
  int K_ = 1, F_ = 0, S_ = 4, W_ = 1, E_ = 0, L_ = 2, FG_ = 1;
  int hist_fpg_ = kFeatPerGroup;  // SML_HIST_FPG=16: half-width feature groups for the per-split histogram
  bool hist_unroll4_ = false;     // SML_HIST_UNROLL=4: 4 gathered rows in flight per thread (A/B knob)
  bool hist_pipe_ = false;        // SML_GBDT_HIST_PIPE=1: software-pipelined histogram loops (A/B knob)
  bool root_pipe_ = false;        // SML_GBDT_ROOT_PIPE=1: software-pipelined root pass (A/B knob)
  bool tight_ = false;            // h LDS plane inside the DS offset range of the g plane (F <= 28; SML_HIST_TIGHT=0 off)
  // lambdarank register kernel: waves per block. SML_RANK_WAVES=4 packs 4 independent waves per block (up
  // to 10 resident per SIMD instead of 4): r4 pass 11 measured it slower (949 vs 860 us per call, ranker
  // fit 33.6M vs 34.0M rows/s), so one-wave blocks stay the default
  int rank_waves_ = 1;
  int rank_nbig_ = 0;       // register-path queries of > 128 documents (the front of rank_order_)
  bool rank_split_ = true;  // SML_RANK_SPLIT=0: one launch of the full kernel for all register-path queries
  int rank_small_waves_ = 1;  // SML_RANK_SMALL_WAVES=4: the small-query launch in 4-wave blocks
  bool rank_treduce_ = true;  // SML_RANK_TREDUCE=0: one pair of wave sums per top document (A/B knob)
  int64_t n_ = 0;
  int32_t bag_n_ = -1;
  DevBuf<uint8_t> bins_, cbins_;           // bins_: own upload when the dataset is not device-resident
  std::shared_ptr<DeviceBins> dev_bins_;   // adopted K1 output (keeps it alive)
  const uint8_t* bins_ptr_ = nullptr;      // row-major bin matrix the kernels read
  DevBuf<float> label_, weight_, g_, h_;
  DevBuf<double> score_;
  DevBuf<int32_t> perm_[2];
  DevBuf<float2> ogh_[2];
  DevBuf<ulonglong2> slab_;
  DevBuf<double2> part_, hist_pool_;
  DevBuf<double> lgain_;
  DevBuf<SplitResult> fbest_, lbest_;
  DevBuf<DLeaf> leaves_;
  DevBuf<int32_t> meta_i_, bag_;
  DevBuf<int8_t> mask_, mono_;
  DevBuf<unsigned int> ghmax_;
  DevBuf<float> ghslot_;   // data-parallel: per-rank slots of the global max |g| / max h
  int64_t scale_n_ = 0;    // global row count: the histogram scale's count bound
  // Fusing reduce / find / choose into one launch (F blocks, slab reduce inside) measured slower on MI355X
  // (2.05 vs 1.97 ms/iter: 28 blocks cannot pull the slabs fast enough; profiles/README, round 2)
  bool skip_last_ = true;  // SML_SKIP_LAST_SPLIT=0: histogram + search the last split's children too
  bool comm_world1_ = false;
  // tree_learner=voting (PV-Tree, C3): local search results, votes, selection and the reduced histograms
  bool voting_ = false;
  int vote_k2_ = 0;          // features reduced per leaf: min(2 top_k, F)
  SplitParams sp_local_{};   // min_data_in_leaf / min_sum_hessian divided by the world size
  DevBuf<SplitResult> floc_;
  DevBuf<double> vote_;
  DevBuf<int32_t> sel_idx_, sel_pos_;
  DevBuf<int8_t> sel_mask_;
  DevBuf<double2> compact_, gh_;
  DevBuf<float> ghmax_partial_;
  // event pairs around this tree's histogram allreduces (device comm time, summed when the tree is read)
  std::vector<hipEvent_t> comm_ev_;
  int comm_used_ = 0;
  hipEvent_t ev_sync_ = nullptr;
  void EnsureCommEvents() {
    if (!comm_ev_.empty()) return;
    comm_ev_.assign(4 * static_cast<size_t>(L_ + 1), nullptr);  // voting: two collectives per split
    for (hipEvent_t& e : comm_ev_) SML_HIP_CHECK(hipEventCreate(&e));
  }
  int tree_seq_ = 0;  // trees grown so far (feature_fraction_bynode node keys)
  bool ghmax_valid_ = false;  // ghmax_ already holds this iteration's class-0 maxima (from grad_kernel)
  int pending_parts_ = 0;     // > 0: ghmax_ is the max over that many block partials, folded by root_init_kernel
  // fused score update + gradients + root histogram (score_grad_hist_kernel)
  bool prep_ok_ = false;      // dataset / config eligible
  bool prep_armed_ = false;   // the last ComputeGradients used an objective with a-priori bounds
  bool prep_valid_ = false;   // g, h and the root slabs match the current scores (set by UpdateScore)
  bool root_ready_ = false;   // ComputeGradients consumed them: the next TrainTree skips its root histogram
  ObjParams prep_params_{};
  int prep_blocks_ = 0;
  int min_rows_hist_ = kMinRowsPerHistBlockDefault;
  double wmax_ = 1.0, ymax_ = 0.0;
  float bound_host_[2] = {-1.f, -1.f};
  DevBuf<float> ghbound_;  // a-priori max |g|, max h: the fused pass's fixed-point scale
  std::vector<int8_t> mask_host_;
  int part_grid_ = 1;
  int part_rows_ = kPartRowsDefault;
  // A feature-lane, bank-conflict-free histogram (lane = feature) measured slower on MI355X (2.28 vs 3.01
  // ms/iter: 16x the memory instructions per row cost more than the conflicts it removes; profiles/README)
  DevBuf<uint8_t> blob_;
  DState* state_ = nullptr;   // two versions: choose_part_kernel reads one and writes the other
  DState* st_cur_ = nullptr;  // version the next hist / reduce / find / choose launches read
  DState* st_next_ = nullptr; // version whose cursor find_split_kernel zeroes (nullptr: none)
  int final_v_ = 0;           // version holding the finished tree's state
  size_t n_ti_ = 0, n_tu_ = 0, n_td_ = 0, n_tl_ = 0;
  size_t off_td_ = 0, off_tl_ = 0, off_ti_ = 0, off_tu_ = 0, blob_bytes_ = 0;
  DevBuf<uint8_t> up_blob_;  // uploaded score-update tree: nodes | cat words | leaf values
  DevBuf<int32_t> leaf_idx_;
  // device row sampling (K8)
  DevBuf<SelectState> sel_;
  DevBuf<uint32_t> sel_key_;
  DevBuf<unsigned int> sel_hist_;
  // lambdarank (K2 ranking)
  bool rank_ready_ = false, rank_regs_ = false, rank_lds_ = false;
  RankTables rank_{};
  DevBuf<int32_t> rank_qb_, rank_scratch_, rank_order_;
  std::vector<std::unique_ptr<DeviceValidSet>> vsets_;
  DevBuf<double> rank_imd_, rank_gain_, rank_lam_, rank_hes_, rank_disc_;
  int32_t* flags_ = nullptr;
  // batched speculative growth
  static constexpr int kBRing = 8;
  bool batch_ok_ = false;
  int spec_k_ = 4;
  int spec_max_ = 4, wide_div_ = 0;  // adaptive round width (bplan_kernel)
  // the fused score pass reads every row's leaf from row_leaf_ (leaf_scatter_kernel) after batched growth;
  // SML_GBDT_ROW_LEAF=0 walks the tree per row instead
  bool row_leaf_on_ = !(std::getenv("SML_GBDT_ROW_LEAF") && std::atoi(std::getenv("SML_GBDT_ROW_LEAF")) == 0);
  bool grew_batched_ = false;
  DevBuf<int4> lseg_, rtab_;
  DevBuf<uint8_t> row_leaf_;
  int blook_ = 1;
  DevBuf<BState> bstate_;
  DevBuf<BNode> bnodes_;
  DevBuf<SplitResult> nbest_;
  int* bflag_host_ = nullptr;
  int* bflag_dev_ = nullptr;
  int plan_cap_ = 0;            // node records allocated for the batched growth (the plan stages them all)
  // index-only partition: interleaved (g, h) of class 0; gh2_valid_: it holds the current gradients; g_stale_:
  // g_ / h_ do not (the fused pass wrote only gh2_) - EnsureGH unpacks before anything reads them
  int64_t comm_bytes0_ = 0;
  bool idx_ok_ = false;
  bool gh2_valid_ = false;
  bool g_stale_ = false;
  DevBuf<float2> gh2_;
  long long* bprof_ = nullptr;  // SML_BPLAN_PROF phase stamps, kPlanProfStride per round
  double bprof_sum_[6] = {0, 0, 0, 0, 0, 0};
  double bprof_tree_[4] = {0, 0, 0, 0};  // rows partitioned, of them in never-popped nodes; expansions, wasted
  long long bprof_trees_ = 0;
  long long bprof_n_ = 0;
  hipEvent_t bev_[kBRing] = {};
  DTree dt_{};
  FeatMeta fm_{};
  void* pinned_ = nullptr;
};

}  // namespace

bool GpuAvailable() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) { (void)hipGetLastError(); return false; }
  return n > 0;
}

std::unique_ptr<TrainBackend> MakeGpuBackend(int device_id) {
  if (!GpuAvailable()) return nullptr;
  return std::unique_ptr<TrainBackend>(new GpuBackend(device_id));
}

}  // namespace sml
