// K12: hogwild mini-batch hashed SGD on the MI355X. One wave64 per example:
// lanes stride over the example's features, gather w[h & mask], reduce the dot
// product with DPP shuffles, evaluate the loss derivative once per wave and
// scatter AdaGrad updates back with float atomics (conflicts are rare in a
// 2^b table, which is what makes hogwild converge like sequential SGD).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <string>
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

__device__ __forceinline__ void ExampleStep(const int64_t* __restrict__ indptr, const uint32_t* __restrict__ idx,
                                            const float* __restrict__ val, const float* __restrict__ labels,
                                            const float* __restrict__ weights, int64_t e, float2* __restrict__ W,
                                            uint64_t mask, float lr, float l2, int loss, int adaptive, float eta_scale,
                                            float* __restrict__ preds, int learn, int lane, float* wloss) {
  const int64_t b = indptr[e], en = indptr[e + 1];
  float s = 0.f;
  for (int64_t p = b + lane; p < en; p += 64) s += W[idx[p] & mask].x * val[p];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (preds && lane == 0) preds[e] = s;
  if (!learn) return;
  const float y = labels[e];
  const float imp = weights ? weights[e] : 1.f;
  float g, l;
  if (loss == 1) {
    const float m = y * s;
    g = -y / (1.f + expf(m));
    l = log1pf(expf(-m));
  } else {
    g = 2.f * (s - y);
    l = (s - y) * (s - y);
  }
  if (lane == 0) *wloss = l * imp;
  g *= imp;
  for (int64_t p = b + lane; p < en; p += 64) {
    const uint64_t h = idx[p] & mask;
    const float x = val[p];
    const float gx = g * x;
    float step;
    if (adaptive) {
      const float G = atomicAdd(&W[h].y, gx * gx) + gx * gx;
      step = lr * gx * rsqrtf(G + 1e-12f);
    } else {
      step = lr * eta_scale * gx;
    }
    if (l2 > 0.f) step += lr * l2 * W[h].x;
    atomicAdd(&W[h].x, -step);
  }
}

__global__ __launch_bounds__(256) void sgd_kernel(const int64_t* __restrict__ indptr, const uint32_t* __restrict__ idx,
                                                  const float* __restrict__ val, const float* __restrict__ labels,
                                                  const float* __restrict__ weights, int64_t n0, int64_t n1,
                                                  float2* __restrict__ W, uint64_t mask, float lr, float l2, int loss,
                                                  int adaptive, float eta_scale, float* __restrict__ preds,
                                                  float* __restrict__ loss_acc, int learn) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t e = n0 + static_cast<int64_t>(blockIdx.x) * kWavesPerBlock + wid;
  __shared__ float wloss[kWavesPerBlock];
  if (lane == 0) wloss[wid] = 0.f;
  if (e < n1) ExampleStep(indptr, idx, val, labels, weights, e, W, mask, lr, l2, loss, adaptive, eta_scale, preds,
                          learn, lane, &wloss[wid]);
  // one loss atomic per block (a same-address atomic per example serialises the launch)
  if (learn) {
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(loss_acc, wloss[0] + wloss[1] + wloss[2] + wloss[3]);
  }
}

__global__ void scale_kernel(float* w, uint64_t n, float s) {
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    w[i] *= s;
}

}  // namespace

struct GpuSgd::Impl {
  hipStream_t stream = nullptr, copy_stream = nullptr;
  std::vector<hipEvent_t> events;
  float2* W = nullptr;
  uint64_t nw = 0;
  int64_t* indptr = nullptr;
  uint32_t* idx = nullptr;
  float *val = nullptr, *lab = nullptr, *wt = nullptr, *pred = nullptr, *loss = nullptr;
  size_t cap_rows = 0, cap_nnz = 0;
  void Reserve(size_t rows, size_t nnz) {
    if (rows > cap_rows) {
      (void)hipFree(indptr); (void)hipFree(lab); (void)hipFree(wt); (void)hipFree(pred);
      VW_HIP_CHECK(hipMalloc(&indptr, (rows + 1) * sizeof(int64_t)));
      VW_HIP_CHECK(hipMalloc(&lab, rows * sizeof(float)));
      VW_HIP_CHECK(hipMalloc(&wt, rows * sizeof(float)));
      VW_HIP_CHECK(hipMalloc(&pred, rows * sizeof(float)));
      cap_rows = rows;
    }
    if (nnz > cap_nnz) {
      (void)hipFree(idx); (void)hipFree(val);
      VW_HIP_CHECK(hipMalloc(&idx, nnz * sizeof(uint32_t)));
      VW_HIP_CHECK(hipMalloc(&val, nnz * sizeof(float)));
      cap_nnz = nnz;
    }
  }
  ~Impl() {
    if (stream) (void)hipStreamSynchronize(stream);
    if (copy_stream) (void)hipStreamSynchronize(copy_stream);
    for (hipEvent_t e : events) (void)hipEventDestroy(e);
    if (copy_stream) (void)hipStreamDestroy(copy_stream);
    (void)hipFree(W); (void)hipFree(indptr); (void)hipFree(idx); (void)hipFree(val);
    (void)hipFree(lab); (void)hipFree(wt); (void)hipFree(pred); (void)hipFree(loss);
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
  VW_HIP_CHECK(hipStreamCreateWithFlags(&impl_->stream, hipStreamNonBlocking));
  VW_HIP_CHECK(hipStreamCreateWithFlags(&impl_->copy_stream, hipStreamNonBlocking));
  impl_->nw = 1ull << cfg.bits;
  VW_HIP_CHECK(hipMalloc(&impl_->W, impl_->nw * sizeof(float2)));
  VW_HIP_CHECK(hipMemsetAsync(impl_->W, 0, impl_->nw * sizeof(float2), impl_->stream));
  VW_HIP_CHECK(hipMalloc(&impl_->loss, sizeof(float)));
  VW_HIP_CHECK(hipMemsetAsync(impl_->loss, 0, sizeof(float), impl_->stream));
  VW_HIP_CHECK(hipStreamSynchronize(impl_->stream));
}

GpuSgd::~GpuSgd() = default;

void GpuSgd::Learn(const int64_t* indptr, const uint32_t* indices, const float* values, const float* labels,
                   const float* weights, int64_t n, int batch, float* preds_out) {
  if (n <= 0) return;
  const size_t nnz = static_cast<size_t>(indptr[n] - indptr[0]);
  impl_->Reserve(n, nnz);
  hipStream_t s = impl_->stream, cs = impl_->copy_stream;
  std::vector<int64_t> ip(indptr, indptr + n + 1);
  for (auto& v : ip) v -= indptr[0];
  VW_HIP_CHECK(hipMemcpyAsync(impl_->indptr, ip.data(), (n + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  VW_HIP_CHECK(hipMemcpyAsync(impl_->lab, labels, n * sizeof(float), hipMemcpyHostToDevice, s));
  if (weights) VW_HIP_CHECK(hipMemcpyAsync(impl_->wt, weights, n * sizeof(float), hipMemcpyHostToDevice, s));
  VW_HIP_CHECK(hipMemsetAsync(impl_->loss, 0, sizeof(float), s));
  const uint64_t mask = impl_->nw - 1;
  batch = std::max(1, batch);
  // The pass's feature ids / values stream in chunks of 16 mini-batches on a copy stream: the
  // (host-blocking, pageable) copy of chunk k+1 runs while the device learns chunk k, so the
  // host->device traffic (8 B per nonzero) hides behind the SGD instead of preceding it.
  const int64_t chunk_rows = static_cast<int64_t>(batch) * 16;
  const int64_t nchunks = (n + chunk_rows - 1) / chunk_rows;
  if (impl_->events.size() < static_cast<size_t>(nchunks)) {
    for (size_t i = impl_->events.size(); i < static_cast<size_t>(nchunks); ++i) {
      hipEvent_t e;
      VW_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      impl_->events.push_back(e);
    }
  }
  auto copy_chunk = [&](int64_t c) {
    const int64_t r0 = c * chunk_rows, r1 = std::min<int64_t>(n, r0 + chunk_rows);
    const size_t p0 = static_cast<size_t>(ip[r0]), p1 = static_cast<size_t>(ip[r1]);
    if (p1 > p0) {
      VW_HIP_CHECK(hipMemcpyAsync(impl_->idx + p0, indices + indptr[0] + p0, (p1 - p0) * sizeof(uint32_t),
                                  hipMemcpyHostToDevice, cs));
      VW_HIP_CHECK(hipMemcpyAsync(impl_->val + p0, values + indptr[0] + p0, (p1 - p0) * sizeof(float),
                                  hipMemcpyHostToDevice, cs));
    }
    VW_HIP_CHECK(hipEventRecord(impl_->events[c], cs));
  };
  copy_chunk(0);
  for (int64_t c = 0; c < nchunks; ++c) {
    VW_HIP_CHECK(hipStreamWaitEvent(s, impl_->events[c], 0));
    const int64_t r0 = c * chunk_rows, r1 = std::min<int64_t>(n, r0 + chunk_rows);
    for (int64_t b0 = r0; b0 < r1; b0 += batch) {
      const int64_t b1 = std::min<int64_t>(r1, b0 + batch);
      const float eta = static_cast<float>(std::pow(examples_ + b0 + 1.0, -static_cast<double>(cfg_.power_t)));
      const int grid = static_cast<int>((b1 - b0 + kWavesPerBlock - 1) / kWavesPerBlock);
      hipLaunchKernelGGL(sgd_kernel, dim3(grid), dim3(64 * kWavesPerBlock), 0, s, impl_->indptr, impl_->idx,
                         impl_->val, impl_->lab, weights ? impl_->wt : nullptr, b0, b1, impl_->W, mask, cfg_.lr,
                         cfg_.l2, cfg_.loss, cfg_.adaptive ? 1 : 0, eta, impl_->pred, impl_->loss, 1);
      VW_HIP_CHECK(hipGetLastError());
    }
    if (c + 1 < nchunks) copy_chunk(c + 1);
  }
  float l = 0;
  VW_HIP_CHECK(hipMemcpyAsync(&l, impl_->loss, sizeof(float), hipMemcpyDeviceToHost, s));
  if (preds_out) VW_HIP_CHECK(hipMemcpyAsync(preds_out, impl_->pred, n * sizeof(float), hipMemcpyDeviceToHost, s));
  VW_HIP_CHECK(hipStreamSynchronize(s));
  examples_ += n;
  sum_loss_ += l;
}

void GpuSgd::Predict(const int64_t* indptr, const uint32_t* indices, const float* values, int64_t n, float* out) {
  if (n <= 0) return;
  const size_t nnz = static_cast<size_t>(indptr[n] - indptr[0]);
  impl_->Reserve(n, nnz);
  hipStream_t s = impl_->stream;
  std::vector<int64_t> ip(indptr, indptr + n + 1);
  for (auto& v : ip) v -= indptr[0];
  VW_HIP_CHECK(hipMemcpyAsync(impl_->indptr, ip.data(), (n + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  VW_HIP_CHECK(hipMemcpyAsync(impl_->idx, indices + indptr[0], nnz * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  VW_HIP_CHECK(hipMemcpyAsync(impl_->val, values + indptr[0], nnz * sizeof(float), hipMemcpyHostToDevice, s));
  const int grid = static_cast<int>((n + kWavesPerBlock - 1) / kWavesPerBlock);
  hipLaunchKernelGGL(sgd_kernel, dim3(grid), dim3(64 * kWavesPerBlock), 0, s, impl_->indptr, impl_->idx, impl_->val,
                     nullptr, nullptr, int64_t(0), n, impl_->W, impl_->nw - 1, 0.f, 0.f, 0, 0, 0.f, impl_->pred,
                     impl_->loss, 0);
  VW_HIP_CHECK(hipGetLastError());
  VW_HIP_CHECK(hipMemcpyAsync(out, impl_->pred, n * sizeof(float), hipMemcpyDeviceToHost, s));
  VW_HIP_CHECK(hipStreamSynchronize(s));
}

void GpuSgd::AllReduceAverage(void* comm, int world) {
  if (world < 1 || !comm) return;  // a world-1 communicator still runs the collective (one-GPU tests)
  hipStream_t s = impl_->stream;
  ncclComm_t c = static_cast<ncclComm_t>(comm);
  const uint64_t nf = impl_->nw * 2;
  ncclResult_t r = ncclAllReduce(impl_->W, impl_->W, nf, ncclFloat, ncclSum, c, s);
  if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL allreduce failed: ") + ncclGetErrorString(r));
  hipLaunchKernelGGL(scale_kernel, dim3(4096), dim3(256), 0, s, reinterpret_cast<float*>(impl_->W), nf, 1.f / world);
  VW_HIP_CHECK(hipGetLastError());
  VW_HIP_CHECK(hipStreamSynchronize(s));
}

uint64_t GpuSgd::NumWeights() const { return impl_->nw; }

void GpuSgd::CopyWeights(float* host_out) const {
  std::vector<float2> tmp(impl_->nw);
  VW_HIP_CHECK(hipMemcpy(tmp.data(), impl_->W, impl_->nw * sizeof(float2), hipMemcpyDeviceToHost));
  for (uint64_t i = 0; i < impl_->nw; ++i) host_out[i] = tmp[i].x;
}

void GpuSgd::SetWeights(const float* host_in) {
  std::vector<float2> tmp(impl_->nw);
  for (uint64_t i = 0; i < impl_->nw; ++i) tmp[i] = make_float2(host_in[i], 0.f);
  VW_HIP_CHECK(hipMemcpy(impl_->W, tmp.data(), impl_->nw * sizeof(float2), hipMemcpyHostToDevice));
}

void* GpuSgd::weights_device() { return impl_->W; }
void* GpuSgd::stream() { return impl_->stream; }

}  // namespace smlvw
