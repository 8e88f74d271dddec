// One-shot peer-to-peer allreduce for small device messages (K21 of SURVEY
// §2.4; call sites C2 §2.5).
//
// The reference reduces LightGBM histograms with lib_lightgbm's TCP socket
// linkers after the driver rendezvous (lightgbm/.../NetworkManager.scala:
// 195-218).  Data-parallel tree growth does one allreduce of the smaller
// child's histogram per split (28 x 255 bins x (g,h) doubles + count ~ 114 KB,
// ~30 per tree) and nothing can overlap it: the next split search needs the
// result.  At that size a ring allreduce is latency-bound (2(N-1) dependent
// hops), so intra-node we do it in ONE kernel and one xGMI hop:
//
//   * every rank owns an uncached (fine-grained) receive area
//     recv[parity][src][cap] plus signal words sig[src][block], exported with
//     hipIpcGetMemHandle and mapped by all peers (handles are exchanged over
//     the base communicator, so no extra rendezvous);
//   * block b of rank r pushes its chunk of the input straight into every
//     peer's recv[parity][r] (posted xGMI writes, no round trip), fences at
//     system scope and raises sig[r][b] = epoch on each peer;
//   * block b then waits for all peers' sig[q][b] and sums the N chunks in
//     fixed rank order, so every rank gets the bitwise-identical result (all
//     ranks must pick the same split) and the result is deterministic.
//
// Two parities make back-to-back calls safe: a rank can only start call k+1
// after all peers raised their call-k signals, which they do after finishing
// call k-1, the last reader of parity (k+1)&1.  Waits are bounded by a
// wall-clock timeout that sets a host-visible error flag (no GPU hang); the
// comm validates itself against the base communicator at start-up and all
// ranks fall back to it together if anything fails.  Messages larger than the
// receive slot go to the base communicator (RCCL multi-channel).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "comm.h"
#include "hip_common.h"

namespace sml {
namespace {

constexpr int kMaxRanks = 8;
constexpr int kP2pThreads = 256;
constexpr int kMaxBlocks = 64;

struct PeerPtrs {
  char* recv[kMaxRanks];     // peer q's receive area base (mapped)
  uint32_t* sig[kMaxRanks];  // peer q's signal words (mapped)
};

// 16-byte vectors of T for the data movement (uncached, xGMI-mapped memory
// wants full-width transactions); VW == 1 handles unaligned buffers.
template <class T, int VW>
struct VecOf {
  T v[VW];
};

// units != nullptr: only the first min(n, *units * per_unit) elements travel (every block still signals, so the
// epochs stay in step); bytes (when set) counts what this rank pushed
template <class T, int VW>
__global__ __launch_bounds__(kP2pThreads) void p2p_allreduce_kernel(PeerPtrs peers, const T* in, T* out, int64_t n,
                                                                    int64_t chunk, int64_t cap_bytes, int rank,
                                                                    int world, uint32_t epoch, long long timeout_ticks,
                                                                    int* err, const int32_t* units, int64_t per_unit,
                                                                    unsigned long long* bytes) {
  using V = VecOf<T, VW>;
  if (units) n = min(n, static_cast<int64_t>(max(0, *units)) * per_unit);
  if (bytes && blockIdx.x == 0 && threadIdx.x == 0)
    atomicAdd(bytes, static_cast<unsigned long long>(n) * sizeof(T) * static_cast<unsigned long long>(world - 1));
  const int b = blockIdx.x;
  const int64_t lo = static_cast<int64_t>(b) * chunk;  // chunk is a multiple of VW
  const int64_t hi = min(n, lo + chunk);
  const int64_t vhi = lo + (hi - lo) / VW * VW;
  const int par = epoch & 1;
  const size_t slot_bytes = static_cast<size_t>(cap_bytes);
  const size_t par_bytes = slot_bytes * kMaxRanks;

  // push my chunk into every peer's recv[par][rank]
  const size_t my_off = par * par_bytes + rank * slot_bytes;
  for (int64_t i = lo + threadIdx.x * VW; i < vhi; i += kP2pThreads * VW) {
    const V v = *reinterpret_cast<const V*>(in + i);
    for (int q = 0; q < world; ++q)
      if (q != rank) *reinterpret_cast<V*>(reinterpret_cast<T*>(peers.recv[q] + my_off) + i) = v;
  }
  for (int64_t i = vhi + threadIdx.x; i < hi; i += kP2pThreads) {
    const T v = in[i];
    for (int q = 0; q < world; ++q)
      if (q != rank) reinterpret_cast<T*>(peers.recv[q] + my_off)[i] = v;
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < world && threadIdx.x != rank) {
    __hip_atomic_store(peers.sig[threadIdx.x] + rank * kMaxBlocks + b, epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // wait for every peer's chunk b
  if (threadIdx.x < world && threadIdx.x != rank) {
    const uint32_t* s = peers.sig[rank] + threadIdx.x * kMaxBlocks + b;
    const long long t0 = wall_clock64();
    while (static_cast<int32_t>(__hip_atomic_load(s, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > timeout_ticks) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __syncthreads();
  __threadfence_system();
  // reduce in rank order (identical on every rank)
  const char* mine = peers.recv[rank] + par * par_bytes;
  for (int64_t i = lo + threadIdx.x * VW; i < vhi; i += kP2pThreads * VW) {
    V acc;
#pragma unroll
    for (int j = 0; j < VW; ++j) acc.v[j] = 0;
    for (int q = 0; q < world; ++q) {
      const V v = (q == rank) ? *reinterpret_cast<const V*>(in + i)
                              : *reinterpret_cast<const V*>(reinterpret_cast<const T*>(mine + q * slot_bytes) + i);
#pragma unroll
      for (int j = 0; j < VW; ++j) acc.v[j] += v.v[j];
    }
    *reinterpret_cast<V*>(out + i) = acc;
  }
  for (int64_t i = vhi + threadIdx.x; i < hi; i += kP2pThreads) {
    T acc = 0;
    for (int q = 0; q < world; ++q)
      acc += (q == rank) ? in[i] : reinterpret_cast<const T*>(mine + q * slot_bytes)[i];
    out[i] = acc;
  }
}

class P2pComm : public Comm {
 public:
  P2pComm(std::shared_ptr<Comm> base, int device, int64_t cap_bytes, double timeout_ms)
      : base_(std::move(base)), rank_(base_->rank()), world_(base_->world()), cap_((cap_bytes + 15) / 16 * 16) {
    if (world_ > kMaxRanks) throw std::runtime_error("p2p allreduce supports at most 8 ranks (one node)");
    if (device >= 0) SML_HIP_CHECK(hipSetDevice(device));
    timeout_ticks_ = static_cast<long long>(timeout_ms * 1e5);  // wall_clock64 runs at 100 MHz
    bool ok = true;
    std::string why;
    try {
      Setup();
    } catch (const std::exception& e) {
      ok = false;
      why = e.what();
    }
    ok = Agree(ok);
    if (ok) {
      try {
        ok = SelfTest();
      } catch (const std::exception& e) {
        ok = false;
        why = e.what();
      }
      ok = Agree(ok);
    }
    active_ = ok;
    if (!ok) {
      reason_ = why.empty() ? "validation failed on some rank" : why;
      Teardown();
    }
  }
  ~P2pComm() override { Teardown(); }

  int rank() const override { return rank_; }
  int world() const override { return world_; }
  bool is_device() const override { return base_->is_device(); }
  bool active() const { return active_; }
  const std::string& reason() const { return reason_; }

  void AllReduceHost(double* buf, int64_t n) override { base_->AllReduceHost(buf, n); }
  void AllReduceHostI64(int64_t* buf, int64_t n) override { base_->AllReduceHostI64(buf, n); }
  void AllReduceDeviceI64(int64_t* buf, int64_t n, void* stream) override {
    if (!Use(n * 8)) return base_->AllReduceDeviceI64(buf, n, stream);
    Launch(reinterpret_cast<long long*>(buf), n, static_cast<hipStream_t>(stream));
  }
  bool AllReduceDeviceI64Active(int64_t* buf, int64_t n_max, const int32_t* units, int64_t per_unit,
                                void* stream) override {
    if (!Use(n_max * 8)) return base_->AllReduceDeviceI64Active(buf, n_max, units, per_unit, stream);
    Launch(reinterpret_cast<long long*>(buf), n_max, static_cast<hipStream_t>(stream), units, per_unit);
    return true;
  }
  // (a blocking read of the device counter: stats time only)
  int64_t DeviceBytes() const override {
    unsigned long long v = 0;
    if (bytes_) SML_HIP_CHECK(hipMemcpy(&v, bytes_, sizeof(v), hipMemcpyDeviceToHost));
    return static_cast<int64_t>(v);
  }
  void AllReduceDeviceF32(float* buf, int64_t n, void* stream) override {
    if (!Use(n * 4)) return base_->AllReduceDeviceF32(buf, n, stream);
    Launch(buf, n, static_cast<hipStream_t>(stream));
  }
  void AllReduceDeviceF64(double* buf, int64_t n, void* stream) override {
    if (!Use(n * 8)) return base_->AllReduceDeviceF64(buf, n, stream);
    Launch(buf, n, static_cast<hipStream_t>(stream));
  }
  void Check() override {
    if (err_ && __atomic_load_n(err_, __ATOMIC_ACQUIRE))
      throw CommError("p2p allreduce timed out waiting for a peer (a rank died or diverged)");
    base_->Check();
  }
  void Abort() override { base_->Abort(); }
  bool aborted() const override { return base_->aborted(); }

 private:
  bool Use(int64_t bytes) const { return active_ && world_ > 1 && bytes <= cap_; }

  template <class T>
  void Launch(T* buf, int64_t n, hipStream_t s, const int32_t* units = nullptr, int64_t per_unit = 0) {
    if (n <= 0) return;
    constexpr int VW = 16 / sizeof(T);
    const bool vec = reinterpret_cast<uintptr_t>(buf) % 16 == 0;
    // ~one 16-byte vector per thread per block; chunks stay multiples of VW
    const int64_t per_block = static_cast<int64_t>(kP2pThreads) * VW;
    const int blocks = static_cast<int>(std::min<int64_t>(kMaxBlocks, (n + per_block - 1) / per_block));
    const int64_t chunk = ((n + blocks - 1) / blocks + VW - 1) / VW * VW;
    ++epoch_;
    if (vec)
      hipLaunchKernelGGL((p2p_allreduce_kernel<T, VW>), dim3(blocks), dim3(kP2pThreads), 0, s, peers_, buf, buf, n,
                         chunk, cap_, rank_, world_, epoch_, timeout_ticks_, err_, units, per_unit, bytes_);
    else
      hipLaunchKernelGGL((p2p_allreduce_kernel<T, 1>), dim3(blocks), dim3(kP2pThreads), 0, s, peers_, buf, buf, n,
                         chunk, cap_, rank_, world_, epoch_, timeout_ticks_, err_, units, per_unit, bytes_);
    SML_HIP_CHECK(hipGetLastError());
  }

  // all-gather of fixed-size byte records through the base host allreduce
  std::vector<uint8_t> AllGatherBytes(const void* mine, size_t bytes) {
    std::vector<double> buf(bytes * world_, 0.0);
    const uint8_t* m = static_cast<const uint8_t*>(mine);
    for (size_t i = 0; i < bytes; ++i) buf[rank_ * bytes + i] = m[i];
    base_->AllReduceHost(buf.data(), static_cast<int64_t>(buf.size()));
    std::vector<uint8_t> out(buf.size());
    for (size_t i = 0; i < buf.size(); ++i) out[i] = static_cast<uint8_t>(buf[i]);
    return out;
  }

  bool Agree(bool ok) {
    double v = ok ? 0.0 : 1.0;
    base_->AllReduceHost(&v, 1);
    return v == 0.0;
  }

  void Setup() {
    const size_t recv_bytes = 2 * static_cast<size_t>(cap_) * kMaxRanks;
    const size_t sig_bytes = sizeof(uint32_t) * kMaxRanks * kMaxBlocks;
    SML_HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&recv_), recv_bytes, hipDeviceMallocUncached));
    SML_HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&sig_), sig_bytes, hipDeviceMallocUncached));
    SML_HIP_CHECK(hipMemset(sig_, 0, sig_bytes));
    SML_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&err_), sizeof(int), hipHostMallocCoherent));
    *err_ = 0;
    SML_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&bytes_), sizeof(unsigned long long)));
    SML_HIP_CHECK(hipMemset(bytes_, 0, sizeof(unsigned long long)));
    SML_HIP_CHECK(hipDeviceSynchronize());
    hipIpcMemHandle_t h[2];
    SML_HIP_CHECK(hipIpcGetMemHandle(&h[0], recv_));
    SML_HIP_CHECK(hipIpcGetMemHandle(&h[1], sig_));
    std::vector<uint8_t> all = AllGatherBytes(h, sizeof(h));
    std::memset(&peers_, 0, sizeof(peers_));
    for (int q = 0; q < world_; ++q) {
      if (q == rank_) {
        peers_.recv[q] = recv_;
        peers_.sig[q] = sig_;
        continue;
      }
      hipIpcMemHandle_t ph[2];
      std::memcpy(ph, all.data() + q * sizeof(h), sizeof(h));
      void* pr = nullptr;
      void* ps = nullptr;
      SML_HIP_CHECK(hipIpcOpenMemHandle(&pr, ph[0], hipIpcMemLazyEnablePeerAccess));
      opened_.push_back(pr);
      SML_HIP_CHECK(hipIpcOpenMemHandle(&ps, ph[1], hipIpcMemLazyEnablePeerAccess));
      opened_.push_back(ps);
      peers_.recv[q] = static_cast<char*>(pr);
      peers_.sig[q] = static_cast<uint32_t*>(ps);
    }
  }

  // exact small-integer sums on both message paths: every rank must agree
  bool SelfTest() {
    struct Restore {  // a broken path must fail fast here, not after the run-time timeout
      long long& t;
      long long v;
      ~Restore() { t = v; }
    } restore{timeout_ticks_, timeout_ticks_};
    timeout_ticks_ = std::min<long long>(timeout_ticks_, 500000000LL);  // 5 s
    const int64_t n = 3001;  // odd, several blocks
    std::vector<double> h(n);
    for (int64_t i = 0; i < n; ++i) h[i] = static_cast<double>((rank_ + 1) * 1000 + i % 977);
    double* d = nullptr;
    hipStream_t s = nullptr;
    SML_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    SML_HIP_CHECK(hipMalloc(&d, sizeof(double) * n));
    bool ok = true;
    for (int rep = 0; rep < 3; ++rep) {  // both parities, back to back (no early exit: epochs stay in step)
      SML_HIP_CHECK(hipMemcpyAsync(d, h.data(), sizeof(double) * n, hipMemcpyHostToDevice, s));
      active_ = true;
      Launch(d, n, s);
      std::vector<double> r(n);
      SML_HIP_CHECK(hipMemcpyAsync(r.data(), d, sizeof(double) * n, hipMemcpyDeviceToHost, s));
      SML_HIP_CHECK(hipStreamSynchronize(s));
      const double ranks = world_ * (world_ + 1) / 2.0;
      for (int64_t i = 0; i < n; ++i)
        ok = ok && r[i] == ranks * 1000 + world_ * static_cast<double>(i % 977);
      ok = ok && !*err_;
    }
    active_ = false;
    (void)hipFree(d);
    (void)hipStreamDestroy(s);
    return ok;
  }

  void Teardown() {
    if (!opened_.empty() || recv_) (void)hipDeviceSynchronize();
    for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
    opened_.clear();
    if (recv_) (void)hipFree(recv_);
    if (sig_) (void)hipFree(sig_);
    if (err_) (void)hipHostFree(err_);
    if (bytes_) (void)hipFree(bytes_);
    bytes_ = nullptr;
    recv_ = nullptr;
    sig_ = nullptr;
    err_ = nullptr;
  }

  std::shared_ptr<Comm> base_;
  int rank_, world_;
  int64_t cap_;
  long long timeout_ticks_ = 0;
  bool active_ = false;
  std::string reason_;
  char* recv_ = nullptr;
  uint32_t* sig_ = nullptr;
  int* err_ = nullptr;
  unsigned long long* bytes_ = nullptr;  // pushed bytes (device memory, bumped by the kernels' block 0)
  uint32_t epoch_ = 0;
  PeerPtrs peers_{};
  std::vector<void*> opened_;
};

}  // namespace

std::shared_ptr<Comm> NewP2pComm(std::shared_ptr<Comm> base, int device, int64_t cap_bytes, double timeout_ms,
                                 std::string* reason) {
  auto c = std::make_shared<P2pComm>(std::move(base), device, cap_bytes, timeout_ms);
  if (reason) *reason = c->active() ? std::string() : c->reason();
  return c;
}

std::vector<double> CommDeviceAllReduce(Comm* c, const std::vector<double>& x, int reps) {
  double* d = nullptr;
  hipStream_t s = nullptr;
  SML_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  SML_HIP_CHECK(hipMalloc(&d, sizeof(double) * std::max<size_t>(1, x.size())));
  std::vector<double> r(x.size());
  for (int i = 0; i < reps; ++i) {
    SML_HIP_CHECK(hipMemcpyAsync(d, x.data(), sizeof(double) * x.size(), hipMemcpyHostToDevice, s));
    c->AllReduceDeviceF64(d, static_cast<int64_t>(x.size()), s);
  }
  SML_HIP_CHECK(hipMemcpyAsync(r.data(), d, sizeof(double) * x.size(), hipMemcpyDeviceToHost, s));
  SML_HIP_CHECK(hipStreamSynchronize(s));
  (void)hipFree(d);
  (void)hipStreamDestroy(s);
  c->Check();
  return r;
}

double CommDeviceAllReduceUs(Comm* c, int64_t n, int iters) {
  double* d = nullptr;
  hipStream_t s = nullptr;
  hipEvent_t e0, e1;
  SML_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  SML_HIP_CHECK(hipMalloc(&d, sizeof(double) * n));
  SML_HIP_CHECK(hipMemsetAsync(d, 0, sizeof(double) * n, s));
  SML_HIP_CHECK(hipEventCreate(&e0));
  SML_HIP_CHECK(hipEventCreate(&e1));
  for (int i = 0; i < 5; ++i) c->AllReduceDeviceF64(d, n, s);
  SML_HIP_CHECK(hipEventRecord(e0, s));
  for (int i = 0; i < iters; ++i) c->AllReduceDeviceF64(d, n, s);
  SML_HIP_CHECK(hipEventRecord(e1, s));
  SML_HIP_CHECK(hipStreamSynchronize(s));
  float ms = 0.f;
  SML_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(d);
  (void)hipStreamDestroy(s);
  c->Check();
  return 1000.0 * ms / iters;
}

}  // namespace sml
