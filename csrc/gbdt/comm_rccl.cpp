// RCCL communicator for data-parallel GBDT (histogram allreduce over xGMI).
// Replaces the reference's LGBM_NetworkInit socket linkers
// (lightgbm/.../NetworkManager.scala:195-218) with one RCCL communicator per
// process/GPU bootstrapped from an ncclUniqueId distributed by the rendezvous.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "comm.h"
#include "hip_common.h"
#include "trace.h"

namespace sml {

#define SML_NCCL_CHECK(expr)                                                              \
  do {                                                                                    \
    ncclResult_t _r = (expr);                                                             \
    if (_r != ncclSuccess)                                                                \
      throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(_r) + " (" #expr ")"); \
  } while (0)

void HostComm::AllReduceDeviceF32(float* buf, int64_t n, void* stream) {
  if (world_ <= 1) return;
  hipStream_t s = static_cast<hipStream_t>(stream);
  std::vector<float> h(n);
  SML_HIP_CHECK(hipMemcpyAsync(h.data(), buf, sizeof(float) * n, hipMemcpyDeviceToHost, s));
  SML_HIP_CHECK(hipStreamSynchronize(s));
  std::vector<double> d(h.begin(), h.end());
  fn_(d.data(), n);
  for (int64_t i = 0; i < n; ++i) h[i] = static_cast<float>(d[i]);
  SML_HIP_CHECK(hipMemcpyAsync(buf, h.data(), sizeof(float) * n, hipMemcpyHostToDevice, s));
  SML_HIP_CHECK(hipStreamSynchronize(s));
}

void HostComm::AllReduceHostI64(int64_t* buf, int64_t n) {
  if (world_ <= 1) return;
  if (fn_i64_) {
    fn_i64_(buf, n);
    return;
  }
  // no integer collective was supplied: exact through the double one in 26-bit limbs (every partial sum of
  // a limb stays far below 2^53 for any realistic world size)
  constexpr int kLimbs = 3;
  std::vector<double> d(static_cast<size_t>(n) * kLimbs);
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t u = static_cast<uint64_t>(buf[i]);
    d[i * kLimbs] = static_cast<double>(u & ((1ull << 26) - 1));
    d[i * kLimbs + 1] = static_cast<double>((u >> 26) & ((1ull << 26) - 1));
    d[i * kLimbs + 2] = static_cast<double>(u >> 52);
  }
  fn_(d.data(), static_cast<int64_t>(d.size()));
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t a = static_cast<uint64_t>(d[i * kLimbs]), b = static_cast<uint64_t>(d[i * kLimbs + 1]),
                   c = static_cast<uint64_t>(d[i * kLimbs + 2]);
    buf[i] = static_cast<int64_t>(a + (b << 26) + (c << 52));  // modulo 2^64: two's complement sums wrap exactly
  }
}

void HostComm::AllReduceDeviceI64(int64_t* buf, int64_t n, void* stream) {
  if (world_ <= 1) return;
  hipStream_t s = static_cast<hipStream_t>(stream);
  std::vector<int64_t> h(n);
  SML_HIP_CHECK(hipMemcpyAsync(h.data(), buf, sizeof(int64_t) * n, hipMemcpyDeviceToHost, s));
  SML_HIP_CHECK(hipStreamSynchronize(s));
  AllReduceHostI64(h.data(), n);
  SML_HIP_CHECK(hipMemcpyAsync(buf, h.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, s));
  SML_HIP_CHECK(hipStreamSynchronize(s));
}

void HostComm::AllReduceDeviceF64(double* buf, int64_t n, void* stream) {
  if (world_ <= 1) return;
  hipStream_t s = static_cast<hipStream_t>(stream);
  std::vector<double> h(n);
  SML_HIP_CHECK(hipMemcpyAsync(h.data(), buf, sizeof(double) * n, hipMemcpyDeviceToHost, s));
  SML_HIP_CHECK(hipStreamSynchronize(s));
  fn_(h.data(), n);
  SML_HIP_CHECK(hipMemcpyAsync(buf, h.data(), sizeof(double) * n, hipMemcpyHostToDevice, s));
  SML_HIP_CHECK(hipStreamSynchronize(s));
}

namespace {

double NowMs() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// The communicator is created non-blocking so that a peer that never reaches (or dies inside) the collective
// init cannot hang the healthy ranks: init polls ncclCommGetAsyncError against a deadline and aborts the
// half-built communicator when it passes (the Python side then retries on every rank together).
class RcclComm : public Comm {
 public:
  RcclComm(const std::string& uid, int rank, int world, int device, double timeout_ms)
      : rank_(rank), world_(world), timeout_ms_(timeout_ms) {
    if (uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("bad ncclUniqueId size");
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    if (device >= 0) SML_HIP_CHECK(hipSetDevice(device));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r = ncclCommInitRankConfig(&comm_, world, id, rank, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) {
      if (comm_) (void)ncclCommAbort(comm_);
      comm_ = nullptr;
      throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(r) + " (ncclCommInitRankConfig)");
    }
    Settle(r, "ncclCommInitRankConfig");
    SML_HIP_CHECK(hipStreamCreateWithFlags(&host_stream_, hipStreamNonBlocking));
  }
  ~RcclComm() override {
    if (comm_) ncclCommDestroy(comm_);  // (null after an abort)
    if (host_stream_) (void)hipStreamSynchronize(host_stream_);
    if (scratch_) (void)hipFree(scratch_);
    if (pinned_) (void)hipHostFree(pinned_);
    if (host_stream_) (void)hipStreamDestroy(host_stream_);
  }
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  bool is_device() const override { return true; }
  // (a world-1 communicator still runs every collective: that is how the one-GPU tests execute this path)
  void AllReduceHost(double* buf, int64_t n) override {
    TraceRange tr("sml::AllReduceHost");
    // small host reductions (root sums, init scores): staged through a persistent device scratch and pinned
    // buffer on the communicator's own stream (no per-call allocation, no device-wide null-stream sync)
    HostReduce(buf, n, ncclDouble);
  }
  void AllReduceDeviceF32(float* buf, int64_t n, void* stream) override {
    if (!comm_) throw CommError("RCCL communicator was aborted");
    Settle(ncclAllReduce(buf, buf, n, ncclFloat, ncclSum, comm_, static_cast<hipStream_t>(stream)), "ncclAllReduce");
  }
  // Polled by the backend while it waits for a tree (RCCL async-error polling): a peer that
  // died or a broken link surfaces as a CommError on every rank instead of a collective that never returns.
  void Check() override {
    if (!comm_) throw CommError("RCCL communicator was aborted");
    ncclResult_t async = ncclSuccess;
    if (ncclCommGetAsyncError(comm_, &async) != ncclSuccess) return;
    if (async != ncclSuccess && async != ncclInProgress) {
      Abort();
      throw CommError(std::string("RCCL communicator failed: ") + ncclGetErrorString(async));
    }
  }
  void Abort() override {
    if (comm_) (void)ncclCommAbort(comm_);  // makes kernels of pending collectives return
    comm_ = nullptr;
  }
  bool aborted() const override { return comm_ == nullptr; }
  void AllReduceDeviceF64(double* buf, int64_t n, void* stream) override {
    if (!comm_) throw CommError("RCCL communicator was aborted");
    Settle(ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, comm_, static_cast<hipStream_t>(stream)), "ncclAllReduce");
  }
  void AllReduceDeviceI64(int64_t* buf, int64_t n, void* stream) override {
    if (!comm_) throw CommError("RCCL communicator was aborted");
    Settle(ncclAllReduce(buf, buf, n, ncclInt64, ncclSum, comm_, static_cast<hipStream_t>(stream)), "ncclAllReduce");
  }
  void AllReduceHostI64(int64_t* buf, int64_t n) override { HostReduce(buf, n, ncclInt64); }

 private:
  // host array -> pinned -> device scratch -> allreduce -> back, all on host_stream_ (8-byte elements)
  void HostReduce(void* buf, int64_t n, ncclDataType_t type) {
    if (!comm_) throw CommError("RCCL communicator was aborted");
    if (n <= 0) return;
    const size_t bytes = sizeof(double) * static_cast<size_t>(n);
    if (bytes > cap_) {
      size_t c = std::max<size_t>(4096, cap_);
      while (c < bytes) c *= 2;
      if (scratch_) SML_HIP_CHECK(hipFree(scratch_));
      if (pinned_) SML_HIP_CHECK(hipHostFree(pinned_));
      scratch_ = nullptr;
      pinned_ = nullptr;
      cap_ = 0;
      SML_HIP_CHECK(hipMalloc(&scratch_, c));
      SML_HIP_CHECK(hipHostMalloc(&pinned_, c, hipHostMallocDefault));
      cap_ = c;
    }
    std::memcpy(pinned_, buf, bytes);
    SML_HIP_CHECK(hipMemcpyAsync(scratch_, pinned_, bytes, hipMemcpyHostToDevice, host_stream_));
    Settle(ncclAllReduce(scratch_, scratch_, n, type, ncclSum, comm_, host_stream_), "ncclAllReduce");
    SML_HIP_CHECK(hipMemcpyAsync(pinned_, scratch_, bytes, hipMemcpyDeviceToHost, host_stream_));
    SML_HIP_CHECK(hipStreamSynchronize(host_stream_));
    std::memcpy(buf, pinned_, bytes);
  }

  // Non-blocking communicators may answer ncclInProgress (init, and the lazy peer connection of a first
  // collective); the next call on the communicator must wait until the state settles. Bounded by the
  // timeout: past it the communicator is aborted and the call fails with CommError.
  void Settle(ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return;
    if (r != ncclInProgress) throw CommError(std::string("RCCL error: ") + ncclGetErrorString(r) + " (" + what + ")");
    const double t0 = NowMs();
    ncclResult_t st = ncclInProgress;
    while (true) {
      if (ncclCommGetAsyncError(comm_, &st) != ncclSuccess) st = ncclInternalError;
      if (st != ncclInProgress) break;
      if (timeout_ms_ > 0 && NowMs() - t0 > timeout_ms_) {
        Abort();
        throw CommError(std::string(what) + " did not complete within " + std::to_string(timeout_ms_) +
                        " ms (a peer rank failed or never joined); communicator aborted");
      }
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    if (st != ncclSuccess) {
      Abort();
      throw CommError(std::string("RCCL error: ") + ncclGetErrorString(st) + " (" + what + ")");
    }
  }

  int rank_, world_;
  double timeout_ms_;
  ncclComm_t comm_ = nullptr;
  hipStream_t host_stream_ = nullptr;  // the host-array reductions' stream
  void* scratch_ = nullptr;            // their device scratch and pinned staging (cap_ bytes each, grow-only)
  void* pinned_ = nullptr;
  size_t cap_ = 0;
};

}  // namespace

std::string RcclGetUniqueId() {
  ncclUniqueId id;
  SML_NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

Comm* NewRcclComm(const std::string& uid, int rank, int world, int device, double timeout_ms) {
  return new RcclComm(uid, rank, world, device, timeout_ms);
}

}  // namespace sml
