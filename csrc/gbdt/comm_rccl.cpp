// RCCL communicator for data-parallel GBDT (histogram allreduce over xGMI).
// Replaces the reference's LGBM_NetworkInit socket linkers
// (lightgbm/.../NetworkManager.scala:195-218) with one RCCL communicator per
// process/GPU bootstrapped from an ncclUniqueId distributed by the rendezvous.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

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
    SML_HIP_CHECK(hipMalloc(&scratch_, 64));
  }
  ~RcclComm() override {
    if (comm_) ncclCommDestroy(comm_);  // (null after an abort)
    if (scratch_) (void)hipFree(scratch_);
  }
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  bool is_device() const override { return true; }
  // (a world-1 communicator still runs every collective: that is how the one-GPU tests execute this path)
  void AllReduceHost(double* buf, int64_t n) override {
    TraceRange tr("sml::AllReduceHost");
    // small host reductions (root sums, init scores): stage through the device
    if (!comm_) throw CommError("RCCL communicator was aborted");
    double* d = nullptr;
    SML_HIP_CHECK(hipMalloc(&d, sizeof(double) * n));
    SML_HIP_CHECK(hipMemcpy(d, buf, sizeof(double) * n, hipMemcpyHostToDevice));
    Settle(ncclAllReduce(d, d, n, ncclDouble, ncclSum, comm_, nullptr), "ncclAllReduce");
    SML_HIP_CHECK(hipStreamSynchronize(nullptr));
    SML_HIP_CHECK(hipMemcpy(buf, d, sizeof(double) * n, hipMemcpyDeviceToHost));
    SML_HIP_CHECK(hipFree(d));
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
  void AllReduceHostI64(int64_t* buf, int64_t n) override {
    if (!comm_) throw CommError("RCCL communicator was aborted");
    int64_t* d = nullptr;
    SML_HIP_CHECK(hipMalloc(&d, sizeof(int64_t) * n));
    SML_HIP_CHECK(hipMemcpy(d, buf, sizeof(int64_t) * n, hipMemcpyHostToDevice));
    Settle(ncclAllReduce(d, d, n, ncclInt64, ncclSum, comm_, nullptr), "ncclAllReduce");
    SML_HIP_CHECK(hipStreamSynchronize(nullptr));
    SML_HIP_CHECK(hipMemcpy(buf, d, sizeof(int64_t) * n, hipMemcpyDeviceToHost));
    SML_HIP_CHECK(hipFree(d));
  }

 private:
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
  void* scratch_ = nullptr;
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
