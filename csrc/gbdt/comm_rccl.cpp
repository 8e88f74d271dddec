// RCCL communicator for data-parallel GBDT (histogram allreduce over xGMI).
// Replaces the reference's LGBM_NetworkInit socket linkers
// (lightgbm/.../NetworkManager.scala:195-218) with one RCCL communicator per
// process/GPU bootstrapped from an ncclUniqueId distributed by the rendezvous.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>
#include <string>
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

class RcclComm : public Comm {
 public:
  RcclComm(const std::string& uid, int rank, int world, int device) : rank_(rank), world_(world) {
    if (uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("bad ncclUniqueId size");
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    if (device >= 0) SML_HIP_CHECK(hipSetDevice(device));
    SML_NCCL_CHECK(ncclCommInitRank(&comm_, world, id, rank));
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
    SML_NCCL_CHECK(ncclAllReduce(d, d, n, ncclDouble, ncclSum, comm_, nullptr));
    SML_HIP_CHECK(hipStreamSynchronize(nullptr));
    SML_HIP_CHECK(hipMemcpy(buf, d, sizeof(double) * n, hipMemcpyDeviceToHost));
    SML_HIP_CHECK(hipFree(d));
  }
  void AllReduceDeviceF32(float* buf, int64_t n, void* stream) override {
    if (!comm_) throw CommError("RCCL communicator was aborted");
    SML_NCCL_CHECK(ncclAllReduce(buf, buf, n, ncclFloat, ncclSum, comm_, static_cast<hipStream_t>(stream)));
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
  void AllReduceDeviceF64(double* buf, int64_t n, void* stream) override {
    if (!comm_) throw CommError("RCCL communicator was aborted");
    SML_NCCL_CHECK(ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, comm_, static_cast<hipStream_t>(stream)));
  }

 private:
  int rank_, world_;
  ncclComm_t comm_ = nullptr;
  void* scratch_ = nullptr;
};

}  // namespace

std::string RcclGetUniqueId() {
  ncclUniqueId id;
  SML_NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

Comm* NewRcclComm(const std::string& uid, int rank, int world, int device) {
  return new RcclComm(uid, rank, world, device);
}

}  // namespace sml
