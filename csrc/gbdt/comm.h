// Collective communication used by data-parallel training (N3/C2 of SURVEY
// §2.3/2.5). The reference runs LightGBM's own socket linkers after a driver
// rendezvous (lightgbm/.../NetworkManager.scala:195-218). Here:
//   * RcclComm: RCCL communicator (one per process/GPU, xGMI intra-node),
//     bootstrapped from an ncclUniqueId handed out by the rendezvous;
//   * HostComm: a host-buffer allreduce supplied by the Python runtime (gloo /
//     TCP) for the CPU backend and for tests without GPUs.
#pragma once
#include <cstdint>
#include <functional>
#include <string>

namespace sml {

class Comm {
 public:
  virtual ~Comm() = default;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  // in-place sum over ranks of a HOST buffer
  virtual void AllReduceHost(double* buf, int64_t n) = 0;
  // in-place sum over ranks of a DEVICE buffer on `stream` (hipStream_t)
  virtual void AllReduceDeviceF32(float* buf, int64_t n, void* stream) = 0;
  virtual void AllReduceDeviceF64(double* buf, int64_t n, void* stream) = 0;
  virtual bool is_device() const { return false; }
};

class HostComm : public Comm {
 public:
  using Fn = std::function<void(double*, int64_t)>;
  HostComm(int rank, int world, Fn fn) : rank_(rank), world_(world), fn_(std::move(fn)) {}
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  void AllReduceHost(double* buf, int64_t n) override { if (world_ > 1) fn_(buf, n); }
  void AllReduceDeviceF32(float*, int64_t, void*) override;
  void AllReduceDeviceF64(double*, int64_t, void*) override;

 private:
  int rank_, world_;
  Fn fn_;
};

// RCCL communicator (defined in comm_rccl.cpp)
std::string RcclGetUniqueId();
Comm* NewRcclComm(const std::string& unique_id, int rank, int world, int device);

}  // namespace sml
