// Collective communication used by data-parallel training (N3/C2 of SURVEY
// §2.3/2.5). The reference runs LightGBM's own socket linkers after a driver
// rendezvous (lightgbm/.../NetworkManager.scala:195-218). Here:
//   * RcclComm: RCCL communicator (one per process/GPU, xGMI intra-node),
//     bootstrapped from an ncclUniqueId handed out by the rendezvous;
//   * HostComm: a host-buffer allreduce supplied by the Python runtime (gloo /
//     TCP) for the CPU backend and for tests without GPUs.
#pragma once
#include <algorithm>
#include <cstdint>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace sml {

// A collective failed or timed out (a peer died, a link broke, ranks diverged). Training must fail on
// every rank instead of ending early with a truncated model (Python: synapseml_amd._gbdt.CommError).
struct CommError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

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
  // exact (associative) sums: the fixed-point histograms of data-parallel training travel as int64, so an
  // N-rank histogram is bitwise the 1-rank histogram of the union of the partitions
  virtual void AllReduceHostI64(int64_t* buf, int64_t n) = 0;
  virtual void AllReduceDeviceI64(int64_t* buf, int64_t n, void* stream) = 0;
  // the same over the first min(n_max, *units * per_unit) elements, `units` a device int the preceding kernels
  // wrote (the batched growth's expansion count): a device-driven transport moves only those; the default
  // (host-sized collectives) reduces all n_max. Returns true if the size was applied on the device.
  virtual bool AllReduceDeviceI64Active(int64_t* buf, int64_t n_max, const int32_t* units, int64_t per_unit,
                                        void* stream) {
    (void)units;
    (void)per_unit;
    AllReduceDeviceI64(buf, n_max, stream);
    return false;
  }
  // bytes this rank moved through a device-driven transport so far (0 if it does not count)
  virtual int64_t DeviceBytes() const { return 0; }
  // element-wise max over ranks of a small HOST buffer, built on the sum: every rank contributes its values in
  // its own slot of a world-sized buffer (exact - the other slots are zeros) and takes the max locally
  void AllReduceHostMax(double* buf, int64_t n) {
    if (world() <= 1) return;
    std::vector<double> all(static_cast<size_t>(n) * world(), 0.0);
    for (int64_t i = 0; i < n; ++i) all[static_cast<size_t>(rank()) * n + i] = buf[i];
    AllReduceHost(all.data(), static_cast<int64_t>(all.size()));
    for (int64_t i = 0; i < n; ++i) {
      double m = all[i];
      for (int q = 1; q < world(); ++q) m = std::max(m, all[static_cast<size_t>(q) * n + i]);
      buf[i] = m;
    }
  }
  virtual bool is_device() const { return false; }
  // raise CommError if an asynchronous collective failed; polled while the backend waits on the device
  virtual void Check() {}
  // unblock collectives stuck on a dead peer (RCCL: ncclCommAbort); the communicator is unusable after
  virtual void Abort() {}
  // true once Abort() ran (a cached communicator in this state must be rebuilt, not reused)
  virtual bool aborted() const { return false; }
};

class HostComm : public Comm {
 public:
  using Fn = std::function<void(double*, int64_t)>;
  using FnI64 = std::function<void(int64_t*, int64_t)>;
  HostComm(int rank, int world, Fn fn, FnI64 fn_i64 = nullptr)
      : rank_(rank), world_(world), fn_(std::move(fn)), fn_i64_(std::move(fn_i64)) {}
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  void AllReduceHost(double* buf, int64_t n) override { if (world_ > 1) fn_(buf, n); }
  void AllReduceHostI64(int64_t* buf, int64_t n) override;
  void AllReduceDeviceF32(float*, int64_t, void*) override;
  void AllReduceDeviceF64(double*, int64_t, void*) override;
  void AllReduceDeviceI64(int64_t*, int64_t, void*) override;

 private:
  int rank_, world_;
  Fn fn_;
  FnI64 fn_i64_;
};

// RCCL communicator (defined in comm_rccl.cpp)
std::string RcclGetUniqueId();
// Non-blocking init bounded by timeout_ms (<= 0: wait forever); a failed or timed-out init aborts the
// half-built communicator and throws CommError.
Comm* NewRcclComm(const std::string& unique_id, int rank, int world, int device, double timeout_ms);

// One-shot P2P (IPC) allreduce for device messages up to cap_bytes, layered on
// `base` (used for the handle exchange, validation, host reductions and large
// messages). Falls back to `base` on every rank if set-up or the start-up
// self-test fails anywhere; *reason then says why. (comm_p2p.hip)
std::shared_ptr<Comm> NewP2pComm(std::shared_ptr<Comm> base, int device, int64_t cap_bytes, double timeout_ms,
                                 std::string* reason);
// test / benchmark helpers: allreduce a host vector through the device path;
// average microseconds per device allreduce of n doubles
std::vector<double> CommDeviceAllReduce(Comm* c, const std::vector<double>& x, int reps);
double CommDeviceAllReduceUs(Comm* c, int64_t n, int iters);

}  // namespace sml
