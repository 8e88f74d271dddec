// Device-resident hashed linear learner (K12/K13 of SURVEY §2.4): the weight
// table (2^b x {w, G}) lives in HBM, mini-batches of CSR examples are learned
// by one wave per example with AdaGrad-style hogwild updates (atomics on the
// touched weights), and the table is averaged across GPUs with RCCL at pass
// boundaries (C4: the reference's spanning-tree AllReduce at endPass).
#pragma once
#include <cstdint>
#include <memory>
#include <string>

namespace smlvw {

struct GpuSgdConfig {
  int bits = 18;
  float lr = 0.5f;
  float power_t = 0.5f;
  float l2 = 0.f;
  int loss = 0;        // 0 squared, 1 logistic
  bool adaptive = true;
};

class GpuSgd {
 public:
  GpuSgd(const GpuSgdConfig& cfg, int device);
  ~GpuSgd();
  // indices are pre-hashed feature ids (masked on device); labels in the
  // loss's convention (logistic: -1/+1). Returns the progressive predictions.
  void Learn(const int64_t* indptr, const uint32_t* indices, const float* values, const float* labels,
             const float* weights, int64_t n, int batch, float* preds_out);
  void Predict(const int64_t* indptr, const uint32_t* indices, const float* values, int64_t n, float* out);
  // in-place sum over ranks of the weight table via the supplied device allreduce, then / world
  void AllReduceAverage(void* nccl_comm_handle, int world);
  uint64_t NumWeights() const;
  void CopyWeights(float* host_out) const;
  void SetWeights(const float* host_in);
  double examples() const { return examples_; }
  double sum_loss() const { return sum_loss_; }
  void* weights_device();
  void* stream();

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
  GpuSgdConfig cfg_;
  double examples_ = 0, sum_loss_ = 0;
};

bool VwGpuAvailable();
// K13: murmur3_32(bytes[offsets[i]:offsets[i+1]], seed) & mask for every i, on the device
void MurmurBatchGpu(const uint8_t* bytes, int64_t nbytes, const int64_t* offsets, int64_t n, uint32_t seed,
                    uint32_t mask, uint32_t* out);

}  // namespace smlvw
