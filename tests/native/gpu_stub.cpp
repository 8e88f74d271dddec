// Host-only build of the GBDT engine (sanitizer targets): no HIP device backend.
#include "backend.h"

namespace sml {
bool GpuAvailable() { return false; }
std::unique_ptr<TrainBackend> MakeGpuBackend(int) { return nullptr; }
}  // namespace sml
