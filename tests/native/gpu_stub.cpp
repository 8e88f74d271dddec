// Host-only build of the GBDT engine (sanitizer targets): no HIP device backend.
#include <stdexcept>

#include "backend.h"
#include "dataset.h"

namespace sml {
bool GpuAvailable() { return false; }
std::unique_ptr<TrainBackend> MakeGpuBackend(int) { return nullptr; }
// datasets of a host-only build never hold device bins
void DatasetDownloadBins(const Dataset&, uint8_t*) { throw std::logic_error("no device bins in a host-only build"); }
}  // namespace sml
