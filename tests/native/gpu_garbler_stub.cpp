// Host-only link stub for the sanitizer builds: the sanitizer harness never
// garbles on a device (GarbleOptions.device = -1), so these must not run.
#include <stdexcept>

#include "hip/gpu_garbler.h"

namespace dash {

struct GpuGarbler::Impl {};

GpuGarbler::GpuGarbler(const std::vector<int>&, const std::vector<int>&, const std::string&, const LabelBank&,
                       const LabelBank&, int) {
    throw std::runtime_error("GPU garbler not linked into the host-only build");
}
GpuGarbler::~GpuGarbler() = default;
void GpuGarbler::sign_layer(uint64_t, const SignPlan&, const CrtLabels&, Array&, Array&, Array&, Array&, CrtLabels&,
                            const std::vector<int>*, const std::vector<i64>*, Array*, Array*) {}
void GpuGarbler::rescale_legacy_iter(uint64_t, int, const RescalePlan&, CrtLabels&,
                                     const std::vector<std::vector<comp_t>>&,
                                     const std::vector<std::vector<comp_t>>&, Array&, Array&, Array&, Array&,
                                     Array&) {}

}  // namespace dash
