// Host-only link stub for the sanitizer builds: the sanitizer harness never
// garbles on a device (GarbleOptions.device = -1), so these must not run.
#include <stdexcept>

#include "hip/gpu_garbler.h"

namespace dash {

struct GpuGarbler::Impl {};

[[noreturn]] static void no_gpu() { throw std::runtime_error("GPU garbler not linked into the host-only build"); }

GpuGarbler::GpuGarbler(const std::vector<int>&, const std::vector<int>&, const std::string&, const LabelBank&,
                       const LabelBank&, int, bool) {
    no_gpu();
}
GpuGarbler::~GpuGarbler() = default;
void GpuGarbler::to_device(const CrtLabels&) { no_gpu(); }
void GpuGarbler::to_host(CrtLabels&) { no_gpu(); }
void GpuGarbler::conv(const ConvGeom&, const i64*, size_t, uint64_t, CrtLabels&) { no_gpu(); }
void GpuGarbler::sign_layer(uint64_t, const SignPlan&, CrtLabels&, Array&, Array&, Array&, Array&,
                            const std::vector<int>*, const std::vector<i64>*, Array*, Array*) {
    no_gpu();
}
void GpuGarbler::rescale_legacy_iter(uint64_t, int, const RescalePlan&, CrtLabels&,
                                     const std::vector<std::vector<comp_t>>&,
                                     const std::vector<std::vector<comp_t>>&, Array&, Array&, Array&, Array&,
                                     Array&) {
    no_gpu();
}
void GpuGarbler::rescale_mrs(uint64_t, const RescaleMrsPlan&, CrtLabels&, Array&) { no_gpu(); }
void GpuGarbler::relu_mrs(uint64_t, const SignMrsPlan&, CrtLabels&, Array&, const std::vector<int>*,
                          const std::vector<i64>*, Array&, Array&) {
    no_gpu();
}
void GpuGarbler::relu_mult(uint64_t, CrtLabels&, const std::vector<i64>*, Array&, Array&) { no_gpu(); }
void GpuGarbler::dense(i64, i64, i64, const i64*, size_t, uint64_t, CrtLabels&) { no_gpu(); }
void GpuGarbler::sumpool(const PoolGeom&, CrtLabels&) { no_gpu(); }
void GpuGarbler::fold_constants(const std::vector<i64>&, i64, CrtLabels&) { no_gpu(); }
void GpuGarbler::save(size_t) { no_gpu(); }
bool GpuGarbler::has_saved(size_t) const { return false; }
void GpuGarbler::restore(size_t, CrtLabels&) { no_gpu(); }
void GpuGarbler::add_saved(size_t, CrtLabels&) { no_gpu(); }
void GpuGarbler::maxpool_begin(const std::vector<std::vector<i64>>&, CrtLabels&) { no_gpu(); }
void GpuGarbler::maxpool_level(uint64_t, int, i64, const SignPlan&, const std::vector<i64>&, Array&, Array&, Array&,
                               Array&, Array&, Array&) {
    no_gpu();
}
void GpuGarbler::maxpool_end(CrtLabels&) { no_gpu(); }
void GpuGarbler::rescale_redash(uint64_t, int, const RescalePlan&, CrtLabels&, const std::vector<std::vector<comp_t>>&,
                                const std::vector<std::vector<comp_t>>&, Array&, Array&) {
    no_gpu();
}
void GpuGarbler::base_ext(uint64_t, const BEPlan&, CrtLabels&, Array&) { no_gpu(); }
void gpu_table_cache_trim() {}
size_t gpu_table_cache_bytes() { return 0; }

}  // namespace dash
