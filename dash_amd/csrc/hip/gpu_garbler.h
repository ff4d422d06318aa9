// GPU garbler for the sign-gadget layers (see garble_gpu.hip). Plain C++
// interface so the host garbler (garbler.cpp) can dispatch to it.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "../gadgets.h"

namespace dash {

class GpuGarbler {
   public:
    GpuGarbler(const std::vector<int>& crt, const std::vector<int>& mrs, const std::string& seed16, const LabelBank& R,
               const LabelBank& Z, int device);
    ~GpuGarbler();
    // ReLU (relu_crt/prefix/mmg/mme set) or Sign layer: tables + next base labels
    void sign_layer(uint64_t layer, const SignPlan& sp, const CrtLabels& cur, Array& ap, Array& c1, Array& c2,
                    Array& sg, CrtLabels& out, const std::vector<int>* relu_crt, const std::vector<i64>* prefix,
                    Array* mmg, Array* mme);
    // one DASH legacy rescale iteration (sign base extension); cur updated in place
    void rescale_legacy_iter(uint64_t layer, int it, const RescalePlan& P, CrtLabels& cur,
                             const std::vector<std::vector<comp_t>>& up, const std::vector<std::vector<comp_t>>& down,
                             Array& tr, Array& ap, Array& c1, Array& c2, Array& sg);

   private:
    struct Impl;
    std::unique_ptr<Impl> impl_;
};

}  // namespace dash
