// Output-label fetch into mapped pinned host memory (kernels_label.hip k_fetch_res, used by runtime.hip)
#pragma once
#include <cstdint>
#include <hip/hip_runtime.h>

#include "launch.h"

namespace dash::dev {
// device bytes of every residue -> mapped pinned host memory in one launch
struct FetchRes {
    const void* in[kMaxRes];
    void* out[kMaxRes];  // device pointers of mapped pinned host buffers
    int64_t bytes[kMaxRes];
    int k;
};
void launch_fetch_res(const FetchRes& a, hipStream_t st);
}  // namespace dash::dev
