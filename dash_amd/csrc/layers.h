// Layer geometry shared by garbler, host evaluator and HIP runtime.
#pragma once

#include "model.h"

namespace dash {

struct ConvGeom {
    i64 C, H, W, F, kh, kw, sh, sw, ph, pw, OH, OW;
    explicit ConvGeom(const Params& p);
    explicit ConvGeom(const GLayer& g) : ConvGeom(g.p) {}
    i64 K() const { return C * kh * kw; }
    i64 out_size() const { return F * OH * OW; }
};

struct PoolGeom {
    i64 C, H, W, kh, kw, sh, sw, OH, OW;
    explicit PoolGeom(const Params& p);
    i64 out_size() const { return C * OH * OW; }
    // flattened input indices of output element o's window (row-major)
    void window(i64 o, std::vector<i64>& idx) const;
};

// Pairwise max-reduction schedule over a window of K values: level l has
// ops[l] pair-max operations; value slots after level l: cnt[l+1].
struct MaxTree {
    std::vector<int> ops, cnt;
    explicit MaxTree(i64 K);
};

inline i64 param1(const Params& p, const char* k, i64 dflt = -1) {
    auto it = p.find(k);
    return (it == p.end() || it->second.empty()) ? dflt : it->second[0];
}
inline const std::vector<i64>& paramv(const Params& p, const char* k) {
    auto it = p.find(k);
    DASH_CHECK(it != p.end(), std::string("missing param ") + k);
    return it->second;
}

// dense input remap for TF (NHWC) flattening: reference cuda_util.h:130
inline i64 dense_src(i64 i, i64 K, i64 ch) { return ch > 0 ? i / ch + (i % ch) * (K / ch) : i; }

std::string arr_name(const char* prefix, int idx, const char* suffix);

}  // namespace dash
