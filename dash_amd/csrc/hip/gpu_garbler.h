// GPU garbler (see garble_gpu.hip). Plain C++ interface so the host garbler
// (garbler.cpp) can dispatch to it.
//
// The garbler's current base labels live on the device between GPU layers
// ("device cur"): the host garbler calls to_device() before a GPU layer when
// its host copy is newer and to_host() before a host layer when the device
// copy is newer, so a run of GPU layers (conv -> rescale -> ReLU -> conv ...)
// never moves labels over PCIe. GPU layers leave the host `cur` stale: they
// only set its shape (p, n, N) and clear its storage.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "../gadgets.h"
#include "../layers.h"

namespace dash {

class GpuGarbler {
   public:
    // hardened: the tables use the hardened encoding's tweaked pads (core.h hard_block) instead of H(K)
    GpuGarbler(const std::vector<int>& crt, const std::vector<int>& mrs, const std::string& seed16, const LabelBank& R,
               const LabelBank& Z, int device, bool hardened = false);
    ~GpuGarbler();
    void to_device(const CrtLabels& cur);
    void to_host(CrtLabels& cur);
    // conv base labels: y = sum_{w != 0 mod p} w*x + (1 + #zero weights)*Z_p (padding reads Z_p);
    // w are the weights reduced mod M ([F][C][kh][kw]), wh their hash_i64 (plan cache key)
    void conv(const ConvGeom& G, const i64* w, size_t nw, uint64_t wh, CrtLabels& cur);
    // ReLU (relu_crt/prefix/mmg/mme set) or Sign layer: tables; device cur -> next base labels
    void sign_layer(uint64_t layer, const SignPlan& sp, CrtLabels& cur, Array& ap, Array& c1, Array& c2, Array& sg,
                    const std::vector<int>* relu_crt, const std::vector<i64>* prefix, Array* mmg, Array* mme);
    // one DASH legacy rescale iteration (sign base extension) on the device cur, in place
    void rescale_legacy_iter(uint64_t layer, int it, const RescalePlan& P, CrtLabels& cur,
                             const std::vector<std::vector<comp_t>>& up, const std::vector<std::vector<comp_t>>& down,
                             Array& tr, Array& ap, Array& c1, Array& c2, Array& sg);

    // legacy rescale as one mixed-radix gadget (gadgets.h RescaleMrsPlan) on the device cur, in place
    void rescale_mrs(uint64_t layer, const RescaleMrsPlan& P, CrtLabels& cur, Array& tab);

    // ReLU with the exact mixed-radix sign (gadgets.h SignMrsPlan) + mixed-modulus half gates; device cur -> next
    void relu_mrs(uint64_t layer, const SignMrsPlan& P, CrtLabels& cur, Array& tab, const std::vector<int>* relu_crt,
                  const std::vector<i64>* prefix, Array& mmg, Array& mme);

    // ReLU whose sign labels the preceding rescale_mrs (P.sign_last) left on the device: mixed-modulus half
    // gates only; device cur -> next
    void relu_mult(uint64_t layer, CrtLabels& cur, const std::vector<i64>* prefix, Array& mmg, Array& mme);

    // dense base labels y_o = sum_{w != 0 mod p} w x_src(i) + (1 + #zero weights) Z_p (w reduced mod M, [out][in],
    // src = dense_src(i, in, channel_tf))
    void dense(i64 in, i64 out, i64 channel_tf, const i64* w, size_t nw, uint64_t wh, CrtLabels& cur);
    // hardened encoding: cur_e += (c[e / group] mod p) R_p (public constants folded into the base labels)
    void fold_constants(const std::vector<i64>& c, i64 group, CrtLabels& cur);
    // window sums of the device cur
    void sumpool(const PoolGeom& G, CrtLabels& cur);
    // device copies of layer outputs a later residual add / in_src layer reads (idx = layer index + 1)
    void save(size_t idx);
    bool has_saved(size_t idx) const;
    void restore(size_t idx, CrtLabels& cur);
    void add_saved(size_t idx, CrtLabels& cur);
    // max pool / max: window values, one ReLU-gadget tree level per call (relu_garble_elem on streams
    // 20 + 2 lv / 21 + 2 lv), then the reduced values become cur
    void maxpool_begin(const std::vector<std::vector<i64>>& win, CrtLabels& cur);
    void maxpool_level(uint64_t layer, int lv, i64 ops, const SignPlan& sp, const std::vector<i64>& prefix, Array& ap,
                       Array& c1, Array& c2, Array& sg, Array& mmg, Array& mme);
    void maxpool_end(CrtLabels& cur);
    // ReDash rescale iteration (base-extension plan) on the device cur, in place
    void rescale_redash(uint64_t layer, int it, const RescalePlan& P, CrtLabels& cur,
                        const std::vector<std::vector<comp_t>>& up, const std::vector<std::vector<comp_t>>& down,
                        Array& tr, Array& be);
    // base-extension layer on the device cur, in place
    void base_ext(uint64_t layer, const BEPlan& P, CrtLabels& cur, Array& be);

    struct Impl;

   private:
    std::unique_ptr<Impl> impl_;
};

// Device blocks of garbled tables freed by their owners return to a small
// per-process cache (exact-size reuse: every GC of one model has the same
// table sizes), so back-to-back garbling skips the driver's allocate-and-clear
// of fresh HBM. Bounded by DASH_GG_CACHE_GB (default 16); trim releases it.
void gpu_table_cache_trim();
size_t gpu_table_cache_bytes();

}  // namespace dash
