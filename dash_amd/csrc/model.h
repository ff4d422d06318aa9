// GarbledModel: the single artefact passed from the garbler to the evaluator
// (offline message), plus the garbler-side secrets and decoder.
//
// The reference keeps garbler and evaluator state inside one object
// (garbling/garbled_circuit_interface.h) and never serializes it; here the
// two roles are split and the model has a versioned binary format
// (docs/WIRE_FORMAT.md) so that garbling and evaluation can run in different
// processes, hosts or devices.
#pragma once

#include <memory>
#include <mutex>
#include <string>

#include "core.h"
#include "gadgets.h"

namespace dash {

enum Kind : int {
    K_DENSE = 0,
    K_CONV = 1,
    K_RELU = 2,
    K_SIGN = 3,
    K_RESCALE = 4,
    K_MAXPOOL = 5,
    K_FLATTEN = 6,
    K_PROJ = 7,
    K_MULT = 8,
    K_MMULT = 9,
    K_MAX = 10,
    K_BASEEXT = 11,
    K_ADD = 12,
    K_SUMPOOL = 13,
};
const char* kind_name(int kind);

using Params = std::map<std::string, std::vector<i64>>;

struct LayerSpec {
    int kind = 0;
    Params p;
};

struct GLayer {
    int kind = 0;
    Params p;
    std::map<std::string, Array> a;
    i64 param(const std::string& k, i64 dflt = -1) const {
        auto it = p.find(k);
        return (it == p.end() || it->second.empty()) ? dflt : it->second[0];
    }
    const std::vector<i64>& vec(const std::string& k) const {
        auto it = p.find(k);
        DASH_CHECK(it != p.end(), std::string("missing layer param ") + k);
        return it->second;
    }
    const Array& arr(const std::string& k) const {
        auto it = a.find(k);
        DASH_CHECK(it != a.end(), std::string("missing layer array ") + k);
        return it->second;
    }
};

struct ModelHeader {
    int version = 4;  // 2: approx tables interleaved [color][digit]; 3: + sign construction flag; 4: + hardened
    int sign_fused = 0;  // 1: sign gadgets use the fused-cast construction (SignPlan::fused)
    // 1: hardened encoding (docs/SECURITY.md): no evaluator-visible constant labels (public-constant wires have
    // label 0: Z_p, bias, shift and padding labels are not shipped) and every table entry is masked by its own
    // tweaked pad (core.h hard_block) instead of the reference's shared H(K)
    int hardened = 0;
    std::vector<int> crt, mrs;
    std::vector<i64> in_dims, out_dims;
    std::vector<int> out_moduli;  // moduli of the output residues
    int max_mod = 0;
};

struct GarbledModel {
    ModelHeader h;
    std::map<std::string, Array> consts;  // evaluator-visible constants (Z_p, shift labels)
    std::vector<GLayer> layers;

    std::string serialize() const;
    // the offline message written straight into a caller buffer (device tables fetched into place)
    // Skeleton form (same-node device transport): arrays written into an evaluator slot through a sink
    // (Device::external; with all_device, every device-resident array) are sent as shape-only placeholders.
    std::string serialize_skeleton(bool all_device = false) const;
    static GarbledModel deserialize_skeleton(const uint8_t* blob, size_t nbytes);
    size_t serialized_size() const;
    size_t serialize_to(uint8_t* out, size_t cap) const;
    static GarbledModel deserialize(const std::string& blob);
    static GarbledModel deserialize(const uint8_t* blob, size_t nbytes);
    size_t table_bytes() const;  // bytes of garbled tables (u128 arrays)
    size_t total_bytes() const;
    LabelBank zero_bank() const;
};

// Held by whoever decodes the outputs (the garbler / client).
struct Decoder {
    std::vector<int> moduli;
    i64 n_out = 0;
    std::vector<Array> dec;  // per residue: u128 [p][n_out] = H(compress(out0 + v*R))
    std::vector<i64> decode(const CrtLabels& out) const;
    std::vector<i64> decode_residues(const CrtLabels& out) const;  // [k][n_out] residues
    // same, from compressed output labels C[j * n_out + e] (wire form of online message #2)
    std::vector<i64> decode_residues_compressed(const u128* C) const;
    std::vector<i64> decode_compressed(const u128* C) const;
    std::string serialize() const;
    static Decoder deserialize(const std::string& blob);
};

// Destination of garbled tables produced on the GPU (zero-copy offline phase): the GPU garbler writes
// table `name` of layer `layer` straight into the returned device buffer (e.g. a HipEvaluator's arena slot,
// HipEvaluator::sink) instead of a buffer of its own; null = no destination for that table.
struct TableSink {
    std::function<std::shared_ptr<Array::Device>(size_t layer, const std::string& name, size_t nbytes)> dest;
};

// A circuit's layer specs converted once, plus the public weights reduced mod M (and their content hash, the
// GPU plan key) shared by every GC garbled from them: per-GC host work no longer scales with the weight count
// (VGG-16: 15 M weights were copied, reduced and hashed for every GC).
struct GarbleSpecs {
    std::vector<LayerSpec> layers;
    struct Weights {
        Array w;            // int64 [out][in] / [F][C][kh][kw], reduced mod M
        uint64_t hash = 0;  // hash_i64 of w
    };
    std::mutex m;
    std::map<std::pair<size_t, i64>, Weights> wcache;  // (layer, M)
};

struct GarbleOptions {
    int nthreads = 0;
    int device = -1;  // >= 0: garble ReLU / Sign / legacy rescale layers on this GPU
    bool fused_sign = true;  // sign gadget construction (gadgets.h SignPlan::fused); false: reference casts
    bool rescale_mrs = false;  // legacy (l-halving) rescale as one mixed-radix gadget (gadgets.h RescaleMrsPlan)
    bool relu_mrs = false;     // ReLU sign by exact mixed-radix conversion (gadgets.h SignMrsPlan)
    // A ReLU right after a mixed-radix rescale takes its sign from that rescale's conversion
    // (gadgets.h RescaleMrsPlan::sign_last); other ReLUs use relu_mrs / the approximate gadget.
    bool relu_joint = false;
    bool hardened = false;  // ModelHeader::hardened
    std::shared_ptr<TableSink> sink;  // GPU-garbled tables go straight to these buffers (device >= 0 only)
    GarbleSpecs* cache = nullptr;     // reduced-weight cache of the specs being garbled (optional)
};

class Garbler {
   public:
    Garbler(const std::vector<int>& crt, const std::vector<int>& mrs, const std::string& seed16, int max_mod = 0);
    GarbledModel garble(const std::vector<LayerSpec>& layers, const std::vector<i64>& in_dims,
                        const GarbleOptions& opt = {});
    // Online message #1: encoded inputs x -> W0 + (x mod p) * R
    CrtLabels encode(const std::vector<i64>& x) const;
    // Same message compressed (16 B per label, the reference's wire size): dst[j * N + e]
    void encode_compressed(const i64* x, i64 N, u128* dst, int nthreads = 0) const;
    // Same message, component-major per residue: dst[j][c * N + e]
    void encode_cm(const i64* x, i64 N, const std::vector<comp_t*>& dst, int nthreads = 0) const;
    const Decoder& decoder() const { return dec_; }
    const std::vector<int>& crt() const { return crt_; }
    i64 crt_modulus() const { return M_; }
    // secrets (exposed for tests / the SGX-style split)
    const LabelBank& offsets() const { return R_; }
    const LabelBank& zeros() const { return Z_; }
    const CrtLabels& input_base() const { return in_base_; }
    // per-layer wall time of the last garble() (reference: BENCHMARK timers, garbled_circuit.h:111-116)
    const std::vector<double>& layer_ms() const { return layer_ms_; }

   private:
    std::vector<int> crt_, mrs_;
    i64 M_ = 1;
    int max_mod_ = 0;
    Prg prg_;
    std::string seed_;
    LabelBank R_, Z_;
    CrtLabels in_base_;
    Decoder dec_;
    std::vector<double> layer_ms_;
    // Input codebook: the compressed label of every (residue j, input element e, value v mod p_j), built
    // once per GC (offline, on first use) so online message #1 is a table lookup per label.
    struct InputCodebook {
        std::mutex m;
        bool built = false;
        int uses = 0;           // encodes so far: a GC encoded once (the protocol's case) never builds the table
        std::vector<u128> tab;  // residue j at off[j]: [N][p_j]
        std::vector<i64> off;
    };
    std::shared_ptr<InputCodebook> codebook_ = std::make_shared<InputCodebook>();
    const InputCodebook* input_codebook() const;
};

// Evaluator-side intermediate values (labels the evaluator computes anyway), per ReLU layer: its input labels
// and the sign labels (mod 2) its half gates are keyed by. Used by the security tests (tests/test_security.py),
// which attack the offline message from exactly this view.
struct EvalTrace {
    std::map<size_t, CrtLabels> relu_in;
    std::map<size_t, Labels> relu_sign;
};

// Host (oracle) evaluator: bit-exact reference for the HIP evaluator.
CrtLabels cpu_evaluate(const GarbledModel& m, const CrtLabels& inputs, int nthreads = 0,
                       std::vector<double>* layer_ms = nullptr, EvalTrace* trace = nullptr);

// Wire-form helpers: compressed labels [k][N] <-> CrtLabels
std::vector<u128> compress_labels(const CrtLabels& L, int nthreads = 0);
CrtLabels decompress_labels(const u128* C, const std::vector<int>& moduli, i64 N, int nthreads = 0);

// Required moduli (for R/Z banks) given bases.
int required_max_modulus(const std::vector<int>& crt, const std::vector<int>& mrs, const std::vector<LayerSpec>& layers,
                         bool rescale_mrs = false);

}  // namespace dash
