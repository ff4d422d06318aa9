#include <cstdio>
#include <cstdlib>
// Host garbler: turns a quantized layer list into a GarbledModel.
//
// Layer-level behaviour follows the reference garbled layers
// (garbling/garbled_circuit.h:129-408 dispatch; garbled_dense.h:88-118,
// garbled_conv2d.h:88-111, garbled_relu.h:119-179, garbled_sign.h,
// garbled_rescale.h:52-73, garbled_maxpool2d.h:64-141, garbled_projection.h,
// garbled_mult.h, garbled_mixed_mod_mult.h, garbled_base_extension.h) and the
// decoding information of garbled_circuit_interface.h:386-415. Work is
// parallel over elements with per-element PRG streams, so the result does not
// depend on the thread count.
#include <chrono>

#include "layers.h"
#include "hip/gpu_garbler.h"

namespace dash {

const char* kind_name(int kind) {
    switch (kind) {
        case K_DENSE: return "dense";
        case K_CONV: return "conv2d";
        case K_RELU: return "approx_relu";
        case K_SIGN: return "sign";
        case K_RESCALE: return "rescale";
        case K_MAXPOOL: return "max_pool";
        case K_FLATTEN: return "flatten";
        case K_PROJ: return "projection";
        case K_MULT: return "mult_layer";
        case K_MMULT: return "mixed_mod_mult_layer";
        case K_MAX: return "max";
        case K_BASEEXT: return "base_extension";
        case K_ADD: return "add";
        case K_SUMPOOL: return "sum_pool";
    }
    return "unknown";
}

std::string arr_name(const char* prefix, int idx, const char* suffix) {
    return std::string(prefix) + std::to_string(idx) + suffix;
}

ConvGeom::ConvGeom(const Params& p) {
    C = param1(p, "C");
    H = param1(p, "H");
    W = param1(p, "W");
    F = param1(p, "F");
    kh = param1(p, "kh");
    kw = param1(p, "kw");
    sh = param1(p, "sh", 1);
    sw = param1(p, "sw", 1);
    ph = param1(p, "ph", 0);
    pw = param1(p, "pw", 0);
    DASH_CHECK(C > 0 && H > 0 && W > 0 && F > 0 && kh > 0 && kw > 0 && sh > 0 && sw > 0, "bad conv geometry");
    OH = (H + 2 * ph - kh) / sh + 1;
    OW = (W + 2 * pw - kw) / sw + 1;
}

PoolGeom::PoolGeom(const Params& p) {
    C = param1(p, "C");
    H = param1(p, "H");
    W = param1(p, "W");
    kh = param1(p, "kh");
    kw = param1(p, "kw");
    sh = param1(p, "sh", kh);
    sw = param1(p, "sw", kw);
    DASH_CHECK(C > 0 && H >= kh && W >= kw && kh > 0 && kw > 0, "bad pool geometry");
    OH = (H - kh) / sh + 1;
    OW = (W - kw) / sw + 1;
}

void PoolGeom::window(i64 o, std::vector<i64>& idx) const {
    idx.clear();
    const i64 c = o / (OH * OW), r = o % (OH * OW), oy = r / OW, ox = r % OW;
    for (i64 dy = 0; dy < kh; ++dy)
        for (i64 dx = 0; dx < kw; ++dx) idx.push_back((c * H + oy * sh + dy) * W + ox * sw + dx);
}

MaxTree::MaxTree(i64 K) {
    int c = static_cast<int>(K);
    cnt.push_back(c);
    while (c > 1) {
        int o = c / 2;
        ops.push_back(o);
        c = o + (c % 2);
        cnt.push_back(c);
    }
}

int required_max_modulus(const std::vector<int>& crt, const std::vector<int>& mrs, const std::vector<LayerSpec>& layers,
                         bool rescale_mrs) {
    int mx = 2;
    for (int p : crt) mx = std::max(mx, p);
    const int k = static_cast<int>(crt.size());
    for (size_t d = 0; d < mrs.size(); ++d) {
        mx = std::max(mx, mrs[d]);
        if (d >= 1) mx = std::max(mx, (k + 1) * mrs[d]);
    }
    for (const auto& l : layers) {
        if (l.kind == K_PROJ) {
            for (auto v : paramv(l.p, "out_mod")) mx = std::max<int>(mx, static_cast<int>(v));
            for (auto v : paramv(l.p, "in_mod")) mx = std::max<int>(mx, static_cast<int>(v));
        }
        if (l.kind == K_MMULT) mx = std::max<int>(mx, static_cast<int>(param1(l.p, "q")));
        if (rescale_mrs && l.kind == K_RESCALE && param1(l.p, "mode", 0) == 0)
            mx = std::max<int>(mx, 2 << static_cast<int>(param1(l.p, "l")));  // the x_u mod 2^(l+1) label
    }
    return mx;
}

// ---------------------------------------------------------------------------
namespace {

// (-v mod M) of every value (the hardened encoding folds public constants c into garbler bases as -c R)
std::vector<i64> neg_mod(const std::vector<i64>& v, i64 M) {
    std::vector<i64> r(v.size());
    for (size_t i = 0; i < v.size(); ++i) r[i] = pmod(-pmod(v[i], M), M);
    return r;
}

// whether the GPU garbler produces hardened gadget tables (else hardened gadget layers garble on the host)
bool gpu_hardened() {
    static const bool on = [] {
        const char* e = std::getenv("DASH_GG_HARD");  // 0: hardened gadget layers on the host garbler (A/B)
        return !(e && e[0] == '0');
    }();
    return on;
}

struct ReluTables {
    Array approx, cast1, cast2, sign, g, e;
};

ReluTables make_relu_tables(const SignPlan& sp, i64 N, i64 sum_crt, int k) {
    ReluTables t;
    t.approx = Array(DType::u128, {N, sp.n_approx});
    if (sp.has_cast1()) t.cast1 = Array(DType::u128, {N, std::max<i64>(sp.n_cast, 1)});
    t.cast2 = Array(DType::u128, {N, std::max<i64>(sp.n_cast, 1)});
    t.sign = Array(DType::u128, {N, sp.n_sign});
    t.g = Array(DType::u128, {N, sum_crt});
    t.e = Array(DType::u128, {N, static_cast<i64>(k), 3});
    return t;
}

void put_relu_tables(GLayer& g, const std::string& pre, ReluTables& t) {
    g.a[pre + "s.approx"] = t.approx;
    if (t.cast1.nbytes) g.a[pre + "s.cast1"] = t.cast1;
    g.a[pre + "s.cast2"] = t.cast2;
    g.a[pre + "s.sign"] = t.sign;
    g.a[pre + "mm.g"] = t.g;
    g.a[pre + "mm.e"] = t.e;
}

// ReLU of one element: x (k residue labels) -> out (k residue labels).
void relu_garble_elem(const SignPlan& sp, const LabelBank& R, const LabelBank& Z, const Prg& prg, u64 s_stream,
                      u64 m_stream, const std::vector<int>& crt, const std::vector<i64>& prefix,
                      const comp_t* const* x0, ReluTables& t, i64 e, comp_t* const* out0, bool hard) {
    const int k = static_cast<int>(crt.size());
    comp_t sig[128];
    comp_t* outs[1] = {sig};
    sign_garble_elem(sp, R, Z, prg, s_stream, x0, t.approx.ptr<u128>() + e * sp.n_approx,
                     sp.has_cast1() ? t.cast1.ptr<u128>() + e * t.cast1.shape[1] : nullptr,
                     t.cast2.ptr<u128>() + e * t.cast2.shape[1],
                     t.sign.ptr<u128>() + e * sp.n_sign, outs, hard);
    u64 ctr = 0;
    const ModInfo& m2 = mod_info(2);
    for (int j = 0; j < k; ++j) {
        const ModInfo& mp = mod_info(crt[j]);
        mixed_mult_garble(x0[j], mp, sig, m2, R, prg, m_stream, ctr, t.g.ptr<u128>() + e * t.g.shape[1] + prefix[j],
                          t.e.ptr<u128>() + (e * k + j) * 3, out0[j], MMTw{hard, m_stream, j, k, true});
    }
}

}  // namespace

// ---------------------------------------------------------------------------
Garbler::Garbler(const std::vector<int>& crt, const std::vector<int>& mrs, const std::string& seed16, int max_mod)
    : crt_(crt), mrs_(mrs) {
    DASH_CHECK(!crt_.empty(), "empty CRT base");
    DASH_CHECK(seed16.size() == 16, "garbler seed must be 16 bytes");
    prg_ = Prg(reinterpret_cast<const uint8_t*>(seed16.data()));
    seed_ = seed16;
    for (int p : crt_) M_ *= p;
    max_mod_ = max_mod;
}

CrtLabels Garbler::encode(const std::vector<i64>& x) const {
    DASH_CHECK(!in_base_.empty(), "garble() must run before encode()");
    const i64 N = in_base_[0].N;
    DASH_CHECK(static_cast<i64>(x.size()) == N, "input size does not match the garbled circuit");
    CrtLabels out;
    for (size_t j = 0; j < crt_.size(); ++j) {
        const int p = crt_[j];
        Labels L(p, N);
        const comp_t* Rp = R_.get(p);
        for (i64 e = 0; e < N; ++e) lab_affine(L.at(e), in_base_[j].at(e), pmod(x[e], p), Rp, L.n, p);
        out.push_back(std::move(L));
    }
    return out;
}

void Garbler::encode_cm(const i64* x, i64 N, const std::vector<comp_t*>& dst, int nthreads) const {
    DASH_CHECK(!in_base_.empty() && in_base_[0].N == N, "input size does not match the garbled circuit");
    DASH_CHECK(dst.size() == crt_.size(), "need one destination per residue");
    const int k = static_cast<int>(crt_.size());
    // residues of every input once, then per residue a (value x component) LUT of v*R mod p
    std::vector<std::vector<uint16_t>> res(k, std::vector<uint16_t>(N));
    for (int j = 0; j < k; ++j)
        for (i64 e = 0; e < N; ++e) res[j][e] = static_cast<uint16_t>(pmod(x[e], crt_[j]));
    i64 total = 0;
    std::vector<i64> start(k + 1, 0);
    for (int j = 0; j < k; ++j) start[j + 1] = start[j] + nr_comps(crt_[j]);
    total = start[k];
    std::vector<std::vector<int16_t>> lut(k);
    for (int j = 0; j < k; ++j) {
        const int p = crt_[j], n = nr_comps(p);
        const comp_t* R = R_.get(p);
        lut[j].resize(static_cast<size_t>(p) * n);
        for (int v = 0; v < p; ++v)
            for (int c = 0; c < n; ++c) lut[j][v * n + c] = static_cast<int16_t>((v * R[c]) % p);
    }
    parallel_for(total, [&](i64 r0, i64 r1) {
        for (i64 r = r0; r < r1; ++r) {
            int j = 0;
            while (start[j + 1] <= r) ++j;
            const int c = static_cast<int>(r - start[j]);
            const int p = crt_[j], n = nr_comps(p);
            const Labels& W0 = in_base_[j];
            const int16_t* L = lut[j].data();
            comp_t* out = dst[j] + static_cast<i64>(c) * N;
            const uint16_t* rv = res[j].data();
            for (i64 e = 0; e < N; ++e) {
                int v = W0.c[e * n + c] + L[rv[e] * n + c];
                out[e] = static_cast<comp_t>(v >= p ? v - p : v);
            }
        }
    }, nthreads);
}

// Builds the input codebook on the second encode (bounded to 256 MiB; larger inputs use the per-label path).
// A GC is single use in the protocol, and its one encode is cheaper per label (k labels per input) than the
// codebook (sum of p_j labels per input); only a reused GC (benchmarks) amortizes the table.
const Garbler::InputCodebook* Garbler::input_codebook() const {
    InputCodebook& cb = *codebook_;
    std::lock_guard<std::mutex> g(cb.m);
    if (cb.built) return cb.tab.empty() ? nullptr : &cb;
    if (++cb.uses < 2) return nullptr;
    cb.built = true;
    if (in_base_.empty()) return nullptr;
    const int k = static_cast<int>(crt_.size());
    const i64 N = in_base_[0].N;
    i64 total = 0;
    cb.off.assign(k + 1, 0);
    for (int j = 0; j < k; ++j) cb.off[j + 1] = cb.off[j] + N * crt_[j];
    total = cb.off[k];
    if (static_cast<size_t>(total) * sizeof(u128) > (size_t(256) << 20)) return nullptr;
    cb.tab.resize(total);
    parallel_for(static_cast<i64>(k) * N, [&](i64 r0, i64 r1) {
        comp_t buf[128];
        for (i64 r = r0; r < r1; ++r) {
            const int j = static_cast<int>(r / N);
            const i64 e = r % N;
            const int p = crt_[j];
            const ModInfo& mi = mod_info(p);
            const comp_t* W0 = in_base_[j].at(e);
            const comp_t* R = R_.get(p);
            for (int c = 0; c < mi.n; ++c) buf[c] = W0[c];
            u128* out = cb.tab.data() + cb.off[j] + e * p;
            for (int v = 0; v < p; ++v) {  // W0 + v*R, stepping v by adding R
                out[v] = compress(buf, mi);
                for (int c = 0; c < mi.n; ++c) {
                    const int t = buf[c] + R[c];
                    buf[c] = static_cast<comp_t>(t >= p ? t - p : t);
                }
            }
        }
    });
    return &cb;
}

void Garbler::encode_compressed(const i64* x, i64 N, u128* dst, int nthreads) const {
    DASH_CHECK(!in_base_.empty() && in_base_[0].N == N, "input size does not match the garbled circuit");
    const int k = static_cast<int>(crt_.size());
    if (const InputCodebook* cb = input_codebook()) {
        // online message #1 = one codebook lookup per label
        for (int j = 0; j < k; ++j) {
            const int p = crt_[j];
            const u128* T = cb->tab.data() + cb->off[j];
            u128* d = dst + static_cast<i64>(j) * N;
            for (i64 e = 0; e < N; ++e) d[e] = T[e * p + pmod(x[e], p)];
        }
        return;
    }
    // per residue a (value x component) table of v*R mod p: one add and one conditional subtract per
    // component (a runtime-divisor 64-bit % per component was most of the cost)
    std::vector<std::vector<int16_t>> lut(k);
    for (int j = 0; j < k; ++j) {
        const int p = crt_[j], n = nr_comps(p);
        const comp_t* R = R_.get(p);
        lut[j].resize(static_cast<size_t>(p) * n);
        for (int v = 0; v < p; ++v)
            for (int c = 0; c < n; ++c) lut[j][static_cast<size_t>(v) * n + c] = static_cast<int16_t>((v * R[c]) % p);
    }
    // four labels of one residue per step (compress4: their Horner chains interleave; a fresh GC's first encode
    // is the batch-1 latency path of the wire form)
    parallel_for(static_cast<i64>(k) * N, [&](i64 r0, i64 r1) {
        comp_t buf[4][128];
        for (i64 r = r0; r < r1;) {
            const int j = static_cast<int>(r / N);
            const i64 e = r % N;
            const i64 cnt = std::min<i64>(4, std::min<i64>(r1 - r, N - e));
            const int p = crt_[j];
            const ModInfo& mi = mod_info(p);
            for (i64 q = 0; q < cnt; ++q) {
                const comp_t* W0 = in_base_[j].at(e + q);
                const int16_t* L = lut[j].data() + static_cast<size_t>(pmod(x[e + q], p)) * mi.n;
                for (int c = 0; c < mi.n; ++c) {
                    const int v = W0[c] + L[c];
                    buf[q][c] = static_cast<comp_t>(v >= p ? v - p : v);
                }
            }
            if (cnt == 4) {
                const comp_t* B[4] = {buf[0], buf[1], buf[2], buf[3]};
                compress4(B, mi, dst + r);
            } else {
                for (i64 q = 0; q < cnt; ++q) dst[r + q] = compress(buf[q], mi);
            }
            r += cnt;
        }
    }, nthreads);
}

std::vector<u128> compress_labels(const CrtLabels& L, int nthreads) {
    const int k = static_cast<int>(L.size());
    const i64 N = k ? L[0].N : 0;
    std::vector<u128> out(static_cast<size_t>(k) * N);
    parallel_for(static_cast<i64>(k) * N, [&](i64 r0, i64 r1) {
        for (i64 r = r0; r < r1; ++r) {
            const int j = static_cast<int>(r / N);
            out[r] = compress(L[j].at(r % N), mod_info(L[j].p));
        }
    }, nthreads);
    return out;
}

CrtLabels decompress_labels(const u128* C, const std::vector<int>& moduli, i64 N, int nthreads) {
    CrtLabels out;
    for (int p : moduli) out.emplace_back(p, N);
    const int k = static_cast<int>(moduli.size());
    parallel_for(static_cast<i64>(k) * N, [&](i64 r0, i64 r1) {
        for (i64 r = r0; r < r1; ++r) {
            const int j = static_cast<int>(r / N);
            const ModInfo& mi = mod_info(moduli[j]);
            comp_t* o = out[j].at(r % N);
            decompress(C[r], o, mi);
            for (int c = 0; c < mi.n; ++c)
                DASH_CHECK(o[c] >= 0 && o[c] < mi.p, "dash integrity: malformed compressed label");
        }
    }, nthreads);
    return out;
}

GarbledModel Garbler::garble(const std::vector<LayerSpec>& layers, const std::vector<i64>& in_dims,
                             const GarbleOptions& opt) {
    const int nt = opt.nthreads;
    const int k = static_cast<int>(crt_.size());
    const int need = required_max_modulus(crt_, mrs_, layers, opt.rescale_mrs);
    max_mod_ = std::max(max_mod_, need);
    GarbledModel m;
    const bool fused = opt.fused_sign;
    const bool hard = opt.hardened;
    m.h.sign_fused = fused ? 1 : 0;
    m.h.hardened = hard ? 1 : 0;
    if (hard) {
        // the hardened encoding keys no projection with a public label (docs/SECURITY.md): the reference's
        // cast construction (zero-label carry) and the legacy rescale (zero-label residue 0 -> sign gadget) do
        DASH_CHECK(fused, "the hardened encoding needs the fused sign construction");
        for (const auto& l : layers)
            DASH_CHECK(!(l.kind == K_RESCALE && param1(l.p, "mode", 0) == 0 && !opt.rescale_mrs),
                       "the hardened encoding has no legacy (sign base extension) rescale; use the mixed-radix "
                       "rescale (rescale_mrs)");
    }
    m.h.crt = crt_;
    m.h.mrs = mrs_;
    m.h.in_dims = in_dims;
    m.h.max_mod = max_mod_;

    // Offset and zero labels for every modulus 2..max_mod
    R_.max_mod = Z_.max_mod = max_mod_;
    R_.lab.assign(max_mod_ + 1, {});
    Z_.lab.assign(max_mod_ + 1, {});
    for (int p = 2; p <= max_mod_; ++p) {
        const int n = nr_comps(p);
        R_.lab[p].resize(n);
        Z_.lab[p].resize(n);
        u64 c1 = 0, c2 = 0;
        prg_.label(stream_id(kGlobalLayer, 1, p), c1, p, n, R_.lab[p].data());
        R_.lab[p][0] = 1;
        if (hard) continue;  // public zero wires have label 0 (nothing shipped)
        prg_.label(stream_id(kGlobalLayer, 2, p), c2, p, n, Z_.lab[p].data());
        Array z(DType::i16, {n});
        std::memcpy(z.ptr<comp_t>(), Z_.lab[p].data(), sizeof(comp_t) * n);
        m.consts["Z." + std::to_string(p)] = z;
    }

    std::unique_ptr<GpuGarbler> gpu;
    if (opt.device >= 0) gpu.reset(new GpuGarbler(crt_, mrs_, seed_, R_, Z_, opt.device, hard));
    // zero-copy offline phase: a GPU-garbled table whose destination the sink knows (an evaluator slot) is
    // written there directly; the model's array then aliases that buffer
    size_t cur_layer = 0;
    auto sinkify = [&](Array& a, const std::string& name) {
        if (!gpu || !opt.sink || !a.nbytes) return;
        auto d = opt.sink->dest(cur_layer, name, a.nbytes);
        if (d) a = Array::on_device(a.dtype, a.shape, std::move(d));
    };
    // a layer's public weights reduced mod M, and their content hash (the GPU plan key): computed once per specs
    // object (GarbleOptions::cache) and shared by every GC garbled from it
    auto reduced_weights = [&](size_t li, const std::vector<i64>& w, std::vector<i64> shape) {
        if (opt.cache) {
            std::lock_guard<std::mutex> lk(opt.cache->m);
            auto it = opt.cache->wcache.find({li, M_});
            if (it != opt.cache->wcache.end() && it->second.w.count() == w.size())
                return std::make_pair(it->second.w, it->second.hash);
        }
        Array wa(DType::i64, std::move(shape));
        DASH_CHECK(wa.count() == w.size(), "weight shape");
        i64* d = wa.ptr<i64>();
        parallel_for(static_cast<i64>(w.size()), [&](i64 b0, i64 b1) {
            for (i64 i = b0; i < b1; ++i) d[i] = pmod(w[i], M_);
        }, nt);
        const uint64_t h = hash_i64(d, w.size());
        if (opt.cache) {
            std::lock_guard<std::mutex> lk(opt.cache->m);
            opt.cache->wcache[{li, M_}] = GarbleSpecs::Weights{wa, h};
        }
        return std::make_pair(wa, h);
    };
    // which copy of `cur` is current: GPU layers read and write the device copy,
    // host layers the host copy; a copy is refreshed only when the other side changed it
    bool host_ok = true, dev_ok = false;

    // Input base labels
    i64 N = 1;
    for (auto d : in_dims) N *= d;
    in_base_.clear();
    codebook_ = std::make_shared<InputCodebook>();  // a new garbling invalidates the input codebook
    for (int j = 0; j < k; ++j) {
        Labels L(crt_[j], N);
        parallel_for(N, [&](i64 b, i64 e_) {
            for (i64 e = b; e < e_; ++e) {
                u64 c = 0;
                prg_.label(stream_id(kGlobalLayer, 3 + j, e), c, L.p, L.n, L.at(e));
            }
        }, nt);
        in_base_.push_back(std::move(L));
    }
    // Rescale shift labels (shared per circuit, reference gci.h:957-980)
    std::vector<std::vector<comp_t>> up_base(k);
    std::map<i64, std::vector<std::vector<comp_t>>> down_base;
    auto get_up = [&]() {
        if (up_base[0].empty()) {
            for (int j = 0; j < k; ++j) {
                const int p = crt_[j], n = nr_comps(p);
                up_base[j].resize(n);
                if (hard) {  // the constant wire's base is -(M/2) R, so its label is 0 (not shipped)
                    std::vector<comp_t> zero(n, 0);
                    lab_affine(up_base[j].data(), zero.data(), -pmod(M_ / 2, p), R_.get(p), n, p);
                    continue;
                }
                u64 c = 0;
                prg_.label(stream_id(kGlobalLayer, 110, j), c, p, n, up_base[j].data());
                Array a(DType::i16, {n});
                lab_affine(a.ptr<comp_t>(), up_base[j].data(), pmod(M_ / 2, p), R_.get(p), n, p);
                m.consts["up." + std::to_string(j)] = a;
            }
        }
    };
    auto get_down = [&](i64 sprod) -> std::vector<std::vector<comp_t>>& {
        auto it = down_base.find(sprod);
        if (it != down_base.end()) return it->second;
        auto& v = down_base[sprod];
        v.resize(k);
        for (int j = 0; j < k; ++j) {
            const int p = crt_[j], n = nr_comps(p);
            v[j].resize(n);
            if (hard) {  // base -c R: label 0
                std::vector<comp_t> zero(n, 0);
                lab_affine(v[j].data(), zero.data(), -pmod(M_ / (2 * sprod), p), R_.get(p), n, p);
                continue;
            }
            u64 c = 0;
            prg_.label(stream_id(kGlobalLayer, 111, (static_cast<u64>(sprod) << 8) | j), c, p, n, v[j].data());
            Array a(DType::i16, {n});
            lab_affine(a.ptr<comp_t>(), v[j].data(), pmod(M_ / (2 * sprod), p), R_.get(p), n, p);
            m.consts["down." + std::to_string(sprod) + "." + std::to_string(j)] = a;
        }
        return v;
    };

    // which layer outputs are referenced by residual adds
    // (and by layers that read an earlier output, param "in_src": projection shortcuts)
    std::vector<int> keep(layers.size() + 1, 0);
    for (const auto& l : layers) {
        if (l.kind == K_ADD) keep[param1(l.p, "src") + 1] = 1;
        auto it = l.p.find("in_src");
        if (it != l.p.end() && !it->second.empty()) keep[it->second[0] + 1] = 1;
    }
    std::vector<CrtLabels> saved(layers.size() + 1);
    std::vector<std::vector<int>> saved_mod(layers.size() + 1);
    std::vector<std::vector<i64>> saved_dims(layers.size() + 1);

    CrtLabels cur = in_base_;
    std::vector<int> cur_mod = crt_;
    std::vector<i64> dims = in_dims;
    if (keep[0]) {
        // with a GPU garbler, outputs read again later (residual adds, in_src) are kept as device copies
        if (gpu) {
            gpu->to_device(cur);
            dev_ok = true;
            gpu->save(0);
        } else {
            saved[0] = cur;
        }
        saved_mod[0] = cur_mod;
        saved_dims[0] = dims;
    }
    std::vector<i64> prefix(k);
    i64 sum_crt = 0;
    for (int j = 0; j < k; ++j) {
        prefix[j] = sum_crt;
        sum_crt += crt_[j];
    }

    layer_ms_.assign(layers.size(), 0.0);
    // joint rescale + ReLU sign: the rescale leaves the sign base labels here (host) or in the GPU garbler
    bool sig_next = false;
    Labels sig_host;
    for (size_t li = 0; li < layers.size(); ++li) {
        const auto t_layer = std::chrono::steady_clock::now();
        const LayerSpec& spec = layers[li];
        cur_layer = li;
        const u64 L = li + 1;
        const bool sig_in = sig_next;  // the previous layer (a mixed-radix rescale) produced this ReLU's sign
        sig_next = false;
        {
            auto it = spec.p.find("in_src");
            if (it != spec.p.end() && !it->second.empty()) {
                const i64 s = it->second[0];
                DASH_CHECK(s >= -1 && s < static_cast<i64>(li), "in_src must name an earlier layer");
                if (gpu) {
                    gpu->restore(static_cast<size_t>(s + 1), cur);
                    host_ok = false;
                    dev_ok = true;
                } else {
                    cur = saved[s + 1];
                    host_ok = true;
                    dev_ok = false;
                }
                cur_mod = saved_mod[s + 1];
                dims = saved_dims[s + 1];
            }
        }
        GLayer g;
        g.kind = spec.kind;
        // copy scalar/list params except the large weight arrays (stored as arrays)
        for (const auto& kv : spec.p)
            if (kv.first != "w" && kv.first != "b") g.p[kv.first] = kv.second;
        const i64 Nin = cur[0].N;
        auto is_crt = [&]() {
            for (int j = 0; j < k; ++j)
                if (cur_mod[j] != crt_[j]) return false;
            return true;
        };

        // legacy rescale as one mixed-radix gadget (RescaleMrsPlan)
        const bool mrs_rescale = opt.rescale_mrs && spec.kind == K_RESCALE && param1(spec.p, "mode", 0) == 0;
        const bool relu_mrs = opt.relu_mrs && spec.kind == K_RELU;
        const bool joint_out = mrs_rescale && opt.relu_joint && li + 1 < layers.size() &&
                               layers[li + 1].kind == K_RELU && param1(layers[li + 1].p, "in_src", -2) == -2;
        // every layer kind but the test-only projection / mult layers garbles on the device when a GPU garbler
        // is present (the legacy rescale's sign base extension needs residue 0 = 2)
        const bool lin_kind = spec.kind == K_CONV || spec.kind == K_DENSE || spec.kind == K_SUMPOOL || spec.kind == K_ADD;
        const bool on_gpu = gpu && (lin_kind || ((!hard || gpu_hardened()) &&
                                    (spec.kind == K_RELU || spec.kind == K_SIGN ||
                                    spec.kind == K_MAXPOOL || spec.kind == K_MAX || spec.kind == K_BASEEXT ||
                                    (spec.kind == K_RESCALE && (param1(spec.p, "mode", 0) != 0 || crt_[0] == 2)))));
        const bool passthru = spec.kind == K_FLATTEN;
        if (on_gpu && !dev_ok) {
            gpu->to_device(cur);
            dev_ok = true;
        } else if (!on_gpu && !passthru && !host_ok) {
            gpu->to_host(cur);
            host_ok = true;
        }
        switch (spec.kind) {
            case K_FLATTEN: {
                dims = {Nin};
                break;
            }
            case K_DENSE: {
                DASH_CHECK(is_crt(), "dense needs CRT-base labels");
                const i64 in = param1(spec.p, "in"), out = param1(spec.p, "out");
                const i64 ch = param1(spec.p, "channel_tf", 0);
                DASH_CHECK(in == Nin, "dense input size mismatch");
                const auto& w = paramv(spec.p, "w");
                const auto& b = paramv(spec.p, "b");
                DASH_CHECK(static_cast<i64>(w.size()) == in * out && static_cast<i64>(b.size()) == out, "dense weight shape");
                const auto rw = reduced_weights(li, w, {out, in});
                const Array& wa = rw.first;
                g.a["w"] = wa;
                CrtLabels nxt;
                for (int j = 0; j < k; ++j) {
                    const int p = crt_[j];
                    const ModInfo& mi = mod_info(p);
                    Labels O(p, out);
                    const comp_t* Zp = Z_.get(p);
                    // garbler-side base of each bias wire: Z_p (its label Z_p + b R is shipped) or, hardened,
                    // -b R (label 0, not shipped)
                    std::vector<comp_t> bbase(static_cast<size_t>(out) * mi.n);
                    if (hard) {
                        for (i64 o = 0; o < out; ++o)
                            lab_affine(bbase.data() + o * mi.n, Zp, -pmod(pmod(b[o], M_), p), R_.get(p), mi.n, p);
                    } else {
                        Array bias(DType::i16, {out, mi.n});
                        for (i64 o = 0; o < out; ++o) {
                            lab_affine(bias.ptr<comp_t>() + o * mi.n, Zp, pmod(pmod(b[o], M_), p), R_.get(p), mi.n, p);
                            std::memcpy(bbase.data() + o * mi.n, Zp, sizeof(comp_t) * mi.n);
                        }
                        g.a[arr_name("bias.", j, "")] = bias;
                    }
                    if (on_gpu) continue;
                    const Labels& I = cur[j];
                    parallel_for(out, [&](i64 b0, i64 b1) {
                        std::vector<i64> acc(mi.n);
                        for (i64 o = b0; o < b1; ++o) {
                            std::fill(acc.begin(), acc.end(), 0);
                            i64 zc = 0;
                            const i64* wr = wa.ptr<i64>() + o * in;
                            for (i64 i = 0; i < in; ++i) {
                                const i64 wv = wr[i] % p;
                                if (wv == 0) {
                                    ++zc;
                                    continue;
                                }
                                const comp_t* x = I.at(dense_src(i, in, ch));
                                for (int c = 0; c < mi.n; ++c) acc[c] += wv * x[c];
                            }
                            comp_t* y = O.at(o);
                            const comp_t* bb = bbase.data() + o * mi.n;
                            for (int c = 0; c < mi.n; ++c) y[c] = static_cast<comp_t>((acc[c] + zc * Zp[c] + bb[c]) % p);
                        }
                    }, nt);
                    nxt.push_back(std::move(O));
                }
                if (on_gpu) {
                    gpu->dense(in, out, ch, wa.ptr<i64>(), wa.count(), rw.second, cur);
                    if (hard) gpu->fold_constants(neg_mod(b, M_), 1, cur);
                } else {
                    cur = std::move(nxt);
                }
                dims = {out};
                break;
            }
            case K_CONV: {
                DASH_CHECK(is_crt(), "conv needs CRT-base labels");
                ConvGeom G(spec.p);
                DASH_CHECK(G.C * G.H * G.W == Nin, "conv input size mismatch");
                const auto& w = paramv(spec.p, "w");
                const auto& b = paramv(spec.p, "b");
                DASH_CHECK(static_cast<i64>(w.size()) == G.F * G.K() && static_cast<i64>(b.size()) == G.F, "conv weight shape");
                const auto rw = reduced_weights(li, w, {G.F, G.C, G.kh, G.kw});
                const Array& wa = rw.first;
                g.a["w"] = wa;
                CrtLabels nxt;
                for (int j = 0; j < k && !hard; ++j) {
                    const int p = crt_[j];
                    const ModInfo& mi = mod_info(p);
                    const comp_t* Zp = Z_.get(p);
                    Array bias(DType::i16, {G.F, mi.n});
                    for (i64 f = 0; f < G.F; ++f)
                        lab_affine(bias.ptr<comp_t>() + f * mi.n, Zp, pmod(pmod(b[f], M_), p), R_.get(p), mi.n, p);
                    g.a[arr_name("bias.", j, "")] = bias;
                }
                if (on_gpu) {
                    gpu->conv(G, wa.ptr<i64>(), wa.count(), rw.second, cur);
                    if (hard) gpu->fold_constants(neg_mod(b, M_), G.OH * G.OW, cur);
                    dims = {G.F, G.OH, G.OW};
                    break;
                }
                for (int j = 0; j < k; ++j) {
                    const int p = crt_[j];
                    const ModInfo& mi = mod_info(p);
                    const comp_t* Zp = Z_.get(p);
                    Labels O(p, G.out_size());
                    const Labels& I = cur[j];
                    parallel_for(G.out_size(), [&](i64 b0, i64 b1) {
                        std::vector<i64> acc(mi.n);
                        for (i64 o = b0; o < b1; ++o) {
                            const i64 f = o / (G.OH * G.OW), r = o % (G.OH * G.OW), oy = r / G.OW, ox = r % G.OW;
                            std::fill(acc.begin(), acc.end(), 0);
                            // bias wire: base Z_p (reference) or -b R (hardened, label 0)
                            i64 zc = hard ? 0 : 1;
                            const i64 bneg = hard ? pmod(-pmod(b[f], M_), p) : 0;
                            const i64* wf = wa.ptr<i64>() + f * G.K();
                            for (i64 c = 0; c < G.C; ++c)
                                for (i64 dy = 0; dy < G.kh; ++dy)
                                    for (i64 dx = 0; dx < G.kw; ++dx) {
                                        const i64 wv = wf[(c * G.kh + dy) * G.kw + dx] % p;
                                        if (wv == 0) {
                                            ++zc;
                                            continue;
                                        }
                                        const i64 iy = oy * G.sh - G.ph + dy, ix = ox * G.sw - G.pw + dx;
                                        const comp_t* x = (iy < 0 || iy >= G.H || ix < 0 || ix >= G.W)
                                                              ? Zp
                                                              : I.at((c * G.H + iy) * G.W + ix);
                                        for (int cc = 0; cc < mi.n; ++cc) acc[cc] += wv * x[cc];
                                    }
                            comp_t* y = O.at(o);
                            const comp_t* Rp = R_.get(p);
                            for (int cc = 0; cc < mi.n; ++cc)
                                y[cc] = static_cast<comp_t>((acc[cc] + zc * Zp[cc] + bneg * Rp[cc]) % p);
                        }
                    }, nt);
                    nxt.push_back(std::move(O));
                }
                cur = std::move(nxt);
                dims = {G.F, G.OH, G.OW};
                break;
            }
            case K_RELU: {
                DASH_CHECK(is_crt(), "relu needs CRT-base labels");
                if (sig_in) {
                    // sign from the preceding rescale (RescaleMrsPlan::sign_last): mixed-modulus half gates only
                    Array tg(DType::u128, {Nin, sum_crt}), te(DType::u128, {Nin, static_cast<i64>(k), 3});
                    if (on_gpu) {
                        sinkify(tg, "mm.g");
                        sinkify(te, "mm.e");
                        gpu->relu_mult(L, cur, &prefix, tg, te);
                    } else {
                        DASH_CHECK(sig_host.N == Nin, "joint ReLU: sign labels missing");
                        CrtLabels nxt;
                        for (int j = 0; j < k; ++j) nxt.emplace_back(crt_[j], Nin);
                        parallel_for(Nin, [&](i64 b0, i64 b1) {
                            const ModInfo& m2 = mod_info(2);
                            for (i64 e = b0; e < b1; ++e) {
                                u64 ctr = 0;
                                for (int j = 0; j < k; ++j)
                                    mixed_mult_garble(cur[j].at(e), mod_info(crt_[j]), sig_host.at(e), m2, R_, prg_,
                                                      stream_id(L, 2, e), ctr, tg.ptr<u128>() + e * sum_crt + prefix[j],
                                                      te.ptr<u128>() + (e * k + j) * 3, nxt[j].at(e),
                                                      MMTw{hard, stream_id(L, 2, e), j, k, true});
                            }
                        }, nt);
                        cur = std::move(nxt);
                    }
                    g.a["mm.g"] = tg;
                    g.a["mm.e"] = te;
                    g.p["smode"] = {2};
                    break;
                }
                if (relu_mrs) {
                    const SignMrsPlan sp(crt_);
                    Array tab(DType::u128, {Nin, std::max<i64>(sp.n_tab, 1)});
                    Array tg(DType::u128, {Nin, sum_crt}), te(DType::u128, {Nin, static_cast<i64>(k), 3});
                    if (on_gpu) {
                        sinkify(tab, "mrs");
                        sinkify(tg, "mm.g");
                        sinkify(te, "mm.e");
                        gpu->relu_mrs(L, sp, cur, tab, &crt_, &prefix, tg, te);
                    } else {
                        CrtLabels nxt;
                        for (int j = 0; j < k; ++j) nxt.emplace_back(crt_[j], Nin);
                        parallel_for(Nin, [&](i64 b0, i64 b1) {
                            std::vector<const comp_t*> x(k);
                            comp_t sig[128];
                            const ModInfo& m2 = mod_info(2);
                            for (i64 e = b0; e < b1; ++e) {
                                for (int j = 0; j < k; ++j) x[j] = cur[j].at(e);
                                sign_mrs_garble_elem(sp, R_, prg_, stream_id(L, 1, e), x.data(),
                                                     tab.ptr<u128>() + e * tab.shape[1], sig, hard);
                                u64 ctr = 0;
                                for (int j = 0; j < k; ++j)
                                    mixed_mult_garble(x[j], mod_info(crt_[j]), sig, m2, R_, prg_, stream_id(L, 2, e), ctr,
                                                      tg.ptr<u128>() + e * sum_crt + prefix[j],
                                                      te.ptr<u128>() + (e * k + j) * 3, nxt[j].at(e),
                                                      MMTw{hard, stream_id(L, 2, e), j, k, true});
                            }
                        }, nt);
                        cur = std::move(nxt);
                    }
                    g.a["mrs"] = tab;
                    g.a["mm.g"] = tg;
                    g.a["mm.e"] = te;
                    g.p["smode"] = {1};
                    break;
                }
                SignPlan sp(crt_, mrs_, {2}, 0, 1, fused);
                ReluTables t = make_relu_tables(sp, Nin, sum_crt, k);
                CrtLabels nxt;
                if (on_gpu) {
                    sinkify(t.approx, "s.approx");
                    sinkify(t.cast1, "s.cast1");
                    sinkify(t.cast2, "s.cast2");
                    sinkify(t.sign, "s.sign");
                    sinkify(t.g, "mm.g");
                    sinkify(t.e, "mm.e");
                    gpu->sign_layer(L, sp, cur, t.approx, t.cast1, t.cast2, t.sign, &crt_, &prefix, &t.g, &t.e);
                    put_relu_tables(g, "", t);
                    break;
                }
                for (int j = 0; j < k; ++j) nxt.emplace_back(crt_[j], Nin);
                parallel_for(Nin, [&](i64 b0, i64 b1) {
                    std::vector<const comp_t*> x(k);
                    std::vector<comp_t*> y(k);
                    for (i64 e = b0; e < b1; ++e) {
                        for (int j = 0; j < k; ++j) {
                            x[j] = cur[j].at(e);
                            y[j] = nxt[j].at(e);
                        }
                        relu_garble_elem(sp, R_, Z_, prg_, stream_id(L, 1, e), stream_id(L, 2, e), crt_, prefix,
                                         x.data(), t, e, y.data(), hard);
                    }
                }, nt);
                put_relu_tables(g, "", t);
                cur = std::move(nxt);
                break;
            }
            case K_SIGN: {
                DASH_CHECK(is_crt(), "sign needs CRT-base labels");
                SignPlan sp(crt_, mrs_, crt_, -1, 1, fused);
                Array ap(DType::u128, {Nin, sp.n_approx}), c1, c2(DType::u128, {Nin, std::max<i64>(sp.n_cast, 1)}),
                    sg(DType::u128, {Nin, sp.n_sign});
                if (sp.has_cast1()) c1 = Array(DType::u128, {Nin, std::max<i64>(sp.n_cast, 1)});
                CrtLabels nxt;
                if (on_gpu) {
                    sinkify(ap, "s.approx");
                    sinkify(c1, "s.cast1");
                    sinkify(c2, "s.cast2");
                    sinkify(sg, "s.sign");
                    gpu->sign_layer(L, sp, cur, ap, c1, c2, sg, nullptr, nullptr, nullptr, nullptr);
                } else {
                    for (int j = 0; j < k; ++j) nxt.emplace_back(crt_[j], Nin);
                }
                if (!on_gpu) parallel_for(Nin, [&](i64 b0, i64 b1) {
                    std::vector<const comp_t*> x(k);
                    std::vector<comp_t*> y(k);
                    for (i64 e = b0; e < b1; ++e) {
                        for (int j = 0; j < k; ++j) {
                            x[j] = cur[j].at(e);
                            y[j] = nxt[j].at(e);
                        }
                        sign_garble_elem(sp, R_, Z_, prg_, stream_id(L, 1, e), x.data(),
                                         ap.ptr<u128>() + e * sp.n_approx,
                                         sp.has_cast1() ? c1.ptr<u128>() + e * c1.shape[1] : nullptr,
                                         c2.ptr<u128>() + e * c2.shape[1], sg.ptr<u128>() + e * sp.n_sign, y.data(), hard);
                    }
                }, nt);
                g.a["s.approx"] = ap;
                if (sp.has_cast1()) g.a["s.cast1"] = c1;
                g.a["s.cast2"] = c2;
                g.a["s.sign"] = sg;
                if (!on_gpu) cur = std::move(nxt);
                break;
            }
            case K_RESCALE: {
                DASH_CHECK(is_crt(), "rescale needs CRT-base labels");
                const i64 mode = param1(spec.p, "mode", 0);
                if (mrs_rescale) {
                    const RescaleMrsPlan P(crt_, static_cast<int>(param1(spec.p, "l")), joint_out);
                    Array tab(DType::u128, {Nin, P.n_tab});
                    if (joint_out && !on_gpu) sig_host = Labels(2, Nin);
                    if (on_gpu) {
                        sinkify(tab, "mrs");
                        gpu->rescale_mrs(L, P, cur, tab);
                    }
                    else parallel_for(Nin, [&](i64 b0, i64 b1) {
                        std::vector<comp_t*> Lp(k);
                        for (i64 e = b0; e < b1; ++e) {
                            for (int j = 0; j < k; ++j) Lp[j] = cur[j].at(e);
                            rescale_mrs_garble_elem(P, R_, prg_, stream_id(L, 30, e), Lp.data(),
                                                    tab.ptr<u128>() + e * P.n_tab,
                                                    joint_out ? sig_host.at(e) : nullptr, hard);
                        }
                    }, nt);
                    g.a["mrs"] = tab;
                    g.p["mode"] = {2};
                    if (joint_out) {
                        g.p["sign_out"] = {1};
                        sig_next = true;
                    }
                    g.p["iters"] = {1};
                    g.p["sprod"] = {P.S};
                    break;
                }
                std::vector<RescalePlan> plans;
                if (mode == 0) {
                    const i64 l = param1(spec.p, "l");
                    DASH_CHECK(l >= 1, "legacy rescale needs l >= 1");
                    for (i64 i = 0; i < l; ++i) plans.emplace_back(crt_, mrs_, std::vector<int>{2}, true, fused);
                } else {
                    std::vector<int> s;
                    for (auto v : paramv(spec.p, "s")) s.push_back(static_cast<int>(v));
                    plans.emplace_back(crt_, mrs_, s, false, fused);
                }
                get_up();
                std::vector<const comp_t*> upp(k);
                for (int j = 0; j < k; ++j) upp[j] = up_base[j].data();
                for (size_t it = 0; it < plans.size(); ++it) {
                    const RescalePlan& P = plans[it];
                    auto& dn = get_down(P.sprod);
                    std::vector<const comp_t*> dnp(k);
                    for (int j = 0; j < k; ++j) dnp[j] = dn[j].data();
                    const std::string pre = arr_name("it", static_cast<int>(it), ".");
                    Array tr(DType::u128, {Nin, P.n_trans});
                    Array ap, c1, c2, sg, be;
                    if (P.sign_be) {
                        ap = Array(DType::u128, {Nin, P.sign.n_approx});
                        if (P.sign.has_cast1()) c1 = Array(DType::u128, {Nin, std::max<i64>(P.sign.n_cast, 1)});
                        c2 = Array(DType::u128, {Nin, std::max<i64>(P.sign.n_cast, 1)});
                        sg = Array(DType::u128, {Nin, P.sign.n_sign});
                    } else {
                        be = Array(DType::u128, {Nin, P.n_be});
                    }
                    if (on_gpu && !P.sign_be) {
                        sinkify(tr, pre + "trans");
                        sinkify(be, pre + "be");
                        gpu->rescale_redash(L, static_cast<int>(it), P, cur, up_base, dn, tr, be);
                    } else if (on_gpu) {
                        sinkify(tr, pre + "trans");
                        sinkify(ap, pre + "s.approx");
                        sinkify(c1, pre + "s.cast1");
                        sinkify(c2, pre + "s.cast2");
                        sinkify(sg, pre + "s.sign");
                        gpu->rescale_legacy_iter(L, static_cast<int>(it), P, cur, up_base, dn, tr, ap, c1, c2, sg);
                    } else parallel_for(Nin, [&](i64 b0, i64 b1) {
                        std::vector<comp_t*> Lp(k);
                        for (i64 e = b0; e < b1; ++e) {
                            for (int j = 0; j < k; ++j) Lp[j] = cur[j].at(e);
                            if (P.sign_be) {
                                rescale_garble_elem(P, R_, Z_, prg_, stream_id(L, 10 + it, e), Lp.data(), upp.data(),
                                                    dnp.data(), tr.ptr<u128>() + e * P.n_trans,
                                                    ap.ptr<u128>() + e * ap.shape[1],
                                                    P.sign.has_cast1() ? c1.ptr<u128>() + e * c1.shape[1] : nullptr,
                                                    c2.ptr<u128>() + e * c2.shape[1], sg.ptr<u128>() + e * sg.shape[1],
                                                    nullptr, hard);
                            } else {
                                rescale_garble_elem(P, R_, Z_, prg_, stream_id(L, 10 + it, e), Lp.data(), upp.data(),
                                                    dnp.data(), tr.ptr<u128>() + e * P.n_trans, nullptr, nullptr,
                                                    nullptr, nullptr, be.ptr<u128>() + e * P.n_be, hard);
                            }
                        }
                    }, nt);
                    g.a[pre + "trans"] = tr;
                    if (P.sign_be) {
                        g.a[pre + "s.approx"] = ap;
                        if (P.sign.has_cast1()) g.a[pre + "s.cast1"] = c1;
                        g.a[pre + "s.cast2"] = c2;
                        g.a[pre + "s.sign"] = sg;
                    } else {
                        g.a[pre + "be"] = be;
                    }
                }
                g.p["iters"] = {static_cast<i64>(plans.size())};
                g.p["sprod"] = {plans[0].sprod};
                break;
            }
            case K_MAXPOOL:
            case K_MAX: {
                DASH_CHECK(is_crt(), "max needs CRT-base labels");
                i64 Nout, K;
                std::vector<std::vector<i64>> win;
                if (spec.kind == K_MAXPOOL) {
                    PoolGeom G(spec.p);
                    DASH_CHECK(G.C * G.H * G.W == Nin, "maxpool input size mismatch");
                    Nout = G.out_size();
                    K = G.kh * G.kw;
                    win.resize(Nout);
                    for (i64 o = 0; o < Nout; ++o) G.window(o, win[o]);
                    dims = {G.C, G.OH, G.OW};
                } else {
                    Nout = 1;
                    K = Nin;
                    win.resize(1);
                    for (i64 i = 0; i < Nin; ++i) win[0].push_back(i);
                    dims = {1};
                }
                MaxTree T(K);
                SignPlan sp(crt_, mrs_, {2}, 0, 1, fused);
                if (on_gpu) {
                    gpu->maxpool_begin(win, cur);
                    for (size_t lv = 0; lv < T.ops.size(); ++lv) {
                        ReluTables t = make_relu_tables(sp, Nout * T.ops[lv], sum_crt, k);
                        const std::string pre = arr_name("lv", static_cast<int>(lv), ".");
                        sinkify(t.approx, pre + "s.approx");
                        sinkify(t.cast1, pre + "s.cast1");
                        sinkify(t.cast2, pre + "s.cast2");
                        sinkify(t.sign, pre + "s.sign");
                        sinkify(t.g, pre + "mm.g");
                        sinkify(t.e, pre + "mm.e");
                        gpu->maxpool_level(L, static_cast<int>(lv), T.ops[lv], sp, prefix, t.approx, t.cast1, t.cast2,
                                           t.sign, t.g, t.e);
                        put_relu_tables(g, pre, t);
                    }
                    gpu->maxpool_end(cur);
                    g.p["levels"] = {static_cast<i64>(T.ops.size())};
                    break;
                }
                // value slots: vals[j] holds Nout x cnt labels (slot-major per output)
                std::vector<Labels> vals;
                for (int j = 0; j < k; ++j) {
                    Labels V(crt_[j], Nout * K);
                    for (i64 o = 0; o < Nout; ++o)
                        for (i64 s = 0; s < K; ++s)
                            std::memcpy(V.at(o * K + s), cur[j].at(win[o][s]), sizeof(comp_t) * V.n);
                    vals.push_back(std::move(V));
                }
                for (size_t lv = 0; lv < T.ops.size(); ++lv) {
                    const i64 ops = T.ops[lv], cnt = T.cnt[lv], cnt1 = T.cnt[lv + 1];
                    ReluTables t = make_relu_tables(sp, Nout * ops, sum_crt, k);
                    std::vector<Labels> nv;
                    for (int j = 0; j < k; ++j) nv.emplace_back(crt_[j], Nout * cnt1);
                    parallel_for(Nout * ops, [&](i64 b0, i64 b1) {
                        std::vector<std::vector<comp_t>> diff(k);
                        std::vector<const comp_t*> x(k);
                        std::vector<comp_t*> y(k);
                        for (int j = 0; j < k; ++j) diff[j].resize(nr_comps(crt_[j]));
                        for (i64 e = b0; e < b1; ++e) {
                            const i64 o = e / ops, q = e % ops;
                            for (int j = 0; j < k; ++j) {
                                const int n = vals[j].n, p = vals[j].p;
                                std::memcpy(diff[j].data(), vals[j].at(o * cnt + 2 * q + 1), sizeof(comp_t) * n);
                                lab_sub(diff[j].data(), vals[j].at(o * cnt + 2 * q), n, p);
                                x[j] = diff[j].data();
                                y[j] = nv[j].at(o * cnt1 + q);
                            }
                            relu_garble_elem(sp, R_, Z_, prg_, stream_id(L, 20 + 2 * lv, e), stream_id(L, 21 + 2 * lv, e),
                                             crt_, prefix, x.data(), t, e, y.data(), hard);
                            for (int j = 0; j < k; ++j)
                                lab_add(y[j], vals[j].at(o * cnt + 2 * q), vals[j].n, vals[j].p);
                        }
                    }, nt);
                    if (cnt % 2)
                        for (int j = 0; j < k; ++j)
                            for (i64 o = 0; o < Nout; ++o)
                                std::memcpy(nv[j].at(o * cnt1 + ops), vals[j].at(o * cnt + cnt - 1), sizeof(comp_t) * nv[j].n);
                    vals = std::move(nv);
                    put_relu_tables(g, arr_name("lv", static_cast<int>(lv), "."), t);
                }
                CrtLabels nxt;
                for (int j = 0; j < k; ++j) {
                    Labels O(crt_[j], Nout);
                    for (i64 o = 0; o < Nout; ++o) std::memcpy(O.at(o), vals[j].at(o), sizeof(comp_t) * O.n);
                    nxt.push_back(std::move(O));
                }
                g.p["levels"] = {static_cast<i64>(T.ops.size())};
                cur = std::move(nxt);
                break;
            }
            case K_SUMPOOL: {
                DASH_CHECK(is_crt(), "sum pool needs CRT-base labels");
                PoolGeom G(spec.p);
                DASH_CHECK(G.C * G.H * G.W == Nin, "sumpool input size mismatch");
                if (on_gpu) {
                    gpu->sumpool(G, cur);
                    dims = {G.C, G.OH, G.OW};
                    break;
                }
                CrtLabels nxt;
                std::vector<i64> w;
                for (int j = 0; j < k; ++j) {
                    Labels O(crt_[j], G.out_size());
                    for (i64 o = 0; o < G.out_size(); ++o) {
                        G.window(o, w);
                        std::memcpy(O.at(o), cur[j].at(w[0]), sizeof(comp_t) * O.n);
                        for (size_t s = 1; s < w.size(); ++s) lab_add(O.at(o), cur[j].at(w[s]), O.n, O.p);
                    }
                    nxt.push_back(std::move(O));
                }
                cur = std::move(nxt);
                dims = {G.C, G.OH, G.OW};
                break;
            }
            case K_ADD: {
                const i64 src = param1(spec.p, "src");
                DASH_CHECK(src >= -1 && src < static_cast<i64>(li), "add: bad source layer");
                if (on_gpu) {
                    gpu->add_saved(static_cast<size_t>(src + 1), cur);
                    break;
                }
                const CrtLabels& other = saved[src + 1];
                DASH_CHECK(!other.empty() && other[0].N == Nin, "add: operand size mismatch");
                for (int j = 0; j < k; ++j)
                    for (i64 e = 0; e < Nin; ++e) lab_add(cur[j].at(e), other[j].at(e), cur[j].n, cur[j].p);
                break;
            }
            case K_PROJ: {
                const auto& inm = paramv(spec.p, "in_mod");
                const auto& outm = paramv(spec.p, "out_mod");
                DASH_CHECK(static_cast<int>(inm.size()) == k && static_cast<int>(outm.size()) == k, "projection moduli");
                CrtLabels nxt;
                for (int j = 0; j < k; ++j) {
                    DASH_CHECK(cur_mod[j] == inm[j], "projection input modulus mismatch");
                    nxt.emplace_back(static_cast<int>(outm[j]), Nin);
                }
                std::vector<Array> tabs;
                for (int j = 0; j < k; ++j) tabs.emplace_back(DType::u128, std::vector<i64>{Nin, inm[j]});
                parallel_for(Nin, [&](i64 b0, i64 b1) {
                    for (i64 e = b0; e < b1; ++e) {
                        u64 ctr = 0;
                        for (int j = 0; j < k; ++j) {
                            const ModInfo& mi = mod_info(static_cast<int>(inm[j]));
                            const ModInfo& mo = mod_info(static_cast<int>(outm[j]));
                            const auto& fn = paramv(spec.p, ("fn." + std::to_string(j)).c_str());
                            prg_.label(stream_id(L, 1, e), ctr, mo.p, mo.n, nxt[j].at(e));
                            garble_proj(cur[j].at(e), R_.get(mi.p), mi, nxt[j].at(e), R_.get(mo.p), mo,
                                        [&fn](int v) { return fn[v]; }, tabs[j].ptr<u128>() + e * mi.p, 1,
                                        Mask{hard, stream_id(L, 1, e), tw_sub(TW_PROJ, j), 0});
                        }
                    }
                }, nt);
                for (int j = 0; j < k; ++j) {
                    g.a[arr_name("t.", j, "")] = tabs[j];
                    cur_mod[j] = static_cast<int>(outm[j]);
                }
                cur = std::move(nxt);
                break;
            }
            case K_MULT: {
                DASH_CHECK(is_crt() && Nin % 2 == 0, "mult layer needs an even number of CRT inputs");
                const i64 No = Nin / 2;
                Array ga(DType::u128, {No, sum_crt}), ea(DType::u128, {No, sum_crt});
                CrtLabels nxt;
                for (int j = 0; j < k; ++j) nxt.emplace_back(crt_[j], No);
                parallel_for(No, [&](i64 b0, i64 b1) {
                    for (i64 e = b0; e < b1; ++e) {
                        u64 ctr = 0;
                        for (int j = 0; j < k; ++j)
                            gen_mult_garble(cur[j].at(2 * e), cur[j].at(2 * e + 1), mod_info(crt_[j]), R_, prg_,
                                            stream_id(L, 1, e), ctr, ga.ptr<u128>() + e * sum_crt + prefix[j],
                                            ea.ptr<u128>() + e * sum_crt + prefix[j], nxt[j].at(e), hard, j);
                    }
                }, nt);
                g.a["g"] = ga;
                g.a["e"] = ea;
                cur = std::move(nxt);
                dims = {No};
                break;
            }
            case K_MMULT: {
                DASH_CHECK(is_crt() && Nin % 2 == 0, "mixed mult layer needs an even number of CRT inputs");
                const int q = static_cast<int>(param1(spec.p, "q"));
                const i64 No = Nin / 2;
                Array ta(DType::u128, {No, sum_crt}), ga(DType::u128, {No, sum_crt}),
                    ea(DType::u128, {No, static_cast<i64>(k), static_cast<i64>(q + 1)});
                CrtLabels nxt;
                for (int j = 0; j < k; ++j) nxt.emplace_back(crt_[j], No);
                const ModInfo& mq = mod_info(q);
                parallel_for(No, [&](i64 b0, i64 b1) {
                    std::vector<comp_t> t0(mq.n);
                    for (i64 e = b0; e < b1; ++e) {
                        u64 ctr = 0;
                        for (int j = 0; j < k; ++j) {
                            const ModInfo& mp = mod_info(crt_[j]);
                            prg_.label(stream_id(L, 1, e), ctr, q, mq.n, t0.data());
                            garble_proj(cur[j].at(2 * e + 1), R_.get(mp.p), mp, t0.data(), R_.get(q), mq,
                                        [](int v) { return static_cast<i64>(v); }, ta.ptr<u128>() + e * sum_crt + prefix[j],
                                        1, Mask{hard, stream_id(L, 1, e), tw_sub(TW_MMT, j), 0});
                            mixed_mult_garble(cur[j].at(2 * e), mp, t0.data(), mq, R_, prg_, stream_id(L, 1, e), ctr,
                                              ga.ptr<u128>() + e * sum_crt + prefix[j],
                                              ea.ptr<u128>() + (e * k + j) * (q + 1), nxt[j].at(e),
                                              MMTw{hard, stream_id(L, 1, e), j, k, false});
                        }
                    }
                }, nt);
                g.a["t"] = ta;
                g.a["g"] = ga;
                g.a["e"] = ea;
                cur = std::move(nxt);
                dims = {No};
                break;
            }
            case K_BASEEXT: {
                DASH_CHECK(is_crt(), "base extension needs CRT-base labels");
                std::vector<int> ext;
                for (auto v : paramv(spec.p, "extra")) ext.push_back(static_cast<int>(v));
                BEPlan P(crt_, ext);
                Array be(DType::u128, {Nin, P.n_tab});
                if (on_gpu) {
                    sinkify(be, "be");
                    gpu->base_ext(L, P, cur, be);
                    g.a["be"] = be;
                    break;
                }
                parallel_for(Nin, [&](i64 b0, i64 b1) {
                    std::vector<comp_t*> Lp(k);
                    for (i64 e = b0; e < b1; ++e) {
                        for (int j = 0; j < k; ++j) Lp[j] = cur[j].at(e);
                        for (int xi : P.extra_idx)
                            std::memcpy(Lp[xi], Z_.get(crt_[xi]), sizeof(comp_t) * nr_comps(crt_[xi]));
                        u64 ctr = 0;
                        be_garble_elem(P, R_, prg_, stream_id(L, 1, e), ctr, Lp.data(), be.ptr<u128>() + e * P.n_tab,
                                       hard);
                    }
                }, nt);
                g.a["be"] = be;
                break;
            }
            default:
                throw std::runtime_error(std::string("dash: cannot garble layer kind ") + std::to_string(spec.kind));
        }
        if (on_gpu) host_ok = false;
        else if (!passthru) dev_ok = false;
        if (keep[li + 1]) {
            if (gpu) {
                if (!dev_ok) {
                    gpu->to_device(cur);
                    dev_ok = true;
                }
                gpu->save(li + 1);
            } else {
                saved[li + 1] = cur;
            }
            saved_mod[li + 1] = cur_mod;
            saved_dims[li + 1] = dims;
        }
        m.layers.push_back(std::move(g));
        layer_ms_[li] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_layer).count();
    }

    if (!host_ok) gpu->to_host(cur);
    // Decoding information (reference gci.h:386-415)
    dec_ = Decoder();
    dec_.moduli = cur_mod;
    dec_.n_out = cur[0].N;
    for (int j = 0; j < k; ++j) {
        const int q = cur_mod[j];
        const ModInfo& mq = mod_info(q);
        Array d(DType::u128, {q, dec_.n_out});
        parallel_for(q, [&](i64 v0, i64 v1) {
            std::vector<comp_t> tmp(mq.n);
            for (i64 v = v0; v < v1; ++v)
                for (i64 e = 0; e < dec_.n_out; ++e) {
                    lab_affine(tmp.data(), cur[j].at(e), v, R_.get(q), mq.n, q);
                    d.ptr<u128>()[v * dec_.n_out + e] = hash(compress(tmp.data(), mq));
                }
        }, nt);
        dec_.dec.push_back(d);
    }
    m.h.out_dims = dims;
    m.h.out_moduli = cur_mod;
    return m;
}

}  // namespace dash
