// Host (oracle) evaluator and decoder. Bit-exact with the HIP evaluator; the
// CPU path of the reference (gci.h:345-380 + every GarbledX::cpu_evaluate).
#include <chrono>
#include "layers.h"

namespace dash {

LabelBank GarbledModel::zero_bank() const {
    LabelBank Z;
    Z.max_mod = h.max_mod;
    Z.lab.assign(h.max_mod + 1, {});
    if (h.hardened) {  // public zero wires have label 0 (docs/SECURITY.md)
        for (int p = 2; p <= h.max_mod; ++p) Z.lab[p].assign(nr_comps(p), 0);
        return Z;
    }
    for (const auto& kv : consts) {
        if (kv.first.rfind("Z.", 0) != 0) continue;
        int p = std::stoi(kv.first.substr(2));
        if (p > h.max_mod) continue;
        const Array& a = kv.second;
        Z.lab[p].assign(a.ptr<comp_t>(), a.ptr<comp_t>() + a.count());
    }
    return Z;
}

size_t GarbledModel::table_bytes() const {
    size_t b = 0;
    for (const auto& l : layers)
        for (const auto& kv : l.a)
            if (kv.second.dtype == DType::u128) b += kv.second.nbytes;
    return b;
}

size_t GarbledModel::total_bytes() const {
    size_t b = 0;
    for (const auto& l : layers)
        for (const auto& kv : l.a) b += kv.second.nbytes;
    for (const auto& kv : consts) b += kv.second.nbytes;
    return b;
}

namespace {

struct ReluTabs {
    const Array *ap, *c1, *c2, *sg, *ga, *ea;
    ReluTabs(const GLayer& g, const std::string& pre)
        : ap(&g.arr(pre + "s.approx")), c1(g.a.count(pre + "s.cast1") ? &g.arr(pre + "s.cast1") : nullptr),
          c2(&g.arr(pre + "s.cast2")),
          sg(&g.arr(pre + "s.sign")), ga(&g.arr(pre + "mm.g")), ea(&g.arr(pre + "mm.e")) {}
};

// s_gate / m_gate: the sign and mixed-mult gadgets' PRG streams (the hardened tweaks' gates)
void relu_eval_elem(const SignPlan& sp, const LabelBank& Z, const std::vector<int>& crt,
                    const std::vector<i64>& prefix, const comp_t* const* x, const ReluTabs& T, i64 e,
                    comp_t* const* out, bool hard, u64 s_gate, u64 m_gate, comp_t* sig_out = nullptr) {
    const int k = static_cast<int>(crt.size());
    comp_t sig[128];
    comp_t* outs[1] = {sig};
    sign_eval_elem(sp, Z, x, T.ap->ptr<u128>() + e * T.ap->shape[1],
                   T.c1 ? T.c1->ptr<u128>() + e * T.c1->shape[1] : nullptr,
                   T.c2->ptr<u128>() + e * T.c2->shape[1], T.sg->ptr<u128>() + e * T.sg->shape[1], outs, hard, s_gate);
    const ModInfo& m2 = mod_info(2);
    if (sig_out) std::memcpy(sig_out, sig, sizeof(comp_t) * m2.n);
    for (int j = 0; j < k; ++j)
        mixed_mult_eval(x[j], mod_info(crt[j]), sig, m2, T.ga->ptr<u128>() + e * T.ga->shape[1] + prefix[j],
                        T.ea->ptr<u128>() + (e * k + j) * 3, out[j], MMTw{hard, m_gate, j, k, true});
}

// a layer array that the hardened encoding does not ship (bias labels): all-zero rows of the same shape
const comp_t* zeros_or(const GLayer& g, const std::string& name, bool hard, size_t n, std::vector<comp_t>& buf) {
    if (!hard) return g.arr(name).ptr<comp_t>();
    buf.assign(n, 0);
    return buf.data();
}

}  // namespace

CrtLabels cpu_evaluate(const GarbledModel& m, const CrtLabels& inputs, int nt, std::vector<double>* layer_ms,
                       EvalTrace* trace) {
    const std::vector<int>& crt = m.h.crt;
    const int k = static_cast<int>(crt.size());
    DASH_CHECK(static_cast<int>(inputs.size()) == k, "input residue count mismatch");
    const LabelBank Z = m.zero_bank();
    const bool fused = m.h.sign_fused != 0;
    const bool hard = m.h.hardened != 0;
    std::vector<i64> prefix(k);
    i64 sum_crt = 0;
    for (int j = 0; j < k; ++j) {
        prefix[j] = sum_crt;
        sum_crt += crt[j];
    }
    std::vector<int> keep(m.layers.size() + 1, 0);
    for (const auto& l : m.layers) {
        if (l.kind == K_ADD) keep[l.param("src") + 1] = 1;
        if (l.p.count("in_src")) keep[l.param("in_src") + 1] = 1;
    }
    std::vector<CrtLabels> saved(m.layers.size() + 1);

    CrtLabels cur = inputs;
    if (keep[0]) saved[0] = cur;
    std::vector<comp_t> zero_const(128, 0);
    auto get_const = [&](const std::string& name) -> const comp_t* {
        if (hard) return zero_const.data();  // shift labels: public constants, label 0
        auto it = m.consts.find(name);
        DASH_CHECK(it != m.consts.end(), "missing model constant " + name);
        return it->second.ptr<comp_t>();
    };

    if (layer_ms) layer_ms->assign(m.layers.size(), 0.0);
    Labels sig_joint;  // sign labels a mixed-radix rescale with sign_out leaves for the next ReLU
    for (size_t li = 0; li < m.layers.size(); ++li) {
        const auto t_layer = std::chrono::steady_clock::now();
        const GLayer& g = m.layers[li];
        const u64 L = li + 1;  // the garbler's layer index (stream ids / hardened tweak gates)
        if (g.p.count("in_src")) cur = saved[g.param("in_src") + 1];
        const i64 Nin = cur[0].N;
        switch (g.kind) {
            case K_FLATTEN:
                break;
            case K_DENSE: {
                const i64 in = g.param("in"), out = g.param("out"), ch = g.param("channel_tf", 0);
                DASH_CHECK(in == Nin, "dense input size mismatch");
                const Array& wa = g.arr("w");
                CrtLabels nxt;
                for (int j = 0; j < k; ++j) {
                    const int p = crt[j];
                    const ModInfo& mi = mod_info(p);
                    const comp_t* Zp = Z.get(p);
                    std::vector<comp_t> zb;
                    const comp_t* bias = zeros_or(g, arr_name("bias.", j, ""), hard, static_cast<size_t>(out) * mi.n, zb);
                    Labels O(p, out);
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
                            const comp_t* bb = bias + o * mi.n;
                            for (int c = 0; c < mi.n; ++c) y[c] = static_cast<comp_t>((acc[c] + zc * Zp[c] + bb[c]) % p);
                        }
                    }, nt);
                    nxt.push_back(std::move(O));
                }
                cur = std::move(nxt);
                break;
            }
            case K_CONV: {
                ConvGeom G(g);
                DASH_CHECK(G.C * G.H * G.W == Nin, "conv input size mismatch");
                const Array& wa = g.arr("w");
                CrtLabels nxt;
                for (int j = 0; j < k; ++j) {
                    const int p = crt[j];
                    const ModInfo& mi = mod_info(p);
                    const comp_t* Zp = Z.get(p);
                    std::vector<comp_t> zb;
                    const comp_t* bias = zeros_or(g, arr_name("bias.", j, ""), hard, static_cast<size_t>(G.F) * mi.n, zb);
                    // weights reduced mod p once
                    std::vector<int32_t> wm(static_cast<size_t>(G.F * G.K()));
                    std::vector<i64> zc(G.F, 0);
                    for (i64 f = 0; f < G.F; ++f)
                        for (i64 q = 0; q < G.K(); ++q) {
                            wm[f * G.K() + q] = static_cast<int32_t>(wa.ptr<i64>()[f * G.K() + q] % p);
                            if (wm[f * G.K() + q] == 0) ++zc[f];
                        }
                    Labels O(p, G.out_size());
                    const Labels& I = cur[j];
                    parallel_for(G.out_size(), [&](i64 b0, i64 b1) {
                        std::vector<int32_t> acc(mi.n);
                        for (i64 o = b0; o < b1; ++o) {
                            const i64 f = o / (G.OH * G.OW), r = o % (G.OH * G.OW), oy = r / G.OW, ox = r % G.OW;
                            std::fill(acc.begin(), acc.end(), 0);
                            const int32_t* wf = wm.data() + f * G.K();
                            for (i64 c = 0; c < G.C; ++c)
                                for (i64 dy = 0; dy < G.kh; ++dy)
                                    for (i64 dx = 0; dx < G.kw; ++dx) {
                                        const int32_t wv = wf[(c * G.kh + dy) * G.kw + dx];
                                        if (wv == 0) continue;
                                        const i64 iy = oy * G.sh - G.ph + dy, ix = ox * G.sw - G.pw + dx;
                                        const comp_t* x = (iy < 0 || iy >= G.H || ix < 0 || ix >= G.W)
                                                              ? Zp
                                                              : I.at((c * G.H + iy) * G.W + ix);
                                        for (int cc = 0; cc < mi.n; ++cc) acc[cc] += wv * x[cc];
                                    }
                            comp_t* y = O.at(o);
                            const comp_t* bb = bias + f * mi.n;
                            for (int cc = 0; cc < mi.n; ++cc)
                                y[cc] = static_cast<comp_t>((acc[cc] + zc[f] * Zp[cc] + bb[cc]) % p);
                        }
                    }, nt);
                    nxt.push_back(std::move(O));
                }
                cur = std::move(nxt);
                break;
            }
            case K_RELU: {
                if (trace) trace->relu_in[li] = cur;
                if (g.param("smode", 0) == 2) {  // sign from the preceding rescale (RescaleMrsPlan::sign_last)
                    DASH_CHECK(sig_joint.N == Nin, "joint ReLU without a preceding sign-producing rescale");
                    if (trace) trace->relu_sign[li] = sig_joint;
                    const Array& tg = g.arr("mm.g");
                    const Array& te = g.arr("mm.e");
                    CrtLabels nxt;
                    for (int j = 0; j < k; ++j) nxt.emplace_back(crt[j], Nin);
                    parallel_for(Nin, [&](i64 b0, i64 b1) {
                        const ModInfo& m2 = mod_info(2);
                        for (i64 e = b0; e < b1; ++e)
                            for (int j = 0; j < k; ++j)
                                mixed_mult_eval(cur[j].at(e), mod_info(crt[j]), sig_joint.at(e), m2,
                                                tg.ptr<u128>() + e * tg.shape[1] + prefix[j],
                                                te.ptr<u128>() + (e * k + j) * 3, nxt[j].at(e),
                                                MMTw{hard, stream_id(L, 2, e), j, k, true});
                    }, nt);
                    cur = std::move(nxt);
                    sig_joint = Labels();
                    break;
                }
                if (g.param("smode", 0) == 1) {  // exact mixed-radix sign (SignMrsPlan)
                    const SignMrsPlan sp(crt);
                    const Array& tab = g.arr("mrs");
                    const Array& tg = g.arr("mm.g");
                    const Array& te = g.arr("mm.e");
                    CrtLabels nxt;
                    for (int j = 0; j < k; ++j) nxt.emplace_back(crt[j], Nin);
                    Labels sigs(2, trace ? Nin : 0);
                    parallel_for(Nin, [&](i64 b0, i64 b1) {
                        std::vector<const comp_t*> x(k);
                        comp_t sig[128];
                        const ModInfo& m2 = mod_info(2);
                        for (i64 e = b0; e < b1; ++e) {
                            for (int j = 0; j < k; ++j) x[j] = cur[j].at(e);
                            sign_mrs_eval_elem(sp, x.data(), tab.ptr<u128>() + e * tab.shape[1], sig, hard,
                                               stream_id(L, 1, e));
                            if (trace) std::memcpy(sigs.at(e), sig, sizeof(comp_t) * m2.n);
                            for (int j = 0; j < k; ++j)
                                mixed_mult_eval(x[j], mod_info(crt[j]), sig, m2, tg.ptr<u128>() + e * tg.shape[1] + prefix[j],
                                                te.ptr<u128>() + (e * k + j) * 3, nxt[j].at(e),
                                                MMTw{hard, stream_id(L, 2, e), j, k, true});
                        }
                    }, nt);
                    if (trace) trace->relu_sign[li] = std::move(sigs);
                    cur = std::move(nxt);
                    break;
                }
                SignPlan sp(crt, m.h.mrs, {2}, 0, 1, fused);
                const ReluTabs T(g, "");
                CrtLabels nxt;
                for (int j = 0; j < k; ++j) nxt.emplace_back(crt[j], Nin);
                Labels sigs(2, trace ? Nin : 0);
                parallel_for(Nin, [&](i64 b0, i64 b1) {
                    std::vector<const comp_t*> x(k);
                    std::vector<comp_t*> y(k);
                    for (i64 e = b0; e < b1; ++e) {
                        for (int j = 0; j < k; ++j) {
                            x[j] = cur[j].at(e);
                            y[j] = nxt[j].at(e);
                        }
                        relu_eval_elem(sp, Z, crt, prefix, x.data(), T, e, y.data(), hard, stream_id(L, 1, e),
                                       stream_id(L, 2, e), trace ? sigs.at(e) : nullptr);
                    }
                }, nt);
                if (trace) trace->relu_sign[li] = std::move(sigs);
                cur = std::move(nxt);
                break;
            }
            case K_SIGN: {
                SignPlan sp(crt, m.h.mrs, crt, -1, 1, fused);
                const Array& ap = g.arr("s.approx");
                const Array* c1 = sp.has_cast1() ? &g.arr("s.cast1") : nullptr;
                const Array& c2 = g.arr("s.cast2");
                const Array& sg = g.arr("s.sign");
                CrtLabels nxt;
                for (int j = 0; j < k; ++j) nxt.emplace_back(crt[j], Nin);
                parallel_for(Nin, [&](i64 b0, i64 b1) {
                    std::vector<const comp_t*> x(k);
                    std::vector<comp_t*> y(k);
                    for (i64 e = b0; e < b1; ++e) {
                        for (int j = 0; j < k; ++j) {
                            x[j] = cur[j].at(e);
                            y[j] = nxt[j].at(e);
                        }
                        sign_eval_elem(sp, Z, x.data(), ap.ptr<u128>() + e * ap.shape[1],
                                       c1 ? c1->ptr<u128>() + e * c1->shape[1] : nullptr,
                                       c2.ptr<u128>() + e * c2.shape[1], sg.ptr<u128>() + e * sg.shape[1], y.data(),
                                       hard, stream_id(L, 1, e));
                    }
                }, nt);
                cur = std::move(nxt);
                break;
            }
            case K_RESCALE: {
                const i64 mode = g.param("mode", 0);
                if (mode == 2) {  // mixed-radix construction of the legacy function
                    const bool so = g.param("sign_out", 0) == 1;
                    const RescaleMrsPlan P(crt, static_cast<int>(g.param("l")), so);
                    const Array& tab = g.arr("mrs");
                    DASH_CHECK(tab.shape[1] == P.n_tab, "mixed-radix rescale table shape");
                    if (so) sig_joint = Labels(2, Nin);
                    parallel_for(Nin, [&](i64 b0, i64 b1) {
                        std::vector<comp_t*> Lp(k);
                        for (i64 e = b0; e < b1; ++e) {
                            for (int j = 0; j < k; ++j) Lp[j] = cur[j].at(e);
                            rescale_mrs_eval_elem(P, Lp.data(), tab.ptr<u128>() + e * P.n_tab,
                                                  so ? sig_joint.at(e) : nullptr, hard, stream_id(L, 30, e));
                        }
                    }, nt);
                    break;
                }
                DASH_CHECK(mode == 0 || mode == 1, "unknown rescale mode " + std::to_string(mode));
                const i64 iters = g.param("iters");
                std::vector<RescalePlan> plans;
                if (mode == 0) {
                    for (i64 i = 0; i < iters; ++i) plans.emplace_back(crt, m.h.mrs, std::vector<int>{2}, true, fused);
                } else {
                    std::vector<int> s;
                    for (auto v : g.vec("s")) s.push_back(static_cast<int>(v));
                    plans.emplace_back(crt, m.h.mrs, s, false, fused);
                }
                std::vector<const comp_t*> up(k), dn(k);
                for (int j = 0; j < k; ++j) up[j] = get_const("up." + std::to_string(j));
                for (size_t it = 0; it < plans.size(); ++it) {
                    const RescalePlan& P = plans[it];
                    for (int j = 0; j < k; ++j)
                        dn[j] = get_const("down." + std::to_string(P.sprod) + "." + std::to_string(j));
                    const std::string pre = arr_name("it", static_cast<int>(it), ".");
                    const Array& tr = g.arr(pre + "trans");
                    const Array* ap = nullptr, *c1 = nullptr, *c2 = nullptr, *sg = nullptr, *be = nullptr;
                    if (P.sign_be) {
                        ap = &g.arr(pre + "s.approx");
                        c1 = P.sign.has_cast1() ? &g.arr(pre + "s.cast1") : nullptr;
                        c2 = &g.arr(pre + "s.cast2");
                        sg = &g.arr(pre + "s.sign");
                    } else {
                        be = &g.arr(pre + "be");
                    }
                    parallel_for(Nin, [&](i64 b0, i64 b1) {
                        std::vector<comp_t*> Lp(k);
                        for (i64 e = b0; e < b1; ++e) {
                            for (int j = 0; j < k; ++j) Lp[j] = cur[j].at(e);
                            if (P.sign_be)
                                rescale_eval_elem(P, Z, Lp.data(), up.data(), dn.data(), tr.ptr<u128>() + e * P.n_trans,
                                                  ap->ptr<u128>() + e * ap->shape[1],
                                                  c1 ? c1->ptr<u128>() + e * c1->shape[1] : nullptr,
                                                  c2->ptr<u128>() + e * c2->shape[1], sg->ptr<u128>() + e * sg->shape[1],
                                                  nullptr, hard, stream_id(L, 10 + it, e));
                            else
                                rescale_eval_elem(P, Z, Lp.data(), up.data(), dn.data(), tr.ptr<u128>() + e * P.n_trans,
                                                  nullptr, nullptr, nullptr, nullptr, be->ptr<u128>() + e * P.n_be, hard,
                                                  stream_id(L, 10 + it, e));
                        }
                    }, nt);
                }
                break;
            }
            case K_MAXPOOL:
            case K_MAX: {
                i64 Nout, K;
                std::vector<std::vector<i64>> win;
                if (g.kind == K_MAXPOOL) {
                    PoolGeom G(g.p);
                    Nout = G.out_size();
                    K = G.kh * G.kw;
                    win.resize(Nout);
                    for (i64 o = 0; o < Nout; ++o) G.window(o, win[o]);
                } else {
                    Nout = 1;
                    K = Nin;
                    win.resize(1);
                    for (i64 i = 0; i < Nin; ++i) win[0].push_back(i);
                }
                MaxTree T(K);
                SignPlan sp(crt, m.h.mrs, {2}, 0, 1, fused);
                std::vector<Labels> vals;
                for (int j = 0; j < k; ++j) {
                    Labels V(crt[j], Nout * K);
                    for (i64 o = 0; o < Nout; ++o)
                        for (i64 s = 0; s < K; ++s) std::memcpy(V.at(o * K + s), cur[j].at(win[o][s]), sizeof(comp_t) * V.n);
                    vals.push_back(std::move(V));
                }
                for (size_t lv = 0; lv < T.ops.size(); ++lv) {
                    const i64 ops = T.ops[lv], cnt = T.cnt[lv], cnt1 = T.cnt[lv + 1];
                    const std::string pre = arr_name("lv", static_cast<int>(lv), ".");
                    std::vector<Labels> nv;
                    for (int j = 0; j < k; ++j) nv.emplace_back(crt[j], Nout * cnt1);
                    const ReluTabs T(g, pre);
                    parallel_for(Nout * ops, [&](i64 b0, i64 b1) {
                        std::vector<std::vector<comp_t>> diff(k);
                        std::vector<const comp_t*> x(k);
                        std::vector<comp_t*> y(k);
                        for (int j = 0; j < k; ++j) diff[j].resize(nr_comps(crt[j]));
                        for (i64 e = b0; e < b1; ++e) {
                            const i64 o = e / ops, q = e % ops;
                            for (int j = 0; j < k; ++j) {
                                const int n = vals[j].n, p = vals[j].p;
                                std::memcpy(diff[j].data(), vals[j].at(o * cnt + 2 * q + 1), sizeof(comp_t) * n);
                                lab_sub(diff[j].data(), vals[j].at(o * cnt + 2 * q), n, p);
                                x[j] = diff[j].data();
                                y[j] = nv[j].at(o * cnt1 + q);
                            }
                            relu_eval_elem(sp, Z, crt, prefix, x.data(), T, e, y.data(), hard,
                                           stream_id(L, 20 + 2 * lv, e), stream_id(L, 21 + 2 * lv, e));
                            for (int j = 0; j < k; ++j) lab_add(y[j], vals[j].at(o * cnt + 2 * q), vals[j].n, vals[j].p);
                        }
                    }, nt);
                    if (cnt % 2)
                        for (int j = 0; j < k; ++j)
                            for (i64 o = 0; o < Nout; ++o)
                                std::memcpy(nv[j].at(o * cnt1 + ops), vals[j].at(o * cnt + cnt - 1), sizeof(comp_t) * nv[j].n);
                    vals = std::move(nv);
                }
                CrtLabels nxt;
                for (int j = 0; j < k; ++j) {
                    Labels O(crt[j], Nout);
                    for (i64 o = 0; o < Nout; ++o) std::memcpy(O.at(o), vals[j].at(o), sizeof(comp_t) * O.n);
                    nxt.push_back(std::move(O));
                }
                cur = std::move(nxt);
                break;
            }
            case K_SUMPOOL: {
                PoolGeom G(g.p);
                CrtLabels nxt;
                std::vector<i64> w;
                for (int j = 0; j < k; ++j) {
                    Labels O(crt[j], G.out_size());
                    for (i64 o = 0; o < G.out_size(); ++o) {
                        G.window(o, w);
                        std::memcpy(O.at(o), cur[j].at(w[0]), sizeof(comp_t) * O.n);
                        for (size_t s = 1; s < w.size(); ++s) lab_add(O.at(o), cur[j].at(w[s]), O.n, O.p);
                    }
                    nxt.push_back(std::move(O));
                }
                cur = std::move(nxt);
                break;
            }
            case K_ADD: {
                const CrtLabels& other = saved[g.param("src") + 1];
                DASH_CHECK(!other.empty() && other[0].N == Nin, "add: operand size mismatch");
                for (int j = 0; j < k; ++j)
                    for (i64 e = 0; e < Nin; ++e) lab_add(cur[j].at(e), other[j].at(e), cur[j].n, cur[j].p);
                break;
            }
            case K_PROJ: {
                const auto& inm = g.vec("in_mod");
                const auto& outm = g.vec("out_mod");
                CrtLabels nxt;
                for (int j = 0; j < k; ++j) nxt.emplace_back(static_cast<int>(outm[j]), Nin);
                parallel_for(Nin, [&](i64 b0, i64 b1) {
                    for (i64 e = b0; e < b1; ++e)
                        for (int j = 0; j < k; ++j) {
                            const ModInfo& mi = mod_info(static_cast<int>(inm[j]));
                            eval_proj(cur[j].at(e), mi, g.arr(arr_name("t.", j, "")).ptr<u128>() + e * mi.p,
                                      mod_info(static_cast<int>(outm[j])), nxt[j].at(e), 1,
                                      Mask{hard, stream_id(L, 1, e), tw_sub(TW_PROJ, j), 0});
                        }
                }, nt);
                cur = std::move(nxt);
                break;
            }
            case K_MULT: {
                const i64 No = Nin / 2;
                const Array& ga = g.arr("g");
                const Array& ea = g.arr("e");
                CrtLabels nxt;
                for (int j = 0; j < k; ++j) nxt.emplace_back(crt[j], No);
                parallel_for(No, [&](i64 b0, i64 b1) {
                    for (i64 e = b0; e < b1; ++e)
                        for (int j = 0; j < k; ++j)
                            gen_mult_eval(cur[j].at(2 * e), cur[j].at(2 * e + 1), mod_info(crt[j]),
                                          ga.ptr<u128>() + e * sum_crt + prefix[j], ea.ptr<u128>() + e * sum_crt + prefix[j],
                                          nxt[j].at(e), hard, stream_id(L, 1, e), j);
                }, nt);
                cur = std::move(nxt);
                break;
            }
            case K_MMULT: {
                const int q = static_cast<int>(g.param("q"));
                const i64 No = Nin / 2;
                const Array& ta = g.arr("t");
                const Array& ga = g.arr("g");
                const Array& ea = g.arr("e");
                const ModInfo& mq = mod_info(q);
                CrtLabels nxt;
                for (int j = 0; j < k; ++j) nxt.emplace_back(crt[j], No);
                parallel_for(No, [&](i64 b0, i64 b1) {
                    std::vector<comp_t> t0(mq.n);
                    for (i64 e = b0; e < b1; ++e)
                        for (int j = 0; j < k; ++j) {
                            const ModInfo& mp = mod_info(crt[j]);
                            eval_proj(cur[j].at(2 * e + 1), mp, ta.ptr<u128>() + e * sum_crt + prefix[j], mq, t0.data(),
                                      1, Mask{hard, stream_id(L, 1, e), tw_sub(TW_MMT, j), 0});
                            mixed_mult_eval(cur[j].at(2 * e), mp, t0.data(), mq, ga.ptr<u128>() + e * sum_crt + prefix[j],
                                            ea.ptr<u128>() + (e * k + j) * (q + 1), nxt[j].at(e),
                                            MMTw{hard, stream_id(L, 1, e), j, k, false});
                        }
                }, nt);
                cur = std::move(nxt);
                break;
            }
            case K_BASEEXT: {
                std::vector<int> ext;
                for (auto v : g.vec("extra")) ext.push_back(static_cast<int>(v));
                BEPlan P(crt, ext);
                const Array& be = g.arr("be");
                parallel_for(Nin, [&](i64 b0, i64 b1) {
                    std::vector<comp_t*> Lp(k);
                    for (i64 e = b0; e < b1; ++e) {
                        for (int j = 0; j < k; ++j) Lp[j] = cur[j].at(e);
                        for (int xi : P.extra_idx) std::memcpy(Lp[xi], Z.get(crt[xi]), sizeof(comp_t) * nr_comps(crt[xi]));
                        be_eval_elem(P, Lp.data(), be.ptr<u128>() + e * P.n_tab, hard, stream_id(L, 1, e));
                    }
                }, nt);
                break;
            }
            default:
                throw std::runtime_error("dash: cannot evaluate layer kind " + std::to_string(g.kind));
        }
        if (keep[li + 1]) saved[li + 1] = cur;
        if (layer_ms)
            (*layer_ms)[li] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_layer).count();
    }
    return cur;
}

// ---------------------------------------------------------------------------
namespace {
// h(j, e) -> hash of output label e of residue j
template <class HashOf>
std::vector<i64> decode_with(const Decoder& d, HashOf&& hash_of) {
    const int k = static_cast<int>(d.moduli.size());
    const i64 n_out = d.n_out;
    std::vector<i64> res(static_cast<size_t>(k) * n_out, -1);
    for (int j = 0; j < k; ++j) {
        const int q = d.moduli[j];
        const u128* D = d.dec[j].ptr<u128>();
        for (i64 e = 0; e < n_out; ++e) {
            const u128 h = hash_of(j, e);
            i64 found = -1;
            for (int v = 0; v < q; ++v)
                if (D[static_cast<i64>(v) * n_out + e] == h) {
                    found = v;
                    break;
                }
            if (found < 0)
                throw std::runtime_error("dash integrity: output label " + std::to_string(e) + " of residue mod " +
                                         std::to_string(q) + " matches no decoding entry");
            res[static_cast<size_t>(j) * n_out + e] = found;
        }
    }
    return res;
}

std::vector<i64> crt_combine(const std::vector<int>& moduli, i64 n_out, const std::vector<i64>& r) {
    const int k = static_cast<int>(moduli.size());
    u128 M = 1;
    for (int q : moduli) M *= static_cast<u128>(q);
    std::vector<i64> val(n_out);
    for (i64 e = 0; e < n_out; ++e) {
        u128 sum = 0;
        for (int j = 0; j < k; ++j) {
            const u128 q = static_cast<u128>(moduli[j]);
            const u128 P = M / q;
            const u128 inv = static_cast<u128>(mul_inv(P % q, static_cast<i64>(q)));
            const u128 t = (static_cast<u128>(r[static_cast<size_t>(j) * n_out + e]) * inv) % q;
            sum = (sum + t * P) % M;
        }
        i64 v = static_cast<i64>(sum);
        if (sum >= M / 2) v = static_cast<i64>(sum) - static_cast<i64>(M);
        val[e] = v;
    }
    return val;
}
}  // namespace

std::vector<i64> Decoder::decode_residues(const CrtLabels& out) const {
    const int k = static_cast<int>(moduli.size());
    DASH_CHECK(static_cast<int>(out.size()) == k, "decode: residue count mismatch");
    for (int j = 0; j < k; ++j)
        DASH_CHECK(out[j].N == n_out && out[j].p == moduli[j], "decode: output label shape mismatch");
    return decode_with(*this, [&](int j, i64 e) { return hash(compress(out[j].at(e), mod_info(moduli[j]))); });
}

std::vector<i64> Decoder::decode_residues_compressed(const u128* C) const {
    return decode_with(*this, [&](int j, i64 e) { return hash(C[static_cast<i64>(j) * n_out + e]); });
}

std::vector<i64> Decoder::decode_compressed(const u128* C) const {
    return crt_combine(moduli, n_out, decode_residues_compressed(C));
}

std::vector<i64> Decoder::decode(const CrtLabels& out) const {
    return crt_combine(moduli, n_out, decode_residues(out));
}

}  // namespace dash
