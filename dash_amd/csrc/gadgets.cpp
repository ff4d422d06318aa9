// Gadget implementations (see gadgets.h for the reference map).
#include "gadgets.h"

namespace dash {

ProjScratch& proj_scratch() {
    thread_local ProjScratch s;
    return s;
}
ProjKeys& proj_keys_scratch() {
    thread_local ProjKeys k;
    return k;
}

namespace {
struct LabelScratch {
    std::vector<comp_t> buf;
    comp_t* get(size_t n) {
        if (buf.size() < n) buf.resize(n);
        return buf.data();
    }
};
LabelScratch& sign_scratch() {
    thread_local LabelScratch s;
    return s;
}
LabelScratch& misc_scratch() {
    thread_local LabelScratch s;
    return s;
}
LabelScratch& be_scratch() {
    thread_local LabelScratch s;
    return s;
}
LabelScratch& rescale_scratch() {
    thread_local LabelScratch s;
    return s;
}
inline void draw(const Prg& prg, u64 stream, u64& ctr, int p, comp_t* out) { prg.label(stream, ctr, p, nr_comps(p), out); }
inline i64 prod_ll(const std::vector<int>& v) {
    i64 r = 1;
    for (int x : v) r *= x;
    return r;
}
}  // namespace

// ---------------------------------------------------------------------------
// Lookup table for the approximate residues: value j of residue i maps to the
// mixed-radix digits of round(frac(alpha_i * j / M) * D), D = prod(mrs).
// Floating point steps mirror the reference so tables agree bit for bit.
std::vector<std::vector<int16_t>> gen_approx_lookup(const std::vector<int>& crt, const std::vector<int>& mrs) {
    const int t = static_cast<int>(mrs.size());
    const long D = prod_ll(mrs);
    const long pk = prod_ll(crt);
    std::vector<std::vector<int16_t>> out(crt.size());
    for (size_t i = 0; i < crt.size(); ++i) {
        const int p = crt[i];
        out[i].assign(static_cast<size_t>(p) * t, 0);
        long double A = static_cast<long double>(pk / p);
        long double alpha = A * static_cast<long double>(mul_inv(static_cast<u128>(static_cast<long long>(A)), p));
        for (int j = 0; j < p; ++j) {
            long double d = alpha * j / pk;
            double dd = static_cast<double>(d);
            dd = std::round(dd * static_cast<double>(D)) / static_cast<double>(D);
            d = static_cast<long double>(dd) * D;
            uint32_t dec = static_cast<uint32_t>(std::round(d));
            for (int q = t - 1; q >= 0; --q) {
                out[i][static_cast<size_t>(j) * t + q] = static_cast<int16_t>(dec % static_cast<uint32_t>(mrs[q]));
                dec /= static_cast<uint32_t>(mrs[q]);
            }
        }
    }
    return out;
}

SignPlan::SignPlan(const std::vector<int>& crt_, const std::vector<int>& mrs_, const std::vector<int>& out, int lo,
                   int up, bool fused_)
    : crt(crt_), mrs(mrs_), out_mod(out), lower(lo), upper(up), fused(fused_) {
    DASH_CHECK(!mrs.empty(), "sign gadget needs a non-empty MRS base");
    DASH_CHECK(mrs[0] % 2 == 0, "sign gadget needs an even most-significant MRS modulus");
    lookup = gen_approx_lookup(crt, mrs);
    const int k = static_cast<int>(crt.size()), t = static_cast<int>(mrs.size());
    crt_prefix.resize(k);
    for (int j = 0; j < k; ++j) {
        crt_prefix[j] = sum_crt;
        sum_crt += crt[j];
    }
    i64 tail = 0;
    for (int d = 1; d < t; ++d) tail += mrs[d];
    n_approx = t * sum_crt;
    n_cast = (k + 1) * tail;
    n_sign = static_cast<i64>(out.size()) * mrs[0];
    max_n = 0;
    for (int p : crt) max_n = std::max(max_n, nr_comps(p));
    for (int m : mrs) max_n = std::max(max_n, nr_comps(m));
    for (int d = 1; d < t; ++d) max_n = std::max(max_n, nr_comps((k + 1) * mrs[d]));
    for (int o : out) max_n = std::max(max_n, nr_comps(o));
}

namespace {
// Fused construction (SignPlan::fused, see gadgets.h). PRG draw order: the
// k*t digit labels (residue-major, modulus digit_mod(d)), then per digit
// d = t-1..1 the carry label (modulus carry_mod(d)), then the outputs.
void sign_garble_fused(const SignPlan& P, const LabelBank& R, const Prg& prg, u64 stream, const comp_t* const* in0,
                       u128* approx, u128* cast2, u128* sign, comp_t* const* out0, bool hard) {
    const int k = static_cast<int>(P.crt.size()), t = static_cast<int>(P.mrs.size());
    const int W = P.max_n;
    comp_t* base = sign_scratch().get(static_cast<size_t>(W) * (k * t + 3));
    comp_t* dig = base;                                    // [k*t][W]
    comp_t* carry = dig + static_cast<size_t>(W) * k * t;  // carry into the current digit
    comp_t* sum = carry + W;
    comp_t* newc = sum + W;
    u64 ctr = 0;
    for (int j = 0; j < k; ++j)
        for (int d = 0; d < t; ++d) draw(prg, stream, ctr, P.digit_mod(d), dig + static_cast<size_t>(W) * (j * t + d));
    ProjKeys& K = proj_keys_scratch();
    for (int j = 0; j < k; ++j) {
        const ModInfo& mi = mod_info(P.crt[j]);
        const auto& lut = P.lookup[j];
        proj_keys(in0[j], R.get(mi.p), mi, K, hard);
        for (int d = 0; d < t; ++d) {
            const ModInfo& mo = mod_info(P.digit_mod(d));
            garble_proj_keys(K, dig + static_cast<size_t>(W) * (j * t + d), R.get(mo.p), mo,
                             [&](int v) { return static_cast<i64>(lut[static_cast<size_t>(v) * t + d]); },
                             approx + t * P.crt_prefix[j] + d, t, Mask{hard, stream, tw_sub(TW_APPROX, j), d});
        }
    }
    bool have_carry = false;
    i64 c2 = 0;
    for (int d = t - 1; d >= 1; --d) {
        const int m = P.mrs[d], mprev = P.mrs[d - 1];
        const ModInfo& mo = mod_info(P.digit_mod(d));
        if (have_carry) std::memcpy(sum, carry, sizeof(comp_t) * mo.n);
        else std::memcpy(sum, dig + static_cast<size_t>(W) * d, sizeof(comp_t) * mo.n);
        for (int j = have_carry ? 0 : 1; j < k; ++j) lab_add(sum, dig + static_cast<size_t>(W) * (j * t + d), mo.n, mo.p);
        const ModInfo& mn = mod_info(P.carry_mod(d));
        draw(prg, stream, ctr, mn.p, newc);
        garble_proj(sum, R.get(mo.p), mo, newc, R.get(mn.p), mn,
                    [m, mprev](int v) { return static_cast<i64>((v / m) % mprev); }, cast2 + c2, 1,
                    Mask{hard, stream, tw_sub(TW_CAST2, d), 0});
        c2 += mo.p;
        std::memcpy(carry, newc, sizeof(comp_t) * mn.n);
        have_carry = true;
    }
    const ModInfo& m0 = mod_info(P.mrs[0]);
    if (have_carry) std::memcpy(sum, carry, sizeof(comp_t) * m0.n);
    else std::memcpy(sum, dig, sizeof(comp_t) * m0.n);
    for (int j = have_carry ? 0 : 1; j < k; ++j) lab_add(sum, dig + static_cast<size_t>(W) * (j * t), m0.n, m0.p);
    const int half = P.mrs[0] / 2;
    for (size_t o = 0; o < P.out_mod.size(); ++o) {
        const ModInfo& mo = mod_info(P.out_mod[o]);
        draw(prg, stream, ctr, mo.p, out0[o]);
        const int lo = P.lower, up = P.upper;
        garble_proj(sum, R.get(m0.p), m0, out0[o], R.get(mo.p), mo,
                    [half, lo, up](int v) { return static_cast<i64>(v < half ? up : lo); }, sign + o * m0.p, 1,
                    Mask{hard, stream, tw_sub(TW_SIGN, 0), static_cast<int>(o)});
    }
}

void sign_eval_fused(const SignPlan& P, const comp_t* const* in, const u128* approx, const u128* cast2,
                     const u128* sign, comp_t* const* out, bool hard, u64 gate) {
    const int k = static_cast<int>(P.crt.size()), t = static_cast<int>(P.mrs.size());
    const int W = P.max_n;
    comp_t* base = sign_scratch().get(static_cast<size_t>(W) * (k * t + 3));
    comp_t* dig = base;
    comp_t* carry = dig + static_cast<size_t>(W) * k * t;
    comp_t* sum = carry + W;
    comp_t* newc = sum + W;
    for (int j = 0; j < k; ++j) {
        const ModInfo& mi = mod_info(P.crt[j]);
        if (hard) {  // one key, t slots of the row's pads
            PadRow pr(compress(in[j], mi), gate, tw_sub(TW_APPROX, j));
            const u128* row = approx + t * P.crt_prefix[j] + static_cast<i64>(color_of(in[j], mi.p)) * t;
            for (int d = 0; d < t; ++d)
                decompress(row[d] - pr.get(d), dig + static_cast<size_t>(W) * (j * t + d), mod_info(P.digit_mod(d)));
            continue;
        }
        for (int d = 0; d < t; ++d)
            eval_proj(in[j], mi, approx + t * P.crt_prefix[j] + d, mod_info(P.digit_mod(d)),
                      dig + static_cast<size_t>(W) * (j * t + d), t);
    }
    bool have_carry = false;
    i64 c2 = 0;
    for (int d = t - 1; d >= 1; --d) {
        const ModInfo& mo = mod_info(P.digit_mod(d));
        if (have_carry) std::memcpy(sum, carry, sizeof(comp_t) * mo.n);
        else std::memcpy(sum, dig + static_cast<size_t>(W) * d, sizeof(comp_t) * mo.n);
        for (int j = have_carry ? 0 : 1; j < k; ++j) lab_add(sum, dig + static_cast<size_t>(W) * (j * t + d), mo.n, mo.p);
        const ModInfo& mn = mod_info(P.carry_mod(d));
        eval_proj(sum, mo, cast2 + c2, mn, newc, 1, Mask{hard, gate, tw_sub(TW_CAST2, d), 0});
        c2 += mo.p;
        std::memcpy(carry, newc, sizeof(comp_t) * mn.n);
        have_carry = true;
    }
    const ModInfo& m0 = mod_info(P.mrs[0]);
    if (have_carry) std::memcpy(sum, carry, sizeof(comp_t) * m0.n);
    else std::memcpy(sum, dig, sizeof(comp_t) * m0.n);
    for (int j = have_carry ? 0 : 1; j < k; ++j) lab_add(sum, dig + static_cast<size_t>(W) * (j * t), m0.n, m0.p);
    PadRow pr(compress(sum, m0), gate, tw_sub(TW_SIGN, 0));
    for (size_t o = 0; o < P.out_mod.size(); ++o) {
        if (hard)
            decompress(sign[o * m0.p + color_of(sum, m0.p)] - pr.get(static_cast<int>(o)), out[o],
                       mod_info(P.out_mod[o]));
        else
            eval_proj(sum, m0, sign + o * m0.p, mod_info(P.out_mod[o]), out[o]);
    }
}
}  // namespace

void sign_garble_elem(const SignPlan& P, const LabelBank& R, const LabelBank& Z, const Prg& prg, u64 stream,
                      const comp_t* const* in0, u128* approx, u128* cast1, u128* cast2, u128* sign,
                      comp_t* const* out0, bool hard) {
    if (P.fused) {
        sign_garble_fused(P, R, prg, stream, in0, approx, cast2, sign, out0, hard);
        return;
    }
    DASH_CHECK(!hard, "the hardened encoding needs the fused sign construction (the reference casts key a "
                      "projection with the public zero label)");
    const int k = static_cast<int>(P.crt.size()), t = static_cast<int>(P.mrs.size());
    const int W = P.max_n;
    comp_t* base = sign_scratch().get(static_cast<size_t>(W) * (k * t + (k + 1) + 4));
    comp_t* mrs_lab = base;                          // [k*t][W]
    comp_t* bases = mrs_lab + static_cast<size_t>(W) * k * t;  // [k+1][W]
    comp_t* carry = bases + static_cast<size_t>(W) * (k + 1);
    comp_t* sum2 = carry + W;
    comp_t* newc = sum2 + W;
    comp_t* sum = newc + W;
    u64 ctr = 0;
    for (int j = 0; j < k; ++j)
        for (int d = 0; d < t; ++d) draw(prg, stream, ctr, P.mrs[d], mrs_lab + static_cast<size_t>(W) * (j * t + d));
    // Step 1: approximate residues in mixed radix
    ProjKeys& K = proj_keys_scratch();
    for (int j = 0; j < k; ++j) {
        const ModInfo& mi = mod_info(P.crt[j]);
        const auto& lut = P.lookup[j];
        proj_keys(in0[j], R.get(mi.p), mi, K);
        for (int d = 0; d < t; ++d) {
            const ModInfo& mo = mod_info(P.mrs[d]);
            garble_proj_keys(K, mrs_lab + static_cast<size_t>(W) * (j * t + d), R.get(mo.p), mo,
                             [&](int v) { return static_cast<i64>(lut[static_cast<size_t>(v) * t + d]); },
                             approx + t * P.crt_prefix[j] + d, t);
        }
    }
    // Step 2: mixed-radix addition from the least significant digit
    {
        const int m_last = P.mrs[t - 1];
        std::memcpy(carry, Z.get(m_last), sizeof(comp_t) * nr_comps(m_last));
    }
    i64 c1 = 0, c2 = 0;
    for (int d = t - 1; d >= 1; --d) {
        const int m = P.mrs[d];
        const ModInfo& mm = mod_info(m);
        const ModInfo& mo = mod_info((k + 1) * m);
        for (int j = 0; j <= k; ++j) draw(prg, stream, ctr, mo.p, bases + static_cast<size_t>(W) * j);
        auto ident = [](int v) { return static_cast<i64>(v); };
        for (int j = 0; j < k; ++j) {
            garble_proj(mrs_lab + static_cast<size_t>(W) * (j * t + d), R.get(m), mm, bases + static_cast<size_t>(W) * j,
                        R.get(mo.p), mo, ident, cast1 + c1);
            c1 += m;
        }
        garble_proj(carry, R.get(m), mm, bases + static_cast<size_t>(W) * k, R.get(mo.p), mo, ident, cast1 + c1);
        c1 += m;
        std::memcpy(sum2, bases, sizeof(comp_t) * mo.n);
        for (int j = 1; j <= k; ++j) lab_add(sum2, bases + static_cast<size_t>(W) * j, mo.n, mo.p);
        const ModInfo& mn = mod_info(P.mrs[d - 1]);
        draw(prg, stream, ctr, mn.p, newc);
        garble_proj(sum2, R.get(mo.p), mo, newc, R.get(mn.p), mn, [m](int v) { return static_cast<i64>(v / m); },
                    cast2 + c2);
        c2 += mo.p;
        std::memcpy(carry, newc, sizeof(comp_t) * mn.n);
    }
    const ModInfo& m0 = mod_info(P.mrs[0]);
    std::memcpy(sum, carry, sizeof(comp_t) * m0.n);
    for (int j = 0; j < k; ++j) lab_add(sum, mrs_lab + static_cast<size_t>(W) * (j * t), m0.n, m0.p);
    // Step 3: most significant digit -> sign value in every output modulus
    const int half = P.mrs[0] / 2;
    for (size_t o = 0; o < P.out_mod.size(); ++o) {
        const ModInfo& mo = mod_info(P.out_mod[o]);
        draw(prg, stream, ctr, mo.p, out0[o]);
        const int lo = P.lower, up = P.upper;
        garble_proj(sum, R.get(m0.p), m0, out0[o], R.get(mo.p), mo,
                    [half, lo, up](int v) { return static_cast<i64>(v < half ? up : lo); }, sign + o * m0.p);
    }
}

void sign_eval_elem(const SignPlan& P, const LabelBank& Z, const comp_t* const* in, const u128* approx,
                    const u128* cast1, const u128* cast2, const u128* sign, comp_t* const* out, bool hard, u64 gate) {
    if (P.fused) {
        sign_eval_fused(P, in, approx, cast2, sign, out, hard, gate);
        return;
    }
    DASH_CHECK(!hard, "the hardened encoding needs the fused sign construction");
    const int k = static_cast<int>(P.crt.size()), t = static_cast<int>(P.mrs.size());
    const int W = P.max_n;
    comp_t* base = sign_scratch().get(static_cast<size_t>(W) * (k * t + (k + 1) + 4));
    comp_t* mrs_lab = base;
    comp_t* casts = mrs_lab + static_cast<size_t>(W) * k * t;
    comp_t* carry = casts + static_cast<size_t>(W) * (k + 1);
    comp_t* sum2 = carry + W;
    comp_t* newc = sum2 + W;
    comp_t* sum = newc + W;
    for (int j = 0; j < k; ++j) {
        const ModInfo& mi = mod_info(P.crt[j]);
        for (int d = 0; d < t; ++d)
            eval_proj(in[j], mi, approx + t * P.crt_prefix[j] + d, mod_info(P.mrs[d]),
                      mrs_lab + static_cast<size_t>(W) * (j * t + d), t);
    }
    {
        const int m_last = P.mrs[t - 1];
        std::memcpy(carry, Z.get(m_last), sizeof(comp_t) * nr_comps(m_last));
    }
    i64 c1 = 0, c2 = 0;
    for (int d = t - 1; d >= 1; --d) {
        const int m = P.mrs[d];
        const ModInfo& mm = mod_info(m);
        const ModInfo& mo = mod_info((k + 1) * m);
        for (int j = 0; j < k; ++j) {
            eval_proj(mrs_lab + static_cast<size_t>(W) * (j * t + d), mm, cast1 + c1, mo, casts + static_cast<size_t>(W) * j);
            c1 += m;
        }
        eval_proj(carry, mm, cast1 + c1, mo, casts + static_cast<size_t>(W) * k);
        c1 += m;
        std::memcpy(sum2, casts, sizeof(comp_t) * mo.n);
        for (int j = 1; j <= k; ++j) lab_add(sum2, casts + static_cast<size_t>(W) * j, mo.n, mo.p);
        const ModInfo& mn = mod_info(P.mrs[d - 1]);
        eval_proj(sum2, mo, cast2 + c2, mn, newc);
        c2 += mo.p;
        std::memcpy(carry, newc, sizeof(comp_t) * mn.n);
    }
    const ModInfo& m0 = mod_info(P.mrs[0]);
    std::memcpy(sum, carry, sizeof(comp_t) * m0.n);
    for (int j = 0; j < k; ++j) lab_add(sum, mrs_lab + static_cast<size_t>(W) * (j * t), m0.n, m0.p);
    for (size_t o = 0; o < P.out_mod.size(); ++o)
        eval_proj(sum, m0, sign + o * m0.p, mod_info(P.out_mod[o]), out[o]);
}

// ---------------------------------------------------------------------------
void mixed_mult_garble(const comp_t* x0, const ModInfo& mp, const comp_t* y0, const ModInfo& mq, const LabelBank& R,
                       const Prg& prg, u64 stream, u64& ctr, u128* g, u128* e, comp_t* out0, const MMTw& tw) {
    const int p = mp.p, q = mq.p;
    comp_t* sk03 = misc_scratch().get(2 * mp.n);
    comp_t* sk04 = sk03 + mp.n;
    const i64 r = x0[0];
    draw(prg, stream, ctr, p, sk03);
    draw(prg, stream, ctr, p, sk04);
    // garbler half gate: x -> x*r
    garble_proj(x0, R.get(p), mp, sk03, R.get(p), mp, [r](int v) { return static_cast<i64>(v) * r; }, g, 1, tw.g());
    // evaluator half gate: y -> -(y + r), payload offset is x0
    garble_proj(y0, R.get(q), mq, sk04, x0, mp, [r, p](int v) { return pmod(-(v + r), p); }, e, 1, tw.e());
    // mini gate: y -> (y + r) mod p
    garble_proj_mini(y0, R.get(q), mq, [r, p](int v) { return pmod(v + r, p); }, e + q, tw.mini(), tw.lane());
    std::memcpy(out0, sk04, sizeof(comp_t) * mp.n);
    lab_sub(out0, sk03, mp.n, p);
}

void mixed_mult_eval(const comp_t* x, const ModInfo& mp, const comp_t* y, const ModInfo& mq, const u128* g,
                     const u128* e, comp_t* out, const MMTw& tw) {
    comp_t* gl = misc_scratch().get(mp.n);
    eval_proj(x, mp, g, mp, gl, 1, tw.g());
    eval_proj(y, mq, e, mp, out, 1, tw.e());
    const i64 ypr = pmod(eval_proj_mini(y, mq, e + mq.p, tw.mini(), tw.lane()), mp.p);
    lab_axpy(out, ypr, x, mp.n, mp.p);
    lab_sub(out, gl, mp.n, mp.p);
}

void gen_mult_garble(const comp_t* x0, const comp_t* y0, const ModInfo& mp, const LabelBank& R, const Prg& prg,
                     u64 stream, u64& ctr, u128* g, u128* e, comp_t* out0, bool hard, int j) {
    const int p = mp.p;
    comp_t* sk03 = misc_scratch().get(2 * mp.n);
    comp_t* sk04 = sk03 + mp.n;
    const i64 r = y0[0];
    draw(prg, stream, ctr, p, sk03);
    draw(prg, stream, ctr, p, sk04);
    garble_proj(x0, R.get(p), mp, sk03, R.get(p), mp, [r](int v) { return static_cast<i64>(v) * r; }, g, 1,
                Mask{hard, stream, tw_sub(TW_MMG, j), 0});
    garble_proj(y0, R.get(p), mp, sk04, x0, mp, [r, p](int v) { return pmod(-(v + r), p); }, e, 1,
                Mask{hard, stream, tw_sub(TW_GME, j), 0});
    std::memcpy(out0, sk04, sizeof(comp_t) * mp.n);
    lab_sub(out0, sk03, mp.n, p);
}

void gen_mult_eval(const comp_t* x, const comp_t* y, const ModInfo& mp, const u128* g, const u128* e, comp_t* out,
                   bool hard, u64 gate, int j) {
    comp_t* gl = misc_scratch().get(mp.n);
    eval_proj(x, mp, g, mp, gl, 1, Mask{hard, gate, tw_sub(TW_MMG, j), 0});
    eval_proj(y, mp, e, mp, out, 1, Mask{hard, gate, tw_sub(TW_GME, j), 0});
    lab_axpy(out, color_of(y, mp.p), x, mp.n, mp.p);
    lab_sub(out, gl, mp.n, mp.p);
}

// ---------------------------------------------------------------------------
BEPlan::BEPlan(const std::vector<int>& mod, const std::vector<int>& ext) : moduli(mod), extra(ext) {
    const int E = static_cast<int>(moduli.size());
    nonext = E - static_cast<int>(extra.size());
    DASH_CHECK(nonext >= 1, "base extension needs at least one non-extended modulus");
    for (int e : extra) {
        auto it = std::find(moduli.begin(), moduli.end(), e);
        DASH_CHECK(it != moduli.end(), "extra modulus not in base");
        extra_idx.push_back(static_cast<int>(it - moduli.begin()));
    }
    std::vector<int> idx(E);
    std::iota(idx.begin(), idx.end(), 0);
    const int ne = static_cast<int>(extra_idx.size());
    for (int i = 1; i <= ne; ++i) std::swap(idx[extra_idx[ne - i]], idx[E - i]);
    swapped.resize(E);
    pos_of.resize(E);
    for (int i = 0; i < E; ++i) {
        swapped[i] = moduli[idx[i]];
        pos_of[idx[i]] = i;
    }
    inv_partial.resize(E);
    for (int i = 0; i + 1 < E; ++i)
        for (int j = i + 1; j < E; ++j) inv_partial[i].push_back(mul_inv(static_cast<u128>(swapped[i]), swapped[j]));
    u128 acc = 1;
    for (int i = 0; i < nonext; ++i) acc *= static_cast<u128>(swapped[i]);
    for (int e : extra) {
        i64 inv_total = mul_inv(acc % static_cast<u128>(e), e);
        invv.push_back(mul_inv(static_cast<u128>(inv_total), e));
    }
    n_tab = 0;
    for (int i = 0; i < nonext; ++i) n_tab += static_cast<i64>(E - i - 1) * swapped[i];
}

void be_garble_elem(const BEPlan& P, const LabelBank& R, const Prg& prg, u64 stream, u64& ctr, comp_t* const* L,
                    u128* tab, bool hard) {
    const int E = static_cast<int>(P.moduli.size());
    // l_w: working copies in swapped order; only the extra residues are
    // written back (non-extended residues stay untouched, as in the reference)
    comp_t* work = be_scratch().get(static_cast<size_t>(128) * E);
    std::vector<comp_t*> lw(E);
    for (int i = 0; i < E; ++i) {
        lw[P.pos_of[i]] = work + 128 * P.pos_of[i];
        std::memcpy(lw[P.pos_of[i]], L[i], sizeof(comp_t) * nr_comps(P.moduli[i]));
    }
    comp_t* out0 = misc_scratch().get(128);
    i64 off = 0;
    for (int i = 0; i < P.nonext; ++i) {
        const ModInfo& mi = mod_info(P.swapped[i]);
        for (int j = 0; j < E - i - 1; ++j) {
            const int tg = i + j + 1;
            const ModInfo& mo = mod_info(P.swapped[tg]);
            draw(prg, stream, ctr, mo.p, out0);
            garble_proj(lw[i], R.get(mi.p), mi, out0, R.get(mo.p), mo, [](int v) { return static_cast<i64>(v); },
                        tab + off, 1, Mask{hard, stream, tw_sub(TW_BE, i), j});
            off += mi.p;
            lab_sub(lw[tg], out0, mo.n, mo.p);
            lab_scale(lw[tg], P.inv_partial[i][j], mo.n, mo.p);
        }
    }
    for (size_t x = 0; x < P.extra.size(); ++x) {
        const int bi = P.extra_idx[x];
        std::memcpy(L[bi], lw[P.pos_of[bi]], sizeof(comp_t) * nr_comps(P.moduli[bi]));
        lab_scale(L[bi], -P.invv[x], nr_comps(P.moduli[bi]), P.moduli[bi]);
    }
}

void be_eval_elem(const BEPlan& P, comp_t* const* L, const u128* tab, bool hard, u64 gate) {
    const int E = static_cast<int>(P.moduli.size());
    comp_t* work = be_scratch().get(static_cast<size_t>(128) * E);
    std::vector<comp_t*> lw(E);
    for (int i = 0; i < E; ++i) {
        lw[P.pos_of[i]] = work + 128 * P.pos_of[i];
        std::memcpy(lw[P.pos_of[i]], L[i], sizeof(comp_t) * nr_comps(P.moduli[i]));
    }
    comp_t* pr = misc_scratch().get(128);
    i64 off = 0;
    for (int i = 0; i < P.nonext; ++i) {
        const ModInfo& mi = mod_info(P.swapped[i]);
        for (int j = 0; j < E - i - 1; ++j) {
            const int tg = i + j + 1;
            const ModInfo& mo = mod_info(P.swapped[tg]);
            eval_proj(lw[i], mi, tab + off, mo, pr, 1, Mask{hard, gate, tw_sub(TW_BE, i), j});
            off += mi.p;
            lab_sub(lw[tg], pr, mo.n, mo.p);
            lab_scale(lw[tg], P.inv_partial[i][j], mo.n, mo.p);
        }
    }
    for (size_t x = 0; x < P.extra.size(); ++x) {
        const int bi = P.extra_idx[x];
        std::memcpy(L[bi], lw[P.pos_of[bi]], sizeof(comp_t) * nr_comps(P.moduli[bi]));
        lab_scale(L[bi], -P.invv[x], nr_comps(P.moduli[bi]), P.moduli[bi]);
    }
}

// ---------------------------------------------------------------------------
RescalePlan::RescalePlan(const std::vector<int>& crt_, const std::vector<int>& mrs, const std::vector<int>& f,
                         bool sbe, bool fused_sign)
    : crt(crt_), factors(f), sign_be(sbe) {
    const int k = static_cast<int>(crt.size());
    std::vector<int> ignored;
    for (int s : factors) {
        auto it = std::find(crt.begin(), crt.end(), s);
        DASH_CHECK(it != crt.end(), "rescale factor must be a CRT modulus");
        int fi = static_cast<int>(it - crt.begin());
        factor_idx.push_back(fi);
        ignored.push_back(fi);
        std::vector<int> act;
        std::vector<i64> iv;
        for (int j = 0; j < k; ++j) {
            if (std::find(ignored.begin(), ignored.end(), j) != ignored.end()) continue;
            act.push_back(j);
            iv.push_back(mul_inv(static_cast<u128>(s), crt[j]));
            n_trans += s;
        }
        active.push_back(act);
        inv.push_back(iv);
        sprod *= s;
    }
    if (sign_be) {
        DASH_CHECK(factors.size() == 1 && factors[0] == 2 && crt[0] == 2,
                   "sign base extension rescale needs factors {2} and crt[0] == 2");
        sign = SignPlan(crt, mrs, {2}, 1, 0, fused_sign);
    } else {
        be = BEPlan(crt, factors);
        n_be = be.n_tab;
    }
}

void rescale_garble_elem(const RescalePlan& P, const LabelBank& R, const LabelBank& Z, const Prg& prg, u64 stream,
                         comp_t* const* L, const comp_t* const* up_base, const comp_t* const* down_base, u128* trans,
                         u128* s_approx, u128* s_cast1, u128* s_cast2, u128* s_sign, u128* be, bool hard) {
    const int k = static_cast<int>(P.crt.size());
    DASH_CHECK(!hard || !P.sign_be, "the hardened encoding has no legacy (sign base extension) rescale: its sign "
                                    "gadget keys a projection with the public zero label; use the mixed-radix rescale");
    for (int j = 0; j < k; ++j) lab_add(L[j], up_base[j], nr_comps(P.crt[j]), P.crt[j]);
    comp_t* out0 = rescale_scratch().get(128);
    u64 ctr = 0;
    i64 off = 0;
    for (size_t f = 0; f < P.factors.size(); ++f) {
        const int s = P.factors[f];
        const int fi = P.factor_idx[f];
        const ModInfo& ms = mod_info(s);
        for (size_t a = 0; a < P.active[f].size(); ++a) {
            const int j = P.active[f][a];
            const ModInfo& mj = mod_info(P.crt[j]);
            draw(prg, stream, ctr, mj.p, out0);
            garble_proj(L[fi], R.get(s), ms, out0, R.get(mj.p), mj, [](int v) { return static_cast<i64>(v); },
                        trans + off, 1, Mask{hard, stream, tw_sub(TW_TRANS, static_cast<uint32_t>(f)), static_cast<int>(a)});
            off += s;
            lab_sub(L[j], out0, mj.n, mj.p);
            lab_scale(L[j], P.inv[f][a], mj.n, mj.p);
        }
    }
    for (int fi : P.factor_idx) std::memcpy(L[fi], Z.get(P.crt[fi]), sizeof(comp_t) * nr_comps(P.crt[fi]));
    if (P.sign_be) {
        comp_t* sig = rescale_scratch().get(128) ;  // reuse: out0 no longer needed
        comp_t* outs[1] = {sig};
        sign_garble_elem(P.sign, R, Z, prg, stream ^ (1ull << 43), L, s_approx, s_cast1, s_cast2, s_sign, outs);
        std::memcpy(L[0], sig, sizeof(comp_t) * nr_comps(2));
    } else {
        be_garble_elem(P.be, R, prg, stream, ctr, L, be, hard);
    }
    for (int j = 0; j < k; ++j) lab_sub(L[j], down_base[j], nr_comps(P.crt[j]), P.crt[j]);
}

void rescale_eval_elem(const RescalePlan& P, const LabelBank& Z, comp_t* const* L, const comp_t* const* up,
                       const comp_t* const* down, const u128* trans, const u128* s_approx, const u128* s_cast1,
                       const u128* s_cast2, const u128* s_sign, const u128* be, bool hard, u64 gate) {
    const int k = static_cast<int>(P.crt.size());
    DASH_CHECK(!hard || !P.sign_be, "the hardened encoding has no legacy (sign base extension) rescale");
    for (int j = 0; j < k; ++j) lab_add(L[j], up[j], nr_comps(P.crt[j]), P.crt[j]);
    comp_t* pr = rescale_scratch().get(128);
    i64 off = 0;
    for (size_t f = 0; f < P.factors.size(); ++f) {
        const int s = P.factors[f];
        const int fi = P.factor_idx[f];
        const ModInfo& ms = mod_info(s);
        for (size_t a = 0; a < P.active[f].size(); ++a) {
            const int j = P.active[f][a];
            const ModInfo& mj = mod_info(P.crt[j]);
            eval_proj(L[fi], ms, trans + off, mj, pr, 1,
                      Mask{hard, gate, tw_sub(TW_TRANS, static_cast<uint32_t>(f)), static_cast<int>(a)});
            off += s;
            lab_sub(L[j], pr, mj.n, mj.p);
            lab_scale(L[j], P.inv[f][a], mj.n, mj.p);
        }
    }
    for (int fi : P.factor_idx) std::memcpy(L[fi], Z.get(P.crt[fi]), sizeof(comp_t) * nr_comps(P.crt[fi]));
    if (P.sign_be) {
        comp_t* sig = rescale_scratch().get(128);
        comp_t* outs[1] = {sig};
        sign_eval_elem(P.sign, Z, L, s_approx, s_cast1, s_cast2, s_sign, outs);
        std::memcpy(L[0], sig, sizeof(comp_t) * nr_comps(2));
    } else {
        be_eval_elem(P.be, L, be, hard, gate);
    }
    for (int j = 0; j < k; ++j) lab_sub(L[j], down[j], nr_comps(P.crt[j]), P.crt[j]);
}

// ---------------------------------------------------------------------------
// Single-shot mixed-radix rescale (gadgets.h RescaleMrsPlan)
RescaleMrsPlan::RescaleMrsPlan(const std::vector<int>& crt_, int l_, bool sign_last_)
    : crt(crt_), l(l_), sign_last(sign_last_) {
    const int kk = k();
    DASH_CHECK(kk >= 2 && crt[0] == 2, "mixed-radix rescale needs CRT residue 0 = 2");
    DASH_CHECK(l >= 1 && l <= 14, "mixed-radix rescale: 1 <= l <= 14");
    for (int j = 1; j < kk; ++j) DASH_CHECK(crt[j] % 2 == 1, "mixed-radix rescale: residues 1.. must be odd");
    S = i64(1) << l;
    T = 2 * S;
    M = 1;
    for (int p : crt) M *= p;
    const i64 h = M / 2;
    U = h + pmod(S - 1 - h % S, S);
    q = (U - (S - 1)) / S;
    ord.clear();
    if (sign_last) {
        for (int j = 1; j < kk; ++j) ord.push_back(j);
        ord.push_back(0);
    } else {
        for (int j = 0; j < kk; ++j) ord.push_back(j);
    }
    B.assign(kk, 1);
    Binv.assign(kk, 1);
    Sinv.assign(kk, 0);
    for (int i = 1; i < kk; ++i) B[i] = B[i - 1] * crt[ord[i - 1]];
    for (int i = 0; i < kk; ++i) Binv[i] = mul_inv(static_cast<u128>(B[i] % crt[ord[i]]), crt[ord[i]]);
    for (int j = 1; j < kk; ++j) Sinv[j] = mul_inv(static_cast<u128>(S % crt[j]), crt[j]);
    dig_off.assign(kk, 0);
    i64 off = 0;
    for (int i = 0; i < kk; ++i) {
        dig_off[i] = off;
        off += static_cast<i64>(crt[ord[i]]) * targets(i);
    }
    fin_off = off;
    n_tab = off + T * kk;
}

i64 RescaleMrsPlan::digit_fn(int i, int t, i64 v) const {
    const i64 pi = crt[ord[i]];
    // digit a_i of x_u; with sign_last the mod-2 key already carries a_{k-1} (U folded in below)
    const i64 a = sign_last && i == k() - 1 ? pmod(v, pi) : pmod((v + U % pi) * Binv[i], pi);
    const i64 m = target_mod(i, t);
    i64 val = a * (B[i] % m);
    if (sign_last && i == 0 && t < k() - 1 && target_res(i, t) == 0) val -= U % m;
    return pmod(val, m);
}

i64 RescaleMrsPlan::final_fn(int j, i64 v) const {
    if (j == 0) return pmod(v / S - q, 2);
    const i64 p = crt[j];
    return pmod((pmod(U, p) - v % S) * Sinv[j] - q, p);
}

void rescale_mrs_garble_elem(const RescaleMrsPlan& P, const LabelBank& R, const Prg& prg, u64 stream,
                             comp_t* const* L, u128* tab, comp_t* sig, bool hard) {
    const int k = P.k();
    constexpr int W = 128;
    // draws, PRG counter order: digit i's target labels (t = 0..k-1-i), then the k final output labels
    int nd = 0;
    for (int i = 0; i < k; ++i) nd += P.targets(i);
    comp_t* buf = rescale_scratch().get(static_cast<size_t>(W) * (nd + k + k + 1));
    std::vector<comp_t*> dig(nd), fin(k), key(k);
    u64 ctr = 0;
    int s = 0;
    for (int i = 0; i < k; ++i)
        for (int t = 0; t < P.targets(i); ++t, ++s) {
            dig[s] = buf + static_cast<size_t>(W) * s;
            draw(prg, stream, ctr, P.target_mod(i, t), dig[s]);
        }
    for (int j = 0; j < k; ++j) {
        fin[j] = buf + static_cast<size_t>(W) * (nd + j);
        draw(prg, stream, ctr, P.crt[j], fin[j]);
    }
    comp_t* acc = buf + static_cast<size_t>(W) * (nd + 2 * k);
    const ModInfo& mT = mod_info(static_cast<int>(P.T));
    std::fill(acc, acc + mT.n, comp_t(0));
    // key base labels: K_i = L_i - sum_{l<i} P_{l,i} (by residue); r = sum_i P_{i,T}
    for (int j = 0; j < k; ++j) {
        key[j] = buf + static_cast<size_t>(W) * (nd + k + j);
        std::memcpy(key[j], L[j], sizeof(comp_t) * nr_comps(P.crt[j]));
    }
    s = 0;
    for (int i = 0; i < k; ++i)
        for (int t = 0; t < P.targets(i); ++t, ++s) {
            if (t == k - 1 - i) {
                lab_add(acc, dig[s], mT.n, mT.p);
            } else {
                const int r = P.target_res(i, t);
                lab_sub(key[r], dig[s], nr_comps(P.crt[r]), P.crt[r]);
            }
        }
    if (P.sign_last && sig) std::memcpy(sig, key[0], sizeof(comp_t) * nr_comps(2));
    ProjKeys& K = proj_keys_scratch();
    s = 0;
    for (int i = 0; i < k; ++i) {
        const ModInfo& mi = mod_info(P.crt[P.ord[i]]);
        proj_keys(key[P.ord[i]], R.get(mi.p), mi, K, hard);
        const int nt = P.targets(i);
        for (int t = 0; t < nt; ++t, ++s) {
            const ModInfo& mo = mod_info(P.target_mod(i, t));
            garble_proj_keys(K, dig[s], R.get(mo.p), mo, [&](int v) { return P.digit_fn(i, t, v); },
                             tab + P.dig_off[i] + t, nt, Mask{hard, stream, tw_sub(TW_MRS, i), t});
        }
    }
    proj_keys(acc, R.get(mT.p), mT, K, hard);
    for (int j = 0; j < k; ++j) {
        const ModInfo& mo = mod_info(P.crt[j]);
        garble_proj_keys(K, fin[j], R.get(mo.p), mo, [&](int v) { return P.final_fn(j, v); }, tab + P.fin_off + j, k,
                         Mask{hard, stream, tw_sub(TW_MRS, k), j});
    }
    // output base labels: Y_j = S^-1 L_j + fin_j (j >= 1), Y_0 = fin_0
    std::memcpy(L[0], fin[0], sizeof(comp_t) * nr_comps(2));
    for (int j = 1; j < k; ++j) {
        const int p = P.crt[j], n = nr_comps(p);
        lab_scale(L[j], P.Sinv[j], n, p);
        lab_add(L[j], fin[j], n, p);
    }
}

void rescale_mrs_eval_elem(const RescaleMrsPlan& P, comp_t* const* L, const u128* tab, comp_t* sig, bool hard,
                           u64 gate) {
    const int k = P.k();
    constexpr int W = 128;
    comp_t* buf = rescale_scratch().get(static_cast<size_t>(W) * (k + 2));
    std::vector<comp_t*> key(k);
    for (int j = 0; j < k; ++j) {
        key[j] = buf + static_cast<size_t>(W) * j;
        std::memcpy(key[j], L[j], sizeof(comp_t) * nr_comps(P.crt[j]));
    }
    const ModInfo& mT = mod_info(static_cast<int>(P.T));
    comp_t* acc = buf + static_cast<size_t>(W) * k;
    comp_t* pr = buf + static_cast<size_t>(W) * (k + 1);
    std::fill(acc, acc + mT.n, comp_t(0));
    for (int i = 0; i < k; ++i) {
        const int r0 = P.ord[i];
        const ModInfo& mi = mod_info(P.crt[r0]);
        const u128 kc = compress(key[r0], mi);
        const u128 h = hard ? 0 : hash(kc);
        PadRow pads(kc, gate, tw_sub(TW_MRS, i));
        const int nt = P.targets(i);
        const u128* row = tab + P.dig_off[i] + static_cast<i64>(color_of(key[r0], mi.p)) * nt;
        for (int t = 0; t < nt; ++t) {
            const ModInfo& mo = mod_info(P.target_mod(i, t));
            decompress(row[t] - (hard ? pads.get(t) : h), pr, mo);
            if (t == nt - 1) lab_add(acc, pr, mo.n, mo.p);
            else lab_sub(key[P.target_res(i, t)], pr, mo.n, mo.p);
        }
    }
    if (P.sign_last && sig) std::memcpy(sig, key[0], sizeof(comp_t) * nr_comps(2));
    const u128 kc = compress(acc, mT);
    const u128 h = hard ? 0 : hash(kc);
    PadRow pads(kc, gate, tw_sub(TW_MRS, k));
    const u128* row = tab + P.fin_off + static_cast<i64>(color_of(acc, mT.p)) * k;
    decompress(row[0] - (hard ? pads.get(0) : h), L[0], mod_info(2));
    for (int j = 1; j < k; ++j) {
        const ModInfo& mo = mod_info(P.crt[j]);
        decompress(row[j] - (hard ? pads.get(j) : h), pr, mo);
        lab_scale(L[j], P.Sinv[j], mo.n, mo.p);
        lab_add(L[j], pr, mo.n, mo.p);
    }
}

// ---------------------------------------------------------------------------
// Exact sign by mixed-radix conversion (gadgets.h SignMrsPlan)
SignMrsPlan::SignMrsPlan(const std::vector<int>& crt_) : crt(crt_) {
    const int kk = k();
    DASH_CHECK(kk >= 2 && crt[0] == 2, "mixed-radix sign needs CRT residue 0 = 2");
    for (int j = 1; j < kk; ++j) DASH_CHECK(crt[j] % 2 == 1, "mixed-radix sign: residues 1.. must be odd");
    for (int p : crt) M *= p;
    U = M / 2;
    ord.clear();
    for (int j = 1; j < kk; ++j) ord.push_back(j);
    ord.push_back(0);
    B.assign(kk, 1);
    Binv.assign(kk, 1);
    for (int i = 1; i < kk; ++i) B[i] = B[i - 1] * crt[ord[i - 1]];
    for (int i = 0; i < kk; ++i) Binv[i] = mul_inv(static_cast<u128>(B[i] % crt[ord[i]]), crt[ord[i]]);
    dig_off.assign(kk - 1, 0);
    i64 off = 0;
    for (int i = 0; i + 1 < kk; ++i) {
        dig_off[i] = off;
        off += static_cast<i64>(crt[ord[i]]) * targets(i);
    }
    n_tab = off;
}

i64 SignMrsPlan::digit_fn(int i, int t, i64 v) const {
    const i64 pi = crt[ord[i]];
    const i64 a = pmod((v + U % pi) * Binv[i], pi);
    const int r = target_res(i, t);
    const i64 m = crt[r];
    i64 val = a * (B[i] % m);
    if (i == 0 && r == ord[k() - 1]) val -= U % m;  // residue 0's key then carries a_{k-1} itself
    return pmod(val, m);
}

void sign_mrs_garble_elem(const SignMrsPlan& P, const LabelBank& R, const Prg& prg, u64 stream,
                          const comp_t* const* x0, u128* tab, comp_t* sig0, bool hard) {
    const int k = P.k();
    constexpr int W = 128;
    int nd = 0;
    for (int i = 0; i + 1 < k; ++i) nd += P.targets(i);
    comp_t* buf = sign_scratch().get(static_cast<size_t>(W) * (nd + k));
    std::vector<comp_t*> dig(std::max(nd, 1)), key(k);
    u64 ctr = 0;
    int s = 0;
    for (int i = 0; i + 1 < k; ++i)
        for (int t = 0; t < P.targets(i); ++t, ++s) {
            dig[s] = buf + static_cast<size_t>(W) * s;
            draw(prg, stream, ctr, P.crt[P.target_res(i, t)], dig[s]);
        }
    for (int j = 0; j < k; ++j) {
        key[j] = buf + static_cast<size_t>(W) * (nd + j);
        std::memcpy(key[j], x0[j], sizeof(comp_t) * nr_comps(P.crt[j]));
    }
    s = 0;
    for (int i = 0; i + 1 < k; ++i)
        for (int t = 0; t < P.targets(i); ++t, ++s) {
            const int r = P.target_res(i, t);
            lab_sub(key[r], dig[s], nr_comps(P.crt[r]), P.crt[r]);
        }
    ProjKeys& K = proj_keys_scratch();
    s = 0;
    for (int i = 0; i + 1 < k; ++i) {
        const ModInfo& mi = mod_info(P.crt[P.ord[i]]);
        proj_keys(key[P.ord[i]], R.get(mi.p), mi, K, hard);
        const int nt = P.targets(i);
        for (int t = 0; t < nt; ++t, ++s) {
            const ModInfo& mo = mod_info(P.crt[P.target_res(i, t)]);
            garble_proj_keys(K, dig[s], R.get(mo.p), mo, [&](int v) { return P.digit_fn(i, t, v); },
                             tab + P.dig_off[i] + t, nt, Mask{hard, stream, tw_sub(TW_SMRS, i), t});
        }
    }
    std::memcpy(sig0, key[P.ord[k - 1]], sizeof(comp_t) * nr_comps(2));
}

void sign_mrs_eval_elem(const SignMrsPlan& P, const comp_t* const* x, const u128* tab, comp_t* sig, bool hard,
                        u64 gate) {
    const int k = P.k();
    constexpr int W = 128;
    comp_t* buf = sign_scratch().get(static_cast<size_t>(W) * (k + 1));
    std::vector<comp_t*> key(k);
    for (int j = 0; j < k; ++j) {
        key[j] = buf + static_cast<size_t>(W) * j;
        std::memcpy(key[j], x[j], sizeof(comp_t) * nr_comps(P.crt[j]));
    }
    comp_t* pr = buf + static_cast<size_t>(W) * k;
    for (int i = 0; i + 1 < k; ++i) {
        const int r0 = P.ord[i];
        const ModInfo& mi = mod_info(P.crt[r0]);
        const u128 kc = compress(key[r0], mi);
        const u128 h = hard ? 0 : hash(kc);
        PadRow pads(kc, gate, tw_sub(TW_SMRS, i));
        const int nt = P.targets(i);
        const u128* row = tab + P.dig_off[i] + static_cast<i64>(color_of(key[r0], mi.p)) * nt;
        for (int t = 0; t < nt; ++t) {
            const int r = P.target_res(i, t);
            const ModInfo& mo = mod_info(P.crt[r]);
            decompress(row[t] - (hard ? pads.get(t) : h), pr, mo);
            lab_sub(key[r], pr, mo.n, mo.p);
        }
    }
    std::memcpy(sig, key[P.ord[k - 1]], sizeof(comp_t) * nr_comps(2));
}

}  // namespace dash
