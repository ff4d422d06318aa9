// Garbled gates and gadgets shared by the host garbler and the host (oracle)
// evaluator. Every gadget is written per *element* (one neuron across all CRT
// residues) so that the garbler, the CPU evaluator and the HIP kernels all
// walk exactly the same sequence of gates and table offsets.
//
// Reference behaviour reproduced here (semantics, not code):
//   projection gate           garbling/gates/projection_gate.h:62-102
//   mini projection           garbling/gates/projection_gate_mini.h:25-56
//   generalized half gate     garbling/gates/generalized_half_gate.h:51-89
//   mixed-modulus half gate   garbling/gates/mixed_mod_half_gate.h:56-104
//   approx-residue lookup     garbling/gadgets/lookup_approx_sign.h:75-101
//   approximate sign gadget   garbling/gadgets/sign_gadget.h:425-671
//   rescale gadget            garbling/gadgets/rescale_gadget.h:115-362
//   base extension gadget     garbling/gadgets/base_extension_gadget.h:70-295
// Table layouts are element-major (see docs/WIRE_FORMAT.md); the reference's
// residue-major rescale layout (rescale_gadget.h:152-175) is not reproduced
// because its own GPU kernel could not read it.
#pragma once

#include "core.h"

namespace dash {

// ---------------------------------------------------------------------------
// Offset (R_p) and zero (Z_p) labels for every modulus 2..max_modulus.
// ---------------------------------------------------------------------------
struct LabelBank {
    int max_mod = 0;
    std::vector<std::vector<comp_t>> lab;  // indexed by modulus
    const comp_t* get(int p) const {
        DASH_CHECK(p >= 2 && p <= max_mod && !lab[p].empty(), "label bank has no entry for modulus " + std::to_string(p));
        return lab[p].data();
    }
};

// ---------------------------------------------------------------------------
// Projection gate
// ---------------------------------------------------------------------------
struct ProjScratch {
    std::vector<comp_t> key, tmp;
    std::vector<u128> kc, hc, payc;
    std::vector<int> colors;
    std::vector<uint8_t> have;
};
ProjScratch& proj_scratch();

// Colors and hashes of the p keys in0 + i*Rin of one input label; shared by
// every projection of that label (the approx step projects one residue label
// into all t MRS digits: one key schedule instead of t).
// The keys of one projection row: kc[i] = compress(in0 + i*Rin), hc[i] = H(kc[i]) (reference masks), and
// per key the hardened pads of the row's tweak, one block at a time (pads of a fan-out row's slots)
struct ProjKeys {
    std::vector<comp_t> key;
    std::vector<u128> kc, hc;
    std::vector<int> colors;
    std::vector<PadRow> pads;
    bool hard = false;
    // mask of key i for mask m (m.hard: pad m.slot of (kc[i], m.gate, m.sub))
    u128 mask(int i, const Mask& m) {
        if (!m.hard) return hc[i];
        PadRow& r = pads[i];
        if (r.gate != m.gate || r.sub != m.sub || r.blk < 0) r = PadRow(kc[i], m.gate, m.sub);
        return r.get(m.slot);
    }
};
// hard: skip the reference hashes (hardened rows use the pads only)
inline void proj_keys(const comp_t* in0, const comp_t* Rin, const ModInfo& mi, ProjKeys& K, bool hard = false) {
    const int pin = mi.p, nin = mi.n;
    K.key.assign(in0, in0 + nin);
    K.kc.resize(pin);
    K.hc.resize(pin);
    K.colors.resize(pin);
    K.hard = hard;
    for (int i = 0; i < pin; ++i) {
        K.kc[i] = compress(K.key.data(), mi);
        K.colors[i] = K.key[0];
        lab_add(K.key.data(), Rin, nin, pin);
    }
    if (hard) K.pads.assign(pin, PadRow());
    else hash_batch(K.kc.data(), K.hc.data(), pin);
}

// table[color(in0 + i*Rin) * stride] = compress(out0 + f(i)*outR) + mask(compress(in0 + i*Rin))
template <class F>
inline void garble_proj_keys(ProjKeys& K, const comp_t* out0, const comp_t* outR, const ModInfo& mo, F&& f,
                             u128* table, int stride = 1, const Mask& mk = Mask()) {
    ProjScratch& s = proj_scratch();
    const int pin = static_cast<int>(K.kc.size());
    s.payc.resize(mo.p);
    s.have.assign(mo.p, 0);
    s.tmp.resize(mo.n);
    for (int i = 0; i < pin; ++i) {
        int c = static_cast<int>(pmod(f(i), mo.p));
        if (!s.have[c]) {
            lab_affine(s.tmp.data(), out0, c, outR, mo.n, mo.p);
            s.payc[c] = compress(s.tmp.data(), mo);
            s.have[c] = 1;
        }
        table[static_cast<i64>(K.colors[i]) * stride] = s.payc[c] + K.mask(i, mk);
    }
}

ProjKeys& proj_keys_scratch();

template <class F>
inline void garble_proj(const comp_t* in0, const comp_t* Rin, const ModInfo& mi, const comp_t* out0,
                        const comp_t* outR, const ModInfo& mo, F&& f, u128* table, int stride = 1,
                        const Mask& mk = Mask()) {
    ProjKeys& K = proj_keys_scratch();
    proj_keys(in0, Rin, mi, K, mk.hard);
    garble_proj_keys(K, out0, outR, mo, std::forward<F>(f), table, stride, mk);
}

// Mini projection: 16-bit payloads t16[color] = f(i) + mask16. Reference: the low 16 bits of H(K), the same
// hash the key's full-entry projection uses (projection_gate_mini.h); hardened: lane `lane` (16 bits) of the
// pad of mk.slot, a slot no full entry of the row uses.
template <class F>
inline void garble_proj_mini(const comp_t* in0, const comp_t* Rin, const ModInfo& mi, F&& f, u128* entry,
                             const Mask& mk = Mask(), int lane = 0) {
    ProjScratch& s = proj_scratch();
    const int pin = mi.p, nin = mi.n;
    DASH_CHECK(pin <= 8, "mini projection supports input moduli <= 8");
    s.key.assign(in0, in0 + nin);
    int16_t* t16 = reinterpret_cast<int16_t*>(entry);
    for (int i = 0; i < pin; ++i) {
        const u128 kc = compress(s.key.data(), mi);
        const u128 h = mk.hard ? (hard_pad(kc, mk.gate, mk.sub, mk.slot) >> (16 * lane)) : hash(kc);
        int color = s.key[0];
        t16[color] = static_cast<int16_t>(static_cast<int16_t>(f(i)) + static_cast<int16_t>(static_cast<uint16_t>(h)));
        lab_add(s.key.data(), Rin, nin, pin);
    }
}

inline int color_of(const comp_t* L, int p) { return static_cast<int>(static_cast<uint16_t>(L[0]) % static_cast<unsigned>(p)); }

// out = decompress(T[color(in) * stride] - mask(compress(in)))
inline void eval_proj(const comp_t* in, const ModInfo& mi, const u128* table, const ModInfo& mo, comp_t* out,
                      int stride = 1, const Mask& mk = Mask()) {
    const u128 kc = compress(in, mi);
    const u128 h = mk.hard ? hard_pad(kc, mk.gate, mk.sub, mk.slot) : hash(kc);
    decompress(table[static_cast<i64>(color_of(in, mi.p)) * stride] - h, out, mo);
}

inline int16_t eval_proj_mini(const comp_t* in, const ModInfo& mi, const u128* entry, const Mask& mk = Mask(),
                              int lane = 0) {
    const u128 kc = compress(in, mi);
    const u128 h = mk.hard ? (hard_pad(kc, mk.gate, mk.sub, mk.slot) >> (16 * lane)) : hash(kc);
    const int16_t* t16 = reinterpret_cast<const int16_t*>(entry);
    return static_cast<int16_t>(t16[color_of(in, mi.p)] - static_cast<int16_t>(static_cast<uint16_t>(h)));
}

// ---------------------------------------------------------------------------
// Approximate sign gadget (per element)
// ---------------------------------------------------------------------------
//
// Two constructions of the same function (SignPlan::fused):
//  * reference (fused = false): per digit d >= 1 every residue's approx label
//    (mod m_d) and the carry (mod m_d) are cast to Z_{(k+1) m_d} by identity
//    projections before the sum (sign_gadget.h:456-546): k + 1 casts per digit;
//  * fused (fused = true): the casts are folded into the projections that
//    produce their inputs. The approx projection of residue j writes digit d
//    directly as a label mod (k+1) m_d (value lut[j][v][d] < m_d), and the
//    carry projection of digit d writes (floor(s / m_d) mod m_{d-1}) directly
//    mod (k+1) m_{d-1} (mod m_0 for the last carry). The least significant
//    digit has no carry-in (the reference adds a cast of the zero label).
//    Every wire carries the same value as in the reference construction, so
//    the gadget computes the same function; it uses k (t-1) + (t-1) fewer
//    projections per element (k = 7, t = 5: 44 -> 12 hashes and table reads
//    on the evaluator side; the cast1 table disappears).
struct SignPlan {
    std::vector<int> crt, mrs, out_mod;
    int lower = 0, upper = 1;
    bool fused = false;
    std::vector<std::vector<int16_t>> lookup;  // [k][v * t + d], d = 0 is most significant
    std::vector<i64> crt_prefix;
    i64 sum_crt = 0;
    i64 n_approx = 0, n_cast = 0, n_sign = 0;  // table entries per element (n_cast: cast2; cast1 too unless fused)
    int max_n = 0;                             // largest label width touched

    SignPlan() = default;
    SignPlan(const std::vector<int>& crt_, const std::vector<int>& mrs_, const std::vector<int>& out, int lo, int up,
             bool fused = false);
    // modulus of residue j's approx output for digit d (and of the digit-d sums)
    int digit_mod(int d) const { return (fused && d >= 1) ? static_cast<int>(crt.size() + 1) * mrs[d] : mrs[d]; }
    // modulus of the carry produced by digit d >= 1 (consumed by digit d - 1)
    int carry_mod(int d) const { return fused ? ((d - 1 >= 1) ? static_cast<int>(crt.size() + 1) * mrs[d - 1] : mrs[0]) : mrs[d - 1]; }
    bool has_cast1() const { return !fused; }
};

std::vector<std::vector<int16_t>> gen_approx_lookup(const std::vector<int>& crt, const std::vector<int>& mrs);

// Garbler: in0[j] = base label of residue j (mod crt[j]); out0[o] receives the
// output base label for out_mod[o].
// hard: hardened masks (core.h Mask) with gate = the gadget's PRG stream `stream` (the evaluator passes the
// same value as `gate`); the hardened encoding needs the fused construction (no constant-keyed carry cast)
void sign_garble_elem(const SignPlan& P, const LabelBank& R, const LabelBank& Z, const Prg& prg, u64 stream,
                      const comp_t* const* in0, u128* approx, u128* cast1, u128* cast2, u128* sign,
                      comp_t* const* out0, bool hard = false);
void sign_eval_elem(const SignPlan& P, const LabelBank& Z, const comp_t* const* in, const u128* approx,
                    const u128* cast1, const u128* cast2, const u128* sign, comp_t* const* out, bool hard = false,
                    u64 gate = 0);

// ---------------------------------------------------------------------------
// Mixed-modulus half gate x (mod p) * y (mod q), q <= 8. Tables: g[p], e[q+1].
// ---------------------------------------------------------------------------
// Hardened tweaks of one mixed half gate (gate = the gadget's PRG stream): the garbler half's key x_j is row
// (TW_MMG, j); the evaluator half's key y is row (TW_MMY, 0) shared by the k residues of a ReLU (shared_y:
// residue j's entry at slot j, its mini at lane j % 8 of slot k + j / 8), or row (TW_MMY, j) of its own
// (entry at slot 0, mini at lane 0 of slot 1)
struct MMTw {
    bool hard = false;
    u64 gate = 0;
    int j = 0, k = 1;
    bool shared_y = true;
    Mask g() const { return Mask{hard, gate, tw_sub(TW_MMG, j), 0}; }
    Mask e() const { return Mask{hard, gate, tw_sub(TW_MMY, shared_y ? 0 : j), shared_y ? j : 0}; }
    Mask mini() const { return Mask{hard, gate, tw_sub(TW_MMY, shared_y ? 0 : j), shared_y ? k + j / 8 : 1}; }
    int lane() const { return shared_y ? j % 8 : 0; }
};
void mixed_mult_garble(const comp_t* x0, const ModInfo& mp, const comp_t* y0, const ModInfo& mq,
                       const LabelBank& R, const Prg& prg, u64 stream, u64& ctr, u128* g, u128* e, comp_t* out0,
                       const MMTw& tw = MMTw());
void mixed_mult_eval(const comp_t* x, const ModInfo& mp, const comp_t* y, const ModInfo& mq, const u128* g,
                     const u128* e, comp_t* out, const MMTw& tw = MMTw());

// Generalized half gate x * y, both mod p. Tables g[p], e[p].
void gen_mult_garble(const comp_t* x0, const comp_t* y0, const ModInfo& mp, const LabelBank& R, const Prg& prg,
                     u64 stream, u64& ctr, u128* g, u128* e, comp_t* out0, bool hard = false, int j = 0);
void gen_mult_eval(const comp_t* x, const comp_t* y, const ModInfo& mp, const u128* g, const u128* e, comp_t* out,
                   bool hard = false, u64 gate = 0, int j = 0);

// ---------------------------------------------------------------------------
// Base extension (ReDash MRS conversion) per element
// ---------------------------------------------------------------------------
struct BEPlan {
    std::vector<int> moduli;        // output (full) base, length E
    std::vector<int> extra;         // moduli to (re)derive
    std::vector<int> extra_idx;     // their indices in `moduli`
    std::vector<int> swapped;       // moduli order used by the MRS loop
    std::vector<int> pos_of;        // for every base index i: position in swapped
    std::vector<std::vector<i64>> inv_partial;  // [i][j] = inv(b_i) mod b_{i+j+1}
    std::vector<i64> invv;          // per extra modulus
    int nonext = 0;
    i64 n_tab = 0;                  // table entries per element
    BEPlan() = default;
    BEPlan(const std::vector<int>& moduli, const std::vector<int>& extra);
};
// L[j] are labels (mod moduli[j]) of one element, updated in place.
void be_garble_elem(const BEPlan& P, const LabelBank& R, const Prg& prg, u64 stream, u64& ctr, comp_t* const* L,
                    u128* tab, bool hard = false);
void be_eval_elem(const BEPlan& P, comp_t* const* L, const u128* tab, bool hard = false, u64 gate = 0);

// ---------------------------------------------------------------------------
// Rescale gadget (one iteration) per element.
//   legacy: factors = {2}, residue 0 recovered by a sign gadget (out {2}, 1/0)
//   redash: factors = s (subset of the CRT base), recovered by base extension
// ---------------------------------------------------------------------------
struct RescalePlan {
    std::vector<int> crt;
    std::vector<int> factors;
    std::vector<int> factor_idx;
    bool sign_be = true;
    i64 n_trans = 0;  // trans-mod entries per element
    std::vector<std::vector<int>> active;  // per factor: residues processed
    std::vector<std::vector<i64>> inv;     // per factor, per active residue: inv(s) mod p
    SignPlan sign;                         // when sign_be
    BEPlan be;                             // otherwise
    i64 n_be = 0;
    i64 sprod = 1;
    RescalePlan() = default;
    RescalePlan(const std::vector<int>& crt, const std::vector<int>& mrs, const std::vector<int>& factors, bool sign_be,
                bool fused_sign = false);
};
// Garbler: L[j] base labels (mod crt[j]) in/out; up/down are the garbler-side
// (offset-free) shift base labels.
void rescale_garble_elem(const RescalePlan& P, const LabelBank& R, const LabelBank& Z, const Prg& prg, u64 stream,
                         comp_t* const* L, const comp_t* const* up_base, const comp_t* const* down_base, u128* trans,
                         u128* s_approx, u128* s_cast1, u128* s_cast2, u128* s_sign, u128* be, bool hard = false);
void rescale_eval_elem(const RescalePlan& P, const LabelBank& Z, comp_t* const* L, const comp_t* const* up,
                       const comp_t* const* down, const u128* trans, const u128* s_approx, const u128* s_cast1,
                       const u128* s_cast2, const u128* s_sign, const u128* be, bool hard = false, u64 gate = 0);

// ---------------------------------------------------------------------------
// Single-shot mixed-radix rescale (the DASH legacy function, new construction)
//
// The legacy gadget divides by S = 2^l with l iterations of "subtract the
// mod-2 residue, halve, recover residue 0 with a sign gadget" (rescale_gadget.h
// :115-242, each iteration a full approximate sign gadget). Composed, the l
// iterations compute y = ceil(x / S) (Rescale._apply). Here the same y comes
// from one exact mixed-radix conversion:
//   x_u = (x + U) mod M with U = S - 1 + S q, U >= M/2 (U ~ M/2)
//   MRS digits a_i of x_u over the CRT base (crt[0] = 2, ascending order):
//     digit i: key K_i = L_i - sum_{l<i} P_{l,i}, a_i = (v_i + U) B_i^-1 mod p_i
//     its table row fans out P_{i,j} = a_i B_i mod p_j to every later residue j
//     and P_{i,T} = a_i B_i mod T (T = 2S) to a power-of-two label
//   r = sum_i P_{i,T} = x_u mod 2S (free additions)
//   final row (T entries): residue j >= 1: Y_j = S^-1 L_j + [(U - r mod S) S^-1 - q]
//                          residue 0:      Y_0 = [(floor(r / S) - q) mod 2]
// so y = floor(x_u / S) - q = ceil(x / S) for every x in [-M/2, M/2 - (U - M/2)):
// only the top U - M/2 < S values of the signed range wrap (they differ from
// the legacy gadget). k + 1 hashes and table reads per element on the
// evaluator instead of l sign gadgets (l = 5, k = 7: 8 instead of ~60), and
// sum_i p_i (k - i) + T k table entries instead of l (2 (k - 1) + sign).
// Table (one row per element): digit i at dig_off[i], [color][k - i] entries
// (targets: the residues of positions i+1..k-1, then T); final rows at
// fin_off, [color][k] (targets: residues 0..k-1).
//
// sign_last (the joint rescale + ReLU sign): positions convert residues
// 1..k-1 and residue 0 (mod 2) LAST, as SignMrsPlan. Its digit a_{k-1} has
// weight B_{k-1} = M/2, so a_{k-1} = [x_u >= M/2] = [x >= M/2 - U] with
// M/2 - U in (-S, 0]; with U mod 2 folded into digit 0's payload for residue
// 0, residue 0's key after the k-1 subtractions IS the label of a_{k-1}. For
// the ReLU that follows, relu(y) = y * a_{k-1} with y = ceil(x / S): y >= 1
// means x >= 1 (sign 1), y <= -1 means x <= -S (sign 0), and y = 0 gives 0
// either way, so the rescale's conversion replaces the ReLU's sign gadget.
// The last position's row has one target (T) and takes a_{k-1} as is.
struct RescaleMrsPlan {
    std::vector<int> crt;
    int l = 0;
    bool sign_last = false;
    i64 S = 1, T = 2, M = 1, U = 0, q = 0;
    std::vector<int> ord;     // position -> residue (identity, or 1..k-1, 0 with sign_last)
    std::vector<i64> B;       // B[i] = prod_{m<i} crt[ord[m]]
    std::vector<i64> Binv;    // B[i]^-1 mod crt[ord[i]]
    std::vector<i64> Sinv;    // S^-1 mod crt[j] (j >= 1)
    std::vector<i64> dig_off; // table offset of digit i's rows
    i64 fin_off = 0, n_tab = 0;
    RescaleMrsPlan() = default;
    RescaleMrsPlan(const std::vector<int>& crt, int l, bool sign_last = false);
    int k() const { return static_cast<int>(crt.size()); }
    int targets(int i) const { return k() - i; }
    // residue of target t < k-1-i of digit i (position i + 1 + t)
    int target_res(int i, int t) const { return ord[i + 1 + t]; }
    // modulus of target t of digit i (residue of position i + 1 + t, the last one T)
    int target_mod(int i, int t) const { return t == k() - 1 - i ? static_cast<int>(T) : crt[ord[i + 1 + t]]; }
    // payload value of digit i, target t, for key value v (a_i B_i reduced mod the target modulus)
    i64 digit_fn(int i, int t, i64 v) const;
    // payload value of final target j for key value v = x_u mod T
    i64 final_fn(int j, i64 v) const;
};
// L[j] (one element's labels mod crt[j]) are replaced by the rescaled labels;
// with sign_last, sig (nullable) receives the mod-2 label of a_{k-1}.
void rescale_mrs_garble_elem(const RescaleMrsPlan& P, const LabelBank& R, const Prg& prg, u64 stream,
                             comp_t* const* L, u128* tab, comp_t* sig = nullptr, bool hard = false);
void rescale_mrs_eval_elem(const RescaleMrsPlan& P, comp_t* const* L, const u128* tab, comp_t* sig = nullptr,
                           bool hard = false, u64 gate = 0);

// ---------------------------------------------------------------------------
// Exact sign by mixed-radix conversion (a construction of the ReLU/Sign
// gadget's sign; the reference approximates it, sign_gadget.h:425-581)
//
// With residue 0 = 2 converted LAST, x_u = x + M/2 = sum_i a_i B_i and the
// last digit's weight is B_{k-1} = M/2, so a_{k-1} = [x_u >= M/2] = [x >= 0]
// exactly. Positions 0..k-2 convert residues 1..k-1 (ascending); digit i's
// table row fans its value a_i B_i out to the later residues (the constant
// -M/2 is folded into digit 0's payload for residue 0), and residue 0's key
// after the k-1 subtractions IS the sign label (mod 2) - no table of its own.
// k-1 hashes on the critical path; sum_{i<k-1} p_{i+1} (k-1-i) table entries
// (k = 7: 147 instead of the approximate gadget's 568) and exact for every x.
// Rows: position i at dig_off[i], [color][k-1-i] (targets: positions i+1..k-1).
struct SignMrsPlan {
    std::vector<int> crt;
    std::vector<int> ord;      // position -> residue: 1, 2, ..., k-1, 0
    i64 M = 1, U = 0;
    std::vector<i64> B, Binv;  // per position: product of the earlier positions' moduli; its inverse mod p
    std::vector<i64> dig_off;
    i64 n_tab = 0;
    SignMrsPlan() = default;
    explicit SignMrsPlan(const std::vector<int>& crt);
    int k() const { return static_cast<int>(crt.size()); }
    int targets(int i) const { return k() - 1 - i; }
    int target_res(int i, int t) const { return ord[i + 1 + t]; }
    i64 digit_fn(int i, int t, i64 v) const;
};
// sign01 base label (mod 2) of one element with residue base labels x0; tables at tab
void sign_mrs_garble_elem(const SignMrsPlan& P, const LabelBank& R, const Prg& prg, u64 stream,
                          const comp_t* const* x0, u128* tab, comp_t* sig0, bool hard = false);
void sign_mrs_eval_elem(const SignMrsPlan& P, const comp_t* const* x, const u128* tab, comp_t* sig, bool hard = false,
                        u64 gate = 0);

}  // namespace dash
