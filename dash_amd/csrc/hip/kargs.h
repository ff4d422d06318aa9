// Kernel argument structs shared by the HIP kernels and the host runtime.
#pragma once

#include <stdint.h>

#include "dev.h"

namespace dash {
namespace dev {

constexpr int kMaxRes = 16;   // max CRT residues on the GPU path
constexpr int kMaxMrs = 16;
constexpr int kMaxOut = 16;

// Label components of activations are stored as bytes: every modulus of the
// GPU path is < 256 (CRT primes, ReDash bases <= 173, power-of-two moduli <=
// 128), so each streaming kernel moves half the bytes of int16 labels. Tables,
// constant labels and the host format stay int16.
typedef uint8_t act_t;
constexpr int kActMaxModulus = 255;

// Residue-major activation description: act[j] -> act_t [B][n_j][N]
struct Act {
    act_t* p[kMaxRes];
    int64_t N;  // elements per GC
};

struct CrtInfo {
    int k;
    int p[kMaxRes];
    int n[kMaxRes];
    int prefix[kMaxRes];
    int sum;
};

// Garbler-side input encoding on the device (k_encode_in), per slot s:
// out_j[s][c][e] = W0_j[s][c][e] + (x[s][e] mod p_j) R_j[s][c] mod p_j
struct EncIn {
    int k;
    int p[kMaxRes];
    int n[kMaxRes];
    const act_t* w0[kMaxRes];  // [n_j][N] component-major input base labels
    const act_t* r[kMaxRes];   // [n_j] the offset R_{p_j}
    act_t* out[kMaxRes];       // [n_j][N] an evaluator slot's input activations (slot s + 1 follows n_j N later)
    int64_t wstride;           // bytes between the encoder slots' W0 / R blocks (grid z = slot)
    // set by launch_encode_in: component prefix of residue j (pre[k] = total) and 1 / p_j
    int pre[kMaxRes + 1];
    float inv[kMaxRes];
};

struct SignArgs {
    CrtInfo crt;
    int t;
    int mrs[kMaxMrs];
    int nout;
    int out_mod[kMaxOut];
    int64_t N;           // elements
    int B;
    int64_t n_approx, n_cast, n_sign;  // table entries per element
    const u128* approx;  // [B][N][n_approx]
    const u128* cast1;   // [B][N][n_cast]
    const u128* cast2;
    const u128* sign;    // [B][N][n_sign]
    u128* mrsP;          // [B][k][t][N] compressed approx outputs
    u128* hx;            // [B][k][N] H(compress(x_j)) (ReLU reuse) - may be null
    uint16_t* colx;      // [B][k][N]
    u128* outP;          // [B][nout][N] compressed sign outputs
    u128* hs;            // [B][N] H(compress(sign mod 2)) when relu != 0
    uint8_t* cs;         // [B][N]
    const u128* zc;      // [B][zc_stride] compressed zero labels, indexed by modulus
    const uint16_t* zcol;  // [B][zc_stride] zero-label colors
    int zc_stride;
    int relu;            // also produce hs / cs for the ReLU multiply
    int16_t* csum;       // [B][t][kCsumComps][N] per-digit sums of the k cast labels (phase B1)
    int64_t c1off[kMaxMrs];  // offset of digit d's block ((k+1) m_d entries) in a cast1 row
    int fused;           // SignPlan::fused: approx outputs are already cast, carries come out cast (no cast1)
    // hardened encoding (dev.h hard_block): hx holds the ReLU garbler half gates' pads, ys the sign label's
    // evaluator-half pads [B][ny][N] (slots 0..k-1 the residues' entries, k.. the packed mini lanes)
    int hard;
    uint64_t sgate0, mgate0;  // gate bases of the sign gadget / the mixed-mult gadget (dev.h gate_base)
    int ny;
    u128* ys;
};
constexpr int kCsumComps = 64;

struct RescaleArgs {
    CrtInfo crt;
    int64_t N;
    int fi, s;
    int add_up;
    int active[kMaxRes];   // 1 if residue is processed by this factor
    int aidx[kMaxRes];     // index among active residues (table offset / s)
    int inv[kMaxRes];      // s^-1 mod p_j
    int64_t n_trans, off;  // entries per element, offset of this factor
    const u128* trans;     // [B][N][n_trans]
    const u128* h0;
    const uint16_t* col0;
    const int16_t* up;     // [B][sum n] per-GC upshift labels (residue-concatenated)
    const int16_t* zero;   // [B][sum n] zero labels of the CRT moduli
    int lab_stride;        // sum_j n_j
    int lab_off[kMaxRes];  // offset of residue j inside up/zero rows
    int hard;              // hardened encoding: trans pads (TW_TRANS, factor) instead of H
    uint64_t gate0;
    int factor;            // index of this factor (the trans row's tweak)
};

// Single-shot mixed-radix rescale (gadgets.h RescaleMrsPlan)
struct MrsArgs {
    CrtInfo crt;
    int T;                         // 2^(l+1): modulus of the x_u mod 2S label (power of two)
    int64_t N, n_tab;
    const u128* tab;               // [B][N][n_tab]
    int64_t dig_off[kMaxRes];      // digit i rows: [color][k - i]
    int64_t fin_off;               // final rows: [color][k]
    int sinv[kMaxRes];             // S^-1 mod p_j (j >= 1)
    u128 hmask;                    // top bit of every log2(T)-bit field (packed mod-T additions)
    u128* pf;                      // [B][k][N] final payloads (chain -> output kernel)
    u128* ps;                      // [B][k(k-1)/2][N] digit payloads for later positions (chain scratch)
    int mode;                      // 0: rescale (position i = residue i, T accumulator, final row -> pf)
                                   // 1: sign (position i = residue (i + 1) mod k; the last key is sign01 -> hs, cs)
                                   // 2: rescale in mode 1's order, the mod-2 key is also the next ReLU's sign
    u128* hs;                      // modes 1, 2: [B][N] hash of the sign label
    uint8_t* cs;                   // modes 1, 2: [B][N] its color
    u128* hx;                      // mode 2: [B][k][N] H(compress(Y_j)) of the outputs (the next ReLU's keys)
    uint16_t* colx;                // mode 2: [B][k][N] their colors
    // hardened encoding (the only one of the mixed-radix constructions): row pads instead of H
    uint64_t gate0;   // this gadget's gate base (rescale: stream slot 30, sign: slot 1)
    uint64_t rgate0;  // modes 1, 2: the ReLU mixed-mult gadget's gate base (its y-row / g-row pads)
    int ny;           // y-row pad slots per element (k entries + packed minis)
    u128* ys;         // modes 1, 2: [B][ny][N] the sign label's y-row pads
    int qpack;        // k_mrs_chain_q: bit 0 four digits per quad reduction (moduli <= 63); >> 1: positions
                      // I < that value take chunk-split keys
};

struct BEArgs {
    int E, nonext;
    int swapped[kMaxRes];    // moduli in MRS order
    int src[kMaxRes];        // residue index of position i
    int inv[kMaxRes][kMaxRes];  // inv_partial[i][j]
    int nextra;
    int extra_pos[kMaxRes];  // position (in swapped order) of extra residue x
    int extra_res[kMaxRes];  // residue index of extra x
    int invv[kMaxRes];
    int64_t N, n_tab;
    const u128* tab;         // [B][N][n_tab]
    int16_t* work;
    int hard;
    uint64_t gate0;
};

struct ProjArgs {
    int k;
    int pin[kMaxRes], pout[kMaxRes];
    const u128* tab[kMaxRes];  // [B][N][pin_j]
    int64_t N;
    int hard;
    uint64_t gate0;
};

struct MultArgs {
    CrtInfo crt;
    int64_t No;  // outputs per GC
    int q;       // 0 = same-modulus multiply, else mixed with modulus q
    const u128* t;  // [B][No][sum]   (mixed only)
    const u128* g;  // [B][No][sum]
    const u128* e;  // same: [B][No][sum]; mixed: [B][No][k][q+1]
    int hard;
    uint64_t gate0;
};

}  // namespace dev
}  // namespace dash
