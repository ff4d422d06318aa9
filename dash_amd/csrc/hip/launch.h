// Host-side launchers for the HIP kernels (implemented in kernels_*.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <vector>

#include "kargs.h"

namespace dash {
namespace dev {


void launch_sign_approx(const SignArgs& a, const Act& x, const ModC* mc, const AesGlobals& g, hipStream_t st);
void launch_sign_chain(const SignArgs& a, int maxn, const ModC* mc, const AesGlobals& g, hipStream_t st);
void launch_unpack(const u128* P, int nres, const Act& out, const CrtInfo& mods, const ModC* mc, int64_t N, int B,
                   hipStream_t st);
void launch_relu_mult(const SignArgs& a, const Act& x, const Act& y, const u128* gtab, const u128* etab,
                      const ModC* mc, hipStream_t st);
void launch_rescale_hash(const Act& x, int fi, int s, const int16_t* up, int up_stride, int add_up, int64_t N, int B,
                         u128* h0, uint16_t* col0, const ModC* mc, const AesGlobals& g, hipStream_t st, int hard = 0);
void launch_rescale_update(const RescaleArgs& a, const Act& x, int B, const ModC* mc, hipStream_t st);
void launch_rescale_post(const Act& x, const CrtInfo& crt, int64_t N, int B, const u128* signP, const int16_t* down,
                         int lab_stride, const int* lab_off, const ModC* mc, hipStream_t st);
void launch_rescale_hash_sign(const u128* signP, const u128* du, int64_t N, int B, u128* h0, uint16_t* col0,
                              const AesGlobals& g, hipStream_t st);
void launch_rescale_update_approx(const RescaleArgs& r, const SignArgs& a, const Act& x, const int16_t* delta,
                                  const u128* zh, int B, const ModC* mc, const AesGlobals& g, hipStream_t st);
void launch_rescale_mrs(const MrsArgs& a, const Act& x, int B, const ModC* mc, const AesGlobals& g, hipStream_t st,
                        bool chain_only = false);
// mixed-radix chain of K residues (mrs_chain.h; instantiated per K in kernels_mrs_*.hip)
template <int K>
void launch_mrs_chain_k(const MrsArgs& a, const Act& x, int B, const ModC* mc, const AesGlobals& g, hipStream_t st);
void launch_rescale_relu_out(const MrsArgs& a, const SignArgs& sa, const Act& x, const Act& y, const u128* gtab,
                             const u128* etab, int B, const ModC* mc, const AesGlobals& g, hipStream_t st);
void launch_relu_joint(const SignArgs& sa, const Act& x, const Act& y, const u128* gtab, const u128* etab, int B,
                       const ModC* mc, const AesGlobals& g, hipStream_t st);
void launch_relu_mrs(const MrsArgs& a, const SignArgs& sa, const Act& x, const Act& y, const u128* gtab,
                     const u128* etab, int B, const ModC* mc, const AesGlobals& g, hipStream_t st);
void launch_base_ext(const BEArgs& a, const Act& x, int B, const ModC* mc, const AesGlobals& g, hipStream_t st);
void launch_proj(const ProjArgs& a, const Act& x, const Act& y, int B, const ModC* mc, const AesGlobals& g,
                 hipStream_t st);
void launch_mult(const MultArgs& a, const Act& x, const Act& y, int B, const ModC* mc, const AesGlobals& g,
                 hipStream_t st);

// label kernels (kernels_label.hip)
void launch_copy_gather(const Act& in, int64_t Nin, const Act& out, int64_t Nout, const int64_t* idx,
                        const CrtInfo& crt, int B, hipStream_t st);
void launch_pair_diff(const Act& v, int64_t Nv, const Act& d, int64_t Nout, int ops, int cnt, const CrtInfo& crt, int B,
                      hipStream_t st);
void launch_pair_add(const Act& v, int64_t Nv, const Act& r, const Act& nv, int64_t Nout, int ops, int cnt, int cnt1,
                     const CrtInfo& crt, int B, hipStream_t st);
void launch_add(const Act& x, const Act& y, int64_t N, const CrtInfo& crt, int B, hipStream_t st);
void launch_window_sum(const Act& in, int64_t Nin, const Act& out, int64_t Nout, const int64_t* idx, int K,
                       const CrtInfo& crt, int B, hipStream_t st);
void launch_aes_bench(u128* out, int blocks, int iters, const AesGlobals& g, hipStream_t st);
void launch_aes_test(const u128* in, u128* out, int64_t n, const AesGlobals& g, hipStream_t st);
void launch_hard_test(const u128* key, const uint64_t* gate, const uint32_t* sub, const uint32_t* blk, u128* out,
                      int64_t n, hipStream_t st);
void launch_codec_test(const int16_t* labels, int64_t N, int q, const ModC* mc, u128* comp, int16_t* decomp,
                       hipStream_t st);

// linear layers (kernels_gemm.hip)
struct DenseArgs {
    CrtInfo crt;
    int64_t K, O;                  // in / out features
    const int16_t* w[kMaxRes];     // [K][O] weights mod p_j (or int8 packs for MFMA)
    const int32_t* zc[kMaxRes];    // [O] zero-weight counts
    const int16_t* bias[kMaxRes];  // [B][O][n_j]
    const int16_t* zero;           // [B][lab_stride]
    int lab_stride;
    int lab_off[kMaxRes];
    const int32_t* src;            // [K] input remap (channel_tf) or null
    // MFMA path (all p <= 255): centered int8 weights [O][Kpad] with the channel_tf remap folded into the
    // column order (w8[o][src(i)] = w[o][i]), zero-padded to Kpad = 64 * ceil(K / 64); null: VALU kernel
    const int8_t* w8[kMaxRes];
    int Kpad;
};
void launch_dense(const DenseArgs& a, const Act& x, const Act& y, int B, hipStream_t st);
// builds the process-wide (residue, component) lookup the VALU dense / conv kernels index blocks with, outside
// any stream capture (HipEvaluator construction calls it)
void prepare_zmap(const CrtInfo& crt);

struct ConvArgs {
    CrtInfo crt;
    int C, H, W, F, kh, kw, sh, sw, ph, pw, OH, OW;
    const int16_t* w[kMaxRes];     // [F][C*kh*kw] weights mod p_j
    const int8_t* w8[kMaxRes];     // [F][Kpad] centered int8 (MFMA path) or null
    int Kpad;
    const int32_t* zc[kMaxRes];    // [F]
    const int16_t* bias[kMaxRes];  // [B][F][n_j]
    const int16_t* zero;           // [B][lab_stride]
    int lab_stride;
    int lab_off[kMaxRes];
    int use_mfma;
    // LDS-image MFMA path (k_conv_img): weights [F16][kh][kw][Cpad] centered int8
    const int8_t* w8r[kMaxRes];
    int Cpad = 0, band = 0, nbands = 0;
    int64_t img_off[kMaxRes + 1];  // first image index of residue j: B * sum_{i<j} n_i
    uint32_t mq[kMaxRes];          // floor(2^32 / p_j): reciprocal for the epilogue's mod p (conv_img_geometry)
    // 24-bit reduction (conv_img_geometry): x mod p = x - p * mulhi_u24(x << sh24, m24) exactly when the
    // accumulator bound keeps x << sh24 below 2^24; sh24 = -1: the 32-bit reduction
    uint32_t m24[kMaxRes];
    int sh24[kMaxRes];
    int ldsS = 0, ldsR = 0;        // LDS image: bytes per position and per input row (conv_img_geometry)
    // tap-unrolled image (conv_unroll_taps): the band is staged per OUTPUT position with the C*kh*kw patch
    // bytes as its channels, the MFMA phase then runs a 1x1 conv (one k-step instead of kh*kw for C << 64).
    // u* hold the layer's own geometry for the staging; the fields above describe the unrolled view.
    int ur = 0;
    int uC = 0, uH = 0, uW = 0, ukh = 0, ukw = 0, ush = 0, usw = 0, uph = 0, upw = 0;
};
void launch_conv(const ConvArgs& a, const Act& x, const Act& y, int B, hipStream_t st);

// k_conv_img geometry: 64-channel chunks (Cpad), the LDS image's position
// stride S and row stride R, and the tallest band of output rows whose input
// rows fit 64 KiB; nbands = 0 if none fits (launch_conv then uses the im2col
// MFMA kernel). S and R are chosen per layer by simulating the MFMA
// B-operand ds_read_b128 of the first 64 output columns over all taps under
// gfx950's banking (64 dword banks, 4 lane groups of 16:
// {0-3,12-15,20-27}, {4-11,16-19,28-31} and the same +32): 4 LDS cycles per
// read is conflict-free. The image is stored channel-last with the staging
// lanes walking channels fastest (ds_write_b32 conflict-free for any S, R).
inline int conv_lds_read_cycles(const ConvArgs& a, int S, int R) {
    static const int G[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                 {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                                 {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                                 {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
    int total = 0;
    for (int t = 0; t < 4; ++t)
        for (int dy = 0; dy < a.kh; ++dy)
            for (int dx = 0; dx < a.kw; ++dx)
                for (int g = 0; g < 4; ++g) {
                    // distinct dwords per bank: at most 16 lanes x 4 dwords land in 64 banks
                    int vals[64][16];
                    int cnt[64] = {0};
                    int worst = 1;
                    for (int i = 0; i < 16; ++i) {
                        const int l = G[g][i];
                        const int col = t * 16 + (l & 15), oy = col / a.OW, ox = col % a.OW;
                        const int base = ((oy * a.sh + dy) * R + (ox * a.sw + dx) * S + (l >> 4) * 16) / 4;
                        for (int d = 0; d < 4; ++d) {
                            const int dw = base + d, bk = dw & 63;
                            bool dup = false;
                            for (int q = 0; q < cnt[bk]; ++q) dup |= vals[bk][q] == dw;
                            if (!dup) {
                                vals[bk][cnt[bk]++] = dw;
                                worst = cnt[bk] > worst ? cnt[bk] : worst;
                            }
                        }
                    }
                    total += worst;
                }
    return total;
}

struct ConvGeomPick {
    int S, R, band, nbands;
};
inline void conv_img_geometry(ConvArgs& a) {
    a.Cpad = (a.C + 63) / 64 * 64;
    for (int j = 0; j < a.crt.k; ++j) {
        const int p = a.crt.p[j];
        a.mq[j] = static_cast<uint32_t>(0x100000000ull / static_cast<uint32_t>(p));
        // x = acc + epilogue constant < 2 * Kpad * half * xmax + (Kpad + 3) p (the epilogue's bound)
        const int half = p / 2;
        const uint64_t xmax = p < 128 ? static_cast<uint64_t>(p - 1) : static_cast<uint64_t>(half);
        const uint64_t X = 2ull * static_cast<uint64_t>(a.Kpad) * half * xmax + (static_cast<uint64_t>(a.Kpad) + 3) * p;
        // smallest sh with m = ceil(2^(32 - sh) / p) < 2^24, i.e. 2^(8 - sh) < p; then q = floor(x m / 2^(32 - sh))
        // is floor(x / p) exactly for x < 2^(24 - sh) and p < 256 (the rounding error stays below 2^-8 < 1 / p)
        a.sh24[j] = -1;
        a.m24[j] = 0;
        if (p >= 2 && p < 256) {
            int sh = 0;
            while (sh <= 8 && (1 << (8 - sh)) >= p) ++sh;
            if (sh <= 8 && X < (1ull << (24 - sh))) {
                const uint64_t m = ((1ull << (32 - sh)) + static_cast<uint64_t>(p) - 1) / static_cast<uint64_t>(p);
                if (m < (1ull << 24)) {
                    a.sh24[j] = sh;
                    a.m24[j] = static_cast<uint32_t>(m);
                }
            }
        }
    }
    // the pick depends on the layer shape only: computed once per shape and process (garbling calls this per GC)
    static std::mutex mu;
    static std::map<std::vector<int>, ConvGeomPick> memo;
    const std::vector<int> key{a.C, a.W, a.pw, a.OH, a.OW, a.kh, a.kw, a.sh, a.sw};
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = memo.find(key);
        if (it != memo.end()) {
            a.ldsS = it->second.S;
            a.ldsR = it->second.R;
            a.band = it->second.band;
            a.nbands = it->second.nbands;
            return;
        }
    }
    const int Wp = a.W + 2 * a.pw;
    // LDS budget per block (A/B knob DASH_CONV_LDS_KB, default 40: measured 64 KiB 21.0, 40 KiB 16.3, 32 KiB 17.9 ms of conv per MiniONN step at 102 GCs): smaller bands leave room for more
    // resident blocks, so one block's staging overlaps another's MFMAs
    static const int64_t budget = [] {
        const char* e = std::getenv("DASH_CONV_LDS_KB");
        const int64_t kb = e ? std::atoll(e) : 40;
        return std::max<int64_t>(8, std::min<int64_t>(64, kb)) * 1024;
    }();
    long best_cyc = -1, best_lds = 0;
    a.band = a.nbands = 0;
    for (int extra : {16, 32, 48, 80}) {
        const int S = a.Cpad + extra;
        for (int rpad = 0; rpad < 256; rpad += 16) {
            const int R = Wp * S + rpad;
            int band = a.OH;
            while (band > 1 && static_cast<int64_t>((band - 1) * a.sh + a.kh) * R > budget) --band;
            const int64_t lds = static_cast<int64_t>((band - 1) * a.sh + a.kh) * R;
            if (lds > budget) continue;
            const long cyc = conv_lds_read_cycles(a, S, R);
            if (best_cyc < 0 || cyc < best_cyc || (cyc == best_cyc && lds < best_lds)) {
                best_cyc = cyc;
                best_lds = lds;
                a.ldsS = S;
                a.ldsR = R;
                a.band = band;
                a.nbands = (a.OH + band - 1) / band;
            }
        }
    }
    std::lock_guard<std::mutex> lk(mu);
    memo[key] = ConvGeomPick{a.ldsS, a.ldsR, a.band, a.nbands};
}

// Switch a layer to the tap-unrolled image when that cuts the MFMA k-steps (few input channels, e.g. the
// RGB first layer: 3x3x3 = 27 patch bytes in one 64-wide k-step instead of 9 steps of 3 real channels each)
// and every residue takes the int8 MFMA path. Unit column stride only (the staging's 8-column loads).
// Call before conv_img_geometry; the caller lays out w8r with conv_w8r.
inline void conv_unroll_taps(ConvArgs& a, int max_p) {
    const int K = a.C * a.kh * a.kw;
    const int steps = a.kh * a.kw * ((a.C + 63) / 64), usteps = (K + 63) / 64;
    const bool ok = [] {
        const char* e = std::getenv("DASH_CONV_UNROLL");
        return !(e && e[0] == '0');
    }();
    if (!ok || a.ur || a.sw != 1 || max_p > 255 || usteps >= steps || a.uW != 0) return;
    a.ur = 1;
    a.uC = a.C; a.uH = a.H; a.uW = a.W; a.ukh = a.kh; a.ukw = a.kw;
    a.ush = a.sh; a.usw = a.sw; a.uph = a.ph; a.upw = a.pw;
    a.C = K; a.H = a.OH; a.W = a.OW;
    a.kh = a.kw = a.sh = a.sw = 1;
    a.ph = a.pw = 0;
}

// Conv kernel geometry for a layer: the tap-unrolled view where it pays (conv_unroll_taps), the LDS band
// image otherwise; when no band of the unrolled view fits the LDS budget (wide outputs, small
// DASH_CONV_LDS_KB) the layer falls back to its own geometry (plain band image, or im2col when nbands = 0).
inline void conv_plan(ConvArgs& a, int max_p, bool unroll) {
    const ConvArgs own = a;
    if (unroll) conv_unroll_taps(a, max_p);
    conv_img_geometry(a);
    if (a.ur && a.nbands == 0) {
        a = own;
        conv_img_geometry(a);
    }
}

// MFMA weight image [F16][kh][kw][Cpad] from the centered im2col weights w8 [F][Kpad] (order ci*kh*kw + dy*kw
// + dx); tap-unrolled layers: [F16][Cpad] with patch channel (dy*kw + dx)*C + ci (the staging's order)
inline std::vector<int8_t> conv_w8r(const ConvArgs& a, const std::vector<int8_t>& w8, int F) {
    const int F16 = (F + 15) / 16 * 16;
    const int C = a.ur ? a.uC : a.C, kh = a.ur ? a.ukh : a.kh, kw = a.ur ? a.ukw : a.kw;
    std::vector<int8_t> r(static_cast<size_t>(F16) * a.kh * a.kw * a.Cpad, 0);
    for (int f = 0; f < F; ++f)
        for (int ci = 0; ci < C; ++ci)
            for (int dy = 0; dy < kh; ++dy)
                for (int dx = 0; dx < kw; ++dx) {
                    const size_t dst = a.ur ? static_cast<size_t>(f) * a.Cpad + (dy * kw + dx) * C + ci
                                            : ((static_cast<size_t>(f) * kh + dy) * kw + dx) * a.Cpad + ci;
                    r[dst] = w8[static_cast<size_t>(f) * a.Kpad + (ci * kh + dy) * kw + dx];
                }
    return r;
}

// int16 matrix transpose out[c][r] = in[r][c] (label-major <-> component-major), kernels_label.hip
void launch_transpose16(const int16_t* in, int16_t* out, int64_t rows, int64_t cols, hipStream_t st);
void launch_narrow(const int16_t* in, act_t* out, int64_t n, hipStream_t st);  // int16 labels -> byte activations
void launch_encode_in(const EncIn& a, const int64_t* x, int64_t N, int slots, hipStream_t st);  // garbler: W0 + x R
void launch_transpose_to_act(const int16_t* in, act_t* out, int64_t rows, int64_t cols, hipStream_t st);
void launch_transpose_from_act(const act_t* in, int16_t* out, int64_t rows, int64_t cols, hipStream_t st);
// the same for every residue of a label set in one launch (grid z = residue): matrix j is rows[j] x cols[j]
struct TrRes {
    const void* in[kMaxRes];
    void* out[kMaxRes];
    int64_t rows[kMaxRes], cols[kMaxRes];
    int k;
};
void launch_transpose_to_act_res(const TrRes& a, hipStream_t st);    // int16 -> bytes
void launch_transpose_from_act_res(const TrRes& a, hipStream_t st);  // bytes -> int16
// elementwise casts of rows[j] * cols[j] contiguous components per residue (layouts already match)
void launch_cast_to_act_res(const TrRes& a, hipStream_t st);    // int16 -> bytes
void launch_cast_from_act_res(const TrRes& a, hipStream_t st);  // bytes -> int16
// per-slot constant scatter (HipEvaluator::load): block i copies `bytes` from src + off to dst0 + b * stride
struct ScatterDesc {
    size_t off;
    uint8_t* dst0;
    size_t stride, bytes;
};
void launch_scatter(const ScatterDesc* d, int n, const uint8_t* src, int b, hipStream_t st);
// the GPU garbler's chunked labels (component q of element e at ((q / 8) * N + e) * 8 + q % 8; rows[j] = n_j,
// cols[j] = N) <-> component-major bytes [n][N]
void launch_unchunk_to_act_res(const TrRes& a, hipStream_t st);
void launch_chunk_from_act_res(const TrRes& a, hipStream_t st);

}  // namespace dev
}  // namespace dash
