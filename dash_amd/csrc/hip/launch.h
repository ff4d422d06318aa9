// Host-side launchers for the HIP kernels (implemented in kernels_*.hip).
#pragma once

#include <hip/hip_runtime.h>

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
                         u128* h0, uint16_t* col0, const ModC* mc, const AesGlobals& g, hipStream_t st);
void launch_rescale_update(const RescaleArgs& a, const Act& x, int B, const ModC* mc, hipStream_t st);
void launch_rescale_post(const Act& x, const CrtInfo& crt, int64_t N, int B, const u128* signP, const int16_t* down,
                         int lab_stride, const int* lab_off, const ModC* mc, hipStream_t st);
void launch_rescale_hash_sign(const u128* signP, const u128* du, int64_t N, int B, u128* h0, uint16_t* col0,
                              const AesGlobals& g, hipStream_t st);
void launch_rescale_update_approx(const RescaleArgs& r, const SignArgs& a, const Act& x, const int16_t* delta,
                                  const u128* zh, int B, const ModC* mc, const AesGlobals& g, hipStream_t st);
void launch_rescale_mrs(const MrsArgs& a, const Act& x, int B, const ModC* mc, const AesGlobals& g, hipStream_t st);
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
};
void launch_dense(const DenseArgs& a, const Act& x, const Act& y, int B, hipStream_t st);

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
};
void launch_conv(const ConvArgs& a, const Act& x, const Act& y, int B, hipStream_t st);

// k_conv_img geometry: 64-channel chunks (Cpad) and the tallest band of output
// rows whose input rows fit the 64 KiB LDS image; nbands = 0 if none fits
// (launch_conv then uses the im2col MFMA kernel).
inline void conv_img_geometry(ConvArgs& a) {
    a.Cpad = (a.C + 63) / 64 * 64;
    const int64_t row_bytes = static_cast<int64_t>(a.W + 2 * a.pw) * (a.Cpad + 16);
    int band = a.OH;
    while (band > 1 && ((band - 1) * a.sh + a.kh) * row_bytes > 65536) --band;
    for (int j = 0; j < a.crt.k; ++j) a.mq[j] = static_cast<uint32_t>(0x100000000ull / static_cast<uint32_t>(a.crt.p[j]));
    if (((band - 1) * a.sh + a.kh) * row_bytes <= 65536) {
        a.band = band;
        a.nbands = (a.OH + band - 1) / band;
    } else {
        a.band = 0;
        a.nbands = 0;
    }
}

// int16 matrix transpose out[c][r] = in[r][c] (label-major <-> component-major), kernels_label.hip
void launch_transpose16(const int16_t* in, int16_t* out, int64_t rows, int64_t cols, hipStream_t st);

}  // namespace dev
}  // namespace dash
