// Garbled linear layers: per-residue modular matrix products on labels.
//   out = (sum_{w != 0 mod p} w * x  +  (#zero weights) * Z_p  +  bias_label) mod p
// The (#zero weights) * Z_p term is the exact algebraic form of the
// reference's per-term "add Z when w == 0 (mod p)" quirk
// (misc/cuda_util.h:105-106, :239-244, label_tensor.h:806-808).
//
// Two conv paths:
//   * VALU (any p): one lane per output position, weights uniform (SGPR).
//   * MFMA int8 (p <= 255): implicit GEMM C[F][n] = W[F][K] * im2col(X)[K][n]
//     on v_mfma_i32_16x16x64_i8 with both operands centered into [-127, 127]
//     (products mod p are unchanged), int32 accumulation, mod-p epilogue fused
//     with the zero-count and bias-label adds. n runs over (GC, component,
//     output position) of one residue, so every residue is one large GEMM.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <type_traits>
#include <vector>

#include "host_util.h"
#include "launch.h"

namespace dash {
namespace dev {

struct ZMap {
    int j[1024];
    int c[1024];
};

__device__ __forceinline__ int32_t mod_p(int32_t v, int p) {
    v %= p;
    return v < 0 ? v + p : v;
}

// grid (ceil(O/256), 1, B*sum_n); z -> (b, j, c)
__global__ __launch_bounds__(256) void k_dense(DenseArgs a, Act x, Act y, const int* zj, const int* zcomp, int sumn) {
    const int z = blockIdx.z;
    const int b = z / sumn, r = z % sumn;
    const int j = zj[r], c = zcomp[r];
    const int64_t o = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (o >= a.O) return;
    const int p = a.crt.p[j], n = a.crt.n[j];
    const act_t* X = x.p[j] + (static_cast<int64_t>(b) * n + c) * a.K;
    const int16_t* W = a.w[j];
    int32_t acc = 0;
    for (int64_t i = 0; i < a.K; ++i) {
        const int64_t s = a.src ? a.src[i] : i;
        acc += static_cast<int32_t>(W[i * a.O + o]) * X[s];
        if ((i & 1023) == 1023) acc %= p;
    }
    const int32_t zc = a.zc[j][o];
    const int16_t zv = a.zero[static_cast<int64_t>(b) * a.lab_stride + a.lab_off[j] + c];
    const int16_t bv = a.bias[j][(static_cast<int64_t>(b) * a.O + o) * n + c];
    y.p[j][(static_cast<int64_t>(b) * n + c) * a.O + o] = static_cast<act_t>(mod_p(acc % p + zc * zv + bv, p));
}

// VALU conv: grid (ceil(OH*OW/256), F, B*sum_n)
__global__ __launch_bounds__(256) void k_conv_valu(ConvArgs a, Act x, Act y, const int* zj, const int* zcomp,
                                                   int sumn) {
    const int z = blockIdx.z;
    const int b = z / sumn, r = z % sumn;
    const int j = zj[r], c = zcomp[r];
    const int f = blockIdx.y;
    const int pos = blockIdx.x * blockDim.x + threadIdx.x;
    const int npos = a.OH * a.OW;
    if (pos >= npos) return;
    const int oy = pos / a.OW, ox = pos % a.OW;
    const int p = a.crt.p[j], n = a.crt.n[j];
    const act_t* X = x.p[j] + (static_cast<int64_t>(b) * n + c) * a.C * a.H * a.W;
    const int16_t* Wf = a.w[j] + static_cast<int64_t>(f) * a.C * a.kh * a.kw;
    const int16_t zv = a.zero[static_cast<int64_t>(b) * a.lab_stride + a.lab_off[j] + c];
    int32_t acc = 0;
    for (int ci = 0; ci < a.C; ++ci) {
        for (int dy = 0; dy < a.kh; ++dy) {
            const int iy = oy * a.sh - a.ph + dy;
            const bool rowok = iy >= 0 && iy < a.H;
            for (int dx = 0; dx < a.kw; ++dx) {
                const int ix = ox * a.sw - a.pw + dx;
                const int32_t w = Wf[(ci * a.kh + dy) * a.kw + dx];
                const int32_t v = (rowok && ix >= 0 && ix < a.W) ? X[(ci * a.H + iy) * a.W + ix] : zv;
                acc += w * v;
            }
        }
        if ((ci & 15) == 15) acc %= p;
    }
    const int32_t zc = a.zc[j][f];
    const int16_t bv = a.bias[j][(static_cast<int64_t>(b) * a.F + f) * n + c];
    y.p[j][((static_cast<int64_t>(b) * n + c) * a.F + f) * npos + pos] =
        static_cast<act_t>(mod_p(acc % p + zc * zv + bv, p));
}

// ---------------------------------------------------------------------------
// MFMA implicit-GEMM conv (int8). Block = 256 threads = 4 waves; tile =
// 64 filters x 64 columns; each wave owns a 16-filter x 64-column slab
// (4 MFMA 16x16 tiles). Columns index (gc, comp, pos) of residue j.
// A (weights) and the im2col B tile are staged in LDS per K-chunk of 64.
typedef int32_t v4i __attribute__((ext_vector_type(4)));
typedef int64_t v2l __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_conv_mfma(ConvArgs a, Act x, Act y, int j, int64_t ncols) {
    __shared__ __attribute__((aligned(16))) int8_t As[64 * 64];   // [f][k]
    __shared__ __attribute__((aligned(16))) int8_t Bs[64 * 64];   // [col][k]
    const int p = a.crt.p[j], n = a.crt.n[j];
    const int npos = a.OH * a.OW;
    const int K = a.C * a.kh * a.kw;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int64_t col0 = static_cast<int64_t>(blockIdx.x) * 64;
    const int f0 = blockIdx.y * 64;
    const int half = p / 2;
    // per-thread B-staging coordinates: thread stages column (tid & 63), k-rows (tid>>6)*16 .. +16
    const int scol = tid & 63, sk0 = (tid >> 6) * 16;
    const int64_t gcol = col0 + scol;
    int sb = 0, sc = 0, soy = 0, sox = 0;
    bool colok = gcol < ncols;
    if (colok) {
        const int64_t per_gc = static_cast<int64_t>(n) * npos;
        sb = static_cast<int>(gcol / per_gc);
        const int64_t r = gcol % per_gc;
        sc = static_cast<int>(r / npos);
        const int pos = static_cast<int>(r % npos);
        soy = pos / a.OW;
        sox = pos % a.OW;
    }
    const act_t* X = x.p[j] + (static_cast<int64_t>(sb) * n + sc) * a.C * a.H * a.W;
    const int16_t zv = colok ? a.zero[static_cast<int64_t>(sb) * a.lab_stride + a.lab_off[j] + sc] : 0;
    const int8_t* W8 = a.w8[j];
    v4i acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = v4i{0, 0, 0, 0};
    for (int k0 = 0; k0 < a.Kpad; k0 += 64) {
        // stage A: 64 filters x 64 k  (16 bytes per thread)
        {
            const int fr = tid >> 2, kc = (tid & 3) * 16;
            const int f = f0 + fr;
            v4i v = v4i{0, 0, 0, 0};
            if (f < a.F) v = *reinterpret_cast<const v4i*>(W8 + static_cast<int64_t>(f) * a.Kpad + k0 + kc);
            *reinterpret_cast<v4i*>(As + fr * 64 + kc) = v;
        }
        // stage B: im2col gather, centered int8
        {
            int8_t vals[16];
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const int kk = k0 + sk0 + t;
                int v = 0;
                if (colok && kk < K) {
                    const int ci = kk / (a.kh * a.kw), rr = kk % (a.kh * a.kw), dy = rr / a.kw, dx = rr % a.kw;
                    const int iy = soy * a.sh - a.ph + dy, ix = sox * a.sw - a.pw + dx;
                    v = (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) ? X[(ci * a.H + iy) * a.W + ix] : zv;
                    if (v > half) v -= p;
                }
                vals[t] = static_cast<int8_t>(v);
            }
            *reinterpret_cast<v4i*>(Bs + scol * 64 + sk0) = *reinterpret_cast<v4i*>(vals);
        }
        __syncthreads();
        // MFMA: wave owns filters [16*wave, +16), columns 64 (4 tiles of 16)
        // operand maps (16x16x64 i8): lane l holds A[row l&15][k = 16*(l>>4) .. +16)
        //                              and B[k = 16*(l>>4) .. +16)[col l&15]
        const v2l av = *reinterpret_cast<const v2l*>(As + (wave * 16 + (lane & 15)) * 64 + (lane >> 4) * 16);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const v2l bv = *reinterpret_cast<const v2l*>(Bs + (t * 16 + (lane & 15)) * 64 + (lane >> 4) * 16);
            acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, acc[t], 0, 0, 0);
        }
        __syncthreads();
    }
    // epilogue: C/D map col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int64_t col = col0 + t * 16 + (lane & 15);
        if (col >= ncols) continue;
        const int64_t per_gc = static_cast<int64_t>(n) * npos;
        const int b = static_cast<int>(col / per_gc);
        const int64_t rr = col % per_gc;
        const int c = static_cast<int>(rr / npos);
        const int pos = static_cast<int>(rr % npos);
        const int16_t zvv = a.zero[static_cast<int64_t>(b) * a.lab_stride + a.lab_off[j] + c];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int f = f0 + wave * 16 + (lane >> 4) * 4 + r;
            if (f >= a.F) continue;
            const int32_t zc = a.zc[j][f];
            const int16_t bv = a.bias[j][(static_cast<int64_t>(b) * a.F + f) * n + c];
            y.p[j][((static_cast<int64_t>(b) * n + c) * a.F + f) * npos + pos] =
                static_cast<act_t>(mod_p(acc[t][r] % p + zc * zvv + bv, p));
        }
    }
}


// ---------------------------------------------------------------------------
// LDS-image MFMA conv. One block = one (GC, label component) image of one
// residue and a band of output rows, 64 filters (4 waves x 16). The input
// band is staged once in LDS as centered int8 in channel-last order
// [row][x][ci] (x stride Cpad+16 bytes: conflict-free ds_read_b128 for 16
// consecutive output columns), padding positions hold the zero label's
// component. The im2col operand is then a plain 16-byte LDS read per lane
// for every (dy, dx, 64-channel chunk): no index arithmetic in the K loop.
// All residues of a layer run in one launch.
__global__ __launch_bounds__(256) void k_conv_img(ConvArgs a, Act x, Act y, int B) {
    extern __shared__ __attribute__((aligned(16))) int8_t img[];
    const int band = static_cast<int>(blockIdx.x % static_cast<unsigned>(a.nbands));
    const int64_t gimg = blockIdx.x / static_cast<unsigned>(a.nbands);
    int j = 0;
    while (j + 1 < a.crt.k && gimg >= a.img_off[j + 1]) ++j;
    if (!a.w8r[j]) return;  // residue handled by the VALU kernel (p > 255)
    const int n = a.crt.n[j], p = a.crt.p[j], half = p / 2;
    const int64_t r0 = gimg - a.img_off[j];
    const int b = static_cast<int>(r0 / n), c = static_cast<int>(r0 % n);
    const int f0 = blockIdx.y * 64;
    const int oy0 = band * a.band;
    const int oy1 = min(a.OH, oy0 + a.band);
    const int iy0 = oy0 * a.sh - a.ph;
    const int in_rows = (oy1 - oy0 - 1) * a.sh + a.kh;
    const int S = a.Cpad + 16, Wp = a.W + 2 * a.pw;
    const int HW = a.H * a.W;
    const act_t* X = x.p[j] + (static_cast<int64_t>(b) * n + c) * a.C * HW;
    const int16_t zv = a.zero[static_cast<int64_t>(b) * a.lab_stride + a.lab_off[j] + c];
    const int zc8 = zv > half ? zv - p : zv;
    const int tid = threadIdx.x;
    // stage the band: each item is a 4-channel x 4-column block transposed in
    // registers into 4 dwords (channel-last); consecutive threads walk x.
    const int c4n = a.Cpad / 4;
    const int WQ = (Wp + 3) / 4;
    const int items = in_rows * WQ * c4n;
    for (int it = tid; it < items; it += 256) {
        const int xq = it % WQ;
        const int t2 = it / WQ;
        const int yq = t2 % in_rows;
        const int c4 = t2 / in_rows;
        const int iy = iy0 + yq;
        const bool rowin = iy >= 0 && iy < a.H;
        uint32_t packed[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int ci = c4 * 4 + q;
            if (ci >= a.C) continue;
            const act_t* row = X + static_cast<int64_t>(ci) * HW + static_cast<int64_t>(iy) * a.W;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int ix = xq * 4 + t - a.pw;
                int v;
                if (rowin && ix >= 0 && ix < a.W) {
                    v = row[ix];
                    if (v > half) v -= p;
                } else {
                    v = zc8;
                }
                packed[t] |= (static_cast<uint32_t>(v) & 0xffu) << (8 * q);
            }
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int xx = xq * 4 + t;
            if (xx < Wp) *reinterpret_cast<uint32_t*>(img + (yq * Wp + xx) * S + c4 * 4) = packed[t];
        }
    }
    __syncthreads();
    const int wave = tid >> 6, lane = tid & 63;
    const int fw = f0 + wave * 16;
    if (fw >= a.F) return;  // wave-uniform; no barrier follows
    const int ncol = (oy1 - oy0) * a.OW;
    const int KK = a.kh * a.kw, CC = a.Cpad / 64;
    const int8_t* Wr = a.w8r[j] + static_cast<int64_t>(fw + (lane & 15)) * (KK * a.Cpad) + (lane >> 4) * 16;
    const int npos = a.OH * a.OW;
    const int32_t* zcp = a.zc[j];
    const int16_t* bias = a.bias[j];
    act_t* Y = y.p[j] + (static_cast<int64_t>(b) * n + c) * a.F * npos;
    for (int col0 = 0; col0 < ncol; col0 += 64) {
        v4i acc[4];
        int base[4];
        bool ok[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            acc[t] = v4i{0, 0, 0, 0};
            const int col = col0 + t * 16 + (lane & 15);
            ok[t] = col < ncol;
            const int oyl = ok[t] ? col / a.OW : 0, ox = ok[t] ? col % a.OW : 0;
            base[t] = ((oyl * a.sh) * Wp + ox * a.sw) * S + (lane >> 4) * 16;
        }
        for (int dy = 0; dy < a.kh; ++dy)
            for (int dx = 0; dx < a.kw; ++dx)
                for (int cc = 0; cc < CC; ++cc) {
                    const v2l av = *reinterpret_cast<const v2l*>(Wr + (dy * a.kw + dx) * a.Cpad + cc * 64);
                    const int off = (dy * Wp + dx) * S + cc * 64;
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const v2l bv = ok[t] ? *reinterpret_cast<const v2l*>(img + base[t] + off) : v2l{0, 0};
                        acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, acc[t], 0, 0, 0);
                    }
                }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            if (!ok[t]) continue;
            const int col = col0 + t * 16 + (lane & 15);
            const int pos = (oy0 + col / a.OW) * a.OW + col % a.OW;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int f = fw + (lane >> 4) * 4 + r;
                if (f >= a.F) continue;
                const int16_t bv = bias[(static_cast<int64_t>(b) * a.F + f) * n + c];
                Y[static_cast<int64_t>(f) * npos + pos] =
                    static_cast<act_t>(mod_p(acc[t][r] % p + zcp[f] * zv + bv, p));
            }
        }
    }
}

// ---------------------------------------------------------------------------
// k_conv_img2: k_conv_img with
//  * the wave's A operand (16 filters x all K steps) loaded once into VGPRs
//    (layers with 1, 4 or 9 k-steps of 64), instead of one 16-B global load per MFMA;
//  * the band staged with 16-B global loads (8 columns of one channel row),
//    transposed to channel-last dwords in registers;
//  * a reciprocal mod p epilogue (one reduction instead of two runtime `%`).
typedef uint32_t u32x4c __attribute__((ext_vector_type(4)));
struct __attribute__((packed, aligned(2))) Row8c {
    u32x4c v;
};
// x mod q for x < 2^(24 - sh) (launch.h sh24 / m24): q = floor(x / p) exactly from one full-rate 24-bit
// multiply-high (the 32-bit one is quarter rate), then one 24-bit multiply-add
__device__ __forceinline__ uint32_t modq_conv24(uint32_t x, int q, uint32_t m, int sh) {
    uint32_t d;
    asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(d) : "v"(x << sh), "s"(m));
    return static_cast<uint32_t>(__mul24(static_cast<int>(d), -q) + static_cast<int>(x));
}
__device__ __forceinline__ uint32_t modq_conv(uint32_t x, uint32_t q, uint32_t mq) {
    // d = floor(x / q) or one less; the remainder (< 2q < 2^24) from the low 24 bits of x - d * q, so the
    // product can be the full-rate 24-bit multiply
    const uint32_t d = __umulhi(x, mq);
    const uint32_t r = (x - __umul24(d, q)) & 0xffffffu;
    return r >= q ? r - q : r;
}

// KSC > 0: the layer has exactly KSC k-steps of 64 (taps x channel chunks), A is held in VGPRs and the
// k-step loop is fully unrolled without branches (runtime-bounded steps made the compiler shuttle the
// accumulators between AGPRs and VGPRs around every MFMA group); KSC = 0: generic streamed-A path.
#ifndef DASH_CONV_ITEMS
#define DASH_CONV_ITEMS 2
#endif
#ifndef DASH_CONV_FW
#define DASH_CONV_FW 16  // filters per wave in the MFMA phase (A/B knob: 32 feeds two MFMAs per B read, measured slower)
#endif
constexpr int kConvFW = DASH_CONV_FW;
static_assert(kConvFW == 16 || kConvFW == 32, "conv: 16 or 32 filters per wave");
#ifndef DASH_CONV_CLAMP
#define DASH_CONV_CLAMP 1  // edge items of the band staging as clamped 8-B loads (0: byte-wise, A/B)
#endif
#ifndef DASH_CONV_BRANCHFREE
#define DASH_CONV_BRANCHFREE 1  // every staging item as one clamped 8-B load + shift + mask (0: full / edge paths, A/B)
#endif
// UR: tap-unrolled band (ConvArgs::ur), a separate instantiation so the channel-chunked staging keeps its
// registers and code
template <int KSC, bool UR>
__global__ __launch_bounds__(256) void k_conv_img2(ConvArgs a, Act x, Act y, int B) {
    constexpr bool AREG = KSC > 0;
    extern __shared__ __attribute__((aligned(16))) int8_t img[];
    const int band = static_cast<int>(blockIdx.x % static_cast<unsigned>(a.nbands));
    const int64_t gimg = blockIdx.x / static_cast<unsigned>(a.nbands);
    int j = 0;
    while (j + 1 < a.crt.k && gimg >= a.img_off[j + 1]) ++j;
    if (!a.w8r[j]) return;  // residue handled by the VALU kernel (p > 255)
    const int n = a.crt.n[j], p = a.crt.p[j], half = p / 2;
    const int64_t r0 = gimg - a.img_off[j];
    const int b = static_cast<int>(r0 / n), c = static_cast<int>(r0 % n);
    const int f0 = blockIdx.y * 64;
    const int oy0 = band * a.band;
    const int oy1 = min(a.OH, oy0 + a.band);
    const int iy0 = oy0 * a.sh - a.ph;
    const int in_rows = (oy1 - oy0 - 1) * a.sh + a.kh;
    const int S = a.ldsS, R = a.ldsR, Wp = a.W + 2 * a.pw;
    // the layer's input image (the unrolled view's a.C/H/W describe the staged band, not the input)
    const int HW = UR ? a.uH * a.uW : a.H * a.W;
    const act_t* X = x.p[j] + (static_cast<int64_t>(b) * n + c) * (UR ? a.uC : a.C) * HW;
    const int16_t zv = a.zero[static_cast<int64_t>(b) * a.lab_stride + a.lab_off[j] + c];
    const int zc8 = zv > half ? zv - p : zv;
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    // Wave tiling of the block's 64 filters x 64 columns per column chunk: kConvFW filters (NG groups of 16) x
    // 16 NT columns per wave; every B operand (image) fragment read from LDS feeds NG MFMAs. 32 filters per wave
    // (half the B reads) measured slower, 2.40 -> 2.69 ms of conv per 24-GC step (132 VGPRs, 3 waves per SIMD),
    // and a build without any B reads from LDS ran no faster (2.43 ms): the conv is not LDS-read bound
    // (profiles/ab/README.md, round 3).
    constexpr int NG = kConvFW / 16, NT = 4 / NG, WF = 64 / kConvFW;
    const int wave_f = wave % WF, wave_c = wave / WF;
    const int fw = f0 + wave_f * kConvFW;  // first filter of the wave (group g: fw + 16 g)
    const int KK = a.kh * a.kw, CC = a.Cpad / 64, KS = KK * CC;
    const int8_t* Wr[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g)
        Wr[g] = a.w8r[j] + static_cast<int64_t>(fw + 16 * g + (lane & 15)) * (KK * a.Cpad) + (lane >> 4) * 16;
    // A operand into VGPRs while the band is staged (padded filter rows exist up to F16)
    v2l av[NG][AREG ? KSC : 1];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        const bool gin = fw + 16 * g < a.F;
#pragma unroll
        for (int s = 0; s < (AREG ? KSC : 1); ++s) {
            const int kk = s / CC, cc = s - kk * CC;
            av[g][s] = (AREG && gin) ? *reinterpret_cast<const v2l*>(Wr[g] + kk * a.Cpad + cc * 64) : v2l{0, 0};
        }
    }
    // epilogue constants first: their global loads are in flight with the A operand and the band staging
    // (issued after the barrier they cost a dependent round trip of their own)
    const int32_t* zcp = a.zc[j];
    const int16_t* bias = a.bias[j];
    const bool rawx = p < 128;
    // |acc| <= Kpad * half * max|x| (weights centered; x centered, or raw residues < p for p < 128);
    // off is a multiple of p above that bound (acc + off >= 0, < 2^31)
    const uint32_t xmax = static_cast<uint32_t>(rawx ? p - 1 : half);
    const uint32_t off =
        static_cast<uint32_t>(p) * (static_cast<uint32_t>(a.Kpad * half) * xmax / static_cast<uint32_t>(p) + 1);
    // col -> (output row in band, column): multiply-high by ceil(2^32 / OW) is exact for col < 2^23
    const uint32_t owm = a.OW > 1 ? 0xffffffffu / static_cast<uint32_t>(a.OW) + 1u : 0u;
    // Transposed product: the MFMA runs with the image as A and the filters as B, so a lane's 4 accumulator
    // rows are 4 consecutive output positions of ONE filter (fw + lane % 16): the epilogue stores them as one
    // dword (4 output bytes) instead of 4 byte stores, and needs one filter's constants per lane. Loaded
    // once (a dependent global load per output inside the column loop cost a round trip per 64 columns).
    uint32_t zq[NG], bq[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        const int fl = fw + 16 * g + (lane & 15);
        zq[g] = bq[g] = 0u;
        if (fl < a.F) {
            zq[g] = static_cast<uint32_t>(zcp[fl]);
            bq[g] = static_cast<uint16_t>(bias[(static_cast<int64_t>(b) * a.F + fl) * n + c]);
        }
    }
    // stage the band: item = (4 channels, 8 columns, row), channel groups fastest across lanes (the
    // channel-last dword stores of a lane group then cover consecutive banks); 4 x 8-B loads -> 8 dwords.
    // Two items per round: both items' loads are issued before either is stored (half the round trips).
    // Operands: for p < 128 the residues themselves (0..p-1 are valid int8, no conversion); otherwise
    // centered into (-p/2, p/2], four bytes at a time (SWAR). The 4 x 4 byte transposes to channel-last
    // dwords are v_perm_b32 pairs. Items that touch the padding or the image edge go byte by byte.
    const uint32_t padb = static_cast<uint32_t>(rawx ? zv : zc8) & 0xffu;
    const uint32_t ck = static_cast<uint32_t>(127 - half) * 0x01010101u;       // b > half <=> bit 7 of b + ck
    const uint32_t csub = static_cast<uint32_t>(256 - p) * 0x01010101u;         // b - p as a byte (b < p)
    auto center4 = [&](uint32_t b) -> uint32_t {
        const uint32_t hi = (b + ck) & 0x80808080u;
        const uint32_t msk = (hi - (hi >> 7)) | hi;  // 0xff in the bytes above half
        return ((b + csub) & msk) | (b & ~msk);
    };
    const int c4n = a.Cpad / 4;
    const int WO = (Wp + 7) / 8;
    const int items = in_rows * WO * c4n;
    // raw[q][h]: channel c4*4+q, columns xo*8 + 4h .. +3 (byte t = column 4h + t), final operand bytes
    // item -> (c4, xo, yq) by multiply-high with ceil(2^32 / d) (exact for item indices < 2^23; the
    // runtime divisions cost ~25 VALU each, 4 per item)
    const uint32_t mc4 = c4n > 1 ? 0xffffffffu / static_cast<uint32_t>(c4n) + 1u : 0u;
    const uint32_t mwo = WO > 1 ? 0xffffffffu / static_cast<uint32_t>(WO) + 1u : 0u;
    // tap-unrolled staging: cq -> (tap, channel), tap -> (dy, dx) the same way (cq < 2^16)
    const uint32_t muc = UR && a.uC > 1 ? 0xffffffffu / static_cast<uint32_t>(a.uC) + 1u : 0u;
    const uint32_t mkw = UR && a.ukw > 1 ? 0xffffffffu / static_cast<uint32_t>(a.ukw) + 1u : 0u;
    // 8 operand bytes of one channel row (tap-unrolled staging): columns ix0 .. ix0 + 7 of `row` (width Wr)
    auto fetch8 = [&](const act_t* row, bool rowin, int ix0, int Wr, uint32_t (&o)[2]) {
        if (Wr >= 8) {
            const int s0 = min(max(ix0, 0), Wr - 8);
            const int sh = ix0 - s0;  // > 0: right edge, < 0: left padding
            // `row` is an in-bounds row (the caller clamps it): the load is unconditional, padding rows and
            // columns are masked (no divergent load, DASH_CONV_BRANCHFREE)
            uint64_t t = *reinterpret_cast<const uint64_t*>(row + s0);
            t = sh >= 8 || sh <= -8 ? 0ull : (sh >= 0 ? t >> (8 * sh) : t << (-8 * sh));
            const int lo = max(0, -ix0), hi = min(8, Wr - ix0);  // valid bytes [lo, hi)
            const uint64_t msk = (rowin && hi > lo)
                                     ? (hi >= 8 ? ~0ull : (1ull << (8 * hi)) - 1ull) & ~((1ull << (8 * lo)) - 1ull)
                                     : 0ull;
            const uint32_t t0 = static_cast<uint32_t>(t), t1 = static_cast<uint32_t>(t >> 32);
            const uint64_t c = (static_cast<uint64_t>(rawx ? t1 : center4(t1)) << 32) | (rawx ? t0 : center4(t0));
            const uint64_t padr = static_cast<uint64_t>(padb) * 0x0101010101010101ull;
            const uint64_t v = (c & msk) | (padr & ~msk);
            o[0] = static_cast<uint32_t>(v);
            o[1] = static_cast<uint32_t>(v >> 32);
        } else {
            o[0] = o[1] = 0u;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int ix = ix0 + u;
                uint32_t v = padb;
                if (rowin && ix >= 0 && ix < Wr) {
                    const int w = row[ix];
                    v = static_cast<uint32_t>(rawx ? w : (w > half ? w - p : w)) & 0xffu;
                }
                o[u >> 2] |= v << (8 * (u & 3));
            }
        }
    };
    auto load_item = [&](int it, uint32_t (&raw)[4][2], int& yq, int& xo, int& c4) {
        const int t2 = c4n > 1 ? static_cast<int>(__umulhi(static_cast<uint32_t>(it), mc4)) : it;
        c4 = it - t2 * c4n;
        yq = WO > 1 ? static_cast<int>(__umulhi(static_cast<uint32_t>(t2), mwo)) : t2;
        xo = t2 - yq * WO;
        if constexpr (UR) {
            // tap-unrolled band: channel cq of output position (row iy0 + yq, column xo * 8 + u) is input
            // channel ci at (row * sh - ph + dy, column - pw + dx), cq = (dy * kw + dx) * C + ci (unit column
            // stride: 8 consecutive input columns)
            // (branch-free: channels past C read channel 0 and are zeroed, rows outside the image read a clamped
            // row and are masked to padding; tap / channel by multiply-high instead of runtime divisions)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int cq = c4 * 4 + q;
                const bool cin = cq < a.C;
                const uint32_t cqc = static_cast<uint32_t>(cin ? cq : 0);
                const int tap = a.uC > 1 ? static_cast<int>(__umulhi(cqc, muc)) : static_cast<int>(cqc);
                const int ci = static_cast<int>(cqc) - tap * a.uC;
                const int dy = a.ukw > 1 ? static_cast<int>(__umulhi(static_cast<uint32_t>(tap), mkw)) : tap;
                const int dx = tap - dy * a.ukw;
                const int iy = (iy0 + yq) * a.ush - a.uph + dy;
                const bool rowin = iy >= 0 && iy < a.uH;
                const int iyc = min(max(iy, 0), a.uH - 1);
                const act_t* row = X + static_cast<int64_t>(ci) * HW + static_cast<int64_t>(iyc) * a.uW;
                uint32_t o[2];
                fetch8(row, rowin, xo * 8 - a.upw + dx, a.uW, o);
                raw[q][0] = cin ? o[0] : 0u;
                raw[q][1] = cin ? o[1] : 0u;
            }
            return;
        }
        const int iy = iy0 + yq;
        const bool rowin = iy >= 0 && iy < a.H;
        const int ix0 = xo * 8 - a.pw;
        if (DASH_CONV_BRANCHFREE && a.W >= 8) {  // (uniform)
            // every item (full, edge, padding row, channel past C) as one in-bounds 8-B load at a clamped row /
            // column / channel, shifted into place and masked: no per-lane path divergence. The branching form
            // ran both the full and the edge path in most waves (the edge columns of a 32-wide image are 2 of
            // its 5 eight-column items) and its exec-mask bookkeeping made the conv issue about as many SALU
            // as VALU instructions (profiles/r05_minionn_b160_headline_pmc.txt)
            const int iyc = min(max(iy, 0), a.H - 1);
            const int s0 = min(max(ix0, 0), a.W - 8);
            const int sh = ix0 - s0;  // > 0: right edge, < 0: left padding
            const int lo = max(0, -ix0), hi = min(8, a.W - ix0);  // valid bytes [lo, hi)
            const uint64_t mrow = (rowin && hi > lo)
                                      ? (hi >= 8 ? ~0ull : (1ull << (8 * hi)) - 1ull) & ~((1ull << (8 * lo)) - 1ull)
                                      : 0ull;
            const uint64_t padr = static_cast<uint64_t>(padb) * 0x0101010101010101ull;
            const act_t* rb = X + static_cast<int64_t>(iyc) * a.W + s0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int ci = c4 * 4 + q;
                const bool cin = ci < a.C;
                uint64_t t = *reinterpret_cast<const uint64_t*>(rb + static_cast<int64_t>(cin ? ci : a.C - 1) * HW);
                t = sh >= 8 || sh <= -8 ? 0ull : (sh >= 0 ? t >> (8 * sh) : t << (-8 * sh));
                const uint32_t t0 = static_cast<uint32_t>(t), t1 = static_cast<uint32_t>(t >> 32);
                const uint64_t c = (static_cast<uint64_t>(rawx ? t1 : center4(t1)) << 32) | (rawx ? t0 : center4(t0));
                const uint64_t v = cin ? (c & mrow) | (padr & ~mrow) : 0ull;  // channels past C: zero operands
                raw[q][0] = static_cast<uint32_t>(v);
                raw[q][1] = static_cast<uint32_t>(v >> 32);
            }
            return;
        }
        const bool full = rowin && ix0 >= 0 && ix0 + 8 <= a.W;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int ci = c4 * 4 + q;
            const act_t* row = X + static_cast<int64_t>(ci) * HW + static_cast<int64_t>(iy) * a.W;
            if (ci >= a.C) {
                raw[q][0] = raw[q][1] = 0u;
            } else if (full) {
                // one 8-B load of 8 byte components (unaligned: global loads take any address on gfx950)
                typedef uint32_t u32x2c __attribute__((ext_vector_type(2)));
                const u32x2c t = *reinterpret_cast<const u32x2c*>(row + ix0);
                raw[q][0] = rawx ? t[0] : center4(t[0]);
                raw[q][1] = rawx ? t[1] : center4(t[1]);
            } else if (DASH_CONV_CLAMP && a.W >= 8) {
                // edge item: one 8-B load clamped into the row, the 8 columns shifted into place and the
                // out-of-image bytes replaced by the padding byte (branch-free; the byte-wise loop below cost
                // 8 dependent loads per channel and diverged from the wave's full items)
                const int s0 = min(max(ix0, 0), a.W - 8);
                const int sh = ix0 - s0;  // > 0: right edge, < 0: left padding
                uint64_t t = 0;
                if (rowin && sh > -8 && sh < 8) t = *reinterpret_cast<const uint64_t*>(row + s0);
                t = sh >= 8 || sh <= -8 ? 0ull : (sh >= 0 ? t >> (8 * sh) : t << (-8 * sh));
                const int lo = max(0, -ix0), hi = min(8, a.W - ix0);  // valid bytes [lo, hi)
                uint64_t msk = 0;
                if (rowin && hi > lo)
                    msk = (hi >= 8 ? ~0ull : (1ull << (8 * hi)) - 1ull) & ~((1ull << (8 * lo)) - 1ull);
                const uint32_t t0 = static_cast<uint32_t>(t), t1 = static_cast<uint32_t>(t >> 32);
                const uint64_t c = (static_cast<uint64_t>(rawx ? t1 : center4(t1)) << 32) | (rawx ? t0 : center4(t0));
                const uint64_t padr = static_cast<uint64_t>(padb) * 0x0101010101010101ull;
                const uint64_t v = (c & msk) | (padr & ~msk);
                raw[q][0] = static_cast<uint32_t>(v);
                raw[q][1] = static_cast<uint32_t>(v >> 32);
            } else {
                raw[q][0] = raw[q][1] = 0u;
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int ix = ix0 + u;
                    uint32_t v = padb;
                    if (rowin && ix >= 0 && ix < a.W) {
                        const int w = row[ix];
                        v = static_cast<uint32_t>(rawx ? w : (w > half ? w - p : w)) & 0xffu;
                    }
                    raw[q][u >> 2] |= v << (8 * (u & 3));
                }
            }
        }
    };
    auto store_item = [&](const uint32_t (&raw)[4][2], int yq, int xo, int c4) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            // [A0 B0 A1 B1], [A2 B2 A3 B3], same for C D; then column t = [A_t B_t C_t D_t]
            const uint32_t ab0 = __builtin_amdgcn_perm(raw[1][h], raw[0][h], 0x05010400u);
            const uint32_t ab1 = __builtin_amdgcn_perm(raw[1][h], raw[0][h], 0x07030602u);
            const uint32_t cd0 = __builtin_amdgcn_perm(raw[3][h], raw[2][h], 0x05010400u);
            const uint32_t cd1 = __builtin_amdgcn_perm(raw[3][h], raw[2][h], 0x07030602u);
            const uint32_t col[4] = {__builtin_amdgcn_perm(cd0, ab0, 0x05040100u), __builtin_amdgcn_perm(cd0, ab0, 0x07060302u),
                                     __builtin_amdgcn_perm(cd1, ab1, 0x05040100u), __builtin_amdgcn_perm(cd1, ab1, 0x07060302u)};
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int xx = xo * 8 + 4 * h + t;
                if (xx < Wp) *reinterpret_cast<uint32_t*>(img + yq * R + xx * S + c4 * 4) = col[t];
            }
        }
    };
    // kConvItems items per round trip: all their loads are issued before any is stored
    constexpr int kConvItems = DASH_CONV_ITEMS;
    for (int it0 = tid; it0 < items; it0 += 256 * kConvItems) {
        uint32_t v[kConvItems][4][2];
        int yq[kConvItems], xo[kConvItems], c4[kConvItems];
#pragma unroll
        for (int u = 0; u < kConvItems; ++u)
            if (it0 + 256 * u < items) load_item(it0 + 256 * u, v[u], yq[u], xo[u], c4[u]);
#pragma unroll
        for (int u = 0; u < kConvItems; ++u)
            if (it0 + 256 * u < items) store_item(v[u], yq[u], xo[u], c4[u]);
    }
    __syncthreads();
    if (fw >= a.F) return;  // wave-uniform; no barrier follows
    const int ncol = (oy1 - oy0) * a.OW;
    const int npos = a.OH * a.OW;
    uint32_t addc[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) addc[g] = off + zq[g] * static_cast<uint32_t>(zv) + bq[g];
    act_t* Y = y.p[j] + (static_cast<int64_t>(b) * n + c) * a.F * npos;
    // dword stores need 4-byte aligned filter rows and band starts, the transposed 16-byte stores 16-byte ones
    const bool dw = (npos & 3) == 0 && ((oy0 * a.OW) & 3) == 0;
    const bool dw16 = (npos & 15) == 0 && ((oy0 * a.OW) & 15) == 0 &&
                      ((reinterpret_cast<uintptr_t>(Y) & 15) == 0);
    const uint32_t mq = a.mq[j];
    const int sh24 = a.sh24[j];
    const uint32_t m24 = a.m24[j];
    // the reduction form is a compile-time choice inside the column loop, which is instantiated for both and
    // entered once (a runtime select per reduced value cost a scalar branch per output byte: the epilogue
    // issued more instructions than the MFMA phase)
    auto red = [&](auto u24, int32_t acc, uint32_t add) -> uint32_t {
        const uint32_t xv = static_cast<uint32_t>(acc) + add;
        if constexpr (decltype(u24)::value) return modq_conv24(xv, p, m24, sh24);
        else return modq_conv(xv, static_cast<uint32_t>(p), mq);
    };
    // tap offsets of the A-in-VGPR path, once per block (the k-step loop then only adds)
    int toff[AREG ? KSC : 1];
    if (AREG) {
#pragma unroll
        for (int s = 0; s < (AREG ? KSC : 1); ++s) {
            const int kk = s / CC, cc = s - kk * CC;
            const int dy = kk / a.kw, dx = kk - dy * a.kw;
            toff[s] = dy * R + dx * S + cc * 64;
        }
    }
    auto columns = [&](auto u24) {
        for (int colw = wave_c * 16 * NT; colw < ncol; colw += 64) {
            v4i acc[NG][NT];
            int base[NT];
    #pragma unroll
            for (int t = 0; t < NT; ++t) {
    #pragma unroll
                for (int g = 0; g < NG; ++g) acc[g][t] = v4i{0, 0, 0, 0};
                const int col = colw + t * 16 + (lane & 15);
                // columns past the band read column 0's operands (valid LDS); their results are never stored
                const int cl = col < ncol ? col : 0;
                const int oyl = a.OW > 1 ? static_cast<int>(__umulhi(static_cast<uint32_t>(cl), owm)) : cl;
                const int ox = cl - oyl * a.OW;
                base[t] = (oyl * a.sh) * R + (ox * a.sw) * S + (lane >> 4) * 16;
            }
            if (AREG) {
                // B operands one k-step ahead: the LDS reads of step s+1 are in flight while step s's MFMAs run
                // (one read ahead left each MFMA waiting out most of an LDS round trip)
                v2l bcur[NT], bnxt[NT];
    #define DASH_CONV_LDB(off) *reinterpret_cast<const v2l*>(img + base[t] + (off))
    #pragma unroll
                for (int t = 0; t < NT; ++t) bcur[t] = DASH_CONV_LDB(toff[0]);
    #pragma unroll
                for (int s = 0; s < (AREG ? KSC : 1); ++s) {
                    if (s + 1 < (AREG ? KSC : 1)) {
    #pragma unroll
                        for (int t = 0; t < NT; ++t) bnxt[t] = DASH_CONV_LDB(toff[(s + 1 < KSC) ? s + 1 : s]);
                    }
                    __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead (the scheduler otherwise sinks them)
    #pragma unroll
                    for (int t = 0; t < NT; ++t)
    #pragma unroll
                        for (int g = 0; g < NG; ++g)
                            acc[g][t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(bcur[t], av[g][s], acc[g][t], 0, 0, 0);
                    __builtin_amdgcn_sched_barrier(0);
    #pragma unroll
                    for (int t = 0; t < NT; ++t) bcur[t] = bnxt[t];
                }
    #undef DASH_CONV_LDB
            } else {
                for (int dy = 0; dy < a.kh; ++dy)
                    for (int dx = 0; dx < a.kw; ++dx)
                        for (int cc = 0; cc < CC; ++cc) {
                            v2l av1[NG];
    #pragma unroll
                            for (int g = 0; g < NG; ++g)
                                av1[g] = fw + 16 * g < a.F ? *reinterpret_cast<const v2l*>(Wr[g] + (dy * a.kw + dx) * a.Cpad + cc * 64)
                                                           : v2l{0, 0};
                            const int offs = dy * R + dx * S + cc * 64;
    #pragma unroll
                            for (int t = 0; t < NT; ++t) {
                                const v2l bv = *reinterpret_cast<const v2l*>(img + base[t] + offs);
    #pragma unroll
                                for (int g = 0; g < NG; ++g)
                                    acc[g][t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(bv, av1[g], acc[g][t], 0, 0, 0);
                            }
                        }
            }
    #pragma unroll
            for (int g = 0; g < NG; ++g) {
                const int fl = fw + 16 * g + (lane & 15);
                if (NT == 4 && dw16 && colw + 64 <= ncol) {
                    // whole 64-column chunk: lane (f, h) holds positions 16 t + 4 h + 0..3 of tile t as one dword; a
                    // 4x4 transpose over (t, h) with v_permlane32_swap / v_permlane16_swap gives it positions
                    // 16 h + 0..15, stored as one 16-byte store per lane (64 contiguous bytes per filter row)
                    uint32_t d[4];
    #pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        uint32_t w = 0;
    #pragma unroll
                        for (int r = 0; r < 4; ++r)
                            w |= red(u24, acc[g][t][r], addc[g]) << (8 * r);
                        d[t] = w;
                    }
                    auto r02 = __builtin_amdgcn_permlane32_swap(d[0], d[2], false, false);
                    d[0] = r02[0];
                    d[2] = r02[1];
                    auto r13 = __builtin_amdgcn_permlane32_swap(d[1], d[3], false, false);
                    d[1] = r13[0];
                    d[3] = r13[1];
                    auto r01 = __builtin_amdgcn_permlane16_swap(d[0], d[1], false, false);
                    d[0] = r01[0];
                    d[1] = r01[1];
                    auto r23 = __builtin_amdgcn_permlane16_swap(d[2], d[3], false, false);
                    d[2] = r23[0];
                    d[3] = r23[1];
                    if (fl < a.F) {
                        act_t* yr = Y + static_cast<int64_t>(fl) * npos + oy0 * a.OW + colw + 16 * (lane >> 4);
                        *reinterpret_cast<uint4*>(yr) = make_uint4(d[0], d[1], d[2], d[3]);
                    }
                    continue;
                }
                if (fl >= a.F) continue;
    #pragma unroll
                for (int t = 0; t < NT; ++t) {
                    // rows r = 0..3: positions colw + 16 t + 4 (lane / 16) + r of filter fl (band rows are whole output rows)
                    const int cb = colw + t * 16 + (lane >> 4) * 4;
                    if (cb >= ncol) continue;
                    const int pos = oy0 * a.OW + cb;
                    uint32_t o[4];
    #pragma unroll
                    for (int r = 0; r < 4; ++r)
                        o[r] = red(u24, acc[g][t][r], addc[g]);
                    act_t* yr = Y + static_cast<int64_t>(fl) * npos + pos;
                    {
                        if (dw && cb + 3 < ncol) {
                            *reinterpret_cast<uint32_t*>(yr) = o[0] | (o[1] << 8) | (o[2] << 16) | (o[3] << 24);
                        } else {
    #pragma unroll
                            for (int r = 0; r < 4; ++r)
                                if (cb + r < ncol) yr[r] = static_cast<act_t>(o[r]);
                        }
                    }
                }
            }
        }
    };
    if (sh24 >= 0) columns(std::true_type{});
    else columns(std::false_type{});
}

// ---------------------------------------------------------------------------
// Dense on MFMA: per residue j one GEMM Y[col][o] = W[o][:] . X[col][:] with
// columns col = (gc, component) of the input labels (each column is K
// contiguous bytes, component-major activations), both operands centered
// int8 (products mod p unchanged), int32 accumulation, then the mod-p
// epilogue with the (#zero weights) * Z_p term and the bias label.
// Block 256 = 4 waves; tile 64 outputs x 64 columns; wave w owns outputs
// [16w, 16w + 16) and 4 column tiles of 16. Operands come straight from
// global memory (16 B per lane per k-step: W rows stay L2-resident, X columns
// are read once), no LDS. Grid (col tiles, O tiles, residues).
__device__ __forceinline__ uint32_t center4p(uint32_t w, int p) {
    // each byte v in [0, p): v > p/2 -> v - p (two's complement byte)
    const int half = p / 2;
    uint32_t r = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        int v = static_cast<int>((w >> (8 * u)) & 0xffu);
        v = v > half ? v - p : v;
        r |= (static_cast<uint32_t>(v) & 0xffu) << (8 * u);
    }
    return r;
}

__global__ __launch_bounds__(256) void k_dense_mfma(DenseArgs a, Act x, Act y, int B) {
    const int j = blockIdx.z;
    const int p = a.crt.p[j], n = a.crt.n[j];
    const int64_t ncols = static_cast<int64_t>(B) * n;
    const int64_t col0 = static_cast<int64_t>(blockIdx.x) * 64;
    if (col0 >= ncols) return;  // block-uniform: this residue has fewer columns than the grid
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int o0 = blockIdx.y * 64 + wave * 16;
    const int K = static_cast<int>(a.K), O = static_cast<int>(a.O);
    const int8_t* W8 = a.w8[j];
    const act_t* X = x.p[j];
    const int kq = (lane >> 4) * 16;  // this lane's 16-byte k slice of each 64-wide step
    const int orow = min(o0 + (lane & 15), O - 1);  // rows past O read a valid row; their results are dropped
    int64_t cols[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) cols[t] = min(col0 + t * 16 + (lane & 15), ncols - 1);
    v4i acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = v4i{0, 0, 0, 0};
    typedef uint32_t u32x4d __attribute__((ext_vector_type(4)));
    for (int k0 = 0; k0 < a.Kpad; k0 += 64) {
        const v2l av = *reinterpret_cast<const v2l*>(W8 + static_cast<int64_t>(orow) * a.Kpad + k0 + kq);
        const int kk = k0 + kq;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            // 16 consecutive k of column cols[t]; bytes at k >= K meet zero weights (the activation buffers have
            // 64 B of slack past the last column, so the over-read stays in bounds)
            const u32x4d raw = *reinterpret_cast<const u32x4d*>(X + cols[t] * K + kk);
            u32x4d c;
#pragma unroll
            for (int u = 0; u < 4; ++u) c[u] = center4p(raw[u], p);
            v2l bv;
            __builtin_memcpy(&bv, &c, 16);
            acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, acc[t], 0, 0, 0);
        }
    }
    // epilogue: C/D map col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int64_t col = col0 + t * 16 + (lane & 15);
        if (col >= ncols) continue;
        const int b = static_cast<int>(col / n), c = static_cast<int>(col - static_cast<int64_t>(b) * n);
        const int32_t zv = a.zero[static_cast<int64_t>(b) * a.lab_stride + a.lab_off[j] + c];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int o = o0 + (lane >> 4) * 4 + r;
            if (o >= O) continue;
            const int32_t bv = a.bias[j][(static_cast<int64_t>(b) * O + o) * n + c];
            y.p[j][col * O + o] = static_cast<act_t>(mod_p(acc[t][r] % p + a.zc[j][o] * zv + bv, p));
        }
    }
}

namespace {
struct ZTab {
    int* dj = nullptr;
    int* dc = nullptr;
    int sumn = 0;
};
// process-wide, keyed by the label widths; built by prepare_zmap at evaluator construction (never inside a
// hipGraph capture: allocation and synchronous copies are not capturable)
std::mutex& ztab_mutex() {
    static std::mutex m;
    return m;
}
std::map<std::vector<int>, ZTab>& ztabs() {
    static auto* t = new std::map<std::vector<int>, ZTab>();  // leaked: device tables live as long as the process
    return *t;
}
std::vector<int> ztab_key(const CrtInfo& crt) { return std::vector<int>(crt.n, crt.n + crt.k); }
}  // namespace

void prepare_zmap(const CrtInfo& crt) {
    std::lock_guard<std::mutex> g(ztab_mutex());
    auto key = ztab_key(crt);
    if (ztabs().count(key)) return;
    ZTab t;
    for (int j = 0; j < crt.k; ++j) t.sumn += crt.n[j];
    std::vector<int> hj(t.sumn), hc(t.sumn);
    int q = 0;
    for (int j = 0; j < crt.k; ++j)
        for (int c = 0; c < crt.n[j]; ++c, ++q) {
            hj[q] = j;
            hc[q] = c;
        }
    HIPCHECK(hipMalloc(&t.dj, t.sumn * sizeof(int)));
    HIPCHECK(hipMalloc(&t.dc, t.sumn * sizeof(int)));
    HIPCHECK(hipMemcpy(t.dj, hj.data(), t.sumn * sizeof(int), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(t.dc, hc.data(), t.sumn * sizeof(int), hipMemcpyHostToDevice));
    ztabs().emplace(std::move(key), t);
}

namespace {
const ZTab& ztab_for(const CrtInfo& crt) {
    std::lock_guard<std::mutex> g(ztab_mutex());
    auto it = ztabs().find(ztab_key(crt));
    DASH_CHECK(it != ztabs().end(), "prepare_zmap was not called for this CRT base");
    return it->second;
}
}  // namespace

void launch_dense(const DenseArgs& a, const Act& x, const Act& y, int B, hipStream_t st) {
    if (a.w8[0]) {
        int maxn = 0;
        for (int j = 0; j < a.crt.k; ++j) maxn = max(maxn, a.crt.n[j]);
        dim3 g(static_cast<unsigned>((static_cast<int64_t>(B) * maxn + 63) / 64), static_cast<unsigned>((a.O + 63) / 64),
               static_cast<unsigned>(a.crt.k));
        hipLaunchKernelGGL(k_dense_mfma, g, dim3(256), 0, st, a, x, y, B);
        return;
    }
    const ZTab& z = ztab_for(a.crt);
    dim3 g(static_cast<unsigned>((a.O + 255) / 256), 1, static_cast<unsigned>(B * z.sumn));
    hipLaunchKernelGGL(k_dense, g, dim3(256), 0, st, a, x, y, z.dj, z.dc, z.sumn);
}

void launch_conv(const ConvArgs& a, const Act& x, const Act& y, int B, hipStream_t st) {
    if (a.use_mfma && a.nbands > 0) {
        const int64_t nimg = a.img_off[a.crt.k];
        const int in_rows = (min(a.band, a.OH) - 1) * a.sh + a.kh;
        const size_t lds = static_cast<size_t>(in_rows) * a.ldsR;
        dim3 g(static_cast<unsigned>(nimg * a.nbands), static_cast<unsigned>((a.F + 63) / 64), 1);
        static const int ver = [] {
            const char* e = std::getenv("DASH_CONV_IMG_VER");
            return e ? std::atoi(e) : 2;
        }();
        const int KS = a.kh * a.kw * (a.Cpad / 64);
        if (ver == 1 && a.ldsS == a.Cpad + 16 && a.ldsR == (a.W + 2 * a.pw) * a.ldsS)
            hipLaunchKernelGGL(k_conv_img, g, dim3(256), lds, st, a, x, y, B);  // A/B: its fixed layout only
        else if (a.ur && KS == 1)
            hipLaunchKernelGGL((k_conv_img2<1, true>), g, dim3(256), lds, st, a, x, y, B);
        else if (a.ur)
            hipLaunchKernelGGL((k_conv_img2<0, true>), g, dim3(256), lds, st, a, x, y, B);
        else if (KS == 9)
            hipLaunchKernelGGL((k_conv_img2<9, false>), g, dim3(256), lds, st, a, x, y, B);
        else if (KS == 4)
            hipLaunchKernelGGL((k_conv_img2<4, false>), g, dim3(256), lds, st, a, x, y, B);
        else if (KS == 1)
            hipLaunchKernelGGL((k_conv_img2<1, false>), g, dim3(256), lds, st, a, x, y, B);
        else
            hipLaunchKernelGGL((k_conv_img2<0, false>), g, dim3(256), lds, st, a, x, y, B);
        bool rest = false;
        for (int j = 0; j < a.crt.k; ++j) rest |= (a.w8r[j] == nullptr);
        if (!rest) return;
    } else if (a.use_mfma) {
        for (int j = 0; j < a.crt.k; ++j) {
            if (!a.w8[j]) continue;
            const int64_t ncols = static_cast<int64_t>(B) * a.crt.n[j] * a.OH * a.OW;
            dim3 g(static_cast<unsigned>((ncols + 63) / 64), static_cast<unsigned>((a.F + 63) / 64), 1);
            hipLaunchKernelGGL(k_conv_mfma, g, dim3(256), 0, st, a, x, y, j, ncols);
        }
        // residues without an int8 image (p > 255) fall through to VALU below
        bool rest = false;
        for (int j = 0; j < a.crt.k; ++j) rest |= (a.w8[j] == nullptr);
        if (!rest) return;
    }
    const ZTab& z = ztab_for(a.crt);
    dim3 g(static_cast<unsigned>((a.OH * a.OW + 255) / 256), static_cast<unsigned>(a.F), static_cast<unsigned>(B * z.sumn));
    hipLaunchKernelGGL(k_conv_valu, g, dim3(256), 0, st, a, x, y, z.dj, z.dc, z.sumn);
}

}  // namespace dev
}  // namespace dash
