// Gadget kernels for gfx950: approximate sign (3 phases), ReLU multiply,
// rescale (legacy sign-BE and ReDash base extension), projection and
// multiplication test gates.
//
// Work decomposition (vs the reference's one-stream-per-residue launches,
// sign_gadget.h:737-795, garbled_relu.h:258-294):
//   phase A  one lane per (GC, residue, element): ONE hash per input label,
//            reused for all |mrs| approx projections and later for the ReLU
//            garbler half-gate (the reference hashes the same key |mrs|+1
//            times); outputs stay compressed (u128).
//   phase B  one lane per (GC, element): the serial mixed-radix carry chain,
//            fully in registers, no device malloc (reference uses new[]).
//   phase C  one lane per (GC, residue, element): ReLU mixed-mod multiply, no
//            AES at all (hashes come from phases A/B).
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "gadget_common.h"

namespace dash {
namespace dev {


// ---------------------------------------------------------------------------
// Phase A tail: the casts Z_{m_d} -> Z_{(k+1) m_d} of residue j's approx
// labels for every digit d >= 1. They do not depend on the carry, so they run
// here, in the lane that just produced the approx labels (still in registers):
// all cast gathers are issued before the paired AES. mrsP[b][j][d] receives
// the approx label for d = 0 and its cast for d >= 1 (phase B1 only sums).
// P[d] = approx label of digit d for d < TM; digits >= TM (t > TM) are
// recomputed from the approx row TA at color `col` (key H).
template <int TM>
__device__ __forceinline__ void approx_casts_out(const AesCtx& aes, const SignArgs& a, const ModC* mc, int j, int b,
                                                 int64_t e, const u128 (&P)[TM], const u128* TA, uint32_t col, u128 H) {
    const int64_t N = a.N;
    const int t = a.t;
    u128* out = a.mrsP + (static_cast<int64_t>(b) * a.crt.k + j) * t * N + e;
    if (a.fused) {
        // fused construction: the approx row already holds every digit in its summation modulus
#pragma unroll
        for (int d = 0; d < TM; ++d)
            if (d < t) out[static_cast<int64_t>(d) * N] = P[d];
        for (int d = TM; d < t; ++d) out[static_cast<int64_t>(d) * N] = TA[col * t + d] - H;
        return;
    }
    const u128* T1 = a.cast1 + (static_cast<int64_t>(b) * N + e) * a.n_cast;
    out[0] = P[0];
    u128 tt[TM];
#pragma unroll
    for (int d = 1; d < TM; ++d)
        if (d < t) {
            const int m = a.mrs[d];
            tt[d] = T1[a.c1off[d] + static_cast<int64_t>(j) * m + u128_mod(P[d], mc[m])];
        }
#pragma unroll
    for (int d = 1; d < TM; d += 2) {
        if (d < t) {
            const bool two = (d + 1 < TM) && (d + 1 < t);
            const u128 PB = (d + 1 < TM) ? P[(d + 1 < TM) ? d + 1 : d] : static_cast<u128>(0);
            u128 HA, HB = 0;
            if (two)
                aes_encrypt2(aes, P[d], PB, HA, HB);
            else
                HA = aes_encrypt(aes, P[d]);
            out[static_cast<int64_t>(d) * N] = tt[d] - HA;
            if (two) out[static_cast<int64_t>(d + 1) * N] = tt[(d + 1 < TM) ? d + 1 : d] - HB;
        }
    }
    for (int d = TM; d < t; ++d) {
        const int m = a.mrs[d];
        const u128 Pd = TA[col * t + d] - H;
        const u128 Td = T1[a.c1off[d] + static_cast<int64_t>(j) * m + u128_mod(Pd, mc[m])];
        out[static_cast<int64_t>(d) * N] = Td - aes_encrypt(aes, Pd);
    }
}

// Phase A: approximate residues + their casts. grid (x, k, B)
template <int TM>
__global__ __launch_bounds__(kAesBlock, kSignApproxMinWaves) void k_sign_approx(SignArgs a, Act x, const ModC* mc, const uint32_t* te0,
                                                     const uint32_t* rk) {
    AES_PROLOGUE(te0, rk);
    const int j = blockIdx.y, b = blockIdx.z;
    const int64_t N = a.N;
    for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < N;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int p = a.crt.p[j];
        const ModC m = mc[p];
        const act_t* L = x.p[j] + static_cast<int64_t>(b) * m.n * N + e;
        const uint32_t col = static_cast<uint16_t>(L[0]) % static_cast<uint32_t>(p);
        const u128* T =
            a.approx + (static_cast<int64_t>(b) * N + e) * a.n_approx + static_cast<int64_t>(a.t) * a.crt.prefix[j];
        // issue the table gathers first: their HBM latency hides under the AES
        u128 P[TM];
#pragma unroll
        for (int d = 0; d < TM; ++d)
            if (d < a.t) P[d] = T[col * a.t + d];
        const u128 C = compress_cm<kSignApproxChunk>(L, N, m);
        const int64_t bke = (static_cast<int64_t>(b) * a.crt.k + j) * N + e;
        if (a.hard) {
            // hardened (fused only): digit d's entry under pad d of (C, sign gate, (TW_APPROX, j)); the ReLU's garbler
            // half gate keyed by the same label gets its own pad (mixed-mult gate, (TW_MMG, j))
            const uint64_t sg = a.sgate0 ^ static_cast<uint64_t>(e);
            u128* out = a.mrsP + (static_cast<int64_t>(b) * a.crt.k + j) * a.t * N + e;
            for (int blk = 0; 4 * blk < a.t; ++blk) {
                u128 pd[4];
                hard_block(C, sg, tw_sub(kTwApprox, j), static_cast<uint32_t>(blk), pd);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int d = 4 * blk + q;
                    if (d < a.t) out[static_cast<int64_t>(d) * N] = T[col * a.t + d] - pd[q];
                }
            }
            if (a.hx) {
                a.hx[bke] = hard_pad(C, a.mgate0 ^ static_cast<uint64_t>(e), tw_sub(kTwMmg, j), 0);
                a.colx[bke] = static_cast<uint16_t>(col);
            }
            continue;
        }
        const u128 H = aes_encrypt(aes, C);
        if (a.hx) {
            a.hx[bke] = H;
            a.colx[bke] = static_cast<uint16_t>(col);
        }
#pragma unroll
        for (int d = 0; d < TM; ++d)
            if (d < a.t) P[d] -= H;
        approx_casts_out<TM>(aes, a, mc, j, b, e, P, T, col, H);
    }
}

// ---------------------------------------------------------------------------
// Phase B1: per MRS digit, the component-wise sum over residues j of the
// phase-A outputs (casts mod (k+1) m_d for d >= 1, approx labels mod m_0 for
// d = 0). No AES and no LDS, so it runs at full occupancy.
// grid (ceil(N/256), t, B): blockIdx.y = t-1 is digit 0, otherwise digit y+1.
template <int MAXN>
__global__ __launch_bounds__(256) void k_sign_castsum(SignArgs a, const ModC* mc) {
    const int b = blockIdx.z;
    const int k = a.crt.k, t = a.t;
    const int d = (static_cast<int>(blockIdx.y) == t - 1) ? 0 : static_cast<int>(blockIdx.y) + 1;
    const int64_t N = a.N;
    const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (e >= N) return;
    const int m = a.mrs[d];
    const int mo = d ? (k + 1) * m : m;
    const ModC Mo = mc[mo];
    const u128* P0 = a.mrsP + (static_cast<int64_t>(b) * k * t + d) * N + e;
    int32_t acc[MAXN];
#pragma unroll
    for (int i = 0; i < MAXN; ++i) acc[i] = 0;
    u128 nk = P0[0];
    for (int j = 0; j < k; ++j) {
        DigitStream s;
        s.init(nk);
        if (j + 1 < k) nk = P0[static_cast<int64_t>(j + 1) * t * N];
#pragma unroll
        for (int i = 0; i < MAXN; ++i)
            if (i < static_cast<int>(Mo.n)) acc[i] += static_cast<int32_t>(s.next(Mo));
    }
    int16_t* S = a.csum + ((static_cast<int64_t>(b) * t + d) * kCsumComps) * N + e;
#pragma unroll
    for (int i = 0; i < MAXN; ++i)
        if (i < static_cast<int>(Mo.n)) S[i * N] = static_cast<int16_t>(modq(static_cast<uint32_t>(acc[i]), Mo));
}

// ---------------------------------------------------------------------------
// Phase B2: the serial mixed-radix carry chain + sign projection. Per digit
// only the carry's cast and the sum's cast2 projection remain on the
// critical path (2 AES + 2 gathers). grid (x, 1, B)
template <int MAXN>
__global__ __launch_bounds__(kAesBlock, kAesMinBlocks) void k_sign_chain(SignArgs a, const ModC* mc, const uint32_t* te0,
                                                    const uint32_t* rk) {
    AES_PROLOGUE(te0, rk);
    const int b = blockIdx.z;
    const int64_t N = a.N;
    const int k = a.crt.k, t = a.t;
    for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < N;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const u128* T1 = a.cast1 + (static_cast<int64_t>(b) * N + e) * a.n_cast;
        const u128* T2 = a.cast2 + (static_cast<int64_t>(b) * N + e) * a.n_cast;
        const int16_t* S = a.csum + static_cast<int64_t>(b) * t * kCsumComps * N + e;
        const int mlast = a.mrs[t - 1];
        u128 carry = a.zc[static_cast<int64_t>(b) * a.zc_stride + mlast];
        uint32_t ccol = a.zcol[static_cast<int64_t>(b) * a.zc_stride + mlast];
        int64_t c1 = 0, c2 = 0;
        int32_t acc[MAXN];
        for (int d = t - 1; d >= 1; --d) {
            const int m = a.mrs[d];
            const int mo = (k + 1) * m;
            const ModC Mo = mc[mo];
            const u128 TA = T1[c1 + static_cast<int64_t>(k) * m + ccol];
            const int16_t* Sd = S + static_cast<int64_t>(d) * kCsumComps * N;
#pragma unroll
            for (int i = 0; i < MAXN; ++i)
                if (i < static_cast<int>(Mo.n)) acc[i] = Sd[i * N];
            const u128 HA = aes_encrypt(aes, carry);
            c1 += static_cast<int64_t>(k + 1) * m;
            DigitStream sa;
            sa.init(TA - HA);
            CompressFwd cf;
            cf.init();
            uint32_t col2 = 0;
#pragma unroll
            for (int i = 0; i < MAXN; ++i)
                if (i < static_cast<int>(Mo.n)) {
                    uint32_t v = static_cast<uint32_t>(acc[i]) + sa.next(Mo);
                    if (v >= static_cast<uint32_t>(mo)) v -= mo;
                    if (i == 0) col2 = v;
                    cf.push(v, Mo);
                }
            const u128 key2 = cf.finish();
            const u128 T2e = T2[c2 + col2];
            const u128 H2 = aes_encrypt(aes, key2);
            carry = T2e - H2;
            c2 += mo;
            ccol = u128_mod(carry, mc[a.mrs[d - 1]]);
        }
        // most significant digit: sum = carry + sum_j mrs[j][0] (the latter from phase B1)
        const int m0 = a.mrs[0];
        const ModC M0 = mc[m0];
        DigitStream sc;
        sc.init(carry);
        CompressFwd cf;
        cf.init();
        uint32_t col = 0;
#pragma unroll
        for (int i = 0; i < MAXN; ++i)
            if (i < static_cast<int>(M0.n)) {
                uint32_t v = static_cast<uint32_t>(S[i * N]) + sc.next(M0);
                if (v >= static_cast<uint32_t>(m0)) v -= m0;
                if (i == 0) col = v;
                cf.push(v, M0);
            }
        const u128 key = cf.finish();
        const u128* TS = a.sign + (static_cast<int64_t>(b) * N + e) * a.n_sign;
        const u128 TS0 = TS[col];
        const u128 H = aes_encrypt(aes, key);
        for (int o = 0; o < a.nout; ++o) {
            const u128 P = (o == 0 ? TS0 : TS[o * m0 + col]) - H;
            a.outP[(static_cast<int64_t>(b) * a.nout + o) * N + e] = P;
            if (a.relu && o == 0) {
                a.hs[static_cast<int64_t>(b) * N + e] = aes_encrypt(aes, P);
                a.cs[static_cast<int64_t>(b) * N + e] = static_cast<uint8_t>(static_cast<uint32_t>(P) & 1u);
            }
        }
    }
}

// Phase B2 of the fused construction (SignPlan::fused): the carry leaves each
// carry projection already in the next digit's summation modulus, so a digit
// costs ONE dependent gather + ONE AES on the critical path (the reference
// construction: two of each). The least significant digit has no carry-in.
// grid (x, 1, B)
template <int MAXN>
__global__ __launch_bounds__(kAesBlock, kAesMinBlocks) void k_sign_chain_fused(SignArgs a, const ModC* mc,
                                                                               const uint32_t* te0, const uint32_t* rk) {
    AES_PROLOGUE(te0, rk);
    const int b = blockIdx.z;
    const int64_t N = a.N;
    const int k = a.crt.k, t = a.t;
    for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < N;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const u128* T2 = a.cast2 + (static_cast<int64_t>(b) * N + e) * a.n_cast;
        const int16_t* S = a.csum + static_cast<int64_t>(b) * t * kCsumComps * N + e;
        u128 carry = 0;
        int64_t c2 = 0;
        int32_t acc[MAXN];
        for (int d = t - 1; d >= 1; --d) {
            const int mo = (k + 1) * a.mrs[d];
            const ModC Mo = mc[mo];
            const int16_t* Sd = S + static_cast<int64_t>(d) * kCsumComps * N;
#pragma unroll
            for (int i = 0; i < MAXN; ++i)
                if (i < static_cast<int>(Mo.n)) acc[i] = Sd[i * N];
            const bool have = d < t - 1;
            DigitStream sa;
            sa.init(carry);
            CompressFwd cf;
            cf.init();
            uint32_t col2 = 0;
#pragma unroll
            for (int i = 0; i < MAXN; ++i)
                if (i < static_cast<int>(Mo.n)) {
                    uint32_t v = static_cast<uint32_t>(acc[i]);
                    if (have) {
                        v += sa.next(Mo);
                        if (v >= static_cast<uint32_t>(mo)) v -= mo;
                    }
                    if (i == 0) col2 = v;
                    cf.push(v, Mo);
                }
            const u128 key2 = cf.finish();
            const u128 T2e = T2[c2 + col2];
            carry = T2e - (a.hard ? hard_pad(key2, a.sgate0 ^ static_cast<uint64_t>(e), tw_sub(kTwCast2, d), 0)
                                  : aes_encrypt(aes, key2));
            c2 += mo;
        }
        const int m0 = a.mrs[0];
        const ModC M0 = mc[m0];
        const bool have = t >= 2;
        DigitStream sc;
        sc.init(carry);
        CompressFwd cf;
        cf.init();
        uint32_t col = 0;
#pragma unroll
        for (int i = 0; i < MAXN; ++i)
            if (i < static_cast<int>(M0.n)) {
                uint32_t v = static_cast<uint32_t>(S[i * N]);
                if (have) {
                    v += sc.next(M0);
                    if (v >= static_cast<uint32_t>(m0)) v -= m0;
                }
                if (i == 0) col = v;
                cf.push(v, M0);
            }
        const u128 key = cf.finish();
        const u128* TS = a.sign + (static_cast<int64_t>(b) * N + e) * a.n_sign;
        const u128 TS0 = TS[col];
        const u128 H = a.hard ? 0 : aes_encrypt(aes, key);
        const uint64_t sg = a.sgate0 ^ static_cast<uint64_t>(e);
        for (int o = 0; o < a.nout; ++o) {
            const u128 P = (o == 0 ? TS0 : TS[o * m0 + col]) - (a.hard ? hard_pad(key, sg, tw_sub(kTwSign, 0), o) : H);
            a.outP[(static_cast<int64_t>(b) * a.nout + o) * N + e] = P;
            if (a.relu && o == 0) {
                if (a.hard) {  // the sign label's y-row pads (ReLU evaluator half gates + minis)
                    const uint64_t mg = a.mgate0 ^ static_cast<uint64_t>(e);
                    for (int blk = 0; 4 * blk < a.ny; ++blk) {
                        u128 pd[4];
                        hard_block(P, mg, tw_sub(kTwMmy, 0), static_cast<uint32_t>(blk), pd);
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            if (4 * blk + q < a.ny) a.ys[(static_cast<int64_t>(b) * a.ny + 4 * blk + q) * N + e] = pd[q];
                    }
                } else {
                    a.hs[static_cast<int64_t>(b) * N + e] = aes_encrypt(aes, P);
                }
                a.cs[static_cast<int64_t>(b) * N + e] = static_cast<uint8_t>(static_cast<uint32_t>(P) & 1u);
            }
        }
    }
}

// Decompress compressed outputs into residue activations. grid (ceil(N/256), nres, B)
__global__ __launch_bounds__(256) void k_unpack(const u128* P, int nres, Act out, CrtInfo mods, const ModC* mc,
                                                int64_t N) {
    const int j = blockIdx.y, b = blockIdx.z;
    const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (e >= N) return;
    const ModC m = mc[mods.p[j]];
    DigitStream s;
    s.init(P[(static_cast<int64_t>(b) * nres + j) * N + e]);
    act_t* o = out.p[j] + static_cast<int64_t>(b) * m.n * N + e;
    for (int i = 0; i < static_cast<int>(m.n); ++i) o[i * N] = static_cast<act_t>(s.next(m));
}

// ---------------------------------------------------------------------------
// Phase C: ReLU = x * sign01(x) via the mixed-modulus half gate.
// grid (ceil(N/256), k, B)
__global__ __launch_bounds__(256) void k_relu_mult(SignArgs a, Act x, Act y, const u128* gtab, const u128* etab,
                                                   const ModC* mc) {
    const int j = blockIdx.y, b = blockIdx.z;
    const int64_t N = a.N;
    const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (e >= N) return;
    const int k = a.crt.k;
    const int p = a.crt.p[j];
    const ModC m = mc[p];
    const int64_t bke = (static_cast<int64_t>(b) * k + j) * N + e;
    const u128 Hx = a.hx[bke];
    const uint32_t colx = a.colx[bke];
    const uint32_t cS = a.cs[static_cast<int64_t>(b) * N + e];
    const int64_t be = static_cast<int64_t>(b) * N + e;
    // reference: one H(sign label) masks all k entries and minis; hardened: entry j under y-row pad j, mini j
    // under lane j % 8 of pad k + j / 8 (MMTw, gadgets.h)
    const u128 HS = a.hard ? a.ys[(static_cast<int64_t>(b) * a.ny + j) * N + e] : a.hs[be];
    const u128 HM = a.hard ? (a.ys[(static_cast<int64_t>(b) * a.ny + k + j / 8) * N + e] >> (16 * (j % 8))) : HS;
    const u128 G = gtab[be * a.crt.sum + a.crt.prefix[j] + colx] - Hx;
    const u128* E3 = etab + (be * k + j) * 3;
    const u128 E = E3[cS] - HS;
    const u128 mini = E3[2];
    const int16_t t16 = static_cast<int16_t>(static_cast<uint16_t>(mini >> (16 * cS)));
    const int16_t ypr16 = static_cast<int16_t>(t16 - static_cast<int16_t>(static_cast<uint16_t>(HM)));
    const uint32_t ypr = modq(static_cast<uint32_t>(static_cast<int32_t>(ypr16) + (p << 15)), m);  // p*2^15 > |ypr16|
    const act_t* X = x.p[j] + static_cast<int64_t>(b) * m.n * N + e;
    act_t* Y = y.p[j] + static_cast<int64_t>(b) * m.n * N + e;
    DigitStream sg, se;
    sg.init(G);
    se.init(E);
    const int n = static_cast<int>(m.n);
    // the next chunk's loads go out before this chunk's stores: vmcnt retires in issue order, so a
    // load issued after a store would also wait for that store
    uint16_t cur[kChunk], nxt[kChunk];
#pragma unroll
    for (int u = 0; u < kChunk; ++u)
        if (u < n) cur[u] = X[static_cast<int64_t>(u) * N];
    for (int i0 = 0; i0 < n; i0 += kChunk) {
#pragma unroll
        for (int u = 0; u < kChunk; ++u)
            if (i0 + kChunk + u < n) nxt[u] = X[static_cast<int64_t>(i0 + kChunk + u) * N];
#pragma unroll
        for (int u = 0; u < kChunk; ++u)
            if (i0 + u < n) {
                const uint32_t g = sg.next(m);
                const uint32_t ev = se.next(m);
                // all terms in [0, p): ev + ypr * x + (p - g) < p^2 + 2p
                Y[static_cast<int64_t>(i0 + u) * N] =
                    static_cast<act_t>(modq(ev + ypr * static_cast<uint32_t>(cur[u]) + static_cast<uint32_t>(p) - g, m));
            }
#pragma unroll
        for (int u = 0; u < kChunk; ++u) cur[u] = nxt[u];
    }
}

// k_relu_mult with the label staged in LDS (stage_ok): a block = (256-element tile, residue j, GC b); the
// per-element gathers go out first, the block's x_j rows come in as 16-byte loads, each lane rewrites its
// column in place and the block stores the y_j rows back as 16-byte stores.
constexpr int kRmBS = 256;
__global__ __launch_bounds__(kRmBS) void k_relu_mult_s(SignArgs a, Act x, Act y, const u128* gtab, const u128* etab,
                                                       const ModC* mc) {
    __shared__ __attribute__((aligned(16))) uint8_t stg[128 * kRmBS];
    const int j = blockIdx.y, b = blockIdx.z;
    const int64_t N = a.N;
    const int tid = static_cast<int>(threadIdx.x);
    const int k = a.crt.k;
    const int p = a.crt.p[j];
    const ModC m = mc[p];
    const int n = static_cast<int>(m.n);
    const act_t* X = x.p[j] + static_cast<int64_t>(b) * n * N;
    act_t* Y = y.p[j] + static_cast<int64_t>(b) * n * N;
    for (int64_t e0 = static_cast<int64_t>(blockIdx.x) * kRmBS; e0 < N; e0 += static_cast<int64_t>(gridDim.x) * kRmBS) {
        const int64_t e = min(e0 + tid, N - 1);
        const int64_t bke = (static_cast<int64_t>(b) * k + j) * N + e;
        const int64_t be = static_cast<int64_t>(b) * N + e;
        const u128 Hx = a.hx[bke];
        const uint32_t colx = a.colx[bke];
        const u128 HS = a.hard ? a.ys[(static_cast<int64_t>(b) * a.ny + j) * N + e] : a.hs[be];
        const u128 HM = a.hard ? (a.ys[(static_cast<int64_t>(b) * a.ny + k + j / 8) * N + e] >> (16 * (j % 8))) : HS;
        const uint32_t cS = a.cs[be];
        const u128* E3 = etab + (be * k + j) * 3;
        const u128 Graw = gtab[be * a.crt.sum + a.crt.prefix[j] + colx];
        const u128 Eraw = E3[cS];
        const u128 mini = E3[2];
        __syncthreads();  // the previous tile's stores have read the image
        lds_stage_rows<kRmBS, 4>(stg, X, N, e0, 0, n);
        __syncthreads();
        const u128 G = Graw - Hx, E = Eraw - HS;
        const int16_t t16 = static_cast<int16_t>(static_cast<uint16_t>(mini >> (16 * cS)));
        const int16_t ypr16 = static_cast<int16_t>(t16 - static_cast<int16_t>(static_cast<uint16_t>(HM)));
        const uint32_t ypr = modq(static_cast<uint32_t>(static_cast<int32_t>(ypr16) + (p << 15)), m);
        if (m.bits == 1) {
            // p = 2 (the residue with the most components, 128): the digits of G and E are their bits, and
            // (e + ypr x + 2 - g) mod 2 = e ^ g ^ (ypr & x): one bit extract and two logic ops per component
            // instead of two 128-bit digit shifts and a reduction
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const uint32_t ge = static_cast<uint32_t>(G >> (32 * w)) ^ static_cast<uint32_t>(E >> (32 * w));
#pragma unroll 8
                for (int u = 0; u < 32; ++u) {
                    const int c = 32 * w + u;
                    if (c >= n) break;
                    uint8_t& v = stg[c * kRmBS + tid];
                    v = static_cast<uint8_t>(((ge >> u) & 1u) ^ (static_cast<uint32_t>(v) & ypr));
                }
            }
        } else if (m.bits) {
            DigitStream sg, se;
            sg.init(G);
            se.init(E);
            for (int c = 0; c < n; ++c) {
                const uint32_t g = sg.next(m);
                const uint32_t ev = se.next(m);
                uint8_t& v = stg[c * kRmBS + tid];
                v = static_cast<uint8_t>(modq(ev + ypr * static_cast<uint32_t>(v) + static_cast<uint32_t>(p) - g, m));
            }
        } else {  // chunk-major (chunk_digit): one divmod per stream per chunk, uniform digit loops
            u128 QG = G, QE = E;
            for (int c0 = 0; c0 < n; c0 += static_cast<int>(m.c)) {
                uint32_t rg = divmod128(QG, m), re = divmod128(QE, m);
                const int cnt = min(static_cast<int>(m.c), n - c0);
                for (int t = 0; t < cnt; ++t) {
                    const uint32_t g = chunk_digit(rg, m);
                    const uint32_t ev = chunk_digit(re, m);
                    uint8_t& v = stg[(c0 + t) * kRmBS + tid];
                    v = static_cast<uint8_t>(modq(ev + ypr * static_cast<uint32_t>(v) + static_cast<uint32_t>(p) - g, m));
                }
            }
        }
        __syncthreads();
        lds_store_rows<kRmBS>(Y, stg, N, e0, 0, n);
    }
}

// ---------------------------------------------------------------------------
// Rescale step 1+2 for one factor: hash the factor residue (optionally after
// the upshift). grid (ceil(N/256), 1, B)
__global__ __launch_bounds__(kAesBlock, kAesMinBlocks) void k_rescale_hash(Act x, int fi, int s, const int16_t* up, int up_stride,
                                                      int add_up, int64_t N, u128* h0, uint16_t* col0,
                                                      const ModC* mc, const uint32_t* te0, const uint32_t* rk,
                                                      int hard) {
    AES_PROLOGUE(te0, rk);
    const int b = blockIdx.z;
    for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < N;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const ModC m = mc[s];
    const act_t* L = x.p[fi] + static_cast<int64_t>(b) * m.n * N + e;
    const int16_t* U = up + static_cast<int64_t>(b) * up_stride;
    // compress of (L + up) mod s, streamed from the least significant component
    CompressFwd cf;
    cf.init();
    uint32_t c0 = 0;
    const int n = static_cast<int>(m.n);
    for (int i0 = 0; i0 < n; i0 += kChunk) {
        uint16_t lv[kChunk];
#pragma unroll
        for (int u = 0; u < kChunk; ++u)
            if (i0 + u < n) lv[u] = static_cast<uint16_t>(L[(i0 + u) * N]);
#pragma unroll
        for (int u = 0; u < kChunk; ++u)
            if (i0 + u < n) {
                uint32_t d = lv[u];
                if (add_up) {
                    d += static_cast<uint16_t>(U[i0 + u]);
                    if (d >= static_cast<uint32_t>(s)) d -= s;
                }
                if (i0 + u == 0) c0 = d;
                cf.push(d, m);
            }
    }
    // hardened: the key itself (each active residue's update lane derives its own pad, k_rescale_update)
    h0[static_cast<int64_t>(b) * N + e] = hard ? cf.finish() : aes_encrypt(aes, cf.finish());
    col0[static_cast<int64_t>(b) * N + e] = static_cast<uint16_t>(c0);
    }
}


// grid (ceil(N/256), k, B)
__global__ __launch_bounds__(256) void k_rescale_update(RescaleArgs a, Act x, const ModC* mc) {
    const int j = blockIdx.y, b = blockIdx.z;
    const int64_t N = a.N;
    const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (e >= N) return;
    const int p = a.crt.p[j];
    const ModC m = mc[p];
    act_t* L = x.p[j] + static_cast<int64_t>(b) * m.n * N + e;
    const int16_t* U = a.up + static_cast<int64_t>(b) * a.lab_stride + a.lab_off[j];
    if (j == a.fi) {
        const int16_t* Zl = a.zero + static_cast<int64_t>(b) * a.lab_stride + a.lab_off[j];
        for (int i = 0; i < static_cast<int>(m.n); ++i) L[i * N] = Zl[i];
        return;
    }
    if (!a.active[j]) return;  // residue of an earlier factor (already zero)
    const int64_t be = static_cast<int64_t>(b) * N + e;
    const u128 mask = a.hard ? hard_pad(a.h0[be], a.gate0 ^ static_cast<uint64_t>(e), tw_sub(kTwTrans, a.factor), a.aidx[j])
                             : a.h0[be];
    const u128 P = a.trans[be * a.n_trans + a.off + static_cast<int64_t>(a.aidx[j]) * a.s + a.col0[be]] - mask;
    DigitStream s;
    s.init(P);
    const int32_t inv = a.inv[j];
    const int n = static_cast<int>(m.n);
    for (int i0 = 0; i0 < n; i0 += kChunk) {
        int16_t lv[kChunk];
#pragma unroll
        for (int u = 0; u < kChunk; ++u)
            if (i0 + u < n) lv[u] = L[(i0 + u) * N];
#pragma unroll
        for (int u = 0; u < kChunk; ++u)
            if (i0 + u < n) {
                uint32_t v = static_cast<uint32_t>(lv[u]) + static_cast<uint32_t>(p) - s.next(m);  // [1, 2p)
                if (a.add_up) v += static_cast<uint32_t>(U[i0 + u]);
                L[(i0 + u) * N] = static_cast<act_t>(modq(v * static_cast<uint32_t>(inv), m));
            }
    }
}

// Downshift (and, for sign base extension, install the recovered mod-2 residue).
// grid (ceil(N/256), k, B)
__global__ __launch_bounds__(256) void k_rescale_post(Act x, CrtInfo crt, int64_t N, const u128* signP,
                                                      const int16_t* down, int lab_stride, const int* lab_off,
                                                      const ModC* mc) {
    const int j = blockIdx.y, b = blockIdx.z;
    const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (e >= N) return;
    const int p = crt.p[j];
    const ModC m = mc[p];
    act_t* L = x.p[j] + static_cast<int64_t>(b) * m.n * N + e;
    const int16_t* D = down + static_cast<int64_t>(b) * lab_stride + lab_off[j];
    const int n = static_cast<int>(m.n);
    if (j == 0 && signP) {
        DigitStream s;
        s.init(signP[static_cast<int64_t>(b) * N + e]);
        for (int i = 0; i < n; ++i) {
            int32_t v = static_cast<int32_t>(s.next(m)) - D[i];
            L[i * N] = static_cast<act_t>(v < 0 ? v + p : v);
        }
        return;
    }
    for (int i0 = 0; i0 < n; i0 += kChunk) {
        int16_t lv[kChunk], dv[kChunk];
#pragma unroll
        for (int u = 0; u < kChunk; ++u)
            if (i0 + u < n) {
                lv[u] = L[(i0 + u) * N];
                dv[u] = D[i0 + u];
            }
#pragma unroll
        for (int u = 0; u < kChunk; ++u)
            if (i0 + u < n) {
                const int32_t v = lv[u] - dv[u];
                L[(i0 + u) * N] = static_cast<act_t>(v < 0 ? v + p : v);
            }
    }
}


// ---------------------------------------------------------------------------
// Legacy (DASH) rescale, fused per iteration:
//   hash   : residue-0 key from the previous iteration's sign payload bits
//            (mod-2 labels: +/- is XOR, so no decompress at all)
//   update : L_j = (L_j + delta_j - proj(L_0)) * 2^-1 streamed digit by digit,
//            compressed on the fly and hashed -> approx projections of the
//            next sign gadget (phase A) in the same pass.
// The downshift of iteration i and the upshift of i+1 collapse into one
// delta = up - down; only the last iteration writes a downshifted result.
__global__ __launch_bounds__(kAesBlock, kAesMinBlocks) void k_rescale_hash_sign(const u128* signP, const u128* du, int64_t N, u128* h0,
                                                           uint16_t* col0, const uint32_t* te0, const uint32_t* rk) {
    AES_PROLOGUE(te0, rk);
    const int b = blockIdx.z;
    for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < N;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const u128 C = signP[static_cast<int64_t>(b) * N + e] ^ du[b];
    h0[static_cast<int64_t>(b) * N + e] = aes_encrypt(aes, C);
    col0[static_cast<int64_t>(b) * N + e] = static_cast<uint16_t>(static_cast<uint32_t>(C) & 1u);
    }
}

// grid (x, k, B). Each component chunk is one dependent HBM round trip (the
// in-place stores keep the next chunk's loads behind them), so the chunk size
// sets the round trips per label; the t approx entries stay live across the
// loop, so larger chunks need the 128-VGPR budget (free here: the 64 KiB AES
// image already limits a CU to 16 waves).
#ifndef DASH_UA_CHUNK
#define DASH_UA_CHUNK 4
#endif
// the mixed-radix chain keeps K-1 digit streams live: at 6 waves/SIMD (80 VGPRs) it spills 240 B per
// lane; 4 waves/SIMD with 128 VGPRs measured faster (6.36 vs 7.04 ms per 24-GC MiniONN step)
constexpr int kChunkUA = DASH_UA_CHUNK;
// CH: components per dependent round trip. Latency-bound launches (batch 1, few waves per SIMD) take 16 (the
// label's n / 4 round trips, 32 for the 128 components of p = 2, were the floor of a small launch)
template <int TM, int CH>
__global__ __launch_bounds__(kAesBlock, DASH_UA_MINBLOCKS) void k_rescale_update_approx(RescaleArgs r, SignArgs a, Act x, const int16_t* delta,
                                                               const u128* zh, const ModC* mc, const uint32_t* te0,
                                                               const uint32_t* rk) {
    AES_PROLOGUE(te0, rk);
    const int j = blockIdx.y, b = blockIdx.z;
    const int64_t N = r.N;
    for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < N;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int p = r.crt.p[j];
    const ModC m = mc[p];
    const int64_t be = static_cast<int64_t>(b) * N + e;
    const u128* TA = a.approx + be * a.n_approx + static_cast<int64_t>(a.t) * a.crt.prefix[j];
    u128 H;
    uint32_t col;
    u128 ent[TM];
    if (j == r.fi) {
        // factor residue is the zero label: constant key per GC
        H = zh[static_cast<int64_t>(b) * a.zc_stride + p];
        col = a.zcol[static_cast<int64_t>(b) * a.zc_stride + p];
#pragma unroll
        for (int d = 0; d < TM; ++d)
            if (d < a.t) ent[d] = TA[col * a.t + d];
    } else {
        const u128 Tt = r.trans[be * r.n_trans + static_cast<int64_t>(r.aidx[j]) * r.s + r.col0[be]];
        const u128 P = Tt - r.h0[be];
        act_t* L = x.p[j] + static_cast<int64_t>(b) * m.n * N + e;
        const int16_t* Dl = delta + static_cast<int64_t>(b) * r.lab_stride + r.lab_off[j];
        DigitStream s;
        s.init(P);
        CompressFwd cf;
        cf.init();
        const int32_t inv = r.inv[j];
        col = 0;
        const int n = static_cast<int>(m.n);
        for (int i0 = 0; i0 < n; i0 += CH) {
            int16_t lv[CH], dv[CH];
#pragma unroll
            for (int u = 0; u < CH; ++u)
                if (i0 + u < n) {
                    lv[u] = L[(i0 + u) * N];
                    dv[u] = Dl[i0 + u];
                }
#pragma unroll
            for (int u = 0; u < CH; ++u)
                if (i0 + u < n) {
                    // lv, dv, digit in [0, p): the sum is in [1, 3p), (sum * inv) mod p in one reduction
                    const uint32_t v = modq((static_cast<uint32_t>(lv[u]) + static_cast<uint32_t>(dv[u]) +
                                             static_cast<uint32_t>(p) - s.next(m)) * static_cast<uint32_t>(inv), m);
                    L[(i0 + u) * N] = static_cast<act_t>(v);
                    cf.push(v, m);
                    if (i0 + u == 0) {
                        col = static_cast<uint32_t>(v);
#pragma unroll
                        for (int d = 0; d < TM; ++d)
                            if (d < a.t) ent[d] = TA[col * a.t + d];
                    }
                }
        }
        H = aes_encrypt(aes, cf.finish());
    }
#pragma unroll
    for (int d = 0; d < TM; ++d)
        if (d < a.t) ent[d] -= H;
    approx_casts_out<TM>(aes, a, mc, j, b, e, ent, TA, col, H);
    }
}



void launch_rescale_hash_sign(const u128* signP, const u128* du, int64_t N, int B, u128* h0, uint16_t* col0,
                              const AesGlobals& g, hipStream_t st) {
    hipLaunchKernelGGL(k_rescale_hash_sign, AES_LAUNCH(N, 1, B), kAesLds, st, signP, du, N, h0, col0, g.te0, g.rk);
}
void launch_rescale_update_approx(const RescaleArgs& r, const SignArgs& a, const Act& x, const int16_t* delta,
                                  const u128* zh, int B, const ModC* mc, const AesGlobals& g, hipStream_t st) {
    // DASH_UA_SMALL=0 keeps the throughput chunk on small launches (A/B)
    static const bool small_on = [] {
        const char* e = std::getenv("DASH_UA_SMALL");
        return !(e && e[0] == '0');
    }();
    // at most two waves per SIMD: the lanes are serial chains of round trips
    const bool small = small_on && r.N * r.crt.k * B <= static_cast<int64_t>(2 * 4 * 64) * num_cus();
    if (a.t <= 5 && small)
        hipLaunchKernelGGL((k_rescale_update_approx<5, 16>), AES_LAUNCH(r.N, r.crt.k, B), kAesLds, st, r, a, x,
                           delta, zh, mc, g.te0, g.rk);
    else if (a.t <= 5)
        hipLaunchKernelGGL((k_rescale_update_approx<5, kChunkUA>), AES_LAUNCH(r.N, r.crt.k, B), kAesLds, st, r, a, x,
                           delta, zh, mc, g.te0, g.rk);
    else if (small)
        hipLaunchKernelGGL((k_rescale_update_approx<8, 16>), AES_LAUNCH(r.N, r.crt.k, B), kAesLds, st, r, a, x,
                           delta, zh, mc, g.te0, g.rk);
    else
        hipLaunchKernelGGL((k_rescale_update_approx<8, kChunkUA>), AES_LAUNCH(r.N, r.crt.k, B), kAesLds, st, r, a,
                           x, delta, zh, mc, g.te0, g.rk);
}



// Output: Y_0 = pf_0 (mod 2), Y_j = S^-1 L_j + pf_j (mod p_j), in place. grid (ceil(N/256), k, B)
__global__ __launch_bounds__(256) void k_rescale_mrs_out(MrsArgs a, Act x, const ModC* mc) {
    const int j = blockIdx.y, b = blockIdx.z;
    const int64_t N = a.N;
    const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (e >= N) return;
    const int k = a.crt.k;
    const ModC m = mc[a.crt.p[j]];
    const int n = static_cast<int>(m.n);
    act_t* L = x.p[j] + static_cast<int64_t>(b) * n * N + e;
    DigitStream s;
    s.init(a.pf[(static_cast<int64_t>(b) * k + j) * N + e]);
    if (j == 0) {
        for (int c = 0; c < n; ++c) L[static_cast<int64_t>(c) * N] = static_cast<act_t>(s.next(m));
        return;
    }
    const uint32_t inv = static_cast<uint32_t>(a.sinv[j]);
    // loads of group c+1 before the stores of group c (as k_relu_mult); 16-digit groups: this kernel runs one
    // short serial walk per lane (batch-1 launches are latency-bound), so fewer, deeper round trips
    constexpr int kG = 2 * kChunk;
    uint16_t cur[kG], nxt[kG];
#pragma unroll
    for (int u = 0; u < kG; ++u)
        if (u < n) cur[u] = L[static_cast<int64_t>(u) * N];
    for (int c0 = 0; c0 < n; c0 += kG) {
#pragma unroll
        for (int u = 0; u < kG; ++u)
            if (c0 + kG + u < n) nxt[u] = L[static_cast<int64_t>(c0 + kG + u) * N];
#pragma unroll
        for (int u = 0; u < kG; ++u)
            if (c0 + u < n)
                L[static_cast<int64_t>(c0 + u) * N] = static_cast<act_t>(modq(cur[u] * inv + s.next(m), m));  // < p^2 + p
#pragma unroll
        for (int u = 0; u < kG; ++u) cur[u] = nxt[u];
    }
}

// Joint rescale + ReLU (MODE 2): the output kernel also produces the next ReLU's garbler half-gate keys
// hx[b][j][e] = H(compress(Y_j)), colx = color (k_label_hash's job) from the components it writes, so the
// rescaled labels are not read back. Residue 0's output is the decompressed payload, its compress the payload.
__global__ __launch_bounds__(kAesBlock, kAesMinBlocks) void k_rescale_mrs_out_hash(MrsArgs a, Act x, const ModC* mc,
                                                                                  const uint32_t* te0,
                                                                                  const uint32_t* rk) {
    (void)te0;
    (void)rk;
    const int j = blockIdx.y, b = blockIdx.z;
    const int64_t N = a.N;
    const int k = a.crt.k;
    const ModC m = mc[a.crt.p[j]];
    const int n = static_cast<int>(m.n);
    for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < N;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        act_t* L = x.p[j] + static_cast<int64_t>(b) * n * N + e;
        const int64_t bke = (static_cast<int64_t>(b) * k + j) * N + e;
        const u128 P = a.pf[bke];
        DigitStream s;
        s.init(P);
        if (j == 0) {
            uint32_t c0 = 0;
            for (int c = 0; c < n; ++c) {
                const uint32_t v = s.next(m);
                if (c == 0) c0 = v;
                L[static_cast<int64_t>(c) * N] = static_cast<act_t>(v);
            }
            a.colx[bke] = static_cast<uint16_t>(c0);
            a.hx[bke] = hard_pad(P, a.rgate0 ^ static_cast<uint64_t>(e), tw_sub(kTwMmg, 0), 0);  // next ReLU g row
            continue;
        }
        const uint32_t inv = static_cast<uint32_t>(a.sinv[j]);
        CompressFwd cf;
        cf.init();
        uint32_t c0 = 0;
        uint16_t cur[kChunk], nxt[kChunk];
#pragma unroll
        for (int u = 0; u < kChunk; ++u)
            if (u < n) cur[u] = L[static_cast<int64_t>(u) * N];
        for (int q0 = 0; q0 < n; q0 += kChunk) {
#pragma unroll
            for (int u = 0; u < kChunk; ++u)
                if (q0 + kChunk + u < n) nxt[u] = L[static_cast<int64_t>(q0 + kChunk + u) * N];
#pragma unroll
            for (int u = 0; u < kChunk; ++u)
                if (q0 + u < n) {
                    const uint32_t v = modq(cur[u] * inv + s.next(m), m);  // < p^2 + p
                    if (q0 + u == 0) c0 = v;
                    L[static_cast<int64_t>(q0 + u) * N] = static_cast<act_t>(v);
                    cf.push(v, m);
                }
#pragma unroll
            for (int u = 0; u < kChunk; ++u) cur[u] = nxt[u];
        }
        a.colx[bke] = static_cast<uint16_t>(c0);
        a.hx[bke] = hard_pad(cf.finish(), a.rgate0 ^ static_cast<uint64_t>(e), tw_sub(kTwMmg, j), 0);
    }
}

// k_rescale_mrs_out_hash with the label staged in LDS (stage_ok): a block = (512-element tile, residue j,
// GC b) walks the label kOhCap components per pass: stage the rows, each lane rewrites its column in place,
// store the rows back (residue 0 only writes the decompressed payload).
constexpr int kOhBS = 512;
constexpr int kOhCap = 40;  // 20 KiB image beside the 32 KiB AES image: three blocks per CU
__global__ __launch_bounds__(kOhBS, kAesMinBlocks) void k_rescale_mrs_out_hash_s(MrsArgs a, Act x, const ModC* mc,
                                                                               const uint32_t* te0, const uint32_t* rk) {
    (void)te0;
    (void)rk;
    __shared__ __attribute__((aligned(16))) uint8_t stg[kOhCap * kOhBS];
    const int j = blockIdx.y, b = blockIdx.z;
    const int64_t N = a.N;
    const int k = a.crt.k;
    const ModC m = mc[a.crt.p[j]];
    const int n = static_cast<int>(m.n);
    const int tid = static_cast<int>(threadIdx.x);
    act_t* L = x.p[j] + static_cast<int64_t>(b) * n * N;
    const uint32_t inv = static_cast<uint32_t>(a.sinv[j]);
    for (int64_t e0 = static_cast<int64_t>(blockIdx.x) * kOhBS; e0 < N; e0 += static_cast<int64_t>(gridDim.x) * kOhBS) {
        const bool valid = e0 + tid < N;
        const int64_t bke = (static_cast<int64_t>(b) * k + j) * N + (valid ? e0 + tid : N - 1);
        const u128 P = a.pf[bke];
        DigitStream s;
        s.init(P);
        CompressFwd cf;
        cf.init();
        u128 Q = P, C = 0, PW = 1;  // chunk-major state (non-power-of-two moduli)
        uint32_t c0 = 0;
        // passes of whole chunks of m.c digits for the chunk-major walk
        const int pass = m.bits ? kOhCap : kOhCap / static_cast<int>(m.c) * static_cast<int>(m.c);
        for (int q0 = 0; q0 < n; q0 += pass) {
            const int cnt = min(pass, n - q0);
            __syncthreads();  // the previous pass's stores have read the image
            if (j != 0) {
                lds_stage_rows<kOhBS, 2>(stg, L, N, e0, q0, cnt);
                __syncthreads();
            }
            if (m.bits && cnt * static_cast<int>(m.bits) <= 64) {
                // power-of-two modulus, the pass's digits in one 64-bit window (residue 0 of the DASH bases: 128
                // one-bit digits, 40 per pass): a shift-and per digit over a fully unrolled, compile-time loop
                // instead of a 128-bit stream shift and scalar loop bookkeeping per digit (24-GC step -1.8 %,
                // profiles/ab/README.md round 6)
                const uint64_t win = static_cast<uint64_t>(s.Q);
                const uint32_t b = m.bits, msk = m.q - 1;
#pragma unroll
                for (int c = 0; c < kOhCap; ++c) {
                    if (c < cnt) {
                        uint8_t& w = stg[c * kOhBS + tid];
                        const uint32_t d = static_cast<uint32_t>(win >> (c * b)) & msk;
                        const uint32_t v = j == 0 ? d : modq(static_cast<uint32_t>(w) * inv + d, m);
                        w = static_cast<uint8_t>(v);
                        if (j != 0) cf.push(v, m);
                    }
                }
                s.Q >>= cnt * b;
                if (q0 == 0) c0 = stg[tid];  // digit 0 of the output (this lane's own LDS byte)
            } else if (m.bits) {
                for (int c = 0; c < cnt; ++c) {
                    uint8_t& w = stg[c * kOhBS + tid];
                    const uint32_t v = j == 0 ? s.next(m) : modq(static_cast<uint32_t>(w) * inv + s.next(m), m);
                    if (q0 + c == 0) c0 = v;
                    w = static_cast<uint8_t>(v);
                    if (j != 0) cf.push(v, m);
                }
            } else {  // chunk-major (chunk_digit): one divmod per chunk, uniform digit loops, one flush per chunk
                // (digit loop unrolled by 4 and the first digit read back after the pass instead of a compare per
                // digit: the loop's scalar bookkeeping was ~40 % of the kernel's instructions, r05 headline PMC)
                for (int k0 = 0; k0 < cnt; k0 += static_cast<int>(m.c)) {
                    uint32_t r = divmod128(Q, m);
                    const int kc = min(static_cast<int>(m.c), cnt - k0);
                    uint32_t acc = 0, pt = 1;
#pragma unroll 4
                    for (int t = 0; t < kc; ++t) {
                        uint8_t& w = stg[(k0 + t) * kOhBS + tid];
                        const uint32_t dd = chunk_digit(r, m);
                        const uint32_t v = j == 0 ? dd : modq(static_cast<uint32_t>(w) * inv + dd, m);
                        w = static_cast<uint8_t>(v);
                        acc += v * pt;
                        pt *= m.q;
                    }
                    C += PW * static_cast<u128>(acc);
                    PW *= static_cast<u128>(m.D);
                }
                if (q0 == 0) c0 = stg[tid];  // digit 0 of the output (this lane's own LDS byte)
            }
            __syncthreads();
            lds_store_rows<kOhBS>(L, stg, N, e0, q0, cnt);
        }
        const u128 H = hard_pad(j == 0 ? P : (m.bits ? cf.finish() : C),
                                a.rgate0 ^ static_cast<uint64_t>(valid ? e0 + tid : N - 1), tw_sub(kTwMmg, j), 0);
        if (valid) {
            a.colx[bke] = static_cast<uint16_t>(c0);
            a.hx[bke] = H;
        }
    }
}

// Joint rescale + ReLU, both outputs in one pass per (element, residue): Y_j (the rescaled label, written in
// place), its hash -> the garbler half gate G = g[color(Y_j)] - H(Y_j) (gathered as soon as the first
// component is known), then relu_j = E + ypr * Y_j - G (k_relu_mult's arithmetic) streamed into y while Y_j
// is read back from the lines this lane just wrote. The sign's hash / color come from chain MODE 2.
#ifndef DASH_RRO_WAVES
#define DASH_RRO_WAVES 4  // k_rescale_relu_out register budget (waves per SIMD): 6 spilled 256 B per lane
#endif
__global__ __launch_bounds__(kAesBlock, DASH_RRO_WAVES) void k_rescale_relu_out(MrsArgs a, SignArgs sa, Act x, Act y,
                                                                              const u128* gtab, const u128* etab,
                                                                              const ModC* mc, const uint32_t* te0,
                                                                              const uint32_t* rk) {
    (void)te0;
    (void)rk;
    const int j = blockIdx.y, b = blockIdx.z;
    const int64_t N = a.N;
    const int k = a.crt.k;
    const int p = a.crt.p[j];
    const ModC m = mc[p];
    const int n = static_cast<int>(m.n);
    const uint32_t inv = static_cast<uint32_t>(a.sinv[j]);
    for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < N;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t be = static_cast<int64_t>(b) * N + e;
        const int64_t bke = (static_cast<int64_t>(b) * k + j) * N + e;
        act_t* L = x.p[j] + static_cast<int64_t>(b) * n * N + e;
        act_t* Y = y.p[j] + static_cast<int64_t>(b) * n * N + e;
        // hardened y-row pads (chain MODE 2 store_ypads): entry j, mini lane j % 8 of slot k + j / 8
        const u128 HS = a.ys[(static_cast<int64_t>(b) * a.ny + j) * N + e];
        const u128 HM = a.ys[(static_cast<int64_t>(b) * a.ny + k + j / 8) * N + e] >> (16 * (j % 8));
        const uint32_t cS = a.cs[be];
        const u128* E3 = etab + (be * k + j) * 3;
        const u128 Eraw = E3[cS];
        const u128 mini = E3[2];
        const u128* grow = gtab + be * sa.crt.sum + sa.crt.prefix[j];
        const u128 P = a.pf[bke];
        DigitStream s;
        s.init(P);
        u128 key, Graw;
        if (j == 0) {
            // Y_0 = decompress(P), compress(Y_0) = P
            uint32_t c0 = 0;
            for (int c = 0; c < n; ++c) {
                const uint32_t v = s.next(m);
                if (c == 0) {
                    c0 = v;
                    Graw = grow[c0];
                }
                L[static_cast<int64_t>(c) * N] = static_cast<act_t>(v);
            }
            key = P;
        } else {
            CompressFwd cf;
            cf.init();
            uint16_t cur[kChunk], nxt[kChunk];
#pragma unroll
            for (int u = 0; u < kChunk; ++u)
                if (u < n) cur[u] = L[static_cast<int64_t>(u) * N];
            for (int q0 = 0; q0 < n; q0 += kChunk) {
#pragma unroll
                for (int u = 0; u < kChunk; ++u)
                    if (q0 + kChunk + u < n) nxt[u] = L[static_cast<int64_t>(q0 + kChunk + u) * N];
#pragma unroll
                for (int u = 0; u < kChunk; ++u)
                    if (q0 + u < n) {
                        const uint32_t v = modq(cur[u] * inv + s.next(m), m);  // < p^2 + p
                        if (q0 + u == 0) Graw = grow[v];
                        L[static_cast<int64_t>(q0 + u) * N] = static_cast<act_t>(v);
                        cf.push(v, m);
                    }
#pragma unroll
                for (int u = 0; u < kChunk; ++u) cur[u] = nxt[u];
            }
            key = cf.finish();
        }
        const u128 G = Graw - hard_pad(key, a.rgate0 ^ static_cast<uint64_t>(e), tw_sub(kTwMmg, j), 0);
        const u128 E = Eraw - HS;
        const int16_t t16 = static_cast<int16_t>(static_cast<uint16_t>(mini >> (16 * cS)));
        const int16_t ypr16 = static_cast<int16_t>(t16 - static_cast<int16_t>(static_cast<uint16_t>(HM)));
        const uint32_t ypr = modq(static_cast<uint32_t>(static_cast<int32_t>(ypr16) + (p << 15)), m);
        DigitStream sg, se;
        sg.init(G);
        se.init(E);
        uint16_t cur[kChunk], nxt[kChunk];
#pragma unroll
        for (int u = 0; u < kChunk; ++u)
            if (u < n) cur[u] = L[static_cast<int64_t>(u) * N];
        for (int i0 = 0; i0 < n; i0 += kChunk) {
#pragma unroll
            for (int u = 0; u < kChunk; ++u)
                if (i0 + kChunk + u < n) nxt[u] = L[static_cast<int64_t>(i0 + kChunk + u) * N];
#pragma unroll
            for (int u = 0; u < kChunk; ++u)
                if (i0 + u < n) {
                    const uint32_t g = sg.next(m);
                    const uint32_t ev = se.next(m);
                    Y[static_cast<int64_t>(i0 + u) * N] =
                        static_cast<act_t>(modq(ev + ypr * static_cast<uint32_t>(cur[u]) + static_cast<uint32_t>(p) - g, m));
                }
#pragma unroll
            for (int u = 0; u < kChunk; ++u) cur[u] = nxt[u];
        }
    }
}

// k_rescale_relu_out with the label staged in LDS (stage_ok, small batches): a block = (256-element tile,
// residue j, GC b) brings x_j's rows in once as 16-byte loads, each lane rescales its column in place and
// hashes it, the block stores the rescaled rows (x in place), then each lane rewrites its column into the
// ReLU output, stored as rows again. The per-lane form streams the label twice with one byte per lane per
// load, n / kChunk dependent round trips per pass. Measured at batch 1 (MiniONN): 90 us per op vs 76 for the
// per-lane form and ~50 + ~50 for the staged output-hash and ReLU-multiply kernels, whose 2.24 ms per step
// beat 2.30 here (64 KiB of LDS per block: two blocks per CU), so the planner only fuses unstaged shapes and
// this form runs under DASH_JOINT_FUSE=1 (A/B).
constexpr int kRroBS = 256;
__global__ __launch_bounds__(kRroBS) void k_rescale_relu_out_s(MrsArgs a, SignArgs sa, Act x, Act y, const u128* gtab,
                                                                const u128* etab, const ModC* mc, const uint32_t* te0,
                                                                const uint32_t* rk) {
    (void)te0;
    (void)rk;
    __shared__ __attribute__((aligned(16))) uint8_t stg[128 * kRroBS];
    const int j = blockIdx.y, b = blockIdx.z;
    const int64_t N = a.N;
    const int k = a.crt.k;
    const int p = a.crt.p[j];
    const ModC m = mc[p];
    const int n = static_cast<int>(m.n);
    const int tid = static_cast<int>(threadIdx.x);
    const uint32_t inv = static_cast<uint32_t>(a.sinv[j]);
    act_t* L = x.p[j] + static_cast<int64_t>(b) * n * N;
    act_t* Y = y.p[j] + static_cast<int64_t>(b) * n * N;
    for (int64_t e0 = static_cast<int64_t>(blockIdx.x) * kRroBS; e0 < N; e0 += static_cast<int64_t>(gridDim.x) * kRroBS) {
        const int64_t e = min(e0 + tid, N - 1);  // spare lanes shadow a real element; the row stores skip them
        const int64_t be = static_cast<int64_t>(b) * N + e;
        const int64_t bke = (static_cast<int64_t>(b) * k + j) * N + e;
        const u128 HS = a.ys[(static_cast<int64_t>(b) * a.ny + j) * N + e];
        const u128 HM = a.ys[(static_cast<int64_t>(b) * a.ny + k + j / 8) * N + e] >> (16 * (j % 8));
        const uint32_t cS = a.cs[be];
        const u128* E3 = etab + (be * k + j) * 3;
        const u128 Eraw = E3[cS];
        const u128 mini = E3[2];
        const u128* grow = gtab + be * sa.crt.sum + sa.crt.prefix[j];
        const u128 P = a.pf[bke];
        __syncthreads();  // the previous tile's row stores have read the image
        if (j != 0) lds_stage_rows<kRroBS, 4>(stg, L, N, e0, 0, n);
        __syncthreads();
        DigitStream s;
        s.init(P);
        CompressFwd cf;
        cf.init();
        u128 Graw = 0;
        // groups of kRroG digits: the group's LDS reads are issued together (one exposed latency per group instead
        // of per digit: a digit's write-back may alias the next digit's read, so the compiler cannot hoist it)
        constexpr int kRroG = 8;
        if (j == 0 && m.bits == 1) {
            // p = 2: Y_0's digits are the bits of P. Its 128 components are the longest label, so the residue-0
            // blocks were the launch's tail when each digit took a 128-bit stream shift
            Graw = grow[static_cast<uint32_t>(P) & 1u];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const uint32_t pw = static_cast<uint32_t>(P >> (32 * w));
#pragma unroll 8
                for (int u = 0; u < 32; ++u) {
                    const int c = 32 * w + u;
                    if (c >= n) break;
                    stg[c * kRroBS + tid] = static_cast<uint8_t>((pw >> u) & 1u);
                }
            }
        }
        for (int c0 = 0; c0 < ((j == 0 && m.bits == 1) ? 0 : n); c0 += kRroG) {
            uint32_t w8[kRroG];
#pragma unroll
            for (int u = 0; u < kRroG; ++u) w8[u] = (j != 0 && c0 + u < n) ? stg[(c0 + u) * kRroBS + tid] : 0u;
#pragma unroll
            for (int u = 0; u < kRroG; ++u) {
                const int c = c0 + u;
                if (c >= n) break;
                const uint32_t v = j == 0 ? s.next(m) : modq(w8[u] * inv + s.next(m), m);
                if (c == 0) Graw = grow[v];
                stg[c * kRroBS + tid] = static_cast<uint8_t>(v);
                if (j != 0) cf.push(v, m);
            }
        }
        const u128 key = j == 0 ? P : cf.finish();
        __syncthreads();
        lds_store_rows<kRroBS>(L, stg, N, e0, 0, n);  // Y_j, the rescaled label
        const u128 G = Graw - hard_pad(key, a.rgate0 ^ static_cast<uint64_t>(e), tw_sub(kTwMmg, j), 0);
        const u128 E = Eraw - HS;
        const int16_t t16 = static_cast<int16_t>(static_cast<uint16_t>(mini >> (16 * cS)));
        const int16_t ypr16 = static_cast<int16_t>(t16 - static_cast<int16_t>(static_cast<uint16_t>(HM)));
        const uint32_t ypr = modq(static_cast<uint32_t>(static_cast<int32_t>(ypr16) + (p << 15)), m);
        DigitStream sg, se;
        sg.init(G);
        se.init(E);
        __syncthreads();  // the row stores have read Y_j
        if (m.bits == 1) {
            // p = 2: (e + ypr y + 2 - g) mod 2 = e ^ g ^ (ypr & y), the digits of G and E being their bits
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const uint32_t ge = static_cast<uint32_t>(G >> (32 * w)) ^ static_cast<uint32_t>(E >> (32 * w));
#pragma unroll 8
                for (int u = 0; u < 32; ++u) {
                    const int c = 32 * w + u;
                    if (c >= n) break;
                    uint8_t& v = stg[c * kRroBS + tid];
                    v = static_cast<uint8_t>(((ge >> u) & 1u) ^ (static_cast<uint32_t>(v) & ypr));
                }
            }
        }
        for (int c0 = 0; c0 < (m.bits == 1 ? 0 : n); c0 += kRroG) {
            uint32_t w8[kRroG];
#pragma unroll
            for (int u = 0; u < kRroG; ++u) w8[u] = c0 + u < n ? stg[(c0 + u) * kRroBS + tid] : 0u;
#pragma unroll
            for (int u = 0; u < kRroG; ++u) {
                const int c = c0 + u;
                if (c >= n) break;
                const uint32_t g = sg.next(m);
                const uint32_t ev = se.next(m);
                stg[c * kRroBS + tid] = static_cast<uint8_t>(modq(ev + ypr * w8[u] + static_cast<uint32_t>(p) - g, m));
            }
        }
        __syncthreads();
        lds_store_rows<kRroBS>(Y, stg, N, e0, 0, n);
    }
}

// Quad form of the joint output (latency-bound launches: batch 1, small layers). Four lanes per (element,
// residue): the label's base-q chunks are dealt over the quad (lane g takes chunks 4j + g, power-of-two moduli
// a quarter of the digits each), every lane runs the payload's chunk divisions and keeps its own chunk, the
// rescaled label's partial keys are summed over the quad. The per-lane forms walk all n digits of three streams
// serially on one lane (~50 us per launch whatever the layer size at batch 1, r05 timeline).
constexpr int kRroQE = 64;  // elements per block (256 threads)
// rows [0, n) of kRroQE elements from e0: 16-byte units when N % 16 == 0, bytes otherwise (tails, tiny layers)
__device__ __forceinline__ void quad_stage_rows(uint8_t* S, const act_t* L, int64_t N, int64_t e0, int n) {
    if (N % 16 == 0) {
        for (int xu = threadIdx.x; xu < n * (kRroQE / 16); xu += blockDim.x) {
            const int row = xu / (kRroQE / 16), part = xu % (kRroQE / 16);
            const int64_t ee = e0 + 16 * part;
            if (ee < N) *reinterpret_cast<uint4*>(S + row * kRroQE + 16 * part) =
                *reinterpret_cast<const uint4*>(L + static_cast<int64_t>(row) * N + ee);
        }
    } else {
        for (int xb = threadIdx.x; xb < n * kRroQE; xb += blockDim.x) {
            const int row = xb / kRroQE, c = xb % kRroQE;
            if (e0 + c < N) S[xb] = L[static_cast<int64_t>(row) * N + e0 + c];
        }
    }
}
__device__ __forceinline__ void quad_store_rows(act_t* L, const uint8_t* S, int64_t N, int64_t e0, int n) {
    if (N % 16 == 0) {
        for (int xu = threadIdx.x; xu < n * (kRroQE / 16); xu += blockDim.x) {
            const int row = xu / (kRroQE / 16), part = xu % (kRroQE / 16);
            const int64_t ee = e0 + 16 * part;
            if (ee < N) *reinterpret_cast<uint4*>(L + static_cast<int64_t>(row) * N + ee) =
                *reinterpret_cast<const uint4*>(S + row * kRroQE + 16 * part);
        }
    } else {
        for (int xb = threadIdx.x; xb < n * kRroQE; xb += blockDim.x) {
            const int row = xb / kRroQE, c = xb % kRroQE;
            if (e0 + c < N) L[static_cast<int64_t>(row) * N + e0 + c] = S[xb];
        }
    }
}
// the quad output forms where a lane-per-element launch would not fill the chip (latency-bound: batch 1, small
// layers); DASH_RRO_QUAD=0 keeps the lane-per-element forms, =2 takes the quad forms at every size (A/B)
static inline bool out_quad_fits(const MrsArgs& a, int B) {
    static const int mode = [] {
        const char* e = std::getenv("DASH_RRO_QUAD");
        return e ? std::atoi(e) : 1;
    }();
    bool fits = mode != 0 && (mode == 2 || (a.N + 255) / 256 * a.crt.k * B <= num_cus());
    for (int j = 0; j < a.crt.k; ++j) fits = fits && a.crt.n[j] <= 128;  // the LDS images hold 128 components
    return fits;
}
__global__ __launch_bounds__(256) void k_rescale_relu_out_q(MrsArgs a, SignArgs sa, Act x, Act y, const u128* gtab,
                                                           const u128* etab, const ModC* mc) {
    __shared__ __attribute__((aligned(16))) uint8_t sL[128 * kRroQE];  // L_j -> Y_j in place
    __shared__ __attribute__((aligned(16))) uint8_t sO[128 * kRroQE];  // ReLU outputs
    const int j = blockIdx.y, b = blockIdx.z;
    const int64_t N = a.N;
    const int k = a.crt.k;
    const int p = a.crt.p[j];
    const ModC m = mc[p];
    const int n = static_cast<int>(m.n);
    const uint32_t q = m.q;
    const int tid = static_cast<int>(threadIdx.x);
    const int el = tid >> 2, g = tid & 3;
    const uint32_t inv = static_cast<uint32_t>(a.sinv[j]);
    act_t* L = x.p[j] + static_cast<int64_t>(b) * n * N;
    act_t* Yo = y.p[j] + static_cast<int64_t>(b) * n * N;
    for (int64_t e0 = static_cast<int64_t>(blockIdx.x) * kRroQE; e0 < N; e0 += static_cast<int64_t>(gridDim.x) * kRroQE) {
        const int64_t e = min(e0 + el, N - 1);  // spare quads shadow a real element; the row stores skip them
        const int64_t be = static_cast<int64_t>(b) * N + e;
        const int64_t bke = (static_cast<int64_t>(b) * k + j) * N + e;
        const u128 HS = a.ys[(static_cast<int64_t>(b) * a.ny + j) * N + e];
        const u128 HM = a.ys[(static_cast<int64_t>(b) * a.ny + k + j / 8) * N + e] >> (16 * (j % 8));
        const uint32_t cS = a.cs[be];
        const u128* E3 = etab + (be * k + j) * 3;
        const u128 mini = E3[2];
        const u128* grow = gtab + be * sa.crt.sum + sa.crt.prefix[j];
        const u128 P = a.pf[bke];
        const u128 Eraw = E3[cS];
        __syncthreads();  // the previous tile's row stores have read the images
        if (j != 0) quad_stage_rows(sL, L, N, e0, n);
        __syncthreads();
        // digit 0 first (every lane): the garbler half gate's row gather overlaps the walk
        u128 Graw;
        {
            uint32_t pd0;
            if (m.bits) {
                pd0 = static_cast<uint32_t>(P) & (q - 1);
            } else {
                u128 t = P;
                uint32_t r = divmod128(t, m);
                pd0 = chunk_digit(r, m);
            }
            const uint32_t v0 = j == 0 ? pd0 : modq(static_cast<uint32_t>(sL[el]) * inv + pd0, m);
            Graw = grow[v0];
        }
        // Y_j = S^-1 L_j + P (mod p), residue 0: Y_0 = decompress(P); the lane's digits and its partial key
        u128 part = 0;
        const int bb = static_cast<int>(m.bits), cpl = (n + 3) >> 2;
        QPow pw;
        if (m.bits) {
            // the lane's digits g cpl .. g cpl + cpl - 1 fit one 64-bit window (bb cpl <= 32 + bb): one 128-bit
            // shift per lane instead of one per digit
            const uint64_t Pw = static_cast<uint64_t>(P >> (bb * g * cpl));
            for (int t = 0; t < cpl; ++t) {
                const int idx = g * cpl + t;
                if (idx >= n) break;
                const uint32_t pd = static_cast<uint32_t>(Pw >> (bb * t)) & (q - 1);
                const uint32_t v = j == 0 ? pd : modq(static_cast<uint32_t>(sL[idx * kRroQE + el]) * inv + pd, m);
                sL[idx * kRroQE + el] = static_cast<uint8_t>(v);
                part |= static_cast<u128>(v) << (bb * idx);
            }
        } else {
            pw.init(m);
            const int c = static_cast<int>(m.c), nch = (n + c - 1) / c;
            u128 Q = P, PW = pw.first(g);
            for (int jj = 0; 4 * jj < nch; ++jj) {
                uint32_t mine = 0;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (4 * jj + u >= nch) break;
                    const uint32_t r = divmod128(Q, m);
                    mine = u == g ? r : mine;
                }
                const int i = 4 * jj + g;
                uint32_t cv = 0, pt = 1;
                for (int t = 0; t < c; ++t) {
                    const int idx = i * c + t;
                    const uint32_t pd = chunk_digit(mine, m);
                    if (idx < n) {
                        const uint32_t v = j == 0 ? pd : modq(static_cast<uint32_t>(sL[idx * kRroQE + el]) * inv + pd, m);
                        sL[idx * kRroQE + el] = static_cast<uint8_t>(v);
                        cv += v * pt;
                    }
                    pt *= q;
                }
                part += PW * static_cast<u128>(cv);
                PW *= pw.d4;
            }
        }
        const u128 key = j == 0 ? P : quad_sum128(part);
        u128 G;
        if constexpr (kQCoop) {  // the quad runs the pad block together (every lane holds the same key)
            uint32_t w[4];
            hard_block_q(key, a.rgate0 ^ static_cast<uint64_t>(e), tw_sub(kTwMmg, j), 0u, g, w);
            G = Graw - quad_gather128(w[0]);
        } else {
            G = Graw - hard_pad(key, a.rgate0 ^ static_cast<uint64_t>(e), tw_sub(kTwMmg, j), 0);
        }
        const u128 E = Eraw - HS;
        const int16_t t16 = static_cast<int16_t>(static_cast<uint16_t>(mini >> (16 * cS)));
        const int16_t ypr16 = static_cast<int16_t>(t16 - static_cast<int16_t>(static_cast<uint16_t>(HM)));
        const uint32_t ypr = modq(static_cast<uint32_t>(static_cast<int32_t>(ypr16) + (p << 15)), m);
        // relu_j = E + ypr Y_j - G, the lane's own digits (k_relu_mult's arithmetic)
        if (m.bits) {
            const uint64_t Gw = static_cast<uint64_t>(G >> (bb * g * cpl)), Ew = static_cast<uint64_t>(E >> (bb * g * cpl));
            for (int t = 0; t < cpl; ++t) {
                const int idx = g * cpl + t;
                if (idx >= n) break;
                const uint32_t gd = static_cast<uint32_t>(Gw >> (bb * t)) & (q - 1);
                const uint32_t ed = static_cast<uint32_t>(Ew >> (bb * t)) & (q - 1);
                sO[idx * kRroQE + el] =
                    static_cast<uint8_t>(modq(ed + ypr * static_cast<uint32_t>(sL[idx * kRroQE + el]) + static_cast<uint32_t>(p) - gd, m));
            }
        } else {
            const int c = static_cast<int>(m.c), nch = (n + c - 1) / c;
            u128 QG = G, QE = E;
            for (int jj = 0; 4 * jj < nch; ++jj) {
                uint32_t mg = 0, me = 0;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (4 * jj + u >= nch) break;
                    const uint32_t rg = divmod128(QG, m);
                    const uint32_t re = divmod128(QE, m);
                    mg = u == g ? rg : mg;
                    me = u == g ? re : me;
                }
                const int i = 4 * jj + g;
                for (int t = 0; t < c; ++t) {
                    const int idx = i * c + t;
                    const uint32_t gd = chunk_digit(mg, m);
                    const uint32_t ed = chunk_digit(me, m);
                    if (idx < n)
                        sO[idx * kRroQE + el] = static_cast<uint8_t>(
                            modq(ed + ypr * static_cast<uint32_t>(sL[idx * kRroQE + el]) + static_cast<uint32_t>(p) - gd, m));
                }
            }
        }
        __syncthreads();
        quad_store_rows(L, sL, N, e0, n);
        quad_store_rows(Yo, sO, N, e0, n);
    }
}

void launch_rescale_relu_out(const MrsArgs& a, const SignArgs& sa, const Act& x, const Act& y, const u128* gtab,
                             const u128* etab, int B, const ModC* mc, const AesGlobals& g, hipStream_t st) {
    static const bool rro_stage = [] {  // DASH_RRO_STAGE=0: the per-lane form (A/B)
        const char* e = std::getenv("DASH_RRO_STAGE");
        return !(e && e[0] == '0');
    }();
    if (out_quad_fits(a, B)) {
        hipLaunchKernelGGL(k_rescale_relu_out_q, dim3(static_cast<unsigned>((a.N + kRroQE - 1) / kRroQE), a.crt.k, B),
                           dim3(256), 0, st, a, sa, x, y, gtab, etab, mc);
        return;
    }
    if (rro_stage && stage_ok(a.N, kRroBS)) {
        hipLaunchKernelGGL(k_rescale_relu_out_s, dim3(static_cast<unsigned>((a.N + kRroBS - 1) / kRroBS), a.crt.k, B),
                           dim3(kRroBS), 0, st, a, sa, x, y, gtab, etab, mc, g.te0, g.rk);
        return;
    }
    hipLaunchKernelGGL(k_rescale_relu_out, AES_LAUNCH(a.N, a.crt.k, B), kAesLds, st, a, sa, x, y, gtab, etab, mc,
                       g.te0, g.rk);
}

// hx[b][j][e] = H(compress(x_j)), colx = color: the ReLU multiply's garbler half gates (exact-sign path;
// the approximate path gets them from k_sign_approx). grid (x, k, B)
__global__ __launch_bounds__(kAesBlock, kAesMinBlocks) void k_label_hash(Act x, CrtInfo crt, int64_t N, u128* hx,
                                                                        uint16_t* colx, const ModC* mc,
                                                                        const uint32_t* te0, const uint32_t* rk,
                                                                        int hard, uint64_t mgate0) {
    AES_PROLOGUE(te0, rk);
    const int j = blockIdx.y, b = blockIdx.z;
    for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < N;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const ModC m = mc[crt.p[j]];
        const act_t* L = x.p[j] + static_cast<int64_t>(b) * m.n * N + e;
        const int64_t bke = (static_cast<int64_t>(b) * crt.k + j) * N + e;
        colx[bke] = static_cast<uint16_t>(static_cast<uint16_t>(L[0]) % m.q);
        const u128 C = compress_cm(L, N, m);
        hx[bke] = hard ? hard_pad(C, mgate0 ^ static_cast<uint64_t>(e), tw_sub(kTwMmg, j), 0) : aes_encrypt(aes, C);
    }
}

// the chain launch of CRT size a.crt.k (per-K units kernels_mrs_*.hip, mrs_chain.h)
static void dispatch_mrs_chain(const MrsArgs& a, const Act& x, int B, const ModC* mc, const AesGlobals& g,
                               hipStream_t st) {
    switch (a.crt.k) {
        case 2: launch_mrs_chain_k<2>(a, x, B, mc, g, st); break;
        case 3: launch_mrs_chain_k<3>(a, x, B, mc, g, st); break;
        case 4: launch_mrs_chain_k<4>(a, x, B, mc, g, st); break;
        case 5: launch_mrs_chain_k<5>(a, x, B, mc, g, st); break;
        case 6: launch_mrs_chain_k<6>(a, x, B, mc, g, st); break;
        case 7: launch_mrs_chain_k<7>(a, x, B, mc, g, st); break;
        case 8: launch_mrs_chain_k<8>(a, x, B, mc, g, st); break;
        case 9: launch_mrs_chain_k<9>(a, x, B, mc, g, st); break;
        case 10: launch_mrs_chain_k<10>(a, x, B, mc, g, st); break;
        case 11: launch_mrs_chain_k<11>(a, x, B, mc, g, st); break;
        case 12: launch_mrs_chain_k<12>(a, x, B, mc, g, st); break;
        default: std::fprintf(stderr, "dash: mixed-radix chains support 2..12 CRT residues\n"); std::abort();
    }
}

void launch_relu_mrs(const MrsArgs& a, const SignArgs& sa, const Act& x, const Act& y, const u128* gtab,
                     const u128* etab, int B, const ModC* mc, const AesGlobals& g, hipStream_t st) {
    hipLaunchKernelGGL(k_label_hash, AES_LAUNCH(a.N, a.crt.k, B), kAesLds, st, x, a.crt, a.N,
                       sa.hx, sa.colx, mc, g.te0, g.rk, sa.hard, sa.mgate0);
    dispatch_mrs_chain(a, x, B, mc, g, st);
    launch_relu_mult(sa, x, y, gtab, etab, mc, st);
}

// ReLU after a sign-producing rescale: the rescale wrote the sign's hash / color (chain MODE 2) and the
// half-gate keys of x (k_rescale_mrs_out_hash); only the mixed-modulus multiply is left
void launch_relu_joint(const SignArgs& sa, const Act& x, const Act& y, const u128* gtab, const u128* etab, int B,
                       const ModC* mc, const AesGlobals& g, hipStream_t st) {
    (void)B;
    (void)g;
    launch_relu_mult(sa, x, y, gtab, etab, mc, st);
}

// Quad form of k_rescale_mrs_out for latency-bound launches (batch 1, small layers): four lanes per (element,
// residue), the payload's chunks dealt over the quad (as k_rescale_relu_out_q's first pass), rows staged and
// stored as 16-byte units.
__global__ __launch_bounds__(256) void k_rescale_mrs_out_q(MrsArgs a, Act x, const ModC* mc) {
    __shared__ __attribute__((aligned(16))) uint8_t sL[128 * kRroQE];
    const int j = blockIdx.y, b = blockIdx.z;
    const int64_t N = a.N;
    const int k = a.crt.k;
    const ModC m = mc[a.crt.p[j]];
    const int n = static_cast<int>(m.n);
    const uint32_t q = m.q;
    const int tid = static_cast<int>(threadIdx.x);
    const int el = tid >> 2, g = tid & 3;
    const uint32_t inv = static_cast<uint32_t>(a.sinv[j]);
    act_t* L = x.p[j] + static_cast<int64_t>(b) * n * N;
    for (int64_t e0 = static_cast<int64_t>(blockIdx.x) * kRroQE; e0 < N; e0 += static_cast<int64_t>(gridDim.x) * kRroQE) {
        const int64_t e = min(e0 + el, N - 1);
        const u128 P = a.pf[(static_cast<int64_t>(b) * k + j) * N + e];
        __syncthreads();
        if (j != 0) quad_stage_rows(sL, L, N, e0, n);
        __syncthreads();
        if (m.bits) {
            const int bb = static_cast<int>(m.bits), cpl = (n + 3) >> 2;
            const uint64_t Pw = static_cast<uint64_t>(P >> (bb * g * cpl));  // (as k_rescale_relu_out_q)
            for (int t = 0; t < cpl; ++t) {
                const int idx = g * cpl + t;
                if (idx >= n) break;
                const uint32_t pd = static_cast<uint32_t>(Pw >> (bb * t)) & (q - 1);
                sL[idx * kRroQE + el] =
                    static_cast<uint8_t>(j == 0 ? pd : modq(static_cast<uint32_t>(sL[idx * kRroQE + el]) * inv + pd, m));
            }
        } else {
            const int c = static_cast<int>(m.c), nch = (n + c - 1) / c;
            u128 Q = P;
            for (int jj = 0; 4 * jj < nch; ++jj) {
                uint32_t mine = 0;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (4 * jj + u >= nch) break;
                    const uint32_t r = divmod128(Q, m);
                    mine = u == g ? r : mine;
                }
                const int i = 4 * jj + g;
                for (int t = 0; t < c; ++t) {
                    const int idx = i * c + t;
                    const uint32_t pd = chunk_digit(mine, m);
                    if (idx < n)
                        sL[idx * kRroQE + el] = static_cast<uint8_t>(
                            j == 0 ? pd : modq(static_cast<uint32_t>(sL[idx * kRroQE + el]) * inv + pd, m));  // < p^2 + p
                }
            }
        }
        __syncthreads();
        quad_store_rows(L, sL, N, e0, n);
    }
}

void launch_rescale_mrs(const MrsArgs& a, const Act& x, int B, const ModC* mc, const AesGlobals& g, hipStream_t st,
                        bool chain_only) {
    dispatch_mrs_chain(a, x, B, mc, g, st);
    if (chain_only) return;  // the joint ReLU's k_rescale_relu_out writes the outputs
    if (a.mode == 2 && stage_ok(a.N, kOhBS))
        hipLaunchKernelGGL(k_rescale_mrs_out_hash_s, grid_aes(a.N, kOhBS, a.crt.k, B), dim3(kOhBS), 0, st, a, x, mc,
                           g.te0, g.rk);
    else if (a.mode == 2)
        hipLaunchKernelGGL(k_rescale_mrs_out_hash, AES_LAUNCH(a.N, a.crt.k, B), kAesLds, st, a, x, mc, g.te0, g.rk);
    else if (out_quad_fits(a, B))
        hipLaunchKernelGGL(k_rescale_mrs_out_q, dim3(static_cast<unsigned>((a.N + kRroQE - 1) / kRroQE), a.crt.k, B),
                           dim3(256), 0, st, a, x, mc);
    else
        hipLaunchKernelGGL(k_rescale_mrs_out, dim3(static_cast<unsigned>((a.N + 255) / 256), a.crt.k, B), dim3(256), 0,
                           st, a, x, mc);
}

// ---------------------------------------------------------------------------
// ReDash base extension (MRS conversion). One lane per (GC, element); the
// working copies live in `work` (component-major, [B][E][128][N]).

__global__ __launch_bounds__(256) void k_base_ext(BEArgs a, Act x, const ModC* mc, const uint32_t* te0,
                                                  const uint32_t* rk) {
    AES_PROLOGUE(te0, rk);
    const int b = blockIdx.z;
    const int64_t N = a.N;
    for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < N;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int E = a.E;
    auto W = [&](int pos) { return a.work + ((static_cast<int64_t>(b) * E + pos) * 128) * N + e; };
    for (int i = 0; i < E; ++i) {
        const ModC m = mc[a.swapped[i]];
        const act_t* src = x.p[a.src[i]] + static_cast<int64_t>(b) * m.n * N + e;
        int16_t* w = W(i);
        col_map(src, w, N, static_cast<int>(m.n), [](int, int16_t v) { return v; });
    }
    const u128* T = a.tab + (static_cast<int64_t>(b) * N + e) * a.n_tab;
    int64_t off = 0;
    for (int i = 0; i < a.nonext; ++i) {
        const ModC mi = mc[a.swapped[i]];
        const int16_t* li = W(i);
        const u128 C = compress_cm(li, N, mi);
        const u128 H = a.hard ? 0 : aes_encrypt(aes, C);
        const uint32_t col = static_cast<uint16_t>(li[0]);
        for (int j = 0; j < E - i - 1; ++j) {
            const int tg = i + j + 1;
            const int q = a.swapped[tg];
            const ModC mo = mc[q];
            const u128 P = T[off + col] - (a.hard ? hard_pad(C, a.gate0 ^ static_cast<uint64_t>(e), tw_sub(kTwBe, i), j) : H);
            off += mi.q;
            DigitStream s;
            s.init(P);
            int16_t* lt = W(tg);
            const int32_t inv = a.inv[i][j];
            col_map(lt, lt, N, static_cast<int>(mo.n), [&](int, int16_t x) {
                int32_t v = x - static_cast<int32_t>(s.next(mo));
                if (v < 0) v += q;
                return static_cast<int16_t>(modq(static_cast<uint32_t>(v * inv), mo));
            });
        }
    }
    for (int xi = 0; xi < a.nextra; ++xi) {
        const int r = a.extra_res[xi];
        const int q = a.swapped[a.extra_pos[xi]];
        const ModC m = mc[q];
        const int16_t* w = W(a.extra_pos[xi]);
        act_t* dst = x.p[r] + static_cast<int64_t>(b) * m.n * N + e;
        const int32_t f = a.invv[xi];  // already negated mod q on the host
        col_map(w, dst, N, static_cast<int>(m.n), [&](int, int16_t v) { return static_cast<int16_t>(modq(static_cast<uint32_t>(v * f), m)); });
    }
    }
}

// ---------------------------------------------------------------------------
// Generic projection layer (test-only Projection). grid (ceil(N/256), k, B)
__global__ __launch_bounds__(kAesBlock, kAesMinBlocks) void k_proj(ProjArgs a, Act x, Act y, const ModC* mc, const uint32_t* te0,
                                              const uint32_t* rk) {
    AES_PROLOGUE(te0, rk);
    const int j = blockIdx.y, b = blockIdx.z;
    const int64_t N = a.N;
    for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < N;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const ModC mi = mc[a.pin[j]], mo = mc[a.pout[j]];
    const act_t* L = x.p[j] + static_cast<int64_t>(b) * mi.n * N + e;
    const u128 C = compress_cm(L, N, mi);
    const u128 H = a.hard ? hard_pad(C, a.gate0 ^ static_cast<uint64_t>(e), tw_sub(kTwProj, j), 0) : aes_encrypt(aes, C);
    const uint32_t col = static_cast<uint16_t>(L[0]) % mi.q;
    const u128 P = a.tab[j][(static_cast<int64_t>(b) * N + e) * mi.q + col] - H;
    DigitStream s;
    s.init(P);
    act_t* O = y.p[j] + static_cast<int64_t>(b) * mo.n * N + e;
    for (int i = 0; i < static_cast<int>(mo.n); ++i) O[i * N] = static_cast<act_t>(s.next(mo));
    }
}

// Generalized half-gate product of pairs (2e, 2e+1), and the mixed-modulus
// variant (second operand first projected to Z_q). grid (ceil(No/256), k, B)
__global__ __launch_bounds__(kAesBlock, kAesMinBlocks) void k_mult(MultArgs a, Act x, Act y, const ModC* mc, const uint32_t* te0,
                                              const uint32_t* rk) {
    AES_PROLOGUE(te0, rk);
    const int j = blockIdx.y, b = blockIdx.z;
    const int64_t No = a.No, Ni = 2 * No;
    for (int64_t o = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; o < No;
         o += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int p = a.crt.p[j];
    const ModC m = mc[p];
    const act_t* X = x.p[j] + static_cast<int64_t>(b) * m.n * Ni + 2 * o;
    const act_t* Yv = X + 1;
    const int64_t bo = static_cast<int64_t>(b) * No + o;
    const uint64_t gt = a.gate0 ^ static_cast<uint64_t>(o);
    const u128 Cx = compress_cm(X, Ni, m);
    const u128 Hx = a.hard ? hard_pad(Cx, gt, tw_sub(kTwMmg, j), 0) : aes_encrypt(aes, Cx);
    const uint32_t colx = static_cast<uint16_t>(X[0]) % p;
    const u128 G = a.g[bo * a.crt.sum + a.crt.prefix[j] + colx] - Hx;
    u128 E;
    int32_t ypr;
    if (a.q == 0) {
        const u128 Cy = compress_cm(Yv, Ni, m);
        const u128 Hy = a.hard ? hard_pad(Cy, gt, tw_sub(kTwGme, j), 0) : aes_encrypt(aes, Cy);
        const uint32_t coly = static_cast<uint16_t>(Yv[0]) % p;
        E = a.e[bo * a.crt.sum + a.crt.prefix[j] + coly] - Hy;
        ypr = static_cast<int32_t>(coly);
    } else {
        const ModC mq = mc[a.q];
        const u128 Cy = compress_cm(Yv, Ni, m);
        const u128 Hy = a.hard ? hard_pad(Cy, gt, tw_sub(kTwMmt, j), 0) : aes_encrypt(aes, Cy);
        const uint32_t coly = static_cast<uint16_t>(Yv[0]) % p;
        const u128 Pt = a.t[bo * a.crt.sum + a.crt.prefix[j] + coly] - Hy;  // compressed label mod q
        u128 Ht, Hm;
        if (a.hard) {  // own row (TW_MMY, j): entry slot 0, mini lane 0 of slot 1
            u128 pd[4];
            hard_block(Pt, gt, tw_sub(kTwMmy, j), 0, pd);
            Ht = pd[0];
            Hm = pd[1];
        } else {
            Ht = Hm = aes_encrypt(aes, Pt);
        }
        const uint32_t colt = u128_mod(Pt, mq);
        const u128* E3 = a.e + (bo * a.crt.k + j) * (a.q + 1);
        E = E3[colt] - Ht;
        const int16_t t16 = static_cast<int16_t>(static_cast<uint16_t>(E3[a.q] >> (16 * colt)));
        ypr = static_cast<int16_t>(t16 - static_cast<int16_t>(static_cast<uint16_t>(Hm)));
        ypr %= p;
        if (ypr < 0) ypr += p;
    }
    DigitStream sg, se;
    sg.init(G);
    se.init(E);
    act_t* O = y.p[j] + static_cast<int64_t>(b) * m.n * No + o;
    const int n = static_cast<int>(m.n);
    for (int i0 = 0; i0 < n; i0 += kChunk) {
        int16_t xv[kChunk];
#pragma unroll
        for (int u = 0; u < kChunk; ++u)
            if (i0 + u < n) xv[u] = X[(i0 + u) * Ni];
#pragma unroll
        for (int u = 0; u < kChunk; ++u)
            if (i0 + u < n) {
                const int32_t gv = static_cast<int32_t>(sg.next(m));
                const int32_t ev = static_cast<int32_t>(se.next(m));
                int32_t v = (ev + ypr * static_cast<int32_t>(xv[u]) - gv) % p;
                if (v < 0) v += p;
                O[(i0 + u) * No] = static_cast<act_t>(v);
            }
    }
    }
}

// ---------------------------------------------------------------------------
// launchers
static inline dim3 grid_for(int64_t n, int bs, int y, int z) {
    return dim3(static_cast<unsigned>((n + bs - 1) / bs), y, z);
}


void launch_sign_approx(const SignArgs& a, const Act& x, const ModC* mc, const AesGlobals& g, hipStream_t st) {
    if (a.t <= 5)
        hipLaunchKernelGGL(k_sign_approx<5>, AES_LAUNCH(a.N, a.crt.k, a.B), kAesLds, st, a, x, mc, g.te0,
                           g.rk);
    else
        hipLaunchKernelGGL(k_sign_approx<8>, AES_LAUNCH(a.N, a.crt.k, a.B), kAesLds, st, a, x, mc, g.te0,
                           g.rk);
}
void launch_sign_chain(const SignArgs& a, int maxn, const ModC* mc, const AesGlobals& g, hipStream_t st) {
    const dim3 gs = grid_for(a.N, 256, a.t, a.B);
    const dim3 gr = grid_aes(a.N, aes_bs(a.N, 1, a.B), 1, a.B), br(aes_bs(a.N, 1, a.B));
    // (measured: folding the castsum pass into the chain lanes is slower, 334 vs 356 inf/s on
    // MiniONN B=24: the chain is latency bound and the castsum's t-fold lane parallelism wins)
    if (maxn <= 24) {  // k = 7 DASH configs (cast outputs mod 8 m_d: <= 22 components)
        hipLaunchKernelGGL(k_sign_castsum<24>, gs, dim3(256), 0, st, a, mc);
        if (a.fused)
            hipLaunchKernelGGL(k_sign_chain_fused<24>, gr, br, kAesLds, st, a, mc, g.te0, g.rk);
        else
            hipLaunchKernelGGL(k_sign_chain<24>, gr, br, kAesLds, st, a, mc, g.te0, g.rk);
    } else if (maxn <= 32) {
        hipLaunchKernelGGL(k_sign_castsum<32>, gs, dim3(256), 0, st, a, mc);
        if (a.fused)
            hipLaunchKernelGGL(k_sign_chain_fused<32>, gr, br, kAesLds, st, a, mc, g.te0, g.rk);
        else
            hipLaunchKernelGGL(k_sign_chain<32>, gr, br, kAesLds, st, a, mc, g.te0, g.rk);
    } else {
        hipLaunchKernelGGL(k_sign_castsum<64>, gs, dim3(256), 0, st, a, mc);
        if (a.fused)
            hipLaunchKernelGGL(k_sign_chain_fused<64>, gr, br, kAesLds, st, a, mc, g.te0, g.rk);
        else
            hipLaunchKernelGGL(k_sign_chain<64>, gr, br, kAesLds, st, a, mc, g.te0, g.rk);
    }
}
void launch_unpack(const u128* P, int nres, const Act& out, const CrtInfo& mods, const ModC* mc, int64_t N, int B,
                   hipStream_t st) {
    hipLaunchKernelGGL(k_unpack, grid_for(N, 256, nres, B), dim3(256), 0, st, P, nres, out, mods, mc, N);
}
void launch_relu_mult(const SignArgs& a, const Act& x, const Act& y, const u128* gtab, const u128* etab,
                      const ModC* mc, hipStream_t st) {
    if (stage_ok(a.N, kRmBS) && x.p[0] != y.p[0]) {
        const unsigned nx = static_cast<unsigned>(std::min<int64_t>((a.N + kRmBS - 1) / kRmBS,
                                                                   std::max(1, 16 * num_cus() / (a.crt.k * a.B))));
        hipLaunchKernelGGL(k_relu_mult_s, dim3(nx, a.crt.k, a.B), dim3(kRmBS), 0, st, a, x, y, gtab, etab, mc);
        return;
    }
    hipLaunchKernelGGL(k_relu_mult, grid_for(a.N, 256, a.crt.k, a.B), dim3(256), 0, st, a, x, y, gtab, etab, mc);
}
void launch_rescale_hash(const Act& x, int fi, int s, const int16_t* up, int up_stride, int add_up, int64_t N, int B,
                         u128* h0, uint16_t* col0, const ModC* mc, const AesGlobals& g, hipStream_t st, int hard) {
    hipLaunchKernelGGL(k_rescale_hash, AES_LAUNCH(N, 1, B), kAesLds, st, x, fi, s, up, up_stride,
                       add_up, N, h0, col0, mc, g.te0, g.rk, hard);
}
void launch_rescale_update(const RescaleArgs& a, const Act& x, int B, const ModC* mc, hipStream_t st) {
    hipLaunchKernelGGL(k_rescale_update, grid_for(a.N, 256, a.crt.k, B), dim3(256), 0, st, a, x, mc);
}
void launch_rescale_post(const Act& x, const CrtInfo& crt, int64_t N, int B, const u128* signP, const int16_t* down,
                         int lab_stride, const int* lab_off, const ModC* mc, hipStream_t st) {
    hipLaunchKernelGGL(k_rescale_post, grid_for(N, 256, crt.k, B), dim3(256), 0, st, x, crt, N, signP, down,
                       lab_stride, lab_off, mc);
}
void launch_base_ext(const BEArgs& a, const Act& x, int B, const ModC* mc, const AesGlobals& g, hipStream_t st) {
    hipLaunchKernelGGL(k_base_ext, grid_aes(a.N, 256, 1, B), dim3(256), kAesLds, st, a, x, mc, g.te0, g.rk);
}
void launch_proj(const ProjArgs& a, const Act& x, const Act& y, int B, const ModC* mc, const AesGlobals& g,
                 hipStream_t st) {
    hipLaunchKernelGGL(k_proj, AES_LAUNCH(a.N, a.k, B), kAesLds, st, a, x, y, mc, g.te0, g.rk);
}
void launch_mult(const MultArgs& a, const Act& x, const Act& y, int B, const ModC* mc, const AesGlobals& g,
                 hipStream_t st) {
    hipLaunchKernelGGL(k_mult, AES_LAUNCH(a.No, a.crt.k, B), kAesLds, st, a, x, y, mc, g.te0, g.rk);
}

}  // namespace dev
}  // namespace dash
