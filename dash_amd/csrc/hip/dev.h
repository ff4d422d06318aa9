// Device library for the CDNA4 (gfx950) garbled-circuit evaluator.
//
//  * AES-128 with one T-table replicated 32x across the LDS banks: lane l
//    always reads copy (l & 31), so a wave64 ds_read_b32 (two 32-lane halves)
//    is bank-conflict free for any byte values. Te1..Te3 are rotations.
//  * Labels live in HBM component-major ([comp][element]) so that lanes
//    walking consecutive elements read/write coalesced; a label never has to
//    be materialised in registers: digit codecs stream.
//      - compress (reverse Horner, chunked 32-bit) reads digits top-down;
//      - compress_fwd (forward, chunked) consumes digits bottom-up and fuses
//        with decompress streams;
//      - decompress streams digits bottom-up from a 128-bit payload by long
//        division by q^c (< 2^32) with a reciprocal (no hardware divide).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dash {
namespace dev {

typedef unsigned __int128 u128;

// ---------------------------------------------------------------------------
// Per-modulus constants (built on the host, see runtime.hip)
struct ModC {
    uint32_t q;      // modulus
    uint32_t n;      // label width
    uint32_t c;      // digits per chunk
    uint32_t D;      // q^c < 2^32
    uint64_t mD;     // floor(2^64 / D)
    uint32_t mq;     // floor(2^32 / q)
    uint32_t bits;   // log2 q if power of two, else 0
    uint32_t dm;     // digit magic: floor(r / q) = mulhi(r, dm) >> ds for r < D (host_util.h make_modc)
    uint32_t ds;
    uint32_t pm;     // label PRG digits per AES block (core.h prg_digits)
    // division by D with a 32-bit reciprocal (Moller-Granlund 2011, "Improved division by invariant
    // integers"): Dn = D << sh normalized to [2^31, 2^32), v = floor((2^64 - 1) / Dn) - 2^32
    uint32_t Dn, v, sh;
};

__device__ __forceinline__ uint64_t mulhi64(uint64_t a, uint64_t b) { return __umul64hi(a, b); }

// floor(x / D), x < D * 2^32 (so the quotient fits 32 bits)
__device__ __forceinline__ uint32_t div64_32(uint64_t x, uint32_t D, uint64_t mD, uint32_t& rem) {
    // mD = floor(2^64 / D) underestimates x / D by less than 2, so one correction (a select, no loop)
    uint64_t q = mulhi64(x, mD);
    uint64_t r = x - q * D;
    if (r >= D) {
        r -= D;
        ++q;
    }
    rem = static_cast<uint32_t>(r);
    return static_cast<uint32_t>(q);
}

// x / q for x < 2^32, q < 2^16
__device__ __forceinline__ uint32_t div32_q(uint32_t x, uint32_t q, uint32_t mq, uint32_t& rem) {
    uint32_t d = __umulhi(x, mq);
    uint32_t r = x - d * q;
    if (r >= q) {
        r -= q;
        ++d;
    }
    rem = r;
    return d;
}

// x mod q for 0 <= x < 2^32: reciprocal multiply + one correction. The
// compiler's `%` by a runtime divisor is a ~25-op v_rcp_iflag sequence (and a
// 64-bit `%` several times that); this is 4-5 ops, a mask for powers of two
// (m.bits is uniform per launch).
__device__ __forceinline__ uint32_t modq(uint32_t x, const ModC& m) {
    if (m.bits) return x & (m.q - 1);
    uint32_t r;
    div32_q(x, m.q, m.mq, r);
    return r;
}

// x mod q for a 64-bit x (q < 2^16): (hi mod q) * (2^32 mod q) + lo mod q
__device__ __forceinline__ uint32_t modq64(uint64_t x, const ModC& m) {
    const uint32_t h = modq(static_cast<uint32_t>(x >> 32), m), l = modq(static_cast<uint32_t>(x), m);
    const uint32_t t = modq(0xffffffffu, m) + 1u;  // 2^32 mod q, or q itself
    return modq(h * t + l, m);
}

// (Q, r) = divmod(Q, D)
// One step of the preinverted division: (u1 * 2^32 + u0) / Dn for u1 < Dn; quotient returned, remainder in r.
// One 32 x 32 -> 64 multiply-add, one 32-bit multiply and two corrections (selects): about half the
// quarter-rate multiplies of the 64-bit reciprocal form (div64_32).
__device__ __forceinline__ uint32_t mg_step(uint32_t u1, uint32_t u0, uint32_t Dn, uint32_t v, uint32_t& r) {
    const uint64_t pr = static_cast<uint64_t>(v) * u1 + u0;
    uint32_t ql = static_cast<uint32_t>(pr);
    uint32_t qh = static_cast<uint32_t>(pr >> 32) + u1 + 1u;
    uint32_t rr = u0 - qh * Dn;
    if (rr > ql) {
        --qh;
        rr += Dn;
    }
    if (rr >= Dn) {
        ++qh;
        rr -= Dn;
    }
    r = rr;
    return qh;
}
// Q / D in place, remainder returned, for D = m.D (odd modulus chunk, D < 2^31 so 1 <= sh <= 31): the
// numerator is shifted by sh (five limbs, the top one below Dn) and divided by Dn limb by limb.
__device__ __forceinline__ uint32_t divmod128(u128& Q, const struct ModC& m) {
    const uint32_t l3 = static_cast<uint32_t>(Q >> 96), l2 = static_cast<uint32_t>(Q >> 64);
    const uint32_t l1 = static_cast<uint32_t>(Q >> 32), l0 = static_cast<uint32_t>(Q);
    const uint32_t sh = m.sh, rs = 32u - sh;  // 1 <= sh <= 31
    const uint32_t u4 = l3 >> rs;
    const uint32_t u3 = __builtin_amdgcn_alignbit(l3, l2, rs), u2 = __builtin_amdgcn_alignbit(l2, l1, rs);
    const uint32_t u1 = __builtin_amdgcn_alignbit(l1, l0, rs), u0 = l0 << sh;
    uint32_t r, q3 = 0, q2 = 0;
    if (l3 | l2) {
        q3 = mg_step(u4, u3, m.Dn, m.v, r);
        q2 = mg_step(r, u2, m.Dn, m.v, r);
    } else {
        r = u2;  // Q < 2^64: the shifted top limbs are u2 = l1 >> (32 - sh) < 2^31 <= Dn, no quotient bits
    }
    const uint32_t q1 = mg_step(r, u1, m.Dn, m.v, r);
    const uint32_t q0 = mg_step(r, u0, m.Dn, m.v, r);
    Q = (static_cast<u128>((static_cast<uint64_t>(q3) << 32) | q2) << 64) | ((static_cast<uint64_t>(q1) << 32) | q0);
    return r >> sh;
}
__device__ __forceinline__ uint32_t divmod128(u128& Q, uint32_t D, uint64_t mD) {
    uint32_t l3 = static_cast<uint32_t>(Q >> 96), l2 = static_cast<uint32_t>(Q >> 64);
    uint32_t l1 = static_cast<uint32_t>(Q >> 32), l0 = static_cast<uint32_t>(Q);
    uint32_t r = 0;
    uint32_t q3 = 0, q2 = 0, q1, q0;
    if (l3 | l2) {
        q3 = div64_32(static_cast<uint64_t>(l3), D, mD, r);
        q2 = div64_32((static_cast<uint64_t>(r) << 32) | l2, D, mD, r);
    }
    q1 = div64_32((static_cast<uint64_t>(r) << 32) | l1, D, mD, r);
    q0 = div64_32((static_cast<uint64_t>(r) << 32) | l0, D, mD, r);
    Q = (static_cast<u128>((static_cast<uint64_t>(q3) << 32) | q2) << 64) | ((static_cast<uint64_t>(q1) << 32) | q0);
    return r;
}

#ifndef DASH_DIGIT_MAGIC
#define DASH_DIGIT_MAGIC 1
#endif
#ifndef DASH_CHUNK_BITS
#define DASH_CHUNK_BITS 31  // D = q^c <= 2^DASH_CHUNK_BITS (31 for the digit magic)
#endif
// Streaming decompress: digits of P in base q, least significant first.
struct DigitStream {
    u128 Q;
    uint32_t r, left;
    __device__ __forceinline__ void init(u128 P) {
        Q = P;
        r = 0;
        left = 0;
    }
    __device__ __forceinline__ uint32_t next(const ModC& m) {
        if (m.bits) {
            uint32_t d = static_cast<uint32_t>(Q) & (m.q - 1);
            Q >>= m.bits;
            return d;
        }
        if (left == 0) {
            r = divmod128(Q, m);
            left = m.c;
        }
        // r < D <= 2^31: exact quotient by multiply-high + shift; the digit (< q < 2^24) from the low
        // 24 bits of r - quot * q, so the product can be the full-rate 24-bit multiply
#if DASH_DIGIT_MAGIC
        const uint32_t quot = __umulhi(r, m.dm) >> m.ds;
        const uint32_t d = (r - __umul24(quot, m.q)) & 0xFFFFFFu;
        r = quot;
#else
        uint32_t d;
        r = div32_q(r, m.q, m.mq, d);
#endif
        --left;
        return d;
    }
};

// Chunk-major digit extraction (callers that walk whole chunks of m.c digits with a wave-uniform trip count):
// r = divmod128(Q, m) starts a chunk, chunk_digit(r, m) returns its next digit. The same digits as
// DigitStream::next without the per-digit chunk bookkeeping.
__device__ __forceinline__ uint32_t chunk_digit(uint32_t& r, const ModC& m) {
#if DASH_DIGIT_MAGIC
    const uint32_t quot = __umulhi(r, m.dm) >> m.ds;
    const uint32_t d = (r - __umul24(quot, m.q)) & 0xFFFFFFu;
    r = quot;
#else
    uint32_t d;
    r = div32_q(r, m.q, m.mq, d);
#endif
    return d;
}

// top digit needs a final reduction (matches host decompress for any payload)
__device__ __forceinline__ uint32_t reduce_top(uint32_t d, const ModC& m) { return d % m.q; }

// Streaming forward compress: push digits from least significant upwards.
// Power-of-two moduli pack digits into a 32-bit word first and place whole
// words into the u128 (one variable 128-bit shift per word, not per digit:
// a mod-2 label has 128 digits).
struct CompressFwd {
    u128 C, PW;
    uint32_t v, pt, cnt, bp, sh;
    __device__ __forceinline__ void init() {
        C = 0;
        PW = 1;
        v = 0;
        pt = 1;
        cnt = 0;
        bp = 0;
        sh = 0;
    }
    __device__ __forceinline__ void push(uint32_t d, const ModC& m) {
        if (m.bits) {
            v |= d << bp;
            bp += m.bits;
            if (bp + m.bits > 32) {
                C |= static_cast<u128>(v) << sh;
                sh += bp;
                v = 0;
                bp = 0;
            }
            return;
        }
        v += d * pt;
        pt *= m.q;
        if (++cnt == m.c) {
            C += PW * static_cast<u128>(v);
            PW *= static_cast<u128>(m.D);
            v = 0;
            pt = 1;
            cnt = 0;
        }
    }
    __device__ __forceinline__ u128 finish() {
        if (bp) C |= static_cast<u128>(v) << sh;  // bits path (bp stays 0 otherwise)
        else if (cnt && v) C += PW * static_cast<u128>(v);
        return C;
    }
};

// Label columns are component-major (stride N). A component loop whose
// iteration waits for its own load pays one HBM round trip per component
// (the compiler does not hoist loads across a runtime-trip-count loop, nor
// past a store to the same column): stage kChunk loads first, then consume.
#ifndef DASH_KCHUNK
#define DASH_KCHUNK 8  // 24 GCs: 16 -> 12.96, 8 -> 12.39, 32 -> 19.44 ms per step (profiles/ab/kchunk*.json)
#endif
constexpr int kChunk = DASH_KCHUNK;

// dst[c * stride] = f(c, src[c * stride]) for c < n, kChunk loads per round
// trip (dst may alias src; f is called in component order)
template <class T, class U, class F>
__device__ __forceinline__ void col_map(const T* src, U* dst, long stride, int n, F&& f) {
    for (int i0 = 0; i0 < n; i0 += kChunk) {
        int16_t v[kChunk];
#pragma unroll
        for (int u = 0; u < kChunk; ++u)
            if (i0 + u < n) v[u] = src[static_cast<long>(i0 + u) * stride];
#pragma unroll
        for (int u = 0; u < kChunk; ++u)
            if (i0 + u < n) dst[static_cast<long>(i0 + u) * stride] = f(i0 + u, v[u]);
    }
}

// compress of a label stored component-major: L[i * stride], streamed from
// the least significant component, kChunk loads in flight per round trip
template <int CH = kChunk, class T>
__device__ __forceinline__ u128 compress_cm(const T* L, long stride, const ModC& m) {
    const int n = m.n;
    CompressFwd cf;
    cf.init();
    for (int i0 = 0; i0 < n; i0 += CH) {
        uint16_t v[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u)
            if (i0 + u < n) v[u] = static_cast<uint16_t>(L[static_cast<long>(i0 + u) * stride]);
#pragma unroll
        for (int u = 0; u < CH; ++u)
            if (i0 + u < n) cf.push(v[u], m);
    }
    return cf.finish();
}

// P mod q (color of a compressed label)
__device__ __forceinline__ uint32_t u128_mod(u128 P, const ModC& m) {
    if (m.bits) return static_cast<uint32_t>(P) & (m.q - 1);
    u128 Q = P;
    uint32_t r = divmod128(Q, m);
    uint32_t d;
    div32_q(r, m.q, m.mq, d);
    return d;
}

// ---------------------------------------------------------------------------
// AES-128 (fixed key 00..0f), T-table form tuned for CDNA4.
//
// LDS image (64 KiB): 256 rows of 256 B; row x holds Te0[x] in words 0..31
// and Te2[x] = ror16(Te0[x]) in words 32..63 (32 copies each). Lane l reads
// copy (l mod 32), so a ds_read_b32 from 32 lanes hits 32 distinct banks
// (bank = (addr/4) mod 32) whatever the indices: conflict-free.
// The byte offset of a lookup, (byte_i(s) << 8) | (4 * (lane mod 32)), is a
// single v_perm_b32; Te2 sits at +128 B (instruction offset field). With
// Te1 = ror8(Te0) and Te3 = ror8(Te2) one AES column costs
//   4 perm + 4 ds_read + xor3 + alignbit + xor3
// (the round key is folded into the rotated xor3 as rol8(rk)): ~7 VALU per
// column vs ~16 for a byte-extract/shift/add/rotate formulation.
// The round keys of the fixed key are compile-time constants (the key is part
// of the scheme, crypto/cpu_aes_engine.h:23-24), so they become literals.
// DASH_AES_COPIES < 32 shrinks the image (2 KiB per copy) at the price of
// (32 / copies)-way bank conflicts: more resident blocks per CU (A/B knob).
#ifndef DASH_AES_COPIES
#define DASH_AES_COPIES 16
#endif
#define DASH_AES_LDS_BYTES (2048 * DASH_AES_COPIES)
#define DASH_AES_LDS_WORDS (DASH_AES_LDS_BYTES / 4)
// Image size for C copies (the garbler's AES-bound kernels use the conflict-free 32-copy image, 64 KiB)
template <int C>
constexpr int aes_lds_words() { return 512 * C; }

__device__ constexpr uint32_t kAesRk[44] = {
    0x00010203u, 0x04050607u, 0x08090a0bu, 0x0c0d0e0fu, 0xd6aa74fdu, 0xd2af72fau, 0xdaa678f1u, 0xd6ab76feu,
    0xb692cf0bu, 0x643dbdf1u, 0xbe9bc500u, 0x6830b3feu, 0xb6ff744eu, 0xd2c2c9bfu, 0x6c590cbfu, 0x0469bf41u,
    0x47f7f7bcu, 0x95353e03u, 0xf96c32bcu, 0xfd058dfdu, 0x3caaa3e8u, 0xa99f9debu, 0x50f3af57u, 0xadf622aau,
    0x5e390f7du, 0xf7a69296u, 0xa7553dc1u, 0x0aa31f6bu, 0x14f9701au, 0xe35fe28cu, 0x440adf4du, 0x4ea9c026u,
    0x47438735u, 0xa41c65b9u, 0xe016baf4u, 0xaebf7ad2u, 0x549932d1u, 0xf0855768u, 0x1093ed9cu, 0xbe2c974eu,
    0x13111d7fu, 0xe3944a17u, 0xf307a78bu, 0x4d2b30c5u};

// LDS image of C copies: row x = C words of Te0[x], then C words of Te2[x] (8 * C bytes per row)
template <int C>
struct AesT {
    static constexpr uint32_t kRow = 8 * C;  // bytes per table row
    static constexpr uint32_t kT2 = 4 * C;   // offset of the Te2 copies inside a row
    const char* T;  // LDS image base
    uint32_t lo;    // 4 * (lane mod C)
};
using AesCtx = AesT<DASH_AES_COPIES>;

__device__ __forceinline__ uint32_t ror32(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }
__device__ __forceinline__ uint32_t rol32c(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// byte offset of row byte_I(s), lane copy (C = 32: D = {0, 0, s.byte[I], lo.byte[0]}, one v_perm_b32)
template <int I, int C>
__device__ __forceinline__ uint32_t aes_off(uint32_t s, uint32_t lo) {
    if constexpr (C == 32) return __builtin_amdgcn_perm(s, lo, 0x0c0c0000u | ((4u + I) << 8));
    else return (((s >> (8 * I)) & 0xffu) * AesT<C>::kRow) | lo;
}
template <int I, int C>
__device__ __forceinline__ uint32_t aes_t0(const AesT<C>& a, uint32_t s) {
    return *reinterpret_cast<const uint32_t*>(a.T + aes_off<I, C>(s, a.lo));
}
template <int I, int C>
__device__ __forceinline__ uint32_t aes_t2(const AesT<C>& a, uint32_t s) {
    return *reinterpret_cast<const uint32_t*>(a.T + aes_off<I, C>(s, a.lo) + AesT<C>::kT2);
}
// three-input XOR in one VALU op (v_bitop3_b32, truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
// one output column of a middle round: Te0[s0.b3]^Te1[s1.b2]^Te2[s2.b1]^Te3[s3.b0]^rk
template <int C>
__device__ __forceinline__ uint32_t aes_col(const AesT<C>& a, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3,
                                            uint32_t rk) {
    const uint32_t u = xor3(aes_t0<2, C>(a, s1), aes_t2<0, C>(a, s3), rol32c(rk, 8));
    return xor3(aes_t0<3, C>(a, s0), aes_t2<1, C>(a, s2), ror32(u, 8));
}
// final round column: S-box bytes sit at Te2.b3, Te0.b2, Te0.b1, Te2.b0
template <int C>
__device__ __forceinline__ uint32_t aes_last(const AesT<C>& a, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3,
                                             uint32_t rk) {
    const uint32_t x1 = __builtin_amdgcn_perm(aes_t2<3, C>(a, s0), aes_t0<2, C>(a, s1), 0x07020c0cu);
    const uint32_t x2 = __builtin_amdgcn_perm(aes_t0<1, C>(a, s2), aes_t2<0, C>(a, s3), 0x0c0c0500u);
    return xor3(x1, x2, rk);
}

template <int C>
__device__ __forceinline__ u128 aes_encrypt(const AesT<C>& a, u128 in) {
    uint32_t s0 = bswap32(static_cast<uint32_t>(in)) ^ kAesRk[0];
    uint32_t s1 = bswap32(static_cast<uint32_t>(in >> 32)) ^ kAesRk[1];
    uint32_t s2 = bswap32(static_cast<uint32_t>(in >> 64)) ^ kAesRk[2];
    uint32_t s3 = bswap32(static_cast<uint32_t>(in >> 96)) ^ kAesRk[3];
#pragma unroll
    for (int r = 1; r < 10; ++r) {
        const uint32_t t0 = aes_col(a, s0, s1, s2, s3, kAesRk[4 * r + 0]);
        const uint32_t t1 = aes_col(a, s1, s2, s3, s0, kAesRk[4 * r + 1]);
        const uint32_t t2 = aes_col(a, s2, s3, s0, s1, kAesRk[4 * r + 2]);
        const uint32_t t3 = aes_col(a, s3, s0, s1, s2, kAesRk[4 * r + 3]);
        s0 = t0;
        s1 = t1;
        s2 = t2;
        s3 = t3;
    }
    const uint32_t o0 = aes_last(a, s0, s1, s2, s3, kAesRk[40]);
    const uint32_t o1 = aes_last(a, s1, s2, s3, s0, kAesRk[41]);
    const uint32_t o2 = aes_last(a, s2, s3, s0, s1, kAesRk[42]);
    const uint32_t o3 = aes_last(a, s3, s0, s1, s2, kAesRk[43]);
    return (static_cast<u128>((static_cast<uint64_t>(bswap32(o3)) << 32) | bswap32(o2)) << 64) |
           ((static_cast<uint64_t>(bswap32(o1)) << 32) | bswap32(o0));
}

// Two independent blocks with interleaved rounds: doubles the LDS-read ILP of
// a latency-bound lane (the serial sign chain).
template <int C>
__device__ __forceinline__ void aes_encrypt2(const AesT<C>& a, u128 inA, u128 inB, u128& outA, u128& outB) {
    uint32_t a0 = bswap32(static_cast<uint32_t>(inA)) ^ kAesRk[0], a1 = bswap32(static_cast<uint32_t>(inA >> 32)) ^ kAesRk[1];
    uint32_t a2 = bswap32(static_cast<uint32_t>(inA >> 64)) ^ kAesRk[2], a3 = bswap32(static_cast<uint32_t>(inA >> 96)) ^ kAesRk[3];
    uint32_t b0 = bswap32(static_cast<uint32_t>(inB)) ^ kAesRk[0], b1 = bswap32(static_cast<uint32_t>(inB >> 32)) ^ kAesRk[1];
    uint32_t b2 = bswap32(static_cast<uint32_t>(inB >> 64)) ^ kAesRk[2], b3 = bswap32(static_cast<uint32_t>(inB >> 96)) ^ kAesRk[3];
#pragma unroll
    for (int r = 1; r < 10; ++r) {
        const uint32_t ta0 = aes_col(a, a0, a1, a2, a3, kAesRk[4 * r + 0]);
        const uint32_t tb0 = aes_col(a, b0, b1, b2, b3, kAesRk[4 * r + 0]);
        const uint32_t ta1 = aes_col(a, a1, a2, a3, a0, kAesRk[4 * r + 1]);
        const uint32_t tb1 = aes_col(a, b1, b2, b3, b0, kAesRk[4 * r + 1]);
        const uint32_t ta2 = aes_col(a, a2, a3, a0, a1, kAesRk[4 * r + 2]);
        const uint32_t tb2 = aes_col(a, b2, b3, b0, b1, kAesRk[4 * r + 2]);
        const uint32_t ta3 = aes_col(a, a3, a0, a1, a2, kAesRk[4 * r + 3]);
        const uint32_t tb3 = aes_col(a, b3, b0, b1, b2, kAesRk[4 * r + 3]);
        a0 = ta0; a1 = ta1; a2 = ta2; a3 = ta3;
        b0 = tb0; b1 = tb1; b2 = tb2; b3 = tb3;
    }
    auto fin = [&](uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3) -> u128 {
        const uint32_t o0 = aes_last(a, s0, s1, s2, s3, kAesRk[40]);
        const uint32_t o1 = aes_last(a, s1, s2, s3, s0, kAesRk[41]);
        const uint32_t o2 = aes_last(a, s2, s3, s0, s1, kAesRk[42]);
        const uint32_t o3 = aes_last(a, s3, s0, s1, s2, kAesRk[43]);
        return (static_cast<u128>((static_cast<uint64_t>(bswap32(o3)) << 32) | bswap32(o2)) << 64) |
               ((static_cast<uint64_t>(bswap32(o1)) << 32) | bswap32(o0));
    };
    outA = fin(a0, a1, a2, a3);
    outB = fin(b0, b1, b2, b3);
}

// ---------------------------------------------------------------------------
// Hardened-encoding pads (core.h hard_block): ChaCha12 on
//   [sigma][K (4 words)][gate lo, gate hi, sub, "HARD"][blk, 0, 0, 0]
// with feed-forward; pad q of the block = words 4q..4q+3. Pure VALU (adds, xors, 32-bit rotates as
// v_alignbit): no LDS image, unlike the T-table AES, so hardened kernels leave the LDS to staging.
constexpr int kDevChaRounds = 12;  // = core.h kChaRounds: part of the hardened encoding, not a tuning knob
__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return __builtin_rotateleft32(x, r); }
#define DASH_QR(a, b, c, d)                 \
    a += b; d = rotl(d ^ a, 16);            \
    c += d; b = rotl(b ^ c, 12);            \
    a += b; d = rotl(d ^ a, 8);             \
    c += d; b = rotl(b ^ c, 7);
__device__ __forceinline__ void hard_block(u128 K, uint64_t gate, uint32_t sub, uint32_t blk, u128 (&out)[4]) {
    const uint32_t k0 = static_cast<uint32_t>(K), k1 = static_cast<uint32_t>(K >> 32);
    const uint32_t k2 = static_cast<uint32_t>(K >> 64), k3 = static_cast<uint32_t>(K >> 96);
    const uint32_t g0 = static_cast<uint32_t>(gate), g1 = static_cast<uint32_t>(gate >> 32);
    uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
    uint32_t x4 = k0, x5 = k1, x6 = k2, x7 = k3, x8 = g0, x9 = g1, x10 = sub, x11 = 0x44524148u;
    uint32_t x12 = blk, x13 = 0, x14 = 0, x15 = 0;
    // NOT unrolled: a kernel inlines this block at every table row it unmasks (the K = 7 chain: ~15 sites), and
    // fully unrolled each copy was ~9 KiB of code, pushing the chain kernels to 70-95 KiB, beyond the
    // instruction cache shared by two CUs. The loop costs 3 scalar instructions per double round.
#pragma unroll 1
    for (int r = 0; r < kDevChaRounds; r += 2) {
        DASH_QR(x0, x4, x8, x12) DASH_QR(x1, x5, x9, x13) DASH_QR(x2, x6, x10, x14) DASH_QR(x3, x7, x11, x15)
        DASH_QR(x0, x5, x10, x15) DASH_QR(x1, x6, x11, x12) DASH_QR(x2, x7, x8, x13) DASH_QR(x3, x4, x9, x14)
    }
    x0 += 0x61707865u; x1 += 0x3320646eu; x2 += 0x79622d32u; x3 += 0x6b206574u;
    x4 += k0; x5 += k1; x6 += k2; x7 += k3; x8 += g0; x9 += g1; x10 += sub; x11 += 0x44524148u;
    x12 += blk;
    auto pk = [](uint32_t a, uint32_t b, uint32_t c, uint32_t d) -> u128 {
        return (static_cast<u128>((static_cast<uint64_t>(d) << 32) | c) << 64) | ((static_cast<uint64_t>(b) << 32) | a);
    };
    out[0] = pk(x0, x1, x2, x3);
    out[1] = pk(x4, x5, x6, x7);
    out[2] = pk(x8, x9, x10, x11);
    out[3] = pk(x12, x13, x14, x15);
}
// Quad-cooperative block (the four lanes of a quad, all active, the same K / gate / sub / blk in each): lane
// j = lane & 3 holds state column j (words j, 4 + j, 8 + j, 12 + j). Column rounds are lane-local; a diagonal
// round rotates rows 1-3 by 1-3 lanes (DPP quad_perm), runs the same quarter round and rotates back. On return
// x[q] = word j of pad q. A quarter of hard_block's VALU work per lane plus six lane moves per double round: a
// latency-bound chain whose lanes each ran a whole block per row (batch 1) waits a quarter as long.
#ifndef DASH_MRS_QCOOP
#define DASH_MRS_QCOOP 1  // A/B knob: quad-cooperative pad blocks in the quad kernels; 0 = block g on lane g
#endif
constexpr bool kQCoop = DASH_MRS_QCOOP != 0;
template <int CTRL>
__device__ __forceinline__ uint32_t qperm(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), CTRL, 0xF, 0xF, false));
}
constexpr int kQRot1 = 0x39, kQRot2 = 0x4E, kQRot3 = 0x93;  // quad_perm: lane i reads lane (i + 1, 2, 3) & 3
__device__ __forceinline__ void hard_block_q(u128 K, uint64_t gate, uint32_t sub, uint32_t blk, int j, uint32_t (&x)[4]) {
    const uint32_t sig = j == 0 ? 0x61707865u : (j == 1 ? 0x3320646eu : (j == 2 ? 0x79622d32u : 0x6b206574u));
    const uint32_t kj = j == 0 ? static_cast<uint32_t>(K)
                               : (j == 1 ? static_cast<uint32_t>(K >> 32)
                                         : (j == 2 ? static_cast<uint32_t>(K >> 64) : static_cast<uint32_t>(K >> 96)));
    const uint32_t cj = j == 0 ? static_cast<uint32_t>(gate)
                               : (j == 1 ? static_cast<uint32_t>(gate >> 32) : (j == 2 ? sub : 0x44524148u));
    const uint32_t dj = j == 0 ? blk : 0u;
    uint32_t a = sig, b = kj, c = cj, d = dj;
#pragma unroll 1
    for (int r = 0; r < kDevChaRounds; r += 2) {
        DASH_QR(a, b, c, d)
        b = qperm<kQRot1>(b);
        c = qperm<kQRot2>(c);
        d = qperm<kQRot3>(d);
        DASH_QR(a, b, c, d)
        b = qperm<kQRot3>(b);
        c = qperm<kQRot2>(c);
        d = qperm<kQRot1>(d);
    }
    x[0] = a + sig;
    x[1] = b + kj;
    x[2] = c + cj;
    x[3] = d + dj;
}
// the 128-bit value whose word j sits in quad lane j, in every lane of the quad
__device__ __forceinline__ u128 quad_gather128(uint32_t w) {
    const uint32_t w0 = qperm<0x00>(w), w1 = qperm<0x55>(w), w2 = qperm<0xAA>(w), w3 = qperm<0xFF>(w);
    return (static_cast<u128>((static_cast<uint64_t>(w3) << 32) | w2) << 64) | ((static_cast<uint64_t>(w1) << 32) | w0);
}
#undef DASH_QR

// Tweak kinds (core.h TweakKind) and the sub word of row `idx`
constexpr uint32_t kTwApprox = 1, kTwCast2 = 3, kTwSign = 4, kTwMmg = 5, kTwMmy = 6, kTwMrs = 7, kTwSmrs = 8,
                   kTwBe = 9, kTwTrans = 10, kTwProj = 11, kTwGme = 12, kTwMmt = 13;
__host__ __device__ __forceinline__ constexpr uint32_t tw_sub(uint32_t kind, uint32_t idx) { return (kind << 16) | (idx & 0xffffu); }
// gate of element e of a gadget whose PRG streams are stream_id(L, slot, e) (core.h): base = stream_id(L, slot, 0)
__host__ __device__ __forceinline__ constexpr uint64_t gate_base(uint64_t layer, uint64_t slot) {
    return (layer << 44) ^ (slot << 36);
}

// E[t] -= pad t of (K, gate, sub) for t < NT (fan-out row of NT entries, blocks of four pads)
template <int NT>
__device__ __forceinline__ void hard_unmask(u128 (&E)[NT], u128 K, uint64_t gate, uint32_t sub) {
#pragma unroll
    for (int b = 0; b < (NT + 3) / 4; ++b) {
        u128 p[4];
        hard_block(K, gate, sub, static_cast<uint32_t>(b), p);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (4 * b + q < NT) E[4 * b + q] -= p[q];
    }
}
// runtime row length nt <= NT
template <int NT>
__device__ __forceinline__ void hard_unmask_n(u128 (&E)[NT], int nt, u128 K, uint64_t gate, uint32_t sub) {
#pragma unroll
    for (int b = 0; b < (NT + 3) / 4; ++b) {
        if (4 * b >= nt) break;
        u128 p[4];
        hard_block(K, gate, sub, static_cast<uint32_t>(b), p);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (4 * b + q < nt) E[4 * b + q] -= p[q];
    }
}
// single pad of slot s
__device__ __forceinline__ u128 hard_pad(u128 K, uint64_t gate, uint32_t sub, int s) {
    u128 p[4];
    hard_block(K, gate, sub, static_cast<uint32_t>(s) >> 2, p);
    const int q = s & 3;
    return q == 0 ? p[0] : (q == 1 ? p[1] : (q == 2 ? p[2] : p[3]));
}

// Global tables: Te0 (256 words); rk kept for the launch ABI (round keys are literals).
struct AesGlobals {
    const uint32_t* te0;
    const uint32_t* rk;
};

// Fill the LDS image; all threads of the block participate.
template <int C = DASH_AES_COPIES>
__device__ __forceinline__ void aes_lds_fill(uint32_t* lds, const uint32_t* te0) {
    // 16-B LDS stores: the 4 words of an aligned quad share the table entry
    // and the rotation, so every block's image costs a quarter of the loads
    // and LDS writes of a word-wise fill
    // kU table loads in flight per thread before their stores: a small block (batch-1 launches shrink to one
    // wave) walks the image in total / nt rounds, and one load round trip per round made the fill a floor of
    // every small AES launch
    constexpr int kU = 8;
    constexpr int total = aes_lds_words<C>() / 4;
    const int nt = blockDim.x * blockDim.y;
    for (int i0 = threadIdx.x + threadIdx.y * blockDim.x; i0 < total; i0 += kU * nt) {
        uint32_t v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int i4 = i0 + u * nt;
            v[u] = i4 < total ? te0[(4 * i4) / (2 * C)] : 0u;
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int i4 = i0 + u * nt;
            if (i4 >= total) break;
            const uint32_t w = ((4 * i4) % (2 * C) >= C) ? ror32(v[u], 16) : v[u];
            reinterpret_cast<uint4*>(lds)[i4] = make_uint4(w, w, w, w);
        }
    }
    __syncthreads();
}

template <int C = DASH_AES_COPIES>
__device__ __forceinline__ AesT<C> aes_ctx(const uint32_t* lds, const uint32_t* /*rk*/) {
    AesT<C> a;
    a.T = reinterpret_cast<const char*>(lds);
    a.lo = (__lane_id() % C) << 2;
    return a;
}

__device__ __forceinline__ u128 ld128(const u128* p) { return *p; }

}  // namespace dev
}  // namespace dash
