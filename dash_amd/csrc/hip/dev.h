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
};

__device__ __forceinline__ uint64_t mulhi64(uint64_t a, uint64_t b) { return __umul64hi(a, b); }

// floor(x / D), x < D * 2^32 (so the quotient fits 32 bits)
__device__ __forceinline__ uint32_t div64_32(uint64_t x, uint32_t D, uint64_t mD, uint32_t& rem) {
    uint64_t q = mulhi64(x, mD);
    uint64_t r = x - q * D;
    while (r >= D) {
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

// (Q, r) = divmod(Q, D)
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
            r = divmod128(Q, m.D, m.mD);
            left = m.c;
        }
        uint32_t d;
        r = div32_q(r, m.q, m.mq, d);
        --left;
        return d;
    }
};

// top digit needs a final reduction (matches host decompress for any payload)
__device__ __forceinline__ uint32_t reduce_top(uint32_t d, const ModC& m) { return d % m.q; }

// Streaming forward compress: push digits from least significant upwards.
struct CompressFwd {
    u128 C, PW;
    uint32_t v, pt, cnt;
    __device__ __forceinline__ void init() {
        C = 0;
        PW = 1;
        v = 0;
        pt = 1;
        cnt = 0;
    }
    __device__ __forceinline__ void push(uint32_t d, const ModC& m) {
        if (m.bits) {
            C |= static_cast<u128>(d) << (m.bits * cnt);
            ++cnt;
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
        if (cnt && v) C += PW * static_cast<u128>(v);
        return C;
    }
};

// compress of a label stored component-major: L[i * stride] (reverse Horner)
__device__ __forceinline__ u128 compress_cm(const int16_t* L, long stride, const ModC& m) {
    const int n = m.n;
    if (m.bits) {
        u128 C = 0;
        for (int i = n - 1; i >= 0; --i) C = (C << m.bits) | static_cast<u128>(static_cast<uint16_t>(L[i * stride]));
        return C;
    }
    int first = n % m.c;
    if (first == 0) first = m.c;
    int i = n - 1;
    uint32_t v = 0;
    for (int t = 0; t < first; ++t, --i) v = v * m.q + static_cast<uint16_t>(L[i * stride]);
    u128 C = v;
    while (i >= 0) {
        v = 0;
        for (int t = 0; t < static_cast<int>(m.c); ++t, --i) v = v * m.q + static_cast<uint16_t>(L[i * stride]);
        C = C * static_cast<u128>(m.D) + v;
    }
    return C;
}

// P mod q (color of a compressed label)
__device__ __forceinline__ uint32_t u128_mod(u128 P, const ModC& m) {
    if (m.bits) return static_cast<uint32_t>(P) & (m.q - 1);
    u128 Q = P;
    uint32_t r = divmod128(Q, m.D, m.mD);
    uint32_t d;
    div32_q(r, m.q, m.mq, d);
    return d;
}

// ---------------------------------------------------------------------------
// AES-128 (fixed key)
struct AesCtx {
    const uint32_t* T;   // LDS: 256 entries x 32 copies
    const uint32_t* rk;  // 44 round key words (big-endian column words)
    uint32_t lane32;
};

__device__ __forceinline__ uint32_t ror32(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ uint32_t te(const AesCtx& a, uint32_t idx) { return a.T[(idx << 5) | a.lane32]; }

__device__ __forceinline__ u128 aes_encrypt(const AesCtx& a, u128 in) {
    const uint32_t* rk = a.rk;
    uint32_t s0 = bswap32(static_cast<uint32_t>(in)) ^ rk[0];
    uint32_t s1 = bswap32(static_cast<uint32_t>(in >> 32)) ^ rk[1];
    uint32_t s2 = bswap32(static_cast<uint32_t>(in >> 64)) ^ rk[2];
    uint32_t s3 = bswap32(static_cast<uint32_t>(in >> 96)) ^ rk[3];
    uint32_t t0, t1, t2, t3;
#pragma unroll
    for (int r = 1; r < 10; ++r) {
        t0 = te(a, s0 >> 24) ^ ror32(te(a, (s1 >> 16) & 0xff), 8) ^ ror32(te(a, (s2 >> 8) & 0xff), 16) ^
             ror32(te(a, s3 & 0xff), 24) ^ rk[4 * r + 0];
        t1 = te(a, s1 >> 24) ^ ror32(te(a, (s2 >> 16) & 0xff), 8) ^ ror32(te(a, (s3 >> 8) & 0xff), 16) ^
             ror32(te(a, s0 & 0xff), 24) ^ rk[4 * r + 1];
        t2 = te(a, s2 >> 24) ^ ror32(te(a, (s3 >> 16) & 0xff), 8) ^ ror32(te(a, (s0 >> 8) & 0xff), 16) ^
             ror32(te(a, s1 & 0xff), 24) ^ rk[4 * r + 2];
        t3 = te(a, s3 >> 24) ^ ror32(te(a, (s0 >> 16) & 0xff), 8) ^ ror32(te(a, (s1 >> 8) & 0xff), 16) ^
             ror32(te(a, s2 & 0xff), 24) ^ rk[4 * r + 3];
        s0 = t0;
        s1 = t1;
        s2 = t2;
        s3 = t3;
    }
    // final round: S-box = byte 2 of Te0 (Te0[x] = 2s | s | s | 3s)
    auto S = [&](uint32_t x) { return (te(a, x) >> 8) & 0xffu; };
    uint32_t o0 = (S(s0 >> 24) << 24) ^ (S((s1 >> 16) & 0xff) << 16) ^ (S((s2 >> 8) & 0xff) << 8) ^ S(s3 & 0xff) ^ rk[40];
    uint32_t o1 = (S(s1 >> 24) << 24) ^ (S((s2 >> 16) & 0xff) << 16) ^ (S((s3 >> 8) & 0xff) << 8) ^ S(s0 & 0xff) ^ rk[41];
    uint32_t o2 = (S(s2 >> 24) << 24) ^ (S((s3 >> 16) & 0xff) << 16) ^ (S((s0 >> 8) & 0xff) << 8) ^ S(s1 & 0xff) ^ rk[42];
    uint32_t o3 = (S(s3 >> 24) << 24) ^ (S((s0 >> 16) & 0xff) << 16) ^ (S((s1 >> 8) & 0xff) << 8) ^ S(s2 & 0xff) ^ rk[43];
    return (static_cast<u128>((static_cast<uint64_t>(bswap32(o3)) << 32) | bswap32(o2)) << 64) |
           ((static_cast<uint64_t>(bswap32(o1)) << 32) | bswap32(o0));
}


// Two independent blocks with interleaved rounds: doubles the LDS-read ILP of
// a latency-bound lane (the serial sign chain) at no extra instructions.
__device__ __forceinline__ void aes_encrypt2(const AesCtx& a, u128 inA, u128 inB, u128& outA, u128& outB) {
    const uint32_t* rk = a.rk;
    uint32_t a0 = bswap32(static_cast<uint32_t>(inA)) ^ rk[0], a1 = bswap32(static_cast<uint32_t>(inA >> 32)) ^ rk[1];
    uint32_t a2 = bswap32(static_cast<uint32_t>(inA >> 64)) ^ rk[2], a3 = bswap32(static_cast<uint32_t>(inA >> 96)) ^ rk[3];
    uint32_t b0 = bswap32(static_cast<uint32_t>(inB)) ^ rk[0], b1 = bswap32(static_cast<uint32_t>(inB >> 32)) ^ rk[1];
    uint32_t b2 = bswap32(static_cast<uint32_t>(inB >> 64)) ^ rk[2], b3 = bswap32(static_cast<uint32_t>(inB >> 96)) ^ rk[3];
#define DASH_AES_COL(s0, s1, s2, s3, r)                                                              \
    (te(a, (s0) >> 24) ^ ror32(te(a, ((s1) >> 16) & 0xff), 8) ^ ror32(te(a, ((s2) >> 8) & 0xff), 16) ^ \
     ror32(te(a, (s3)&0xff), 24) ^ rk[r])
#pragma unroll
    for (int r = 1; r < 10; ++r) {
        uint32_t ta0 = DASH_AES_COL(a0, a1, a2, a3, 4 * r + 0);
        uint32_t tb0 = DASH_AES_COL(b0, b1, b2, b3, 4 * r + 0);
        uint32_t ta1 = DASH_AES_COL(a1, a2, a3, a0, 4 * r + 1);
        uint32_t tb1 = DASH_AES_COL(b1, b2, b3, b0, 4 * r + 1);
        uint32_t ta2 = DASH_AES_COL(a2, a3, a0, a1, 4 * r + 2);
        uint32_t tb2 = DASH_AES_COL(b2, b3, b0, b1, 4 * r + 2);
        uint32_t ta3 = DASH_AES_COL(a3, a0, a1, a2, 4 * r + 3);
        uint32_t tb3 = DASH_AES_COL(b3, b0, b1, b2, 4 * r + 3);
        a0 = ta0; a1 = ta1; a2 = ta2; a3 = ta3;
        b0 = tb0; b1 = tb1; b2 = tb2; b3 = tb3;
    }
#undef DASH_AES_COL
    auto S = [&](uint32_t x) { return (te(a, x) >> 8) & 0xffu; };
    auto last = [&](uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3) -> u128 {
        uint32_t o0 = (S(s0 >> 24) << 24) ^ (S((s1 >> 16) & 0xff) << 16) ^ (S((s2 >> 8) & 0xff) << 8) ^ S(s3 & 0xff) ^ rk[40];
        uint32_t o1 = (S(s1 >> 24) << 24) ^ (S((s2 >> 16) & 0xff) << 16) ^ (S((s3 >> 8) & 0xff) << 8) ^ S(s0 & 0xff) ^ rk[41];
        uint32_t o2 = (S(s2 >> 24) << 24) ^ (S((s3 >> 16) & 0xff) << 16) ^ (S((s0 >> 8) & 0xff) << 8) ^ S(s1 & 0xff) ^ rk[42];
        uint32_t o3 = (S(s3 >> 24) << 24) ^ (S((s0 >> 16) & 0xff) << 16) ^ (S((s1 >> 8) & 0xff) << 8) ^ S(s2 & 0xff) ^ rk[43];
        return (static_cast<u128>((static_cast<uint64_t>(bswap32(o3)) << 32) | bswap32(o2)) << 64) |
               ((static_cast<uint64_t>(bswap32(o1)) << 32) | bswap32(o0));
    };
    outA = last(a0, a1, a2, a3);
    outB = last(b0, b1, b2, b3);
}

// Global tables: Te0 (256 words) and the fixed-key round keys (44 words).
struct AesGlobals {
    const uint32_t* te0;
    const uint32_t* rk;
};

#define DASH_AES_LDS_WORDS (256 * 32)
// Fill the replicated LDS table; all threads of the block participate.
__device__ __forceinline__ void aes_lds_fill(uint32_t* lds, const uint32_t* te0) {
    for (int i = threadIdx.x + threadIdx.y * blockDim.x; i < DASH_AES_LDS_WORDS; i += blockDim.x * blockDim.y)
        lds[i] = te0[i >> 5];
    __syncthreads();
}

__device__ __forceinline__ AesCtx aes_ctx(const uint32_t* lds, const uint32_t* rk) {
    AesCtx a;
    a.T = lds;
    a.rk = rk;
    a.lane32 = threadIdx.x & 31;
    return a;
}

__device__ __forceinline__ u128 ld128(const u128* p) { return *p; }

}  // namespace dev
}  // namespace dash
