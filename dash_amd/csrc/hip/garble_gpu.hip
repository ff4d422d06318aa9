// GPU garbler for the sign-gadget layers (ReLU, Sign, DASH legacy rescale).
//
// Garbling is data independent: every random label comes from the AES-CTR
// PRG at a position (stream, counter) fixed by the gadget structure, and a
// projection table entry depends only on its input/output base labels. The
// CPU garbler walks each element serially (gadgets.cpp sign_garble_elem,
// mixed_mult_garble, rescale_garble_elem); here the same structure is turned
// into three massively parallel passes per gadget:
//   draw    one thread per (element, label slot): PRG labels at their counters
//   derive  one thread per element: label sums feeding later projections
//   project one thread per (element, table entry): key + i*R_in, AES, payload
// and the result is byte-identical with the CPU garbler (tests compare the
// serialized models). Reference parity: sign_gadget.h:425-581,
// garbled_relu.h:119-179, rescale_gadget.h:115-242.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <map>
#include <tuple>
#include <memory>
#include <mutex>
#include <string>

#include "../layers.h"
#include "dev.h"
#include "gpu_garbler.h"
#include "kargs.h"
#include "launch.h"
#include "host_util.h"

namespace dash {
using namespace dev;
using namespace hostutil;

namespace gg {

// The garbling stream of the calling thread (DevCtx::st, set by every GpuGarbler entry point): a
// non-blocking stream per device, so garbling never synchronizes with evaluation streams.
thread_local hipStream_t tl_st = nullptr;

constexpr int kW = 128;  // label slot width (max components)

// label reference kinds
enum Src : int { S_INPUT = 0, S_SLOT = 1, S_ZERO = 2 };
// projection functions
enum Fn : int { F_IDENT = 0, F_LUT = 1, F_DIV = 2, F_SIGN = 3, F_MULR = 4, F_NEGR = 5, F_DIVMOD = 6, F_FAN = 7 };
// output offset kinds
enum OutR : int { R_BANK = 0, R_INPUT = 1 };

struct Draw {
    int slot, q, ctr;  // label slot, modulus, first counter block
};
struct Proj {
    int in_kind, in_idx, pin;    // input label (input residue / slot / zero label of pin)
    int out_slot, pout;          // output base label slot
    int fn, a0, a1, a2;          // function + parameters
    int outr_kind, outr_idx;     // R_pout or input residue label
    int table, stride;           // table id, entry stride
    int64_t off;                 // entry offset inside the element's table row
    int64_t first;               // first global entry index of this projection
    int pay1;                    // unused by the kernels (k_emit's bank indices: EProj::pay1)
    // hardened encoding (core.h Mask): the row's tweak sub word and the pad slot of its first target (fan-out
    // rows F_LUT / F_FAN use slot hslot + d for target d); the gate is the gadget's PRG stream
    uint32_t hsub = 0;
    int hslot = 0;
};

struct Tables {
    u128* t[8];        // per table id: [N][row]
    int64_t row[8];    // entries per element
};

struct Ctx {
    const int16_t* R;    // [max_mod + 1][kW]
    const int16_t* Z;    // [max_mod + 1][kW]
    const ModC* mc;      // [max_mod + 1]
    uint32_t rk[44];     // PRG (seed) round keys
    const uint32_t* te0;
    // multiples of this GC's offsets, per modulus p (null until a projection of that modulus needs them):
    // iR[p] = [p][4 * chunks(n_p)] words, row i = the components i * R_p[q] mod p packed two per word
    const uint32_t* const* iR;
    int hard;  // hardened encoding: HC holds the compressed keys, k_emit / k_relu_finish derive tweaked pads
};

// Chunked component-major labels (all device labels of the GPU garbler): the
// components of an element are grouped in chunks of 8 (16 bytes); chunk c8 of
// element e of a label set of N elements sits at base + (c8 * N + e) * 8. A
// wave of lanes walking consecutive elements reads a chunk with one coalesced
// 16-byte load per lane (1 KiB contiguous per wave), and a lane gets 8
// components per load instruction. A single uniform label row (R_p, Z_p) is
// the same view with chunk stride 8 (components contiguous).
constexpr int kCh = 8;
__host__ __device__ constexpr int64_t chunks_of(int n) { return (n + kCh - 1) / kCh; }

// strided label view: component q at p[(q >> 3) * cs + (q & 7)], chunk c8 (16-B aligned) at p + c8 * cs
struct LRef {
    const int16_t* p;
    int64_t cs;
};
__host__ __device__ __forceinline__ LRef row_ref(const int16_t* row) { return LRef{row, kCh}; }

// input labels, per residue: element e's view is {p + e * es, cs}: chunked sets have es = 8,
// cs = 8 N; es = 0, cs = 8 broadcasts one label row to every element (the legacy rescale's Z_2 residue)
struct In {
    const int16_t* p[kMaxRes];
    int64_t es[kMaxRes], cs[kMaxRes];
    int n[kMaxRes];
};

// ------------------------------------------------------------------ device
// AES-bound garbling kernels use the conflict-free 32-copy LDS image (dev.h AesT)
constexpr int kGAes = 32;
using GAes = AesT<kGAes>;
constexpr int kGAesWords = aes_lds_words<kGAes>();

template <int C>
__device__ __forceinline__ u128 aes_keyed(const AesT<C>& a, u128 in, const uint32_t* rk) {
    uint32_t s0 = bswap32(static_cast<uint32_t>(in)) ^ rk[0];
    uint32_t s1 = bswap32(static_cast<uint32_t>(in >> 32)) ^ rk[1];
    uint32_t s2 = bswap32(static_cast<uint32_t>(in >> 64)) ^ rk[2];
    uint32_t s3 = bswap32(static_cast<uint32_t>(in >> 96)) ^ rk[3];
#pragma unroll
    for (int r = 1; r < 10; ++r) {
        const uint32_t t0 = aes_col(a, s0, s1, s2, s3, rk[4 * r + 0]);
        const uint32_t t1 = aes_col(a, s1, s2, s3, s0, rk[4 * r + 1]);
        const uint32_t t2 = aes_col(a, s2, s3, s0, s1, rk[4 * r + 2]);
        const uint32_t t3 = aes_col(a, s3, s0, s1, s2, rk[4 * r + 3]);
        s0 = t0;
        s1 = t1;
        s2 = t2;
        s3 = t3;
    }
    const uint32_t o0 = aes_last(a, s0, s1, s2, s3, rk[40]);
    const uint32_t o1 = aes_last(a, s1, s2, s3, s0, rk[41]);
    const uint32_t o2 = aes_last(a, s2, s3, s0, s1, rk[42]);
    const uint32_t o3 = aes_last(a, s3, s0, s1, s2, rk[43]);
    return (static_cast<u128>((static_cast<uint64_t>(bswap32(o3)) << 32) | bswap32(o2)) << 64) |
           ((static_cast<uint64_t>(bswap32(o1)) << 32) | bswap32(o0));
}

// two independent blocks under the PRG key, rounds interleaved (twice the LDS-read ILP of one lane)
template <int C>
__device__ __forceinline__ void aes_keyed2(const AesT<C>& a, u128 inA, u128 inB, const uint32_t* rk, u128& outA,
                                           u128& outB) {
    uint32_t a0 = bswap32(static_cast<uint32_t>(inA)) ^ rk[0], a1 = bswap32(static_cast<uint32_t>(inA >> 32)) ^ rk[1];
    uint32_t a2 = bswap32(static_cast<uint32_t>(inA >> 64)) ^ rk[2], a3 = bswap32(static_cast<uint32_t>(inA >> 96)) ^ rk[3];
    uint32_t b0 = bswap32(static_cast<uint32_t>(inB)) ^ rk[0], b1 = bswap32(static_cast<uint32_t>(inB >> 32)) ^ rk[1];
    uint32_t b2 = bswap32(static_cast<uint32_t>(inB >> 64)) ^ rk[2], b3 = bswap32(static_cast<uint32_t>(inB >> 96)) ^ rk[3];
#pragma unroll
    for (int r = 1; r < 10; ++r) {
        const uint32_t ta0 = aes_col(a, a0, a1, a2, a3, rk[4 * r + 0]);
        const uint32_t tb0 = aes_col(a, b0, b1, b2, b3, rk[4 * r + 0]);
        const uint32_t ta1 = aes_col(a, a1, a2, a3, a0, rk[4 * r + 1]);
        const uint32_t tb1 = aes_col(a, b1, b2, b3, b0, rk[4 * r + 1]);
        const uint32_t ta2 = aes_col(a, a2, a3, a0, a1, rk[4 * r + 2]);
        const uint32_t tb2 = aes_col(a, b2, b3, b0, b1, rk[4 * r + 2]);
        const uint32_t ta3 = aes_col(a, a3, a0, a1, a2, rk[4 * r + 3]);
        const uint32_t tb3 = aes_col(a, b3, b0, b1, b2, rk[4 * r + 3]);
        a0 = ta0; a1 = ta1; a2 = ta2; a3 = ta3;
        b0 = tb0; b1 = tb1; b2 = tb2; b3 = tb3;
    }
    auto fin = [&](uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3) -> u128 {
        const uint32_t o0 = aes_last(a, s0, s1, s2, s3, rk[40]);
        const uint32_t o1 = aes_last(a, s1, s2, s3, s0, rk[41]);
        const uint32_t o2 = aes_last(a, s2, s3, s0, s1, rk[42]);
        const uint32_t o3 = aes_last(a, s3, s0, s1, s2, rk[43]);
        return (static_cast<u128>((static_cast<uint64_t>(bswap32(o3)) << 32) | bswap32(o2)) << 64) |
               ((static_cast<uint64_t>(bswap32(o1)) << 32) | bswap32(o0));
    };
    outA = fin(a0, a1, a2, a3);
    outB = fin(b0, b1, b2, b3);
}

__device__ __forceinline__ uint64_t stream_of(uint64_t layer, uint64_t slot, uint64_t e, uint64_t mask) {
    return ((layer << 44) ^ (slot << 36) ^ e) ^ mask;
}

struct Gadget {
    const Draw* draws;
    int ndraws, nslots;
    const Proj* projs;
    int nprojs;
    int64_t entries;  // per element
    int nblk;         // AES-CTR blocks drawn per element (sum over draws)
    uint64_t layer, sslot, mask;  // PRG stream of this gadget: stream_of(layer, sslot, e, mask)
    int16_t* S;       // scratch: slot s is a chunked label set of kW components ([kW / 8][N][8]) at S + s * kW * N
    u128* PB;         // key-hash scratch of the binary (mod-2) mini gates: [2][N] (k_bin_keys)
    int64_t N;
    int mrs[kMaxMrs]; // MRS base of the sign gadget (per-digit output moduli of the fanned-out approx projections)
    u128* BK;             // [bank rows][N] payloads (k_bank -> k_emit)
    u128* HC;             // [entries][N] key hashes (k_hash -> k_emit), entry = first + color
    uint16_t* CC;         // [entries][N] the entry index i of that color
};

// slot s as a chunked label set, and element e's view of it
__host__ __device__ __forceinline__ int16_t* slot_base(const Gadget& g, int s) {
    return g.S + static_cast<int64_t>(s) * kW * g.N;
}
__device__ __forceinline__ LRef slot_ref(const Gadget& g, int s, int64_t e) {
    return LRef{slot_base(g, s) + e * kCh, g.N * kCh};
}

typedef uint32_t u32x4a __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4a ld_chunk(LRef a, int c8) { return *reinterpret_cast<const u32x4a*>(a.p + c8 * a.cs); }
__device__ __forceinline__ void st_chunk(int16_t* p, const u32x4a& v) { *reinterpret_cast<u32x4a*>(p) = v; }
__device__ __forceinline__ void unpack8(const u32x4a& v, uint32_t (&d)[8]) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        d[2 * u] = v[u] & 0xffffu;
        d[2 * u + 1] = v[u] >> 16;
    }
}
__device__ __forceinline__ u32x4a pack8(const uint32_t (&d)[8]) {
    u32x4a v;
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = d[2 * u] | (d[2 * u + 1] << 16);
    return v;
}
__device__ __forceinline__ void add8(uint32_t (&acc)[8], const u32x4a& v) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        acc[2 * u] += v[u] & 0xffffu;
        acc[2 * u + 1] += v[u] >> 16;
    }
}

// Stage a gadget's small descriptor array (draws / projections) in LDS so the
// per-thread binary search costs LDS, not dependent global round trips.
constexpr int kMaxDesc = 224;  // 224 x 80-B Proj (17.5 KiB) beside the AES image (dev.h)
constexpr int kGB = 512;        // threads per block of the AES-bound garbling kernels
template <class T>
__device__ __forceinline__ void lds_stage(T* dst, const T* src, int n) {
    const int words = n * static_cast<int>(sizeof(T) / 4);
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d = reinterpret_cast<uint32_t*>(dst);
    for (int i = threadIdx.x; i < words; i += blockDim.x) d[i] = s[i];
}

constexpr int kTile = 64;
#ifndef DASH_GG_PB
#define DASH_GG_PB 512
#endif
constexpr int kPB = DASH_GG_PB;  // threads per k_project block (A/B knob)

__device__ __forceinline__ int rfl(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint32_t rflu(uint32_t x) {
    return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(x)));
}
__device__ __forceinline__ int64_t rfl64(int64_t x) {
    const uint64_t u = static_cast<uint64_t>(x);
    const uint64_t lo = rflu(static_cast<uint32_t>(u)), hi = rflu(static_cast<uint32_t>(u >> 32));
    return static_cast<int64_t>(lo | (hi << 32));
}
__device__ __forceinline__ ModC rfl_modc(const ModC& m) {
    ModC r;
    r.q = rflu(m.q);
    r.n = rflu(m.n);
    r.c = rflu(m.c);
    r.D = rflu(m.D);
    r.mD = static_cast<uint64_t>(rfl64(static_cast<int64_t>(m.mD)));
    r.mq = rflu(m.mq);
    r.bits = rflu(m.bits);
    r.dm = rflu(m.dm);
    r.ds = rflu(m.ds);
    r.pm = rflu(m.pm);
    r.Dn = rflu(m.Dn);
    r.v = rflu(m.v);
    r.sh = rflu(m.sh);
    return r;
}
__device__ __forceinline__ Proj rfl_proj(const Proj& p) {
    Proj r;
    r.in_kind = rfl(p.in_kind);
    r.in_idx = rfl(p.in_idx);
    r.pin = rfl(p.pin);
    r.out_slot = rfl(p.out_slot);
    r.pout = rfl(p.pout);
    r.fn = rfl(p.fn);
    r.a0 = rfl(p.a0);
    r.a1 = rfl(p.a1);
    r.a2 = rfl(p.a2);
    r.outr_kind = rfl(p.outr_kind);
    r.outr_idx = rfl(p.outr_idx);
    r.table = rfl(p.table);
    r.stride = rfl(p.stride);
    r.off = rfl64(p.off);
    r.first = rfl64(p.first);
    r.pay1 = rfl(p.pay1);
    r.hsub = rflu(p.hsub);
    r.hslot = rfl(p.hslot);
    return r;
}

// One thread per (draw, element), draw-major: the 64 lanes of a wave are
// consecutive elements of one draw (uniform modulus, width and counter), each
// producing its whole label: AES-CTR blocks ctr, ctr+1, ... of its stream,
// ModC::pm consecutive components (Prg::label order) per block as the base-q
// digits of the block (DigitStream). Components are gathered 8 at a time in a
// 128-bit shift register and stored as 16-byte chunks: one coalesced KiB per
// wave per chunk, and chunk padding past n is written as zeros.
#ifndef DASH_GG_DRAW_PAIRS
#define DASH_GG_DRAW_PAIRS 1  // A/B knob: a label's AES-CTR blocks computed up front, two interleaved (0: one by one)
#endif
constexpr bool kDrawPairs = DASH_GG_DRAW_PAIRS != 0;
template <int C>
__global__ __launch_bounds__(kGB) void k_draw(Ctx c, Gadget g) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_aes[aes_lds_words<C>()];
    aes_lds_fill<C>(lds_aes, c.te0);
    const AesT<C> aes = aes_ctx<C>(lds_aes, nullptr);
    const int64_t N = g.N;
    const int64_t tiles = (N + kTile - 1) / kTile;
    const int64_t nw = tiles * g.ndraws;
    const int lane = static_cast<int>(threadIdx.x) & (kTile - 1);
    const int64_t wpb = kGB / kTile;
    const int64_t w0 = static_cast<int64_t>(blockIdx.x) * wpb + rfl(static_cast<int>(threadIdx.x) / kTile);
    const int64_t wstep = static_cast<int64_t>(gridDim.x) * wpb;
    const int64_t cs = N * kCh;
    for (int64_t w = w0; w < nw; w += wstep) {
        const int di = static_cast<int>(w / tiles);
        const int64_t tile = w - static_cast<int64_t>(di) * tiles;
        const int64_t e = tile * kTile + lane;
        const Draw d{rfl(g.draws[di].slot), rfl(g.draws[di].q), rfl(g.draws[di].ctr)};
        const ModC m = rfl_modc(c.mc[d.q]);
        const int n = static_cast<int>(m.n), pm = static_cast<int>(m.pm);
        if (e >= N) continue;
        const uint64_t stream = stream_of(g.layer, g.sslot, static_cast<uint64_t>(e), g.mask);
        int16_t* out = slot_base(g, d.slot) + e * kCh;
        DigitStream ds;
        u128 acc = 0;  // pending components, the oldest in the low 16 bits once 8 are in
        int blk = 0, left = 0;
        // the label's AES-CTR blocks up front (<= 3: q^pm <= 2^64 and q^n <= 2^128), two interleaved at a time
        const int nb = (n + pm - 1) / pm;
        const u128 base = static_cast<u128>(stream) << 64;
        u128 B[3];
        if (kDrawPairs && nb >= 2) {
            aes_keyed2(aes, base | static_cast<uint64_t>(d.ctr), base | static_cast<uint64_t>(d.ctr + 1), c.rk, B[0], B[1]);
            if (nb >= 3) B[2] = aes_keyed(aes, base | static_cast<uint64_t>(d.ctr + 2), c.rk);
        } else if (kDrawPairs) {
            B[0] = aes_keyed(aes, base | static_cast<uint64_t>(d.ctr), c.rk);
        }
        auto push = [&](int q, uint32_t dg) {
            acc = (acc >> 16) | (static_cast<u128>(dg) << 112);
            if ((q & 7) == 7) {
                u32x4a v;
                v[0] = static_cast<uint32_t>(acc);
                v[1] = static_cast<uint32_t>(acc >> 32);
                v[2] = static_cast<uint32_t>(acc >> 64);
                v[3] = static_cast<uint32_t>(acc >> 96);
                st_chunk(out + (q >> 3) * cs, v);
            }
        };
        if (m.bits) {
            for (int q = 0; q < n; ++q) {
                if (left == 0) {
                    if (kDrawPairs && nb <= 3) ds.init(blk == 0 ? B[0] : (blk == 1 ? B[1] : B[2]));
                    else ds.init(aes_keyed(aes, base | static_cast<uint64_t>(d.ctr + blk), c.rk));
                    ++blk;
                    left = pm;
                }
                push(q, ds.next(m));
                --left;
            }
        } else {
            // chunk-major (dev.h chunk_digit): per block, one divmod per chunk of m.c digits and a uniform digit
            // loop (the digits DigitStream::next yields)
            int q = 0;
            for (int bi = 0; bi < nb; ++bi) {
                u128 Q = (kDrawPairs && nb <= 3) ? (bi == 0 ? B[0] : (bi == 1 ? B[1] : B[2]))
                                                 : aes_keyed(aes, base | static_cast<uint64_t>(d.ctr + bi), c.rk);
                const int bcnt = min(pm, n - bi * pm);
                for (int k0 = 0; k0 < bcnt; k0 += static_cast<int>(m.c)) {
                    uint32_t r = divmod128(Q, m);
                    const int kc = min(static_cast<int>(m.c), bcnt - k0);
                    for (int t = 0; t < kc; ++t, ++q) push(q, chunk_digit(r, m));
                }
            }
        }
        if (n & 7) {  // last partial chunk: shift the pending components down, zeros above
            const u128 last = acc >> (16 * (8 - (n & 7)));
            u32x4a v;
            v[0] = static_cast<uint32_t>(last);
            v[1] = static_cast<uint32_t>(last >> 32);
            v[2] = static_cast<uint32_t>(last >> 64);
            v[3] = static_cast<uint32_t>(last >> 96);
            st_chunk(out + (n >> 3) * cs, v);
        }
    }
}

__device__ __forceinline__ LRef label_ref(const Ctx& c, const Gadget& g, const In& in, int64_t e, int kind, int idx,
                                          int q) {
    if (kind == S_INPUT) return LRef{in.p[idx] + e * in.es[idx], in.cs[idx]};
    if (kind == S_SLOT) return slot_ref(g, idx, e);
    return row_ref(c.Z + static_cast<int64_t>(q) * kW);
}

// sign derive: sum2[q] = sum_{j<=k} bases[q][j]; sum = carry_final + sum_j mrs[j][0]
struct SignSlots {
    int k, t;
    int mrs[kMaxMrs];
    int sum2_slot0, sum_slot, bases_slot0, newc_slot0, mrs_slot0, stride_q;  // stride_q = k + 2 (fused: 1)
    int fused;              // SignPlan::fused: digit sums read the approx outputs + the previous carry directly
    int dmod[kMaxMrs];      // fused: modulus of digit d's labels (SignPlan::digit_mod)
};

// dst = sum of `cnt` source slots (src0 + i * step) [+ one extra label ex] mod m; 8 components per step
__device__ __forceinline__ void slot_sum(const Gadget& g, int64_t e, int dst, int src0, int step, int cnt, LRef ex,
                                         bool has_ex, const ModC& m) {
    const int n = static_cast<int>(m.n);
    const LRef d = slot_ref(g, dst, e);
    for (int c8 = 0; c8 < chunks_of(n); ++c8) {
        uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (has_ex) add8(acc, ld_chunk(ex, c8));
        for (int i = 0; i < cnt; ++i) add8(acc, ld_chunk(slot_ref(g, src0 + i * step, e), c8));
#pragma unroll
        for (int u = 0; u < 8; ++u) acc[u] = modq(acc[u], m);
        st_chunk(const_cast<int16_t*>(d.p) + c8 * d.cs, pack8(acc));  // chunks past n stay inside the slot
    }
}

// grid (elements, t): y = q is one digit sum (the fused sums read the previous carry, which the carry
// projections of k_project produce later, so every q is independent here)
__global__ __launch_bounds__(256) void k_sign_derive(Ctx c, Gadget g, SignSlots s) {
    const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (e >= g.N) return;
    const int k = s.k, t = s.t;
    const LRef none{nullptr, 0};
    if (s.fused) {
        // digit q (d = t-1-q): sum_j approx[j][d] (+ carry of the previous digit, none for q = 0);
        // MSD: sum_j approx[j][0] + last carry (none when t = 1)
        {
            const int q = blockIdx.y;
            const int d = t - 1 - q;
            const ModC Mo = c.mc[s.dmod[d]];
            const int dst = d == 0 ? s.sum_slot : s.sum2_slot0 + q;
            slot_sum(g, e, dst, s.mrs_slot0 + d, t, k, q > 0 ? slot_ref(g, s.newc_slot0 + q - 1, e) : none, q > 0, Mo);
        }
        return;
    }
    const int q = blockIdx.y;
    if (q + 1 < t) {
        const int d = t - 1 - q;
        const ModC Mo = c.mc[(k + 1) * s.mrs[d]];
        slot_sum(g, e, s.sum2_slot0 + q, s.bases_slot0 + q * s.stride_q, 1, k + 1, none, false, Mo);
        return;
    }
    const int m0 = s.mrs[0];
    const ModC M0 = c.mc[m0];
    const LRef carry = t >= 2 ? slot_ref(g, s.newc_slot0 + (t - 2) * s.stride_q, e)
                              : row_ref(c.Z + static_cast<int64_t>(m0) * kW);
    slot_sum(g, e, s.sum_slot, s.mrs_slot0, t, k, carry, true, M0);
}

// Digits (a_q + f * b_q) mod m, q < m.n, of a per-lane label a and an offset label b, pushed into cf. Chunks
// are loaded kLd at a time (one memory round trip per 8 kLd components instead of one per 8). BU: b is a
// wave-uniform row (R_q), moved to SGPRs (readfirstlane), so it costs no vector registers. KEY: f is the key
// index i = (col - a_0) mod m, computed from the first loaded chunk (R[0] = 1: the key's color is col).
constexpr int kLd = 4;
template <bool BU, bool KEY>
__device__ __forceinline__ void push_lin(CompressFwd& cf, LRef a, LRef b, uint32_t& f, const ModC& m, uint32_t col = 0) {
    const int n = static_cast<int>(m.n);
    const int nc = static_cast<int>(chunks_of(n));
    for (int c0 = 0; c0 < nc; c0 += kLd) {
        u32x4a av[kLd], bv[kLd];
#pragma unroll
        for (int h = 0; h < kLd; ++h) {
            if (c0 + h < nc) {
                av[h] = ld_chunk(a, c0 + h);
                bv[h] = ld_chunk(b, c0 + h);
            }
        }
        if (KEY && c0 == 0) {
            const uint32_t x0 = av[0][0] & 0xffffu;
            f = col + m.q - x0;
            if (f >= m.q) f -= m.q;
        }
#pragma unroll
        for (int h = 0; h < kLd; ++h) {
            if (c0 + h >= nc) break;
            uint32_t bs[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) bs[u] = BU ? rflu(bv[h][u]) : bv[h][u];
            const int q0 = (c0 + h) * 8;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t x = (u & 1) ? (av[h][u >> 1] >> 16) : (av[h][u >> 1] & 0xffffu);
                const uint32_t y = (u & 1) ? (bs[u >> 1] >> 16) : (bs[u >> 1] & 0xffffu);
                if (q0 + u < n) cf.push(modq(x + f * y, m), m);
            }
        }
    }
}

// one thread per (element, table entry). Element-tiled order: the 64 lanes of
// a wavefront are 64 consecutive elements of one tile, all on the SAME table
// entry r, so the projection descriptor, i, the label widths (loop trip
// counts), the moduli and the function are wave-uniform. They are moved to
// SGPRs explicitly (readfirstlane): the digit loops then branch on scalar
// conditions instead of exec masks, and the compressor's running power of the
// modulus is scalar work issued beside the vector digits. Labels are chunked
// component-major: one coalesced 16-byte load per lane covers 8 components;
// consecutive waves walk the entries of the same 64 elements.
// Projections in two passes, so no lane carries a long dependent chain (key
// loads -> compress -> AES -> payload loads -> compress -> store):
//   k_hash  one lane per (element, color c of a projection): the entry i whose
//           key x + i*R has color c (R[0] = 1: i = c - x[0] mod p), its hash
//           H(compress(key)) and i -> HC / CC [first + c][N];
//   k_emit  one block per (table, 64-element tile, segment of kSeg table
//           positions): every lane computes the entry of one element at one
//           position (payload o + f(i)*R, inline or from the payload bank, + H)
//           into an LDS image of the tile's row segments, which is then written
//           out as 64 contiguous runs of kSeg x 16 bytes.
// Table rows are element-major ([N][row]) and permuted by color, so a wave of
// consecutive elements at one position writes 64 lines 16 bytes each; the LDS
// image turns that into full-line stores.
// Element-tiled order: the 64 lanes of a wavefront are 64 consecutive elements
// of one tile, all on the SAME work item, so the projection descriptor, the
// label widths (loop trip counts), the moduli and the function are
// wave-uniform and moved to SGPRs (readfirstlane); labels are chunked
// component-major, so one coalesced 16-byte load per lane covers 8 components.
__device__ __forceinline__ int find_proj(const Proj* sp, int n, int64_t r) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {  // last projection with first <= r (uniform search)
        const int mid = (lo + hi + 1) >> 1;
        if (rfl64(sp[mid].first) <= r) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

template <int C>
__global__ __launch_bounds__(kPB) void k_hash(Ctx c, Gadget g, In in) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_aes[aes_lds_words<C>()];
    aes_lds_fill<C>(lds_aes, c.te0);
    const AesT<C> aes = aes_ctx<C>(lds_aes, nullptr);
    const Proj* sp = g.projs;  // wave-uniform reads (scalar / broadcast loads)
    const int64_t N = g.N;
    const int64_t tiles = (N + kTile - 1) / kTile;
    const int64_t nw = tiles * g.entries;  // wave work items (tile, entry)
    const int lane = static_cast<int>(threadIdx.x) & (kTile - 1);
    const int64_t wpb = kPB / kTile;
    const int64_t w0 = static_cast<int64_t>(blockIdx.x) * wpb + rfl(static_cast<int>(threadIdx.x) / kTile);
    const int64_t wstep = static_cast<int64_t>(gridDim.x) * wpb;
    for (int64_t w = w0; w < nw; w += wstep) {
        const int64_t tile = w / g.entries;
        const int64_t r = w - tile * g.entries;
        const Proj P = rfl_proj(sp[find_proj(sp, g.nprojs, r)]);
        const uint32_t col = static_cast<uint32_t>(r - P.first);
        const ModC mi = rfl_modc(c.mc[P.pin]);
        // the last tile's spare lanes recompute element N-1 (uniform control flow) and skip the store
        const int64_t e_raw = tile * kTile + lane;
        const int64_t e = e_raw < N ? e_raw : N - 1;
        const LRef x = label_ref(c, g, in, e, P.in_kind, P.in_idx, P.pin);
        uint32_t i = 0;
        CompressFwd kc;
        kc.init();
        push_lin<true, true>(kc, x, row_ref(c.R + static_cast<int64_t>(P.pin) * kW), i, mi, col);
        const u128 H = c.hard ? kc.finish() : aes_encrypt(aes, kc.finish());
        if (e_raw < N) {
            g.HC[r * N + e] = H;
            g.CC[r * N + e] = static_cast<uint16_t>(i);
        }
    }
}

// Key hashes, one wave per (64-element tile, hash job), a job = up to kHJ consecutive colors of one
// projection: the input label comes from HBM once, the job's later colors re-read it from the CU's L1
// (a wave's label is <= 16 KiB), and the waves of a block are few jobs, not few entries. (Holding the label
// in registers instead spilled: 8 chunks x 16 B per lane plus the unrolled compress exceed 128 VGPRs.)
constexpr int kHJ = 8;  // colors per hash job
struct HashJob {
    int proj, c0;
};
template <int C>
__global__ __launch_bounds__(kPB, 4) void k_hash_jobs(Ctx c, Gadget g, In in, const HashJob* jobs, int njobs) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_aes[aes_lds_words<C>()];
    aes_lds_fill<C>(lds_aes, c.te0);
    const AesT<C> aes = aes_ctx<C>(lds_aes, nullptr);
    const int64_t N = g.N;
    const int64_t tiles = (N + kTile - 1) / kTile;
    const int64_t nw = tiles * njobs;
    const int lane = static_cast<int>(threadIdx.x) & (kTile - 1);
    const int64_t wpb = kPB / kTile;
    const int64_t w0 = static_cast<int64_t>(blockIdx.x) * wpb + rfl(static_cast<int>(threadIdx.x) / kTile);
    const int64_t wstep = static_cast<int64_t>(gridDim.x) * wpb;
    for (int64_t w = w0; w < nw; w += wstep) {
        const int64_t tile = w / njobs;
        const int jb = static_cast<int>(w - tile * njobs);
        const int pi = rfl(jobs[jb].proj), c0 = rfl(jobs[jb].c0);
        const Proj P = rfl_proj(g.projs[pi]);
        const ModC mi = rfl_modc(c.mc[P.pin]);
        const uint32_t p = static_cast<uint32_t>(P.pin);
        const int c1 = min(P.pin, c0 + kHJ);
        const int64_t e_raw = tile * kTile + lane;
        const int64_t e = e_raw < N ? e_raw : N - 1;
        const LRef x = label_ref(c, g, in, e, P.in_kind, P.in_idx, P.pin);
        const int16_t* R = c.R + static_cast<int64_t>(P.pin) * kW;
        for (int col = c0; col < c1; ++col) {
            uint32_t i = 0;
            CompressFwd kc;
            kc.init();
            push_lin<true, true>(kc, x, row_ref(R), i, mi, static_cast<uint32_t>(col));
            const u128 H = c.hard ? kc.finish() : aes_encrypt(aes, kc.finish());
            if (e_raw < N) {
                g.HC[(P.first + col) * N + e] = H;
                g.CC[(P.first + col) * N + e] = static_cast<uint16_t>(i);
            }
        }
    }
}

// ---- uniform-offset compression: compress(x + a) for a per-lane label x and a wave-uniform row a
#ifndef DASH_GG_ALIGNED_GROUPS
#define DASH_GG_ALIGNED_GROUPS 1  // A/B knob: chunk-aligned digit groups (compress_xa_g); 0 = runtime groups only
#endif
constexpr bool kAlignedGroups = DASH_GG_ALIGNED_GROUPS != 0;
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t w) { return __builtin_bit_cast(u16x2, w); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }

// C * d + v for d, v < 2^24 (four 32-bit limbs, carries by 64-bit adds)
__device__ __forceinline__ u128 mad128_24(u128 C, uint32_t d, uint32_t v) {
    const uint64_t lo = static_cast<uint64_t>(C), hi = static_cast<uint64_t>(C >> 64);
    const uint64_t l0 = static_cast<uint64_t>(static_cast<uint32_t>(lo)) * d + v;
    const uint64_t l1 = static_cast<uint64_t>(static_cast<uint32_t>(lo >> 32)) * d + (l0 >> 32);
    const uint64_t h0 = static_cast<uint64_t>(static_cast<uint32_t>(hi)) * d + (l1 >> 32);
    const uint64_t h1 = static_cast<uint64_t>(static_cast<uint32_t>(hi >> 32)) * d + (h0 >> 32);
    return (static_cast<u128>((h1 << 32) | static_cast<uint32_t>(h0)) << 64) |
           ((l1 << 32) | static_cast<uint32_t>(l0));
}

// Digits d_q = (x_q + a_q) mod q (q < n; padding components count as 0) of a per-lane chunked label x and a
// uniform row a (a_q < q, two components
// per word, chunk c8 at words 4 c8 .. 4 c8 + 3; same-address broadcast loads), compressed as sum_q d_q q^q by
// Horner's rule from the top chunk: two digits per packed 16-bit add / subtract / min, one 24-bit multiply-add
// (or shift-or for a power of two) per digit, a 128-bit merge per group of digits below 2^24 (the group
// bookkeeping is scalar). d0 = digit 0 (the color when a_0 = i and x's color is x_0).
template <bool PW2>
__device__ __forceinline__ u128 compress_xa_t(LRef x, const uint32_t* a, const ModC& m, uint32_t& d0) {
    const int nc = static_cast<int>(chunks_of(static_cast<int>(m.n)));
    const uint32_t q = m.q, b = m.bits;
    int g = 1;  // digits per group: q^g <= 2^24 (power of two: 24 / b bits)
    uint32_t D = q;
    if (PW2) {
        g = static_cast<int>(24 / b);
        D = 1u << (b * g);
    } else {
        while (static_cast<uint64_t>(D) * q <= (1u << 24)) {
            D *= q;
            ++g;
        }
    }
    const u16x2 qq = {static_cast<unsigned short>(q), static_cast<unsigned short>(q)};
    const u16x2 msk = {static_cast<unsigned short>(q - 1), static_cast<unsigned short>(q - 1)};
    u128 C = 0;
    uint32_t v = 0;
    int r = (8 * nc - 1) % g;  // digits after the current one in its group (groups are aligned at digit 0)
    uint32_t dlow = 0;
    // kLd chunks of x and of the row in flight per round trip, consumed from the most significant chunk
    for (int c0 = nc - 1; c0 >= 0; c0 -= kLd) {
        u32x4a xv[kLd], av[kLd];
#pragma unroll
        for (int h = 0; h < kLd; ++h) {
            if (c0 - h >= 0) {
                xv[h] = ld_chunk(x, c0 - h);
                av[h] = *reinterpret_cast<const u32x4a*>(a + 4 * (c0 - h));
            }
        }
#pragma unroll
        for (int h = 0; h < kLd; ++h) {
            if (c0 - h < 0) break;
            uint32_t t[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const u16x2 sm = as_u16x2(xv[h][u]) + as_u16x2(av[h][u]);
                t[u] = PW2 ? as_u32(sm & msk) : as_u32(__builtin_elementwise_min(sm, sm - qq));
            }
            const int qb = 8 * (c0 - h);  // first component of this chunk
#pragma unroll
            for (int k = 7; k >= 0; --k) {
                // chunk padding (components >= n) is not guaranteed zero in reused label blocks: digit 0
                const uint32_t d = qb + k >= static_cast<int>(m.n) ? 0u
                                   : ((k & 1) ? (t[k >> 1] >> 16) : (t[k >> 1] & 0xffffu));
                v = PW2 ? ((v << b) | d) : __umul24(v, q) + d;
                if (r == 0) {
                    C = mad128_24(C, D, v);
                    v = 0;
                    r = g - 1;
                } else {
                    --r;
                }
            }
            dlow = t[0] & 0xffffu;
        }
    }
    d0 = dlow;
    return C;
}
// Chunk-aligned digit groups: G | 8 digits with q^G <= 2^24 (G = 8 for q <= 8, 4 for q <= 64). The groups then
// start at the chunk boundaries, so after the digit loop is unrolled the flush points are compile-time positions,
// and only the top chunk can hold padding components (masked once, four ANDs). The digit loop carries no scalar
// bookkeeping: the runtime-group form above issued more SALU than VALU instructions in k_bank (1.26 G SALU vs
// 0.99 G VALU per 4 MiniONN GCs, profiles/r05_garble_pmc_hardened_4gc.txt), and the CU's one scalar unit serves
// all four SIMDs. Same integer as the runtime-group form (exact Horner, any grouping).
__device__ __forceinline__ void top_chunk_mask(uint32_t (&t)[4], int valid) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
        t[u] &= (2 * u < valid ? 0xffffu : 0u) | (2 * u + 1 < valid ? 0xffff0000u : 0u);
}
template <int G>
__device__ __forceinline__ u128 compress_xa_g(LRef x, const uint32_t* a, const ModC& m, uint32_t& d0) {
    const int nc = static_cast<int>(chunks_of(static_cast<int>(m.n)));
    const uint32_t q = m.q;
    uint32_t D = 1;
#pragma unroll
    for (int i = 0; i < G; ++i) D *= q;
    const u16x2 qq = {static_cast<unsigned short>(q), static_cast<unsigned short>(q)};
    u128 C = 0;
    uint32_t dlow = 0;
    for (int c0 = nc - 1; c0 >= 0; c0 -= kLd) {
        u32x4a xv[kLd], av[kLd];
#pragma unroll
        for (int h = 0; h < kLd; ++h) {
            if (c0 - h >= 0) {
                xv[h] = ld_chunk(x, c0 - h);
                av[h] = *reinterpret_cast<const u32x4a*>(a + 4 * (c0 - h));
            }
        }
#pragma unroll
        for (int h = 0; h < kLd; ++h) {
            if (c0 - h < 0) break;
            uint32_t t[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const u16x2 sm = as_u16x2(xv[h][u]) + as_u16x2(av[h][u]);
                t[u] = as_u32(__builtin_elementwise_min(sm, sm - qq));
            }
            const int valid = static_cast<int>(m.n) - 8 * (c0 - h);
            if (valid < 8) top_chunk_mask(t, valid);  // uniform: the top chunk only
            uint32_t v = 0;
#pragma unroll
            for (int k = 7; k >= 0; --k) {
                const uint32_t d = (k & 1) ? (t[k >> 1] >> 16) : (t[k >> 1] & 0xffffu);
                v = __umul24(v, q) + d;
                if (k % G == 0) {
                    C = mad128_24(C, D, v);
                    v = 0;
                }
            }
            dlow = t[0] & 0xffffu;
        }
    }
    d0 = dlow;
    return C;
}
__device__ __forceinline__ u128 compress_xa(LRef x, const uint32_t* a, const ModC& m, uint32_t& d0) {
    if (kAlignedGroups && m.q <= 8) return compress_xa_g<8>(x, a, m, d0);
    if (kAlignedGroups && m.q <= 64) return compress_xa_g<4>(x, a, m, d0);
    return m.bits ? compress_xa_t<true>(x, a, m, d0) : compress_xa_t<false>(x, a, m, d0);
}

// Two keys of one label x with two uniform rows a1, a2 (two entry indices): x is read once, and the two
// Horner chains (and the two AES blocks that follow) are independent work for the same lane.
template <bool PW2>
__device__ __forceinline__ void compress_xa2_t(LRef x, const uint32_t* a1, const uint32_t* a2, const ModC& m, u128& C1,
                                               u128& C2, uint32_t& d01, uint32_t& d02) {
    const int nc = static_cast<int>(chunks_of(static_cast<int>(m.n)));
    const uint32_t q = m.q, b = m.bits;
    int g = 1;
    uint32_t D = q;
    if (PW2) {
        g = static_cast<int>(24 / b);
        D = 1u << (b * g);
    } else {
        while (static_cast<uint64_t>(D) * q <= (1u << 24)) {
            D *= q;
            ++g;
        }
    }
    const u16x2 qq = {static_cast<unsigned short>(q), static_cast<unsigned short>(q)};
    const u16x2 msk = {static_cast<unsigned short>(q - 1), static_cast<unsigned short>(q - 1)};
    C1 = 0;
    C2 = 0;
    uint32_t v1 = 0, v2 = 0;
    int r = (8 * nc - 1) % g;
    uint32_t l1 = 0, l2 = 0;
    constexpr int kL2 = 2;  // chunks in flight per round trip (x plus two rows each)
    for (int c0 = nc - 1; c0 >= 0; c0 -= kL2) {
        u32x4a xv[kL2], av[kL2], bv[kL2];
#pragma unroll
        for (int h = 0; h < kL2; ++h) {
            if (c0 - h >= 0) {
                xv[h] = ld_chunk(x, c0 - h);
                av[h] = *reinterpret_cast<const u32x4a*>(a1 + 4 * (c0 - h));
                bv[h] = *reinterpret_cast<const u32x4a*>(a2 + 4 * (c0 - h));
            }
        }
#pragma unroll
        for (int h = 0; h < kL2; ++h) {
            if (c0 - h < 0) break;
            uint32_t t1[4], t2[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const u16x2 s1 = as_u16x2(xv[h][u]) + as_u16x2(av[h][u]);
                const u16x2 s2 = as_u16x2(xv[h][u]) + as_u16x2(bv[h][u]);
                t1[u] = PW2 ? as_u32(s1 & msk) : as_u32(__builtin_elementwise_min(s1, s1 - qq));
                t2[u] = PW2 ? as_u32(s2 & msk) : as_u32(__builtin_elementwise_min(s2, s2 - qq));
            }
            const int qb = 8 * (c0 - h);
#pragma unroll
            for (int k = 7; k >= 0; --k) {
                const bool pad = qb + k >= static_cast<int>(m.n);
                const uint32_t e1 = pad ? 0u : ((k & 1) ? (t1[k >> 1] >> 16) : (t1[k >> 1] & 0xffffu));
                const uint32_t e2 = pad ? 0u : ((k & 1) ? (t2[k >> 1] >> 16) : (t2[k >> 1] & 0xffffu));
                v1 = PW2 ? ((v1 << b) | e1) : __umul24(v1, q) + e1;
                v2 = PW2 ? ((v2 << b) | e2) : __umul24(v2, q) + e2;
                if (r == 0) {
                    C1 = mad128_24(C1, D, v1);
                    C2 = mad128_24(C2, D, v2);
                    v1 = v2 = 0;
                    r = g - 1;
                } else {
                    --r;
                }
            }
            l1 = t1[0] & 0xffffu;
            l2 = t2[0] & 0xffffu;
        }
    }
    d01 = l1;
    d02 = l2;
}
// compress_xa2_t with chunk-aligned groups (compress_xa_g)
template <int G>
__device__ __forceinline__ void compress_xa2_g(LRef x, const uint32_t* a1, const uint32_t* a2, const ModC& m, u128& C1,
                                               u128& C2, uint32_t& d01, uint32_t& d02) {
    const int nc = static_cast<int>(chunks_of(static_cast<int>(m.n)));
    const uint32_t q = m.q;
    uint32_t D = 1;
#pragma unroll
    for (int i = 0; i < G; ++i) D *= q;
    const u16x2 qq = {static_cast<unsigned short>(q), static_cast<unsigned short>(q)};
    C1 = 0;
    C2 = 0;
    uint32_t l1 = 0, l2 = 0;
    constexpr int kL2 = 2;
    for (int c0 = nc - 1; c0 >= 0; c0 -= kL2) {
        u32x4a xv[kL2], av[kL2], bv[kL2];
#pragma unroll
        for (int h = 0; h < kL2; ++h) {
            if (c0 - h >= 0) {
                xv[h] = ld_chunk(x, c0 - h);
                av[h] = *reinterpret_cast<const u32x4a*>(a1 + 4 * (c0 - h));
                bv[h] = *reinterpret_cast<const u32x4a*>(a2 + 4 * (c0 - h));
            }
        }
#pragma unroll
        for (int h = 0; h < kL2; ++h) {
            if (c0 - h < 0) break;
            uint32_t t1[4], t2[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const u16x2 s1 = as_u16x2(xv[h][u]) + as_u16x2(av[h][u]);
                const u16x2 s2 = as_u16x2(xv[h][u]) + as_u16x2(bv[h][u]);
                t1[u] = as_u32(__builtin_elementwise_min(s1, s1 - qq));
                t2[u] = as_u32(__builtin_elementwise_min(s2, s2 - qq));
            }
            const int valid = static_cast<int>(m.n) - 8 * (c0 - h);
            if (valid < 8) {
                top_chunk_mask(t1, valid);
                top_chunk_mask(t2, valid);
            }
            uint32_t v1 = 0, v2 = 0;
#pragma unroll
            for (int k = 7; k >= 0; --k) {
                const uint32_t e1 = (k & 1) ? (t1[k >> 1] >> 16) : (t1[k >> 1] & 0xffffu);
                const uint32_t e2 = (k & 1) ? (t2[k >> 1] >> 16) : (t2[k >> 1] & 0xffffu);
                v1 = __umul24(v1, q) + e1;
                v2 = __umul24(v2, q) + e2;
                if (k % G == 0) {
                    C1 = mad128_24(C1, D, v1);
                    C2 = mad128_24(C2, D, v2);
                    v1 = v2 = 0;
                }
            }
            l1 = t1[0] & 0xffffu;
            l2 = t2[0] & 0xffffu;
        }
    }
    d01 = l1;
    d02 = l2;
}
__device__ __forceinline__ void compress_xa2(LRef x, const uint32_t* a1, const uint32_t* a2, const ModC& m, u128& C1,
                                             u128& C2, uint32_t& d01, uint32_t& d02) {
    if (kAlignedGroups && m.q <= 8) compress_xa2_g<8>(x, a1, a2, m, C1, C2, d01, d02);
    else if (kAlignedGroups && m.q <= 64) compress_xa2_g<4>(x, a1, a2, m, C1, C2, d01, d02);
    else if (m.bits) compress_xa2_t<true>(x, a1, a2, m, C1, C2, d01, d02);
    else compress_xa2_t<false>(x, a1, a2, m, C1, C2, d01, d02);
}

#ifndef DASH_GG_HASH_PAIRS
#define DASH_GG_HASH_PAIRS 1  // A/B knob: two entry indices per k_hash_iu step (0: one)
#endif
constexpr bool kHashPairs = DASH_GG_HASH_PAIRS != 0;
// Key hashes with the entry index i uniform across the wave (one wave per (64-element tile, hash job), a job =
// up to kHJ consecutive i of one projection): key = x + i R_pin, i.e. digits x_q + (i R_q mod p) with the
// multiple row iR[pin][i] read from scalar memory; the key's color (digit 0, R_0 = 1) places the hash:
// HC / CC[first + color][e] = H, i.
// HARD (hardened encoding): the keys themselves, no AES, so no LDS image either (it capped the kernel at two
// 512-thread blocks per CU and cost a 64 KiB fill per block): k_hash_iu 2.15 -> 1.74 ms per 4 MiniONN GCs
template <int C, bool HARD>
__global__ __launch_bounds__(kPB, HARD ? 5 : 4) void k_hash_iu(Ctx c, Gadget g, In in, const HashJob* jobs, int njobs) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_aes[HARD ? 4 : aes_lds_words<C>()];
    if (!HARD) aes_lds_fill<C>(lds_aes, c.te0);
    const AesT<C> aes = aes_ctx<C>(lds_aes, nullptr);
    const int64_t N = g.N;
    const int64_t tiles = (N + kTile - 1) / kTile;
    const int64_t nw = tiles * njobs;
    const int lane = static_cast<int>(threadIdx.x) & (kTile - 1);
    const int64_t wpb = kPB / kTile;
    const int64_t w0 = static_cast<int64_t>(blockIdx.x) * wpb + rfl(static_cast<int>(threadIdx.x) / kTile);
    const int64_t wstep = static_cast<int64_t>(gridDim.x) * wpb;
    for (int64_t w = w0; w < nw; w += wstep) {
        const int64_t tile = w / njobs;
        const int jb = static_cast<int>(w - tile * njobs);
        const int pi = rfl(jobs[jb].proj), c0 = rfl(jobs[jb].c0);
        const Proj P = rfl_proj(g.projs[pi]);
        const ModC mi = rfl_modc(c.mc[P.pin]);
        const int c1 = min(P.pin, c0 + kHJ);
        const int64_t e_raw = tile * kTile + lane;
        const int64_t e = e_raw < N ? e_raw : N - 1;
        const LRef x = label_ref(c, g, in, e, P.in_kind, P.in_idx, P.pin);
        const int words = 4 * static_cast<int>(chunks_of(static_cast<int>(mi.n)));
        const uint32_t* rows = c.iR[P.pin];
        int i = c0;
        if (kHashPairs) {
            // two entry indices per step: one pass over x, two interleaved AES blocks (twice the LDS-read ILP)
            for (; i + 1 < c1; i += 2) {
                u128 k1, k2, H1, H2;
                uint32_t col1, col2;
                compress_xa2(x, rows + static_cast<int64_t>(i) * words, rows + static_cast<int64_t>(i + 1) * words, mi,
                             k1, k2, col1, col2);
                if (HARD) {  // hardened: the keys themselves (k_emit derives each entry's tweaked pad)
                    H1 = k1;
                    H2 = k2;
                } else {
                    aes_encrypt2(aes, k1, k2, H1, H2);
                }
                if (e_raw < N) {  // rows by entry index (coalesced); CC = color - i (k_emit inverts in LDS)
                    g.HC[(P.first + i) * N + e] = H1;
                    g.CC[(P.first + i) * N + e] = static_cast<uint16_t>(static_cast<int>(col1) - i);
                    g.HC[(P.first + i + 1) * N + e] = H2;
                    g.CC[(P.first + i + 1) * N + e] = static_cast<uint16_t>(static_cast<int>(col2) - (i + 1));
                }
            }
        }
        for (; i < c1; ++i) {
            uint32_t col;
            const u128 key = compress_xa(x, rows + static_cast<int64_t>(i) * words, mi, col);
            const u128 H = HARD ? key : aes_encrypt(aes, key);
            if (e_raw < N) {
                g.HC[(P.first + i) * N + e] = H;
                g.CC[(P.first + i) * N + e] = static_cast<uint16_t>(static_cast<int>(col) - i);
            }
        }
    }
}

// the multiple rows iR[p] of this GC's offsets (k_hash_iu, k_bank_iu): dst[i][w] = (i R_2w mod p) |
// (i R_2w+1 mod p) << 16 for the components of chunks(n_p) chunks (padding components are 0)
struct IrJob {
    uint32_t* dst;
    int p, words;
};
constexpr int kMaxIr = 32;
struct IrArgs {
    IrJob j[kMaxIr];
    int n;
};
__global__ __launch_bounds__(256) void k_iR(Ctx c, IrArgs a) {
    const IrJob J = a.j[blockIdx.y];
    const ModC m = c.mc[J.p];
    const int16_t* R = c.R + static_cast<int64_t>(J.p) * kW;
    const int64_t total = static_cast<int64_t>(J.p) * J.words;
    for (int64_t x = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; x < total;
         x += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const uint32_t i = static_cast<uint32_t>(x / J.words);
        const int wd = static_cast<int>(x - static_cast<int64_t>(i) * J.words);
        const uint32_t r0 = modq(i * static_cast<uint32_t>(R[2 * wd]), m);
        const uint32_t r1 = modq(i * static_cast<uint32_t>(R[2 * wd + 1]), m);
        J.dst[x] = r0 | (r1 << 16);
    }
}

// the 8 low bits (mod-2 components) of a chunk, component q at bit q
__device__ __forceinline__ uint32_t bits8(const u32x4a& v) {
    uint32_t b = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) b |= ((v[u] & 1u) | ((v[u] >> 15) & 2u)) << (2 * u);
    return b;
}

// LDS AES image copies of the AES-bound kernels (A/B knob DASH_GG_AES_COPIES = 16 | 32): 32 copies are
// bank-conflict free (64 KiB: 2 blocks per CU), 16 copies halve the image (2-way conflicts, more blocks)
inline int gg_aes_copies() {
    static const int v = [] {
        const char* e = std::getenv("DASH_GG_AES_COPIES");
        return e && std::atoi(e) == 16 ? 16 : 32;
    }();
    return v;
}
inline auto draw_kernel() { return gg_aes_copies() == 16 ? k_draw<16> : k_draw<32>; }
inline auto hash_kernel() { return gg_aes_copies() == 16 ? k_hash<16> : k_hash<32>; }
inline auto hash_jobs_kernel() { return gg_aes_copies() == 16 ? k_hash_jobs<16> : k_hash_jobs<32>; }
inline auto hash_iu_kernel(bool hard) {
    if (hard) return k_hash_iu<16, true>;
    return gg_aes_copies() == 16 ? k_hash_iu<16, false> : k_hash_iu<32, false>;
}
// DASH_GG_KEYS (A/B knob): 2 (default) = uniform-i key hashes and bank payloads from the offsets' multiple rows
// (compress_xa); 1 = multiple rows for the bank payloads only; 0 = the round-3 per-lane forms
// DASH_GG_FUSED (A/B knob): 1 = hardened k_emit computes its own keys and bank payloads (no HC / CC / BK round
// trip); 0 (default) = staged from k_hash_iu / k_bank. Measured and rejected (profiles/ab/README.md, round 6):
// byte-identical, but k_emit went 5.58 -> 9.22 ms per 4 MiniONN GCs while the k_hash_iu / k_bank time it removed
// was 2.76 ms (garbler kernels 18.5 -> 19.4 ms): the block's compress phase serialises with its pad and store
// phases, and a wave spans two key rows of possibly different moduli (te <= 32)
inline bool gg_emit_fused() {
    static const bool v = [] {
        const char* e = std::getenv("DASH_GG_FUSED");
        return e && std::atoi(e) == 1;
    }();
    return v;
}
inline int gg_hash_mode() {
    static const int v = [] {
        const char* e = std::getenv("DASH_GG_KEYS");
        return e ? std::atoi(e) : 2;
    }();
    return v;
}
// DASH_GG_HASH=entry: one wave per (tile, entry) (k_hash); default: per (tile, hash job) (k_hash_jobs).
// Rejected (profiles/ab/README.md): a block per (tile, projection) with the label staged in LDS (9.8 -> 17.6 ms
// per 4 GCs: most projections have 3-17 colors, most of the block's waves idled at its barriers), and a wave per
// (tile, projection) stepping packed-byte keys x + i*R incrementally (22.1 ms: fewer, longer serial work items
// and the unrolled compress's uniform constants spilled 146 SGPRs).
inline bool gg_hash_jobs() {
    static const bool v = [] {
        const char* e = std::getenv("DASH_GG_HASH");
        return !(e && std::string(e) == "entry");
    }();
    return v;
}

// ---- k_emit: table rows assembled per tile of elements in LDS
// A table entry is T[color] = payload + H, payload = o + v * R (mod pout) with
// v = f(i, d) taking few distinct values per (projection, target d), so every
// distinct payload of an element is computed once into a bank row, and an
// entry is two LDS lookups and an add. A k_emit block owns a scope (a
// contiguous range of table positions covering whole projections) for te
// consecutive elements:
//   1a  stage the scope's key hashes and entry indices (HC / CC rows, coalesced)
//   1b  compute the scope's bank payloads (lanes: consecutive elements of a bank row)
//   2   one lane per (element, position): bank row of (i, d) + H -> the table,
//       te contiguous runs of span x 16 bytes (full-line stores)
constexpr uint32_t kHole = 0xffffffffu;  // position map: no projection writes here
constexpr int kEB = 256;                 // k_emit threads
struct BankRow {
    int slot, pout, v, res;  // payload = slot label + v * (res < 0 ? R_pout : input label of residue res) mod pout
};
struct EProj {
    uint32_t hsub;  // hardened tweak (Proj::hsub / hslot)
    int hslot;
    int first;  // first key-hash entry (HC / CC row)
    int pay1;   // element-independent f: bix base (bank row of (i, d) at bix[pay1 + i * t + d]);
                // F_MULR / F_NEGR: scope-relative bank row of v = 0 (rows v = 0 .. pout - 1)
    int16_t fn, t, res;
    uint16_t pout;
    int in_idx;  // the projection's input label (fused key hashes: Emit::fused)
    int16_t in_kind;
    uint16_t pin;
};
static_assert(sizeof(EProj) == 32, "EProj: 32 B (224 of them are staged in k_emit's LDS)");
struct Scope {
    int table, tsh;  // table id; te = 1 << tsh elements per block
    int a, span;     // table positions [a, a + span)
    int r0, ne;      // key-hash entries [r0, r0 + ne)
    int b0, nb;      // bank rows [b0, b0 + nb)
    int bx0, nbx;    // bank indices [bx0, bx0 + nbx) of its element-independent projections
    int q0, nq;      // hardened: pad quads [q0, q0 + nq) covering the span (Emit::quads)
    int64_t blk0;    // first block of the scope
};
struct Emit {
    int by_i;  // key hashes stored by entry index i with CC = color - i (k_hash_iu); else by color with CC = i
    // fused (hardened, every bank row an R-offset row): the block computes its tile's keys and bank payloads
    // itself (compress_xa over the offsets' multiple rows) instead of loading k_hash_iu's / k_bank's output
    int fused;
    const Scope* sc;
    int nsc, nep;
    int64_t blocks;
    const uint32_t* map;  // table t's positions at map + map_off[t]: projection << 24 | color << 12 | target
    int64_t map_off[8];
    const uint16_t* bix;
    const BankRow* rows;
    const EProj* ep;
    // hardened: runs of <= 4 consecutive positions of one key whose pads come from ONE ChaCha block (same
    // projection and color, consecutive fan-out targets, same block of 4 slots), (position - scope a) << 3 | count
    const uint32_t* quads;
};

// Bank payloads: one wave per (64-element tile, bank row), lanes = consecutive elements (the row's slot,
// modulus and offset kind are wave-uniform): BK[row][N] = slot label + v * offset (mod pout), compressed.
__device__ __forceinline__ u128 bank_payload(const Ctx& c, const Gadget& g, const In& in, const BankRow* rows, int row,
                                             int64_t e) {
    const int slot = rfl(rows[row].slot), pout = rfl(rows[row].pout), res = rfl(rows[row].res);
    uint32_t f = rflu(static_cast<uint32_t>(rows[row].v));
    const ModC mo = rfl_modc(c.mc[pout]);
    if (res < 0 && c.iR != nullptr && c.iR[pout] != nullptr) {
        // uniform offset v R_pout: its multiple row (compress_xa)
        const int words = 4 * static_cast<int>(chunks_of(static_cast<int>(mo.n)));
        uint32_t d0;
        return compress_xa(slot_ref(g, slot, e), c.iR[pout] + static_cast<int64_t>(f) * words, mo, d0);
    }
    CompressFwd pc;
    pc.init();
    if (res < 0) push_lin<true, false>(pc, slot_ref(g, slot, e), row_ref(c.R + static_cast<int64_t>(pout) * kW), f, mo);
    else push_lin<false, false>(pc, slot_ref(g, slot, e), LRef{in.p[res] + e * in.es[res], in.cs[res]}, f, mo);
    return pc.finish();
}

// Bank payloads: one wave per (64-element tile, bank job), lanes = consecutive elements (the rows' slot,
// modulus and offset kind are wave-uniform): BK[row][N] = slot label + v * offset (mod pout), compressed. A job
// is one row or two rows of the same slot label and R offset (two values v): the label is read once for both.
struct BankJob {
    int r0, r1;  // r1 < 0: a single row
};
__global__ __launch_bounds__(256) void k_bank(Ctx c, Gadget g, In in, const BankRow* rows, const BankJob* jobs,
                                              int njobs) {
    const int64_t N = g.N;
    const int64_t tiles = (N + kTile - 1) / kTile;
    const int64_t nw = tiles * njobs;
    const int lane = static_cast<int>(threadIdx.x) & (kTile - 1);
    const int64_t wpb = 256 / kTile;
    const int64_t w0 = static_cast<int64_t>(blockIdx.x) * wpb + rfl(static_cast<int>(threadIdx.x) / kTile);
    const int64_t wstep = static_cast<int64_t>(gridDim.x) * wpb;
    for (int64_t w = w0; w < nw; w += wstep) {
        // tile-major: the rows of one slot label (a target's values) run in neighbouring waves, so the label's
        // re-reads hit L2 (row-major order re-fetched it from HBM for every value)
        const int64_t tile = w / njobs;
        const int jb = static_cast<int>(w - tile * njobs);
        const int r0 = rfl(jobs[jb].r0), r1 = rfl(jobs[jb].r1);
        const int64_t e_raw = tile * kTile + lane;
        const int64_t e = e_raw < N ? e_raw : N - 1;
        if (r1 >= 0) {  // (host-checked: same slot, same modulus, R offsets, multiple rows present)
            const int slot = rfl(rows[r0].slot), pout = rfl(rows[r0].pout);
            const uint32_t f0 = rflu(static_cast<uint32_t>(rows[r0].v)), f1 = rflu(static_cast<uint32_t>(rows[r1].v));
            const ModC mo = rfl_modc(c.mc[pout]);
            const int words = 4 * static_cast<int>(chunks_of(static_cast<int>(mo.n)));
            const uint32_t* rp = c.iR[pout];
            u128 P0, P1;
            uint32_t d0, d1;
            compress_xa2(slot_ref(g, slot, e), rp + static_cast<int64_t>(f0) * words, rp + static_cast<int64_t>(f1) * words,
                         mo, P0, P1, d0, d1);
            if (e_raw < N) {
                g.BK[static_cast<int64_t>(r0) * N + e] = P0;
                g.BK[static_cast<int64_t>(r1) * N + e] = P1;
            }
        } else {
            const u128 P = bank_payload(c, g, in, rows, r0, e);
            if (e_raw < N) g.BK[static_cast<int64_t>(r0) * N + e] = P;
        }
    }
}

__global__ __launch_bounds__(kEB) void k_emit(Ctx c, Gadget g, In in, Tables tb, Emit em) {
    extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
    __shared__ EProj sep[kMaxDesc];
    lds_stage(sep, em.ep, em.nep);
    __syncthreads();
    const int64_t N = g.N;
    for (int64_t b = blockIdx.x; b < em.blocks; b += gridDim.x) {
        int lo = 0, hi = em.nsc - 1;
        while (lo < hi) {  // last scope with blk0 <= b (uniform)
            const int mid = (lo + hi + 1) >> 1;
            if (rfl64(em.sc[mid].blk0) <= b) lo = mid;
            else hi = mid - 1;
        }
        const Scope S = em.sc[lo];
        const int tsh = rfl(S.tsh), te = 1 << tsh;
        const int64_t e0 = (b - rfl64(S.blk0)) << tsh;
        const int ne = rfl(S.ne), nb = rfl(S.nb), r0 = rfl(S.r0), span = rfl(S.span), a = rfl(S.a);
        // LDS rows of te + 1 entries: rows of different hashes / payloads start 4 banks apart, so the lanes of
        // a ds_read_b128 group (consecutive positions: different rows, one element) hit distinct banks
        const int te1 = te + 1;
        const int bx0 = rfl(S.bx0), nbx = rfl(S.nbx);
        u128* HCL = reinterpret_cast<u128*>(dyn);
        u128* PBL = HCL + ne * te1;
        uint16_t* CCL = reinterpret_cast<uint16_t*>(PBL + nb * te1);
        // by_i: IDX[color row][el] = the row of the entry index with that color (the inverse of CCL's deltas)
        uint16_t* IDX = CCL + ((ne * te1 + 1) & ~1);
        uint32_t* MAP = reinterpret_cast<uint32_t*>(IDX + (em.by_i ? ((ne * te1 + 1) & ~1) : 0));
        uint16_t* BIX = reinterpret_cast<uint16_t*>(MAP + span);
        const int table = rfl(S.table);
        // 1: the tile's key hashes, entry indices and bank payloads (coalesced rows of te elements, kUn loads in
        // flight per thread), the scope's position map and bank indices
        constexpr int kUn = 4;
        const int b0 = rfl(S.b0);
        const int nh = ne << tsh, nall = (ne + nb) << tsh;
        if (em.fused) {
            // 1 (fused): item (row, element). A key row r0 + rr is entry index i of the projection holding it: its key
            // x + i R_pin lands at the row of its color (CCL = i, as k_hash does); a bank row is slot label + v R_pout.
            // The lanes of a wave are consecutive elements of one or two rows (uniform moduli in the common case).
            for (int x = threadIdx.x; x < nall; x += kEB) {
                const int rr = x >> tsh, el = x & (te - 1);
                const int64_t e = min(e0 + el, N - 1);
                if (x < nh) {
                    const int r = r0 + rr;
                    int lo = 0, hi = em.nep - 1;
                    while (lo < hi) {  // the projection holding key row r (projections are in `first` order)
                        const int mid = (lo + hi + 1) >> 1;
                        if (sep[mid].first <= r) lo = mid;
                        else hi = mid - 1;
                    }
                    const EProj& P = sep[lo];
                    const int i = r - P.first;
                    const ModC mi = c.mc[P.pin];
                    const int words = 4 * static_cast<int>(chunks_of(static_cast<int>(mi.n)));
                    uint32_t col;
                    const u128 key = compress_xa(label_ref(c, g, in, e, P.in_kind, P.in_idx, P.pin),
                                                 c.iR[P.pin] + static_cast<int64_t>(i) * words, mi, col);
                    const int rc = P.first - r0 + static_cast<int>(col);
                    HCL[rc * te1 + el] = key;
                    CCL[rc * te1 + el] = static_cast<uint16_t>(i);
                } else {
                    const BankRow B = em.rows[b0 + rr - ne];
                    const ModC mo = c.mc[B.pout];
                    const int words = 4 * static_cast<int>(chunks_of(static_cast<int>(mo.n)));
                    uint32_t d0;
                    PBL[(rr - ne) * te1 + el] =
                        compress_xa(slot_ref(g, B.slot, e), c.iR[B.pout] + static_cast<int64_t>(B.v) * words, mo, d0);
                }
            }
        }
        for (int x0 = threadIdx.x; !em.fused && x0 < nall; x0 += kUn * kEB) {
            u128 hv[kUn];
            uint16_t cv[kUn];
#pragma unroll
            for (int u = 0; u < kUn; ++u) {
                const int x = x0 + u * kEB;
                if (x >= nall) continue;
                const int rr = x >> tsh;
                const int64_t e = min(e0 + (x & (te - 1)), N - 1);
                if (x < nh) {
                    hv[u] = g.HC[(r0 + rr) * N + e];
                    cv[u] = g.CC[(r0 + rr) * N + e];
                } else {
                    hv[u] = g.BK[(b0 + rr - ne) * N + e];
                }
            }
#pragma unroll
            for (int u = 0; u < kUn; ++u) {
                const int x = x0 + u * kEB;
                if (x >= nall) continue;
                const int rr = x >> tsh, el = x & (te - 1);
                if (x < nh) {
                    HCL[rr * te1 + el] = hv[u];
                    CCL[rr * te1 + el] = cv[u];
                } else {
                    PBL[(rr - ne) * te1 + el] = hv[u];
                }
            }
        }
        const uint32_t* gmap = em.map + em.map_off[table] + a;
        for (int x = threadIdx.x; x < span; x += kEB) MAP[x] = gmap[x];
        for (int x = threadIdx.x; x < nbx; x += kEB) BIX[x] = em.bix[bx0 + x];
        // hardened: the scope's pad runs too, so a quad's descriptor chain (run -> position map -> projection ->
        // entry row -> key) is LDS reads only
        uint32_t* QDL = reinterpret_cast<uint32_t*>(BIX + ((nbx + 1) & ~1));
        if (c.hard) {
            const uint32_t* QD = em.quads + rfl(S.q0);
            const int nq = rfl(S.nq);
            for (int x = threadIdx.x; x < nq; x += kEB) QDL[x] = QD[x];
        }
        __syncthreads();
        if (em.by_i) {
            // the colors of a projection's keys are a permutation of its entry indices: invert in LDS,
            // IDX[row of color c][el] = row of the entry index whose key has color c (delta = c - i)
            for (int x = threadIdx.x; x < nh; x += kEB) {
                const int rr = x >> tsh, el = x & (te - 1);
                const int delta = static_cast<int16_t>(CCL[rr * te1 + el]);
                IDX[(rr + delta) * te1 + el] = static_cast<uint16_t>(rr);
            }
            __syncthreads();
        }
        u128* T = tb.t[table];
        const int64_t row = tb.row[table];
        if (c.hard) {
            // 2 (hardened): one ChaCha block per quad (up to 4 entries of one key: a fan-out row's consecutive
            // targets share a block), quad-fastest over the tile's elements. (Rejected, profiles/ab/README.md:
            // loading the next quad's descriptor chain before this quad's pad block, and a prefetch of the next
            // tile's staging loads: k_emit unchanged.)
            const int nq = rfl(S.nq);
            const int totq = nq * te;
            const float inv_nq = 1.0f / static_cast<float>(nq);
            for (int x = threadIdx.x; x < totq; x += kEB) {
                int el = static_cast<int>(static_cast<float>(x) * inv_nq);
                if (el * nq > x) --el;
                else if ((el + 1) * nq <= x) ++el;
                const int q = x - el * nq;
                const int64_t e = e0 + el;
                if (e >= N) continue;
                const uint32_t qd = QDL[q];
                const int p0 = static_cast<int>(qd >> 3), cnt = static_cast<int>(qd & 7u);
                const uint32_t m0 = MAP[p0];
                const EProj P = sep[m0 >> 24];
                int rr = P.first + static_cast<int>((m0 >> 12) & 0xfffu) - r0;  // the color's row
                int i;
                if (em.by_i) {
                    rr = IDX[rr * te1 + el];
                    i = rr - (P.first - r0);
                } else {
                    i = CCL[rr * te1 + el];
                }
                const int d0 = static_cast<int>(m0 & 0xfffu);
                const bool fan = P.fn == F_LUT || P.fn == F_FAN;
                const int s0 = P.hslot + (fan ? d0 : 0);
                u128 pad[4];
                hard_block(HCL[rr * te1 + el], stream_of(g.layer, g.sslot, static_cast<uint64_t>(e), g.mask), P.hsub,
                           static_cast<uint32_t>(s0) >> 2, pad);
                u128* dst = T + e * row + a + p0;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (u >= cnt) break;
                    int br;
                    if (P.fn == F_MULR || P.fn == F_NEGR) {  // never fan-out: cnt == 1
                        const int xr = in.p[P.res][e * in.es[P.res]];
                        int w = P.fn == F_MULR ? (i * xr) % P.pout : -(i + xr) % P.pout;
                        if (w < 0) w += P.pout;
                        br = P.pay1 + w;
                    } else {
                        br = BIX[P.pay1 - bx0 + i * P.t + d0 + u];
                    }
                    const int qq = (s0 + u) & 3;
                    const u128 h = qq == 0 ? pad[0] : (qq == 1 ? pad[1] : (qq == 2 ? pad[2] : pad[3]));
                    const u128 v = PBL[br * te1 + el] + h;
                    u32x4a w;
                    w[0] = static_cast<uint32_t>(v);
                    w[1] = static_cast<uint32_t>(v >> 32);
                    w[2] = static_cast<uint32_t>(v >> 64);
                    w[3] = static_cast<uint32_t>(v >> 96);
                    *reinterpret_cast<u32x4a*>(dst + u) = w;
                }
            }
            __syncthreads();
            continue;
        }
        // 2: entries, position-fastest (contiguous per element), kUn independent LDS-only chains per thread
        const int total = span * te;
        const float inv_span = 1.0f / static_cast<float>(span);
        for (int x0 = threadIdx.x; x0 < total; x0 += kUn * kEB) {
            uint32_t mm[kUn];
            int el[kUn], pp[kUn];
#pragma unroll
            for (int u = 0; u < kUn; ++u) {
                const int x = x0 + u * kEB;
                int q = static_cast<int>(static_cast<float>(x) * inv_span);
                if (q * span > x) --q;
                else if ((q + 1) * span <= x) ++q;
                el[u] = q;
                pp[u] = x - q * span;
                mm[u] = (x < total && e0 + q < N) ? MAP[pp[u]] : kHole;
            }
            u128 v[kUn];
#pragma unroll
            for (int u = 0; u < kUn; ++u) {
                if (mm[u] == kHole) continue;
                const EProj P = sep[mm[u] >> 24];
                int rr = P.first + static_cast<int>((mm[u] >> 12) & 0xfffu) - r0;  // the color's row
                int i;
                if (em.by_i) {
                    rr = IDX[rr * te1 + el[u]];  // the entry index's row
                    i = rr - (P.first - r0);
                } else {
                    i = CCL[rr * te1 + el[u]];
                }
                int br;
                if (P.fn == F_MULR || P.fn == F_NEGR) {
                    const int64_t e = e0 + el[u];
                    const int xr = in.p[P.res][e * in.es[P.res]];
                    int w = P.fn == F_MULR ? (i * xr) % P.pout : -(i + xr) % P.pout;
                    if (w < 0) w += P.pout;
                    br = P.pay1 + w;
                } else {
                    br = BIX[P.pay1 - bx0 + i * P.t + static_cast<int>(mm[u] & 0xfffu)];
                }
                v[u] = PBL[br * te1 + el[u]] + HCL[rr * te1 + el[u]];
            }
#pragma unroll
            for (int u = 0; u < kUn; ++u) {
                if (mm[u] == kHole) continue;
                u32x4a w;
                w[0] = static_cast<uint32_t>(v[u]);
                w[1] = static_cast<uint32_t>(v[u] >> 32);
                w[2] = static_cast<uint32_t>(v[u] >> 64);
                w[3] = static_cast<uint32_t>(v[u] >> 96);
                *reinterpret_cast<u32x4a*>(T + (e0 + el[u]) * row + a + pp[u]) = w;
            }
        }
        __syncthreads();
    }
}

// Mixed-radix rescale (gadgets.h RescaleMrsPlan), garbler side of the free
// operations, one thread per element, 8 components per load: key base labels
// K_i = L_i - sum_{l<i} P_{l,i}, the mod-T accumulator r = sum_i P_{i,T}, then
// the output base labels (in place) Y_0 = F_0, Y_j = S^-1 L_j + F_j.
constexpr int kMaxY = 160;  // (residue, chunk) work items: sum of chunks_of(n_j) over residues + accumulator
struct MrsG {
    int k, T;
    int crt[kMaxRes], sinv[kMaxRes];
    int nsub[kMaxRes];
    int sub[kMaxRes][kMaxRes];  // digit-target slots subtracted from residue j's key
    int tslot[kMaxRes];         // slot of digit i's T target
    int key0, acc, fin0;
    int16_t* L[kMaxRes];  // chunked [n_j / 8][N][8], updated in place
    int yj[kMaxY], yc[kMaxY];  // k_mrs_derive grid y -> (residue j (k: accumulator), chunk)
};

// grid (elements, work items y): item y = (residue j, chunk c8), j = k the accumulator; one chunk per thread,
// so all of a thread's loads are one memory round trip (a chunk loop paid one per chunk)
__global__ __launch_bounds__(256) void k_mrs_derive(Ctx c, Gadget g, MrsG a) {
    const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (e >= g.N) return;
    const int64_t cs = g.N * kCh;
    const int k = a.k;
    const int j = a.yj[blockIdx.y], c8 = a.yc[blockIdx.y];
    if (j < k) {
        const int p = a.crt[j];
        const ModC m = c.mc[p];
        const int ns = a.nsub[j];
        int16_t* Lj = a.L[j] + e * kCh;
        const LRef K = slot_ref(g, a.key0 + j, e), F = slot_ref(g, a.fin0 + j, e);
        const u32x4a xv = *reinterpret_cast<const u32x4a*>(Lj + c8 * cs);
        const u32x4a fvv = ld_chunk(F, c8);
        uint32_t x[8];
        unpack8(xv, x);
        // key: L_j - sum of the digit payload labels aimed at residue j (loads batched kLd at a time)
        uint32_t kv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) kv[u] = x[u] + static_cast<uint32_t>(p) * static_cast<uint32_t>(ns);
        for (int l0 = 0; l0 < ns; l0 += kLd) {
            u32x4a sv[kLd];
#pragma unroll
            for (int h = 0; h < kLd; ++h)
                if (l0 + h < ns) sv[h] = ld_chunk(slot_ref(g, a.sub[j][l0 + h], e), c8);
#pragma unroll
            for (int h = 0; h < kLd; ++h) {
                if (l0 + h >= ns) break;
                uint32_t t[8];
                unpack8(sv[h], t);
#pragma unroll
                for (int u = 0; u < 8; ++u) kv[u] -= t[u];
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) kv[u] = modq(kv[u], m);
        st_chunk(const_cast<int16_t*>(K.p) + c8 * K.cs, pack8(kv));
        // output base label (in place): Y_0 = F_0, Y_j = S^-1 L_j + F_j (chunk padding stays in the block)
        uint32_t fv[8], yv[8];
        unpack8(fvv, fv);
#pragma unroll
        for (int u = 0; u < 8; ++u) yv[u] = j == 0 ? fv[u] : modq(x[u] * static_cast<uint32_t>(a.sinv[j]) + fv[u], m);
        st_chunk(Lj + c8 * cs, pack8(yv));
        return;
    }
    const LRef A = slot_ref(g, a.acc, e);
    uint32_t av[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int l0 = 0; l0 < k; l0 += kLd) {
        u32x4a tv[kLd];
#pragma unroll
        for (int h = 0; h < kLd; ++h)
            if (l0 + h < k) tv[h] = ld_chunk(slot_ref(g, a.tslot[l0 + h], e), c8);
#pragma unroll
        for (int h = 0; h < kLd; ++h)
            if (l0 + h < k) add8(av, tv[h]);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) av[u] &= static_cast<uint32_t>(a.T - 1);
    st_chunk(const_cast<int16_t*>(A.p) + c8 * A.cs, pack8(av));
}

// Mixed-radix sign (gadgets.h SignMrsPlan): key base labels
// K_r = x_r - sum of the digit-target labels aimed at residue r (slot lists).
struct MrsSG {
    int k;
    int crt[kMaxRes];
    int nsub[kMaxRes];
    int sub[kMaxRes][kMaxRes];  // slots subtracted from residue r's key
    int key0;                   // key slot of residue r = key0 + r
};
// grid (elements, residue r)
__global__ __launch_bounds__(256) void k_mrs_sign_derive(Ctx c, Gadget g, In in, MrsSG a) {
    const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (e >= g.N) return;
    {
        const int r = blockIdx.y;
        const int p = a.crt[r];
        const ModC m = c.mc[p];
        const int nc = static_cast<int>(chunks_of(in.n[r])), ns = a.nsub[r];
        const LRef x{in.p[r] + e * in.es[r], in.cs[r]};
        const LRef K = slot_ref(g, a.key0 + r, e);
        for (int c8 = 0; c8 < nc; ++c8) {
            uint32_t kv[8];
            unpack8(ld_chunk(x, c8), kv);
#pragma unroll
            for (int u = 0; u < 8; ++u) kv[u] += static_cast<uint32_t>(p) * static_cast<uint32_t>(ns);
            for (int l = 0; l < ns; ++l) {
                uint32_t sv[8];
                unpack8(ld_chunk(slot_ref(g, a.sub[r][l], e), c8), sv);
#pragma unroll
                for (int u = 0; u < 8; ++u) kv[u] -= sv[u];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) kv[u] = modq(kv[u], m);
            st_chunk(const_cast<int16_t*>(K.p) + c8 * K.cs, pack8(kv));
        }
    }
}

// ReLU mixed-mod half gates beyond the g/e projections: mini gate payloads
// (16-bit, e[q]) and the output base labels out0[j] = sk04 - sk03.
// Grid (elements, residue j): per thread the two mini entries of (e, j) and
// the chunks of out0[j].
struct MiniArgs {
    int k;
    int crt[kMaxRes];
    int sig_slot, sk_slot0;  // sk03_j = sk_slot0 + 2j, sk04_j = +1
    int16_t* out[kMaxRes];   // next base labels, chunked
};

__global__ __launch_bounds__(256) void k_relu_finish(Ctx c, Gadget g, In in, Tables tb, MiniArgs m, const u128* hk) {
    const int j = blockIdx.y;
    const int64_t N = g.N;
    const int p = m.crt[j], nc = static_cast<int>(chunks_of(in.n[j]));
    const ModC mp = c.mc[p];
    const int16_t* R2 = c.R + 2 * kW;
    for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < N;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int r = in.p[j][e * in.es[j]];
        const int sig0 = slot_ref(g, m.sig_slot, e).p[0];
        // mini gate y -> (y + r) mod p, 16-bit payload at t16[color] of entry e[k][2]; key hashes: k_bin_keys
        int16_t* t16 = reinterpret_cast<int16_t*>(tb.t[5] + (e * m.k + j) * 3 + 2);
        for (int i = 0; i < 2; ++i) {
            const uint32_t color = static_cast<uint32_t>(sig0 + i * R2[0]) & 1u;
            // hardened: lane j % 8 of pad k + j / 8 of the sign label's y row (MMTw, gadgets.h)
            const u128 H = c.hard ? (hard_pad(hk[i * N + e], stream_of(g.layer, g.sslot, static_cast<uint64_t>(e), g.mask),
                                              tw_sub(kTwMmy, 0), m.k + j / 8) >> (16 * (j % 8)))
                                  : hk[i * N + e];
            const int fv = (i + r) % p;
            t16[color] = static_cast<int16_t>(static_cast<int16_t>(fv) + static_cast<int16_t>(static_cast<uint16_t>(H)));
        }
        const LRef s3 = slot_ref(g, m.sk_slot0 + 2 * j, e), s4 = slot_ref(g, m.sk_slot0 + 2 * j + 1, e);
        int16_t* o = m.out[j] + e * kCh;
        for (int c8 = 0; c8 < nc; ++c8) {
            uint32_t a[8], b[8];
            unpack8(ld_chunk(s4, c8), a);
            unpack8(ld_chunk(s3, c8), b);
#pragma unroll
            for (int u = 0; u < 8; ++u) a[u] = modq(a[u] + static_cast<uint32_t>(p) - b[u], mp);
            st_chunk(o + c8 * N * kCh, pack8(a));
        }
    }
}

// Legacy rescale, before the sign gadget: L += up; trans projections of the
// mod-2 residue into every other residue; L_j = (L_j - out0_j) * 2^-1; L_0 = Z_2.
struct RsArgs {
    int k;
    int crt[kMaxRes];
    int inv[kMaxRes];
    int ctr[kMaxRes];          // first trans-label AES-CTR block of residue j
    int16_t* L[kMaxRes];       // chunked, updated in place
    const int16_t* up;         // [k][kW]
    const int16_t* down;       // [k][kW]
    uint64_t layer, sslot;     // trans stream = stream_of(layer, sslot, e, 0)
};

// Keys x + i*R_2 (i = 0, 1) of a mod-2 label x [+ add], hashed once per
// element (hk[i][N]). Both users need the same two hashes for all k residues:
// the legacy rescale's trans projections of L_0 + up_0 and the ReLU mini
// gates of the sign output. A mod-2 label compresses to its component bits,
// so the key is a bit pack and key 1 is key 0 XOR the bits of R_2. x is a
// chunked label set (16 chunks of 8 components), add a uniform row.
__global__ __launch_bounds__(kGB) void k_bin_keys(Ctx c, const int16_t* x, const int16_t* add, u128* hk, int64_t N) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_aes[kGAesWords];
    aes_lds_fill<kGAes>(lds_aes, c.te0);
    const GAes aes = aes_ctx<kGAes>(lds_aes, nullptr);
    const LRef R2 = row_ref(c.R + 2 * kW);
    uint32_t rb[4] = {0, 0, 0, 0}, ab[4] = {0, 0, 0, 0};
#pragma unroll
    for (int c8 = 0; c8 < 16; ++c8) {
        rb[c8 >> 2] |= bits8(ld_chunk(R2, c8)) << (8 * (c8 & 3));
        if (add) ab[c8 >> 2] |= bits8(ld_chunk(row_ref(add), c8)) << (8 * (c8 & 3));
    }
    const u128 rbits = (static_cast<u128>((static_cast<uint64_t>(rb[3]) << 32) | rb[2]) << 64) |
                       ((static_cast<uint64_t>(rb[1]) << 32) | rb[0]);
    const u128 abits = (static_cast<u128>((static_cast<uint64_t>(ab[3]) << 32) | ab[2]) << 64) |
                       ((static_cast<uint64_t>(ab[1]) << 32) | ab[0]);
    for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < N;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const LRef xe{x + e * kCh, N * kCh};
        uint32_t k0[4] = {0, 0, 0, 0};
#pragma unroll
        for (int c8 = 0; c8 < 16; ++c8) k0[c8 >> 2] |= bits8(ld_chunk(xe, c8)) << (8 * (c8 & 3));
        const u128 key0 = ((static_cast<u128>((static_cast<uint64_t>(k0[3]) << 32) | k0[2]) << 64) |
                           ((static_cast<uint64_t>(k0[1]) << 32) | k0[0])) ^ abits;  // mod-2 add = XOR of the bits
        u128 h0, h1;
        if (c.hard) {  // hardened: the keys (k_relu_finish derives the mini pads)
            h0 = key0;
            h1 = key0 ^ rbits;
        } else {
            aes_encrypt2(aes, key0, key0 ^ rbits, h0, h1);
        }
        hk[e] = h0;
        hk[N + e] = h1;
    }
}

// One thread per (element, residue j >= 1) (grid y = j - 1): the trans
// projection of the mod-2 residue into residue j plus the in-place update of
// L_j. The trans output label is drawn one AES-CTR block at a time and
// consumed at once (no per-thread label array, no scratch). L_0 is not
// written here: the sign gadget reads Z_2 for residue 0 directly (In with a
// zero element stride) and k_rescale_post_g overwrites L_0 afterwards.
__global__ __launch_bounds__(kGB) void k_rescale_pre(Ctx c, RsArgs a, Tables tb, const u128* hk, int64_t N) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_aes[kGAesWords];
    aes_lds_fill<kGAes>(lds_aes, c.te0);
    const GAes aes = aes_ctx<kGAes>(lds_aes, nullptr);
    const int j = 1 + static_cast<int>(blockIdx.y);
    const int p = a.crt[j];
    const ModC mj = c.mc[p];
    const int n = static_cast<int>(mj.n), pm = static_cast<int>(mj.pm);
    const int16_t* R2 = c.R + 2 * kW;
    const int16_t* Rp = c.R + static_cast<int64_t>(p) * kW;
    const int16_t* upj = a.up + j * kW;
    const int64_t cs = N * kCh;
    for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < N;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        // hashes of the two trans rows' keys (L_0 + up_0) + i*R_2: k_bin_keys
        const int l00 = a.L[0][e * kCh];
        const uint32_t color0 = static_cast<uint32_t>(l00 + a.up[0]) & 1u;
        const u128 H0 = hk[e], H1 = hk[N + e];
        const uint64_t stream = stream_of(a.layer, a.sslot, static_cast<uint64_t>(e), 0);
        int16_t* L = a.L[j] + e * kCh;
        CompressFwd p0, p1;
        p0.init();
        p1.init();
        for (int q0 = 0, blk = 0; q0 < n; q0 += pm, ++blk) {
            DigitStream ds;
            ds.init(aes_keyed(aes, (static_cast<u128>(stream) << 64) | static_cast<uint64_t>(a.ctr[j] + blk), c.rk));
            const int cnt = min(pm, n - q0);
            for (int h = 0; h < cnt; ++h) {
                const int q = q0 + h;
                const uint32_t o = ds.next(mj);
                p0.push(o, mj);
                p1.push(modq(o + static_cast<uint32_t>(Rp[q]), mj), mj);
                int16_t& Lq = L[(q >> 3) * cs + (q & 7)];
                int v = Lq + upj[q];
                if (v >= p) v -= p;
                v -= static_cast<int>(o);
                if (v < 0) v += p;
                Lq = static_cast<int16_t>(modq(static_cast<uint32_t>(v * a.inv[j]), mj));
            }
        }
        u128* row = tb.t[6] + e * tb.row[6] + (j - 1) * 2;
        const uint32_t color1 = static_cast<uint32_t>(l00 + a.up[0] + R2[0]) & 1u;
        row[color0] = p0.finish() + H0;
        row[color1] = p1.finish() + H1;
    }
}

// After the sign gadget: L_0 = sign output; L -= down. Elementwise over
// (residue j = blockIdx.y, chunked index (c8 * N + e) * 8 + u).
__global__ __launch_bounds__(256) void k_rescale_post_g(Ctx c, RsArgs a, Gadget g, int sig_slot) {
    const int j = blockIdx.y;
    const int p = a.crt[j];
    const int64_t nc = chunks_of(static_cast<int>(c.mc[p].n));
    const int16_t* dn = a.down + j * kW;
    int16_t* L = a.L[j];
    const int64_t N = g.N;
    const int16_t* sig = slot_base(g, sig_slot);
    for (int64_t x = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; x < N * nc * kCh;
         x += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int q = static_cast<int>(x / (N * kCh)) * kCh + static_cast<int>(x & (kCh - 1));
        const int v = (j == 0 ? sig[x] : L[x]) - dn[q];
        L[x] = static_cast<int16_t>(v < 0 ? v + p : v);
    }
}

// ---------------------------------------------------------------------------
// Label algebra of the remaining layer kinds (dense, sum / max pooling, residual
// add, ReDash rescale, base extension). All labels are chunked component-major
// (kCh), so each thread moves one 16-byte chunk (8 components) of one element.

// dst = ca a + cb b + cr r (mod p), any operand optional. A label set has element stride 8 and chunk stride
// 8 N; a uniform row (R_p, Z_p, a shift label) element stride 0 and chunk stride 8. Chunk padding past n stays 0
// when the operands' padding is 0 (draws, rows and every kernel here keep it 0).
struct LinJob {
    int16_t* dst;
    const int16_t* a;
    const int16_t* b;
    const int16_t* r;
    int64_t aes, acs, bes, bcs;
    int p, nc;
    int ca, cb, cr;
};
constexpr int kMaxLin = 24;
struct LinArgs {
    LinJob j[kMaxLin];
    int n;
    int64_t N;
};
__global__ __launch_bounds__(256) void k_lin(Ctx c, LinArgs a) {
    const LinJob J = a.j[blockIdx.y];
    const ModC m = c.mc[J.p];
    const int64_t N = a.N, total = N * J.nc;
    const uint32_t ca = J.ca, cb = J.cb, cr = J.cr;
    for (int64_t x = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; x < total;
         x += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int c8 = static_cast<int>(x / N);
        const int64_t e = x - static_cast<int64_t>(c8) * N;
        uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t[8];
        if (J.a) {
            unpack8(*reinterpret_cast<const u32x4a*>(J.a + e * J.aes + c8 * J.acs), t);
#pragma unroll
            for (int u = 0; u < 8; ++u) acc[u] += ca * t[u];
        }
        if (J.b) {
            unpack8(*reinterpret_cast<const u32x4a*>(J.b + e * J.bes + c8 * J.bcs), t);
#pragma unroll
            for (int u = 0; u < 8; ++u) acc[u] += cb * t[u];
        }
        if (J.r) {
            unpack8(*reinterpret_cast<const u32x4a*>(J.r + c8 * kCh), t);
#pragma unroll
            for (int u = 0; u < 8; ++u) acc[u] += cr * t[u];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc[u] = modq(acc[u], m);
        st_chunk(J.dst + (static_cast<int64_t>(c8) * N + e) * kCh, pack8(acc));
    }
}

// Gathered sums: dst[e] (+)= sum_t cf[t] src[map[e K + t]] (mod p); map entries < 0 are skipped. Max-pool
// window gathers, pair differences and recombination, sum-pool windows.
constexpr int kMaxTerms = 16;
struct GsJob {
    int16_t* dst;
    const int16_t* src;
    int p, nc;
    int cf[kMaxTerms];
};
struct GsArgs {
    GsJob j[kMaxRes];
    int n, K, acc;
    int64_t N, Nsrc;
    const int32_t* map;
};
__global__ __launch_bounds__(256) void k_gsum(Ctx c, GsArgs a) {
    const GsJob& J = a.j[blockIdx.y];
    const ModC m = c.mc[J.p];
    const int64_t N = a.N, total = N * J.nc;
    for (int64_t x = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; x < total;
         x += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int c8 = static_cast<int>(x / N);
        const int64_t e = x - static_cast<int64_t>(c8) * N;
        int16_t* d = J.dst + (static_cast<int64_t>(c8) * N + e) * kCh;
        uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t[8];
        if (a.acc) unpack8(*reinterpret_cast<const u32x4a*>(d), acc);
        for (int s = 0; s < a.K; ++s) {
            const int32_t src = a.map[e * a.K + s];
            if (src < 0) continue;
            unpack8(*reinterpret_cast<const u32x4a*>(J.src + (static_cast<int64_t>(c8) * a.Nsrc + src) * kCh), t);
            const uint32_t f = static_cast<uint32_t>(J.cf[s]);
#pragma unroll
            for (int u = 0; u < 8; ++u) acc[u] += f * t[u];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc[u] = modq(acc[u], m);
        st_chunk(d, pack8(acc));
    }
}

// Hardened encoding (garbler.cpp): public constants c_g (one per group of `group` consecutive elements, e.g.
// a conv filter's bias) folded into the base labels, y_e += c_{e / group} R_p (mod p), so the constant wires
// need no evaluator-visible label. Grid (element x chunk work, residue j).
struct FoldJob {
    int16_t* dst;
    const int32_t* c;  // [groups] constants reduced mod p
    int p, nc;
};
struct FoldArgs {
    FoldJob j[kMaxRes];
    int64_t N, group;
};
__global__ __launch_bounds__(256) void k_fold(Ctx c, FoldArgs a) {
    const FoldJob& J = a.j[blockIdx.y];
    const ModC m = c.mc[J.p];
    const int16_t* Rp = c.R + static_cast<int64_t>(J.p) * kW;
    const int64_t N = a.N, total = N * J.nc;
    for (int64_t x = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; x < total;
         x += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int c8 = static_cast<int>(x / N);
        const int64_t e = x - static_cast<int64_t>(c8) * N;
        int16_t* d = J.dst + (static_cast<int64_t>(c8) * N + e) * kCh;
        const uint32_t f = static_cast<uint32_t>(J.c[e / a.group]);
        uint32_t acc[8], t[8];
        unpack8(*reinterpret_cast<const u32x4a*>(d), acc);
        unpack8(*reinterpret_cast<const u32x4a*>(Rp + c8 * kCh), t);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc[u] = modq(acc[u] + f * t[u], m);
        st_chunk(d, pack8(acc));
    }
}

// Dense base labels y_o = sum_i w_oi x_i + zc_o Z_p (mod p), weights reduced mod p and transposed ([in][out],
// rows already in the channel_tf source order), zc_o = 1 + #(w_oi = 0 mod p) (the reference's zero-weight Z
// quirk, and the bias label's Z). Block: 64 outputs x 4 input groups for one (chunk, residue); the groups'
// partial sums meet in LDS.
struct DnJob {
    int16_t* dst;
    const int16_t* x;
    const int16_t* wt;
    const int32_t* zc;
    int p, nc;
};
struct DnArgs {
    DnJob j[kMaxRes];
    int n, in, out, otiles;
};
__global__ __launch_bounds__(256) void k_gdense(Ctx c, DnArgs a) {
    __shared__ uint32_t part[3][64][9];
    const DnJob J = a.j[blockIdx.y];
    const int c8 = static_cast<int>(blockIdx.x) / a.otiles;
    if (c8 >= J.nc) return;
    const int o = (static_cast<int>(blockIdx.x) - c8 * a.otiles) * 64 + (threadIdx.x & 63);
    const int grp = threadIdx.x >> 6;
    const ModC m = c.mc[J.p];
    const int64_t xcs = static_cast<int64_t>(a.in) * kCh;
    uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t[8];
    if (o < a.out) {
        int since = 0;
        for (int i = grp; i < a.in; i += 4) {
            const uint32_t w = static_cast<uint16_t>(J.wt[static_cast<int64_t>(i) * a.out + o]);
            if (w) {
                unpack8(*reinterpret_cast<const u32x4a*>(J.x + c8 * xcs + static_cast<int64_t>(i) * kCh), t);
#pragma unroll
                for (int u = 0; u < 8; ++u) acc[u] += w * t[u];
            }
            if (++since == 256) {  // w, x < p <= 2048: 256 products stay below 2^30 on top of a residue
                since = 0;
#pragma unroll
                for (int u = 0; u < 8; ++u) acc[u] = modq(acc[u], m);
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc[u] = modq(acc[u], m);
    }
    if (grp > 0) {
#pragma unroll
        for (int u = 0; u < 8; ++u) part[grp - 1][threadIdx.x & 63][u] = acc[u];
    }
    __syncthreads();
    if (grp == 0 && o < a.out) {
        unpack8(*reinterpret_cast<const u32x4a*>(c.Z + static_cast<int64_t>(J.p) * kW + c8 * kCh), t);
        const uint32_t zc = static_cast<uint32_t>(J.zc[o]);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            uint32_t v = acc[u] + part[0][o & 63][u] + part[1][o & 63][u] + part[2][o & 63][u];
            v = modq(v, m) + modq(zc, m) * t[u];
            acc[u] = modq(v, m);
        }
        st_chunk(J.dst + (static_cast<int64_t>(c8) * a.out + o) * kCh, pack8(acc));
    }
}

// ------------------------------------------------------------------- host
struct SignLayout {
    std::vector<Draw> draws;
    std::vector<Proj> projs;
    int fan[kMaxMrs] = {};  // output modulus of the approx fan-out per digit
    SignSlots ss{};
    int nslots = 0;
    int out_slot0 = 0;
    int64_t entries = 0;
};

// Fused construction (gadgets.cpp sign_garble_fused): digit labels, carries, outputs.
SignLayout sign_layout_fused(const SignPlan& P, int extra_slots) {
    SignLayout L;
    const int k = static_cast<int>(P.crt.size()), t = static_cast<int>(P.mrs.size());
    int slot = 0, ctr = 0;
    auto draw = [&](int q) {
        L.draws.push_back({slot, q, ctr});
        ctr += prg_blocks(q);
        return slot++;
    };
    const int dig0 = slot;
    for (int j = 0; j < k; ++j)
        for (int d = 0; d < t; ++d) draw(P.digit_mod(d));
    const int newc0 = slot;
    for (int q = 0; q + 1 < t; ++q) draw(P.carry_mod(t - 1 - q));
    L.out_slot0 = slot;
    for (int o : P.out_mod) draw(o);
    const int sum2_0 = slot;
    slot += std::max(0, t - 1);
    const int sum_slot = slot++;
    L.nslots = slot + extra_slots;
    L.ss.k = k;
    L.ss.t = t;
    L.ss.fused = 1;
    for (int d = 0; d < t; ++d) {
        L.ss.mrs[d] = P.mrs[d];
        L.ss.dmod[d] = P.digit_mod(d);
        L.fan[d] = P.digit_mod(d);
    }
    L.ss.sum2_slot0 = sum2_0;
    L.ss.sum_slot = sum_slot;
    L.ss.bases_slot0 = 0;
    L.ss.newc_slot0 = newc0;
    L.ss.mrs_slot0 = dig0;
    L.ss.stride_q = 1;
    int64_t first = 0;
    auto add = [&](Proj p) {
        p.first = first;
        first += p.pin;
        L.projs.push_back(p);
    };
    for (int j = 0; j < k; ++j) {
        Proj ap{S_INPUT, j, P.crt[j], dig0 + j * t, P.mrs[0], F_LUT, j, 0, t, R_BANK, 0, 0, t, t * P.crt_prefix[j], 0};
        ap.hsub = tw_sub(kTwApprox, static_cast<uint32_t>(j));  // slots = digits
        add(ap);
    }
    int64_t c2 = 0;
    for (int q = 0; q + 1 < t; ++q) {
        const int d = t - 1 - q;
        const int mo = P.digit_mod(d);
        Proj cp{S_SLOT, sum2_0 + q, mo, newc0 + q, P.carry_mod(d), F_DIVMOD, P.mrs[d], P.mrs[d - 1], 0, R_BANK, 0,
                2, 1, c2, 0};
        cp.hsub = tw_sub(kTwCast2, static_cast<uint32_t>(d));
        add(cp);
        c2 += mo;
    }
    const int m0 = P.mrs[0];
    for (size_t o = 0; o < P.out_mod.size(); ++o) {
        Proj sp{S_SLOT, sum_slot, m0, L.out_slot0 + static_cast<int>(o), P.out_mod[o], F_SIGN, m0 / 2, P.lower, P.upper,
                R_BANK, 0, 3, 1, static_cast<int64_t>(o) * m0, 0};
        sp.hsub = tw_sub(kTwSign, 0);
        sp.hslot = static_cast<int>(o);
        add(sp);
    }
    L.entries = first;
    return L;
}

// Mirrors sign_garble_elem: draw order = PRG counter order.
SignLayout sign_layout(const SignPlan& P, int extra_slots) {
    if (P.fused) return sign_layout_fused(P, extra_slots);
    SignLayout L;
    const int k = static_cast<int>(P.crt.size()), t = static_cast<int>(P.mrs.size());
    int slot = 0, ctr = 0;
    auto draw = [&](int q) {
        L.draws.push_back({slot, q, ctr});
        ctr += prg_blocks(q);
        return slot++;
    };
    const int mrs0 = slot;
    for (int j = 0; j < k; ++j)
        for (int d = 0; d < t; ++d) draw(P.mrs[d]);
    const int stride_q = k + 2;
    const int bases0 = slot;
    for (int q = 0; q + 1 < t; ++q) {
        const int d = t - 1 - q;
        for (int j = 0; j <= k; ++j) draw((k + 1) * P.mrs[d]);
        draw(P.mrs[d - 1]);  // newc
    }
    L.out_slot0 = slot;
    for (int o : P.out_mod) draw(o);
    // derived slots
    const int sum2_0 = slot;
    slot += std::max(0, t - 1);
    const int sum_slot = slot++;
    L.nslots = slot + extra_slots;
    L.ss.k = k;
    L.ss.t = t;
    for (int d = 0; d < t; ++d) {
        L.ss.mrs[d] = P.mrs[d];
        L.ss.dmod[d] = P.mrs[d];
        L.fan[d] = P.mrs[d];
    }
    L.ss.sum2_slot0 = sum2_0;
    L.ss.sum_slot = sum_slot;
    L.ss.bases_slot0 = bases0;
    L.ss.newc_slot0 = bases0 + (k + 1);
    L.ss.mrs_slot0 = mrs0;
    L.ss.stride_q = stride_q;
    // projections (table ids: 0 approx, 1 cast1, 2 cast2, 3 sign)
    int64_t first = 0;
    auto add = [&](Proj p) {
        p.first = first;
        first += p.pin;
        L.projs.push_back(p);
    };
    // approx: ONE projection per residue j fanned out over the t digits (same input key and hash for all
    // digits; per digit d: output slot mrs0 + j*t + d, modulus mrs[d], table offset + d), see k_project
    for (int j = 0; j < k; ++j)
        add(Proj{S_INPUT, j, P.crt[j], mrs0 + j * t, P.mrs[0], F_LUT, j, 0, t, R_BANK, 0, 0, t,
                 t * P.crt_prefix[j], 0});
    int64_t c1 = 0, c2 = 0;
    for (int q = 0; q + 1 < t; ++q) {
        const int d = t - 1 - q;
        const int m = P.mrs[d], mo = (k + 1) * m;
        for (int j = 0; j <= k; ++j) {
            Proj p{};
            if (j < k) {
                p.in_kind = S_SLOT;
                p.in_idx = mrs0 + j * t + d;
            } else if (q == 0) {
                p.in_kind = S_ZERO;  // carry of the least significant digit: Z_{m_last}
                p.in_idx = 0;
            } else {
                p.in_kind = S_SLOT;
                p.in_idx = bases0 + (q - 1) * stride_q + (k + 1);  // newc of the previous digit
            }
            p.pin = m;
            p.out_slot = bases0 + q * stride_q + j;
            p.pout = mo;
            p.fn = F_IDENT;
            p.outr_kind = R_BANK;
            p.table = 1;
            p.stride = 1;
            p.off = c1;
            c1 += m;
            add(p);
        }
        add(Proj{S_SLOT, sum2_0 + q, mo, bases0 + q * stride_q + (k + 1), P.mrs[d - 1], F_DIV, m, 0, 0, R_BANK, 0, 2, 1,
                 c2, 0});
        c2 += mo;
    }
    const int m0 = P.mrs[0];
    for (size_t o = 0; o < P.out_mod.size(); ++o)
        add(Proj{S_SLOT, sum_slot, m0, L.out_slot0 + static_cast<int>(o), P.out_mod[o], F_SIGN, m0 / 2, P.lower, P.upper,
                 R_BANK, 0, 3, 1, static_cast<int64_t>(o) * m0, 0});
    L.entries = first;
    return L;
}

// Structure-only device constants (gadget descriptors, public conv weights):
// identical for every GC of a model, so they are uploaded once per process and
// reused. A fresh hipMalloc + hipMemcpy + hipFree per gadget made every layer
// drain the GPU queue before the host could prepare the next one.
struct ConstCache {
    std::mutex m;
    std::map<std::tuple<int, uint64_t, size_t>, std::pair<std::string, void*>> map;
};
inline ConstCache& const_cache() {
    static ConstCache* c = new ConstCache();  // leaked: lives as long as the process
    return *c;
}
template <class T>
const T* dconst(const T* h, size_t n) {
    const size_t bytes = n * sizeof(T);
    const char* b = reinterpret_cast<const char*>(h);
    uint64_t x = 1469598103934665603ull;  // FNV-1a
    for (size_t i = 0; i < bytes; ++i) x = (x ^ static_cast<uint8_t>(b[i])) * 1099511628211ull;
    int dev = 0;
    HIPCHECK(hipGetDevice(&dev));
    ConstCache& c = const_cache();
    std::lock_guard<std::mutex> g(c.m);
    auto key = std::make_tuple(dev, x, bytes);
    auto it = c.map.find(key);
    if (it != c.map.end() && it->second.first.compare(0, std::string::npos, b, bytes) == 0)
        return static_cast<const T*>(it->second.second);
    void* d = nullptr;
    HIPCHECK(hipMalloc(&d, std::max<size_t>(1, bytes)));
    if (bytes) HIPCHECK(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice));
    if (it != c.map.end()) return static_cast<const T*>(d);  // hash collision: keep the first entry, leak this one
    c.map.emplace(key, std::make_pair(std::string(b, bytes), d));
    return static_cast<const T*>(d);
}

}  // namespace gg


// DASH_GG_TRACE=1: per-call phase timings on stderr (upload / alloc / kernels / download)
struct PhaseTrace {
    bool on = std::getenv("DASH_GG_TRACE") != nullptr;
    const char* what;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now(), t = t0;
    std::string line;
    explicit PhaseTrace(const char* w) : what(w) {}
    void mark(const char* phase) {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        line += std::string(" ") + phase + "=" + std::to_string(std::chrono::duration<double, std::milli>(n - t).count());
        t = n;
    }
    ~PhaseTrace() {
        if (on) std::fprintf(stderr, "[gg] %s%s\n", what, line.c_str());
    }
};

// ------------------------------------------------------- table block cache
namespace {
struct BlockCache {
    std::mutex m;
    // (device, stream, bytes): a block is reused only on the stream that released it (stream-ordered reuse;
    // two garbling contexts never hand each other a block their queued kernels may still touch)
    std::multimap<std::tuple<int, hipStream_t, size_t>, void*> free;
    size_t cached = 0;
    size_t cap = static_cast<size_t>(std::getenv("DASH_GG_CACHE_GB") ? std::atof(std::getenv("DASH_GG_CACHE_GB")) * 1e9
                                                                      : 16e9);
};
BlockCache& block_cache() {
    static BlockCache* c = new BlockCache();  // leaked: deleters may run during static destruction
    return *c;
}

void* cache_get(int device, hipStream_t st, size_t bytes) {
    BlockCache& c = block_cache();
    {
        std::lock_guard<std::mutex> g(c.m);
        auto it = c.free.find(std::make_tuple(device, st, bytes));
        if (it != c.free.end()) {
            void* p = it->second;
            c.free.erase(it);
            c.cached -= bytes;
            return p;
        }
    }
    void* p = nullptr;
    HIPCHECK(hipMalloc(&p, bytes));
    return p;
}

void cache_put(int device, hipStream_t st, void* p, size_t bytes) {
    if (!p) return;
    BlockCache& c = block_cache();
    {
        std::lock_guard<std::mutex> g(c.m);
        if (c.cached + bytes <= c.cap) {
            c.free.emplace(std::make_tuple(device, st, bytes), p);
            c.cached += bytes;
            return;
        }
    }
    (void)hipFree(p);
}
}  // namespace

void gpu_table_cache_trim() {
    BlockCache& c = block_cache();
    std::lock_guard<std::mutex> g(c.m);
    for (auto& kv : c.free) (void)hipFree(kv.second);
    c.free.clear();
    c.cached = 0;
}

size_t gpu_table_cache_bytes() {
    BlockCache& c = block_cache();
    std::lock_guard<std::mutex> g(c.m);
    return c.cached;
}

namespace {
inline unsigned blocks_for(int64_t n, int bs, int cap = 65536) {
    return static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((n + bs - 1) / bs, cap)));
}

// a cached device block with RAII return to the cache (or a borrowed buffer: never cached or freed)
struct DevBlock {
    void* p = nullptr;
    size_t bytes = 0;
    int device = 0;
    bool borrowed = false;
    hipStream_t st = nullptr;  // the garbling stream that allocated (and last used) the block
    DevBlock() = default;
    DevBlock(const DevBlock&) = delete;
    DevBlock& operator=(const DevBlock&) = delete;
    DevBlock(DevBlock&& o) noexcept { *this = std::move(o); }
    DevBlock& operator=(DevBlock&& o) noexcept {
        release();
        p = o.p;
        bytes = o.bytes;
        device = o.device;
        borrowed = o.borrowed;
        st = o.st;
        o.p = nullptr;
        return *this;
    }
    ~DevBlock() { release(); }
    void alloc(int dev, size_t b) {
        release();
        device = dev;
        bytes = std::max<size_t>(16, b);
        borrowed = false;
        st = gg::tl_st;
        p = cache_get(dev, st, bytes);
    }
    void borrow(int dev, void* q, size_t b) {
        release();
        device = dev;
        bytes = b;
        borrowed = true;
        p = q;
    }
    void release() {
        if (p && !borrowed) cache_put(device, st, p, bytes);
        p = nullptr;
    }
    template <class T>
    T* as() const {
        return static_cast<T*>(p);
    }
};

struct DevTable {
    DevBlock b;
    int64_t row = 0;
    // zero: only for tables whose entries are not all written by the kernels (the ReLU e table's
    // mini entry fills 2 of its 8 int16 slots); every other table is fully covered, since the
    // colors of a projection's p keys are a permutation of Z_p (R[0] = 1).
    // target: the model array this table becomes; when it already names an external device buffer
    // (GarbleOptions::sink: an evaluator's arena slot) the kernels write there directly.
    void alloc(int device, int64_t N, int64_t r, const Array& target, bool zero = false) {
        row = r;
        const size_t bytes = static_cast<size_t>(N) * r * sizeof(u128);
        if (target.device_resident() && target.dev->external) {
            DASH_CHECK(target.nbytes == bytes && target.dev->device == device, "gpu garbler: table sink size mismatch");
            b.borrow(device, const_cast<void*>(target.device_ptr()), bytes);
        } else {
            b.alloc(device, bytes);
        }
        if (zero) HIPCHECK(hipMemsetAsync(b.p, 0, b.bytes, gg::tl_st));
    }
    u128* p() const { return b.as<u128>(); }
    // hand the buffer to `a` as a device-resident array (kept in HBM; the
    // evaluator on this node copies it device-to-device). Its deleter returns
    // the block to the cache. A borrowed (sink) buffer already is `a`'s.
    void to_array(Array& a, int device) {
        if (b.borrowed) {
            DASH_CHECK(a.device_ptr() == b.p, "gpu garbler: sink table rebound");
            b.p = nullptr;
            return;
        }
        DASH_CHECK(a.nbytes <= b.bytes && (a.nbytes == static_cast<size_t>(b.bytes) || a.nbytes < 16),
                   "gpu garbler: table size mismatch");
        auto d = std::make_shared<Array::Device>();
        const size_t bytes = b.bytes;
        const hipStream_t st = b.st;
        d->p = std::shared_ptr<void>(b.p, [device, st, bytes](void* x) { cache_put(device, st, x, bytes); });
        b.p = nullptr;
        d->device = device;
        d->fetch = [device](void* h, const void* dv, size_t n) {
            HIPCHECK(hipSetDevice(device));
            HIPCHECK(hipMemcpy(h, dv, n, hipMemcpyDeviceToHost));
        };
        a = Array::on_device(a.dtype, a.shape, std::move(d));
    }
};

// k_draw grid: one lane per (draw, element), elements padded to whole waves
// A/B knob DASH_GG_DRAW_BLOCKS: grid cap of k_draw (grid-stride; every block fills its 32 / 64 KiB LDS AES image)
inline int draw_block_cap() {
    static const int v = [] {
        const char* e = std::getenv("DASH_GG_DRAW_BLOCKS");
        return e ? std::max(1, std::atoi(e)) : 16384;
    }();
    return v;
}
unsigned draw_grid(const gg::Gadget& g) {
    const int64_t lanes = (g.N + gg::kTile - 1) / gg::kTile * gg::kTile * g.ndraws;
    return blocks_for(lanes, gg::kGB, draw_block_cap());
}

// AES-CTR blocks per element: draws are laid out back to back in counter order
int draw_blocks(const std::vector<gg::Draw>& d) {
    if (d.empty()) return 0;
    return d.back().ctr + prg_blocks(d.back().q);
}

void check_desc(const gg::Gadget& g) {
    DASH_CHECK(g.ndraws <= gg::kMaxDesc && g.nprojs <= gg::kMaxDesc,
               "gpu garbler: gadget descriptor exceeds the LDS-staged limit");
}

// run the three sign-gadget passes for N elements with input labels `in`
// key-hash scratch of the calling thread's garbling context (DevCtx, grow-only): [entries][N] hashes + colors
std::pair<u128*, uint16_t*> hc_scratch(size_t entries, int64_t N);
u128* bank_scratch(size_t rows, int64_t N);
const uint32_t* const* ensure_iR(const gg::Ctx& c, const std::vector<int>& mods);

// Host-side function data of a projection set (the value f(i, d) of every entry): k_emit reads bank rows
// and bank indices built from it here, so none of it is needed on the device.
struct ProjFns {
    const std::vector<int16_t>* flut = nullptr;  // F_FAN values [a0 + i * t + d]
    const std::vector<int>* fan = nullptr;       // F_FAN target moduli [a1 + d]
    const std::vector<int16_t>* lut = nullptr;   // F_LUT approx lookup, residue j's [p][t] at lut_off[j]
    const int* lut_off = nullptr;
};

// k_emit dynamic LDS budget per block (A/B knob DASH_GG_EMIT_LDS_KB): smaller scopes per block, more
// resident blocks per CU to overlap one block's staging loads with another's table stores. With the hardened
// encoding's ChaCha pads (VALU-heavy) 24 KiB measured best: garble + load 7.8 / 7.4 / 7.0 ms per MiniONN GC at
// 48 / 16 / 24 KiB (profiles/ab/README.md, round 5)
inline size_t emit_lds_budget() {
    static const size_t v = [] {
        const char* e = std::getenv("DASH_GG_EMIT_LDS_KB");
        const int kb = e ? std::atoi(e) : 24;
        return static_cast<size_t>(std::min(56, std::max(8, kb))) << 10;
    }();
    return v;
}

// The projections of a gadget: k_hash (one key hash per (element, color)), then k_emit over scopes. Host
// preparation, cached by content per gadget structure (dconst): the per-table position maps, the scopes
// (contiguous position ranges covering whole projections, te elements per block within the LDS budget),
// the deduplicated bank rows of every scope and the (i, d) -> bank row index of every projection.
// g.draws / label slots must be ready (same stream).
void project(const gg::Ctx& c, gg::Gadget& g, const gg::In& in, const gg::Tables& tb, const std::vector<gg::Proj>& pr,
             const ProjFns& fx = ProjFns()) {
    DASH_CHECK(!pr.empty() && pr.size() <= 255, "gpu garbler: projection count outside [1, 255]");
    const int np = static_cast<int>(pr.size());
    auto is_fan = [](const gg::Proj& p) { return p.fn == gg::F_LUT || p.fn == gg::F_FAN; };
    auto elem_dep = [](const gg::Proj& p) { return p.fn == gg::F_MULR || p.fn == gg::F_NEGR; };
    auto targets = [&](const gg::Proj& p) { return is_fan(p) ? p.stride : 1; };
    auto extent = [&](const gg::Proj& p) {
        return is_fan(p) ? static_cast<int64_t>(p.pin) * p.stride : static_cast<int64_t>(p.pin - 1) * p.stride + 1;
    };
    auto pout_of = [&](const gg::Proj& p, int d) {
        if (p.fn == gg::F_LUT) return g.mrs[d];
        if (p.fn == gg::F_FAN) return (*fx.fan)[p.a1 + d];
        return p.pout;
    };
    auto value = [&](const gg::Proj& p, int i, int d) -> int {  // f(i, d) mod pout, element-independent f
        const int t = targets(p), po = pout_of(p, d);
        int64_t f;
        switch (p.fn) {
            case gg::F_LUT: f = (*fx.lut)[fx.lut_off[p.a0] + i * t + d]; break;
            case gg::F_FAN: f = (*fx.flut)[p.a0 + i * t + d]; break;
            case gg::F_DIV: f = i / p.a0; break;
            case gg::F_DIVMOD: f = (i / p.a0) % p.a1; break;
            case gg::F_SIGN: f = i < p.a0 ? p.a2 : p.a1; break;
            default: f = i;
        }
        f %= po;
        return static_cast<int>(f < 0 ? f + po : f);
    };
    for (const auto& p : pr) {
        DASH_CHECK(p.pin >= 2 && p.pin <= 4096 && targets(p) < 4096, "gpu garbler: projection shape out of range");
        DASH_CHECK(p.table >= 0 && p.table < 8 && tb.t[p.table] != nullptr && tb.row[p.table] > 0,
                   "gpu garbler: projection into an unallocated table");
        DASH_CHECK(p.fn != gg::F_LUT || (fx.lut && fx.lut_off), "gpu garbler: F_LUT projection without its lookup");
        DASH_CHECK(p.fn != gg::F_FAN || (fx.flut && fx.fan), "gpu garbler: F_FAN projection without its values");
    }
    gg::Emit em{};
    em.by_i = 0;
    // position maps
    std::vector<uint32_t> map;
    for (int t = 0; t < 8; ++t) {
        bool used = false;
        for (const auto& p : pr) used |= p.table == t;
        if (!used) continue;
        const int64_t row = tb.row[t];
        const size_t m0 = map.size();
        em.map_off[t] = static_cast<int64_t>(m0);
        map.resize(m0 + static_cast<size_t>(row), gg::kHole);
        for (int pi = 0; pi < np; ++pi) {
            const auto& p = pr[pi];
            if (p.table != t) continue;
            const int nt = targets(p);
            for (int col = 0; col < p.pin; ++col)
                for (int d = 0; d < nt; ++d) {
                    const int64_t pos = p.off + (is_fan(p) ? static_cast<int64_t>(col) * nt + d : static_cast<int64_t>(col) * p.stride);
                    DASH_CHECK(pos >= 0 && pos < row && map[m0 + pos] == gg::kHole,
                               "gpu garbler: projection table positions overlap or overflow the row");
                    map[m0 + pos] = (static_cast<uint32_t>(pi) << 24) | (static_cast<uint32_t>(col) << 12) |
                                    static_cast<uint32_t>(d);
                }
        }
    }
    // scopes: projections by (table, offset); overlapping spans must share a scope, adjacent ones are grouped
    // while the group stays small (te >= 8)
    std::vector<int> order(np);
    for (int i = 0; i < np; ++i) order[i] = i;
    std::sort(order.begin(), order.end(), [&](int x, int y) {
        return std::tie(pr[x].table, pr[x].off) < std::tie(pr[y].table, pr[y].off);
    });
    const bool by_i0 = gg::gg_hash_mode() == 2 && !std::any_of(pr.begin(), pr.end(), [](const gg::Proj& p) {
        return p.pin >= 32768;
    });
    // fused (hardened, no element-dependent payload offsets): k_emit computes its tile's keys and bank payloads,
    // no k_hash_iu / k_bank launches and no HC / CC / BK round trip through HBM
    const bool fused = by_i0 && c.hard && gg::gg_emit_fused() && std::none_of(pr.begin(), pr.end(), [](const gg::Proj& p) {
        return p.outr_kind == gg::R_INPUT;
    });
    const bool by_i = by_i0 && !fused;
    auto elem_bytes = [&](int64_t ne, int64_t nb) { return ne * (16 + 2 + (by_i ? 2 : 0)) + nb * 16; };
    auto rows_bound = [&](const gg::Proj& p) {  // bank rows upper bound
        int64_t n = 0;
        for (int d = 0; d < targets(p); ++d) n += std::min<int64_t>(elem_dep(p) ? pout_of(p, d) : p.pin, pout_of(p, d));
        return n;
    };
    std::vector<std::vector<int>> groups;
    {
        int64_t gend = -1, gne = 0, gnb = 0;
        int gt = -1;
        for (int pi : order) {
            const auto& p = pr[pi];
            const bool overlap = p.table == gt && p.off < gend;
            const bool near = p.table == gt && p.off <= gend + 8 &&
                              elem_bytes(gne + p.pin, gnb + rows_bound(p)) * 9 <= static_cast<int64_t>(emit_lds_budget());
            if (groups.empty() || !(overlap || near)) {
                groups.push_back({});
                gend = -1;
                gne = gnb = 0;
                gt = p.table;
            }
            groups.back().push_back(pi);
            gend = std::max(gend, p.off + extent(p));
            gne += p.pin;
            gnb += rows_bound(p);
        }
    }
    std::vector<gg::EProj> ep(np);
    std::vector<uint16_t> bix;
    std::vector<gg::BankRow> rows;
    std::vector<gg::Scope> sc;
    std::vector<uint32_t> quads;
    size_t lds_max = 0;
    const auto N = g.N;
    for (const auto& grp : groups) {
        gg::Scope S{};
        S.table = pr[grp[0]].table;
        int64_t a = INT64_MAX, end = 0, r0 = INT64_MAX, r1 = 0;
        for (int pi : grp) {
            a = std::min(a, pr[pi].off);
            end = std::max(end, pr[pi].off + extent(pr[pi]));
            r0 = std::min(r0, pr[pi].first);
            r1 = std::max(r1, pr[pi].first + pr[pi].pin);
        }
        S.a = static_cast<int>(a);
        S.span = static_cast<int>(end - a);
        S.r0 = static_cast<int>(r0);
        S.ne = static_cast<int>(r1 - r0);
        S.b0 = static_cast<int>(rows.size());
        S.bx0 = static_cast<int>(bix.size());
        std::map<std::tuple<int, int, int, int>, int> dedup;
        auto row_of = [&](int slot, int po, int v, int res) {
            auto key = std::make_tuple(slot, po, v, res);
            auto it = dedup.find(key);
            if (it != dedup.end()) return it->second;
            const int r = static_cast<int>(rows.size()) - S.b0;
            rows.push_back(gg::BankRow{slot, po, v, res});
            dedup.emplace(key, r);
            return r;
        };
        for (int pi : grp) {
            const auto& p = pr[pi];
            gg::EProj& E = ep[pi];
            E.first = static_cast<int>(p.first);
            E.hsub = p.hsub;
            E.hslot = p.hslot;
            DASH_CHECK(p.pout > 0 && p.pout < 65536 && p.a0 < 32768, "gpu garbler: projection outside the emit descriptor");
            E.fn = static_cast<int16_t>(p.fn);
            E.t = static_cast<int16_t>(targets(p));
            E.res = static_cast<int16_t>(elem_dep(p) ? p.a0 : -1);
            E.pout = static_cast<uint16_t>(p.pout);
            E.in_kind = static_cast<int16_t>(p.in_kind);
            E.in_idx = p.in_idx;
            E.pin = static_cast<uint16_t>(p.pin);
            const int res = p.outr_kind == gg::R_INPUT ? p.outr_idx : -1;
            if (elem_dep(p)) {
                E.pay1 = static_cast<int>(rows.size()) - S.b0;
                for (int v = 0; v < p.pout; ++v) rows.push_back(gg::BankRow{p.out_slot, p.pout, v, res});
            } else {
                E.pay1 = static_cast<int>(bix.size());
                for (int i = 0; i < p.pin; ++i)
                    for (int d = 0; d < E.t; ++d) {
                        const int r = row_of(is_fan(p) ? p.out_slot + d : p.out_slot, pout_of(p, d), value(p, i, d), res);
                        DASH_CHECK(r < 65536, "gpu garbler: bank row index overflow");
                        bix.push_back(static_cast<uint16_t>(r));
                    }
            }
        }
        S.nb = static_cast<int>(rows.size()) - S.b0;
        S.nbx = static_cast<int>(bix.size()) - S.bx0;
        S.q0 = static_cast<int>(quads.size());
        if (c.hard) {
            // runs of positions sharing one pad block: same projection and color, consecutive fan-out targets
            int open = -1;  // index of the run being extended
            uint32_t pm = 0;
            for (int64_t pos = a; pos < end; ++pos) {
                const uint32_t m = map[em.map_off[S.table] + pos];
                if (m == gg::kHole) {
                    open = -1;
                    continue;
                }
                const auto& p = pr[m >> 24];
                const int d = static_cast<int>(m & 0xfffu);
                const int slot = p.hslot + (is_fan(p) ? d : 0);
                if (open >= 0 && is_fan(p) && (m >> 12) == (pm >> 12) && d == static_cast<int>(pm & 0xfffu) + 1 &&
                    (quads[open] & 7u) < 4 && (slot >> 2) == ((slot - 1) >> 2)) {
                    ++quads[open];
                } else {
                    DASH_CHECK(pos - a < (1 << 28), "gpu garbler: table scope too wide for the pad runs");
                    quads.push_back(static_cast<uint32_t>(pos - a) << 3 | 1u);
                    open = static_cast<int>(quads.size()) - 1;
                }
                pm = m;
            }
        }
        S.nq = static_cast<int>(quads.size()) - S.q0;
        const size_t per = static_cast<size_t>(elem_bytes(S.ne, S.nb));
        // position map, bank indices and (hardened) the pad runs staged in LDS
        const size_t fixed = static_cast<size_t>(S.span) * 4 + static_cast<size_t>(S.nbx) * 2 + 16 +
                             (c.hard ? static_cast<size_t>(S.nq) * 4 + 4 : 0);
        auto lds_of = [&](int sh) { return ((1u << sh) + 1) * per + fixed; };
        int tsh = 5;
        while (tsh > 0 && lds_of(tsh) > emit_lds_budget()) --tsh;
        DASH_CHECK(lds_of(tsh) <= (64u << 10) - sizeof(gg::EProj) * gg::kMaxDesc, "gpu garbler: projection scope exceeds LDS");
        S.tsh = tsh;
        lds_max = std::max(lds_max, lds_of(tsh));
        S.blk0 = em.blocks;
        em.blocks += (N + (1 << tsh) - 1) >> tsh;
        sc.push_back(S);
    }
    g.projs = gg::dconst(pr.data(), pr.size());
    g.nprojs = np;
    em.map = gg::dconst(map.data(), map.size());
    em.bix = gg::dconst(bix.data(), bix.size());
    em.rows = gg::dconst(rows.data(), rows.size());
    em.ep = gg::dconst(ep.data(), ep.size());
    em.quads = quads.empty() ? nullptr : gg::dconst(quads.data(), quads.size());
    em.nep = np;
    em.sc = gg::dconst(sc.data(), sc.size());
    em.nsc = static_cast<int>(sc.size());
    if (!fused) {
        auto hc = hc_scratch(static_cast<size_t>(g.entries), g.N);
        g.HC = hc.first;
        g.CC = hc.second;
        g.BK = bank_scratch(rows.size(), g.N);
    }
    check_desc(g);
    const int64_t lanes = (g.N + gg::kTile - 1) / gg::kTile * gg::kTile;
    // multiple rows of the projections' input moduli (uniform-i key hashes) and of the bank rows' R offsets
    gg::Ctx cc = c;
    const bool iu = by_i;  // k_hash_iu writes the by-index layout k_emit then inverts
    em.by_i = by_i ? 1 : 0;
    em.fused = fused ? 1 : 0;
    {
        std::vector<int> mods;
        for (const auto& p : pr) mods.push_back(p.pin);
        for (const auto& r : rows)
            if (r.res < 0) mods.push_back(r.pout);
        std::sort(mods.begin(), mods.end());
        mods.erase(std::unique(mods.begin(), mods.end()), mods.end());
        if (gg::gg_hash_mode() != 0) cc.iR = ensure_iR(c, mods);
    }
    // (rejected, profiles/ab/README.md: one block per label group with the label staged in LDS, 7.2 -> 7.6-8.2 ms
    // per 4 GCs, and one wave per group stepping packed-byte payloads o + v*off incrementally, 10.7 ms)
    if (fused) DASH_CHECK(cc.iR != nullptr, "gpu garbler: fused emit without the offsets' multiple rows");
    if (!rows.empty() && !fused) {
        // bank jobs: neighbouring rows of one slot label with R offsets pair up (one label read, two payloads)
        std::vector<gg::BankJob> bj;
        const bool pairs = gg::gg_hash_mode() == 2;
        for (size_t r = 0; r < rows.size(); ++r) {
            const auto& a = rows[r];
            if (pairs && r + 1 < rows.size()) {
                const auto& b = rows[r + 1];
                if (a.res < 0 && b.res < 0 && a.slot == b.slot && a.pout == b.pout && a.pout < 32768) {
                    bj.push_back(gg::BankJob{static_cast<int>(r), static_cast<int>(r + 1)});
                    ++r;
                    continue;
                }
            }
            bj.push_back(gg::BankJob{static_cast<int>(r), -1});
        }
        const gg::BankJob* dbj = gg::dconst(bj.data(), bj.size());
        hipLaunchKernelGGL(gg::k_bank, dim3(blocks_for(lanes * static_cast<int64_t>(bj.size()), 256, 32768)), dim3(256), 0,
                           gg::tl_st, cc, g, in, em.rows, dbj, static_cast<int>(bj.size()));
    }
    if (fused) {
    } else if (iu) {
        std::vector<gg::HashJob> hj;
        for (int pi = 0; pi < np; ++pi)
            for (int c0 = 0; c0 < pr[pi].pin; c0 += gg::kHJ) hj.push_back(gg::HashJob{pi, c0});
        const gg::HashJob* dj = gg::dconst(hj.data(), hj.size());
        hipLaunchKernelGGL(gg::hash_iu_kernel(cc.hard != 0), dim3(blocks_for(lanes * static_cast<int64_t>(hj.size()), gg::kPB, 16384)),
                           dim3(gg::kPB), 0, gg::tl_st, cc, g, in, dj, static_cast<int>(hj.size()));
    } else if (gg::gg_hash_jobs()) {
        std::vector<gg::HashJob> hj;
        for (int pi = 0; pi < np; ++pi)
            for (int c0 = 0; c0 < pr[pi].pin; c0 += gg::kHJ) hj.push_back(gg::HashJob{pi, c0});
        const gg::HashJob* dj = gg::dconst(hj.data(), hj.size());
        hipLaunchKernelGGL(gg::hash_jobs_kernel(), dim3(blocks_for(lanes * static_cast<int64_t>(hj.size()), gg::kPB, 16384)),
                           dim3(gg::kPB), 0, gg::tl_st, c, g, in, dj, static_cast<int>(hj.size()));
    } else {
        hipLaunchKernelGGL(gg::hash_kernel(), dim3(blocks_for(lanes * g.entries, gg::kPB, 16384)), dim3(gg::kPB), 0,
                           gg::tl_st, c, g, in);
    }
    hipLaunchKernelGGL(gg::k_emit, dim3(static_cast<unsigned>(std::min<int64_t>(em.blocks, 65536))), dim3(gg::kEB),
                       lds_max, gg::tl_st, fused ? cc : c, g, in, tb, em);
}

void run_sign(const gg::Ctx& c, const gg::SignLayout& L, gg::Gadget& g, const gg::In& in, const gg::Tables& tb,
              const ProjFns& fx) {
    g.draws = gg::dconst(L.draws.data(), L.draws.size());
    g.ndraws = static_cast<int>(L.draws.size());
    g.projs = gg::dconst(L.projs.data(), L.projs.size());
    g.nprojs = static_cast<int>(L.projs.size());
    g.entries = L.entries;
    g.nblk = draw_blocks(L.draws);
    for (int d = 0; d < L.ss.t; ++d) g.mrs[d] = L.fan[d];
    check_desc(g);
    hipLaunchKernelGGL(gg::draw_kernel(), dim3(draw_grid(g)), dim3(gg::kGB), 0, gg::tl_st, c, g);
    hipLaunchKernelGGL(gg::k_sign_derive, dim3(blocks_for(g.N, 256), L.ss.t), dim3(256), 0, gg::tl_st, c, g, L.ss);
    project(c, g, in, tb, L.projs, fx);
    HIPCHECK(hipGetLastError());
}

// host labels whose authoritative copy is on the device: shape only
void set_stale(CrtLabels& cur, const std::vector<int>& mods, int64_t N) {
    cur.assign(mods.size(), Labels());
    for (size_t j = 0; j < mods.size(); ++j) {
        cur[j].p = mods[j];
        cur[j].n = nr_comps(mods[j]);
        cur[j].N = N;
    }
}
}  // namespace

namespace gg {
// End of a layer's launches. Everything of a GC runs in order on the null
// stream, so the next layer (and block reuse through the table cache) needs no
// host-device sync: the host prepares layer i+1 while the GPU runs layer i.
// Only temporary device allocations force a drain before they are freed;
// DASH_GG_SYNC=1 restores per-layer syncs (exact per-layer garbling timers).
inline void end_layer(std::vector<void*>& tmp) {
    static const bool sync = std::getenv("DASH_GG_SYNC") != nullptr;
    if (sync || !tmp.empty()) HIPCHECK(hipStreamSynchronize(tl_st));
    for (void* p : tmp) (void)hipFree(p);
    tmp.clear();
}
}  // namespace gg

// Per-device garbling context, shared by every GpuGarbler of the process: the non-blocking garbling stream,
// modulus constants and AES table, the pinned staging ring and the grow-only gadget scratch. A GpuGarbler
// holds the context's lock for its lifetime (one garbling per device at a time; concurrent GarbledCircuit
// constructions on one device queue up), so the per-GC setup is a few async copies: no allocation, no
// device-wide synchronization, nothing that would stall or serialize the evaluator's streams.
struct DevCtx {
    std::mutex m;
    int device = 0;
    hipStream_t st = nullptr;
    dev::ModC* mc = nullptr;
    int mc_max = 0;
    uint32_t* te0 = nullptr;
    // pinned staging + device ring for per-GC uploads (R, Z, shift labels), copied asynchronously on st
    static constexpr size_t kRing = 8u << 20;
    char* ring_h = nullptr;
    char* ring_d = nullptr;
    size_t ring_off = 0;
    // grow-only gadget scratch (label slots) and payload bank reused by every layer and GC
    int16_t* S = nullptr;
    size_t S_bytes = 0;
    u128* PB = nullptr;
    size_t PB_bytes = 0;
    void init(int dev) {
        device = dev;
        HIPCHECK(hipSetDevice(dev));
        HIPCHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&ring_h), kRing));
        HIPCHECK(hipMalloc(reinterpret_cast<void**>(&ring_d), kRing));
        auto te = make_te0();
        HIPCHECK(hipMalloc(reinterpret_cast<void**>(&te0), te.size() * sizeof(uint32_t)));
        HIPCHECK(hipMemcpy(te0, te.data(), te.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    // ModC table covering moduli up to max_mod (grows; rebuilt on the stream, waited for before reuse)
    const dev::ModC* modc(int max_mod) {
        if (max_mod > mc_max) {
            HIPCHECK(hipStreamSynchronize(st));  // earlier kernels may still read the old table
            if (mc) HIPCHECK(hipFree(mc));
            std::vector<dev::ModC> h(max_mod + 1);
            for (int q = 2; q <= max_mod; ++q) h[q] = make_modc(q);
            HIPCHECK(hipMalloc(reinterpret_cast<void**>(&mc), h.size() * sizeof(dev::ModC)));
            HIPCHECK(hipMemcpy(mc, h.data(), h.size() * sizeof(dev::ModC), hipMemcpyHostToDevice));
            mc_max = max_mod;
        }
        return mc;
    }
    template <class T>
    const T* stage(const T* h, size_t n) {
        const size_t bytes = (n * sizeof(T) + 255) / 256 * 256;
        DASH_CHECK(bytes <= kRing, "gpu garbler: staging ring too small");
        if (ring_off + bytes > kRing) {  // wrap: earlier copies must have landed before their staging is reused
            HIPCHECK(hipStreamSynchronize(st));
            ring_off = 0;
        }
        std::memcpy(ring_h + ring_off, h, n * sizeof(T));
        HIPCHECK(hipMemcpyAsync(ring_d + ring_off, ring_h + ring_off, n * sizeof(T), hipMemcpyHostToDevice, st));
        const T* d = reinterpret_cast<const T*>(ring_d + ring_off);
        ring_off += bytes;
        return d;
    }
    // pinned host buffer of the label hand-offs (to_device / to_host): DMA copies instead of the runtime's
    // chunked pageable staging (dozens of blit kernels per GC); grow-only, reused once the stream has drained
    char* pin_h = nullptr;
    size_t pin_bytes = 0;
    char* pinned(size_t bytes) {
        if (bytes > pin_bytes) {
            HIPCHECK(hipStreamSynchronize(st));
            if (pin_h) (void)hipHostFree(pin_h);
            HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&pin_h), bytes));
            pin_bytes = bytes;
        }
        return pin_h;
    }
    int16_t* scratch(size_t bytes) {
        if (bytes > S_bytes) {
            HIPCHECK(hipStreamSynchronize(st));
            if (S) (void)hipFree(S);
            HIPCHECK(hipMalloc(reinterpret_cast<void**>(&S), bytes));
            S_bytes = bytes;
        }
        return S;
    }
    u128* pbank(size_t rows, int64_t N) {
        const size_t bytes = std::max<size_t>(16, rows * static_cast<size_t>(N) * sizeof(u128));
        if (bytes > PB_bytes) {
            HIPCHECK(hipStreamSynchronize(st));
            if (PB) (void)hipFree(PB);
            HIPCHECK(hipMalloc(reinterpret_cast<void**>(&PB), bytes));
            PB_bytes = bytes;
        }
        return PB;
    }
    // bank payloads between k_bank and k_emit
    u128* BK = nullptr;
    size_t BK_n = 0;
    u128* bank(size_t rows, int64_t N) {
        const size_t n = std::max<size_t>(1, rows * static_cast<size_t>(N));
        if (n > BK_n) {
            HIPCHECK(hipStreamSynchronize(st));
            if (BK) (void)hipFree(BK);
            HIPCHECK(hipMalloc(reinterpret_cast<void**>(&BK), n * sizeof(u128)));
            BK_n = n;
        }
        return BK;
    }
    // multiple rows iR[p] of the current GC's offsets (k_iR): per-modulus grow-only buffers, valid for the
    // garbling generation that computed them (a new GpuGarbler = new offsets R = new generation)
    uint64_t iR_gen = 0;
    std::map<int, std::pair<uint32_t*, uint64_t>> iR_buf;  // p -> (buffer, generation)
    const uint32_t* const* iR_dev = nullptr;                // staged pointer table of the current generation
    bool iR_dirty = true;
    // key hashes / colors between k_hash and k_emit
    u128* HC = nullptr;
    uint16_t* CC = nullptr;
    size_t HC_n = 0;
    std::pair<u128*, uint16_t*> hc(size_t entries, int64_t N) {
        const size_t n = std::max<size_t>(1, entries * static_cast<size_t>(N));
        if (n > HC_n) {
            HIPCHECK(hipStreamSynchronize(st));
            if (HC) (void)hipFree(HC);
            if (CC) (void)hipFree(CC);
            HIPCHECK(hipMalloc(reinterpret_cast<void**>(&HC), n * sizeof(u128)));
            HIPCHECK(hipMalloc(reinterpret_cast<void**>(&CC), n * sizeof(uint16_t)));
            HC_n = n;
        }
        return {HC, CC};
    }
};
thread_local DevCtx* tl_dc = nullptr;  // the calling thread's garbling context (set by Impl::enter)
namespace {  // the same (translation-unit) anonymous namespace as its declaration above run_sign
std::pair<u128*, uint16_t*> hc_scratch(size_t entries, int64_t N) {
    DASH_CHECK(tl_dc != nullptr, "gpu garbler: no garbling context on this thread");
    return tl_dc->hc(entries, N);
}
u128* bank_scratch(size_t rows, int64_t N) {
    DASH_CHECK(tl_dc != nullptr, "gpu garbler: no garbling context on this thread");
    return tl_dc->bank(rows, N);
}
// the iR pointer table with rows for every modulus of `mods` (k_iR launches for those missing in this
// generation); moduli >= 32768 get none (their users keep the generic per-lane form)
const uint32_t* const* ensure_iR(const gg::Ctx& c, const std::vector<int>& mods) {
    DASH_CHECK(tl_dc != nullptr, "gpu garbler: no garbling context on this thread");
    DevCtx& d = *tl_dc;
    gg::IrArgs a{};
    auto flush = [&]() {
        if (!a.n) return;
        int64_t mx = 1;
        for (int i = 0; i < a.n; ++i) mx = std::max<int64_t>(mx, static_cast<int64_t>(a.j[i].p) * a.j[i].words);
        hipLaunchKernelGGL(gg::k_iR, dim3(blocks_for(mx, 256, 1024), a.n), dim3(256), 0, gg::tl_st, c, a);
        a.n = 0;
    };
    for (int p : mods) {
        if (p < 2 || p >= 32768 || p > d.mc_max) continue;
        auto& slot = d.iR_buf[p];
        if (slot.first && slot.second == d.iR_gen) continue;
        const int words = 4 * static_cast<int>(gg::chunks_of(nr_comps(p)));
        if (!slot.first) {
            HIPCHECK(hipStreamSynchronize(gg::tl_st));  // no kernel of this context may still hold the stage ring
            HIPCHECK(hipMalloc(reinterpret_cast<void**>(&slot.first), static_cast<size_t>(p) * words * sizeof(uint32_t)));
        }
        slot.second = d.iR_gen;
        d.iR_dirty = true;
        a.j[a.n++] = gg::IrJob{slot.first, p, words};
        if (a.n == gg::kMaxIr) flush();
    }
    flush();
    if (d.iR_dirty) {
        std::vector<const uint32_t*> tab(static_cast<size_t>(d.mc_max) + 1, nullptr);
        for (const auto& kv : d.iR_buf)
            if (kv.second.second == d.iR_gen && kv.first <= d.mc_max) tab[kv.first] = kv.second.first;
        d.iR_dev = d.stage(tab.data(), tab.size());
        d.iR_dirty = false;
    }
    return d.iR_dev;
}
}  // namespace
// A free garbling context of the device, locked for the caller: up to DASH_GG_CONTEXTS (default 8) per
// device, so that many garblings (threads, e.g. the serving engine's refill workers) run on their own streams
// at once and fill each other's launch gaps and latency stalls; one more waits for the first context.
std::unique_lock<std::mutex> acquire_ctx(int device, DevCtx*& out) {
    static std::mutex m;
    static auto* pools = new std::map<int, std::vector<DevCtx*>>();  // leaked: lives as long as the process
    static const size_t cap = [] {
        const char* e = std::getenv("DASH_GG_CONTEXTS");
        return static_cast<size_t>(std::max(1, e ? std::atoi(e) : 8));  // = the serving engine's 8 refill workers
    }();
    DevCtx* first = nullptr;
    {
        std::lock_guard<std::mutex> g(m);
        auto& pool = (*pools)[device];
        for (DevCtx* c : pool) {
            std::unique_lock<std::mutex> l(c->m, std::try_to_lock);
            if (l.owns_lock()) {
                out = c;
                return l;
            }
        }
        if (pool.size() < cap) {
            DevCtx* c = new DevCtx();
            c->init(device);
            pool.push_back(c);
            out = c;
            return std::unique_lock<std::mutex>(c->m);
        }
        first = pool.front();
    }
    out = first;
    return std::unique_lock<std::mutex>(first->m);  // every context busy: queue on the first one
}

struct GpuGarbler::Impl {
    DevCtx* dcp = nullptr;
    std::unique_lock<std::mutex> lock;
    DevCtx& dc;
    gg::Ctx c{};
    // device cur: per residue label-major [N][n_j]
    std::vector<DevBlock> cur;
    std::vector<int> cur_mod;
    int64_t cur_N = 0;
    int max_mod = 0;
    std::vector<int> crt;
    int k = 0;
    int device = 0;
    // approx-sign lookup (gen_approx_lookup: residue j's [p][t] at lut_off[j]) for the F_LUT bank rows
    std::vector<int16_t> lut;
    int lut_off[kMaxRes] = {};
    ProjFns lut_fns() const { return ProjFns{nullptr, nullptr, &lut, lut_off}; }
    // sign base labels a sign_last mixed-radix rescale leaves for the next ReLU ([N][kW], relu_mult)
    // the sign label a sign_last mixed-radix rescale leaves in its scratch slot sig_slot (scratch at sig_S)
    // for the next ReLU's relu_mult, which reuses that scratch in place (no copy out and back)
    int sig_slot = -1;
    int64_t sig_N = 0;
    const int16_t* sig_S = nullptr;
    // device copies of layer outputs that a later residual add or in_src layer reads (index = layer + 1)
    struct Saved {
        std::vector<DevBlock> L;
        std::vector<int> mods;
        int64_t N = 0;
    };
    std::map<size_t, Saved> saved;
    // max pool in progress: value slots [Nout][cnt] (output-major) of the current tree level
    std::vector<DevBlock> mp_V;
    int64_t mp_Nout = 0, mp_cnt = 0;
    explicit Impl(int dev) : lock(acquire_ctx(dev, dcp)), dc(*dcp), device(dev) {}
    template <class T>
    const T* stage(const T* h, size_t n) { return dc.stage(h, n); }
    int16_t* scratch(size_t bytes) { return dc.scratch(bytes); }
    u128* pbank(size_t rows, int64_t N) { return dc.pbank(rows, N); }
    std::vector<DevBlock> alloc_labels(const std::vector<int>& mods, int64_t N) {
        std::vector<DevBlock> v(mods.size());
        for (size_t j = 0; j < mods.size(); ++j)
            v[j].alloc(device, static_cast<size_t>(N) * gg::chunks_of(nr_comps(mods[j])) * gg::kCh * sizeof(int16_t));
        return v;
    }
    void check_cur(const CrtLabels& host) const {
        DASH_CHECK(host.size() == cur.size() && !host.empty() && host[0].N == cur_N,
                   "gpu garbler: device labels out of sync with the host garbler");
        for (size_t j = 0; j < host.size(); ++j) DASH_CHECK(host[j].p == cur_mod[j], "gpu garbler: modulus mismatch");
    }
    void enter() {
        bind_device(device, dc.st, "gpu garbler");  // also on garbling worker threads (one Impl per context)
        gg::tl_st = dc.st;
        tl_dc = &dc;
    }
    ~Impl() {
        // garble() returns with every table written; blocks released below are reused in stream order
        (void)hipStreamSynchronize(dc.st);
        cur.clear();
        (void)hipGetLastError();  // teardown errors are ignored: do not leave them for a later HIPCHECK
    }
};

GpuGarbler::GpuGarbler(const std::vector<int>& crt, const std::vector<int>& mrs, const std::string& seed16,
                       const LabelBank& R, const LabelBank& Z, int device, bool hardened)
    : impl_(new Impl(device)) {
    Impl& I = *impl_;
    I.enter();
    I.c.hard = hardened ? 1 : 0;
    I.crt = crt;
    I.k = static_cast<int>(crt.size());
    I.max_mod = R.max_mod;
    std::vector<int16_t> hR((R.max_mod + 1) * gg::kW, 0), hZ((R.max_mod + 1) * gg::kW, 0);
    for (int p = 2; p <= R.max_mod; ++p) {
        if (R.lab[p].empty()) continue;
        std::copy(R.lab[p].begin(), R.lab[p].end(), hR.begin() + p * gg::kW);
        std::copy(Z.lab[p].begin(), Z.lab[p].end(), hZ.begin() + p * gg::kW);
    }
    I.c.R = I.stage(hR.data(), hR.size());
    I.c.Z = I.stage(hZ.data(), hZ.size());
    I.c.mc = I.dc.modc(R.max_mod);
    I.c.te0 = I.dc.te0;
    ++I.dc.iR_gen;  // this GC's offsets R: every multiple row is recomputed on first use
    I.dc.iR_dirty = true;
    I.c.iR = nullptr;
    auto rk = round_key_words(reinterpret_cast<const uint8_t*>(seed16.data()));
    std::copy(rk.begin(), rk.end(), I.c.rk);
    if (!mrs.empty()) {
        auto lut = gen_approx_lookup(crt, mrs);
        for (int j = 0; j < I.k; ++j) {
            I.lut_off[j] = static_cast<int>(I.lut.size());
            I.lut.insert(I.lut.end(), lut[j].begin(), lut[j].end());
        }
    }
}

GpuGarbler::~GpuGarbler() {
    if (impl_) impl_->enter();
}

// Device labels are chunked component-major (gg::kCh): host label-major rows are transposed on the host
// around the (rare) host<->device hand-offs.
void GpuGarbler::to_device(const CrtLabels& cur) {
    Impl& I = *impl_;
    I.enter();
    DASH_CHECK(!cur.empty(), "gpu garbler: no labels");
    I.cur_mod.clear();
    for (const auto& l : cur) I.cur_mod.push_back(l.p);
    I.cur_N = cur[0].N;
    I.cur = I.alloc_labels(I.cur_mod, I.cur_N);
    // every residue transposed into one pinned block (the stream is idle: the previous hand-off synchronized
    // or the context was just acquired), one DMA copy per residue
    size_t total = 0;
    for (const auto& L : cur) total += static_cast<size_t>(gg::chunks_of(L.n)) * gg::kCh * L.N;
    int16_t* t = reinterpret_cast<int16_t*>(I.dc.pinned(std::max<size_t>(16, total * sizeof(int16_t))));
    for (size_t j = 0; j < cur.size(); ++j) {
        const Labels& L = cur[j];
        DASH_CHECK(L.c.size() == static_cast<size_t>(L.N) * L.n, "gpu garbler: host labels are stale");
        const size_t cnt = static_cast<size_t>(gg::chunks_of(L.n)) * gg::kCh * L.N;
        std::fill(t, t + cnt, int16_t(0));
        for (i64 e = 0; e < L.N; ++e)
            for (int q = 0; q < L.n; ++q)
                t[((static_cast<size_t>(q >> 3)) * L.N + e) * gg::kCh + (q & 7)] = L.c[static_cast<size_t>(e) * L.n + q];
        HIPCHECK(hipMemcpyAsync(I.cur[j].p, t, cnt * sizeof(int16_t), hipMemcpyHostToDevice, gg::tl_st));
        t += cnt;
    }
}

void GpuGarbler::to_host(CrtLabels& cur) {
    Impl& I = *impl_;
    I.enter();
    I.check_cur(cur);
    size_t total = 0;
    for (const auto& L : cur) total += static_cast<size_t>(L.N) * gg::chunks_of(L.n) * gg::kCh;
    // pinned(): a growth synchronizes the stream before the old block is freed (an earlier to_device's copies)
    int16_t* t0 = reinterpret_cast<int16_t*>(I.dc.pinned(std::max<size_t>(16, total * sizeof(int16_t))));
    int16_t* t = t0;
    for (size_t j = 0; j < cur.size(); ++j) {
        const size_t cnt = static_cast<size_t>(cur[j].N) * gg::chunks_of(cur[j].n) * gg::kCh;
        HIPCHECK(hipMemcpyAsync(t, I.cur[j].p, cnt * sizeof(int16_t), hipMemcpyDeviceToHost, gg::tl_st));
        t += cnt;
    }
    HIPCHECK(hipStreamSynchronize(gg::tl_st));
    t = t0;
    for (size_t j = 0; j < cur.size(); ++j) {
        Labels& L = cur[j];
        L.c.resize(static_cast<size_t>(L.N) * L.n);
        for (i64 e = 0; e < L.N; ++e)
            for (int q = 0; q < L.n; ++q)
                L.c[static_cast<size_t>(e) * L.n + q] = t[((static_cast<size_t>(q >> 3)) * L.N + e) * gg::kCh + (q & 7)];
        t += static_cast<size_t>(L.N) * gg::chunks_of(L.n) * gg::kCh;
    }
}

namespace {
struct ConvPlanKey {
    int dev;
    uint64_t wh;
    std::vector<i64> geom;
    std::vector<int> mods;
    bool operator<(const ConvPlanKey& o) const {
        return std::tie(dev, wh, geom, mods) < std::tie(o.dev, o.wh, o.geom, o.mods);
    }
};
// prepared MFMA conv arguments (weights images, zero counts, zero bias rows in device memory), per process
std::map<ConvPlanKey, dev::ConvArgs>& conv_plans() {
    static auto* m = new std::map<ConvPlanKey, dev::ConvArgs>();  // leaked: device buffers live as long as the process
    return *m;
}
std::mutex& conv_plans_mutex() {
    static std::mutex m;
    return m;
}
}  // namespace

// Conv base labels = the evaluator's garbled conv applied to the zero labels:
// y = W x + (#zero weights + 1) Z (the +1 is the bias label's Z_p, the bias
// itself being public), through the same int8 MFMA implicit-GEMM kernel
// (launch_conv, one launch for all residues). The garbler's chunked labels
// are unchunked into the kernel's component-major byte activations and its
// output chunked back (one launch each for all residues). The public per-layer setup
// (centered int8 weight images, zero counts, all-zero bias rows) is built
// once per process and looked up by a hash of the weights.
void GpuGarbler::conv(const ConvGeom& G, const i64* w, size_t nw, uint64_t wh, CrtLabels& cur) {
    Impl& I = *impl_;
    I.enter();
    I.check_cur(cur);
    PhaseTrace tr_("conv");
    const int K = static_cast<int>(G.K());
    const int F = static_cast<int>(G.F);
    DASH_CHECK(static_cast<i64>(nw) == G.F * G.K(), "gpu garbler: conv weight shape");
    DASH_CHECK(G.C * G.H * G.W == I.cur_N, "gpu garbler: conv input size mismatch");
    DASH_CHECK(static_cast<int>(I.cur_mod.size()) <= kMaxRes, "gpu garbler: too many residues");
    std::vector<int> mods = I.cur_mod;
    const int64_t Nin = I.cur_N, Nout = G.out_size();
    std::vector<DevBlock> out = I.alloc_labels(mods, Nout);
    dev::ConvArgs a{};
    {
        ConvPlanKey key{I.device, wh, {G.C, G.H, G.W, G.F, G.kh, G.kw, G.sh, G.sw, G.ph, G.pw}, mods};
        std::lock_guard<std::mutex> lk(conv_plans_mutex());
        auto it = conv_plans().find(key);
        if (it != conv_plans().end()) {
            a = it->second;
        } else {
            a.crt.k = static_cast<int>(mods.size());
            for (int j = 0; j < a.crt.k; ++j) {
                a.crt.p[j] = mods[j];
                a.crt.n[j] = nr_comps(mods[j]);
                a.crt.prefix[j] = a.crt.sum;
                a.crt.sum += mods[j];
            }
            a.C = static_cast<int>(G.C); a.H = static_cast<int>(G.H); a.W = static_cast<int>(G.W);
            a.F = F; a.kh = static_cast<int>(G.kh); a.kw = static_cast<int>(G.kw);
            a.sh = static_cast<int>(G.sh); a.sw = static_cast<int>(G.sw);
            a.ph = static_cast<int>(G.ph); a.pw = static_cast<int>(G.pw);
            a.OH = static_cast<int>(G.OH); a.OW = static_cast<int>(G.OW);
            a.Kpad = (K + 63) / 64 * 64;
            a.use_mfma = 1;
            int max_p = 0;
            for (int j = 0; j < a.crt.k; ++j) max_p = std::max(max_p, mods[j]);
            dev::conv_plan(a, max_p, true);
            a.lab_stride = 0;
            a.img_off[0] = 0;
            for (int j = 0; j < a.crt.k; ++j) {
                const int p = mods[j], n = a.crt.n[j];
                DASH_CHECK(p <= dev::kActMaxModulus, "gpu garbler: conv residue modulus above 255");
                a.lab_off[j] = p * gg::kW;
                a.img_off[j + 1] = a.img_off[j] + n;
                std::vector<int16_t> wm(static_cast<size_t>(F) * K);
                std::vector<int8_t> w8(static_cast<size_t>(F) * a.Kpad, 0);
                std::vector<int32_t> zc(F, 1);
                for (int f = 0; f < F; ++f)
                    for (int q = 0; q < K; ++q) {
                        const int v = static_cast<int>(w[static_cast<size_t>(f) * K + q] % p);
                        wm[static_cast<size_t>(f) * K + q] = static_cast<int16_t>(v);
                        if (v == 0) ++zc[f];
                        w8[static_cast<size_t>(f) * a.Kpad + q] = static_cast<int8_t>(v > p / 2 ? v - p : v);
                    }
                a.w[j] = gg::dconst(wm.data(), wm.size());
                a.zc[j] = gg::dconst(zc.data(), zc.size());
                std::vector<int16_t> zb(static_cast<size_t>(F) * n, 0);
                a.bias[j] = gg::dconst(zb.data(), zb.size());
                a.w8[j] = nullptr;
                a.w8r[j] = nullptr;
                if (a.nbands > 0) {
                    const std::vector<int8_t> w8r = dev::conv_w8r(a, w8, F);
                    a.w8r[j] = gg::dconst(w8r.data(), w8r.size());
                } else {
                    a.w8[j] = gg::dconst(w8.data(), w8.size());
                }
            }
            conv_plans().emplace(std::move(key), a);
        }
    }
    a.zero = I.c.Z;  // this GC's zero labels: component c of residue j at Z[p_j * kW + c]
    // chunked int16 labels <-> the kernel's component-major byte activations
    std::vector<DevBlock> xin(mods.size()), yout(mods.size());
    dev::Act x{}, y{};
    x.N = Nin;
    y.N = Nout;
    dev::TrRes ti{}, to{};
    ti.k = to.k = a.crt.k;
    for (int j = 0; j < a.crt.k; ++j) {
        const int n = a.crt.n[j];
        xin[j].alloc(I.device, static_cast<size_t>(Nin) * n);
        yout[j].alloc(I.device, static_cast<size_t>(Nout) * n);
        ti.in[j] = I.cur[j].as<int16_t>();
        ti.out[j] = xin[j].as<dev::act_t>();
        ti.rows[j] = n;
        ti.cols[j] = Nin;
        to.in[j] = yout[j].as<dev::act_t>();
        to.out[j] = out[j].as<int16_t>();
        to.rows[j] = n;
        to.cols[j] = Nout;
        x.p[j] = xin[j].as<dev::act_t>();
        y.p[j] = yout[j].as<dev::act_t>();
    }
    dev::launch_unchunk_to_act_res(ti, gg::tl_st);  // all residues in one launch
    dev::launch_conv(a, x, y, 1, gg::tl_st);
    dev::launch_chunk_from_act_res(to, gg::tl_st);
    // xin / yout return to the block cache; later users are ordered behind these kernels on the stream
    HIPCHECK(hipGetLastError());
    std::vector<void*> tmp;
    gg::end_layer(tmp);
    tr_.mark("kernels");
    I.cur = std::move(out);
    I.cur_N = Nout;
    set_stale(cur, mods, I.cur_N);
}

// Sign gadget (+ the ReLU's mixed-modulus half gates when prefix/mmg/mme are set) over N elements whose input
// labels are `in`: PRG streams (layer, sslot_s) for the sign and (layer, sslot_m) for the half gates. Returns
// the output base labels (out_mod of the plan, or the CRT base for a ReLU). Shared by Sign, ReLU and every
// level of a max pool (relu_garble_elem with its own stream slots).
static std::vector<DevBlock> sign_core(GpuGarbler::Impl& I, uint64_t layer, uint64_t sslot_s, uint64_t sslot_m,
                                       const SignPlan& sp, const gg::In& in, int64_t N, Array& ap, Array& c1,
                                       Array& c2, Array& sg, const std::vector<i64>* prefix, Array* mmg, Array* mme,
                                       std::vector<int>& omods) {
    const int k = I.k;
    const bool relu = prefix != nullptr;
    // relu: 2 slots per residue for the mixed-mult output labels sk03/sk04
    gg::SignLayout L = gg::sign_layout(sp, relu ? 2 * k : 0);
    int sk0 = L.nslots - (relu ? 2 * k : 0);
    int16_t* S = I.scratch(static_cast<size_t>(N) * L.nslots * gg::kW * sizeof(int16_t));
    DevTable tA, t1, t2, tS, tG, tE;
    tA.alloc(I.device, N, ap.shape[1], ap);
    if (sp.has_cast1()) t1.alloc(I.device, N, c1.shape[1], c1);
    t2.alloc(I.device, N, c2.shape[1], c2);
    tS.alloc(I.device, N, sg.shape[1], sg);
    gg::Tables tb{};
    tb.t[0] = tA.p(); tb.row[0] = tA.row;
    tb.t[1] = t1.p(); tb.row[1] = t1.row;
    tb.t[2] = t2.p(); tb.row[2] = t2.row;
    tb.t[3] = tS.p(); tb.row[3] = tS.row;
    if (relu) {
        tG.alloc(I.device, N, mmg->shape[1], *mmg);
        tE.alloc(I.device, N, static_cast<int64_t>(k) * 3, *mme, true);
        tb.t[4] = tG.p(); tb.row[4] = tG.row;
        tb.t[5] = tE.p(); tb.row[5] = tE.row;
    }
    gg::Gadget g{};
    g.layer = layer;
    g.sslot = sslot_s;
    g.mask = 0;
    g.S = S;
    g.PB = I.pbank(2, N);
    g.N = N;
    g.nslots = L.nslots;
    run_sign(I.c, L, g, in, tb, I.lut_fns());
    omods = relu ? I.crt : sp.out_mod;
    std::vector<DevBlock> out = I.alloc_labels(omods, N);
    if (relu) {
        // mixed-mult draws (stream slot sslot_m, counters run over the residues) and the g/e projections
        std::vector<gg::Draw> dr;
        std::vector<gg::Proj> pr;
        int ctr = 0;
        int64_t first = 0;
        for (int j = 0; j < k; ++j) {
            const int p = I.crt[j];
            dr.push_back({sk0 + 2 * j, p, ctr});
            ctr += prg_blocks(p);
            dr.push_back({sk0 + 2 * j + 1, p, ctr});
            ctr += prg_blocks(p);
        }
        for (int j = 0; j < k; ++j) {
            const int p = I.crt[j];
            gg::Proj a{gg::S_INPUT, j, p, sk0 + 2 * j, p, gg::F_MULR, j, 0, 0, gg::R_BANK, 0, 4, 1, (*prefix)[j], first};
            a.hsub = tw_sub(kTwMmg, static_cast<uint32_t>(j));
            first += p;
            pr.push_back(a);
        }
        for (int j = 0; j < k; ++j) {
            const int p = I.crt[j];
            gg::Proj b{gg::S_SLOT, L.out_slot0, 2, sk0 + 2 * j + 1, p, gg::F_NEGR, j, 0, 0, gg::R_INPUT, j, 5, 1,
                       static_cast<int64_t>(j) * 3, first};
            b.hsub = tw_sub(kTwMmy, 0);  // the sign label's y row, slot j
            b.hslot = j;
            first += 2;
            pr.push_back(b);
        }
        // the e table row is [k][3]: projection entries land at j*3 + color
        gg::Gadget gm = g;
        gm.sslot = sslot_m;
        gm.draws = gg::dconst(dr.data(), dr.size());
        gm.ndraws = static_cast<int>(dr.size());
        gm.projs = gg::dconst(pr.data(), pr.size());
        gm.nprojs = static_cast<int>(pr.size());
        gm.entries = first;
        gm.nblk = draw_blocks(dr);
        check_desc(gm);
        hipLaunchKernelGGL(gg::draw_kernel(), dim3(draw_grid(gm)), dim3(gg::kGB), 0, gg::tl_st, I.c, gm);
        project(I.c, gm, in, tb, pr);
        gg::MiniArgs ma{};
        ma.k = k;
        for (int j = 0; j < k; ++j) ma.crt[j] = I.crt[j];
        ma.sig_slot = L.out_slot0;
        ma.sk_slot0 = sk0;
        for (int j = 0; j < k; ++j) ma.out[j] = out[j].as<int16_t>();
        // the sign gadget's payload bank (>= 2 rows, its readers are done: same stream) now holds the two
        // mini-gate key hashes of the sign output
        hipLaunchKernelGGL(gg::k_bin_keys, dim3(blocks_for(N, gg::kGB, 8192)), dim3(gg::kGB), 0, gg::tl_st, I.c,
                           static_cast<const int16_t*>(gg::slot_base(g, L.out_slot0)),
                           static_cast<const int16_t*>(nullptr), g.PB, N);
        hipLaunchKernelGGL(gg::k_relu_finish, dim3(blocks_for(N, 256, 4096), k), dim3(256), 0, gg::tl_st, I.c, gm, in,
                           tb, ma, static_cast<const u128*>(g.PB));
        tG.to_array(*mmg, I.device);
        tE.to_array(*mme, I.device);
    } else {
        // sign layer outputs: out0[o] slots (one per output residue) are already component-major [n][N] blocks
        for (size_t o = 0; o < omods.size(); ++o)
            HIPCHECK(hipMemcpyAsync(out[o].p, gg::slot_base(g, L.out_slot0 + static_cast<int>(o)),
                                    static_cast<size_t>(gg::chunks_of(nr_comps(omods[o]))) * gg::kCh * N * sizeof(int16_t),
                                    hipMemcpyDeviceToDevice, gg::tl_st));
    }
    HIPCHECK(hipGetLastError());
    tA.to_array(ap, I.device);
    if (sp.has_cast1()) t1.to_array(c1, I.device);
    t2.to_array(c2, I.device);
    tS.to_array(sg, I.device);
    return out;
}

// chunked label set of N elements as a projection / derive input
static gg::In labels_in(const std::vector<DevBlock>& L, const std::vector<int>& mods, int64_t N) {
    gg::In in{};
    for (size_t j = 0; j < L.size(); ++j) {
        in.p[j] = L[j].as<int16_t>();
        in.n[j] = nr_comps(mods[j]);
        in.es[j] = gg::kCh;
        in.cs[j] = N * gg::kCh;
    }
    return in;
}

void GpuGarbler::sign_layer(uint64_t layer, const SignPlan& sp, CrtLabels& cur, Array& ap, Array& c1, Array& c2,
                            Array& sg, const std::vector<int>* relu_crt, const std::vector<i64>* prefix, Array* mmg,
                            Array* mme) {
    Impl& I = *impl_;
    I.enter();
    I.check_cur(cur);
    PhaseTrace tr_(relu_crt ? "relu" : "sign");
    const int64_t N = I.cur_N;
    std::vector<void*> tmp;
    std::vector<int> omods;
    std::vector<DevBlock> out = sign_core(I, layer, 1, 2, sp, labels_in(I.cur, I.crt, N), N, ap, c1, c2, sg,
                                          relu_crt ? prefix : nullptr, mmg, mme, omods);
    gg::end_layer(tmp);
    tr_.mark("kernels");
    I.cur = std::move(out);
    I.cur_mod = omods;
    set_stale(cur, omods, N);
}

void GpuGarbler::rescale_legacy_iter(uint64_t layer, int it, const RescalePlan& P, CrtLabels& cur,
                                     const std::vector<std::vector<comp_t>>& up,
                                     const std::vector<std::vector<comp_t>>& down, Array& tr, Array& ap, Array& c1,
                                     Array& c2, Array& sg) {
    Impl& I = *impl_;
    I.enter();
    I.check_cur(cur);
    PhaseTrace tr_("rescale_iter");
    const int64_t N = I.cur_N;
    const int k = I.k;
    std::vector<void*> tmp;
    std::vector<int16_t> hup(k * gg::kW, 0), hdn(k * gg::kW, 0);
    for (int j = 0; j < k; ++j) {
        std::copy(up[j].begin(), up[j].end(), hup.begin() + j * gg::kW);
        std::copy(down[j].begin(), down[j].end(), hdn.begin() + j * gg::kW);
    }
    gg::RsArgs ra{};
    ra.k = k;
    for (int j = 0; j < k; ++j) {
        ra.crt[j] = I.crt[j];
        ra.L[j] = I.cur[j].as<int16_t>();
        ra.inv[j] = 0;
    }
    // inverses of 2 for the active residues (plan order = residues 1..k-1)
    for (size_t a = 0; a < P.active[0].size(); ++a) ra.inv[P.active[0][a]] = static_cast<int>(P.inv[0][a]);
    ra.up = I.stage(hup.data(), hup.size());
    ra.down = I.stage(hdn.data(), hdn.size());
    ra.layer = layer;
    ra.sslot = 10 + it;
    DevTable tT, tA, t1, t2, tS;
    tT.alloc(I.device, N, tr.shape[1], tr);
    tA.alloc(I.device, N, ap.shape[1], ap);
    if (P.sign.has_cast1()) t1.alloc(I.device, N, c1.shape[1], c1);
    t2.alloc(I.device, N, c2.shape[1], c2);
    tS.alloc(I.device, N, sg.shape[1], sg);
    gg::Tables tb{};
    tb.t[0] = tA.p(); tb.row[0] = tA.row;
    tb.t[1] = t1.p(); tb.row[1] = t1.row;
    tb.t[2] = t2.p(); tb.row[2] = t2.row;
    tb.t[3] = tS.p(); tb.row[3] = tS.row;
    tb.t[6] = tT.p(); tb.row[6] = tT.row;
    tr_.mark("alloc");
    for (int j = 1, ctr = 0; j < k; ++j) {
        ra.ctr[j] = ctr;
        ctr += prg_blocks(I.crt[j]);
    }
    gg::SignLayout L = gg::sign_layout(P.sign, 0);
    // rows 0-1: the trans key hashes (k_bin_keys -> k_rescale_pre)
    u128* PB = I.pbank(2, N);
    hipLaunchKernelGGL(gg::k_bin_keys, dim3(blocks_for(N, gg::kGB, 8192)), dim3(gg::kGB), 0, gg::tl_st, I.c,
                       static_cast<const int16_t*>(ra.L[0]), ra.up, PB, N);
    hipLaunchKernelGGL(gg::k_rescale_pre, dim3(blocks_for(N, gg::kGB, 2048), k - 1), dim3(gg::kGB), 0, gg::tl_st, I.c,
                       ra, tb, PB, N);
    int16_t* S = I.scratch(static_cast<size_t>(N) * L.nslots * gg::kW * sizeof(int16_t));
    gg::In in{};
    for (int j = 0; j < k; ++j) {
        in.p[j] = I.cur[j].as<int16_t>();
        in.n[j] = nr_comps(I.crt[j]);
        in.es[j] = gg::kCh;  // chunked component-major
        in.cs[j] = N * gg::kCh;
    }
    DASH_CHECK(I.crt[0] == 2, "gpu garbler: legacy rescale needs residue 0 = 2");
    in.p[0] = I.c.Z + 2 * gg::kW;  // residue 0 is Z_2 for every element (zero element stride)
    in.es[0] = 0;
    in.cs[0] = gg::kCh;
    gg::Gadget g{};
    g.layer = layer;
    g.sslot = 10 + it;
    g.mask = 1ull << 43;  // nested sign stream (rescale_garble_elem)
    g.S = S;
    g.PB = I.pbank(2, N);
    g.N = N;
    g.nslots = L.nslots;
    run_sign(I.c, L, g, in, tb, I.lut_fns());
    hipLaunchKernelGGL(gg::k_rescale_post_g, dim3(blocks_for(N * 128, 256, 4096), k), dim3(256), 0, gg::tl_st, I.c, ra,
                       g, L.out_slot0);
    HIPCHECK(hipGetLastError());
    gg::end_layer(tmp);
    tr_.mark("kernels");
    tT.to_array(tr, I.device);
    tA.to_array(ap, I.device);
    if (P.sign.has_cast1()) t1.to_array(c1, I.device);
    t2.to_array(c2, I.device);
    tS.to_array(sg, I.device);
    set_stale(cur, I.cur_mod, N);
}

// ReLU mixed-modulus half gates out_j = x_j * sig (relu_garble_elem's mixed_mult_garble order): draws of the
// sk03/sk04 labels (slots sk0 + 2j, + 1) on PRG stream 2 of g.layer, the g (F_MULR) and e (F_NEGR) projections
// into tables 4 / 5, the mini payloads and output base labels. g.S holds the sign label at sig_slot.
static std::vector<DevBlock> relu_mult_gates(GpuGarbler::Impl& I, const gg::Gadget& g, const gg::In& in,
                                             gg::Tables& tb, int sig_slot, int sk0, const std::vector<i64>& prefix) {
    const int64_t N = g.N;
    const int k = I.k;
    std::vector<DevBlock> out = I.alloc_labels(I.crt, N);
    std::vector<gg::Draw> dm;
    std::vector<gg::Proj> pm;
    int c2 = 0;
    int64_t f2 = 0;
    for (int j = 0; j < k; ++j) {
        const int p = I.crt[j], n = nr_comps(p);
        dm.push_back({sk0 + 2 * j, p, c2});
        c2 += prg_blocks(p);
        dm.push_back({sk0 + 2 * j + 1, p, c2});
        c2 += prg_blocks(p);
    }
    for (int j = 0; j < k; ++j) {
        const int p = I.crt[j];
        gg::Proj q{gg::S_INPUT, j, p, sk0 + 2 * j, p, gg::F_MULR, j, 0, 0, gg::R_BANK, 0, 4, 1, prefix[j], f2};
        q.hsub = tw_sub(kTwMmg, static_cast<uint32_t>(j));
        f2 += p;
        pm.push_back(q);
    }
    for (int j = 0; j < k; ++j) {
        const int p = I.crt[j];
        gg::Proj q{gg::S_SLOT, sig_slot, 2, sk0 + 2 * j + 1, p, gg::F_NEGR, j, 0, 0, gg::R_INPUT, j, 5, 1,
                   static_cast<int64_t>(j) * 3, f2};
        q.hsub = tw_sub(kTwMmy, 0);
        q.hslot = j;
        f2 += 2;
        pm.push_back(q);
    }
    gg::Gadget gm = g;
    gm.sslot = 2;
    gm.PB = I.pbank(2, N);
    gm.draws = gg::dconst(dm.data(), dm.size());
    gm.ndraws = static_cast<int>(dm.size());
    gm.projs = gg::dconst(pm.data(), pm.size());
    gm.nprojs = static_cast<int>(pm.size());
    gm.entries = f2;
    gm.nblk = draw_blocks(dm);
    check_desc(gm);
    hipLaunchKernelGGL(gg::draw_kernel(), dim3(draw_grid(gm)), dim3(gg::kGB), 0, gg::tl_st, I.c, gm);
    project(I.c, gm, in, tb, pm);
    gg::MiniArgs ma{};
    ma.k = k;
    for (int j = 0; j < k; ++j) ma.crt[j] = I.crt[j];
    ma.sig_slot = sig_slot;
    ma.sk_slot0 = sk0;
    for (int j = 0; j < k; ++j) ma.out[j] = out[j].as<int16_t>();
    hipLaunchKernelGGL(gg::k_bin_keys, dim3(blocks_for(N, gg::kGB, 8192)), dim3(gg::kGB), 0, gg::tl_st, I.c,
                       static_cast<const int16_t*>(gg::slot_base(g, sig_slot)), static_cast<const int16_t*>(nullptr),
                       gm.PB, N);
    hipLaunchKernelGGL(gg::k_relu_finish, dim3(blocks_for(N, 256, 4096), k), dim3(256), 0, gg::tl_st, I.c, gm, in,
                       tb, ma, static_cast<const u128*>(gm.PB));
    return out;
}

// ReLU with the mixed-radix sign: draw the digit-target labels (sign_mrs_garble_elem order) -> keys ->
// fan-out projections; residue 0's key slot is the sign label; then the mixed-modulus half gates exactly as
// in sign_layer's ReLU branch.
void GpuGarbler::relu_mrs(uint64_t layer, const SignMrsPlan& P, CrtLabels& cur, Array& tab,
                          const std::vector<int>* relu_crt, const std::vector<i64>* prefix, Array& mmg, Array& mme) {
    Impl& I = *impl_;
    I.enter();
    I.check_cur(cur);
    PhaseTrace tr_("relu_mrs");
    (void)relu_crt;
    const int64_t N = I.cur_N;
    const int k = I.k;
    DASH_CHECK(P.k() == k, "gpu garbler: mixed-radix sign plan mismatch");
    std::vector<gg::Draw> dr;
    std::vector<gg::Proj> pr;
    std::vector<int> fan;
    std::vector<int16_t> flut;
    gg::MrsSG a{};
    a.k = k;
    int slot = 0, ctr = 0;
    std::vector<int> dig0(k, 0);
    for (int i = 0; i + 1 < k; ++i) {
        dig0[i] = slot;
        for (int t = 0; t < P.targets(i); ++t) {
            const int r = P.target_res(i, t);
            a.sub[r][a.nsub[r]++] = slot;
            dr.push_back({slot++, P.crt[r], ctr});
            ctr += prg_blocks(P.crt[r]);
        }
    }
    a.key0 = slot;
    slot += k;
    const int sig_slot = a.key0 + P.ord[k - 1];
    const int sk0 = slot;
    slot += 2 * k;
    const int nslots = slot;
    int64_t first = 0;
    for (int i = 0; i + 1 < k; ++i) {
        const int nt = P.targets(i), r0 = P.ord[i];
        const int a0 = static_cast<int>(flut.size()), a1 = static_cast<int>(fan.size());
        for (int v = 0; v < P.crt[r0]; ++v)
            for (int t = 0; t < nt; ++t) flut.push_back(static_cast<int16_t>(P.digit_fn(i, t, v)));
        for (int t = 0; t < nt; ++t) fan.push_back(P.crt[P.target_res(i, t)]);
        gg::Proj p{};
        p.in_kind = gg::S_SLOT; p.in_idx = a.key0 + r0; p.pin = P.crt[r0];
        p.out_slot = dig0[i]; p.pout = P.crt[P.target_res(i, 0)]; p.fn = gg::F_FAN; p.a0 = a0; p.a1 = a1;
        p.outr_kind = gg::R_BANK; p.table = 0; p.stride = nt; p.off = P.dig_off[i]; p.first = first;
        p.hsub = tw_sub(kTwSmrs, static_cast<uint32_t>(i));
        first += P.crt[r0];
        pr.push_back(p);
    }
    for (int j = 0; j < k; ++j) a.crt[j] = P.crt[j];
    DevTable tT, tG, tE;
    tT.alloc(I.device, N, tab.shape[1], tab);
    tG.alloc(I.device, N, mmg.shape[1], mmg);
    tE.alloc(I.device, N, static_cast<int64_t>(k) * 3, mme, true);
    gg::Tables tb{};
    tb.t[0] = tT.p(); tb.row[0] = tT.row;
    tb.t[4] = tG.p(); tb.row[4] = tG.row;
    tb.t[5] = tE.p(); tb.row[5] = tE.row;
    gg::In in{};
    for (int j = 0; j < k; ++j) {
        in.p[j] = I.cur[j].as<int16_t>();
        in.n[j] = nr_comps(I.crt[j]);
        in.es[j] = gg::kCh;  // chunked component-major
        in.cs[j] = N * gg::kCh;
    }
    gg::Gadget g{};
    g.layer = layer;
    g.sslot = 1;
    g.mask = 0;
    g.S = I.scratch(static_cast<size_t>(N) * nslots * gg::kW * sizeof(int16_t));
    g.PB = I.pbank(2, N);
    g.N = N;
    g.nslots = nslots;
    g.draws = gg::dconst(dr.data(), dr.size());
    g.ndraws = static_cast<int>(dr.size());
    g.projs = gg::dconst(pr.data(), pr.size());
    g.nprojs = static_cast<int>(pr.size());
    g.entries = first;
    g.nblk = draw_blocks(dr);

    check_desc(g);
    std::vector<void*> tmp;
    hipLaunchKernelGGL(gg::draw_kernel(), dim3(draw_grid(g)), dim3(gg::kGB), 0, gg::tl_st, I.c, g);
    hipLaunchKernelGGL(gg::k_mrs_sign_derive, dim3(blocks_for(N, 256), k), dim3(256), 0, gg::tl_st, I.c, g, in, a);
    project(I.c, g, in, tb, pr, ProjFns{&flut, &fan});
    // mixed-modulus half gates (as sign_layer's ReLU branch, sign label = residue 0's key slot)
    std::vector<DevBlock> out = relu_mult_gates(I, g, in, tb, sig_slot, sk0, *prefix);
    HIPCHECK(hipGetLastError());
    gg::end_layer(tmp);
    tr_.mark("kernels");
    tT.to_array(tab, I.device);
    tG.to_array(mmg, I.device);
    tE.to_array(mme, I.device);
    I.cur = std::move(out);
    set_stale(cur, I.crt, N);
}

// Mixed-radix rescale: draw (digit-target labels, then the k final labels, in
// rescale_mrs_garble_elem's PRG order) -> derive keys / outputs -> fan-out
// projections (one per digit, one final).
void GpuGarbler::rescale_mrs(uint64_t layer, const RescaleMrsPlan& P, CrtLabels& cur, Array& tab) {
    Impl& I = *impl_;
    I.enter();
    I.check_cur(cur);
    PhaseTrace tr_("rescale_mrs");
    const int64_t N = I.cur_N;
    const int k = I.k;
    DASH_CHECK(P.k() == k && static_cast<int>(P.T) <= I.max_mod, "gpu garbler: mixed-radix rescale plan mismatch");
    std::vector<gg::Draw> dr;
    std::vector<gg::Proj> pr;
    std::vector<int> fan;
    std::vector<int16_t> flut;
    gg::MrsG a{};
    a.k = k;
    a.T = static_cast<int>(P.T);
    int slot = 0, ctr = 0;
    std::vector<int> dig0(k, 0);
    for (int i = 0; i < k; ++i) {
        dig0[i] = slot;
        for (int t = 0; t < P.targets(i); ++t) {
            const int q = P.target_mod(i, t);
            if (t == k - 1 - i) {
                a.tslot[i] = slot;
            } else {
                const int r = P.target_res(i, t);
                a.sub[r][a.nsub[r]++] = slot;
            }
            dr.push_back({slot++, q, ctr});
            ctr += prg_blocks(q);
        }
    }
    a.fin0 = slot;
    for (int j = 0; j < k; ++j) {
        dr.push_back({slot++, P.crt[j], ctr});
        ctr += prg_blocks(P.crt[j]);
    }
    a.key0 = slot;
    slot += k;
    a.acc = slot++;
    const int nslots = slot;
    int64_t first = 0;
    for (int i = 0; i < k; ++i) {
        const int nt = P.targets(i), r0 = P.ord[i];
        const int a0 = static_cast<int>(flut.size()), a1 = static_cast<int>(fan.size());
        for (int v = 0; v < P.crt[r0]; ++v)
            for (int t = 0; t < nt; ++t) flut.push_back(static_cast<int16_t>(P.digit_fn(i, t, v)));
        for (int t = 0; t < nt; ++t) fan.push_back(P.target_mod(i, t));
        gg::Proj p{};
        p.in_kind = gg::S_SLOT; p.in_idx = a.key0 + r0; p.pin = P.crt[r0];
        p.out_slot = dig0[i]; p.pout = P.target_mod(i, 0); p.fn = gg::F_FAN; p.a0 = a0; p.a1 = a1;
        p.outr_kind = gg::R_BANK; p.table = 0; p.stride = nt; p.off = P.dig_off[i]; p.first = first;
        p.hsub = tw_sub(kTwMrs, static_cast<uint32_t>(i));
        first += P.crt[r0];
        pr.push_back(p);
    }
    {
        const int a0 = static_cast<int>(flut.size()), a1 = static_cast<int>(fan.size());
        for (int v = 0; v < P.T; ++v)
            for (int j = 0; j < k; ++j) flut.push_back(static_cast<int16_t>(P.final_fn(j, v)));
        for (int j = 0; j < k; ++j) fan.push_back(P.crt[j]);
        // T entries but only p_j distinct payloads per target j (k_emit's bank rows)
        gg::Proj p{};
        p.in_kind = gg::S_SLOT; p.in_idx = a.acc; p.pin = static_cast<int>(P.T);
        p.out_slot = a.fin0; p.pout = P.crt[0]; p.fn = gg::F_FAN; p.a0 = a0; p.a1 = a1;
        p.outr_kind = gg::R_BANK; p.table = 0; p.stride = k; p.off = P.fin_off; p.first = first;
        p.hsub = tw_sub(kTwMrs, static_cast<uint32_t>(k));
        first += P.T;
        pr.push_back(p);
    }
    for (int j = 0; j < k; ++j) {
        a.crt[j] = P.crt[j];
        a.sinv[j] = static_cast<int>(P.Sinv[j]);
        a.L[j] = I.cur[j].as<int16_t>();
    }
    DevTable tT;
    tT.alloc(I.device, N, P.n_tab, tab);
    gg::Tables tb{};
    tb.t[0] = tT.p();
    tb.row[0] = tT.row;
    gg::Gadget g{};
    g.layer = layer;
    g.sslot = 30;
    g.mask = 0;
    g.S = I.scratch(static_cast<size_t>(N) * nslots * gg::kW * sizeof(int16_t));
    g.PB = nullptr;
    g.N = N;
    g.nslots = nslots;
    g.draws = gg::dconst(dr.data(), dr.size());
    g.ndraws = static_cast<int>(dr.size());
    g.projs = gg::dconst(pr.data(), pr.size());
    g.nprojs = static_cast<int>(pr.size());
    g.entries = first;
    g.nblk = draw_blocks(dr);

    check_desc(g);
    gg::In in{};
    std::vector<void*> tmp;
    hipLaunchKernelGGL(gg::draw_kernel(), dim3(draw_grid(g)), dim3(gg::kGB), 0, gg::tl_st, I.c, g);
    int ny = 0;
    for (int j = 0; j <= k; ++j) {
        const int nc = static_cast<int>(gg::chunks_of(nr_comps(j < k ? P.crt[j] : static_cast<int>(P.T))));
        for (int c8 = 0; c8 < nc; ++c8) {
            DASH_CHECK(ny < gg::kMaxY, "gpu garbler: mixed-radix derive work items");
            a.yj[ny] = j;
            a.yc[ny++] = c8;
        }
    }
    hipLaunchKernelGGL(gg::k_mrs_derive, dim3(blocks_for(N, 256), ny), dim3(256), 0, gg::tl_st, I.c, g, a);
    project(I.c, g, in, tb, pr, ProjFns{&flut, &fan});
    if (P.sign_last) {
        // residue 0's key slot is the sign label of the ReLU that follows (relu_mult)
        I.sig_slot = a.key0;
        I.sig_N = N;
        I.sig_S = g.S;
    }
    HIPCHECK(hipGetLastError());
    gg::end_layer(tmp);
    tr_.mark("kernels");
    tT.to_array(tab, I.device);
    set_stale(cur, I.cur_mod, N);
}

// ReLU whose sign came out of the preceding mixed-radix rescale (RescaleMrsPlan::sign_last, I.sig_slot): the
// mixed-modulus half gates only; device cur -> next base labels.
void GpuGarbler::relu_mult(uint64_t layer, CrtLabels& cur, const std::vector<i64>* prefix, Array& mmg, Array& mme) {
    Impl& I = *impl_;
    I.enter();
    I.check_cur(cur);
    PhaseTrace tr_("relu_mult");
    const int64_t N = I.cur_N;
    const int k = I.k;
    DASH_CHECK(I.sig_slot >= 2 * k && I.sig_N == N, "gpu garbler: joint ReLU without a preceding sign-producing rescale");
    // the rescale's scratch in place: the sign label stays in its slot, the mixed-multiply output labels take
    // slots 0 .. 2k - 1 (the rescale's digit-target labels, dead by now); no slot above the sign is needed,
    // so the grow-only scratch is not reallocated
    const int sig_slot = I.sig_slot, sk0 = 0, nslots = sig_slot + 1;
    DevTable tG, tE;
    tG.alloc(I.device, N, mmg.shape[1], mmg);
    tE.alloc(I.device, N, static_cast<int64_t>(k) * 3, mme, true);
    gg::Tables tb{};
    tb.t[4] = tG.p(); tb.row[4] = tG.row;
    tb.t[5] = tE.p(); tb.row[5] = tE.row;
    gg::In in{};
    for (int j = 0; j < k; ++j) {
        in.p[j] = I.cur[j].as<int16_t>();
        in.n[j] = nr_comps(I.crt[j]);
        in.es[j] = gg::kCh;  // chunked component-major
        in.cs[j] = N * gg::kCh;
    }
    gg::Gadget g{};
    g.layer = layer;
    g.sslot = 2;
    g.mask = 0;
    g.S = I.scratch(static_cast<size_t>(N) * nslots * gg::kW * sizeof(int16_t));
    DASH_CHECK(g.S == I.sig_S, "gpu garbler: garbling scratch moved between the rescale and its joint ReLU");
    g.N = N;
    g.nslots = nslots;
    std::vector<DevBlock> out = relu_mult_gates(I, g, in, tb, sig_slot, sk0, *prefix);
    HIPCHECK(hipGetLastError());
    std::vector<void*> tmp;
    gg::end_layer(tmp);
    tr_.mark("kernels");
    tG.to_array(mmg, I.device);
    tE.to_array(mme, I.device);
    I.cur = std::move(out);
    I.sig_slot = -1;
    I.sig_N = 0;
    I.sig_S = nullptr;
    set_stale(cur, I.crt, N);
}

// ===========================================================================
// Remaining layer kinds on the device: dense, sum pool, residual add (device
// copies of saved outputs), max pool / max (trees of ReLU gadgets), ReDash
// rescale (trans projections + base extension) and the base-extension layer.
// Each is byte-identical to the host garbler (garbler.cpp; tests compare the
// serialized models), so a GC of any zoo model is garbled without host round
// trips of its labels.
namespace {

size_t label_bytes(int p, int64_t N) {
    return static_cast<size_t>(N) * gg::chunks_of(nr_comps(p)) * gg::kCh * sizeof(int16_t);
}

gg::LinJob lin_job(int16_t* dst, int p) {
    gg::LinJob j{};
    j.dst = dst;
    j.p = p;
    j.nc = static_cast<int>(gg::chunks_of(nr_comps(p)));
    return j;
}
// operands: a / b label sets of N elements (element stride 8, chunk stride 8 N), r a uniform row
void lin_a(gg::LinJob& j, const int16_t* a, int64_t N, int64_t coef) {
    j.a = a;
    j.aes = gg::kCh;
    j.acs = N * gg::kCh;
    j.ca = static_cast<int>(pmod(coef, j.p));
}
void lin_b(gg::LinJob& j, const int16_t* b, int64_t N, int64_t coef) {
    j.b = b;
    j.bes = gg::kCh;
    j.bcs = N * gg::kCh;
    j.cb = static_cast<int>(pmod(coef, j.p));
}
void lin_r(gg::LinJob& j, const int16_t* r, int64_t coef) {
    j.r = r;
    j.cr = static_cast<int>(pmod(coef, j.p));
}

void launch_lin(const gg::Ctx& c, const std::vector<gg::LinJob>& jobs, int64_t N) {
    for (size_t s0 = 0; s0 < jobs.size(); s0 += gg::kMaxLin) {
        gg::LinArgs a{};
        a.n = static_cast<int>(std::min<size_t>(gg::kMaxLin, jobs.size() - s0));
        a.N = N;
        int ncmax = 1;
        for (int i = 0; i < a.n; ++i) {
            a.j[i] = jobs[s0 + i];
            ncmax = std::max(ncmax, a.j[i].nc);
        }
        hipLaunchKernelGGL(gg::k_lin, dim3(blocks_for(N * ncmax, 256, 8192), a.n), dim3(256), 0, gg::tl_st, c, a);
    }
}

// dst[e] (+)= sum_t cf_j[t] src[map[e K + t]] for every residue j (cf of residue j: coef(p_j, t))
template <class Coef>
void launch_gsum(const gg::Ctx& c, const std::vector<DevBlock>& dst, const std::vector<DevBlock>& src,
                 const std::vector<int>& mods, int64_t N, int64_t Nsrc, const int32_t* map, int K, bool acc,
                 Coef coef) {
    DASH_CHECK(K >= 1 && K <= gg::kMaxTerms && mods.size() <= static_cast<size_t>(kMaxRes),
               "gpu garbler: gathered sum shape");
    gg::GsArgs a{};
    a.n = static_cast<int>(mods.size());
    a.K = K;
    a.acc = acc ? 1 : 0;
    a.N = N;
    a.Nsrc = Nsrc;
    a.map = map;
    int ncmax = 1;
    for (int j = 0; j < a.n; ++j) {
        a.j[j].dst = dst[j].as<int16_t>();
        a.j[j].src = src[j].as<int16_t>();
        a.j[j].p = mods[j];
        a.j[j].nc = static_cast<int>(gg::chunks_of(nr_comps(mods[j])));
        for (int t = 0; t < K; ++t) a.j[j].cf[t] = static_cast<int>(pmod(coef(mods[j], t), mods[j]));
        ncmax = std::max(ncmax, a.j[j].nc);
    }
    hipLaunchKernelGGL(gg::k_gsum, dim3(blocks_for(N * ncmax, 256, 8192), a.n), dim3(256), 0, gg::tl_st, c, a);
}

struct DensePlanKey {
    int dev;
    uint64_t wh;
    std::vector<i64> geom;
    std::vector<int> mods;
    bool operator<(const DensePlanKey& o) const {
        return std::tie(dev, wh, geom, mods) < std::tie(o.dev, o.wh, o.geom, o.mods);
    }
};
struct DensePlan {
    const int16_t* wt[kMaxRes];
    const int32_t* zc[kMaxRes];
};
std::map<DensePlanKey, DensePlan>& dense_plans() {
    static auto* m = new std::map<DensePlanKey, DensePlan>();  // leaked: device buffers live as long as the process
    return *m;
}
std::mutex& dense_plans_mutex() {
    static std::mutex m;
    return m;
}

// residue labels (chunked) and a working-copy area for the base-extension stages of one gadget
struct BeStage {
    std::vector<std::vector<int>> slot;  // [i][j]: drawn output label of stage i's projection to target i+j+1
};

// BEPlan draws in be_garble_elem's PRG order, appended to dr (slots from `slot`, counters from `ctr`)
BeStage be_draws(const BEPlan& P, std::vector<gg::Draw>& dr, int& slot, int& ctr) {
    BeStage st;
    const int E = static_cast<int>(P.moduli.size());
    st.slot.resize(P.nonext);
    for (int i = 0; i < P.nonext; ++i)
        for (int j = 0; j < E - i - 1; ++j) {
            const int q = P.swapped[i + j + 1];
            st.slot[i].push_back(slot);
            dr.push_back({slot++, q, ctr});
            ctr += prg_blocks(q);
        }
    return st;
}

// be_garble_elem on the device: working copies lw (slots lw0 + position in the swapped order) of the labels
// Lp (residue i of P.moduli); per non-extended stage i the identity projections of lw[i] into every later
// modulus (table `table`, entries in be_garble_elem's order), then lw[t] = (lw[t] - out) inv; the extended
// residues come back scaled by -invv. Draws (st) must be done.
void be_run(GpuGarbler::Impl& I, gg::Gadget& g, const BEPlan& P, const std::vector<int16_t*>& Lp, const BeStage& st,
            int lw0, gg::Tables& tb, int table) {
    const int E = static_cast<int>(P.moduli.size());
    const int64_t N = g.N;
    std::vector<gg::LinJob> jobs;
    for (int i = 0; i < E; ++i) {
        gg::LinJob j = lin_job(gg::slot_base(g, lw0 + P.pos_of[i]), P.moduli[i]);
        lin_a(j, Lp[i], N, 1);
        jobs.push_back(j);
    }
    launch_lin(I.c, jobs, N);
    int64_t off = 0;
    gg::In none{};
    for (int i = 0; i < P.nonext; ++i) {
        std::vector<gg::Proj> pr;
        int64_t first = 0;
        for (int j = 0; j < E - i - 1; ++j) {
            const int tg = i + j + 1;
            gg::Proj p{gg::S_SLOT, lw0 + i, P.swapped[i], st.slot[i][j], P.swapped[tg], gg::F_IDENT, 0, 0, 0,
                       gg::R_BANK, 0, table, 1, off, first};
            p.hsub = tw_sub(kTwBe, static_cast<uint32_t>(i));
            p.hslot = j;
            off += P.swapped[i];
            first += P.swapped[i];
            pr.push_back(p);
        }
        g.entries = first;
        project(I.c, g, none, tb, pr);
        jobs.clear();
        for (int j = 0; j < E - i - 1; ++j) {
            const int tg = i + j + 1, q = P.swapped[tg];
            const i64 inv = P.inv_partial[i][j];
            gg::LinJob J = lin_job(gg::slot_base(g, lw0 + tg), q);
            lin_a(J, gg::slot_base(g, lw0 + tg), N, inv);
            lin_b(J, gg::slot_base(g, st.slot[i][j]), N, -inv);
            jobs.push_back(J);
        }
        launch_lin(I.c, jobs, N);
    }
    jobs.clear();
    for (size_t x = 0; x < P.extra.size(); ++x) {
        const int bi = P.extra_idx[x];
        gg::LinJob J = lin_job(Lp[bi], P.moduli[bi]);
        lin_a(J, gg::slot_base(g, lw0 + P.pos_of[bi]), N, -P.invv[x]);
        jobs.push_back(J);
    }
    launch_lin(I.c, jobs, N);
}

}  // namespace

void GpuGarbler::save(size_t idx) {
    Impl& I = *impl_;
    I.enter();
    Impl::Saved sv;
    sv.mods = I.cur_mod;
    sv.N = I.cur_N;
    sv.L = I.alloc_labels(sv.mods, sv.N);
    for (size_t j = 0; j < sv.mods.size(); ++j)
        HIPCHECK(hipMemcpyAsync(sv.L[j].p, I.cur[j].p, label_bytes(sv.mods[j], sv.N), hipMemcpyDeviceToDevice, gg::tl_st));
    I.saved[idx] = std::move(sv);
}

bool GpuGarbler::has_saved(size_t idx) const { return impl_->saved.count(idx) != 0; }

void GpuGarbler::restore(size_t idx, CrtLabels& cur) {
    Impl& I = *impl_;
    I.enter();
    auto it = I.saved.find(idx);
    DASH_CHECK(it != I.saved.end(), "gpu garbler: no device copy of that layer output");
    const Impl::Saved& sv = it->second;
    I.cur = I.alloc_labels(sv.mods, sv.N);
    for (size_t j = 0; j < sv.mods.size(); ++j)
        HIPCHECK(hipMemcpyAsync(I.cur[j].p, sv.L[j].p, label_bytes(sv.mods[j], sv.N), hipMemcpyDeviceToDevice, gg::tl_st));
    I.cur_mod = sv.mods;
    I.cur_N = sv.N;
    set_stale(cur, I.cur_mod, I.cur_N);
}

// residual add: cur += saved output (free addition of base labels, garbler.cpp K_ADD)
void GpuGarbler::add_saved(size_t idx, CrtLabels& cur) {
    Impl& I = *impl_;
    I.enter();
    I.check_cur(cur);
    auto it = I.saved.find(idx);
    DASH_CHECK(it != I.saved.end() && it->second.N == I.cur_N && it->second.mods == I.cur_mod,
               "gpu garbler: add operand missing or of another shape");
    std::vector<gg::LinJob> jobs;
    for (size_t j = 0; j < I.cur_mod.size(); ++j) {
        gg::LinJob J = lin_job(I.cur[j].as<int16_t>(), I.cur_mod[j]);
        lin_a(J, I.cur[j].as<int16_t>(), I.cur_N, 1);
        lin_b(J, it->second.L[j].as<int16_t>(), I.cur_N, 1);
        jobs.push_back(J);
    }
    launch_lin(I.c, jobs, I.cur_N);
    HIPCHECK(hipGetLastError());
}

// dense base labels (garbler.cpp K_DENSE): y_o = sum_{w != 0 mod p} w x_src(i) + (1 + #zero weights) Z_p
void GpuGarbler::dense(i64 in, i64 out, i64 ch, const i64* w, size_t nw, uint64_t wh, CrtLabels& cur) {
    Impl& I = *impl_;
    I.enter();
    I.check_cur(cur);
    PhaseTrace tr_("dense");
    DASH_CHECK(I.cur_N == in && static_cast<i64>(nw) == in * out, "gpu garbler: dense shape");
    const int k = static_cast<int>(I.cur_mod.size());
    DensePlan plan{};
    {
        DensePlanKey key{I.device, wh, {in, out, ch}, I.cur_mod};
        std::lock_guard<std::mutex> lk(dense_plans_mutex());
        auto it = dense_plans().find(key);
        if (it != dense_plans().end()) {
            plan = it->second;
        } else {
            for (int j = 0; j < k; ++j) {
                const int p = I.cur_mod[j];
                DASH_CHECK(p <= 2048, "gpu garbler: dense residue modulus above 2048");
                std::vector<int16_t> wt(static_cast<size_t>(in) * out);
                std::vector<int32_t> zc(out, 1);
                for (i64 o = 0; o < out; ++o)
                    for (i64 i = 0; i < in; ++i) {
                        const int v = static_cast<int>(w[static_cast<size_t>(o * in + i)] % p);
                        if (v == 0) ++zc[o];
                        wt[static_cast<size_t>(dense_src(i, in, ch)) * out + o] = static_cast<int16_t>(v);
                    }
                plan.wt[j] = gg::dconst(wt.data(), wt.size());
                plan.zc[j] = gg::dconst(zc.data(), zc.size());
            }
            dense_plans().emplace(std::move(key), plan);
        }
    }
    std::vector<DevBlock> y = I.alloc_labels(I.cur_mod, out);
    gg::DnArgs a{};
    a.n = k;
    a.in = static_cast<int>(in);
    a.out = static_cast<int>(out);
    a.otiles = static_cast<int>((out + 63) / 64);
    int ncmax = 1;
    for (int j = 0; j < k; ++j) {
        a.j[j] = gg::DnJob{y[j].as<int16_t>(), I.cur[j].as<int16_t>(), plan.wt[j], plan.zc[j], I.cur_mod[j],
                           static_cast<int>(gg::chunks_of(nr_comps(I.cur_mod[j])))};
        ncmax = std::max(ncmax, a.j[j].nc);
    }
    hipLaunchKernelGGL(gg::k_gdense, dim3(a.otiles * ncmax, k), dim3(256), 0, gg::tl_st, I.c, a);
    HIPCHECK(hipGetLastError());
    tr_.mark("kernels");
    I.cur = std::move(y);
    I.cur_N = out;
    set_stale(cur, I.cur_mod, out);
}

// hardened encoding: y_e += (c[e / group] mod p_j) R_pj on the device cur (c: one public constant per group,
// already negated / reduced mod M by the caller)
void GpuGarbler::fold_constants(const std::vector<i64>& c, i64 group, CrtLabels& cur) {
    Impl& I = *impl_;
    I.enter();
    I.check_cur(cur);
    DASH_CHECK(group >= 1 && static_cast<i64>(c.size()) * group == I.cur_N, "gpu garbler: constant fold shape");
    gg::FoldArgs a{};
    a.N = I.cur_N;
    a.group = group;
    int ncmax = 1;
    const int k = static_cast<int>(I.cur_mod.size());
    for (int j = 0; j < k; ++j) {
        const int p = I.cur_mod[j];
        std::vector<int32_t> cj(c.size());
        for (size_t g = 0; g < c.size(); ++g) cj[g] = static_cast<int32_t>(pmod(c[g], p));
        a.j[j] = gg::FoldJob{I.cur[j].as<int16_t>(), gg::dconst(cj.data(), cj.size()), p,
                             static_cast<int>(gg::chunks_of(nr_comps(p)))};
        ncmax = std::max(ncmax, a.j[j].nc);
    }
    const int64_t work = I.cur_N * ncmax;
    const int blocks = static_cast<int>(std::min<int64_t>((work + 255) / 256, 4096));
    hipLaunchKernelGGL(gg::k_fold, dim3(blocks, k), dim3(256), 0, gg::tl_st, I.c, a);
    HIPCHECK(hipGetLastError());
}

// sum pool (garbler.cpp K_SUMPOOL): window sums of base labels
void GpuGarbler::sumpool(const PoolGeom& G, CrtLabels& cur) {
    Impl& I = *impl_;
    I.enter();
    I.check_cur(cur);
    DASH_CHECK(G.C * G.H * G.W == I.cur_N, "gpu garbler: sum pool input size");
    const int64_t Nout = G.out_size();
    const int K = static_cast<int>(G.kh * G.kw);
    std::vector<int32_t> map(static_cast<size_t>(Nout) * K);
    std::vector<i64> win;
    for (int64_t o = 0; o < Nout; ++o) {
        G.window(o, win);
        for (int s = 0; s < K; ++s) map[static_cast<size_t>(o) * K + s] = static_cast<int32_t>(win[s]);
    }
    std::vector<DevBlock> y = I.alloc_labels(I.cur_mod, Nout);
    // windows of more than kMaxTerms values: accumulate term groups (the map is re-cut per group)
    for (int t0 = 0; t0 < K; t0 += gg::kMaxTerms) {
        const int Kt = std::min(gg::kMaxTerms, K - t0);
        std::vector<int32_t> mt(static_cast<size_t>(Nout) * Kt);
        for (int64_t o = 0; o < Nout; ++o)
            for (int t = 0; t < Kt; ++t) mt[static_cast<size_t>(o) * Kt + t] = map[static_cast<size_t>(o) * K + t0 + t];
        launch_gsum(I.c, y, I.cur, I.cur_mod, Nout, I.cur_N, gg::dconst(mt.data(), mt.size()), Kt, t0 > 0,
                    [](int, int) { return 1; });
    }
    HIPCHECK(hipGetLastError());
    I.cur = std::move(y);
    I.cur_N = Nout;
    set_stale(cur, I.cur_mod, Nout);
}

// max pool / max (garbler.cpp K_MAXPOOL / K_MAX): the window values, then per tree level the pair differences,
// a ReLU gadget (streams 20 + 2 lv / 21 + 2 lv), and max = relu(b - a) + a, the odd value carried
void GpuGarbler::maxpool_begin(const std::vector<std::vector<i64>>& win, CrtLabels& cur) {
    Impl& I = *impl_;
    I.enter();
    I.check_cur(cur);
    const int64_t Nout = static_cast<int64_t>(win.size());
    DASH_CHECK(Nout > 0, "gpu garbler: empty max pool");
    const int64_t K = static_cast<int64_t>(win[0].size());
    std::vector<int32_t> map(static_cast<size_t>(Nout * K));
    for (int64_t o = 0; o < Nout; ++o) {
        DASH_CHECK(static_cast<int64_t>(win[o].size()) == K, "gpu garbler: ragged max pool windows");
        for (int64_t s = 0; s < K; ++s) map[static_cast<size_t>(o * K + s)] = static_cast<int32_t>(win[o][s]);
    }
    I.mp_V = I.alloc_labels(I.cur_mod, Nout * K);
    launch_gsum(I.c, I.mp_V, I.cur, I.cur_mod, Nout * K, I.cur_N, gg::dconst(map.data(), map.size()), 1, false,
                [](int, int) { return 1; });
    I.mp_Nout = Nout;
    I.mp_cnt = K;
}

void GpuGarbler::maxpool_level(uint64_t layer, int lv, i64 ops, const SignPlan& sp, const std::vector<i64>& prefix,
                               Array& ap, Array& c1, Array& c2, Array& sg, Array& mmg, Array& mme) {
    Impl& I = *impl_;
    I.enter();
    PhaseTrace tr_("maxpool_level");
    const int64_t Nout = I.mp_Nout, cnt = I.mp_cnt, cnt1 = ops + cnt % 2, Nd = Nout * ops;
    DASH_CHECK(ops >= 1 && 2 * ops <= cnt, "gpu garbler: max tree level shape");
    // pair differences D[o ops + q] = V[o cnt + 2q + 1] - V[o cnt + 2q]
    std::vector<int32_t> dm(static_cast<size_t>(Nd) * 2), am(static_cast<size_t>(Nout * cnt1)),
        ym(static_cast<size_t>(Nout * cnt1));
    for (int64_t o = 0; o < Nout; ++o) {
        for (int64_t q = 0; q < ops; ++q) {
            dm[static_cast<size_t>((o * ops + q) * 2)] = static_cast<int32_t>(o * cnt + 2 * q + 1);
            dm[static_cast<size_t>((o * ops + q) * 2 + 1)] = static_cast<int32_t>(o * cnt + 2 * q);
        }
        for (int64_t q = 0; q < cnt1; ++q) {
            am[static_cast<size_t>(o * cnt1 + q)] = static_cast<int32_t>(q < ops ? o * cnt + 2 * q : o * cnt + cnt - 1);
            ym[static_cast<size_t>(o * cnt1 + q)] = q < ops ? static_cast<int32_t>(o * ops + q) : -1;
        }
    }
    std::vector<DevBlock> D = I.alloc_labels(I.crt, Nd);
    launch_gsum(I.c, D, I.mp_V, I.crt, Nd, Nout * cnt, gg::dconst(dm.data(), dm.size()), 2, false,
                [](int p, int t) { return t == 0 ? 1 : p - 1; });
    std::vector<int> omods;
    std::vector<DevBlock> Y = sign_core(I, layer, 20 + 2 * lv, 21 + 2 * lv, sp, labels_in(D, I.crt, Nd), Nd, ap, c1, c2,
                                        sg, &prefix, &mmg, &mme, omods);
    std::vector<DevBlock> nv = I.alloc_labels(I.crt, Nout * cnt1);
    launch_gsum(I.c, nv, I.mp_V, I.crt, Nout * cnt1, Nout * cnt, gg::dconst(am.data(), am.size()), 1, false,
                [](int, int) { return 1; });
    launch_gsum(I.c, nv, Y, I.crt, Nout * cnt1, Nd, gg::dconst(ym.data(), ym.size()), 1, true,
                [](int, int) { return 1; });
    HIPCHECK(hipGetLastError());
    tr_.mark("kernels");
    I.mp_V = std::move(nv);
    I.mp_cnt = cnt1;
}

void GpuGarbler::maxpool_end(CrtLabels& cur) {
    Impl& I = *impl_;
    I.enter();
    DASH_CHECK(I.mp_cnt == 1, "gpu garbler: max tree not reduced to one value");
    I.cur = std::move(I.mp_V);
    I.cur_N = I.mp_Nout;
    I.cur_mod = I.crt;
    I.mp_Nout = I.mp_cnt = 0;
    set_stale(cur, I.cur_mod, I.cur_N);
}

// ReDash rescale iteration (rescale_garble_elem with a base-extension plan): L += up; per factor the identity
// projections of L[fi] into every active residue (trans table), L_j = (L_j - out) s^-1; L[fi] = Z; base
// extension of the factors' residues (be table); L -= down. One PRG stream (layer, 10 + it), counters in
// rescale_garble_elem's order.
void GpuGarbler::rescale_redash(uint64_t layer, int it, const RescalePlan& P, CrtLabels& cur,
                                const std::vector<std::vector<comp_t>>& up,
                                const std::vector<std::vector<comp_t>>& down, Array& tr, Array& be) {
    Impl& I = *impl_;
    I.enter();
    I.check_cur(cur);
    PhaseTrace tr_("rescale_redash");
    DASH_CHECK(!P.sign_be && I.cur_mod == I.crt, "gpu garbler: ReDash rescale plan mismatch");
    const int64_t N = I.cur_N;
    const int k = I.k;
    std::vector<int16_t> hup(k * gg::kW, 0), hdn(k * gg::kW, 0);
    for (int j = 0; j < k; ++j) {
        std::copy(up[j].begin(), up[j].end(), hup.begin() + j * gg::kW);
        std::copy(down[j].begin(), down[j].end(), hdn.begin() + j * gg::kW);
    }
    const int16_t* dup = I.stage(hup.data(), hup.size());
    const int16_t* ddn = I.stage(hdn.data(), hdn.size());
    // draws: trans outputs (factor, active residue), then the base extension's
    std::vector<gg::Draw> dr;
    int slot = 0, ctr = 0;
    std::vector<std::vector<int>> ts(P.factors.size());
    for (size_t f = 0; f < P.factors.size(); ++f)
        for (int j : P.active[f]) {
            ts[f].push_back(slot);
            dr.push_back({slot++, P.crt[j], ctr});
            ctr += prg_blocks(P.crt[j]);
        }
    BeStage st = be_draws(P.be, dr, slot, ctr);
    const int lw0 = slot;
    slot += k;
    const int nslots = slot;
    DevTable tT, tB;
    tT.alloc(I.device, N, tr.shape[1], tr);
    tB.alloc(I.device, N, be.shape[1], be);
    gg::Tables tb{};
    tb.t[6] = tT.p(); tb.row[6] = tT.row;
    tb.t[7] = tB.p(); tb.row[7] = tB.row;
    gg::Gadget g{};
    g.layer = layer;
    g.sslot = 10 + it;
    g.mask = 0;
    g.S = I.scratch(static_cast<size_t>(N) * nslots * gg::kW * sizeof(int16_t));
    g.N = N;
    g.nslots = nslots;
    g.draws = gg::dconst(dr.data(), dr.size());
    g.ndraws = static_cast<int>(dr.size());
    g.nblk = draw_blocks(dr);
    check_desc(g);
    hipLaunchKernelGGL(gg::draw_kernel(), dim3(draw_grid(g)), dim3(gg::kGB), 0, gg::tl_st, I.c, g);
    std::vector<int16_t*> L(k);
    for (int j = 0; j < k; ++j) L[j] = I.cur[j].as<int16_t>();
    std::vector<gg::LinJob> jobs;
    for (int j = 0; j < k; ++j) {
        gg::LinJob J = lin_job(L[j], I.crt[j]);
        lin_a(J, L[j], N, 1);
        lin_r(J, dup + j * gg::kW, 1);
        jobs.push_back(J);
    }
    launch_lin(I.c, jobs, N);
    const gg::In in = labels_in(I.cur, I.crt, N);
    int64_t off = 0;
    for (size_t f = 0; f < P.factors.size(); ++f) {
        const int s = P.factors[f], fi = P.factor_idx[f];
        std::vector<gg::Proj> pr;
        int64_t first = 0;
        for (size_t a = 0; a < P.active[f].size(); ++a) {
            const int j = P.active[f][a];
            gg::Proj tp{gg::S_INPUT, fi, s, ts[f][a], P.crt[j], gg::F_IDENT, 0, 0, 0, gg::R_BANK, 0, 6, 1, off, first};
            tp.hsub = tw_sub(kTwTrans, static_cast<uint32_t>(f));
            tp.hslot = static_cast<int>(a);
            pr.push_back(tp);
            off += s;
            first += s;
        }
        g.entries = first;
        project(I.c, g, in, tb, pr);
        jobs.clear();
        for (size_t a = 0; a < P.active[f].size(); ++a) {
            const int j = P.active[f][a];
            gg::LinJob J = lin_job(L[j], P.crt[j]);
            lin_a(J, L[j], N, P.inv[f][a]);
            lin_b(J, gg::slot_base(g, ts[f][a]), N, -P.inv[f][a]);
            jobs.push_back(J);
        }
        launch_lin(I.c, jobs, N);
    }
    jobs.clear();
    for (int fi : P.factor_idx) {
        gg::LinJob J = lin_job(L[fi], P.crt[fi]);
        lin_r(J, I.c.Z + static_cast<int64_t>(P.crt[fi]) * gg::kW, 1);
        jobs.push_back(J);
    }
    launch_lin(I.c, jobs, N);
    be_run(I, g, P.be, L, st, lw0, tb, 7);
    jobs.clear();
    for (int j = 0; j < k; ++j) {
        gg::LinJob J = lin_job(L[j], I.crt[j]);
        lin_a(J, L[j], N, 1);
        lin_r(J, ddn + j * gg::kW, -1);
        jobs.push_back(J);
    }
    launch_lin(I.c, jobs, N);
    HIPCHECK(hipGetLastError());
    std::vector<void*> tmp;
    gg::end_layer(tmp);
    tr_.mark("kernels");
    tT.to_array(tr, I.device);
    tB.to_array(be, I.device);
    set_stale(cur, I.cur_mod, N);
}

// base-extension layer (garbler.cpp K_BASEEXT): the extra residues start from Z, then be_garble_elem on
// stream (layer, 1), counters from 0
void GpuGarbler::base_ext(uint64_t layer, const BEPlan& P, CrtLabels& cur, Array& be) {
    Impl& I = *impl_;
    I.enter();
    I.check_cur(cur);
    DASH_CHECK(P.moduli == I.cur_mod, "gpu garbler: base extension plan mismatch");
    const int64_t N = I.cur_N;
    const int E = static_cast<int>(P.moduli.size());
    std::vector<gg::Draw> dr;
    int slot = 0, ctr = 0;
    BeStage st = be_draws(P, dr, slot, ctr);
    const int lw0 = slot;
    slot += E;
    DevTable tB;
    tB.alloc(I.device, N, be.shape[1], be);
    gg::Tables tb{};
    tb.t[7] = tB.p(); tb.row[7] = tB.row;
    gg::Gadget g{};
    g.layer = layer;
    g.sslot = 1;
    g.mask = 0;
    g.S = I.scratch(static_cast<size_t>(N) * slot * gg::kW * sizeof(int16_t));
    g.N = N;
    g.nslots = slot;
    g.draws = gg::dconst(dr.data(), dr.size());
    g.ndraws = static_cast<int>(dr.size());
    g.nblk = draw_blocks(dr);
    check_desc(g);
    if (!dr.empty()) hipLaunchKernelGGL(gg::draw_kernel(), dim3(draw_grid(g)), dim3(gg::kGB), 0, gg::tl_st, I.c, g);
    std::vector<int16_t*> L(E);
    for (int j = 0; j < E; ++j) L[j] = I.cur[j].as<int16_t>();
    std::vector<gg::LinJob> jobs;
    for (int xi : P.extra_idx) {
        gg::LinJob J = lin_job(L[xi], P.moduli[xi]);
        lin_r(J, I.c.Z + static_cast<int64_t>(P.moduli[xi]) * gg::kW, 1);
        jobs.push_back(J);
    }
    launch_lin(I.c, jobs, N);
    be_run(I, g, P, L, st, lw0, tb, 7);
    HIPCHECK(hipGetLastError());
    std::vector<void*> tmp;
    gg::end_layer(tmp);
    tB.to_array(be, I.device);
    set_stale(cur, I.cur_mod, N);
}

}  // namespace dash
