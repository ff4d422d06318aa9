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
    int pay1;                    // 1 + payload bank row of f-index 0 (F_SIGN, F_DIV, F_DIVMOD); 0: computed inline
    int pad_;
    int64_t first_out;           // first global output (entry x target) index (k_emit; set by gg::project)
};

// A projection whose function takes few distinct values (sign: 2, carry: k+1)
// has few distinct payloads o + f*R: they are computed once per element into a
// payload bank (row-major [row][N], coalesced) instead of once per table entry.
struct PayDesc {
    int out_slot, pout, f;  // payload = slot label + f * R_pout (f already reduced mod pout)
};

struct Tables {
    u128* t[8];        // per table id: [N][row]
    int64_t row[8];    // entries per element
};

struct Ctx {
    const int16_t* R;    // [max_mod + 1][kW]
    const int16_t* Z;    // [max_mod + 1][kW]
    const ModC* mc;      // [max_mod + 1]
    const int16_t* lut;  // approx lookup [k][p][t] flattened, offsets lut_off[j]
    int lut_off[kMaxRes];
    uint32_t rk[44];     // PRG (seed) round keys
    const uint32_t* te0;
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
__device__ __forceinline__ u128 aes_keyed(const AesCtx& a, u128 in, const uint32_t* rk) {
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
    u128* PB;         // payload bank [row][N] (PayDesc rows)
    int64_t N;
    int mrs[kMaxMrs]; // MRS base of the sign gadget (per-digit output moduli of the fanned-out approx projections)
    const int16_t* flut;  // F_FAN: payload values [a0 + i * stride + target] (reduced mod the target modulus)
    const int* fan;       // F_FAN: target moduli [a1 + target]
    const int* fbank;     // F_FAN: [a1 + target] 1 + payload bank row of value 0 (k_payloads), 0: computed inline
    int64_t outputs;      // per element: table entries written (sum over projections of entries x targets)
    u128* HC;             // [entries][N] key hashes (k_hash -> k_emit)
    uint8_t* CC;          // [entries][N] key colors
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
constexpr int kMaxDesc = 224;  // 224 x 72-B Proj (16 KiB) beside the AES image (dev.h)
constexpr int kGB = 512;        // threads per block of the AES-bound garbling kernels
template <class T>
__device__ __forceinline__ void lds_stage(T* dst, const T* src, int n) {
    const int words = n * static_cast<int>(sizeof(T) / 4);
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d = reinterpret_cast<uint32_t*>(dst);
    for (int i = threadIdx.x; i < words; i += blockDim.x) d[i] = s[i];
}

// One thread per (AES-CTR block, element), block-major: the lanes of a wave are
// consecutive elements drawing the same block, so the binary search is (mostly)
// wave-uniform and the stores land in neighbouring chunks. Block b of a draw
// yields ModC::pm consecutive components (Prg::label order) as the base-q
// digits of the block (DigitStream: one 128-bit long division per chunk of
// digits).
__global__ __launch_bounds__(kGB) void k_draw(Ctx c, Gadget g) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_aes[DASH_AES_LDS_WORDS];
    __shared__ Draw sd[kMaxDesc];
    lds_stage(sd, g.draws, g.ndraws);
    aes_lds_fill(lds_aes, c.te0);
    const AesCtx aes = aes_ctx(lds_aes, nullptr);
    const int64_t N = g.N;
    const int64_t total = N * g.nblk;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int b = static_cast<int>(i / N);
        const int64_t e = i - static_cast<int64_t>(b) * N;
        int lo = 0, hi = g.ndraws - 1;
        while (lo < hi) {  // last draw with ctr <= b
            const int mid = (lo + hi + 1) >> 1;
            if (sd[mid].ctr <= b) lo = mid;
            else hi = mid - 1;
        }
        const Draw d = sd[lo];
        const ModC m = c.mc[d.q];
        const int j = static_cast<int>(m.pm) * (b - d.ctr);
        const int cnt = min(static_cast<int>(m.pm), static_cast<int>(m.n) - j);
        const uint64_t stream = stream_of(g.layer, g.sslot, static_cast<uint64_t>(e), g.mask);
        DigitStream ds;
        ds.init(aes_keyed(aes, (static_cast<u128>(stream) << 64) | static_cast<uint64_t>(b), c.rk));
        int16_t* out = slot_base(g, d.slot) + e * kCh;
        const int64_t cs = N * kCh;
        for (int u = 0; u < cnt; ++u) {
            const int q = j + u;
            out[(q >> 3) * cs + (q & 7)] = static_cast<int16_t>(ds.next(m));
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

// digits (a_q + f * b_q) mod m of a per-lane label a and a wave-uniform row b (R_q: components in [0, m)),
// pushed into cf, 8 per chunk load. The row's chunk is moved to SGPRs (readfirstlane of a uniform load), so it
// costs no vector registers and its unpacking is scalar work.
__device__ __forceinline__ void push_row(CompressFwd& cf, LRef a, const int16_t* b, uint32_t f, const ModC& m) {
    const int n = static_cast<int>(m.n);
    const int nc = static_cast<int>(chunks_of(n));
    for (int c8 = 0; c8 < nc; ++c8) {
        const u32x4a av = ld_chunk(a, c8);
        const u32x4a bv = *reinterpret_cast<const u32x4a*>(b + c8 * kCh);
        uint32_t bs[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) bs[u] = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(bv[u])));
        const int q0 = c8 * 8;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint32_t x = (u & 1) ? (av[u >> 1] >> 16) : (av[u >> 1] & 0xffffu);
            const uint32_t y = (u & 1) ? (bs[u >> 1] >> 16) : (bs[u >> 1] & 0xffffu);
            if (q0 + u < n) cf.push(modq(x + f * y, m), m);
        }
    }
}
// the same with a per-lane offset label b (the evaluator half gate's offset is the input label x0)
__device__ __forceinline__ void push_row2(CompressFwd& cf, LRef a, LRef b, uint32_t f, const ModC& m) {
    const int n = static_cast<int>(m.n);
    const int nc = static_cast<int>(chunks_of(n));
    for (int c8 = 0; c8 < nc; ++c8) {
        uint32_t a0[8], b0[8];
        unpack8(ld_chunk(a, c8), a0);
        unpack8(ld_chunk(b, c8), b0);
        const int q0 = c8 * 8;
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (q0 + u < n) cf.push(modq(a0[u] + f * b0[u], m), m);
    }
}

// key = x + i*R (mod m), compressed from the least significant digit (R: uniform row)
__device__ __forceinline__ u128 proj_key(LRef x, const int16_t* R, int i, const ModC& m, uint32_t& color) {
    CompressFwd kc;
    kc.init();
    push_row(kc, x, R, static_cast<uint32_t>(i), m);
    color = modq(static_cast<uint32_t>(static_cast<uint16_t>(x.p[0]) + i * static_cast<uint16_t>(R[0])), m);
    return kc.finish();
}

// payload = o + f*R (mod m), o, f, R in [0, m) (R: uniform row)
__device__ __forceinline__ u128 proj_payload(LRef o, const int16_t* R, uint32_t f, const ModC& m) {
    CompressFwd pc;
    pc.init();
    push_row(pc, o, R, f, m);
    return pc.finish();
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
    r.first_out = rfl64(p.first_out);
    return r;
}

// Projections in two passes, so no lane carries a long dependent chain (key
// loads -> compress -> AES -> payload loads -> compress -> store):
//   k_hash  one lane per (element, table entry): key = x + i*R, H(compress(key)),
//           color -> HC / CC [entry][N];
//   k_emit  one lane per (element, entry, target): payload (inline, or from the
//           payload bank) + H -> the entry's table slot.
// Element-tiled order: the 64 lanes of a wavefront are 64 consecutive elements
// of one tile, all on the SAME work item, so the projection descriptor, i, the
// label widths (loop trip counts), the moduli and the function are
// wave-uniform and moved to SGPRs (readfirstlane); labels are chunked
// component-major, so one coalesced 16-byte load per lane covers 8 components.
__device__ __forceinline__ int find_proj(const Proj* sp, int n, int64_t r, bool by_out) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {  // last projection with first (first_out) <= r (uniform search)
        const int mid = (lo + hi + 1) >> 1;
        if (rfl64(by_out ? sp[mid].first_out : sp[mid].first) <= r) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__global__ __launch_bounds__(kPB) void k_hash(Ctx c, Gadget g, In in) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_aes[DASH_AES_LDS_WORDS];
    __shared__ Proj sp[kMaxDesc];
    lds_stage(sp, g.projs, g.nprojs);
    aes_lds_fill(lds_aes, c.te0);
    const AesCtx aes = aes_ctx(lds_aes, nullptr);
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
        const Proj P = rfl_proj(sp[find_proj(sp, g.nprojs, r, false)]);
        const int i = static_cast<int>(r - P.first);
        const ModC mi = rfl_modc(c.mc[P.pin]);
        // the last tile's spare lanes recompute element N-1 (uniform control flow) and skip the store
        const int64_t e_raw = tile * kTile + lane;
        const int64_t e = e_raw < N ? e_raw : N - 1;
        uint32_t color;
        const u128 H = aes_encrypt(aes, proj_key(label_ref(c, g, in, e, P.in_kind, P.in_idx, P.pin),
                                                 c.R + static_cast<int64_t>(P.pin) * kW, i, mi, color));
        if (e_raw < N) {
            g.HC[r * N + e] = H;
            g.CC[r * N + e] = static_cast<uint8_t>(color);
        }
    }
}

__global__ __launch_bounds__(256) void k_emit(Ctx c, Gadget g, In in, Tables tb) {
    __shared__ Proj sp[kMaxDesc];
    lds_stage(sp, g.projs, g.nprojs);
    __syncthreads();
    const int64_t N = g.N;
    const int64_t tiles = (N + kTile - 1) / kTile;
    const int64_t nw = tiles * g.outputs;  // wave work items (tile, output)
    const int lane = static_cast<int>(threadIdx.x) & (kTile - 1);
    const int64_t wpb = blockDim.x / kTile;
    const int64_t w0 = static_cast<int64_t>(blockIdx.x) * wpb + rfl(static_cast<int>(threadIdx.x) / kTile);
    const int64_t wstep = static_cast<int64_t>(gridDim.x) * wpb;
    for (int64_t w = w0; w < nw; w += wstep) {
        const int64_t tile = w / g.outputs;
        const int64_t o = w - tile * g.outputs;
        const Proj P = rfl_proj(sp[find_proj(sp, g.nprojs, o, true)]);
        const bool fan = P.fn == F_LUT || P.fn == F_FAN;
        const int t = fan ? P.stride : 1;
        const int local = static_cast<int>(o - P.first_out);
        const int i = local / t, d = local - i * t;
        const int64_t r = P.first + i;
        const int64_t e_raw = tile * kTile + lane;
        const int64_t e = e_raw < N ? e_raw : N - 1;
        const u128 H = g.HC[r * N + e];
        const uint32_t color = g.CC[r * N + e];
        u128 pay;
        if (P.fn == F_LUT) {
            // approx fan-out: digit d's payload mrs0_slot + d + lut[j][i][d] * R_{m_d}
            const int pout = rfl(g.mrs[d]);
            int64_t cm = c.lut[c.lut_off[P.a0] + i * t + d] % pout;
            if (cm < 0) cm += pout;
            pay = proj_payload(slot_ref(g, P.out_slot + d, e), c.R + static_cast<int64_t>(pout) * kW,
                               static_cast<uint32_t>(cm), rfl_modc(c.mc[pout]));
        } else if (P.fn == F_FAN) {
            // generic fan-out: target d writes slot out_slot + d, modulus fan[a1 + d], value flut[a0 + i * t + d]
            const uint32_t cm = static_cast<uint32_t>(rfl(g.flut[P.a0 + i * t + d]));
            const int bk = g.fbank ? rfl(g.fbank[P.a1 + d]) : 0;
            if (bk) {
                // few distinct values (e.g. the rescale's final projection: T = 2^(l+1) entries, p_j values)
                pay = g.PB[static_cast<int64_t>(bk - 1 + static_cast<int>(cm)) * N + e];
            } else {
                const int pout = rfl(g.fan[P.a1 + d]);
                pay = proj_payload(slot_ref(g, P.out_slot + d, e), c.R + static_cast<int64_t>(pout) * kW, cm,
                                   rfl_modc(c.mc[pout]));
            }
        } else if (P.pay1 > 0) {
            // few distinct payloads: precomputed per element by k_payloads
            const int idx = P.fn == F_SIGN ? (i < P.a0 ? 1 : 0) : i / P.a0;  // F_SIGN: 0 lower / 1 upper; F_DIV(MOD): i / m
            pay = g.PB[static_cast<int64_t>(P.pay1 - 1 + idx) * N + e];
        } else {
            int64_t f;
            switch (P.fn) {
                case F_DIV: f = i / P.a0; break;
                case F_DIVMOD: f = (i / P.a0) % P.a1; break;
                case F_SIGN: f = i < P.a0 ? P.a2 : P.a1; break;  // a0 = half, a1 = lower, a2 = upper
                case F_MULR: f = static_cast<int64_t>(i) * in.p[P.a0][e * in.es[P.a0]]; break;
                case F_NEGR: f = -(static_cast<int64_t>(i) + in.p[P.a0][e * in.es[P.a0]]); break;
                default: f = i;
            }
            int64_t cm = f % P.pout;
            if (cm < 0) cm += P.pout;
            const ModC mo = rfl_modc(c.mc[P.pout]);
            if (P.outr_kind == R_BANK) {
                pay = proj_payload(slot_ref(g, P.out_slot, e), c.R + static_cast<int64_t>(P.pout) * kW,
                                   static_cast<uint32_t>(cm), mo);
            } else {
                CompressFwd pc;
                pc.init();
                push_row2(pc, slot_ref(g, P.out_slot, e), label_ref(c, g, in, e, S_INPUT, P.outr_idx, 0),
                          static_cast<uint32_t>(cm), mo);
                pay = pc.finish();
            }
        }
        if (e_raw < N) {
            const int64_t slot = fan ? static_cast<int64_t>(color) * t + d : static_cast<int64_t>(color) * P.stride;
            tb.t[P.table][e * tb.row[P.table] + P.off + slot] = pay + H;
        }
    }
}

// Mixed-radix rescale (gadgets.h RescaleMrsPlan), garbler side of the free
// operations, one thread per element, 8 components per load: key base labels
// K_i = L_i - sum_{l<i} P_{l,i}, the mod-T accumulator r = sum_i P_{i,T}, then
// the output base labels (in place) Y_0 = F_0, Y_j = S^-1 L_j + F_j.
struct MrsG {
    int k, T;
    int crt[kMaxRes], sinv[kMaxRes];
    int nsub[kMaxRes];
    int sub[kMaxRes][kMaxRes];  // digit-target slots subtracted from residue j's key
    int tslot[kMaxRes];         // slot of digit i's T target
    int key0, acc, fin0;
    int16_t* L[kMaxRes];  // chunked [n_j / 8][N][8], updated in place
};

// grid (elements, k + 1): y = j < k derives residue j, y = k the accumulator
__global__ __launch_bounds__(256) void k_mrs_derive(Ctx c, Gadget g, MrsG a) {
    const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (e >= g.N) return;
    const int64_t cs = g.N * kCh;
    const int k = a.k;
    const int y = blockIdx.y;
    if (y < k) {
        const int j = y;
        const int p = a.crt[j];
        const ModC m = c.mc[p];
        const int nc = static_cast<int>(chunks_of(static_cast<int>(m.n))), ns = a.nsub[j];
        int16_t* Lj = a.L[j] + e * kCh;
        const LRef K = slot_ref(g, a.key0 + j, e), F = slot_ref(g, a.fin0 + j, e);
        for (int c8 = 0; c8 < nc; ++c8) {
            uint32_t x[8];
            unpack8(*reinterpret_cast<const u32x4a*>(Lj + c8 * cs), x);
            // key: L_j - sum of the digit payload labels aimed at residue j
            uint32_t kv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) kv[u] = x[u] + static_cast<uint32_t>(p) * static_cast<uint32_t>(ns);
            for (int l = 0; l < ns; ++l) {
                uint32_t sv[8];
                unpack8(ld_chunk(slot_ref(g, a.sub[j][l], e), c8), sv);
#pragma unroll
                for (int u = 0; u < 8; ++u) kv[u] -= sv[u];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) kv[u] = modq(kv[u], m);
            st_chunk(const_cast<int16_t*>(K.p) + c8 * K.cs, pack8(kv));
            // output base label (in place): Y_0 = F_0, Y_j = S^-1 L_j + F_j (chunk padding stays in the block)
            uint32_t fv[8], yv[8];
            unpack8(ld_chunk(F, c8), fv);
#pragma unroll
            for (int u = 0; u < 8; ++u) yv[u] = j == 0 ? fv[u] : modq(x[u] * static_cast<uint32_t>(a.sinv[j]) + fv[u], m);
            st_chunk(Lj + c8 * cs, pack8(yv));
        }
        return;
    }
    const int ncT = static_cast<int>(chunks_of(static_cast<int>(c.mc[a.T].n)));
    const LRef A = slot_ref(g, a.acc, e);
    for (int c8 = 0; c8 < ncT; ++c8) {
        uint32_t av[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int l = 0; l < k; ++l) add8(av, ld_chunk(slot_ref(g, a.tslot[l], e), c8));
#pragma unroll
        for (int u = 0; u < 8; ++u) av[u] &= static_cast<uint32_t>(a.T - 1);
        st_chunk(const_cast<int16_t*>(A.p) + c8 * A.cs, pack8(av));
    }
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

// Payload bank: one thread per (row, element), rows = PayDesc entries.
__global__ __launch_bounds__(256) void k_payloads(Ctx c, Gadget g, const PayDesc* pd, int npd) {
    const int64_t total = g.N * npd;
    for (int64_t x = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; x < total;
         x += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int r = static_cast<int>(x / g.N);
        const int64_t e = x - static_cast<int64_t>(r) * g.N;
        const PayDesc d = pd[r];
        // a wave may straddle two rows (N is not a multiple of 64): the offset row is per lane here
        CompressFwd pc;
        pc.init();
        push_row2(pc, slot_ref(g, d.out_slot, e), row_ref(c.R + static_cast<int64_t>(d.pout) * kW),
                  static_cast<uint32_t>(d.f), c.mc[d.pout]);
        g.PB[x] = pc.finish();
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
            const u128 H = hk[i * N + e];
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
__device__ __forceinline__ uint32_t bits8(const u32x4a& v) {
    uint32_t b = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) b |= ((v[u] & 1u) | ((v[u] >> 15) & 2u)) << (2 * u);
    return b;
}
__global__ __launch_bounds__(kGB) void k_bin_keys(Ctx c, const int16_t* x, const int16_t* add, u128* hk, int64_t N) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_aes[DASH_AES_LDS_WORDS];
    aes_lds_fill(lds_aes, c.te0);
    const AesCtx aes = aes_ctx(lds_aes, nullptr);
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
        aes_encrypt2(aes, key0, key0 ^ rbits, h0, h1);
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
    __shared__ __attribute__((aligned(16))) uint32_t lds_aes[DASH_AES_LDS_WORDS];
    aes_lds_fill(lds_aes, c.te0);
    const AesCtx aes = aes_ctx(lds_aes, nullptr);
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

// ------------------------------------------------------------------- host
struct SignLayout {
    std::vector<Draw> draws;
    std::vector<Proj> projs;
    std::vector<PayDesc> pays;
    int fan[kMaxMrs] = {};  // output modulus of the approx fan-out per digit
    SignSlots ss{};
    int nslots = 0;
    int out_slot0 = 0;
    int64_t entries = 0;
};

// Route projection p's payloads through the payload bank: row idx < nidx holds
// out_slot + f(idx) * R_pout.
template <class F>
Proj banked(SignLayout& L, Proj p, int nidx, F&& f) {
    p.pay1 = static_cast<int>(L.pays.size()) + 1;
    for (int idx = 0; idx < nidx; ++idx) {
        int64_t cm = static_cast<int64_t>(f(idx)) % p.pout;
        if (cm < 0) cm += p.pout;
        L.pays.push_back(PayDesc{p.out_slot, p.pout, static_cast<int>(cm)});
    }
    return p;
}
inline Proj banked_sign(SignLayout& L, const Proj& p) {  // F_SIGN: row 0 = lower (a1), row 1 = upper (a2)
    return banked(L, p, 2, [&](int idx) { return idx ? p.a2 : p.a1; });
}

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
    for (int j = 0; j < k; ++j)
        add(Proj{S_INPUT, j, P.crt[j], dig0 + j * t, P.mrs[0], F_LUT, j, 0, t, R_BANK, 0, 0, t,
                 t * P.crt_prefix[j], 0});
    int64_t c2 = 0;
    for (int q = 0; q + 1 < t; ++q) {
        const int d = t - 1 - q;
        const int mo = P.digit_mod(d);
        const Proj cp{S_SLOT, sum2_0 + q, mo, newc0 + q, P.carry_mod(d), F_DIVMOD, P.mrs[d], P.mrs[d - 1], 0, R_BANK, 0,
                      2, 1, c2, 0};
        add(banked(L, cp, (mo + cp.a0 - 1) / cp.a0, [&](int idx) { return idx % cp.a1; }));
        c2 += mo;
    }
    const int m0 = P.mrs[0];
    for (size_t o = 0; o < P.out_mod.size(); ++o)
        add(banked_sign(L, Proj{S_SLOT, sum_slot, m0, L.out_slot0 + static_cast<int>(o), P.out_mod[o], F_SIGN, m0 / 2,
                                P.lower, P.upper, R_BANK, 0, 3, 1, static_cast<int64_t>(o) * m0, 0}));
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
        add(banked(L, Proj{S_SLOT, sum2_0 + q, mo, bases0 + q * stride_q + (k + 1), P.mrs[d - 1], F_DIV, m, 0, 0, R_BANK,
                           0, 2, 1, c2, 0},
                   (mo + m - 1) / m, [](int idx) { return idx; }));
        c2 += mo;
    }
    const int m0 = P.mrs[0];
    for (size_t o = 0; o < P.out_mod.size(); ++o)
        add(banked_sign(L, Proj{S_SLOT, sum_slot, m0, L.out_slot0 + static_cast<int>(o), P.out_mod[o], F_SIGN, m0 / 2,
                                P.lower, P.upper, R_BANK, 0, 3, 1, static_cast<int64_t>(o) * m0, 0}));
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
std::pair<u128*, uint8_t*> hc_scratch(size_t entries, int64_t N);

// The projections of a gadget: output indices (entry x target) assigned, descriptors staged, then k_hash and
// k_emit on the garbling stream. g.draws / labels / payload bank must be ready (same stream).
void project(const gg::Ctx& c, gg::Gadget& g, const gg::In& in, const gg::Tables& tb, std::vector<gg::Proj> pr) {
    int64_t outs = 0;
    for (auto& p : pr) {
        p.first_out = outs;
        const bool fan = p.fn == gg::F_LUT || p.fn == gg::F_FAN;
        outs += static_cast<int64_t>(p.pin) * (fan ? p.stride : 1);
    }
    g.projs = gg::dconst(pr.data(), pr.size());
    g.nprojs = static_cast<int>(pr.size());
    g.outputs = outs;
    auto hc = hc_scratch(static_cast<size_t>(g.entries), g.N);
    g.HC = hc.first;
    g.CC = hc.second;
    check_desc(g);
    const int64_t lanes = (g.N + gg::kTile - 1) / gg::kTile * gg::kTile;
    hipLaunchKernelGGL(gg::k_hash, dim3(blocks_for(lanes * g.entries, gg::kPB, 16384)), dim3(gg::kPB), 0, gg::tl_st, c, g,
                       in);
    hipLaunchKernelGGL(gg::k_emit, dim3(blocks_for(lanes * g.outputs, 256, 16384)), dim3(256), 0, gg::tl_st, c, g, in, tb);
}

void run_sign(const gg::Ctx& c, const gg::SignLayout& L, gg::Gadget& g, const gg::In& in, const gg::Tables& tb,
              std::vector<void*>& tmp) {
    g.draws = gg::dconst(L.draws.data(), L.draws.size());
    g.ndraws = static_cast<int>(L.draws.size());
    g.projs = gg::dconst(L.projs.data(), L.projs.size());
    g.nprojs = static_cast<int>(L.projs.size());
    g.entries = L.entries;
    g.nblk = draw_blocks(L.draws);
    for (int d = 0; d < L.ss.t; ++d) g.mrs[d] = L.fan[d];
    check_desc(g);
    hipLaunchKernelGGL(gg::k_draw, dim3(blocks_for(g.N * g.nblk, gg::kGB, 8192)), dim3(gg::kGB), 0, gg::tl_st, c, g);
    hipLaunchKernelGGL(gg::k_sign_derive, dim3(blocks_for(g.N, 256), L.ss.t), dim3(256), 0, gg::tl_st, c, g, L.ss);
    if (!L.pays.empty()) {
        DASH_CHECK(g.PB != nullptr, "gpu garbler: payload bank not allocated");
        const gg::PayDesc* pd = gg::dconst(L.pays.data(), L.pays.size());
        const int npd = static_cast<int>(L.pays.size());
        hipLaunchKernelGGL(gg::k_payloads, dim3(blocks_for(g.N * npd, 256, 16384)), dim3(256), 0, gg::tl_st, c, g, pd, npd);
    }
    project(c, g, in, tb, L.projs);
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
    // key hashes / colors between k_hash and k_emit
    u128* HC = nullptr;
    uint8_t* CC = nullptr;
    size_t HC_n = 0;
    std::pair<u128*, uint8_t*> hc(size_t entries, int64_t N) {
        const size_t n = std::max<size_t>(1, entries * static_cast<size_t>(N));
        if (n > HC_n) {
            HIPCHECK(hipStreamSynchronize(st));
            if (HC) (void)hipFree(HC);
            if (CC) (void)hipFree(CC);
            HIPCHECK(hipMalloc(reinterpret_cast<void**>(&HC), n * sizeof(u128)));
            HIPCHECK(hipMalloc(reinterpret_cast<void**>(&CC), n));
            HC_n = n;
        }
        return {HC, CC};
    }
};
thread_local DevCtx* tl_dc = nullptr;  // the calling thread's garbling context (set by Impl::enter)
namespace {  // the same (translation-unit) anonymous namespace as its declaration above run_sign
std::pair<u128*, uint8_t*> hc_scratch(size_t entries, int64_t N) {
    DASH_CHECK(tl_dc != nullptr, "gpu garbler: no garbling context on this thread");
    return tl_dc->hc(entries, N);
}
}  // namespace
// A free garbling context of the device, locked for the caller: up to DASH_GG_CONTEXTS (default 2) per
// device, so two garblings (two threads, e.g. the serving engine's refill workers) run on two streams at
// once and fill each other's launch gaps; a third waits for the first context to free up.
std::unique_lock<std::mutex> acquire_ctx(int device, DevCtx*& out) {
    static std::mutex m;
    static auto* pools = new std::map<int, std::vector<DevCtx*>>();  // leaked: lives as long as the process
    static const size_t cap = [] {
        const char* e = std::getenv("DASH_GG_CONTEXTS");
        return static_cast<size_t>(std::max(1, e ? std::atoi(e) : 2));
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
    // sign base labels a sign_last mixed-radix rescale leaves for the next ReLU ([N][kW], relu_mult)
    DevBlock sig;
    int64_t sig_N = 0;
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
        HIPCHECK(hipSetDevice(device));
        gg::tl_st = dc.st;
        tl_dc = &dc;
    }
    ~Impl() {
        // garble() returns with every table written; blocks released below are reused in stream order
        (void)hipStreamSynchronize(dc.st);
        cur.clear();
        sig = DevBlock();
    }
};

GpuGarbler::GpuGarbler(const std::vector<int>& crt, const std::vector<int>& mrs, const std::string& seed16,
                       const LabelBank& R, const LabelBank& Z, int device)
    : impl_(new Impl(device)) {
    Impl& I = *impl_;
    I.enter();
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
    auto rk = round_key_words(reinterpret_cast<const uint8_t*>(seed16.data()));
    std::copy(rk.begin(), rk.end(), I.c.rk);
    if (!mrs.empty()) {
        auto lut = gen_approx_lookup(crt, mrs);
        std::vector<int16_t> flat;
        for (int j = 0; j < I.k; ++j) {
            I.c.lut_off[j] = static_cast<int>(flat.size());
            flat.insert(flat.end(), lut[j].begin(), lut[j].end());
        }
        I.c.lut = gg::dconst(flat.data(), flat.size());
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
    std::vector<int16_t> t;
    for (size_t j = 0; j < cur.size(); ++j) {
        const Labels& L = cur[j];
        DASH_CHECK(L.c.size() == static_cast<size_t>(L.N) * L.n, "gpu garbler: host labels are stale");
        t.assign(static_cast<size_t>(gg::chunks_of(L.n)) * gg::kCh * L.N, 0);
        for (i64 e = 0; e < L.N; ++e)
            for (int q = 0; q < L.n; ++q)
                t[((static_cast<size_t>(q >> 3)) * L.N + e) * gg::kCh + (q & 7)] = L.c[static_cast<size_t>(e) * L.n + q];
        // pageable source: staged before the call returns, ordered on the garbling stream
        HIPCHECK(hipMemcpyAsync(I.cur[j].p, t.data(), t.size() * sizeof(int16_t), hipMemcpyHostToDevice, gg::tl_st));
    }
}

void GpuGarbler::to_host(CrtLabels& cur) {
    Impl& I = *impl_;
    I.enter();
    I.check_cur(cur);
    std::vector<std::vector<int16_t>> t(cur.size());
    for (size_t j = 0; j < cur.size(); ++j) {
        t[j].resize(static_cast<size_t>(cur[j].N) * gg::chunks_of(cur[j].n) * gg::kCh);
        HIPCHECK(hipMemcpyAsync(t[j].data(), I.cur[j].p, t[j].size() * sizeof(int16_t), hipMemcpyDeviceToHost,
                                gg::tl_st));
    }
    HIPCHECK(hipStreamSynchronize(gg::tl_st));
    for (size_t j = 0; j < cur.size(); ++j) {
        Labels& L = cur[j];
        L.c.resize(static_cast<size_t>(L.N) * L.n);
        for (i64 e = 0; e < L.N; ++e)
            for (int q = 0; q < L.n; ++q)
                L.c[static_cast<size_t>(e) * L.n + q] = t[j][((static_cast<size_t>(q >> 3)) * L.N + e) * gg::kCh + (q & 7)];
    }
}

namespace {
// 64-bit mix hash of a weight vector (public conv weights: the per-layer MFMA setup is cached by content)
uint64_t weights_hash(const std::vector<i64>& w) {
    uint64_t h = 0x9e3779b97f4a7c15ull ^ w.size();
    for (i64 v : w) {
        h ^= static_cast<uint64_t>(v) + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
        h *= 0xff51afd7ed558ccdull;
    }
    return h;
}
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
void GpuGarbler::conv(const ConvGeom& G, const std::vector<i64>& w, CrtLabels& cur) {
    Impl& I = *impl_;
    I.enter();
    I.check_cur(cur);
    PhaseTrace tr_("conv");
    const int K = static_cast<int>(G.K());
    const int F = static_cast<int>(G.F);
    DASH_CHECK(static_cast<i64>(w.size()) == G.F * G.K(), "gpu garbler: conv weight shape");
    DASH_CHECK(G.C * G.H * G.W == I.cur_N, "gpu garbler: conv input size mismatch");
    DASH_CHECK(static_cast<int>(I.cur_mod.size()) <= kMaxRes, "gpu garbler: too many residues");
    std::vector<int> mods = I.cur_mod;
    const int64_t Nin = I.cur_N, Nout = G.out_size();
    std::vector<DevBlock> out = I.alloc_labels(mods, Nout);
    dev::ConvArgs a{};
    {
        ConvPlanKey key{I.device, weights_hash(w), {G.C, G.H, G.W, G.F, G.kh, G.kw, G.sh, G.sw, G.ph, G.pw}, mods};
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

void GpuGarbler::sign_layer(uint64_t layer, const SignPlan& sp, CrtLabels& cur, Array& ap, Array& c1, Array& c2,
                            Array& sg, const std::vector<int>* relu_crt, const std::vector<i64>* prefix, Array* mmg,
                            Array* mme) {
    Impl& I = *impl_;
    I.enter();
    I.check_cur(cur);
    PhaseTrace tr_(relu_crt ? "relu" : "sign");
    const int64_t N = I.cur_N;
    const int k = I.k;
    std::vector<void*> tmp;
    const bool relu = relu_crt != nullptr;
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
    tr_.mark("alloc");
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
    g.S = S;
    g.PB = I.pbank(std::max<size_t>(2, L.pays.size()), N);
    g.N = N;
    g.nslots = L.nslots;
    run_sign(I.c, L, g, in, tb, tmp);
    std::vector<int> omods = relu ? I.crt : sp.out_mod;
    std::vector<DevBlock> out = I.alloc_labels(omods, N);
    if (relu) {
        // mixed-mult draws (stream slot 2, counters run over the residues) and the g/e projections
        std::vector<gg::Draw> dr;
        std::vector<gg::Proj> pr;
        int ctr = 0;
        int64_t first = 0;
        for (int j = 0; j < k; ++j) {
            const int p = I.crt[j], n = nr_comps(p);
            dr.push_back({sk0 + 2 * j, p, ctr});
            ctr += prg_blocks(p);
            dr.push_back({sk0 + 2 * j + 1, p, ctr});
            ctr += prg_blocks(p);
        }
        for (int j = 0; j < k; ++j) {
            const int p = I.crt[j];
            gg::Proj a{gg::S_INPUT, j, p, sk0 + 2 * j, p, gg::F_MULR, j, 0, 0, gg::R_BANK, 0, 4, 1, (*prefix)[j], first};
            first += p;
            pr.push_back(a);
        }
        for (int j = 0; j < k; ++j) {
            const int p = I.crt[j];
            gg::Proj b{gg::S_SLOT, L.out_slot0, 2, sk0 + 2 * j + 1, p, gg::F_NEGR, j, 0, 0, gg::R_INPUT, j, 5, 1,
                       static_cast<int64_t>(j) * 3, first};
            first += 2;
            pr.push_back(b);
        }
        // the e table row is [k][3]: projection entries land at j*3 + color
        gg::Gadget gm = g;
        gm.sslot = 2;
        gm.draws = gg::dconst(dr.data(), dr.size());
        gm.ndraws = static_cast<int>(dr.size());
        gm.projs = gg::dconst(pr.data(), pr.size());
        gm.nprojs = static_cast<int>(pr.size());
        gm.entries = first;
        gm.nblk = draw_blocks(dr);
        check_desc(gm);
        hipLaunchKernelGGL(gg::k_draw, dim3(blocks_for(N * gm.nblk, gg::kGB, 8192)), dim3(gg::kGB), 0, gg::tl_st, I.c, gm);
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
    gg::end_layer(tmp);
    tr_.mark("kernels");
    tA.to_array(ap, I.device);
    if (sp.has_cast1()) t1.to_array(c1, I.device);
    t2.to_array(c2, I.device);
    tS.to_array(sg, I.device);
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
    // the payload bank is sized once for both users: rows 0-1 hold the trans key hashes until the sign gadget's
    // k_payloads (later on the same stream) overwrites them
    u128* PB = I.pbank(std::max<size_t>(2, L.pays.size()), N);
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
    g.PB = I.pbank(std::max<size_t>(2, L.pays.size()), N);
    g.N = N;
    g.nslots = L.nslots;
    run_sign(I.c, L, g, in, tb, tmp);
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
        f2 += p;
        pm.push_back(q);
    }
    for (int j = 0; j < k; ++j) {
        const int p = I.crt[j];
        gg::Proj q{gg::S_SLOT, sig_slot, 2, sk0 + 2 * j + 1, p, gg::F_NEGR, j, 0, 0, gg::R_INPUT, j, 5, 1,
                   static_cast<int64_t>(j) * 3, f2};
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
    hipLaunchKernelGGL(gg::k_draw, dim3(blocks_for(N * gm.nblk, gg::kGB, 8192)), dim3(gg::kGB), 0, gg::tl_st, I.c, gm);
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
    g.flut = gg::dconst(flut.data(), flut.size());
    g.fan = gg::dconst(fan.data(), fan.size());
    check_desc(g);
    std::vector<void*> tmp;
    hipLaunchKernelGGL(gg::k_draw, dim3(blocks_for(N * g.nblk, gg::kGB, 8192)), dim3(gg::kGB), 0, gg::tl_st, I.c, g);
    hipLaunchKernelGGL(gg::k_mrs_sign_derive, dim3(blocks_for(N, 256), k), dim3(256), 0, gg::tl_st, I.c, g, in, a);
    project(I.c, g, in, tb, pr);
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
    std::vector<int> fan, fbank;
    std::vector<int16_t> flut;
    std::vector<gg::PayDesc> pays;
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
        first += P.crt[r0];
        pr.push_back(p);
    }
    {
        const int a0 = static_cast<int>(flut.size()), a1 = static_cast<int>(fan.size());
        for (int v = 0; v < P.T; ++v)
            for (int j = 0; j < k; ++j) flut.push_back(static_cast<int16_t>(P.final_fn(j, v)));
        for (int j = 0; j < k; ++j) fan.push_back(P.crt[j]);
        // T entries but only p_j distinct payloads per target j: payload bank rows fin_j + f * R_{p_j}
        fbank.assign(fan.size(), 0);
        for (int j = 0; j < k; ++j) {
            fbank[a1 + j] = static_cast<int>(pays.size()) + 1;
            for (int f = 0; f < P.crt[j]; ++f) pays.push_back(gg::PayDesc{a.fin0 + j, P.crt[j], f});
        }
        gg::Proj p{};
        p.in_kind = gg::S_SLOT; p.in_idx = a.acc; p.pin = static_cast<int>(P.T);
        p.out_slot = a.fin0; p.pout = P.crt[0]; p.fn = gg::F_FAN; p.a0 = a0; p.a1 = a1;
        p.outr_kind = gg::R_BANK; p.table = 0; p.stride = k; p.off = P.fin_off; p.first = first;
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
    g.PB = I.pbank(std::max<size_t>(1, pays.size()), N);
    g.N = N;
    g.nslots = nslots;
    g.draws = gg::dconst(dr.data(), dr.size());
    g.ndraws = static_cast<int>(dr.size());
    g.projs = gg::dconst(pr.data(), pr.size());
    g.nprojs = static_cast<int>(pr.size());
    g.entries = first;
    g.nblk = draw_blocks(dr);
    g.flut = gg::dconst(flut.data(), flut.size());
    g.fan = gg::dconst(fan.data(), fan.size());
    g.fbank = gg::dconst(fbank.data(), fbank.size());
    check_desc(g);
    gg::In in{};
    std::vector<void*> tmp;
    hipLaunchKernelGGL(gg::k_draw, dim3(blocks_for(N * g.nblk, gg::kGB, 8192)), dim3(gg::kGB), 0, gg::tl_st, I.c, g);
    if (!pays.empty()) {
        const gg::PayDesc* pd = gg::dconst(pays.data(), pays.size());
        const int npd = static_cast<int>(pays.size());
        hipLaunchKernelGGL(gg::k_payloads, dim3(blocks_for(N * npd, 256, 16384)), dim3(256), 0, gg::tl_st, I.c, g, pd, npd);
    }
    hipLaunchKernelGGL(gg::k_mrs_derive, dim3(blocks_for(N, 256), k + 1), dim3(256), 0, gg::tl_st, I.c, g, a);
    project(I.c, g, in, tb, pr);
    if (P.sign_last) {
        // residue 0's key slot is the sign label of the ReLU that follows (relu_mult)
        I.sig.alloc(I.device, static_cast<size_t>(N) * gg::kW * sizeof(int16_t));
        I.sig_N = N;
        // the mod-2 key slot is a contiguous component-major block [128][N]
        HIPCHECK(hipMemcpyAsync(I.sig.p, gg::slot_base(g, a.key0), static_cast<size_t>(N) * gg::kW * sizeof(int16_t),
                                hipMemcpyDeviceToDevice, gg::tl_st));
    }
    HIPCHECK(hipGetLastError());
    gg::end_layer(tmp);
    tr_.mark("kernels");
    tT.to_array(tab, I.device);
    set_stale(cur, I.cur_mod, N);
}

// ReLU whose sign came out of the preceding mixed-radix rescale (RescaleMrsPlan::sign_last, I.sig): the
// mixed-modulus half gates only; device cur -> next base labels.
void GpuGarbler::relu_mult(uint64_t layer, CrtLabels& cur, const std::vector<i64>* prefix, Array& mmg, Array& mme) {
    Impl& I = *impl_;
    I.enter();
    I.check_cur(cur);
    PhaseTrace tr_("relu_mult");
    const int64_t N = I.cur_N;
    const int k = I.k;
    DASH_CHECK(I.sig.p && I.sig_N == N, "gpu garbler: joint ReLU without a preceding sign-producing rescale");
    const int sig_slot = 0, sk0 = 1, nslots = 1 + 2 * k;
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
    g.N = N;
    g.nslots = nslots;
    HIPCHECK(hipMemcpyAsync(gg::slot_base(g, sig_slot), I.sig.p, static_cast<size_t>(N) * gg::kW * sizeof(int16_t),
                            hipMemcpyDeviceToDevice, gg::tl_st));
    std::vector<DevBlock> out = relu_mult_gates(I, g, in, tb, sig_slot, sk0, *prefix);
    HIPCHECK(hipGetLastError());
    std::vector<void*> tmp;
    gg::end_layer(tmp);
    tr_.mark("kernels");
    tG.to_array(mmg, I.device);
    tE.to_array(mme, I.device);
    I.cur = std::move(out);
    I.sig = DevBlock();
    I.sig_N = 0;
    set_stale(cur, I.crt, N);
}

}  // namespace dash
