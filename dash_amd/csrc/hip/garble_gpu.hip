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
#include <memory>

#include "../layers.h"
#include "dev.h"
#include "gpu_garbler.h"
#include "kargs.h"
#include "host_util.h"

namespace dash {
using namespace dev;
using namespace hostutil;

namespace gg {

constexpr int kW = 128;  // label slot width (max components)

// label reference kinds
enum Src : int { S_INPUT = 0, S_SLOT = 1, S_ZERO = 2 };
// projection functions
enum Fn : int { F_IDENT = 0, F_LUT = 1, F_DIV = 2, F_SIGN = 3, F_MULR = 4, F_NEGR = 5 };
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

// input labels: per residue a label-major array [N][n_j]
struct In {
    const int16_t* p[kMaxRes];
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

// Prg::label (core.h): two components per AES-CTR block
__device__ __forceinline__ void prg_label(const AesCtx& a, const uint32_t* rk, uint64_t stream, uint64_t ctr,
                                          const ModC& m, int16_t* out) {
    const int n = static_cast<int>(m.n);
    for (int j = 0; j < n; j += 2) {
        const u128 blk = (static_cast<u128>(stream) << 64) | (ctr + static_cast<uint64_t>(j >> 1));
        const u128 r = aes_keyed(a, blk, rk);
        out[j] = static_cast<int16_t>(modq64(static_cast<uint64_t>(r), m));
        if (j + 1 < n) out[j + 1] = static_cast<int16_t>(modq64(static_cast<uint64_t>(r >> 64), m));
    }
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
    uint64_t layer, sslot, mask;  // PRG stream of this gadget: stream_of(layer, sslot, e, mask)
    int16_t* S;       // scratch [N][nslots][kW]
    int64_t N;
};

// one thread per (element, draw)
__global__ __launch_bounds__(256) void k_draw(Ctx c, Gadget g) {
    __shared__ uint32_t lds_aes[DASH_AES_LDS_WORDS];
    aes_lds_fill(lds_aes, c.te0);
    const AesCtx aes = aes_ctx(lds_aes, nullptr);
    const int64_t total = g.N * g.ndraws;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t e = i / g.ndraws;
        const Draw d = g.draws[i % g.ndraws];
        int16_t* out = g.S + (e * g.nslots + d.slot) * kW;
        prg_label(aes, c.rk, stream_of(g.layer, g.sslot, static_cast<uint64_t>(e), g.mask), d.ctr, c.mc[d.q], out);
    }
}

__device__ __forceinline__ const int16_t* label_ref(const Ctx& c, const Gadget& g, const In& in, int64_t e, int kind,
                                                    int idx, int q) {
    if (kind == S_INPUT) return in.p[idx] + e * in.n[idx];
    if (kind == S_SLOT) return g.S + (e * g.nslots + idx) * kW;
    return c.Z + static_cast<int64_t>(q) * kW;
}

// sign derive: sum2[q] = sum_{j<=k} bases[q][j]; sum = carry_final + sum_j mrs[j][0]
struct SignSlots {
    int k, t;
    int mrs[kMaxMrs];
    int sum2_slot0, sum_slot, bases_slot0, newc_slot0, mrs_slot0, stride_q;  // stride_q = k + 2
};

__global__ __launch_bounds__(256) void k_sign_derive(Ctx c, Gadget g, SignSlots s) {
    const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (e >= g.N) return;
    int16_t* S = g.S + e * g.nslots * kW;
    const int k = s.k, t = s.t;
    for (int q = 0; q + 1 < t; ++q) {
        const int d = t - 1 - q;
        const int mo = (k + 1) * s.mrs[d];
        const ModC Mo = c.mc[mo];
        const int n = static_cast<int>(Mo.n);
        int16_t* dst = S + (s.sum2_slot0 + q) * kW;
        const int16_t* b0 = S + (s.bases_slot0 + q * s.stride_q) * kW;
        for (int i = 0; i < n; ++i) {
            int v = 0;
            for (int j = 0; j <= k; ++j) v += b0[j * kW + i];
            dst[i] = static_cast<int16_t>(modq(static_cast<uint32_t>(v), Mo));
        }
    }
    const int m0 = s.mrs[0];
    const int n0 = static_cast<int>(c.mc[m0].n);
    const int16_t* carry = t >= 2 ? S + (s.newc_slot0 + (t - 2) * s.stride_q) * kW : c.Z + static_cast<int64_t>(m0) * kW;
    int16_t* sum = S + s.sum_slot * kW;
    for (int i = 0; i < n0; ++i) {
        int v = carry[i];
        for (int j = 0; j < k; ++j) v += S[(s.mrs_slot0 + j * t) * kW + i];
        sum[i] = static_cast<int16_t>(modq(static_cast<uint32_t>(v), c.mc[m0]));
    }
}

// one thread per (element, table entry)
__global__ __launch_bounds__(256) void k_project(Ctx c, Gadget g, In in, Tables tb) {
    __shared__ uint32_t lds_aes[DASH_AES_LDS_WORDS];
    aes_lds_fill(lds_aes, c.te0);
    const AesCtx aes = aes_ctx(lds_aes, nullptr);
    const int64_t total = g.N * g.entries;
    for (int64_t gi = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; gi < total;
         gi += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t e = gi / g.entries;
        const int64_t r = gi % g.entries;
        int lo = 0, hi = g.nprojs - 1;
        while (lo < hi) {  // last projection with first <= r
            const int mid = (lo + hi + 1) >> 1;
            if (g.projs[mid].first <= r) lo = mid;
            else hi = mid - 1;
        }
        const Proj P = g.projs[lo];
        const int i = static_cast<int>(r - P.first);
        const ModC mi = c.mc[P.pin], mo = c.mc[P.pout];
        const int16_t* inl = label_ref(c, g, in, e, P.in_kind, P.in_idx, P.pin);
        const int16_t* Rin = c.R + static_cast<int64_t>(P.pin) * kW;
        // key = in + i*Rin (mod pin), compressed streaming from the least significant digit
        CompressFwd kc;
        kc.init();
        uint32_t color = 0;
        for (int q = 0; q < static_cast<int>(mi.n); ++q) {
            const uint32_t v = modq(static_cast<uint32_t>(inl[q] + i * Rin[q]), mi);
            if (q == 0) color = v;
            kc.push(v, mi);
        }
        const u128 H = aes_encrypt(aes, kc.finish());
        // function value
        int64_t f;
        switch (P.fn) {
            case F_LUT: f = c.lut[c.lut_off[P.a0] + i * P.a2 + P.a1]; break;  // a0 = j, a1 = d, a2 = t
            case F_DIV: f = i / P.a0; break;
            case F_SIGN: f = i < P.a0 ? P.a2 : P.a1; break;  // a0 = half, a1 = lower, a2 = upper
            case F_MULR: {
                const int16_t* x = label_ref(c, g, in, e, S_INPUT, P.a0, 0);
                f = static_cast<int64_t>(i) * x[0];
                break;
            }
            case F_NEGR: {
                const int16_t* x = label_ref(c, g, in, e, S_INPUT, P.a0, 0);
                f = -(static_cast<int64_t>(i) + x[0]);
                break;
            }
            default: f = i;
        }
        int64_t cm = f % P.pout;
        if (cm < 0) cm += P.pout;
        const int16_t* ol = g.S + (e * g.nslots + P.out_slot) * kW;
        const int16_t* oR = P.outr_kind == R_BANK ? c.R + static_cast<int64_t>(P.pout) * kW
                                                  : label_ref(c, g, in, e, S_INPUT, P.outr_idx, 0);
        CompressFwd pc;
        pc.init();
        for (int q = 0; q < static_cast<int>(mo.n); ++q) {
            // ol, cm, oR in [0, pout): < pout^2 + pout, 32-bit reduction
            pc.push(modq(static_cast<uint32_t>(ol[q]) + static_cast<uint32_t>(cm) * static_cast<uint32_t>(oR[q]), mo), mo);
        }
        tb.t[P.table][e * tb.row[P.table] + P.off + static_cast<int64_t>(color) * P.stride] = pc.finish() + H;
    }
}

// ReLU mixed-mod half gates beyond the g/e projections: mini gate payloads
// (16-bit, e[q]) and the output base labels out0[j] = sk04 - sk03.
struct MiniArgs {
    int k;
    int crt[kMaxRes];
    int sig_slot, sk_slot0;  // sk03_j = sk_slot0 + 2j, sk04_j = +1
    int16_t* out[kMaxRes];   // next base labels [N][n_j]
};

__global__ __launch_bounds__(256) void k_relu_finish(Ctx c, Gadget g, In in, Tables tb, MiniArgs m) {
    __shared__ uint32_t lds_aes[DASH_AES_LDS_WORDS];
    aes_lds_fill(lds_aes, c.te0);
    const AesCtx aes = aes_ctx(lds_aes, nullptr);
    const int64_t total = g.N * m.k;
    for (int64_t gi = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; gi < total;
         gi += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t e = gi / m.k;
        const int j = static_cast<int>(gi % m.k);
        const int p = m.crt[j];
        const int16_t* x = in.p[j] + e * in.n[j];
        const int16_t* sig = g.S + (e * g.nslots + m.sig_slot) * kW;
        const ModC m2 = c.mc[2];
        const int16_t* R2 = c.R + 2 * kW;
        const int r = x[0];
        // mini gate y -> (y + r) mod p, 16-bit payload at t16[color] of entry e[k][2]
        int16_t* t16 = reinterpret_cast<int16_t*>(tb.t[5] + (e * m.k + j) * 3 + 2);
        for (int i = 0; i < 2; ++i) {
            CompressFwd kc;
            kc.init();
            uint32_t color = 0;
            for (int q = 0; q < static_cast<int>(m2.n); ++q) {
                const uint32_t v = static_cast<uint32_t>(sig[q] + i * R2[q]) & 1u;
                if (q == 0) color = v;
                kc.push(v, m2);
            }
            const u128 H = aes_encrypt(aes, kc.finish());
            const int fv = (i + r) % p;
            t16[color] = static_cast<int16_t>(static_cast<int16_t>(fv) + static_cast<int16_t>(static_cast<uint16_t>(H)));
        }
        const int16_t* s3 = g.S + (e * g.nslots + m.sk_slot0 + 2 * j) * kW;
        const int16_t* s4 = s3 + kW;
        int16_t* o = m.out[j] + e * in.n[j];
        for (int q = 0; q < in.n[j]; ++q) {
            int v = s4[q] - s3[q];
            o[q] = static_cast<int16_t>(v < 0 ? v + p : v);
        }
    }
}

// Legacy rescale, before the sign gadget: L += up; trans projections of the
// mod-2 residue into every other residue; L_j = (L_j - out0_j) * 2^-1; L_0 = Z_2.
struct RsArgs {
    int k;
    int crt[kMaxRes];
    int inv[kMaxRes];
    int16_t* L[kMaxRes];       // [N][n_j], updated in place
    const int16_t* up;         // [k][kW]
    const int16_t* down;       // [k][kW]
    uint64_t layer, sslot;     // trans stream = stream_of(layer, sslot, e, 0)
};

__global__ __launch_bounds__(256) void k_rescale_pre(Ctx c, RsArgs a, Tables tb, int64_t N) {
    __shared__ uint32_t lds_aes[DASH_AES_LDS_WORDS];
    aes_lds_fill(lds_aes, c.te0);
    const AesCtx aes = aes_ctx(lds_aes, nullptr);
    for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < N;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        for (int j = 0; j < a.k; ++j) {
            const int p = a.crt[j], n = static_cast<int>(c.mc[p].n);
            int16_t* L = a.L[j] + e * n;
            for (int q = 0; q < n; ++q) {
                int v = L[q] + a.up[j * kW + q];
                L[q] = static_cast<int16_t>(v >= p ? v - p : v);
            }
        }
        const uint64_t stream = stream_of(a.layer, a.sslot, static_cast<uint64_t>(e), 0);
        uint64_t ctr = 0;
        int16_t out0[kW];
        const int16_t* L0 = a.L[0] + e * c.mc[2].n;
        const ModC m2 = c.mc[2];
        for (int j = 1; j < a.k; ++j) {
            const int p = a.crt[j];
            const ModC mj = c.mc[p];
            prg_label(aes, c.rk, stream, ctr, mj, out0);
            ctr += (mj.n + 1) / 2;
            const int16_t* Rp = c.R + static_cast<int64_t>(p) * kW;
            for (int i = 0; i < 2; ++i) {
                CompressFwd kc;
                kc.init();
                uint32_t color = 0;
                for (int q = 0; q < static_cast<int>(m2.n); ++q) {
                    const uint32_t v = static_cast<uint32_t>(L0[q] + i * c.R[2 * kW + q]) & 1u;
                    if (q == 0) color = v;
                    kc.push(v, m2);
                }
                const u128 H = aes_encrypt(aes, kc.finish());
                CompressFwd pc;
                pc.init();
                for (int q = 0; q < static_cast<int>(mj.n); ++q)
                    pc.push(modq(static_cast<uint32_t>(out0[q] + i * Rp[q]), mj), mj);
                tb.t[6][e * tb.row[6] + (j - 1) * 2 + color] = pc.finish() + H;
            }
            int16_t* L = a.L[j] + e * mj.n;
            for (int q = 0; q < static_cast<int>(mj.n); ++q) {
                int v = L[q] - out0[q];
                if (v < 0) v += p;
                L[q] = static_cast<int16_t>(modq(static_cast<uint32_t>(v * a.inv[j]), mj));
            }
        }
        int16_t* Lz = a.L[0] + e * m2.n;
        for (int q = 0; q < static_cast<int>(m2.n); ++q) Lz[q] = c.Z[2 * kW + q];
    }
}

// After the sign gadget: L_0 = sign output; L -= down.
__global__ __launch_bounds__(256) void k_rescale_post_g(Ctx c, RsArgs a, Gadget g, int sig_slot) {
    const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (e >= g.N) return;
    const int16_t* sig = g.S + (e * g.nslots + sig_slot) * kW;
    for (int j = 0; j < a.k; ++j) {
        const int p = a.crt[j], n = static_cast<int>(c.mc[p].n);
        int16_t* L = a.L[j] + e * n;
        for (int q = 0; q < n; ++q) {
            int v = (j == 0 ? sig[q] : L[q]) - a.down[j * kW + q];
            L[q] = static_cast<int16_t>(v < 0 ? v + p : v);
        }
    }
}

// ------------------------------------------------------------------- host
struct SignLayout {
    std::vector<Draw> draws;
    std::vector<Proj> projs;
    SignSlots ss{};
    int nslots = 0;
    int out_slot0 = 0;
    int64_t entries = 0;
};

// Mirrors sign_garble_elem: draw order = PRG counter order.
SignLayout sign_layout(const SignPlan& P, int extra_slots) {
    SignLayout L;
    const int k = static_cast<int>(P.crt.size()), t = static_cast<int>(P.mrs.size());
    int slot = 0, ctr = 0;
    auto draw = [&](int q) {
        L.draws.push_back({slot, q, ctr});
        ctr += (nr_comps(q) + 1) / 2;
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
    for (int d = 0; d < t; ++d) L.ss.mrs[d] = P.mrs[d];
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
    for (int j = 0; j < k; ++j)
        for (int d = 0; d < t; ++d)
            add(Proj{S_INPUT, j, P.crt[j], mrs0 + j * t + d, P.mrs[d], F_LUT, j, d, t, R_BANK, 0, 0, t,
                     t * P.crt_prefix[j] + d, 0});
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
        add(Proj{S_SLOT, sum_slot, m0, L.out_slot0 + static_cast<int>(o), P.out_mod[o], F_SIGN, m0 / 2, P.lower,
                 P.upper, R_BANK, 0, 3, 1, static_cast<int64_t>(o) * m0, 0});
    L.entries = first;
    return L;
}

template <class T>
T* dput(const T* h, size_t n, std::vector<void*>& owned) {
    T* d = nullptr;
    HIPCHECK(hipMalloc(reinterpret_cast<void**>(&d), std::max<size_t>(1, n) * sizeof(T)));
    if (n) HIPCHECK(hipMemcpy(d, h, n * sizeof(T), hipMemcpyHostToDevice));
    owned.push_back(d);
    return d;
}

}  // namespace gg

struct GpuGarbler::Impl {
    gg::Ctx c{};
    std::vector<void*> owned;
    int max_mod = 0;
    std::vector<int> crt;
    int k = 0;
    int device = 0;
    ~Impl() {
        for (void* p : owned) (void)hipFree(p);
    }
};

GpuGarbler::GpuGarbler(const std::vector<int>& crt, const std::vector<int>& mrs, const std::string& seed16,
                       const LabelBank& R, const LabelBank& Z, int device)
    : impl_(new Impl) {
    HIPCHECK(hipSetDevice(device));
    Impl& I = *impl_;
    I.device = device;
    I.crt = crt;
    I.k = static_cast<int>(crt.size());
    I.max_mod = R.max_mod;
    std::vector<int16_t> hR((R.max_mod + 1) * gg::kW, 0), hZ((R.max_mod + 1) * gg::kW, 0);
    for (int p = 2; p <= R.max_mod; ++p) {
        if (R.lab[p].empty()) continue;
        std::copy(R.lab[p].begin(), R.lab[p].end(), hR.begin() + p * gg::kW);
        std::copy(Z.lab[p].begin(), Z.lab[p].end(), hZ.begin() + p * gg::kW);
    }
    I.c.R = gg::dput(hR.data(), hR.size(), I.owned);
    I.c.Z = gg::dput(hZ.data(), hZ.size(), I.owned);
    std::vector<dev::ModC> mc(R.max_mod + 1);
    for (int q = 2; q <= R.max_mod; ++q) mc[q] = make_modc(q);
    I.c.mc = gg::dput(mc.data(), mc.size(), I.owned);
    auto te = make_te0();
    I.c.te0 = gg::dput(te.data(), te.size(), I.owned);
    auto rk = round_key_words(reinterpret_cast<const uint8_t*>(seed16.data()));
    std::copy(rk.begin(), rk.end(), I.c.rk);
    if (!mrs.empty()) {
        auto lut = gen_approx_lookup(crt, mrs);
        std::vector<int16_t> flat;
        for (int j = 0; j < I.k; ++j) {
            I.c.lut_off[j] = static_cast<int>(flat.size());
            flat.insert(flat.end(), lut[j].begin(), lut[j].end());
        }
        I.c.lut = gg::dput(flat.data(), flat.size(), I.owned);
    }
}

GpuGarbler::~GpuGarbler() = default;

namespace {
inline unsigned blocks_for(int64_t n, int bs, int cap = 65536) {
    return static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((n + bs - 1) / bs, cap)));
}

struct DevLabels {
    std::vector<int16_t*> p;
    std::vector<void*> owned;
    ~DevLabels() {
        for (void* q : owned) (void)hipFree(q);
    }
};

void upload_labels(const CrtLabels& L, DevLabels& d) {
    for (const auto& l : L) {
        int16_t* x = nullptr;
        HIPCHECK(hipMalloc(reinterpret_cast<void**>(&x), std::max<size_t>(1, l.c.size()) * sizeof(int16_t)));
        HIPCHECK(hipMemcpy(x, l.c.data(), l.c.size() * sizeof(int16_t), hipMemcpyHostToDevice));
        d.p.push_back(x);
        d.owned.push_back(x);
    }
}

void download_labels(const DevLabels& d, CrtLabels& L) {
    for (size_t j = 0; j < L.size(); ++j)
        HIPCHECK(hipMemcpy(L[j].c.data(), d.p[j], L[j].c.size() * sizeof(int16_t), hipMemcpyDeviceToHost));
}

struct DevTable {
    u128* p = nullptr;
    int64_t row = 0;
    size_t bytes = 0;
    ~DevTable() {
        if (p) (void)hipFree(p);
    }
    void alloc(int64_t N, int64_t r) {
        row = r;
        bytes = static_cast<size_t>(N) * r * sizeof(u128);
        HIPCHECK(hipMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(16, bytes)));
        HIPCHECK(hipMemset(p, 0, std::max<size_t>(16, bytes)));
    }
    // hand the buffer to `a` as a device-resident array (kept in HBM; the
    // evaluator on this node copies it device-to-device)
    void to_array(Array& a, int device) {
        DASH_CHECK(a.nbytes == bytes, "gpu garbler: table size mismatch");
        auto d = std::make_shared<Array::Device>();
        d->p = std::shared_ptr<void>(p, [](void* x) { (void)hipFree(x); });
        p = nullptr;
        d->device = device;
        d->fetch = [device](void* h, const void* dv, size_t n) {
            HIPCHECK(hipSetDevice(device));
            HIPCHECK(hipMemcpy(h, dv, n, hipMemcpyDeviceToHost));
        };
        a = Array::on_device(a.dtype, a.shape, std::move(d));
    }
};

// run the three sign-gadget passes for N elements with input labels `in`
void run_sign(const gg::Ctx& c, const gg::SignLayout& L, gg::Gadget& g, const gg::In& in, const gg::Tables& tb,
              std::vector<void*>& tmp) {
    g.draws = gg::dput(L.draws.data(), L.draws.size(), tmp);
    g.ndraws = static_cast<int>(L.draws.size());
    g.projs = gg::dput(L.projs.data(), L.projs.size(), tmp);
    g.nprojs = static_cast<int>(L.projs.size());
    g.entries = L.entries;
    hipLaunchKernelGGL(gg::k_draw, dim3(blocks_for(g.N * g.ndraws, 256, 8192)), dim3(256), 0, nullptr, c, g);
    hipLaunchKernelGGL(gg::k_sign_derive, dim3(blocks_for(g.N, 256)), dim3(256), 0, nullptr, c, g, L.ss);
    hipLaunchKernelGGL(gg::k_project, dim3(blocks_for(g.N * g.entries, 256, 16384)), dim3(256), 0, nullptr, c, g, in,
                       tb);
    HIPCHECK(hipGetLastError());
}
}  // namespace

void GpuGarbler::sign_layer(uint64_t layer, const SignPlan& sp, const CrtLabels& cur, Array& ap, Array& c1, Array& c2,
                            Array& sg, CrtLabels& out, const std::vector<int>* relu_crt, const std::vector<i64>* prefix,
                            Array* mmg, Array* mme) {
    Impl& I = *impl_;
    const int64_t N = cur[0].N;
    const int k = I.k;
    std::vector<void*> tmp;
    DevLabels din;
    upload_labels(cur, din);
    const bool relu = relu_crt != nullptr;
    // relu: 2 slots per residue for the mixed-mult output labels sk03/sk04
    gg::SignLayout L = gg::sign_layout(sp, relu ? 2 * k : 0);
    int sk0 = L.nslots - (relu ? 2 * k : 0);
    int16_t* S = nullptr;
    HIPCHECK(hipMalloc(reinterpret_cast<void**>(&S), static_cast<size_t>(N) * L.nslots * gg::kW * sizeof(int16_t)));
    tmp.push_back(S);
    DevTable tA, t1, t2, tS, tG, tE;
    tA.alloc(N, ap.shape[1]);
    t1.alloc(N, c1.shape[1]);
    t2.alloc(N, c2.shape[1]);
    tS.alloc(N, sg.shape[1]);
    gg::Tables tb{};
    tb.t[0] = tA.p; tb.row[0] = tA.row;
    tb.t[1] = t1.p; tb.row[1] = t1.row;
    tb.t[2] = t2.p; tb.row[2] = t2.row;
    tb.t[3] = tS.p; tb.row[3] = tS.row;
    if (relu) {
        tG.alloc(N, mmg->shape[1]);
        tE.alloc(N, static_cast<int64_t>(k) * 3);
        tb.t[4] = tG.p; tb.row[4] = tG.row;
        tb.t[5] = tE.p; tb.row[5] = tE.row;
    }
    gg::In in{};
    for (int j = 0; j < k; ++j) {
        in.p[j] = din.p[j];
        in.n[j] = nr_comps(I.crt[j]);
    }
    gg::Gadget g{};
    g.layer = layer;
    g.sslot = 1;
    g.mask = 0;
    g.S = S;
    g.N = N;
    g.nslots = L.nslots;
    run_sign(I.c, L, g, in, tb, tmp);
    DevLabels dout;
    if (relu) {
        // mixed-mult draws (stream slot 2, counters run over the residues) and the g/e projections
        std::vector<gg::Draw> dr;
        std::vector<gg::Proj> pr;
        int ctr = 0;
        int64_t first = 0;
        for (int j = 0; j < k; ++j) {
            const int p = I.crt[j], n = nr_comps(p);
            dr.push_back({sk0 + 2 * j, p, ctr});
            ctr += (n + 1) / 2;
            dr.push_back({sk0 + 2 * j + 1, p, ctr});
            ctr += (n + 1) / 2;
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
        gm.draws = gg::dput(dr.data(), dr.size(), tmp);
        gm.ndraws = static_cast<int>(dr.size());
        gm.projs = gg::dput(pr.data(), pr.size(), tmp);
        gm.nprojs = static_cast<int>(pr.size());
        gm.entries = first;
        hipLaunchKernelGGL(gg::k_draw, dim3(blocks_for(N * gm.ndraws, 256, 8192)), dim3(256), 0, nullptr, I.c, gm);
        hipLaunchKernelGGL(gg::k_project, dim3(blocks_for(N * gm.entries, 256, 16384)), dim3(256), 0, nullptr, I.c, gm,
                           in, tb);
        gg::MiniArgs ma{};
        ma.k = k;
        for (int j = 0; j < k; ++j) ma.crt[j] = I.crt[j];
        ma.sig_slot = L.out_slot0;
        ma.sk_slot0 = sk0;
        for (int j = 0; j < k; ++j) {
            int16_t* x = nullptr;
            HIPCHECK(hipMalloc(reinterpret_cast<void**>(&x), out[j].c.size() * sizeof(int16_t)));
            dout.p.push_back(x);
            dout.owned.push_back(x);
            ma.out[j] = x;
        }
        hipLaunchKernelGGL(gg::k_relu_finish, dim3(blocks_for(N * k, 256, 8192)), dim3(256), 0, nullptr, I.c, gm, in,
                           tb, ma);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipDeviceSynchronize());
        download_labels(dout, out);
        tG.to_array(*mmg, I.device);
        tE.to_array(*mme, I.device);
    } else {
        HIPCHECK(hipDeviceSynchronize());
        // sign layer outputs: out0[o] slots (one per CRT residue) -> label-major host labels
        std::vector<int16_t> hs(static_cast<size_t>(N) * L.nslots * gg::kW);
        HIPCHECK(hipMemcpy(hs.data(), S, hs.size() * sizeof(int16_t), hipMemcpyDeviceToHost));
        for (int o = 0; o < k; ++o) {
            const int n = out[o].n;
            for (int64_t e = 0; e < N; ++e)
                std::memcpy(out[o].at(e), hs.data() + (e * L.nslots + L.out_slot0 + o) * gg::kW, n * sizeof(int16_t));
        }
    }
    tA.to_array(ap, I.device);
    t1.to_array(c1, I.device);
    t2.to_array(c2, I.device);
    tS.to_array(sg, I.device);
    for (void* p : tmp) (void)hipFree(p);
}

void GpuGarbler::rescale_legacy_iter(uint64_t layer, int it, const RescalePlan& P, CrtLabels& cur,
                                     const std::vector<std::vector<comp_t>>& up,
                                     const std::vector<std::vector<comp_t>>& down, Array& tr, Array& ap, Array& c1,
                                     Array& c2, Array& sg) {
    Impl& I = *impl_;
    const int64_t N = cur[0].N;
    const int k = I.k;
    std::vector<void*> tmp;
    DevLabels dL;
    upload_labels(cur, dL);
    std::vector<int16_t> hup(k * gg::kW, 0), hdn(k * gg::kW, 0);
    for (int j = 0; j < k; ++j) {
        std::copy(up[j].begin(), up[j].end(), hup.begin() + j * gg::kW);
        std::copy(down[j].begin(), down[j].end(), hdn.begin() + j * gg::kW);
    }
    gg::RsArgs ra{};
    ra.k = k;
    for (int j = 0; j < k; ++j) {
        ra.crt[j] = I.crt[j];
        ra.L[j] = dL.p[j];
        ra.inv[j] = 0;
    }
    // inverses of 2 for the active residues (plan order = residues 1..k-1)
    for (size_t a = 0; a < P.active[0].size(); ++a) ra.inv[P.active[0][a]] = static_cast<int>(P.inv[0][a]);
    ra.up = gg::dput(hup.data(), hup.size(), tmp);
    ra.down = gg::dput(hdn.data(), hdn.size(), tmp);
    ra.layer = layer;
    ra.sslot = 10 + it;
    DevTable tT, tA, t1, t2, tS;
    tT.alloc(N, tr.shape[1]);
    tA.alloc(N, ap.shape[1]);
    t1.alloc(N, c1.shape[1]);
    t2.alloc(N, c2.shape[1]);
    tS.alloc(N, sg.shape[1]);
    gg::Tables tb{};
    tb.t[0] = tA.p; tb.row[0] = tA.row;
    tb.t[1] = t1.p; tb.row[1] = t1.row;
    tb.t[2] = t2.p; tb.row[2] = t2.row;
    tb.t[3] = tS.p; tb.row[3] = tS.row;
    tb.t[6] = tT.p; tb.row[6] = tT.row;
    hipLaunchKernelGGL(gg::k_rescale_pre, dim3(blocks_for(N, 256, 4096)), dim3(256), 0, nullptr, I.c, ra, tb, N);
    gg::SignLayout L = gg::sign_layout(P.sign, 0);
    int16_t* S = nullptr;
    HIPCHECK(hipMalloc(reinterpret_cast<void**>(&S), static_cast<size_t>(N) * L.nslots * gg::kW * sizeof(int16_t)));
    tmp.push_back(S);
    gg::In in{};
    for (int j = 0; j < k; ++j) {
        in.p[j] = dL.p[j];
        in.n[j] = nr_comps(I.crt[j]);
    }
    gg::Gadget g{};
    g.layer = layer;
    g.sslot = 10 + it;
    g.mask = 1ull << 43;  // nested sign stream (rescale_garble_elem)
    g.S = S;
    g.N = N;
    g.nslots = L.nslots;
    run_sign(I.c, L, g, in, tb, tmp);
    hipLaunchKernelGGL(gg::k_rescale_post_g, dim3(blocks_for(N, 256)), dim3(256), 0, nullptr, I.c, ra, g, L.out_slot0);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipDeviceSynchronize());
    download_labels(dL, cur);
    tT.to_array(tr, I.device);
    tA.to_array(ap, I.device);
    t1.to_array(c1, I.device);
    t2.to_array(c2, I.device);
    tS.to_array(sg, I.device);
    for (void* p : tmp) (void)hipFree(p);
}

}  // namespace dash
