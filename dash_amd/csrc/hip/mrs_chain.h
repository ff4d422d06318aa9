// Mixed-radix chain kernels (gadgets.h RescaleMrsPlan / SignMrsPlan), per CRT size K. The templates live
// here and are instantiated per K in separate translation units (kernels_mrs_*.hip), so a change to the chain
// rebuilds a few K in parallel instead of one unit holding all K = 2..12 (docs/BUILD.md).
#pragma once

#include "gadget_common.h"

namespace dash {
namespace dev {

// ---------------------------------------------------------------------------
// Single-shot mixed-radix rescale (gadgets.h RescaleMrsPlan): the serial part
// runs one lane per (GC, element), K (the CRT size) is a template parameter so
// the payload matrix P[l][j] (digit l -> later residue j) lives in registers
// with static indices. Digit i's key is residue i's label minus the payloads
// of the earlier digits, streamed from HBM, compressed and hashed; its row
// ([color][K - i] contiguous entries) is gathered while the AES runs. The
// power-of-two label r = x_u mod 2S is accumulated packed (per-field adds, no
// decompress), its hash selects the final row; the K final payloads go to
// a.pf for the elementwise output kernel.
__device__ __forceinline__ u128 add_packed(u128 a, u128 b, u128 hmask) {
    return ((a & ~hmask) + (b & ~hmask)) ^ ((a ^ b) & hmask);
}

// Digit i's key streams residue i's label in chunks of kMrsChunk components,
// the next chunk's loads issued before the current one is consumed. The
// payloads P_{l,j} of digit l for later residues j go to a per-lane scratch
// (a.ps, [B][pair][N], coalesced) and are read back when digit j starts:
// holding them in registers (up to K(K-1)/2 u128) spilled.
#ifndef DASH_MRS_CHUNK
#define DASH_MRS_CHUNK 4  // 8: mode-2 chain spilled 84 B/lane, 4: 28 (mode 0: 52 -> 0); 24 GCs 13.07 -> 12.96 ms
#endif
constexpr int kMrsChunk = DASH_MRS_CHUNK;
#ifndef DASH_MRS_M2CH
#define DASH_MRS_M2CH 16  // components per load batch of the mod-2 key (modes 1, 2)
#endif
template <int K>
__device__ __forceinline__ constexpr int mrs_pair(int l, int j) {  // l < j < K
    return l * (2 * K - l - 1) / 2 + (j - l - 1);
}

// Hardened encoding (the only encoding of the mixed-radix constructions, docs/SECURITY.md): position i's row
// is unmasked with the pads of (key, gate, (TW_MRS | TW_SMRS, i)), the final row with (acc, gate, (TW_MRS, K)).
template <int MODE>
__device__ __forceinline__ constexpr uint32_t mrs_row_sub(int i) {
    return tw_sub(MODE == 1 ? kTwSmrs : kTwMrs, static_cast<uint32_t>(i));
}
// The sign label (mod 2) keys the next ReLU's k evaluator half gates and their minis: its y-row pads go to
// ys[b][s][e], s < ny (the ReLU multiply subtracts them instead of a shared H(key))
__device__ __forceinline__ void store_ypads(const MrsArgs& a, u128 key, int b, int64_t N, int64_t e) {
    const uint64_t g = a.rgate0 ^ static_cast<uint64_t>(e);
    for (int blk = 0; 4 * blk < a.ny; ++blk) {
        u128 p[4];
        hard_block(key, g, tw_sub(kTwMmy, 0), static_cast<uint32_t>(blk), p);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (4 * blk + q < a.ny) a.ys[(static_cast<int64_t>(b) * a.ny + 4 * blk + q) * N + e] = p[q];
    }
}

// MODE 1 (exact sign, gadgets.h SignMrsPlan): positions convert residues
// 1..K-1, the last position is residue 0 (mod 2): its key is the bit pack of
// L_0 XOR the K-1 payloads aimed at it (mod-2 subtraction), i.e. the sign
// label itself; only its hash and color are produced (the ReLU multiply).
// MODE 2 (joint rescale + ReLU sign, RescaleMrsPlan::sign_last): MODE 1's
// order with MODE 0's T target on every row (the mod-2 position's row has only
// that one) and final row; the mod-2 key's hash and color go to hs / cs.
#ifndef DASH_CHAIN2_WAVES
#define DASH_CHAIN2_WAVES 4  // mode 2 (joint rescale + sign) register budget in waves per SIMD
#endif
template <int K, int MODE>
__global__ __launch_bounds__(kAesBlock, MODE == 2 ? DASH_CHAIN2_WAVES : DASH_UA_MINBLOCKS) void k_mrs_chain(MrsArgs a, Act x, const ModC* mc,
                                                                          const uint32_t* te0, const uint32_t* rk) {
    (void)te0;
    (void)rk;
    const int b = blockIdx.z;
    const int64_t N = a.N;
    constexpr int NP = K * (K - 1) / 2 > 0 ? K * (K - 1) / 2 : 1;
    for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < N;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const u128* row0 = a.tab + (static_cast<int64_t>(b) * N + e) * a.n_tab;
        u128* PS = a.ps + static_cast<int64_t>(b) * NP * N + e;
        u128 acc = 0;
#pragma unroll
        for (int i = 0; i < (MODE >= 1 ? K - 1 : K); ++i) {
            const int r = MODE >= 1 ? (i + 1) % K : i;  // residue converted at position i
            const ModC m = mc[a.crt.p[r]];
            const int n = static_cast<int>(m.n);
            const act_t* L = x.p[r] + static_cast<int64_t>(b) * n * N + e;
            DigitStream ds[K > 1 ? K - 1 : 1];
#pragma unroll
            for (int l = 0; l < i; ++l) ds[l].init(PS[static_cast<int64_t>(mrs_pair<K>(l, i)) * N]);
            CompressFwd cf;
            cf.init();
            uint32_t col = 0;
            uint16_t cur[kMrsChunk], nxt[kMrsChunk];
#pragma unroll
            for (int u = 0; u < kMrsChunk; ++u)
                if (u < n) cur[u] = static_cast<uint16_t>(L[static_cast<int64_t>(u) * N]);
            for (int c0 = 0; c0 < n; c0 += kMrsChunk) {
#pragma unroll
                for (int u = 0; u < kMrsChunk; ++u)
                    if (c0 + kMrsChunk + u < n) nxt[u] = static_cast<uint16_t>(L[static_cast<int64_t>(c0 + kMrsChunk + u) * N]);
#pragma unroll
                for (int u = 0; u < kMrsChunk; ++u)
                    if (c0 + u < n) {
                        uint32_t d = cur[u];
#pragma unroll
                        for (int l = 0; l < i; ++l) {
                            const uint32_t s = ds[l].next(m);
                            d = d >= s ? d - s : d + m.q - s;
                        }
                        if (c0 + u == 0) col = d;
                        cf.push(d, m);
                    }
#pragma unroll
                for (int u = 0; u < kMrsChunk; ++u) cur[u] = nxt[u];
            }
            constexpr int kExtra = MODE == 1 ? 0 : 1;        // rescale rows end with the T target
            const int nt = K - 1 - i + kExtra;
            const u128* row = row0 + a.dig_off[i] + static_cast<int64_t>(col) * nt;
            u128 E[K];
#pragma unroll
            for (int t = 0; t < nt; ++t) E[t] = row[t];
            hard_unmask_n<K>(E, nt, cf.finish(), a.gate0 ^ static_cast<uint64_t>(e), mrs_row_sub<MODE>(i));
#pragma unroll
            for (int t = 0; t < K - 1 - i; ++t) PS[static_cast<int64_t>(mrs_pair<K>(i, i + 1 + t)) * N] = E[t];
            if (MODE != 1) acc = add_packed(acc, E[K - 1 - i], a.hmask);
        }
        if (MODE >= 1) {
            // last position: residue 0 (mod 2): compress = bit pack, subtraction = XOR
            const ModC m = mc[a.crt.p[0]];
            const act_t* L = x.p[0] + static_cast<int64_t>(b) * m.n * N + e;
            u128 key = compress_cm<DASH_MRS_M2CH>(L, N, m);
#pragma unroll
            for (int l = 0; l < K - 1; ++l) key ^= PS[static_cast<int64_t>(mrs_pair<K>(l, K - 1)) * N];
            const uint32_t c = static_cast<uint32_t>(key) & 1u;
            u128 E = 0;
            if (MODE == 2)  // the sign digit's T payload row (one entry)
                E = row0[a.dig_off[K - 1] + c] - hard_pad(key, a.gate0 ^ static_cast<uint64_t>(e), mrs_row_sub<MODE>(K - 1), 0);
            store_ypads(a, key, b, N, e);
            a.cs[static_cast<int64_t>(b) * N + e] = static_cast<uint8_t>(c);
            if (MODE == 2) acc = add_packed(acc, E, a.hmask);
        }
        if (MODE == 1) continue;
        const uint32_t col = static_cast<uint32_t>(acc) & static_cast<uint32_t>(a.T - 1);
        const u128* row = row0 + a.fin_off + static_cast<int64_t>(col) * K;
        u128 F[K];
#pragma unroll
        for (int j = 0; j < K; ++j) F[j] = row[j];
        hard_unmask<K>(F, acc, a.gate0 ^ static_cast<uint64_t>(e), mrs_row_sub<0>(K));
#pragma unroll
        for (int j = 0; j < K; ++j) a.pf[(static_cast<int64_t>(b) * K + j) * N + e] = F[j];
    }
}

// LDS-staged chain (N % 16 == 0, N >= kMrsBS): a block owns kMrsBS consecutive elements and walks the
// positions in lockstep; residue r's label bytes for the block are brought into LDS by the whole block,
// kMrsCap components per pass, as 16-byte loads that are all in flight at once, and each lane then reads its
// components from LDS. The per-lane form (k_mrs_chain) loaded one byte per lane per component, kMrsChunk
// at a time: ~n / 4 dependent HBM round trips per position, 65 % of its cycles waiting (r03 roofline:
// 0.87 TB/s fetched). Outputs, payload scratch and table gathers are per lane as before.
constexpr int kMrsBS = 512;   // elements (lanes) per block
constexpr int kMrsCap = 64;   // components staged per pass (kMrsCap * kMrsBS = 32 KiB)
#ifndef DASH_STAGE_U
#define DASH_STAGE_U 2  // 16-byte loads in flight per thread while staging (4 pushed the chain into spills)
#endif
constexpr int kStageU = DASH_STAGE_U;
#ifndef DASH_STAGE_RD
#define DASH_STAGE_RD 4  // LDS component reads batched per lane
#endif
constexpr int kStageRd = DASH_STAGE_RD;
// one position of k_mrs_chain_s, I a compile-time constant (constant stream counts and pair indices)
template <int K, int MODE, int I>
__device__ __forceinline__ void chain_s_pos(const MrsArgs& a, uint64_t gate, const ModC* mc, const Act& x,
                                            uint8_t* stg, int b, int64_t N, int64_t e0, int tid, bool valid,
                                            const u128* row0, u128* PS, u128& acc) {
    constexpr int kLast = MODE >= 1 ? K - 1 : K;
    if constexpr (I < kLast) {
        constexpr int i = I;
        {
            constexpr int r = MODE >= 1 ? (i + 1) % K : i;
            const ModC m = mc[a.crt.p[r]];
            const int n = static_cast<int>(m.n);
            const act_t* L = x.p[r] + static_cast<int64_t>(b) * n * N;
            uint32_t col = 0;
            u128 key;
            constexpr int kExtra = MODE == 1 ? 0 : 1;
            constexpr int nt = K - 1 - i + kExtra;
            u128 pf0 = 0, pf1 = 0;  // the row's first and last entries, loaded as soon as the row index is known
            if constexpr (r == 0) {  // residue 0, the base's power of two (mrs_staged checks): per-digit streams
                DigitStream ds[K > 1 ? K - 1 : 1];
#pragma unroll
                for (int l = 0; l < i; ++l) ds[l].init(PS[static_cast<int64_t>(mrs_pair<K>(l, i)) * N]);
                CompressFwd cf;
                cf.init();
                for (int c0 = 0; c0 < n; c0 += kMrsCap) {
                    const int cnt = min(kMrsCap, n - c0);
                    __syncthreads();
                    lds_stage_rows<kMrsBS, kStageU>(stg, L, N, e0, c0, cnt);
                    __syncthreads();
                    for (int c = 0; c < cnt; ++c) {
                        uint32_t d = valid ? stg[c * kMrsBS + tid] : 0u;  // spare lanes read no staged bytes
#pragma unroll
                        for (int l = 0; l < i; ++l) {
                            const uint32_t s = ds[l].next(m);
                            d = d >= s ? d - s : d + m.q - s;
                        }
                        if (c0 + c == 0) {
                            col = d;
                            // the row index is the key's first digit: start the row's first / last entry loads
                            // now, so the gather overlaps the rest of the digit walk (block-uniform branch)
                            const u128* rowp = row0 + a.dig_off[i] + static_cast<int64_t>(col) * nt;
                            pf0 = rowp[0];
                            pf1 = rowp[nt - 1];
                        }
                        cf.push(d, m);
                    }
                }
                key = cf.finish();
            } else {
                // chunk-major walk (as k_mrs_chain_w): passes of whole chunks, one divmod per stream per chunk of
                // m.c digits, wave-uniform digit loops, one compress flush per chunk
                u128 Q[K > 1 ? K - 1 : 1];
#pragma unroll
                for (int l = 0; l < i; ++l) Q[l] = PS[static_cast<int64_t>(mrs_pair<K>(l, i)) * N];
                u128 C = 0, PW = 1;
                const int mcn = static_cast<int>(m.c);
                const int pass = kMrsCap / mcn * mcn;
                for (int p0 = 0; p0 < n; p0 += pass) {
                    const int pcnt = min(pass, n - p0);
                    __syncthreads();
                    lds_stage_rows<kMrsBS, kStageU>(stg, L, N, e0, p0, pcnt);
                    __syncthreads();
                    for (int c0 = 0; c0 < pcnt; c0 += mcn) {
                        uint32_t rr[K > 1 ? K - 1 : 1];
#pragma unroll
                        for (int l = 0; l < i; ++l) rr[l] = divmod128(Q[l], m);
                        const int cnt = min(mcn, pcnt - c0);
                        uint32_t v = 0, pt = 1;
                        auto digit = [&](int t) -> uint32_t {
                            uint32_t d = valid ? stg[(c0 + t) * kMrsBS + tid] : 0u;
#pragma unroll
                            for (int l = 0; l < i; ++l) {
                                const uint32_t sd = chunk_digit(rr[l], m);
                                d = d >= sd ? d - sd : d + m.q - sd;
                            }
                            return d;
                        };
                        int t0 = 0;
                        if (p0 + c0 == 0) {  // (uniform) digit 0 peeled: its row gather starts at once, and the
                                             // digit loop below carries no per-digit compare
                            const uint32_t d = digit(0);
                            col = d;
                            const u128* rowp = row0 + a.dig_off[i] + static_cast<int64_t>(col) * nt;
                            pf0 = rowp[0];
                            pf1 = rowp[nt - 1];
                            v = d;
                            pt = m.q;
                            t0 = 1;
                        }
#pragma unroll 2
                        for (int t = t0; t < cnt; ++t) {
                            const uint32_t d = digit(t);
                            v += d * pt;
                            pt *= m.q;
                        }
                        C += PW * static_cast<u128>(v);
                        PW *= static_cast<u128>(m.D);
                    }
                }
                key = C;
            }
            const u128* row = row0 + a.dig_off[i] + static_cast<int64_t>(col) * nt;
            u128 E[K];
            E[0] = pf0;
#pragma unroll
            for (int t = 1; t < nt - 1; ++t) E[t] = row[t];  // the lines were brought in by the early loads
            if (nt > 1) E[nt - 1] = pf1;
            hard_unmask_n<K>(E, nt, key, gate, mrs_row_sub<MODE>(i));
            if (valid) {
#pragma unroll
                for (int t = 0; t < K - 1 - i; ++t) PS[static_cast<int64_t>(mrs_pair<K>(i, i + 1 + t)) * N] = E[t];
            }
            if constexpr (MODE != 1) acc = add_packed(acc, E[K - 1 - i], a.hmask);
        }
        chain_s_pos<K, MODE, I + 1>(a, gate, mc, x, stg, b, N, e0, tid, valid, row0, PS, acc);
    }
}

template <int K, int MODE>
__global__ __launch_bounds__(kMrsBS, MODE == 2 ? DASH_CHAIN2_WAVES : DASH_UA_MINBLOCKS) void k_mrs_chain_s(
    MrsArgs a, Act x, const ModC* mc, const uint32_t* te0, const uint32_t* rk) {
    (void)te0;
    (void)rk;
    __shared__ __attribute__((aligned(16))) uint8_t stg[kMrsCap * kMrsBS];
    const int b = blockIdx.z;
    const int64_t N = a.N;
    constexpr int NP = K * (K - 1) / 2 > 0 ? K * (K - 1) / 2 : 1;
    const int tid = static_cast<int>(threadIdx.x);
    for (int64_t e0 = static_cast<int64_t>(blockIdx.x) * kMrsBS; e0 < N; e0 += static_cast<int64_t>(gridDim.x) * kMrsBS) {
        const bool valid = e0 + tid < N;
        const int64_t e = valid ? e0 + tid : N - 1;  // spare lanes shadow a real element, store nothing
        const u128* row0 = a.tab + (static_cast<int64_t>(b) * N + e) * a.n_tab;
        u128* PS = a.ps + static_cast<int64_t>(b) * NP * N + e;
        u128 acc = 0;
        const uint64_t gate = a.gate0 ^ static_cast<uint64_t>(e);
        chain_s_pos<K, MODE, 0>(a, gate, mc, x, stg, b, N, e0, tid, valid, row0, PS, acc);
        if (MODE >= 1) {
            const ModC m = mc[a.crt.p[0]];
            const int n = static_cast<int>(m.n);
            const act_t* L = x.p[0] + static_cast<int64_t>(b) * n * N;
            CompressFwd cf;
            cf.init();
            u128 kb = 0;  // mod-2 residue: the components' bits packed 32 at a time (one shift-or each)
            for (int c0 = 0; c0 < n; c0 += kMrsCap) {
                const int cnt = min(kMrsCap, n - c0);
                __syncthreads();
                lds_stage_rows<kMrsBS, kStageU>(stg, L, N, e0, c0, cnt);
                __syncthreads();
                if (m.bits == 1) {
                    for (int w0 = 0; w0 < cnt; w0 += 32) {
                        uint32_t w = 0;
#pragma unroll 8
                        for (int u = 0; u < 32; ++u)
                            if (w0 + u < cnt) w |= (valid ? static_cast<uint32_t>(stg[(w0 + u) * kMrsBS + tid]) : 0u) << u;
                        kb |= static_cast<u128>(w) << (c0 + w0);
                    }
                } else {
                    for (int c = 0; c < cnt; ++c) cf.push(valid ? stg[c * kMrsBS + tid] : 0u, m);
                }
            }
            u128 key = m.bits == 1 ? kb : cf.finish();
#pragma unroll
            for (int l = 0; l < K - 1; ++l) key ^= PS[static_cast<int64_t>(mrs_pair<K>(l, K - 1)) * N];
            const uint32_t c = static_cast<uint32_t>(key) & 1u;
            u128 E = 0;
            if (MODE == 2) E = row0[a.dig_off[K - 1] + c] - hard_pad(key, gate, mrs_row_sub<MODE>(K - 1), 0);
            if (valid) {
                store_ypads(a, key, b, N, e);
                a.cs[static_cast<int64_t>(b) * N + e] = static_cast<uint8_t>(c);
            }
            if (MODE == 2) acc = add_packed(acc, E, a.hmask);
        }
        if (MODE == 1) continue;
        const uint32_t colf = static_cast<uint32_t>(acc) & static_cast<uint32_t>(a.T - 1);
        const u128* row = row0 + a.fin_off + static_cast<int64_t>(colf) * K;
        u128 F[K];
#pragma unroll
        for (int j = 0; j < K; ++j) F[j] = row[j];
        hard_unmask<K>(F, acc, gate, mrs_row_sub<0>(K));
        if (valid) {
#pragma unroll
            for (int j = 0; j < K; ++j) a.pf[(static_cast<int64_t>(b) * K + j) * N + e] = F[j];
        }
    }
}

// Latency form of the staged chain (small launches: batch 1). The per-lane form streams each position's label
// from HBM (n / kMrsChunk dependent round trips per position) and passes the pair payloads P_{l,i} between
// positions through HBM; at batch 1 a launch is one wave per SIMD, so every one of those round trips is
// exposed (~0.17 ms per rescale whatever N is). Here a block owns kMrsWBS consecutive elements:
//  * the label rows of EVERY residue come into LDS once, in one loop over all rows with kWaveU 16-byte loads in
//    flight per thread, before the chain starts;
//  * the positions read their components from LDS with no barrier;
//  * the K(K-1)/2 pair payloads stay in registers (one wave per SIMD: the whole 512-VGPR file is the lane's).
constexpr int kMrsWBS = 256;
constexpr int kWaveU = 8;
// one position of k_mrs_chain_w, I a compile-time constant (the pair payloads PS stay in registers). The wave
// form is compiled for bases whose residue 0 is the only power of two (first-primes bases: p_0 = 2, the rest
// odd; mrs_wave_lds checks it): each position then carries one digit path instead of both, which keeps the
// kernel's code closer to the instruction cache.
template <int K, int MODE, int I>
__device__ __forceinline__ void chain_w_pos(const MrsArgs& a, uint64_t gate, const ModC* mc, const uint8_t* wst,
                                            const int* roff, int tid, bool valid, const u128* row0, u128* PS,
                                            u128& acc) {
    constexpr int kLast = MODE >= 1 ? K - 1 : K;
    if constexpr (I < kLast) {
        constexpr int r = MODE >= 1 ? (I + 1) % K : I;
        const ModC m = mc[a.crt.p[r]];
        const int n = static_cast<int>(m.n);
        const uint8_t* Ls = wst + roff[r] * kMrsWBS + tid;
        uint32_t col = 0;
        u128 key;
        constexpr int kExtra = MODE == 1 ? 0 : 1;
        constexpr int nt = K - 1 - I + kExtra;
        u128 pf0 = 0, pf1 = 0;  // the row's first and last entries, loaded as soon as the row index is known
        if constexpr (r == 0) {  // residue 0: the base's power of two (per-digit streams)
            DigitStream ds[I > 0 ? I : 1];
#pragma unroll
            for (int l = 0; l < I; ++l) ds[l].init(PS[mrs_pair<K>(l, I)]);
            CompressFwd cf;
            cf.init();
            for (int c = 0; c < n; ++c) {
                uint32_t d = valid ? Ls[c * kMrsWBS] : 0u;
#pragma unroll
                for (int l = 0; l < I; ++l) {
                    const uint32_t s = ds[l].next(m);
                    d = d >= s ? d - s : d + m.q - s;
                }
                if (c == 0) {
                    col = d;
                    // the row index is the key's first digit: the gather overlaps the rest of the digit walk
                    const u128* rowp = row0 + a.dig_off[I] + static_cast<int64_t>(col) * nt;
                    pf0 = rowp[0];
                    pf1 = rowp[nt - 1];
                }
                cf.push(d, m);
            }
            key = cf.finish();
        } else {  // odd residue
            // chunk-major walk: every stream shares the modulus, so one divmod per stream per chunk of m.c
            // digits, then the chunk's digits with a wave-uniform trip count, one compress flush per chunk
            // (the same digits and compress as DigitStream / CompressFwd, without their per-digit bookkeeping)
            u128 Q[I > 0 ? I : 1];
#pragma unroll
            for (int l = 0; l < I; ++l) Q[l] = PS[mrs_pair<K>(l, I)];
            u128 C = 0, PW = 1;
            for (int c0 = 0; c0 < n; c0 += static_cast<int>(m.c)) {
                uint32_t rr[I > 0 ? I : 1];
#pragma unroll
                for (int l = 0; l < I; ++l) rr[l] = divmod128(Q[l], m);
                const int cnt = min(static_cast<int>(m.c), n - c0);
                uint32_t v = 0, pt = 1;
                for (int t = 0; t < cnt; ++t) {
                    uint32_t d = valid ? Ls[(c0 + t) * kMrsWBS] : 0u;
#pragma unroll
                    for (int l = 0; l < I; ++l) {
                        const uint32_t sd = chunk_digit(rr[l], m);
                        d = d >= sd ? d - sd : d + m.q - sd;
                    }
                    if (c0 + t == 0) {
                        col = d;
                        const u128* rowp = row0 + a.dig_off[I] + static_cast<int64_t>(col) * nt;
                        pf0 = rowp[0];
                        pf1 = rowp[nt - 1];
                    }
                    v += d * pt;
                    pt *= m.q;
                }
                C += PW * static_cast<u128>(v);
                PW *= static_cast<u128>(m.D);
            }
            key = C;
        }
        const u128* row = row0 + a.dig_off[I] + static_cast<int64_t>(col) * nt;
        u128 E[nt > 0 ? nt : 1];
        E[0] = pf0;
#pragma unroll
        for (int t = 1; t < nt - 1; ++t) E[t] = row[t];  // the lines were brought in by the early loads
        if constexpr (nt > 1) E[nt - 1] = pf1;
        if constexpr (nt > 0) hard_unmask<nt>(E, key, gate, mrs_row_sub<MODE>(I));
#pragma unroll
        for (int t = 0; t < K - 1 - I; ++t) PS[mrs_pair<K>(I, I + 1 + t)] = E[t];
        if constexpr (MODE != 1) acc = add_packed(acc, E[K - 1 - I], a.hmask);
        chain_w_pos<K, MODE, I + 1>(a, gate, mc, wst, roff, tid, valid, row0, PS, acc);
    }
}

template <int K, int MODE>
__global__ __launch_bounds__(kMrsWBS, 1) void k_mrs_chain_w(MrsArgs a, Act x, const ModC* mc, const uint32_t* te0,
                                                            const uint32_t* rk) {
    (void)te0;
    (void)rk;
    extern __shared__ __attribute__((aligned(16))) uint8_t wst[];  // row g (residue r, component c) at g * kMrsWBS
    const int b = blockIdx.z;
    const int64_t N = a.N;
    constexpr int NP = K * (K - 1) / 2 > 0 ? K * (K - 1) / 2 : 1;
    const int tid = static_cast<int>(threadIdx.x);
    int roff[K + 1];
    const act_t* src[K];
    roff[0] = 0;
#pragma unroll
    for (int r = 0; r < K; ++r) {
        const int n = static_cast<int>(mc[a.crt.p[r]].n);
        roff[r + 1] = roff[r] + n;
        src[r] = x.p[r] + static_cast<int64_t>(b) * n * N;
    }
    const int units = roff[K] * (kMrsWBS / 16);
    for (int64_t e0 = static_cast<int64_t>(blockIdx.x) * kMrsWBS; e0 < N; e0 += static_cast<int64_t>(gridDim.x) * kMrsWBS) {
        __syncthreads();  // the previous tile's readers are done
        if (N % 16 != 0) {
            // rows not 16-byte aligned (tiny layers, e.g. a 10-logit head): each lane stages its own column, one
            // byte per row, kWaveBU loads in flight (unit xu = row * kMrsWBS + tid, its LDS offset)
            constexpr int kWaveBU = 32;
            const int bunits = roff[K] * kMrsWBS;
            const int64_t e = e0 + tid;
            for (int x0 = tid; x0 < bunits; x0 += kWaveBU * kMrsWBS) {
                uint32_t v[kWaveBU];
#pragma unroll
                for (int h = 0; h < kWaveBU; ++h) {
                    const int xu = x0 + h * kMrsWBS;
                    const int g = xu / kMrsWBS;
                    const act_t* row = src[0] + static_cast<int64_t>(g) * N;
#pragma unroll
                    for (int r = 1; r < K; ++r)
                        if (g >= roff[r]) row = src[r] + static_cast<int64_t>(g - roff[r]) * N;
                    v[h] = (xu < bunits && e < N) ? static_cast<uint32_t>(row[e]) : 0u;
                }
#pragma unroll
                for (int h = 0; h < kWaveBU; ++h) {
                    const int xu = x0 + h * kMrsWBS;
                    if (xu < bunits) wst[xu] = static_cast<uint8_t>(v[h]);
                }
            }
        } else
        for (int x0 = tid; x0 < units; x0 += kWaveU * kMrsWBS) {
            uint4 v[kWaveU];
#pragma unroll
            for (int h = 0; h < kWaveU; ++h) {
                const int xu = x0 + h * kMrsWBS;
                const int g = xu >> 4;
                const int64_t e = e0 + 16 * (xu & 15);
                const act_t* row = src[0] + static_cast<int64_t>(g) * N;
#pragma unroll
                for (int r = 1; r < K; ++r)
                    if (g >= roff[r]) row = src[r] + static_cast<int64_t>(g - roff[r]) * N;
                if (xu < units && e < N) v[h] = *reinterpret_cast<const uint4*>(row + e);
            }
#pragma unroll
            for (int h = 0; h < kWaveU; ++h) {
                const int xu = x0 + h * kMrsWBS;
                if (xu < units) *reinterpret_cast<uint4*>(wst + (xu >> 4) * kMrsWBS + 16 * (xu & 15)) = v[h];
            }
        }
        __syncthreads();
        const bool valid = e0 + tid < N;
        const int64_t e = valid ? e0 + tid : N - 1;  // spare lanes shadow a real element, store nothing
        const u128* row0 = a.tab + (static_cast<int64_t>(b) * N + e) * a.n_tab;
        u128 PS[NP];
        u128 acc = 0;
        const uint64_t gate = a.gate0 ^ static_cast<uint64_t>(e);
        chain_w_pos<K, MODE, 0>(a, gate, mc, wst, roff, tid, valid, row0, PS, acc);
        if (MODE >= 1) {
            const ModC m = mc[a.crt.p[0]];
            const int n = static_cast<int>(m.n);
            const uint8_t* Ls = wst + tid;
            CompressFwd cf;
            cf.init();
            for (int c = 0; c < n; ++c) cf.push(valid ? Ls[c * kMrsWBS] : 0u, m);
            u128 key = cf.finish();
#pragma unroll
            for (int l = 0; l < K - 1; ++l) key ^= PS[mrs_pair<K>(l, K - 1)];
            const uint32_t cb = static_cast<uint32_t>(key) & 1u;
            u128 E = 0;
            if (MODE == 2) E = row0[a.dig_off[K - 1] + cb] - hard_pad(key, gate, mrs_row_sub<MODE>(K - 1), 0);
            if (valid) {
                store_ypads(a, key, b, N, e);
                a.cs[static_cast<int64_t>(b) * N + e] = static_cast<uint8_t>(cb);
            }
            if (MODE == 2) acc = add_packed(acc, E, a.hmask);
        }
        if (MODE == 1) continue;
        const uint32_t colf = static_cast<uint32_t>(acc) & static_cast<uint32_t>(a.T - 1);
        const u128* row = row0 + a.fin_off + static_cast<int64_t>(colf) * K;
        u128 F[K];
#pragma unroll
        for (int j = 0; j < K; ++j) F[j] = row[j];
        hard_unmask<K>(F, acc, gate, mrs_row_sub<0>(K));
        if (valid) {
#pragma unroll
            for (int j = 0; j < K; ++j) a.pf[(static_cast<int64_t>(b) * K + j) * N + e] = F[j];
        }
    }
}

// ---------------------------------------------------------------------------
// Quad form of the wave chain (batch-1 latency). At batch 1 a chain launch is one wave per SIMD and every
// element is a serial walk of K positions (~100 us per launch whatever the layer size, r05 batch-1 trace).
// Here four lanes share one element:
//  * position I's I payload streams are dealt to the quad's lanes (stream l to lane l % 4), each lane
//    decompresses its own, and the per-digit sums are all-reduced over the quad with two DPP adds;
//  * every lane then has the key digits and compresses the key (the same value in all four lanes);
//  * the row's entries and their pad blocks are split over the lanes (entries 4g..4g+3 and ChaCha block g on
//    lane g) and broadcast back with DPP, so the pair payloads stay replicated in every lane's registers;
//  * the final row likewise: lane g unmasks and stores outputs 4g..4g+3.
// Four times the lanes of the wave form, and per lane about a quarter of the decompression work.
constexpr int kMrsQE = 64;            // elements per block
constexpr int kMrsQBS = 4 * kMrsQE;   // threads per block (quads of consecutive lanes)
template <int S>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v) {  // the value of quad lane S, in every lane of the quad
    return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), S * 0x55, 0xF, 0xF, false));
}
template <int S>
__device__ __forceinline__ u128 quad_bcast128(u128 v) {
    const uint32_t w0 = quad_bcast<S>(static_cast<uint32_t>(v)), w1 = quad_bcast<S>(static_cast<uint32_t>(v >> 32));
    const uint32_t w2 = quad_bcast<S>(static_cast<uint32_t>(v >> 64)), w3 = quad_bcast<S>(static_cast<uint32_t>(v >> 96));
    return (static_cast<u128>((static_cast<uint64_t>(w3) << 32) | w2) << 64) | ((static_cast<uint64_t>(w1) << 32) | w0);
}
// sum over the quad of v < q, mod q (every lane gets it): xor-1 then xor-2 partners (quad_perm 1032 / 2301)
__device__ __forceinline__ uint32_t quad_sum_mod(uint32_t v, uint32_t q) {
    uint32_t s = v + static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0xB1, 0xF, 0xF, false));
    s = s >= q ? s - q : s;
    uint32_t t = s + static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(s), 0x4E, 0xF, 0xF, false));
    return t >= q ? t - q : t;
}
// byte-wise sum over the quad of four packed values (each byte < 64): every byte of the result < 4 * 64
__device__ __forceinline__ uint32_t quad_sum_bytes(uint32_t v) {
    const uint32_t s = v + static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0xB1, 0xF, 0xF, false));
    return s + static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(s), 0x4E, 0xF, 0xF, false));
}
// Chunk-split key (positions with at most kQSplit payload streams): the key's base-q chunks are dealt over the
// quad, lane g taking chunks 4j + g, so each lane walks a quarter of the digits; every lane runs the streams'
// chunk divisions (cheap next to the digit walk) and keeps its own chunk's value, and the lanes' partial keys
// sum over the quad. The stream-split form (below) replicates the whole digit walk on every lane.
constexpr int kQSplit = 5;  // compiled for positions I <= kQSplit; the launch picks the limit (DASH_MRS_QSPLIT)
template <int NSTR>
__device__ __forceinline__ u128 quad_key_split(const uint8_t* Ls, const ModC& m, int g, bool valid, u128 (&Q)[NSTR > 0 ? NSTR : 1]) {
    const int n = static_cast<int>(m.n);
    if (m.bits) {  // power of two (no streams): lane g packs digits [g * cpl, (g + 1) * cpl) at bit b * t
        const int cpl = (n + 3) >> 2, b = static_cast<int>(m.bits);
        u128 P = 0;
        for (int t = 0; t < cpl; ++t) {
            const int idx = g * cpl + t;
            if (valid && idx < n) P |= static_cast<u128>(Ls[idx * kMrsQE]) << (b * idx);
        }
        return quad_sum128(P);  // disjoint bit ranges: the sum is the OR
    }
    const int c = static_cast<int>(m.c);
    const uint32_t q = m.q;
    const int nch = (n + c - 1) / c;
    QPow pw;
    pw.init(m);
    u128 PW = pw.first(g), P = 0;
    for (int j = 0; 4 * j < nch; ++j) {
        uint32_t mine[NSTR > 0 ? NSTR : 1];
        if constexpr (NSTR > 0) {
#pragma unroll
            for (int l = 0; l < NSTR; ++l) mine[l] = 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (4 * j + u >= nch) break;
#pragma unroll
                for (int l = 0; l < NSTR; ++l) {
                    const uint32_t rr = divmod128(Q[l], m);
                    mine[l] = u == g ? rr : mine[l];
                }
            }
        }
        const int i = 4 * j + g;
        uint32_t v = 0, pt = 1;
        for (int t = 0; t < c; ++t) {
            const int idx = i * c + t;
            uint32_t d = 0;
            if (valid && idx < n) d = Ls[idx * kMrsQE];
            if constexpr (NSTR > 0) {
                uint32_t S = 0;
#pragma unroll
                for (int l = 0; l < NSTR; ++l) {
                    S += chunk_digit(mine[l], m);
                    S = S >= q ? S - q : S;
                }
                d = d >= S ? d - S : d + q - S;
                if (idx >= n) d = 0;
            }
            v += d * pt;
            pt *= q;
        }
        P += PW * static_cast<u128>(v);
        PW *= pw.d4;
    }
    return quad_sum128(P);
}
template <int K, int MODE, int I>
__device__ __forceinline__ void chain_q_pos(const MrsArgs& a, uint64_t gate, const ModC* mc, const uint8_t* wst,
                                            const int* roff, int el, int g, bool valid, const u128* row0, u128* PS,
                                            u128& acc) {
    constexpr int kLast = MODE >= 1 ? K - 1 : K;
    if constexpr (I < kLast) {
        constexpr int r = MODE >= 1 ? (I + 1) % K : I;
        const ModC m = mc[a.crt.p[r]];
        const int n = static_cast<int>(m.n);
        const uint8_t* Ls = wst + roff[r] * kMrsQE + el;  // the four lanes of a quad read the same byte (broadcast)
        constexpr int kExtra = MODE == 1 ? 0 : 1;
        constexpr int nt = K - 1 - I + kExtra;
        uint32_t col = 0;
        u128 key;
        // kQCoop: every lane loads the whole row (the quad's loads share their lines); else this lane's entries
        // 4g .. 4g + 3
        constexpr int kNE = kQCoop ? nt : 4;
        u128 Eo[kNE];
#pragma unroll
        for (int t = 0; t < kNE; ++t) Eo[t] = 0;
        auto fetch_row = [&](uint32_t c) {  // issued as soon as the row index (the key's first digit) is known
            const u128* rowp = row0 + a.dig_off[I] + static_cast<int64_t>(c) * nt;
#pragma unroll
            for (int q = 0; q < kNE; ++q)
                if (kQCoop || 4 * g + q < nt) Eo[q] = rowp[kQCoop ? q : 4 * g + q];
        };
        bool split = false;  // positions I < (qpack >> 1): chunk-split (DASH_MRS_QSPLIT=-1: the stream-split walk)
        if constexpr (I <= kQSplit) split = I < (a.qpack >> 1);
        if (split) {
            // the row index (the key's first digit) first, so the row loads overlap the digit walk
            u128 Q[I > 0 ? I : 1];
            uint32_t d0 = valid ? Ls[0] : 0u;
            if constexpr (I > 0) {
#pragma unroll
                for (int l = 0; l < I; ++l) Q[l] = PS[mrs_pair<K>(l, I)];
                uint32_t S0 = 0;
                if (m.bits) {
#pragma unroll
                    for (int l = 0; l < I; ++l) S0 += static_cast<uint32_t>(Q[l]) & (m.q - 1);
                    S0 &= m.q - 1;
                } else {
#pragma unroll
                    for (int l = 0; l < I; ++l) {
                        u128 t = Q[l];
                        uint32_t c0 = divmod128(t, m);
                        S0 += chunk_digit(c0, m);
                        S0 = S0 >= m.q ? S0 - m.q : S0;
                    }
                }
                d0 = d0 >= S0 ? d0 - S0 : d0 + m.q - S0;
            }
            col = d0;
            fetch_row(col);
            key = quad_key_split<I>(Ls, m, g, valid, Q);
        } else if constexpr (r == 0) {  // residue 0, the base's power of two: mode 0 position 0, no payload streams
            CompressFwd cf;
            cf.init();
            for (int c = 0; c < n; ++c) {
                const uint32_t d = valid ? Ls[c * kMrsQE] : 0u;
                if (c == 0) {
                    col = d;
                    fetch_row(col);
                }
                cf.push(d, m);
            }
            key = cf.finish();
        } else {
            constexpr int NS = I > 0 ? (I + 3) / 4 : 1;  // streams per lane: l = g + 4 s < I
            u128 Q[NS];
#pragma unroll
            for (int s2 = 0; s2 < NS; ++s2) {
                Q[s2] = 0;
#pragma unroll
                for (int l = 4 * s2; l < 4 * s2 + 4 && l < I; ++l)  // static register indices, selected per lane
                    if (g == l - 4 * s2) Q[s2] = PS[mrs_pair<K>(l, I)];
            }
            u128 C = 0, PW = 1;
            const int mcn = static_cast<int>(m.c);
            const uint32_t q = m.q;
            for (int c0 = 0; c0 < n; c0 += mcn) {
                uint32_t rr[NS];
#pragma unroll
                for (int s2 = 0; s2 < NS; ++s2) rr[s2] = I > 0 ? divmod128(Q[s2], m) : 0u;  // no stream: Q = 0
                const int cnt = min(mcn, n - c0);
                uint32_t v = 0, pt = 1;
                if (I > 0 && (a.qpack & 1) && q <= 63) {
                    // four digits per quad reduction: the lane's digit sums packed in bytes (each < q), two DPP
                    // adds leave every byte < 4q <= 252, then each byte is reduced mod q
                    for (int t0 = 0; t0 < cnt; t0 += 4) {
                        uint32_t pk = 0;
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            if (t0 + u >= cnt) break;
                            uint32_t sd = 0;
#pragma unroll
                            for (int s2 = 0; s2 < NS; ++s2) {
                                sd += chunk_digit(rr[s2], m);
                                sd = sd >= q ? sd - q : sd;
                            }
                            pk |= sd << (8 * u);
                        }
                        pk = quad_sum_bytes(pk);
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            if (t0 + u >= cnt) break;
                            uint32_t S = (pk >> (8 * u)) & 0xffu;
                            S = S >= 2 * q ? S - 2 * q : S;
                            S = S >= q ? S - q : S;
                            uint32_t d = valid ? Ls[(c0 + t0 + u) * kMrsQE] : 0u;
                            d = d >= S ? d - S : d + q - S;
                            if (c0 + t0 + u == 0) {
                                col = d;
                                fetch_row(col);
                            }
                            v += d * pt;
                            pt *= q;
                        }
                    }
                } else {
                    for (int t = 0; t < cnt; ++t) {
                        uint32_t S = 0;
                        if constexpr (I > 0) {
                            uint32_t sd = 0;
#pragma unroll
                            for (int s2 = 0; s2 < NS; ++s2) {
                                sd += chunk_digit(rr[s2], m);
                                sd = sd >= q ? sd - q : sd;
                            }
                            S = quad_sum_mod(sd, q);  // the digit sum of all I streams
                        }
                        uint32_t d = valid ? Ls[(c0 + t) * kMrsQE] : 0u;
                        d = d >= S ? d - S : d + q - S;
                        if (c0 + t == 0) {
                            col = d;
                            fetch_row(col);
                        }
                        v += d * pt;
                        pt *= q;
                    }
                }
                C += PW * static_cast<u128>(v);
                PW *= static_cast<u128>(m.D);
            }
            key = C;
        }
        // every lane takes every entry: pair payloads for the later positions, the T target for acc
        u128 E[nt];
        if constexpr (kQCoop) {
            // the quad runs the row's pad blocks together and gathers each pad into every lane
#pragma unroll
            for (int bk = 0; bk < (nt + 3) / 4; ++bk) {
                uint32_t w[4];
                hard_block_q(key, gate, mrs_row_sub<MODE>(I), static_cast<uint32_t>(bk), g, w);
#pragma unroll
                for (int qq = 0; qq < 4; ++qq)
                    if (4 * bk + qq < nt) E[4 * bk + qq] = Eo[4 * bk + qq] - quad_gather128(w[qq]);
            }
        } else {
            if (4 * g < nt) {  // lane g's pad block (entries 4g .. 4g + 3)
                u128 pd[4];
                hard_block(key, gate, mrs_row_sub<MODE>(I), static_cast<uint32_t>(g), pd);
#pragma unroll
                for (int qq = 0; qq < 4; ++qq)
                    if (4 * g + qq < nt) Eo[qq] -= pd[qq];
            }
#pragma unroll
            for (int t = 0; t < nt; ++t) {
                const u128 own = Eo[t % 4];
                E[t] = (t >> 2) == 0 ? quad_bcast128<0>(own) : (t >> 2) == 1 ? quad_bcast128<1>(own)
                       : (t >> 2) == 2 ? quad_bcast128<2>(own) : quad_bcast128<3>(own);
            }
        }
#pragma unroll
        for (int t = 0; t < K - 1 - I; ++t) PS[mrs_pair<K>(I, I + 1 + t)] = E[t];
        if constexpr (MODE != 1) acc = add_packed(acc, E[K - 1 - I], a.hmask);
        chain_q_pos<K, MODE, I + 1>(a, gate, mc, wst, roff, el, g, valid, row0, PS, acc);
    }
}

template <int K, int MODE>
__global__ __launch_bounds__(kMrsQBS, 2) void k_mrs_chain_q(MrsArgs a, Act x, const ModC* mc) {
    extern __shared__ __attribute__((aligned(16))) uint8_t wst[];  // row gg (residue r, component c) at gg * kMrsQE
    const int b = blockIdx.z;
    const int64_t N = a.N;
    constexpr int NP = K * (K - 1) / 2 > 0 ? K * (K - 1) / 2 : 1;
    const int tid = static_cast<int>(threadIdx.x);
    const int el = tid >> 2, g = tid & 3;
    int roff[K + 1];
    const act_t* src[K];
    roff[0] = 0;
#pragma unroll
    for (int r = 0; r < K; ++r) {
        const int n = static_cast<int>(mc[a.crt.p[r]].n);
        roff[r + 1] = roff[r] + n;
        src[r] = x.p[r] + static_cast<int64_t>(b) * n * N;
    }
    for (int64_t e0 = static_cast<int64_t>(blockIdx.x) * kMrsQE; e0 < N; e0 += static_cast<int64_t>(gridDim.x) * kMrsQE) {
        __syncthreads();  // the previous tile's readers are done
        if (N % 16 == 0) {
            // 16-byte units: row gg's kMrsQE bytes are kMrsQE / 16 units
            constexpr int W = kMrsQE / 16;
            const int units = roff[K] * W;
            for (int x0 = tid; x0 < units; x0 += 4 * kMrsQBS) {
                uint4 v[4];
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                    const int xu = x0 + h * kMrsQBS;
                    const int gg = xu / W;
                    const int64_t e = e0 + 16 * (xu % W);
                    const act_t* row = src[0] + static_cast<int64_t>(gg) * N;
#pragma unroll
                    for (int r = 1; r < K; ++r)
                        if (gg >= roff[r]) row = src[r] + static_cast<int64_t>(gg - roff[r]) * N;
                    if (xu < units && e < N) v[h] = *reinterpret_cast<const uint4*>(row + e);
                }
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                    const int xu = x0 + h * kMrsQBS;
                    if (xu < units) *reinterpret_cast<uint4*>(wst + (xu / W) * kMrsQE + 16 * (xu % W)) = v[h];
                }
            }
        } else {
            const int bunits = roff[K] * kMrsQE;  // one byte per (row, element)
            for (int xu = tid; xu < bunits; xu += kMrsQBS) {
                const int gg = xu / kMrsQE;
                const int64_t e = e0 + xu % kMrsQE;
                const act_t* row = src[0] + static_cast<int64_t>(gg) * N;
#pragma unroll
                for (int r = 1; r < K; ++r)
                    if (gg >= roff[r]) row = src[r] + static_cast<int64_t>(gg - roff[r]) * N;
                wst[xu] = e < N ? static_cast<uint8_t>(row[e]) : 0;
            }
        }
        __syncthreads();
        const bool valid = e0 + el < N;
        const int64_t e = valid ? e0 + el : N - 1;  // spare quads shadow a real element, store nothing
        const u128* row0 = a.tab + (static_cast<int64_t>(b) * N + e) * a.n_tab;
        u128 PS[NP];
        u128 acc = 0;
        const uint64_t gate = a.gate0 ^ static_cast<uint64_t>(e);
        chain_q_pos<K, MODE, 0>(a, gate, mc, wst, roff, el, g, valid, row0, PS, acc);
        if (MODE >= 1) {
            // residue 0 (mod 2): bit pack of L_0 XOR the K - 1 payloads aimed at it = the sign label (all lanes)
            const ModC m = mc[a.crt.p[0]];
            const int n = static_cast<int>(m.n);
            const uint8_t* Ls = wst + el;
            u128 key;
            if (m.bits == 1) {
                // lane g packs components 32 g .. 32 g + 31 as one word and the quad's words are summed (disjoint
                // bits): every lane used to walk all 128 components through the compressor
                uint32_t w = 0;
#pragma unroll 8
                for (int u = 0; u < 32; ++u) {
                    const int c = 32 * g + u;
                    if (valid && c < n) w |= static_cast<uint32_t>(Ls[c * kMrsQE]) << u;
                }
                key = quad_sum128(static_cast<u128>(w) << (32 * g));
            } else {
                CompressFwd cf;
                cf.init();
                for (int c = 0; c < n; ++c) cf.push(valid ? Ls[c * kMrsQE] : 0u, m);
                key = cf.finish();
            }
#pragma unroll
            for (int l = 0; l < K - 1; ++l) key ^= PS[mrs_pair<K>(l, K - 1)];
            const uint32_t cb = static_cast<uint32_t>(key) & 1u;
            u128 E = 0;
            if (MODE == 2) {
                if constexpr (kQCoop) {
                    uint32_t w[4];
                    hard_block_q(key, gate, mrs_row_sub<MODE>(K - 1), 0u, g, w);
                    E = row0[a.dig_off[K - 1] + cb] - quad_gather128(w[0]);
                } else {
                    E = row0[a.dig_off[K - 1] + cb] - hard_pad(key, gate, mrs_row_sub<MODE>(K - 1), 0);
                }
            }
            if (kQCoop && valid) {
                // the next ReLU's y-row pads: the quad runs each block, lane j stores word j of its pads
                const uint64_t gy = a.rgate0 ^ static_cast<uint64_t>(e);
                for (int bk = 0; 4 * bk < a.ny; ++bk) {
                    uint32_t w[4];
                    hard_block_q(key, gy, tw_sub(kTwMmy, 0), static_cast<uint32_t>(bk), g, w);
#pragma unroll
                    for (int qq = 0; qq < 4; ++qq)
                        if (4 * bk + qq < a.ny)
                            reinterpret_cast<uint32_t*>(a.ys + (static_cast<int64_t>(b) * a.ny + 4 * bk + qq) * N + e)[g] = w[qq];
                }
                if (g == 0) a.cs[static_cast<int64_t>(b) * N + e] = static_cast<uint8_t>(cb);
            }
            if (!kQCoop && valid) {
                // the next ReLU's y-row pads: block g on lane g
                const uint64_t gy = a.rgate0 ^ static_cast<uint64_t>(e);
                if (4 * g < a.ny) {
                    u128 pd[4];
                    hard_block(key, gy, tw_sub(kTwMmy, 0), static_cast<uint32_t>(g), pd);
#pragma unroll
                    for (int qq = 0; qq < 4; ++qq)
                        if (4 * g + qq < a.ny) a.ys[(static_cast<int64_t>(b) * a.ny + 4 * g + qq) * N + e] = pd[qq];
                }
                if (g == 0) a.cs[static_cast<int64_t>(b) * N + e] = static_cast<uint8_t>(cb);
            }
            if (MODE == 2) acc = add_packed(acc, E, a.hmask);
        }
        if (MODE == 1) continue;
        const uint32_t colf = static_cast<uint32_t>(acc) & static_cast<uint32_t>(a.T - 1);
        const u128* row = row0 + a.fin_off + static_cast<int64_t>(colf) * K;
        if constexpr (kQCoop) {
            // output 4 bk + g on lane g under pad g of block bk (the quad runs the block, gathers every pad)
#pragma unroll
            for (int bk = 0; bk < (K + 3) / 4; ++bk) {
                const bool mine = 4 * bk + g < K;
                const u128 F = mine ? row[4 * bk + g] : u128(0);
                uint32_t w[4];
                hard_block_q(acc, gate, mrs_row_sub<0>(K), static_cast<uint32_t>(bk), g, w);
                u128 pd = 0;
#pragma unroll
                for (int qq = 0; qq < 4; ++qq) {
                    const u128 p = quad_gather128(w[qq]);
                    pd = qq == g ? p : pd;
                }
                if (valid && mine) a.pf[(static_cast<int64_t>(b) * K + 4 * bk + g) * N + e] = F - pd;
            }
        } else if (4 * g < K) {  // outputs 4g .. 4g + 3 under pad block g
            u128 F[4], pd[4];
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) F[qq] = 4 * g + qq < K ? row[4 * g + qq] : u128(0);
            hard_block(acc, gate, mrs_row_sub<0>(K), static_cast<uint32_t>(g), pd);
            if (valid) {
#pragma unroll
                for (int qq = 0; qq < 4; ++qq)
                    if (4 * g + qq < K) a.pf[(static_cast<int64_t>(b) * K + 4 * g + qq) * N + e] = F[qq] - pd[qq];
            }
        }
    }
}

// bases whose residue 0 is the single power of two: the wave and staged chain forms compile one digit path per position
static inline bool mrs_odd_base(const CrtInfo& crt) {
    if ((crt.p[0] & (crt.p[0] - 1)) != 0) return false;
    for (int r = 1; r < crt.k; ++r)
        if ((crt.p[r] & 1) == 0) return false;
    return true;
}
// dynamic LDS of k_mrs_chain_w (every residue's rows for kMrsWBS elements), 0 when the form does not apply
static inline size_t mrs_wave_lds(const MrsArgs& a, int B) {
    static const bool on = [] {
        const char* e = std::getenv("DASH_MRS_WAVE");
        return !(e && e[0] == '0');
    }();
    // only launches of at most one block per CU: above that the per-lane form keeps more waves resident (24 GCs,
    // MiniONN: 11.29 ms per step per-lane vs 11.56 with this form on every small-block launch)
    // only bases whose residue 0 is the single power of two (the form's positions carry one digit path each)
    if (!mrs_odd_base(a.crt)) return 0;
    // (rows that are not 16-byte aligned: byte-wise staging, only for single-block layers)
    if (!on || (a.N % 16 != 0 && a.N > kMrsWBS) || (a.N + kMrsWBS - 1) / kMrsWBS * B > num_cus()) return 0;
    size_t sum = 0;
    for (int r = 0; r < a.crt.k; ++r) sum += static_cast<size_t>(std::floor(128.0 / std::log2(static_cast<double>(a.crt.p[r]))));  // core.h nr_comps
    const size_t bytes = sum * kMrsWBS;
    if (bytes > (160u << 10)) return 0;  // the hardened chain holds no AES image
    return bytes;
}

// the quad form replaces the wave form where that applies (DASH_MRS_QUAD=0: the wave form, A/B)
static inline bool mrs_quad_on() {
    static const bool on = [] {
        const char* e = std::getenv("DASH_MRS_QUAD");
        return !(e && e[0] == '0');
    }();
    return on;
}
// launches k_mrs_chain_w<K, MODE> (or its quad form) with wl bytes of dynamic LDS (the per-kernel limit is raised
// once)
template <int K, int MODE>
static void launch_chain_w(const MrsArgs& a, const Act& x, int B, size_t wl, const ModC* mc, const AesGlobals& g,
                           hipStream_t st) {
    if (mrs_quad_on()) {
        static const int qpack = [] {  // A/B knobs DASH_MRS_QPACK=0 (one quad reduction per digit), DASH_MRS_QSPLIT=0
            const char* e = std::getenv("DASH_MRS_QPACK");
            const char* f = std::getenv("DASH_MRS_QSPLIT");  // the last chunk-split position (-1: none)
            const int lim = f ? std::max(-1, std::min(kQSplit, std::atoi(f))) : 3;
            return (e && e[0] == '0' ? 0 : 1) | ((lim + 1) << 1);
        }();
        MrsArgs aq = a;
        aq.qpack = qpack;
        const size_t ql = wl / kMrsWBS * kMrsQE;  // every residue's rows for kMrsQE elements
        const dim3 gq(static_cast<unsigned>((a.N + kMrsQE - 1) / kMrsQE), 1, B);
        hipLaunchKernelGGL((k_mrs_chain_q<K, MODE>), gq, dim3(kMrsQBS), ql, st, aq, x, mc);
        return;
    }
    static const bool raised = [] {
        return hipFuncSetAttribute(reinterpret_cast<const void*>(&k_mrs_chain_w<K, MODE>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                   160 << 10) == hipSuccess;
    }();
    (void)raised;
    const dim3 gw(static_cast<unsigned>((a.N + kMrsWBS - 1) / kMrsWBS), 1, B);
    hipLaunchKernelGGL((k_mrs_chain_w<K, MODE>), gw, dim3(kMrsWBS), wl, st, a, x, mc, g.te0, g.rk);
}

// the staged chain holds two 512-lane blocks per CU: below two blocks per CU (batch-1 latency) the per-lane form,
// whose block size shrinks to spread a small launch over every CU, is faster
static inline bool mrs_staged(const MrsArgs& a, int B) {
    return mrs_odd_base(a.crt) && stage_ok(a.N, kMrsBS) && (a.N + kMrsBS - 1) / kMrsBS * B >= 2 * num_cus();
}


// One chain launch for K residues: the wave-staged form for launches of at most one block per CU (batch-1
// latency), the LDS-staged form for large ones, the per-lane form between; a.mode picks rescale / sign / joint.
template <int K>
void launch_mrs_chain_k(const MrsArgs& a, const Act& x, int B, const ModC* mc, const AesGlobals& g, hipStream_t st) {
    const bool stg = mrs_staged(a, B);
    const size_t wl = stg ? 0 : mrs_wave_lds(a, B);
    const dim3 gc = stg ? grid_aes(a.N, kMrsBS, 1, B) : grid_aes(a.N, aes_bs(a.N, 1, B), 1, B);
    const dim3 bc(stg ? kMrsBS : aes_bs(a.N, 1, B));
    if (a.mode == 1) {
        if (wl) launch_chain_w<K, 1>(a, x, B, wl, mc, g, st);
        else if (stg) hipLaunchKernelGGL((k_mrs_chain_s<K, 1>), gc, bc, 0, st, a, x, mc, g.te0, g.rk);
        else hipLaunchKernelGGL((k_mrs_chain<K, 1>), gc, bc, 0, st, a, x, mc, g.te0, g.rk);
    } else if (a.mode == 2) {
        if (wl) launch_chain_w<K, 2>(a, x, B, wl, mc, g, st);
        else if (stg) hipLaunchKernelGGL((k_mrs_chain_s<K, 2>), gc, bc, 0, st, a, x, mc, g.te0, g.rk);
        else hipLaunchKernelGGL((k_mrs_chain<K, 2>), gc, bc, 0, st, a, x, mc, g.te0, g.rk);
    } else {
        if (wl) launch_chain_w<K, 0>(a, x, B, wl, mc, g, st);
        else if (stg) hipLaunchKernelGGL((k_mrs_chain_s<K, 0>), gc, bc, 0, st, a, x, mc, g.te0, g.rk);
        else hipLaunchKernelGGL((k_mrs_chain<K, 0>), gc, bc, 0, st, a, x, mc, g.te0, g.rk);
    }
}

}  // namespace dev
}  // namespace dash
