// Shared pieces of the gadget kernels (kernels_gadget.hip and the per-K mixed-radix chain units
// kernels_mrs_*.hip): launch geometry, the AES LDS prologue, LDS row staging.
#pragma once

#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "kargs.h"
#include "launch.h"

namespace dash {
namespace dev {

constexpr size_t kAesLds = 0;  // AES image is static LDS

// AES kernels hold the LDS image (dev.h: 32 KiB at 16 copies) per block; the
// second launch bound is the minimum number of waves per SIMD, so it sets the
// register budget: 4 -> 128 VGPRs, 6 -> 80, 8 -> 64. Measured on MiniONN,
// 24 GCs, one stream (ms per step, scripts/ab_online.py): 64 KiB image at 4
// waves/SIMD 20.9; 32 KiB image at 6 waves/SIMD 19.7 (the mixed-radix chain
// 7.4 -> 6.9 ms, approx phase 4.5 -> 4.1); at 8 waves/SIMD the chain spills
// (9.3 ms). The approx phase has its own knob (8 waves: 4.0-4.3 ms, within the
// box-to-box noise of 6) and the chain its own (DASH_UA_MINBLOCKS, 4 waves).
// The 2-way bank conflicts of 16 copies cost less than the extra resident
// waves buy: these kernels wait on HBM, AES is ~3 % of their time.
#ifndef DASH_AES_BLOCK
#define DASH_AES_BLOCK 512
#endif
constexpr int kAesBlock = DASH_AES_BLOCK;
#ifndef DASH_AES_MINBLOCKS
#define DASH_AES_MINBLOCKS 6
#endif
constexpr int kAesMinBlocks = DASH_AES_MINBLOCKS;  // minimum waves per SIMD (register budget)
#ifndef DASH_SA_MINBLOCKS
#define DASH_SA_MINBLOCKS 6
#endif
constexpr int kSignApproxMinWaves = DASH_SA_MINBLOCKS;
#ifndef DASH_SA_CHUNK
#define DASH_SA_CHUNK 16
#endif
constexpr int kSignApproxChunk = DASH_SA_CHUNK;  // label loads in flight per lane in the approx phase

// AES kernels stride over their elements so the LDS image is filled once per
// resident block: resident blocks per CU (register budget: waves per SIMD x 4
// SIMDs x 64 lanes / block size; LDS: 160 KiB / image), x4 for tail balance.
static int num_cus() {
    static int cus = [] {
        int dev = 0, n = 256;
        if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        return n;
    }();
    return cus;
}
static int aes_block_cap(int bs) {
    const int waves = std::max(kAesMinBlocks, kSignApproxMinWaves);
    const int resident = std::max(1, std::min(waves * 256 / bs, 160 * 1024 / DASH_AES_LDS_BYTES));
    return 4 * resident * num_cus();
}
static inline dim3 grid_aes(int64_t n, int bs, int y, int z) {
    int64_t nx = (n + bs - 1) / bs;
    const int64_t capx = std::max<int64_t>(1, aes_block_cap(bs) / (static_cast<int64_t>(y) * z));
    return dim3(static_cast<unsigned>(std::min(nx, capx)), y, z);
}
// Block size of an AES kernel over n x y x z lanes: kAesBlock when the launch
// fills every CU at that size, else halved (down to one wave) until it does.
// Small launches (batch-1 latency, the late small layers) then spread over all
// CUs with few waves per SIMD, and their lanes are serial chains: a wave that
// has its SIMD to itself finishes sooner.
static inline int aes_bs(int64_t n, int y, int z) {
    const int64_t lanes = n * y * z;
    int bs = kAesBlock;
    while (bs > 64 && lanes < static_cast<int64_t>(bs) * num_cus()) bs >>= 1;
    return bs;
}
#define AES_LAUNCH(n, y, z) grid_aes((n), aes_bs((n), (y), (z)), (y), (z)), dim3(aes_bs((n), (y), (z)))

// static (not dynamic) LDS: its address is a link-time constant, so the
// table base folds into the ds_read offset field
#define AES_PROLOGUE(tab, rk)                    \
    __shared__ __attribute__((aligned(16))) uint32_t lds_aes[DASH_AES_LDS_WORDS]; \
    aes_lds_fill(lds_aes, tab);                   \
    const AesCtx aes = aes_ctx(lds_aes, rk)

// ---------------------------------------------------------------------------
// LDS staging of component-major byte labels (rows of N bytes, N % 16 == 0): a block owning BS consecutive
// elements moves rows [c0, c0 + cnt) of its tile between HBM and an LDS image S[c][BS] with 16-byte
// accesses, U of them in flight per thread. Lanes then walk their own element's components in LDS. A lane
// streaming its own column from HBM moves one byte per lane per load (64 B per wave instruction) with a
// few loads in flight: the streaming kernels sat at 0.2-1.5 TB/s, 65-70 % of cycles waiting (r03 roofline).
template <int BS, int U>
__device__ __forceinline__ void lds_stage_rows(uint8_t* S, const act_t* L, int64_t N, int64_t e0, int c0, int cnt) {
    constexpr int W = BS / 16;  // 16-byte units per row
    const int units = cnt * W;
    for (int x0 = threadIdx.x; x0 < units; x0 += U * BS) {
        uint4 v[U];
#pragma unroll
        for (int h = 0; h < U; ++h) {
            const int x = x0 + h * BS;
            const int64_t e = e0 + 16 * (x % W);
            if (x < units && e < N) v[h] = *reinterpret_cast<const uint4*>(L + static_cast<int64_t>(c0 + x / W) * N + e);
        }
#pragma unroll
        for (int h = 0; h < U; ++h) {
            const int x = x0 + h * BS;
            if (x < units) *reinterpret_cast<uint4*>(S + (x / W) * BS + 16 * (x % W)) = v[h];
        }
    }
}
template <int BS>
__device__ __forceinline__ void lds_store_rows(act_t* L, const uint8_t* S, int64_t N, int64_t e0, int c0, int cnt) {
    constexpr int W = BS / 16;
    const int units = cnt * W;
    for (int x = threadIdx.x; x < units; x += BS) {
        const int64_t e = e0 + 16 * (x % W);
        if (e < N)
            *reinterpret_cast<uint4*>(L + static_cast<int64_t>(c0 + x / W) * N + e) =
                *reinterpret_cast<const uint4*>(S + (x / W) * BS + 16 * (x % W));
    }
}
// the staged kernels where the shape allows (whole 16-byte rows, at least one full block); A/B knob
// DASH_MRS_STAGE=0 keeps the per-lane forms
static inline bool stage_ok(int64_t N, int bs) {
    static const bool on = [] {
        const char* e = std::getenv("DASH_MRS_STAGE");
        return !(e && e[0] == '0');
    }();
    return on && N % 16 == 0 && N >= bs;
}

// the mixed-radix chain keeps K-1 digit streams live: at 6 waves/SIMD (80 VGPRs) it spills 240 B per
// lane; 4 waves/SIMD with 128 VGPRs measured faster (6.36 vs 7.04 ms per 24-GC MiniONN step)
#ifndef DASH_UA_MINBLOCKS
#define DASH_UA_MINBLOCKS 4
#endif

// u128 sum over the quad, every lane gets it (two DPP rounds on the four 32-bit words, carries by the adds)
template <int CTRL>
__device__ __forceinline__ u128 dpp128(u128 v) {
    const uint32_t w0 = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(static_cast<uint32_t>(v)), CTRL, 0xF, 0xF, false));
    const uint32_t w1 = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(static_cast<uint32_t>(v >> 32)), CTRL, 0xF, 0xF, false));
    const uint32_t w2 = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(static_cast<uint32_t>(v >> 64)), CTRL, 0xF, 0xF, false));
    const uint32_t w3 = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(static_cast<uint32_t>(v >> 96)), CTRL, 0xF, 0xF, false));
    return (static_cast<u128>((static_cast<uint64_t>(w3) << 32) | w2) << 64) | ((static_cast<uint64_t>(w1) << 32) | w0);
}
__device__ __forceinline__ u128 quad_sum128(u128 v) {
    v += dpp128<0xB1>(v);
    return v + dpp128<0x4E>(v);
}
struct QPow {  // D^1 .. D^4 of a modulus (D = q^c < 2^31): lane g's first chunk weight and the group step
    u128 d1, d2, d3, d4;
    __device__ __forceinline__ void init(const ModC& m) {
        d1 = static_cast<u128>(m.D);
        d2 = d1 * d1;
        d3 = d2 * d1;
        d4 = d2 * d2;
    }
    __device__ __forceinline__ u128 first(int g) const {
        return g == 0 ? static_cast<u128>(1) : (g == 1 ? d1 : (g == 2 ? d2 : d3));
    }
};

}  // namespace dev
}  // namespace dash
