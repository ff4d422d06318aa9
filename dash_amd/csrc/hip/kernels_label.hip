// Free (non-cryptographic) label kernels: gathers, pair differences / sums
// for the max-pool reduction tree, residual add, window sums, plus small
// parity-test kernels for the AES and digit codecs.
#include <algorithm>

#include "launch.h"
#include "fetch.h"

namespace dash {
namespace dev {

// out[b][j][c][o] = in[b][j][c][idx[o]]     grid (ceil(Nout*n_max/256), k, B)
__global__ __launch_bounds__(256) void k_copy_gather(Act in, int64_t Nin, Act out, int64_t Nout, const int64_t* idx,
                                                     CrtInfo crt) {
    const int j = blockIdx.y, b = blockIdx.z;
    const int n = crt.n[j];
    const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= Nout * n) return;
    const int64_t c = t / Nout, o = t % Nout;
    out.p[j][(static_cast<int64_t>(b) * n + c) * Nout + o] = in.p[j][(static_cast<int64_t>(b) * n + c) * Nin + idx[o]];
}

// d[..][o*ops+q] = v[..][o*cnt+2q+1] - v[..][o*cnt+2q]
__global__ __launch_bounds__(256) void k_pair_diff(Act v, int64_t Nv, Act d, int64_t Nout, int ops, int cnt,
                                                   CrtInfo crt) {
    const int j = blockIdx.y, b = blockIdx.z;
    const int n = crt.n[j], p = crt.p[j];
    const int64_t Nd = Nout * ops;
    const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= Nd * n) return;
    const int64_t c = t / Nd, e = t % Nd, o = e / ops, q = e % ops;
    const act_t* V = v.p[j] + (static_cast<int64_t>(b) * n + c) * Nv + o * cnt + 2 * q;
    int32_t x = V[1] - V[0];
    d.p[j][(static_cast<int64_t>(b) * n + c) * Nd + e] = static_cast<act_t>(x < 0 ? x + p : x);
}

// nv[o*cnt1+q] = v[o*cnt+2q] + r[o*ops+q]; odd leftover copied to slot ops
__global__ __launch_bounds__(256) void k_pair_add(Act v, int64_t Nv, Act r, Act nv, int64_t Nout, int ops, int cnt,
                                                  int cnt1, CrtInfo crt) {
    const int j = blockIdx.y, b = blockIdx.z;
    const int n = crt.n[j], p = crt.p[j];
    const int64_t Nn = Nout * cnt1, Nr = Nout * ops;
    const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= Nn * n) return;
    const int64_t c = t / Nn, e = t % Nn, o = e / cnt1, q = e % cnt1;
    const act_t* V = v.p[j] + (static_cast<int64_t>(b) * n + c) * Nv + o * cnt;
    act_t val;
    if (q < ops) {
        int32_t x = V[2 * q] + r.p[j][(static_cast<int64_t>(b) * n + c) * Nr + o * ops + q];
        val = static_cast<act_t>(x >= p ? x - p : x);
    } else {
        val = V[cnt - 1];
    }
    nv.p[j][(static_cast<int64_t>(b) * n + c) * Nn + e] = val;
}

__global__ __launch_bounds__(256) void k_add(Act x, Act y, int64_t N, CrtInfo crt) {
    const int j = blockIdx.y, b = blockIdx.z;
    const int n = crt.n[j], p = crt.p[j];
    const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= N * n) return;
    const int64_t off = static_cast<int64_t>(b) * n * N + t;
    int32_t v = x.p[j][off] + y.p[j][off];
    x.p[j][off] = static_cast<act_t>(v >= p ? v - p : v);
}

// out[o] = sum_s in[idx[o*K+s]]
__global__ __launch_bounds__(256) void k_window_sum(Act in, int64_t Nin, Act out, int64_t Nout, const int64_t* idx,
                                                    int K, CrtInfo crt) {
    const int j = blockIdx.y, b = blockIdx.z;
    const int n = crt.n[j], p = crt.p[j];
    const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= Nout * n) return;
    const int64_t c = t / Nout, o = t % Nout;
    const act_t* I = in.p[j] + (static_cast<int64_t>(b) * n + c) * Nin;
    int32_t acc = 0;
    for (int s = 0; s < K; ++s) acc += I[idx[o * K + s]];
    out.p[j][(static_cast<int64_t>(b) * n + c) * Nout + o] = static_cast<act_t>(acc % p);
}

__global__ __launch_bounds__(512) void k_aes_test(const u128* in, u128* out, int64_t n, const uint32_t* te0,
                                                  const uint32_t* rk) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_aes[DASH_AES_LDS_WORDS];
    aes_lds_fill(lds_aes, te0);
    const AesCtx aes = aes_ctx(lds_aes, rk);
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x)
        out[i] = aes_encrypt(aes, in[i]);
}

// hardened pads (dev.h hard_block) of n keys: out[4 i + q] = pad q of block blk[i] of (key[i], gate[i], sub[i])
__global__ __launch_bounds__(256) void k_hard_test(const u128* key, const uint64_t* gate, const uint32_t* sub,
                                                   const uint32_t* blk, u128* out, int64_t n) {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        u128 p[4];
        hard_block(key[i], gate[i], sub[i], blk[i], p);
#pragma unroll
        for (int q = 0; q < 4; ++q) out[4 * i + q] = p[q];
    }
}

// Throughput probe: every lane runs `iters` x 2 chained encryptions.
__global__ __launch_bounds__(512) void k_aes_bench(u128* out, int iters, const uint32_t* te0) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_aes[DASH_AES_LDS_WORDS];
    aes_lds_fill(lds_aes, te0);
    const AesCtx aes = aes_ctx(lds_aes, nullptr);
    const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    u128 x = static_cast<u128>(i), y = ~static_cast<u128>(i);
    for (int it = 0; it < iters; ++it) aes_encrypt2(aes, x, y, x, y);
    out[i] = x ^ y;
}

// labels: component-major [n][N]; comp[e] = compress, decomp = decompress(comp)
__global__ __launch_bounds__(256) void k_codec_test(const int16_t* L, int64_t N, int q, const ModC* mc, u128* comp,
                                                    int16_t* decomp) {
    const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (e >= N) return;
    const ModC m = mc[q];
    const u128 C = compress_cm(L + e, N, m);
    comp[e] = C;
    DigitStream s;
    s.init(C);
    CompressFwd f;
    f.init();
    for (int i = 0; i < static_cast<int>(m.n); ++i) {
        uint32_t d = s.next(m);
        decomp[i * N + e] = static_cast<int16_t>(d);
        f.push(d, m);
    }
    // forward compress must agree with reverse Horner
    if (f.finish() != C) decomp[e] = -1;
}

static inline dim3 g1(int64_t n, int y, int z) { return dim3(static_cast<unsigned>((n + 255) / 256), y, z); }
static inline int64_t nmax(const CrtInfo& c) {
    int m = 0;
    for (int j = 0; j < c.k; ++j) m = c.n[j] > m ? c.n[j] : m;
    return m;
}

void launch_copy_gather(const Act& in, int64_t Nin, const Act& out, int64_t Nout, const int64_t* idx,
                        const CrtInfo& crt, int B, hipStream_t st) {
    hipLaunchKernelGGL(k_copy_gather, g1(Nout * nmax(crt), crt.k, B), dim3(256), 0, st, in, Nin, out, Nout, idx, crt);
}
void launch_pair_diff(const Act& v, int64_t Nv, const Act& d, int64_t Nout, int ops, int cnt, const CrtInfo& crt,
                      int B, hipStream_t st) {
    hipLaunchKernelGGL(k_pair_diff, g1(Nout * ops * nmax(crt), crt.k, B), dim3(256), 0, st, v, Nv, d, Nout, ops, cnt,
                       crt);
}
void launch_pair_add(const Act& v, int64_t Nv, const Act& r, const Act& nv, int64_t Nout, int ops, int cnt, int cnt1,
                     const CrtInfo& crt, int B, hipStream_t st) {
    hipLaunchKernelGGL(k_pair_add, g1(Nout * cnt1 * nmax(crt), crt.k, B), dim3(256), 0, st, v, Nv, r, nv, Nout, ops,
                       cnt, cnt1, crt);
}
void launch_add(const Act& x, const Act& y, int64_t N, const CrtInfo& crt, int B, hipStream_t st) {
    hipLaunchKernelGGL(k_add, g1(N * nmax(crt), crt.k, B), dim3(256), 0, st, x, y, N, crt);
}
void launch_window_sum(const Act& in, int64_t Nin, const Act& out, int64_t Nout, const int64_t* idx, int K,
                       const CrtInfo& crt, int B, hipStream_t st) {
    hipLaunchKernelGGL(k_window_sum, g1(Nout * nmax(crt), crt.k, B), dim3(256), 0, st, in, Nin, out, Nout, idx, K,
                       crt);
}
// out[c][r] = in[r][c]: 64x64 tiles through LDS (row pitch 65: conflict-free
// column reads), both global sides coalesced; element types may differ (label
// components < 256: int16 host layout <-> byte activations).
// grid (ceil(cols/64), ceil(rows/64))
template <class Tin, class Tout>
__global__ __launch_bounds__(256) void k_transpose(const Tin* __restrict__ in, Tout* __restrict__ out, int64_t rows,
                                                   int64_t cols) {
    __shared__ int16_t t[64][65];
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const int64_t c0 = static_cast<int64_t>(blockIdx.x) * 64, r0 = static_cast<int64_t>(blockIdx.y) * 64;
    for (int y = ty; y < 64; y += 4) {
        const int64_t r = r0 + y, c = c0 + tx;
        if (r < rows && c < cols) t[y][tx] = static_cast<int16_t>(in[r * cols + c]);
    }
    __syncthreads();
    for (int y = ty; y < 64; y += 4) {
        const int64_t c = c0 + y, r = r0 + tx;
        if (r < rows && c < cols) out[c * rows + r] = static_cast<Tout>(t[tx][y]);
    }
}
template <class Tin, class Tout>
__global__ __launch_bounds__(256) void k_transpose_res(TrRes a) {
    __shared__ int16_t t[64][65];
    const int j = blockIdx.z;
    const int64_t rows = a.rows[j], cols = a.cols[j];
    const int64_t c0 = static_cast<int64_t>(blockIdx.x) * 64, r0 = static_cast<int64_t>(blockIdx.y) * 64;
    if (c0 >= cols || r0 >= rows) return;  // block-uniform: this residue's matrix is smaller than the grid
    const Tin* __restrict__ in = static_cast<const Tin*>(a.in[j]);
    Tout* __restrict__ out = static_cast<Tout*>(a.out[j]);
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int y = ty; y < 64; y += 4) {
        const int64_t r = r0 + y, c = c0 + tx;
        if (r < rows && c < cols) t[y][tx] = static_cast<int16_t>(in[r * cols + c]);
    }
    __syncthreads();
    for (int y = ty; y < 64; y += 4) {
        const int64_t c = c0 + y, r = r0 + tx;
        if (r < rows && c < cols) out[c * rows + r] = static_cast<Tout>(t[tx][y]);
    }
}
// grid (blocks, residue): out[j][x] = in[j][x], x < rows[j] * cols[j]; 4 components per lane-iteration
template <class Tin, class Tout>
__global__ __launch_bounds__(256) void k_cast_res(TrRes a) {
    const int j = blockIdx.y;
    const int64_t n = a.rows[j] * a.cols[j];
    const Tin* __restrict__ in = static_cast<const Tin*>(a.in[j]);
    Tout* __restrict__ out = static_cast<Tout*>(a.out[j]);
    for (int64_t x = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; x < n;
         x += static_cast<int64_t>(gridDim.x) * blockDim.x)
        out[x] = static_cast<Tout>(in[x]);
}
// grid (blocks, residue) over the component-major index x = q * N + e
template <bool TO_ACT>
__global__ __launch_bounds__(256) void k_chunk_res(TrRes a) {
    const int j = blockIdx.y;
    const int64_t N = a.cols[j], n = a.rows[j] * N;
    for (int64_t x = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; x < n;
         x += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t q = x / N, e = x - q * N;
        const int64_t cx = ((q >> 3) * N + e) * 8 + (q & 7);
        if (TO_ACT)
            static_cast<act_t*>(a.out[j])[x] = static_cast<act_t>(static_cast<const int16_t*>(a.in[j])[cx]);
        else
            static_cast<int16_t*>(a.out[j])[cx] = static_cast<int16_t>(static_cast<const act_t*>(a.in[j])[x]);
    }
}
__global__ __launch_bounds__(256) void k_narrow(const int16_t* __restrict__ in, act_t* __restrict__ out, int64_t n) {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x)
        out[i] = static_cast<act_t>(in[i]);
}
void launch_narrow(const int16_t* in, act_t* out, int64_t n, hipStream_t st) {
    const unsigned nb = static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 16384)));
    hipLaunchKernelGGL(k_narrow, dim3(nb), dim3(256), 0, st, in, out, n);
}

// Output labels of every residue written straight into mapped pinned host memory by one launch, instead of one
// copy-engine transfer per residue (k = 7 D2H copies were ~35 us of a 1.5 ms batch-1 latency, r05 timeline).
// grid (blocks, k); 16-byte stores where both sides are 16-byte aligned. The stream synchronize after the launch
// makes the stores visible to the host (system-scope release at the kernel's end, fenced here as well).
__global__ __launch_bounds__(256) void k_fetch_res(FetchRes a) {
    const int j = blockIdx.y;
    const int64_t nb = a.bytes[j];
    const uint8_t* s = static_cast<const uint8_t*>(a.in[j]);
    uint8_t* d = static_cast<uint8_t*>(a.out[j]);
    const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
    const int64_t t0 = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    const bool al = ((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 15u) == 0;
    const int64_t n16 = al ? nb / 16 : 0;
    for (int64_t i = t0; i < n16; i += stride)
        reinterpret_cast<uint4*>(d)[i] = reinterpret_cast<const uint4*>(s)[i];
    for (int64_t i = n16 * 16 + t0; i < nb; i += stride) d[i] = s[i];
    __threadfence_system();
}
void launch_fetch_res(const FetchRes& a, hipStream_t st) {
    int64_t mx = 1;
    for (int j = 0; j < a.k; ++j) mx = std::max(mx, a.bytes[j]);
    const unsigned nb = static_cast<unsigned>(std::min<int64_t>((mx / 16 + 255) / 256 + 1, 64));
    hipLaunchKernelGGL(k_fetch_res, dim3(nb, static_cast<unsigned>(a.k)), dim3(256), 0, st, a);
}

// Online message #1 encoded on the device by the garbler (core.h lab_affine per component, reference
// garbled_circuit_interface.h garble_inputs): grid (ceil(N / 1024), k, slots). A block owns one (slot, residue)
// and 1024 elements: the modulus is uniform, each lane reduces its 4 inputs mod p once and walks the residue's
// component rows with 4-byte loads and stores (independent iterations, unrolled). The first round-6 form (one lane
// per (residue, component, element), the residue found per lane) issued three dependent round trips per lane for
// one byte: 333 us per 20-GC MiniONN launch, 599 us per 41 GCs; one row per block: 224 us per 41 GCs; this form:
// 248 us per 55 GCs (r06 headline traces, profiles/r06_headline_b165_kernels_final.txt).
// Both reductions (x mod p, (w + v r) mod p) are a float-reciprocal quotient plus one correction, exact below
// 2^22; an input beyond that takes the 64-bit path.
__device__ __forceinline__ uint32_t mod_small(int64_t x, uint32_t p, float inv) {
    if (x > -(int64_t(1) << 22) && x < (int64_t(1) << 22)) {
        const int32_t xi = static_cast<int32_t>(x);
        int32_t r = xi - static_cast<int32_t>(floorf(static_cast<float>(xi) * inv)) * static_cast<int32_t>(p);
        if (r < 0) r += p;
        if (r >= static_cast<int32_t>(p)) r -= p;
        return static_cast<uint32_t>(r);
    }
    const int64_t r = x % static_cast<int64_t>(p);
    return static_cast<uint32_t>(r < 0 ? r + p : r);
}
constexpr int kEncPerLane = 4;
__global__ __launch_bounds__(256) void k_encode_in(EncIn a, const int64_t* __restrict__ x, int64_t N) {
    const int s = blockIdx.z;
    const int j = static_cast<int>(blockIdx.y);  // residue (uniform)
    const int n = a.n[j];
    const uint32_t p = static_cast<uint32_t>(a.p[j]);
    const float inv = a.inv[j];
    const act_t* rr = a.r[j] + s * a.wstride;
    const act_t* w0 = a.w0[j] + s * a.wstride;
    act_t* o0 = a.out[j] + static_cast<int64_t>(s) * n * N;
    const int64_t* xs = x + static_cast<int64_t>(s) * N;
    // rows of this residue are 4-byte aligned when N is and the slot bases are (uniform)
    const bool al = N % kEncPerLane == 0 &&
                    ((reinterpret_cast<uintptr_t>(w0) | reinterpret_cast<uintptr_t>(o0)) & 3u) == 0;
    const int64_t step = static_cast<int64_t>(gridDim.x) * 256 * kEncPerLane;
    for (int64_t e = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) * kEncPerLane; e < N; e += step) {
        // x mod p once per element, then every component row of the residue
        uint32_t v[kEncPerLane];
#pragma unroll
        for (int u = 0; u < kEncPerLane; ++u) v[u] = e + u < N ? mod_small(xs[e + u], p, inv) : 0u;
        if (al) {
            // kEncRows rows' loads issued before any of their stores (the output rows may alias the inputs as far
            // as the compiler knows, so a plain loop made every row one full round trip)
            constexpr int kEncRows = 8;
            for (int c0 = 0; c0 < n; c0 += kEncRows) {
                uint32_t r8[kEncRows], w8[kEncRows];
#pragma unroll
                for (int h = 0; h < kEncRows; ++h) {
                    const int c = min(c0 + h, n - 1);
                    r8[h] = rr[c];
                    w8[h] = *reinterpret_cast<const uint32_t*>(w0 + static_cast<int64_t>(c) * N + e);
                }
#pragma unroll
                for (int h = 0; h < kEncRows; ++h) {
                    if (c0 + h >= n) break;
                    uint32_t o4 = 0;
#pragma unroll
                    for (int u = 0; u < kEncPerLane; ++u)
                        o4 |= mod_small(((w8[h] >> (8 * u)) & 0xffu) + v[u] * r8[h], p, inv) << (8 * u);
                    *reinterpret_cast<uint32_t*>(o0 + static_cast<int64_t>(c0 + h) * N + e) = o4;
                }
            }
        } else {
            for (int c = 0; c < n; ++c) {
                const uint32_t r = rr[c];
                for (int u = 0; u < kEncPerLane && e + u < N; ++u) {
                    const int64_t f = static_cast<int64_t>(c) * N + e + u;
                    o0[f] = static_cast<act_t>(mod_small(w0[f] + v[u] * r, p, inv));
                }
            }
        }
    }
}
void launch_encode_in(const EncIn& a0, const int64_t* x, int64_t N, int slots, hipStream_t st) {
    EncIn a = a0;
    a.pre[0] = 0;
    for (int j = 0; j < a.k; ++j) {
        a.pre[j + 1] = a.pre[j] + a.n[j];
        a.inv[j] = 1.0f / static_cast<float>(a.p[j]);
    }
    if (slots > 65535) throw std::runtime_error("encode_in: more than 65535 slots in one launch");
    const int64_t bx = (N + 256 * kEncPerLane - 1) / (256 * kEncPerLane);
    hipLaunchKernelGGL(k_encode_in, dim3(static_cast<unsigned>(std::min<int64_t>(bx, 4096)), static_cast<unsigned>(a.k),
                                         static_cast<unsigned>(slots)),
                       dim3(256), 0, st, a, x, N);
}

static inline dim3 grid_tr(int64_t rows, int64_t cols) {
    return dim3(static_cast<unsigned>((cols + 63) / 64), static_cast<unsigned>((rows + 63) / 64));
}
void launch_transpose16(const int16_t* in, int16_t* out, int64_t rows, int64_t cols, hipStream_t st) {
    hipLaunchKernelGGL((k_transpose<int16_t, int16_t>), grid_tr(rows, cols), dim3(256), 0, st, in, out, rows, cols);
}
void launch_transpose_to_act(const int16_t* in, act_t* out, int64_t rows, int64_t cols, hipStream_t st) {
    hipLaunchKernelGGL((k_transpose<int16_t, act_t>), grid_tr(rows, cols), dim3(256), 0, st, in, out, rows, cols);
}
void launch_transpose_from_act(const act_t* in, int16_t* out, int64_t rows, int64_t cols, hipStream_t st) {
    hipLaunchKernelGGL((k_transpose<act_t, int16_t>), grid_tr(rows, cols), dim3(256), 0, st, in, out, rows, cols);
}

static inline dim3 grid_tr_res(const TrRes& a) {
    int64_t r = 1, c = 1;
    for (int j = 0; j < a.k; ++j) {
        r = std::max(r, a.rows[j]);
        c = std::max(c, a.cols[j]);
    }
    return dim3(static_cast<unsigned>((c + 63) / 64), static_cast<unsigned>((r + 63) / 64), static_cast<unsigned>(a.k));
}
void launch_transpose_to_act_res(const TrRes& a, hipStream_t st) {
    hipLaunchKernelGGL((k_transpose_res<int16_t, act_t>), grid_tr_res(a), dim3(256), 0, st, a);
}
void launch_transpose_from_act_res(const TrRes& a, hipStream_t st) {
    hipLaunchKernelGGL((k_transpose_res<act_t, int16_t>), grid_tr_res(a), dim3(256), 0, st, a);
}

static inline dim3 grid_cast_res(const TrRes& a) {
    int64_t mx = 1;
    for (int j = 0; j < a.k; ++j) mx = std::max(mx, a.rows[j] * a.cols[j]);
    return dim3(static_cast<unsigned>(std::min<int64_t>((mx + 255) / 256, 4096)), static_cast<unsigned>(a.k));
}
void launch_cast_to_act_res(const TrRes& a, hipStream_t st) {
    hipLaunchKernelGGL((k_cast_res<int16_t, act_t>), grid_cast_res(a), dim3(256), 0, st, a);
}
void launch_cast_from_act_res(const TrRes& a, hipStream_t st) {
    hipLaunchKernelGGL((k_cast_res<act_t, int16_t>), grid_cast_res(a), dim3(256), 0, st, a);
}

void launch_unchunk_to_act_res(const TrRes& a, hipStream_t st) {
    hipLaunchKernelGGL(k_chunk_res<true>, grid_cast_res(a), dim3(256), 0, st, a);
}
void launch_chunk_from_act_res(const TrRes& a, hipStream_t st) {
    hipLaunchKernelGGL(k_chunk_res<false>, grid_cast_res(a), dim3(256), 0, st, a);
}

// one block per descriptor; 4-byte words where source, destination and size allow, bytes otherwise
__global__ __launch_bounds__(256) void k_scatter(const ScatterDesc* d, const uint8_t* src, int b) {
    const ScatterDesc c = d[blockIdx.x];
    const uint8_t* s = src + c.off;
    uint8_t* t = c.dst0 + static_cast<size_t>(b) * c.stride;
    if (((reinterpret_cast<uintptr_t>(t) | reinterpret_cast<uintptr_t>(s) | c.bytes) & 3) == 0) {
        for (size_t i = threadIdx.x; i < c.bytes / 4; i += blockDim.x)
            reinterpret_cast<uint32_t*>(t)[i] = reinterpret_cast<const uint32_t*>(s)[i];
    } else {
        for (size_t i = threadIdx.x; i < c.bytes; i += blockDim.x) t[i] = s[i];
    }
}
void launch_scatter(const ScatterDesc* d, int n, const uint8_t* src, int b, hipStream_t st) {
    hipLaunchKernelGGL(k_scatter, dim3(static_cast<unsigned>(n)), dim3(256), 0, st, d, src, b);
}

void launch_aes_test(const u128* in, u128* out, int64_t n, const AesGlobals& g, hipStream_t st) {
    const unsigned nb = static_cast<unsigned>(std::min<int64_t>((n + 511) / 512, 2048));
    hipLaunchKernelGGL(k_aes_test, dim3(nb), dim3(512), 0, st, in, out, n, g.te0, g.rk);
}
void launch_aes_bench(u128* out, int blocks, int iters, const AesGlobals& g, hipStream_t st) {
    hipLaunchKernelGGL(k_aes_bench, dim3(blocks), dim3(512), 0, st, out, iters, g.te0);
}
void launch_hard_test(const u128* key, const uint64_t* gate, const uint32_t* sub, const uint32_t* blk, u128* out,
                      int64_t n, hipStream_t st) {
    hipLaunchKernelGGL(k_hard_test, dim3(static_cast<unsigned>(std::min<int64_t>((n + 255) / 256, 1024))), dim3(256), 0,
                       st, key, gate, sub, blk, out, n);
}
void launch_codec_test(const int16_t* labels, int64_t N, int q, const ModC* mc, u128* comp, int16_t* decomp,
                       hipStream_t st) {
    hipLaunchKernelGGL(k_codec_test, g1(N, 1, 1), dim3(256), 0, st, labels, N, q, mc, comp, decomp);
}

}  // namespace dev
}  // namespace dash
