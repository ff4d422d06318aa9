// dash_amd native core: scalar domain, CRT math, label primitives, fixed-key
// AES hash (AES-NI), AES-CTR label PRG and a small thread pool.
//
// Behavioural parity with the reference (UzL-ITS/dash):
//   * label width n_p = floor(128 / log2 p)         dash/include/garbling/label_tensor.h:1353-1357
//   * compress C = sum_j L_j p^j (uint128, L_0 LSD)   label_tensor.h:715-724
//   * H(C) = AES-128_K(LE bytes of C), K = 00..0f     crypto/cpu_aes_engine.h:23-40
//   * color = component 0, offsets have R[0] = 1      label_tensor.h:1303-1307
//   * CRT helpers (signed modulo, mul_inv, CRT)      misc/util.h:43-156
// The implementation is new: chunked Horner/long-division digit codecs,
// pipelined AES-NI, a deterministic AES-CTR PRG (the reference uses RDRAND,
// which makes garbling non-reproducible and impossible to mirror on the GPU).
#pragma once

#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace dash {

using u128 = unsigned __int128;
using i64 = int64_t;
using u64 = uint64_t;
using comp_t = int16_t;  // one label component ("crt_val_t" in the reference)

#define DASH_CHECK(cond, msg)                                                 \
    do {                                                                      \
        if (!(cond)) throw std::runtime_error(std::string("dash: ") + (msg)); \
    } while (0)

// ----------------------------------------------------------------------------
// Scalar / CRT math
// ----------------------------------------------------------------------------
inline int nr_comps(i64 p) {
    // Same floating point formula as the reference so label widths match for
    // every modulus (including prime powers such as 32).
    return static_cast<int>(std::floor(128.0 / std::log2(static_cast<double>(p))));
}

// Label PRG digits per AES-CTR block. The m least significant base-p digits of a
// uniform 128-bit block are uniform on Z_p^m up to statistical distance
// p^m / 2^128, so m is the largest count with p^m <= 2^64 (distance <= 2^-64);
// for p = 2^b all 128 / b digits (exact). p = 7: 22 digits per block instead of
// 2 (one 64-bit half per component), i.e. 3 AES per 45-component label, not 23.
inline int prg_digits(i64 p) {
    if ((p & (p - 1)) == 0) {
        int b = 0;
        while ((i64(1) << b) < p) ++b;
        return 128 / b;
    }
    int m = 0;
    unsigned __int128 v = 1;
    while (v * static_cast<unsigned __int128>(p) <= (static_cast<unsigned __int128>(1) << 64)) {
        v *= static_cast<unsigned __int128>(p);
        ++m;
    }
    return m;
}
// AES-CTR blocks of one label
inline int prg_blocks(i64 p) {
    const int m = prg_digits(p);
    return (nr_comps(p) + m - 1) / m;
}

inline i64 pmod(i64 a, i64 p) {
    i64 r = a % p;
    return r < 0 ? r + p : r;
}

// Multiplicative inverse of a mod b (extended Euclid), b < 2^16.
inline i64 mul_inv(u128 a, i64 b) {
    if (b == 1) return 1;
    i64 b0 = b;
    i64 x0 = 0, x1 = 1;
    u128 aa = a;
    u128 bb = static_cast<u128>(b);
    while (aa > 1) {
        if (bb == 0) throw std::runtime_error("dash: mul_inv of non-invertible value");
        i64 q = static_cast<i64>(aa / bb);
        u128 t = bb;
        bb = aa % bb;
        aa = t;
        i64 tx = x0;
        x0 = x1 - q * x0;
        x1 = tx;
    }
    if (x1 < 0) x1 += b0;
    return x1;
}

std::vector<int> first_primes(int k);

// ----------------------------------------------------------------------------
// Label digit codecs (compress / decompress)
// ----------------------------------------------------------------------------
struct ModInfo {
    int p = 0;        // modulus
    int n = 0;        // components per label
    int chunk = 1;    // digits per 32-bit chunk (p^chunk < 2^32)
    u64 pchunk = 1;   // p^chunk
    bool pow2 = false;
    int bits = 0;     // log2 p when pow2
    int prg_m = 2;    // label PRG digits per AES block (prg_digits)
};

const ModInfo& mod_info(int p);

// C = sum_j L[j] * p^j  (mod 2^128)
inline u128 compress(const comp_t* L, const ModInfo& m) {
    const int n = m.n;
    if (m.pow2) {
        u128 C = 0;
        for (int j = n - 1; j >= 0; --j) C = (C << m.bits) | static_cast<u128>(static_cast<uint16_t>(L[j]));
        return C;
    }
    // Horner over chunks of `chunk` digits evaluated in 64-bit, then folded in
    // 128-bit: C = C * p^c + chunk_value.
    u128 C = 0;
    int j = n - 1;
    const u64 p = static_cast<u64>(m.p);
    int first = n % m.chunk;
    if (first == 0) first = m.chunk;
    // leading (partial) chunk
    {
        u64 v = 0;
        for (int t = 0; t < first; ++t, --j) v = v * p + static_cast<u64>(static_cast<uint16_t>(L[j]));
        C = v;
    }
    while (j >= 0) {
        u64 v = 0;
        for (int t = 0; t < m.chunk; ++t, --j) v = v * p + static_cast<u64>(static_cast<uint16_t>(L[j]));
        C = C * static_cast<u128>(m.pchunk) + v;
    }
    return C;
}

// compress() of four labels of one modulus at once: four independent Horner chains interleaved, so the
// dependent 64-bit multiply-adds of one label overlap those of the other three (the host input encoder's
// online message #1, Garbler::encode_compressed)
inline void compress4(const comp_t* const L[4], const ModInfo& m, u128 out[4]) {
    const int n = m.n;
    if (m.pow2) {
        for (int q = 0; q < 4; ++q) out[q] = compress(L[q], m);
        return;
    }
    const u64 p = static_cast<u64>(m.p);
    int j = n - 1;
    int first = n % m.chunk;
    if (first == 0) first = m.chunk;
    u128 C[4];
    {
        u64 v[4] = {0, 0, 0, 0};
        for (int t = 0; t < first; ++t, --j)
            for (int q = 0; q < 4; ++q) v[q] = v[q] * p + static_cast<u64>(static_cast<uint16_t>(L[q][j]));
        for (int q = 0; q < 4; ++q) C[q] = v[q];
    }
    while (j >= 0) {
        u64 v[4] = {0, 0, 0, 0};
        for (int t = 0; t < m.chunk; ++t, --j)
            for (int q = 0; q < 4; ++q) v[q] = v[q] * p + static_cast<u64>(static_cast<uint16_t>(L[q][j]));
        for (int q = 0; q < 4; ++q) C[q] = C[q] * static_cast<u128>(m.pchunk) + v[q];
    }
    for (int q = 0; q < 4; ++q) out[q] = C[q];
}

// Inverse of compress for a valid C (< p^n). For arbitrary C the first n-1
// digits are the base-p digits and the top digit is reduced mod p.
inline void decompress(u128 C, comp_t* L, const ModInfo& m) {
    const int n = m.n;
    if (m.pow2) {
        const u128 mask = (static_cast<u128>(1) << m.bits) - 1;
        for (int j = 0; j < n; ++j) {
            L[j] = static_cast<comp_t>(static_cast<int>(C & mask));
            C >>= m.bits;
        }
        L[n - 1] = static_cast<comp_t>(static_cast<int>(L[n - 1]) % m.p);
        return;
    }
    const u64 D = m.pchunk;
    const u64 p = static_cast<u64>(m.p);
    int j = 0;
    while (j < n) {
        // (C, r) = divmod(C, D) with D < 2^32
        u64 hi = static_cast<u64>(C >> 64), lo = static_cast<u64>(C);
        u64 qh = hi / D, r = hi % D;
        u64 x1 = (r << 32) | (lo >> 32);
        u64 q1 = x1 / D;
        r = x1 % D;
        u64 x0 = (r << 32) | (lo & 0xffffffffull);
        u64 q0 = x0 / D;
        r = x0 % D;
        C = (static_cast<u128>(qh) << 64) | (static_cast<u128>(q1) << 32) | q0;
        int cnt = std::min(m.chunk, n - j);
        for (int t = 0; t < cnt; ++t, ++j) {
            L[j] = static_cast<comp_t>(r % p);
            r /= p;
        }
    }
    // top digit: (floor(C_orig / p^(n-1))) mod p  -- matches the reference's
    // final `%= modulus` for in-range payloads.
    (void)C;
}

// ----------------------------------------------------------------------------
// Label vector arithmetic (component-wise mod p)
// ----------------------------------------------------------------------------
inline void lab_add(comp_t* a, const comp_t* b, int n, int p) {
    for (int i = 0; i < n; ++i) {
        int v = a[i] + b[i];
        a[i] = static_cast<comp_t>(v >= p ? v - p : v);
    }
}
inline void lab_sub(comp_t* a, const comp_t* b, int n, int p) {
    for (int i = 0; i < n; ++i) {
        int v = a[i] - b[i];
        a[i] = static_cast<comp_t>(v < 0 ? v + p : v);
    }
}
// a = a * c mod p  (c any signed integer)
inline void lab_scale(comp_t* a, i64 c, int n, int p) {
    i64 cc = pmod(c, p);
    for (int i = 0; i < n; ++i) a[i] = static_cast<comp_t>((a[i] * cc) % p);
}
// a = a + c*b mod p
inline void lab_axpy(comp_t* a, i64 c, const comp_t* b, int n, int p) {
    i64 cc = pmod(c, p);
    for (int i = 0; i < n; ++i) a[i] = static_cast<comp_t>((a[i] + cc * b[i]) % p);
}
// out = base + c*off mod p
inline void lab_affine(comp_t* out, const comp_t* base, i64 c, const comp_t* off, int n, int p) {
    i64 cc = pmod(c, p);
    for (int i = 0; i < n; ++i) out[i] = static_cast<comp_t>((base[i] + cc * off[i]) % p);
}

// ----------------------------------------------------------------------------
// AES-128 (AES-NI)
// ----------------------------------------------------------------------------
struct AesKey {
    __m128i rk[11];
};
void aes_expand(const uint8_t key[16], AesKey& out);
// Round keys in the byte order a portable/GPU implementation needs (11x16 B).
void aes_round_key_bytes(const AesKey& k, uint8_t out[176]);

inline __m128i aes_enc_block(__m128i x, const AesKey& k) {
    x = _mm_xor_si128(x, k.rk[0]);
    for (int r = 1; r < 10; ++r) x = _mm_aesenc_si128(x, k.rk[r]);
    return _mm_aesenclast_si128(x, k.rk[10]);
}

inline __m128i u128_to_m(u128 v) {
    __m128i r;
    std::memcpy(&r, &v, 16);
    return r;
}
inline u128 m_to_u128(__m128i v) {
    u128 r;
    std::memcpy(&r, &v, 16);
    return r;
}

// The fixed-key hash used for every gate (key 00 01 .. 0f).
const AesKey& fixed_key();
inline u128 hash(u128 x) { return m_to_u128(aes_enc_block(u128_to_m(x), fixed_key())); }
void hash_batch(const u128* in, u128* out, size_t n);

// ----------------------------------------------------------------------------
// Hardened-encoding hash (docs/SECURITY.md): a tweakable hash of a compressed
// key label K, H(K, gate, sub, blk) = the ChaCha12 block function (feed-forward
// included) on the state
//   [sigma0..3][K (4 words, LE)][gate lo, gate hi, sub, "HARD"][blk, 0, 0, 0]
// whose 512-bit output is four 128-bit pads (pad q = words 4q..4q+3, LE). The
// table entry of slot s of a projection row is masked by pad (s mod 4) of
// block s / 4, and (gate, sub) is unique per row within a GC, so no two
// entries of a GC share a pad: unlike the reference's fixed-key AES H(K), a
// key that feeds several outputs (fan-out rows, a ReLU's k half gates, a
// half gate's mini table) gets an independent pad per output.
// ----------------------------------------------------------------------------
constexpr int kChaRounds = 12;
constexpr uint32_t kHardTag = 0x44524148u;  // "HARD"

inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// ChaCha block function with `rounds` rounds (even) and feed-forward; in/out 16 words
inline void chacha_core(const uint32_t in[16], uint32_t out[16], int rounds) {
    uint32_t x[16];
    for (int i = 0; i < 16; ++i) x[i] = in[i];
    auto qr = [&x](int a, int b, int c, int d) {
        x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 16);
        x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 12);
        x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 8);
        x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 7);
    };
    for (int r = 0; r < rounds; r += 2) {
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15);
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14);
    }
    for (int i = 0; i < 16; ++i) out[i] = x[i] + in[i];
}

// The four pads of block `blk` of key K under tweak (gate, sub)
inline void hard_block(u128 K, u64 gate, uint32_t sub, uint32_t blk, u128 pads[4]) {
    uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                      static_cast<uint32_t>(K), static_cast<uint32_t>(K >> 32), static_cast<uint32_t>(K >> 64),
                      static_cast<uint32_t>(K >> 96), static_cast<uint32_t>(gate), static_cast<uint32_t>(gate >> 32),
                      sub, kHardTag, blk, 0u, 0u, 0u};
    uint32_t o[16];
    chacha_core(s, o, kChaRounds);
    for (int q = 0; q < 4; ++q)
        pads[q] = (static_cast<u128>((static_cast<u64>(o[4 * q + 3]) << 32) | o[4 * q + 2]) << 64) |
                  ((static_cast<u64>(o[4 * q + 1]) << 32) | o[4 * q]);
}

// pad of slot s
inline u128 hard_pad(u128 K, u64 gate, uint32_t sub, int s) {
    u128 p[4];
    hard_block(K, gate, sub, static_cast<uint32_t>(s) >> 2, p);
    return p[s & 3];
}

// The pads of one (key, tweak) row, one block computed at a time as slots are asked for
struct PadRow {
    u128 K = 0;
    u64 gate = 0;
    uint32_t sub = 0;
    int blk = -1;
    u128 p[4];
    PadRow() = default;
    PadRow(u128 k, u64 g, uint32_t s) : K(k), gate(g), sub(s) {}
    u128 get(int s) {
        if ((s >> 2) != blk) {
            blk = s >> 2;
            hard_block(K, gate, sub, static_cast<uint32_t>(blk), p);
        }
        return p[s & 3];
    }
};

// Tweak kinds (the high 16 bits of `sub`; the low bits index the row inside the gadget)
enum TweakKind : uint32_t {
    TW_APPROX = 1,  // sign gadget: residue j's approx row (slots: digits)
    TW_CAST1 = 2,   // reference casts (non-hardened only)
    TW_CAST2 = 3,   // sign gadget: digit d's carry projection
    TW_SIGN = 4,    // sign gadget: MSD -> outputs (slots: output moduli)
    TW_MMG = 5,     // mixed / generalized half gate, garbler half (key x_j)
    TW_MMY = 6,     // mixed half gate, evaluator half + mini (key y; slots: residues, then the packed minis)
    TW_MRS = 7,     // mixed-radix rescale rows (i < k: digit rows; i = k: final row)
    TW_SMRS = 8,    // mixed-radix sign rows
    TW_BE = 9,      // base extension rows
    TW_TRANS = 10,  // ReDash rescale: factor residue -> active residues
    TW_PROJ = 11,   // projection layer
    TW_GME = 12,    // generalized half gate, evaluator half (key y_j)
    TW_MMT = 13,    // mixed-mult layer: the residue-j mod transform (key x_2e+1)
};
inline uint32_t tw_sub(TweakKind k, uint32_t idx) { return (static_cast<uint32_t>(k) << 16) | (idx & 0xffffu); }

// A table mask: the reference's H(K) (hard == false) or the hardened pad of slot `slot`
struct Mask {
    bool hard = false;
    u64 gate = 0;
    uint32_t sub = 0;
    int slot = 0;
    Mask with_slot(int s) const {
        Mask m = *this;
        m.slot = s;
        return m;
    }
};

// ----------------------------------------------------------------------------
// Deterministic label PRG: AES-128-CTR keyed with the garbler seed.
// block(stream, ctr) = AES_k(stream << 64 | ctr); each block yields two
// 64-bit samples; component = sample mod p (bias <= p / 2^64).
// ----------------------------------------------------------------------------
struct Prg {
    AesKey key;
    explicit Prg(const uint8_t seed[16]) { aes_expand(seed, key); }
    Prg() {
        uint8_t z[16] = {0};
        aes_expand(z, key);
    }
    // n components of a uniform label mod p: block b = AES_seed(stream || ctr + b) gives components
    // b*m .. b*m + m - 1 as its least significant base-p digits (m = prg_digits(p)); ctr advances by
    // prg_blocks(p). The GPU garbler (garble_gpu.hip k_draw) produces the same digits.
    inline void label(u64 stream, u64& ctr, int p, int n, comp_t* out) const {
        const ModInfo& mi = mod_info(p);
        const int m = mi.prg_m;
        for (int j = 0; j < n; j += m) {
            u128 blk = (static_cast<u128>(stream) << 64) | ctr++;
            u128 V = m_to_u128(aes_enc_block(u128_to_m(blk), key));
            const int cnt = std::min(m, n - j);
            if (mi.pow2) {
                for (int u = 0; u < cnt; ++u, V >>= mi.bits) out[j + u] = static_cast<comp_t>(static_cast<u64>(V) & (p - 1));
                continue;
            }
            for (int u = 0; u < cnt;) {
                u64 r = static_cast<u64>(V % mi.pchunk);  // chunk of `chunk` digits
                V /= mi.pchunk;
                for (int c = 0; c < mi.chunk && u < cnt; ++c, ++u) {
                    out[j + u] = static_cast<comp_t>(r % static_cast<u64>(p));
                    r /= static_cast<u64>(p);
                }
            }
        }
    }
};

// Stream identifiers: distinct (layer, slot, element) triples never collide.
// 64-bit mix hash of an int64 array (public weights: GPU plan cache keys)
inline uint64_t hash_i64(const i64* w, size_t n) {
    uint64_t h = 0x9e3779b97f4a7c15ull ^ n;
    for (size_t i = 0; i < n; ++i) {
        h ^= static_cast<uint64_t>(w[i]) + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
        h *= 0xff51afd7ed558ccdull;
    }
    return h;
}

inline u64 stream_id(u64 layer, u64 slot, u64 elem) {
    return (layer << 44) ^ (slot << 36) ^ elem;
}
constexpr u64 kGlobalLayer = 0xFFFFF;

// ----------------------------------------------------------------------------
// Thread pool / parallel_for (static chunking, deterministic results)
// ----------------------------------------------------------------------------
int default_threads();
void set_default_threads(int n);
void parallel_for(i64 n, const std::function<void(i64, i64)>& body, int nthreads = 0);

// ----------------------------------------------------------------------------
// Typed, 64-byte aligned n-d array (the unit of the GarbledModel format)
// ----------------------------------------------------------------------------
enum class DType : uint8_t { i16 = 0, i32 = 1, i64 = 2, u128 = 3, u8 = 4 };
inline size_t dtype_size(DType d) {
    switch (d) {
        case DType::i16: return 2;
        case DType::i32: return 4;
        case DType::i64: return 8;
        case DType::u128: return 16;
        case DType::u8: return 1;
    }
    return 1;
}

// Large host buffers: anonymous mmap (already zero) advised to use 2 MiB
// transparent huge pages. In a VM every 4 KiB first-touch fault is an exit
// that serializes the worker threads; huge pages cut the faults 512x so the
// garbler and the host evaluator scale with threads.
void* big_alloc(size_t bytes, bool* zeroed);
void big_free(void* p, size_t bytes);
constexpr size_t kBigAlloc = size_t(1) << 20;

template <class T>
struct BigAllocator {
    using value_type = T;
    BigAllocator() = default;
    template <class U>
    BigAllocator(const BigAllocator<U>&) {}
    T* allocate(size_t n) { return static_cast<T*>(big_alloc(n * sizeof(T), nullptr)); }
    void deallocate(T* p, size_t n) { big_free(p, n * sizeof(T)); }
    template <class U>
    bool operator==(const BigAllocator<U>&) const { return true; }
    template <class U>
    bool operator!=(const BigAllocator<U>&) const { return false; }
};

struct Array {
    // Device-resident payload: the GPU garbler leaves its tables in HBM so the
    // evaluator on the same node copies them device-to-device (no PCIe round
    // trip). The host copy is fetched on first host access (serialize, CPU
    // evaluator, numpy), once, thread-safely, and shared by every copy.
    struct Device {
        std::shared_ptr<void> p;  // device buffer (deleter frees it)
        int device = -1;
        std::function<void(void* host, const void* dev, size_t n)> fetch;
        std::once_flag once;
        std::shared_ptr<uint8_t> host;
        // the buffer belongs to someone else (a HIP evaluator's table arena slot the GPU garbler wrote
        // into): `p` does not own it, and it is valid only while that slot holds this model
        bool external = false;
    };

    DType dtype = DType::u8;
    std::vector<i64> shape;
    std::shared_ptr<uint8_t> buf;
    size_t nbytes = 0;
    std::shared_ptr<Device> dev;
    // placeholder of a skeleton model (GarbledModel::deserialize_skeleton): the bytes were written straight into
    // the evaluator's table slot by the garbler (cross-process sink); no host or device payload here
    bool in_slot = false;

    Array() = default;
    Array(DType dt, std::vector<i64> shp) : dtype(dt), shape(std::move(shp)) {
        nbytes = shape_bytes();
        buf = host_alloc(nbytes);
    }
    // an array whose bytes live in a device buffer (no host storage until first host access)
    static Array on_device(DType dt, std::vector<i64> shp, std::shared_ptr<Device> d) {
        Array a;
        a.dtype = dt;
        a.shape = std::move(shp);
        a.nbytes = a.shape_bytes();
        a.dev = std::move(d);
        return a;
    }
    bool device_resident() const { return dev && dev->p; }
    const void* device_ptr() const { return device_resident() ? dev->p.get() : nullptr; }
    size_t count() const { return nbytes / dtype_size(dtype); }
    template <typename T>
    T* ptr() {
        return reinterpret_cast<T*>(host_bytes());
    }
    template <typename T>
    const T* ptr() const {
        return reinterpret_cast<const T*>(host_bytes());
    }
    uint8_t* host_bytes() const {
        DASH_CHECK(!in_slot, "array bytes live in an evaluator table slot (skeleton model): no host copy");
        if (!device_resident()) return buf.get();
        Device* d = dev.get();
        const size_t n = nbytes;
        std::call_once(d->once, [d, n] {
            d->host = host_alloc(n);
            d->fetch(d->host.get(), d->p.get(), n);
        });
        return d->host.get();
    }

   private:
    size_t shape_bytes() const {
        size_t cnt = 1;
        for (auto s : shape) cnt *= static_cast<size_t>(s);
        return cnt * dtype_size(dtype);
    }
    static std::shared_ptr<uint8_t> host_alloc(size_t nbytes) {
        size_t alloc = (nbytes + 63) & ~size_t(63);
        if (alloc == 0) alloc = 64;
        bool zeroed = false;
        uint8_t* p = static_cast<uint8_t*>(big_alloc(alloc, &zeroed));
        if (!zeroed) std::memset(p, 0, alloc);
        return std::shared_ptr<uint8_t>(p, [alloc](uint8_t* q) { big_free(q, alloc); });
    }
};

// ----------------------------------------------------------------------------
// Label tensor: N labels mod p, label-major (the n components of one label are
// contiguous), element index = flattened semantic index.
// ----------------------------------------------------------------------------
struct Labels {
    int p = 0;
    int n = 0;
    i64 N = 0;
    std::vector<comp_t, BigAllocator<comp_t>> c;
    Labels() = default;
    Labels(int p_, i64 N_) : p(p_), n(nr_comps(p_)), N(N_), c(static_cast<size_t>(N_) * nr_comps(p_), 0) {}
    comp_t* at(i64 i) { return c.data() + i * n; }
    const comp_t* at(i64 i) const { return c.data() + i * n; }
};
using CrtLabels = std::vector<Labels>;  // one Labels per residue

}  // namespace dash
