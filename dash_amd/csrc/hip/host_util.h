// Host-side helpers shared by the HIP translation units: error checking,
// AES T-table / round-key images and modulus constants for the device codecs.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "../core.h"
#include "dev.h"

namespace dash {

#define HIPCHECK(x)                                                                                      \
    do {                                                                                                 \
        hipError_t e_ = (x);                                                                             \
        if (e_ != hipSuccess)                                                                            \
            throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) + " at " + __FILE__ + \
                                     ":" + std::to_string(__LINE__));                                    \
    } while (0)

namespace hostutil {

// --------------------------------------------------------- device binding
// DASH_DEBUG_DEVICE=1: every native entry that launches or allocates checks that the calling thread's current
// device and the stream it was handed belong to the object's device (a rank or worker thread that never set its
// device would otherwise launch on device 0 with another device's pointers).
inline bool debug_device_checks() {
    static const bool on = [] {
        const char* e = std::getenv("DASH_DEBUG_DEVICE");
        return e && e[0] == '1';
    }();
    return on;
}
inline void check_device(int dev, hipStream_t st, const char* where) {
    int cur = -1;
    HIPCHECK(hipGetDevice(&cur));
    if (cur != dev)
        throw std::runtime_error(std::string("dash: ") + where + " runs on device " + std::to_string(cur) +
                                 ", its object lives on device " + std::to_string(dev));
    if (st) {
        hipDevice_t sd = -1;
        HIPCHECK(hipStreamGetDevice(st, &sd));
        if (static_cast<int>(sd) != dev)
            throw std::runtime_error(std::string("dash: ") + where + " got a stream of device " +
                                     std::to_string(sd) + ", its object lives on device " + std::to_string(dev));
    }
}
// Make `dev` current for this thread (cheap: a thread-local store) and, in debug mode, check the stream.
inline void bind_device(int dev, hipStream_t st, const char* where) {
    HIPCHECK(hipSetDevice(dev));
    if (debug_device_checks()) check_device(dev, st, where);
}

// --------------------------------------------------------------- AES tables
inline uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = static_cast<uint8_t>((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return r;
}
inline std::vector<uint32_t> make_te0() {
    // S-box from the GF(2^8) inverse and the AES affine map
    uint8_t sbox[256];
    for (int x = 0; x < 256; ++x) {
        uint8_t inv = 0;
        if (x)
            for (int y = 1; y < 256; ++y)
                if (gmul(static_cast<uint8_t>(x), static_cast<uint8_t>(y)) == 1) {
                    inv = static_cast<uint8_t>(y);
                    break;
                }
        uint8_t s = inv;
        uint8_t r = s;
        for (int i = 0; i < 4; ++i) {
            r = static_cast<uint8_t>((r << 1) | (r >> 7));
            s ^= r;
        }
        sbox[x] = static_cast<uint8_t>(s ^ 0x63);
    }
    std::vector<uint32_t> te(256);
    for (int x = 0; x < 256; ++x) {
        uint8_t s = sbox[x];
        te[x] = (static_cast<uint32_t>(gmul(s, 2)) << 24) | (static_cast<uint32_t>(s) << 16) |
                (static_cast<uint32_t>(s) << 8) | gmul(s, 3);
    }
    return te;
}
inline std::vector<uint32_t> fixed_round_key_words() {
    uint8_t rk[176];
    aes_round_key_bytes(fixed_key(), rk);
    std::vector<uint32_t> w(44);
    for (int i = 0; i < 44; ++i)
        w[i] = (static_cast<uint32_t>(rk[4 * i]) << 24) | (static_cast<uint32_t>(rk[4 * i + 1]) << 16) |
               (static_cast<uint32_t>(rk[4 * i + 2]) << 8) | rk[4 * i + 3];
    return w;
}

inline dev::ModC make_modc(int q) {
    dev::ModC m{};
    m.q = q;
    m.n = nr_comps(q);
    m.pm = static_cast<uint32_t>(prg_digits(q));
    if ((q & (q - 1)) == 0) {
        int b = 0;
        while ((1 << b) < q) ++b;
        m.bits = b;
        m.c = 1;
        m.D = q;
        return m;
    }
    // chunks of c digits with D = q^c <= 2^31, so that floor(r / q) for r < D is one multiply-high and a
    // shift: with s = ceil(log2 q) - 1 and dm = ceil(2^(32+s) / q) < 2^32, the error e = dm*q - 2^(32+s) < q
    // gives r*e < D*q <= 2^31 * 2^(s+1) = 2^(32+s), hence floor(r*dm / 2^(32+s)) = floor(r / q)
    uint64_t D = q;
    int c = 1;
    while (D * static_cast<uint64_t>(q) <= (1ull << DASH_CHUNK_BITS)) {
        D *= q;
        ++c;
    }
    m.c = c;
    m.D = static_cast<uint32_t>(D);
    m.mD = static_cast<uint64_t>((static_cast<u128>(1) << 64) / D);
    int bl = 0;
    while ((D >> bl) != 0) ++bl;
    m.sh = static_cast<uint32_t>(32 - bl);  // D < 2^31: 1 <= sh
    m.Dn = static_cast<uint32_t>(D << m.sh);
    m.v = static_cast<uint32_t>(~0ull / static_cast<uint64_t>(m.Dn) - (1ull << 32));
    m.mq = static_cast<uint32_t>((1ull << 32) / static_cast<uint64_t>(q));
    int s = 0;
    while ((1 << (s + 1)) < q) ++s;  // 2^s < q <= 2^(s+1)
    const uint64_t two = 1ull << (32 + s);
    m.dm = static_cast<uint32_t>((two + q - 1) / q);
    m.ds = static_cast<uint32_t>(s);
    if (DASH_DIGIT_MAGIC && (static_cast<u128>(D) * (static_cast<uint64_t>(m.dm) * q - two) > two || q >= (1 << 24))) {
        std::fprintf(stderr, "dash: no 32-bit digit magic for modulus %d\n", q);
        std::abort();
    }
    return m;
}

}  // namespace


// AES-128 round keys of an arbitrary key as big-endian column words (device layout)
inline std::vector<uint32_t> round_key_words(const uint8_t key16[16]) {
    AesKey k;
    aes_expand(key16, k);
    uint8_t rk[176];
    aes_round_key_bytes(k, rk);
    std::vector<uint32_t> w(44);
    for (int i = 0; i < 44; ++i)
        w[i] = (static_cast<uint32_t>(rk[4 * i]) << 24) | (static_cast<uint32_t>(rk[4 * i + 1]) << 16) |
               (static_cast<uint32_t>(rk[4 * i + 2]) << 8) | rk[4 * i + 3];
    return w;
}

}  // namespace dash
