// Versioned binary format of GarbledModel and Decoder (docs/WIRE_FORMAT.md).
// Little-endian, length-prefixed; every array carries dtype + shape.
#include "model.h"

namespace dash {

namespace {
constexpr char kModelMagic[8] = {'D', 'A', 'M', 'D', 'G', 'C', '0', '1'};
constexpr char kDecMagic[8] = {'D', 'A', 'M', 'D', 'D', 'E', 'C', '1'};

// Writer over an output byte range (or a size count when out == nullptr): the offline message is written
// once, straight into the caller's buffer (a send buffer), and a device-resident array (GPU garbler tables)
// is fetched from HBM directly into its place, with no intermediate host copy.
constexpr uint8_t kInSlot = 0x80;  // skeleton dtype flag: shape only, the bytes are in the evaluator's slot

struct W {
    uint8_t* out = nullptr;
    size_t cap = 0;
    size_t off = 0;
    int skeleton = 0;  // 1: external device arrays as placeholders; 2: every device-resident array
    void raw(const void* p, size_t n) {
        if (out) {
            DASH_CHECK(off + n <= cap, "serialize: output buffer too small");
            std::memcpy(out + off, p, n);
        }
        off += n;
    }
    void u32(uint32_t v) { raw(&v, 4); }
    void i64v(i64 v) { raw(&v, 8); }
    void str(const std::string& x) {
        u32(static_cast<uint32_t>(x.size()));
        raw(x.data(), x.size());
    }
    void ivec(const std::vector<i64>& v) {
        u32(static_cast<uint32_t>(v.size()));
        for (auto x : v) i64v(x);
    }
    void ivec32(const std::vector<int>& v) {
        u32(static_cast<uint32_t>(v.size()));
        for (auto x : v) i64v(x);
    }
    void arr(const Array& a) {
        uint8_t dt = static_cast<uint8_t>(a.dtype);
        if (skeleton && a.device_resident() && (skeleton == 2 || a.dev->external)) {
            dt |= kInSlot;
            raw(&dt, 1);
            ivec(a.shape);
            i64v(static_cast<i64>(a.nbytes));
            return;
        }
        raw(&dt, 1);
        ivec(a.shape);
        i64v(static_cast<i64>(a.nbytes));
        if (out && a.device_resident() && !a.dev->host) {
            DASH_CHECK(off + a.nbytes <= cap, "serialize: output buffer too small");
            a.dev->fetch(out + off, a.device_ptr(), a.nbytes);
            off += a.nbytes;
        } else if (out) {
            raw(a.ptr<uint8_t>(), a.nbytes);
        } else {
            off += a.nbytes;
        }
    }
};

struct Rd {
    const uint8_t* s;
    size_t n;
    size_t off = 0;
    Rd(const uint8_t* p, size_t len) : s(p), n(len) {}
    explicit Rd(const std::string& x) : s(reinterpret_cast<const uint8_t*>(x.data())), n(x.size()) {}
    void raw(void* p, size_t k) {
        DASH_CHECK(off + k <= n, "truncated blob");
        std::memcpy(p, s + off, k);
        off += k;
    }
    uint32_t u32() {
        uint32_t v;
        raw(&v, 4);
        return v;
    }
    i64 i64v() {
        i64 v;
        raw(&v, 8);
        return v;
    }
    std::string str() {
        uint32_t k = u32();
        DASH_CHECK(off + k <= n, "truncated blob");
        std::string r(reinterpret_cast<const char*>(s + off), k);
        off += k;
        return r;
    }
    std::vector<i64> ivec() {
        uint32_t k = u32();
        DASH_CHECK(static_cast<size_t>(k) * 8 <= n - off, "truncated blob");
        std::vector<i64> v(k);
        for (auto& x : v) x = i64v();
        return v;
    }
    std::vector<int> ivec32() {
        auto v = ivec();
        return std::vector<int>(v.begin(), v.end());
    }
    bool skeleton = false;
    Array arr() {
        uint8_t dt;
        raw(&dt, 1);
        if (skeleton && (dt & kInSlot)) {
            dt &= static_cast<uint8_t>(~kInSlot);
            DASH_CHECK(dt <= 4, "bad dtype");
            Array a;
            a.dtype = static_cast<DType>(dt);
            a.shape = ivec();
            size_t cnt = 1;
            for (auto d : a.shape) {
                DASH_CHECK(d >= 0 && (d == 0 || cnt <= (size_t(1) << 50) / static_cast<size_t>(d)), "bad array shape");
                cnt *= static_cast<size_t>(d);
            }
            a.nbytes = cnt * dtype_size(a.dtype);
            DASH_CHECK(static_cast<size_t>(i64v()) == a.nbytes, "array size mismatch");
            a.in_slot = true;
            return a;
        }
        DASH_CHECK(dt <= 4, "bad dtype");
        auto shape = ivec();
        size_t cnt = 1;
        for (auto d : shape) {
            DASH_CHECK(d >= 0 && (d == 0 || cnt <= n / static_cast<size_t>(d)), "bad array shape");
            cnt *= static_cast<size_t>(d);
        }
        DASH_CHECK(n - off >= 8 && cnt * dtype_size(static_cast<DType>(dt)) <= n - off - 8, "array larger than the blob");
        Array a(static_cast<DType>(dt), shape);
        i64 nb = i64v();
        DASH_CHECK(static_cast<size_t>(nb) == a.nbytes, "array size mismatch");
        raw(a.ptr<uint8_t>(), a.nbytes);
        return a;
    }
};
}  // namespace

namespace {
void write_model(const GarbledModel& m, W& w) {
    const auto& h = m.h;
    const auto& consts = m.consts;
    const auto& layers = m.layers;
    w.raw(kModelMagic, 8);
    w.u32(4u);
    w.u32(static_cast<uint32_t>(h.sign_fused));
    w.u32(static_cast<uint32_t>(h.hardened));
    w.ivec32(h.crt);
    w.ivec32(h.mrs);
    w.ivec(h.in_dims);
    w.ivec(h.out_dims);
    w.ivec32(h.out_moduli);
    w.i64v(h.max_mod);
    w.u32(static_cast<uint32_t>(consts.size()));
    for (const auto& kv : consts) {
        w.str(kv.first);
        w.arr(kv.second);
    }
    w.u32(static_cast<uint32_t>(layers.size()));
    for (const auto& l : layers) {
        w.u32(static_cast<uint32_t>(l.kind));
        w.u32(static_cast<uint32_t>(l.p.size()));
        for (const auto& kv : l.p) {
            w.str(kv.first);
            w.ivec(kv.second);
        }
        w.u32(static_cast<uint32_t>(l.a.size()));
        for (const auto& kv : l.a) {
            w.str(kv.first);
            w.arr(kv.second);
        }
    }
}
}  // namespace

size_t GarbledModel::serialized_size() const {
    W w;
    write_model(*this, w);
    return w.off;
}

size_t GarbledModel::serialize_to(uint8_t* out, size_t cap) const {
    W w;
    w.out = out;
    w.cap = cap;
    write_model(*this, w);
    return w.off;
}

std::string GarbledModel::serialize() const {
    std::string s(serialized_size(), '\0');
    serialize_to(reinterpret_cast<uint8_t*>(&s[0]), s.size());
    return s;
}

GarbledModel GarbledModel::deserialize(const std::string& blob) {
    return deserialize(reinterpret_cast<const uint8_t*>(blob.data()), blob.size());
}

namespace {
GarbledModel read_model(Rd& r, size_t nbytes);
}

GarbledModel GarbledModel::deserialize(const uint8_t* blob, size_t nbytes) {
    Rd r(blob, nbytes);
    return read_model(r, nbytes);
}

GarbledModel GarbledModel::deserialize_skeleton(const uint8_t* blob, size_t nbytes) {
    Rd r(blob, nbytes);
    r.skeleton = true;
    return read_model(r, nbytes);
}

std::string GarbledModel::serialize_skeleton(bool all_device) const {
    W sz;
    sz.skeleton = all_device ? 2 : 1;
    write_model(*this, sz);
    std::string s(sz.off, '\0');
    W w;
    w.out = reinterpret_cast<uint8_t*>(&s[0]);
    w.cap = s.size();
    w.skeleton = sz.skeleton;
    write_model(*this, w);
    return s;
}

namespace {
GarbledModel read_model(Rd& r, size_t nbytes) {
    char mg[8];
    r.raw(mg, 8);
    DASH_CHECK(std::memcmp(mg, kModelMagic, 8) == 0, "not a garbled model blob");
    GarbledModel m;
    m.h.version = static_cast<int>(r.u32());
    DASH_CHECK(m.h.version >= 2 && m.h.version <= 4, "unsupported garbled model version (expected 2..4)");
    m.h.sign_fused = m.h.version >= 3 ? static_cast<int>(r.u32()) : 0;
    DASH_CHECK(m.h.sign_fused == 0 || m.h.sign_fused == 1, "bad sign construction flag");
    m.h.hardened = m.h.version >= 4 ? static_cast<int>(r.u32()) : 0;
    DASH_CHECK(m.h.hardened == 0 || m.h.hardened == 1, "bad hardened flag");
    m.h.version = 4;
    m.h.crt = r.ivec32();
    m.h.mrs = r.ivec32();
    m.h.in_dims = r.ivec();
    m.h.out_dims = r.ivec();
    m.h.out_moduli = r.ivec32();
    m.h.max_mod = static_cast<int>(r.i64v());
    uint32_t nc = r.u32();
    for (uint32_t i = 0; i < nc; ++i) {
        std::string k = r.str();
        m.consts[k] = r.arr();
    }
    uint32_t nl = r.u32();
    for (uint32_t i = 0; i < nl; ++i) {
        GLayer g;
        g.kind = static_cast<int>(r.u32());
        uint32_t np = r.u32();
        for (uint32_t q = 0; q < np; ++q) {
            std::string k = r.str();
            g.p[k] = r.ivec();
        }
        uint32_t na = r.u32();
        for (uint32_t q = 0; q < na; ++q) {
            std::string k = r.str();
            g.a[k] = r.arr();
        }
        m.layers.push_back(std::move(g));
    }
    DASH_CHECK(r.off == nbytes, "trailing bytes after garbled model");
    return m;
}
}  // namespace

std::string Decoder::serialize() const {
    auto put = [this](W& w) {
        w.raw(kDecMagic, 8);
        w.ivec32(moduli);
        w.i64v(n_out);
        w.u32(static_cast<uint32_t>(dec.size()));
        for (const auto& a : dec) w.arr(a);
    };
    W sz;
    put(sz);
    std::string s(sz.off, '\0');
    W w;
    w.out = reinterpret_cast<uint8_t*>(&s[0]);
    w.cap = s.size();
    put(w);
    return s;
}

Decoder Decoder::deserialize(const std::string& blob) {
    Rd r(blob);
    char mg[8];
    r.raw(mg, 8);
    DASH_CHECK(std::memcmp(mg, kDecMagic, 8) == 0, "not a decoder blob");
    Decoder d;
    d.moduli = r.ivec32();
    d.n_out = r.i64v();
    uint32_t n = r.u32();
    for (uint32_t i = 0; i < n; ++i) d.dec.push_back(r.arr());
    return d;
}

}  // namespace dash
