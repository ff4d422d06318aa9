// Python bindings of the native core (pybind11).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "dataloader.h"
#include "hip/gpu_garbler.h"
#include "layers.h"
#include "onnx.h"

namespace py = pybind11;
using namespace dash;

namespace dash {
void register_hip_bindings(py::module_& m);  // runtime_hip.cpp / runtime_stub.cpp
}

namespace {

u128 py_to_u128(py::int_ v) {
    py::int_ mask64 = py::int_(0xFFFFFFFFFFFFFFFFull);
    py::object lo = v & mask64;
    py::object hi = (v >> py::int_(64)) & mask64;
    return (static_cast<u128>(hi.cast<uint64_t>()) << 64) | lo.cast<uint64_t>();
}
py::int_ u128_to_py(u128 x) {
    py::int_ hi(static_cast<uint64_t>(x >> 64)), lo(static_cast<uint64_t>(x));
    return py::int_((hi << py::int_(64)) | lo);
}

Params to_params(const py::dict& d) {
    Params p;
    for (auto item : d) {
        std::string key = py::str(item.first);
        py::object v = py::reinterpret_borrow<py::object>(item.second);
        py::array_t<i64, py::array::c_style | py::array::forcecast> a = py::array_t<i64, py::array::c_style | py::array::forcecast>::ensure(v);
        if (!a) {
            a = py::array_t<i64, py::array::c_style | py::array::forcecast>(py::array(py::make_tuple(v)));
        }
        std::vector<i64> vec(a.data(), a.data() + a.size());
        p[key] = std::move(vec);
    }
    return p;
}

py::dict from_params(const Params& p) {
    py::dict d;
    for (const auto& kv : p) d[py::str(kv.first)] = py::cast(kv.second);
    return d;
}

py::array array_view(const Array& a, py::object owner) {
    std::vector<py::ssize_t> shape(a.shape.begin(), a.shape.end());
    switch (a.dtype) {
        case DType::i16: return py::array_t<int16_t>(shape, a.ptr<int16_t>(), owner);
        case DType::i32: return py::array_t<int32_t>(shape, a.ptr<int32_t>(), owner);
        case DType::i64: return py::array_t<int64_t>(shape, a.ptr<int64_t>(), owner);
        case DType::u8: return py::array_t<uint8_t>(shape, a.ptr<uint8_t>(), owner);
        case DType::u128: {
            shape.push_back(2);
            return py::array_t<uint64_t>(shape, a.ptr<uint64_t>(), owner);
        }
    }
    return py::none();
}

py::list labels_to_py(const CrtLabels& L) {
    py::list out;
    for (const auto& x : L) {
        py::array_t<int16_t> arr({static_cast<py::ssize_t>(x.N), static_cast<py::ssize_t>(x.n)});
        std::memcpy(arr.mutable_data(), x.c.data(), x.c.size() * sizeof(comp_t));
        out.append(py::make_tuple(x.p, arr));
    }
    return out;
}

CrtLabels labels_from_py(const py::list& l) {
    CrtLabels out;
    for (auto item : l) {
        py::tuple t = item.cast<py::tuple>();
        int p = t[0].cast<int>();
        auto arr = py::array_t<int16_t, py::array::c_style | py::array::forcecast>::ensure(t[1]);
        DASH_CHECK(arr && arr.ndim() == 2, "labels must be (N, n) int16 arrays");
        Labels L(p, arr.shape(0));
        DASH_CHECK(arr.shape(1) == L.n, "label width does not match modulus");
        std::memcpy(L.c.data(), arr.data(), L.c.size() * sizeof(comp_t));
        out.push_back(std::move(L));
    }
    return out;
}

std::vector<LayerSpec> specs_from_py(const py::list& l) {
    std::vector<LayerSpec> out;
    for (auto item : l) {
        py::tuple t = item.cast<py::tuple>();
        LayerSpec s;
        s.kind = t[0].cast<int>();
        s.p = to_params(t[1].cast<py::dict>());
        out.push_back(std::move(s));
    }
    return out;
}

py::array_t<uint64_t> u128_array(const u128* src, py::ssize_t k, py::ssize_t n) {
    py::array_t<uint64_t> out({k, n, static_cast<py::ssize_t>(2)});
    if (k * n) std::memcpy(out.mutable_data(), src, sizeof(u128) * k * n);
    return out;
}

const u128* u128_data(const py::array_t<uint64_t, py::array::c_style | py::array::forcecast>& a, py::ssize_t k,
                      py::ssize_t n) {
    DASH_CHECK(a.ndim() == 3 && a.shape(0) == k && a.shape(1) == n && a.shape(2) == 2,
               "compressed labels must be a (k, N, 2) uint64 array");
    return reinterpret_cast<const u128*>(a.data());
}

class IntegrityError : public std::exception {};

// serialize_into / deserialize_buffer read or write bi.size bytes straight from bi.ptr: only a 1-D, C-contiguous
// byte buffer describes that memory (a strided or negative-stride view would send the copy past the view)
void check_contig_bytes(const py::buffer_info& bi, const char* who) {
    DASH_CHECK(bi.itemsize == 1 && bi.ndim == 1 && (bi.shape[0] <= 1 || bi.strides[0] == 1),
               std::string(who) + " needs a 1-D C-contiguous byte buffer");
}

}  // namespace

PYBIND11_MODULE(_dash_native, m) {
    m.doc() = "dash_amd native core: labels, AES, garbler, host evaluator, HIP runtime";
    static py::exception<std::runtime_error> integrity_exc(m, "IntegrityError");
    py::register_exception_translator([](std::exception_ptr p) {
        try {
            if (p) std::rethrow_exception(p);
        } catch (const std::runtime_error& e) {
            if (std::string(e.what()).rfind("dash integrity", 0) == 0) {
                PyErr_SetString(integrity_exc.ptr(), e.what());
                return;
            }
            throw;
        }
    });

    m.def("nr_comps", &nr_comps);
    m.def("gpu_table_cache_trim", &gpu_table_cache_trim, "release the GPU garbler's cached table blocks");
    m.def("gpu_table_cache_bytes", &gpu_table_cache_bytes);
    m.def("first_primes", &first_primes);
    m.def("mul_inv", [](py::int_ a, i64 b) { return mul_inv(py_to_u128(a), b); });
    m.def("set_num_threads", &set_default_threads);
    m.def("get_num_threads", &default_threads);
    m.def("aes_hash", [](py::int_ x) { return u128_to_py(hash(py_to_u128(x))); }, "fixed-key AES-128 of a 128-bit int");
    m.def("chacha_block", [](std::vector<uint32_t> state, int rounds) {
        DASH_CHECK(state.size() == 16, "ChaCha state is 16 words");
        std::vector<uint32_t> out(16);
        chacha_core(state.data(), out.data(), rounds);
        return out;
    }, "ChaCha block function (rounds rounds, feed-forward) of a 16-word state");
    m.def("hard_pads", [](py::int_ key, uint64_t gate, uint32_t sub, uint32_t blk) {
        u128 p[4];
        hard_block(py_to_u128(key), gate, sub, blk, p);
        py::list out;
        for (auto v : p) out.append(u128_to_py(v));
        return out;
    }, "the four hardened-encoding pads of block blk of key K under tweak (gate, sub)");
    m.def("stream_id", &stream_id);
    m.def("aes_hash_array", [](py::array_t<uint64_t, py::array::c_style | py::array::forcecast> a) {
        DASH_CHECK(a.ndim() == 2 && a.shape(1) == 2, "expected (n, 2) uint64 array");
        py::array_t<uint64_t> out({a.shape(0), static_cast<py::ssize_t>(2)});
        hash_batch(reinterpret_cast<const u128*>(a.data()), reinterpret_cast<u128*>(out.mutable_data()), a.shape(0));
        return out;
    });
    m.def("aes_encrypt_block", [](py::bytes key, py::bytes block) {
        std::string k = key, b = block;
        DASH_CHECK(k.size() == 16 && b.size() == 16, "key and block must be 16 bytes");
        AesKey ak;
        aes_expand(reinterpret_cast<const uint8_t*>(k.data()), ak);
        __m128i x;
        std::memcpy(&x, b.data(), 16);
        x = aes_enc_block(x, ak);
        char out[16];
        std::memcpy(out, &x, 16);
        return py::bytes(out, 16);
    });
    m.def("aes_round_keys", [](py::bytes key) {
        std::string k = key;
        DASH_CHECK(k.size() == 16, "key must be 16 bytes");
        AesKey ak;
        aes_expand(reinterpret_cast<const uint8_t*>(k.data()), ak);
        uint8_t rk[176];
        aes_round_key_bytes(ak, rk);
        return py::bytes(reinterpret_cast<char*>(rk), 176);
    });
    m.def("compress", [](py::array_t<int16_t, py::array::c_style | py::array::forcecast> a, int p) {
        const ModInfo& mi = mod_info(p);
        DASH_CHECK(a.size() == mi.n, "label length mismatch");
        return u128_to_py(compress(a.data(), mi));
    });
    m.def("decompress", [](py::int_ c, int p) {
        const ModInfo& mi = mod_info(p);
        py::array_t<int16_t> out(mi.n);
        decompress(py_to_u128(c), out.mutable_data(), mi);
        return out;
    });
    m.def("gen_approx_lookup", &gen_approx_lookup);
    m.def("prg_label", [](py::bytes seed, uint64_t stream, uint64_t ctr, int p) {
        std::string s = seed;
        DASH_CHECK(s.size() == 16, "seed must be 16 bytes");
        Prg prg(reinterpret_cast<const uint8_t*>(s.data()));
        py::array_t<int16_t> out(nr_comps(p));
        prg.label(stream, ctr, p, nr_comps(p), out.mutable_data());
        return out;
    });
    m.def("kind_name", &kind_name);

    // Single gates of the native garbler with caller-chosen labels (wire-compatibility vectors: the tests
    // rebuild the reference's formulas in a pure-Python oracle and compare table bytes). Tables come back as
    // uint64 (entries, 2) = (lo, hi) of each 16-byte entry.
    using I16 = py::array_t<int16_t, py::array::c_style | py::array::forcecast>;
    auto table_out = [](const std::vector<u128>& t) {
        py::array_t<uint64_t> out({static_cast<py::ssize_t>(t.size()), static_cast<py::ssize_t>(2)});
        auto o = out.mutable_unchecked<2>();
        for (size_t i = 0; i < t.size(); ++i) {
            o(i, 0) = static_cast<uint64_t>(t[i]);
            o(i, 1) = static_cast<uint64_t>(t[i] >> 64);
        }
        return out;
    };
    auto check_label = [](const I16& a, int p, const char* what) {
        DASH_CHECK(a.size() == nr_comps(p), std::string(what) + ": label length does not match its modulus");
    };
    m.def("garble_projection_gate", [=](I16 in0, I16 Rin, int pin, I16 out0, I16 outR, int pout, std::vector<i64> f) {
        check_label(in0, pin, "in0"); check_label(Rin, pin, "Rin"); check_label(out0, pout, "out0");
        check_label(outR, pout, "outR");
        DASH_CHECK(static_cast<int>(f.size()) == pin, "one function value per input value");
        std::vector<u128> t(pin);
        garble_proj(in0.data(), Rin.data(), mod_info(pin), out0.data(), outR.data(), mod_info(pout),
                    [&](int v) { return f[v]; }, t.data());
        return table_out(t);
    }, "projection gate T[color(in0 + i Rin)] = compress(out0 + f(i) outR) + H(compress(in0 + i Rin))");
    m.def("garble_mini_gate", [=](I16 in0, I16 Rin, int pin, std::vector<i64> f) {
        check_label(in0, pin, "in0"); check_label(Rin, pin, "Rin");
        DASH_CHECK(static_cast<int>(f.size()) == pin, "one function value per input value");
        std::vector<u128> t(1, 0);
        garble_proj_mini(in0.data(), Rin.data(), mod_info(pin), [&](int v) { return f[v]; }, t.data());
        return table_out(t);
    }, "mini projection: int16 payloads f(i) + (int16)H at slot color of one 16-byte entry");
    m.def("garble_mixed_mod_gate", [=](I16 x0, int p, I16 y0, int q, I16 Rp, I16 Rq, py::bytes seed, uint64_t stream) {
        check_label(x0, p, "x0"); check_label(y0, q, "y0"); check_label(Rp, p, "Rp"); check_label(Rq, q, "Rq");
        std::string sd = seed;
        DASH_CHECK(sd.size() == 16, "seed must be 16 bytes");
        Prg prg(reinterpret_cast<const uint8_t*>(sd.data()));
        LabelBank R;
        R.max_mod = std::max(p, q);
        R.lab.assign(R.max_mod + 1, {});
        R.lab[p].assign(Rp.data(), Rp.data() + Rp.size());
        R.lab[q].assign(Rq.data(), Rq.data() + Rq.size());
        std::vector<u128> g(p), e(q + 1, 0);
        py::array_t<int16_t> out0(nr_comps(p));
        u64 ctr = 0;
        mixed_mult_garble(x0.data(), mod_info(p), y0.data(), mod_info(q), R, prg, stream, ctr, g.data(), e.data(),
                          out0.mutable_data());
        return py::make_tuple(table_out(g), table_out(e), out0);
    }, "mixed-modulus half gate x (mod p) * y (mod q): garbler table [p], evaluator table [q + 1] (q full entries, "
       "then the mini entry), output base label; sk03 / sk04 drawn from Prg(seed) on `stream`");

    py::class_<GarbleSpecs, std::shared_ptr<GarbleSpecs>>(m, "GarbleSpecs",
        "a circuit's layer specs converted once; its public weights are reduced mod M once per CRT modulus and "
        "shared by every GC garbled from it")
        .def(py::init([](const py::list& layers) {
            auto s = std::make_shared<GarbleSpecs>();
            s->layers = specs_from_py(layers);
            return s;
        }))
        .def_property_readonly("num_layers", [](const GarbleSpecs& s) { return s.layers.size(); });

    py::class_<GarbledModel, std::shared_ptr<GarbledModel>>(m, "GarbledModel")
        .def("serialize", [](const GarbledModel& g) { return py::bytes(g.serialize()); })
        .def_static("deserialize", [](py::bytes b) { return std::make_shared<GarbledModel>(GarbledModel::deserialize(std::string(b))); })
        .def("serialized_size", &GarbledModel::serialized_size)
        .def("serialize_into", [](const GarbledModel& g, py::buffer b) {
            py::buffer_info bi = b.request(true);
            check_contig_bytes(bi, "serialize_into");
            const size_t cap = static_cast<size_t>(bi.size);
            py::gil_scoped_release nogil;
            return g.serialize_to(static_cast<uint8_t*>(bi.ptr), cap);
        }, "write the offline message into a writable buffer (>= serialized_size() bytes) -> bytes written; "
           "device-resident tables are fetched straight into it")
        .def("serialize_skeleton", [](const GarbledModel& g, bool all_device) { return py::bytes(g.serialize_skeleton(all_device)); },
             py::arg("all_device") = false,
             "the offline message without the tables the garbler wrote into an evaluator slot (device transport); "
             "all_device: every device-resident array as a placeholder (an evaluator template)")
        .def_static("deserialize_skeleton", [](py::buffer b) {
            py::buffer_info bi = b.request();
            check_contig_bytes(bi, "deserialize_skeleton");
            const auto* p = static_cast<const uint8_t*>(bi.ptr);
            const size_t n = static_cast<size_t>(bi.size) * static_cast<size_t>(bi.itemsize);
            py::gil_scoped_release rel;
            return std::make_shared<GarbledModel>(GarbledModel::deserialize_skeleton(p, n));
        })
        .def_static("deserialize_buffer", [](py::buffer b) {
            py::buffer_info bi = b.request();
            check_contig_bytes(bi, "deserialize_buffer");
            const size_t n = static_cast<size_t>(bi.size);
            const uint8_t* p = static_cast<const uint8_t*>(bi.ptr);
            py::gil_scoped_release nogil;
            return std::make_shared<GarbledModel>(GarbledModel::deserialize(p, n));
        }, "parse an offline message from any byte buffer (no intermediate copy)")
        .def_property_readonly("crt", [](const GarbledModel& g) { return g.h.crt; })
        .def_property_readonly("mrs", [](const GarbledModel& g) { return g.h.mrs; })
        .def_property_readonly("in_dims", [](const GarbledModel& g) { return g.h.in_dims; })
        .def_property_readonly("out_dims", [](const GarbledModel& g) { return g.h.out_dims; })
        .def_property_readonly("out_moduli", [](const GarbledModel& g) { return g.h.out_moduli; })
        .def_property_readonly("max_mod", [](const GarbledModel& g) { return g.h.max_mod; })
        .def_property_readonly("sign_fused", [](const GarbledModel& g) { return g.h.sign_fused != 0; })
        .def_property_readonly("hardened", [](const GarbledModel& g) { return g.h.hardened != 0; })
        .def("const_names", [](const GarbledModel& g) {
            std::vector<std::string> v;
            for (const auto& kv : g.consts) v.push_back(kv.first);
            return v;
        }, "names of the evaluator-visible constant labels the offline message ships (none when hardened)")
        .def("const_array", [](std::shared_ptr<GarbledModel> g, const std::string& name) {
            return array_view(g->consts.at(name), py::cast(g));
        })
        .def_property_readonly("num_layers", [](const GarbledModel& g) { return g.layers.size(); })
        .def("table_bytes", &GarbledModel::table_bytes)
        .def("total_bytes", &GarbledModel::total_bytes)
        .def("layer_kind", [](const GarbledModel& g, size_t i) { return g.layers.at(i).kind; })
        .def("layer_params", [](const GarbledModel& g, size_t i) { return from_params(g.layers.at(i).p); })
        .def("layer_arrays", [](std::shared_ptr<GarbledModel> g, size_t i) {
            py::dict d;
            py::object owner = py::cast(g);
            for (const auto& kv : g->layers.at(i).a) d[py::str(kv.first)] = array_view(kv.second, owner);
            return d;
        })
        .def("consts", [](std::shared_ptr<GarbledModel> g) {
            py::dict d;
            py::object owner = py::cast(g);
            for (const auto& kv : g->consts) d[py::str(kv.first)] = array_view(kv.second, owner);
            return d;
        })
        .def("flip_table_bit", [](GarbledModel& g, size_t layer, const std::string& name, size_t entry, int bit) {
            // fault injection for integrity tests
            Array& a = g.layers.at(layer).a.at(name);
            DASH_CHECK(a.dtype == DType::u128 && entry < a.count(), "bad fault-injection target");
            a.ptr<u128>()[entry] ^= (static_cast<u128>(1) << bit);
        });

    py::class_<Decoder, std::shared_ptr<Decoder>>(m, "Decoder")
        .def("decode", [](const Decoder& d, const py::list& labels) {
            auto v = d.decode(labels_from_py(labels));
            return py::array_t<i64>(v.size(), v.data());
        })
        .def("decode_residues", [](const Decoder& d, const py::list& labels) {
            auto v = d.decode_residues(labels_from_py(labels));
            return py::array_t<i64>({static_cast<py::ssize_t>(d.moduli.size()), static_cast<py::ssize_t>(d.n_out)}, v.data());
        })
        .def("decode_compressed", [](const Decoder& d, py::array_t<uint64_t, py::array::c_style | py::array::forcecast> c) {
            return d.decode_compressed(u128_data(c, d.moduli.size(), d.n_out));
        })
        .def("decode_residues_compressed", [](const Decoder& d, py::array_t<uint64_t, py::array::c_style | py::array::forcecast> c) {
            auto r = d.decode_residues_compressed(u128_data(c, d.moduli.size(), d.n_out));
            py::array_t<i64> out({static_cast<py::ssize_t>(d.moduli.size()), static_cast<py::ssize_t>(d.n_out)});
            std::memcpy(out.mutable_data(), r.data(), r.size() * sizeof(i64));
            return out;
        })
        .def_property_readonly("moduli", [](const Decoder& d) { return d.moduli; })
        .def_property_readonly("n_out", [](const Decoder& d) { return d.n_out; })
        .def("serialize", [](const Decoder& d) { return py::bytes(d.serialize()); })
        .def_static("deserialize", [](py::bytes b) { return std::make_shared<Decoder>(Decoder::deserialize(std::string(b))); })
        .def("tables", [](std::shared_ptr<Decoder> d) {
            py::list l;
            py::object owner = py::cast(d);
            for (const auto& a : d->dec) l.append(array_view(a, owner));
            return l;
        });

    py::class_<TableSink, std::shared_ptr<TableSink>>(m, "TableSink");
    py::class_<Garbler, std::shared_ptr<Garbler>>(m, "Garbler")
        .def(py::init([](std::vector<int> crt, std::vector<int> mrs, py::bytes seed, int max_mod) {
                 return std::make_shared<Garbler>(crt, mrs, std::string(seed), max_mod);
             }),
             py::arg("crt"), py::arg("mrs"), py::arg("seed"), py::arg("max_mod") = 0)
        .def("garble", [](Garbler& g, std::shared_ptr<GarbleSpecs> specs, std::vector<i64> in_dims, int nthreads,
                          int device, bool fused_sign, bool rescale_mrs, bool relu_mrs, bool relu_joint,
                          std::shared_ptr<TableSink> sink, bool hardened) {
            GarbleOptions o;
            o.hardened = hardened;
            o.sink = std::move(sink);
            o.nthreads = nthreads;
            o.device = device;
            o.fused_sign = fused_sign;
            o.rescale_mrs = rescale_mrs;
            o.relu_mrs = relu_mrs;
            o.relu_joint = relu_joint;
            o.cache = specs.get();
            GarbledModel gm;
            {
                py::gil_scoped_release rel;
                gm = g.garble(specs->layers, in_dims, o);
            }
            return std::make_shared<GarbledModel>(std::move(gm));
        }, py::arg("layers"), py::arg("in_dims"), py::arg("nthreads") = 0, py::arg("device") = -1,
           py::arg("fused_sign") = true, py::arg("rescale_mrs") = false,
           py::arg("relu_mrs") = false, py::arg("relu_joint") = false, py::arg("sink") = nullptr,
           py::arg("hardened") = false)
        .def("garble", [](Garbler& g, const py::list& layers, std::vector<i64> in_dims, int nthreads, int device,
                          bool fused_sign, bool rescale_mrs, bool relu_mrs, bool relu_joint,
                          std::shared_ptr<TableSink> sink, bool hardened) {
            auto specs = specs_from_py(layers);
            GarbleOptions o;
            o.hardened = hardened;
            o.sink = std::move(sink);
            o.nthreads = nthreads;
            o.device = device;
            o.fused_sign = fused_sign;
            o.rescale_mrs = rescale_mrs;
            o.relu_mrs = relu_mrs;
            o.relu_joint = relu_joint;
            GarbledModel gm;
            {
                py::gil_scoped_release rel;
                gm = g.garble(specs, in_dims, o);
            }
            return std::make_shared<GarbledModel>(std::move(gm));
        }, py::arg("layers"), py::arg("in_dims"), py::arg("nthreads") = 0, py::arg("device") = -1,
           py::arg("fused_sign") = true, py::arg("rescale_mrs") = false,
           py::arg("relu_mrs") = false, py::arg("relu_joint") = false, py::arg("sink") = nullptr,
           py::arg("hardened") = false)
        .def("layer_ms", [](const Garbler& g) { return g.layer_ms(); })
        .def("encode", [](const Garbler& g, py::array_t<i64, py::array::c_style | py::array::forcecast> x) {
            std::vector<i64> v(x.data(), x.data() + x.size());
            return labels_to_py(g.encode(v));
        })
        .def("encode_cm", [](const Garbler& g, py::array_t<i64, py::array::c_style | py::array::forcecast> x) {
            // online message #1 in component-major layout: one (n_j, N) int16 array per residue
            const i64 N = x.size();
            py::list out;
            std::vector<py::array_t<int16_t>> arrs;
            std::vector<comp_t*> dst;
            for (int p : g.crt()) {
                arrs.emplace_back(std::vector<py::ssize_t>{nr_comps(p), static_cast<py::ssize_t>(N)});
                dst.push_back(arrs.back().mutable_data());
            }
            {
                py::gil_scoped_release rel;
                g.encode_cm(x.data(), N, dst);
            }
            for (auto& a : arrs) out.append(a);
            return out;
        })
        .def("encode_compressed", [](const Garbler& g, py::array_t<i64, py::array::c_style | py::array::forcecast> x) {
            const i64 N = x.size();
            std::vector<u128> buf(g.crt().size() * N);
            {
                py::gil_scoped_release rel;
                g.encode_compressed(x.data(), N, buf.data());
            }
            return u128_array(buf.data(), g.crt().size(), N);
        })
        .def("decoder", [](const Garbler& g) { return std::make_shared<Decoder>(g.decoder()); })
        .def_property_readonly("crt_modulus", &Garbler::crt_modulus)
        .def("offset_label", [](const Garbler& g, int p) {
            const comp_t* r = g.offsets().get(p);
            return py::array_t<int16_t>(nr_comps(p), r);
        })
        .def("zero_label", [](const Garbler& g, int p) {
            const comp_t* r = g.zeros().get(p);
            return py::array_t<int16_t>(nr_comps(p), r);
        })
        .def("input_base", [](const Garbler& g) { return labels_to_py(g.input_base()); });

    m.def("compress_labels", [](const py::list& labels) {
        CrtLabels L = labels_from_py(labels);
        auto c = compress_labels(L);
        return u128_array(c.data(), L.size(), L.empty() ? 0 : L[0].N);
    });
    m.def("decompress_labels", [](py::array_t<uint64_t, py::array::c_style | py::array::forcecast> c,
                                  const std::vector<int>& moduli) {
        DASH_CHECK(c.ndim() == 3, "compressed labels must be (k, N, 2)");
        const i64 N = c.shape(1);
        CrtLabels L = decompress_labels(u128_data(c, moduli.size(), N), moduli, N);
        return labels_to_py(L);
    });
    m.def("cpu_evaluate", [](std::shared_ptr<GarbledModel> gm, const py::list& labels, int nthreads) {
        CrtLabels in = labels_from_py(labels);
        CrtLabels out;
        {
            py::gil_scoped_release rel;
            out = cpu_evaluate(*gm, in, nthreads);
        }
        return labels_to_py(out);
    }, py::arg("model"), py::arg("labels"), py::arg("nthreads") = 0);
    m.def("cpu_evaluate_trace", [](std::shared_ptr<GarbledModel> gm, const py::list& labels, int nthreads) {
        auto in = labels_from_py(labels);
        EvalTrace tr;
        CrtLabels out;
        {
            py::gil_scoped_release rel;
            out = cpu_evaluate(*gm, in, nthreads, nullptr, &tr);
        }
        py::dict relu;
        for (const auto& kv : tr.relu_sign) {
            const Labels& S = kv.second;
            py::array_t<int16_t> sa({static_cast<py::ssize_t>(S.N), static_cast<py::ssize_t>(S.n)});
            std::memcpy(sa.mutable_data(), S.c.data(), S.c.size() * sizeof(comp_t));
            relu[py::int_(kv.first)] = py::make_tuple(labels_to_py(tr.relu_in.at(kv.first)), sa);
        }
        return py::make_tuple(labels_to_py(out), relu);
    }, py::arg("model"), py::arg("labels"), py::arg("nthreads") = 0,
       "host evaluation that also returns, per ReLU layer, (input labels, sign labels): the evaluator's own "
       "intermediate values (security tests)");
    m.def("cpu_evaluate_timed", [](std::shared_ptr<GarbledModel> gm, const py::list& labels, int nthreads) {
        CrtLabels in = labels_from_py(labels);
        CrtLabels out;
        std::vector<double> ms;
        {
            py::gil_scoped_release rel;
            out = cpu_evaluate(*gm, in, nthreads, &ms);
        }
        return py::make_tuple(labels_to_py(out), ms);
    }, py::arg("model"), py::arg("labels"), py::arg("nthreads") = 0);

    // ---------------------------------------------------------------- ONNX
    m.def("onnx_parse", [](py::bytes blob) {
        onnx::Model mdl;
        {
            std::string s = blob;
            py::gil_scoped_release rel;
            mdl = onnx::parse_model(s);
        }
        auto tensor = [](const onnx::Tensor& t) {
            py::dict d;
            d["name"] = t.name;
            d["data_type"] = t.data_type;
            d["dims"] = t.dims;
            std::vector<py::ssize_t> shape(t.dims.begin(), t.dims.end());
            py::array_t<float> v(static_cast<py::ssize_t>(t.values.size()));
            if (!t.values.empty()) std::memcpy(v.mutable_data(), t.values.data(), t.values.size() * sizeof(float));
            d["values"] = v;
            d["ivalues"] = t.ivalues;
            return d;
        };
        py::dict out;
        out["ir_version"] = mdl.ir_version;
        out["opset"] = mdl.opset;
        out["producer_name"] = mdl.producer_name;
        out["producer_version"] = mdl.producer_version;
        py::list nodes;
        for (const auto& n : mdl.graph.nodes) {
            py::dict nd;
            nd["name"] = n.name;
            nd["op_type"] = n.op_type;
            nd["inputs"] = n.inputs;
            nd["outputs"] = n.outputs;
            py::dict attrs;
            for (const auto& a : n.attributes) {
                if (!a.ints.empty()) attrs[py::str(a.name)] = a.ints;
                else if (!a.floats.empty()) attrs[py::str(a.name)] = a.floats;
                else if (a.t) attrs[py::str(a.name)] = tensor(*a.t);
                else if (a.has_i) attrs[py::str(a.name)] = a.i;
                else if (a.has_f) attrs[py::str(a.name)] = a.f;
                else attrs[py::str(a.name)] = py::bytes(a.s);
            }
            nd["attrs"] = attrs;
            nodes.append(nd);
        }
        out["nodes"] = nodes;
        py::list inits;
        for (const auto& t : mdl.graph.initializers) inits.append(tensor(t));
        out["initializers"] = inits;
        auto vis = [](const std::vector<onnx::ValueInfo>& v) {
            py::list l;
            for (const auto& vi : v) {
                py::dict d;
                d["name"] = vi.name;
                d["elem_type"] = vi.elem_type;
                d["dims"] = vi.dims;
                l.append(d);
            }
            return l;
        };
        out["inputs"] = vis(mdl.graph.inputs);
        out["outputs"] = vis(mdl.graph.outputs);
        return out;
    });

    // ------------------------------------------------------------ datasets
    auto dataset_to_py = [](const Dataset& d) {
        auto split = [](const ImageSet& s) {
            py::array_t<uint8_t> x({static_cast<py::ssize_t>(s.n), static_cast<py::ssize_t>(s.c),
                                    static_cast<py::ssize_t>(s.h), static_cast<py::ssize_t>(s.w)});
            if (!s.pixels.empty()) std::memcpy(x.mutable_data(), s.pixels.data(), s.pixels.size());
            py::array_t<uint8_t> y(static_cast<py::ssize_t>(s.labels.size()));
            if (!s.labels.empty()) std::memcpy(y.mutable_data(), s.labels.data(), s.labels.size());
            return py::make_tuple(x, y);
        };
        return py::make_tuple(split(d.train), split(d.test));
    };
    m.def("load_mnist", [dataset_to_py](const std::string& dir) { return dataset_to_py(load_mnist(dir)); });
    m.def("load_cifar10", [dataset_to_py](const std::string& dir) { return dataset_to_py(load_cifar10(dir)); });

    dash::register_hip_bindings(m);
}
