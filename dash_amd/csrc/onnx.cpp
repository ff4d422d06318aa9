// Minimal ONNX (protobuf wire format) reader.
//
// The reference links libprotobuf + generated onnx.proto3 classes
// (circuit/onnx_modelloader.h:20-54). Neither protoc nor the onnx package is
// available on the MI355X image, and the loader only needs a handful of
// message types, so this file decodes the wire format directly: ModelProto ->
// GraphProto -> {NodeProto, TensorProto (initializers), ValueInfoProto}.
// Attributes are kept *by name* (the reference indexes them positionally,
// onnx_modelloader.h:280-295, which breaks across exporters).
#include "onnx.h"

#include <cstring>
#include <fstream>
#include <sstream>

namespace dash {
namespace onnx {
namespace {

struct Reader {
    const uint8_t* p;
    const uint8_t* end;

    bool done() const { return p >= end; }
    uint64_t varint() {
        uint64_t v = 0;
        int shift = 0;
        while (true) {
            DASH_CHECK(p < end, "onnx: truncated varint");
            uint8_t b = *p++;
            v |= static_cast<uint64_t>(b & 0x7F) << shift;
            if (!(b & 0x80)) break;
            shift += 7;
            DASH_CHECK(shift < 64, "onnx: varint too long");
        }
        return v;
    }
    uint32_t fixed32() {
        DASH_CHECK(end - p >= 4, "onnx: truncated fixed32");
        uint32_t v;
        std::memcpy(&v, p, 4);
        p += 4;
        return v;
    }
    uint64_t fixed64() {
        DASH_CHECK(end - p >= 8, "onnx: truncated fixed64");
        uint64_t v;
        std::memcpy(&v, p, 8);
        p += 8;
        return v;
    }
    Reader sub() {
        uint64_t n = varint();
        DASH_CHECK(static_cast<uint64_t>(end - p) >= n, "onnx: truncated length-delimited field");
        Reader r{p, p + n};
        p += n;
        return r;
    }
    std::string str() {
        Reader r = sub();
        return std::string(reinterpret_cast<const char*>(r.p), r.end - r.p);
    }
    void skip(int wt) {
        switch (wt) {
            case 0: varint(); break;
            case 1: fixed64(); break;
            case 2: sub(); break;
            case 5: fixed32(); break;
            default: DASH_CHECK(false, "onnx: unsupported wire type " + std::to_string(wt));
        }
    }
};

float as_float(uint32_t bits) {
    float f;
    std::memcpy(&f, &bits, 4);
    return f;
}

// repeated scalar field: packed (wire type 2) or one element (wire type 0/5)
void read_ints(Reader& r, int wt, std::vector<int64_t>& out) {
    if (wt == 2) {
        Reader s = r.sub();
        while (!s.done()) out.push_back(static_cast<int64_t>(s.varint()));
    } else {
        out.push_back(static_cast<int64_t>(r.varint()));
    }
}
void read_floats(Reader& r, int wt, std::vector<float>& out) {
    if (wt == 2) {
        Reader s = r.sub();
        while (!s.done()) out.push_back(as_float(s.fixed32()));
    } else {
        out.push_back(as_float(r.fixed32()));
    }
}
void read_doubles(Reader& r, int wt, std::vector<double>& out) {
    auto one = [&](Reader& rr) {
        uint64_t b = rr.fixed64();
        double d;
        std::memcpy(&d, &b, 8);
        out.push_back(d);
    };
    if (wt == 2) {
        Reader s = r.sub();
        while (!s.done()) one(s);
    } else {
        one(r);
    }
}

Tensor parse_tensor(Reader r) {
    Tensor t;
    std::string raw;
    std::vector<float> fdata;
    std::vector<int64_t> i32, i64;
    std::vector<double> ddata;
    while (!r.done()) {
        uint64_t key = r.varint();
        int field = static_cast<int>(key >> 3), wt = static_cast<int>(key & 7);
        switch (field) {
            case 1: read_ints(r, wt, t.dims); break;
            case 2: t.data_type = static_cast<int>(r.varint()); break;
            case 4: read_floats(r, wt, fdata); break;
            case 5: read_ints(r, wt, i32); break;
            case 7: read_ints(r, wt, i64); break;
            case 8: t.name = r.str(); break;
            case 9: raw = r.str(); break;
            case 10: read_doubles(r, wt, ddata); break;
            case 14: DASH_CHECK(r.varint() == 0, "onnx: external tensor data is not supported"); break;
            default: r.skip(wt);
        }
    }
    int64_t numel = 1;
    for (auto d : t.dims) numel *= d;
    if (!raw.empty()) {
        // raw_data is always little endian (ONNX spec); x86 hosts read it as-is
        switch (t.data_type) {
            case 1: {  // FLOAT
                DASH_CHECK(static_cast<int64_t>(raw.size()) == 4 * numel, "onnx: float raw_data size mismatch");
                t.values.resize(numel);
                std::memcpy(t.values.data(), raw.data(), raw.size());
                break;
            }
            case 11: {  // DOUBLE
                t.values.resize(numel);
                for (int64_t i = 0; i < numel; ++i) {
                    double d;
                    std::memcpy(&d, raw.data() + 8 * i, 8);
                    t.values[i] = static_cast<float>(d);
                }
                t.ivalues.resize(0);
                break;
            }
            case 7: {  // INT64
                DASH_CHECK(static_cast<int64_t>(raw.size()) == 8 * numel, "onnx: int64 raw_data size mismatch");
                t.ivalues.resize(numel);
                std::memcpy(t.ivalues.data(), raw.data(), raw.size());
                break;
            }
            case 6: {  // INT32
                t.ivalues.resize(numel);
                for (int64_t i = 0; i < numel; ++i) {
                    int32_t v;
                    std::memcpy(&v, raw.data() + 4 * i, 4);
                    t.ivalues[i] = v;
                }
                break;
            }
            default: DASH_CHECK(false, "onnx: unsupported tensor data type " + std::to_string(t.data_type));
        }
    } else if (!fdata.empty()) {
        t.values = std::move(fdata);
    } else if (!ddata.empty()) {
        t.values.assign(ddata.begin(), ddata.end());
    } else if (!i64.empty()) {
        t.ivalues = std::move(i64);
    } else if (!i32.empty()) {
        t.ivalues = std::move(i32);
    }
    if (t.values.empty() && !t.ivalues.empty())
        for (auto v : t.ivalues) t.values.push_back(static_cast<float>(v));
    return t;
}

Attribute parse_attribute(Reader r) {
    Attribute a;
    while (!r.done()) {
        uint64_t key = r.varint();
        int field = static_cast<int>(key >> 3), wt = static_cast<int>(key & 7);
        switch (field) {
            case 1: a.name = r.str(); break;
            case 2: a.f = as_float(r.fixed32()); a.has_f = true; break;
            case 3: a.i = static_cast<int64_t>(r.varint()); a.has_i = true; break;
            case 4: a.s = r.str(); break;
            case 5: a.t = std::make_shared<Tensor>(parse_tensor(r.sub())); break;
            case 7: read_floats(r, wt, a.floats); break;
            case 8: read_ints(r, wt, a.ints); break;
            case 20: a.type = static_cast<int>(r.varint()); break;
            default: r.skip(wt);
        }
    }
    return a;
}

Node parse_node(Reader r) {
    Node n;
    while (!r.done()) {
        uint64_t key = r.varint();
        int field = static_cast<int>(key >> 3), wt = static_cast<int>(key & 7);
        switch (field) {
            case 1: n.inputs.push_back(r.str()); break;
            case 2: n.outputs.push_back(r.str()); break;
            case 3: n.name = r.str(); break;
            case 4: n.op_type = r.str(); break;
            case 5: n.attributes.push_back(parse_attribute(r.sub())); break;
            case 7: n.domain = r.str(); break;
            default: r.skip(wt);
        }
    }
    return n;
}

// TensorShapeProto.Dimension
int64_t parse_dim(Reader r) {
    int64_t v = -1;
    while (!r.done()) {
        uint64_t key = r.varint();
        int field = static_cast<int>(key >> 3), wt = static_cast<int>(key & 7);
        if (field == 1) v = static_cast<int64_t>(r.varint());
        else r.skip(wt);  // dim_param (symbolic, e.g. batch) -> -1
    }
    return v;
}

ValueInfo parse_value_info(Reader r) {
    ValueInfo vi;
    while (!r.done()) {
        uint64_t key = r.varint();
        int field = static_cast<int>(key >> 3), wt = static_cast<int>(key & 7);
        if (field == 1) {
            vi.name = r.str();
        } else if (field == 2) {  // TypeProto
            Reader tp = r.sub();
            while (!tp.done()) {
                uint64_t k2 = tp.varint();
                if ((k2 >> 3) == 1) {  // tensor_type
                    Reader tt = tp.sub();
                    while (!tt.done()) {
                        uint64_t k3 = tt.varint();
                        int f3 = static_cast<int>(k3 >> 3), w3 = static_cast<int>(k3 & 7);
                        if (f3 == 1) {
                            vi.elem_type = static_cast<int>(tt.varint());
                        } else if (f3 == 2) {  // shape
                            Reader sh = tt.sub();
                            while (!sh.done()) {
                                uint64_t k4 = sh.varint();
                                if ((k4 >> 3) == 1) vi.dims.push_back(parse_dim(sh.sub()));
                                else sh.skip(static_cast<int>(k4 & 7));
                            }
                        } else {
                            tt.skip(w3);
                        }
                    }
                } else {
                    tp.skip(static_cast<int>(k2 & 7));
                }
            }
        } else {
            r.skip(wt);
        }
    }
    return vi;
}

Graph parse_graph(Reader r) {
    Graph g;
    while (!r.done()) {
        uint64_t key = r.varint();
        int field = static_cast<int>(key >> 3), wt = static_cast<int>(key & 7);
        switch (field) {
            case 1: g.nodes.push_back(parse_node(r.sub())); break;
            case 2: g.name = r.str(); break;
            case 5: g.initializers.push_back(parse_tensor(r.sub())); break;
            case 11: g.inputs.push_back(parse_value_info(r.sub())); break;
            case 12: g.outputs.push_back(parse_value_info(r.sub())); break;
            default: r.skip(wt);
        }
    }
    return g;
}

}  // namespace

const Attribute* Node::attr(const std::string& n) const {
    for (const auto& a : attributes)
        if (a.name == n) return &a;
    return nullptr;
}

Model parse_model(const std::string& bytes) {
    Model m;
    Reader r{reinterpret_cast<const uint8_t*>(bytes.data()), reinterpret_cast<const uint8_t*>(bytes.data()) + bytes.size()};
    bool have_graph = false;
    while (!r.done()) {
        uint64_t key = r.varint();
        int field = static_cast<int>(key >> 3), wt = static_cast<int>(key & 7);
        switch (field) {
            case 1: m.ir_version = static_cast<int64_t>(r.varint()); break;
            case 2: m.producer_name = r.str(); break;
            case 3: m.producer_version = r.str(); break;
            case 7: m.graph = parse_graph(r.sub()); have_graph = true; break;
            case 8: {  // OperatorSetIdProto {domain=1, version=2}
                Reader o = r.sub();
                while (!o.done()) {
                    uint64_t k2 = o.varint();
                    if ((k2 >> 3) == 2) m.opset = static_cast<int64_t>(o.varint());
                    else o.skip(static_cast<int>(k2 & 7));
                }
                break;
            }
            default: r.skip(wt);
        }
    }
    DASH_CHECK(have_graph, "onnx: model has no graph");
    return m;
}

Model parse_model_file(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    DASH_CHECK(f.good(), "onnx: cannot open " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    return parse_model(ss.str());
}

}  // namespace onnx
}  // namespace dash
