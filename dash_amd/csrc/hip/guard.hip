// The garbler's exact run-time range guard on the GPU (dash_amd/garbling/guard.py RangeGuard).
//
// The garbled circuit computes modulo M = prod(CRT base) and its non-linear gadgets read signed values in
// [-M/2, M/2); the mixed-radix rescale (gadgets.h RescaleMrsPlan) is exact only below Rescale.mrs_limit(M).
// The garbler holds the plaintext input and the public weights, so per input it evaluates the quantized model
// exactly (int64 activations, 32x32 -> 64-bit products) and flags every input whose gadget inputs leave their
// exact range. It runs on its own high-priority stream beside the garbled evaluation of the same inputs; the
// flags land in mapped host memory and are read before any result is released.
//
// One launch per layer over a chunk of inputs:
//   k_g_conv   a lane per (input, 4 filters, output pixel): pixel-fastest, so the filter block is wave-uniform
//              (its weights are scalar loads) and a wave reads 64 neighbouring input pixels per tap
//   k_g_dense  a lane per (input, output)
//   k_g_elem   rescale / ReLU / sign / residual add / value-preserving layers, with the gadget range check
//   k_g_pool   max / sum pooling (max pooling: the window's inputs and its max - min span, which bounds every
//              difference b - a the pairwise max tree feeds its ReLU gadgets)
//   k_g_out    the outputs' signed range
// Flags per input (int32): bit 0 = a range violation, bit 1 = an activation beyond the int32 operand range of
// the linear layers (the exact int64 host model decides those, guard.py).
// Reference semantics: rescale_gadget.h:115-242 (exact on the whole signed range), circuit.h:159-265 (range
// tracking); the reference has no run-time guard.
#include <hip/hip_runtime.h>

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <vector>

#include "host_util.h"

namespace py = pybind11;

namespace dash {
namespace guard {

enum Kind : int { G_CONV = 0, G_DENSE = 1, G_HALVE = 2, G_DIV = 3, G_RELU = 4, G_SIGN = 5, G_MAXPOOL = 6,
                  G_SUMPOOL = 7, G_ADD = 8, G_IDENT = 9 };
constexpr int kBad = 1, kUncertain = 2;

__device__ __forceinline__ void flag(int* flags, int64_t b, int f) { atomicOr(flags + b, f); }

// operand of a 32 x 32 -> 64-bit product: x itself when it fits, else 0 and the input is marked uncertain
__device__ __forceinline__ int32_t operand(int64_t x, bool& wide) {
    const int32_t v = static_cast<int32_t>(x);
    wide |= static_cast<int64_t>(v) != x;
    return v;
}

// elementwise layers fused into the epilogue of the layer before them (guard.py native_spec): each checks its
// input against its gadget range, then applies its function
struct PostOp {
    int kind, check, l;
    int64_t lo, hi, S, c;
};
constexpr int kMaxPost = 6;
struct Post {
    int n;
    PostOp op[kMaxPost];
};
__device__ __forceinline__ int64_t floordiv(int64_t a, int64_t s) {
    int64_t q = a / s;
    if ((a % s != 0) && (a < 0)) --q;
    return q;
}
__device__ __forceinline__ int64_t run_post(const Post& P, int64_t v, bool& bad) {
    for (int i = 0; i < P.n; ++i) {
        const PostOp& o = P.op[i];
        if (o.check && (v < o.lo || v >= o.hi)) bad = true;
        switch (o.kind) {
            case G_HALVE:
                for (int s = 0; s < o.l; ++s) v = (v + o.c) >> 1;  // floor((v + c) / 2), two's complement
                break;
            case G_DIV: v = floordiv(v + o.c, o.S); break;
            case G_RELU: v = v > 0 ? v : 0; break;
            case G_SIGN: v = v >= 0 ? 1 : -1; break;
            default: break;
        }
    }
    return v;
}

struct ConvP {
    const int64_t* x;
    int64_t* y;
    const int32_t* w;  // [F][C][kh][kw]
    const int64_t* bias;
    int* flags;
    int C, H, W, F, kh, kw, sh, sw, ph, pw, OH, OW;
    int64_t in_size, out_size;
    int64_t asafe;  // I24: operands |x| <= asafe keep every partial sum inside int32 (host bound, see Layer)
    Post post;
};
constexpr int kFB = 8;  // filters per lane (one input load feeds kFB multiply-adds)
// I24: 24 x 24-bit multiply-adds into int32 accumulators (v_mad_i32_i24, full rate), exact for operands up to
// the layer's safe bound; a larger operand marks the input uncertain. Otherwise 32 x 32 -> 64-bit products.
// Lanes = output pixels, padded to whole waves per (input, filter block): the filter block is wave-uniform, so
// its weights are scalar loads (KH x KW > 0: the taps unrolled, a channel's taps merged into wide scalar loads).
// PAD = false: no tap of a valid output pixel leaves the image (no bounds checks).
template <int KH, int KW, bool I24, bool PAD>
__global__ __launch_bounds__(256) void k_g_conv(ConvP p, int64_t total) {
    const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= total) return;
    const int OHW = p.OH * p.OW;
    const int OHWp = (OHW + 63) & ~63;
    const int nfb = (p.F + kFB - 1) / kFB;
    const int pix = static_cast<int>(t % OHWp);
    const int64_t r = t / OHWp;
    const int fb = __builtin_amdgcn_readfirstlane(static_cast<int>(r % nfb));
    const int64_t b = static_cast<int64_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(r / nfb)));
    if (pix >= OHW) return;
    const int kh = KH ? KH : p.kh, kw = KW ? KW : p.kw;
    const int oy = pix / p.OW, ox = pix - oy * p.OW;
    const int f0 = fb * kFB;
    const int K = p.C * kh * kw;
    const int64_t* xb = p.x + b * p.in_size;
    int64_t acc[kFB];
    int32_t a32[kFB];
#pragma unroll
    for (int j = 0; j < kFB; ++j) acc[j] = 0, a32[j] = 0;
    const int32_t* wf[kFB];
#pragma unroll
    for (int j = 0; j < kFB; ++j) wf[j] = p.w + static_cast<int64_t>(min(f0 + j, p.F - 1)) * K;
    bool wide = false;
    const int iy0 = oy * p.sh - p.ph, ix0 = ox * p.sw - p.pw;
    const int64_t HW = static_cast<int64_t>(p.H) * p.W;
#pragma unroll 2
    for (int c = 0; c < p.C; ++c) {
        const int64_t* xc = xb + c * HW;
        const int kc = c * kh * kw;
#pragma unroll
        for (int dy = 0; dy < kh; ++dy) {
            const int iy = iy0 + dy;
            const bool rowok = !PAD || (iy >= 0 && iy < p.H);
            const int64_t* xr = xc + static_cast<int64_t>(iy) * p.W;
#pragma unroll
            for (int dx = 0; dx < kw; ++dx) {
                const int ix = ix0 + dx;
                const int64_t xv = (!PAD || (rowok && ix >= 0 && ix < p.W)) ? xr[ix] : 0;
                const int k = kc + dy * kw + dx;
                if (I24) {
                    wide |= xv > p.asafe || xv < -p.asafe;
                    const int32_t xo = static_cast<int32_t>(xv);
#pragma unroll
                    for (int j = 0; j < kFB; ++j) a32[j] += __mul24(xo, wf[j][k]);
                } else {
                    const int32_t xo = operand(xv, wide);
#pragma unroll
                    for (int j = 0; j < kFB; ++j) acc[j] += static_cast<int64_t>(xo) * wf[j][k];
                }
            }
        }
    }
    if (wide) flag(p.flags, b, kUncertain);
    int64_t* yb = p.y + b * p.out_size;
    bool bad = false;
#pragma unroll
    for (int j = 0; j < kFB; ++j) {
        const int f = f0 + j;
        if (f < p.F)
            yb[static_cast<int64_t>(f) * OHW + pix] =
                run_post(p.post, (I24 ? static_cast<int64_t>(a32[j]) : acc[j]) + p.bias[f], bad);
    }
    if (bad) flag(p.flags, b, kBad);
}

struct DenseP {
    const int64_t* x;
    int64_t* y;
    const int32_t* w;  // [out][in]
    const int64_t* bias;
    const int32_t* perm;  // channel_tf: input element of column k (null: identity)
    int* flags;
    int64_t in, out, in_size, out_size;
    Post post;
};
__global__ __launch_bounds__(256) void k_g_dense(DenseP p, int64_t total) {
    const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= total) return;
    const int64_t o = t % p.out, b = t / p.out;
    const int64_t* xb = p.x + b * p.in_size;
    const int32_t* wr = p.w + o * p.in;
    int64_t acc = 0;
    bool wide = false, bad = false;
    for (int64_t k = 0; k < p.in; ++k) {
        const int64_t xv = xb[p.perm ? p.perm[k] : k];
        acc += static_cast<int64_t>(operand(xv, wide)) * wr[k];
    }
    if (wide) flag(p.flags, b, kUncertain);
    p.y[b * p.out_size + o] = run_post(p.post, acc + p.bias[o], bad);
    if (bad) flag(p.flags, b, kBad);
}

// a chain of elementwise layers (the head and its fused successors) or a residual add followed by one
struct ElemP {
    const int64_t* x;
    const int64_t* x2;  // add: the residual source (null: none)
    int64_t* y;
    int* flags;
    int64_t n, in_size, in2_size, out_size;
    Post post;
};
__global__ __launch_bounds__(256) void k_g_elem(ElemP p, int64_t total) {
    const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= total) return;
    const int64_t i = t % p.n, b = t / p.n;
    int64_t v = p.x[b * p.in_size + i];
    if (p.x2) v += p.x2[b * p.in2_size + i];
    bool bad = false;
    p.y[b * p.out_size + i] = run_post(p.post, v, bad);
    if (bad) flag(p.flags, b, kBad);
}

struct PoolP {
    const int64_t* x;
    int64_t* y;
    int* flags;
    int maxp, check;
    int64_t lo, hi, span_max;
    int C, H, W, kh, kw, sh, sw, OH, OW;
    int64_t in_size, out_size;
    Post post;
};
__global__ __launch_bounds__(256) void k_g_pool(PoolP p, int64_t total) {
    const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= total) return;
    const int64_t per = static_cast<int64_t>(p.C) * p.OH * p.OW;
    const int64_t o = t % per, b = t / per;
    const int ox = static_cast<int>(o % p.OW);
    const int oy = static_cast<int>((o / p.OW) % p.OH);
    const int c = static_cast<int>(o / (static_cast<int64_t>(p.OW) * p.OH));
    const int64_t* xb = p.x + b * p.in_size + static_cast<int64_t>(c) * p.H * p.W;
    int64_t mx = INT64_MIN, mn = INT64_MAX, sum = 0;
    for (int dy = 0; dy < p.kh; ++dy)
        for (int dx = 0; dx < p.kw; ++dx) {
            const int64_t v = xb[static_cast<int64_t>(oy * p.sh + dy) * p.W + ox * p.sw + dx];
            mx = v > mx ? v : mx;
            mn = v < mn ? v : mn;
            sum += v;
        }
    bool bad = p.check && (mn < p.lo || mx >= p.hi || (p.maxp && mx - mn > p.span_max));
    p.y[b * p.out_size + o] = run_post(p.post, p.maxp ? mx : sum, bad);
    if (bad) flag(p.flags, b, kBad);
}

__global__ __launch_bounds__(256) void k_g_out(const int64_t* x, int* flags, int64_t lo, int64_t hi, int64_t n,
                                               int64_t stride, int64_t total) {
    const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= total) return;
    const int64_t i = t % n, b = t / n;
    const int64_t v = x[b * stride + i];
    if (v < lo || v >= hi) flag(flags, b, kBad);
}

// flags of a chunk zeroed / copied to the ticket's mapped host flags by kernels: a captured hipMemsetAsync of
// the flags did not take effect on graph replays (stale flags of an earlier check survived, bench on a full GPU)
__global__ __launch_bounds__(256) void k_g_zero(int* flags, int64_t n) {
    const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t < n) flags[t] = 0;
}
__global__ __launch_bounds__(256) void k_g_fetch(const int* flags, int* host, int64_t n) {
    const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t < n) host[t] = flags[t];
    __threadfence_system();
}

// ------------------------------------------------------------------ host
struct Layer {
    int kind, src;  // src: context index of the input (0 = circuit input, i + 1 = output of layer i)
    int buf;        // activation buffer of this layer's output
    int64_t in_size, out_size;
    int check = 0;
    int64_t lo = 0, hi = 0, span_max = 0, S = 1, c = 0;
    int l = 0;
    int C = 0, H = 0, W = 0, F = 0, kh = 0, kw = 0, sh = 1, sw = 1, ph = 0, pw = 0, OH = 0, OW = 0;
    int add_src = -1;  // G_ADD: context index of the residual
    int32_t* w = nullptr;
    int64_t* bias = nullptr;
    int32_t* perm = nullptr;
    // conv: operands |x| <= asafe keep every partial sum inside int32 (asafe * max_f sum_k |w_fk| <= 2^31 - 1;
    // the bias is added in int64) and inside the 24-bit multiplier; 0 = the 64-bit product form
    int64_t asafe = 0;
    Post post{};  // elementwise layers applied to this layer's output (an elementwise head: its own op first)
};

inline int knob(const char* name, int dflt) {
    const char* e = std::getenv(name);
    return e ? std::atoi(e) : dflt;
}
inline unsigned blocks_of(int64_t total) { return static_cast<unsigned>((total + 255) / 256); }

class DevRangeGuard {
   public:
    // layers: dicts built by garbling/guard.py (_native_spec); ctx_buf: activation buffer of every context
    // index (0 = input); nbuf buffers of buf_elems int64 per input each
    DevRangeGuard(int device, const py::list& layers, int64_t input_size, std::vector<int> ctx_buf,
                  std::vector<int64_t> buf_elems, int64_t out_lo, int64_t out_hi, int chunk)
        : dev_(device), N_(input_size), ctx_buf_(std::move(ctx_buf)), buf_elems_(std::move(buf_elems)),
          out_lo_(out_lo), out_hi_(out_hi), chunk_(chunk) {
        DASH_CHECK(chunk_ >= 1 && chunk_ <= 4096, "DevRangeGuard: chunk out of range");
        hostutil::bind_device(dev_, nullptr, "DevRangeGuard");
        for (auto item : layers) {
            py::dict d = item.cast<py::dict>();
            Layer L{};
            L.kind = d["kind"].cast<int>();
            L.src = d["src"].cast<int>();
            L.buf = d["buf"].cast<int>();
            L.in_size = d["in_size"].cast<int64_t>();
            L.out_size = d["out_size"].cast<int64_t>();
            if (d.contains("check") && d["check"].cast<bool>()) {
                L.check = 1;
                L.lo = d["lo"].cast<int64_t>();
                L.hi = d["hi"].cast<int64_t>();
            }
            auto geti = [&](const char* k, int dflt) { return d.contains(k) ? d[k].cast<int>() : dflt; };
            L.span_max = d.contains("span_max") ? d["span_max"].cast<int64_t>() : 0;
            L.S = d.contains("S") ? d["S"].cast<int64_t>() : 1;
            L.c = d.contains("c") ? d["c"].cast<int64_t>() : 0;
            L.l = geti("l", 0);
            L.C = geti("C", 0), L.H = geti("H", 0), L.W = geti("W", 0), L.F = geti("F", 0);
            L.kh = geti("kh", 0), L.kw = geti("kw", 0), L.sh = geti("sh", 1), L.sw = geti("sw", 1);
            L.ph = geti("ph", 0), L.pw = geti("pw", 0), L.OH = geti("OH", 0), L.OW = geti("OW", 0);
            L.add_src = geti("add_src", -1);
            if (d.contains("post")) {
                py::list ops = d["post"].cast<py::list>();
                DASH_CHECK(ops.size() <= static_cast<size_t>(kMaxPost), "DevRangeGuard: too many fused layers");
                for (auto o : ops) {
                    py::dict od = o.cast<py::dict>();
                    PostOp& op = L.post.op[L.post.n++];
                    op.kind = od["kind"].cast<int>();
                    DASH_CHECK(op.kind >= G_HALVE && op.kind <= G_SIGN || op.kind == G_IDENT,
                               "DevRangeGuard: fused layer kind");
                    op.check = od.contains("check") && od["check"].cast<bool>() ? 1 : 0;
                    op.lo = op.check ? od["lo"].cast<int64_t>() : 0;
                    op.hi = op.check ? od["hi"].cast<int64_t>() : 0;
                    op.l = od.contains("l") ? od["l"].cast<int>() : 0;
                    op.S = od.contains("S") ? od["S"].cast<int64_t>() : 1;
                    op.c = od.contains("c") ? od["c"].cast<int64_t>() : 0;
                    DASH_CHECK(op.kind != G_DIV || op.S >= 1, "DevRangeGuard: rescale divisor");
                    DASH_CHECK(op.l >= 0 && op.l < 63, "DevRangeGuard: rescale halvings");
                }
            }
            DASH_CHECK(L.kind == G_CONV || L.kind == G_DENSE || L.kind == G_MAXPOOL || L.kind == G_SUMPOOL ||
                           L.kind == G_ADD || L.kind == G_IDENT,
                       "DevRangeGuard: unknown layer kind (elementwise layers come as fused ops)");
            DASH_CHECK(L.src >= 0 && static_cast<size_t>(L.src) < ctx_buf_.size(), "DevRangeGuard: bad source");
            DASH_CHECK(L.buf >= 0 && static_cast<size_t>(L.buf) < buf_elems_.size(), "DevRangeGuard: bad buffer");
            DASH_CHECK(L.out_size <= buf_elems_[L.buf], "DevRangeGuard: buffer too small");
            DASH_CHECK(L.kind != G_DIV || L.S >= 1, "DevRangeGuard: rescale divisor");
            if (L.kind == G_CONV) {
                DASH_CHECK(L.C > 0 && L.H > 0 && L.W > 0 && L.F > 0 && L.kh > 0 && L.kw > 0 && L.OH > 0 && L.OW > 0,
                           "DevRangeGuard: conv geometry");
                DASH_CHECK(L.in_size == static_cast<int64_t>(L.C) * L.H * L.W &&
                               L.out_size == static_cast<int64_t>(L.F) * L.OH * L.OW,
                           "DevRangeGuard: conv sizes");
                DASH_CHECK((L.OH - 1) * L.sh - L.ph + L.kh <= L.H + L.ph && (L.OW - 1) * L.sw - L.pw + L.kw <= L.W + L.pw,
                           "DevRangeGuard: conv output dims");
            }
            if (L.kind == G_MAXPOOL || L.kind == G_SUMPOOL) {
                DASH_CHECK((L.OH - 1) * L.sh + L.kh <= L.H && (L.OW - 1) * L.sw + L.kw <= L.W &&
                               L.in_size == static_cast<int64_t>(L.C) * L.H * L.W &&
                               L.out_size == static_cast<int64_t>(L.C) * L.OH * L.OW,
                           "DevRangeGuard: pool geometry");
            }
            if (L.kind == G_CONV || L.kind == G_DENSE) {
                auto w = d["w"].cast<py::array_t<int32_t, py::array::c_style | py::array::forcecast>>();
                auto b = d["b"].cast<py::array_t<int64_t, py::array::c_style | py::array::forcecast>>();
                const int64_t rows = L.kind == G_CONV ? L.F : L.out_size;
                const int64_t K = L.kind == G_CONV ? static_cast<int64_t>(L.C) * L.kh * L.kw : L.in_size;
                DASH_CHECK(w.size() == rows * K && b.size() == rows, "DevRangeGuard: weight / bias shape");
                L.w = upload(w.data(), w.size());
                L.bias = upload(b.data(), b.size());
                if (L.kind == G_CONV) {
                    int64_t wsum = 1, wmax = 0;
                    for (int64_t f = 0; f < rows; ++f) {
                        int64_t s = 0;
                        for (int64_t k = 0; k < K; ++k) {
                            const int64_t v = std::abs(static_cast<int64_t>(w.data()[f * K + k]));
                            s += v;
                            wmax = std::max(wmax, v);
                        }
                        wsum = std::max(wsum, s);
                    }
                    const int64_t lim24 = (int64_t(1) << 23) - 1;
                    L.asafe = wmax <= lim24 ? std::min(lim24, ((int64_t(1) << 31) - 1) / wsum) : 0;
                    if (knob("DASH_GUARD_I24", 1) == 0) L.asafe = 0;  // A/B: the 64-bit product form
                }
                if (L.kind == G_DENSE && d.contains("perm") && !d["perm"].is_none()) {
                    auto pm = d["perm"].cast<py::array_t<int32_t, py::array::c_style | py::array::forcecast>>();
                    DASH_CHECK(pm.size() == L.in_size, "DevRangeGuard: permutation size");
                    for (py::ssize_t k = 0; k < pm.size(); ++k)
                        DASH_CHECK(pm.data()[k] >= 0 && pm.data()[k] < L.in_size, "DevRangeGuard: permutation entry");
                    L.perm = upload(pm.data(), pm.size());
                }
            }
            if (L.kind == G_ADD)
                DASH_CHECK(L.add_src >= 0 && static_cast<size_t>(L.add_src) < ctx_buf_.size(), "DevRangeGuard: add source");
            if (L.kind == G_ADD || L.kind == G_IDENT)
                DASH_CHECK(L.in_size == L.out_size, "DevRangeGuard: elementwise layer changes the size");
            layers_.push_back(L);
        }
        DASH_CHECK(!layers_.empty(), "DevRangeGuard: empty circuit");
        DASH_CHECK(ctx_buf_.size() >= 2, "DevRangeGuard: context map size");
        // buffers: chunk inputs each
        for (int64_t e : buf_elems_) {
            int64_t* p = nullptr;
            HIPCHECK(hipMalloc(reinterpret_cast<void**>(&p), sizeof(int64_t) * e * chunk_));
            bufs_.push_back(p);
        }
        // stream priority (A/B knob DASH_GUARD_PRIO = 0 low, 1 normal, 2 high): high by default, so the check
        // never waits behind the evaluation it overlaps
        int lo_pri = 0, hi_pri = 0;
        HIPCHECK(hipDeviceGetStreamPriorityRange(&lo_pri, &hi_pri));
        const int pk = knob("DASH_GUARD_PRIO", 2);
        const int pri = pk >= 2 ? hi_pri : (pk == 1 ? (lo_pri + hi_pri) / 2 : lo_pri);
        HIPCHECK(hipStreamCreateWithPriority(&st_, hipStreamNonBlocking, pri));
    }
    ~DevRangeGuard() {
        (void)hipSetDevice(dev_);
        (void)hipStreamSynchronize(st_);
        for (auto& t : tickets_) release(t);
        for (auto* p : bufs_) (void)hipFree(p);
        for (auto* p : owned_) (void)hipFree(p);
        (void)hipStreamDestroy(st_);
        (void)hipGetLastError();
    }
    DevRangeGuard(const DevRangeGuard&) = delete;
    DevRangeGuard& operator=(const DevRangeGuard&) = delete;

    // start the check of B inputs (x: [B][N] int64) on the guard's stream; returns a ticket for wait()
    int submit(const int64_t* x, int64_t B) {
        std::lock_guard<std::mutex> lk(mu_);
        hostutil::bind_device(dev_, st_, "DevRangeGuard::submit");
        int id = -1;
        for (size_t i = 0; i < tickets_.size(); ++i)
            if (!tickets_[i].busy) { id = static_cast<int>(i); break; }
        if (id < 0) {
            tickets_.emplace_back();
            id = static_cast<int>(tickets_.size()) - 1;
        }
        Ticket& t = tickets_[id];
        if (t.cap < B) {
            release(t);
            t.cap = std::max<int64_t>(B, chunk_);
            HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&t.x_h), sizeof(int64_t) * t.cap * N_));
            HIPCHECK(hipMalloc(reinterpret_cast<void**>(&t.x_d), sizeof(int64_t) * t.cap * N_));
            HIPCHECK(hipMalloc(reinterpret_cast<void**>(&t.flags_d), sizeof(int) * t.cap));
            HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&t.flags_h), sizeof(int) * t.cap, hipHostMallocMapped));
            HIPCHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&t.flags_hd), t.flags_h, 0));
            HIPCHECK(hipEventCreateWithFlags(&t.done, hipEventDisableTiming));
        }
        t.busy = true;
        t.B = B;
        std::memcpy(t.x_h, x, sizeof(int64_t) * B * N_);
        // the whole check (H2D, one launch per layer and chunk, flags D2H) as one graph per (ticket, batch size):
        // one launch instead of ~2 per layer, no gaps between the small layer kernels
        if (knob("DASH_GUARD_GRAPH", 1) == 0) {  // A/B: stream launches
            enqueue(t, B);
            HIPCHECK(hipEventRecord(t.done, st_));
            return id;
        }
        auto it = t.graphs.find(B);
        if (it == t.graphs.end()) {
            if (t.graphs.size() >= 8) drop_graphs(t);
            HIPCHECK(hipStreamBeginCapture(st_, hipStreamCaptureModeThreadLocal));
            enqueue(t, B);
            hipGraph_t g = nullptr;
            HIPCHECK(hipStreamEndCapture(st_, &g));
            hipGraphExec_t ge = nullptr;
            const hipError_t e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
            (void)hipGraphDestroy(g);
            HIPCHECK(e);
            it = t.graphs.emplace(B, ge).first;
        }
        HIPCHECK(hipGraphLaunch(it->second, st_));
        HIPCHECK(hipEventRecord(t.done, st_));
        return id;
    }
    // the flags of a ticket (blocks until its check has run); the ticket is free again afterwards
    std::vector<int> wait(int id) {
        Ticket* t;
        {
            std::lock_guard<std::mutex> lk(mu_);
            DASH_CHECK(id >= 0 && static_cast<size_t>(id) < tickets_.size() && tickets_[id].busy,
                       "DevRangeGuard: unknown ticket");
            t = &tickets_[id];
        }
        HIPCHECK(hipEventSynchronize(t->done));
        std::lock_guard<std::mutex> lk(mu_);
        std::vector<int> out(t->flags_h, t->flags_h + t->B);
        t->busy = false;
        return out;
    }
    int64_t input_size() const { return N_; }
    size_t device_bytes() const {
        size_t s = 0;
        for (int64_t e : buf_elems_) s += sizeof(int64_t) * e * chunk_;
        return s;
    }

   private:
    struct Ticket {
        int64_t cap = 0, B = 0;
        int64_t* x_h = nullptr;
        int64_t* x_d = nullptr;
        int* flags_d = nullptr;
        int* flags_h = nullptr;
        int* flags_hd = nullptr;  // flags_h as seen from the device (mapped)
        hipEvent_t done = nullptr;
        bool busy = false;
        std::map<int64_t, hipGraphExec_t> graphs;  // batch size -> the captured check
    };
    static void drop_graphs(Ticket& t) {
        for (auto& kv : t.graphs) (void)hipGraphExecDestroy(kv.second);
        t.graphs.clear();
    }
    void release(Ticket& t) {
        if (t.done) (void)hipEventSynchronize(t.done);
        drop_graphs(t);
        if (t.x_h) (void)hipHostFree(t.x_h);
        if (t.x_d) (void)hipFree(t.x_d);
        if (t.flags_d) (void)hipFree(t.flags_d);
        if (t.flags_h) (void)hipHostFree(t.flags_h);
        if (t.done) (void)hipEventDestroy(t.done);
        t = Ticket{};
    }
    template <class T>
    T* upload(const T* src, size_t n) {
        T* p = nullptr;
        HIPCHECK(hipMalloc(reinterpret_cast<void**>(&p), sizeof(T) * std::max<size_t>(n, 1)));
        if (n) HIPCHECK(hipMemcpy(p, src, sizeof(T) * n, hipMemcpyHostToDevice));
        owned_.push_back(p);
        return p;
    }
    void enqueue(const Ticket& t, int64_t B) {
        HIPCHECK(hipMemcpyAsync(t.x_d, t.x_h, sizeof(int64_t) * B * N_, hipMemcpyHostToDevice, st_));
        hipLaunchKernelGGL(k_g_zero, dim3(blocks_of(B)), dim3(256), 0, st_, t.flags_d, B);
        for (int64_t b0 = 0; b0 < B; b0 += chunk_) run_chunk(t, b0, std::min<int64_t>(chunk_, B - b0));
        hipLaunchKernelGGL(k_g_fetch, dim3(blocks_of(B)), dim3(256), 0, st_, t.flags_d, t.flags_hd, B);
    }
    // context index -> (pointer, per-input stride); index 0 of a chunk is the ticket's input rows
    std::pair<const int64_t*, int64_t> ctx(const Ticket& t, int idx, int64_t b0) const {
        if (idx == 0) return {t.x_d + b0 * N_, N_};
        const int buf = ctx_buf_[idx];
        return {bufs_[buf], buf_elems_[buf]};
    }
    using ConvK = void (*)(ConvP, int64_t);
    template <int KH, int KW>
    static ConvK conv_for(bool i24, bool pad) {
        return i24 ? (pad ? k_g_conv<KH, KW, true, true> : k_g_conv<KH, KW, true, false>)
                   : (pad ? k_g_conv<KH, KW, false, true> : k_g_conv<KH, KW, false, false>);
    }
    static ConvK conv_kernel(const Layer& L) {
        const bool i24 = L.asafe > 0, pad = L.ph > 0 || L.pw > 0;
        if (L.kh == 3 && L.kw == 3) return conv_for<3, 3>(i24, pad);
        if (L.kh == 2 && L.kw == 2) return conv_for<2, 2>(i24, pad);
        if (L.kh == 1 && L.kw == 1) return conv_for<1, 1>(i24, pad);
        return conv_for<0, 0>(i24, pad);
    }
    void run_chunk(const Ticket& t, int64_t b0, int64_t B) {
        int* flags = t.flags_d + b0;
        for (size_t i = 0; i < layers_.size(); ++i) {
            const Layer& L = layers_[i];
            auto in = ctx(t, L.src, b0);
            int64_t* y = bufs_[L.buf];
            const int64_t ys = buf_elems_[L.buf];
            switch (L.kind) {
                case G_CONV: {
                    ConvP p{in.first, y, L.w, L.bias, flags, L.C, L.H, L.W, L.F, L.kh, L.kw, L.sh, L.sw, L.ph, L.pw,
                            L.OH, L.OW, in.second, ys, L.asafe, L.post};
                    const int64_t ohwp = (static_cast<int64_t>(L.OH) * L.OW + 63) & ~int64_t(63);
                    const int64_t total = B * ((L.F + kFB - 1) / kFB) * ohwp;
                    hipLaunchKernelGGL(conv_kernel(L), dim3(blocks_of(total)), dim3(256), 0, st_, p, total);
                    break;
                }
                case G_DENSE: {
                    DenseP p{in.first, y, L.w, L.bias, L.perm, flags, L.in_size, L.out_size, in.second, ys, L.post};
                    const int64_t total = B * L.out_size;
                    hipLaunchKernelGGL(k_g_dense, dim3(blocks_of(total)), dim3(256), 0, st_, p, total);
                    break;
                }
                case G_MAXPOOL:
                case G_SUMPOOL: {
                    PoolP p{in.first, y, flags, L.kind == G_MAXPOOL, L.check, L.lo, L.hi, L.span_max, L.C, L.H, L.W,
                            L.kh, L.kw, L.sh, L.sw, L.OH, L.OW, in.second, ys, L.post};
                    const int64_t total = B * L.out_size;
                    hipLaunchKernelGGL(k_g_pool, dim3(blocks_of(total)), dim3(256), 0, st_, p, total);
                    break;
                }
                default: {
                    auto in2 = L.kind == G_ADD ? ctx(t, L.add_src, b0) : std::make_pair<const int64_t*, int64_t>(nullptr, 0);
                    ElemP p{in.first, in2.first, y, flags, L.out_size, in.second, in2.second, ys, L.post};
                    const int64_t total = B * L.out_size;
                    hipLaunchKernelGGL(k_g_elem, dim3(blocks_of(total)), dim3(256), 0, st_, p, total);
                }
            }
        }
        const Layer& last = layers_.back();
        const int64_t total = B * last.out_size;
        hipLaunchKernelGGL(k_g_out, dim3(blocks_of(total)), dim3(256), 0, st_, bufs_[last.buf], flags, out_lo_,
                           out_hi_, last.out_size, buf_elems_[last.buf], total);
    }

    int dev_;
    int64_t N_;
    std::vector<int> ctx_buf_;
    std::vector<int64_t> buf_elems_;
    int64_t out_lo_, out_hi_;
    int chunk_;
    std::vector<Layer> layers_;
    std::vector<int64_t*> bufs_;
    std::vector<void*> owned_;
    std::deque<Ticket> tickets_;  // stable addresses: wait() holds one while submit() appends
    hipStream_t st_ = nullptr;
    std::mutex mu_;
};

}  // namespace guard

void register_guard_bindings(py::module_& m) {
    using guard::DevRangeGuard;
    py::class_<DevRangeGuard>(m, "DevRangeGuard")
        .def(py::init<int, const py::list&, int64_t, std::vector<int>, std::vector<int64_t>, int64_t, int64_t, int>(),
             py::arg("device"), py::arg("layers"), py::arg("input_size"), py::arg("ctx_buf"), py::arg("buf_elems"),
             py::arg("out_lo"), py::arg("out_hi"), py::arg("chunk") = 64)
        .def("submit", [](DevRangeGuard& g, py::array_t<int64_t, py::array::c_style | py::array::forcecast> x) {
            DASH_CHECK(x.ndim() == 2 && x.shape(1) == g.input_size(), "DevRangeGuard.submit: x must be (B, N)");
            const int64_t B = x.shape(0);
            const int64_t* p = x.data();
            py::gil_scoped_release rel;
            return g.submit(p, B);
        })
        .def("wait", &DevRangeGuard::wait, py::call_guard<py::gil_scoped_release>())
        .def("device_bytes", &DevRangeGuard::device_bytes)
        .def("input_size", &DevRangeGuard::input_size);
}

}  // namespace dash
