// Host-code sanitizer harness: garble + host-evaluate + decode
// small circuits with every gadget on the multi-threaded path, built with
// -fsanitize=address,undefined (or thread). Exit code 0 = decoded outputs
// equal the plaintext expectations computed here.
#include <cstdio>
#include <random>

#include "model.h"

using namespace dash;

static int check(const char* name, const std::vector<i64>& got, const std::vector<i64>& want) {
    if (got != want) {
        std::fprintf(stderr, "%s: mismatch\n", name);
        for (size_t i = 0; i < got.size() && i < want.size(); ++i)
            std::fprintf(stderr, "  %zu: got %lld want %lld\n", i, (long long)got[i], (long long)want[i]);
        return 1;
    }
    std::printf("%s ok\n", name);
    return 0;
}

int main() {
    int fails = 0;
    const std::string seed(16, 'z');
    std::mt19937 rng(7);
    // dense 16 -> 8, relu, rescale (legacy l = 1: sign-gadget and mixed-radix constructions), sign
    for (int mrs_rescale = 0; mrs_rescale < 2; ++mrs_rescale) {
        const i64 I = 16, O = 8;
        std::vector<i64> W(I * O), b(O), x(I);
        for (auto& v : W) v = static_cast<i64>(rng() % 7) - 3;
        for (auto& v : b) v = static_cast<i64>(rng() % 11) - 5;
        for (auto& v : x) v = static_cast<i64>(rng() % 41) - 20;
        std::vector<LayerSpec> L(4);
        L[0].kind = K_DENSE;
        L[0].p["in"] = {I};
        L[0].p["out"] = {O};
        L[0].p["w"] = W;
        L[0].p["b"] = b;
        L[1].kind = K_RELU;
        L[2].kind = K_RESCALE;
        L[2].p["mode"] = {0};
        L[2].p["l"] = {1};
        L[3].kind = K_SIGN;
        const std::vector<int> crt = first_primes(8);
        const std::vector<int> mrs = {102, 7, 7, 6, 6, 6};
        Garbler g(crt, mrs, seed, required_max_modulus(crt, mrs, L, mrs_rescale != 0));
        GarbleOptions opt;
        opt.nthreads = 8;
        opt.rescale_mrs = mrs_rescale != 0;
        opt.relu_mrs = mrs_rescale != 0;  // and the exact mixed-radix sign
        GarbledModel m = g.garble(L, {I}, opt);
        CrtLabels in = g.encode(x);
        CrtLabels out = cpu_evaluate(m, in, 8);
        std::vector<i64> want(O);
        for (i64 o = 0; o < O; ++o) {
            i64 acc = b[o];
            for (i64 i = 0; i < I; ++i) acc += W[o * I + i] * x[i];
            acc = acc > 0 ? acc : 0;
            acc = (acc + 1) / 2;  // legacy rescale rounds up (ceil(x / 2) for x >= 0)
            want[o] = acc >= 0 ? 1 : -1;
        }
        fails += check(mrs_rescale ? "dense+relu+rescale(mrs)+sign" : "dense+relu+rescale+sign", g.decoder().decode(out),
                       want);
    }
    // conv 2x6x6 -> 3x6x6 (3x3, pad 1), maxpool 2x2, ReDash rescale by the first modulus
    {
        const i64 C = 2, H = 6, W = 6, F = 3;
        std::vector<i64> Wt(F * C * 9), b(F), x(C * H * W);
        for (auto& v : Wt) v = static_cast<i64>(rng() % 5) - 2;
        for (auto& v : b) v = static_cast<i64>(rng() % 9) - 4;
        for (auto& v : x) v = static_cast<i64>(rng() % 21) - 10;
        std::vector<LayerSpec> L(3);
        L[0].kind = K_CONV;
        L[0].p = {{"C", {C}}, {"H", {H}}, {"W", {W}}, {"F", {F}}, {"kh", {3}}, {"kw", {3}}, {"sh", {1}}, {"sw", {1}},
                  {"ph", {1}}, {"pw", {1}}, {"w", Wt}, {"b", b}};
        L[1].kind = K_MAXPOOL;
        L[1].p = {{"C", {F}}, {"H", {H}}, {"W", {W}}, {"kh", {2}}, {"kw", {2}}};
        L[2].kind = K_RESCALE;
        L[2].p = {{"mode", {1}}, {"s", {32}}};
        const std::vector<int> crt = {32, 3, 5, 7, 11, 13, 17};
        const std::vector<int> mrs = {10, 9, 9, 8, 7, 7, 6};
        Garbler g(crt, mrs, seed, required_max_modulus(crt, mrs, L));
        GarbleOptions opt;
        opt.nthreads = 8;
        GarbledModel m = g.garble(L, {C, H, W}, opt);
        // serialization round trip on the way
        GarbledModel m2 = GarbledModel::deserialize(m.serialize());
        CrtLabels out = cpu_evaluate(m2, g.encode(x), 8);
        i64 M = 1;
        for (int p : crt) M *= p;
        const i64 S = 32, off = (M / 2) % S;
        std::vector<i64> conv(F * H * W), want;
        for (i64 f = 0; f < F; ++f)
            for (i64 oy = 0; oy < H; ++oy)
                for (i64 ox = 0; ox < W; ++ox) {
                    i64 acc = b[f];
                    for (i64 c = 0; c < C; ++c)
                        for (i64 dy = 0; dy < 3; ++dy)
                            for (i64 dx = 0; dx < 3; ++dx) {
                                const i64 iy = oy + dy - 1, ix = ox + dx - 1;
                                if (iy >= 0 && iy < H && ix >= 0 && ix < W)
                                    acc += Wt[((f * C + c) * 3 + dy) * 3 + dx] * x[(c * H + iy) * W + ix];
                            }
                    conv[(f * H + oy) * W + ox] = acc;
                }
        for (i64 f = 0; f < F; ++f)
            for (i64 oy = 0; oy < H / 2; ++oy)
                for (i64 ox = 0; ox < W / 2; ++ox) {
                    i64 mx = conv[(f * H + 2 * oy) * W + 2 * ox];
                    for (int q = 1; q < 4; ++q) mx = std::max(mx, conv[(f * H + 2 * oy + q / 2) * W + 2 * ox + q % 2]);
                    const i64 num = mx + off;
                    want.push_back(num >= 0 ? num / S : -((-num + S - 1) / S));  // floor division
                }
        fails += check("conv+maxpool+redash_rescale", g.decoder().decode(out), want);
    }
    return fails;
}
