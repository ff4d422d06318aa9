// Native MNIST (idx) and CIFAR-10 (binary batches) readers.
// Reference counterpart: misc/dataloader.h:48-121 (dlib-based). Images are
// returned as uint8 in [C][H][W] order, the layout every layer assumes.
#include "dataloader.h"

#include <fstream>
#include <sstream>

namespace dash {
namespace {

std::string slurp(const std::string& path, bool required) {
    std::ifstream f(path, std::ios::binary);
    if (!f.good()) {
        DASH_CHECK(!required, "dataloader: cannot open " + path);
        return {};
    }
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

uint32_t be32(const std::string& s, size_t off) {
    const auto* b = reinterpret_cast<const uint8_t*>(s.data()) + off;
    return (uint32_t(b[0]) << 24) | (uint32_t(b[1]) << 16) | (uint32_t(b[2]) << 8) | uint32_t(b[3]);
}

void read_idx_images(const std::string& path, bool required, ImageSet& out) {
    std::string s = slurp(path, required);
    if (s.empty()) return;
    DASH_CHECK(s.size() >= 16 && be32(s, 0) == 0x00000803, "dataloader: bad idx3 magic in " + path);
    const uint32_t n = be32(s, 4), rows = be32(s, 8), cols = be32(s, 12);
    DASH_CHECK(s.size() >= 16 + size_t(n) * rows * cols, "dataloader: truncated " + path);
    out.n = n;
    out.c = 1;
    out.h = rows;
    out.w = cols;
    out.pixels.assign(s.begin() + 16, s.begin() + 16 + size_t(n) * rows * cols);
}

void read_idx_labels(const std::string& path, bool required, ImageSet& out) {
    std::string s = slurp(path, required);
    if (s.empty()) return;
    DASH_CHECK(s.size() >= 8 && be32(s, 0) == 0x00000801, "dataloader: bad idx1 magic in " + path);
    const uint32_t n = be32(s, 4);
    DASH_CHECK(s.size() >= 8 + size_t(n), "dataloader: truncated " + path);
    out.labels.assign(s.begin() + 8, s.begin() + 8 + n);
}

void read_cifar_batch(const std::string& path, bool required, ImageSet& out) {
    std::string s = slurp(path, required);
    if (s.empty()) return;
    constexpr size_t rec = 1 + 3 * 32 * 32;
    DASH_CHECK(s.size() % rec == 0, "dataloader: CIFAR-10 batch size is not a multiple of 3073: " + path);
    const size_t n = s.size() / rec;
    out.c = 3;
    out.h = 32;
    out.w = 32;
    for (size_t i = 0; i < n; ++i) {
        out.labels.push_back(static_cast<uint8_t>(s[i * rec]));
        // record: R plane, G plane, B plane, each row-major -> already [C][H][W]
        out.pixels.insert(out.pixels.end(), s.begin() + i * rec + 1, s.begin() + (i + 1) * rec);
    }
    out.n += n;
}

}  // namespace

Dataset load_mnist(const std::string& dir) {
    Dataset d;
    read_idx_images(dir + "/train-images-idx3-ubyte", false, d.train);
    read_idx_labels(dir + "/train-labels-idx1-ubyte", false, d.train);
    read_idx_images(dir + "/t10k-images-idx3-ubyte", true, d.test);
    read_idx_labels(dir + "/t10k-labels-idx1-ubyte", true, d.test);
    DASH_CHECK(d.test.labels.size() == d.test.n, "dataloader: MNIST test image/label count mismatch");
    DASH_CHECK(d.train.labels.size() == d.train.n, "dataloader: MNIST train image/label count mismatch");
    return d;
}

Dataset load_cifar10(const std::string& dir) {
    Dataset d;
    for (int i = 1; i <= 5; ++i) read_cifar_batch(dir + "/data_batch_" + std::to_string(i) + ".bin", false, d.train);
    read_cifar_batch(dir + "/test_batch.bin", true, d.test);
    return d;
}

}  // namespace dash
