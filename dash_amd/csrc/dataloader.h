// Dataset readers (MNIST idx, CIFAR-10 binary). Reference: misc/dataloader.h.
#pragma once

#include <string>
#include <vector>

#include "core.h"

namespace dash {

struct ImageSet {
    size_t n = 0, c = 0, h = 0, w = 0;
    std::vector<uint8_t> pixels;  // [n][c][h][w]
    std::vector<uint8_t> labels;  // [n]
};

struct Dataset {
    ImageSet train, test;
};

// dir holds {train,t10k}-{images-idx3,labels-idx1}-ubyte (train files optional)
Dataset load_mnist(const std::string& dir);
// dir holds data_batch_{1..5}.bin (optional) and test_batch.bin
Dataset load_cifar10(const std::string& dir);

}  // namespace dash
