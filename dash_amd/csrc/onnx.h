// Minimal ONNX model reader (protobuf wire format, no libprotobuf).
// Reference counterpart: circuit/onnx_modelloader.h:33-129.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "core.h"

namespace dash {
namespace onnx {

struct Tensor {
    std::string name;
    int data_type = 0;            // TensorProto.DataType (1 = FLOAT, 7 = INT64, ...)
    std::vector<int64_t> dims;
    std::vector<float> values;    // every numeric tensor, as float
    std::vector<int64_t> ivalues; // integer tensors (shapes for Reshape, ...)
};

struct Attribute {
    std::string name;
    int type = 0;
    float f = 0.f;
    int64_t i = 0;
    bool has_f = false, has_i = false;
    std::string s;
    std::vector<float> floats;
    std::vector<int64_t> ints;
    std::shared_ptr<Tensor> t;
};

struct Node {
    std::string name, op_type, domain;
    std::vector<std::string> inputs, outputs;
    std::vector<Attribute> attributes;
    const Attribute* attr(const std::string& n) const;
};

struct ValueInfo {
    std::string name;
    int elem_type = 0;
    std::vector<int64_t> dims;  // -1 for symbolic dimensions
};

struct Graph {
    std::string name;
    std::vector<Node> nodes;
    std::vector<Tensor> initializers;
    std::vector<ValueInfo> inputs, outputs;
};

struct Model {
    int64_t ir_version = 0, opset = 0;
    std::string producer_name, producer_version;
    Graph graph;
};

Model parse_model(const std::string& bytes);
Model parse_model_file(const std::string& path);

}  // namespace onnx
}  // namespace dash
