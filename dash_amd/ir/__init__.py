"""Plaintext model IR: layers, circuit, quantization, bases, ONNX import."""
