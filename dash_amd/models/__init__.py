"""Model zoo (paper architectures + LeNet-5 / VGG-16 / ResNet-18)."""
from .zoo import ARCHS, BENCH_CONFIGS, build_circuit, canonical, input_dims, quantized_inputs, synthetic_inputs  # noqa: F401
