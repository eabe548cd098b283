"""cxxnet_amd: an MI355X-native convolutional-network training framework with
cxxnet's capabilities (.conf networks, CLI tasks, checkpoint format, Python API).

Compute path: hand-written gfx950 HIP kernels (MFMA implicit-GEMM convolution,
fused layer kernels, fused optimizer) on NHWC bf16 activations; one process per GPU
with RCCL over xGMI for data parallelism; a native C++ runtime for the config
language, graph description, checkpoint PODs, data IO and metrics.
"""
__version__ = "0.1.0"

from . import native  # noqa: F401
