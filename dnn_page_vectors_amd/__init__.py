"""dnn_page_vectors_amd — MI355X-native page-vector (DSSM / CDSSM two-tower) engine.

Capabilities of ``collawolley/dnn_page_vectors`` re-designed for AMD MI355X (gfx950):
hand-written HIP/CDNA4 kernels for the hot ops, PyTorch-ROCm as the tensor/autograd
host, RCCL over xGMI for data parallelism and cross-GPU in-batch negatives, and a C++
host runtime for featurisation.  See README.md and SURVEY.md.
"""
__version__ = "0.1.0"

from .config import Configuration, preset_config, PRESETS  # noqa: F401
