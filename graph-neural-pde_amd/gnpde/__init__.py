"""gnpde — MI355X-native GRAND/BLEND ODE right-hand side.

Drop-in for the hot path of alimt1992/graph-neural-pde: the ODEFunc / ODEblock
classes keep the reference's signatures (see model_configurations.set_function
/ set_block); the arithmetic runs in hand-written gfx950 HIP kernels behind the
C ABI of include/gnpde.h (libgnpde.so, loaded by gnpde._lib with no fallback).
"""
from . import _lib, ops  # noqa: F401
from .base_classes import GraphData, ODEblock, ODEFunc  # noqa: F401
from .block_constant import ConstantODEblock  # noqa: F401
from .block_mixed import MixedODEblock  # noqa: F401
from .block_transformer_hard_attention import HardAttODEblock  # noqa: F401
from .block_transformer_attention import AttODEblock  # noqa: F401
from .function_laplacian_diffusion import LaplacianODEFunc  # noqa: F401
from .function_transformer_attention import ODEFuncTransformerAtt, SpGraphTransAttentionLayer  # noqa: F401
from .model_configurations import set_block, set_function  # noqa: F401
from .integrator import odeint  # noqa: F401
from .utils import MaxNFEException  # noqa: F401

__version__ = "0.1.0"


def native_library_path():
    return _lib.LIB_PATH


def build_info():
    """Loaded library path, the source hash compiled into it and whether it
    matches the sources of this tree."""
    lib, src = _lib.build_id(), _lib.source_hash()
    return {"library": _lib.LIB_PATH, "build_id": lib, "source_hash": src, "fresh": lib == src}
