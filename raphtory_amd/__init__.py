"""raphtory_amd — MI355X-native windowed temporal-analysis path of Raphtory.

The product is ``_build/librgpu.so`` (HIP kernels for gfx950 + host packer behind the C ABI of
``include/rgpu.h``).  This package is its host side: ctypes bindings (``_native``), the
per-partition ``TemporalGraph``, the Analyser / AnalysisTask mirror (``analysis``), the
partition function (``partition``) and the synthetic spouts (``synth``).
"""
from ._native import NativeUnavailable  # noqa: F401
from .graph import RGPUError, TemporalGraph  # noqa: F401
from .partition import get_partition, get_worker  # noqa: F401
from . import rgev  # noqa: F401

__all__ = ["TemporalGraph", "RGPUError", "NativeUnavailable", "get_partition", "get_worker"]
