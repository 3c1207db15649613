"""bwagpu — Python host side of the MI355X seed-extension engine (ctypes over
include/bwagpu.h).  The product is lib/libbwagpu.so; this package only moves
arrays across the C ABI and never computes alignments itself."""
from . import abi
from .engine import Batch, BwaGpuError, Engine, compact, unflatten

__all__ = ["abi", "Batch", "BwaGpuError", "Engine", "compact", "unflatten"]
