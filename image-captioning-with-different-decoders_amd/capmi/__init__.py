"""capmi -- MI355X-native kernels and runtime for the 'attention' captioning training step.

Importing ``capmi`` loads libcapmi.so (HIP, gfx950) and fails loudly if it is
missing: the HIP kernels are the only compute path for device tensors.
"""
from ._lib import ABI_VERSION, EXPORTS, LIB_PATH, CapmiError, lib  # noqa: F401

__all__ = ["ABI_VERSION", "EXPORTS", "LIB_PATH", "CapmiError", "lib"]
