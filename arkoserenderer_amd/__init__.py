"""arkoserenderer_amd — MI355X-native DDGI probe-update path for Arkose.

The hot path is HIP for gfx950 in arkoserenderer_amd/csrc (libark_ddgi.so),
reached through the C-ABI in include/ark_ddgi.h. This package holds the Python
host mirror of the reference node interface (ddgi.py), the scene inputs
(scene.py) and the ctypes binding (abi.py).
"""
from . import abi  # noqa: F401

__all__ = ["abi", "ddgi", "scene"]
