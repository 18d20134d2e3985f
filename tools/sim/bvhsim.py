"""Loader of tools/lib/libark_bvhsim.so: the host traversal simulator of the BVH8
(tools/sim/bvh_trace_sim.cpp), a tool kept out of the product library libark_ddgi.so."""
import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "..", "lib", "libark_bvhsim.so")
_lib = None


def load(build: bool = True) -> C.CDLL:
    """The simulator library (built by `make -C tools/sim`, which __graft_entry__.build()
    runs; `build` makes it here when it is missing)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB) and build:
        subprocess.run(["make", "-j4"], cwd=HERE, check=True)
    lib = C.CDLL(LIB)
    lib.ark_ddgi_debug_bvh8_trace_stats.restype = C.c_int
    lib.ark_ddgi_debug_bvh8_trace_stats.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_int, C.POINTER(C.c_uint64), C.c_void_p]
    _lib = lib
    return lib
