"""udpdk_amd — MI355X-native UDPDK datapath.

The product is the C/HIP shared library ``libudpdk_amd.so`` next to this file (C ABI in
``include/udpdk_gpu.h`` and ``include/udpdk_api.h``). This Python package is the test and
benchmark driver: ctypes bindings (:mod:`udpdk_amd.abi`), the synthetic frame generator of
SURVEY.md §8(d) (:mod:`udpdk_amd.frames`) and multi-GPU shard bookkeeping
(:mod:`udpdk_amd.shard`). There is no Python or CPU fallback for the datapath: if the library
is missing, :func:`udpdk_amd.abi.lib` raises.
"""

__all__ = ["abi", "frames", "shard"]
