"""newsched_amd -- MI355X-native block-execution path for the newsched GNU Radio runtime.

Product code: HIP kernels + C-ABI (csrc/ -> lib/libnsh_hip.so, include/nsh_hip.h) and the
C++17 host runtime restating newsched's block/buffer/scheduler API (runtime/, schedulers/,
blocklib/ -> lib/libnewsched.so). `nsh` and `nsr` are the ctypes views of the two
libraries. There is no CPU fallback: importing a binding whose library is missing raises.
"""
from . import nsh  # noqa: F401

__all__ = ["nsh", "nsr"]
