"""Device ops: hand-written HIP kernels for gfx950 plus torch CPU references.

Every op dispatches on the tensor's device: CUDA(HIP) tensors run the kernels
in ``lazzaro_amd/_lib/liblzk.so`` (raising if the library is missing), CPU
tensors run the fp32 torch reference of the same op (the CPU test tier).
"""
from . import _lib  # noqa: F401
from .search import flat_topk  # noqa: F401
