"""Probe: wrap a raw HIP allocation (rocfm p2p_malloc) as a torch tensor via __cuda_array_interface__."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rocfm.ops import hip  # noqa: E402

H = hip()
torch.cuda.set_device(0)
ptr = H.p2p_malloc(4096 * 4, 0)


class _Raw:
    def __init__(self, p, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (p, False), "version": 3,
                                         "strides": None}


t = torch.as_tensor(_Raw(ptr, 4096), device="cuda")
print("wrapped", t.device, t.dtype, t.shape, hex(t.data_ptr()), hex(ptr))
t.fill_(3.0)
t[10] = 7.0
print("sum", float(t.sum()), "ok" if t.data_ptr() == ptr and float(t.sum()) == 3.0 * 4095 + 7.0 else "MISMATCH")
