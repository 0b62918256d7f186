"""Minimal ctypes access to the HIP runtime that libq3t.so itself links (device buffers for the C-ABI drop-in tests,
without a second HIP runtime from a framework wheel in the same process)."""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "qwen3-tts-jetson_amd"))
import q3t  # noqa: E402,F401  (loads libq3t.so and with it libamdhip64.so.7)

_hip = C.CDLL("libamdhip64.so.7")
_hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
_hip.hipFree.argtypes = [C.c_void_p]
_hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
_hip.hipDeviceSynchronize.argtypes = []
_hip.hipGetDeviceCount.argtypes = [C.POINTER(C.c_int)]
H2D, D2H = 1, 2


def device_count():
    n = C.c_int(0)
    return n.value if _hip.hipGetDeviceCount(C.byref(n)) == 0 else 0


class DevBuf:
    """device copy of a numpy array (freed on close / garbage collection)"""

    def __init__(self, arr=None, nbytes=None):
        self.nbytes = int(arr.nbytes if arr is not None else nbytes)
        self.ptr = C.c_void_p()
        assert _hip.hipMalloc(C.byref(self.ptr), max(self.nbytes, 4)) == 0, "hipMalloc failed"
        if arr is not None:
            a = np.ascontiguousarray(arr)
            assert _hip.hipMemcpy(self.ptr, a.ctypes.data_as(C.c_void_p), self.nbytes, H2D) == 0

    @property
    def p(self):
        return self.ptr.value

    def get(self, dtype, count):
        out = np.empty(count, dtype)
        assert _hip.hipDeviceSynchronize() == 0
        assert _hip.hipMemcpy(out.ctypes.data_as(C.c_void_p), self.ptr, out.nbytes, D2H) == 0
        return out

    def close(self):
        if self.ptr:
            _hip.hipFree(self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def sync():
    assert _hip.hipDeviceSynchronize() == 0
