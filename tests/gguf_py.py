"""Minimal numpy GGUF (v2/v3) reader for test tooling (memory-mapped, F32/F16 tensors only)."""
import struct

import numpy as np

_SCALAR = {0: "<B", 1: "<b", 2: "<H", 3: "<h", 4: "<I", 5: "<i", 6: "<f", 7: "<?", 10: "<Q", 11: "<q", 12: "<d"}


class GGUF:
    def __init__(self, path):
        self.path = path
        self.mm = np.memmap(path, dtype=np.uint8, mode="r")
        buf = self.mm
        self._p = 0
        assert bytes(buf[:4]) == b"GGUF", "bad magic"
        self._p = 4
        self.version = self._u32()
        nt = self._u64()
        nkv = self._u64()
        self.kv = {}
        for _ in range(nkv):
            k = self._str()
            t = self._u32()
            self.kv[k] = self._val(t)
        self.tensors = {}
        order = []
        for _ in range(nt):
            name = self._str()
            nd = self._u32()
            ne = [self._u64() for _ in range(nd)]
            typ = self._u32()
            off = self._u64()
            self.tensors[name] = (ne, typ, off)
            order.append(name)
        self.order = order
        align = int(self.kv.get("general.alignment", 32))
        self.data_off = (self._p + align - 1) // align * align

    def _rd(self, fmt):
        n = struct.calcsize(fmt)
        v = struct.unpack(fmt, bytes(self.mm[self._p:self._p + n]))[0]
        self._p += n
        return v

    def _u32(self):
        return self._rd("<I")

    def _u64(self):
        return self._rd("<Q")

    def _str(self):
        n = self._u64()
        s = bytes(self.mm[self._p:self._p + n]).decode("utf-8")
        self._p += n
        return s

    def _val(self, t):
        if t == 8:
            return self._str()
        if t == 9:
            et = self._u32()
            n = self._u64()
            return [self._val(et) for _ in range(n)]
        return self._rd(_SCALAR[t])

    def tensor(self, name):
        """numpy array in PyTorch (row-major, reversed ne) order."""
        ne, typ, off = self.tensors[name]
        dt = {0: np.float32, 1: np.float16}[typ]
        n = int(np.prod(ne))
        start = self.data_off + off
        a = np.frombuffer(self.mm, dtype=dt, count=n, offset=start)
        return a.reshape(list(reversed(ne)))
