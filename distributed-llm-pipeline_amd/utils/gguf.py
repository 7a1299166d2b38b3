"""GGUF v3 writer and (pure-python) reader.

The reference loads `baronllm-llama3.1-v1-q6_k.gguf` through llama.cpp
(`orchestrator/src/main.rs:39-40`); the format is reconstructed in SURVEY.md §2.8.
The production reader is the native C++ one (`csrc/runtime/gguf.cpp`, mmap, zero copy);
this module is the writer used by the synthetic-model generator and a python reader used
as a cross-check oracle in tests.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Any

import numpy as np

from . import quants as Q

GGUF_MAGIC = 0x46554747
GGUF_VERSION = 3

# value types
U8, I8, U16, I16, U32, I32, F32T, BOOL, STRING, ARRAY, U64, I64, F64 = range(13)
_FMT = {U8: "<B", I8: "<b", U16: "<H", I16: "<h", U32: "<I", I32: "<i", F32T: "<f",
        BOOL: "<?", U64: "<Q", I64: "<q", F64: "<d"}


def _wstr(b: bytearray, s: str | bytes):
    if isinstance(s, str):
        s = s.encode("utf-8")
    b += struct.pack("<Q", len(s))
    b += s


def _infer_vtype(v: Any) -> int:
    if isinstance(v, bool):
        return BOOL
    if isinstance(v, int):
        return I32 if -2**31 <= v < 2**31 else I64
    if isinstance(v, float):
        return F32T
    if isinstance(v, (str, bytes)):
        return STRING
    if isinstance(v, (list, tuple, np.ndarray)):
        return ARRAY
    raise TypeError(type(v))


@dataclass
class _Tensor:
    name: str
    shape: tuple            # ggml order: ne[0] innermost
    qtype: int
    data: Any               # bytes-like or callable returning bytes (lazy)
    nbytes: int


@dataclass
class GGUFWriter:
    path: str
    alignment: int = 32
    kv: list = field(default_factory=list)
    tensors: list = field(default_factory=list)

    def add(self, key: str, value: Any, vtype: int | None = None, elem_type: int | None = None):
        self.kv.append((key, value, vtype if vtype is not None else _infer_vtype(value), elem_type))

    def add_tensor(self, name: str, data, qtype: int, shape_ggml: tuple, nbytes: int | None = None):
        """shape_ggml: (ne0, ne1, ...) with ne0 contiguous. data: bytes/ndarray or a callable."""
        if nbytes is None:
            nbytes = Q.tensor_bytes(qtype, shape_ggml)
        if not callable(data):
            arr = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
            assert arr.nbytes == nbytes, (name, arr.nbytes, nbytes)
            data = arr
        self.tensors.append(_Tensor(name, tuple(int(s) for s in shape_ggml), qtype, data, nbytes))

    def _kv_bytes(self) -> bytearray:
        b = bytearray()
        for key, v, vt, et in self.kv:
            _wstr(b, key)
            b += struct.pack("<I", vt)
            if vt == STRING:
                _wstr(b, v)
            elif vt == ARRAY:
                items = list(v)
                if et is None:
                    et = _infer_vtype(items[0]) if items else I32
                b += struct.pack("<IQ", et, len(items))
                if et == STRING:
                    for s in items:
                        _wstr(b, s)
                else:
                    arr = np.asarray(items, dtype=np.dtype(_FMT[et][1:]).newbyteorder("<"))
                    b += arr.tobytes()
            else:
                b += struct.pack(_FMT[vt], v)
        return b

    def write(self):
        if not any(k == "general.alignment" for k, *_ in self.kv):
            self.add("general.alignment", self.alignment, U32)
        hdr = bytearray()
        hdr += struct.pack("<IIQQ", GGUF_MAGIC, GGUF_VERSION, len(self.tensors), len(self.kv))
        hdr += self._kv_bytes()
        offset = 0
        offsets = []
        for t in self.tensors:
            offsets.append(offset)
            offset += (t.nbytes + self.alignment - 1) // self.alignment * self.alignment
        for t, off in zip(self.tensors, offsets):
            _wstr(hdr, t.name)
            hdr += struct.pack("<I", len(t.shape))
            hdr += struct.pack("<%dQ" % len(t.shape), *t.shape)
            hdr += struct.pack("<IQ", t.qtype, off)
        pad = (-len(hdr)) % self.alignment
        hdr += b"\0" * pad
        with open(self.path, "wb") as f:
            f.write(hdr)
            for t in self.tensors:
                data = t.data() if callable(t.data) else t.data
                data = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
                assert data.nbytes == t.nbytes, (t.name, data.nbytes, t.nbytes)
                f.write(data.tobytes())
                f.write(b"\0" * ((-t.nbytes) % self.alignment))


@dataclass
class GGUFTensorInfo:
    name: str
    shape: tuple
    qtype: int
    offset: int
    nbytes: int


class GGUFReader:
    """Pure-python GGUF v2/v3 reader (np.memmap), used as a test oracle."""

    def __init__(self, path: str):
        self.path = path
        self.mm = np.memmap(path, dtype=np.uint8, mode="r")
        self.pos = 0
        magic, ver = struct.unpack_from("<II", self.mm, 0)
        if magic != GGUF_MAGIC:
            raise ValueError("not a GGUF file")
        self.version = ver
        self.pos = 8
        n_t, n_kv = self._u("<QQ")
        self.kv: dict[str, Any] = {}
        for _ in range(n_kv):
            k = self._str()
            (vt,) = self._u("<I")
            self.kv[k] = self._val(vt)
        self.alignment = int(self.kv.get("general.alignment", 32))
        infos = []
        for _ in range(n_t):
            name = self._str()
            (nd,) = self._u("<I")
            shape = self._u("<%dQ" % nd)
            qt, off = self._u("<IQ")
            infos.append((name, tuple(shape), qt, off))
        data_start = (self.pos + self.alignment - 1) // self.alignment * self.alignment
        self.data_start = data_start
        self.tensors: dict[str, GGUFTensorInfo] = {}
        for name, shape, qt, off in infos:
            nb = Q.tensor_bytes(qt, shape) if qt in Q.BLOCK else 0
            self.tensors[name] = GGUFTensorInfo(name, shape, qt, data_start + off, nb)

    def _u(self, fmt):
        v = struct.unpack_from(fmt, self.mm, self.pos)
        self.pos += struct.calcsize(fmt)
        return v

    def _str(self):
        (n,) = self._u("<Q")
        s = bytes(self.mm[self.pos:self.pos + n]).decode("utf-8", errors="replace")
        self.pos += n
        return s

    def _val(self, vt):
        if vt == STRING:
            return self._str()
        if vt == ARRAY:
            et, n = self._u("<IQ")
            if et == STRING:
                return [self._str() for _ in range(n)]
            dt = np.dtype(_FMT[et][1:]).newbyteorder("<")
            arr = np.frombuffer(self.mm, dtype=dt, count=n, offset=self.pos).copy()
            self.pos += n * dt.itemsize
            return arr
        (v,) = self._u(_FMT[vt])
        return v

    def raw(self, name: str) -> np.ndarray:
        t = self.tensors[name]
        return np.asarray(self.mm[t.offset:t.offset + t.nbytes])

    def tensor_f32(self, name: str) -> np.ndarray:
        """Dequantized tensor in numpy row-major order (reversed ggml shape)."""
        t = self.tensors[name]
        y = Q.dequantize(self.raw(name), t.qtype)
        return y.reshape(tuple(reversed(t.shape)))
