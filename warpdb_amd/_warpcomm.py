"""ctypes binding of include/warpcomm.h (libwarpdb.so): one RCCL communicator
per rank whose collectives run on the query's own stream.

The exchange step of a row-sharded query (the reference
gathers every shard's dense result on the host, src/multi_gpu_utils.cpp:23-60)
is one collective between a partials kernel and a merge kernel.  Through
torch.distributed that collective runs on the process group's internal
stream, fenced by two cross-stream event waits; here it is enqueued on the
stream the kernels use, so stream order is the only synchronisation.
"""
from __future__ import annotations

import ctypes
import os

from . import _warpexec as wx

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libwarpdb.so")
ID_BYTES = 128
SUM, MAX, MIN = 0, 1, 2

_lib = None


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FileNotFoundError(f"{LIB_PATH} is missing: build it with `make -C warpdb_amd`")
    wx.load()  # libwarpexec first (libwarpdb links it)
    lib = ctypes.CDLL(LIB_PATH)
    P, I32, I64, E, S = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_char_p, ctypes.c_size_t
    sig = {
        "wx_comm_unique_id": [P, E, S],
        "wx_comm_init": [P, I32, I32, I32, ctypes.POINTER(ctypes.c_void_p), E, S],
        "wx_comm_all_reduce": [P, P, P, I64, I32, I32, P, E, S],
        "wx_comm_all_gather": [P, P, P, I64, P, E, S],
        "wx_comm_destroy": [P, E, S],
    }
    for name, argtypes in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = ctypes.c_int
    for name in ("wx_comm_rank", "wx_comm_size"):
        getattr(lib, name).argtypes = [P]
        getattr(lib, name).restype = ctypes.c_int32
    _lib = lib
    return lib


EXPORTED_SYMBOLS = ("wx_comm_unique_id", "wx_comm_init", "wx_comm_all_reduce", "wx_comm_all_gather",
                    "wx_comm_rank", "wx_comm_size", "wx_comm_destroy")


def unique_id() -> bytes:
    lib = load()
    buf = ctypes.create_string_buffer(ID_BYTES)
    err = ctypes.create_string_buffer(1024)
    wx._check(lib.wx_comm_unique_id(buf, err, len(err)), err)
    return buf.raw


class Comm:
    """This rank's communicator (collective construction: every rank calls
    it with the id rank 0 made)."""

    def __init__(self, comm_id: bytes, n_ranks: int, rank: int, device: int):
        if len(comm_id) != ID_BYTES:
            raise ValueError("a communicator id is 128 bytes")
        self._lib = load()
        self._h = ctypes.c_void_p()
        self._id = ctypes.create_string_buffer(comm_id, ID_BYTES)
        err = ctypes.create_string_buffer(1024)
        wx._check(self._lib.wx_comm_init(self._id, n_ranks, rank, device, ctypes.byref(self._h), err, len(err)),
                  err)
        self.n_ranks, self.rank, self.device = n_ranks, rank, device

    def all_reduce(self, src: int, dst: int, count: int, dtype: int, op: int, stream: int) -> None:
        err = ctypes.create_string_buffer(1024)
        wx._check(self._lib.wx_comm_all_reduce(self._h, src, dst, count, dtype, op, stream or None, err, len(err)),
                  err)

    def all_gather(self, src: int, dst: int, nbytes: int, stream: int) -> None:
        err = ctypes.create_string_buffer(1024)
        wx._check(self._lib.wx_comm_all_gather(self._h, src, dst, nbytes, stream or None, err, len(err)), err)

    def close(self) -> None:
        if self._h:
            err = ctypes.create_string_buffer(1024)
            st = self._lib.wx_comm_destroy(self._h, err, len(err))
            self._h = ctypes.c_void_p()
            wx._check(st, err)
