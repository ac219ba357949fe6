"""Arrow exports of query results: the reference's host
query_arrow (src/arrow_utils.cpp:37-94, bindings/python/pywarpdb.cpp:18-37)
plus zero-copy ArrowDeviceArrays in HBM (device_type ARROW_DEVICE_ROCM,
include/arrow_c_abi.h:126,140-155 of the reference) and the compacted
struct<value: float32, row: int64> result.  Device buffers are read back with
hipMemcpy and compared bit for bit with the oracle; releasing the capsule
must return the HBM.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

import oracle_lib as ora
import synth

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
TEST_CSV = os.path.join(HERE, "golden", "test.csv")
ARROW_DEVICE_ROCM = 10


class ArrowArray(ctypes.Structure):
    pass


ArrowArray._fields_ = [("length", ctypes.c_int64), ("null_count", ctypes.c_int64), ("offset", ctypes.c_int64),
                       ("n_buffers", ctypes.c_int64), ("n_children", ctypes.c_int64),
                       ("buffers", ctypes.POINTER(ctypes.c_void_p)),
                       ("children", ctypes.POINTER(ctypes.POINTER(ArrowArray))),
                       ("dictionary", ctypes.POINTER(ArrowArray)), ("release", ctypes.c_void_p),
                       ("private_data", ctypes.c_void_p)]


class ArrowSchema(ctypes.Structure):
    pass


ArrowSchema._fields_ = [("format", ctypes.c_char_p), ("name", ctypes.c_char_p), ("metadata", ctypes.c_char_p),
                        ("flags", ctypes.c_int64), ("n_children", ctypes.c_int64),
                        ("children", ctypes.POINTER(ctypes.POINTER(ArrowSchema))),
                        ("dictionary", ctypes.POINTER(ArrowSchema)), ("release", ctypes.c_void_p),
                        ("private_data", ctypes.c_void_p)]


class ArrowDeviceArray(ctypes.Structure):
    _fields_ = [("array", ArrowArray), ("device_id", ctypes.c_int64), ("device_type", ctypes.c_int32),
                ("sync_event", ctypes.c_void_p), ("reserved", ctypes.c_int64 * 3)]


def _ptr(cap, name):
    get = ctypes.pythonapi.PyCapsule_GetPointer
    get.restype = ctypes.c_void_p
    get.argtypes = [ctypes.py_object, ctypes.c_char_p]
    return get(cap, name)


def _hip():
    lib = ctypes.CDLL("libamdhip64.so")
    lib.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    lib.hipMemcpy.restype = ctypes.c_int
    return lib


def d2h(ptr, n, dtype):
    out = np.empty(n, dtype)
    if n:
        assert _hip().hipMemcpy(out.ctypes.data, ptr, out.nbytes, 2) == 0  # hipMemcpyDeviceToHost
    return out


def write_csv(path, cols):
    with open(path, "w") as f:
        f.write(",".join(cols) + "\n")
        for row in zip(*cols.values()):
            f.write(",".join("%.9g" % float(x) for x in row) + "\n")


@pytest.fixture(scope="module")
def big_db(tmp_path_factory):
    from warpdb_amd import pywarpdb as pw

    n = 2_000_003
    cols = synth.c2_table(n)
    path = str(tmp_path_factory.mktemp("arrow") / "arrow_big.csv")
    write_csv(path, cols)
    return pw.WarpDB(path), cols


def test_device_dense_export_zero_copy():
    from warpdb_amd import pywarpdb as pw

    db = pw.WarpDB(TEST_CSV)
    arr_cap, sch_cap = db.query_arrow_device("price * quantity WHERE price > 10")
    a = ArrowDeviceArray.from_address(_ptr(arr_cap, b"arrow_device_array"))
    s = ArrowSchema.from_address(_ptr(sch_cap, b"arrow_schema"))
    assert a.device_type == ARROW_DEVICE_ROCM and a.device_id == 0
    assert s.format == b"f" and a.array.length == 4 and a.array.n_buffers == 2 and not a.array.buffers[0]
    v = d2h(a.array.buffers[1], 4, np.float32)
    assert v.tolist() == [31.5, 80.0, 30.5, 150.0]


def test_device_dense_matches_oracle_and_release_frees_hbm(big_db):
    db, cols = big_db
    n = len(cols["price"])
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info()
    arr_cap, sch_cap = db.query_arrow_device("price * quantity WHERE price > 15")
    a = ArrowDeviceArray.from_address(_ptr(arr_cap, b"arrow_device_array"))
    assert a.device_type == ARROW_DEVICE_ROCM and a.array.length == n
    v = d2h(a.array.buffers[1], n, np.float32)
    fill = np.zeros(n, np.float32)
    expect = ora.dense(ora.HostTable(cols), "price * quantity", "price > 15", fill)
    assert np.array_equal(v.view(np.uint32), expect.view(np.uint32))
    free1, _ = torch.cuda.mem_get_info()
    del arr_cap, sch_cap, a
    free2, _ = torch.cuda.mem_get_info()
    assert free2 - free1 >= 4 * n - (2 << 20), (free0, free1, free2)


def test_host_compact_export_roundtrip_pyarrow():
    pa = pytest.importorskip("pyarrow")
    from warpdb_amd import pywarpdb as pw

    db = pw.WarpDB(TEST_CSV)
    arr_cap, sch_cap = db.query_arrow_compact("price * quantity WHERE price > 15")
    a = pa.Array._import_from_c(_ptr(arr_cap, None), _ptr(sch_cap, None))
    assert a.type == pa.struct([pa.field("value", pa.float32(), nullable=False),
                                pa.field("row", pa.int64(), nullable=False)])
    assert a.to_pylist() == [{"value": 80.0, "row": 1}, {"value": 30.5, "row": 2}, {"value": 150.0, "row": 3}]


def test_device_compact_export_matches_oracle(big_db):
    db, cols = big_db
    arr_cap, sch_cap = db.query_arrow_device_compact("price * quantity WHERE price > 15")
    a = ArrowDeviceArray.from_address(_ptr(arr_cap, b"arrow_device_array"))
    s = ArrowSchema.from_address(_ptr(sch_cap, b"arrow_schema"))
    assert a.device_type == ARROW_DEVICE_ROCM and s.format == b"+s" and s.n_children == 2
    assert s.children[0].contents.format == b"f" and s.children[0].contents.name == b"value"
    assert s.children[1].contents.format == b"l" and s.children[1].contents.name == b"row"
    rv, ri = ora.project_filter(ora.HostTable(cols), "price * quantity", "price > 15")
    m = a.array.length
    assert m == len(ri) and a.array.n_children == 2
    vals = d2h(a.array.children[0].contents.buffers[1], m, np.float32)
    rows = d2h(a.array.children[1].contents.buffers[1], m, np.int64)
    assert np.array_equal(rows, ri) and np.array_equal(vals.view(np.uint32), rv.view(np.uint32))
