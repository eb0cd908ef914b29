"""CPU: the C-ABI library loads and exports exactly what include/horreum_gpu.h
declares; struct layouts agree; no compute call is made (no GPU here)."""
import ctypes
import os

import numpy as np
import pytest

from horreum_amd import abi


def test_library_exports_every_header_symbol():
    lib = abi.load_library()
    names = abi.header_exports()
    assert len(names) >= 15
    for name in names:
        assert hasattr(lib, name), name
        assert name in abi._PROTOS, f"{name} has no ctypes prototype"


def test_abi_version_and_status_strings():
    lib = abi.load_library()
    assert lib.hg_abi_version() == 6
    for st in abi.Status:
        s = lib.hg_status_string(int(st)).decode()
        assert s and s != "unknown status", st
    assert lib.hg_block_count(16, 3) == 6  # src/sstable/index.rs:85-117: 6 blocks
    assert lib.hg_block_count(0, 3) == 0


def test_struct_layouts():
    assert abi.SPAN_DTYPE.itemsize == 16
    assert abi.PAIR_DTYPE.itemsize == 24
    assert abi.BLOCK_DTYPE.itemsize == 24
    assert abi.DECODE_RESULT_DTYPE.itemsize == 24
    assert abi.ENCODE_RESULT_DTYPE.itemsize == 16
    assert ctypes.sizeof(abi.HgErr) == 16
    from oracle import oracle
    assert oracle.SPAN_DTYPE == abi.SPAN_DTYPE and oracle.PAIR_DTYPE == abi.PAIR_DTYPE


def test_invalid_args_rejected_without_device():
    lib = abi.load_library()
    assert lib.hg_ctx_create(0, None) == abi.Status.INVALID_ARG
    assert lib.hg_ctx_destroy(None) == abi.Status.INVALID_ARG
    n = ctypes.c_uint64()
    assert lib.hg_decode_dev(None, None, 0, None, 0, ctypes.byref(n), None) == abi.Status.INVALID_ARG


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(abi.HorreumGpuError):
        abi._lib_backup = abi._lib
        try:
            abi._lib = None
            abi.load_library(str(tmp_path / "nope.so"))
        finally:
            abi._lib = abi._lib_backup


def test_engine_refuses_without_gpu():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from horreum_amd.engine import Engine
    with pytest.raises(abi.HorreumGpuError):
        Engine(0)


def test_knobs_set_get_clear():
    """hg_set_knob: the library's only run-time switches (no environment
    reads); unknown names are refused, value < 0 clears."""
    lib = abi.load_library()
    v = ctypes.c_int64()
    assert lib.hg_get_knob(b"HG_DECODE_BP", ctypes.byref(v)) == 0 and v.value == -1
    assert lib.hg_set_knob(b"HG_DECODE_BP", 64) == 0
    assert lib.hg_get_knob(b"HG_DECODE_BP", ctypes.byref(v)) == 0 and v.value == 64
    assert lib.hg_set_knob(b"HG_DECODE_BP", -1) == 0
    assert lib.hg_get_knob(b"HG_DECODE_BP", ctypes.byref(v)) == 0 and v.value == -1
    assert lib.hg_set_knob(b"HG_NO_SUCH_KNOB", 1) == abi.Status.INVALID_ARG
    assert lib.hg_set_knob(None, 1) == abi.Status.INVALID_ARG
    assert abi.knob_value("HG_MERGE_SERIAL", "exact") == 2
    assert abi.knob_value("HG_DECODE_BATCH", "streams") == 1


def test_library_reads_no_environment():
    """The release library's behaviour cannot be changed by a service's
    environment: no getenv / secure_getenv import in libhorreum_gpu.so."""
    import subprocess
    out = subprocess.run(["nm", "-D", "--undefined-only", abi.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    assert "getenv" not in out, [l for l in out.splitlines() if "getenv" in l]
