"""ctypes binding of include/horreum_gpu.h (libhorreum_gpu.so).

Loading is strict: there is no CPU fallback anywhere in the product path.  If
the shared library is missing or cannot be loaded, importing the engine raises
HorreumGpuError with the build command.
"""
import ctypes
import enum
import os
import re

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HG_LIBRARY") or os.path.join(PKG_DIR, "libhorreum_gpu.so")
HEADER_PATH = os.path.join(os.path.dirname(PKG_DIR), "include", "horreum_gpu.h")


class HorreumGpuError(RuntimeError):
    """A C-ABI call failed (status code + message)."""

    def __init__(self, status, msg=""):
        self.status = int(status)
        text = f"{status_string(self.status)} ({self.status})"
        if self.status == Status.HIP:
            site = last_hip_error()
            if site:
                text += f" at {site}"
        super().__init__(f"{msg}: {text}" if msg else text)


class Status(enum.IntEnum):
    OK = 0
    TRUNCATED_HEADER = 1
    TRUNCATED_BODY = 2
    LEN_OVERFLOW = 3
    SPAN_RANGE = 4
    CAPACITY = 5
    INVALID_ARG = -1
    HIP = -2
    TOO_LARGE = -3
    INTERNAL = -4
    EMPTY_MERGE = -5
    UNSORTED = -6


# ---- struct layouts (must match include/horreum_gpu.h) -------------------------
SPAN_DTYPE = np.dtype([("off", "<u8"), ("klen", "<u4"), ("vlen", "<u4")])
PAIR_DTYPE = np.dtype([("key_off", "<u8"), ("val_off", "<u8"), ("klen", "<u4"), ("vlen", "<u4")])
BLOCK_DTYPE = np.dtype([("first_rec", "<u8"), ("position", "<u8"), ("length", "<u8")])
DECODE_RESULT_DTYPE = np.dtype([("n_records", "<u8"), ("kind", "<i4"), ("reserved", "<u4"),
                                ("err_offset", "<u8")])
ENCODE_RESULT_DTYPE = np.dtype([("out_len", "<u8"), ("kind", "<i4"), ("reserved", "<u4")])
KEY_DTYPE = np.dtype([("off", "<u8"), ("len", "<u4"), ("reserved", "<u4")])
LOOKUP_DTYPE = np.dtype([("rec", "<u8"), ("val_off", "<u8"), ("vlen", "<u4"), ("found", "<i4")])
MERGE_RESULT_DTYPE = np.dtype([("n_out", "<u8"), ("kind", "<i4"), ("table", "<u4"),
                               ("index", "<u8")])


class HgErr(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("reserved", ctypes.c_uint32),
                ("offset", ctypes.c_uint64)]


class HgMergeResult(ctypes.Structure):
    _fields_ = [("n_out", ctypes.c_uint64), ("kind", ctypes.c_int32),
                ("table", ctypes.c_uint32), ("index", ctypes.c_uint64)]


def header_exports(path=HEADER_PATH):
    """Function names declared in include/horreum_gpu.h."""
    text = open(path, encoding="utf-8").read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(hg_[a-z_0-9]+)\s*\(", text)))


_u8p = ctypes.c_void_p
_vp = ctypes.c_void_p
_u64 = ctypes.c_uint64
_u32 = ctypes.c_uint32
_PROTOS = {
    "hg_abi_version": (ctypes.c_int, []),
    "hg_set_knob": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int64]),
    "hg_get_knob": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64)]),
    "hg_status_string": (ctypes.c_char_p, [ctypes.c_int]),
    "hg_last_hip_error": (ctypes.c_char_p, []),
    "hg_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    "hg_ctx_destroy": (ctypes.c_int, [_vp]),
    "hg_ctx_set_stream": (ctypes.c_int, [_vp, _vp]),
    "hg_ctx_trim": (ctypes.c_int, [_vp]),
    "hg_ctx_use_own_stream": (ctypes.c_int, [_vp]),
    "hg_ctx_stream": (_vp, [_vp]),
    "hg_ctx_synchronize": (ctypes.c_int, [_vp]),
    "hg_ctx_reserve": (ctypes.c_int, [_vp, _u64, _u64]),
    "hg_decode_dev": (ctypes.c_int, [_vp, _u8p, _u64, _vp, _u64, ctypes.POINTER(_u64),
                                     ctypes.POINTER(HgErr)]),
    "hg_decode_dev_async": (ctypes.c_int, [_vp, _u8p, _u64, _vp, _u64, _vp]),
    "hg_decode_host": (ctypes.c_int, [_vp, _u8p, _u64, _vp, _u64, ctypes.POINTER(_u64),
                                      ctypes.POINTER(HgErr)]),
    "hg_encode_dev": (ctypes.c_int, [_vp, _u8p, _vp, _u64, _u8p, _u64, _vp, _u32, _vp,
                                     ctypes.POINTER(_u64)]),
    "hg_encode_dev_async": (ctypes.c_int, [_vp, _u8p, _vp, _u64, _u8p, _u64, _vp, _u32, _vp,
                                           _vp]),
    "hg_encode_host": (ctypes.c_int, [_vp, _u8p, _u64, _vp, _u64, _u8p, _u64, _vp, _u32, _vp,
                                      ctypes.POINTER(_u64)]),
    "hg_block_count": (_u64, [_u64, _u32]),
    "hg_keyindex_bytes": (_u64, [_u64]),
    "hg_keyindex_build_dev_async": (ctypes.c_int, [_vp, _u8p, _u64, _vp, _u64, _vp]),
    "hg_lookup_dev_async": (ctypes.c_int, [_vp, _u8p, _vp, _vp, _u64, ctypes.c_uint32, _u8p, _vp, _u64, _vp]),
    "hg_lookup_host": (ctypes.c_int, [_vp, _u8p, _u64, ctypes.c_uint32, _u8p, _u64, _vp, _u64, _vp]),
    # batch decode(ctx, n, tables**, lens*, spans**, caps*, results)
    "hg_decode_batch_dev_async": (ctypes.c_int, [_vp, _u32, _vp, _vp, _vp, _vp, _vp]),
    # merge(ctx, ntables, arena, arena_len, table_off*, spans**, counts*, out, cap, result)
    "hg_merge_dev": (ctypes.c_int, [_vp, _u32, _u8p, _u64, _vp, _vp, _vp, _vp, _u64,
                                    ctypes.POINTER(HgMergeResult)]),
    "hg_merge_dev_async": (ctypes.c_int, [_vp, _u32, _u8p, _u64, _vp, _vp, _vp, _vp, _u64, _vp]),
    # compact(ctx, ntables, tables**, lens*, out, cap, out_len*, stride, blocks, result*)
    "hg_host_register": (ctypes.c_int, [_vp, _u64]),
    "hg_host_unregister": (ctypes.c_int, [_vp]),
    "hg_host_is_pinned": (ctypes.c_int, [_vp]),
    "hg_compact_host": (ctypes.c_int, [_vp, _u32, _vp, _vp, _u8p, _u64, ctypes.POINTER(_u64),
                                       _u32, _vp, ctypes.POINTER(HgMergeResult)]),
    # compact_dev(ctx, ntables, arena, arena_len, table_off*, lens*, out, cap, out_len*, stride,
    #             blocks, result*)
    "hg_compact_dev": (ctypes.c_int, [_vp, _u32, _u8p, _u64, _vp, _vp, _u8p, _u64,
                                      ctypes.POINTER(_u64), _u32, _vp,
                                      ctypes.POINTER(HgMergeResult)]),
    # range decode(ctx, sst, len, begin, stop, entry, spans, cap, [n*, exit*, err* | result])
    "hg_decode_range_dev_async": (ctypes.c_int, [_vp, _u8p, _u64, _u64, _u64, _u64, _vp, _u64,
                                                 _vp]),
    "hg_decode_range_dev": (ctypes.c_int, [_vp, _u8p, _u64, _u64, _u64, _u64, _vp, _u64,
                                           ctypes.POINTER(_u64), ctypes.POINTER(_u64),
                                           ctypes.POINTER(HgErr)]),
    "hg_decode_guess_entry_dev": (ctypes.c_int, [_vp, _u8p, _u64, _u64, ctypes.POINTER(_u64)]),
    "hg_encoded_size": (ctypes.c_int, [_vp, _vp, _u64, ctypes.POINTER(_u64)]),
    # multi(ctxs**, nctx, ...)
    "hg_multi_decode_host": (ctypes.c_int, [_vp, _u32, _u32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "hg_multi_decode_file_host": (ctypes.c_int, [_vp, _u32, _u8p, _u64, _vp, _u64,
                                                 ctypes.POINTER(_u64), ctypes.POINTER(HgErr)]),
    "hg_multi_compact_host": (ctypes.c_int, [_vp, _u32, _u32, _vp, _vp, _u8p, _u64,
                                             ctypes.POINTER(_u64), _u32, _vp,
                                             ctypes.POINTER(HgMergeResult)]),
    "hg_multi_compact_dev": (ctypes.c_int, [_vp, _u32, _u32, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                            ctypes.POINTER(HgMergeResult)]),
}

_lib = None


def load_library(path=LIB_PATH):
    """Load libhorreum_gpu.so once; raise HorreumGpuError if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise HorreumGpuError(Status.HIP, f"{path} not built (run: make -C horreum_amd/csrc)")
    # One HIP runtime per process: torch bundles libamdhip64.so.7 and our
    # library needs the same SONAME.  Loading torch first makes the dynamic
    # linker reuse its copy, so device pointers and streams are shared.
    try:
        import torch  # noqa: F401
    except ImportError:  # pragma: no cover - standalone C users
        pass
    try:
        lib = ctypes.CDLL(path)
    except OSError as e:  # pragma: no cover - environment specific
        raise HorreumGpuError(Status.HIP, f"cannot load {path}: {e}") from e
    for name, (res, args) in _PROTOS.items():
        fn = getattr(lib, name, None)
        if fn is None:  # an older experimental build (A/B tools); tests/test_abi.py checks exports
            continue
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


# Knobs (hg_set_knob): the library reads no environment variables.  Values
# are integers; the words the A/B scripts used to put in the environment
# are mapped here.
KNOB_WORDS = {"HG_DECODE_BATCH": {"streams": 1}, "HG_MERGE_SERIAL": {"exact": 2},
              "HG_COMPACT_ENCODE": {"pairs": 1}}


def knob_value(name, value):
    if isinstance(value, str):
        words = KNOB_WORDS.get(name, {})
        if value in words:
            return words[value]
        if name == "HG_MERGE_SERIAL":  # any other word: the reference loop
            return 1
        return int(value)
    return int(value)


def set_knob(name, value):
    """Set library knob `name` (value < 0 clears it; see hg_set_knob)."""
    lib = load_library()
    if not hasattr(lib, "hg_set_knob"):  # an older experimental build reads the environment
        if int(knob_value(name, value)) < 0:
            os.environ.pop(name, None)
        else:
            os.environ[name] = str(value)
        return
    rc = lib.hg_set_knob(name.encode(), knob_value(name, value))
    if rc != 0:
        raise HorreumGpuError(rc, f"hg_set_knob({name})")


def knobs_from_env(environ=None):
    """Tools only (A/B scripts): forward HG_* knob variables of the
    environment to the library.  The product never calls this."""
    environ = os.environ if environ is None else environ
    lib = load_library()
    if not hasattr(lib, "hg_set_knob"):
        return []
    done = []
    for name, value in environ.items():
        if not name.startswith("HG_"):
            continue
        try:
            v = knob_value(name, value)
        except ValueError:  # not a knob (HG_LIBRARY, HG_BENCH_*, ...)
            continue
        if lib.hg_set_knob(name.encode(), v) == 0:
            done.append(name)
    return done


def status_string(status):
    # (the loaded library's text; never loads it here: a HorreumGpuError
    # raised by load_library itself formats its status through this)
    if _lib is not None:
        return _lib.hg_status_string(int(status)).decode()
    return Status(status).name if status in Status._value2member_map_ else "unknown"


def last_hip_error():
    """Where the most recent HG_ERR_HIP came from (hg_last_hip_error)."""
    global _lib
    if _lib is None:
        return ""
    return _lib.hg_last_hip_error().decode()


def check(status, what=""):
    if status != 0:
        raise HorreumGpuError(status, what)
    return status
