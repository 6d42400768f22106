"""ctypes binding of libeegfx.so (include/eegfx.h).

The library is built in-tree by ``__graft_entry__.build()`` (``make -C
eeg_dataanalysispackage_amd/csrc``).  There is no fallback: if the shared object is missing or
does not load, every entry point raises -- the product path never substitutes a CPU
implementation.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, Structure, c_char, c_char_p, c_double, c_float, c_int, c_int32,
                    c_int64, c_uint64, c_void_p)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libeegfx.so")

# ---- constants (eegfx.h) -----------------------------------------------------------------------
EEGFX_OK = 0
EEGFX_EINVAL = -1
EEGFX_EIO = -2
EEGFX_EFORMAT = -3
EEGFX_EHIP = -4
EEGFX_ENOMEM = -5
EEGFX_ERANGE = -6
EEGFX_ENOTSUP = -7
INT_16 = 0
IEEE_FLOAT_32 = 1
MEM_HOST = 0
MEM_DEVICE = 1
EXACT = 0
FMA = 1
PRESTIMULUS = 100
POSTSTIMULUS = 750

STATUS_NAMES = {
    EEGFX_EINVAL: "EINVAL", EEGFX_EIO: "EIO", EEGFX_EFORMAT: "EFORMAT", EEGFX_EHIP: "EHIP",
    EEGFX_ENOMEM: "ENOMEM", EEGFX_ERANGE: "ERANGE", EEGFX_ENOTSUP: "ENOTSUP",
}


class ChannelInfo(Structure):
    _fields_ = [("number", c_int32), ("name", c_char * 64), ("reference", c_char * 64),
                ("resolution", c_double), ("unit", c_char * 32)]


class HeaderInfo(Structure):
    _fields_ = [("n_channels", c_int32), ("binary_format", c_int32), ("multiplexed", c_int32),
                ("sampling_interval_us", c_double), ("data_file", c_char * 512),
                ("marker_file", c_char * 512)]


class Marker(Structure):
    _fields_ = [("number", c_int32), ("type", c_char * 64), ("description", c_char * 64),
                ("position", c_int64), ("size", c_int64), ("channel", c_int32),
                ("stimulus_index", c_int32)]


class GatherOp(Structure):
    _fields_ = [("kind", c_int32), ("peer", c_int32), ("row", c_int64), ("rows", c_int64)]


GATHER_SEND, GATHER_RECV, GATHER_COPY = 0, 1, 2


class EegfxError(RuntimeError):
    """A non-zero status of the C ABI (carries the code and eegfx_last_error())."""

    def __init__(self, code: int, message: str):
        super().__init__(f"[{STATUS_NAMES.get(code, code)}] {message}")
        self.code = code


# Exported symbols with their (restype, argtypes).  tests/test_library_abi.py checks this table
# against include/eegfx.h and the shared object's dynamic symbol table.
SIGNATURES = {
    "eegfx_version": (c_char_p, []),
    "eegfx_last_error": (c_char_p, []),
    "eegfx_device_count": (c_int, [POINTER(c_int)]),
    "eegfx_ctx_create": (c_int, [c_int, POINTER(c_void_p)]),
    "eegfx_ctx_set_stream": (c_int, [c_void_p, c_void_p]),
    "eegfx_ctx_stream": (c_int, [c_void_p, POINTER(c_void_p)]),
    "eegfx_ctx_set_numerics": (c_int, [c_void_p, c_int]),
    "eegfx_ctx_synchronize": (c_int, [c_void_p]),
    "eegfx_ctx_guard_stats": (c_int, [c_void_p, POINTER(c_int64), POINTER(c_int64), c_int]),
    "eegfx_ctx_guard_detail": (c_int, [c_void_p, POINTER(c_int64), POINTER(c_int64),
                                       POINTER(c_int64), c_int]),
    "eegfx_ctx_kernel_stats": (c_int, [c_void_p, POINTER(c_int64), POINTER(c_double),
                                       POINTER(c_int64)]),
    "eegfx_ctx_set_timing": (c_int, [c_void_p, c_int]),
    "eegfx_ctx_set_mailbox": (c_int, [c_void_p, c_int]),
    "eegfx_ctx_get_mailbox": (c_int, [c_void_p, POINTER(c_int32), POINTER(c_int32)]),
    "eegfx_ctx_destroy": (c_int, [c_void_p]),
    "eegfx_read_header": (c_int, [c_char_p, POINTER(HeaderInfo), POINTER(ChannelInfo), c_int32]),
    "eegfx_read_markers": (c_int, [c_char_p, POINTER(Marker), c_int64, POINTER(c_int64)]),
    "eegfx_recording_frames": (c_int, [c_char_p, c_char_p, POINTER(c_int64)]),
    "eegfx_read_raw": (c_int, [c_void_p, c_char_p, c_char_p, c_void_p, c_int64, c_int]),
    "eegfx_plan_markers": (c_int, [POINTER(Marker), c_int64, c_int64, c_int32, POINTER(c_int64),
                                   c_void_p, c_void_p, POINTER(c_int64)]),
    "eegfx_cut_epochs_f64": (c_int, [c_void_p, c_void_p, c_int32, c_int64, c_int32, c_void_p,
                                     c_void_p, c_int32, c_void_p, c_int64, c_void_p, c_int]),
    "eegfx_extract_features_f64": (c_int, [c_void_p, c_void_p, c_int64, c_int32, c_int32,
                                           c_int32, c_int32, c_int32, c_void_p, c_int]),
    "eegfx_process_recording": (c_int, [c_void_p, c_void_p, c_int32, c_int64, c_int32, c_void_p,
                                        c_void_p, c_int32, c_void_p, c_int64, c_void_p, c_int]),
    "eegfx_process_recording_epochs": (c_int, [c_void_p, c_void_p, c_int32, c_int64, c_int32,
                                               c_void_p, c_void_p, c_int32, c_void_p, c_int64,
                                               c_void_p, c_void_p, c_int]),
    "eegfx_synth_recording": (c_int, [c_void_p, c_void_p, c_int64, c_int32, c_uint64]),
    "eegfx_logreg_sgd_train": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32,
                                       c_double, c_double, c_double, c_double, c_void_p,
                                       POINTER(c_int32), c_int]),
    "eegfx_logreg_sgd_train_partitioned": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int32,
                                                   c_int32, c_double, c_double, c_double, c_double,
                                                   c_int32, c_void_p, POINTER(c_int32), c_int]),
    "eegfx_spark_sample": (c_int, [c_int64, c_double, c_int32, c_int64, c_void_p,
                                   POINTER(c_int64)]),
    "eegfx_logreg_predict": (c_int, [c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_double,
                                     c_double, c_void_p, c_int]),
    "eegfx_svm_sgd_train": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32,
                                    c_double, c_double, c_double, c_double, c_void_p,
                                    POINTER(c_int32), c_int]),
    "eegfx_svm_predict": (c_int, [c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_double,
                                  c_double, c_void_p, c_int]),
    "eegfx_plan_markers_device": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int32,
                                          POINTER(c_int64), c_void_p, c_void_p, POINTER(c_int64),
                                          c_int]),
    "eegfx_shard_range": (c_int, [c_int64, c_int32, c_int32, POINTER(c_int64), POINTER(c_int64)]),
    "eegfx_gather_schedule": (c_int, [c_int64, c_int32, c_void_p, c_void_p]),
    "eegfx_comm_unique_id": (c_int, [c_void_p]),
    "eegfx_comm_create": (c_int, [c_void_p, c_int32, c_int32, c_void_p, POINTER(c_void_p)]),
    "eegfx_comm_init_all": (c_int, [POINTER(c_void_p), c_int32, POINTER(c_void_p)]),
    "eegfx_comm_rank": (c_int, [c_void_p, POINTER(c_int32), POINTER(c_int32)]),
    "eegfx_gather": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_void_p]),
    "eegfx_gather_root": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int32, c_void_p]),
    "eegfx_gather_root_plan": (c_int, [c_int64, c_int32, c_int32, c_int32, POINTER(GatherOp),
                                       POINTER(c_int32)]),
    "eegfx_group_start": (c_int, []),
    "eegfx_group_end": (c_int, []),
    "eegfx_comm_destroy": (c_int, [c_void_p]),
    "eegfx_process_recording_streamed": (c_int, [c_void_p, c_void_p, c_int32, c_int64, c_int32,
                                                 c_void_p, c_void_p, c_int32, c_void_p, c_int64,
                                                 c_void_p, c_int64]),
    "eegfx_odp_create": (c_int, [c_void_p, POINTER(c_char_p), c_int32, POINTER(c_void_p)]),
    "eegfx_odp_load_data": (c_int, [c_void_p]),
    "eegfx_odp_error": (c_char_p, [c_void_p]),
    "eegfx_odp_num_epochs": (c_int64, [c_void_p]),
    "eegfx_odp_get_data": (c_int, [c_void_p, c_void_p]),
    "eegfx_odp_get_labels": (c_int, [c_void_p, c_void_p]),
    "eegfx_odp_get_positions": (c_int, [c_void_p, c_void_p, c_void_p]),
    "eegfx_odp_get_features": (c_int, [c_void_p, c_int32, c_int32, c_int32, c_int32, c_void_p]),
    "eegfx_odp_destroy": (None, [c_void_p]),
}

_lib = None


def lib() -> ctypes.CDLL:
    """Loads libeegfx.so once (raises if it is missing -- no fallback)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch wheels bundle their own libamdhip64.so.7 and
        # libhsa-runtime64.so.  Loading torch first makes libeegfx's libamdhip64.so.7 dependency
        # resolve (by SONAME) to that same runtime, so torch tensors and eegfx contexts share one
        # device context.  Without torch, the ROCm runtime under /opt/rocm is used.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run __graft_entry__.build() "
                              "(make -C eeg_dataanalysispackage_amd/csrc)")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


class EegfxRangeError(EegfxError, IndexError):
    """ERANGE: a marker position the reference would not cut (OffLineDataProvider.java:220-225,
    copyOfRange's ArrayIndexOutOfBoundsException) -- an IndexError that keeps the status code."""


def check(rc: int) -> None:
    if rc != EEGFX_OK:
        msg = lib().eegfx_last_error().decode(errors="replace")
        raise (EegfxRangeError if rc == EEGFX_ERANGE else EegfxError)(rc, msg)


def ptr(a) -> c_void_p:
    """Address of a numpy array (host) or torch tensor (device) as a void*."""
    if a is None:
        return c_void_p(0)
    if hasattr(a, "data_ptr"):
        return c_void_p(a.data_ptr())
    return c_void_p(a.ctypes.data)
