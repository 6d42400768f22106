"""Device context and the compute entry points of libeegfx (include/eegfx.h).

Arrays may be numpy arrays (host memory: the library stages them through HBM and returns after
the results are copied back) or torch tensors on a ROCm device (device memory: the work is
enqueued on the context stream and the call returns without synchronising).
"""
from __future__ import annotations

import ctypes
from ctypes import c_int, c_int64, c_void_p
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import check, lib, ptr


def _is_device(a) -> bool:
    return hasattr(a, "is_cuda") and a.is_cuda


def _mem(*arrays) -> int:
    kinds = {_is_device(a) for a in arrays if a is not None}
    if len(kinds) != 1:
        raise ValueError("all buffers of one call must live in the same memory (host or device)")
    return _lib.MEM_DEVICE if kinds.pop() else _lib.MEM_HOST


def _contig(a, dtype):
    if _is_device(a):
        if not a.is_contiguous():
            raise ValueError("device tensors must be contiguous")
        return a
    return np.ascontiguousarray(a, dtype=dtype)


class Context:
    """One HIP device + stream (eegfx_ctx).  numerics: "exact" (bit-exact to the reference
    order of operations, default), "fma" (fused multiply-add filter bank, <= 1e-9 relative) or
    "mfma" (the window as one 16x512 fp64 operator on the matrix cores, <= 1e-9 relative; layouts
    without a matrix kernel run the "fma" filter bank)."""

    def __init__(self, device: int = 0, numerics: str = "exact"):
        h = c_void_p()
        check(lib().eegfx_ctx_create(device, ctypes.byref(h)))
        self._h = h
        self.device = device
        self.set_numerics(numerics)

    # -- context ----------------------------------------------------------------------------------
    @property
    def handle(self) -> c_void_p:
        if self._h is None:
            raise RuntimeError("context destroyed")
        return self._h

    def set_numerics(self, numerics: str) -> None:
        mode = {"exact": _lib.EXACT, "fma": _lib.FMA, "mfma": _lib.MFMA}[numerics]
        check(lib().eegfx_ctx_set_numerics(self.handle, mode))
        self.numerics = numerics

    def set_stream(self, stream_handle: Optional[int]) -> None:
        check(lib().eegfx_ctx_set_stream(self.handle, c_void_p(stream_handle or 0)))

    def set_timing(self, enable: bool) -> None:
        check(lib().eegfx_ctx_set_timing(self.handle, 1 if enable else 0))

    def synchronize(self) -> None:
        check(lib().eegfx_ctx_synchronize(self.handle))

    def kernel_stats(self):
        """(timed launches, summed duration in ms, algorithmic bytes) of the dominant kernel
        since timing was (re)enabled -- HIP events on the context stream."""
        n, ms, by = c_int64(), ctypes.c_double(), c_int64()
        check(lib().eegfx_ctx_kernel_stats(self.handle, ctypes.byref(n), ctypes.byref(ms),
                                           ctypes.byref(by)))
        return int(n.value), float(ms.value), int(by.value)

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            lib().eegfx_ctx_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter teardown order
        try:
            self.close()
        except Exception:
            pass

    # -- compute ----------------------------------------------------------------------------------
    @staticmethod
    def _sel(cols: Sequence[int], res: Sequence[float]):
        cols_a = np.ascontiguousarray(cols, dtype=np.int32)
        res_a = np.ascontiguousarray(res, dtype=np.float32)
        if cols_a.shape != res_a.shape or cols_a.ndim != 1:
            raise ValueError("cols and res must be 1-D of equal length")
        return cols_a, res_a

    def cut_epochs(self, raw, n_channels_total: int, cols, res, pos, out=None):
        """Raw multiplexed recording (int16 or float32, n_frames x n_channels_total) ->
        baseline-corrected epochs double[n][C][750] (OffLineDataProvider.java:216-233)."""
        cols_a, res_a = self._sel(cols, res)
        fmt = _fmt(raw)
        n_frames = _numel(raw) // n_channels_total
        pos = _contig(pos, np.int64)
        n = _numel(pos)
        C = len(cols_a)
        if out is None:
            out = _empty_like_mem(raw, (n, C, _lib.POSTSTIMULUS), "float64")
        mem = _mem(raw, pos, out)
        check(lib().eegfx_cut_epochs_f64(self.handle, ptr(raw), fmt, n_frames, n_channels_total,
                                         ptr(cols_a), ptr(res_a), C, ptr(pos), n, ptr(out), mem))
        return out

    def extract_features(self, epochs, name=8, epoch_size=512, skip=175, feature_size=16,
                         out=None):
        """Batched WaveletTransform.extractFeatures over epochs double[n][C][750]."""
        epochs = _contig(epochs, np.float64)
        shape = tuple(epochs.shape)
        if len(shape) != 3 or shape[2] != _lib.POSTSTIMULUS:
            raise ValueError(f"epochs must be [n][C][750], got {shape}")
        n, C = shape[0], shape[1]
        if out is None:
            out = _empty_like_mem(epochs, (n, C * feature_size), "float64")
        mem = _mem(epochs, out)
        check(lib().eegfx_extract_features_f64(self.handle, ptr(epochs), n, C, name, epoch_size,
                                               skip, feature_size, ptr(out), mem))
        return out

    def process_recording(self, raw, n_channels_total: int, cols, res, pos, out=None):
        """Fused hot path: raw recording + marker positions -> dwt-8 features [n][16*C]."""
        cols_a, res_a = self._sel(cols, res)
        fmt = _fmt(raw)
        n_frames = _numel(raw) // n_channels_total
        pos = _contig(pos, np.int64)
        n = _numel(pos)
        C = len(cols_a)
        if out is None:
            out = _empty_like_mem(raw, (n, 16 * C), "float64")
        mem = _mem(raw, pos, out)
        check(lib().eegfx_process_recording(self.handle, ptr(raw), fmt, n_frames,
                                            n_channels_total, ptr(cols_a), ptr(res_a), C,
                                            ptr(pos), n, ptr(out), mem))
        return out

    def plan_markers(self, positions, stimulus_index, n_frames: int, guessed: int,
                     balance: int = 0):
        """Marker planning (OffLineDataProvider.java:200-265) on the device as a parallel scan
        (eegfx_plan_markers_device): returns (positions, labels, balance) like
        brainvision.plan_markers.  positions / stimulus_index: host or device arrays."""
        from ctypes import byref
        if _is_device(positions):
            import torch
            n = int(positions.numel())
            pos_out = torch.empty(max(1, n), dtype=torch.int64, device=positions.device)
            lab_out = torch.empty(max(1, n), dtype=torch.float64, device=positions.device)
        else:
            positions = np.ascontiguousarray(positions, dtype=np.int64)
            stimulus_index = np.ascontiguousarray(stimulus_index, dtype=np.int32)
            n = positions.size
            pos_out = np.empty(max(1, n), dtype=np.int64)
            lab_out = np.empty(max(1, n), dtype=np.float64)
        bal = c_int64(balance)
        k = c_int64()
        check(lib().eegfx_plan_markers_device(self.handle, ptr(positions), ptr(stimulus_index), n,
                                              int(n_frames), int(guessed), byref(bal),
                                              ptr(pos_out), ptr(lab_out), byref(k),
                                              _mem(positions, stimulus_index, pos_out)))
        return pos_out[:k.value], lab_out[:k.value], bal.value

    def process_recording_streamed(self, raw, n_channels_total: int, cols, res, pos,
                                   chunk_frames: int = 1 << 23, out=None):
        """configs[4]: the fused path over a host-resident recording streamed to the device in
        chunks (eegfx_process_recording_streamed); raw/pos/out are host (numpy) arrays."""
        cols_a, res_a = self._sel(cols, res)
        if _is_device(raw):
            raise ValueError("process_recording_streamed takes a host recording")
        raw = np.ascontiguousarray(raw)
        fmt = _fmt(raw)
        n_frames = raw.size // n_channels_total
        pos = np.ascontiguousarray(pos, dtype=np.int64)
        n = pos.size
        C = len(cols_a)
        if out is None:
            out = np.empty((n, 16 * C), dtype=np.float64)
        check(lib().eegfx_process_recording_streamed(
            self.handle, ptr(raw), fmt, n_frames, n_channels_total, ptr(cols_a), ptr(res_a), C,
            ptr(pos), n, ptr(out), int(chunk_frames)))
        return out

    def synth_recording(self, dst, n_channels: int, seed: int) -> None:
        """Fills a device int16 tensor (n_frames x n_channels) with the synthetic recording."""
        if not _is_device(dst):
            raise ValueError("synth_recording writes a device tensor")
        n_frames = dst.numel() // n_channels
        check(lib().eegfx_synth_recording(self.handle, ptr(dst), n_frames, n_channels,
                                          ctypes.c_uint64(seed)))


def dwt8_operator() -> np.ndarray:
    """The fe=dwt-8 window transform as a 16 x 512 matrix (host; eegfx_dwt8_operator):
    row r of the first 16 coefficients (a6 ++ d6, before normalisation) of a window x is
    ``M[r] @ x`` -- the operator the "mfma" numerics applies on the FP64 matrix cores."""
    m = np.empty((16, 512), dtype=np.float64)
    check(lib().eegfx_dwt8_operator(ptr(m)))
    return m


def device_count() -> int:
    n = c_int()
    check(lib().eegfx_device_count(ctypes.byref(n)))
    return n.value


def _numel(a) -> int:
    return int(a.numel()) if hasattr(a, "numel") and callable(a.numel) else int(np.asarray(a).size)


def _fmt(raw) -> int:
    name = str(raw.dtype)
    if name.endswith("int16"):
        return _lib.INT_16
    if name.endswith("float32"):
        return _lib.IEEE_FLOAT_32
    raise ValueError(f"raw samples must be int16 or float32, got {raw.dtype}")


def _empty_like_mem(ref, shape, dtype: str):
    if _is_device(ref):
        import torch
        return torch.empty(shape, dtype=getattr(torch, dtype), device=ref.device)
    return np.empty(shape, dtype=dtype)
