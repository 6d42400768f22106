"""Device context and the compute entry points of libeegfx (include/eegfx.h).

Arrays may be numpy arrays (host memory: the library stages them through HBM and returns after
the results are copied back) or torch tensors on a ROCm device (device memory: the work is
enqueued on the context stream and the call returns without synchronising).  Device calls are
ordered with torch's current stream on both sides: the context stream waits for the work that
produced the inputs, and torch's stream waits for the kernels before anything later uses (or
frees) the buffers.  Marker positions held in device memory are validated by the kernels; a
violation raises ``IndexError`` (the reference's ArrayIndexOutOfBoundsException) from the next
call that synchronises the context (``Context.synchronize()``, or any host-memory call); device
results are unspecified until such a call has returned without error.
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


_TORCH_NAMES = {np.dtype(np.float64): "float64", np.dtype(np.int64): "int64",
                np.dtype(np.int32): "int32", np.dtype(np.float32): "float32",
                np.dtype(np.int16): "int16"}


def _contig(a, dtype):
    """Host arrays are converted to `dtype`; device tensors are passed as they are, so they must
    already have it (the kernels read the raw bytes: an int32 position tensor read as int64 would
    address past its allocation)."""
    if _is_device(a):
        want = _TORCH_NAMES[np.dtype(dtype)]
        if str(a.dtype) != "torch." + want:
            raise ValueError(f"device tensor has dtype {a.dtype}, expected torch.{want}")
        if not a.is_contiguous():
            raise ValueError("device tensors must be contiguous")
        return a
    return np.ascontiguousarray(a, dtype=dtype)


def _check_out(out, shape, dtype="float64"):
    """A caller-supplied output: right shape, dtype and contiguity (the kernels write it raw)."""
    if tuple(out.shape) != tuple(shape):
        raise ValueError(f"out has shape {tuple(out.shape)}, expected {tuple(shape)}")
    if _is_device(out):
        if str(out.dtype) != "torch." + dtype or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous torch.{dtype} tensor")
    elif out.dtype != np.dtype(dtype) or not out.flags["C_CONTIGUOUS"]:
        raise ValueError(f"out must be a C-contiguous {dtype} array")
    return out


class Context:
    """One HIP device + stream (eegfx_ctx).  numerics: "exact" (bit-exact to the reference
    order of operations, default) or "fma" (fused multiply-add filter bank, <= 1e-9 relative)."""

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
        modes = {"exact": _lib.EXACT, "fma": _lib.FMA}
        if numerics not in modes:
            raise ValueError(f"numerics must be one of {sorted(modes)}, got {numerics!r}")
        mode = modes[numerics]
        check(lib().eegfx_ctx_set_numerics(self.handle, mode))
        self.numerics = numerics

    def set_stream(self, stream_handle: Optional[int]) -> None:
        check(lib().eegfx_ctx_set_stream(self.handle, c_void_p(stream_handle or 0)))

    def stream_handle(self) -> int:
        """The hipStream_t the context enqueues on."""
        h = c_void_p()
        check(lib().eegfx_ctx_stream(self.handle, ctypes.byref(h)))
        return int(h.value or 0)

    def _enter_device(self, ref):
        """Orders the context stream after torch's current stream (the producers of the inputs);
        returns the pair for _leave_device, or None when they are the same stream."""
        import torch
        cur = torch.cuda.current_stream(ref.device)
        mine = self.stream_handle()
        if cur.cuda_stream == mine:
            return None
        ext = torch.cuda.ExternalStream(mine, device=ref.device)
        ext.wait_stream(cur)
        return cur, ext

    @staticmethod
    def _leave_device(pair) -> None:
        """Orders torch's current stream after the kernels just enqueued."""
        if pair is not None:
            cur, ext = pair
            cur.wait_stream(ext)

    def _call(self, mem, ref, fn, *args):
        pair = self._enter_device(ref) if mem == _lib.MEM_DEVICE else None
        try:
            check(fn(*args))
        finally:
            self._leave_device(pair)

    def set_timing(self, enable: bool) -> None:
        check(lib().eegfx_ctx_set_timing(self.handle, 1 if enable else 0))

    def synchronize(self) -> None:
        """Waits for the context stream.  Raises IndexError when a kernel met a device-resident
        marker position the reference would not cut (OffLineDataProvider.java:220-225)."""
        check(lib().eegfx_ctx_synchronize(self.handle))  # ERANGE -> EegfxRangeError (IndexError)

    def kernel_stats(self):
        """(timed launches, summed duration in ms, algorithmic bytes) of the dominant kernel
        since timing was (re)enabled -- HIP events on the context stream."""
        n, ms, by = c_int64(), ctypes.c_double(), c_int64()
        check(lib().eegfx_ctx_kernel_stats(self.handle, ctypes.byref(n), ctypes.byref(ms),
                                           ctypes.byref(by)))
        return int(n.value), float(ms.value), int(by.value)

    def guard_stats(self, reset: bool = False):
        """(rows checked, rows recomputed under EXACT) of the fma numerics' conditioning guard
        since the context was created or last reset (eegfx_ctx_guard_stats; synchronises)."""
        a, b = c_int64(), c_int64()
        check(lib().eegfx_ctx_guard_stats(self.handle, ctypes.byref(a), ctypes.byref(b),
                                          1 if reset else 0))
        return int(a.value), int(b.value)

    def set_mailbox(self, enable: bool) -> None:
        """Opt-in resident server for small host extract batches (eegfx_ctx_set_mailbox): the
        per-epoch drop-in without a launch per call.  Disable it before a device-wide
        synchronisation (torch.cuda.synchronize), which would wait for the resident kernel."""
        check(lib().eegfx_ctx_set_mailbox(self.handle, 1 if enable else 0))

    def mailbox_state(self):
        """(enabled, resident) of the context's per-epoch server (eegfx_ctx_get_mailbox): at most
        4 contexts of a process hold a started server on a device; the others use the launch
        path."""
        a, b = ctypes.c_int32(), ctypes.c_int32()
        check(lib().eegfx_ctx_get_mailbox(self.handle, ctypes.byref(a), ctypes.byref(b)))
        return bool(a.value), bool(b.value)

    def guard_detail(self, reset: bool = False):
        """(rows checked, rows that went to the guard's second stage, rows recomputed under EXACT)
        since the context was created or last reset (eegfx_ctx_guard_detail; synchronises)."""
        a, b, c = c_int64(), c_int64(), c_int64()
        check(lib().eegfx_ctx_guard_detail(self.handle, ctypes.byref(a), ctypes.byref(b),
                                           ctypes.byref(c), 1 if reset else 0))
        return int(a.value), int(b.value), int(c.value)

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
        raw = _raw(raw)
        fmt = _fmt(raw)
        n_frames = _frames(raw, n_channels_total)
        pos = _contig(pos, np.int64)
        n = _numel(pos)
        C = len(cols_a)
        if out is None:
            out = _empty_like_mem(raw, (n, C, _lib.POSTSTIMULUS), "float64")
        _check_out(out, (n, C, _lib.POSTSTIMULUS))
        mem = _mem(raw, pos, out)
        self._call(mem, raw, lib().eegfx_cut_epochs_f64, self.handle, ptr(raw), fmt, n_frames,
                   n_channels_total, ptr(cols_a), ptr(res_a), C, ptr(pos), n, ptr(out), mem)
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
        _check_out(out, (n, C * feature_size))
        mem = _mem(epochs, out)
        self._call(mem, epochs, lib().eegfx_extract_features_f64, self.handle, ptr(epochs), n, C,
                   name, epoch_size, skip, feature_size, ptr(out), mem)
        return out

    def process_recording(self, raw, n_channels_total: int, cols, res, pos, out=None):
        """Fused hot path: raw recording + marker positions -> dwt-8 features [n][16*C]."""
        cols_a, res_a = self._sel(cols, res)
        raw = _raw(raw)
        fmt = _fmt(raw)
        n_frames = _frames(raw, n_channels_total)
        pos = _contig(pos, np.int64)
        n = _numel(pos)
        C = len(cols_a)
        if out is None:
            out = _empty_like_mem(raw, (n, 16 * C), "float64")
        _check_out(out, (n, 16 * C))
        mem = _mem(raw, pos, out)
        self._call(mem, raw, lib().eegfx_process_recording, self.handle, ptr(raw), fmt, n_frames,
                   n_channels_total, ptr(cols_a), ptr(res_a), C, ptr(pos), n, ptr(out), mem)
        return out

    def process_recording_epochs(self, raw, n_channels_total: int, cols, res, pos, out=None,
                                 epochs_out=None):
        """getData() and extractFeatures in one pass (eegfx_process_recording_epochs): returns
        (features [n][16*C], epochs [n][C][750]), each equal to its own call."""
        cols_a, res_a = self._sel(cols, res)
        raw = _raw(raw)
        fmt = _fmt(raw)
        n_frames = _frames(raw, n_channels_total)
        pos = _contig(pos, np.int64)
        n = _numel(pos)
        C = len(cols_a)
        if out is None:
            out = _empty_like_mem(raw, (n, 16 * C), "float64")
        if epochs_out is None:
            epochs_out = _empty_like_mem(raw, (n, C, _lib.POSTSTIMULUS), "float64")
        _check_out(out, (n, 16 * C))
        _check_out(epochs_out, (n, C, _lib.POSTSTIMULUS))
        mem = _mem(raw, pos, out, epochs_out)
        self._call(mem, raw, lib().eegfx_process_recording_epochs, self.handle, ptr(raw), fmt,
                   n_frames, n_channels_total, ptr(cols_a), ptr(res_a), C, ptr(pos), n, ptr(out),
                   ptr(epochs_out), mem)
        return out, epochs_out

    def plan_markers(self, positions, stimulus_index, n_frames: int, guessed: int,
                     balance: int = 0):
        """Marker planning (OffLineDataProvider.java:200-265) on the device as a parallel scan
        (eegfx_plan_markers_device): returns (positions, labels, balance) like
        brainvision.plan_markers.  positions / stimulus_index: host or device arrays."""
        from ctypes import byref
        if _is_device(positions):
            import torch
            positions = _contig(positions, np.int64)
            stimulus_index = _contig(stimulus_index, np.int32)
            n = int(positions.numel())
            if int(stimulus_index.numel()) != n:
                raise ValueError("positions and stimulus_index must have the same length")
            pos_out = torch.empty(max(1, n), dtype=torch.int64, device=positions.device)
            lab_out = torch.empty(max(1, n), dtype=torch.float64, device=positions.device)
        else:
            positions = np.ascontiguousarray(positions, dtype=np.int64)
            stimulus_index = np.ascontiguousarray(stimulus_index, dtype=np.int32)
            n = positions.size
            if stimulus_index.size != n:
                raise ValueError("positions and stimulus_index must have the same length")
            pos_out = np.empty(max(1, n), dtype=np.int64)
            lab_out = np.empty(max(1, n), dtype=np.float64)
        bal = c_int64(balance)
        k = c_int64()
        mem = _mem(positions, stimulus_index, pos_out)
        self._call(mem, positions, lib().eegfx_plan_markers_device, self.handle, ptr(positions),
                   ptr(stimulus_index), n, int(n_frames), int(guessed), byref(bal), ptr(pos_out),
                   ptr(lab_out), byref(k), mem)
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
        n_frames = _frames(raw, n_channels_total)
        pos = np.ascontiguousarray(pos, dtype=np.int64)
        n = pos.size
        C = len(cols_a)
        if out is None:
            out = np.empty((n, 16 * C), dtype=np.float64)
        _check_out(out, (n, 16 * C))
        check(lib().eegfx_process_recording_streamed(
            self.handle, ptr(raw), fmt, n_frames, n_channels_total, ptr(cols_a), ptr(res_a), C,
            ptr(pos), n, ptr(out), int(chunk_frames)))
        return out

    def synth_recording(self, dst, n_channels: int, seed: int) -> None:
        """Fills a device int16 tensor (n_frames x n_channels) with the synthetic recording."""
        if not _is_device(dst):
            raise ValueError("synth_recording writes a device tensor")
        dst = _contig(dst, np.int16)
        n_frames = _frames(dst, n_channels)
        self._call(_lib.MEM_DEVICE, dst, lib().eegfx_synth_recording, self.handle, ptr(dst),
                   n_frames, n_channels, ctypes.c_uint64(seed))


def device_count() -> int:
    n = c_int()
    check(lib().eegfx_device_count(ctypes.byref(n)))
    return n.value


def _frames(raw, n_channels_total: int) -> int:
    """Frames of a multiplexed recording of n_channels_total channels: the channel count must be
    positive, divide the buffer, and match the second dimension of a 2-D recording."""
    ct = int(n_channels_total)
    if ct < 1:
        raise ValueError(f"n_channels_total must be >= 1, got {n_channels_total}")
    shape = tuple(raw.shape)
    if len(shape) == 2 and shape[1] != ct:
        raise ValueError(f"recording has {shape[1]} channels per frame, n_channels_total is {ct}")
    total = _numel(raw)
    if total % ct:
        raise ValueError(f"{total} samples do not divide into frames of {ct} channels")
    return total // ct


def _numel(a) -> int:
    return int(a.numel()) if hasattr(a, "numel") and callable(a.numel) else int(np.asarray(a).size)


def _raw(raw):
    """The recording: a contiguous int16 / float32 array (host) or tensor (device)."""
    _fmt(raw)
    if _is_device(raw):
        if not raw.is_contiguous():
            raise ValueError("device tensors must be contiguous")
        return raw
    return np.ascontiguousarray(raw)


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
