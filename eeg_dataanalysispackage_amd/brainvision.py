"""Native BrainVision reader and marker planner (csrc/brainvision.cpp) -- Python view.

Replaces the eegloader-hdfs 2.4 calls of OffLineDataProvider.processEEGFiles
(``getChannelInfo`` :167-168, ``readMarkerList`` :196) and the per-marker selection loop
(:200-265) with the native implementation in libeegfx.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import check, lib


@dataclass
class ChannelInfo:
    number: int       # 1-based (ChannelInfo.getNumber())
    name: str         # ChannelInfo.getName()
    reference: str
    resolution: float
    unit: str         # ChannelInfo.getUnits()


@dataclass
class Header:
    n_channels: int
    binary_format: int  # _lib.INT_16 | _lib.IEEE_FLOAT_32
    multiplexed: bool
    sampling_interval_us: float
    data_file: str
    marker_file: str
    channels: List[ChannelInfo]


@dataclass
class EEGMarker:
    number: int
    type: str
    stimulus: str        # EEGMarker.getStimulus(): the description field
    position: int        # EEGMarker.getPosition()
    size: int
    channel: int
    stimulus_index: int  # digits(stimulus) - 1, or -1


def _s(b: bytes) -> str:
    return b.decode("utf-8", errors="replace")


def read_header(vhdr_path: str) -> Header:
    info = _lib.HeaderInfo()
    check(lib().eegfx_read_header(vhdr_path.encode(), ctypes.byref(info), None, 0))
    chans = (_lib.ChannelInfo * max(1, 4096))()
    check(lib().eegfx_read_header(vhdr_path.encode(), ctypes.byref(info), chans, 4096))
    # the header may list fewer Ch<n> entries than NumberOfChannels
    out = []
    for c in chans:
        if c.number == 0:
            break
        out.append(ChannelInfo(c.number, _s(c.name), _s(c.reference), c.resolution, _s(c.unit)))
    return Header(info.n_channels, info.binary_format, bool(info.multiplexed),
                  info.sampling_interval_us, _s(info.data_file), _s(info.marker_file), out)


def read_markers(vmrk_path: str) -> List[EEGMarker]:
    n = ctypes.c_int64()
    check(lib().eegfx_read_markers(vmrk_path.encode(), None, 0, ctypes.byref(n)))
    arr = (_lib.Marker * max(1, n.value))()
    check(lib().eegfx_read_markers(vmrk_path.encode(), arr, n.value, ctypes.byref(n)))
    return [EEGMarker(m.number, _s(m.type), _s(m.description), m.position, m.size, m.channel,
                      m.stimulus_index) for m in arr[:n.value]]


def recording_frames(vhdr_path: str, eeg_path: str) -> int:
    n = ctypes.c_int64()
    check(lib().eegfx_recording_frames(vhdr_path.encode(), eeg_path.encode(), ctypes.byref(n)))
    return n.value


def read_raw(vhdr_path: str, eeg_path: str) -> np.ndarray:
    """Raw multiplexed samples as [n_frames][n_channels] (int16 or float32), host memory."""
    h = read_header(vhdr_path)
    nf = recording_frames(vhdr_path, eeg_path)
    dt = np.int16 if h.binary_format == _lib.INT_16 else np.float32
    out = np.empty((nf, h.n_channels), dtype=dt)
    check(lib().eegfx_read_raw(None, vhdr_path.encode(), eeg_path.encode(),
                               ctypes.c_void_p(out.ctypes.data), out.nbytes, _lib.MEM_HOST))
    return out


def _marker_array(markers: Sequence[EEGMarker]):
    arr = (_lib.Marker * max(1, len(markers)))()
    for i, m in enumerate(markers):
        arr[i].number = m.number
        arr[i].type = m.type.encode()[:63]
        arr[i].description = m.stimulus.encode()[:63]
        arr[i].position = m.position
        arr[i].size = m.size
        arr[i].channel = m.channel
        arr[i].stimulus_index = m.stimulus_index
    return arr


def plan_markers(markers: Sequence[EEGMarker], n_frames: int, guessed: int,
                 balance: int = 0) -> Tuple[np.ndarray, np.ndarray, int]:
    """OffLineDataProvider.java:200-265 selection: returns (positions, labels, balance)."""
    arr = _marker_array(markers)
    n = len(markers)
    pos = np.empty(max(1, n), dtype=np.int64)
    lab = np.empty(max(1, n), dtype=np.float64)
    bal = ctypes.c_int64(balance)
    k = ctypes.c_int64()
    check(lib().eegfx_plan_markers(arr, n, n_frames, guessed, ctypes.byref(bal),
                                   ctypes.c_void_p(pos.ctypes.data),
                                   ctypes.c_void_p(lab.ctypes.data), ctypes.byref(k)))
    return pos[:k.value].copy(), lab[:k.value].copy(), bal.value
