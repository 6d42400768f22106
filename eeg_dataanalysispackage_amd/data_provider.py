"""OffLineDataProvider -- the reference's data-provider API on the MI355X path.

Mirrors DataTransformation/OffLineDataProvider.java: ``OffLineDataProvider(args)`` (:78),
``loadData()`` (:88-98), ``getData()`` (:370), ``getDataLabels()`` (:377), with the same argument
formats (``[info.txt]`` or ``[file.eeg, guessed, ...]``), the same per-file skip rules and the
same error behaviour: ``loadData`` never raises -- it logs the fatal error, keeps what was loaded
and exposes the message as ``last_error``.  Paths are local files (the reference reads HDFS).

Decode, epoch cut and baseline correction run on the GPU (csrc/kernels.hip); the epochs stay
resident in HBM and ``getData()`` copies them back.
"""
from __future__ import annotations

import ctypes
import logging
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import check, lib
from .context import Context

log = logging.getLogger(__name__)


class OffLineDataProvider:
    def __init__(self, args: Sequence[str], context: Optional[Context] = None,
                 plan_only: bool = False):
        """plan_only=True: parse, select and label on the host only (no GPU, no epochs)."""
        self.args = list(args)
        self._ctx = None if plan_only else (context if context is not None else Context())
        argv = (ctypes.c_char_p * max(1, len(self.args)))(*[a.encode() for a in self.args])
        h = ctypes.c_void_p()
        handle = self._ctx.handle if self._ctx is not None else None
        check(lib().eegfx_odp_create(handle, argv, len(self.args), ctypes.byref(h)))
        self._h = h
        self.last_error = ""
        log.info("Started OffLineDataProvider with arguments %s", self.args)

    def loadData(self) -> None:
        rc = lib().eegfx_odp_load_data(self._h)
        self.last_error = lib().eegfx_odp_error(self._h).decode(errors="replace")
        if rc != _lib.EEGFX_OK:
            log.critical(self.last_error)  # logger.fatal(e.getMessage()) -- swallowed

    def num_epochs(self) -> int:
        return int(lib().eegfx_odp_num_epochs(self._h))

    def getData(self) -> np.ndarray:
        """Epochs as double[n][3][750] (Fz, Cz, Pz)."""
        n = self.num_epochs()
        out = np.empty((n, 3, _lib.POSTSTIMULUS), dtype=np.float64)
        if n:
            check(lib().eegfx_odp_get_data(self._h, ctypes.c_void_p(out.ctypes.data)))
        return out

    def getDataLabels(self) -> List[float]:
        n = self.num_epochs()
        out = np.empty(max(1, n), dtype=np.float64)
        check(lib().eegfx_odp_get_labels(self._h, ctypes.c_void_p(out.ctypes.data)))
        return [float(v) for v in out[:n]]

    def getPositions(self):
        """Marker positions and source-file index of every selected epoch (not in the Java API;
        exposes the bit-exact marker offsets for parity tests)."""
        n = self.num_epochs()
        pos = np.empty(max(1, n), dtype=np.int64)
        fid = np.empty(max(1, n), dtype=np.int32)
        check(lib().eegfx_odp_get_positions(self._h, ctypes.c_void_p(pos.ctypes.data),
                                            ctypes.c_void_p(fid.ctypes.data)))
        return pos[:n], fid[:n]

    def getFeatures(self, name=8, epoch_size=512, skip=175, feature_size=16) -> np.ndarray:
        """fe=dwt-8 features of the resident epochs, computed on the device."""
        n = self.num_epochs()
        out = np.empty((n, 3 * feature_size), dtype=np.float64)
        if n:
            check(lib().eegfx_odp_get_features(self._h, name, epoch_size, skip, feature_size,
                                               ctypes.c_void_p(out.ctypes.data)))
        return out

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            lib().eegfx_odp_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
