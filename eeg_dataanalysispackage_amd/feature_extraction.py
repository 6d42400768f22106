"""IFeatureExtraction / WaveletTransform -- the fe=dwt-8 plugin on the MI355X path.

Mirrors FeatureExtraction/IFeatureExtraction.java:27-35 and WaveletTransform.java:40-246:
constructor ``WaveletTransform(name, epochSize, skipSamples, featureSize)`` (:82-87), the
validating setters (:160-212) raising ``ValueError`` where Java raises
IllegalArgumentException, ``getFeatureDimension()`` = FEATURE_SIZE * 3 / 1 (:150-152), and
``extractFeatures(epoch)`` for one ``double[3][750]`` epoch returning a fresh 48-vector.
``extractFeaturesBatch`` is the batched form the GPU is built for (one launch per batch).
"""
from __future__ import annotations

import abc
from typing import Optional

import numpy as np

from . import _lib
from .context import Context

CHANNELS = (1, 2, 3)          # WaveletTransform.java:47
DOWN_SMPL_FACTOR = 1          # :57


class IFeatureExtraction(abc.ABC):
    @abc.abstractmethod
    def extractFeatures(self, epoch) -> np.ndarray:
        ...

    @abc.abstractmethod
    def getFeatureDimension(self) -> int:
        ...


class WaveletTransform(IFeatureExtraction):
    def __init__(self, name: int = 8, epochSize: int = 512, skipSamples: int = 175,
                 featureSize: int = 16, context: Optional[Context] = None):
        # The 4-argument Java constructor assigns without validation (:82-87).
        self.NAME = name
        self.EPOCH_SIZE = epochSize
        self.SKIP_SAMPLES = skipSamples
        self.FEATURE_SIZE = featureSize
        self._ctx = context

    @property
    def context(self) -> Context:
        if self._ctx is None:
            self._ctx = Context()
        return self._ctx

    # -- IFeatureExtraction -----------------------------------------------------------------------
    def extractFeatures(self, epoch) -> np.ndarray:
        e = np.asarray(epoch, dtype=np.float64)
        if e.ndim != 2 or e.shape[0] < len(CHANNELS) or e.shape[1] < _lib.POSTSTIMULUS:
            raise IndexError(f"epoch must be double[>=3][750], got {e.shape}")
        batch = np.ascontiguousarray(e[None, :len(CHANNELS), :_lib.POSTSTIMULUS])
        return self.extractFeaturesBatch(batch)[0]

    def getFeatureDimension(self) -> int:
        return self.FEATURE_SIZE * len(CHANNELS) // DOWN_SMPL_FACTOR

    # -- batched form ------------------------------------------------------------------------------
    def extractFeaturesBatch(self, epochs, out=None):
        """epochs: double[n][C][750] (numpy or device tensor) -> features [n][C*FEATURE_SIZE]."""
        return self.context.extract_features(epochs, self.NAME, self.EPOCH_SIZE,
                                             self.SKIP_SAMPLES, self.FEATURE_SIZE, out=out)

    # -- setters (:160-212) ------------------------------------------------------------------------
    def setWaveletName(self, name: int) -> None:
        if 0 <= name <= 17:
            self.NAME = name
        else:
            raise ValueError("Wavelet Name must be >= 0 and <= 17")

    def setEpochSize(self, epochSize: int) -> None:
        if 0 < epochSize <= _lib.POSTSTIMULUS:
            self.EPOCH_SIZE = epochSize
        else:
            raise ValueError(f"Epoch Size must be > 0 and <= {_lib.POSTSTIMULUS}")

    def setSkipSamples(self, skipSamples: int) -> None:
        if 0 < skipSamples <= _lib.POSTSTIMULUS:
            self.SKIP_SAMPLES = skipSamples
        else:
            raise ValueError(f"Skip Samples must be > 0 and <= {_lib.POSTSTIMULUS}")

    def setFeatureSize(self, featureSize: int) -> None:
        if 0 < featureSize <= 1024:
            self.FEATURE_SIZE = featureSize
        else:
            raise ValueError("Feature Size must be > 0 and <= 1024")

    def __str__(self) -> str:
        return (f"DWT: EPOCH_SIZE: {self.EPOCH_SIZE} FEATURE_SIZE: {self.FEATURE_SIZE} "
                f"WAVELETNAME: {self.NAME} SKIP_SAMPLES: {self.SKIP_SAMPLES}\n")

    def __eq__(self, other) -> bool:
        return (isinstance(other, WaveletTransform) and self.EPOCH_SIZE == other.EPOCH_SIZE
                and self.SKIP_SAMPLES == other.SKIP_SAMPLES and self.NAME == other.NAME
                and self.FEATURE_SIZE == other.FEATURE_SIZE)

    def __hash__(self) -> int:
        r = self.EPOCH_SIZE
        r = 31 * r + self.SKIP_SAMPLES
        r = 31 * r + self.NAME
        return 31 * r + self.FEATURE_SIZE
