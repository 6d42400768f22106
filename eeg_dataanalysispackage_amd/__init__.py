"""MI355X-native epoch-to-feature path of EEG_DataAnalysisPackage.

Host mirror of the reference's hot-path API over the libeegfx C ABI (include/eegfx.h):

* :class:`OffLineDataProvider` -- DataTransformation/OffLineDataProvider.java
* :class:`IFeatureExtraction`, :class:`WaveletTransform` -- FeatureExtraction/*.java (fe=dwt-8)
* :class:`Context` -- device/stream + the batched and fused compute entry points
* :mod:`brainvision` -- native .vhdr/.vmrk reader and marker planner
"""
from ._lib import EegfxError, LIB_PATH, lib
from .brainvision import (ChannelInfo, EEGMarker, Header, plan_markers, read_header,
                          read_markers, read_raw, recording_frames)
from .context import Context, device_count
from .data_provider import OffLineDataProvider
from .feature_extraction import IFeatureExtraction, WaveletTransform

__all__ = [
    "Context", "ChannelInfo", "EEGMarker", "EegfxError", "Header", "IFeatureExtraction",
    "LIB_PATH", "OffLineDataProvider", "WaveletTransform", "device_count", "lib",
    "plan_markers", "read_header", "read_markers", "read_raw", "recording_frames",
]
