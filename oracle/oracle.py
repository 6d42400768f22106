"""CPU oracle of the reference epoch-to-feature path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker / CPU baseline.  The product (eeg_dataanalysispackage_amd/) never
imports it.

* numerics: liboracle.so, the C restatement in eegfx_oracle.c (built by oracle/Makefile);
* host logic: a pure-Python restatement of the reference's control flow, each function citing
  the reference file:line it follows (paths relative to the reference checkout,
  src/main/java/cz/zcu/kiv/...).  BrainVision parsing restates the un-vendored
  eegloader-hdfs 2.4 jar (pom.xml:84-88) from the file format and the reference's call sites.

Pinned against the reference's own goldens in tests/test_oracle_golden.py.
"""
from __future__ import annotations

import ctypes
import os
import re
import subprocess
from ctypes import c_double, c_int, c_int64, c_void_p
from typing import Dict, List, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
PRE, POST = 100, 750  # Const.java:61-62

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.oracle_decode_epochs.argtypes = [c_void_p, c_int, c_int64, c_int, c_void_p, c_void_p,
                                           c_int, c_void_p, c_int64, c_void_p]
        L.oracle_extract_features.argtypes = [c_void_p, c_int64, c_int, c_int, c_int, c_int, c_int,
                                              c_void_p]
        L.oracle_process_recording.argtypes = [c_void_p, c_int, c_int64, c_int, c_void_p, c_void_p,
                                               c_int, c_void_p, c_int64, c_int, c_int, c_int, c_int,
                                               c_int, c_void_p]
        L.oracle_process_recording_fast.argtypes = [c_void_p, c_int, c_int64, c_int, c_void_p,
                                                    c_void_p, c_int, c_void_p, c_int64, c_int,
                                                    c_int, c_int, c_int, c_void_p]
        L.oracle_process_recording_fast.restype = c_int
        L.oracle_extract_features_fast.argtypes = [c_void_p, c_int64, c_int, c_int, c_int, c_int,
                                                   c_void_p]
        L.oracle_extract_features_fast.restype = c_int
        for f in (L.oracle_decode_epochs, L.oracle_extract_features, L.oracle_process_recording):
            f.restype = None
        _lib = L
    return _lib


def _p(a: np.ndarray) -> c_void_p:
    return c_void_p(a.ctypes.data)


# ---- numerics (liboracle) -------------------------------------------------------------------------
def decode_epochs(raw: np.ndarray, cols: Sequence[int], res: Sequence[float],
                  pos: Sequence[int]) -> np.ndarray:
    """a3 + a5..a7 -> double[n][C][750] (OffLineDataProvider.java:216-233)."""
    raw = np.ascontiguousarray(raw)
    fmt = 0 if raw.dtype == np.int16 else 1
    n_frames, ct = raw.shape
    cols_a = np.ascontiguousarray(cols, dtype=np.int32)
    res_a = np.ascontiguousarray(res, dtype=np.float32)
    pos_a = np.ascontiguousarray(pos, dtype=np.int64)
    out = np.empty((len(pos_a), len(cols_a), POST), dtype=np.float64)
    lib().oracle_decode_epochs(_p(raw), fmt, n_frames, ct, _p(cols_a), _p(res_a), len(cols_a),
                               _p(pos_a), len(pos_a), _p(out))
    return out


def extract_features(epochs: np.ndarray, skip=175, win=512, nfeat=16,
                     faithful=True) -> np.ndarray:
    """WaveletTransform.extractFeatures per epoch (WaveletTransform.java:107-141)."""
    ep = np.ascontiguousarray(epochs, dtype=np.float64)
    n, C, _ = ep.shape
    out = np.empty((n, C * nfeat), dtype=np.float64)
    lib().oracle_extract_features(_p(ep), n, C, skip, win, nfeat, 1 if faithful else 0, _p(out))
    return out


def extract_features_fast(epochs: np.ndarray, skip=175, win=512, nfeat=16) -> np.ndarray:
    """The optimised CPU extractFeatures (channels share the vector lanes); bit-identical to
    extract_features.  The per-thread CPU rate beside the drop-in (bench.py --workload dropin)."""
    ep = np.ascontiguousarray(epochs, dtype=np.float64)
    n, C, _ = ep.shape
    out = np.empty((n, C * nfeat), dtype=np.float64)
    if lib().oracle_extract_features_fast(_p(ep), n, C, skip, win, nfeat, _p(out)) != 0:
        raise ValueError("extract_features_fast: win must be 512, nfeat <= 16, skip + win <= 750")
    return out


def process_recording(raw: np.ndarray, cols, res, pos, faithful=True, nthreads=1,
                      skip=175, win=512, nfeat=16) -> np.ndarray:
    raw = np.ascontiguousarray(raw)
    fmt = 0 if raw.dtype == np.int16 else 1
    n_frames, ct = raw.shape
    cols_a = np.ascontiguousarray(cols, dtype=np.int32)
    res_a = np.ascontiguousarray(res, dtype=np.float32)
    pos_a = np.ascontiguousarray(pos, dtype=np.int64)
    out = np.empty((len(pos_a), len(cols_a) * nfeat), dtype=np.float64)
    lib().oracle_process_recording(_p(raw), fmt, n_frames, ct, _p(cols_a), _p(res_a),
                                   len(cols_a), _p(pos_a), len(pos_a), skip, win, nfeat,
                                   1 if faithful else 0, nthreads, _p(out))
    return out


def process_recording_fast(raw: np.ndarray, cols, res, pos, nthreads=1, skip=175, win=512,
                           nfeat=16) -> np.ndarray:
    """The optimised CPU baseline: minimal cascade over only the frames that reach
    the features, epochs vectorised in groups; bit-identical to process_recording (bench.py's
    cpu_baseline leg; tests/test_oracle_golden.py pins it)."""
    raw = np.ascontiguousarray(raw)
    fmt = 0 if raw.dtype == np.int16 else 1
    n_frames, ct = raw.shape
    cols_a = np.ascontiguousarray(cols, dtype=np.int32)
    res_a = np.ascontiguousarray(res, dtype=np.float32)
    pos_a = np.ascontiguousarray(pos, dtype=np.int64)
    out = np.empty((len(pos_a), len(cols_a) * nfeat), dtype=np.float64)
    rc = lib().oracle_process_recording_fast(_p(raw), fmt, n_frames, ct, _p(cols_a), _p(res_a),
                                             len(cols_a), _p(pos_a), len(pos_a), skip, win, nfeat,
                                             nthreads, _p(out))
    if rc != 0:
        raise ValueError("process_recording_fast: win must be 512, nfeat <= 16, skip + win <= 750")
    return out


# ---- host logic (pure Python restatement) -------------------------------------------------------
class JavaError(Exception):
    """Stands for the Java exception the reference would raise (name in .kind)."""

    def __init__(self, kind: str, msg: str = ""):
        super().__init__(f"{kind}: {msg}")
        self.kind = kind


def java_parse_int(s: str) -> int:
    """Integer.parseInt: optional sign, ASCII digits, int32 range."""
    if not re.fullmatch(r"[+-]?[0-9]+", s):
        raise JavaError("NumberFormatException", f'For input string: "{s}"')
    v = int(s)
    if not -2**31 <= v < 2**31:
        raise JavaError("NumberFormatException", f'For input string: "{s}"')
    return v


def java_split_space(s: str) -> List[str]:
    """String.split(" "): trailing empty strings removed."""
    parts = s.split(" ")
    while parts and parts[-1] == "":
        parts.pop()
    if not parts and s == "":
        return [""]
    return parts


def read_lines(path: str) -> List[str]:
    """BufferedReader.readLine over a file (\\n, \\r\\n, \\r terminators)."""
    with open(path, "rb") as f:
        text = f.read().decode("utf-8", errors="replace")
    lines = re.split(r"\r\n|\n|\r", text)
    if lines and lines[-1] == "":
        lines.pop()
    return lines


def read_vhdr(path: str) -> Dict:
    """eegloader getChannelInfo + header fields (OffLineDataProvider.java:167-168)."""
    sec = ""
    info = {"n_channels": None, "binary_format": "INT_16", "orientation": "MULTIPLEXED",
            "channels": []}
    for raw in read_lines(path):
        line = raw.strip()
        if not line or line.startswith(";"):
            continue
        if line.startswith("["):
            sec = line.lower()
            if sec == "[comment]":
                break
            continue
        if "=" not in line:
            continue
        k, v = line.split("=", 1)
        k = k.strip()
        if sec == "[common infos]" and k == "NumberOfChannels":
            info["n_channels"] = int(v)
        elif sec == "[common infos]" and k == "DataOrientation":
            info["orientation"] = v.strip()
        elif sec == "[binary infos]" and k == "BinaryFormat":
            info["binary_format"] = v.strip()
        elif sec == "[channel infos]" and k.startswith("Ch"):
            f = v.split(",")
            name = f[0].replace("\\1", ",")
            res = float(f[2]) if len(f) > 2 and f[2].strip() else 1.0
            info["channels"].append((int(k[2:]), name, res))
    return info


def read_vmrk(path: str) -> List[Tuple[str, str, int]]:
    """eegloader readMarkerList: (type, description, position) in file order (:196)."""
    sec = ""
    out = []
    for raw in read_lines(path):
        line = raw.strip()
        if not line or line.startswith(";"):
            continue
        if line.startswith("["):
            sec = line.lower()
            continue
        if sec == "[marker infos]" and line.startswith("Mk") and "=" in line:
            f = line.split("=", 1)[1].split(",")
            out.append((f[0].replace("\\1", ","), f[1].replace("\\1", ","), int(f[2])))
    return out


def stimulus_index(desc: str) -> int:
    """OffLineDataProvider.java:207-214: replaceAll("[\\\\D]", "") then parseInt - 1, or -1."""
    d = re.sub(r"[^0-9]", "", desc)
    return java_parse_int(d) - 1 if d else -1


def plan_markers(markers, n_frames: int, guessed: int, balance: int):
    """OffLineDataProvider.java:200-265 for one file -> (positions, labels, balance)."""
    pos, lab = [], []
    for _typ, desc, p in markers:
        si = stimulus_index(desc)
        if p - PRE < 0 or p - PRE > n_frames:  # copyOfRange AIOOBE, caught :262-264
            continue
        target = si + 1 == guessed
        if target and balance <= 0:
            pos.append(p); lab.append(1.0); balance += 1
        elif (not target) and balance >= 0:
            pos.append(p); lab.append(0.0); balance -= 1
    return pos, lab, balance


def load_info_txt(path: str) -> Dict[str, int]:
    """loadFilesFromInfoTxt (:283-319); dict keeps LinkedHashMap insertion order."""
    files: Dict[str, int] = {}
    for line in read_lines(path):
        if len(line) == 0 or line[0] == "#":
            continue
        parts = java_split_space(line)
        if len(parts) > 1:
            try:
                files[parts[0]] = java_parse_int(parts[1])
            except JavaError:
                raise JavaError("IllegalArgumentException",
                                f"Line {line} contains an improper number format")
    return files


def data_provider(args: Sequence[str]):
    """OffLineDataProvider(args).loadData() -> (epochs[n][3][750], labels, positions, error).

    handleInput (:111-141), processEEGFiles (:147-268), setFileNames (:327-365); like loadData
    (:88-98) any exception stops loading and what was loaded is kept."""
    epochs: List[np.ndarray] = []
    labels: List[float] = []
    positions: List[int] = []
    error = ""
    idx = {"fz": 0, "cz": 0, "pz": 0}
    balance = 0
    try:
        if len(args) <= 0 or len(args) > 6:
            raise JavaError("IllegalArgumentException", "Please enter the input ...")
        loc = args[0]
        if len(loc) < 4:
            raise JavaError("StringIndexOutOfBoundsException", "")
        if loc[-4:] == ".eeg":
            prefix = ""
            if len(args) < 2:
                raise JavaError("ArrayIndexOutOfBoundsException", "1")
            files = {loc: java_parse_int(args[1])}
        elif loc[-4:] == ".txt":
            if "/" not in loc:
                raise JavaError("StringIndexOutOfBoundsException", "-1")
            prefix = loc[:loc.rindex("/")] + "/"
            files = load_info_txt(loc)
        else:
            raise JavaError("IllegalArgumentException", "Please enter the input ...")
        for key, guessed in files.items():
            path = prefix + key
            if len(path) <= 4 or path[-4:] != ".eeg":
                continue
            base = path[:path.rindex(".")]
            vhdr, vmrk = base + ".vhdr", base + ".vmrk"
            if not (os.path.isfile(vhdr) and os.path.isfile(vmrk) and os.path.isfile(path)):
                continue
            h = read_vhdr(vhdr)
            for num, name, _res in h["channels"]:
                n = name.lower()
                if n == "fz":
                    idx["fz"] = num
                elif n == "cz":
                    idx["cz"] = num
                if n == "pz":
                    idx["pz"] = num
            ct = h["n_channels"]
            dt = np.int16 if h["binary_format"] == "INT_16" else np.float32
            raw = np.fromfile(path, dtype="<" + np.dtype(dt).str[1:])
            raw = raw[: (raw.size // ct) * ct].reshape(-1, ct)
            sel = [idx["fz"], idx["cz"], idx["pz"]]
            if min(sel) < 1 or max(sel) > ct:
                raise JavaError("ChannelNotFound", str(sel))
            resmap = {num: r for num, _n, r in h["channels"]}
            cols = [s - 1 for s in sel]
            res = [resmap.get(s, 1.0) for s in sel]
            markers = read_vmrk(vmrk)
            # stimulus parse errors surface in marker order: plan up to the failing marker
            good, err = [], None
            for m in markers:
                try:
                    stimulus_index(m[1])
                except JavaError as ex:
                    err = ex
                    break
                good.append(m)
            pos, lab, balance = plan_markers(good, raw.shape[0], guessed, balance)
            if pos:
                epochs.extend(decode_epochs(raw, cols, res, pos))
            labels.extend(lab)
            positions.extend(pos)
            if err is not None:
                raise err
    except JavaError as ex:
        error = str(ex)
    ep = np.array(epochs) if epochs else np.zeros((0, 3, POST))
    return ep, labels, positions, error


# ---- reference-style checks ------------------------------------------------------------------------
def java_epoch_sum(epochs: np.ndarray) -> float:
    """OfflineDataProviderTest.java:71-80: per-row sums then total, in Java order."""
    total = 0.0
    for ep in epochs:
        for row in ep:
            rs = 0.0
            for v in row.tolist():
                rs += v
            total += rs
    return total


def java_feature_sum(features: np.ndarray) -> float:
    """FeatureExtractionTest.java:96-105: per-vector sums then total, in Java order."""
    total = 0.0
    for f in features:
        s = 0.0
        for v in f.tolist():
            s += v
        total += s
    return total
