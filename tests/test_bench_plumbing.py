"""bench.py's measurement plumbing on CPU: the algorithmic byte counts of SURVEY.md 8d and the
readers of the committed profiles that fill `roofline.traffic` and `roofline.ceiling` in the
bench line (the GPU side is timed on the box)."""
import json
import os

import numpy as np
import pytest

import bench
from conftest import REPO


def test_algorithmic_bytes_per_epoch():
    assert bench.bytes_per_epoch(3, 3) == 4064
    assert bench.bytes_per_epoch(32, 32) == 43272     # configs[3]
    # fma: levels 1-5 as the collapsed 280-tap filter (16 x 280 + 16 x 10 MAC per channel);
    # EXACT: the a-path cascade (5,120 MAC per channel)
    assert bench.FLOP_PER_SIGNAL["fma"] == 2 * (16 * 280 + 16 * 10)
    assert bench.FLOP_PER_SIGNAL["exact"] * 3 == 30720


def test_traffic_reader_takes_the_newest_summary():
    key = "fused_dwt8_c3_int16_1000000_fma"
    got = bench.traffic_from_profiles(key)
    assert got is not None and got["workload_key"] == key
    pdir = os.path.join(REPO, "profiles")
    names = sorted((f for f in os.listdir(pdir) if f.endswith(".json") and "traffic" in f and
                    json.load(open(os.path.join(pdir, f))).get("workload_key") == key),
                   key=bench.run_tag_order)
    assert names[-1].startswith("r06zz_")  # the newest run (round 6)
    assert got == json.load(open(os.path.join(pdir, names[-1])))
    # FETCH_SIZE x2 (gfx950) + WRITE_SIZE over the algorithmic 3,476 B per epoch: a few % over
    assert 1.0 <= got["hbm_bytes_per_launch"] / 3.476e9 < 1.1
    assert bench.traffic_from_profiles("no such workload") is None


def test_run_tags_order_like_spreadsheet_columns():
    tags = ["r03ab_x", "r02n_x", "r03k_x", "r03aa_x", "r03z_x", "r03h_x", "r01b_x"]
    assert sorted(tags, key=bench.run_tag_order) == [
        "r01b_x", "r02n_x", "r03h_x", "r03k_x", "r03z_x", "r03aa_x", "r03ab_x"]


def test_ceiling_reader_scales_to_the_launch():
    k = json.load(open(os.path.join(REPO, bench.CEILING_FILE)))["kernels"]["window_kernel<int16,3> fma"]
    c = bench.ceiling_from_profiles(3, "fma", 500_000, 0.5, 1_738_000_000)
    assert c["ms"] == pytest.approx(k["ceiling_ms"] * 500_000 / k["epochs_per_launch"], abs=1e-4)
    assert c["frac"] == pytest.approx(1.738e9 / (c["ms"] * 1e-3) / 8e12, rel=1e-3)
    assert c["kernel_over_ceiling"] == pytest.approx(c["ms"] / 0.5, rel=1e-3)
    assert 0.5 < c["frac"] < 0.8            # the measured power-capped bound, not HBM's 1.0
    assert bench.ceiling_from_profiles(3, "exact", 1, 1.0, 1) is None
    assert bench.ceiling_from_profiles(7, "fma", 1, 1.0, 1) is None


def test_whole_path_ceiling_adds_the_baseline_pass():
    d = json.load(open(os.path.join(REPO, bench.CEILING_FILE)))
    b = d["baseline_kernel<int16,3>"]["ms_alone"]
    w = d["kernels"]["window_kernel<int16,3> fma"]["ceiling_ms"]
    c = bench.whole_path_ceiling(3, "fma", 1_000_000, 1.0, 4064)
    assert c["ms"] == pytest.approx(b + w, abs=1e-4)
    assert c["frac"] == pytest.approx(4.064e9 / ((b + w) * 1e-3) / 8e12, rel=1e-3)
    assert 0.5 < c["frac"] < 0.8
    # configs[3]: baseline_any_kernel's measured time + the 32-channel window kernel's bound
    b32 = d["baseline_any_kernel<int16> c32"]
    w32 = d["kernels"]["window_c32_kernel fma"]
    n = w32["epochs_per_launch"]
    c32 = bench.whole_path_ceiling(32, "fma", n, 2.0, 43272)
    assert c32["ms"] == pytest.approx(b32["ms_alone"] * n / b32["epochs_per_launch"]
                                      + w32["ceiling_ms"], abs=1e-4)
    assert 0.5 < c32["frac"] < 0.9
    assert bench.whole_path_ceiling(16, "fma", 1, 1.0, 1) is None
    assert bench.whole_path_ceiling(3, "exact", 1, 1.0, 1) is None


def test_watchdog_reports_the_line_and_exits_when_a_phase_hangs():
    """A multi-rank phase that never returns (a gather stuck in RCCL) must not cost the extraction
    line: rank 0 prints it with the phase's error and the process exits 0."""
    import subprocess
    import sys
    code = ("import sys, time; sys.path.insert(0, %r); import bench\n"
            "w = bench._Watchdog(); w.arm(0.5, {'metric': 'm', 'value': 1.0}, 'gather hung')\n"
            "time.sleep(30)\n") % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=20)
    assert r.returncode == 0
    line = json.loads(r.stdout.strip())
    assert line["value"] == 1.0 and line["gather"]["error"] == "gather hung"


def test_watchdog_disarmed_phase_does_not_fire():
    import time
    w = bench._Watchdog()
    w.arm(0.2, None, "teardown")
    w.disarm()
    time.sleep(0.4)  # still alive: the timer was cancelled


def test_gather_row_checksum_detects_misplaced_shards():
    """bench.py's gather legs compare every shard on the root with its rank's own checksum
    (unit norms alone pass a misplaced or duplicated shard)."""
    import torch
    rng = np.random.default_rng(3)
    shards = [torch.from_numpy(rng.standard_normal((50, 48))) for _ in range(3)]
    sums = [bench.row_checksum(s) for s in shards]
    full = torch.cat(shards)
    assert [bench.row_checksum(full[r * 50:(r + 1) * 50]) for r in range(3)] == sums
    swapped = torch.cat([shards[1], shards[0], shards[2]])
    assert bench.row_checksum(swapped[:50]) != sums[0]
    dup = torch.cat([shards[0], shards[0], shards[2]])
    assert bench.row_checksum(dup[50:100]) != sums[1]
    rows = shards[2].clone()
    rows[[3, 4]] = rows[[4, 3]]                       # two rows exchanged inside a shard
    assert bench.row_checksum(rows) != sums[2]


def test_live_energy_leg_arithmetic():
    """whole_path.energy: step energy from the accumulator over the untimed steps, the bound
    step_J / cap and its ratio to the timed step (a stand-in meter: 1.4 kW drawn, cap 1.4 kW)."""
    import time as _time

    class FakeTorch:
        class cuda:
            @staticmethod
            def synchronize(dev):
                pass

    class Meter:
        ok = True
        j = 0.0

        def joules(self):
            return self.j

        def cap_w(self):
            return 1400.0

    m = Meter()

    def step():   # each step: 0.88 ms of wall time at 1.4 kW
        m.j += 1400.0 * 0.88e-3
        _time.sleep(0.0)

    e = bench.energy_leg(m, FakeTorch, None, step, 0.88, 1_000_000, 4064, min_ms=10.0)
    assert e["available"] and e["steps"] >= 10
    assert abs(e["step_J"] - 1.232) < 1e-9
    assert abs(e["bound_ms"] - 0.88) < 1e-4 and abs(e["step_over_bound"] - 1.0) < 1e-3
    assert abs(e["frac_at_bound"] - 4064e6 / 0.88e-3 / 8e12) < 1e-3
    off = bench.energy_leg(None, FakeTorch, None, step, 0.88, 1, 4064)
    assert off["available"] is False
