"""Socket power of the bench's GPU with nothing running, and with back-to-back tiny kernels (clocks
up, almost no work), from the SMU's energy accumulator -- how much of the baseline pass's 1.24 kW
(0.174 J over 0.14 ms, profiles/r05_ceiling.json) is the chip being on rather than its work.
    python3 tools/probes/idle_power.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402  (EnergyMeter only)

dev = torch.device("cuda:0")
m = bench.EnergyMeter(torch, 0)
if not m.ok:
    print("energy meter unavailable:", m.why)
    sys.exit(0)
x = torch.zeros(64, device=dev)
torch.cuda.synchronize()


def watts(fn, secs=0.6):
    torch.cuda.synchronize()
    j0, t0 = m.joules(), time.perf_counter()
    while time.perf_counter() - t0 < secs:
        fn()
    torch.cuda.synchronize()
    j1, t1 = m.joules(), time.perf_counter()
    return (j1 - j0) / (t1 - t0)


def tiny():
    for _ in range(200):
        x.add_(1.0)


def big():
    y = torch.empty(1 << 28, dtype=torch.uint8, device=dev)
    for _ in range(4):
        y.fill_(1)


print(f"cap {m.cap_w():.0f} W")
for label, fn in (("idle (host sleeps)", lambda: time.sleep(0.01)), ("tiny kernels back to back", tiny),
                  ("idle again", lambda: time.sleep(0.01)), ("HBM fill 256 MB x4", big),
                  ("tiny kernels again", tiny)):
    print(f"{label:28s} {watts(fn):7.1f} W")
