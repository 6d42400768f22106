"""Slowest HIP runtime calls in a rocprofv3 --hip-trace CSV (the drop-in's multi-thread stalls).

    python3 tools/probes/api_stalls.py DIR/run_hip_api_trace.csv [threshold_us] [skip,functions]

Prints, per API function, the call count and how many took longer than the threshold, then the
40 slowest calls with their thread and start time (relative to the first call), and for each of
the 5 slowest the calls of other threads that overlap it by more than half the threshold.
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    thr = float(sys.argv[2]) if len(sys.argv) > 2 else 500.0
    skip = set(sys.argv[3].split(",")) if len(sys.argv) > 3 else set()
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            rows.append((r["Function"], int(r["Thread_Id"]), t0, t1))
    if not rows:
        print("no rows")
        return
    base = min(r[2] for r in rows)
    per = defaultdict(lambda: [0, 0, 0.0])
    for fn, _, t0, t1 in rows:
        d = (t1 - t0) / 1e3
        p = per[fn]
        p[0] += 1
        p[1] += d > thr
        p[2] = max(p[2], d)
    print(f"{len(rows)} calls; per function: count, over {thr:.0f} us, max us")
    for fn, (n, over, mx) in sorted(per.items(), key=lambda kv: -kv[1][2])[:25]:
        print(f"  {fn:40s} {n:8d} {over:6d} {mx:10.1f}")
    slow = sorted((r for r in rows if r[0] not in skip), key=lambda r: r[2] - r[3])[:40]
    print("slowest calls: function, thread, start ms, us")
    for fn, tid, t0, t1 in slow:
        print(f"  {fn:40s} {tid:8d} {(t0 - base) / 1e6:10.3f} {(t1 - t0) / 1e3:9.1f}")
    for fn, tid, t0, t1 in slow[:5]:
        ov = [r for r in rows if r[1] != tid and min(t1, r[3]) - max(t0, r[2]) > thr * 500]
        print(f"overlapping {fn} of thread {tid} at {(t0 - base) / 1e6:.3f} ms: {len(ov)} calls")
        for r in sorted(ov, key=lambda r: r[2])[:16]:
            print(f"    {r[0]:40s} {r[1]:8d} {(r[2] - base) / 1e6:10.3f} {(r[3] - r[2]) / 1e3:9.1f}")


def around(path, err_path, min_us=50.0):
    """For each slowest call that dropin_bench reported (stderr: tid, at_ns, duration), the runtime
    calls of every thread overlapping it that took more than min_us, and the stalled thread's own."""
    import re
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            rows.append((r["Function"], int(r["Thread_Id"]), int(r["Start_Timestamp"]),
                         int(r["End_Timestamp"])))
    pat = re.compile(r"(\w+) threads (\d+) slowest #(\d+): ([\d.]+) us .*tid (\d+) at_ns (\d+)")
    for line in open(err_path):
        m = pat.search(line)
        if not m:
            continue
        leg, T, rank, dur, tid, at = m.groups()
        t0 = int(at)
        t1 = t0 + int(float(dur) * 1e3)
        print(f"== {leg} T{T} #{rank}: {dur} us, tid {tid}")
        for fn, th, a, b in sorted(rows, key=lambda r: r[2]):
            if min(t1, b) - max(t0, a) <= 0:
                continue
            if th == int(tid) or (b - a) / 1e3 > min_us:
                print(f"    {'*' if th == int(tid) else ' '} {fn:32s} {th:8d} {(a - t0) / 1e3:9.1f} {(b - a) / 1e3:9.1f}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--around":
        around(sys.argv[2], sys.argv[3])
    else:
        main()
