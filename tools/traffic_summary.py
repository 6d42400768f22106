#!/usr/bin/env python3
"""HBM traffic per launch of one kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

    python tools/traffic_summary.py --fetch DIR --write DIR --kernel window_kernel \
        --workload-key fused_dwt8_c3_int16_1000000_fma --out profiles/r02c_traffic_fma.json

Corrections (MI355X_MICROARCH.md, "HBM"): both counters are in KiB; on gfx950 FETCH_SIZE reports
half the bytes of a wide (16 B/lane) streaming read, so it is doubled; WRITE_SIZE is exact for
16 B/lane streaming stores.  The window_kernel reads the recording with 16 B/lane LDS-DMA
(global_load_lds_dwordx4) and writes features with 16 B/lane stores, the calibrated widths.
"""
import argparse
import csv
import glob
import json
import os
import statistics


def per_dispatch(d, counter, kernel):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter or kernel not in row["Kernel_Name"]:
                    continue
                key = (f, row["Dispatch_Id"])
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel} under {d}")
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", default="window_kernel")
    ap.add_argument("--workload-key", required=True)
    ap.add_argument("--algorithmic-bytes", type=int, default=0)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fetch = per_dispatch(a.fetch, "FETCH_SIZE", a.kernel)
    write = per_dispatch(a.write, "WRITE_SIZE", a.kernel)
    fetch_kib, write_kib = statistics.median(fetch), statistics.median(write)
    total = 2 * fetch_kib * 1024 + write_kib * 1024
    d = {
        "workload_key": a.workload_key,
        "kernel": a.kernel,
        "dispatches": {"fetch": len(fetch), "write": len(write)},
        "FETCH_SIZE_kib_median": fetch_kib,
        "WRITE_SIZE_kib_median": write_kib,
        "read_bytes_per_launch": 2 * fetch_kib * 1024,
        "write_bytes_per_launch": write_kib * 1024,
        "hbm_bytes_per_launch": total,
        "correction": "FETCH_SIZE x2 (gfx950 wide-read half count), both KiB -> bytes",
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, "
                  "--kernel-include-regex " + a.kernel,
    }
    if a.algorithmic_bytes:
        d["algorithmic_bytes_per_launch"] = a.algorithmic_bytes
        d["traffic_over_algorithmic"] = round(total / a.algorithmic_bytes, 4)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(d, fh, indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
