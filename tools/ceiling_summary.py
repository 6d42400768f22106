#!/usr/bin/env python3
"""The attainable bound of the window kernels and of the whole step, from one power study
(tools/power_study.sh with PMC=1 for c3 and c32, plus tools/baseline_power.sh, one GPU box).

  python3 tools/ceiling_summary.py <power dir> <out.json>

Method: every VALU instruction of these kernels occupies its SIMD four cycles
(SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU = 1.00), so the VALU issue time of a launch is
SQ_INSTS_VALU x 4 / 1,024 SIMDs / the shader clock the chip holds under the kernel's own sustained
load (mean of the eight XCD clocks amd-smi reports mid-run).  The kernel cannot finish before its
VALU work has issued, and under load it sits at the 1.4 kW socket cap, which sets that clock.
The whole step adds baseline_kernel, which runs below the cap at full clock and is bound by its
memory pattern: its ceiling is its own measured time.
"""
import glob
import json
import os
import re
import sys

SIMDS = 256 * 4
HBM_PEAK = 8.0e12
KERNELS = {  # workload -> (name, epochs per launch, algorithmic bytes per launch)
    "c3": ("window_kernel<int16,3> fma", 1_000_000, 3476 * 1_000_000),
    "c32": ("window_c32_kernel fma", 250_000, 37000 * 250_000),
}
STEP_BYTES_C3 = 4064 * 1_000_000  # the whole path, 3-channel int16


def smi(path):
    txt = open(path).read()
    watts = float(re.search(r"SOCKET_POWER:\s*([\d.]+)\s*W", txt).group(1))
    clocks = [float(m) for m in re.findall(r"GFX_\d+:\s*\n\s*CLK:\s*([\d.]+)\s*MHz", txt)]
    return watts, sum(clocks) / len(clocks), clocks


def probe_ms(path):
    return float(re.search(r"([\d.]+) ms per launch", open(path).read()).group(1))


def counters(d):
    tot = {}
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        import csv
        per = {}
        for r in csv.DictReader(open(f)):
            k = (r["Dispatch_Id"], r["Counter_Name"])
            per[k] = per.get(k, 0.0) + float(r["Counter_Value"])
        for (disp, c), v in per.items():
            tot.setdefault(c, []).append(v)
    return {c: sorted(v)[len(v) // 2] for c, v in tot.items()}


def main():
    src, out = sys.argv[1], sys.argv[2]
    res = {"what": "Attainable bound of the window kernels (VALU issue at the power-capped clock) "
                   "and of the whole c3 step (baseline_kernel at its own measured time + the "
                   "window kernel's bound); tools/ceiling_summary.py over " + src,
           "method": __doc__.split("Method (DESIGN.md §5.1): ")[1].strip(),
           "kernels": {}}
    for wl, (name, n, nbytes) in KERNELS.items():
        if not os.path.exists(f"{src}/window_probe_{wl}.txt"):
            continue
        watts, mhz, clocks = smi(f"{src}/window_probe_{wl}_smi.txt")
        ms = probe_ms(f"{src}/window_probe_{wl}.txt")
        c = {}
        for d in sorted(glob.glob(f"{src}/pmc_{wl}_*")):
            if os.path.isdir(d):
                c.update(counters(d))
        valu = c["SQ_INSTS_VALU"]
        ceil_ms = valu * 4 / SIMDS / (mhz * 1e6) * 1e3
        res["kernels"][name] = {
            "epochs_per_launch": n, "algorithmic_bytes_per_launch": nbytes,
            "SQ_INSTS_VALU": valu, "SQ_ACTIVE_INST_VALU": c.get("SQ_ACTIVE_INST_VALU"),
            "SQ_INSTS_VALU_FMA_F64": c.get("SQ_INSTS_VALU_FMA_F64"),
            "SQ_INSTS_VALU_CVT": c.get("SQ_INSTS_VALU_CVT"), "SQ_WAVES": c.get("SQ_WAVES"),
            "valu_instr_per_wave": round(valu / c["SQ_WAVES"], 1),
            "clock_MHz_under_load": round(mhz), "xcd_clocks_MHz": clocks, "socket_W": watts,
            "kernel_ms_sustained": ms, "ceiling_ms": round(ceil_ms, 4),
            "hbm_frac_at_ceiling": round(nbytes / (ceil_ms * 1e-3) / HBM_PEAK, 4),
            "kernel_over_ceiling": round(ceil_ms / ms, 4)}
    if os.path.exists(f"{src}/baseline.txt"):
        watts, mhz, _ = smi(f"{src}/baseline_smi.txt")
        bms = probe_ms(f"{src}/baseline.txt")
        w = res["kernels"].get(KERNELS["c3"][0])
        res["baseline_kernel<int16,3>"] = {"ms_alone": bms, "socket_W": watts,
                                           "clock_MHz": round(mhz)}
        if w:
            step = bms + w["ceiling_ms"]
            res["whole_path_c3"] = {
                "ceiling_ms": round(step, 4), "bytes_per_epoch": 4064,
                "hbm_frac_at_ceiling": round(STEP_BYTES_C3 / (step * 1e-3) / HBM_PEAK, 4),
                "measured_ms_sustained": round(bms + w["kernel_ms_sustained"], 4)}
    if os.path.exists(f"{src}/step.txt") and os.path.exists(f"{src}/baseline.txt"):
        # the per-step energy budget: at the 1.4 kW socket cap a step cannot take
        # less than its energy / 1,400 W; the energies of the two passes from their own sustained
        # runs (watts x launch time), against the step measured back to back
        sw, smhz, _ = smi(f"{src}/step_smi.txt")
        sms = probe_ms(f"{src}/step.txt")
        bw, _, _ = smi(f"{src}/baseline_smi.txt")
        bms = probe_ms(f"{src}/baseline.txt")
        w = res["kernels"].get(KERNELS["c3"][0])
        if w:
            e_base = bw * bms * 1e-3
            e_win = w["socket_W"] * w["kernel_ms_sustained"] * 1e-3
            t_min = (e_base + e_win) / 1400.0 * 1e3
            res["energy_budget_c3"] = {
                "baseline_J": round(e_base, 4), "window_J_at_cap": round(e_win, 4),
                "step_J_measured": round(sw * sms * 1e-3, 4), "step_W": sw,
                "step_clock_MHz": round(smhz), "step_ms_sustained": sms,
                "min_step_ms_at_1400W": round(t_min, 4),
                "whole_path_frac_at_energy_bound": round(STEP_BYTES_C3 / (t_min * 1e-3) / HBM_PEAK, 4),
                "step_ms_for_frac_0.60": round(STEP_BYTES_C3 / (0.6 * HBM_PEAK) * 1e3, 4)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1)[:3000])


if __name__ == "__main__":
    main()
