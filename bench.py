#!/usr/bin/env python3
"""Benchmark of the epoch-to-feature hot path (BASELINE.json metric, configs[1] per GPU).

One step = one pass of the fused raw -> dwt-8 feature kernels over one batch of synthetic epochs
(3 channels, multiplexed int16 @ 1000 Hz, one marker every 1000 frames), inputs already resident
in HBM: 1,000,000 epochs at N = 1 (configs[1]); at N > 1 every rank (torch.distributed, RCCL)
extracts its own 8,000,000-epoch shard, so N = 8 is configs[2]'s 64M epochs (weak scaling:
epochs are independent, no data-path collective).  The feature gather to rank 0 is timed after
the extraction steps and reported beside `value` (`gather`, `extract_plus_gather`).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--numerics exact|fma]

Rank 0 prints ONE JSON line (see DESIGN.md "Measurement").  Extra legs:
  roofline      the dominant kernel (window_kernel): its algorithmic bytes per launch / its
                average launch duration, measured with HIP events that the context records on
                the stream the kernel runs on, against 8.0 TB/s (MI355X_MICROARCH.md); traffic =
                HBM bytes per launch from the committed rocprofv3 PMC summary (else null);
  cpu_baseline  the C restatement (oracle/, reference-faithful full pyramid) timed on the host
                cores on a bounded sample of the same workload (rank 0's shard; at N > 1 after
                the gather legs).
"""
import argparse
import json
import os
import re
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "epochs/sec feature-extracted (whole node) + % HBM roofline, 1/2/4/8 GPUs"


def bytes_per_epoch(ct, C):
    """Whole-path algorithmic bytes: 612 frames in + 8 B marker + 16*C doubles out
    (3 ch: 4,064 B; 32 ch: 43,272 B)."""
    return 612 * ct * 2 + 8 + 16 * C * 8


HBM_PEAK_GBS = 8000.0                          # MI355X_MICROARCH.md: 8.0 TB/s spec
FP64_VECTOR_PEAK_TFS = 78.6                    # vendor fp64 vector spec (not in the guide)
FP64_FMA_MEASURED_TFS = 55.8                   # v_fma_f64 probe on this part (git show c3ab853:profiles/r01/r01b_perf_study.json)
# fp64 filter-bank flops per channel: fma numerics run levels 1-5 as the collapsed 280-tap filter
# (16 x 280 + level 6's 16 x 10 = 4,640 MAC, dwt8.h), EXACT the level-by-level a-path cascade
# (5,120 MAC)
FLOP_PER_SIGNAL = {"fma": 2 * 4640, "exact": 2 * 5120}
FRAMES_PER_EPOCH = 1000                        # one marker per second at 1000 Hz
SEED = 0x5EED
WINDOW_KERNEL = "window_kernel<int16,3>"
WORKLOADS = {
    "c3": {"ct": 3, "C": 3, "desc": "configs[1]: synthetic 1M epochs x 3 ch (Fz/Cz/Pz) multiplexed "
                                    "int16 @1000 Hz -> fe=dwt-8 48-dim L2-normalised features, per GPU"},
    "c3dist": {"ct": 3, "C": 3, "desc": "configs[2]: synthetic multiplexed int16 recordings, "
                                        "3 ch (Fz/Cz/Pz) @1000 Hz, epoch-sharded over the GPUs, "
                                        "8M epochs per rank (64M over 8xMI355X) -> fe=dwt-8 "
                                        "48-dim L2-normalised features"},
    "c32": {"ct": 32, "C": 32, "desc": "configs[3]: synthetic epochs x full 32-channel montage, "
                                       "multiplexed int16 @1000 Hz, every channel through the DWT -> "
                                       "512-dim L2-normalised features, per GPU"},
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=50,
                    help="untimed steps; ~50 ms of sustained load brings the clocks to their steady (power-capped) state")
    ap.add_argument("--epochs", type=int, default=None,
                    help="epochs per GPU per step (default: 1,000,000 = configs[1] at N = 1; "
                         "8,000,000 per rank = configs[2]'s 64M epochs over 8 GPUs when N > 1)")
    ap.add_argument("--workload", choices=["c3", "c32", "stream", "dropin", "logreg", "svm"],
                    default="c3",
                    help="c3: configs[1] (Fz/Cz/Pz, 48-dim, the headline); c32: configs[3] (full "
                         "32-channel montage, every channel through the DWT, 512-dim); stream: "
                         "configs[4] (4 h recordings in pinned host memory, a marker every 100 ms, "
                         "streamed to the device in chunks); dropin: configs[0]'s per-epoch "
                         "IFeatureExtraction calls and the info.txt flow through the C ABI "
                         "(latency, per calling thread); logreg: the downstream classifier "
                         "(MLlib LogisticRegressionWithSGD, 100 full-batch iterations) on the 1M "
                         "48-dim feature rows of c3; svm: the same with SVMWithSGD")
    ap.add_argument("--chunk-frames", type=int, default=1 << 23, help="stream workload chunk")
    ap.add_argument("--spacing", type=int, default=FRAMES_PER_EPOCH,
                    help="c3/c32: frames between markers (default 1000, the headline; < 687 makes "
                         "windows overlap and the window DMA cached instead of streaming)")
    ap.add_argument("--lib", default=None,
                    help="study only: another build of libeegfx.so to load (A/B of library builds)")
    ap.add_argument("--numerics", choices=["exact", "fma"], default="fma",
                    help="fma: fused filter bank (<=1e-9 of the reference, the north_star bound); "
                         "exact: the reference's operation order, bit-identical")
    ap.add_argument("--alt-steps", type=int, default=10,
                    help="steps of a second, untimed-for-value pass in the other numerics mode "
                         "(reported under 'alt_numerics'; 0 disables)")
    ap.add_argument("--cpu-sample", type=int, default=500_000,
                    help="epochs in the CPU-baseline sample (0 disables)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0: every available host core (affinity, capped by a cgroup CPU quota)")
    ap.add_argument("--no-gather", action="store_true", help="skip the RCCL feature gather legs")
    ap.add_argument("--settle-ms", type=float, default=100.0,
                    help="untimed steps after the warmup for at least this much wall time, so the "
                         "timed steps start past the clock's power-cap transient (reported as "
                         "config.settle; DESIGN.md §7); 0 disables")
    ap.add_argument("--plant", default=None, metavar="KIND:RATE",
                    help="c3 study only (DESIGN.md §3.1): overwrite the spans [pos-100, pos+750) of "
                         "a fraction RATE of the markers, evenly spread, with 'flat' (constant "
                         "samples, the flat stretch of DoD2015_01: certified by the guard's second "
                         "stage) or 'null' (a Nyquist-alternating +-1000-count signal on the DC "
                         "level, in the filters' null space: recomputed under EXACT) windows")
    ap.add_argument("--trace-steps", action="store_true",
                    help="study only: device time of every warmup and timed step (HIP events "
                         "between steps), reported under 'step_trace'")
    ap.add_argument("--gather-timeout", type=float, default=300.0,
                    help="seconds the gather legs may take before rank 0 reports the extraction "
                         "line without them and every rank exits")
    ap.add_argument("--dist-backend", default="nccl",
                    help="rehearsal only: 'gloo' runs the N>1 control flow without RCCL")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal only: every rank uses cuda:0 (a one-GPU box)")
    ap.add_argument("--force-dist", action="store_true",
                    help="rehearsal only: run the N>1 code path (process group, C-ABI gather) "
                         "even with one rank")
    return ap.parse_args()


def run_tag_order(name):
    """Order of the run tags that prefix profiles/ files: r<round><letters>, the letters counted
    like spreadsheet columns (r03z < r03aa < r03ab), so the newest run sorts last."""
    m = re.match(r"r(\d+)([a-z]*)", name)
    if not m:
        return (-1, 0, name)
    return (int(m.group(1)), len(m.group(2)), m.group(2))


def traffic_from_profiles(workload_key):
    """HBM bytes per launch from the committed PMC summary (profiles/*traffic*.json): the newest
    run's file for the workload."""
    best = None
    pdir = os.path.join(REPO, "profiles")
    if not os.path.isdir(pdir):
        return None
    for f in sorted(os.listdir(pdir), key=run_tag_order):
        if f.endswith(".json") and "traffic" in f:
            try:
                d = json.load(open(os.path.join(pdir, f)))
            except Exception:
                continue
            if d.get("workload_key") == workload_key and d.get("hbm_bytes_per_launch"):
                best = d
    return best


CEILING_FILE = os.path.join("profiles", "r05_ceiling.json")


def ceiling_from_profiles(C, numerics, n, kernel_ms, kernel_bytes):
    """The attainable bound of the dominant kernel (profiles/r05_ceiling.json, written by
    tools/ceiling_summary.py): its VALU issue time at the clock the chip holds under the kernel's
    own sustained power draw (SQ counters + amd-smi under load), scaled to this launch's epochs,
    next to the live kernel time."""
    if numerics != "fma":
        return None
    key = {3: "window_kernel<int16,3> fma", 32: "window_c32_kernel fma"}.get(C)
    try:
        k = json.load(open(os.path.join(REPO, CEILING_FILE)))["kernels"][key]
    except Exception:
        return None
    ms = k["ceiling_ms"] * n / k["epochs_per_launch"]
    return {"bound": "VALU issue at the power-capped clock (1.4 kW socket cap)",
            "ms": round(ms, 4),
            "frac": round(kernel_bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "kernel_over_ceiling": round(ms / kernel_ms, 4),
            "valu_instr_per_wave": k["valu_instr_per_wave"],
            "clock_MHz_under_load": k["clock_MHz_under_load"],
            "source": CEILING_FILE}


def whole_path_ceiling(C, numerics, n, step_ms, bpe):
    """The attainable bound of the whole step: the baseline pass at its own measured time (it
    runs below the power cap, bound by its memory pattern) plus the window kernel's VALU bound,
    scaled to this launch's epochs (profiles/r05_ceiling.json): the c3 step (baseline_kernel +
    window_kernel) and the configs[3] step (baseline_any_kernel + window_c32_kernel).  For c3 also
    the energy bound: the step's measured energy (baseline pass below the cap + window kernel at
    the cap) over the 1.4 kW cap, the shortest step this instruction stream allows."""
    if numerics != "fma" or C not in (3, 32):
        return None
    try:
        d = json.load(open(os.path.join(REPO, CEILING_FILE)))
        if C == 3:
            base = d["baseline_kernel<int16,3>"]
            b = base["ms_alone"] * n / base.get("epochs_per_launch", 1_000_000)
            w = d["kernels"]["window_kernel<int16,3> fma"]
        else:
            base = d["baseline_any_kernel<int16> c32"]
            b = base["ms_alone"] * n / base["epochs_per_launch"]
            w = d["kernels"]["window_c32_kernel fma"]
    except Exception:
        return None
    ms = b + w["ceiling_ms"] * n / w["epochs_per_launch"]
    out = {"ms": round(ms, 4), "frac": round(n * bpe / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "step_over_ceiling": round(ms / step_ms, 4),
           "baseline_kernel_ms_alone": b, "source": CEILING_FILE}
    e = d.get("energy_budget_c3") if C == 3 else None
    if e:
        ems = e["min_step_ms_at_1400W"] * n / w["epochs_per_launch"]
        out["energy_bound"] = {"ms": round(ems, 4),
                               "frac": round(n * bpe / (ems * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                               "step_over_bound": round(ems / step_ms, 4),
                               "step_J": e["step_J_measured"], "cap_W": e["step_W"],
                               "measured_on": "the box of " + CEILING_FILE + " (this box: "
                                              "whole_path.energy)"}
    return out


class EnergyMeter:
    """Socket energy of the bench's GPU, read from the SMU's energy accumulator (amdsmi, read-only:
    no setting changes), and the socket power cap.  Unavailable (no amdsmi, no permission, device
    not matched by PCI address) -> ok False and `why` says so; the bench line then carries null."""

    def __init__(self, torch, dev_index):
        self.h, self.why, self.smi = None, None, None
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            self.smi = amdsmi
            p = torch.cuda.get_device_properties(dev_index)
            want = (int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id))
            for h in amdsmi.amdsmi_get_processor_handles():
                dom, bus, devfn = amdsmi.amdsmi_get_gpu_device_bdf(h).split(":")
                if (int(dom, 16), int(bus, 16), int(devfn.split(".")[0], 16)) == want:
                    self.h = h
                    break
            if self.h is None:
                self.why = f"no amdsmi device at PCI {want}"
            else:
                self.joules()
        except Exception as e:  # reported, never fatal
            self.h, self.why = None, repr(e)[:200]

    @property
    def ok(self):
        return self.h is not None

    def joules(self):
        e = self.smi.amdsmi_get_energy_count(self.h)
        return e["energy_accumulator"] * e["counter_resolution"] * 1e-6

    def cap_w(self):
        c = self.smi.amdsmi_get_power_cap_info(self.h)["power_cap"]
        return c / 1e6 if c > 1e5 else float(c)  # microwatts on this stack


def energy_leg(meter, torch, dev, step, step_ms, n, bpe, min_ms=300.0):
    """The live energy bound of the step: untimed steps after the timed region,
    for at least min_ms, bracketed by the socket's energy accumulator.  A step cannot be shorter
    than its energy over the socket power cap, so bound_ms = step_J / cap_W, and step_over_bound =
    bound_ms / step_ms (the timed step) = the power drawn as a fraction of the cap: near 1 means the
    step is energy-bound at the cap on this box, and only less energy per epoch makes it faster."""
    if meter is None or not meter.ok:
        return {"available": False, "why": getattr(meter, "why", "not measured")}
    k = max(10, int(min_ms / max(step_ms, 1e-3)))
    torch.cuda.synchronize(dev)
    j0, t0 = meter.joules(), time.perf_counter()
    for _ in range(k):
        step()
    torch.cuda.synchronize(dev)
    j1, t1 = meter.joules(), time.perf_counter()
    cap = meter.cap_w()
    e = (j1 - j0) / k
    bound_ms = e / cap * 1e3
    return {"available": True, "steps": k, "step_J": round(e, 5),
            "mean_W": round((j1 - j0) / (t1 - t0), 1), "cap_W": round(cap, 1),
            "bound_ms": round(bound_ms, 4),
            "frac_at_bound": round(n * bpe / (bound_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "step_over_bound": round(bound_ms / step_ms, 4),
            "source": "amdsmi energy accumulator over the untimed steps after the timed region"}


_JSON_OUT = None


def emit(line):
    """Prints the one JSON line on the process's original stdout (fd 1 at start-up)."""
    out = _JSON_OUT or sys.stdout
    print(json.dumps(line), file=out, flush=True)


def _stdout_to_stderr():
    """Everything else written to fd 1 -- RCCL's version banner at communicator creation, runtime
    chatter -- goes to stderr, so stdout carries exactly the bench line."""
    global _JSON_OUT
    sys.stdout.flush()
    _JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)


def main():
    args = parse()
    _stdout_to_stderr()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus > 1 must be launched with torch.distributed.run")
    distributed = world > 1 or args.force_dist
    dev = torch.device("cuda", 0 if args.same_device else local)
    torch.cuda.set_device(dev)
    if distributed:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    if args.lib:
        from eeg_dataanalysispackage_amd import _lib
        _lib.LIB_PATH = os.path.abspath(args.lib)
    import eeg_dataanalysispackage_amd as fx

    if args.workload == "stream":
        return bench_stream(args, rank, world, dev, dist if distributed else None)
    if args.workload == "dropin":
        return bench_dropin(args, rank, world, dev, dist if distributed else None)
    if args.workload in ("logreg", "svm"):
        return bench_logreg(args, rank, world, dev, dist if distributed else None)
    wl = WORKLOADS[args.workload]
    if args.workload == "c3" and distributed:
        wl = WORKLOADS["c3dist"]  # the N > 1 line is configs[2]: 8M epochs per rank
    ct, C = wl["ct"], wl["C"]
    if args.epochs is None:
        if args.workload == "c32":
            args.epochs = 250_000  # 16 GB recording + 1 GB of 512-dim features per GPU
        elif distributed:
            args.epochs = 8_000_000  # 48 GB recording + 3.07 GB of features per rank
        else:
            args.epochs = 1_000_000
    n = args.epochs
    if args.workload == "c3" and not distributed and n == 8_000_000:
        wl = dict(WORKLOADS["c3dist"], desc="configs[2]: one rank's 8M-epoch shard on one GPU "
                                            "(synthetic multiplexed int16, 3 ch @1000 Hz, 48 GB "
                                            "recording) -> fe=dwt-8 48-dim L2-normalised features")
    elif args.workload == "c3" and not distributed and n != 1_000_000:
        wl = dict(wl, desc=wl["desc"].replace("1M epochs", f"{n} epochs (not the configs[1] size)"))
    sp = args.spacing
    if sp < 100:
        raise SystemExit("--spacing must be >= 100 frames")
    n_frames = sp * n + 2000
    ctx = fx.Context(dev.index, numerics=args.numerics)
    meter = EnergyMeter(torch, dev.index)
    # A dedicated (non-null) torch stream shared with the context: the kernels run on it, so the
    # HIP events recorded on it bracket exactly the launches of the timed region.
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)

    raw = torch.empty((n_frames, ct), dtype=torch.int16, device=dev)
    ctx.synth_recording(raw, ct, SEED + rank)
    pos = torch.arange(sp, sp * (n + 1), sp, dtype=torch.int64, device=dev)
    out = torch.empty((n, 16 * C), dtype=torch.float64, device=dev)
    cols, res = list(range(C)), [0.1] * C
    planted = plant_windows(torch, raw, pos, args.plant) if args.plant else None

    def step():
        ctx.process_recording(raw, ct, cols, res, pos, out=out)

    trace = {"warmup": [], "timed": []} if args.trace_steps else None
    ctx.guard_stats(reset=True)

    def traced(k, key):
        if trace is None:
            for _ in range(k):
                step()
            return
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(k + 1)]
        evs[0].record(stream)
        for i in range(k):
            step()
            evs[i + 1].record(stream)
        trace[key] = evs

    traced(args.warmup, "warmup")
    torch.cuda.synchronize(dev)
    # Settle: the first ~25 launches after idle run at a clock that first overshoots, then sinks
    # below and recovers to the power-capped steady state (step trace, git show c3ab853:profiles/r04c/driver_gap);
    # a short --warmup would otherwise time that transient.  Reported, not counted as warmup.
    settle_steps, s0 = 0, time.perf_counter()
    while (time.perf_counter() - s0) * 1e3 < args.settle_ms:
        for _ in range(10):
            step()
        settle_steps += 10
        torch.cuda.synchronize(dev)
    settle_ms = (time.perf_counter() - s0) * 1e3
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)

    ctx.guard_detail(reset=True)  # the guard counters then cover exactly the timed steps
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ctx.set_timing(True)  # HIP events around each window_kernel launch, on the context stream
    t0 = time.perf_counter()
    ev0.record(stream)
    traced(args.steps, "timed")
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    step_ms = ev0.elapsed_time(ev1) / args.steps      # both kernels, device clock
    launches, win_total_ms, win_bytes = ctx.kernel_stats()
    ctx.set_timing(False)
    if launches != args.steps:
        raise RuntimeError(f"timed {launches} window_kernel launches for {args.steps} steps")
    kernel_ms = win_total_ms / launches                 # average window_kernel launch duration
    kernel_bytes = win_bytes // launches                # algorithmic bytes per launch
    guard_checked, guard_rechecked, guard_redone = ctx.guard_detail()  # the timed steps (fma)

    t = torch.tensor([elapsed, kernel_ms, step_ms], dtype=torch.float64, device=dev)
    if distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kernel_ms, step_ms = float(t[0]), float(t[1]), float(t[2])
    energy = energy_leg(meter, torch, dev, step, step_ms, n, bytes_per_epoch(ct, C))

    # the other numerics mode, same buffers (reported beside the headline, not as value)
    alt = None
    if args.alt_steps > 0:
        other = "exact" if args.numerics != "exact" else "fma"
        ctx.set_numerics(other)
        step()
        torch.cuda.synchronize(dev)
        a0 = time.perf_counter()
        for _ in range(args.alt_steps):
            step()
        torch.cuda.synchronize(dev)
        at = torch.tensor([time.perf_counter() - a0], dtype=torch.float64, device=dev)
        if distributed:
            dist.all_reduce(at, op=dist.ReduceOp.MAX)
        alt = {"numerics": other, "value": round(world * n * args.alt_steps / float(at[0]), 1),
               "ms_per_step": round(float(at[0]) / args.alt_steps * 1e3, 4)}
        ctx.set_numerics(args.numerics)
        step()  # leave `out` in the headline mode for the checks below
        torch.cuda.synchronize(dev)

    # sanity of the produced features (unit rows) -- outside the timed region
    norms = torch.linalg.vector_norm(out, dim=1)
    ok_norm = bool(torch.all(torch.isfinite(norms)) and torch.max(torch.abs(norms - 1)) < 1e-12)

    line = None
    if rank == 0:
        workload_key = f"fused_dwt8_c{C}_int16_{n}_{args.numerics}"
        if sp != FRAMES_PER_EPOCH:
            workload_key += f"_spacing{sp}"
        value = world * n * args.steps / elapsed
        achieved = kernel_bytes / (kernel_ms * 1e-3) / 1e9
        bpe = bytes_per_epoch(ct, C)
        path_gbs = n * bpe / (step_ms * 1e-3) / 1e9
        kernels = (["baseline_kernel<int16,3>", WINDOW_KERNEL] if C == 3 else
                   ["baseline_any_kernel<int16>",
                    "window_c32_kernel" if C == 32 else "window_wide_kernel<int16>"])
        prof = traffic_from_profiles(workload_key)
        line = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "epochs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": wl["desc"],
                "epochs_per_gpu": n,
                "marker_spacing_frames": sp,
                "channels": C,
                "numerics": args.numerics,
                "kernels": kernels,
                "unit_rows_check": ok_norm,
                "guard": guard_report(args, fx, dev, guard_checked, guard_rechecked,
                                      guard_redone),
                "planted": planted,
                "settle": {"min_ms": args.settle_ms, "ms": round(settle_ms, 1),
                           "steps": settle_steps,
                           "note": "untimed steps between the warmup and the timed region, until "
                                   "min_ms of wall time has passed (the power-cap clock "
                                   "transient of the first ~25 launches)"},
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": (round(prof["hbm_bytes_per_launch"]) if prof else None),
                "kernel": kernels[1],
                "kernel_ms": round(kernel_ms, 4),
                "bytes_per_launch": kernel_bytes,
                "bytes_per_epoch": kernel_bytes // n,
                "traffic_source": (prof.get("source") if prof else None),
                "whole_path": {"ms": round(step_ms, 4), "bytes_per_epoch": bpe,
                               "GBps": round(path_gbs, 1),
                               "frac": round(path_gbs / HBM_PEAK_GBS, 4),
                               "energy": energy,
                               "ceiling": whole_path_ceiling(C, args.numerics, n, step_ms, bpe)},
                # the other side of the kernel's balance: fp64 filter-bank flops
                # (5,120 MAC per signal) against the vector fp64 peak, and the VALU issue share
                # of the kernel's cycles from the committed SQ counter pass
                "fp64": {"flop_per_epoch": FLOP_PER_SIGNAL[args.numerics] * C,
                         "achieved_TFs": round(FLOP_PER_SIGNAL[args.numerics] * C * n
                                               / (kernel_ms * 1e-3) / 1e12, 2),
                         "peak_TFs": FP64_VECTOR_PEAK_TFS,
                         "measured_fma_peak_TFs": FP64_FMA_MEASURED_TFS,
                         "frac": round(FLOP_PER_SIGNAL[args.numerics] * C * n / (kernel_ms * 1e-3)
                                       / 1e12 / FP64_VECTOR_PEAK_TFS, 4)},
                "ceiling": ceiling_from_profiles(C, args.numerics, n, kernel_ms, kernel_bytes),
            },
            "cpu_baseline": None,
        }

    if line is not None and alt:
        line["alt_numerics"] = alt
    if line is not None and trace is not None:
        line["step_trace"] = {k: [round(a.elapsed_time(b), 4) for a, b in zip(v, v[1:])]
                              for k, v in trace.items()}

    # The gathers are the first RCCL traffic between the ranks' own communicators; a hang there
    # must not cost the extraction line (or keep every rank alive until the launcher's limit).
    watchdog = _Watchdog()
    gather = None
    if distributed and not args.no_gather:
        watchdog.arm(args.gather_timeout, line,
                     f"gather legs did not finish within {args.gather_timeout} s")
        try:
            gather = bench_gather(args, ctx, out, n, C, rank, world, dev, dist)
        except Exception as exc:  # the extraction line above must still be reported
            gather = {"op": None, "ms": None, "error": f"{type(exc).__name__}: {exc}"[:300]}
        watchdog.disarm()

    # rank 0's host cores on a bounded sample of its own shard; at N > 1 after the gather legs,
    # so the timed extraction and gathers ran with every rank's host threads quiet
    cpu = None
    if rank == 0 and args.cpu_sample > 0:
        cpu = cpu_baseline(args, raw, out, ct, C, sp)
        if distributed:
            cpu["sample"] += (f"; rank 0 of {world}, after the gather legs (the other ranks idle "
                              "in teardown)")

    if rank == 0:
        line["cpu_baseline"] = cpu
        if gather:
            line["gather"] = gather
            if gather.get("ms") is not None:
                # extract + gather: the whole feature matrix on rank 0 (the product leg)
                line["extract_plus_gather"] = {
                    "value": round(world * n / ((elapsed / args.steps) + gather["ms"] * 1e-3), 1),
                    "unit": "epochs/s", "gather_op": gather["op"]}
        emit(line)

    if distributed:
        # the line is out; do not hang in teardown (rank 0 may still be timing the CPU baseline
        # while the other ranks get here)
        watchdog.arm(180 if rank else 60, None, "teardown")
    ctx.close()
    if distributed:
        dist.destroy_process_group()
    watchdog.disarm()


def guard_report(args, fx, dev, checked, rechecked, redone):
    """The fma conditioning guard over the timed steps: rows checked, rows that
    failed the a-priori test and went to the second stage (the row's measured max |x|), rows that
    failed that too and were recomputed under EXACT; and the same on every marker of the
    reference's two recordings (tests/golden/test-data, the repo's copies), outside the timed
    region."""
    if args.numerics != "fma":
        return None
    rep = {"rows_checked": checked, "rows_rechecked": rechecked, "rows_recomputed": redone,
           "rate": (redone / checked) if checked else None, "reference_recordings": {}}
    data = os.path.join(REPO, "tests", "golden", "test-data", "DoD")
    c = fx.Context(dev.index, numerics="fma")
    try:
        for stem in ("DoD2015_01", "DoD_2015_02"):
            base = os.path.join(data, stem)
            raw = fx.read_raw(base + ".vhdr", base + ".eeg")
            allpos = [m.position for m in fx.read_markers(base + ".vmrk") if m.position >= 100]
            c.guard_detail(reset=True)
            c.process_recording(raw, raw.shape[1], [0, 1, 2], [0.1] * 3, allpos)
            k, rc, r = c.guard_detail()
            rep["reference_recordings"][stem] = {"markers": k, "rows_rechecked": rc,
                                                 "rows_recomputed": r}
    except Exception as exc:  # the recordings are test fixtures; report, do not fail the line
        rep["reference_recordings"] = {"error": f"{type(exc).__name__}: {exc}"[:200]}
    finally:
        c.close()
    return rep


def plant_selection(n, rate):
    """Indices of the markers --plant overwrites: round(rate * n) of them, evenly spread over
    [0, n) (marker i when floor((i + 1) * rate) > floor(i * rate))."""
    i = np.arange(n, dtype=np.float64)
    return np.nonzero(np.floor((i + 1) * rate) > np.floor(i * rate))[0]


def plant_windows(torch, raw, pos, spec, chunk=100_000):
    """--plant KIND:RATE (study only): overwrite the frames [pos-100, pos+750) of the selected
    markers, every channel, with 'flat' samples (the value at pos-100, held: the flat stretch of
    DoD2015_01) or 'null' samples (DC + 1000 (-1)^f counts: a Nyquist-alternating window, which
    the 12-decimal low-pass taps cancel to rounding level).  Markers are spaced >= 850 frames
    apart, so the spans do not overlap."""
    kind, _, rate = spec.partition(":")
    rate = float(rate)
    if kind not in ("flat", "null") or not 0.0 <= rate <= 1.0:
        raise SystemExit("--plant KIND:RATE with KIND flat|null and 0 <= RATE <= 1")
    sel = torch.from_numpy(plant_selection(pos.numel(), rate)).to(pos.device)
    span = torch.arange(-100, 750, device=pos.device, dtype=torch.int64)
    for a in range(0, sel.numel(), chunk):
        p = pos[sel[a:a + chunk]]
        idx = p[:, None] + span[None, :]                     # [m, 850] frames
        if kind == "flat":
            v = raw[p - 100][:, None, :].expand(-1, span.numel(), -1)
        else:
            sign = 1 - 2 * (idx & 1)
            v = (-25000 + 1000 * sign)[:, :, None].expand(-1, -1, raw.shape[1])
        raw[idx.reshape(-1)] = v.reshape(-1, raw.shape[1]).to(raw.dtype)
    torch.cuda.synchronize(raw.device)
    return {"kind": kind, "rate": rate, "markers": int(sel.numel()),
            "note": "study workload, not the headline: the selected markers' spans overwritten "
                    "on the device before the run"}


class _Watchdog:
    """Ends the process if a multi-rank phase hangs: rank 0 first prints the bench line (when it
    has not been printed yet) with the phase's error, so the extraction measurement survives."""

    def __init__(self):
        self._timer = None

    def arm(self, seconds, line, what):
        import threading

        def fire():
            if line is not None:
                line["gather"] = {"op": None, "ms": None, "error": what}
                emit(line)
            sys.stderr.write(f"bench.py: {what}; exiting\n")
            sys.stderr.flush()
            os._exit(0)  # the phase is outside the measurement; its error is in the line

        self.disarm()
        self._timer = threading.Timer(seconds, fire)
        self._timer.daemon = True
        self._timer.start()

    def disarm(self):
        if self._timer is not None:
            self._timer.cancel()
            self._timer = None


def row_checksum(rows):
    """Order-sensitive exact checksum of a block of feature rows (torch float64 [n][F]): the rows'
    bits as int64, weighted by their 1-based row index, summed with wraparound -- exact, so equal
    wherever the same rows are summed; a shard moved, duplicated or altered changes it."""
    import torch
    bits = rows.contiguous().view(torch.int64)
    idx = torch.arange(1, rows.shape[0] + 1, dtype=torch.int64, device=rows.device)[:, None]
    return int((bits * idx).sum())


def bench_gather(args, ctx, out, n, C, rank, world, dev, dist):
    """The only exchange of the path: assembling the [world*n][16C] feature matrix
    in rank (= getData()) order.  Product leg: eegfx_gather_root through the C ABI -- the matrix
    on rank 0 only, the reference's single consumer (OffLineDataProvider.java:370-372,
    LogisticRegressionClassifier.java:87-94) -- by grouped RCCL send/recv over xGMI, every shard
    crossing one link once, on a communicator created from an RCCL unique id that rank 0 ships
    over the torch process group.  Beside it: eegfx_gather (the matrix on every rank, one RCCL
    broadcast per rank), and the same two exchanges through torch.distributed
    (isend/irecv to rank 0; all_gather_into_tensor + pad / concat).  All are timed outside the
    extraction steps (2 warm + 5 timed, max over ranks) and check the rows they deliver."""
    import torch
    from eeg_dataanalysispackage_amd.sharding import Comm, gather_features, gather_features_root

    def timed(fn, reps=5):
        fn()
        fn()
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            res = fn()
        torch.cuda.synchronize(dev)
        t = torch.tensor([(time.perf_counter() - t0) / reps], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return res, float(t[0]) * 1e3

    # every rank's checksum of its own rows, gathered once (a few bytes over the process group)
    own = torch.tensor([row_checksum(out)], dtype=torch.int64,
                       device=dev if args.dist_backend == "nccl" else "cpu")
    sums = [torch.zeros_like(own) for _ in range(world)]
    dist.all_gather(sums, own)
    sums = [int(t) for t in sums]

    def every_rank(flag):
        """True when `flag` holds on every rank (a MIN over the process group)."""
        t = torch.tensor([1 if flag else 0], dtype=torch.int64,
                         device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(int(t[0]))

    def root_ok(full):
        """rank 0 holds every rank's rows in rank order, each shard bit-identical to what its
        rank computed (checksums of the shards, not only unit norms: a misplaced or duplicated
        shard fails); the other ranks receive nothing -- checked on every rank."""
        if rank != 0:
            return every_rank(full is None)
        return every_rank(all(row_checksum(full[r * n:(r + 1) * n]) == sums[r]
                              for r in range(world)))

    bpr = n * 16 * C * 8
    res = {"bytes_per_rank": bpr, "rows": world * n, "root": 0,
           "root_inbound_bytes": bpr * (world - 1)}
    if args.dist_backend == "nccl":
        uid = [Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = Comm(ctx, world, rank, uid[0])
        full = (torch.empty((world * n, 16 * C), dtype=torch.float64, device=dev)
                if rank == 0 else None)
        got, ms = timed(lambda: comm.gather_root(out, world * n, root=0, out=full))
        res.update({"op": "eegfx_gather_root (RCCL grouped send/recv to rank 0)",
                    "ms": round(ms, 3), "rows_check": root_ok(got),
                    "root_inbound_GBps": round(bpr * (world - 1) / (ms * 1e-3) / 1e9, 1)})
        del full, got
        full = torch.empty((world * n, 16 * C), dtype=torch.float64, device=dev)
        full, ms_b = timed(lambda: comm.gather(out, world * n, out=full))
        res["all_ranks"] = {"op": "eegfx_gather (RCCL broadcast per rank, grouped)",
                            "ms": round(ms_b, 3),
                            "rows_check": every_rank(all(
                                row_checksum(full[r * n:(r + 1) * n]) == sums[r]
                                for r in range(world)))}
        comm.close()
        del full
        got, ms_r = timed(lambda: gather_features_root(out, world * n, 0))
        res["torch_root_p2p"] = {"ms": round(ms_r, 3), "rows_check": root_ok(got)}
        del got
    else:
        res.update({"op": None, "ms": None, "note": "C-ABI gathers need RCCL (rehearsal backend)"})
    full, ms_t = timed(lambda: gather_features(out, world * n))
    res["torch_all_gather"] = {"ms": round(ms_t, 3),
                               "rows_check": every_rank(all(
                                   row_checksum(full[r * n:(r + 1) * n]) == sums[r]
                                   for r in range(world)))}
    del full
    if res["ms"] is None:
        res["op"], res["ms"] = "torch all_gather_into_tensor", round(ms_t, 3)
    return res


def bench_dropin(args, rank, world, dev, dist):
    """configs[0] through the C ABI, latency-bound: the reference calls
    IFeatureExtraction.extractFeatures once per epoch (Spark map closures,
    LogisticRegressionClassifier.java:55-61,90; serial loops, NeuralNetworkClassifier.java:78-86;
    FeatureExtractionTest.java:62-67) and loads test-data/info.txt through OffLineDataProvider.
    Reported per calling thread (one context per thread, as include/eegfx.h prescribes):
      single_epoch  eegfx_extract_features_f64 on one host epoch (the JNI drop-in), median latency;
      threads       the same call from T threads at once, each with its own context;
      info_txt      OffLineDataProvider(info.txt).loadData() + features of its 11 epochs;
    and beside them the C port (oracle, one thread) on the same epoch."""
    import threading
    import torch
    import eeg_dataanalysispackage_amd as fx
    from oracle import oracle
    data = os.path.join(REPO, "tests", "golden", "test-data")
    base = os.path.join(data, "DoD", "DoD2015_01")
    raw = fx.read_raw(base + ".vhdr", base + ".eeg")
    pos, _, _ = fx.plan_markers(fx.read_markers(base + ".vmrk"), raw.shape[0], 1)
    ep = oracle.decode_epochs(raw, [0, 1, 2], [0.1] * 3, pos)
    reps = max(200, args.steps * 10)

    def lat(fn, k=reps):
        for _ in range(20):
            fn()
        ts = []
        for _ in range(k):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)), float(np.percentile(ts, 99))

    ctx = fx.Context(dev.index, numerics=args.numerics)
    one = np.ascontiguousarray(ep[:1])
    outb = np.empty((1, 48))
    med, p99 = lat(lambda: ctx.extract_features(one, out=outb))
    want = oracle.extract_features(one)
    parity = bool(np.array_equal(outb, want) if args.numerics == "exact"
                  else np.max(np.abs(outb - want)) <= 1e-9)
    fe = fx.WaveletTransform(context=ctx)
    med_fe, _ = lat(lambda: fe.extractFeatures(ep[0]))
    # T threads, one context each, calling concurrently (Spark local[T])
    threads = {}
    for T in (2, 4, 8):
        ctxs = [fx.Context(dev.index, numerics=args.numerics) for _ in range(T)]
        per = [0.0] * T
        k = reps // 2

        def work(i):
            o = np.empty((1, 48))
            for _ in range(10):
                ctxs[i].extract_features(one, out=o)
            t0 = time.perf_counter()
            for _ in range(k):
                ctxs[i].extract_features(one, out=o)
            per[i] = (time.perf_counter() - t0) / k
        th = [threading.Thread(target=work, args=(i,)) for i in range(T)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        for c in ctxs:
            c.close()
        threads[str(T)] = {"per_thread_epochs_per_s": round(1.0 / float(np.mean(per)), 1),
                           "aggregate_epochs_per_s": round(sum(1.0 / p for p in per), 1)}
    # info.txt end to end (configs[0]'s data) through the C-ABI provider
    info = os.path.join(data, "infoTrain.txt")

    def info_flow():
        odp = fx.OffLineDataProvider([info], context=ctx)
        odp.loadData()
        f = odp.getFeatures()
        odp.close()
        return f
    med_info, _ = lat(info_flow, k=max(20, args.steps))
    f_info = info_flow()
    # the C port on the same epoch, one thread (the per-thread rate of the CPU baseline)
    med_cpu, _ = lat(lambda: oracle.extract_features(one, faithful=True), k=reps)
    ctx.close()
    # the same calls from native code (tools/dropin_bench.hip: what a JNI caller sees, no Python)
    native = None
    exe = os.path.join(REPO, "tools", "dropin_bench")
    if os.path.exists(exe):
        import subprocess
        r = subprocess.run([exe, REPO, str(reps), "0" if args.numerics == "exact" else "1"],
                           capture_output=True, text=True, timeout=300)
        if r.returncode == 0:
            native = json.loads(r.stdout)
        else:
            native = {"error": r.stderr[-500:]}
    value = (native["single_epoch"]["epochs_per_s"] if native and "single_epoch" in native
             else 1.0 / med)
    if rank == 0:
        emit(({
            "metric": "per-call IFeatureExtraction latency through the C ABI (configs[0] drop-in)",
            "value": round(value, 1), "unit": "epochs/s per calling thread",
            "n_gpus": world, "steps": reps, "warmup": 20, "ms_per_step": round(med * 1e3, 4),
            "higher_is_better": True, "scaling": "none", "vs_baseline": None, "dtype": "f64",
            "data": "reference test-data (DoD2015_01, infoTrain.txt)",
            "config": {"workload": "configs[0]: one host epoch per eegfx_extract_features_f64 "
                                   "call (zero-copy pinned staging), numerics " + args.numerics,
                       "parity": parity},
            "native_c_abi": native,
            "python": {"single_epoch_median_us": round(med * 1e6, 2), "p99_us": round(p99 * 1e6, 2),
                       "WaveletTransform_median_us": round(med_fe * 1e6, 2), "threads": threads},
            "info_txt": {"epochs": int(f_info.shape[0]), "median_ms": round(med_info * 1e3, 3),
                         "epochs_per_s": round(f_info.shape[0] / med_info, 1),
                         "feature_sum": oracle.java_feature_sum(f_info)},
            "cpu_baseline": {"value": round((native or {}).get("cpu_port_single_thread", {}).get(
                                 "epochs_per_s") or 1.0 / med_cpu, 1),
                             "unit": "epochs/s per thread", "cores": 1, "kind": "port",
                             "sample": "the same epoch, oracle C restatement (full pyramid), "
                                       f"median of {reps} calls from C (Python: "
                                       f"{round(1.0 / med_cpu, 1)} epochs/s)",
                             "optimised": (native or {}).get("cpu_optimised_single_thread")},
        }))


def bench_stream(args, rank, world, dev, dist):
    """configs[4]: long recordings streamed from pinned host memory (eegfx_process_recording_
    streamed).  Per GPU: four 4-hour 3-channel recordings back to back (57.6M frames, 346 MB int16)
    with a marker every 100 frames (dense, overlapping epochs: 576k per step).  The bound is the
    host link: every frame crosses PCIe once per step."""
    import torch
    import eeg_dataanalysispackage_amd as fx
    nf = 4 * 4 * 3600 * 1000
    step_frames = 100
    ctx = fx.Context(dev.index, numerics=args.numerics)
    d_raw = torch.empty((nf, 3), dtype=torch.int16, device=dev)
    ctx.synth_recording(d_raw, 3, SEED + rank)
    host = torch.empty((nf, 3), dtype=torch.int16, pin_memory=True)
    host.copy_(d_raw)
    del d_raw
    raw = host.numpy()
    pos = np.arange(step_frames * 2, nf - 700, step_frames, dtype=np.int64)
    n = len(pos)
    out = torch.empty((n, 48), dtype=torch.float64, pin_memory=True).numpy()

    def step():
        ctx.process_recording_streamed(raw, 3, [0, 1, 2], [0.1] * 3, pos,
                                       chunk_frames=args.chunk_frames, out=out)

    for _ in range(max(1, args.warmup)):
        step()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    el = time.perf_counter() - t0
    if dist:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t[0])
    ok = bool(np.all(np.isfinite(out)) and np.max(np.abs(np.linalg.norm(out, axis=1) - 1)) < 1e-12)
    # the host-link bound of a step: the same bytes moved by plain concurrent copies (the
    # recording host -> device on one stream, the feature rows device -> host on another)
    d_in = torch.empty(nf * 3, dtype=torch.int16, device=dev)
    d_out = torch.empty((n, 48), dtype=torch.float64, device=dev)
    h_out = torch.from_numpy(out)
    s_in, s_out = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    flat = host.view(-1)

    def copies():
        with torch.cuda.stream(s_in):
            d_in.copy_(flat, non_blocking=True)
        with torch.cuda.stream(s_out):
            h_out.copy_(d_out, non_blocking=True)

    def timed_copies(fn, reps=5):
        fn()
        torch.cuda.synchronize(dev)
        c0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - c0) / reps * 1e3

    def upload_only():
        with torch.cuda.stream(s_in):
            d_in.copy_(flat, non_blocking=True)

    def download_only():
        with torch.cuda.stream(s_out):
            h_out.copy_(d_out, non_blocking=True)

    copy_ms = timed_copies(copies)
    # each direction alone on this box: the link's rates differ by box
    up_ms, down_ms = timed_copies(upload_only), timed_copies(download_only)
    del d_in, d_out
    cpu = None
    if rank == 0 and args.cpu_sample > 0:
        # the same recordings and marker grid on the host cores (BASELINE.json configs[4])
        cpu = cpu_baseline(args, torch.from_numpy(raw), torch.from_numpy(out), 3, 3,
                           sp=step_frames, first=int(pos[0]), n_epochs=n,
                           what="first streamed 4 h recording (a marker every 100 frames)")
    if rank == 0:
        h2d = nf * 6 * args.steps / el / 1e9
        emit(({
            "metric": METRIC, "value": round(world * n * args.steps / el, 1), "unit": "epochs/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": "configs[4]: four 4 h 3-channel int16 recordings per GPU in "
                                   "pinned host memory, a marker every 100 frames, streamed in "
                                   f"{args.chunk_frames}-frame chunks",
                       "epochs_per_gpu": n, "numerics": args.numerics, "unit_rows_check": ok},
            "host_link": {"bound": "pcie", "h2d_GBps": round(h2d, 2),
                          "bytes_per_step": nf * 6, "d2h_bytes_per_step": n * 48 * 8,
                          "copy_only_ms": round(copy_ms, 3),
                          "upload_alone_ms": round(up_ms, 3), "download_alone_ms": round(down_ms, 3),
                          "frac": round(copy_ms / (el / args.steps * 1e3), 4),
                          "note": "every frame crosses the host link once per step and every "
                                  "feature row once back; copy_only_ms = the same bytes moved by "
                                  "two concurrent plain copies (the bound), frac = that / step"},
            "cpu_baseline": cpu,
        }))
    ctx.close()


def bench_logreg(args, rank, world, dev, dist):
    """LogisticRegressionClassifier's training (MLlib LogisticRegressionWith
    SGD defaults: 100 iterations, step 1.0, regParam 0.01, full batch) on the device-resident
    feature rows of the c3 workload.  A step = one whole training run; value = rows x iterations
    per second; the roofline is the gradient pass, which reads the n x 48 rows + labels once per
    iteration.  --workload svm: SVMClassifier's SVMWithSGD (HingeGradient), same defaults."""
    import torch
    import eeg_dataanalysispackage_amd as fx
    from eeg_dataanalysispackage_amd import classification as clf
    svm = args.workload == "svm"
    train = clf.svm_sgd_train if svm else clf.sgd_train
    algo = "SVMWithSGD" if svm else "LogisticRegressionWithSGD"
    n = args.epochs or 1_000_000
    ctx = fx.Context(dev.index, numerics=args.numerics)
    raw = torch.empty((FRAMES_PER_EPOCH * n + 2000, 3), dtype=torch.int16, device=dev)
    ctx.synth_recording(raw, 3, SEED + rank)
    pos = torch.arange(FRAMES_PER_EPOCH, FRAMES_PER_EPOCH * (n + 1), FRAMES_PER_EPOCH,
                       dtype=torch.int64, device=dev)
    X = ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos)
    del raw
    ctx.synchronize()
    # labels: the sign of a fixed direction plus noise (deterministic), both classes present
    g = torch.Generator(device=dev).manual_seed(SEED)
    w0 = torch.randn(48, generator=g, device=dev, dtype=torch.float64)
    y = ((X @ w0 + 0.1 * torch.randn(n, generator=g, device=dev, dtype=torch.float64)) > 0)
    y = y.to(torch.float64).contiguous()
    torch.cuda.synchronize(dev)
    iters = clf.DEFAULT_NUM_ITERATIONS

    def step():
        return train(ctx, X, y, iters, clf.DEFAULT_STEP_SIZE, clf.DEFAULT_REG_PARAM,
                     clf.DEFAULT_MINI_BATCH_FRACTION, convergence_tol=0.0)

    for _ in range(max(1, min(args.warmup, 5))):
        w, it = step()
    steps = max(1, min(args.steps, 20))
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        w, it = step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t[0])
    per_iter = elapsed / steps / it
    bytes_iter = n * 48 * 8 + n * 8
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        from oracle import mllib_logreg as ref
        k = min(n, 100_000)
        Xh, yh = X[:k].cpu().numpy(), y[:k].cpu().numpy()
        c0 = time.perf_counter()
        wr, itr = ref.sgd_train(Xh, yh, iters, 1.0, 0.01, convergence_tol=0.0,
                                gradient="hinge" if svm else "logistic")
        cdt = time.perf_counter() - c0
        wg, itg = train(ctx, Xh, yh, iters, 1.0, 0.01, convergence_tol=0.0)
        cpu = {"value": round(k * itr / cdt, 1), "unit": "rows*iterations/s", "cores": 1,
               "kind": "port",
               "sample": f"first {k} rows, numpy restatement of MLlib 1.6.2 "
                         f"{algo} ({itr} iterations, one partition), "
                         f"{cdt:.2f} s wall",
               "gpu_parity_on_sample": bool(np.linalg.norm(wg - wr) <= 1e-9 * np.linalg.norm(wr))}
    if rank == 0:
        emit(({
            "metric": f"{'SVM' if svm else 'logistic-regression'} SGD rows*iterations/s (MLlib "
                      f"{algo}, full batch) on the dwt-8 feature rows",
            "value": round(world * n * it * steps / elapsed, 1),
            "unit": "rows*iterations/s", "n_gpus": world, "steps": steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"{args.workload}: 100 iterations, step 1.0, regParam 0.01 over "
                                   "the c3 feature rows (1M x 48 per GPU), labels from a fixed "
                                   "direction",
                       "rows_per_gpu": n, "features": 48, "iterations": it},
            "roofline": {"bound": "hbm", "achieved": round(bytes_iter / per_iter / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(bytes_iter / per_iter / 1e9 / HBM_PEAK_GBS, 4),
                         "traffic": None, "kernel": "lr_grad16_kernel + lr_update_kernel",
                         "bytes_per_iteration": bytes_iter,
                         "ms_per_iteration": round(per_iter * 1e3, 4)},
            "cpu_baseline": cpu}))
    ctx.close()


def host_cores():
    """The host cores this process may run on: the CPU affinity set, capped by a cgroup CPU quota
    when one is set (a GPU box shares its host: nproc shows every CPU of the machine, the quota
    the box's share).  Returns (cores, details)."""
    import math
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / period
        except (OSError, ValueError):
            pass
    cores = min(aff, max(1, math.floor(quota))) if quota else aff
    return cores, {"affinity": aff, "os_cpu_count": os.cpu_count(), "cgroup_quota_cpus": quota}


def cpu_baseline(args, raw, gpu_out, ct, C, sp=FRAMES_PER_EPOCH, first=None, n_epochs=None,
                 what="rank-0 synthetic recording"):
    """C restatement of the Java algorithm (oracle/, reference-faithful full 6-level pyramid),
    threads over contiguous epoch ranges, on a bounded sample of the same synthetic workload.

    SURVEY.md 8(d): the reference-faithful variant is `value`; beside it the optimised CPU
    restatement (oracle.process_recording_fast: minimal cascade over only the 612 frames that reach
    the features, 4 epochs per AVX2 vector, bit-identical features), and both at one thread on a
    smaller sample.  Every leg is the median of 5 timed runs after a warm-up."""
    from oracle import oracle
    avail, cores_info = host_cores()
    # SURVEY 8d / BASELINE.md: N = every core of the host available to this run (Spark local[*],
    # Utils/SparkInitializer.java:44); --cpu-threads overrides
    threads = args.cpu_threads or avail
    first = sp if first is None else first
    k = min(args.cpu_sample if C == 3 else args.cpu_sample // 10,
            args.epochs if n_epochs is None else n_epochs)
    k1 = max(1, min(k // 25, 20000 if C == 3 else 2000))  # one-thread sample
    host = raw[: first + sp * k + 2000].cpu().numpy()
    pos = np.arange(first, first + sp * k, sp, dtype=np.int64)
    cols = list(range(C))

    def run(h, p, faithful, nthreads):
        if faithful:
            return oracle.process_recording(h, cols, [0.1] * C, p, faithful=True,
                                            nthreads=nthreads)
        return oracle.process_recording_fast(h, cols, [0.1] * C, p, nthreads=nthreads)

    def leg(n, faithful, nthreads, reps=5):
        h = host[: first + sp * n + 2000]
        run(h[: sp * 200 + 2000], pos[: min(200, n)], faithful, nthreads)
        times, feats = [], None
        for _ in range(reps):
            t0 = time.perf_counter()
            feats = run(h, pos[:n], faithful, nthreads)
            times.append(time.perf_counter() - t0)
        dt = float(np.median(times))
        return n / dt, dt, feats

    value, dt, feats = leg(k, True, threads)
    gpu = gpu_out[:k].cpu().numpy()
    if args.numerics == "exact":
        parity = bool(np.array_equal(gpu, feats, equal_nan=True))
    else:
        parity = bool(np.max(np.abs(gpu - feats)) <= 1e-9)
    faithful_1, _, _ = leg(k1, True, 1)
    minimal_n, _, feats_min = leg(k, False, threads)
    minimal_1, _, _ = leg(k1, False, 1)
    t16 = None
    if threads != 16 and avail >= 16:  # the earlier rounds' 16-thread leg, for comparison
        t16 = {"value": round(leg(k, True, 16)[0], 1), "cores": 16, "sample_epochs": k}
    return {
        "value": round(value, 1),
        "unit": "epochs/s",
        "cores": threads,
        "host_cores": cores_info,
        "kind": "port",
        "sample": f"first {k} epochs of the {what}, C restatement of the "
                  f"Java path (full 6-level pyramid), {threads} threads over contiguous ranges, "
                  f"median of 5 runs of {dt:.2f} s wall",
        "gpu_parity_on_sample": parity,
        "variants": {
            "faithful_1_thread": {"value": round(faithful_1, 1), "sample_epochs": k1},
            "optimised": {"value": round(minimal_n, 1), "cores": threads, "sample_epochs": k,
                                "bit_identical_to_faithful": bool(np.array_equal(
                                    feats, feats_min, equal_nan=True))},
            "optimised_1_thread": {"value": round(minimal_1, 1), "sample_epochs": k1},
            "faithful_16_threads": t16,
        },
    }


if __name__ == "__main__":
    main()
