import sys, os, time, numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import eeg_dataanalysispackage_amd as fx
ctx = fx.Context(0, numerics="fma")
nf = 57_600_000
d = torch.empty((nf, 3), dtype=torch.int16, device="cuda")
ctx.synth_recording(d, 3, 5)
hp = torch.empty((nf, 3), dtype=torch.int16, pin_memory=True); hp.copy_(d)
pg = d.cpu().numpy()
pos = np.arange(200, nf - 700, 100, dtype=np.int64)
outp = torch.empty((len(pos), 48), dtype=torch.float64, pin_memory=True).numpy()
for name, raw, out in [("pinned", hp.numpy(), outp), ("pageable", pg, None)]:
    for chunk in (1 << 20, 1 << 22, 1 << 24):
        ctx.process_recording_streamed(raw, 3, [0,1,2], [0.1]*3, pos, chunk_frames=chunk, out=out)
        t = time.perf_counter()
        for _ in range(3):
            ctx.process_recording_streamed(raw, 3, [0,1,2], [0.1]*3, pos, chunk_frames=chunk, out=out)
        dt = (time.perf_counter() - t) / 3
        print(name, chunk, f"{dt*1e3:.1f} ms  {nf*6/dt/1e9:.1f} GB/s  {len(pos)/dt/1e6:.1f} Mep/s")
t = time.perf_counter(); x = torch.empty((nf,3), dtype=torch.int16, device="cuda"); x.copy_(hp, non_blocking=True); torch.cuda.synchronize(); print("raw H2D", nf*6/(time.perf_counter()-t)/1e9, "GB/s")
