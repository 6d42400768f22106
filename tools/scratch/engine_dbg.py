import sys, os, numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import eeg_dataanalysispackage_amd as fx
ctx = fx.Context(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
nf = 1000 * n + 2000
dev = torch.device("cuda", 0)
raw = torch.empty((nf, 3), dtype=torch.int16, device=dev)
ctx.synth_recording(raw, 3, 0x5EED)
pos = torch.arange(1000, 1000 + 1000 * n, 1000, dtype=torch.int64, device=dev)
out = ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos); ctx.synchronize()
out2 = ctx.process_recording(raw, 3, [0, 1, 2], [0.1] * 3, pos); ctx.synchronize()
f = out.cpu().numpy(); f2 = out2.cpu().numpy()
nrm = np.linalg.norm(f, axis=1)
bad = np.where(~np.isfinite(nrm) | (np.abs(nrm - 1) > 1e-12))[0]
diff = np.where(np.any(f != f2, axis=1))[0]
print("n", n, "bad rows", len(bad), bad[:20], "nondeterministic rows", len(diff), diff[:20])
if len(bad): print(f[bad[0]][:8], nrm[bad[:5]])
os.environ["EEGFX_ENGINE"] = "0"
