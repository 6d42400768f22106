#!/bin/bash
set -euo pipefail
echo -n "default: "; timeout -k 10 200 python bench.py --workload stream --steps 20 --warmup 3 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["host_link"]["h2d_GBps"])'
echo -n "SDMA=0: "; HSA_ENABLE_SDMA=0 timeout -k 10 200 python bench.py --workload stream --steps 20 --warmup 3 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["host_link"]["h2d_GBps"])'
python3 - <<'PY'
import torch, time
for sdma in ["default"]:
    n = 345_600_000
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    o = torch.empty(221_000_000, dtype=torch.uint8, device="cuda")
    ho = torch.empty(221_000_000, dtype=torch.uint8, pin_memory=True)
    for _ in range(3): d.copy_(h, non_blocking=True)
    torch.cuda.synchronize(); t=time.perf_counter()
    for _ in range(10): d.copy_(h, non_blocking=True)
    torch.cuda.synchronize(); dt=(time.perf_counter()-t)/10
    print("H2D alone GB/s", round(n/dt/1e9,1))
    torch.cuda.synchronize(); t=time.perf_counter()
    for _ in range(10): ho.copy_(o, non_blocking=True)
    torch.cuda.synchronize(); dt=(time.perf_counter()-t)/10
    print("D2H alone GB/s", round(221e6/dt/1e9,1))
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize(); t=time.perf_counter()
    for _ in range(10):
        with torch.cuda.stream(s1): d.copy_(h, non_blocking=True)
        with torch.cuda.stream(s2): ho.copy_(o, non_blocking=True)
    torch.cuda.synchronize(); dt=(time.perf_counter()-t)/10
    print("both concurrently: ms", round(dt*1e3,2), "H2D-equiv GB/s", round(n/dt/1e9,1), "total GB/s", round((n+221e6)/dt/1e9,1))
PY
