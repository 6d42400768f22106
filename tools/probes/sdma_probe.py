"""Device-to-host copies on an SDMA engine (ROCr hsa_amd_memory_async_copy) instead of the HIP
runtime's blit kernel, alone and beside a 346 MB upload -- does the host link split differently
between the two directions (configs[4]: uploads at 46-50 GB/s beside blit downloads)?
    python3 tools/probes/sdma_probe.py
"""
import ctypes as ct
import time

import torch

dev = torch.device("cuda:0")
torch.cuda.init()
hsa = ct.CDLL("libhsa-runtime64.so")


class Agent(ct.Structure):
    _fields_ = [("handle", ct.c_uint64)]


class Signal(ct.Structure):
    _fields_ = [("handle", ct.c_uint64)]


assert hsa.hsa_init() == 0
gpus, cpus = [], []
CB = ct.CFUNCTYPE(ct.c_int, Agent, ct.c_void_p)


def each(agent, _):
    kind = ct.c_int(-1)
    hsa.hsa_agent_get_info(agent, 17, ct.byref(kind))  # HSA_AGENT_INFO_DEVICE
    (gpus if kind.value == 1 else cpus if kind.value == 0 else []).append(Agent(agent.handle))
    return 0


cb = CB(each)
assert hsa.hsa_iterate_agents(cb, None) == 0
print(f"{len(gpus)} GPU agent(s), {len(cpus)} CPU agent(s)")
gpu, cpu = gpus[0], cpus[0]
hsa.hsa_amd_memory_async_copy.argtypes = [ct.c_void_p, Agent, ct.c_void_p, Agent, ct.c_size_t,
                                          ct.c_uint32, ct.c_void_p, Signal]
hsa.hsa_signal_create.argtypes = [ct.c_int64, ct.c_uint32, ct.c_void_p, ct.POINTER(Signal)]
hsa.hsa_signal_wait_scacquire.argtypes = [Signal, ct.c_int, ct.c_int64, ct.c_uint64, ct.c_int]
hsa.hsa_signal_wait_scacquire.restype = ct.c_int64
hsa.hsa_signal_store_relaxed.argtypes = [Signal, ct.c_int64]

UP, DOWN = 345_600_000, 221_180_544
h_in = torch.empty(UP, dtype=torch.uint8, pin_memory=True)
d_in = torch.empty(UP, dtype=torch.uint8, device=dev)
h_out = torch.empty(DOWN, dtype=torch.uint8, pin_memory=True)
d_out = torch.ones(DOWN, dtype=torch.uint8, device=dev)
s_in, s_out = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
sig_d, sig_u = Signal(), Signal()
assert hsa.hsa_signal_create(1, 0, None, ct.byref(sig_d)) == 0
assert hsa.hsa_signal_create(1, 0, None, ct.byref(sig_u)) == 0
torch.cuda.synchronize()


def sdma(dst, dst_agent, src, src_agent, n, sig):
    hsa.hsa_signal_store_relaxed(sig, 1)
    st = hsa.hsa_amd_memory_async_copy(dst, dst_agent, src, src_agent, n, 0, None, sig)
    assert st == 0, f"hsa_amd_memory_async_copy: status {st:#x}"


def wait(sig):
    hsa.hsa_signal_wait_scacquire(sig, 2, 1, 2**63 - 1, 1)  # until < 1


def leg(label, up, down):
    res = []
    for _ in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if up == "hip":
            with torch.cuda.stream(s_in):
                d_in.copy_(h_in, non_blocking=True)
        elif up == "sdma":
            sdma(d_in.data_ptr(), gpu, h_in.data_ptr(), cpu, UP, sig_u)
        if down == "hip":
            with torch.cuda.stream(s_out):
                h_out.copy_(d_out, non_blocking=True)
        elif down == "sdma":
            sdma(h_out.data_ptr(), cpu, d_out.data_ptr(), gpu, DOWN, sig_d)
        if up == "sdma":
            wait(sig_u)
        if down == "sdma":
            wait(sig_d)
        torch.cuda.synchronize()
        res.append((time.perf_counter() - t0) * 1e3)
    ms = sorted(res[1:])[1]
    print(f"{label:40s} {ms:7.3f} ms")


leg("upload alone (HIP)", "hip", None)
leg("upload alone (SDMA)", "sdma", None)
leg("download alone (HIP blit)", None, "hip")
leg("download alone (SDMA)", None, "sdma")
leg("pair: HIP up + HIP blit down", "hip", "hip")
leg("pair: HIP up + SDMA down", "hip", "sdma")
leg("pair: SDMA up + SDMA down", "sdma", "sdma")
ok = bool((h_out[:1 << 20] == 1).all())
print("download contents ok:", ok)
