"""Probe: do gloo collectives / P2P accept CUDA tensors here (two ranks on one GPU)?"""
import os
import torch
import torch.distributed as dist

dist.init_process_group("gloo")
r = dist.get_rank()
torch.cuda.set_device(0)
t = torch.full((4,), r + 1, dtype=torch.int64, device="cuda")
out = [torch.zeros(4, dtype=torch.int64, device="cuda") for _ in range(2)]
res = {}
try:
    dist.all_gather(out, t)
    res["all_gather"] = [o.tolist() for o in out]
except Exception as e:  # noqa: BLE001
    res["all_gather"] = repr(e)[:120]
try:
    if r == 0:
        w = dist.batch_isend_irecv([dist.P2POp(dist.isend, t, 1)])
    else:
        b = torch.zeros(4, dtype=torch.int64, device="cuda")
        w = dist.batch_isend_irecv([dist.P2POp(dist.irecv, b, 0)])
    for x in w:
        x.wait()
    res["p2p"] = "ok" if r == 0 else b.tolist()
except Exception as e:  # noqa: BLE001
    res["p2p"] = repr(e)[:160]
try:
    dist.broadcast(t, 0)
    res["broadcast"] = t.tolist()
except Exception as e:  # noqa: BLE001
    res["broadcast"] = repr(e)[:120]
print(r, res, flush=True)
dist.destroy_process_group()
