"""A/B of the root's k_shard_unpack reading an IPC receive buffer of each
memory kind: uncached (the default now), fine-grained
and plain hipMalloc, on one GPU.  A real round pack of an 8 GiB B7 shard
(128 KiB per block: the largest round, 256 MiB) is copied into a buffer of
each kind by lz4mtHipIpcAllocKind, then unpacked into a mirror 20 times;
prints the mean kernel time (HIP events) and the rate per kind.

    python tools/unpack_ab.py [GiB]
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
    n = int(gib * (1 << 30)) // (4 << 20) * (4 << 20)
    sd = L.make_sd(7, stream_checksum=False, block_checksum=True)
    cap = 128 << 10
    src = L.gen_synthetic(n, seed=42)
    ws = L.shard_workspace(n, sd)
    L.shard_reset(n, sd, ws)
    L.shard_encode(src, sd, ws)
    torch.cuda.synchronize()
    pb = L.shard_pack_bound(n, sd, cap)
    pack = torch.empty(pb, dtype=torch.uint8, device="cuda")
    L.shard_pack(src, sd, ws, pack, cap, 1)
    torch.cuda.synchronize()
    packed = int.from_bytes(bytes(pack[24:32].cpu().numpy().tobytes()), "little")
    mirror = L.shard_workspace(n, sd)
    st = torch.cuda.current_stream()
    out = {"shard_bytes": n, "pack_bytes": packed, "reps": 20, "kinds": {}}
    for want, name in ((2, "uncached"), (1, "fine-grained"), (0, "coarse-grained (hipMalloc)")):
        ptr, h, k = ctypes.c_void_p(), (ctypes.c_uint8 * 64)(), ctypes.c_int(-1)
        if L.lib.lz4mtHipIpcAllocKind(pb, ctypes.byref(ptr), h, want, ctypes.byref(k)) != 0:
            out["kinds"][name] = "allocation / IPC export failed"
            continue
        if k.value != want:
            out["kinds"][name] = f"not available (got kind {k.value})"
            L.lib.lz4mtHipFree(ptr)
            continue
        assert L.lib.lz4mtHipCopyAsync(ptr, ctypes.c_void_p(pack.data_ptr()), packed,
                                       ctypes.c_void_p(st.cuda_stream)) == 0
        ts = []
        for _ in range(21):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            r = L.lib.lz4mtHipShardUnpack(ptr, n, ctypes.byref(sd), ctypes.c_void_p(mirror.data_ptr()),
                                          mirror.numel(), ctypes.c_void_p(st.cuda_stream))
            b.record()
            assert r == 0
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        ms = sum(ts[1:]) / len(ts[1:])
        out["kinds"][name] = {"unpack_ms": round(ms, 4), "GBps": round(packed / ms / 1e6, 1)}
        L.lib.lz4mtHipFree(ptr)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
