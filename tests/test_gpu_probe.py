"""The encoders' table probe and its fallback.

The product encoders probe the LZ4 hash table with ONE LDS exchange per
lane (ds_wrxchg_rtn_b32 / ds_mskor_rtn_b32), which reproduces LZ4 1.9.3's
sequential inserts (reference call site src/lz4mt.cpp:391)
only because gfx950 applies a wave's same-address exchanges in ascending
lane order -- measured, not architected.  The library checks that once per
device (k_xchg_order) and, when it fails, runs the read-back probe
instantiation of every encoder instead (read, write a marker, read back,
resolve same-bucket predecessors exactly), which assumes no ordering.
LZ4MT_AMD_ENC_PROBE=readback forces that path; it must write the reference's
bytes everywhere the exchange path does: golden blocks and frames, the
256 MiB App. F known answers, -BD frames (the LINK kernels), and a frame
encoded while its stream is captured into a graph before any check ran."""
import ctypes
import random

import pytest
import torch

import oracle
from conftest import bd_data, read_golden

pytestmark = pytest.mark.gpu

L = None


@pytest.fixture(scope="module", autouse=True)
def lib():
    global L
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    import lz4mt_amd
    L = lz4mt_amd
    return L


@pytest.fixture
def readback(monkeypatch):
    monkeypatch.setenv("LZ4MT_AMD_ENC_PROBE", "readback")
    assert L.lib.lz4mtHipEncoderProbe() == 0
    yield
    monkeypatch.delenv("LZ4MT_AMD_ENC_PROBE")
    assert L.lib.lz4mtHipEncoderProbe() == 1


def dev(b):
    t = torch.empty(max(len(b), 1), dtype=torch.uint8, device="cuda")
    if b:
        t[:len(b)].copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8))
    return t[:len(b)]


def host(t):
    return bytes(t.cpu().numpy().tobytes())


def test_order_check_and_probe_selection():
    """On gfx950 the check passes (1; -1 would be a HIP error, 0 a failed
    order) and the exchange probe is the one in use."""
    assert L.lib.lz4mtHipCheckEncoderOrder() == 1
    assert L.lib.lz4mtHipEncoderProbe() == 1


def test_readback_golden_blocks_and_frames(readback, golden, golden_inputs):
    import hashlib
    for v in golden["blocks"]:
        data = golden_inputs[v["input"]][:v["n"]]
        c = L.compress_block(data, v["cap"])
        assert len(c) == v["ret"] and hashlib.sha1(c).hexdigest() == v["sha1"], v
    for f in golden["frames"]:
        data = golden_inputs[f["input"]]
        sd = L.make_sd(f["bid"], f["stream_checksum"], f["block_checksum"])
        assert host(L.compress_frame(dev(data), sd)) == read_golden(f["file"]), f["file"]


def test_readback_fuzz_vs_oracle(readback):
    """Collision-heavy inputs (3-letter alphabets, short periods) exercise the
    read-back path's same-bucket predecessor resolution; every table kind:
    byU16 (64 KiB blocks), the 3-byte table (256 KiB), byU32."""
    rnd = random.Random(11)
    syn = oracle.gen_synthetic(1 << 20, 3)
    for n in (70_000, 262_144, 1 << 20):
        for kind in range(3):
            if kind == 0:
                d = syn[:n]
            elif kind == 1:
                d = bytes(rnd.randrange(3) for _ in range(n))
            else:
                d = (bytes(rnd.randrange(256) for _ in range(rnd.randrange(1, 70))) * (n // 8))[:n]
            for cap in (n, n - 1):
                assert L.compress_block(d, cap) == oracle.compress_block(d, cap), (n, kind, cap)
    data = bytes(rnd.randrange(4) for _ in range(3 << 20))
    for bid in (4, 5, 6, 7):
        sd = L.make_sd(bid, stream_checksum=True, block_checksum=True)
        assert host(L.compress_frame(dev(data), sd)) == oracle.compress_frame(data, oracle.params(bid, True, True)), bid


@pytest.mark.parametrize("row", [((0, 1, 7), 133159392, 0x1686045A), ((0, 1, 4), 131956528, 0xAB492B3C),
                                 ((0, 1, 5), 136145906, 0xE62BB3AC), ((1, 0, 6), 133770948, 0x7D1BC1BA)])
def test_readback_known_answers_256mib(readback, row):
    """SURVEY.md App. F known answers (frame size + XXH32) through the
    read-back probe: k_encode (B7), k_encode16 (B4), k_encode_p17 (B5) and
    k_encode at B6 with the content checksum."""
    (sc, bc, bid), size, h = row
    src = L.gen_synthetic(256 << 20)
    fr = L.compress_frame(src, L.make_sd(bid, bool(sc), bool(bc)))
    assert fr.numel() == size and L.xxh32(fr) == h


def test_readback_block_dependent_frames(readback, golden):
    """-BD frames (k_link_warm, k_encode_linked_round / _chain, k_encode_linked)."""
    for f in golden["bd_frames"]:
        sd = L.make_sd(f["bid"], f["stream_checksum"], f["block_checksum"], block_dependence=True)
        assert host(L.compress_frame(dev(bd_data(f)), sd)) == read_golden(f["file"]), f["name"]


def test_readback_sharded_encode(readback):
    """k_encode_pub (the streamed gather's encoder) through the read-back
    probe: the shard's records equal the single-call frame's."""
    n = (24 << 20) + 77
    src = L.gen_synthetic(n, seed=9)
    sd = L.make_sd(7, stream_checksum=False, block_checksum=True)
    want = L.compress_frame(src, sd)
    ws = L.shard_workspace(n, sd)
    L.shard_reset(n, sd, ws)
    L.shard_encode(src, sd, ws)
    body = L.shard_body_bytes(n, sd, ws)
    hdr = L.frame_header(sd)
    out = torch.empty(len(hdr) + body + 4, dtype=torch.uint8, device="cuda")
    out[:len(hdr)] = torch.frombuffer(bytearray(hdr), dtype=torch.uint8).cuda()
    L.shard_assemble(src, n, sd, ws, out[len(hdr):len(hdr) + body])
    out[len(hdr) + body:] = 0
    assert torch.equal(out, want)


def test_capture_before_any_check_is_exact(monkeypatch, golden_inputs):
    """a compress captured into a graph on a device whose order
    check has not run yet takes the read-back probe (the check synchronises
    and cannot run inside a capture), so the replayed graph is exact
    either way.  A fresh process guarantees the device is unchecked."""
    import subprocess
    import sys
    import os
    code = r'''
import ctypes, sys, torch
sys.path.insert(0, sys.argv[1])
import lz4mt_amd as L
data = open(sys.argv[2], "rb").read()
src = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
sd = L.make_sd(5, False, True)
cap = L.frame_bound(src.numel(), sd)
frame = torch.zeros(cap, dtype=torch.uint8, device="cuda")
fsz = torch.zeros(2, dtype=torch.int64, device="cuda")
ws = L.compress_workspace(src.numel(), sd)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    r = L.lib.lz4mtHipCompressFrameAsync(ctypes.c_void_p(src.data_ptr()), src.numel(),
        ctypes.c_void_p(frame.data_ptr()), cap, ctypes.c_void_p(fsz.data_ptr()), ctypes.byref(sd),
        ctypes.c_void_p(ws.data_ptr()), ws.numel(), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert r == 0
g.replay()
torch.cuda.synchronize()
sys.stdout.buffer.write(bytes(frame[:int(fsz[0].item())].cpu().numpy().tobytes()))
'''
    import tempfile
    data = golden_inputs["syn300k"] * 4
    with tempfile.NamedTemporaryFile(suffix=".bin") as f:
        f.write(data)
        f.flush()
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        r = subprocess.run([sys.executable, "-c", code, root, f.name], capture_output=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout == oracle.compress_frame(data, oracle.params(5, False, True))
