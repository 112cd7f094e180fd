"""GPU parity for block-dependent (-BD) frames, SURVEY.md §8(f) #4.

Compress: the reference's compressBlockDependency (src/lz4mt.cpp:460-538)
replayed on liblz4 1.9.3 with its exact call sequence gives the golden
frames (tests/golden/make_golden.py: bd_frame_reference for 64 / 256 KiB
blocks, bd_frame_contiguous for 1 / 4 MiB blocks, where the reference reads
each block over its own dictionary -- DESIGN.md).  The device encoder must
write the same bytes, through the device frame engine and through
lz4mtCompress (one batch and many).

Decompress: decompressBlockDependency (src/lz4mt.cpp:737-845): the golden
frames decode to their inputs; damaged frames give the oracle's result code
and bytes (the block checksum is checked before a block is written there).
"""
import pytest
import torch
import xxhash

import oracle
from conftest import bd_data, bd_input, read_golden

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


def dev(b):
    t = torch.empty(max(len(b), 1), dtype=torch.uint8, device="cuda")
    if b:
        t[:len(b)].copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8))
    return t[:len(b)]


def host(t):
    return bytes(t.cpu().numpy().tobytes())


def _sd(f):
    return L.make_sd(f["bid"], f["stream_checksum"], f["block_checksum"], block_dependence=True)


def test_bd_golden_frames_device(golden):
    for f in golden["bd_frames"]:
        data = bd_data(f)
        frame = read_golden(f["file"])
        got = host(L.compress_frame(dev(data), _sd(f)))
        assert got == frame, f["name"]
        out, r = L.decompress_frame(dev(frame))
        assert r == 0 and host(out) == data, f["name"]


@pytest.mark.parametrize("rounds", ["1", "2", "serial", "chain2", "chain3-1", "chain0"])
def test_bd_rounds_and_serial_finish(golden, monkeypatch, rounds):
    """The parallel rounds capped at 1 or 2 leave blocks unsettled: the serial
    kernel finishes from the first unsettled block (its entry table exact);
    "serial" runs the one-wave kernel alone; "chainG[-R]" runs the chained
    rounds with G blocks per chain (capped at R rounds), "chain0" the
    one-block-per-wave rounds at every block size.  Same bytes as the
    reference."""
    if rounds == "serial":
        monkeypatch.setenv("LZ4MT_AMD_BD_SERIAL", "1")
    elif rounds.startswith("chain"):
        g, _, r = rounds[5:].partition("-")
        monkeypatch.setenv("LZ4MT_AMD_BD_CHAIN", g)
        if r:
            monkeypatch.setenv("LZ4MT_AMD_BD_ROUNDS", r)
    else:
        monkeypatch.setenv("LZ4MT_AMD_BD_ROUNDS", rounds)
    for f in golden["bd_frames"]:
        data = bd_data(f)
        assert host(L.compress_frame(dev(data), _sd(f))) == read_golden(f["file"]), (f["name"], rounds)
        out, r = L.decompress_frame(dev(read_golden(f["file"])))
        assert r == 0 and host(out) == data, (f["name"], rounds)
    for f in golden["bd_known"]:
        if f["bytes"] > (64 << 20):
            continue
        data = bd_data(f)
        frame = L.compress_frame(dev(data), _sd(f))
        assert (frame.numel(), L.xxh32(frame)) == (f["size"], f["xxh32"]), (f["name"], rounds)


def test_bd_known_answers_device(golden):
    for f in golden["bd_known"]:
        data = bd_data(f)
        assert xxhash.xxh32(data).intdigest() == f["content_xxh32"]
        frame = L.compress_frame(dev(data), _sd(f))
        assert (frame.numel(), L.xxh32(frame)) == (f["size"], f["xxh32"]), f["name"]
        out, r = L.decompress_frame(frame)
        assert r == 0 and L.xxh32(out) == f["content_xxh32"], f["name"]


@pytest.mark.parametrize("mode", ["DEVICE", "PARALLEL", "SEQUENTIAL"])
@pytest.mark.parametrize("batches", ["one", "many"])
def test_bd_callback_api(golden, monkeypatch, mode, batches):
    """lz4mtCompress / lz4mtDecompress on -BD frames: the device engine in
    every mode (the reference bypasses ctx.compress / ctx.decompress for
    them); with small batches the lz4 table and the 64 KiB history carry
    across batches."""
    if batches == "many":
        monkeypatch.setenv("LZ4MT_AMD_BATCH0_MIB", "1")
        monkeypatch.setenv("LZ4MT_AMD_BATCH_MIB", "1")
    m = {"DEVICE": L.MODE_DEVICE, "PARALLEL": L.MODE_PARALLEL, "SEQUENTIAL": L.MODE_SEQUENTIAL}[mode]
    for f in golden["bd_frames"] + [k for k in golden["bd_known"] if k["bid"] >= 6]:
        data = bd_data(f)
        r, frame = L.compress(data, _sd(f), mode=m)
        assert r == 0, (f["name"], L.result_to_string(r))
        if "file" in f:
            assert frame == read_golden(f["file"]), (f["name"], mode, batches)
        else:
            assert (len(frame), xxhash.xxh32(frame).intdigest()) == (f["size"], f["xxh32"]), (f["name"], mode)
        r, out, sd = L.decompress(frame, len(data) + 64, mode=m)
        assert r == 0 and out == data, (f["name"], mode, batches, L.result_to_string(r))
        assert sd.flg.blockIndependence == 0


@pytest.mark.parametrize("api", ["device", "DEVICE", "PARALLEL"])
def test_bd_damaged_frames_vs_oracle(golden, api):
    """Flipped bytes, truncations and rewritten size words in -BD frames:
    the oracle's result code (decompressBlockDependency order: size, data,
    checksum word, checksum, decode, write) and its bytes."""
    import random
    rnd = random.Random({"device": 1, "DEVICE": 2, "PARALLEL": 3}[api])
    f = golden["bd_frames"][0]   # 64 KiB blocks, block checksums
    data = bd_data(f)
    frame = read_golden(f["file"])
    cap = len(data) + (1 << 20)
    for it in range(40):
        b = bytearray(frame)
        kind = it % 3
        if kind == 0:
            b[rnd.randrange(7, len(b))] ^= 1 << rnd.randrange(8)
        elif kind == 1:
            del b[rnd.randrange(8, len(b)):]
        else:
            a = rnd.randrange(7, len(b) - 4)
            b[a:a + 4] = rnd.randrange(1 << 32).to_bytes(4, "little")
        rw, ow = oracle.decompress_frame(bytes(b), cap)
        if api == "device":
            out = torch.empty(cap, dtype=torch.uint8, device="cuda")
            o, r = L.decompress_frame(dev(bytes(b)), out=out, check=False)
            got = host(o)
        else:
            r, got, _ = L.decompress(bytes(b), cap, mode=L.MODE_DEVICE if api == "DEVICE" else L.MODE_PARALLEL)
        assert r == rw, (it, kind, L.result_to_string(r), L.result_to_string(rw))
        assert got == ow, (it, kind, len(got), len(ow))


@pytest.mark.parametrize("period", [60000, 65535, 200_000])
def test_bd_long_chains(monkeypatch, period):
    """Input repeating with a period near the 64 KiB window: every block's
    bytes come from the previous block's, so a wrong history propagates
    block after block and the decoder's rounds cannot settle before the
    serial finish takes over (60000 / 65535 with 64 KiB blocks).  The
    parallel encode and decode must give the serial kernels' bytes, and the
    oracle must decode the frame to the input."""
    rnd = __import__("random").Random(period)
    unit = bytes(rnd.randrange(256) for _ in range(period))
    data = (unit * (3_000_000 // period + 1))[:3_000_000]
    for bid in (4, 5):
        sd = L.make_sd(bid, True, True, block_dependence=True)
        fr = host(L.compress_frame(dev(data), sd))
        monkeypatch.setenv("LZ4MT_AMD_BD_SERIAL", "1")
        assert host(L.compress_frame(dev(data), sd)) == fr, (period, bid)
        o_ser, r_ser = L.decompress_frame(dev(fr))
        monkeypatch.delenv("LZ4MT_AMD_BD_SERIAL")
        out, r = L.decompress_frame(dev(fr))
        assert r == 0 and r_ser == 0 and host(out) == data and host(o_ser) == data, (period, bid)
        rw, ow = oracle.decompress_frame(fr, len(data) + (1 << 20))
        assert rw == 0 and ow == data


@pytest.mark.parametrize("bid", [4, 5])
def test_bd_parallel_equals_serial_64mib(monkeypatch, bid):
    """64 MiB of App. F input (1024 / 256 blocks): the parallel rounds write
    the one-wave serial kernel's frame, and both decoders give the input
    back (size-independent check beside the 9 MiB known answers)."""
    src = L.gen_synthetic(64 << 20, seed=77)
    sd = L.make_sd(bid, False, True, block_dependence=True)
    fr = L.compress_frame(src, sd)
    monkeypatch.setenv("LZ4MT_AMD_BD_SERIAL", "1")
    fr_ser = L.compress_frame(src, sd)
    out_ser, r_ser = L.decompress_frame(fr)
    monkeypatch.delenv("LZ4MT_AMD_BD_SERIAL")
    assert fr.numel() == fr_ser.numel() and torch.equal(fr, fr_ser)
    out, r = L.decompress_frame(fr)
    assert r == 0 and r_ser == 0 and torch.equal(out, src) and torch.equal(out_ser, src)


@pytest.mark.parametrize("api", ["device", "DEVICE", "PARALLEL"])
def test_bd_reference_written_b6_b7_frames(golden, api):
    """-BD frames the reference itself writes with 1 and 4 MiB blocks
    (compressBlockDependency on liblz4 1.9.3, src/lz4mt.cpp:460-538: after
    LZ4_slideInputBuffer each block is read over its own dictionary, so the
    bytes differ from this library's contiguous stream and on App. F input
    they do not decode back).  Decoding them is what a user with existing
    -BD archives does: lz4mtDecompress must give decompressBlockDependency's
    bytes and result (src/lz4mt.cpp:737-845, 997-1007), here pinned by
    liblz4's LZ4_decompress_safe_withPrefix64k (make_golden.py
    bd_decompress_reference) and the oracle."""
    from lz4mt_amd import RESULT_NAMES
    for f in golden["bd_ref_decode"]:
        frame = read_golden(f["file"])
        assert (len(frame), xxhash.xxh32(frame).intdigest()) == (f["size"], f["xxh32"]), f["name"]
        cap = f["bytes"] + (1 << (8 + 2 * f["bid"])) + (1 << 20)   # room for a whole block past the end
        if api == "device":
            out = torch.empty(cap, dtype=torch.uint8, device="cuda")
            o, r = L.decompress_frame(dev(frame), out=out, check=False)
            got = host(o)
        else:
            r, got, _ = L.decompress(frame, cap, mode=L.MODE_DEVICE if api == "DEVICE" else L.MODE_PARALLEL)
        assert RESULT_NAMES[r] == f["result"], (f["name"], api, RESULT_NAMES[r])
        assert (len(got), xxhash.xxh32(got).intdigest()) == (f["out_bytes"], f["out_xxh32"]), (f["name"], api)
        rw, ow = oracle.decompress_frame(frame, cap)
        assert (r, got) == (rw, ow), (f["name"], api)


def test_bd_async_calls_on_two_streams(golden):
    """Two asynchronous -BD compress calls from one thread on two streams,
    nothing synchronised in between (lz4mtHipCompressFrameAsyncEx): each
    call's plan, carried table and round scratch live in its own workspace,
    so both frames are the reference's (the golden -BD frames)."""
    import ctypes
    fs = [f for f in golden["bd_frames"] if f["bytes"] >= 1_000_000][:2]
    assert len(fs) == 2
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    jobs = []
    for f, st in zip(fs, streams):
        data = dev(bd_data(f))
        sd = _sd(f)
        cap = L.frame_bound(data.numel(), sd)
        out = torch.empty(cap, dtype=torch.uint8, device="cuda")
        ws = L.compress_workspace(data.numel(), sd)
        fsz = torch.zeros(1, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()   # inputs ready before the side streams read them
        jobs.append((f, data, sd, out, ws, fsz, st))
    for f, data, sd, out, ws, fsz, st in jobs * 2:   # A, B, A, B back to back
        r = L.lib.lz4mtHipCompressFrameAsyncEx(ctypes.c_void_p(data.data_ptr()), data.numel(),
                                               ctypes.c_void_p(out.data_ptr()), out.numel(),
                                               ctypes.c_void_p(fsz.data_ptr()), ctypes.byref(sd), 0,
                                               ctypes.c_void_p(ws.data_ptr()), ws.numel(),
                                               ctypes.c_void_p(st.cuda_stream))
        assert r == 0
    torch.cuda.synchronize()
    for f, data, sd, out, ws, fsz, st in jobs:
        assert host(out[:int(fsz[0].item())]) == read_golden(f["file"]), f["name"]


def _ref_entries(golden):
    """The reference-written 1 / 4 MiB -BD frames: fixtures (bd_ref_decode) and
    known answers over several full blocks (bd_ref_known), with their inputs."""
    from oracle import gen_synthetic
    out = []
    for f in golden["bd_ref_decode"] + golden["bd_ref_known"]:
        data = bd_input(f["bytes"], f["seed"]) if f["kind"] == "bd" else gen_synthetic(f["bytes"], f["seed"])
        out.append((f, data))
    return out


@pytest.mark.parametrize("api,batches,path", [
    ("device", "one", "rounds"), ("device", "one", "serial"), ("device", "one", "round1"),
    ("DEVICE", "one", "rounds"), ("DEVICE", "many", "rounds"), ("PARALLEL", "many", "rounds"),
])
def test_bd_reference_bytes_mode(golden, monkeypatch, api, batches, path):
    """LZ4MT_AMD_BD_REFERENCE=1: -BD frames with 1 and 4 MiB blocks written
    byte for byte as the reference writes them (compressBlockDependency,
    src/lz4mt.cpp:460-538, translate() at 486-488: lz4 1.9.3's
    LZ4_slideInputBuffer returns the dictionary's own address, so from the
    second block on each full block is read over its own dictionary).  Pinned
    by frames liblz4 1.9.3 wrote with the reference's call sequence
    (make_golden.py bd_frame_reference): fixtures and size + XXH32 known
    answers.  Parallel rounds, the one-wave serial kernel, one round + the
    serial finish, the callback engine in one and many batches."""
    monkeypatch.setenv("LZ4MT_AMD_BD_REFERENCE", "1")
    if path == "serial":
        monkeypatch.setenv("LZ4MT_AMD_BD_SERIAL", "1")
    if path == "round1":
        monkeypatch.setenv("LZ4MT_AMD_BD_ROUNDS", "1")
    if batches == "many":
        monkeypatch.setenv("LZ4MT_AMD_BATCH0_MIB", "1")
        monkeypatch.setenv("LZ4MT_AMD_BATCH_MIB", "1")
    for f, data in _ref_entries(golden):
        sd = L.make_sd(f["bid"], stream_checksum=f["stream_checksum"], block_checksum=f["block_checksum"],
                       block_dependence=True)
        if api == "device":
            frame = host(L.compress_frame(dev(data), sd))
        else:
            r, frame = L.compress(data, sd, mode=L.MODE_DEVICE if api == "DEVICE" else L.MODE_PARALLEL)
            assert r == 0, (f["name"], L.result_to_string(r))
        if "file" in f:
            assert frame == read_golden(f["file"]), (f["name"], api, batches, path)
        else:
            assert (len(frame), xxhash.xxh32(frame).intdigest()) == (f["size"], f["xxh32"]), (f["name"], api, path)


def test_bd_reference_bytes_mode_off_is_the_decodable_stream(golden):
    """Without the knob the same inputs give the contiguous (decodable)
    stream: a different frame wherever a full block follows the first, and
    it decodes back to the input."""
    for f, data in _ref_entries(golden)[-2:]:
        sd = L.make_sd(f["bid"], stream_checksum=f["stream_checksum"], block_checksum=f["block_checksum"],
                       block_dependence=True)
        frame = L.compress_frame(dev(data), sd)
        assert (frame.numel(), xxhash.xxh32(host(frame)).intdigest()) != (f["size"], f["xxh32"]), f["name"]
        out, r = L.decompress_frame(frame)
        assert r == 0 and host(out) == data, f["name"]
