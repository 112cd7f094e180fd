"""Test configuration: `gpu` marker, repo root on sys.path, golden fixtures."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


def read_golden(rel):
    with open(os.path.join(GOLDEN, rel), "rb") as f:
        return f.read()


@pytest.fixture(scope="session")
def golden_inputs(golden):
    return {k: read_golden(v["file"]) for k, v in golden["inputs"].items()}


@pytest.fixture(scope="session")
def decode_blob():
    return read_golden("decode_blocks.bin")


def with_stream_size(frame, n):
    """The same frame with FLG.3 set and the u64 content size in the header
    (src/lz4mt.cpp:335-369: magic, FLG, BD, [size], HC over FLG..size)."""
    import struct
    import xxhash
    flg, bd = frame[4] | 0x08, frame[5]
    desc = bytes([flg, bd]) + struct.pack("<Q", n)
    hc = (xxhash.xxh32(desc, seed=0).intdigest() >> 8) & 0xFF
    return frame[:4] + desc + bytes([hc]) + frame[7:]


@pytest.fixture(scope="session")
def known_answers():
    with open(os.path.join(GOLDEN, "known_answers.json")) as f:
        return json.load(f)


def checksum_of_checksums(t, chunk=16 << 20):
    """XXH32 over the little-endian u32 XXH32 digests of consecutive ``chunk``
    pieces of a device tensor (the "chunks" values of known_answers.json);
    the digests come from the library (lz4mtHipXxh32Chunks)."""
    import xxhash

    import lz4mt_amd as L
    d = L.xxh32_chunks(t, chunk).cpu().numpy().astype("<u4").tobytes()
    return xxhash.xxh32(d).intdigest()


def bd_data(f):
    """The input of a -BD golden entry: its "kind" (default "bd" =
    bd_input) at f["bytes"] / f["seed"]; "zeros", "random" (every block
    raw) and "mixed" (random, zero and bd_input pieces) cover the edge
    cases (tests/golden/make_golden.py)."""
    import random

    from oracle import gen_random
    n, seed, kind = f["bytes"], f["seed"], f.get("kind", "bd")
    if kind == "zeros":
        return bytes(n)
    if kind == "random":
        return gen_random(n, seed)
    if kind == "mixed":
        rnd = random.Random(seed)
        out = bytearray()
        while len(out) < n:
            k = rnd.randrange(3)
            m = rnd.randrange(1, 120_000)
            out += gen_random(m, rnd.randrange(1 << 30)) if k == 0 else bytes(m) if k == 1 else \
                bd_input(m, rnd.randrange(1 << 30))
        return bytes(out[:n])
    return bd_input(n, seed)


def bd_input(n, seed):
    """Block-dependent (-BD) test input with matches across block
    boundaries: App. F text with pieces re-copied from up to 64 KiB back
    (deterministic on any host; tests/golden/make_golden.py uses it)."""
    import random

    from oracle import gen_synthetic
    rnd = random.Random(seed)
    base = gen_synthetic(n + 65536, seed)
    out = bytearray()
    pos = 0
    while len(out) < n:
        if len(out) > 70000 and rnd.random() < 0.5:
            a = len(out) - rnd.randrange(4, 65535)
            out += out[a:a + rnd.randrange(4, 300)]
        else:
            k = rnd.randrange(1, 200)
            out += base[pos:pos + k]
            pos += k
    return bytes(out[:n])
