"""The exchange-probe window of encode_block_v5 (LZ4MT_ENC_XCHG, the
hash-product tag LZ4MT_ENC_HTAG), restated lane by lane in
tools/enc_model.py (encode_xchg), against the oracle on the CPU: with the
exchanges applied in ascending lane order -- the hardware property the
kernel relies on and lz4mtHipCheckEncoderOrder checks on the device -- each
lane's candidate is LZ4 1.9.3's sequential one, so the
blocks are byte-identical, also on a 3-letter alphabet where same-bucket
collisions and tag aliases are frequent."""
import os
import random
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import oracle  # noqa: E402
import enc_model  # noqa: E402


def _cases():
    rnd = random.Random(1)
    syn = oracle.gen_synthetic(1 << 20, 3)
    yield "appf", syn[:70000]
    yield "appf_odd", syn[333:333 + 100003]
    yield "abc", bytes(rnd.randrange(3) for _ in range(65547))
    yield "period37", (bytes(rnd.randrange(256) for _ in range(37)) * 2500)[:90000]
    yield "zeros", bytes(80000)
    yield "random", oracle.gen_random(70000, 5)


@pytest.mark.parametrize("name,data", list(_cases()), ids=[c[0] for c in _cases()])
def test_exchange_probe_model_matches_oracle(name, data):
    n = len(data)
    for cap in (n, n + n // 255 + 16):   # lz4mt's cap = n (limitedOutput) and an unlimited one
        assert enc_model.encode(data, cap, xchg=True) == oracle.compress_block(data, cap), (name, cap)
