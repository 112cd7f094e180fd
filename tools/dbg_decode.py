"""Finds the first golden decode vector the GPU gets wrong and explains which
LZ4 sequence produced the first wrong byte (host-side parse of the block)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import lz4mt_amd as L  # noqa: E402
import oracle  # noqa: E402

g = json.load(open(os.path.join(ROOT, "tests/golden/golden.json")))
blob = open(os.path.join(ROOT, "tests/golden/decode_blocks.bin"), "rb").read()


def sequences(blk):
    ip, op, out = 0, 0, []
    while ip < len(blk):
        t = blk[ip]; s0 = ip; ip += 1
        lit = t >> 4
        if lit == 15:
            while True:
                b = blk[ip]; ip += 1; lit += b
                if b != 255: break
        lp = ip; ip += lit
        if ip >= len(blk):
            out.append((s0, op, lit, 0, 0)); break
        off = blk[ip] | (blk[ip + 1] << 8); ip += 2
        ml = (t & 15) + 4
        if (t & 15) == 15:
            while True:
                b = blk[ip]; ip += 1; ml += b
                if b != 255: break
        out.append((s0, op, lit, off, ml)); op += lit + ml
    return out


for v in g["decode"]:
    if v["variant"] != "valid":
        continue
    blk = blob[v["off"]:v["off"] + v["len"]]
    r, got = L.decompress_block(blk, v["cap"])
    r2, want = oracle.decompress_block(blk, v["cap"])
    if got != want:
        i = next(k for k in range(min(len(got), len(want))) if got[k] != want[k])
        print("vector", {k: v[k] for k in ("src", "cap", "len")}, "ret", r, r2, "first diff at", i,
              "wrong bytes", sum(1 for a, b in zip(got, want) if a != b))
        seqs = sequences(blk)
        for n, (s0, op, lit, off, ml) in enumerate(seqs):
            if op <= i < op + lit + ml:
                for m in range(max(0, n - 3), min(len(seqs), n + 3)):
                    s = seqs[m]
                    print("  seq", m, "tok@", s[0], "op", s[1], "lit", s[2], "off", s[3], "ml", s[4],
                          "<-- first wrong" if m == n else "")
                break
        print("  got ", got[i - 8:i + 24].hex())
        print("  want", want[i - 8:i + 24].hex())
        break
else:
    print("all valid decode vectors OK")
