"""False candidates per sequence that the encoder's tag must filter
(tools/split_sim.c false_cands), App. F input: 64 KiB blocks on lz4's byU16
table (k_encode16) and 4 MiB blocks on byU32 (k_encode).  With t tag bits
each false candidate becomes an extra round trip with probability 2^-t, so
the table's LDS size (tag bits) trades against round trips per sequence.
usage: python tools/tag_sim.py"""
import ctypes
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402  (the App. F generator; test infrastructure)

so = "/tmp/split_sim.so"
subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", "-o", so,
                       os.path.join(os.path.dirname(os.path.abspath(__file__)), "split_sim.c")])
lib = ctypes.CDLL(so)
data = oracle.gen_synthetic(32 << 20, 42)
for name, bm, u16 in (("B4 byU16 (k_encode16)", 64 << 10, 1), ("B7 byU32 (k_encode)", 4 << 20, 0)):
    pr, fc, seqs = ctypes.c_uint64(0), ctypes.c_uint64(0), 0
    for off in range(0, len(data), bm):
        blk = data[off:off + bm]
        buf = ctypes.create_string_buffer(blk, len(blk))
        seqs += lib.false_cands(buf, len(blk), u16, ctypes.byref(pr), ctypes.byref(fc))
    f = fc.value / seqs
    print(f"{name}: {seqs} sequences, {pr.value / seqs:.1f} probes and {f:.2f} false candidates per sequence; "
          "extra round trips per sequence by tag bits: " +
          ", ".join(f"{t}b {f / 2 ** t:.3f}" for t in (2, 4, 6, 7, 8, 9, 10)))
