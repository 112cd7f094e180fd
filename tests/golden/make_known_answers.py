"""Generates tests/golden/known_answers.json: known answers for the large
BASELINE.json configs (frame size, XXH32 of the frame and of the content,
and the chunked "checksum of checksums" of both: XXH32 over the LE u32
XXH32 digests of consecutive 16 MiB pieces).

The frames are computed by the pinned CPU oracle (oracle/lz4_oracle.c,
orc_stream_known_answer: the App. F input streamed batch by batch through
the lz4mt frame writer, reference src/lz4mt.cpp:335-457, 898-935).  The
oracle itself is pinned at 256 MiB by SURVEY.md App. F (checked first, below)
and by liblz4 1.9.3 (tests/test_oracle.py).

Run:  python tests/golden/make_known_answers.py
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle  # noqa: E402

CHUNK = 16 << 20
GiB = 1 << 30
# name -> (bytes, block id, stream checksum, block checksum, what it pins)
CASES = {
    "configs1_8gib_b7_SxBX": (8 * GiB, 7, False, True, "BASELINE configs[1] (-Sx -BX), the bench workload"),
    "8gib_b7_default": (8 * GiB, 7, True, False, "default flags: serial content checksum over 8 GiB"),
    "configs2_32gib_b7_SxBX": (32 * GiB, 7, False, True,
                               "BASELINE configs[2]: 32 GiB stream, frame and record offsets past 2^32"),
    "10gib_b6_SxBX": (10 * GiB, 6, False, True, "1 MiB blocks: parallel frame walk over a frame past 2^32"),
    "8gib_b5_SxBX": (8 * GiB, 5, False, True, "sweep: 256 KiB blocks (32768) at the bench size"),
    "8gib_b4_SxBX": (8 * GiB, 4, False, True, "sweep: 64 KiB blocks (131072, lz4's byU16 table, k_encode16)"),
}


def main():
    t0 = time.time()
    pin = oracle.known_answer(256 << 20, oracle.params(7, False, True), chunk=CHUNK)
    assert (pin["frame_size"], pin["frame_xxh32"], pin["content_xxh32"]) == (133159392, 0x1686045A, 0xE6F24EBA)
    out = {"chunk": CHUNK, "seed": 42, "generator": "SURVEY.md App. F", "cases": {}}
    only = [a for a in sys.argv[1:] if a in CASES]   # regenerate just these (merged into the file)
    if only:
        out = json.load(open(os.path.join(HERE, "known_answers.json")))
    for name, (n, bid, sck, bck, what) in CASES.items():
        if only and name not in only:
            continue
        ka = oracle.known_answer(n, oracle.params(bid, sck, bck), seed=42, chunk=CHUNK, threads=os.cpu_count() or 8)
        ka.update({"bytes": n, "block_id": bid, "stream_checksum": sck, "block_checksum": bck, "pins": what})
        out["cases"][name] = ka
        print(name, ka, f"{time.time() - t0:.0f}s", flush=True)
    with open(os.path.join(HERE, "known_answers.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
