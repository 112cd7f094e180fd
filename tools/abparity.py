"""Quick parity screen of an A/B build (LZ4MT_AMD_LIB=exp_libs/<v>.so): frames
of App. F text, a collision-heavy mixed input, random bytes and words of a
small random vocabulary at block ids 4..7 against
the CPU oracle, plus the 256 MiB B7 -Sx -BX known answer.  Prints one line;
exit 1 on a mismatch.  (The full parity suite runs on the build that is
kept: tools/gpu_round.sh abtest / tests.)"""
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402
import oracle  # noqa: E402


def main():
    name = os.path.basename(os.environ.get("LZ4MT_AMD_LIB", "product"))
    rnd = random.Random(5)
    syn = oracle.gen_synthetic(12 << 20, 9)
    mixed = bytearray(syn[:6 << 20])
    for s in range(0, len(mixed), 1 << 20):   # 3-letter stretches: many same-bucket collisions
        for i in range(s, s + 200_000):
            mixed[i] = 97 + rnd.randrange(3)
    # every byte value in every hash-input position: random bytes, and words
    # drawn from a small random vocabulary (many matches, varied 5-byte keys)
    rand = rnd.randbytes(6 << 20)
    vocab = [rnd.randbytes(rnd.randrange(3, 12)) for _ in range(4000)]
    words = bytearray()
    while len(words) < (6 << 20):
        words += vocab[rnd.randrange(len(vocab))]
    bad = []
    for label, data in (("appf", syn), ("mixed", bytes(mixed)), ("random", rand), ("vocab", bytes(words[:6 << 20]))):
        src = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
        for bid in (4, 5, 6, 7):
            for sck, bck in ((False, True), (True, False)):
                fr = L.compress_frame(src, L.make_sd(bid, sck, bck))
                got = bytes(fr.cpu().numpy().tobytes())
                if got != oracle.compress_frame(data, oracle.params(bid, sck, bck)):
                    bad.append((label, bid, sck, bck))
                out, r = L.decompress_frame(fr)
                if r != 0 or not torch.equal(out, src):
                    bad.append(("decode", label, bid, sck, bck))
    t = L.gen_synthetic(256 << 20)
    fr = L.compress_frame(t, L.make_sd(7, False, True))
    if (fr.numel(), L.xxh32(fr)) != (133159392, 0x1686045A):
        bad.append("known answer 256 MiB B7 -Sx -BX")
    out, r = L.decompress_frame(fr)
    if r != 0 or L.xxh32(out) != 0xE6F24EBA:
        bad.append("decode of the 256 MiB known answer")
    print(f"{name}: parity {'OK' if not bad else 'MISMATCH ' + str(bad)}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
