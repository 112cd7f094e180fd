"""Per-window (encoder) / per-sequence (decoder) SQ counter summary of a
tools/gpu_round.sh `sq` pass: rocprofv3 --pmc SQ_* over tools/kprof.py 2
(2 GiB App. F, 4 MiB blocks), divided by the window and sequence counts
tools/kstats.py 2 measured on the same input (its diagnostic twins count
them).  SQ cycle counters are quad-cycles (MI355X_MICROARCH.md): x4 for
shader cycles.
usage: python tools/sqsum.py <rocprof dir> <kstats.txt>"""
import csv
import glob
import re
import sys

f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
ks = open(sys.argv[2]).read()
windows = int(re.search(r"windows (\d+)", ks).group(1))
seqs = int(re.search(r"sequences (\d+)", ks).group(1))
agg = {}
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].strip()
    if k in ("k_encode", "k_decode"):
        agg.setdefault(k, {})
        agg[k][r["Counter_Name"]] = agg[k].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
units = {"k_encode": windows, "k_decode": seqs}
print(f"windows {windows}, sequences {seqs} (2 GiB App. F, 4 MiB blocks)")
for k, v in agg.items():
    per = {a.replace("SQ_", ""): round(b / units[k], 1) for a, b in sorted(v.items())}
    cyc = {c: round(per[c] * 4) for c in ("WAVE_CYCLES", "WAIT_ANY", "ACTIVE_INST_ANY") if c in per}
    print(k, "per", "window" if k == "k_encode" else "sequence", per, "shader cycles", cyc)
