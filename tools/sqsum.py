"""Per-window / per-sequence SQ counter summary of a tools/kprof.py 2 PMC run."""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = {}
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:20]
    if k in ("k_encode", "k_decode"):
        agg.setdefault(k, {})
        agg[k][r["Counter_Name"]] = agg[k].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
units = {"k_encode": 265152366 / 4, "k_decode": 252137000 / 4}   # windows / sequences in 2 GiB
for k, v in agg.items():
    print(k, "per", "window" if k == "k_encode" else "sequence", {a.replace("SQ_", ""): round(b / units[k], 1) for a, b in sorted(v.items())})
