"""Summarises a tools/prof.sh run into profiles/<tag>_pmc.json: per kernel,
average duration (kernel trace), FETCH_SIZE and WRITE_SIZE per launch in
bytes (rocprofv3 reports KiB).  gfx950 note (MI355X_MICROARCH.md): FETCH_SIZE
counts HALF the bytes of 16-B-per-lane streaming reads; other access widths
are uncalibrated, so both the raw and the x2 figure are kept.
usage: python tools/pmcsum.py gpurun_out/prof_<tag> profiles/<tag>_pmc.json"""
import csv
import glob
import json
import sys

src, dst = sys.argv[1], sys.argv[2]
out = {}
for name, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
    f = glob.glob(f"{src}/{name}/*counter_collection.csv")[0]
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if not k.startswith("k_"):
            continue
        e = out.setdefault(k, {"launches": {}, "fetch_bytes": [], "write_bytes": [], "ns": []})
        v = float(r["Counter_Value"]) * 1024.0
        (e["fetch_bytes"] if counter == "FETCH_SIZE" else e["write_bytes"]).append(v)
        e["ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
res = {}
for k, e in out.items():
    fb = max(e["fetch_bytes"]) if e["fetch_bytes"] else 0.0
    wb = max(e["write_bytes"]) if e["write_bytes"] else 0.0
    res[k] = {"fetch_bytes": fb, "fetch_bytes_x2": 2 * fb, "write_bytes": wb,
              "traffic_bytes": fb + wb, "max_ns": max(e["ns"])}
stats = glob.glob(f"{src}/trace/*kernel_stats.csv")
if stats:
    for r in csv.DictReader(open(stats[0])):
        if r["Name"] in res:
            res[r["Name"]]["trace_avg_ns"] = float(r["AverageNs"])
            res[r["Name"]]["trace_calls"] = int(r["Calls"])
json.dump({"workload": "tools/kprof.py 8: 8 GiB App. F synthetic, 4 MiB blocks, -Sx -BX", "kernels": res},
          open(dst, "w"), indent=1)
print(json.dumps(res, indent=1))
