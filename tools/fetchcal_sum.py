"""Summarises the FETCH_SIZE calibration pass (tools/fetch_cal.py under
rocprofv3 --pmc FETCH_SIZE): per load width, FETCH_SIZE / bytes read and the
implied read rate (bytes / kernel duration), which must not exceed the
achievable HBM rate for the factor to be accepted.
usage: python tools/fetchcal_sum.py <rocprof dir> [GiB]"""
import csv
import glob
import json
import re
import sys

N = int(float(sys.argv[2] if len(sys.argv) > 2 else 8) * (1 << 30))
ACHIEVABLE = 6.3e12   # MI355X_MICROARCH.md: achievable HBM read rate
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
ORDER = [1, 1, 4, 4, 8, 8, 16, 16]   # tools/fetch_cal.py's launches (the trace drops the template argument)
rows = {}
cal = [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == "FETCH_SIZE" and
       re.match(r"(void )?(lz4mt::shard::)?k_fetch_cal", r["Kernel_Name"])]
cal.sort(key=lambda r: int(r["Dispatch_Id"]))
for w, r in zip(ORDER, cal):
    ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    rows.setdefault(w, []).append((float(r["Counter_Value"]) * 1024.0, ns))
res = {}
for w, v in sorted(rows.items()):
    runs = [{"fetch_bytes": fb, "factor": round(fb / N, 4), "ns": ns, "implied_TBps": round(N / ns / 1e3, 3),
             "physical": N / (ns * 1e-9) <= ACHIEVABLE} for fb, ns in v]
    ok = [x for x in runs if x["physical"]]
    res[f"width_{w}"] = {"runs": runs,
                         "factor": round(sum(x["factor"] for x in ok) / len(ok), 4) if ok else None}
print(json.dumps({"bytes_read_per_launch": N, "achievable_Bps": ACHIEVABLE, "widths": res}, indent=1))
