"""Summarises a tools/prof.sh run into profiles/<tag>_pmc.json (and, with
--current, profiles/pmc_current.json, which bench.py reads): per kernel the
average duration (kernel trace) and FETCH_SIZE / WRITE_SIZE per launch in
bytes (rocprofv3 reports KiB) on 8 GiB of App. F input, 4 MiB blocks,
-Sx -BX (flg 0x70) -- the bench configuration, recorded in "config" so
bench.py uses it only for that configuration.

Calibration (MI355X_MICROARCH.md: gfx950 FETCH_SIZE counts ~1/2 of the bytes
of wide streaming reads; other widths need a known byte count): the same
kernels on 8 GiB of random bytes, where every block is stored raw, so
k_encode streams its source once (n bytes) and k_decode copies n raw bytes;
fetch_factor = FETCH_SIZE / n.  k_xxh32_frame_blocks (reads exactly the
stored bytes) is the cross-check on the App. F run.
usage: python tools/pmcsum.py gpurun_out/prof_<tag> <tag> [--current]"""
import csv
import glob
import json
import sys

src, tag = sys.argv[1], sys.argv[2]
N = 8 << 30


def counters(run):
    out = {}
    for name, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        f = glob.glob(f"{src}/{name}_{run}/*counter_collection.csv")[0]
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].strip()
            if not k.startswith("k_"):
                continue
            e = out.setdefault(k, {"fetch_bytes": [], "write_bytes": [], "ns": []})
            (e["fetch_bytes"] if counter == "FETCH_SIZE" else e["write_bytes"]).append(float(r["Counter_Value"]) * 1024.0)
            e["ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return {k: {"fetch_bytes": max(e["fetch_bytes"] or [0.0]), "write_bytes": max(e["write_bytes"] or [0.0]),
                "max_ns": max(e["ns"])} for k, e in out.items()}


appf, rnd = counters("appf"), counters("random")
for k in appf.values():
    k["traffic_raw"] = k["fetch_bytes"] + k["write_bytes"]
stats = glob.glob(f"{src}/trace/*kernel_stats.csv")
if stats:
    for r in csv.DictReader(open(stats[0])):
        name = r["Name"].split("(")[0].strip()
        if name in appf:
            appf[name]["trace_avg_ns"] = float(r["AverageNs"])
            appf[name]["trace_calls"] = int(r["Calls"])
# k_encode: its source stream (n bytes, every launch) is counted at the
# factor the random-input run measures; what App. F input fetches beyond that
# (candidate-verify and match-count words: 256-B wave loads) at the guide's
# 1/2.  k_decode: the raw-copy run gives the factor of its 16-B-per-lane reads.
cal = {}
if "k_encode" in rnd:
    cal["k_encode"] = {"stream_bytes": N, "stream_factor": rnd["k_encode"]["fetch_bytes"] / N, "other_factor": 0.5,
                       "how": "source stream calibrated by k_encode over 8 GiB of random bytes (all blocks raw: the "
                              "source streamed once, n bytes known); the remaining fetches at the guide's x2",
                       "fetch_raw": rnd["k_encode"]["fetch_bytes"], "write_raw": rnd["k_encode"]["write_bytes"]}
if "k_decode" in rnd:
    cal["k_decode"] = {"fetch_factor": rnd["k_decode"]["fetch_bytes"] / N,
                       "how": "k_decode over the raw-block frame of 8 GiB of random bytes (n bytes copied)",
                       "fetch_raw": rnd["k_decode"]["fetch_bytes"], "write_raw": rnd["k_decode"]["write_bytes"]}
res = {"tag": tag, "config": {"bytes": N, "block_bytes": 4 << 20, "flg": 0x70,
                              "workload": "tools/kprof.py 8: 8 GiB App. F synthetic, 4 MiB blocks, -Sx -BX"},
       "kernels": appf, "calibration": cal, "random_input": rnd}
json.dump(res, open(f"profiles/{tag}_pmc.json", "w"), indent=1)
if "--current" in sys.argv:
    json.dump(res, open("profiles/pmc_current.json", "w"), indent=1)
print(json.dumps({"kernels": {k: appf[k] for k in ("k_encode", "k_decode") if k in appf}, "calibration": cal},
                 indent=1))
