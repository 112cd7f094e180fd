"""Summarises a tools/prof.sh run into profiles/<tag>_pmc.json (and, with
--current, profiles/pmc_current.json, which bench.py reads): per kernel the
average duration (kernel trace) and FETCH_SIZE / WRITE_SIZE per launch in
bytes (rocprofv3 reports KiB) on 8 GiB of App. F input, 4 MiB blocks,
-Sx -BX (flg 0x70) -- the bench configuration, recorded in "config" so
bench.py uses it only for that configuration.

Calibration: FETCH_SIZE / bytes of a kernel that reads a known byte count
exactly once at the load widths these kernels use (tools/fetch_cal.py,
summarised by tools/fetchcal_sum.py into the json given as the third
argument); bench.py divides each kernel's FETCH_SIZE by that factor.
With --bid=K (K != 7) the profile is the configs[4] sweep point of block id
K (appf runs only): profiles/pmc_b<K>.json, its encoder kernel
(k_encode16 at 64 KiB, k_encode_p17 at 256 KiB) calibrated like k_encode.
With --gib=G (G != 8) the input is G GiB (tools/kprof.py G): --gib=32 is
configs[2]'s 32 GiB stream, written to profiles/pmc_dec32.json (bench.py's
--decompress-only line reads its k_decode traffic there).
usage: python tools/pmcsum.py <gpu_round dir> <tag> [fcal_summary.json] [--current] [--bid=K] [--gib=G]"""
import csv
import glob
import json
import sys

src, tag = sys.argv[1], sys.argv[2]
GIB = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--gib=")), 8))
N = GIB << 30


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


bid = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--bid=")), 7))
appf = counters("appf")
rnd = counters("random") if bid == 7 and GIB == 8 else {}
for k in appf.values():
    k["traffic_raw"] = k["fetch_bytes"] + k["write_bytes"]
stats = glob.glob(f"{src}/trace/*kernel_stats.csv")
if stats:
    for r in csv.DictReader(open(stats[0])):
        name = r["Name"].split("(")[0].strip()
        if name in appf:
            appf[name]["trace_avg_ns"] = float(r["AverageNs"])
            appf[name]["trace_calls"] = int(r["Calls"])
# Calibration: FETCH_SIZE / bytes of a kernel that reads
# a known byte count exactly once (tools/fetch_cal.py: k_fetch_cal over 8 GiB
# with 1-, 4-, 8- and 16-byte loads per lane, the widths k_encode / k_decode
# use), accepted only at a physically possible rate (tools/fetchcal_sum.py).
# The random-input runs stay as diagnostics: k_encode does NOT stream random
# input once (its probe step grows after misses), so their ratio is a
# coverage, not a counter factor.
cal = {}
fc_path = sys.argv[3] if len(sys.argv) > 3 and not sys.argv[3].startswith("--") else None
enc_kernels = ("k_encode", "k_encode16", "k_encode_p17", "k_decode")
fc = json.load(open(fc_path)) if fc_path else None
if fc:
    facs = {w: v["factor"] for w, v in fc["widths"].items() if v["factor"]}
    f_lo, f_hi = min(facs.values()), max(facs.values())
    how = ("FETCH_SIZE / bytes read by k_fetch_cal (8 GiB read exactly once; tools/fetch_cal.py) per load width: " +
           ", ".join(f"{w.split('_')[1]} B {f}" for w, f in sorted(facs.items(), key=lambda x: int(x[0].split('_')[1]))) +
           f"; implied rates <= {fc['achievable_Bps'] / 1e12:.1f} TB/s")
    for k in enc_kernels:
        cal[k] = {"fetch_factor": (f_lo + f_hi) / 2, "fetch_factor_range": [f_lo, f_hi], "how": how,
                  "source": fc_path}
if "k_encode" in rnd:
    cal.setdefault("diagnostics", {})["k_encode_random_input_coverage"] = {
        "fetch_raw": rnd["k_encode"]["fetch_bytes"], "bytes": N,
        "note": "k_encode over 8 GiB of random bytes (every block raw): FETCH_SIZE / n, the probe coverage times "
                "the counter factor -- not a calibration"}
bm = 1 << (8 + 2 * bid)
res = {"tag": tag, "config": {"bytes": N, "block_bytes": bm, "flg": 0x70,
                              "workload": f"tools/kprof.py {GIB} --bid={bid}: {GIB} GiB App. F synthetic, {bm >> 10} KiB "
                                          "blocks, -Sx -BX"},
       "kernels": appf, "calibration": cal, "random_input": rnd}
out = (f"profiles/pmc_dec{GIB}.json" if GIB != 8 else
       f"profiles/{tag}_pmc.json" if bid == 7 else f"profiles/pmc_b{bid}.json")
json.dump(res, open(out, "w"), indent=1)
if "--current" in sys.argv:
    json.dump(res, open("profiles/pmc_current.json", "w"), indent=1)
print(json.dumps({"kernels": {k: appf[k] for k in enc_kernels if k in appf}, "calibration": cal},
                 indent=1))
