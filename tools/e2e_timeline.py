"""GPU timeline (kernels + copies) of the measured pass of tools/e2e_one.py from
a rocprofv3 --kernel-trace --memory-copy-trace run:
python tools/e2e_timeline.py <dir with *_kernel_trace.csv and *_memory_copy_trace.csv>"""
import csv
import glob
import os
import sys

d = sys.argv[1]
K = list(csv.DictReader(open(glob.glob(os.path.join(d, "*kernel_trace.csv"))[0])))
M = list(csv.DictReader(open(glob.glob(os.path.join(d, "*memory_copy_trace.csv"))[0])))
ev = [(int(k["Start_Timestamp"]), int(k["End_Timestamp"]), "K", k["Kernel_Name"].split("(")[0].replace("lz4mt::", ""),
       k["Stream_Id"], k["Queue_Id"], int(k["Grid_Size_X"]) // 64) for k in K]
ev += [(int(m["Start_Timestamp"]), int(m["End_Timestamp"]), "C", m["Direction"].replace("MEMORY_COPY_", ""),
        m["Stream_Id"], "-", 0) for m in M]
ev.sort()
enc = [e for e in ev if e[3] == "k_encode"]
nper = len(enc) // 2   # two passes; the second is measured
start = enc[nper][0] - 50_000_000 if nper else ev[0][0]
keep = {"k_encode", "k_decode", "k_frame_assemble", "k_xxh32_stored", "k_xxh32_frame_blocks"}
t0 = None
print("start_ms end_ms dur_ms kind name stream queue workgroups (ms from the first event shown)")
for e in ev:
    if e[0] < start:
        continue
    t0 = e[0] if t0 is None else t0
    if e[2] == "C" or e[3] in keep:
        print(f"{(e[0] - t0) / 1e6:8.1f} {(e[1] - t0) / 1e6:8.1f} {(e[1] - e[0]) / 1e6:7.1f} {e[2]} {e[3]:24s} "
              f"s{e[4]} q{e[5]} wg{e[6]}")
