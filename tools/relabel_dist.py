"""Re-labels committed N > 1 bench records with bench.py's round-6 labels
(VERDICT r05 item 1): `config.workload` says configs[3] only for a 64 GiB
run, `config.parallelism` names the transport that moved the records.
Measured values are untouched; a `relabelled` note records the change.
usage: python tools/relabel_dist.py profiles/<file>.json ..."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def relabel(line):
    cfg = line["config"]
    world = line["n_gpus"]
    bid = {64 << 10: 4, 256 << 10: 5, 1 << 20: 6, 4 << 20: 7}[cfg.get("block_bytes", 4 << 20)]
    strong = line.get("scaling") == "strong"
    old_w, old_p = cfg["workload"], cfg.get("parallelism")
    head, rest = old_w.split(": ", 1) if ": " in old_w else (old_w, "")
    if strong and rest.startswith("ONE "):
        pass
    elif strong and head.startswith("configs[3]: ONE"):
        rest = head[len("configs[3]: "):] + (": " + rest if rest else "")
    total = cfg.get("bytes_total") or cfg.get("bytes_per_gpu", 0) * world
    if not total:   # round-2 records: "<x> GiB/GPU" in the label only
        total = int(float(old_w.split(" GiB/GPU")[0].split()[-1]) * (1 << 30)) * world
    new_head = bench.workload_id(world, bid, n_total=total, strong=strong)
    cfg["workload"] = f"{new_head}: {rest}" if rest else new_head
    gather = str(line.get("gather") or "")
    streamed = gather.startswith("streamed")
    # records older than round 4 name the transport only inside `gather`; the
    # one-GPU rehearsals all ran over gloo (file names say so)
    transport = (line.get("transport") or gather.rsplit(", ", 1)[-1].rstrip(")")) if streamed else None
    backend = line.get("backend") or "gloo"
    cfg["parallelism"] = bench.parallelism_label(world, True, streamed, transport, backend)
    line["relabelled"] = (f"round 6 (VERDICT r05 item 1): labels recomputed by bench.workload_id / "
                          f"parallelism_label; was workload={old_w!r}, parallelism={old_p!r}; "
                          f"measured values unchanged")
    return line


for path in sys.argv[1:]:
    text = open(path).read()
    out = []
    for ln in text.splitlines():
        s = ln.strip()
        if s.startswith("{") and '"n_gpus"' in s:
            d = json.loads(s)
            if "relabelled" not in d and (d.get("n_gpus", 1) > 1 or
                                          "configs[3]" in d.get("config", {}).get("workload", "")):
                ln = json.dumps(relabel(d))
        out.append(ln)
    open(path, "w").write("\n".join(out) + ("\n" if text.endswith("\n") else ""))
    print(path)
