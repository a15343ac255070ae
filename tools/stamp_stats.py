"""Stamp a rocprofv3 kernel summary with the library build it profiled.

    python tools/stamp_stats.py BENCH_LINE.json run_kernel_stats.csv CONFIG

BENCH_LINE.json: the bench line the profiled command printed (its build_id).  Writes <csv stem>.meta.json
beside the summary: {"build_id", "config", "kernels": {kernel: {"calls", "avg_ms", "frames", "instrumented_step"}}}.
With run_kernel_trace.csv beside the summary, each kernel also gets its launches split per frame (frames end at
k_final): "frames" = [[calls, avg_ms], ...] in order, and "instrumented_step" = the last frame's, the one bench.py
--events times with HIP events on one stream (the timed two-stream steps may split a frame into other launches, so
only that frame's launches are the same launches as the live figure).  bench.py looks for the
committed profiles/*_kernel_stats.meta.json of the build it times and config it runs, and reports that summary's
average launch time of the dominant kernel beside its own live (HIP event) figure (roofline.rocprof)."""
import csv
import json
import os
import re
import sys

line, stats, cfg = sys.argv[1:4]
bid = None
for ln in open(line, errors="replace"):
    ln = ln.strip()
    if ln.startswith("{") and '"build_id"' in ln:
        bid = json.loads(ln)["build_id"]
if bid is None:
    sys.exit(f"{line}: no bench line with a build_id")
kernels = {}
for row in csv.DictReader(open(stats)):
    m = re.search(r"jsrt::(k_\w+)(<[^>]*>)?", row["Name"])
    if m:
        kernels[m.group(1) + (m.group(2) or "")] = {"calls": int(row["Calls"]), "avg_ms": float(row["AverageNs"]) * 1e-6}
trace = os.path.join(os.path.dirname(stats), "run_kernel_trace.csv")
if os.path.exists(trace):
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    frames, cur = [], {}
    for row in rows:
        m = re.search(r"jsrt::(k_\w+)(<[^>]*>)?", row["Kernel_Name"])
        if not m:
            continue
        k = m.group(1) + (m.group(2) or "")
        cur.setdefault(k, []).append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6)
        if m.group(1) == "k_final":
            frames.append(cur)
            cur = {}
    for k, v in kernels.items():
        per = [[len(f[k]), sum(f[k]) / len(f[k])] for f in frames if f.get(k)]
        if per:
            v["frames"] = per
            v["instrumented_step"] = {"calls": per[-1][0], "avg_ms": per[-1][1]}
meta = os.path.splitext(stats)[0] + ".meta.json"
with open(meta, "w") as f:
    json.dump({"build_id": bid, "config": cfg, "stats": os.path.basename(stats), "kernels": kernels}, f, indent=1)
print(meta, bid)
