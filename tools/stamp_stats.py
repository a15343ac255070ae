"""Stamp a rocprofv3 kernel summary with the library build it profiled.

    python tools/stamp_stats.py BENCH_LINE.json run_kernel_stats.csv CONFIG

BENCH_LINE.json: the bench line the profiled command printed (its build_id).  Writes <csv stem>.meta.json
beside the summary: {"build_id", "config", "kernels": {kernel: {"calls", "avg_ms"}}}.  bench.py looks for the
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
meta = os.path.splitext(stats)[0] + ".meta.json"
with open(meta, "w") as f:
    json.dump({"build_id": bid, "config": cfg, "stats": os.path.basename(stats), "kernels": kernels}, f, indent=1)
print(meta, bid)
