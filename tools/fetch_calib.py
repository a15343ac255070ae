"""Ratios of rocprofv3's FETCH_SIZE / WRITE_SIZE to the bytes tools/fetch_calib.hip moved, per access shape.

    python tools/fetch_calib.py DIR_FETCH DIR_WRITE known.json

DIR_*: the rocprofv3 --pmc output directories of the two passes; known.json: the program's stdout (bytes per
kernel).  Reads the second dispatch of each kernel (the first pays first-touch effects)."""
import csv
import glob
import json
import os
import sys


def per_kernel(d, counter):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter:
                continue
            k = row["Kernel_Name"].split("(")[0].strip()
            vals.setdefault(k, {}).setdefault(int(row["Dispatch_Id"]), 0.0)
            vals[k][int(row["Dispatch_Id"])] += float(row["Counter_Value"])
    return {k: v[sorted(v)[-1]] * 1024 for k, v in vals.items()}  # KB -> B, last dispatch


fetch, write = per_kernel(sys.argv[1], "FETCH_SIZE"), per_kernel(sys.argv[2], "WRITE_SIZE")
known = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
out = {}
for k in ("read4", "read16"):
    out[k] = {"bytes": known[k], "FETCH_SIZE": fetch.get(k), "ratio": fetch.get(k, 0) / known[k]}
for k in ("write4", "write16"):
    out[k] = {"bytes": known[k], "WRITE_SIZE": write.get(k), "ratio": write.get(k, 0) / known[k]}
out["scat4"] = {"bytes": known["scat4_bytes"], "lines": known["scat4_lines"], "WRITE_SIZE": write.get("scat4"),
                "ratio_to_bytes": write.get("scat4", 0) / known["scat4_bytes"],
                "bytes_per_line": write.get("scat4", 0) / known["scat4_lines"]}
print(json.dumps(out, indent=1))
