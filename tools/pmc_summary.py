"""Summarise rocprofv3 --pmc csv passes per render kernel (k_gen, k_extend<PF>, k_shade<PF>, ...):
counter sums over all dispatches of that kernel, plus derived per-wave figures.

    python tools/pmc_summary.py <pmc dir> [--config NAME --merge profiles/pmc_summary.json]

--merge adds {NAME: {"kernels": {kernel: {counter: sum, "dispatches": n}}, "build_id": id}} to the committed
summary that bench.py reads for roofline.traffic and the VALU figures.  build_id: the library build the passes
ran (the bench line each pass printed, <pmc dir>/p<k>.log); passes of different builds are refused, and bench.py
flags a roofline whose counters come from another build than the one it times."""
import csv
import glob
import json
import os
import re
import sys

root = sys.argv[1]


def pass_build_ids(root):
    """The build_id of the bench line each pass printed (p<k>.log), when the logs are still there."""
    ids = {}
    for f in sorted(glob.glob(os.path.join(root, "p*.log"))):
        for line in open(f, errors="replace"):
            line = line.strip()
            if line.startswith("{") and '"build_id"' in line:
                try:
                    ids[os.path.basename(f)] = json.loads(line)["build_id"]
                except (ValueError, KeyError):
                    pass
    return ids


ids = pass_build_ids(root)
if len(set(ids.values())) > 1:
    sys.exit(f"pmc passes of different library builds: {ids}")
build_id = next(iter(ids.values()), None)
if build_id is None and os.path.exists(os.path.join(root, "summary.json")):  # logs removed: the first summary's id
    build_id = json.load(open(os.path.join(root, "summary.json"))).get("__build_id__")
print(f"build_id {build_id}")
tot, disp = {}, {}
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        m = re.search(r"jsrt::(k_\w+)(<[^>]*>)?", row.get("Kernel_Name", ""))
        if not m:
            continue
        k = m.group(1) + (m.group(2) or "")
        name = row["Counter_Name"]
        tot.setdefault(k, {})
        tot[k][name] = tot[k].get(name, 0.0) + float(row["Counter_Value"])
        disp.setdefault(k, {}).setdefault(name, set()).add(row.get("Dispatch_Id"))
out = {}
for k in sorted(tot):
    t = tot[k]
    print(f"== {k}")
    for c in sorted(t):
        print(f"   {c:28s} {t[c]:.6g}  (dispatches {len(disp[k][c])})")
    w = t.get("SQ_WAVES")
    if w:
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"):
            if c in t:
                print(f"   {c + ' / wave':28s} {t[c] / w:.5g}")
        for c in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC",
                  "SQ_INST_CYCLES_VMEM_RD", "SQ_INST_CYCLES_VMEM_WR", "SQ_INST_CYCLES_SMEM", "SQ_WAIT_INST_LDS"):
            if c in t:
                print(f"   {c + ' / wave (x4 cyc)':28s} {4 * t[c] / w:.5g}")
    if t.get("SQ_THREAD_CYCLES_VALU") and t.get("SQ_ACTIVE_INST_VALU"):
        print(f"   VALU lane utilisation        {t['SQ_THREAD_CYCLES_VALU'] / (64 * t['SQ_ACTIVE_INST_VALU']):.3f}")
    out[k] = dict(t)
    out[k]["dispatches"] = max(len(v) for v in disp[k].values())
with open(os.path.join(root, "summary.json"), "w") as f:
    json.dump(dict(out, __build_id__=build_id), f, indent=1)
if "--merge" in sys.argv:
    cfg = sys.argv[sys.argv.index("--config") + 1]
    dst = sys.argv[sys.argv.index("--merge") + 1]
    allp = json.load(open(dst)) if os.path.exists(dst) else {}
    allp[cfg] = {"source": os.path.relpath(root) + " (rocprofv3 --pmc passes, bench.py --steps 1 --warmup 0)", "steps": 1,
                 "kernels": out, "build_id": build_id}
    with open(dst, "w") as f:
        json.dump(allp, f, indent=1, sort_keys=True)
