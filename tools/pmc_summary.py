"""Summarise rocprofv3 --pmc csv passes for the render kernel (sum over its dispatches)."""
import csv, glob, os, sys
root = sys.argv[1]
tot = {}
disp = {}
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if "render_kernel" not in row.get("Kernel_Name", ""):
            continue
        name = row["Counter_Name"]
        tot[name] = tot.get(name, 0.0) + float(row["Counter_Value"])
        disp.setdefault(name, set()).add(row.get("Dispatch_Id"))
for k in sorted(tot):
    print(f"{k:32s} {tot[k]:.6g}  (dispatches {len(disp[k])})")
v = tot.get("SQ_INSTS_VALU"); w = tot.get("SQ_WAVES")
if v and w:
    print(f"VALU insts per wave: {v / w:.4g}")
if tot.get("SQ_THREAD_CYCLES_VALU") and tot.get("SQ_ACTIVE_INST_VALU"):
    print(f"VALU lane utilisation: {tot['SQ_THREAD_CYCLES_VALU'] / (64 * tot['SQ_ACTIVE_INST_VALU']):.3f}")
