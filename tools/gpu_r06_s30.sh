#!/bin/bash
# round 6 s30: diagnosis of the slow first runs (wall time well above the summed kernel time): bunny 8-step benches in
# a row, each with its process CPU time and context switches (resource.getrusage of the child)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3 4 5; do
  timeout -k 10 300 python - $i <<'PY' | tee -a gpurun_out/diag_s30.txt || exit 1
import json, resource, subprocess, sys, time
i = sys.argv[1]
t = time.time()
with open(f"gpurun_out/diag_s30_{i}.json", "w") as out, open(f"gpurun_out/diag_s30_{i}.err", "w") as err:
    rc = subprocess.call([sys.executable, "bench.py", "--config", "bunny", "--steps", "8", "--warmup", "1",
                          "--no-cpu-baseline", "--ab"], stdout=out, stderr=err)
wall = time.time() - t
ru = resource.getrusage(resource.RUSAGE_CHILDREN)
d = json.load(open(f"gpurun_out/diag_s30_{i}.json"))
print(i, rc, round(d["value"] / 1e6, 1), round(d["ms_per_step"], 1), round(d["kernel_ms_per_step"], 1),
      "wall", round(wall, 1), "user", round(ru.ru_utime, 1), "sys", round(ru.ru_stime, 1), "invol", ru.ru_nivcsw,
      "vol", ru.ru_nvcsw, "load", open("/proc/loadavg").read().split()[:3], flush=True)
sys.exit(rc)
PY
done
