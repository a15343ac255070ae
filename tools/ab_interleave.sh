#!/bin/bash
# Interleaved A/B with repeats (round 6): REPS rounds, each running every spec once in turn, so box drift hits
# every spec alike; then one summary line per spec (mean, min, max of value and of each stage time).
#   bash tools/ab_interleave.sh CFG STEPS REPS NAME=[VAR=VALUE[,VAR=VALUE]][@LIB] ...
#   (LIB: a library variant name under _build (libjsrt_<LIB>.so); no @: the default library)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
CFG=$1; STEPS=$2; REPS=$3; shift 3
for rep in $(seq 1 $REPS); do
  for spec in "$@"; do
    name=${spec%%=*}; rest=${spec#*=}
    envs=${rest%%@*}; lib=""
    [[ "$rest" == *@* ]] && lib=$PWD/jsraytracer_amd/_build/libjsrt_${rest##*@}.so
    out=gpurun_out/abi_${CFG}_${name}_$rep
    ( IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
      [ -n "$lib" ] && export JSRT_LIB=$lib
      timeout -k 10 300 python bench.py --config $CFG --steps $STEPS --warmup 1 --no-cpu-baseline --ab > $out.json 2> $out.err )
    rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || { echo "FAILED $name rep $rep rc=$rc"; tail -5 $out.err; exit $rc; }
    python -c "import json; d=json.load(open('$out.json')); p=d.get('parity') or {}; print('$name', $rep, '%.1f'%(d['value']/1e6), 'parity=%s'%p.get('pass'), flush=True)"
  done
done
python - "$CFG" "$REPS" "$@" <<'EOF'
import json, sys
cfg, reps, specs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
for spec in specs:
    name = spec.split("=", 1)[0]
    ds = [json.load(open(f"gpurun_out/abi_{cfg}_{name}_{r}.json")) for r in range(1, reps + 1)]
    v = [d["value"] / 1e6 for d in ds]
    st = {}
    for d in ds:
        for k, x in d.get("stages_ms_per_step", {}).items():
            st.setdefault(k, []).append(x)
    par = all((d.get("parity") or {}).get("pass", True) for d in ds)
    print(f"{name:10s} M/s mean {sum(v)/len(v):7.1f} min {min(v):7.1f} max {max(v):7.1f}  parity={par}  stages(ms, mean [min-max]): " +
          ", ".join(f"{k} {sum(x)/len(x):.2f} [{min(x):.2f}-{max(x):.2f}]" for k, x in st.items() if max(x) > 0.05))
EOF
