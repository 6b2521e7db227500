#!/bin/bash
# A/B of k_step builds with per-variant environments (e.g. LDS table sizes):
#   SPECS="base: wg512:ORBIT_LDS_ENTRIES=5632,ORBIT_LDS_SLOTS=7296" TAG=x bash tools/gpu_ab2.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out; mkdir -p "$O"; T=${TAG:-ab2}
D=$R/nbody-orbit-analysis_amd/variants
for rep in ${REPS:-1 2 3}; do
  for spec in $SPECS; do
    v=${spec%%:*}; envs=${spec#*:}
    lib=""; [ -f "$D/lib_$v.so" ] && lib="$D/lib_$v.so"     # else the default build
    ( export ORBIT_HIP_LIB=$lib; for kv in ${envs//,/ }; do export "$kv"; done
      timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline \
        > "$O/ab_${T}_${v}_$rep.json" 2> "$O/ab_${T}_${v}_$rep.err" )
    rc=$?; echo "$v rep$rep rc=$rc $(grep -o 'k_step [0-9.]* ms' "$O/ab_${T}_${v}_$rep.err") $(python3 -c "import json;print(round(json.load(open('$O/ab_${T}_${v}_$rep.json'))['ms_per_step'],4))" 2>/dev/null)"
    [ $rc = 0 ] || { tail -5 "$O/ab_${T}_${v}_$rep.err"; exit $rc; }
  done
done
