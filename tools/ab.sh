#!/bin/bash
# A/B of k_step build variants on the bench workload: alternating bench runs (k_step ms
# from HIP events), then per-item stamps of the stamp builds.  Usage:
#   VARS="base ntst" STAMPS="stamps stampsnt" TAG=x bash tools/ab.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out; mkdir -p "$O"; T=${TAG:-ab}
D=$R/nbody-orbit-analysis_amd/variants
for rep in ${REPS:-1 2}; do
  for v in ${VARS:-base}; do
    lib=""; [ "$v" != base ] && lib="$D/lib_$v.so"
    ORBIT_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline \
      > "$O/ab_${T}_${v}_$rep.json" 2> "$O/ab_${T}_${v}_$rep.err"
    rc=$?; echo "$v rep$rep rc=$rc $(grep -o 'k_step [0-9.]* ms' "$O/ab_${T}_${v}_$rep.err")"
    [ $rc = 0 ] || exit $rc
  done
done
for v in ${STAMPS:-}; do
  ORBIT_HIP_LIB=$D/lib_$v.so timeout -k 10 300 python tools/stamps.py > "$O/ab_${T}_$v.stamps" 2>&1
  rc=$?; echo "== $v rc=$rc"; grep -v amdgpu.ids "$O/ab_${T}_$v.stamps" | tail -8; [ $rc = 0 ] || exit $rc
done
