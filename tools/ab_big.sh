#!/bin/bash
# A/B of build variants on configs[1] (1e7 f64 particles in 100 large halos: every halo on
# the partitioned large-halo path); ms_per_step from bench.py, alternating runs.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out; mkdir -p "$O"; T=${TAG:-abbig}
D=$R/nbody-orbit-analysis_amd/variants
for rep in ${REPS:-1 2}; do
  for v in ${VARS:-base}; do
    lib=""; [ "$v" != base ] && lib="$D/lib_$v.so"
    ORBIT_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline \
      --dtype float64 --particles 1e7 --halos 100 > "$O/${T}_${v}_$rep.json" 2> "$O/${T}_${v}_$rep.err"
    rc=$?; echo "$v rep$rep rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$O/${T}_${v}_$rep.json")"
    [ $rc = 0 ] || exit $rc
  done
done
