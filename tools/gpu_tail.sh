#!/bin/bash
# Dispatch-tail experiment: k_step at 1e8 particles with 10000 (configs[2]), 9984 (= 39 x 256)
# and 10240 (= 40 x 256) halos, alternating on one box; then the stamps build's tail figures.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out; mkdir -p "$O"
for rep in 1 2; do
  for h in 10000 9984 10240; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --halos $h \
      > "$O/tail_${h}_$rep.json" 2> "$O/tail_${h}_$rep.err"
    rc=$?; echo "halos $h rep$rep rc=$rc $(grep -o 'k_step [0-9.]* ms' "$O/tail_${h}_$rep.err")"
    [ $rc = 0 ] || exit $rc
  done
done
ORBIT_HIP_LIB=$R/nbody-orbit-analysis_amd/variants/lib_stamps.so timeout -k 10 300 \
  python tools/stamps.py > "$O/tail_stamps.txt" 2>&1 || exit $?
grep -v amdgpu.ids "$O/tail_stamps.txt" | tail -6
