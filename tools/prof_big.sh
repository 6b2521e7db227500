# rocprof kernel stats of configs[1] for library variants: VARS="base jrs2k:ENV=V,..."
set -u
cd $GRAFT_REPO_ROOT; R=$(pwd); O=$R/gpurun_out; mkdir -p $O; D=$R/nbody-orbit-analysis_amd/variants; T=${TAG:-pb}
for ve in ${VARS:-base}; do
  v=${ve%%:*}; e=""; [ "$ve" != "$v" ] && e=${ve#*:}
  lib=""; [ "$v" != base ] && lib=$D/lib_$v.so
  for kv in ${e//,/ }; do export "$kv"; done
  export ORBIT_HIP_LIB=$lib
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $O/prof_${T}_$v -o run -- python3 $R/bench.py --dtype float64 --particles 1e7 --halos 100 \
      --steps 10 --warmup 3 --no-cpu-baseline > $O/${T}_$v.json 2> $O/${T}_$v.err )
  rc=$?; echo "== $ve"; python3 tools/kstats.py $O/prof_${T}_$v | grep -E "k_|gather|scan" | head -12; [ $rc = 0 ] || exit $rc
  for kv in ${e//,/ }; do unset "${kv%%=*}"; done
done
