# configs[1] (1e7 f64, 100 large halos) A/B of library variants + environment settings
#   VARS="base:ENV=1,ENV2=2 jrs2k:ORBIT_PART_ENTRIES=2048" bash tools/ab_big.sh
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out; mkdir -p $O; D=nbody-orbit-analysis_amd/variants; T=${TAG:-big}
for rep in ${REPS:-1 2}; do
  for ve in ${VARS:-base}; do
    v=${ve%%:*}; e=""; [ "$ve" != "$v" ] && e=${ve#*:}
    lib=""; [ "$v" != base ] && lib=$D/lib_$v.so
    env ORBIT_HIP_LIB=$lib ${e//,/ } timeout -k 10 300 python bench.py --dtype float64 --particles 1e7 --halos 100 \
      --steps 10 --warmup 3 --no-cpu-baseline > $O/${T}_${v}_$rep.json 2> $O/${T}_${v}_$rep.err
    rc=$?; echo "$ve rep$rep $(grep -o 'k_step [0-9.]* ms' $O/${T}_${v}_$rep.err)"; [ $rc = 0 ] || exit $rc
  done
done
