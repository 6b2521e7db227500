# alternating bench runs of one library under environment settings: ENVS="A=1 A=0"
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out; mkdir -p $O; T=${TAG:-env}
for rep in ${REPS:-1 2}; do
  for e in ${ENVS:-X=1}; do
    env ${e//,/ } timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} \
      > $O/${T}_${e//[=,]/_}_$rep.json 2> $O/${T}_${e//[=,]/_}_$rep.err
    rc=$?; echo "$e rep$rep $(grep -o 'k_step [0-9.]* ms' $O/${T}_${e//[=,]/_}_$rep.err)"; [ $rc = 0 ] || exit $rc
  done
done
