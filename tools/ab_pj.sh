# k_stepp (previous-table join) vs k_step: GPU tests on k_stepp, then alternating benches
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out; mkdir -p $O; T=${TAG:-pj}
if [ "${SKIP_TESTS:-0}" = 0 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $O/gpu_tests_$T.log 2>&1; rc=$?; tail -3 $O/gpu_tests_$T.log; [ $rc = 0 ] || exit $rc
fi
for rep in ${REPS:-1 2}; do
  for v in ${PJV:-1 0}; do
    ORBIT_PJOIN=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} \
      > $O/ab_${T}_${v}_$rep.json 2> $O/ab_${T}_${v}_$rep.err
    rc=$?; echo "pj=$v rep$rep $(grep -o 'k_step [0-9.]* ms' $O/ab_${T}_${v}_$rep.err) $(grep -o '"ms_per_step": [0-9.]*' $O/ab_${T}_${v}_$rep.json)"; [ $rc = 0 ] || exit $rc
  done
done
