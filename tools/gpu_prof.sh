#!/bin/bash
# rocprofv3 kernel-trace stats of bench.py, the FETCH/WRITE PMC passes of k_step
# (tools/pmc.sh -> profiles/pmc_k_step.json), and the end-to-end benches.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out; mkdir -p "$O"; T=${TAG:-r02}
if [ "${SKIP_PROF:-0}" != 1 ]; then
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$O/prof_$T" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline \
    > "$O/bench_prof_$T.json" 2> "$O/bench_prof_$T.err" )
rc=$?; echo "rocprof rc=$rc"; [ $rc = 0 ] || exit $rc
find "$O/prof_$T" -name '*kernel_stats.csv' -exec head -8 {} \;
fi
if [ "${SKIP_PMC:-0}" != 1 ]; then
TAG=$T PMC_FILE=$R/tools/pmc_bytes.txt bash tools/pmc.sh > "$O/pmc_$T.out" 2>&1
rc=$?; echo "pmc rc=$rc"; tail -3 "$O/pmc_$T.out"; [ $rc = 0 ] || exit $rc
N0=$(python3 -c "import json;print(json.load(open('$O/bench_prof_$T.json'))['config']['particles_per_step_per_gpu'])" 2>/dev/null || echo 100000000)
python3 tools/pmc_summary.py "$O/pmc_$T" 99998874 "$O/pmc_k_step_$T.json"
fi
if [ "${SKIP_E2E:-0}" != 1 ]; then
for m in "--device-loader" ""; do
  timeout -k 10 400 python tools/bench_e2e.py --snapshots 7 $m > "$O/e2e_${T}${m:+_dev}.json" 2> "$O/e2e_${T}${m:+_dev}.err"
  rc=$?; echo "e2e [$m] rc=$rc"; cat "$O/e2e_${T}${m:+_dev}.json"; [ $rc = 0 ] || exit $rc
done
fi
