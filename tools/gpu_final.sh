#!/bin/bash
# Round-end style session: GPU tests, smoke, default bench, rocprofv3 kernel stats,
# k_step PMC traffic and the end-to-end benches.  Stops at the first failing step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out; mkdir -p "$O"; T=${TAG:-final}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > "$O/gpu_tests_$T.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$O/gpu_tests_$T.log"; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_$T.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$O/smoke_$T.log"; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python bench.py > "$O/bench_$T.json" 2> "$O/bench_$T.err"
rc=$?; echo "bench rc=$rc"; cat "$O/bench_$T.json"; [ $rc = 0 ] || exit $rc
SKIP_PMC=${SKIP_PMC:-0} SKIP_E2E=${SKIP_E2E:-0} TAG=$T bash tools/gpu_prof.sh
