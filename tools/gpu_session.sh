#!/bin/bash
# One GPU session on the MI355X box: GPU tests -> bench -> rocprofv3 kernel trace.
# Stops at the first crash / time-out (exit codes 124, 134, 137, 139) as the pool requires.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p "$O"
TAG=${TAG:-r01}
BENCH_ARGS=${BENCH_ARGS:-}
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }

if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > "$O/gpu_tests_$TAG.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$O/gpu_tests_$TAG.log"; fatal $rc pytest
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_$TAG.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 "$O/smoke_$TAG.log"; fatal $rc smoke
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 900 python bench.py $BENCH_ARGS > "$O/bench_$TAG.json" 2> "$O/bench_$TAG.err"
  rc=$?; echo "bench rc=$rc"; tail -4 "$O/bench_$TAG.err"; cat "$O/bench_$TAG.json"; fatal $rc bench
fi
if [ "${SKIP_PROF:-0}" != 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG" -o run \
    -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline $BENCH_ARGS \
    > "$O/bench_prof_$TAG.json" 2> "$O/bench_prof_$TAG.err"
  rc=$?; echo "rocprof rc=$rc"; tail -2 "$O/bench_prof_$TAG.err"; fatal $rc rocprof
  find "$O/prof_$TAG" -name '*kernel_stats.csv' -exec head -12 {} \;
fi
