#!/bin/bash
# GPU session for SURVEY §8(f) rows f3/f4: parity tests, benchmark, rocprof kernel stats.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out; mkdir -p "$O"; T=${TAG:-post}
timeout -k 10 300 python -u -m pytest tests/test_gpu_post.py -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf > "$O/t_$T.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 "$O/t_$T.log"; grep -E "^FAILED" "$O/t_$T.log" | head -5
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python -u tools/bench_post.py ${WHICH:+--which $WHICH} > "$O/bp_$T.jsonl" 2> "$O/bp_$T.err"
rc=$?; echo "bench_post rc=$rc"; tail -3 "$O/bp_$T.err"; cat "$O/bp_$T.jsonl"; [ $rc = 0 ] || exit $rc
if [ "${PROF:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$T" -o run \
    -- python3 "$R/tools/bench_post.py" ${WHICH:+--which $WHICH} > "$O/bp_prof_$T.jsonl" 2> "$O/bp_prof_$T.err"
  rc=$?; echo "rocprof rc=$rc"; [ $rc = 0 ] || exit $rc
  find "$O/prof_$T" -name '*kernel_stats.csv' -exec cut -c1-160 {} \; | head -24
fi
