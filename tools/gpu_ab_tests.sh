#!/bin/bash
# GPU tests of the default build, then an A/B of k_step variants (tools/ab.sh) and
# their stamp builds.  Stops at the first failure or crash.
#   VARS="base old" STAMPS="stamps oldstamps" TAG=x bash tools/gpu_ab_tests.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out; mkdir -p "$O"; T=${TAG:-abt}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
      --timeout-method thread > "$O/gpu_tests_$T.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$O/gpu_tests_$T.log"; [ $rc = 0 ] || exit $rc
fi
TAG=$T bash tools/ab.sh
