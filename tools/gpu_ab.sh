#!/bin/bash
# GPU tests (base build and, with TEST_VARIANT, one variant library), then tools/ab.sh.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out; mkdir -p "$O"; T=${TAG:-ab}
if [ -n "${TEST_VARIANT:-}" ]; then
  ORBIT_HIP_LIB=$R/nbody-orbit-analysis_amd/variants/lib_$TEST_VARIANT.so timeout -k 10 500 \
    python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf \
    > "$O/t_${T}_$TEST_VARIANT.log" 2>&1
  rc=$?; echo "tests[$TEST_VARIANT] rc=$rc"; tail -2 "$O/t_${T}_$TEST_VARIANT.log"; [ $rc = 0 ] || exit $rc
fi
TAG=$T bash tools/ab.sh
