#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
for v in ${VARIANTS:-BASE GATHER INSERT FRAME STORE1 PHASE3}; do
  echo "=== $v"
  ORBIT_HIP_LIB=$R/nbody-orbit-analysis_amd/variants/lib_st_$v.so timeout -k 10 300 python tools/stamps.py 2>&1 | grep -E "span|phase|total|barrier"
  rc=${PIPESTATUS[0]}; case $rc in 124|134|137|139) echo FATAL; exit $rc;; esac
done
