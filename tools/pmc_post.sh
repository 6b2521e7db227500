#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the f3/f4 kernels over tools/bench_post.py (one rocprofv3
# pass per counter; counters only, no trace domains), reduced by tools/pmc_post.py.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/pmcpost_${TAG:-x}; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "k_collate|k_central|k_mp_" \
    --output-format csv -d "$O/$c" -o run -- python3 "$R/tools/bench_post.py" \
    > "$O/$c.out" 2> "$O/$c.err"
  rc=$?; echo "post $c rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
python3 "$R/tools/pmc_post.py" "$O" "$O/pmc_post.json"
