#!/bin/bash
# Kernel-variant sweep on the MI355X box: name lib entries slots
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out; mkdir -p "$O"
TAG=${TAG:-sweep}
STEPS=${STEPS:-4}
: > "$O/$TAG.jsonl"
while read -r name lib entries slots; do
  [ -z "$name" ] && continue
  ORBIT_HIP_LIB=$R/nbody-orbit-analysis_amd/variants/$lib ORBIT_LDS_ENTRIES=$entries ORBIT_LDS_SLOTS=$slots \
    timeout -k 10 300 python bench.py --steps $STEPS --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} \
    > "$O/${TAG}_$name.json" 2> "$O/${TAG}_$name.err"
  rc=$?
  echo "$name rc=$rc $(grep -o 'k_step [0-9.]* ms' "$O/${TAG}_$name.err") $(grep -o 'items/step.*' "$O/${TAG}_$name.err")"
  case $rc in 124|134|137|139) echo "FATAL $rc"; exit $rc;; esac
  python -c "import json,sys; d=json.load(open('$O/${TAG}_$name.json')); print(json.dumps({'name':'$name','value':d['value'],'ms':d['ms_per_step'],'kms':d['roofline']['kernel_ms'],'frac':d['roofline']['frac']}))" >> "$O/$TAG.jsonl" 2>/dev/null
done < "${SWEEP_FILE:-tools/sweep.txt}"
cat "$O/$TAG.jsonl"
