#!/bin/bash
# Quick GPU check: GPU tests, one bench (k_step time), instruction-count PMC pass.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out; mkdir -p "$O"; T=${TAG:-q}
timeout -k 10 400 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf > "$O/t_$T.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 "$O/t_$T.log"; grep -E "^FAILED" "$O/t_$T.log" | head -5
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$O/b_$T.json" 2> "$O/b_$T.err"
rc=$?; echo "bench rc=$rc $(grep -o 'k_step [0-9.]* ms' "$O/b_$T.err")"; case $rc in 0) ;; *) exit $rc;; esac
if [ "${PMC:-1}" = 1 ]; then
TAG=$T VARIANTS="${VARIANTS:-base}" COUNTERS="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" bash tools/pmc_variants.sh 2>&1 | tail -3
fi
