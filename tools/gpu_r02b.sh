#!/bin/bash
# GPU tests, 1-GPU bench, and 2-rank gloo rehearsals (weak / strong) of bench.py's
# ShardedEngine leg on one GPU.  Stops at the first failing step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out; mkdir -p "$O"; T=${TAG:-r02}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf > "$O/t_$T.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$O/t_$T.log"; grep -E "^FAILED" "$O/t_$T.log" | head; [ $rc = 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS:-} > "$O/b_$T.json" 2> "$O/b_$T.err"
rc=$?; echo "bench rc=$rc"; tail -3 "$O/b_$T.err"; grep -o '"value": [0-9.e+]*\|"frac": [0-9.]*' "$O/b_$T.json"; [ $rc = 0 ] || exit $rc
for sc in weak strong; do
  P=2.5e7; [ $sc = strong ] && P=1e8
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo --scaling $sc --particles $P \
    --no-cpu-baseline > "$O/b2_${sc}_$T.json" 2> "$O/b2_${sc}_$T.err"
  rc=$?; echo "bench N=2 gloo $sc rc=$rc"; grep -v Warning "$O/b2_${sc}_$T.err" | tail -3; cat "$O/b2_${sc}_$T.json"; [ $rc = 0 ] || exit $rc
done
