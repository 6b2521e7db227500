#!/bin/bash
# One parameterised GPU session on the MI355X box (run through gpurun).  Steps run in
# the order given and the session stops at the first failing step (a crash, abort or
# time-out ends it: nothing more touches the GPU after one).
#
#   STEPS="tests smoke bench prof pmc" TAG=r03a bash tools/gpu.sh
#
# steps:
#   tests     python -m pytest tests -m gpu ($TESTS selects files / -k, default all)
#   smoke     __graft_entry__.smoke()
#   bench     bench.py $BENCH_ARGS (default workload, CPU baseline included)
#   prof      rocprofv3 --kernel-trace --stats over bench.py --steps 10
#   pmc       FETCH_SIZE / WRITE_SIZE passes over k_step -> pmc_k_step_$TAG.json
#   big       configs[1] (1e7 f64, 100 large halos) bench + rocprof
#   e2e       tools/bench_e2e.py with a device loader and with a host loader
#   e2es      tools/bench_e2e.py --sharded, world 2 over gloo (presharded, whole)
#   otf       tools/bench_onthefly.py $OTF_ARGS (configs[4] one-GPU share)
#   post      tools/bench_post.py (+ rocprof)
#   b2        bench.py --gpus 2 over gloo on this one GPU ($B2_SCALING, default strong)
#   ab        alternating bench runs of library variants ($VARS, tools/variants.sh)
#   pab       the same for tools/bench_post.py ($PAB_WHICH, default mainprog)
#   pprof     rocprofv3 kernel stats of tools/bench_post.py per variant in $VARS
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out; mkdir -p "$O"; T=${TAG:-x}
ok() { local rc=$1; echo "[$2] rc=$rc"; [ "$rc" = 0 ] || exit "$rc"; }
prof() {   # prof <dir> <timeout> <python args...>: kernel trace + stats of one command
  local d=$1 t=$2; shift 2
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 "$t" rocprofv3 --kernel-trace --stats \
      --output-format csv -d "$d" -o run -- python3 "$@" )
}

for step in ${STEPS:-tests smoke bench}; do
case $step in
tests)
  timeout -k 10 ${TESTS_TIMEOUT:-1500} python -u -m pytest ${TESTS:-tests} -m gpu -x -q -rf \
    -p no:cacheprovider --timeout ${TEST_TIMEOUT:-300} --timeout-method thread \
    > "$O/gpu_tests_$T.log" 2>&1
  rc=$?; tail -3 "$O/gpu_tests_$T.log"; ok $rc tests ;;
smoke)
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_$T.log" 2>&1
  rc=$?; tail -2 "$O/smoke_$T.log"; ok $rc smoke ;;
bench)
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$O/bench_$T.json" 2> "$O/bench_$T.err"
  rc=$?; tail -3 "$O/bench_$T.err"; cat "$O/bench_$T.json"; ok $rc bench ;;
prof)
  prof "$O/prof_$T" 400 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} \
    > "$O/bench_prof_$T.json" 2> "$O/bench_prof_$T.err"
  rc=$?; python3 tools/kstats.py "$O/prof_$T" | head -8
  python3 tools/trace_window.py "$O/prof_$T" ${RAMP:-30} ${WARM:-5} ${STEPS_T:-20} "$O/trace_window_$T.json"; ok $rc prof ;;
pmc)
  TAG=$T PMC_FILE=${PMC_FILE:-$R/tools/pmc_bytes.txt} bash tools/pmc.sh > "$O/pmc_$T.out" 2>&1
  rc=$?; tail -3 "$O/pmc_$T.out"; ok $rc pmc
  N0=$(grep -o 'particles_per_step_per_gpu": [0-9]*' "$O/bench_prof_$T.json" 2>/dev/null | grep -o '[0-9]*$' || true)
  python3 tools/pmc_summary.py "$O/pmc_$T" "${N0:-99998874}" "$O/pmc_k_step_$T.json"; ok $? pmc_summary ;;
big)
  prof "$O/prof_big_$T" 400 "$R/bench.py" --dtype float64 --particles 1e7 --halos 100 \
    --steps 10 --warmup 3 --no-cpu-baseline > "$O/big_$T.json" 2> "$O/big_$T.err"
  rc=$?; cat "$O/big_$T.json"; python3 tools/kstats.py "$O/prof_big_$T"; ok $rc big ;;
envsweep)
  # bench.py $BENCH_ARGS under environment settings ($ENVS: space-separated NAME=VALUE,NAME=VALUE)
  for rep in ${REPS:-1 2}; do
    for e in ${ENVS:-ORBIT_DIRECT=1}; do
      env ${e//,/ } timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline \
        ${BENCH_ARGS:-} > "$O/es_${T}_${e}_$rep.json" 2> "$O/es_${T}_${e}_$rep.err"
      rc=$?; echo "$e rep$rep $(grep -o 'k_step [0-9.]* ms' "$O/es_${T}_${e}_$rep.err") $(grep -o '"ms_per_step": [0-9.]*' "$O/es_${T}_${e}_$rep.json")"; ok $rc "envsweep $e"
    done
  done ;;
pmcbig)
  TAG=$T bash tools/pmc_big.sh > "$O/pmcbig_$T.out" 2>&1
  rc=$?; tail -8 "$O/pmcbig_$T.out"; ok $rc pmcbig ;;
pstamps)
  # per-work-group phases of the large-halo kernels (stamps build: tools/variants.sh with
  # a "stamps -DOA_STAMPS=1" line)
  ORBIT_HIP_LIB=$R/nbody-orbit-analysis_amd/variants/lib_stamps.so timeout -k 10 300 \
    python tools/part_stamps.py > "$O/pstamps_$T.txt" 2>&1
  rc=$?; tail -12 "$O/pstamps_$T.txt"; ok $rc pstamps ;;
stamps)
  # per-work-group phases of k_step (stamps build: tools/variants.sh "stamps -DOA_STAMPS=1")
  ORBIT_HIP_LIB=$R/nbody-orbit-analysis_amd/variants/lib_${STAMPS_LIB:-stamps}.so timeout -k 10 300 \
    python tools/stamps.py > "$O/stamps_$T.txt" 2>&1
  rc=$?; tail -22 "$O/stamps_$T.txt"; ok $rc stamps ;;
bigsweep)
  # configs[1] under environment settings ($BIG_ENVS: space-separated NAME=VALUE,NAME=VALUE)
  for rep in ${REPS:-1 2}; do
    for e in ${BIG_ENVS:-ORBIT_PART_ENTRIES=4096}; do
      env ${e//,/ } timeout -k 10 300 python bench.py --dtype float64 --particles 1e7 --halos 100 \
        --steps 10 --warmup 3 --no-cpu-baseline > "$O/bs_${T}_${e}_$rep.json" 2> "$O/bs_${T}_${e}_$rep.err"
      rc=$?; echo "$e rep$rep $(grep -o 'k_step [0-9.]* ms' "$O/bs_${T}_${e}_$rep.err")"; ok $rc "bigsweep $e"
    done
  done ;;
e2e)
  for m in "--device-loader" ""; do
    timeout -k 10 400 python tools/bench_e2e.py --snapshots ${E2E_SNAPS:-14} $m \
      > "$O/e2e_$T${m:+_dev}.json" 2> "$O/e2e_$T${m:+_dev}.err"
    rc=$?; cat "$O/e2e_$T${m:+_dev}.json"; ok $rc "e2e $m"
  done ;;
e2es)
  # the sharded driver end to end: world-2 gloo rehearsal on this one GPU
  for c in presharded whole; do
    ORBIT_DIRECT=${B2_DIRECT:-0} timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port ${E2E_PORT:-29521} tools/bench_e2e.py --sharded \
      --backend gloo --contract $c --scaling ${E2E_SCALING:-strong} --snapshots ${E2E_SNAPS:-12} \
      > "$O/e2es_${c}_$T.json" 2> "$O/e2es_${c}_$T.err"
    rc=$?; grep -v Warning "$O/e2es_${c}_$T.err" | tail -2; cat "$O/e2es_${c}_$T.json"; ok $rc "e2es $c"
  done ;;
otf)
  timeout -k 10 600 python tools/bench_onthefly.py ${OTF_ARGS:-} > "$O/otf_$T.json" 2> "$O/otf_$T.err"
  rc=$?; tail -3 "$O/otf_$T.err"; cat "$O/otf_$T.json"; ok $rc otf ;;
post)
  timeout -k 10 400 python -u tools/bench_post.py > "$O/post_$T.jsonl" 2> "$O/post_$T.err"
  rc=$?; cat "$O/post_$T.jsonl"; ok $rc post
  prof "$O/prof_post_$T" 400 "$R/tools/bench_post.py" > /dev/null 2> "$O/post_prof_$T.err"
  rc=$?; python3 tools/kstats.py "$O/prof_post_$T"; ok $rc post_prof ;;
b2)
  sc=${B2_SCALING:-strong}
  # ORBIT_DIRECT=0: two processes share this one GPU, whose time slicing can hold a
  # k_step item's predecessor off the CUs past the direct records' look-back bound (a
  # production run has one process per GPU); the rehearsal checks the plumbing
  ORBIT_DIRECT=${B2_DIRECT:-0} timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port ${B2_PORT:-29517} bench.py --gpus 2 --steps 5 --warmup 2 \
    --backend gloo --scaling "$sc" --no-cpu-baseline ${B2_ARGS:-} > "$O/b2_${sc}_$T.json" 2> "$O/b2_${sc}_$T.err"
  rc=$?; grep -v Warning "$O/b2_${sc}_$T.err" | tail -3; cat "$O/b2_${sc}_$T.json"; ok $rc b2 ;;
ab)
  D=$R/nbody-orbit-analysis_amd/variants
  for rep in ${REPS:-1 2}; do
    for v in ${VARS:-base}; do
      lib=""; [ "$v" != base ] && lib="$D/lib_$v.so"
      ORBIT_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline \
        ${BENCH_ARGS:-} > "$O/ab_${T}_${v}_$rep.json" 2> "$O/ab_${T}_${v}_$rep.err"
      rc=$?; echo "$v rep$rep $(grep -o 'k_step [0-9.]* ms' "$O/ab_${T}_${v}_$rep.err") \
$(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*' "$O/ab_${T}_${v}_$rep.json" | tr '\n' ' ')"; ok $rc "ab $v"
    done
  done ;;
pab)
  D=$R/nbody-orbit-analysis_amd/variants
  for rep in ${REPS:-1 2}; do
    for v in ${VARS:-base}; do
      lib=""; [ "$v" != base ] && lib="$D/lib_$v.so"
      ORBIT_HIP_LIB=$lib timeout -k 10 300 python tools/bench_post.py --which ${PAB_WHICH:-mainprog} \
        > "$O/pab_${T}_${v}_$rep.jsonl" 2> "$O/pab_${T}_${v}_$rep.err"
      rc=$?; echo "$v rep$rep $(grep -o '"ms_per_[a-z]*": [0-9.]*\|identical to the GPU: [A-Za-z]*' "$O/pab_${T}_${v}_$rep.jsonl" | tr '\n' ' ')"
      ok $rc "pab $v"
    done
  done ;;
pprof)   # per-kernel stats of tools/bench_post.py for each library variant in $VARS
  D=$R/nbody-orbit-analysis_amd/variants
  for v in ${VARS:-base}; do
    lib=""; [ "$v" != base ] && lib="$D/lib_$v.so"
    ORBIT_HIP_LIB=$lib prof "$O/pprof_${T}_$v" 300 "$R/tools/bench_post.py" --which ${PAB_WHICH:-collate} \
      > "$O/pprof_${T}_$v.jsonl" 2> "$O/pprof_${T}_$v.err"
    rc=$?; echo "== $v $(grep -o '"ms_per_[a-z]*": [0-9.]*' "$O/pprof_${T}_$v.jsonl")"
    python3 tools/kstats.py "$O/pprof_${T}_$v" | head -6; ok $rc "pprof $v"
  done ;;
cal)
  # FETCH_SIZE / WRITE_SIZE per access width (tools/ubench/fetch_cal, built on the CPU host)
  for c in FETCH_SIZE WRITE_SIZE; do
    ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv \
        -d "$O/cal_$T/$c" -o run -- "$R/tools/ubench/fetch_cal" ) > "$O/cal_${T}_$c.out" 2>&1
    rc=$?; tail -1 "$O/cal_${T}_$c.out"; ok $rc "cal $c"
  done
  python3 tools/fetch_cal.py "$O/cal_$T" "$O/cal_${T}_FETCH_SIZE.out" > "$O/fetch_cal_$T.json"; ok $? cal_summary ;;
pmcpost)
  TAG=$T bash tools/pmc_post.sh > "$O/pmcpost_$T.out" 2>&1
  rc=$?; tail -12 "$O/pmcpost_$T.out"; ok $rc pmcpost ;;
*) echo "unknown step $step"; exit 2 ;;
esac
done
