set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out; mkdir -p "$O"; T=${TAG:-r02b}
timeout -k 10 500 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf > "$O/t_$T.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 "$O/t_$T.log"
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > "$O/b_$T.json" 2> "$O/b_$T.err"
rc=$?; echo "bench rc=$rc"; tail -3 "$O/b_$T.err"; cat "$O/b_$T.json"; [ $rc = 0 ] || exit $rc
ORBIT_HIP_LIB=$R/nbody-orbit-analysis_amd/variants/lib_stamps.so timeout -k 10 300 python tools/stamps.py > "$O/stamps_$T.txt" 2>&1
rc=$?; echo "stamps rc=$rc"; tail -15 "$O/stamps_$T.txt"
