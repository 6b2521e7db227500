set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out; mkdir -p $O
D=nbody-orbit-analysis_amd/variants
run() { # tag env...
  local t=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --halos ${H} > $O/wg_$t.json 2> $O/wg_$t.err
  local rc=$?; echo "$t H=$H $(grep -o 'k_step [0-9.]* ms' $O/wg_$t.err) $(grep -o 'items/step [0-9]* (large halos [0-9]*)' $O/wg_$t.err) $(grep -o '"ms_per_step": [0-9.]*' $O/wg_$t.json)"; [ $rc = 0 ] || exit $rc
}
for rep in 1 2; do
 H=25000 run base25_$rep ORBIT_HIP_LIB=
 H=25000 run wg25_$rep ORBIT_HIP_LIB=$D/lib_wg512.so ORBIT_LDS_ENTRIES=5632 ORBIT_LDS_SLOTS=8192
 H=10000 run base10_$rep ORBIT_HIP_LIB=
done
