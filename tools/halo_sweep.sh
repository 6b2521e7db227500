set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out; mkdir -p $O
for H in ${HS:-10000 12500 15000 20000}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --halos $H > $O/hs_$H.json 2> $O/hs_$H.err
  rc=$?; echo "H=$H $(grep -o 'k_step [0-9.]* ms' $O/hs_$H.err) $(grep -o 'items/step [0-9]* (large halos [0-9]*)' $O/hs_$H.err)"; [ $rc = 0 ] || exit $rc
done
