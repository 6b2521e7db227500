set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 600 python tools/bench_onthefly.py --steps 4 > $O/otfab_new_$rep.json 2> $O/otfab_new_$rep.err || exit 1
  echo "new $rep $(grep -o '"compute_ms_per_step": [0-9.]*\|"ms_per_step": [0-9.]*' $O/otfab_new_$rep.json | tr '\n' ' ')"
  (cd old_r05 && timeout -k 10 600 python tools/bench_onthefly.py --steps 4 > $O/otfab_old_$rep.json 2> $O/otfab_old_$rep.err) || exit 1
  echo "old $rep $(grep -o '"compute_ms_per_step": [0-9.]*\|"ms_per_step": [0-9.]*' $O/otfab_old_$rep.json | tr '\n' ' ')"
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_otf -o run -- python3 $R/tools/bench_onthefly.py --steps 3 > $O/otf_prof.json 2> $O/otf_prof.err || exit 1
python3 $R/tools/kstats.py $O/prof_otf | head -12
