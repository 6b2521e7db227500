# On-the-fly stream A/B: this tree against the worktree in old_r06/ (built in place),
# alternating, the old tree first
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out; mkdir -p $O
for rep in ${REPS:-1 2 3}; do
  (cd old_r06 && timeout -k 10 600 python tools/bench_onthefly.py --steps 4 > $O/otfab2_old_$rep.json 2> $O/otfab2_old_$rep.err) || exit 1
  echo "old $rep $(grep -o '"compute_ms_per_step": [0-9.]*\|"ms_per_step": [0-9.]*' $O/otfab2_old_$rep.json | tr '\n' ' ')"
  timeout -k 10 600 python tools/bench_onthefly.py --steps 4 > $O/otfab2_new_$rep.json 2> $O/otfab2_new_$rep.err || exit 1
  echo "new $rep $(grep -o '"compute_ms_per_step": [0-9.]*\|"ms_per_step": [0-9.]*' $O/otfab2_new_$rep.json | tr '\n' ' ')"
done
