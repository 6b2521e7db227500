#!/bin/bash
# Large-halo path (k_big_frame / k_big_join) at configs[1]'s halo size with varying
# halo counts: per-particle cost against the tables' total footprint.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out; mkdir -p "$O"; T=${TAG:-big}
for cfg in ${CFGS:-1e7:100 2.5e6:25 1e6:10}; do
  set -- ${cfg/:/ }
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$O/prof_${T}_$2" -o run -- python3 "$R/bench.py" --dtype float64 --particles $1 --halos $2 \
      --steps 10 --warmup 3 --no-cpu-baseline > "$O/b_${T}_$2.json" 2> "$O/b_${T}_$2.err" )
  rc=$?; echo "cfg $cfg rc=$rc"; [ $rc = 0 ] || exit $rc
  python3 -c "import json;d=json.load(open('$O/b_${T}_$2.json'));print(d['ms_per_step'], d['roofline'])"
  python3 tools/kstats.py "$O/prof_${T}_$2"
done
