#!/bin/bash
# PMC passes for k_step (separate rocprofv3 runs, counters only with kernel trace off).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/pmc_${TAG:-r01}; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $counters --kernel-include-regex "${KREGEX:-k_step}" --output-format csv \
      -d "$O/p$i" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} \
      > "$O/p$i.out" 2> "$O/p$i.err"
  rc=$?; echo "pass $i ($counters) rc=$rc"
  case $rc in 124|134|137|139) echo FATAL; exit $rc;; esac
done < "${PMC_FILE:-$R/tools/pmc.txt}"
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
acc = collections.defaultdict(list)
for f in sorted(glob.glob(O + '/p*/**/*counter_collection.csv', recursive=True)):
    rows = list(csv.DictReader(open(f)))
    per = collections.defaultdict(float)
    for r in rows:
        per[(r['Dispatch_Id'], r['Counter_Name'])] += float(r['Counter_Value'])
    for (d, c), v in per.items():
        acc[c].append(v)
for c, vs in sorted(acc.items()):
    print('%-28s n=%d mean=%.4g last=%.4g' % (c, len(vs), sum(vs) / len(vs), vs[-1]))
PY
