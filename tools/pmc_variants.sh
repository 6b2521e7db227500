#!/bin/bash
# One PMC pass (counters in $COUNTERS) over k_step of bench.py for each library
# variant in $VARIANTS (nbody-orbit-analysis_amd/variants/lib_<v>.so; "base" = in-tree).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/pmcv_${TAG:-x}; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for v in $VARIANTS; do
  lib=$R/nbody-orbit-analysis_amd/variants/lib_$v.so; [ "$v" = base ] && lib=$R/nbody-orbit-analysis_amd/liborbit_hip.so
  ORBIT_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --pmc $COUNTERS --kernel-include-regex 'k_step' --output-format csv \
      -d "$O/$v" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$O/$v.out" 2> "$O/$v.err"
  rc=$?; echo "$v rc=$rc"
  case $rc in 124|134|137|139) echo FATAL; exit $rc;; esac
done
python3 - "$O" $VARIANTS <<'PY'
import csv, glob, sys, collections
O, vs = sys.argv[1], sys.argv[2:]
for v in vs:
    f = glob.glob(O + '/' + v + '/**/*counter_collection.csv', recursive=True)
    if not f: print(v, 'no data'); continue
    per = collections.defaultdict(float)
    disp = collections.defaultdict(float)
    for r in csv.DictReader(open(f[0])):
        per[(int(r['Dispatch_Id']), r['Counter_Name'])] += float(r['Counter_Value'])
    last = max(d for d, _ in per)
    print(v.ljust(10), '  '.join('%s=%.4g' % (c, x) for (d, c), x in sorted(per.items()) if d == last))
PY
