# FETCH_SIZE / WRITE_SIZE of each large-halo kernel at configs[1] (one rocprofv3 pass per
# counter and kernel; FETCH_SIZE doubled per MI355X_MICROARCH.md for 16-B streams)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/pmcbig_${TAG:-x}; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for k in ${KERNELS:-k_part_join k_part_scatter k_gather_recs}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 120 rocprofv3 --pmc $c --kernel-include-regex "$k" --output-format csv \
      -d "$O/${k}_$c" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline \
      --dtype float64 --particles 1e7 --halos 100 > "$O/${k}_$c.out" 2> "$O/${k}_$c.err"
    rc=$?; echo "$k $c rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
  done
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections, os
O = sys.argv[1]
for d in sorted(glob.glob(O + '/*_*SIZE')):
    per = collections.defaultdict(float)
    for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            per[r['Dispatch_Id']] += float(r['Counter_Value'])
    v = list(per.values())
    print('%-28s n=%d  per launch KB: mean %.0f  last %.0f' % (os.path.basename(d), len(v), sum(v) / max(len(v), 1), v[-1] if v else 0))
PY
