# World-2 rehearsal (gloo, both ranks on this one GPU) of the sharded on-the-fly stream:
# apsis IDs and angle changes through the shared host buffer (ORBIT_OTF_STAGE=1) against
# gathering them to rank 0 (=0).  PARTICLES: the global snapshot size.
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out; mkdir -p $O; T=${TAG:-otfst}
for rep in ${REPS:-1 2}; do
  for st in 1 0; do
    ORBIT_DIRECT=0 ORBIT_OTF_STAGE=$st timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29600 + rep * 2 + st)) \
      tools/bench_onthefly.py --sharded --backend gloo --particles ${PARTICLES:-5e7} --steps ${STEPS:-6} \
      > $O/${T}_stage${st}_$rep.json 2> $O/${T}_stage${st}_$rep.err
    rc=$?
    echo "stage=$st rep$rep $(grep -o '"ms_per_step": [0-9.]*' $O/${T}_stage${st}_$rep.json) $(grep -o "sharded phases.*" $O/${T}_stage${st}_$rep.err | head -1)"
    [ $rc = 0 ] || exit $rc
  done
done
