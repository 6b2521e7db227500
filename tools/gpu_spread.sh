for sp in 32 64 128; do
  ORBIT_PART_SPREAD=$sp CFGS="1e7:100" TAG=sp$sp bash tools/gpu_big.sh 2>&1 | grep -E "k_part|rc=|^[0-9]" | cut -c1-120 || exit 1
done
