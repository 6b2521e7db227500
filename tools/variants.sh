#!/bin/bash
# Build diagnostic / tuning variants of liborbit_hip.so in-tree (CPU side, before a
# gpurun call): each line of $VARIANT_FILE is "name -Dflag ...".
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
D=$R/nbody-orbit-analysis_amd/variants; mkdir -p "$D"
SRC="$R/nbody-orbit-analysis_amd/csrc/orbit_hip.hip $R/nbody-orbit-analysis_amd/csrc/orbit_post.hip"
pids=()
while read -r name flags; do
  [ -z "$name" ] && continue
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
    -fno-fast-math -mllvm -amdgpu-atomic-optimizer-strategy=None -I"$R/include" $flags -o "$D/lib_$name.so" $SRC &
  pids+=($!)
  if [ ${#pids[@]} -ge 6 ]; then wait "${pids[0]}"; pids=("${pids[@]:1}"); fi
done < "${VARIANT_FILE:-$R/tools/variants.txt}"
wait
ls -la "$D"
