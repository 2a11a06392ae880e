#!/bin/bash
# Same-box occupancy A/B of the BVH rayColor kernels after pathTrace moved to 6 waves:
# random spheres (sphere-group kernel, librtmi_g6 = 6 waves/SIMD) and the bunny box
# (simple-scene mesh kernel, librtmi_bs6 = 6 waves/SIMD) against the shipped 5, two rounds interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r03i_occ}; mkdir -p $O
for r in 1 2; do
  for sv in "spheres default" "spheres g6" "bunny default" "bunny bs6"; do
    set -- $sv
    lib=raytracingthenextweekcuda_amd/librtmi.so; [ $2 != default ] && lib=raytracingthenextweekcuda_amd/librtmi_$2.so
    RTMI_LIB=$lib timeout -k 10 300 python bench.py --scene $1 --no-cpu-baseline > $O/bench_$1_$2_$r.log 2>&1 || exit $?
    echo "$r $1 $2 $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$1_$2_$r.log)"
  done
done
