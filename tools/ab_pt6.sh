#!/bin/bash
# Same-box A/B of the pathTrace kernel builds on materialball (librtmi = shipped, librtmi_ptd5 =
# pixel derived from the work item at 5 waves/SIMD, librtmi_pt6 = the same at 6), two rounds interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r03h_pt6}; mkdir -p $O
for r in 1 2; do
  for v in default ptd5 pt6; do
    lib=raytracingthenextweekcuda_amd/librtmi.so; [ $v != default ] && lib=raytracingthenextweekcuda_amd/librtmi_$v.so
    RTMI_LIB=$lib timeout -k 10 300 python bench.py --scene materialball --no-cpu-baseline > $O/bench_materialball_${v}_$r.log 2>&1 || exit $?
    echo "$r $v done"
  done
done
