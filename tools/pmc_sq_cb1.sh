#!/bin/bash
# SQ issue counters of the timed CB1 layout (--in-flight-layout, full spp, --no-overlap) for the in-tree
# library and A/B libraries (ALT="librtmi_x.so ..."): gpurun_out/$TAG/sq_<lib>/p<i>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-sqcb1}
for lib in librtmi.so ${ALT:-}; do
  d=$O/sq_${lib%.so}_${SCENE:-cornellbox1}
  mkdir -p $d
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    RTMI_LIB=raytracingthenextweekcuda_amd/$lib timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $d/p$i -o pmc -- \
      python3 bench.py --scene ${SCENE:-cornellbox1} --steps 2 --warmup 1 --no-cpu-baseline --no-overlap ${LAYOUT:---in-flight-layout} > $d/p$i.log 2>&1 || exit $?
  done
done
echo done
