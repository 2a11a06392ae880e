#!/bin/bash
# SQ counter groups (lane utilisation, issue, waits) of the render kernel per scene:
# SCENES="cornellbox1 bunny materialball" bash tools/pmc_sq_scenes.sh -> gpurun_out/pmcsq_<scene>/p<i>
# LIB=librtmi_x.so profiles an A/B library of the same sources instead (-> pmcsq_<scene>_librtmi_x).
set -u
export TMPDIR=/tmp
for scene in ${SCENES:-cornellbox1 bunny materialball}; do
  d=gpurun_out/pmcsq_$scene${LIB:+_${LIB%.so}}
  mkdir -p $d
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_INSTS_VMEM_WR" \
             "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    RTMI_LIB=${LIB:+raytracingthenextweekcuda_amd/$LIB} timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $d/p$i -o pmc -- \
      python3 bench.py --scene $scene --steps 1 --warmup 1 --no-cpu-baseline --no-overlap --spp 16 > $d/p$i.log 2>&1 || exit $?
  done
done
echo done
