#!/bin/bash
# SQ counter groups (lane utilisation, issue, waits) of the render kernel per scene:
# SCENES="cornellbox1 bunny materialball" bash tools/pmc_sq_scenes.sh -> gpurun_out/pmcsq_<scene>/p<i>
set -u
export TMPDIR=/tmp
for scene in ${SCENES:-cornellbox1 bunny materialball}; do
  mkdir -p gpurun_out/pmcsq_$scene
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_INSTS_VMEM_WR"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmcsq_$scene/p$i -o pmc -- \
      python3 bench.py --scene $scene --steps 1 --warmup 1 --no-cpu-baseline --spp 16 > gpurun_out/pmcsq_$scene/p$i.log 2>&1 || exit $?
  done
done
echo done
