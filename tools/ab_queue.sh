#!/bin/bash
# Work-queue A/B (RTMI_QUEUE=1) over refill-threshold builds; parity first.
set -u
RTMI_QUEUE=1 timeout -k 10 500 python -m pytest tests -m gpu -q -rf -x > gpurun_out/gpu_queue.log 2>&1; echo "queue pytest rc=$?"; tail -2 gpurun_out/gpu_queue.log
for sc in ${SCENES:-cornellbox1 spheres}; do
  echo "static $sc $(RTMI_QUEUE=0 timeout -k 10 300 python bench.py --scene $sc --steps 5 --warmup 1 --no-cpu-baseline | grep -o '"ms_per_step": [0-9.]*')"
  for v in ${VARIANTS:-default rf4 rf32}; do
    lib=raytracingthenextweekcuda_amd/librtmi.so
    [ "$v" != "default" ] && lib=raytracingthenextweekcuda_amd/librtmi_$v.so
    echo "queue $v $sc $(RTMI_LIB=$lib RTMI_QUEUE=1 timeout -k 10 300 python bench.py --scene $sc --steps 5 --warmup 1 --no-cpu-baseline | grep -o '"ms_per_step": [0-9.]*')"
  done
done
