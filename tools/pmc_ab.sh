set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcab
for v in base default; do
  lib=raytracingthenextweekcuda_amd/librtmi.so
  [ "$v" != "default" ] && lib=raytracingthenextweekcuda_amd/librtmi_$v.so
  export RTMI_LIB=$lib
  timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmcab/$v -o pmc -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmcab/$v.log 2>&1 || exit $?
done
echo done
