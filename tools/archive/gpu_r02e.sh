set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02e
RTMI_LIB=raytracingthenextweekcuda_amd/librtmi_stamps.so timeout -k 10 200 python tools/stamps_breakdown.py cornellbox1 media suzanne spheres bunny > gpurun_out/r02e/stamps.log 2>&1 || exit $?
for sc in spheres suzanne cornellbox1; do
  for v in default r4 r8; do
    lib=raytracingthenextweekcuda_amd/librtmi.so
    [ "$v" != "default" ] && lib=raytracingthenextweekcuda_amd/librtmi_$v.so
    echo "== $sc $v" >> gpurun_out/r02e/refill_shards.log
    SCENE=$sc RTMI_LIB=$lib timeout -k 10 300 python tools/shard_balance.py 1:2 8:2 >> gpurun_out/r02e/refill_shards.log 2>&1 || exit $?
  done
done
timeout -k 10 300 python bench.py > gpurun_out/r02e/bench.log 2>&1 || exit $?
echo done
