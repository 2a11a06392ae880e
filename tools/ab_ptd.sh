#!/bin/bash
# Same-box pathTrace A/B behind DESIGN §4 (late round 3; profiles/r03/ptd/). Libraries as built then:
# librtmi.so = RT_PT_DERIVE at 5 waves, librtmi_pt6.so = -DRT_PT_WAVES=6, librtmi_base.so = -DRT_PT_DERIVE=0.
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r03i_ptd; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_pathtrace.py tests/test_variants.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_pt_default.log 2>&1 || exit $?
echo default-tests ok
RTMI_LIB=raytracingthenextweekcuda_amd/librtmi_pt6.so timeout -k 10 300 python -u -m pytest tests/test_pathtrace.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_pt_pt6.log 2>&1 || exit $?
echo pt6-tests ok
for r in 1 2; do
  for v in base default pt6; do
    lib=raytracingthenextweekcuda_amd/librtmi.so; [ $v != default ] && lib=raytracingthenextweekcuda_amd/librtmi_$v.so
    RTMI_LIB=$lib timeout -k 10 300 python bench.py --scene materialball --no-cpu-baseline > $O/bench_materialball_${v}_$r.log 2>&1 || exit $?
    echo "$r $v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_materialball_${v}_$r.log)"
  done
done
