#!/bin/bash
# Same-box A/B of library builds on the BVH scenes: VARIANTS="base default" SPP=16
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${VARIANTS:-base default}; do
  lib=raytracingthenextweekcuda_amd/librtmi.so
  [ "$v" != "default" ] && lib=raytracingthenextweekcuda_amd/librtmi_$v.so
  echo "== $v"
  RTMI_LIB=$lib timeout -k 10 200 python tools/traversal_stats.py ${SPP:-16} 2>&1 | grep -v amdgpu.ids || exit $?
done
