#!/bin/bash
# Same-box A/B: bench.py alternating the shipped library and RTMI_LIB variants, REPS rounds.
#   TAG=ab SCENES="cornellbox1" ALT="librtmi_x.so" REPS=3 bash tools/ab_alternate.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab}
mkdir -p "$O"
for r in $(seq 1 ${REPS:-3}); do
  for sc in ${SCENES:-cornellbox1}; do
    timeout -k 10 300 python bench.py --scene $sc --no-cpu-baseline ${BENCH_ARGS:-} > "$O/${sc}_base_$r.log" 2>&1 || exit $?
    for alt in ${ALT:-}; do
      RTMI_LIB=raytracingthenextweekcuda_amd/$alt timeout -k 10 300 python bench.py --scene $sc --no-cpu-baseline ${BENCH_ARGS:-} > "$O/${sc}_${alt%.so}_$r.log" 2>&1 || exit $?
    done
  done
done
python3 - "$O" <<'PY'
import glob, json, os, sys, collections
res = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*_*_[0-9]*.log"))):
    key = os.path.basename(f).rsplit("_", 1)[0]
    for line in open(f):
        if line.startswith("{"):
            res[key].append(json.loads(line)["roofline"]["kernel_ms"])
for k, v in sorted(res.items()):
    print(f"{k:40s} kernel_ms {' '.join(f'{x:.3f}' for x in v)}  min {min(v):.3f}")
PY
