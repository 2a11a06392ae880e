"""Summarise tools/pmc_sq_scenes.sh: per scene, the render kernel's VALU lane utilisation
(SQ_THREAD_CYCLES_VALU / 64 / SQ_ACTIVE_INST_VALU), VALU issue share of wave cycles and waits, L2 hit rate.
  python tools/sq_summary.py bunny bunny_librtmi_noleafbatch   (the gpurun_out/pmcsq_<name> directories)"""
import collections
import csv
import glob
import sys

for scene in sys.argv[1:] or ["cornellbox1", "bunny", "materialball"]:
    agg = collections.defaultdict(float)
    for f in glob.glob(f"gpurun_out/pmcsq_{scene}/p*/**/*counter_collection.csv", recursive=True):
        disp = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if "render_kernel" in r["Kernel_Name"] or "pathtrace_kernel" in r["Kernel_Name"]:
                disp[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        last = max(d for d, _ in disp) if disp else None
        for (d, c), v in disp.items():
            if d == last:
                agg[c] = v
    if not agg:
        continue
    util = agg["SQ_THREAD_CYCLES_VALU"] / 64.0 / max(agg["SQ_ACTIVE_INST_VALU"], 1)
    print(f"{scene}: VALU lane utilisation {util:.3f}; VALU insts {agg['SQ_INSTS_VALU']:.3g}, SALU "
          f"{agg['SQ_INSTS_SALU']:.3g}, LDS {agg['SQ_INSTS_LDS']:.3g}, VMEM rd {agg['SQ_INSTS_VMEM_RD']:.3g}, "
          f"branch {agg['SQ_INSTS_BRANCH']:.3g}; wave cycles: wait(waitcnt) {agg['SQ_WAIT_ANY'] / agg['SQ_WAVE_CYCLES']:.3f} "
          f"issue-stall {agg['SQ_WAIT_INST_ANY'] / agg['SQ_WAVE_CYCLES']:.3f} active {agg['SQ_ACTIVE_INST_ANY'] / agg['SQ_WAVE_CYCLES']:.3f}"
          + (f"; L2 hit rate {agg['TCC_HIT_sum'] / max(agg['TCC_HIT_sum'] + agg['TCC_MISS_sum'], 1):.3f} "
             f"({agg['TCC_MISS_sum']:.3g} misses)" if "TCC_HIT_sum" in agg else ""))
