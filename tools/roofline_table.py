"""DESIGN.md §5 table rows from the committed evidence: bench lines (ms/frame, segments),
profiles/valu_issue.json (SQ_INSTS_VALU per segment) and profiles/pmc_traffic.json (HBM
bytes per launch).
  python tools/roofline_table.py <dir with bench_<scene>.log files>
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VALU_GINST_PER_CU = 4 * 2.4 / 2  # G wave64 VALU instructions / s per CU (bench.py)
PEAK_HBM = 8000.0  # GB/s
SCENES = ["cornellbox1", "spheres", "bunny", "media", "materialball", "suzanne"]


def main(src):
    valu = json.load(open(os.path.join(REPO, "profiles", "valu_issue.json")))["workloads"]
    traffic = json.load(open(os.path.join(REPO, "profiles", "pmc_traffic.json")))
    print("| workload | kernel variant | ms/frame | kernel ms (isolated) | G segments/s | VALU inst / segment | "
          "VALU issue (frac) | VALU lane util | useful frac | SALU inst / segment (frac of 1 per CU-cycle) | "
          "HBM bytes / launch (frac) |")
    for sc in SCENES:
        f = os.path.join(src, f"bench_{sc}.log")
        if not os.path.exists(f) and sc == "cornellbox1":  # the default line (gpu_session.sh BENCH=1)
            f = os.path.join(src, "bench.log")
        if not os.path.exists(f):
            continue
        line = next(json.loads(s) for s in open(f) if s.startswith("{"))
        wl = line["config"]["workload"]
        segs = line["config"]["segments_per_frame"]
        kms = line["roofline"]["kernel_ms"]
        v = valu.get(wl, {}).get("valu_insts_per_segment")
        lu = valu.get(wl, {}).get("valu_lane_util")
        t = traffic.get(wl, {}).get("hbm_bytes_per_launch")
        sv = valu.get(wl, {}).get("salu_insts_per_segment")
        # the device's CUs as the line measured them (its VALU peak = CUs x 4.8 G/s), as bench.py's salu_frac
        n_cu = line["config"].get("n_cu") or round(line["roofline"]["peak"] / VALU_GINST_PER_CU)
        PEAK_VALU = n_cu * VALU_GINST_PER_CU
        sf = sv * segs / (n_cu * 2.4e9 * kms * 1e-3) if sv else None
        ach = v * segs / (kms * 1e-3) / 1e9 if v else None
        hbm = t / (kms * 1e-3) / 1e9 if t else None
        print(f"| {wl} | `{line['config'].get('variant')}` | {line['ms_per_step']:.3f} | {kms:.3f} | {segs / (line['ms_per_step'] * 1e-3) / 1e9:.2f} | "
              f"{v:.2f} | {ach:.0f} G/s ({ach / PEAK_VALU:.3f}) | "
              + (f"{lu:.3f} | {ach / PEAK_VALU * lu:.3f} | " if lu else "— | — | ")
              + (f"{sv:.2f} ({sf:.3f}) | " if sv else "— | ")
              + (f"{t / 1e9:.2f} GB ({hbm / PEAK_HBM:.4f}) |" if t else "— |"))


if __name__ == "__main__":
    main(sys.argv[1])
