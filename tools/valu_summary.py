"""VALU-issue roofline inputs from rocprofv3 PMC passes.

  python tools/valu_summary.py calibrate <probe_dir_10000> <probe_dir_20000> [valu_probe.json]
      -> profiles/<round>/valu_probe.json: SQ_INSTS_VALU of tools/valu_probe at two trip
         counts; their difference must be waves x 8 x d_iters (the whole chip, exactly).
  python tools/valu_summary.py lanes <probe_dir_64> <probe_dir_16>
      -> the lane-utilisation counter ratio SQ_THREAD_CYCLES_VALU / 64 / SQ_ACTIVE_INST_VALU of
         tools/valu_probe with 64 and 16 active lanes per wave (expected 1 and 0.25).
  python tools/valu_summary.py workload <pmc_dir> <bench_log> [out_json]
      -> merges {workload: valu_insts_per_segment, ...} into profiles/valu_issue.json, from
         the render/pathtrace kernel dispatches of a `--pmc SQ_INSTS_VALU SQ_WAVES
         GRBM_GUI_ACTIVE ...` pass over bench.py and that bench's own JSON line (segments).
"""
import collections
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def dispatches(pmc_dir, match=None):
    out = collections.OrderedDict()
    for f in sorted(glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            if match and not any(m in r["Kernel_Name"] for m in match):
                continue
            d = out.setdefault(int(r["Dispatch_Id"]), {"kernel": r["Kernel_Name"], "counters": collections.Counter(),
                                                        "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
            d["counters"][r["Counter_Name"]] += float(r["Counter_Value"])
    return out


def calibrate(d1, d2, probe_json=None):
    a, b = dispatches(d1, ["valu_probe"]), dispatches(d2, ["valu_probe"])
    ia = [v["counters"]["SQ_INSTS_VALU"] for v in a.values()]
    ib = [v["counters"]["SQ_INSTS_VALU"] for v in b.values()]
    waves = next(iter(a.values()))["counters"]["SQ_WAVES"]
    it1, it2 = [int(os.path.basename(os.path.normpath(d)).rsplit("_", 1)[1]) for d in (d1, d2)]
    delta = ib[0] - ia[0]
    expect = waves * 8 * (it2 - it1)
    res = {"probe": "tools/valu_probe.hip: 8 independent v_fma_f32 per trip per wave",
           "waves": waves, "iters": [it1, it2], "sq_insts_valu": [ia[0], ib[0]],
           "delta": delta, "expected_delta_whole_chip": expect, "ratio": delta / expect,
           "extra_per_wave": (ia[0] - waves * 8 * it1) / waves,
           "verdict": "SQ_INSTS_VALU counts wave64 VALU instructions of the whole chip"
           if abs(delta / expect - 1) < 1e-6 else "NOT whole-chip: check normalisation"}
    if probe_json and os.path.exists(probe_json):
        for line in open(probe_json):
            if line.startswith("{"):
                res["timed"] = json.loads(line)
    return res


def lane_util(c):
    """Mean active lanes per issued wave64 VALU instruction, as a fraction of 64."""
    if not c.get("SQ_ACTIVE_INST_VALU") or "SQ_THREAD_CYCLES_VALU" not in c:
        return None
    return c["SQ_THREAD_CYCLES_VALU"] / 64.0 / c["SQ_ACTIVE_INST_VALU"]


def lanes(d64, d16):
    out = {"probe": "tools/valu_probe: the same VALU loop run by 64 or 16 lanes of each wave"}
    for name, d, want in (("active_64", d64, 1.0), ("active_16", d16, 0.25)):
        ds = dispatches(d, ["valu_probe"])
        v = list(ds.values())[-1]["counters"]
        out[name] = {"sq_thread_cycles_valu": v.get("SQ_THREAD_CYCLES_VALU"),
                     "sq_active_inst_valu": v.get("SQ_ACTIVE_INST_VALU"),
                     "sq_insts_valu": v.get("SQ_INSTS_VALU"), "lane_util": lane_util(v), "expected": want}
    return out


def workload(pmc_dir, bench_log, out_json):
    line = next(json.loads(s) for s in open(bench_log) if s.startswith("{"))
    wl = line["config"]["workload"]
    segs = line["config"]["segments_per_frame"]
    # only the launched variant's dispatches (bench.py's line names it; rt_kernel_variant_name)
    variant = line["config"].get("variant")
    ds = dispatches(pmc_dir, [variant] if variant else ["render_kernel", "pathtrace_kernel"])
    if not ds:
        raise SystemExit(f"{pmc_dir}: no dispatch of {variant!r}")
    insts = [v["counters"]["SQ_INSTS_VALU"] for v in ds.values()]
    # every dispatch of the pass renders the same frame (warm-up + timed): take their mean
    per_launch = sum(insts) / len(insts)
    clk = [v["counters"]["GRBM_GUI_ACTIVE"] / 8 / (v["ns"] * 1e-9) / 1e9 for v in ds.values() if v["ns"] > 0]
    tot = collections.Counter()
    for v in ds.values():
        tot.update(v["counters"])
    ent = {"kernel": next(iter(ds.values()))["kernel"].split("(")[0],
           "valu_insts_per_launch": per_launch, "spread": (max(insts) - min(insts)) / per_launch,
           "segments_per_launch": segs, "valu_insts_per_segment": per_launch / segs,
           "effective_clock_ghz": sum(clk) / len(clk) if clk else None,
           "dispatches": len(insts), "source": os.path.relpath(pmc_dir, REPO),
           # VALU lane utilisation (SQ_THREAD_CYCLES_VALU / 64 / SQ_ACTIVE_INST_VALU, calibrated with
           # tools/valu_probe's active-lane mode) and the wave-cycle shares, summed over the dispatches
           "valu_lane_util": lane_util(tot),
           "wait_inst_any_share": (tot["SQ_WAIT_INST_ANY"] / tot["SQ_WAVE_CYCLES"]) if tot.get("SQ_WAVE_CYCLES") else None,
           "wait_any_share": (tot["SQ_WAIT_ANY"] / tot["SQ_WAVE_CYCLES"]) if tot.get("SQ_WAVE_CYCLES") else None,
           # what bench.py checks before using the entry: the launched symbol and the kernel sources
           "variant": variant, "kernel_source_sha": line["config"].get("kernel_source_sha")}
    # the scalar side, from the sibling pmc_salu_<scene> pass (gpu_session.sh VALU=...) when present:
    # SALU instructions per segment (the CU's one scalar ALU issues at most one per cycle)
    sdir = pmc_dir.replace("pmc_valu_", "pmc_salu_")
    sds = dispatches(sdir, [variant] if variant else ["render_kernel", "pathtrace_kernel"]) if sdir != pmc_dir else {}
    if sds:
        salu = [v["counters"]["SQ_INSTS_SALU"] for v in sds.values()]
        stot = collections.Counter()
        for v in sds.values():
            stot.update(v["counters"])
        n = len(salu)
        ent.update({"salu_insts_per_segment": sum(salu) / n / segs,
                    "smem_insts_per_segment": stot["SQ_INSTS_SMEM"] / n / segs,
                    "branch_insts_per_segment": stot["SQ_INSTS_BRANCH"] / n / segs,
                    "salu_source": os.path.relpath(sdir, REPO)})
    d = json.load(open(out_json)) if os.path.exists(out_json) else {}
    d.setdefault("note", "SQ_INSTS_VALU (whole chip, wave64 instructions; calibrated in profiles/r02/valu_probe.json) "
                         "of the bench workload's render kernel per traced segment; bench.py multiplies it by the "
                         "live launch's segments and divides by the live kernel time")
    d.setdefault("workloads", {})[wl] = ent
    with open(out_json, "w") as fh:
        json.dump(d, fh, indent=1, sort_keys=True)
    return wl, ent


if __name__ == "__main__":
    if sys.argv[1] == "calibrate":
        print(json.dumps(calibrate(*sys.argv[2:5]), indent=1))
    elif sys.argv[1] == "lanes":
        print(json.dumps(lanes(*sys.argv[2:4]), indent=1))
    else:
        out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(REPO, "profiles", "valu_issue.json")
        print(workload(sys.argv[2], sys.argv[3], out))
