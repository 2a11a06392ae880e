"""tools/valu_summary.py workload on synthetic rocprofv3 counter files (CPU only): the per-segment VALU count,
the lane utilisation and the wait shares from the VALU pass, the SALU / SMEM / branch counts from the sibling
pmc_salu_<scene> pass, averaged over the launched variant's dispatches only, and the symbol and digest recorded
for bench.py's check."""
import csv
import importlib.util
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("valu_summary", os.path.join(REPO, "tools", "valu_summary.py"))
vs = importlib.util.module_from_spec(spec)
spec.loader.exec_module(vs)

VARIANT = "render_kernel<false, true, false, false, 3>"
KERNEL = "void rt::render_kernel<false, true, false, false, 3>(rt::RenderLaunch, ...)"
OTHER = "rt::combine_kernel(rt::RenderLaunch, float*)"


def write_pass(d, rows):
    os.makedirs(os.path.join(d, "host", "1"), exist_ok=True)
    with open(os.path.join(d, "host", "1", "pmc_counter_collection.csv"), "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value",
                                           "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for disp, name, counters in rows:
            for c, v in counters.items():
                w.writerow({"Dispatch_Id": disp, "Kernel_Name": name, "Counter_Name": c, "Counter_Value": v,
                            "Start_Timestamp": 0, "End_Timestamp": 5_000_000})


def test_workload_entry_merges_valu_and_salu_passes(tmp_path):
    segs = 1000
    valu = {"SQ_INSTS_VALU": 24000, "SQ_WAVES": 64, "GRBM_GUI_ACTIVE": 8 * 5_000_000 * 2.4,
            "SQ_ACTIVE_INST_VALU": 24000, "SQ_THREAD_CYCLES_VALU": 24000 * 64 * 0.625, "SQ_WAIT_ANY": 30,
            "SQ_WAIT_INST_ANY": 20, "SQ_WAVE_CYCLES": 100, "SQ_BUSY_CYCLES": 1}
    write_pass(str(tmp_path / "pmc_valu_cornellbox1"),
               [(1, KERNEL, valu), (2, OTHER, {"SQ_INSTS_VALU": 9e9}), (3, KERNEL, dict(valu, SQ_INSTS_VALU=26000))])
    salu = {"SQ_INSTS_SALU": 8000, "SQ_INSTS_SMEM": 1000, "SQ_INSTS_BRANCH": 2500, "SQ_WAVES": 64}
    write_pass(str(tmp_path / "pmc_salu_cornellbox1"), [(1, KERNEL, salu), (2, OTHER, {"SQ_INSTS_SALU": 7e9})])
    line = {"config": {"workload": "cornellbox1_512x512_spp128_d8_n1", "segments_per_frame": segs,
                       "variant": VARIANT, "kernel_source_sha": "0123456789abcdef"}}
    log = tmp_path / "pmc_valu_cornellbox1.log"
    log.write_text("noise\n" + json.dumps(line) + "\n")
    out = tmp_path / "valu_issue.json"
    wl, ent = vs.workload(str(tmp_path / "pmc_valu_cornellbox1"), str(log), str(out))
    assert wl == "cornellbox1_512x512_spp128_d8_n1"
    assert ent["valu_insts_per_segment"] == 25.0  # mean of the variant's two dispatches, not the combine pass
    assert ent["dispatches"] == 2
    assert abs(ent["valu_lane_util"] - 0.625) < 1e-12
    assert ent["wait_any_share"] == 0.3 and ent["wait_inst_any_share"] == 0.2
    assert ent["salu_insts_per_segment"] == 8.0 and ent["smem_insts_per_segment"] == 1.0
    assert ent["branch_insts_per_segment"] == 2.5
    assert ent["variant"] == VARIANT and ent["kernel_source_sha"] == "0123456789abcdef"
    assert json.load(open(out))["workloads"][wl]["salu_insts_per_segment"] == 8.0
