"""Summarise per-scene rocprofv3 runs (tools/gpu_profiles.sh) into
profiles/pmc_traffic.json and copy the evidence into profiles/<round>/.

HBM bytes per launch of the render kernel = FETCH_SIZE x 2 (gfx950 counts half
of the streamed reads, MI355X_MICROARCH.md) + WRITE_SIZE, both in KB (1024 B),
averaged over the kernel's launches in the PMC pass.
Usage: python tools/pmc_summary.py <round> [scene ...]
       RTMI_PMC_SRC=gpurun_out/<tag> python tools/pmc_summary.py <round> [scene ...]
"""
import csv
import glob
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, os.environ.get("RTMI_PMC_SRC", "gpurun_out"))
KERNELS = ("render_kernel", "pathtrace_kernel")


def kernel_mean(path, counter):
    vals = {}
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter or not any(k in row["Kernel_Name"] for k in KERNELS):
            continue
        vals.setdefault(row["Dispatch_Id"], 0.0)
        vals[row["Dispatch_Id"]] += float(row["Counter_Value"])
    return sum(vals.values()) / len(vals) if vals else None


def workload(scene):
    log = os.path.join(OUT, f"prof_{scene}.log")
    for line in open(log):
        if line.startswith("{"):
            return json.loads(line)["config"]["workload"], json.loads(line)
    raise RuntimeError(f"no bench line in {log}")


def main():
    rnd = sys.argv[1]
    scenes = sys.argv[2:] or ["cornellbox1", "spheres", "bunny", "materialball", "media"]
    dst = os.path.join(REPO, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    jpath = os.path.join(REPO, "profiles", "pmc_traffic.json")
    table = json.load(open(jpath)) if os.path.exists(jpath) else {}
    for scene in scenes:
        wl, line = workload(scene)
        stats = glob.glob(os.path.join(OUT, f"prof_{scene}", "**", "*kernel_stats.csv"), recursive=True)
        if stats:
            shutil.copy(stats[0], os.path.join(dst, f"kernel_stats_{scene}.csv"))
        shutil.copy(os.path.join(OUT, f"prof_{scene}.log"), os.path.join(dst, f"bench_{scene}_under_rocprof.log"))
        vals = {}
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            f = glob.glob(os.path.join(OUT, f"pmc_{scene}_{c}", "**", "*counter_collection.csv"), recursive=True)
            if not f:
                continue
            vals[c] = kernel_mean(f[0], c)
            shutil.copy(f[0], os.path.join(dst, f"pmc_{scene}_{c.lower()}.csv"))
        if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:
            hbm = (2.0 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024.0
            table[wl] = {
                "fetch_size_kb": round(vals["FETCH_SIZE"], 1),
                "write_size_kb": round(vals["WRITE_SIZE"], 1),
                "hbm_bytes_per_launch": hbm,
                "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes "
                          "(tools/gpu_profiles.sh); FETCH_SIZE doubled per MI355X_MICROARCH.md "
                          "(gfx950 counts half of streamed reads); KB = 1024 B",
                "source": f"profiles/{rnd}/pmc_{scene}_fetch_size.csv, profiles/{rnd}/pmc_{scene}_write_size.csv",
            }
            print(scene, wl, "HBM bytes/launch", hbm, "kernel_ms", line["roofline"]["kernel_ms"])
    json.dump(table, open(jpath, "w"), indent=1)


if __name__ == "__main__":
    main()
