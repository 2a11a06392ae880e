"""Summarise per-scene rocprofv3 runs (tools/gpu_session.sh) into profiles/pmc_traffic.json and
copy the evidence into profiles/<round>/.

HBM bytes per launch of the render kernel = FETCH_SIZE x 2 (gfx950 counts half of the streamed
reads, MI355X_MICROARCH.md) + WRITE_SIZE, both in KB (1024 B), averaged over the launched
variant's dispatches in the PMC pass (FETCH_SIZE and WRITE_SIZE in separate passes). Each entry
records the kernel symbol and the kernel-source digest of the pass's own bench line, which
bench.py checks before it uses the entry.
Usage: RTMI_PMC_SRC=gpurun_out/<tag> python tools/pmc_summary.py <round> [scene ...]
"""
import csv
import glob
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, os.environ.get("RTMI_PMC_SRC", "gpurun_out"))


def bench_line(log):
    for line in open(log):
        if line.startswith("{"):
            return json.loads(line)
    raise RuntimeError(f"no bench line in {log}")


def kernel_mean(path, counter, variant):
    vals, names = {}, set()
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter or variant not in row["Kernel_Name"]:
            continue
        names.add(row["Kernel_Name"].split("(")[0])
        vals.setdefault(row["Dispatch_Id"], 0.0)
        vals[row["Dispatch_Id"]] += float(row["Counter_Value"])
    if len(names) != 1:
        raise SystemExit(f"{path}: {counter} dispatches of {variant!r}: {sorted(names)}")
    return sum(vals.values()) / len(vals), names.pop()


def main():
    rnd = sys.argv[1]
    scenes = sys.argv[2:] or ["cornellbox1", "spheres", "bunny", "materialball", "media", "suzanne"]
    dst = os.path.join(REPO, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    jpath = os.path.join(REPO, "profiles", "pmc_traffic.json")
    table = json.load(open(jpath)) if os.path.exists(jpath) else {}
    for scene in scenes:
        vals, lines = {}, {}
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            f = glob.glob(os.path.join(OUT, f"pmc_{scene}_{c}", "**", "*counter_collection.csv"), recursive=True)
            if not f:
                continue
            lines[c] = bench_line(os.path.join(OUT, f"pmc_{scene}_{c}.log"))
            vals[c] = kernel_mean(f[0], c, lines[c]["config"]["variant"])
            shutil.copy(f[0], os.path.join(dst, f"pmc_{scene}_{c.lower()}.csv"))
            shutil.copy(os.path.join(OUT, f"pmc_{scene}_{c}.log"), os.path.join(dst, f"pmc_{scene}_{c.lower()}.log"))
        if len(vals) < 2:
            continue
        a, b = lines["FETCH_SIZE"]["config"], lines["WRITE_SIZE"]["config"]
        assert a["workload"] == b["workload"] and a["kernel_source_sha"] == b["kernel_source_sha"], (a, b)
        hbm = (2.0 * vals["FETCH_SIZE"][0] + vals["WRITE_SIZE"][0]) * 1024.0
        table[a["workload"]] = {
            "fetch_size_kb": round(vals["FETCH_SIZE"][0], 1),
            "write_size_kb": round(vals["WRITE_SIZE"][0], 1),
            "hbm_bytes_per_launch": hbm,
            "kernel": vals["FETCH_SIZE"][1],
            "kernel_source_sha": a["kernel_source_sha"],
            "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes "
                      "(tools/gpu_session.sh); FETCH_SIZE doubled per MI355X_MICROARCH.md "
                      "(gfx950 counts half of streamed reads); KB = 1024 B",
            "source": f"profiles/{rnd}/pmc_{scene}_fetch_size.csv, profiles/{rnd}/pmc_{scene}_write_size.csv",
        }
        print(scene, a["workload"], vals["FETCH_SIZE"][1], "HBM bytes/launch", hbm)
    json.dump(table, open(jpath, "w"), indent=1)


if __name__ == "__main__":
    main()
