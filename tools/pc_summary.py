"""Digest of a stochastic PC-sampling run (tools/pc_sample.sh): samples of the render kernel per
instruction, per instruction class and per stall reason, with the instruction text and the
disassembly neighbourhood of the hottest PCs.
  python tools/pc_summary.py gpurun_out/<tag>/pcs_<scene> [kernel substring] [top]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else "render_kernel"
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
files = [f for f in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True) if "pc_sampling" in os.path.basename(f)]
if not files:
    raise SystemExit(f"no pc_sampling csv under {d}: {glob.glob(os.path.join(d, '**', '*'), recursive=True)[:20]}")
rows = []
for f in files:
    with open(f) as fh:
        rows += list(csv.DictReader(fh))
print("files:", files, "rows:", len(rows))
print("columns:", list(rows[0].keys()) if rows else None)
kcol = next((c for c in rows[0] if "Kernel" in c or "kernel" in c), None) if rows else None
icol = next((c for c in ("Instruction", "instruction") if rows and c in rows[0]), None)
sel = [r for r in rows if not kcol or want in r.get(kcol, "")] if rows else []
print(f"samples in {want!r}: {len(sel)} of {len(rows)}")
if not sel:
    raise SystemExit(0)
by_inst = collections.Counter()
by_op = collections.Counter()
stall = collections.Counter()
issued = collections.Counter()
for r in sel:
    ins = (r.get(icol) or "?").strip() if icol else "?"
    key = (r.get("Code_Object_Offset") or r.get("Pc") or r.get("PC") or "", ins)
    by_inst[key] += 1
    by_op[ins.split()[0] if ins else "?"] += 1
    for c in r:
        if "Stall" in c or "stall" in c:
            stall[(c, r[c])] += 1
        if "Issued" in c or "issued" in c:
            issued[(c, r[c])] += 1
n = len(sel)
print("\nby opcode:")
for k, v in by_op.most_common(30):
    print(f"  {v / n:6.3f} {k}")
if stall:
    print("\nstall reasons:")
    for k, v in stall.most_common(20):
        print(f"  {v / n:6.3f} {k}")
if issued:
    print("\nissued:")
    for k, v in issued.most_common(10):
        print(f"  {v / n:6.3f} {k}")
print(f"\ntop {top} instructions:")
for (pc, ins), v in by_inst.most_common(top):
    print(f"  {v / n:6.4f} {pc:>12} {ins}")
