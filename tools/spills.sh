#!/bin/bash
# Register / spill / LDS census of the kernels in csrc/build/rt_kernel.s (make asm).
f=${1:-raytracingthenextweekcuda_amd/csrc/build/rt_kernel.s}
grep -E "^\s+\.(name|vgpr_count|vgpr_spill_count|sgpr_spill_count|private_segment_fixed_size|sgpr_count|group_segment_fixed_size):" "$f" |
  awk '{k=$1; v=$2; gsub(/[.:]/,"",k); d[k]=v; if (k=="vgpr_spill_count") {n=d["name"]; sub(/^_ZN2rt[0-9]+/,"",n);
       printf "%-46s vgpr %3s spill %3s | sgpr %3s spill %3s | scratch %3s B | static lds %s\n", substr(n,1,46), d["vgpr_count"], v, d["sgpr_count"], d["sgpr_spill_count"], d["private_segment_fixed_size"], d["group_segment_fixed_size"]}}'
