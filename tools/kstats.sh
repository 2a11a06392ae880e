#!/bin/bash
# Per-kernel register / scratch / LDS summary of the megakernel TU's assembly (make asm).
#   bash tools/kstats.sh [asm file]   (default raytracingthenextweekcuda_amd/csrc/build/rt_kernel.s)
f=${1:-$(dirname "$0")/../raytracingthenextweekcuda_amd/csrc/build/rt_kernel.s}
awk '/^[ \t]*\.size[ \t]+_ZN2rt/ {split($2,a,","); name=a[1]}
     /; NumVgprs:/ {v=$3} /; ScratchSize:/ {sc=$3} /; TotalNumSgprs:/ {sg=$3} /; Occupancy:/ {occ=$3}
     /; LDSByteSize:/ {lds=$3; n=name; sub(/EvNS_12RenderLaunch.*/,"",n); sub(/^_ZN2rt[0-9]+/,"",n);
       printf "%-48s vgpr %3s sgpr %3s scratch %3s lds %6s\n", n, v, sg, sc, lds}' "$f"
