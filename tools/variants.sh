#!/bin/bash
# Build A/B variants of librtmi.so (experiments only): tools/variants.sh name "-DFLAG=.."
set -e
cd "$(dirname "$0")/../raytracingthenextweekcuda_amd/csrc"
make -s -j4 BUILD=build_$1 OUT=../librtmi_$1.so EXTRA="$2"
