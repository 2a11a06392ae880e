#!/bin/bash
# A/B library of the current sources with extra compile flags (same-box comparisons through RTMI_LIB):
#   bash tools/build_ab.sh <name> "<EXTRA flags>"   ->  raytracingthenextweekcuda_amd/librtmi_<name>.so
# (its own object directory csrc/build_<name>; rt_build_flags reports RT_BUILD_AB for non-default switches)
set -e
name=$1; shift
cd "$(dirname "$0")/../raytracingthenextweekcuda_amd/csrc"
make -s -j8 OUT=../librtmi_$name.so BUILD=build_$name EXTRA="$*" 2>&1 | grep -v "warning: argument unused" || true
ls -la ../librtmi_$name.so
