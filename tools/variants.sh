#!/bin/bash
# Build A/B variants of libaicp_hip.so (CPU side): bash tools/variants.sh NAME "FLAGS" [NAME "FLAGS" ...]
# Each lands in build_ab/lib_NAME.so; run them with tools/run_variants.sh NAME...
set -e
cd "$(dirname "$0")/.."
mkdir -p build_ab
while [ $# -ge 2 ]; do
  make -s -j8 -C aicp_mapping_amd/csrc OUT=$PWD/build_ab/lib_$1.so OBJDIR=build_$1 EXTRA="$2" >/dev/null
  echo "built build_ab/lib_$1.so ($2)"
  shift 2
done
