#!/bin/bash
# Build A/B variants of libptsvgf into path-tracing-svgf_amd/lib_exp/<name> (run here; they travel to the box).
# usage: bash tools/exp_build.sh name "EXTRA FLAGS" [name "FLAGS" ...]
set -e
cd "$(dirname "$0")/../path-tracing-svgf_amd"
while [ $# -gt 1 ]; do
  make -s -j8 OUT="lib_exp/$1" EXTRA="$2" "lib_exp/$1/libptsvgf.so" "lib_exp/$1/libptsvgf_host.so"
  shift 2
done
