#!/bin/bash
# Build timing-experiment variants of libgsr.so (results are NOT correct; timing only).
# Usage: tools/build_variants.sh NAME "-DFLAG ..." [NAME "-D..." ...]  → build_var/libgsr_NAME.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -ge 2 ]; do
  make -s -C "$ROOT/pose-splatter_amd/csrc" -j8 OUT="$ROOT/build_var/libgsr_$1.so" \
       OBJDIR="$ROOT/build_var/obj_$1" EXTRA="$2"
  shift 2
done
