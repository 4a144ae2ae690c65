#!/bin/bash
# Per-kernel VGPRs / scratch / occupancy / LDS of the HIP sources (compiler remarks, gfx950).
# Usage: tools/resource_usage.sh [file.hip ...]   (EXTRA="-D..." for a variant)
HERE=$(cd "$(dirname "$0")" && pwd)
cd "$HERE/../pose-splatter_amd/csrc"
for f in ${@:-*.hip}; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -I../../include -fno-slp-vectorize $EXTRA \
    --cuda-device-only -c "$f" -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 | python3 "$HERE/resource_usage.py" "$f"
done
