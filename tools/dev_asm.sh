#!/bin/bash
# Device assembly of the headline forward instance only (-DENFLOW_DEV_ONLY), for
# instruction-mix / register checks while editing flow_device.h:
#   bash tools/dev_asm.sh OUT.s [extra hipcc flags]
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-/tmp/dev_flow.s}; shift || true
hipcc --offload-arch=gfx950 -O3 -std=c++17 -I "$ROOT/include" -DENFLOW_DEV_ONLY "$@" --cuda-device-only -S \
  -o "$OUT" "$ROOT/enflow_amd/csrc/enflow_flow.hip" 2>&1 | grep -v "hip-link"
