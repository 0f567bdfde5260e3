#!/bin/bash
# Time the moments kernel with its MFMAs and/or loads stubbed out (make probe PROBE=1|2|3), to
# split a launch into memory, matrix-core and fixed (locate / combine / finalise) time.
# Run on the GPU box from the repo root; restores the real library at the end.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
LIB=$ROOT/cc-mpc_amd/ccmpc/libccmpc.so
OUT=$ROOT/gpurun_out/variants
mkdir -p "$OUT"
cp "$LIB" "$OUT/libccmpc.real.so"
for V in real 1 2 3; do
  if [ "$V" != real ]; then cp "$ROOT/cc-mpc_amd/csrc/build_p$V/libccmpc.so" "$LIB"; fi
  echo "== variant $V" | tee -a "$OUT/times.txt"
  timeout -k 10 300 python3 "$ROOT/tools/probe_moments.py" ALL time 0 >> "$OUT/times.txt" 2>&1
done
cp "$OUT/libccmpc.real.so" "$LIB"
