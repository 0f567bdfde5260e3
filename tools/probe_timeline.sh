#!/bin/bash
# Per-workgroup phase timeline (PROBE=4 build), run on the GPU box from the repo root.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
LIB=$ROOT/cc-mpc_amd/ccmpc/libccmpc.so
OUT=$ROOT/gpurun_out/variants
mkdir -p "$OUT"
cp "$LIB" /tmp/libccmpc.real.so
cp "$ROOT/cc-mpc_amd/csrc/${PROBE_LIB:-build_p4}/libccmpc.so" "$LIB"
timeout -k 10 300 python3 "$ROOT/tools/probe_phases.py" $JOBS > "$OUT/timeline.txt" 2>&1
cp /tmp/libccmpc.real.so "$LIB"
