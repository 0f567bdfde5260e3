#!/bin/bash
# Placement vs finish time (PROBE=4 build), run on the GPU box from the repo root.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
LIB=$ROOT/cc-mpc_amd/ccmpc/libccmpc.so
OUT=$ROOT/gpurun_out/variants
mkdir -p "$OUT"
cp "$LIB" /tmp/libccmpc.real.so
cp "$ROOT/cc-mpc_amd/csrc/build_p4/libccmpc.so" "$LIB"
rc=0
for a in ${CASES:-"C4 moments" "C4 cycle" "C5 moments" "C2 cycle"}; do
  timeout -k 10 200 python3 "$ROOT/tools/probe_balance.py" $a >> "$OUT/balance.txt" 2>&1 || { rc=$?; break; }
done
cp /tmp/libccmpc.real.so "$LIB"
exit $rc
