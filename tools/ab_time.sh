#!/bin/bash
# A/B kernel timing of alternative libccmpc.so builds (LIBS="build_x build_y", relative to
# cc-mpc_amd/csrc; "main" = the in-tree library), run on the GPU box from the repo root.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
LIB=$ROOT/cc-mpc_amd/ccmpc/libccmpc.so
OUT=$ROOT/gpurun_out/variants
mkdir -p "$OUT"
cp "$LIB" /tmp/libccmpc.real.so
rc=0
for rep in 1 2; do
  for v in ${LIBS:-main}; do
    if [ "$v" = main ]; then cp /tmp/libccmpc.real.so "$LIB"; else cp "$ROOT/cc-mpc_amd/csrc/$v/libccmpc.so" "$LIB"; fi
    echo "== $v (rep $rep)" >> "$OUT/ab.txt"
    timeout -k 10 200 python3 "$ROOT/tools/probe_moments.py" x time 0 >> "$OUT/ab.txt" 2>&1 || { rc=$?; break 2; }
  done
done
cp /tmp/libccmpc.real.so "$LIB"
exit $rc
