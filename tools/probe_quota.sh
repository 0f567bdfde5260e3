#!/bin/bash
# Wave-quota sweep of the large-input path (PROBE=8 build: CCMPC_LG_WQ override), GPU box.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
LIB=$ROOT/cc-mpc_amd/ccmpc/libccmpc.so
OUT=$ROOT/gpurun_out/variants
mkdir -p "$OUT"
cp "$LIB" /tmp/libccmpc.real.so
cp "$ROOT/cc-mpc_amd/csrc/build_p8/libccmpc.so" "$LIB"
rc=0
for q in ${QUOTAS:-8 7 6}; do
  echo "== lg_wq $q" >> "$OUT/quota.txt"
  CCMPC_LG_WQ=$q timeout -k 10 200 python3 "$ROOT/tools/probe_moments.py" x time 0 >> "$OUT/quota.txt" 2>&1 || { rc=$?; break; }
done
cp /tmp/libccmpc.real.so "$LIB"
exit $rc
