#!/bin/bash
# UTCL1 (address translation) counters for the C4 / C5 moments launches (GPU box, repo root).
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/tlb
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for CFG in C4full C4 C5; do
  timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum --kernel-trace -d "$OUT/$CFG/a" -o run --output-format csv -- python3 "$ROOT/tools/probe_moments.py" $CFG moments 10 > "$OUT/$CFG.a.log" 2>&1
  timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum --kernel-trace -d "$OUT/$CFG/b" -o run --output-format csv -- python3 "$ROOT/tools/probe_moments.py" $CFG moments 10 > "$OUT/$CFG.b.log" 2>&1
done
