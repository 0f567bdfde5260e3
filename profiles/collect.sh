#!/bin/bash
# Profile collection for one round (run on the GPU box via gpurun, from the repo root):
#   bash profiles/collect.sh r01
# 1. rocprofv3 --kernel-trace --stats of the default bench workload (C2)      -> kernel durations
# 2. rocprofv3 --pmc FETCH_SIZE (own pass, kernel trace only)                   -> HBM read bytes
# 3. rocprofv3 --pmc WRITE_SIZE (own pass, kernel trace only)                   -> HBM write bytes
# then profiles/summarize.py writes profiles/<round>/summary.json (per-kernel averages, with the
# gfx950 FETCH_SIZE x2 correction of MI355X_MICROARCH.md "HBM").
# Counter passes never combine --pmc with sys/runtime/hip/hsa tracing.
set -euo pipefail
ROUND=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$ROUND
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
BENCH="python3 $ROOT/bench.py --no-cpu --steps 300 --warmup 30"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- $BENCH > "$OUT/trace_bench.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/fetch" -o run --output-format csv -- $BENCH > "$OUT/fetch_bench.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/write" -o run --output-format csv -- $BENCH > "$OUT/write_bench.log" 2>&1
# summary lands under gpurun_out/ (merged back); copy into profiles/<round>/ afterwards with
#   python profiles/summarize.py gpurun_out/prof_<round> profiles/<round>
python3 "$ROOT/profiles/summarize.py" "$OUT" "$OUT/summary"
