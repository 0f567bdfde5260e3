#!/bin/bash
# Counter passes for the C4/C5 moments kernel (run on the GPU box from the repo root).
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/probe
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 60 "$ROOT/tools/mfma_f64_rate" > "$OUT/mfma_rate.txt" 2>&1
cd /tmp
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
for CFG in C4 C5; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/$CFG/trace" -o run --output-format csv -- python3 "$ROOT/tools/probe_moments.py" $CFG moments 100 > "$OUT/$CFG.trace.log" 2>&1
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d "$OUT/$CFG/sq" -o run --output-format csv -- python3 "$ROOT/tools/probe_moments.py" $CFG moments 20 > "$OUT/$CFG.sq.log" 2>&1
  timeout -k 10 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace -d "$OUT/$CFG/mfma" -o run --output-format csv -- python3 "$ROOT/tools/probe_moments.py" $CFG moments 20 > "$OUT/$CFG.mfma.log" 2>&1
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/$CFG/fetch" -o run --output-format csv -- python3 "$ROOT/tools/probe_moments.py" $CFG moments 20 > "$OUT/$CFG.fetch.log" 2>&1
done
