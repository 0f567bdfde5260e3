#!/bin/bash
# Per-configuration kernel profiles (run on the GPU box via gpurun, from the repo root):
#   bash profiles/collect_configs.sh r02
# For each BASELINE configuration's one-launch cycle (tools/probe_moments.py; C4full and C5
# rotate over 3 copies of the store so every launch streams from HBM, not the 256 MiB
# Infinity Cache):
#   1. rocprofv3 --kernel-trace --stats              -> per-kernel durations
#   2. rocprofv3 --pmc FETCH_SIZE   (own pass, kernel trace only)
#   3. rocprofv3 --pmc WRITE_SIZE   (own pass, kernel trace only)
# then profiles/summarize.py writes gpurun_out/prof_<round>_<config>/summary/summary.json.
set -euo pipefail
ROUND=${1:-r02}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
# cycle configs (tools/probe_moments.py) and planning-step configs (tools/step_replay.py: the
# whole step graph, every kernel of the step)
ALL=("C2 1 400" "C3-1e3 1 400" "C3-2e4 1 400" "C3 1 400" "C4 1 200" "C4full 3 30" "C5 3 60"
     "step_c2 0 300" "step_c1_100k 0 200" "step_pred_c2 0 300" "step_pred_dev_c2 0 300"
     "step_pred_dev_100k 0 200")
for spec in "${ALL[@]}"; do
  set -- $spec
  if [ -n "${ONLY:-}" ] && [[ ",$ONLY," != *",$1,"* ]]; then continue; fi
  CFG=$1; ROT=$2; IT=$3
  OUT=$ROOT/gpurun_out/prof_${ROUND}_${CFG}
  mkdir -p "$OUT"
  if [[ $CFG == step_* ]]; then
    RUN="python3 $ROOT/tools/step_replay.py $CFG $IT"
  else
    RUN="python3 $ROOT/tools/probe_moments.py $CFG cycle $IT"
  fi
  ROTATE=$ROT timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- $RUN > "$OUT/trace.log" 2>&1
  ROTATE=$ROT timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/fetch" -o run --output-format csv -- $RUN > "$OUT/fetch.log" 2>&1
  ROTATE=$ROT timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/write" -o run --output-format csv -- $RUN > "$OUT/write.log" 2>&1
  python3 "$ROOT/profiles/summarize.py" "$OUT" "$OUT/summary" > "$OUT/summary.txt"
  echo "$CFG done"
done
