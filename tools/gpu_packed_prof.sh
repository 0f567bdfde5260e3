# rocprofv3 kernel stats of step graph replays with the input copy in the placement's first
# launch (CCMPC_STEP_PACKED=1) and as its own kernel (0)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in step_c2 step_pred_dev_c2; do
  for m in 0 1; do
    CCMPC_STEP_PACKED=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/pk_${cfg}_$m -o run -- python3 tools/step_replay.py $cfg 200 \
      > gpurun_out/pk_${cfg}_$m.log 2>&1
  done
done
