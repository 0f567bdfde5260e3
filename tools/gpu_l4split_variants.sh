# The split L4 at C1's 100 000 particles under build variants (gpurun_probe/libccmpc_<v>.so):
# rocprofv3 kernel stats of the step graph's replays, and the step lines
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in base c4096 c4096p8 c8192p8; do
  lib=cc-mpc_amd/ccmpc/libccmpc.so
  [ $v = base ] || lib=gpurun_probe/libccmpc_$v.so
  CCMPC_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/l4v_$v -o run -- python3 tools/step_replay.py step_c1_100k 200 \
    > gpurun_out/l4v_$v.log 2>&1
  echo "== $v" >> gpurun_out/l4v_steps.jsonl
  CCMPC_LIB=$lib timeout -k 10 200 python3 -u tools/bench_steps.py dropin_100k dropin_pred_100k_dev \
    >> gpurun_out/l4v_steps.jsonl 2>&1
done
