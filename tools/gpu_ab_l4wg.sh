# L4 A/B on the GPU box: the step graph's L4 as one workgroup per (cell, t) (ccmpc_l4) against
# the split form (ccmpc_l4_split).  The L4 / step tests with the one-workgroup form forced, then
# the drop-in step lines under both settings, alternated.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-l4wg}
mkdir -p gpurun_out
CCMPC_L4_ONE_WG_MAX=1000000 timeout -k 10 400 python -u -m pytest -x -v --timeout 120 \
  --timeout-method thread -m gpu tests/test_gpu_core.py tests/test_gpu_fused.py \
  tests/test_gpu_planner.py tests/test_gpu_step.py tests/test_gpu_step_modes.py \
  > gpurun_out/${tag}_tests.log 2>&1
for r in 1 2; do
  for m in 0 8192; do
    echo "== round $r one_wg_max $m" >> gpurun_out/${tag}_steps.jsonl
    CCMPC_L4_ONE_WG_MAX=$m timeout -k 10 200 python -u tools/bench_steps.py dropin dropin_pp \
      dropin_pred_dev >> gpurun_out/${tag}_steps.jsonl 2>&1
  done
done
