# The step's input copy inside the placement's first launch (ccmpc_*_packed) against the
# separate copy kernel: the step / harness GPU tests, then the drop-in step lines under both
# settings, alternated (CCMPC_STEP_PACKED)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-packed}
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_step.py tests/test_gpu_step_modes.py tests/test_gpu_episode.py \
  tests/test_gpu_harness.py tests/test_gpu_planner.py tests/test_gpu_fused.py \
  > gpurun_out/${tag}_tests.log 2>&1
for r in 1 2 3; do
  for m in 0 2; do
    echo "== round $r packed $m" >> gpurun_out/${tag}_steps.jsonl
    CCMPC_STEP_PACKED=$m timeout -k 10 300 python -u tools/bench_steps.py dropin dropin_pp \
      dropin_pred_dev >> gpurun_out/${tag}_steps.jsonl 2>&1
  done
done
