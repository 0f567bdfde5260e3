# L4 on the GPU box: the L4 / step tests, phase timelines (PROBE=4 build in
# gpurun_probe/), then the drop-in step lines.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-l4a}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_planner.py tests/test_gpu_step.py \
  tests/test_gpu_step_modes.py tests/test_gpu_milp.py > gpurun_out/${tag}_tests.log 2>&1
bash tools/gpu_probe.sh ${tag} 100000:1 5000:4
timeout -k 10 300 python -u tools/bench_steps.py dropin dropin_100k > gpurun_out/${tag}_steps.jsonl 2>&1
