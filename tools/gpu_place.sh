# Placement on the GPU box: the sampler / bucketing / step tests, phase timelines (PROBE=4
# build in gpurun_probe/), the drop-in step lines at C2's shape and at 100 000 particles.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-pla}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_sample_bucket.py tests/test_gpu_load_predictions.py tests/test_gpu_fused.py \
  tests/test_gpu_step_modes.py tests/test_gpu_step.py tests/test_gpu_core.py > gpurun_out/${tag}_tests.log 2>&1
bash tools/gpu_probe.sh ${tag} 100000:1 5000:4
timeout -k 10 300 python -u tools/bench_steps.py dropin_100k dropin_pred_100k_dev dropin_100k dropin_pred_100k_dev > gpurun_out/${tag}_steps.jsonl 2>&1
