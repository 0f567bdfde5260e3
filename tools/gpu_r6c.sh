set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sample_bucket.py tests/test_gpu_load_predictions.py > gpurun_out/r6c_tests.log 2>&1
bash tools/gpu_probe.sh r6c 100000:1 5000:4
timeout -k 10 300 python -u tools/bench_steps.py dropin dropin_100k dropin_pred_dev dropin_pred_100k_dev > gpurun_out/r6c_steps.log 2>&1
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_step_modes.py tests/test_gpu_harness.py tests/test_gpu_episode.py tests/test_gpu_planner.py > gpurun_out/r6c_tests2.log 2>&1
