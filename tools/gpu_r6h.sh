set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_step_modes.py tests/test_gpu_harness.py tests/test_gpu_load_predictions.py > gpurun_out/r6h_tests.log 2>&1
timeout -k 10 300 python -u tools/bench_steps.py dropin_pred_dev dropin_pred_100k_dev dropin_pred_dev > gpurun_out/r6h_steps.log 2>&1
