set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sample_bucket.py tests/test_gpu_load_predictions.py > gpurun_out/r6b_tests.log 2>&1
bash tools/gpu_probe.sh r6b_nw4 100000:1
CCMPC_PLACE_WIDE2=1 bash tools/gpu_probe.sh r6b_wide2 100000:1
CCMPC_PLACE_V2=1 bash tools/gpu_probe.sh r6b_v2 5000:4
CCMPC_PLACE_V2=1 CCMPC_RARE_TWO_PASS=1 bash tools/gpu_probe.sh r6b_v2tp 5000:4
timeout -k 10 300 python -u tools/bench_steps.py dropin dropin_100k > gpurun_out/r6b_steps.log 2>&1
CCMPC_PLACE_WIDE2=1 timeout -k 10 300 python -u tools/bench_steps.py dropin_100k > gpurun_out/r6b_steps_wide2.log 2>&1
CCMPC_PLACE_V2=1 timeout -k 10 300 python -u tools/bench_steps.py dropin > gpurun_out/r6b_steps_v2.log 2>&1
timeout -k 10 300 python -u tools/bench_steps.py dropin_pred dropin_pred_dev dropin_pred_100k dropin_pred_100k_dev > gpurun_out/r6b_steps_pred.log 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_harness.py tests/test_gpu_step_modes.py tests/test_gpu_episode.py > gpurun_out/r6b_tests2.log 2>&1
