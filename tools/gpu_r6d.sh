set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sample_bucket.py tests/test_gpu_load_predictions.py > gpurun_out/r6d_tests.log 2>&1
bash tools/gpu_probe.sh r6d 100000:1
timeout -k 10 300 python -u tools/bench_steps.py dropin_100k > gpurun_out/r6d_steps.log 2>&1
