# QP on the GPU box: the QP test files, then the QP bench lines.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-qpa}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_qp_gi.py tests/test_gpu_mpc.py tests/test_gpu_episode.py tests/test_gpu_milp.py > gpurun_out/${tag}_tests.log 2>&1
timeout -k 10 300 python -u tools/bench_steps.py qp1_t8 qp qp1_t12 qp_t12 > gpurun_out/${tag}_bench.jsonl 2>&1
