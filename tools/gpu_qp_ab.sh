# QP step A/B on the GPU box: the GI tests, then the 30-step T = 8 scene, the T = 8 / 12 batches
# and the single frames (tools/qp_probe.py, tools/bench_steps.py)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-qpb}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_qp_gi.py tests/test_gpu_mpc.py tests/test_gpu_milp.py > gpurun_out/${tag}_tests.log 2>&1
QP_FIRST=59 timeout -k 10 200 python -u tools/qp_probe.py 8 1 > gpurun_out/${tag}_scene59.log 2>&1
timeout -k 10 300 python -u tools/bench_steps.py qp1_t8 qp qp1_t12 qp_t12 > gpurun_out/${tag}_bench.jsonl 2>&1
