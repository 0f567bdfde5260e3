set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_qp_gi.py tests/test_gpu_mpc.py > gpurun_out/r6i_tests.log 2>&1
for ns in 2; do CCMPC_QP_GI_NOSTEP=$ns timeout -k 10 300 python -u tools/bench_steps.py qp qp1_t8 > gpurun_out/r6i_qp_ns$ns.log 2>&1; done
