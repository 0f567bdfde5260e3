set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mpc.py tests/test_gpu_qp_gi.py tests/test_gpu_episode.py tests/test_gpu_harness.py tests/test_gpu_milp.py > gpurun_out/t_qp.log 2>&1
for r in 1 2; do
CCMPC_QP_FUSED_LTV=0 timeout -k 10 200 python -u tools/time_frame.py > gpurun_out/time_frame_unfused_$r.log 2>&1
CCMPC_QP_FUSED_LTV=1 timeout -k 10 200 python -u tools/time_frame.py > gpurun_out/time_frame_fused_$r.log 2>&1
done
