set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mpc.py tests/test_gpu_qp_gi.py tests/test_gpu_lds_poison.py tests/test_gpu_milp.py > gpurun_out/t_qp.log 2>&1
CCMPC_LIB=cc-mpc_amd/csrc/build_vtr/libccmpc.so timeout -k 10 120 python -u tools/qp_debug.py 101 h 60 > gpurun_out/qp_trace_setup.log 2>&1
timeout -k 10 200 python -u tools/ab_qp.py method > gpurun_out/ab_qp.log 2>&1
timeout -k 10 200 python -u tools/time_frame.py > gpurun_out/time_frame.log 2>&1
