set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_qp_gi.py tests/test_gpu_mpc.py tests/test_gpu_milp.py tests/test_gpu_lds_poison.py > gpurun_out/t_split.log 2>&1
for r in 1 2; do
for m in 0 1; do
echo "== split $m" >> gpurun_out/ab_split.log
CCMPC_QP_GI_SPLIT=$m CCMPC_QP_METHOD=gi timeout -k 10 200 python -u tools/ab_qp.py child 2>&1 | grep -v amdgpu >> gpurun_out/ab_split.log
CCMPC_QP_GI_SPLIT=$m timeout -k 10 200 python -u tools/profile_milp.py 2>&1 | grep " ms " | head -8 | awk '{print $1}' | tr '\n' ' ' >> gpurun_out/ab_split.log
echo >> gpurun_out/ab_split.log
done
done
