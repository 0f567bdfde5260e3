set -e
mkdir -p gpurun_out
for r in 1 2; do
for v in default vgi; do
if [ $v = default ]; then L=cc-mpc_amd/ccmpc/libccmpc.so; else L=cc-mpc_amd/csrc/build_$v/libccmpc.so; fi
echo "== $v" >> gpurun_out/ab_gionly.log
CCMPC_LIB=$L CCMPC_QP_METHOD=gi timeout -k 10 200 python -u tools/ab_qp.py child 2>&1 | grep -v amdgpu >> gpurun_out/ab_gionly.log
CCMPC_LIB=$L timeout -k 10 200 python -u tools/frame_split.py 2>&1 | grep "qp wait\|total" >> gpurun_out/ab_gionly.log
done
done
