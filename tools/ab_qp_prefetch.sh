set -e
mkdir -p gpurun_out
for v in vtr vtr0; do
echo "== $v" >> gpurun_out/ab_pf.log
CCMPC_LIB=cc-mpc_amd/csrc/build_$v/libccmpc.so timeout -k 10 120 python -u tools/qp_debug.py 101 h 60 2>&1 | grep -v amdgpu | head -4 >> gpurun_out/ab_pf.log
done
for r in 1 2; do
for v in default vpf0; do
echo "== frame $v" >> gpurun_out/ab_pf.log
if [ $v = default ]; then L=cc-mpc_amd/ccmpc/libccmpc.so; else L=cc-mpc_amd/csrc/build_$v/libccmpc.so; fi
CCMPC_LIB=$L timeout -k 10 200 python -u tools/frame_split.py 2>&1 | grep "qp wait\|total" >> gpurun_out/ab_pf.log
done
done
