set -e
mkdir -p gpurun_out
for r in 1 2; do
for v in vp4 vp4r16; do
echo "== $v" >> gpurun_out/ab_rare.log
CCMPC_LIB=cc-mpc_amd/csrc/build_$v/libccmpc.so timeout -k 10 120 python -u tools/probe_step.py --reps 3 2>&1 | grep -A1 "^rares\|^cycle" >> gpurun_out/ab_rare.log
done
done
