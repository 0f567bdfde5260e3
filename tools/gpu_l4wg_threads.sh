# The one-workgroup L4 (ccmpc_l4) at 512 / 1024 threads per workgroup: phase timelines
# (tools/probe_l4.py, PROBE=4 builds in gpurun_probe/) and rocprofv3 kernel stats of the C2 step
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in 512 1024; do
  CCMPC_LIB=gpurun_probe/libccmpc_w$v.so timeout -k 10 120 python3 -u tools/probe_l4.py \
    > gpurun_out/l4wg_w${v}_probe.log 2>&1
  CCMPC_L4_ONE_WG_MAX=8192 CCMPC_LIB=gpurun_probe/libccmpc_w$v.so timeout -k 10 120 \
    rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/l4wg_w$v -o run \
    -- python3 tools/step_replay.py step_c2 200 > gpurun_out/l4wg_w${v}_prof.log 2>&1
done
