# rocprofv3 kernel stats of the C2 step graph's replays with the split L4 (0) and the
# one-workgroup L4 (8192)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for m in 0 8192; do
  CCMPC_L4_ONE_WG_MAX=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/l4wg_prof_$m -o run -- python3 tools/step_replay.py step_c2 200 \
    > gpurun_out/l4wg_prof_$m.log 2>&1
done
