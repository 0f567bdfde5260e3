set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_probe.sh r6e_ho1 100000:1
CCMPC_SUPER_HANDOFF=0 bash tools/gpu_probe.sh r6e_ho0 100000:1
timeout -k 10 300 python -u tools/bench_steps.py dropin_100k > gpurun_out/r6e_steps_ho1.log 2>&1
CCMPC_SUPER_HANDOFF=0 timeout -k 10 300 python -u tools/bench_steps.py dropin_100k > gpurun_out/r6e_steps_ho0.log 2>&1
