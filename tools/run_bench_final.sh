set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u bench.py > gpurun_out/bench_r05b.json 2> gpurun_out/bench_r05b.err
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r05b_steps20.json 2> gpurun_out/bench_r05b_steps20.err
CCMPC_LIB=cc-mpc_amd/csrc/build_vtr/libccmpc.so timeout -k 10 120 python -u tools/qp_debug.py 101 h 60 > gpurun_out/qp_trace_setup.log 2>&1
CCMPC_LIB=cc-mpc_amd/csrc/build_vtr/libccmpc.so timeout -k 10 120 python -u tools/qp_debug.py 105 h 60 >> gpurun_out/qp_trace_setup.log 2>&1
