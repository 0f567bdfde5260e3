set -o pipefail
mkdir -p gpurun_out/s46
STEP_TIMEOUT=300 bash tools/gpu_session.sh s46 \
 "python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu" \
 "python -u bench.py > gpurun_out/s46/bench_default.json" \
 "cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/s46/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py > $GRAFT_REPO_ROOT/gpurun_out/s46/bench_rocprof_line.json" \
 "python -u tools/time_step_split.py"
