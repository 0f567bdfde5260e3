# r03 final measurement session (GPU box, repo root): full GPU suite, the default bench line,
# rocprofv3 --kernel-trace --stats of the same command, the per-configuration PMC profiles.
set -o pipefail
mkdir -p gpurun_out/s55
STEP_TIMEOUT=600 bash tools/gpu_session.sh s55 \
 "python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu" \
 "python -u bench.py > gpurun_out/s55/bench_default.json" \
 "cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/s55/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py > $GRAFT_REPO_ROOT/gpurun_out/s55/bench_rocprof_line.json" \
 "bash profiles/collect_configs.sh r03g"
