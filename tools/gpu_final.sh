# Round-end check on the GPU box (repo root): the GPU tests, smoke(), the default bench and the
# driver's 20-step bench, then a rocprofv3 --stats pass over the bench.  Optional tag argument:
# output files gpurun_out/final<tag>_*.
set -e
T=${1:-}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/final${T}_gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final${T}_smoke.log 2>&1
timeout -k 10 600 python -u bench.py > gpurun_out/final${T}_bench.json 2> gpurun_out/final${T}_bench.err
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/final${T}_bench_steps20.json 2> gpurun_out/final${T}_bench_steps20.err
if [ -n "${ROCPROF:-}" ]; then
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final${T}_prof -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu > gpurun_out/final${T}_bench_rocprof_run.json 2> gpurun_out/final${T}_rocprof.err
fi
