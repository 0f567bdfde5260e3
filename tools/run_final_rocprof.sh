set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final_prof_csv -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu > gpurun_out/final_bench_rocprof_run.json 2> gpurun_out/final_rocprof.err
