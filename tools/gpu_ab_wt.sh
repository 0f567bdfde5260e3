# A/B of write-through particle stores (gpurun_probe/libccmpc_wt.so, _p4wt.so) on the GPU box
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=$GRAFT_REPO_ROOT/gpurun_probe
mkdir -p gpurun_out
CCMPC_LIB=$P/libccmpc_wt.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sample_bucket.py tests/test_gpu_load_predictions.py > gpurun_out/wt_tests.log 2>&1
for lib in p4 p4wt; do
  CCMPC_LIB=$P/libccmpc_$lib.so timeout -k 10 200 python -u tools/probe_step.py --N 100000 --O 1 --reps 3 > gpurun_out/wt_probe_${lib}_100k.log 2>&1
  CCMPC_LIB=$P/libccmpc_$lib.so timeout -k 10 200 python -u tools/probe_step.py --N 5000 --O 4 --reps 3 > gpurun_out/wt_probe_${lib}_c2.log 2>&1
done
for r in 1 2; do
  timeout -k 10 300 python -u tools/bench_steps.py dropin dropin_100k > gpurun_out/wt_steps_base_$r.jsonl 2>&1
  CCMPC_LIB=$P/libccmpc_wt.so timeout -k 10 300 python -u tools/bench_steps.py dropin dropin_100k > gpurun_out/wt_steps_wt_$r.jsonl 2>&1
done
