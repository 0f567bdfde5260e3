# The cycle's work-item geometry at T <= 8 (8-wave items in-tree, 4-wave items as
# csrc/build_nw2): cycle configs and the drop-in step lines alternated, then the whole GPU suite
# on the variant library (CCMPC_LIB)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ONLY=C2,C3-1e3,C3-2e4,C3-1e5 timeout -k 10 400 python3 -u tools/ab_configs.py main build_nw2 \
  main build_nw2 > gpurun_out/ab_item_waves.log 2>&1
for v in main nw2 main nw2; do
  lib=cc-mpc_amd/ccmpc/libccmpc.so
  [ $v = main ] || lib=cc-mpc_amd/csrc/build_$v/libccmpc.so
  echo "== $v" >> gpurun_out/ab_item_waves_steps.jsonl
  CCMPC_LIB=$lib timeout -k 10 200 python3 -u tools/bench_steps.py dropin dropin_100k \
    >> gpurun_out/ab_item_waves_steps.jsonl 2>&1
done
CCMPC_LIB=cc-mpc_amd/csrc/build_nw2/libccmpc.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests \
  > gpurun_out/ab_item_waves_tests.log 2>&1
CCMPC_LIB=cc-mpc_amd/csrc/build_nw2/libccmpc.so timeout -k 10 600 python -u bench.py \
  > gpurun_out/ab_item_waves_bench.json 2> gpurun_out/ab_item_waves_bench.err
CCMPC_LIB=cc-mpc_amd/csrc/build_nw2/libccmpc.so timeout -k 10 600 python -u bench.py --steps 20 \
  --warmup 5 > gpurun_out/ab_item_waves_bench20.json 2> gpurun_out/ab_item_waves_bench20.err
