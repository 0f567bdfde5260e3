# Generic step A/B on the GPU box: the step GPU tests (unless SKIP_TESTS=1), then
# tools/bench_steps.py lines under each value of an environment switch, alternated over rounds.
#   bash tools/gpu_ab_env.sh TAG VAR "V1 V2" [ROUNDS] [LINES...]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; var=$2; vals=$3; rounds=${4:-2}; shift 4 || shift $#
lines=${*:-dropin dropin_pp dropin_100k dropin_pred_dev}
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest -x -q --timeout 120 \
  --timeout-method thread -m gpu tests/test_gpu_step.py tests/test_gpu_step_modes.py \
  tests/test_gpu_episode.py tests/test_gpu_harness.py > gpurun_out/${tag}_tests.log 2>&1
for r in $(seq $rounds); do
  for m in $vals; do
    echo "== round $r $var $m" >> gpurun_out/${tag}_steps.jsonl
    env $var=$m timeout -k 10 300 python -u tools/bench_steps.py $lines \
      >> gpurun_out/${tag}_steps.jsonl 2>&1
  done
done
