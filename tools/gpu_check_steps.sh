# The whole GPU suite, then every drop-in step line (tools/bench_steps.py)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-chk}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
  > gpurun_out/${tag}_tests.log 2>&1
timeout -k 10 300 python -u tools/bench_steps.py dropin dropin_pp dropin_100k dropin_pred \
  dropin_pred_dev dropin_pred_100k_dev > gpurun_out/${tag}_steps.jsonl 2>&1
