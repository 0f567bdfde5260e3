set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r6f_tests.log 2>&1
ONLY=step_c2,step_c1_100k,step_pred_c2,step_pred_dev_c2,step_pred_dev_100k timeout -k 10 600 bash profiles/collect_configs.sh r06 > gpurun_out/r6f_prof.log 2>&1
timeout -k 10 400 python -u tools/bench_steps.py dropin dropin_pp dropin_100k dropin_pred dropin_pred_dev dropin_pred_100k dropin_pred_100k_dev > gpurun_out/r6f_steps.log 2>&1
