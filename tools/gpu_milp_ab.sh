# MILP on the GPU box: the MILP GPU tests, then tools/profile_milp_split.py with the root's
# children solved ahead (CCMPC_MILP_SPECULATE=1) and without, alternated
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-milp}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_milp.py > gpurun_out/${tag}_tests.log 2>&1
for r in 1 2; do
  for m in 0 1; do
    echo "== round $r speculate $m" >> gpurun_out/${tag}_split.log
    CCMPC_MILP_SPECULATE=$m timeout -k 10 200 python -u tools/profile_milp_split.py \
      >> gpurun_out/${tag}_split.log 2>&1
  done
done
