# QP lines with the in-tree library and csrc/<variant>/libccmpc.so, alternating, on one box
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
v=$1; tag=${2:-qpab}
mkdir -p gpurun_out
for r in 1 2; do
  CCMPC_LIB=$GRAFT_REPO_ROOT/cc-mpc_amd/csrc/$v/libccmpc.so timeout -k 10 300 python -u tools/bench_steps.py qp1_t8 qp qp1_t12 qp_t12 > gpurun_out/${tag}_${v}_$r.jsonl 2>&1
  timeout -k 10 300 python -u tools/bench_steps.py qp1_t8 qp qp1_t12 qp_t12 > gpurun_out/${tag}_main_$r.jsonl 2>&1
done
