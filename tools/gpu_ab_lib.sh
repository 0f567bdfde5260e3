# A/B of the in-tree library against csrc/<variant>/libccmpc.so on the GPU box: the cycle
# configs (tools/ab_configs.py, twice, alternating) and the headline bench line (no CPU leg, no
# sweep, no C4), twice each.  Args: variant name, tag.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
v=$1; tag=${2:-ab}
mkdir -p gpurun_out
ONLY=C2,C3-1e3,C3-1e5,C4/8,C5 timeout -k 10 500 python -u tools/ab_configs.py main $v main $v > gpurun_out/${tag}_configs.log 2>&1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-sweep --no-c4 > gpurun_out/${tag}_bench_main_$r.json 2> gpurun_out/${tag}_bench_main_$r.err
  CCMPC_LIB=$GRAFT_REPO_ROOT/cc-mpc_amd/csrc/$v/libccmpc.so timeout -k 10 300 python -u bench.py --no-cpu --no-sweep --no-c4 > gpurun_out/${tag}_bench_${v}_$r.json 2> gpurun_out/${tag}_bench_${v}_$r.err
done
