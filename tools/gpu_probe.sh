# PROBE=4 phase timelines of the planning step (tools/probe_step.py) with the probe build copied
# to gpurun_probe/ (build_p* does not travel); args: tag, then "N:O" pairs
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
for s in "$@"; do
  N=${s%%:*}; O=${s##*:}
  CCMPC_LIB=$GRAFT_REPO_ROOT/gpurun_probe/libccmpc_p4.so timeout -k 10 200 python -u tools/probe_step.py --N $N --O $O --reps 3 > gpurun_out/${tag}_N${N}_O${O}.log 2>&1
done
