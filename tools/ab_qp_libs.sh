#!/bin/bash
# A/B of library builds on the planning QP (GPU box, repo root): one child per build and round,
#   bash tools/ab_qp_libs.sh main build_e3 build_e4 ...      ("main" = the in-tree library)
for rnd in 1 2; do
  for b in "$@"; do
    if [ "$b" = main ]; then lib=cc-mpc_amd/ccmpc/libccmpc.so; else lib=cc-mpc_amd/csrc/$b/libccmpc.so; fi
    echo -n "$b "
    CCMPC_LIB=$lib CCMPC_QP_WAVES=1 timeout -k 10 120 python -u tools/ab_qp.py child 2>/dev/null || exit $?
  done
done
