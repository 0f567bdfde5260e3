#!/bin/bash
# Build an alternative libccmpc.so with extra compile flags (every source: the knobs live in
# shared headers) -> cc-mpc_amd/csrc/build_NAME/libccmpc.so, for tools/ab_configs.py:
#   tools/build_variant.sh d3 "-DCCMPC_DEPTH=3"
set -euo pipefail
cd "$(dirname "$0")/../cc-mpc_amd/csrc"
make -s -j8 OBJDIR="build_$1" OUT="build_$1/libccmpc.so" EXTRA="${2:-}" >/dev/null
echo "built build_$1/libccmpc.so (${2:-})"
