#!/bin/bash
# tools/gpr.sh TIMEOUT 'COMMAND' - rebuild the in-tree library and examples
# (the GPU box runs what is in the tree, it does not build), then send
# COMMAND to the GPU box through gpurun.
set -e
cd "$(dirname "$0")/.."
make -s -C ix_amd/csrc 2>&1 | grep -v hip-link || true
exec /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
