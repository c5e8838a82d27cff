#!/bin/bash
# Build libixgrx.so from git revision REV into tools/ablib/NAME.so (for
# same-process A/B timing against the working tree: tools/ab_lib.py).
# usage: tools/build_rev.sh REV NAME
set -e
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$ROOT/build/rev_$NAME
rm -rf "$T" && mkdir -p "$T" "$ROOT/tools/ablib"
git -C "$ROOT" archive "$REV" ix_amd/csrc include examples | tar -x -C "$T"
make -s -C "$T/ix_amd/csrc" OUT="$ROOT/tools/ablib/$NAME.so" OBJ="$T/obj" 2>&1 | grep -v hip-link || true
ls -la "$ROOT/tools/ablib/$NAME.so"
