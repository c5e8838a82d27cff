#!/bin/bash
# Build the working tree's library with a python-regex edit applied to the
# kernel source, into tools/ablib/NAME.so (same-process A/B: tools/ab_lib.py).
# usage: tools/build_variant.sh NAME 'python expression on s (the source text)'
# (VFILE=ixgrx_tx.hip etc. to edit another source of ix_amd/csrc)
set -e
NAME=$1; EXPR=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$ROOT/build/var_$NAME
rm -rf "$T" && mkdir -p "$T/ix_amd" "$ROOT/tools/ablib"
cp -r "$ROOT/ix_amd/csrc" "$T/ix_amd/" && cp -r "$ROOT/include" "$T/"
python3 - "$T/ix_amd/csrc/${VFILE:-ixgrx_kernels.hip}" "$EXPR" <<'PY'
import re, sys
p, expr = sys.argv[1], sys.argv[2]
s = open(p).read()
t = eval(expr, {"re": re, "s": s})
assert t != s, "variant edit changed nothing"
open(p, "w").write(t)
PY
make -s -C "$T/ix_amd/csrc" OUT="$ROOT/tools/ablib/$NAME.so" OBJ="$T/obj" 2>&1 | grep -v hip-link || true
ls -la "$ROOT/tools/ablib/$NAME.so"
