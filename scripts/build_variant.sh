#!/bin/bash
# Build an alternative libccamd.so for same-box A/B measurements (bench.py / tests pick it up through
# CCAMD_LIB=build/var/NAME/libccamd.so).  usage: scripts/build_variant.sh NAME [GIT_REV|-] [HIPCC FLAGS...]
# GIT_REV '-' (default): the working tree's engine source.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; REV=${2:--}; shift; [ $# -gt 0 ] && shift
OUT=$ROOT/build/var/$NAME
mkdir -p "$OUT"
if [ "$REV" = "-" ]; then cp "$ROOT/consensuscruncher_amd/csrc/cc_engine.hip" "$ROOT/build/var/cc_engine_$NAME.hip"
else git -C "$ROOT" show "$REV:consensuscruncher_amd/csrc/cc_engine.hip" > "$ROOT/build/var/cc_engine_$NAME.hip"; fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" -o "$OUT/libccamd.so" \
    "$ROOT/build/var/cc_engine_$NAME.hip" -ldl
echo "$OUT/libccamd.so"
