#!/bin/bash
# Build the product library of a git revision (or the working tree, rev "WT")
# with extra -D switches into ntt-gpu-qtesla_amd/lib/ab/<name>.so, for the
# interleaved one-process A/B of tools/ab.py.
#   tools/build_ab.sh <name> <rev|WT> [extra hipcc flags...]
set -euo pipefail
name=$1 rev=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${AB_OUT:-$ROOT/ntt-gpu-qtesla_amd/lib/ab}
mkdir -p "$OUT"
if [ "$rev" = WT ]; then
    src=$ROOT
else
    src=$(mktemp -d)
    git -C "$ROOT" archive "$rev" ntt-gpu-qtesla_amd/csrc include | tar -x -C "$src"
fi
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall "$@" -shared -o "$OUT/$name.so" \
    "$src/ntt-gpu-qtesla_amd/csrc/ntt_kernels.hip" "$src/ntt-gpu-qtesla_amd/csrc/nussbaumer.hip" \
    "$src/ntt-gpu-qtesla_amd/csrc/host_stream.cpp"
[ "$rev" = WT ] || rm -rf "$src"
echo "$OUT/$name.so"
