#!/bin/bash
# Build the engine of git revision $1 into artes_amd/lib/libartes_hip_$2.so (A/B timing; development tool).
set -e
REV=$1; TAG=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" artes_amd/csrc include | tar -x -C "$TMP"
# the Makefile's flags (artes_amd/csrc/Makefile)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -munsafe-fp-atomics -w \
    -mllvm -disable-machine-licm -mllvm -amdgpu-sched-strategy=max-ilp \
    -o "$ROOT/artes_amd/lib/libartes_hip_$TAG.so" "$TMP/artes_amd/csrc/transport.hip"
rm -rf "$TMP"
echo "built artes_amd/lib/libartes_hip_$TAG.so from $REV"
