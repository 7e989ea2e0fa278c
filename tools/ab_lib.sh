#!/bin/bash
# Builds a variant of libmfa_amd.so in which ONE kernel source is taken from a git revision:
#   bash tools/ab_lib.sh <rev> <csrc file name> <tag>  ->  tools/ablib/libmfa_<tag>.so
# (the other objects are the current build's).  Load it with MFA_LIB=... for process-level A/B.
set -euo pipefail
REV=$1; SRC=$2; TAG=$3
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/metal-flash-attention-plus_amd
TMP=$(mktemp -d)
git -C "$ROOT" show "$REV:metal-flash-attention-plus_amd/csrc/$SRC" > "$TMP/$SRC"
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-slp-vectorize -w -I$PKG/csrc"
case $SRC in attention_fwd_v2.hip|attention_fwd_stream.hip|attention_fwd_pipe.hip|attention_fwd_kv8.hip|attention_bwd_fast.hip)
  FLAGS="$FLAGS -mllvm -amdgpu-mfma-vgpr-form";; esac
/opt/rocm/bin/hipcc $FLAGS -c "$TMP/$SRC" -o "$TMP/variant.o"
OBJS=$(ls "$PKG"/build/*.o | grep -v "/${SRC%.hip}.o$")
mkdir -p "$ROOT/tools/ablib"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/tools/ablib/libmfa_$TAG.so" $OBJS "$TMP/variant.o"
rm -rf "$TMP"
echo "tools/ablib/libmfa_$TAG.so"
