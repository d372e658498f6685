#!/bin/bash
# Build libmvreg_hip.so variants with one source recompiled under extra flags (ablation experiments).
# usage: tools/build_variant.sh <source.hip> <name> <flags...>   -> tools/vsp/<name>.so
set -eu
R="$(cd "$(dirname "$0")/.." && pwd)"
SRC=$1; NAME=$2; shift 2
C="$R/3d_multiview_reg_amd/csrc"
mkdir -p "$R/tools/vsp/obj"
base=$(basename "$SRC" .hip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I"$R/include" -Wall -Wno-unused-function "$@" \
  -c "$C/$SRC" -o "$R/tools/vsp/obj/$NAME.o"
objs=$(ls "$C"/build/*.o | grep -v "/$base.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/tools/vsp/$NAME.so" $objs "$R/tools/vsp/obj/$NAME.o"
