#!/bin/bash
# Build libmvreg_hip.so variants with one source recompiled under extra flags (ablation experiments).
# usage: tools/build_variant.sh <source.hip> <name> <flags...>   -> tools/vsp/<name>.so
# The variant's mvr_source_hash is the base build's hash + the variant's name and flags.
set -eu
R="$(cd "$(dirname "$0")/.." && pwd)"
SRC=$1; NAME=$2; shift 2
C="$R/3d_multiview_reg_amd/csrc"
mkdir -p "$R/tools/vsp/obj"
make -s -C "$C" >/dev/null
base=$(basename "$SRC" .hip)
HASH=$(cd "$C" && cat $(ls *.hip *.hpp | sort) ../../include/mvreg.h | sha256sum | cut -c1-16)
FL="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$R/include -Wall -Wno-unused-function"
$FL "$@" -c "$C/$SRC" -o "$R/tools/vsp/obj/$NAME.o"
$FL -DMVR_SRC_HASH="\"$HASH+$NAME:$*\"" -c "$C/prof.hip" -o "$R/tools/vsp/obj/${NAME}_prof.o"
objs=$(ls "$C"/build/*.o | grep -v "/$base.o" | grep -v "/prof.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/tools/vsp/$NAME.so" $objs "$R/tools/vsp/obj/$NAME.o" \
  "$R/tools/vsp/obj/${NAME}_prof.o"
