#!/bin/bash
# Variant build of libmvreg_hip.so for same-box A/B runs: tools/vbuild.sh <name> "<extra hipcc flags>"
# -> tools/vsp/<name>.so (objects under tools/vsp/obj/<name>); load it with MVR_LIB=tools/vsp/<name>.so.
set -eu
R="$(cd "$(dirname "$0")/.." && pwd)"
NAME=$1; EXTRA=${2:-}
C="$R/3d_multiview_reg_amd/csrc"
O="$R/tools/vsp/obj/$NAME"
mkdir -p "$O"
HASH=$(cat $(ls "$C"/*.hip "$C"/*.hpp | sort) "$R/include/mvreg.h" | sha256sum | cut -c1-16)
HASH="$HASH+$(echo "$EXTRA" | sha256sum | cut -c1-6)"
for f in "$C"/*.hip; do
  b=$(basename "$f" .hip)
  x=""; [ "$b" = prof ] && x="-DMVR_SRC_HASH=\"$HASH\""; [ "$b" = feat_nn ] && x="-fno-slp-vectorize"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I"$R/include" -Wall -Wno-unused-function $x $EXTRA \
    -c "$f" -o "$O/$b.o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/tools/vsp/$NAME.so" "$O"/*.o
echo "built tools/vsp/$NAME.so ($HASH)"
