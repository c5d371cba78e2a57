#!/bin/bash
# Build an experimental copy of liboctvr_hip.so with extra -D flags: scripts/build_variant.sh NAME -DX=Y ...
# Output: opencv-octvr_amd/lib/variants/NAME.so (select it with OCTVR_HIP_LIB=...).
# SRC=<repo checkout> builds that checkout's sources instead (e.g. a git worktree of an older commit).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
B=/tmp/octvr_variant_$NAME; mkdir -p $B "$ROOT/opencv-octvr_amd/lib/variants"
SRC=${SRC:-$ROOT}
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I$SRC/include -I$SRC/opencv-octvr_amd/csrc $*"
OBJS=
for f in octvr_hip.cpp async.cpp fastmapper.cpp seams.cpp tiling.cpp multiband_host.cpp masks.cpp morph.cpp kernels.hip multiband.hip fastmapper.hip; do
  o=$B/${f%.*}_${f##*.}.o
  X=; [[ $f == *.hip ]] && X="-x hip"
  /opt/rocm/bin/hipcc $FLAGS $X -c "$SRC/opencv-octvr_amd/csrc/$f" -o $o &
  OBJS="$OBJS $o"
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$ROOT/opencv-octvr_amd/lib/variants/$NAME.so" $OBJS -lpthread -lz
