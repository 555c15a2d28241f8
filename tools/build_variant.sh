#!/bin/bash
# A/B build of libclipk.so with extra compile flags for some sources (default gemm.hip):
#   tools/build_variant.sh <tag> "<-Dflags>" [source.hip ...]
# -> build_ab/<tag>/libclipk.so (load it with CLIPK_LIB=...). Other objects from build/.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
PKG=$R/few-shot-prompt-learning-for-vision-language-models-in-imbalanced-datasets_amd
TAG=$1; FLAGS=$2; shift 2
SRCS=${@:-gemm.hip}
OUT=$R/build_ab/$TAG
mkdir -p $OUT
OBJS=""
SKIP=""
for SRC in $SRCS; do
  OBJ=$OUT/${SRC%.hip}.o
  EXTRA=""
  case $SRC in attention*.hip) EXTRA="-mllvm -amdgpu-mfma-vgpr-form=1";; esac
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $EXTRA $FLAGS -c $PKG/csrc/$SRC -o $OBJ
  OBJS="$OBJS $OBJ"
  SKIP="$SKIP|/${SRC%.hip}.o$"
done
OTHERS=$(ls $PKG/build/*.o | grep -Ev "${SKIP:1}")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $OUT/libclipk.so $OBJS $OTHERS
echo built $OUT/libclipk.so
