#!/bin/bash
# A/B build of libclipk.so with extra compile flags for one source (default gemm.hip):
#   tools/build_variant.sh <tag> "<-Dflags>" [source.hip]
# -> build_ab/<tag>/libclipk.so (load it with CLIPK_LIB=...). Other objects from build/.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
PKG=$R/few-shot-prompt-learning-for-vision-language-models-in-imbalanced-datasets_amd
TAG=$1; FLAGS=$2; SRC=${3:-gemm.hip}
OUT=$R/build_ab/$TAG
mkdir -p $OUT
OBJ=$OUT/${SRC%.hip}.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $FLAGS -c $PKG/csrc/$SRC -o $OBJ
OTHERS=$(ls $PKG/build/*.o | grep -v "/${SRC%.hip}.o$")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $OUT/libclipk.so $OBJ $OTHERS
echo built $OUT/libclipk.so
