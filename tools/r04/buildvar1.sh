#!/bin/bash
# Variant library with ONE source file recompiled under extra flags, linked against the tree's other objects
# (build/obj from `make`): ab/<name>.so. usage: tools/r04/buildvar1.sh <name> <file.hip> [-DFLAG=1 ...]
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
name=$1; src=$2; shift 2
C=$R/image-captioning-with-different-decoders_amd/csrc
O=$R/build/obj
mkdir -p $R/ab/$name.d
obj=$R/ab/$name.d/${src%.hip}.o
(cd $C && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -Wall -Wno-unused-result "$@" -c $src -o $obj)
others=$(ls $O/*.o | grep -v "/${src%.hip}.o$")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $R/ab/$name.so $others $obj
rm -rf $R/ab/$name.d
echo "built ab/$name.so ($src $*)"
