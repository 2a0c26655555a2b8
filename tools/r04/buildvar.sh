#!/bin/bash
# Build a variant libcapmi.so with extra compile flags into ab/<name>.so (kernel A/B builds; CAPMI_LIB=ab/<name>.so)
# usage: tools/r04/buildvar.sh <name> [-DFLAG=1 ...]
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
name=$1; shift
C=$R/image-captioning-with-different-decoders_amd/csrc
mkdir -p $R/ab/$name.d
make -s -C $C -j8 OBJDIR=$R/ab/$name.d OUTDIR=$R/ab/$name.d \
  CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -Wall -Wno-unused-result $*"
mv $R/ab/$name.d/libcapmi.so $R/ab/$name.so
rm -rf $R/ab/$name.d
echo "built ab/$name.so ($*)"
