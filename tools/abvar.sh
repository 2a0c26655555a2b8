#!/bin/bash
# Build a variant libcapmi.so with extra compile flags into ab/<name>.so (kernel A/B and diagnostic builds,
# loaded with CAPMI_LIB=ab/<name>.so). usage: [ONLY="gemm_x3p gemm_x3"] tools/abvar.sh <name> [-DFLAG=1 ...]
# ONLY: recompile just these sources with the flags and link them with the in-tree objects (build/obj).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
C=$R/image-captioning-with-different-decoders_amd/csrc
D=$R/ab/$name.d
rm -rf $D && mkdir -p $D
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -Wall -Wno-unused-result $*"
if [ -n "$ONLY" ]; then
  make -s -C $C -j8 >/dev/null  # the in-tree objects are current
  cp $R/build/obj/*.o $D/
  for f in $ONLY; do rm -f $D/$f.o; done
  touch $D/*.o
fi
make -s -C $C -j8 OBJDIR=$D OUTDIR=$D CXXFLAGS="$FLAGS"
mv $D/libcapmi.so $R/ab/$name.so
rm -rf $D
echo "built ab/$name.so ($*${ONLY:+; only $ONLY})"
