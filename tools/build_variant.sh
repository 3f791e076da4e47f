#!/bin/bash
# Builds libctcext.so with extra compile flags into ab/lib<name>.so (same-box
# A/B variants; the in-tree build is untouched).  usage: tools/build_variant.sh name "-DX=1 ..."
set -e
R=$(cd $(dirname $0)/.. && pwd)
D=/tmp/ctcx_variant_$1
rm -rf $D && mkdir -p $D/csrc $D/ctcext_amd/lib $D/include
cp $R/ctc-beam-search-op_amd/csrc/*.hip $R/ctc-beam-search-op_amd/csrc/*.h $R/ctc-beam-search-op_amd/csrc/Makefile $D/csrc/
mkdir -p $D/../include 2>/dev/null || true
cp $R/include/ctcext.h $D/include/
sed -i "s#-falign-loops=32#-falign-loops=32 $2#" $D/csrc/Makefile
sed -i "s#../../include/ctcext.h#../include/ctcext.h#" $D/csrc/Makefile
sed -i 's#"../../include/ctcext.h"#"../include/ctcext.h"#' $D/csrc/ctcext_capi.hip
make -s -j10 -C $D/csrc OUT=../ctcext_amd/lib/libctcext.so 2>&1 | grep -E "error" || true
mkdir -p $R/ab
cp $D/ctcext_amd/lib/libctcext.so $R/ab/lib$1.so
echo "built ab/lib$1.so"
