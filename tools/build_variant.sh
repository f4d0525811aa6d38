#!/bin/bash
# Build an N2-only dev library variant from a copy of csrc/ with some headers replaced:
#   tools/build_variant.sh TAG "DEVFLAGS" [file.h=/path/to/replacement.h ...]
# -> aiqmc/libaiqmc_hip_TAG.so (AIQMC_LIB_VARIANT=TAG); for interleaved A/B (tools/ab_variants.sh).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd
TAG=$1; FLAGS=$2; shift 2
W=/tmp/aq_variant_$TAG
rm -rf $W; mkdir -p $W/pkg/csrc $W/include
cp $PKG/csrc/*.h $PKG/csrc/*.hip $PKG/csrc/Makefile $W/pkg/csrc/
cp $ROOT/include/*.h $W/include/
for r in "$@"; do cp "${r#*=}" "$W/pkg/csrc/${r%%=*}"; done
make -C $W/pkg/csrc dev DEVTAG=$TAG DEVFLAGS="$FLAGS" OUTDIR=$PKG/aiqmc -j4 > $W/build.log 2>&1 || { tail -20 $W/build.log; exit 1; }
echo "built $PKG/aiqmc/libaiqmc_hip_$TAG.so"
