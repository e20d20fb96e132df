#!/bin/bash
# build_variant.sh NAME SED_EXPR [EXTRA_HIPFLAGS]: experimental kernel build into variants/NAME/libgrt.so
set -e
NAME=$1; EXPR=$2; FLAGS=$3
ROOT=$(cd $(dirname $0)/.. && pwd)
W=/tmp/var/$NAME; rm -rf $W; mkdir -p $W; cp -r $ROOT/gr_raytracer_amd/csrc $W/csrc
sed -i "$EXPR" $W/csrc/device/geodesic.hip
mkdir -p $ROOT/variants/$NAME
make -s -j8 ALLOW_UNSTAMPED=1 -C $W/csrc INC=$ROOT/include OUT=$ROOT/variants/$NAME BUILD=$W/obj EXTRA_HIPFLAGS="$FLAGS" $ROOT/variants/$NAME/libgrt.so 2>&1 | grep -E "error" || true
ls -la $ROOT/variants/$NAME/libgrt.so
