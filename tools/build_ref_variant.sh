#!/bin/bash
# build_ref_variant.sh NAME [GIT_REV=HEAD] (env EXTRA: extra hipcc flags): libgrt.so of a committed revision's csrc into
# variants/NAME (same-box A/B against the working tree's build, tools/time_variants.py)
set -e
NAME=$1; REV=${2:-HEAD}
ROOT=$(cd $(dirname $0)/.. && pwd)
W=/tmp/var/$NAME; rm -rf $W; mkdir -p $W
git -C $ROOT archive $REV gr_raytracer_amd/csrc include | tar -x -C $W
mkdir -p $ROOT/variants/$NAME
make -s -j8 ALLOW_UNSTAMPED=1 -C $W/gr_raytracer_amd/csrc INC=$W/include OUT=$ROOT/variants/$NAME BUILD=$W/obj EXTRA_HIPFLAGS="$EXTRA" \
  $ROOT/variants/$NAME/libgrt.so 2>&1 | grep -E "error" || true
ls -la $ROOT/variants/$NAME/libgrt.so
