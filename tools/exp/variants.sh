#!/bin/bash
# Build experiment variants of libsift_mi.so (compile-time -D switches) into
# tools/exp/v_<name>/, e.g.
#   bash tools/exp/variants.sh noscan=-DSIFT_EXP_ORIENT_NOSCAN noexp=-DSIFT_EXP_ORIENT_NOEXP
# then time one with: SIFT_MI_LIB=tools/exp/v_noscan/libsift_mi.so python bench.py ...
cd "$(dirname "$0")/../.." || exit 2
for spec in "$@"; do
  name=${spec%%=*}; defs=${spec#*=}
  make -s -C sift-features_amd/csrc -j8 OUT="$PWD/tools/exp/v_$name/libsift_mi.so" OBJ="$PWD/tools/exp/v_$name/build" EXTRA="$defs" || exit 1
done
