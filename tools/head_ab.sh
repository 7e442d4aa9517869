#!/bin/bash
# A/B of the octave-0 head kernels (tools/ubench_kernels head): the default
# build, the packed-row-pass build (ubench_kernels_pk) and a strip workgroup
# target sweep.  Run via gpurun.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
N=${1:-64}
for b in ubench_kernels ubench_kernels_pk; do
  [ -x tools/$b ] || continue
  echo "== $b"
  timeout -k 10 120 ./tools/$b head $N || exit $?
done
for wg in 3072 4096 8192 12288; do
  echo "== SIFT_MI_STRIP_WG=$wg"
  SIFT_MI_STRIP_WG=$wg timeout -k 10 120 ./tools/ubench_kernels head $N | grep round || exit $?
done
