#!/bin/bash
# A/B libraries under jylis_amd/_ab/ (git-ignored, shipped to the GPU box):
#   head           the committed tree (git archive HEAD)
#   NAME=-DFLAGS   the working tree built with extra defines
# usage: scripts/build_ab.sh head "rt1=-DJY_RT_SLICES=1" ...
set -eu
cd "$(dirname "$0")/.."
mkdir -p jylis_amd/_ab
for v in "$@"; do
  if [ "$v" = head ]; then
    rm -rf /tmp/jy_head && mkdir -p /tmp/jy_head
    git archive HEAD jylis_amd include | tar -x -C /tmp/jy_head
    make -s -j8 -C /tmp/jy_head/jylis_amd OUT=$PWD/jylis_amd/_ab/libjylis_head.so
  else
    name=${v%%=*}; flags=${v#*=}
    make -s -j8 -C jylis_amd BUILD=_ab/_b_$name OUT=_ab/libjylis_$name.so EXTRA="$flags"
  fi
done
ls -la jylis_amd/_ab/*.so
