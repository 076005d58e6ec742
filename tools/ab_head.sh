#!/bin/bash
# Builds rnnlogic_amd/_build/variants/head.so from the last commit's ground.hip /
# graph.cpp / internal.h (the working tree's other objects), for A/B runs.
set -e
REPO=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p $T/x/csrc $T/include $REPO/rnnlogic_amd/_build/variants
cp $REPO/include/rnnlogic_hip.h $T/include/
for f in ground.hip internal.h graph.cpp; do git -C $REPO show HEAD:rnnlogic_amd/csrc/$f > $T/x/csrc/$f; done
cd $T/x/csrc
B="--offload-arch=gfx950 -O3 -fPIC -std=c++17"
hipcc $B -c ground.hip -o g.o
hipcc $B -c graph.cpp -o gr.o
O=$REPO/rnnlogic_amd/_build
hipcc --offload-arch=gfx950 -shared -fPIC gr.o g.o $O/rotate.hip.o $O/encode.hip.o $O/batch.hip.o $O/mine.hip.o -o $O/variants/head.so
rm -rf $T
echo $O/variants/head.so
