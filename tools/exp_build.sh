#!/bin/bash
# Experimental build of libsr_hip.so: conv3x3.hip (or $SRC) recompiled with extra flags, linked with
# the other objects of the current build -> abl/lib<tag>.so (A/B only; never the shipped library).
# usage: bash tools/exp_build.sh <tag> "<flags>"
set -e
cd "$(dirname "$0")/../basicsr4rs_amd/csrc"
TAG=$1; FLAGS=$2; SRC=${SRC:-conv3x3}
mkdir -p /tmp/exp ../../abl
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $FLAGS -c $SRC.hip -o /tmp/exp/${SRC}_$TAG.o
OBJS=$(ls ../lib/obj/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../abl/lib$TAG.so $OBJS /tmp/exp/${SRC}_$TAG.o
echo "abl/lib$TAG.so"
