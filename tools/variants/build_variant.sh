#!/bin/bash
# Build a library variant on the host: the in-tree objects with ONE source
# recompiled under extra defines, linked to tools/variants/lib_<tag>.so
# (same header revision, so RNVP_LIB_PATH accepts it):
#   bash tools/variants/build_variant.sh TAG SOURCE.hip "-DNAME=VALUE ..."
set -e
TAG=$1; SRC=$2; DEFS=$3
C=$(cd $(dirname $0)/../../dl-normalizing-flows_amd/csrc && pwd)
V=$(cd $(dirname $0) && pwd)
make -C $C -s
W=$(mktemp -d); cp $C/build/*.o $W/
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -I$C/../../include -I$C -Wall -Wno-unused-function \
  -Wno-unused-variable $DEFS -c $C/$SRC -o $W/${SRC%.hip}.o
TL=$(python3 -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
g++ -shared -o $V/lib_$TAG.so $W/*.o -L$TL -lamdhip64 -Wl,-rpath,$TL -Wl,--no-undefined
rm -rf $W
echo built $V/lib_$TAG.so
