#!/bin/bash
# Build an A/B variant of the product library with extra -D flags:
#   bash tools/build_variant.sh NAME "-DGLFSX_SCHED=1 ..."
# -> glfs_amd/libglfsx_NAME.so (load it with GLFSX_LIB=...; A/B runs only)
set -e
NAME=$1; DEFS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=/tmp/glfsx_var_$NAME
rm -rf $D && mkdir -p $D/glfs_amd && cp -r $ROOT/glfs_amd/csrc $D/glfs_amd/ && cp -r $ROOT/include $D/
rm -f $D/glfs_amd/csrc/*.o
make -s -C $D/glfs_amd/csrc HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $DEFS"
cp $D/glfs_amd/libglfsx.so $ROOT/glfs_amd/libglfsx_$NAME.so
echo "built glfs_amd/libglfsx_$NAME.so ($DEFS)"
