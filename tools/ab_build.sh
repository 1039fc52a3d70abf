#!/bin/bash
# A/B builds of libjrq for the GPU box (tools only): ab_build.sh NAME SRC.hip builds
# ab/libjrq_NAME.so with csrc/crc64.hip replaced by SRC.hip (the other objects from lib/obj);
# run a leg against it with JRQ_LIB=ab/libjrq_NAME.so.
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2
mkdir -p ab/obj_$name
cp sofa-jraft_amd/csrc/*.h ab/obj_$name/
cp "$src" ab/obj_$name/crc64.hip
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I include -c ab/obj_$name/crc64.hip -o ab/obj_$name/crc64.o
objs=$(ls sofa-jraft_amd/lib/obj/*.o | grep -v crc64.o)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ab/libjrq_$name.so ab/obj_$name/crc64.o $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf ab/obj_$name
