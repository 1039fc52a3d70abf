#!/bin/bash
# Build an A/B variant of libjrq.so into ab/<name>/libjrq.so (tools/ab_inproc.py loads several
# side by side).  usage: tools/ab_build.sh NAME "EXTRA HIPCC FLAGS" [crc64.hip override]
set -e
cd "$(dirname "$0")/.."
name=$1; flags=$2; crc=${3:-sofa-jraft_amd/csrc/crc64.hip}
out=ab/$name; mkdir -p $out
srcs="sofa-jraft_amd/csrc/quorum.hip sofa-jraft_amd/csrc/table.hip sofa-jraft_amd/csrc/append_entries.hip sofa-jraft_amd/csrc/commit_fanout.hip sofa-jraft_amd/csrc/v2_decode.hip sofa-jraft_amd/csrc/engine.hip"
objs=""
for s in $crc $srcs; do
  o=$out/$(basename $s .hip).o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Isofa-jraft_amd/csrc $flags -c $s -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $out/libjrq.so $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built $out/libjrq.so"
