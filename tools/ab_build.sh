#!/bin/bash
# Build an A/B variant of libjrq.so into ab/<name>/libjrq.so (tools/ab_inproc.py loads several
# side by side).  usage: [SRC=dir/with/csrc] tools/ab_build.sh NAME "EXTRA HIPCC FLAGS" [crc64.hip override]
# (SRC: another tree's sofa-jraft_amd/csrc, e.g. an earlier commit's sources extracted under ab/)
set -e
cd "$(dirname "$0")/.."
name=$1; flags=$2; src=${SRC:-sofa-jraft_amd/csrc}; crc=${3:-$src/crc64.hip}
out=ab/$name; mkdir -p $out
srcs="$src/quorum.hip $src/table.hip $src/append_entries.hip $src/commit_fanout.hip $src/v2_decode.hip $src/engine.hip"
objs=""
for s in $crc $srcs; do
  o=$out/$(basename $s .hip).o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$src $flags -c $s -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $out/libjrq.so $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built $out/libjrq.so"
