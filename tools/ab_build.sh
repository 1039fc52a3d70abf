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
# jrq_build_id(): the variant's own sources' hash (as the Makefile does for the product library)
sha=$(python3 sofa-jraft_amd/jraft_amd/_srcsha.py $src)
printf 'static const char id[] = "JRQ_BUILD_ID=%s";\nconst char *jrq_build_id(void) { return id + 13; }\n' $sha > $out/build_id.c
gcc -O2 -fPIC -c $out/build_id.c -o $out/build_id.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $out/libjrq.so $objs $out/build_id.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built $out/libjrq.so"
