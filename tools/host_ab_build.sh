#!/bin/bash
# Build an A/B variant of the host mirror + drive into ab/<name>/ (libjraft_host.so,
# libjraft_drive.so and a copy of the tree's libjrq.so, found through $ORIGIN), for
# tools/gpu_check.sh `dab` / `hab`.  usage: [HOST_SRC=file] tools/host_ab_build.sh NAME "EXTRA G++ FLAGS"
# (HOST_SRC: another jraft_host.cpp, e.g. an earlier commit's; it includes the tree's jraft_host.h)
set -e
cd "$(dirname "$0")/.."
name=$1; flags=$2; out=ab/$name; mkdir -p $out
src=${HOST_SRC:-sofa-jraft_amd/host/jraft_host.cpp}
cp sofa-jraft_amd/lib/libjrq.so $out/
g++ -O2 -std=c++17 -fPIC -fno-semantic-interposition -Wall -Wextra $flags -shared -o $out/libjraft_host.so \
  -Isofa-jraft_amd/host $src -L$out -ljrq -lpthread -Wl,-rpath,'$ORIGIN'
g++ -O2 -std=c++17 -fPIC -fno-semantic-interposition -Wall -Wextra $flags -shared -o $out/libjraft_drive.so \
  sofa-jraft_amd/host/jraft_drive.cpp -Isofa-jraft_amd/host -L$out -ljraft_host -ljrq -Wl,-rpath,'$ORIGIN'
echo "built $out"
