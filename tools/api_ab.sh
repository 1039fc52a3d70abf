#!/bin/bash
# Alternating A/B of the host mirror's per-call cost on the GPU box (CPU only): the tree's
# jraft_host.cpp against a variant directory (tools/api_probe.py --host-src), N rounds each,
# one log line per run.  usage: tools/api_ab.sh VARIANT_DIR [ROUNDS] [THREADS]
cd "$(dirname "$0")/.."
var=$1; n=${2:-5}; th=${3:-1,16}
python tools/api_probe.py --threads 1 --epochs 2 --no-build > /dev/null 2>&1 || true
for i in $(seq $n); do
  timeout -k 10 200 python tools/api_probe.py --threads $th --epochs 4 --host-src $var/jraft_host.cpp | sed 's/^/variant /' || exit 1
  timeout -k 10 200 python tools/api_probe.py --threads $th --epochs 4 | sed 's/^/tree /' || exit 1
done
