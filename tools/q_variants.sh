#!/bin/bash
# A/B the quorum pair-kernel variants (JRQ_Q_VARIANT, quorum.hip) on C3 through bench.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for v in ${QV:-0 1 2 3 0}; do
  JRQ_Q_VARIANT=$v timeout -k 10 180 python bench.py --no-cpu --no-crc --steps 50 --warmup 5 > gpurun_out/qv_$v.json 2> gpurun_out/qv_$v.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/qv_$v.json')); r=d['roofline']; print('variant $v', round(d['ms_per_step']*1e3,2), 'us/step', round(r['kernel_ms']*1e3,2), 'us/kernel', round(r['achieved']), 'GB/s', 'lease', round(d['next_rows']['lease_check']['roofline']['achieved']))"
done
