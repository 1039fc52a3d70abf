#!/bin/bash
# CRC64 rounds-kernel timelines for a few launch shapes (tools/crc_timeline.hip).
# TL_BINS selects builds: crc_timeline (production), crc_timeline_nosetup / _notail
# (diagnostic builds with -DJRQ_DIAG_NO_SETUP / -DJRQ_DIAG_NO_TAIL; results not bit-exact).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for b in ${TL_BINS:-crc_timeline}; do
  for g in ${TL_SHAPES:-"256,0,0" "256,0,1" "256,4352,0" "240,0,1" "128,0,1"}; do
    echo "## $b $g"
    timeout -k 10 60 ./tools/$b ${g//,/ } || exit $?
  done
done > gpurun_out/timeline.log 2>&1
cat gpurun_out/timeline.log
