#!/bin/bash
# PMC passes on the CRC64 rounds kernel (C5 / C1 via tools/crc_once.py) and the quorum kernel
# (C3); one counter group per pass, each pass its own process and time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null || exit 2
mkdir -p gpurun_out
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM"; do
  i=$((i+1))
  for cfg in ${CFGS:-C5 C3}; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc${i}_$cfg -o run --output-format csv -- python tools/crc_once.py $cfg 3 > gpurun_out/pmc${i}_$cfg.log 2>&1
    rc=$?; echo "pmc$i $cfg rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc${i}_$cfg.log; exit $rc; fi
  done
done
