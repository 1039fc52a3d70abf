#!/bin/bash
# A/B legs on the GPU box (tools only): AB_VARIANTS="a b" AB_LEGS=C5,C1,v2 bash tools/ab_run.sh
# runs bench.py --legs $AB_LEGS once per ab/libjrq_<variant>.so (built by tools/ab_build.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
i=0
for v in ${AB_VARIANTS:-cur}; do
  i=$((i + 1))
  JRQ_LIB=ab/libjrq_$v.so timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu \
    --legs ${AB_LEGS:-C5,C1,v2} > gpurun_out/ab_${i}_$v.log 2>&1 || exit 1
done
