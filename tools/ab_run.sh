#!/bin/bash
# A/B legs on the GPU box (tools only): AB_VARIANTS="a b:ENV=1" AB_LEGS=C5,C1,v2 bash tools/ab_run.sh
# runs bench.py --legs $AB_LEGS once per variant: library ab/libjrq_<name>.so (built by
# tools/ab_build.sh; "lib" = the in-tree one) and optional VAR=value environment settings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
i=0
for spec in ${AB_VARIANTS:-lib}; do
  i=$((i + 1))
  name=${spec%%:*}
  envs=""
  [ "$spec" != "$name" ] && envs=$(echo "${spec#*:}" | tr ',' ' ')
  lib=ab/libjrq_$name.so
  [ "$name" = lib ] && lib=sofa-jraft_amd/lib/libjrq.so
  env JRQ_LIB=$lib $envs timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu \
    --legs ${AB_LEGS:-C5,C1,v2} > gpurun_out/ab_${i}_$name.log 2>&1 || exit 1
done
