cd $GRAFT_REPO_ROOT
for v in default head dup dupwait; do
  if [ $v = default ]; then unset JRQ_LIB; else export JRQ_LIB=ab/libjrq_$v.so; fi
  timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu --legs C5,C1,v2 > gpurun_out/ab_$v.log 2>&1 || exit 1
done
