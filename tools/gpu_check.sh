#!/bin/bash
# GPU session driver: each GPU step under its own time limit; stop at the first
# crash / abort / timeout (exit >= 124), continue past ordinary test failures (exit 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-"tests smoke bench"}
for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -v -x -p no:cacheprovider --timeout 240 --timeout-method thread --durations=15 ;;
    crc)   run crc_tests 600 python -m pytest tests/test_gpu_crc.py -q -x -p no:cacheprovider --timeout 300 ;;
    quorum) run quorum_tests 600 python -m pytest tests/test_gpu_quorum.py -q -x -p no:cacheprovider --timeout 300 ;;
    quick) run bench_quick 600 python bench.py --steps 20 --warmup 3 --no-cpu ;;
    legs)  run bench_legs 600 python bench.py --steps 20 --warmup 3 --no-cpu --legs ${BENCH_LEGS:-quorum,table,drive,C2} ;;
    smoke) run smoke 300 python __graft_entry__.py smoke ;;
    bench) run bench 600 python bench.py --steps 20 --warmup 3 --detail gpurun_out/bench_detail.json ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu ;;
    profd) run prof_drive 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/profd -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu --legs table,drive ;;
    tbl)   run table_tests 600 python -m pytest tests/test_gpu_table.py -q -x -p no:cacheprovider --timeout 300 ;;
    pmc)   # one rocprofv3 --pmc pass per (leg, counter): every kernel name then carries one workload
           for leg in ${PMC_LEGS:-quorum C2 C2L C3K C5 C1 table v2 snapshot lease readindex tick fanout ae}; do
             for c in FETCH_SIZE WRITE_SIZE; do
               run pmc_${leg}_$c 180 rocprofv3 --kernel-trace --pmc $c -d gpurun_out/pmc_${leg}_$c -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu --legs $leg
             done
           done ;;
    rdreq) # read-request sizes (exact read bytes = 32 n32 + 64 n64 + 128 n128), one pass per leg
           for leg in ${PMC_LEGS:-quorum C2 C2L C3K C5 C1 table v2 snapshot lease readindex tick fanout ae}; do
             run pmc_${leg}_RDREQ 180 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d gpurun_out/pmc_${leg}_RDREQ -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu --legs $leg
           done ;;
    host)  run host_test 300 ./tests/_build/host_test gpu ;;
    babl)  # the bench legs once per variant library (A/B of legs ab_inproc.py lacks)
           for v in ${AB_LIBS:-base}; do
             run bench_${TAG:-sel}_$v 600 env JRAFT_AMD_AB_LIB=ab/$v/libjrq.so python bench.py --steps 20 --warmup 5 --no-cpu --legs ${BENCH_LEGS:-table} --detail gpurun_out/bench_${TAG:-sel}_${v}_detail.json
           done ;;
    dab)   # the drive leg once per variant host build (ab/<v>/libjraft_drive.so + its libs), alternating
           i=0; for v in ${AB_LIBS:-base}; do i=$((i+1))
             run drive_${i}_$v 300 env JRAFT_AMD_AB_DRIVE=ab/$v/libjraft_drive.so python bench.py --steps 5 --warmup 2 --no-cpu --legs drive --detail gpurun_out/drive_${i}_${v}_detail.json
           done ;;
    hab)   # host-mirror builds round-robin, one process per run (tools/drive_ab.py), medians per
           # variant; AB_SPECS: the variant list itself (NAME=path[:VAR=VALUE] ...)
           run hab_${TAG:-sel} 900 python tools/drive_ab.py ${AB_SPECS:-$(for v in ${AB_LIBS:-hA}; do echo $v=ab/$v/libjraft_drive.so; done)} --flush-threads "${FLUSH_THREADS:-}" --rounds ${ROUNDS:-5} --epochs ${EPOCHS:-10} --threads ${THREADS:-16} --active ${ACTIVE:-1.0} ;;
    ab)    run ab_${TAG:-sel} 600 env AB_LEGS=${AB_LEGS:-C3,C5f,C1f,archive} python tools/ab_inproc.py ${AB_VARIANTS:-base=ab/base/libjrq.so} ;;
    tpab)  # the resident table epoch, every group committing, libjrq variants side by side
           for P in ${TP_PEERS:-5}; do
             run tpab_${TAG:-sel}_P$P 300 env P=$P FLAG_FRAC=${FLAG_FRAC:-0} python tools/table_peers_ab.py ${TP_VARIANTS:-base=ab/base/libjrq.so}
           done ;;
    fulltrace) # the default bench run under the tracer: the printed line, the full result and one
           # kernel trace of the same launches (tools/leg_traces.py --trace -> <tag>_leg_kernels.json)
           run fulltrace 900 rocprofv3 --kernel-trace --stats -d gpurun_out/full -o run --output-format csv -- python bench.py --detail gpurun_out/full_detail.json
           python tools/leg_traces.py --trace gpurun_out/full --detail gpurun_out/full_detail.json > gpurun_out/full_leg_kernels.json
           rm -f gpurun_out/full/run_kernel_trace.csv ;;
    legtrace) # one kernel trace per bench leg (tools/leg_traces.py -> profiles/<tag>_leg_kernels.json)
           for leg in ${TRACE_LEGS:-quorum table C2 C2L C3K C5 C1 ae v2 snapshot lease fanout}; do
             run legtrace_$leg 180 rocprofv3 --kernel-trace -d gpurun_out/legtrace_$leg -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu --legs $leg
           done ;;
    tsel)  run tests_${TAG:-sel} 900 python -u -m pytest ${TESTS:-tests/test_gpu_table.py} -x -q -p no:cacheprovider --timeout 240 --timeout-method thread ;;
    bsel)  run bench_${TAG:-sel} 600 python bench.py --steps 20 --warmup 5 --no-cpu --legs ${BENCH_LEGS:-quorum} --detail gpurun_out/bench_${TAG:-sel}_detail.json ;;
    sqpmc) run sqpmc_${TRACE_LEGS:-v2} 120 rocprofv3 --kernel-trace --pmc ${SQ_COUNTERS:-SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_BUSY_CYCLES} -d gpurun_out/sqpmc_${TRACE_LEGS:-v2} -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu --legs ${TRACE_LEGS:-v2} ;;
    trace) run trace_${TRACE_LEGS:-v2} 300 rocprofv3 --kernel-trace -d gpurun_out/trace_${TRACE_LEGS:-v2} -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu --legs ${TRACE_LEGS:-v2} ;;
    probe) run pin_probe 120 python tools/pin_cache_probe.py ;;
    drive) run drive_tests 300 python -u -m pytest tests/test_host_drive.py -v -x -p no:cacheprovider --timeout 240 --timeout-method thread ;;
  esac
done
