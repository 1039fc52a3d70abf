# round 6: the sharded batch (N engines in one process) -- GPU tests, then the drive leg
set -e
export TESTS="tests/test_host_drive.py tests/test_host_cpp.py tests/test_jni.py -m gpu"
STEPS="tsel" TAG=shard bash tools/gpu_check.sh
STEPS="legs" BENCH_LEGS="drive" bash tools/gpu_check.sh
