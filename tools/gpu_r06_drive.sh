# round 6: order-free ack records -- GPU tests of the table / host path, then the drive leg
set -e
export TESTS="tests/test_gpu_table_acks.py tests/test_gpu_table.py tests/test_host_drive.py tests/test_host_cpp.py tests/test_jni.py -m gpu"
STEPS="tsel" TAG=acks bash tools/gpu_check.sh
STEPS="legs" BENCH_LEGS="table,drive" bash tools/gpu_check.sh
STEPS="probe" bash tools/gpu_check.sh
