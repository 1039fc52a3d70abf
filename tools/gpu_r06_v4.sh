# round 6: the v4 table epoch -- GPU tests of the table path, then A/B against the v3 build
set -e
export TESTS="tests/test_gpu_table.py tests/test_gpu_c1.py tests/test_jni.py tests/test_host_drive.py tests/test_host_cpp.py -m gpu"
export TP_VARIANTS="v3=ab/v3/libjrq.so il7=ab/il7/libjrq.so v4=sofa-jraft_amd/lib/libjrq.so"
STEPS="tsel" TAG=v4 bash tools/gpu_check.sh
STEPS="tpab" TAG=f0 FLAG_FRAC=0 TP_PEERS="5" bash tools/gpu_check.sh
STEPS="tpab" TAG=f1 FLAG_FRAC=0.01 TP_PEERS="5 3 9" bash tools/gpu_check.sh
STEPS="tpab" TAG=f10 FLAG_FRAC=0.1 TP_PEERS="5" bash tools/gpu_check.sh
