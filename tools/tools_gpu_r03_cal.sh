set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "lstm" -m gpu > gpurun_out/r03/lstm_tests2.log 2>&1
rc=$?; echo "op tests rc=$rc"; [ $rc -le 1 ] || exit $rc
NPROB=1,2,3,4,6,8,10 FORCE_BS=0,4,8 GROUPS=8 timeout -k 10 400 python -u tools/tools_lstm_groups.py > gpurun_out/r03/lstm_cal2.log 2>&1
