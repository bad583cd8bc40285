set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 400 python -u tools/tools_mx_parity.py > gpurun_out/r03/mx_parity.log 2>&1
echo "parity rc=$?"
