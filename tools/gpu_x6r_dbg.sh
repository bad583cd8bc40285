set -o pipefail
for d in 0 1 2 3 4; do echo "== DBG $d"; DBG=$d STAMPS=1 timeout -k 10 60 python tools/gemm_one.py 19200 256 256 8 3 2>/dev/null | grep "wave [04]" || exit 1; done
