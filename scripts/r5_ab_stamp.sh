set -e -o pipefail
bash scripts/r5_ab.sh $1 3
timeout -k 10 300 python scripts/stamp_wb.py lib_ab/wbstamp.so > gpurun_out/$1/stamp.log 2>&1
tail -8 gpurun_out/$1/stamp.log
