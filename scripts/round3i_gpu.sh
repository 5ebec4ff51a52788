set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3i
mkdir -p $O
cd $R
WSD0=28688128 timeout -k 10 300 python scripts/ws_diff.py lib_ab/wbl1.so lib_ab/wbl6.so > $O/wsdiff.log 2>&1; tail -60 $O/wsdiff.log
