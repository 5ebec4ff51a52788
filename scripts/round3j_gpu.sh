set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3j
mkdir -p $O
cd $R
for v in wm4 wm2; do
  timeout -k 10 300 python scripts/wb_check.py lib_ab/wbtest_$v.so > $O/wb_$v.log 2>&1; echo $v; grep -E "B=65536|bounds|leftover" $O/wb_$v.log
done
