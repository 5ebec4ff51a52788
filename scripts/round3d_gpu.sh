# Round 3d: A/B of loop unrolling (forward t loop x3; backward t loops x2) against HEAD's kernels
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3d
mkdir -p $O
cd $R
timeout -k 10 400 python scripts/kbench.py lib_ab/fwdrcp.so lib_ab/unroll_f.so lib_ab/unroll_fb.so --rounds 5 --sustain 20 > $O/kb.log 2>&1
cat $O/kb.log
