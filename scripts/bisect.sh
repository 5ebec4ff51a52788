set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=forging-control_amd/lib
timeout -k 10 300 python scripts/kbench.py $L/libfcr_f32.so $L/libfcr.so $L/libfcr_bisB.so $L/libfcr_bisC.so $L/libfcr_bisD.so $L/libfcr_bisBCD.so --batch 2048 --rounds 1 > gpurun_out/bisect.log 2>&1
grep lib gpurun_out/bisect.log
