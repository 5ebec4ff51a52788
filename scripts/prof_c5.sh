# config 5 (B = 65 536, N = 25, H = 256): kernel trace of one kbench round of the default build
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c5 -o c5 -- python3 $R/scripts/kbench.py $R/forging-control_amd/lib/libfcr.so --batch 65536 --horizon 25 --hidden 256 --rounds 1 > $R/gpurun_out/prof_c5.log 2>&1
