# config-5 fused wide cell: A/B against the default (rocBLAS + cell kernel) and a kernel-stats profile of it
set -e
R=$GRAFT_REPO_ROOT
L=$R/forging-control_amd/lib
timeout -k 10 300 python3 $R/scripts/kbench.py $L/libfcr_rb.so $L/libfcr.so --batch 65536 --horizon 25 --hidden 256 --rounds 2 > $R/gpurun_out/kb_wf.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_wf -o wf -- python3 $R/scripts/kbench.py $L/libfcr.so --batch 65536 --horizon 25 --hidden 256 --rounds 1 > $R/gpurun_out/prof_wf.log 2>&1
