set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ctr
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $R/gpurun_out/ctr/list.txt 2>&1 || true
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/ctr/p$i -o c -- python3 $R/scripts/kbench.py $R/forging-control_amd/lib/libfcr.so --rounds 1 --batch 32768 > $R/gpurun_out/ctr/p$i.log 2>&1 || echo "pass $i failed"
done
echo done
