# config-5 fused wide cell: stall/LDS counters, each pass its own run (kbench on the fused build)
set -e
R=$GRAFT_REPO_ROOT
L=$R/forging-control_amd/lib
cd /tmp && export TMPDIR=/tmp
i=0
for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pmc_wf$i -o p -- python3 $R/scripts/kbench.py $L/libfcr_wf.so --batch 65536 --horizon 25 --hidden 256 --rounds 1 > $R/gpurun_out/pmc_wf$i.log 2>&1
done
