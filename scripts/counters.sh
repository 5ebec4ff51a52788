# SQ / LDS counters of the rollout kernels, one rocprofv3 pass per counter group (kbench at B=32768)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ctr
cd /tmp && export TMPDIR=/tmp
i=0
for C in "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32" "SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_MFMA_F16 SQ_INSTS_VMEM" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/ctr/p$i -o c -- python3 $R/scripts/kbench.py $R/forging-control_amd/lib/libfcr.so --rounds 1 --batch 32768 > $R/gpurun_out/ctr/p$i.log 2>&1 || echo "pass $i failed"
done
echo done
