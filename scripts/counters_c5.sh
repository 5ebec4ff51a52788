# SQ / LDS counters of config 5's two cell kernels, one rocprofv3 pass per counter group (kbench, B = 65 536, H = 256,
# N = 2, every window kept); summary: python scripts/ctr_summary.py gpurun_out/ctr5 wide
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ctr5
cd /tmp && export TMPDIR=/tmp
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL" "SQ_INSTS_VMEM SQ_INSTS_VALU_MFMA_F16 SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_WRITE_REQ_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/ctr5/p$i -o c -- python3 $R/scripts/kbench.py $R/forging-control_amd/lib/libfcr.so --rounds 1 --batch 65536 --horizon 2 --hidden 256 --keep-budget 272000000000 > $R/gpurun_out/ctr5/p$i.log 2>&1 || echo "pass $i failed"
done
echo done
