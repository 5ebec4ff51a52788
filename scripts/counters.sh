# SQ / LDS / HBM counters of the rollout kernels, one rocprofv3 pass per counter group (MI355X_MICROARCH.md: rocprofv3
# does not split groups over passes), each pass one kbench.py process.
#   usage: scripts/counters.sh OUTDIR LIB [kbench args...]     (on the GPU box; summary: scripts/ctr_summary.py OUTDIR)
#   e.g.   scripts/counters.sh gpurun_out/ctr_c3 forging-control_amd/lib/libfcr.so --batch 262144 --precision 1
#          scripts/counters.sh gpurun_out/ctr_c5 forging-control_amd/lib/libfcr.so --batch 65536 --horizon 2 \
#              --hidden 256 --keep-budget 272000000000
# PASS_SEL (env, optional): space-separated pass numbers to run (default: all)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$(realpath -m ${1:?outdir}); LIB=$(realpath ${2:?lib}); shift 2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
PASSES=("SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32"
        "SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_MFMA_F16 SQ_INSTS_VMEM"
        "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
        "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
        "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU"
        "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"
        "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL"
        "SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA"
        "FETCH_SIZE"
        "WRITE_SIZE")
SEL=${PASS_SEL:-$(seq 1 ${#PASSES[@]})}
for i in $SEL; do
  timeout -s KILL 240 rocprofv3 --pmc ${PASSES[$((i-1))]} --output-format csv -d $OUT/p$i -o c -- \
    python3 $R/scripts/kbench.py $LIB --rounds 1 "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo "counters done: $OUT"
