set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/micro
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/micro/lds -o m -- $R/scripts/micro/lds_conflict > $R/gpurun_out/micro/lds.log 2>&1
cat $R/gpurun_out/micro/lds.log
python3 - <<'PY'
import csv, os
R = os.environ["GRAFT_REPO_ROOT"]
for r in csv.DictReader(open(f"{R}/gpurun_out/micro/lds/m_counter_collection.csv")):
    print(r["Kernel_Name"][:40], r["Counter_Name"], r["Counter_Value"])
PY
