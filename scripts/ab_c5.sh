# Config-5 A/B of two builds in ONE process (scripts/kbench.py; B 65 536, N 25, H 256): every window kept, then the
# library's default keep budget. usage: scripts/ab_c5.sh OUTDIR LIB_A LIB_B [rounds]
set -e -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$1; A=$2; B=$3; RND=${4:-3}
mkdir -p $OUT
cd $R
timeout -k 10 400 python scripts/kbench.py $A $B --batch 65536 --horizon 25 --hidden 256 --rounds $RND \
  --keep-budget 272000000000 > $OUT/ab_c5_keepall.log 2>&1
tail -6 $OUT/ab_c5_keepall.log
timeout -k 10 400 python scripts/kbench.py $A $B --batch 65536 --horizon 25 --hidden 256 --rounds $RND \
  > $OUT/ab_c5_default.log 2>&1
tail -6 $OUT/ab_c5_default.log
