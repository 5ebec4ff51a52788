set -e -o pipefail
bash scripts/r5_ab.sh actz 3
mkdir -p gpurun_out/actu
timeout -k 10 400 python scripts/kbench.py lib_ab/prod.so lib_ab/actu.so --batch 65536 --horizon 25 --hidden 256 --rounds 2 --keep-budget 272000000000 > gpurun_out/actu/ab_c5_keepall.log 2>&1
tail -3 gpurun_out/actu/ab_c5_keepall.log
