# A/B of wide_gemm_cell_kernel mainloop variants (config 5), one process, interleaved; args: libs
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python scripts/kbench.py "$@" --hidden 256 --horizon 25 --rounds 3 > gpurun_out/kb_wg.log 2>&1
cat gpurun_out/kb_wg.log
