set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "wide or config5" -x -q --timeout 200 --timeout-method thread > gpurun_out/wide_tests.log 2>&1
tail -2 gpurun_out/wide_tests.log
timeout -k 10 300 python scripts/kbench.py lib_ab/t1.so lib_ab/t4.so lib_ab/t8.so --hidden 256 --horizon 25 --rounds 3 > gpurun_out/kb_rowg.log 2>&1
cat gpurun_out/kb_rowg.log
timeout -k 10 300 python bench.py --gpus 2 --share-gpu --steps 5 --warmup 2 --no-cpu-baseline --grad-check off > gpurun_out/rehearse2.log 2>&1
tail -c 600 gpurun_out/rehearse2.log
