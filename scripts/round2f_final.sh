# Round 2f final: A/B of the row-gradient reduction, GPU suite, config-5 bench line + kernel statistics,
# then the wide-path parity tests on the DPP variant
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2g
mkdir -p $O
timeout -k 10 300 python $R/scripts/kbench.py $R/lib_ab/lb4.so $R/lib_ab/dpp.so --hidden 256 --horizon 25 --rounds 3 > $O/kb_dpp.log 2>&1
cat $O/kb_dpp.log
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
tail -1 $O/gputest.log
timeout -k 10 300 python $R/bench.py --hidden 256 --horizon 25 --batch 65536 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c5.log 2>&1
tail -c 200 $O/bench_c5.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5trace -o c5 -- python3 $R/bench.py --hidden 256 --horizon 25 --batch 65536 --steps 2 --warmup 1 --no-cpu-baseline --grad-check off > $O/c5trace.log 2>&1
echo trace ok
cd $R && cp lib_ab/dpp.so forging-control_amd/lib/libfcr.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "wide or config5" -x -q --timeout 200 --timeout-method thread > $O/wide_dpp.log 2>&1
tail -1 $O/wide_dpp.log
