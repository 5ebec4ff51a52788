# Round-5 measurement call: the wide hidden sizes under a kernel trace (no vendor-library kernel may appear), the
# config-5 line at the library's default keep budget, and the surrogate step at H = 256.
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/widetrace -o wide -- python3 -m pytest $R/tests/test_gpu_parity.py -m gpu -q -k "wide_path_hidden_sizes" -p no:cacheprovider > $O/widetrace.log 2>&1
tail -2 $O/widetrace.log
cd $R
timeout -k 10 600 python3 bench.py --horizon 25 --hidden 256 --steps 5 --warmup 2 --no-cpu-baseline > $O/c5_default.log 2>&1
tail -c 600 $O/c5_default.log
timeout -k 10 300 python3 scripts/bench_surrogate.py --hidden 256 --B 256 4096 65536 --steps 10 > $O/sur256.log 2>&1
cat $O/sur256.log
