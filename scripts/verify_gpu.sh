# GPU: full parity suite, smoke(), the default bench line and (with PROF=1) its rocprofv3 kernel stats
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/verify
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/verify/pytest.log 2>&1 || { tail -40 gpurun_out/verify/pytest.log; exit 1; }
tail -3 gpurun_out/verify/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/verify/smoke.log 2>&1 || { tail -20 gpurun_out/verify/smoke.log; exit 1; }
tail -1 gpurun_out/verify/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/verify/bench.log 2>&1 || { tail -20 gpurun_out/verify/bench.log; exit 1; }
tail -1 gpurun_out/verify/bench.log
if [ "${PROF:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/verify/prof -o v -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/verify/prof.log 2>&1
  echo prof done
fi
