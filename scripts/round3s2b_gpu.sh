# A/B: forward fragment reads issued ahead of the region's MFMAs (FCR_FWD_RDFIRST=1) against the base build
set -o pipefail
O=gpurun_out/r3s2b
mkdir -p $O
timeout -k 10 500 python -u scripts/kbench.py lib_ab/base.so lib_ab/rdf.so --rounds 3 --sustain 30 > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
grep lib $O/kbench.log
