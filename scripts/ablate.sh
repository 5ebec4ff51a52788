# Diagnostic: build the ablation variants (results are garbage by design) into lib/ for kbench timing.
#   FCR_ABLATE=1: fragment reads and operand splits stay, MFMAs go; FCR_ABLATE=2: cell pointwise goes;
#   FCR_ABLATE=3: no sequence-slab traffic (h/c/dx loads become opaque registers, stores go).
set -e
cd "$(dirname "$0")/.."
SRC=forging-control_amd/csrc
for v in ${VARIANTS:-1 2 3}; do
  /opt/rocm/bin/hipcc -O3 -fno-slp-vectorize --offload-arch=gfx950 -std=c++17 -shared -fPIC -DFCR_ABLATE=$v \
    -I include -I $SRC $SRC/fcr_abi.hip $SRC/fcr_rows.hip -o forging-control_amd/lib/libfcr_abl$v.so -lrocblas
done
