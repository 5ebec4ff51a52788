# Build lib_ab/<name>.so from a git revision (default HEAD) for A/B timing against the working tree (scripts/kbench.py).
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}; NAME=${2:-old}
T=$(mktemp -d)
mkdir -p lib_ab
git archive $REV forging-control_amd/csrc include | tar -x -C $T
/opt/rocm/bin/hipcc -O3 -fno-slp-vectorize --offload-arch=gfx950 -std=c++17 -shared -fPIC -I $T/include \
  -I $T/forging-control_amd/csrc $T/forging-control_amd/csrc/fcr_abi.hip $T/forging-control_amd/csrc/fcr_rows.hip \
  -o lib_ab/$NAME.so
rm -rf $T
