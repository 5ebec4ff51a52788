# Build lib_ab/NAME.so from the working tree with extra compiler flags (A/B timing with scripts/kbench.py).
# usage: scripts/build_variant.sh NAME [extra hipcc flags...]
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p lib_ab
/opt/rocm/bin/hipcc -O3 -fno-slp-vectorize --offload-arch=gfx950 -std=c++17 -shared -fPIC -I include \
  -I forging-control_amd/csrc "$@" forging-control_amd/csrc/fcr_abi.hip forging-control_amd/csrc/fcr_rows.hip \
  -o lib_ab/$NAME.so
