#!/bin/bash
# Device assembly of the library's two translation units, for ISA-identity checks of source-only
# refactors: scripts/isa_dump.sh OUTDIR [extra hipcc flags]; then diff two OUTDIRs (isa_diff below).
# Comments and the compiler's ident/version lines are stripped so only instructions and metadata remain.
set -euo pipefail
out=${1:?outdir}; shift
root=$(cd "$(dirname "$0")/.." && pwd)
src=$root/forging-control_amd/csrc
mkdir -p "$out"
for f in fcr_abi fcr_rows; do
  /opt/rocm/bin/hipcc -O3 -fno-slp-vectorize --offload-arch=gfx950 -std=c++17 --cuda-device-only -S \
    -I "$root/include" -I "$src" "$@" "$src/$f.hip" -o "$out/$f.s"
  grep -v -E '^\s*(;|//)|\.ident|^\s*$|__hip_cuid_' "$out/$f.s" | sed -e 's/\s*;.*$//' -e 's/\.LBB[0-9]*_/.LBB_/g' -e 's/post_getpc[0-9]*/post_getpc/g' > "$out/$f.clean.s"
done
