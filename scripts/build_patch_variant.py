"""Build lib_ab/NAME.so from a copy of the sources with textual patches applied (bounding builds and A/B variants for
scripts/kbench.py; the product sources are never touched). usage:
    python scripts/build_patch_variant.py NAME PATCHES.json [extra hipcc flags...]
PATCHES.json: [[file relative to csrc, old text, new text], ...]; every old text must occur exactly once."""
import json
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
name, spec = sys.argv[1], sys.argv[2]
tmp = tempfile.mkdtemp()
src = os.path.join(tmp, "csrc")
shutil.copytree(os.path.join(ROOT, "forging-control_amd", "csrc"), src)
for f, old, new in json.load(open(spec)):
    p = os.path.join(src, f)
    s = open(p).read()
    assert s.count(old) == 1, (f, old[:80], s.count(old))
    open(p, "w").write(s.replace(old, new))
os.makedirs(os.path.join(ROOT, "lib_ab"), exist_ok=True)
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-fno-slp-vectorize", "--offload-arch=gfx950", "-std=c++17", "-shared", "-fPIC",
       "-I", os.path.join(ROOT, "include"), "-I", src, *sys.argv[3:], os.path.join(src, "fcr_abi.hip"),
       os.path.join(src, "fcr_rows.hip"), "-o", os.path.join(ROOT, "lib_ab", name + ".so")]
subprocess.check_call(cmd)
shutil.rmtree(tmp)
print("built lib_ab/%s.so" % name)
