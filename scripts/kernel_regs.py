"""Per-kernel register / scratch / LDS budget from a device assembly file (scripts/isa_dump.sh output):
    python scripts/kernel_regs.py FILE.s [name substring ...]
next_free_vgpr (VGPR+AGPR allocation request), scratch bytes per lane (private_segment_fixed_size: > 0 = spills),
static LDS, and the waves per SIMD the register allocation allows (MI355X_MICROARCH.md §Register files)."""
import re
import sys

path, keys = sys.argv[1], sys.argv[2:]
cur, rows = None, []
for line in open(path):
    m = re.match(r"\s*\.amdhsa_kernel (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        continue
    if cur is None:
        continue
    m = re.match(r"\s*\.amdhsa_(next_free_vgpr|private_segment_fixed_size|group_segment_fixed_size|accum_offset|"
                 r"next_free_sgpr) (\d+)", line)
    if m:
        cur[m.group(1)] = int(m.group(2))
    if re.match(r"\s*\.end_amdhsa_kernel", line):
        rows.append(cur)
        cur = None
for r in rows:
    if keys and not any(k in r["name"] for k in keys):
        continue
    v = r.get("next_free_vgpr", 0)
    alloc = (v + 7) // 8 * 8
    waves = min(8, 512 // alloc) if alloc else 8
    print(f"{r['name'][:70]:70s} vgpr {v:3d} (agpr from {r.get('accum_offset', 0):3d}) scratch {r.get('private_segment_fixed_size', 0):4d} "
          f"lds {r.get('group_segment_fixed_size', 0):6d} waves/SIMD {waves}")
