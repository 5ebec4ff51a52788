"""Exhaustive check of the backward weight image layout (fcr_img.h: staggered rows, no swizzle).

Every read of the recomputed forward product (ds_read_b64 row reads) and of the transposed product
(ds_read_b64_tr_b16) must fetch the intended weights; each lane's address must be (its own base) +
(an instruction constant), so the constant is the ds offset and no address VALU is needed; and no
instruction may have an LDS bank conflict (64 banks x 4 B; b64 reads serviced as two 32-lane groups:
bank pair (a/8) mod 32, MI355X_MICROARCH.md §LDS). Mirrors img_row_start / img_unit / Img in fcr_img.h.

    python scripts/img_layout_check.py      # prints (HS, layer, units/row, tile units, conflicts)
"""


def geom(HS, layer):
    nsl = HS + 2 if layer == 0 else 2 * HS
    kb = (nsl + 7) // 8
    U = 32 if kb > 2 else 16                    # 8-B units per row
    tile = 536 if U == 32 else 268              # one slot's 16 staggered rows, in units
    return nsl, kb, U, tile


def row_start(m, U):
    """unit offset of row m (0..15) inside its slot's tile"""
    if U == 32:
        return 33 * m + (8 if m >= 8 else 0)
    k = m % 4 + 4 * (m // 8)                    # 16-unit rows in pairs (k, k+16 mod 32) of one 32-unit block
    return 33 * k + (4 if k >= 4 else 0) + 16 * ((m // 4) % 2)


def unit(kb, q, h0, U):
    return q * (U // 4) + 2 * kb + h0


def addr(R, sigma, grp, U, tile):
    """byte address (in the hi image) of weight (gate row R, combined slot sigma, lane group grp)"""
    slot, m = R >> 4, R & 15
    return 8 * (slot * tile + row_start(m, U) + unit(sigma >> 3, grp, (sigma & 7) >> 2, U)) + 2 * (sigma & 3)


def check(HS, layer):
    nsl, KB, U, tile = geom(HS, layer)
    rows = 16 * HS
    img = {}
    for R in range(rows):
        assert row_start(R & 15, U) + U <= tile
        for sigma in range(8 * KB):
            for grp in range(4):
                a = addr(R, sigma, grp, U, tile)
                assert a not in img, "overlap"
                img[a] = (R, sigma, grp)
    fconf = 0
    for r in range(HS):
        for kb in range(KB):
            for h0 in range(2):
                const = 8 * (r * tile + 2 * kb + h0)
                for half in range(2):
                    banks = []
                    for l in range(32 * half, 32 * half + 32):
                        m, q = l & 15, l >> 4
                        base = 8 * (row_start(m, U) + q * (U // 4))          # img_lane fb
                        a = base + const
                        for e in range(4):
                            assert img[a + 2 * e] == (16 * r + m, 8 * kb + 4 * h0 + e, q)
                        banks.append((a // 8) % 32)
                    fconf = max(fconf, 32 - len(set(banks)))
    tconf = 0
    NB, KBB = (nsl + 3) // 4, (HS + 1) // 2
    for tau in range(NB):
        for kbb in range(KBB):
            for jj in range(2):
                slot = 2 * kbb + jj
                if slot >= HS:
                    continue
                const = 8 * (slot * tile + 2 * (tau >> 1) + (tau & 1))
                fetched = {}
                for half in range(2):
                    banks = []
                    for l in range(32 * half, 32 * half + 32):
                        g, i = l >> 4, l & 15
                        mt, p = 4 * g + (i >> 2), i & 3
                        base = 8 * (row_start(mt, U) + p * (U // 4))        # img_lane tb
                        a = base + const
                        banks.append((a // 8) % 32)
                        fetched[l] = a
                    tconf = max(tconf, 32 - len(set(banks)))
                # transpose semantics: lane (g, i) element er = element (i&3) of source lane 16g+4er+(i>>2)
                for l in range(64):
                    g, i = l >> 4, l & 15
                    for er in range(4):
                        src = 16 * g + 4 * er + (i >> 2)
                        R, sigma, grp = img[fetched[src] + 2 * (i & 3)]
                        assert (R, sigma, grp) == (16 * slot + 4 * g + er, 4 * tau + (i & 3), i >> 2)
    return U, tile, fconf, tconf


if __name__ == "__main__":
    for HS in (4, 8, 13):
        for layer in (0, 1):
            U, tile, f, t = check(HS, layer)
            print(f"HS={HS:2d} layer={'0' if layer == 0 else '>=1'}: {U} units/row, tile {tile} units, "
                  f"row-read conflicts {f}, transposed-read conflicts {t}")
            assert f == 0 and t == 0
