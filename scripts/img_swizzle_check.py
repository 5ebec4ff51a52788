import numpy as np, itertools
def f_swz(m, RB):
    b = lambda x, i: (x >> i) & 1
    if RB == 256:   # bits: m0->b0, m1->b3, m2->b4, m3->b2
        return b(m,0) | (b(m,1) << 3) | (b(m,2) << 4) | (b(m,3) << 2)
    else:           # RB == 128: m1->b0, m2->b3, m3->b2 (m0 via row parity)
        return b(m,1) | (b(m,2) << 3) | (b(m,3) << 2)
def phys_unit(R, w, RB):
    return w ^ f_swz(R & 15, RB)
def byte_addr(R, w, e, RB):
    return R * RB + 8 * phys_unit(R, w, RB) + 2 * e
def bankpair(addr):   # b64-granular bank pair within the 64 banks
    return (addr // 8) % 32

def check(HS, layer):
    NSL = HS + 2 if layer == 0 else 2 * HS
    KB = (NSL + 7) // 8
    RB = max(128, 64 * KB)
    U = RB // 8
    NB = (NSL + 3) // 4
    KBB = (HS + 1) // 2
    rows = 16 * HS
    # logical matrix A_log[R][col] with unique values (R,col) -> id
    img = {}
    for R in range(rows):
        for col in range(U * 4):
            w, e = col // 4, col % 4
            a = byte_addr(R, w, e, RB)
            assert a not in img
            img[a] = (R, col)
    assert max(img) < rows * RB
    # forward reads: tile r, block kb, lane l: 2 b64 reads (units 2c, 2c+1), c = 4kb+q
    conf = 0
    for r in range(HS):
        for kb in range(KB):
            for h0 in range(2):
                for half in range(2):
                    bp = []
                    for l in range(32 * half, 32 * half + 32):
                        m, q = l & 15, l >> 4
                        R = 16 * r + m
                        w = 2 * (4 * kb + q) + h0
                        a = byte_addr(R, w, 0, RB)
                        for e in range(4):
                            got = img[a + 2 * e]
                            exp_col = kb * 32 + q * 8 + 4 * h0 + e
                            assert got == (R, exp_col), (got, R, exp_col)
                        bp.append(bankpair(a))
                    conf = max(conf, 32 - len(set(bp)))
    fconf = conf
    # backward transposed reads: tile tau, block kbb, jj; lane 4q'+p of group g supplies row q', chunk p
    conf = 0
    for tau in range(NB):
        for kbb in range(KBB):
            for jj in range(2):
                slot = 2 * kbb + jj
                if slot >= HS:
                    continue
                for half in range(2):
                    bp = []
                    for l in range(32 * half, 32 * half + 32):
                        g, i = l >> 4, l & 15
                        qq, p = i >> 2, i & 3
                        R = 16 * slot + 4 * g + qq
                        w = 8 * (tau >> 1) + 2 * p + (tau & 1)
                        a = byte_addr(R, w, 0, RB)
                        bp.append(bankpair(a))
                        # data: lane i of the group receives column i of the 4 rows: element qq' = row qq'
                    conf = max(conf, 32 - len(set(bp)))
                    # verify semantic: lane (g, i) element e_row gets A'[m'=i][k'=8g+4jj+e_row]
                    for l in range(32 * half, 32 * half + 32):
                        g, i = l >> 4, l & 15
                        for er in range(4):
                            src_lane = 16 * g + 4 * er + (i >> 2)
                            sg, si = src_lane >> 4, src_lane & 15
                            R = 16 * slot + 4 * sg + (si >> 2)
                            w = 8 * (tau >> 1) + 2 * (si & 3) + (tau & 1)
                            a = byte_addr(R, w, i & 3, RB)
                            Rg, col = img[a]
                            # intended: row = unit 4*slot+g gate er ; col = combined slot sigma=4tau+(i&3), grp i>>2
                            sigma = 4 * tau + (i & 3)
                            exp_col = (sigma >> 3) * 32 + (i >> 2) * 8 + (sigma & 7)
                            assert Rg == 16 * slot + 4 * g + er and col == exp_col, (Rg, col)
    return RB, fconf, conf
for HS in (4, 8, 13):
    for layer in (0, 1):
        print(HS, layer, check(HS, layer))
