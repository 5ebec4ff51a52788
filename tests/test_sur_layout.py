"""Exhaustive check of the surrogate weight-gradient kernel's LDS layouts (csrc/fcr_sur.h, sur_wgrad_kernel).

Mirrors sur_rowA / sur_rowB, the staging writes and the lane addresses of the transposed reads
(ds_read_b64_tr_b16: within each 16-lane group g, lane i's element er is element i & 3 of the 8-B unit
addressed by lane 16 g + 4 er + (i >> 2); scripts/img_layout_check.py uses the same model), and checks for
HS = 4, 8, 13 and both layer kinds that
  * no two staged values share LDS bytes and every row stays inside its region,
  * every A fragment lane holds dG[row k][R = 16 mt + (lane & 15)] for k = 32 kk + 8 g + j, and every B
    fragment lane holds in[row k][n = 16 nt + (lane & 15)] — the MFMA operand layouts,
  * no transposed read has an LDS bank conflict (64 banks x 4 B; b64 reads serviced per 32 lanes: bank pair
    (address / 8) mod 32, MI355X_MICROARCH.md).
"""
import pytest

KW, KC = 2, 2
KR = 16 * KW * KC
SA, SB = 544, 768


def rowA(k):
    return k * 544 + 128 * ((k >> 3) & 1) + 128 * (k >> 4)


def rowB(k):
    return k * 768 + 8 * ((k & 3) + 4 * ((k >> 3) & 1))


def geometry(HS, L0):
    KBB = (HS + 1) // 2
    RA = (2 * HS + 3) // 4
    NT = RA + 1 if L0 else 2 * RA
    a_bytes = rowA(KR - 1) + 32 * 2 * KBB
    a_pad = (a_bytes + 255) // 256 * 256
    return KBB, RA, NT, a_pad


def staged(HS, L0):
    """byte -> what the staging writes there (A hi image only; lo is the same layout A_PAD further)."""
    KBB, RA, NT, a_pad = geometry(HS, L0)
    A, B = {}, {}
    for k in range(KR):
        for kbb in range(KBB):
            for qq in range(4):
                for u in range(2):           # the two 8-B halves of a 16-B dgate piece: slots 2 kbb, 2 kbb + 1
                    for gate in range(4):
                        addr = rowA(k) + 32 * (2 * kbb + u) + 8 * qq + 2 * gate
                        R = 16 * (2 * kbb + u) + 4 * qq + gate
                        assert addr not in A
                        A[addr] = (k, R)
                        assert addr + 2 <= a_pad
    for k in range(KR):
        for rr in range(2):
            region = (256 if rr == 0 else 0) if L0 else 256 * rr
            for qq in range(4):
                if L0 and rr == 0:
                    halves = 4                # (hi x_q, lo x_q, hi x_4, lo x_4)
                else:
                    halves = 32               # 16 record words
                for h in range(halves):
                    addr = rowB(k) + region + 64 * qq + 2 * h
                    assert addr not in B
                    if L0 and rr == 0:
                        n = 16 * RA + 4 * qq + h
                    else:
                        rec = 0 if (L0 or rr == 0) else 1   # layer 0: the h record is the first one
                        n = 16 * (rec * RA + h // 4) + 4 * qq + (h % 4) if h // 4 < RA else None
                    B[addr] = (k, n)
                    assert addr + 2 <= KR * SB
    return A, B


@pytest.mark.parametrize("HS", [4, 8, 13])
@pytest.mark.parametrize("L0", [False, True])
def test_transposed_reads_fetch_the_operands_without_conflicts(HS, L0):
    KBB, RA, NT, a_pad = geometry(HS, L0)
    A, B = staged(HS, L0)
    for kk in range(KR // 32):
        oA, oB = rowA(32 * kk) - rowA(0), rowB(32 * kk) - rowB(0)
        hA, hB = rowA(4) - rowA(0), rowB(4) - rowB(0)
        for h in range(2):
            reads = [("A", mt, lambda L, mt=mt: rowA(8 * (L >> 4) + ((L >> 2) & 3)) + 8 * (L & 3) + oA + h * hA + 32 * mt)
                     for mt in range(HS)]
            for nt in range(NT):
                rg = 0 if nt < RA else 256
                aa = nt if nt < RA else nt - RA
                reads.append(("B", nt, lambda L, rg=rg, aa=aa: rowB(8 * (L >> 4) + ((L >> 2) & 3)) + 64 * (L & 3) + oB + h * hB
                              + rg + 8 * aa))
            for kind, tile, addr_of in reads:
                addr = [addr_of(L) for L in range(64)]
                for half in range(2):
                    banks = {(addr[L] // 8) % 32 for L in range(32 * half, 32 * half + 32)}
                    assert len(banks) == 32, (kind, tile, kk, h, half)
                for L in range(64):
                    g, i = L >> 4, L & 15
                    for er in range(4):
                        src = 16 * g + 4 * er + (i >> 2)
                        got = (A if kind == "A" else B).get(addr[src] + 2 * (i & 3))
                        k = 32 * kk + 8 * g + 4 * h + er
                        if kind == "A":
                            assert got == (k, 16 * tile + i), (tile, L, er, got)
                        else:
                            want = 16 * tile + i
                            assert got is not None and got[0] == k, (tile, L, er, got)
                            # a column past the record's 2 HS halves is padding (never decoded)
                            if got[1] is not None:
                                assert got[1] == want, (tile, L, er, got)
