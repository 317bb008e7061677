"""CPU: brute-force checks of the GEMM kernels' LDS image layouts (csrc/gemm.hip).

Each check restates the kernel's address formulas (rc_sw / rc_off, crh_src / crh_lane / frag_crh)
and verifies, for every lane:
  - consistency: the bytes a fragment read takes are the logical operand elements the MFMA
    fragment wants, given where the global_load_lds staging put them (1 KiB per wave
    instruction, lane l -> bytes [16 l, 16 l + 16) of the piece);
  - bank-conflict freedom under MI355X_MICROARCH.md's LDS model: bank = (byte / 4) mod 64,
    ds_read_b128 served in four 16-lane groups, ds_read_b64_tr_b16 in two 32-lane groups;
    a group is conflict-free when its lanes' dwords fall on distinct banks.
"""
import itertools

import pytest

B128_GROUPS = [
    [*range(0, 4), *range(12, 16), *range(20, 28)],
    [*range(4, 12), *range(16, 20), *range(28, 32)],
    [*range(32, 36), *range(44, 48), *range(52, 60)],
    [*range(36, 44), *range(48, 52), *range(60, 64)],
]
B64_GROUPS = [list(range(0, 32)), list(range(32, 64))]


def _conflict_free(addr_of_lane, groups, nbytes):
    for grp in groups:
        banks = []
        for lane in grp:
            a = addr_of_lane(lane)
            assert a % nbytes == 0
            banks += [(a // 4 + d) % 64 for d in range(nbytes // 4)]
        if len(set(banks)) != len(banks):
            return False
    return True


# ---------------------------------------------------------------- RC images (row = i, 16-B chunks of r)

def rc_sw(bk, row):
    return ((row & 1) | ((row >> 1) & 2)) if bk == 32 else ((row >> 1) & 7)


def rc_off(bk, row, c):
    return row * bk * 2 + ((c ^ rc_sw(bk, row)) << 4)


@pytest.mark.parametrize("bk", [32, 64])
def test_rc_fragment_reads_conflict_free_and_consistent(bk):
    # staging (gemm_tile lane_offsets, RC): piece t, lane l -> image row t*RPI + l/CPR, logical chunk
    # (l % CPR) ^ rc_sw(row), written at 16 l of the piece
    cpr, rpi = bk // 8, 64 // (bk // 8)
    where = {}
    for t in range(256 * bk * 2 // 1024):
        for lane in range(64):
            row = t * rpi + lane // cpr
            c = (lane % cpr) ^ rc_sw(bk, row)
            where[(row, c)] = t * 1024 + 16 * lane
    for row, c in where:
        assert where[(row, c)] == rc_off(bk, row, c)  # the read formula finds what staging wrote
    for s, kk in itertools.product(range(16), range(bk // 32)):
        # fragment s (rows 16 s .. 16 s + 15), k-substep kk: lane reads row 16 s + (l & 15), chunk 4 kk + (l >> 4)
        f = lambda lane: rc_off(bk, s * 16 + (lane & 15), kk * 4 + (lane >> 4))
        assert _conflict_free(f, B128_GROUPS, 16)


# ---------------------------------------------------------------- half-blocked CR images

def crh_src(rows, t, lane):
    """(k-row, first column) of the 8 bf16 lane `lane` stages for piece t (gemm.hip crh_src)."""
    fp = rows // 32
    kb, s2 = divmod(t, fp)
    rr = lane >> 2
    h = ((lane >> 1) & 1) ^ ((rr >> 3) & 1)
    return kb * 16 + rr, s2 * 32 + h * 16 + (lane & 1) * 8


def crh_lane(rows, lane, hi, h):
    g, i = lane >> 4, lane & 15
    q, p = i >> 2, i & 3
    rr = 8 * (g & 1) + q + 4 * hi
    return (g >> 1) * (rows // 32) * 1024 + 64 * rr + 32 * (h ^ ((rr >> 3) & 1)) + 8 * p


@pytest.mark.parametrize("rows,bk", [(256, 32), (128, 32), (256, 64)])
def test_cr_half_blocked_reads_consistent_and_conflict_free(rows, bk):
    # staging: element (k-row, column) -> LDS byte
    byte_of = {}
    for t in range(rows * bk * 2 // 1024):
        for lane in range(64):
            kr, col = crh_src(rows, t, lane)
            for e in range(8):
                byte_of[(kr, col + e)] = t * 1024 + 16 * lane + 2 * e
    assert len(byte_of) == rows * bk
    for kk, s in itertools.product(range(bk // 32), range(rows // 16)):
        off = (2 * kk * (rows // 32) + s // 2) * 1024  # frag_crh's immediate
        for hi in (0, 1):
            addr = lambda lane: crh_lane(rows, lane, hi, s & 1) + off
            # the 8 B a lane reads hold k-row kk*32 + 8g + q + 4hi, columns 16 s + 4p .. 4p + 3
            for lane in range(64):
                g, i = lane >> 4, lane & 15
                q, p = i >> 2, i & 3
                kr = kk * 32 + 8 * g + q + 4 * hi
                for e in range(4):
                    assert byte_of[(kr, 16 * s + 4 * p + e)] == addr(lane) + 2 * e
            assert _conflict_free(addr, B64_GROUPS, 8)


def test_cr_swizzled_rows_reads_conflict_free():
    # the swizzled-row CR image that pgemm.inc and VIT_CR_HB=0 builds keep (cr_swz / cr_off, ROWS = 256)
    def cr_f(r):
        return ((r & 3) << 2) | ((r >> 2) & 3)

    def cr_off(r, c):
        return r * 256 * 2 + ((((c & ~15) | ((c & 15) ^ cr_f(r)))) << 4)

    for s in range(16):
        for hi in (0, 1):
            def addr(lane):
                g, i = lane >> 4, lane & 15
                q, p = i >> 2, i & 3
                return cr_off(8 * g + q + 4 * hi, 2 * s + (p >> 1)) + (p & 1) * 8
            assert _conflict_free(addr, B64_GROUPS, 8)
