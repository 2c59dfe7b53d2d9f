"""CPU: the edge-tile row layout tables (csrc/tower_edge.h, Cfg::EDGE of the trunk kernel) are a
bijection between the 252 cells of six Connect4 boards and 252 of the rows 0..255 (the other 4 are
padding, EDGE_ROW = 255), every tap's source row is the neighbour cell's row (a zero row 256..271 off
the board), tiles 0 / 1 / 6 / 7 hold only x = 0 / y = 0 / x = 6 / y = 5 cells (the taps the kernel
skips for them read zero padding only), and every B-fragment read of the trunk is LDS-bank-conflict
free under the ds_read_b128 bank rule (MI355X_MICROARCH.md §LDS: 16-lane groups {0-3,12-15,20-27},
{4-11,16-19,28-31}; 272-B rows = one 16-B slot per row)."""
import os
import re

HDR = os.path.join(os.path.dirname(__file__), "..", "self_play_reinforcement_learning_amd", "csrc", "tower_edge.h")
GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]


def _arr(src, name):
    m = re.search(r"#define %s_INIT \{(.*?)\}" % name, src, re.S)
    return [int(x) for x in re.findall(r"\d+", m.group(1))]


def _tables():
    src = open(HDR).read()
    return _arr(src, "EDGE_ROW"), _arr(src, "EDGE_CELL_ROW"), _arr(src, "EDGE_NBR")


def test_edge_tables():
    er, cr, nb = _tables()
    assert len(er) == 256 and len(cr) == 6 * 7 * 6 and len(nb) == 9 * 256
    cells = set()
    for r in range(256):
        v = er[r]
        if v == 255:  # padding row: every tap reads a zero row
            assert all(256 <= nb[tap * 256 + r] < 272 for tap in range(9))
            continue
        b, x, y = v >> 6, (v >> 3) & 7, v & 7
        assert b < 6 and x < 7 and y < 6 and (b, x, y) not in cells
        cells.add((b, x, y))
        assert cr[(b * 7 + x) * 6 + y] == r
        for tap in range(9):
            nx, ny = x + tap // 3 - 1, y + tap % 3 - 1
            got = nb[tap * 256 + r]
            if 0 <= nx < 7 and 0 <= ny < 6:
                assert got == cr[(b * 7 + nx) * 6 + ny]
            else:
                assert 256 <= got < 272
    assert len(cells) == 252 and sum(v == 255 for v in er) == 4
    # the skipped (tile, tap) pairs: 3 per edge tile, 12 in all
    dead = {0: (0, 1, 2), 1: (0, 3, 6), 6: (6, 7, 8), 7: (2, 5, 8)}
    for t, taps in dead.items():
        for tap in taps:
            assert all(256 <= nb[tap * 256 + r] < 272 for r in range(32 * t, 32 * t + 32)), (t, tap)


def test_edge_reads_bank_conflict_free():
    """Every (tile, tap) operand read the kernel issues: within each 16-lane group the source rows that
    share a 16-B slot (row mod 16) are one and the same row (a broadcast), never two."""
    er, _, nb = _tables()
    reads = 0
    for t in range(8):
        for tap in range(9):
            src = [nb[tap * 256 + 32 * t + l] for l in range(32)]
            if all(s >= 256 for s in src):
                continue  # a skipped (tile, tap): no read
            reads += 1
            for g in GROUPS:
                per = {}
                for l in g:
                    per.setdefault(src[l] % 16, set()).add(src[l])
                assert max(len(s) for s in per.values()) == 1, (t, tap, g)
    assert reads == 60


def _m16_lane_row(n):
    """tower_m16.h lane_row: MFMA column n of a 16x16x32 B fragment h stands for tile row lane_row(n) + h."""
    in_a = n < 4 or n >= 12
    i = (n if n < 4 else n - 8) if in_a else n - 4
    return (0 if in_a else 16) + 2 * i


def test_m16_reads_bank_conflict_free():
    """The 16x16x32 trunk's B-fragment reads (csrc/tower_m16.h): lane 16 q + n of fragment (tile t, h)
    reads 16 B of row nbr[tap][32 t + lane_row(n) + h] at byte offset 64 k + 16 q, i.e. 16-B slot
    (row + q + 4 k) mod 16; every 16-lane group of every k-step of every live (tile, tap) read touches 16
    distinct slots (or the same row: a broadcast).  With column n on row 16 h + n (round 4) the model
    gives 50 % conflict cycles (measured 44 % of the kernel's LDS cycles)."""
    _, _, nb = _tables()
    groups = GROUPS + [[l + 32 for l in g] for g in GROUPS]
    assert sorted(_m16_lane_row(n) + h for h in (0, 1) for n in range(16)) == list(range(32))
    reads = 0
    for t in range(8):
        for tap in range(9):
            if all(nb[tap * 256 + 32 * t + l] >= 256 for l in range(32)):
                continue
            for h in (0, 1):
                reads += 1
                for k in range(4):
                    for g in groups:
                        per = {}
                        for l in g:
                            q, n = l >> 4, l & 15
                            s = nb[tap * 256 + 32 * t + _m16_lane_row(n) + h]
                            per.setdefault((s + q + 4 * k) % 16, set()).add(s)
                        assert max(len(s) for s in per.values()) == 1, (t, tap, h, k, g)
    assert reads == 120
