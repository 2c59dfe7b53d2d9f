"""Edge-tile row layout of a 6-board Connect4 tile (tower.hip Cfg::EDGE), conflict-free by construction.

Writes self_play_reinforcement_learning_amd/csrc/tower_edge.h: EDGE_ROW (row -> board/x/y, 255 =
padding), EDGE_CELL_ROW (cell -> row) and EDGE_NBR ([tap][row] -> source row, zero rows off the board).

Constraints (the kernel skips these (tile, tap) MFMAs): tile 0 holds only x = 0 cells, tile 1 only
y = 0, tile 6 only x = 6, tile 7 only y = 5 (padding rows may sit anywhere; the kernel tests
EDGE_ROW[r] != 255), so their dx = -1 / dy = -1 / dx = +1 / dy = +1 taps read zero padding only.

Bank model (MI355X_MICROARCH.md §LDS): a B-fragment read is one ds_read_b128 per (tile, tap, k-step);
its 16-lane groups are {0-3,12-15,20-27} and {4-11,16-19,28-31} (+32), bank = (addr / 4) mod 64, and
the 272-B LDS rows shift each row by one 16-B slot, so lane l of a group touches slot
(source row + chunk) mod 16 and a group is conflict-free iff its 16 source rows are distinct mod 16.
Both groups hold 16 different lane residues l mod 16.

Shift-invariant colouring: every cell (b, x, y) gets the residue kappa = (u x + v y + t_b) mod 16 and
is placed at a row of that residue (lane l = kappa or kappa + 16 of its tile).  A tap (dx, dy) maps a
cell to one whose residue is kappa + (u dx + v dy), the same shift for every lane, so the source rows
of a group stay distinct at every tap; an off-board lane (or a padding row) reads the zero row of
the residue its virtual neighbour would have (rows 256..271 have residues 0..15).  Every B-fragment
read of the trunk (and of the stem and the epilogue's residual reads, tap 4) is then conflict-free.
The placement of cells into (tile, residue) bins with the tile classes above is a max-flow problem;
(u, v, t_b) are searched until all 252 cells fit.  The round-1 to round-3 layout (row order from a
local search with row = slot, modelled 1.42-way sharing) measured 33 % bank-conflict cycles.

    python scripts/edge_layout_model.py                 # the recorded parameters (instant)
    python scripts/edge_layout_model.py --search [--seed S] [--tries N]
"""
import argparse
import os
import random

GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
ROWS, ZROW, NZ = 256, 256, 16
W, H, B = 7, 6, 6
CELLS = [(b, x, y) for b in range(B) for x in range(W) for y in range(H)]
EDGE_TILES = {0: lambda c: c[1] == 0, 1: lambda c: c[2] == 0, 6: lambda c: c[1] == W - 1, 7: lambda c: c[2] == H - 1}
INTERIOR = (2, 3, 4, 5)
# (u, v, t_0..t_5) found by --search (seed 2, relaxed padding); reproduces the shipped tower_edge.h
RECORDED = (6, 13, (0, 15, 13, 2, 11, 14))


def kappa(c, u, v, t):
    return (c[1] * u + c[2] * v + t[c[0]]) % 16


def place(u, v, t, fixed_padding=False):
    """Max-flow placement of the 252 cells into bins (edge tile, residue) of 2 rows and (interior,
    residue) of 8 rows.  Returns (cells placed, {cell: (tile class, residue)})."""
    import numpy as np
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import maximum_flow

    bins = [(T, r) for T in (0, 1, 6, 7, "I") for r in range(16)]
    bi = {b: i for i, b in enumerate(bins)}

    def cap(T, r):
        if T == "I":
            return 8
        return 1 if (fixed_padding and T == 7 and r >= 12) else 2

    n = len(CELLS)
    src, sink = 0, 1 + n + len(bins)
    rows, cols, caps = [], [], []
    for i, c in enumerate(CELLS):
        rows.append(src), cols.append(1 + i), caps.append(1)
        k = kappa(c, u, v, t)
        for T in [T for T, f in EDGE_TILES.items() if f(c)] + ["I"]:
            rows.append(1 + i), cols.append(1 + n + bi[(T, k)]), caps.append(1)
    for j, (T, r) in enumerate(bins):
        rows.append(1 + n + j), cols.append(sink), caps.append(cap(T, r))
    g = csr_matrix((np.array(caps, dtype=np.int32), (rows, cols)), shape=(sink + 1, sink + 1))
    res = maximum_flow(g, src, sink)
    flow = res.flow.tocsr() if hasattr(res, "flow") else res.residual.tocsr()
    out = {}
    for i, c in enumerate(CELLS):
        row = flow.getrow(1 + i)
        for j, f in zip(row.indices, row.data):
            if f > 0 and 1 + n <= j < sink:
                out[c] = bins[j - 1 - n]
    return res.flow_value, out


def rows_from_placement(pl, u, v, t):
    """Row table: bin (edge tile T, residue r) -> rows 32T + r and 32T + r + 16; (interior, r) -> the
    two rows of residue r in each of tiles 2..5.  Padding rows (None) fill what is left."""
    rows = [None] * ROWS
    slots = {}
    for T in (0, 1, 6, 7):
        for r in range(16):
            slots[(T, r)] = [32 * T + r, 32 * T + r + 16]
    for r in range(16):
        slots[("I", r)] = [32 * T + r + 16 * h for T in INTERIOR for h in (0, 1)]
    for c in sorted(pl):  # deterministic: cells in (b, x, y) order take a bin's rows in order
        rows[slots[pl[c]].pop(0)] = c
    return rows


def nbr_table(rows, u, v):
    inv = {c: r for r, c in enumerate(rows) if c is not None}
    nbr = [[0] * ROWS for _ in range(9)]
    for tap in range(9):
        dx, dy = tap // 3 - 1, tap % 3 - 1
        shift = (u * dx + v * dy) % 16
        for r in range(ROWS):
            c = rows[r]
            if c is not None and 0 <= c[1] + dx < W and 0 <= c[2] + dy < H:
                nbr[tap][r] = inv[(c[0], c[1] + dx, c[2] + dy)]
            else:  # the zero row of the residue the virtual neighbour would have
                nbr[tap][r] = ZROW + (r % 16 + shift) % 16
    return nbr


def on_board(c, tap):
    return c is not None and 0 <= c[1] + tap // 3 - 1 < W and 0 <= c[2] + tap % 3 - 1 < H


def live(rows, T, tap):
    return any(on_board(rows[r], tap) for r in range(T * 32, T * 32 + 32))


def bank_cost(rows, nbr):
    """Sum over the live (tile, tap) reads and lane groups of the max number of DISTINCT source rows
    that share one 16-B slot (1 = conflict-free; identical rows broadcast), and the read count."""
    tot = n = 0
    for T in range(8):
        for tap in range(9):
            if not live(rows, T, tap):
                continue
            for g in GROUPS:
                per = {}
                for l in g:
                    s = nbr[tap][T * 32 + l]
                    per.setdefault(s % 16, set()).add(s)
                tot += max(len(x) for x in per.values())
                n += 1
    return tot, n


def check(rows, nbr):
    """The invariants the kernel relies on (also tests/test_tower_edge_layout.py)."""
    cells = [c for c in rows if c is not None]
    assert len(cells) == len(set(cells)) == B * W * H
    for T, f in EDGE_TILES.items():
        assert all(rows[r] is None or f(rows[r]) for r in range(32 * T, 32 * T + 32)), T


def write_header(rows, nbr, path, note):
    enc = [255 if c is None else c[0] * 64 + c[1] * 8 + c[2] for c in rows]
    inv = {c: r for r, c in enumerate(rows) if c is not None}
    cell_row = [inv[(b, x, y)] for b in range(B) for x in range(W) for y in range(H)]
    flat = [val for tap in range(9) for val in nbr[tap]]

    def arr(name, vals):
        body = ", \\\n".join("    " + ", ".join(str(x) for x in vals[i:i + 24]) for i in range(0, len(vals), 24))
        return "#define %s_INIT { \\\n%s }\n" % (name, body)

    hdr = ("// tower_edge.h — generated by scripts/edge_layout_model.py (%s).\n"
           "// Edge-tile row layout of a 6-board Connect4 tile (Cfg::EDGE): row r holds cell (b, x, y) =\n"
           "// (v >> 6, (v >> 3) & 7, v & 7) of v = EDGE_ROW[r] (255 = padding row); EDGE_CELL_ROW[(b * 7 + x) * 6 + y]\n"
           "// is its row; EDGE_NBR[tap * 256 + r] the source row of tap (dx, dy) = (tap / 3 - 1, tap %% 3 - 1),\n"
           "// a zero row (256 + i) off the board.  Tiles 0 / 1 / 6 / 7 hold only x = 0 / y = 0 / x = 6 /\n"
           "// y = 5 cells, so their dx = -1 / dy = -1 / dx = +1 / dy = +1 taps read zero padding only.\n"
           "// Row r holds a cell of residue (u x + v y + t_b) mod 16 = r mod 16: every B-fragment read is\n"
           "// bank-conflict free at every tap.\n"
           "#pragma once\n" % note) + arr("EDGE_ROW", enc) + arr("EDGE_CELL_ROW", cell_row) + arr("EDGE_NBR", flat)
    with open(path, "w") as f:
        f.write(hdr)


def search(seed, tries, fixed_padding):
    rnd = random.Random(seed)
    best = (-1, None)
    for i in range(tries):
        u, v = rnd.randrange(16), rnd.randrange(16)
        t = (0,) + tuple(rnd.randrange(16) for _ in range(B - 1))
        n, _ = place(u, v, t, fixed_padding)
        if n > best[0]:
            best = (n, (u, v, t))
            print(f"try {i}: {n} of {len(CELLS)} cells placed with u={u} v={v} t={t}", flush=True)
        if n == len(CELLS):
            break
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--search", action="store_true")
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--tries", type=int, default=20000)
    ap.add_argument("--fixed-padding", action="store_true", help="padding rows only at 252..255")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                  "self_play_reinforcement_learning_amd", "csrc", "tower_edge.h"))
    args = ap.parse_args()
    if args.search:
        n, (u, v, t) = search(args.seed, args.tries, args.fixed_padding)
        if n != len(CELLS):
            raise SystemExit(f"no conflict-free placement found ({n} of {len(CELLS)} cells)")
    else:
        u, v, t = RECORDED
    n, pl = place(u, v, t, args.fixed_padding)
    assert n == len(CELLS), n
    rows = rows_from_placement(pl, u, v, t)
    nbr = nbr_table(rows, u, v)
    check(rows, nbr)
    cost, reads = bank_cost(rows, nbr)
    note = "u=%d v=%d t=%s: modelled bank sharing %.3f per 16-lane read over %d reads" % (u, v, list(t), cost / reads,
                                                                                          reads)
    print(note)
    write_header(rows, nbr, args.out, note)


if __name__ == "__main__":
    main()
