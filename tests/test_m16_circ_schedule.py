"""CPU check of the circular-halo schedule of the 7x7 kernel (conv_m16.hip, CIRC, round 6).

The kernel streams chunk c + 1's halo into circular LDS planes while chunk c computes; a piece that
lands too late, or overwrites a piece some wave still reads, gives wrong maps only on the GPU and
perhaps only sometimes.  This restates the kernel's per-tile schedule (region sizes, issue pairs,
physical pieces) and its ordering rules, and checks every tile of the launch shapes the kernel runs,
piece by piece:

* a piece written by waves 4-7 at the start of their pair gp is visible to every wave from pair
  gp + 2 on (their vmcnt wait at pair gp + 1, then the ring barrier they meet in its middle);
* when waves 4-7 start pair gp, waves 0-3 are inside pair gp, so the piece's previous content must
  not be read at pair gp or later;
* the first chunk is loaded by the prologue (every wave, drained) into physical pieces 0 .. nh-1.

Pairs are counted over the tile's chunks (25 per chunk: 24 tap pairs + the 49th tap with its zero
padding tap); tap t of a chunk is read at its pair t // 2.
"""
import numpy as np
import pytest

KS, R, KSQ, PAIRS = 7, 3, 49, 25
CP = 28  # 28-KiB planes (staggered 6-tap ring): 1-KiB pieces per plane


def tile_schedule(rows, pitch):
    """conv_m16.hip: np, R1 / R2 / R3 sizes and whether the tile runs circular."""
    np_ = (rows * pitch + 63) // 64
    op = max(2 * np_ - CP, 0)
    early = (6 * pitch) // 64
    r2 = min(op, early)
    r3 = op - r2
    r1 = np_ - op
    circ = np_ <= CP and (r3 == 0 or ((np_ - r3) * 64) // pitch >= rows - 2 * R)
    return np_, r1, r2, r3, circ


def issue_pairs(p, c, cb0, cb1, np_, r1, r2, r3):
    """(chunk, jlo, jhi) the waves 4-7 issue at pair p of chunk c (conv_m16.hip's schedule)."""
    has_next = c + 1 < cb1
    if p < 2:
        j0 = np_ - r3
        jm = j0 + (r3 + 1) // 2
        jlo = j0 if p == 0 else jm
        jhi = (jm if p == 0 else np_) if c > cb0 else jlo
        return c, jlo, jhi
    if p <= 20:
        jlo = (p - 2) * r1 // 19
        return c + 1, jlo, ((p - 1) * r1 // 19 if has_next else jlo)
    if p <= 22:
        jm = r1 + (r2 + 1) // 2
        jlo = r1 if p == 21 else jm
        return c + 1, jlo, ((jm if p == 21 else r1 + r2) if has_next else jlo)
    return c + 1, 0, 0


def piece_read_pairs(q, pitch, npieces):
    """Per local piece of a chunk: (first, last) pair that reads it (-1 / -1: none)."""
    first = np.full(npieces + 8, 10 ** 9)
    last = np.full(npieces + 8, -1)
    for t in range(KSQ):
        off = (t // KS) * pitch + t % KS
        pc = (q + off) // 64
        p = t // 2
        np.minimum.at(first, pc, p)
        np.maximum.at(last, pc, p)
    return first, last


def check_tile(q, rows, pitch, nh, cb0, cb1):
    np_, r1, r2, r3, circ = tile_schedule(rows, pitch)
    if not circ:
        return False
    assert r1 + r2 + r3 == np_ and min(r1, r2, r3) >= 0
    first, last = piece_read_pairs(q, pitch, np_)
    assert last[np_:].max() < 0, "a tap reads past the tile's pieces"
    # physical piece -> (chunk, local piece, write time, first read, last read) of its occupants
    write = {}  # (chunk, j) -> gp issued (None: prologue)
    for c in range(cb0, cb1):
        for p in range(PAIRS):
            cc, jlo, jhi = issue_pairs(p, c, cb0, cb1, np_, r1, r2, r3)
            for j in range(jlo, jhi):
                assert (cc, j) not in write, ("piece issued twice", cc, j)
                write[(cc, j)] = (c - cb0) * PAIRS + p
    occ = {}
    base = 0
    for c in range(cb0, cb1):
        g0 = (c - cb0) * PAIRS
        for j in range(np_):
            rd0, rd1 = first[j], last[j]
            if c == cb0:
                assert j < nh
                w = None
            else:
                assert (c, j) in write, ("piece never loaded", c, j)
                w = write[(c, j)]
                if rd1 >= 0:
                    assert g0 + rd0 >= w + 2, ("read before visible", c, j, g0 + rd0, w)
            ph = (base + j) % CP
            for (pc, pj, pw, p0, p1) in occ.get(ph, []):
                if pc == c:
                    continue
                if p1 >= 0:  # the previous occupant's reads end before this write is issued
                    wt = -1 if w is None else w
                    assert p1 < wt, ("overwrite while read", c, j, pc, pj, p1, wt)
            occ.setdefault(ph, []).append((c, j, w, g0 + rd0 if rd1 >= 0 else -1, g0 + rd1 if rd1 >= 0 else -1))
        base = (base + np_) % CP
    return True


def launch_tiles(n, h, w, npx):
    cap, hw = 64 * npx, h * w
    total = n * hw
    pitch = w + 2 * R  # tight pitch (raster_tiling's first variant for conv_m16)
    rows_max, tiles = 0, []
    for i in range((total + cap - 1) // cap):
        P0, P1 = i * cap, min(i * cap + cap, total) - 1
        f0, f1 = P0 // hw, P1 // hw
        ya, yb = (P0 - f0 * hw) // w, (P1 - f1 * hw) // w
        rows = yb - ya + 1 + 2 * R if f0 == f1 else (h - ya + 2 * R) + (yb + 1 + 2 * R)
        rows_max = max(rows_max, rows)
        tiles.append((P0, P1, f0, f1, ya))
    nh = (rows_max * pitch + 63) // 64
    return tiles, pitch, nh, hw


@pytest.mark.parametrize("n,h,w,npx,c16,ksplit", [
    (232, 46, 46, 10, 8, 1), (232, 46, 46, 10, 12, 1),   # the headline's Mconv2-5 / Mconv1
    (38, 46, 46, 10, 8, 1), (57, 46, 46, 8, 12, 1),     # round-3 batches, 512-px tiles
    (16, 46, 46, 5, 8, 1), (2, 46, 46, 6, 8, 2),        # small launches, split K
    (64, 46, 82, 10, 8, 1), (16, 69, 123, 9, 12, 1),    # C5, a C4 scale
    (16, 92, 164, 10, 8, 1), (116, 46, 46, 7, 8, 4),
])
def test_circular_halo_schedule(n, h, w, npx, c16, ksplit):
    tiles, pitch, nh, hw = launch_tiles(n, h, w, npx)
    if nh > CP:
        pytest.skip("halo planes over 28 KiB: the launch is not staggered, so not circular")
    ran = 0
    for (P0, P1, f0, f1, ya) in tiles:
        if f0 != f1:
            continue  # crossing a frame border: drained
        P = np.arange(P0, P1 + 1)
        pp = P - f0 * hw
        q = (pp // w - ya) * pitch + pp % w
        rows = (P1 - f0 * hw) // w - ya + 1 + 2 * R
        per = c16 // ksplit
        for split in range(ksplit):
            cb0 = split * per
            if per > 1 and check_tile(q, rows, pitch, nh, cb0, cb0 + per):
                ran += 1
    if (h, w) == (46, 46) and npx >= 8:
        assert ran > 0.6 * len(tiles) * ksplit, (ran, len(tiles))  # most tiles of the headline run circular


def test_headline_tiles_are_mostly_circular():
    """At 640-px tiles on 46 x 46 maps (tight pitch 52) every tile of one frame qualifies."""
    tiles, pitch, nh, hw = launch_tiles(232, 46, 46, 10)
    one = [t for t in tiles if t[2] == t[3]]
    circ = [tile_schedule((t[1] - t[2] * hw) // 46 - t[4] + 1 + 6, pitch)[4] for t in one]
    assert pitch == 52 and nh <= CP
    assert all(circ), sum(circ)
    assert 0.6 < len(one) / len(tiles) < 0.8, len(one) / len(tiles)
