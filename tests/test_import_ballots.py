"""The k2himport kernels' ballot compositions (round 6), restated on the host.

Pass A's wave function (`wave_gfn`), its block newline prefix (`nl_prefix_block`) and pass B's
per-lane entry states (`wave_state_in`) in `k2hash_amd/csrc/k2h_import_dev.hip` replace wave
scans of span functions over the two-state getline machine of tests/k2himport.cc:81-86 (mode
K reads a key up to its TAB, mode V a value up to its newline).  Each lane's span acts on the
state as a function: per entry mode its exit mode, record ends, last field boundary; plus its
last NUL.  These tests restate the kernels' ballot arithmetic -- the nearest fixed-exit lane
below, the parity of swapping lanes in between, per-bit prefix counts, the highest lane with a
boundary -- lane for lane in Python and check it against the plain sequential composition on
random span functions.  They pin the algebra; `-m gpu` tests (tests/test_import.py) pin the
kernels themselves against the reference's own getline loop.
"""
import random

WAVE = 64


def popc(x):
    return bin(x).count("1")


def ballot(pred):
    return sum(1 << i for i, p in enumerate(pred) if p)


def highest(mask):
    return mask.bit_length() - 1


def random_lanes(rng, sparse=False):
    """Span functions of one wave: exit mode per entry, record ends per entry (a span of at most
    six events ends at most 3 records; a span re-read from the file, up to 64), boundary
    positions per entry (unit-relative + 1, increasing with the lane; 0: none), last NUL."""
    lanes = []
    for i in range(WAVE):
        if sparse and rng.random() < 0.8:
            lanes.append(((0, 1), (0, 0), (0, 0), 0))  # no event: the identity
            continue
        big = rng.random() < 0.02
        ex = (rng.randint(0, 1), rng.randint(0, 1))
        cnt = tuple(rng.randint(0, 64 if big else 3) for _ in range(2))
        last = tuple(i * 128 + rng.randint(1, 128) if rng.random() < 0.6 else 0 for _ in range(2))
        nul = i * 128 + rng.randint(1, 128) if rng.random() < 0.1 else 0
        lanes.append((ex, cnt, last, nul))
    return lanes


def entry_modes(lanes, m_entry):
    """Each lane's entry mode from ballots (wave_state_in / wave_gfn): the nearest lane below
    with a fixed exit mode (or the wave's entry mode), flipped by the swapping lanes between."""
    bfix = ballot(ex[0] == ex[1] for ex, *_ in lanes)
    bk = ballot(ex[0] != 0 for ex, *_ in lanes)
    bswap = ballot(ex[0] != 0 and ex[1] == 0 for ex, *_ in lanes)
    out = []
    for lane in range(WAVE + 1):  # lane WAVE: the wave's exit mode
        below = (1 << lane) - 1
        mf = bfix & below
        jf = highest(mf) if mf else 0
        flips = bswap & below & (~((2 << jf) - 1) if mf else -1)
        out.append((((bk >> jf) if mf else m_entry) ^ popc(flips)) & 1)
    return out


def test_wave_state_in_matches_sequential_composition():
    rng = random.Random(0x6B32)
    for _ in range(600):
        lanes = random_lanes(rng, sparse=rng.random() < 0.3)
        su = dict(m=rng.randint(0, 1), r=rng.randint(0, 10**6), fs=rng.randint(0, 9), ln=rng.randint(0, 9))
        base = 1 << 30
        ref, s = [], dict(su)
        for ex, cnt, last, nul in lanes:
            ref.append(dict(s))
            m = s["m"]
            s = dict(m=ex[m], r=s["r"] + cnt[m], fs=base + last[m] if last[m] else s["fs"],
                     ln=base + nul if nul else s["ln"])
        modes = entry_modes(lanes, su["m"])
        cnts = [lanes[i][1][modes[i]] for i in range(WAVE)]
        lasts = [lanes[i][2][modes[i]] for i in range(WAVE)]
        nb = 7 if any(c > 3 for c in cnts) else 2
        bits = [ballot((c >> b) & 1 for c in cnts) for b in range(nb)]
        hl, hn = ballot(x != 0 for x in lasts), ballot(lane[3] != 0 for lane in lanes)
        for i in range(WAVE):
            below = (1 << i) - 1
            pc = sum(popc(bits[b] & below) << b for b in range(nb))
            got = dict(m=modes[i], r=su["r"] + pc,
                       fs=base + lasts[highest(hl & below)] if hl & below else su["fs"],
                       ln=base + lanes[highest(hn & below)][3] if hn & below else su["ln"])
            assert got == ref[i]
        assert sum(popc(bits[b]) << b for b in range(nb)) == s["r"] - su["r"]  # the unit's record ends


def test_wave_gfn_matches_sequential_composition():
    rng = random.Random(0x6B33)
    for _ in range(600):
        lanes = random_lanes(rng, sparse=rng.random() < 0.3)
        for e in (0, 1):
            m, r, last, ln = e, 0, 0, 0
            for ex, cnt, lst, nul in lanes:
                r += cnt[m]
                last = lst[m] or last
                ln = nul or ln
                m = ex[m]
            modes = entry_modes(lanes, e)
            cnts = [lanes[i][1][modes[i]] for i in range(WAVE)]
            lasts = [lanes[i][2][modes[i]] for i in range(WAVE)]
            nb = 7 if any(c > 3 for c in cnts) else 2
            total = sum(popc(ballot((c >> b) & 1 for c in cnts)) << b for b in range(nb))
            h = ballot(x != 0 for x in lasts)
            hn = ballot(lane[3] != 0 for lane in lanes)
            assert (modes[WAVE], total, lasts[highest(h)] if h else 0) == (m, r, last)
            assert (lanes[highest(hn)][3] if hn else 0) == ln


def test_nl_prefix_block_matches_sequential_scan():
    """NlSum over a 128-thread block: bit 0 has newline, bit 1 open (no cut after it), bits 2+
    its position; compose(x, y) = y if y has a newline, else x closed when y holds a cut."""
    def compose(x, y):
        return y if y & 1 else (x & (~0 if y & 2 else ~2))

    rng = random.Random(0x6B34)
    for _ in range(3000):
        vs = []
        for _ in range(128):
            u = rng.random()
            vs.append(2 if u < 0.3 else 0 if u < 0.5 else 1 | (rng.randint(0, 1) << 1) | (rng.randint(0, 16383) << 2))
        ref, acc = [], 2
        for v in vs:
            ref.append(acc)
            acc = compose(acc, v)
        got, agg0 = [], 2
        for w in range(2):
            wv = vs[WAVE * w:WAVE * (w + 1)]
            bnl, bcut = ballot(v & 1 for v in wv), ballot(not v & 2 for v in wv)
            agg = 0 if bcut else 2
            if bnl:
                ja = highest(bnl)
                agg = wv[ja] & ~2 if (bcut >> ja) >> 1 else wv[ja]
            prev = agg0 if w else 2
            for lane in range(WAVE):
                below = (1 << lane) - 1
                m, cb = bnl & below, bcut & below
                j = highest(m) if m else 0
                closed = ((cb >> j) >> 1) != 0 if m else cb != 0
                p = wv[j] if m else prev
                got.append(p & ~2 if closed else p)
            if w == 0:
                agg0 = agg
        assert got == ref
