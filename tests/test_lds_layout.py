"""LDS layouts of conv_fwd_kernel (async-rl_amd/csrc/conv_fwd.hip) and the LSTM gate / BPTT
kernels (lstm.hip), checked on the CPU.

The layout constants are read from the kernel source. The address formulas are
restated here: a1_pos / a1_off (conv_fwd.hip:117-119), the conv1 epilogue
stores (:247, :501-504), the conv2 a1 / W2 fragment reads (:519-523, :556-569)
and the conv1 W1 fragment reads (:266). Two kinds of property are checked:
  * correctness: the a1 slots of the 400 pixels x 2 channel halves are
    distinct and lie inside a plane; the epilogue's 8-byte stores cover each
    slot's 16 bytes exactly once; conv2 reads only slots the epilogue wrote;
  * the bank model the round-4 layout was built for (MI355X_MICROARCH.md,
    LDS): each ds_read_b128 lane group of a conv2 a1 read and of a W1 / W2
    fragment read touches 16 distinct 16-byte bank quads, i.e. no extra cycles.
"""
import os
import re
from collections import defaultdict

SRC = os.path.join(os.path.dirname(__file__), "..", "async-rl_amd", "csrc", "conv_fwd.hip")

# ds_read_b128: four groups of 16 lanes, each served in one pass over 64 banks
B128_GROUPS = [
    [0, 1, 2, 3, 12, 13, 14, 15] + list(range(20, 28)),
    list(range(4, 12)) + [16, 17, 18, 19, 28, 29, 30, 31],
    [32, 33, 34, 35, 44, 45, 46, 47] + list(range(52, 60)),
    list(range(36, 44)) + [48, 49, 50, 51, 60, 61, 62, 63],
]
C1_P, C2_P = 400, 81


def _const(src, name):
    m = re.search(r"constexpr int [^;]*\b%s = ([^;,]+)[;,]" % name, src)
    assert m, name
    return m.group(1).strip()


def layout():
    src = open(SRC).read()
    wrow = int(_const(src, "WROW"))
    a1_ps = int(_const(src, "A1_PS"))
    assert _const(src, "A1_HALF") == "4 * A1_PS"
    a1_half = 4 * a1_ps
    assert _const(src, "A1P") == "2 * A1_HALF * 16"
    return wrow, a1_ps, a1_half, 2 * a1_half * 16


WROW, A1_PS, A1_HALF, A1P = layout()


def a1_pos(Y, X):
    return 9 * Y + X if X < 9 else 90 + ((9 * Y + 15) & 15)


def a1_off(y, x, h):
    return (h * A1_HALF + ((y & 1) * 2 + (x & 1)) * A1_PS + a1_pos(y >> 1, x >> 1)) << 4


def b128_extra(addrs):
    """Extra LDS cycles of one ds_read_b128 (64 lane byte addresses, 16-B aligned)."""
    extra = 0
    for grp in B128_GROUPS:
        quads = defaultdict(set)
        for lane in grp:
            a = addrs[lane]
            quads[(a >> 4) & 15].add(a >> 4)   # 64 banks = 16 quads of 4 dwords
        extra += max(len(v) for v in quads.values()) - 1
    return extra


def test_a1_slots_distinct_and_inside_a_plane():
    seen = {}
    for y in range(20):
        for x in range(20):
            for h in range(2):
                o = a1_off(y, x, h)
                assert 0 <= o and o + 16 <= A1P
                assert o not in seen, (y, x, h, seen.get(o))
                seen[o] = (y, x, h)
    assert len(seen) == 2 * C1_P


def test_epilogue_stores_cover_each_slot_once():
    # lane (g, col) of conv1 tile t holds oc 4g..4g+3 of position p = 16 t + col and stores them as
    # one 8-byte chunk per split plane at a1_off(oy, ox, g >> 1) + 8 (g & 1)
    written = defaultdict(int)
    for t in range(25):
        for g in range(4):
            for col in range(16):
                p = 16 * t + col
                oy, ox = divmod(p, 20)
                o = a1_off(oy, ox, g >> 1) + (g & 1) * 8
                for b in range(o, o + 8):
                    written[b] += 1
    assert set(written.values()) == {1}
    slots = {a1_off(y, x, h) for y in range(20) for x in range(20) for h in range(2)}
    assert {b & ~15 for b in written} == slots
    assert len(written) == 16 * len(slots)


def conv2_a1_reads(m, tap):
    """Byte addresses of one conv2 a1 fragment read (plane 0) of m-tile m, tap = 2 s + (g >> 1)
    of lane group g: lane (g, col) reads position 16 m + col (rows past 81 read position - 16)."""
    addrs = [None] * 64
    for lane in range(64):
        g, col = lane >> 4, lane & 15
        pos = 16 * m + col
        pc = pos if pos < C2_P else pos - 16
        oy, ox = divmod(pc, 9)
        tp = tap + (g >> 1)
        addrs[lane] = a1_off(2 * oy + (tp >> 2), 2 * ox + (tp & 3), g & 1)
    return addrs


def test_conv2_reads_only_written_slots():
    slots = {a1_off(y, x, h) for y in range(20) for x in range(20) for h in range(2)}
    for m in range(6):
        for s in range(8):
            for a in conv2_a1_reads(m, 2 * s):
                assert a in slots


def test_conv2_a1_reads_conflict_free():
    for m in range(6):
        for s in range(8):
            assert b128_extra(conv2_a1_reads(m, 2 * s)) == 0, (m, s)


def test_weight_fragment_reads_conflict_free():
    for s in range(8):
        # conv2 W2: lane (g, col), oc = 16 nt + col, k-step s: oc row, 32-byte tap block, 16-byte half
        for nt in range(2):
            w2 = [(16 * nt + (l & 15)) * WROW + (2 * s + ((l >> 4) >> 1)) * 32 + ((l >> 4) & 1) * 16
                  for l in range(64)]
            assert b128_extra(w2) == 0, ("W2", s, nt)
        # conv1 W1: lane (g, col), oc = col: row col, k = 8 (4 s + g) .. + 7
        w1 = [(l & 15) * WROW + (4 * s + (l >> 4)) * 16 for l in range(64)]
        assert b128_extra(w1) == 0, ("W1", s)


def test_old_layout_conflicts_are_detected():
    # the model is not vacuous: the round-3 weight row of 528 B (1 slot mod 16) conflicts
    w1 = [(l & 15) * 528 + (4 * 0 + (l >> 4)) * 16 for l in range(64)]
    assert b128_extra(w1) > 0


LSTM_SRC = os.path.join(os.path.dirname(__file__), "..", "async-rl_amd", "csrc", "lstm.hip")


def lstm_ld():
    m = re.search(r"constexpr int LSTM_LD = (\d+);", open(LSTM_SRC).read())
    assert m
    return int(m.group(1))


def lstm_reads(ld, row0, k):
    """One f32x4 fragment read of the LSTM gate / BPTT kernels (lstm.hip:138-139, :398): lane
    (q, col) reads staged row row0 + col (ld float4 per row) at float4 column q + 4 k."""
    return [((row0 + (l & 15)) * ld + (l >> 4) + 4 * k) * 16 for l in range(64)]


def test_lstm_fragment_reads_conflict_free():
    ld = lstm_ld()
    for row0 in (0, 16, 32, 48, 64, 80):
        for k in range(8):
            assert b128_extra(lstm_reads(ld, row0, k)) == 0, (ld, row0, k)
    # the round-3 stride of 33 float4 (1 mod 16) puts two rows of a lane group on one quad
    assert b128_extra(lstm_reads(33, 0, 0)) > 0
