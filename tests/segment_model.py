"""Python model of the segmented long-pretoken path (encode.hip, k_seg_init / k_seg_first /
k_seg_enc / k_seg_check / k_seg_join / k_seg_out): the pretoken is cut at the ASCII chars BPE.tokenize skips
(/root/reference/src/model/bpe.zig:192-208), around inert chars (a symbol in no merge) and
before whitespace with a mergeable symbol; every group of segments is encoded alone
with its round profile recorded, each boundary between groups is checked by replaying
the two profiles in the reference's merge order (bpe.zig:214-253), and crossed
boundaries join their groups until none is crossed. Test infrastructure: it states the
algorithm the kernel implements so that its exactness can be checked against the
reference loop (oracle.RefTokenizer.bpe_tokenize) on many random cases on the CPU."""
from oracle.oracle import codepoint_slices

INF = 1 << 62


def _value(merges, a, b):
    v = merges.get((a, b))
    return INF if v is None else v[0]


def bpe_profile(merges, syms):
    """The reference rounds on a symbol list; returns (final symbols, rounds) with one
    (rank, new_id, merged the first symbol, merged the last symbol) per round."""
    w = list(syms)
    rounds = []
    while len(w) > 1:
        best, br = None, INF
        for i in range(len(w) - 1):
            r = _value(merges, w[i], w[i + 1])
            if r < br:
                br, best = r, (w[i], w[i + 1])
        if best is None:
            break
        nid = merges[best][1]
        le = re = False
        i = 0
        while i < len(w) - 1:
            if w[i] == best[0] and w[i + 1] == best[1]:
                le = le or i == 0
                re = re or i + 1 == len(w) - 1
                w[i] = nid
                del w[i + 1]
            else:
                i += 1
        rounds.append((br, nid, le, re))
    return w, rounds


def crossed(merges, left, right):
    """Does the two-group process of (left | right) merge the pair straddling them?
    left/right: (initial symbols, rounds). A tie with a group's next round counts as
    crossed (always safe: joining groups is exact)."""
    x, y = left[0][-1], right[0][0]
    lr, rr = left[1], right[1]
    ng = max([k + 1 for k, r in enumerate(lr) if r[3]], default=0)
    nh = max([k + 1 for k, r in enumerate(rr) if r[2]], default=0)
    i = j = 0
    b = _value(merges, x, y)
    while True:
        hc = lr[i][0] if i < ng else INF
        hd = rr[j][0] if j < nh else INF
        if b < INF and b <= hc and b <= hd:
            return True
        if hc == INF and hd == INF:
            return False
        chg = False
        if hc <= hd:
            if lr[i][3]:
                x, chg = lr[i][1], True
            i += 1
        if hd <= hc:
            if rr[j][2]:
                y, chg = rr[j][1], True
            j += 1
        if chg:
            b = _value(merges, x, y)


def crossed_edges(merges, left, right):
    """crossed() as the kernel computes it (encode.hip seg_crossed_core): only the rounds that
    changed left's last symbol (RE) and right's first (LE) are walked; a pair ends at the
    next entry of either list, and its merge crosses if its value <= that entry's."""
    x, y = left[0][-1], right[0][0]
    re = [(r[0], r[1]) for r in left[1] if r[3]]
    le = [(r[0], r[1]) for r in right[1] if r[2]]
    i = j = 0
    while True:
        hc = re[i][0] if i < len(re) else INF
        hd = le[j][0] if j < len(le) else INF
        b = _value(merges, x, y)
        if b < INF and b <= min(hc, hd):
            return True
        if hc == INF and hd == INF:
            return False
        if hc <= hd:
            x = re[i][1]
            i += 1
        if hd <= hc:
            y = le[j][1]
            j += 1


def merges_ordered(merges):
    """tokenizer.cpp merges_ordered: does every merge rank after every merge creating one of
    its parts (a token made by several merges: the largest of their ranks)? Then a group's
    round values strictly increase and crossed_edges() == crossed(); otherwise the library
    keeps such a table off the segmented path."""
    made = {}
    for (_a, _b), (r, n) in merges.items():
        made[n] = max(made.get(n, -1), r)
    return all(r > made.get(a, -1) and r > made.get(b, -1) for (a, b), (r, _n) in merges.items())


WS = b" \t\n\r\x0b\x0c"


def cut_classes(tok):
    """Per ASCII byte: 'drop' (no id, no unk: bpe.zig:192-208), 'inert' (its symbol -- own
    id or the unk id, bpe.zig:198-205 -- is in no merge on either side), 'cut' (whitespace
    with a mergeable symbol), or None (an ordinary char)."""
    unk_id = tok.vocab.get(tok.unk) if tok.unk is not None else None
    sides = set()
    for (a, b) in tok.merges:
        sides.add(a)
        sides.add(b)
    cls = []
    for c in range(128):
        sym = tok.vocab.get(bytes([c]), unk_id)
        if sym is None:
            cls.append("drop")
        elif sym not in sides:
            cls.append("inert")
        elif c in WS:
            cls.append("cut")
        else:
            cls.append(None)
    return cls, unk_id


def segments(tok, seq: bytes):
    """The kernel's segments of a pretoken (k_seg_init): runs of kept bytes, cut after a
    dropped byte, around an inert char (a segment of its own) and before a whitespace cut.
    Returns [(start, end, inert)]."""
    cls, _ = cut_classes(tok)
    kind = [cls[c] if c < 0x80 else None for c in seq]
    segs, cur = [], None
    for i, k in enumerate(kind):
        if k == "drop":
            if cur is not None:
                segs.append((cur, i, False))
                cur = None
            continue
        brk = k in ("inert", "cut") or (i > 0 and kind[i - 1] == "inert")
        if cur is not None and brk:
            segs.append((cur, i, False))
            cur = None
        if k == "inert":
            segs.append((i, i + 1, True))
            continue
        if cur is None:
            cur = i
    if cur is not None:
        segs.append((cur, len(seq), False))
    return segs


def segmented_bpe(tok, seq: bytes, edges=False):
    """BPE.tokenize of one pretoken by segments; None where the kernel does not segment
    (fewer than two segments). Returns [(id, start, end)]. edges: check the boundaries as
    the kernel does (crossed_edges; exact for ordered merge tables only)."""
    check = crossed_edges if edges else crossed
    _, unk_id = cut_classes(tok)
    segs = segments(tok, seq)
    if len(segs) < 2:
        return None
    cache = {}

    def run(g):  # group = (first segment, end segment)
        if g not in cache:
            a, b = segs[g[0]][0], segs[g[1] - 1][1]
            s0 = []
            for (s, e) in codepoint_slices(seq[a:b]):
                tid = tok.vocab.get(seq[a:b][s:e], unk_id)
                if tid is not None:
                    s0.append(tid)
            if not s0:  # every char dropped: an empty group, joined with its neighbours
                cache[g] = ([], [], [])
                return cache[g]
            fin, rounds = bpe_profile(tok.merges, s0)
            toks = [(t, s + a, e + a) for (t, s, e) in tok.bpe_tokenize(seq[a:b])]
            assert [t[0] for t in toks] == fin
            cache[g] = (s0, rounds, toks)
        return cache[g]

    def inert(g):
        return g[1] - g[0] == 1 and segs[g[0]][2]

    groups = [(k, k + 1) for k in range(len(segs))]
    while True:
        changed, new, cur = False, [], groups[0]
        for nxt in groups[1:]:
            if inert(cur) or inert(nxt):  # never crossed
                new.append(cur)
                cur = nxt
                continue
            L, R = run(cur), run(nxt)
            if not L[0] or not R[0] or check(tok.merges, L, R):
                cur, changed = (cur[0], nxt[1]), True
            else:
                new.append(cur)
                cur = nxt
        new.append(cur)
        groups = new
        if not changed:
            break
    out = []
    for g in groups:
        out += run(g)[2]
    return out
