"""Multi-line access traces for the split / combine tests (core.cc:139-266):
the hotspot generator's lines with a byte offset and a size drawn per access
(some zero, some crossing one or more line boundaries, some ending exactly on
a boundary)."""
import numpy as np


def gen_multiline(tiles, per_tile, hot_lines=16, seed=7, max_size=200):
    from oracle import pyoracle as po
    a, m, offs = po.gen_trace(tiles, per_tile, hot_lines=hot_lines)
    rng = np.random.default_rng(seed)
    off = rng.integers(0, 64, len(a)).astype(np.uint64)
    size = rng.integers(1, max_size + 1, len(a)).astype(np.uint32)
    k = rng.random(len(a))
    size[k < 0.05] = 0                                        # no access, gap carried
    edge = (k >= 0.05) & (k < 0.15)                           # end exactly on a line boundary
    size[edge] = (64 - off[edge] + 64 * rng.integers(0, 3, int(edge.sum()))).astype(np.uint32)
    return a + off, size, m, offs


def split_reference(addr, size, meta, offs, line=64):
    """core.cc:139-201 as a literal loop (the line addresses and the meta words
    gg_split_accesses must produce)."""
    la, lm, first = [], [], []
    for t in range(len(offs) - 1):
        carry = 0
        for i in range(int(offs[t]), int(offs[t + 1])):
            first.append(len(la))
            gap = carry + ((int(meta[i]) & 0x7FFFFFFF) >> 1)
            if int(size[i]) == 0:
                carry = gap
                continue
            carry = 0
            b, e = int(addr[i]), int(addr[i]) + int(size[i])
            ba, ea = b - b % line, e - e % line
            a = ba
            j = 0
            while a <= ea:
                off = b % line if a == ba else 0
                sz = (e % line) - off if a == ea else line - off
                if not (a == ea and sz == 0):
                    la.append(a)
                    w = int(meta[i]) & 1
                    lm.append(w | (gap << 1) if j == 0 else w | 0x80000000)
                    j += 1
                a += line
    first.append(len(la))
    first = np.array(first, np.uint64)
    return np.array(la, np.uint64), np.array(lm, np.uint32), first, first[np.asarray(offs, np.int64)]
