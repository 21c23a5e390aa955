"""A step-level model of the cell table's parallel chain placement
(build_cells: k_cells_fill, k_over_heads + max-scan, k_cells_place).  Every record's atomic steps run in a random interleaving with the
others', including records whose runs share a chain (equal fingerprint low bits,
equal stride) and entries of other homes sitting in the chain cells.  The check
is the probe's walk rule (k_probe, prefix_contain_walk, k_lookup_key): every
record is found from its home cell, moving to the next cell of its
fingerprint's chain while the current one is full with the chain flag on its
last slot.  Kernel-level parity runs on the GPU (test_gpu_parity
test_exchange_mode_options, the exchange scale digests)."""
import random

import pytest

K = 8  # kCell


def stride(n, fp):
    return 1 if (n & (n - 1)) else 1 + 2 * (fp & 1023)


def next_cell(c, n, fp):
    return (c + stride(n, fp)) % n


def chain_cell(c, n, fp, s):  # next_cell applied s times
    return (c + s * stride(n, fp)) % n


class TableFull(Exception):
    pass


def place(n_cells, recs, foreign, rnd):
    """recs: (home, fp, tag); returns the cells and their chain flags."""
    cells = [[None] * K for _ in range(n_cells)]
    flag = [False] * n_cells
    for c, e in foreign:  # entries of other homes already in the table
        if None in cells[c]:
            cells[c][cells[c].index(None)] = e
    recs = sorted(recs, key=lambda r: (r[0], r[1] & 7))  # the radix sort: (cell, low fp bits)
    n = len(recs)
    over, first = [False] * n, [False] * n
    for i, (c, fp, _) in enumerate(recs):
        r = 0
        while r < K and i - r - 1 >= 0 and recs[i - r - 1][0] == c:
            r += 1
        if r < K:  # k_cells_fill
            cells[c][r] = recs[i]
            flag[c] |= r == K - 1 and i + 1 < n and recs[i + 1][0] == c
        else:
            over[i] = True
            first[i] = not (i >= K + 1 and recs[i - K - 1][0] == c)
    head = [i if over[i] and (first[i] or recs[i][1] != recs[i - 1][1]) else 0 for i in range(n)]
    start, m = [], 0
    for h in head:  # inclusive max-scan
        m = max(m, h)
        start.append(m)

    def record(i):  # k_cells_place, one yield per memory step
        c, fp, _ = recs[i]
        x = i - start[i]
        slot = x % K
        more = slot == K - 1 and i + 1 < n and recs[i + 1][0] == c and recs[i + 1][1] == fp
        at = chain_cell(c, n_cells, fp, 1 + x // K)
        yield
        if cells[at][slot] is None:  # CAS
            cells[at][slot] = recs[i]
            flag[at] |= more
            return
        for _ in range(n_cells):  # taken: cell_insert from here on
            snap, snapflag = list(cells[at]), flag[at]
            yield
            for s in range(K):
                if snap[s] is None:
                    yield
                    if cells[at][s] is None:
                        cells[at][s] = recs[i]
                        return
            if not snapflag or snap[K - 1] is None:
                yield
                flag[at] = True
            at = next_cell(at, n_cells, fp)
        raise TableFull

    live = [record(i) for i in range(n) if over[i]]
    while live:
        j = rnd.randrange(len(live))
        try:
            next(live[j])
        except StopIteration:
            live.pop(j)
    return recs, cells, flag


def reachable(rec, cells, flag, n_cells):
    at = rec[0]
    for _ in range(n_cells + 1):
        if rec in cells[at]:
            return True
        if not (cells[at][K - 1] is not None and flag[at]):
            return False
        at = next_cell(at, n_cells, rec[1])
    return False


def test_parallel_chain_placement_keeps_every_record_reachable():
    done = 0
    for seed in range(400):
        rnd = random.Random(seed)
        n_cells = rnd.choice([16, 64, 13, 29, 1024])
        recs = []
        for k in range(rnd.randint(1, n_cells * K // 4)):
            if rnd.random() < 0.6:  # heavy homes; fingerprints sharing low bits and strides
                recs.append((rnd.randrange(2), rnd.choice([5, 1029, 7, 29]), k))
            else:
                recs.append((rnd.randrange(n_cells), rnd.randrange(1 << 19), k))
        # entries of other homes in the chain cells (not in any home of recs:
        # k_cells_fill owns those)
        homes = {r[0] for r in recs}
        foreign = [(c, ("f", k)) for k, c in enumerate(rnd.randrange(n_cells) for _ in range(n_cells // 2))
                   if c not in homes]
        try:
            placed, cells, flag = place(n_cells, recs, foreign, rnd)
        except TableFull:
            continue
        for r in placed:
            assert reachable(r, cells, flag, n_cells), (seed, r)
        done += 1
    assert done > 350


def test_chain_cell_is_next_cell_repeated():
    for n in (13, 16, 1024, 1 << 20):
        for fp in (0, 5, 1023, 1024, (1 << 19) - 1):
            c = 7 % n
            at = c
            for s in range(1, 40):
                at = next_cell(at, n, fp)
                assert chain_cell(c, n, fp, s) == at


if __name__ == "__main__":
    pytest.main([__file__, "-q"])
