"""The sweeps' item dealing over the XCDs (le_sweep.hip sweep_item / sweep_grid), restated
on the host: every light item is taken by exactly one workgroup of the launch grid, for
blocks of B table entries (B = 1 round-robin, the default 8, larger) and for one contiguous
range per XCD (B = -1), with heavy items first.  Pure integer logic, no GPU."""
import pytest


def grid8(n):
    return (n + 7) & ~7


def sweep_grid(items, item_bound, B):
    per = items // item_bound if item_bound > 0 else 1
    return grid8(items + 8 + (8 * B * per if B > 0 else 0))


def sweep_item(b, nt_entries, nh_entries, per_entry, B):
    nt, nh = nt_entries * per_entry, nh_entries * per_entry
    h8 = (nh + 7) & ~7
    if b < h8:
        return b if b < nh else -1
    bl, nl = b - h8, nt - nh
    if B > 0:
        Bi = B * per_entry
        k, x = bl >> 3, bl & 7
        it = ((k // Bi) * 8 + x) * Bi + (k % Bi)
        return nh + it if it < nl else -1
    per = (nl + 7) >> 3
    if (bl >> 3) >= per:
        return -1
    it = (bl & 7) * per + (bl >> 3)
    return nh + it if it < nl else -1


@pytest.mark.parametrize("B", [-1, 1, 3, 8, 34])
@pytest.mark.parametrize("per_entry", [1, 3])
@pytest.mark.parametrize("nt,nh,bound", [(1, 0, 1), (7, 0, 9), (100, 0, 100), (997, 13, 1000), (4096, 200, 4500),
                                         (43008, 0, 43008), (12, 12, 12)])
def test_every_item_once(B, per_entry, nt, nh, bound):
    grid = sweep_grid(bound * per_entry, bound, B)
    taken = [sweep_item(b, nt, nh, per_entry, B) for b in range(grid)]
    got = sorted(t for t in taken if t >= 0)
    assert got == list(range(nt * per_entry)), (B, per_entry, nt, nh)


def test_blocks_stay_on_one_xcd():
    # hardware deals workgroup b to XCD b mod 8: a block of B entries x per_entry items is one XCD's
    B, per_entry, nt = 8, 3, 4096
    grid = sweep_grid(nt * per_entry, nt, B)
    xcd = {}
    for b in range(grid):
        it = sweep_item(b, nt, 0, per_entry, B)
        if it >= 0:
            xcd[it] = b & 7
    Bi = B * per_entry
    for start in range(0, nt * per_entry, Bi):
        assert len({xcd[i] for i in range(start, min(start + Bi, nt * per_entry))}) == 1
