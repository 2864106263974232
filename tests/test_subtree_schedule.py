"""CPU mirror of nmt.hip subtree_kernel's per-lane schedule (the fused NMT
levels of the k = 256 / 512 jobs).  The kernel walks an S-leaf subtree in post
order, one node per iteration, with the next iteration's memory operands
loaded one iteration ahead and pending left siblings in a per-level stack slot.
This replays exactly that index logic on symbolic nodes and checks that every
node is hashed from its true children, that each stack load reads the value
last stored to that slot (no overwrite in between), and that the root is the
subtree's root.  The GPU tests (test_gpu_parity k = 256 / 512, the config-4
variant test at 16 squares) check the bytes."""
import pytest


def kernel_schedule(S: int):
    slog = S.bit_length() - 1
    leaves = [("leaf", i) for i in range(S)]
    stack = {}                      # level -> value stored there
    hashes = []
    nL, nR = leaves[0], leaves[1]
    j, lvl, pos = 0, 0, 0
    cur = None
    for it in range(S - 1):
        merge = it > 0 and (pos & 1)
        L, R = nL, (cur if merge else nR)
        nlvl, npos = (lvl + 1, pos >> 1) if merge else (1, j)
        if not merge:
            j += 1
        if it + 2 < S:
            if npos & 1:
                nL = stack[nlvl]
            else:
                nL, nR = leaves[2 * j], leaves[2 * j + 1]
        cur = ("node", nlvl, npos, L, R)
        hashes.append(cur)
        if not (npos & 1) and nlvl < slog:
            stack[nlvl] = cur
        lvl, pos = nlvl, npos
    return cur, hashes


def reference_tree(lo: int, n: int, level: int, index: int):
    if n == 1:
        return ("leaf", lo)
    a = reference_tree(lo, n // 2, level - 1, 2 * index)
    b = reference_tree(lo + n // 2, n // 2, level - 1, 2 * index + 1)
    return ("node", level, index, a, b)


@pytest.mark.parametrize("S", [4, 8, 16, 32, 64, 128, 256])
def test_subtree_post_order_matches_tree(S):
    root, hashes = kernel_schedule(S)
    slog = S.bit_length() - 1
    assert root == reference_tree(0, S, slog, 0)
    assert len(hashes) == S - 1
    # every node exactly once
    assert len({(h[1], h[2]) for h in hashes}) == S - 1
