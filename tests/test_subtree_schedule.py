"""CPU mirror of nmt.hip subtree_kernel's per-lane schedule (the fused NMT
levels).  The kernel walks an S-leaf subtree in post order, one node per
iteration, with pending left siblings in a per-level stack slot.  The product
kernel loads each iteration's operands at use (kernel_schedule: a leaf pair,
or on a merge the stored left sibling from stack_slot(lvl)); round 3's first
form loaded them one iteration ahead (prefetch_schedule; the build is
tools/probes/nmt_variants.patch).  Both replay exactly the kernel's index
logic on symbolic nodes; the tests check that every node is hashed from its
true children, that each stack load reads the value last stored to that slot
(no overwrite in between), and that the root is the subtree's root.  The GPU tests (test_gpu_parity k = 256 / 512, the config-4
variant test at 16 squares) check the bytes."""
import pytest


def kernel_schedule(S: int):
    """The product loop (operands loaded at use)."""
    slog = S.bit_length() - 1
    leaves = [("leaf", i) for i in range(S)]
    stack = {}                      # level -> value stored there
    hashes = []
    cur = None
    j, lvl, pos = 0, 0, 0
    for it in range(S - 1):
        merge = it > 0 and (pos & 1)
        if merge:
            L, R = stack[lvl], cur     # pa = stack_slot(lvl); R <- cur
        else:
            L, R = leaves[2 * j], leaves[2 * j + 1]
        nlvl, npos = (lvl + 1, pos >> 1) if merge else (1, j)
        if not merge:
            j += 1
        cur = ("node", nlvl, npos, L, R)
        hashes.append(cur)
        if not (npos & 1) and nlvl < slog:
            stack[nlvl] = cur
        lvl, pos = nlvl, npos
    return cur, hashes


def prefetch_schedule(S: int):
    """Round 3's first form (next operands loaded one iteration ahead)."""
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


@pytest.mark.parametrize("schedule", [kernel_schedule, prefetch_schedule])
@pytest.mark.parametrize("S", [4, 8, 16, 32, 64, 128, 256])
def test_subtree_post_order_matches_tree(S, schedule):
    root, hashes = schedule(S)
    slog = S.bit_length() - 1
    assert root == reference_tree(0, S, slog, 0)
    assert len(hashes) == S - 1
    # every node exactly once
    assert len({(h[1], h[2]) for h in hashes}) == S - 1
