"""CPU mirror of tree_top_kernel's index arithmetic (nmt.hip), plain and with
the wide first level (kTopWide: a thread per parent over 2 kTopThreads
parents, tpw = 4 kTopThreads / n_in trees per workgroup, its output in the
helpers' LDS rows, lane pairs from the second level on), and of the engine's
choice of the fused top (engine.hip top_fuse_nodes).  Nodes are combined with
an order-sensitive stand-in for hash_node, so a wrong pairing, tree offset or
buffer alias changes the roots.  The GPU parity tests check the kernel itself
(k = 128 / 256 / 512 squares against the oracle fixtures)."""
import pytest

K_TOP_THREADS = 128


def combine(a, b):
    return ("n", a, b)


def tree_top_model(trees, n_in, wide):
    """trees: list of per-tree input node lists (n_in each) -> roots, as the
    kernel's workgroups compute them."""
    tpw = (4 if wide else 2) * K_TOP_THREADS // n_in
    n_trees = len(trees)
    roots = [None] * n_trees
    for wg in range((n_trees + tpw - 1) // tpw):
        buf = [[None] * K_TOP_THREADS for _ in range(2)]
        wide_out = [None] * (2 * K_TOP_THREADS)
        cur = 0
        if wide:
            half = n_in // 2
            for tid in range(2 * K_TOP_THREADS):
                j, p = tid // half, tid % half
                g = wg * tpw + j
                if j < tpw and g < n_trees:
                    wide_out[tid] = combine(trees[g][2 * p], trees[g][2 * p + 1])
        m = n_in // 2 if wide else n_in
        o = [None] * K_TOP_THREADS
        while m >= 2:
            half = m // 2
            src = wide_out if (wide and m == n_in // 2) else buf[cur]
            nxt = [None] * K_TOP_THREADS
            for u in range(K_TOP_THREADS):   # pair units
                j, p = u // half, u % half
                g = wg * tpw + j
                if not (j < tpw and g < n_trees):
                    continue
                if m == n_in and not wide:   # first level from global memory
                    L, R = trees[g][2 * p], trees[g][2 * p + 1]
                else:
                    L, R = src[j * m + 2 * p], src[j * m + 2 * p + 1]
                o[u] = combine(L, R)
                if m > 2:
                    nxt[u] = o[u]
            buf[cur ^ 1] = nxt
            cur ^= 1
            m //= 2
        for u in range(tpw):
            g = wg * tpw + u
            if g < n_trees:
                roots[g] = o[u]
    return roots


def reference_root(nodes):
    while len(nodes) > 1:
        nodes = [combine(nodes[2 * i], nodes[2 * i + 1]) for i in range(len(nodes) // 2)]
    return nodes[0]


@pytest.mark.parametrize("n_in,wide,n_trees", [(32, False, 64), (128, False, 12), (256, False, 5),
                                               (64, True, 40), (128, True, 64), (256, True, 7), (512, True, 3),
                                               (8, True, 130)])
def test_tree_top_indexing(n_in, wide, n_trees):
    trees = [[("leaf", t, i) for i in range(n_in)] for t in range(n_trees)]
    assert tree_top_model(trees, n_in, wide) == [reference_root(t) for t in trees]


def top_fuse_nodes(W, n, top_wide=2):
    """engine.hip Engine::top_fuse_nodes (auto mode): (top, wide)."""
    m = W
    while m >= 2:
        if n * 2 * W * (m // 2) < 65536:
            if m > 256:
                return 0, False
            t, e = m, 0
            while e < top_wide and 2 * t <= W and 2 * t <= 512 and 2 * t >= 8 and 2 * n * 2 * W * (t // 2) <= 131072:
                t *= 2
                e += 1
            return t, t > m
        m //= 2
    return 0, False


def test_top_fuse_choice():
    # config 2 (k = 128, one square): the whole tree in the top, first level wide
    assert top_fuse_nodes(256, 1) == (256, True)
    # config 3 (k = 512, one square): two levels more than the lane-pair level 32
    assert top_fuse_nodes(1024, 1) == (128, True)
    assert top_fuse_nodes(1024, 1, top_wide=0) == (32, False)
    # k = 256
    assert top_fuse_nodes(512, 1) == (256, True)
    # config 4 batches: no tree top (the subtree launch writes the roots)
    assert top_fuse_nodes(256, 128) == (0, False)
    # tiny squares: the whole tree, never wide below 8 nodes
    assert top_fuse_nodes(4, 1) == (4, False)
    for W in (4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048):
        for n in (1, 2, 3, 4, 8, 16, 64, 256):
            t, wide = top_fuse_nodes(W, n)
            assert t <= W and t <= (512 if wide else 256)
            if wide:
                # the lane pairs of the second level fit two waves per SIMD
                assert 8 <= t and 2 * n * 2 * W * (t // 4) <= 131072
