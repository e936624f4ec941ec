"""Control-flow model of the leaf-pair heap walk (csrc/rt_kernels.hip `heap_run`) against the reference's
`intersect_all_node` (shader_tris.wgsl:268-301), on random heaps with arbitrary node-test outcomes.

The walk's path depends only on which nodes the ray's slab test accepts (intersect_node has no best-t test), so
a set of "hit" nodes stands for any ray; empty nodes (the reference's inverted default boxes) are just nodes that
hit. The kernel's version must reach the same triangles in the same order, make the same node tests, and stop at
the same 600-step cap (checked here with smaller caps too, so that the cap falls on every kind of loop body).
The GPU parity tests check the real kernels against the oracle's counts; this pins the transformation itself.
"""
import random

import pytest


def reference_walk(n, m, hit, cap=600):
    """shader_tris.wgsl:268-301, statement by statement: (triangles tested in order, node tests)."""
    i, step, tris, nodes = 1, 0, [], 0
    while step < cap:
        step += 1
        if i < n:
            nodes += 1
            if hit(i):
                i *= 2
                continue
        if i >= n:
            j = i - n
            if j >= m:
                break
            tris.append(j)
        while i & 1:
            i //= 2
        if i == 0:
            break
        i += 1
    return tris, nodes


def pair_walk(n, m, hit, cap=600, flush_every=None):
    """heap_run as written: one node test per iteration, a hit bottom node appends its two leaves as one entry;
    the node count is derived as steps - triangles at the end of a run (runs end at a flush when
    `flush_every` is set, as a suspended walk does)."""
    pair = 1 << 31
    i, step, tris_n, nodes, out = 1, 0, 0, 0, []
    walking = True
    if i >= n:  # n == 1
        if m:
            out.append(0)
            tris_n += 1
            step += 1
        return out, step - tris_n
    while walking:
        step0, tris0, entries = step, tris_n, []
        while walking and (flush_every is None or len(entries) < flush_every):
            step += 1
            h = hit(i)
            down = h and 2 * i < n
            if h and not down:
                j0 = 2 * i - n
                if j0 + 2 <= m and step <= cap - 2:
                    entries.append(j0 | pair)
                    tris_n += 2
                    step += 2
                else:
                    walking = False
                    if step < cap and j0 < m:
                        entries.append(j0)
                        tris_n += 1
                        step += 1
            ip1 = i + 1
            up = ip1 >> ((ip1 & -ip1).bit_length() - 1)
            if not down and up == 1:
                walking = False
            i = 2 * i if down else up
            if step >= cap:
                walking = False
        for e in entries:
            out.append(e & ~pair)
            if e & pair:
                out.append((e & ~pair) + 1)
        nodes += (step - step0) - (tris_n - tris0)
    return out, nodes


@pytest.mark.parametrize("seed", range(4))
def test_pair_walk_matches_reference_walk(seed):
    rng = random.Random(seed)
    for _ in range(3000):
        n = 1 << rng.randint(0, 11)
        m = rng.randint(0, n) if rng.random() < 0.7 else rng.randint(max(0, n - 3), n)
        p = rng.random()
        hits = {x for x in range(1, n) if rng.random() < p}
        cap = rng.choice([600, 600, 1, 2, 3, 5, 7, 13, 40, 101])
        flush = rng.choice([None, 1, 3, 8])
        want = reference_walk(n, m, hits.__contains__, cap)
        got = pair_walk(n, m, hits.__contains__, cap, flush)
        assert got == want, (n, m, cap, flush, sorted(hits)[:20])


def test_pair_walk_with_reference_empty_nodes():
    """Trees as Tree::build leaves them (tree.rs:58-66): nodes over leaves >= m keep the inverted default box,
    which every finite ray's slab test accepts, so the walk ends at the first empty leaf."""
    rng = random.Random(7)
    for m in (1, 2, 3, 5, 979, 1000, 1024):
        n = 1
        while n < m:
            n *= 2
        for _ in range(200):
            p = rng.random()
            real = {x for x in range(1, n) if rng.random() < p}

            def hit(i, real=real, n=n, m=m):
                lo = i
                while lo < n:
                    lo *= 2
                return (lo - n) >= m or i in real  # leftmost leaf beyond m: empty subtree

            assert pair_walk(n, m, hit) == reference_walk(n, m, hit)
