"""CPU exactness model of the sign-ordered node test against the reference's intersect_node
(shader_tris.wgsl:150-159) in IEEE f32, minNum / maxNum for min / max (the build's numerics contract).

The heap walk's kernels (rt_kernels.hip node_slab_so) read each node as (lo, hi, lo) per axis — lo <= hi after a
per-axis swap done on the host (renderer.cpp pack_nodes_so) — at an offset chosen by the sign of 1/d, so the near
plane comes first and the slab test needs no per-axis min / max:

    tnear_k = (near_k - o_k) * inv_k,  tfar_k = (far_k - o_k) * inv_k
    hit = max3(tnear) <= min3(tfar) && min3(tfar) >= 0

Equal to the reference whenever every 1/d component is finite (the kernels fall back to the reference formula, on the
same layout, for a wave with any infinite or NaN component) and no bound is NaN (the host disables the layout then):
with lo <= hi and inv finite and nonzero, RN is monotone, so (lo - o) * inv and (hi - o) * inv are ordered by the sign
of inv and min / max pick exactly the near / far value; the swap only reorders the pair min / max take. Zeros of either
sign only enter comparisons, where -0 == +0; infinite bounds or overflowing differences stay ordered. The cases where the forms differ (NaN from 0 x inf when a direction
component is +-0 or denormal, NaN bounds) are the ones the predicate excludes — checked here too."""
import numpy as np

F = np.float32
MAXREF = F(3.40282e38)  # FLT_MAX_REF, shader_*.wgsl:4


def reference_hit(o, inv, mn, mx):
    t0 = (mn - o) * inv
    t1 = (mx - o) * inv
    tmin = np.fmin(t0, t1)
    tmax = np.fmax(t0, t1)
    tminf = np.fmax(np.fmax(tmin[..., 0], tmin[..., 1]), tmin[..., 2])
    tmaxf = np.fmin(np.fmin(tmax[..., 0], tmax[..., 1]), tmax[..., 2])
    return (tminf <= tmaxf) & (tmaxf >= F(0))


def pack_so(mn, mx):
    """Host layout: per axis lo <= hi (swapped where the node had min > max: padding nodes, inverted boxes)."""
    lo = np.where(mn > mx, mx, mn)
    hi = np.where(mn > mx, mn, mx)
    return lo, hi


def so_hit(o, inv, lo, hi):
    neg = np.signbit(inv)
    near = np.where(neg, hi, lo)
    far = np.where(neg, lo, hi)
    tn = (near - o) * inv
    tf = (far - o) * inv
    tminf = np.fmax(np.fmax(tn[..., 0], tn[..., 1]), tn[..., 2])
    tmaxf = np.fmin(np.fmin(tf[..., 0], tf[..., 1]), tf[..., 2])
    return (tminf <= tmaxf) & (tmaxf >= F(0))


def usable(inv, mn, mx, o=None):
    """The kernels' predicate for the sign-ordered form: finite 1/d and origin (wave-uniform in the kernel) and no
    NaN bound (per tree, on the host)."""
    ok = np.all(np.isfinite(inv), axis=-1) & ~np.any(np.isnan(mn) | np.isnan(mx), axis=-1)
    return ok if o is None else ok & np.all(np.isfinite(o), axis=-1)


def _check(o, d, mn, mx):
    with np.errstate(all="ignore"):
        inv = F(1) / d
        ref = reference_hit(o, inv, mn, mx)
        lo, hi = pack_so(mn, mx)
        so = so_hit(o, inv, lo, hi)
    ok = usable(inv, mn, mx, o)
    bad = ok & (ref != so)
    assert not bad.any(), (o[bad][:3], d[bad][:3], mn[bad][:3], mx[bad][:3])
    return ok, ref, so


def _unit(rng, n):
    d = rng.standard_normal((n, 3)).astype(F)
    return (d / np.sqrt((d * d).sum(-1, keepdims=True))).astype(F)


def test_random_boxes_and_rays():
    rng = np.random.default_rng(1)
    n = 400_000
    o = (rng.standard_normal((n, 3)) * 3).astype(F)
    c = (rng.standard_normal((n, 3)) * 3).astype(F)
    h = np.abs(rng.standard_normal((n, 3))).astype(F)
    aim = c - o + rng.standard_normal((n, 3)).astype(F)  # rays roughly at the boxes: both outcomes common
    d = (aim / np.sqrt((aim * aim).sum(-1, keepdims=True))).astype(F)
    d[: n // 2] = _unit(rng, n // 2)
    ok, ref, _ = _check(o, d, c - h, c + h)
    assert ok.all() and 0.1 < ref.mean() < 0.9


def test_padding_and_inverted_nodes():
    """Padding nodes (min = +MAX, max = -MAX), which the reference passes for every ray, and boxes inverted on
    one axis only."""
    rng = np.random.default_rng(2)
    n = 100_000
    o = (rng.standard_normal((n, 3)) * 2).astype(F)
    d = _unit(rng, n)
    mn = np.full((n, 3), MAXREF, F)
    mx = np.full((n, 3), -MAXREF, F)
    ok, ref, so = _check(o, d, mn, mx)
    assert ok.all() and ref.all() and so.all()
    c = rng.standard_normal((n, 3)).astype(F)
    h = np.abs(rng.standard_normal((n, 3))).astype(F)
    mn, mx = c - h, c + h
    ax = rng.integers(0, 3, n)
    mn[np.arange(n), ax], mx[np.arange(n), ax] = mx[np.arange(n), ax].copy(), mn[np.arange(n), ax].copy()
    _check(o, d, mn, mx)


def test_origins_on_planes_zeros_and_flat_boxes():
    """lo - o = 0 (+0, and -0 where bounds / origin are -0), flat boxes (lo = hi), origins inside and on corners."""
    rng = np.random.default_rng(3)
    n = 200_000
    d = _unit(rng, n)
    grid = np.array([-1.0, -0.0, 0.0, 0.5, 1.0], F)
    mn = grid[rng.integers(0, 5, (n, 3))]
    mx = grid[rng.integers(0, 5, (n, 3))]
    o = grid[rng.integers(0, 5, (n, 3))]
    ok, ref, _ = _check(o, d, mn, mx)
    assert ok.all() and ref.any() and not ref.all()


def test_huge_bounds_and_tiny_directions():
    """Bounds near FLT_MAX_REF (products overflow to +-inf, still ordered) and direction components down to 2^-120
    (1/d finite but huge); below 2^-126 / exactly +-0 the predicate excludes the ray."""
    rng = np.random.default_rng(4)
    n = 200_000
    d = _unit(rng, n)
    k = rng.integers(0, 3, n)
    d[np.arange(n), k] = (np.ldexp(1.0, -rng.integers(60, 121, n)) * rng.choice([-1.0, 1.0], n)).astype(F)
    o = (rng.standard_normal((n, 3))).astype(F)
    big = np.array([-MAXREF, -1e30, -1.0, 1.0, 1e30, MAXREF], F)
    mn = big[rng.integers(0, 3, (n, 3))]
    mx = big[rng.integers(3, 6, (n, 3))]
    ok, _, _ = _check(o, d, mn, mx)
    assert ok.all()


def test_the_excluded_cases_do_differ():
    """Why the predicate is needed: a +-0 direction component with the origin on the plane (0 x inf = NaN) changes
    the reference's min / max (minNum drops the NaN) but not the same way in the sign-ordered form; NaN bounds too."""
    o = np.array([[0.5, 0.0, 0.5]], F)
    d = np.array([[1.0, 0.0, 0.0]], F)
    mn = np.array([[1.0, 0.0, 0.0]], F)
    mx = np.array([[2.0, 1.0, 1.0]], F)
    with np.errstate(all="ignore"):
        inv = F(1) / d
        lo, hi = pack_so(mn, mx)
        assert not usable(inv, mn, mx).any()
        assert reference_hit(o, inv, mn, mx)[0] != so_hit(o, inv, lo, hi)[0]
    mn2 = np.array([[np.nan, 0.0, 0.0]], F)
    assert not usable(np.ones((1, 3), F), mn2, mx).any()
