"""The planner's tree scans (nearest, near set) against a numpy restatement of the oracle's
(oracle/smp_oracle.cpp Planner::nearest / Planner::near_set, which follow birrt_star.cpp:4076-4133 and
4272-4324): integer ids must match exactly.  Trees are synthetic: uniform and clustered configurations, costs
with many ties, constant / ascending / descending costs, and nodes placed on the near radius.  Every case runs in the
four forms the planner uses: the workgroup's own scans (nearest, near_set), a distributed scan's slice functions over the
whole range (slice_nn, slice_near), and the fused nearest + near set of connect (near_set<20, true>, slice_near<true>)."""

MODES = {"local": {}, "slice": {"slices": True}, "fused": {"fused": True}, "fused_slice": {"slices": True, "fused": True},
         "slice_inl": {"slices": True, "inline": True}, "fused_slice_inl": {"slices": True, "fused": True, "inline": True}}
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def ref_scans(q, cost, x, r, excl):
    s = np.zeros(len(q))
    for j in range(8):  # same order of operations as the oracle's dist(): s += d * d, j ascending
        d = q[:, j] - x[j]
        s = s + d * d
    d = np.sqrt(s)
    ids = np.arange(len(q))
    nearest = int(np.argmin(d)) if d.min() < 10000.0 else 0
    near = ids[(d < r) & (ids != excl)]
    order = near[np.lexsort((near, cost[near]))]
    k = len(order)
    t = min(20, k)
    return nearest, k, order[:t], order[k - t:]


def make_tree(rng, n, kind):
    q = rng.uniform(-3, 3, (n, 8))
    if kind == "ties":
        cost = np.floor(rng.uniform(0, 6, n) * 2) / 2
    elif kind == "const":
        cost = np.full(n, 2.5)
    elif kind == "asc":
        cost = np.sort(rng.uniform(0, 10, n))
    elif kind == "desc":
        cost = -np.sort(-rng.uniform(0, 10, n))
    else:
        cost = rng.uniform(0, 10, n)
    if n:
        cost[0] = 0.0
    return q, cost


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("n", [1, 5, 63, 64, 65, 511, 513, 2049, 9001])
@pytest.mark.parametrize("kind", ["rand", "ties", "const", "asc", "desc"])
def test_tree_scans_match_oracle(n, kind, mode):
    from squirrel_motion_planner_amd import probes
    rng = np.random.default_rng(n * 7 + len(kind))
    q, cost = make_tree(rng, n, kind)
    r = 4.0
    queries, excl = [], []
    for k in range(6):
        i = int(rng.integers(0, n))
        queries.append(q[i] + rng.normal(0, 0.5 * k, 8))
        excl.append(i if k % 2 == 0 else -1)
    # nodes exactly on / just inside / just outside the radius of query 0
    x0 = queries[0]
    for t, f in enumerate((1.0, 1.0 - 1e-15, 1.0 + 1e-15, 1.0 - 1e-13, 1.0 + 1e-13)):
        if t + 1 < n:
            e = np.zeros(8)
            e[t % 8] = r * f
            q[t + 1] = x0 + e
    queries = np.array(queries)
    got = probes.tree_scan(q, cost, queries, excl, r, **MODES[mode])
    for k in range(len(queries)):
        nn, kk, lo, hi = ref_scans(q, cost, queries[k], r, excl[k])
        assert got["nearest"][k] == nn, (k, got["nearest"][k], nn)
        assert got["k"][k] == kk
        t = len(lo)
        assert list(got["lo"][k][:t]) == list(lo), (k, got["lo"][k], lo)
        assert list(got["hi"][k][:t]) == list(hi), (k, got["hi"][k], hi)
        assert (got["lo"][k][t:] == -1).all() and (got["hi"][k][t:] == -1).all()


@pytest.mark.parametrize("mode", list(MODES))
def test_tree_scans_clustered_radius(mode):
    """Dense cluster around the query: every node near, k >> 20."""
    from squirrel_motion_planner_amd import probes
    rng = np.random.default_rng(5)
    n = 6000
    x = rng.uniform(-1, 1, 8)
    q = x + rng.normal(0, 0.3, (n, 8))
    cost = np.round(rng.uniform(0, 3, n), 2)
    got = probes.tree_scan(q, cost, x[None, :], [17], 4.0, reps=3, **MODES[mode])
    nn, kk, lo, hi = ref_scans(q, cost, x, 4.0, 17)
    assert got["nearest"][0] == nn and got["k"][0] == kk == n - 1
    assert list(got["lo"][0]) == list(lo) and list(got["hi"][0]) == list(hi)


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("kind", ["rand", "asc", "desc", "ties"])
def test_tree_scans_three_chunks(kind, mode):
    """17000 nodes: three register chunks of the near set, running lists carried across chunks."""
    from squirrel_motion_planner_amd import probes
    rng = np.random.default_rng(11)
    q, cost = make_tree(rng, 17000, kind)
    q *= 0.5
    queries = q[[3, 9000, 16999]] + 0.1
    excl = [3, -1, 16999]
    got = probes.tree_scan(q, cost, queries, excl, 4.0, **MODES[mode])
    for k in range(3):
        nn, kk, lo, hi = ref_scans(q, cost, queries[k], 4.0, excl[k])
        assert got["nearest"][k] == nn and got["k"][k] == kk
        assert list(got["lo"][k]) == list(lo) and list(got["hi"][k]) == list(hi)
