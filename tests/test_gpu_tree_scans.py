"""The planner's tree scans (nearest, near set) against a numpy restatement of the oracle's
(oracle/smp_oracle.cpp Planner::nearest / Planner::near_set, which follow birrt_star.cpp:4076-4133 and
4272-4324): integer ids must match exactly.  Trees are synthetic: uniform and clustered configurations, costs
with many ties, constant / ascending / descending costs, and nodes placed on the near radius.  Every case runs in the
four forms the planner uses: the workgroup's own scans (nearest, near_set), a distributed scan's slice functions over the
whole range (slice_nn, slice_near), and the fused nearest + near set of connect (near_set<20, true>, slice_near<true>).

What the planner runs: the "local" forms below 2048 nodes (fp64 register path); from 2048 nodes the local scans and every
slice of a distributed scan go through the inlined fp32-prefilter forms (slice_inl / fused_slice_inl, and "local" /
"fused" at n >= 2048, which call them).  The "slice" / "fused_slice" modes run the fp64 slice functions slice_nn /
slice_near, which the planner keeps only as the fallback of a histogram that cannot split its costs; they stay here as a
cross-check of that fallback."""

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


@pytest.mark.parametrize("mode", ["local", "fused", "slice_inl", "fused_slice_inl"])
@pytest.mark.parametrize("n", [2048, 5000])
def test_fp32_prefilter_near_ties(n, mode):
    """Nearest-node ties and near-ties that the fp32 copy cannot separate (nn32_finish's candidate threshold decides
    which threads rescan in fp64): exact duplicates of one configuration at ids spread over threads and waves (the first
    strict minimum is the lowest id), nodes within 1e-9 .. 1e-7 of the query (equal in fp32, ordered in fp64), a second
    cluster at the same fp32 distance, and nodes on the radius within the fp32 error band.  Run in the fp32 forms the
    planner uses (local scans of 2048+ nodes, helper / publisher slices)."""
    from squirrel_motion_planner_amd import probes
    rng = np.random.default_rng(n + len(mode))
    q = rng.uniform(-3, 3, (n, 8))
    cost = rng.uniform(0, 10, n)
    cost[0] = 0.0
    x = rng.uniform(-2, 2, 8)
    base = x + np.array([0.3, -0.2, 0.1, 0.05, 0.0, 0.0, 0.0, 0.0])
    # duplicates of one node (equal fp64 distance) at ids across threads / waves / the slice's node stride
    dup = [n - 1, 1500, 777, 513, 64, 65]
    for i in dup:
        q[i] = base
    # nodes within 1e-9 .. 1e-7 of the query in one joint: identical in fp32, different in fp64
    tiny = [(901, 1e-7), (902, -3e-8), (1903 % n, 1e-9), (17, 5e-8)]
    queries, excl = [], []
    for k, (i, d) in enumerate(tiny):
        e = np.zeros(8)
        e[k % 8] = d
        q[i] = x + e
    queries.append(x.copy())
    excl.append(-1)
    # query 1: the duplicates are the nearest (no node closer): first strict minimum = lowest duplicate id
    queries.append(base + np.array([1e-8, 0, 0, 0, 0, 0, 0, 0]))
    excl.append(-1)
    # query 2: two clusters at fp32-equal distances (mirror images), the fp64 distances differ in the last bits
    x2 = rng.uniform(-1, 1, 8)
    for t, i in enumerate((300, 1200, 2046)):
        e = np.zeros(8)
        e[3] = 0.25 + (t - 1) * 1e-12
        q[i] = x2 + (e if t % 2 == 0 else -e)
    queries.append(x2)
    excl.append(1200)
    # query 3: nodes on the radius within the fp32 error band, costs tied
    x3 = rng.uniform(-1, 1, 8)
    r = 4.0
    for t, f in enumerate((1.0, 1.0 - 1e-9, 1.0 + 1e-9, 1.0 - 1e-7, 1.0 + 1e-7, 1.0 - 3e-8)):
        e = np.zeros(8)
        e[(t + 2) % 8] = r * f
        q[100 + 37 * t] = x3 + e
        cost[100 + 37 * t] = 4.5
    queries.append(x3)
    excl.append(-1)
    queries = np.array(queries)
    got = probes.tree_scan(q, cost, queries, excl, r, **MODES[mode])
    for k in range(len(queries)):
        nn, kk, lo, hi = ref_scans(q, cost, queries[k], r, excl[k])
        assert got["nearest"][k] == nn, (k, got["nearest"][k], nn)
        assert got["k"][k] == kk
        t = len(lo)
        assert list(got["lo"][k][:t]) == list(lo), (k, got["lo"][k], lo)
        assert list(got["hi"][k][:t]) == list(hi), (k, got["hi"][k], hi)
    nn1 = ref_scans(q, cost, queries[1], r, -1)[0]
    assert nn1 == min(dup)
