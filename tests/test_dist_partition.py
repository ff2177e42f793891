"""Host-side checks of the multi-GPU partition, no GPU needed: subtrees of the
assembly tree per rank, the fronts above them shared by their ranks as a 1D block-cyclic column
partition (smlu_plan_partition), each rank's device allocation (smlu_plan_rank_memory) and the
critical-path projection (smlu_plan_project)."""
import numpy as np
import pytest

import smlu
from smlu import matrices as mats


@pytest.mark.parametrize("nparts", [1, 2, 3, 4, 8])
def test_partition_owners_and_shared_fronts(nparts):
    A = mats.poisson3d(14)
    P = smlu.Plan(A)
    first, parent, level = P.supernodes()
    owner, nshared = P.partition(nparts)
    ns = len(parent)
    assert owner.shape == (ns,)
    assert owner.min() >= -1 and owner.max() < nparts
    if nparts == 1:
        assert (owner == 0).all() and nshared == 0
        return
    assert nshared == int((owner == -1).sum()) and nshared >= 1
    # every rank owns subtree work
    assert set(np.unique(owner[owner >= 0])) == set(range(nparts))
    # a shared front's parent is shared too (groups only grow towards the root), and an
    # ordinary front's parent is either on the same rank or shared
    for s in range(ns):
        p = parent[s]
        if p < 0:
            continue
        if owner[s] == -1:
            assert owner[p] == -1
        else:
            assert owner[p] in (owner[s], -1)


def test_rank_memory_splits_the_factor_store():
    A = mats.poisson3d(20)
    P = smlu.Plan(A)
    one = P.rank_memory(1, 0)
    for nparts in (2, 4):
        mem = [P.rank_memory(nparts, r) for r in range(nparts)]
        store = sum(m[0] for m in mem)
        # every factor entry lives on exactly one rank (block padding aside)
        assert 0.98 * one[0] <= store <= 1.05 * one[0] + 1e6
        assert max(m[0] for m in mem) < one[0]
        assert all(m[2] > 0 for m in mem)


def test_projection_scales_on_the_3d_model():
    A = mats.poisson3d(48)
    P = smlu.Plan(A)
    t1s = []
    for nparts in (1, 2, 4):
        t, t1 = P.project(nparts, tflops=50.0, gbs=100.0, lat_us=20.0)
        t1s.append(t1)
        if nparts == 1:
            assert t == pytest.approx(t1)
        else:
            assert t < t1
    assert len(set(round(x, 9) for x in t1s)) == 1


def test_partition_is_deterministic():
    A = mats.poisson3d(12)
    o1, k1 = smlu.Plan(A).partition(4)
    o2, k2 = smlu.Plan(A).partition(4)
    assert np.array_equal(o1, o2) and k1 == k2


def _subtree_ranks(owner, parent):
    """Ranks owning ordinary fronts in each front's subtree (children precede parents)."""
    ns = len(parent)
    R = [set() for _ in range(ns)]
    for s in range(ns):
        if owner[s] >= 0:
            R[s].add(int(owner[s]))
        if parent[s] >= 0:
            R[parent[s]] |= R[s]
    return R


@pytest.mark.parametrize("nparts", [2, 3, 4, 8])
@pytest.mark.parametrize("case", ["poisson3d", "random"])
def test_proportional_mapping_groups(nparts, case):
    # proportional mapping: sibling subtrees use disjoint ranks (their shared fronts run
    # concurrently) except for light subtrees packed whole onto one rank, so each rank works on at
    # most one shared front per tree level
    A = mats.poisson3d(20) if case == "poisson3d" else mats.random_dominant(3000, 0.003, seed=5)
    P = smlu.Plan(A)
    first, parent, level = P.supernodes()
    owner, nshared = P.partition(nparts)
    R = _subtree_ranks(owner, parent)
    kids = {}
    for s in range(len(parent)):
        if parent[s] >= 0:
            kids.setdefault(int(parent[s]), []).append(s)
    for s in np.flatnonzero(owner == -1):
        ch = kids.get(int(s), [])
        for i in range(len(ch)):
            for j in range(i + 1, len(ch)):
                # siblings share a rank only when one of them is packed whole onto it
                if R[ch[i]] & R[ch[j]]:
                    assert min(len(R[ch[i]]), len(R[ch[j]])) == 1, (s, ch[i], ch[j])
    for lv in np.unique(level):   # shared fronts of one tree level never share a rank
        seen = set()
        for s in np.flatnonzero((owner == -1) & (level == lv)):
            assert not (seen & R[s]), lv
            seen |= R[s]


def test_projection_eight_ranks_beats_four():
    # the proportional mapping keeps scaling from 4 to 8 ranks (bin-packing regressed from 4 to 8
    # ranks).  With the calibrated model (round 5: level-batched fronts, 0.32 ms per level, 80 us per
    # panel step) 64^3 is latency-bound, so the gain is small but must stay monotone.
    P = smlu.Plan(mats.poisson3d(64))
    sp = {k: P.project(k, tflops=52.0, gbs=100.0, lat_us=20.0) for k in (2, 4, 8)}
    s = {k: v[1] / v[0] for k, v in sp.items()}
    assert 1.0 < s[2] < s[4] < s[8], s


def test_projection_calibrated_one_gpu():
    # N = 1 of the model against the measured one-GPU refactor (round 5, profiles/r05): C2 2D 512^2
    # 7.9 ms, 3D 64^3 (smaller fronts, the per-level latency dominates); the 128^3 point (0.49 s) is
    # checked by tools/partition_projection.py (its 10 s analysis is too long for this suite)
    t, t1 = smlu.Plan(mats.poisson2d(512)).project(1)
    assert t == pytest.approx(t1)
    assert 5e-3 <= t1 <= 11e-3, t1
