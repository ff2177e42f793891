"""Host-side checks of the multi-GPU partition: proportional mapping of the
assembly tree onto ranks (smlu_plan_partition), no GPU needed."""
import numpy as np
import pytest

import smlu
from smlu import matrices as mats


def _tree(P):
    first, parent, level = P.supernodes()
    return first, parent, level


@pytest.mark.parametrize("nparts", [1, 2, 3, 4, 8])
def test_partition_covers_tree_and_exchange_levels(nparts):
    A = mats.poisson3d(14)
    P = smlu.Plan(A)
    first, parent, level = _tree(P)
    owner, xl = P.partition(nparts)
    ns = len(parent)
    assert owner.shape == (ns,)
    assert owner.min() >= 0 and owner.max() < nparts
    if nparts == 1:
        assert (owner == 0).all() and xl.size == 0
        return
    # every rank gets work
    assert set(np.unique(owner)) == set(range(nparts))
    # exchange levels are exactly the levels of fronts with a child on another rank
    expect = sorted({int(level[parent[s]]) for s in range(ns)
                     if parent[s] >= 0 and owner[parent[s]] != owner[s]})
    assert list(xl) == expect
    # a subtree owned by a single rank stays on it: below the exchange fronts ownership is
    # inherited, i.e. a child differs from its parent only where the parent's rank set splits
    crossings = sum(1 for s in range(ns) if parent[s] >= 0 and owner[parent[s]] != owner[s])
    assert crossings >= nparts - 1


def test_partition_balances_subtree_work():
    A = mats.poisson3d(20)
    P = smlu.Plan(A)
    w = P.front_flops()
    owner, _ = P.partition(4)
    first, parent, level = _tree(P)
    # work of the fronts below the top separators, per rank: within a factor 2.5 of the mean
    top = {int(s) for s in range(len(parent)) if parent[s] >= 0 and owner[parent[s]] != owner[s]}
    load = np.zeros(4)
    for s in range(len(parent)):
        load[owner[s]] += w[s]
    assert load.max() <= 2.5 * load.mean(), load
    assert len(top) >= 3


def test_partition_is_deterministic():
    A = mats.poisson3d(12)
    o1, x1 = smlu.Plan(A).partition(4)
    o2, x2 = smlu.Plan(A).partition(4)
    assert np.array_equal(o1, o2) and np.array_equal(x1, x2)
