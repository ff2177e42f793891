"""The collective schedule of the multi-GPU partition, built on the host for every rank (no device):
C3 (3D Poisson 128^3) and C4 (256^3, BASELINE configs[3]) at 8 ranks, the driver's scaling runs.

Each rank's schedule comes from the same code that smlu_dist_create runs (smlu_plan_rank_schedule:
build_schedule without the uploads).  The checks are the ones a deadlock or a mismatched transfer
would break on the first 8-GPU run:

* pairing: for every ordered rank pair (a, b), the sizes of a's sends to b, in a's step order,
  equal the sizes of b's receives from a, in b's step order (RCCL matches point-to-point
  transfers between two ranks in issue order);
* broadcasts: every member of a broadcast group runs a broadcast step with the same root, the
  same byte count and the same group, in the same position of its sequence of that group's steps;
* progress: executing every rank's steps in order, where a step completes once each of its
  transfers has been posted by both sides (a rendezvous model: no transfer is buffered), the
  factor, forward and backward sequences all run to the end -- no cyclic wait;
* memory: every rank's device allocation (factor store, scratch, staging, schedule buffers)
  fits one MI355X's 288 GB.

Reference intent: the MPI rank split of src/SharedMemSparseLU.jl:107,128."""
import collections
import time

import numpy as np
import pytest

import smlu
from smlu import matrices as mats

HBM_BYTES = 288e9


def transfers(step, me):
    """(sends, recvs) of one step: lists of (peer, bytes), bytes > 0 (rccl_bcast: root -> members)."""
    if step["type"] == "bcast":
        if step["bytes"] <= 0:
            return [], []
        if me == step["root"]:
            return [(g, step["bytes"]) for g in step["group"] if g != me], []
        return [], [(step["root"], step["bytes"])]
    sends = [(p, s) for p, s, _ in step["peers"] if s > 0]
    recvs = [(p, r) for p, _, r in step["peers"] if r > 0]
    return sends, recvs


def check_collective(scheds, nranks):
    """Pairing, broadcast agreement and progress of every sequence; returns per-sequence totals."""
    totals = {}
    for seq in ("fac", "fwd", "bwd"):
        steps = [[s for s in scheds[r] if s["seq"] == seq] for r in range(nranks)]
        # pairing per ordered pair, in issue order
        sent = collections.defaultdict(list)
        recv = collections.defaultdict(list)
        for r in range(nranks):
            for st in steps[r]:
                s, v = transfers(st, r)
                for p, b in s:
                    sent[(r, p)].append(b)
                for p, b in v:
                    recv[(p, r)].append(b)
        for key in set(sent) | set(recv):
            assert sent[key] == recv[key], (seq, key, len(sent[key]), len(recv[key]))
        # broadcasts: the k-th broadcast of a group is the same step on every member
        byg = collections.defaultdict(dict)
        for r in range(nranks):
            for st in steps[r]:
                if st["type"] == "bcast":
                    assert r in st["group"] and st["root"] in st["group"]
                    byg[tuple(st["group"])].setdefault(r, []).append((st["root"], st["bytes"]))
        for g, per in byg.items():
            assert set(per) == set(g), (seq, g, sorted(per))
            first = per[g[0]]
            for r in g:
                assert per[r] == first, (seq, g, r)
        # progress: rendezvous execution of all ranks' sequences
        pos = [0] * nranks
        done = [set() for _ in range(nranks)]   # completed transfer ids of the current step
        ordinal = collections.Counter()          # per (a, b): transfers posted so far by the sender
        ordinal_r = collections.Counter()        # ... and by the receiver
        post = [None] * nranks

        def posts(r):
            """Transfer ids of rank r's current step: ('s'|'r', a, b, k) with the per-pair ordinal."""
            if post[r] is None:
                s, v = transfers(steps[r][pos[r]], r)
                ids = []
                for p, _ in s:
                    ids.append(("s", r, p, ordinal[(r, p)]))
                    ordinal[(r, p)] += 1
                for p, _ in v:
                    ids.append(("r", p, r, ordinal_r[(p, r)]))
                    ordinal_r[(p, r)] += 1
                post[r] = ids
            return post[r]

        moved, nsteps = 0, sum(len(x) for x in steps)
        while True:
            progress = False
            active = {}
            for r in range(nranks):
                if pos[r] < len(steps[r]):
                    for t in posts(r):
                        active[t] = r
            for t, r in active.items():
                kind, a, b, k = t
                other = ("r", a, b, k) if kind == "s" else ("s", a, b, k)
                if other in active:
                    done[r].add(t)
            for r in range(nranks):
                while pos[r] < len(steps[r]) and set(posts(r)) <= done[r]:
                    done[r] -= set(post[r])
                    post[r] = None
                    pos[r] += 1
                    moved += 1
                    progress = True
                    if pos[r] < len(steps[r]):
                        posts(r)
            if all(pos[r] == len(steps[r]) for r in range(nranks)):
                break
            assert progress, (seq, "cyclic wait", pos, [len(x) for x in steps])
        assert moved == nsteps
        totals[seq] = (nsteps, sum(sum(v) for v in sent.values()))
    return totals


def build_all(N, nranks, workers=3):
    """Every rank's schedule, `workers` at a time (the library call releases the GIL; each call
    holds its own copy of the plan: 256^3 about 6 GB)."""
    from concurrent.futures import ThreadPoolExecutor
    A = mats.poisson3d(N)
    P = smlu.Plan(A, ordering="nd")
    del A
    with ThreadPoolExecutor(max_workers=workers) as ex:
        out = list(ex.map(lambda r: P.rank_schedule(nranks, r), range(nranks)))
    return P, [o[0] for o in out], [o[1] for o in out]


@pytest.mark.parametrize("N", [40, 128, 256])
def test_eight_rank_schedule_pairs_and_fits(N):
    t0 = time.time()
    P, scheds, infos = build_all(N, 8)
    totals = check_collective(scheds, 8)
    # the partition really shares the top fronts and moves data in every sequence
    assert sum(i["shared_fronts"] for i in infos) > 0
    for seq in ("fac", "fwd", "bwd"):
        assert totals[seq][0] > 0 and totals[seq][1] > 0, (seq, totals[seq])
    for r, i in enumerate(infos):
        assert i["device_bytes"] <= HBM_BYTES, (r, i["device_bytes"] / 1e9)
        assert i["device_bytes"] >= i["store_bytes"] + i["scratch_bytes"]
    # the per-rank store + scratch agree with the partition's memory query
    for r in (0, 7):
        st, sc, _ = P.rank_memory(8, r)
        # (the device store is padded by 64 columns of the tallest front for k_urows' reads)
        assert st <= infos[r]["store_bytes"] <= 1.02 * st + 4e6 and sc == infos[r]["scratch_bytes"]
    mx = max(i["device_bytes"] for i in infos) / 1e9
    print(f"\n{N}^3 / 8 ranks: max device {mx:.1f} GB per rank, steps/bytes {totals}, "
          f"{time.time() - t0:.0f} s")


def test_checker_catches_mismatches():
    # the checker itself: a wrong byte count, a missing receive and a crossed order all fail
    good = [[{"seq": "fac", "type": "exchange", "peers": [(1, 8, 0)]},
             {"seq": "fac", "type": "exchange", "peers": [(1, 0, 16)]}],
            [{"seq": "fac", "type": "exchange", "peers": [(0, 0, 8)]},
             {"seq": "fac", "type": "exchange", "peers": [(0, 16, 0)]}]]
    check_collective(good, 2)
    bad_bytes = [list(good[0]), [{"seq": "fac", "type": "exchange", "peers": [(0, 0, 9)]}, good[1][1]]]
    with pytest.raises(AssertionError):
        check_collective(bad_bytes, 2)
    crossed = [[good[0][1], good[0][0]], [good[1][0], good[1][1]]]   # rank 0 receives before it sends
    with pytest.raises(AssertionError):
        check_collective(crossed, 2)
    bc = [[{"seq": "fac", "type": "bcast", "root": 0, "bytes": 8, "group": [0, 1]}],
          [{"seq": "fac", "type": "bcast", "root": 0, "bytes": 16, "group": [0, 1]}]]
    with pytest.raises(AssertionError):
        check_collective(bc, 2)
