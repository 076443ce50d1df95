"""The config-4 sweep's answer checked against the oracle: the bench's whole 1M-subset sweep (kp_consolidate_argmin:
device simulation + device argmax) on the 10k-node cluster, then
  * the returned best subset re-simulated by the oracle: identical computeConsolidation record, and the best's
    savings equal the maximum over the device's per-subset results of its chunk (a second, read-all launch);
  * firstNConsolidationOption's winner (the binary search replayed over the device's prefix results) equal to the
    same search replayed over the oracle's prefix records committed in tests/golden/fullsize_digests.json.
The upstream semantics are SURVEY a19 (computeConsolidation, filterByPrice, firstNConsolidationOption)."""
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

N_SUBSETS = 1_000_000


def test_sweep_subsets_split_invariant():
    """The sweep's subsets do not depend on how chunks are split over ranks (CPU)."""
    from kpamd import disruption
    cands = np.arange(300, dtype=np.uint32) * 3
    n = 3 * disruption.SWEEP_CHUNK // 2
    offs, nodes, base = disruption.sweep_subsets(cands, n)
    assert base == 0 and len(offs) == n + 1
    o1, n1, b1 = disruption.sweep_subsets(cands, n, 1, 2)
    assert b1 == disruption.SWEEP_CHUNK
    lo = offs[b1]
    assert (nodes[lo:lo + len(n1)] == n1).all() and (o1 == offs[b1:] - lo).all()
    sizes = np.diff(offs)
    assert sizes.min() >= 1 and sizes.max() <= 100 and set(np.unique(nodes)) <= set(cands.tolist())


@pytest.mark.gpu
def test_sweep_best_and_first_n_vs_oracle(ctx, catalog):
    import kpamd
    import make_fullsize_digests as mk
    from kpamd import disruption, synth
    from oracle import pyoracle
    cl = synth.config4(catalog, n_nodes=10_000, seed=4)
    offs, nodes, _ = disruption.sweep_subsets(cl.candidates, N_SUBSETS)
    plan = kpamd.ClusterPlan(ctx, cl)
    try:
        choice, _ = disruption.sweep(plan, offs, nodes)
        best = choice["subset"]
        assert best >= 0 and sum(choice["counts"]) == N_SUBSETS
        sub = [int(x) for x in nodes[offs[best]:offs[best + 1]]]
        # the argmax: the best's chunk simulated again with every result read back
        c = best // disruption.SWEEP_CHUNK
        lo, hi = c * disruption.SWEEP_CHUNK, min(N_SUBSETS, (c + 1) * disruption.SWEEP_CHUNK)
        co = (offs[lo:hi + 1] - offs[lo]).astype(np.uint32)
        _, res, _ = plan.argmin(co, nodes[offs[lo]:offs[hi]], base_index=lo, read_all=True)
        # firstNConsolidationOption over the device's prefix results
        mids = disruption.MultiNodeConsolidation.search_prefixes(len(cl.candidates))
        pres, _ = plan.simulate([list(cl.candidates[:m + 1]) for m in mids])
    finally:
        plan.close()
    want, _ = pyoracle.simulate_batch(cl, [sub])
    assert mk.sim_record(choice["result"]) == mk.sim_record(want[0])
    nonnoop = res["savings"][res["decision"] != 0]
    assert choice["result"]["savings"] == nonnoop.max()
    assert best - lo == int(np.nonzero((res["decision"] != 0) & (res["savings"] == nonnoop.max()))[0][0])
    digests = json.load(open(os.path.join(HERE, "golden", "fullsize_digests.json")))["config4-10000"]["prefixes"]
    dec = lambda rec: {"decision": rec[0], "n_options": rec[5]}
    hit_dev = disruption.MultiNodeConsolidation.replay(len(cl.candidates), dict(zip(mids, pres)))
    hit_ora = disruption.MultiNodeConsolidation.replay(len(cl.candidates), dict(zip(mids, [dec(r) for r in digests])))
    assert hit_dev is not None and hit_ora is not None and hit_dev[0] == hit_ora[0]
    assert mk.sim_record(hit_dev[1]) == digests[mids.index(hit_ora[0])]
