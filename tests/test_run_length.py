"""The fast lane's run-length commit. In Solves whose queue runs of one shape-level
are the rule (deployments created in bursts: kp_solve picks the continuation variant when most queue neighbours share
their shape; kp_overrides.fast_lane forces either variant), the fast lane commits the next k pods of a run onto the NodeClaim the run
is filling in one step when, for each of them one at a time, the reference would do the same: sort.Slice leaves the
NodeClaim in place (the next entry's len(Pods) is not below its own), the first-fit scan starts at it, and Fits over
its remaining types holds with every requested resource under the threshold value it last passed. Parity: device ==
the one-pod-at-a-time oracle (which never batches), on burst problems where runs are cut by every one of those
conditions, with the variant forced on and off; the stats count the batched pods."""
import pytest


def _solve(ctx, prob, cont, ov):
    import kpamd
    ov(fast_lane=2 if cont else 1)
    return kpamd.Scheduler(ctx, prob).solve()


@pytest.mark.gpu
@pytest.mark.parametrize("n_pods,seed", [(3_000, 5), (12_000, 6), (20_000, 2)])
def test_burst_run_length_equals_oracle(ctx, catalog, ov, n_pods, seed):
    from kpamd import synth
    from oracle import pyoracle
    from test_gpu_parity import check_same
    prob = synth.config2(catalog, n_pods=n_pods, seed=seed, burst=True)
    want = pyoracle.solve(prob)
    on = _solve(ctx, prob, True, ov)
    check_same(on, want)
    assert on["stats"]["run_length_pods"] > n_pods // 4, on["stats"]["run_length_pods"]
    off = _solve(ctx, prob, False, ov)
    check_same(off, want)
    assert off["stats"]["run_length_pods"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_forced_run_length_on_random_problems(ctx, catalog, ov, seed):
    """Limits, taints, minValues, relaxations (re-queued pods: lastLen), several catalogues: the continuation variant
    forced on equals the oracle."""
    from kpamd import synth
    from oracle import pyoracle
    from test_gpu_parity import check_same
    prob = synth.random_problem(catalog, 1600 + seed, n_types=150, n_pods=600, n_pools=3, n_shapes=6)
    check_same(_solve(ctx, prob, True, ov), pyoracle.solve(prob))


@pytest.mark.gpu
def test_run_cut_by_thresholds_and_ties(ctx, catalog, ov):
    """Runs of identical pods onto NodeClaims whose remaining types shrink as the requests cross allocatable values
    (every m5 size), and two shape-levels alternating in blocks so NodeClaims tie on len(Pods) (sort.Slice moves)."""
    import numpy as np
    from kpamd import synth
    from kpamd.model import NodePool, PodShape, Problem
    from oracle import pyoracle
    from test_gpu_parity import check_same
    pool = NodePool("m5", 0, 0, [("karpenter.k8s.aws/instance-family", "In", ["m5"]),
                                 ("karpenter.sh/capacity-type", "In", ["on-demand"])])
    shapes = [PodShape(synth.req_res(250, 512)), PodShape(synth.req_res(250, 512), tolerations=[("x", "Exists", "", "")]),
              PodShape(synth.req_res(1000, 2048))]
    blocks = [0] * 40 + [1] * 40 + [0] * 25 + [2] * 30 + [1] * 60 + [0] * 100 + [2] * 10 + [1] * 5
    shape = np.asarray(blocks, dtype=np.uint32)
    creation = (1_750_000_000 + np.arange(len(blocks))).astype(np.int64)
    uid = np.arange(1, len(blocks) + 1, dtype=np.uint64)
    prob = Problem([catalog], [pool], shapes, shape, creation, uid, name="run-cuts")
    want = pyoracle.solve(prob)
    got = _solve(ctx, prob, True, ov)
    check_same(got, want)
    assert got["stats"]["run_length_pods"] > 0
