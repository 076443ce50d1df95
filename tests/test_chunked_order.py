"""The spilled newNodeClaims order (solve_kernel past its LDS sort capacity) against the oracle, bit-exact.

Past kp_overrides.sort_capacity NodeClaims the sorted order leaves LDS for the chunked order (blocks of <= 64 NodeClaims in global
memory, directory in LDS); when the directory is full it continues on the flat global arrays. The LDS capacity is
forced small here (kp_overrides.sort_capacity) so that every path runs on small batches: stable moves within a chunk and across
chunks, appended NodeClaims, chunk splits and emptied chunks, the literal pdqsort (12 < n < 50) with its rebuild,
the chunk dead marks, and the fallback to the flat order mid-Solve (kp_overrides.chunk_capacity lowers the directory's size).
"""
import pytest

from test_gpu_parity import check_same, run_both

pytestmark = pytest.mark.gpu

MODE_FLAT, MODE_LDS, MODE_CHUNKED = 0, 1, 2


def _solve(ctx, prob, ov, sort_cap, chk_maxc=None):
    # chunk_capacity 0 is the full directory; the flat-order case (no chunks) asks for -1 -> clamped to 0 chunks
    ov(sort_capacity=sort_cap, chunk_capacity=0 if chk_maxc is None else (chk_maxc if chk_maxc > 0 else -1))
    got, want = run_both(ctx, prob)
    check_same(got, want)
    return got["stats"]["order_chunks"], len(got["nodeclaims"])


@pytest.mark.parametrize("sort_cap", [1, 5, 9])  # (config 2 at 2.5k pods makes 11 NodeClaims)
def test_chunked_config2(ctx, catalog, ov, sort_cap):
    from kpamd import synth
    oc, n = _solve(ctx, synth.config2(catalog, n_pods=2500, seed=11), ov, sort_cap)
    assert n > sort_cap and oc[4] == MODE_CHUNKED
    assert oc[3] >= 1  # built at the spill (and rebuilt after each literal pdqsort)


@pytest.mark.parametrize("seed,sort_cap", [(5, 64), (6, 64), (5, 8)])
def test_chunked_config5_splits(ctx, catalog, ov, seed, sort_cap):
    """config 5 (20 pools, GPU/Neuron pools): hundreds of NodeClaims whose stable moves cross chunks, split full ones
    and empty others; from 8 NodeClaims on, the literal pdqsort (12 < n < 50) and its rebuilds as well."""
    from kpamd import synth
    oc, n = _solve(ctx, synth.config5(catalog, n_pods=4000, seed=seed), ov, sort_cap)
    assert oc[4] == MODE_CHUNKED and n > 64
    assert oc[1] > 0 and oc[2] > 0, oc  # splits and emptied chunks both happened


def test_flat_order_when_chunks_off(ctx, catalog, ov):
    from kpamd import synth
    oc, n = _solve(ctx, synth.config2(catalog, n_pods=2500, seed=11), ov, 5, chk_maxc=0)
    assert oc[4] == MODE_FLAT and n > 5


def test_chunk_directory_full_falls_back(ctx, catalog, ov):
    """A directory of 3 chunks overflows mid-Solve: the order continues on the flat global arrays."""
    from kpamd import synth
    oc, n = _solve(ctx, synth.config5(catalog, n_pods=3000, seed=5), ov, 40, chk_maxc=3)
    assert oc[4] == MODE_FLAT and n > 3 * 64, (oc, n)


def test_lds_order_below_capacity(ctx, catalog, ov):
    from kpamd import synth
    oc, n = _solve(ctx, synth.config2(catalog, n_pods=400, seed=7), ov, 8192)
    assert oc[4] == MODE_LDS and oc[3] == 0


def test_chunked_topology(ctx, catalog, ov):
    """Spread owners (no dead marks: their failures depend on the counts) on the chunked order."""
    from kpamd import synth
    prob = synth.config3(catalog, n_pods=3000, n_deployments=40, n_existing=60)
    oc, n = _solve(ctx, prob, ov, 16)
    assert oc[4] == MODE_CHUNKED and n > 16


@pytest.mark.parametrize("limit_div,sort_cap", [(300, 8), (500, 8), (500, 64)])
def test_chunked_memo_runs(ctx, catalog, ov, limit_div, sort_cap):
    """Binding limits on the chunked order: many pods fail every placement, so the fast lane's unschedulable memo takes
    runs of them at once (window entries on lanes), up to the pop that ends the Solve once a pass makes no progress, with
    the queue shorter than the 64-entry window at the end (its ring wraps onto re-pushed entries)."""
    from kpamd import synth
    prob = synth.config5(catalog, n_pods=4000, seed=5, limit_div=limit_div)
    oc, n = _solve(ctx, prob, ov, sort_cap)
    assert oc[4] == MODE_CHUNKED and n > sort_cap
