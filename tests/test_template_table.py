"""SURVEY §8e "feasibility precompute" (e2): the per-Solve table of template options per (shape-level, NodePool
template) that kp_solve_prepare_comm computes in shape-level row ranges, one per rank, and all-gathers; solve_kernel
reads one entry per template attempt instead of re-filtering the template's types.

CPU: the row partition, and the exchange step over a world-size-2 gloo group (each rank fills its rows of a table
with the oracle's CompatibleAvailableFilter for (NodePool requirements, pod shape) rows, pads its chunk, all-gathers;
the reassembled table equals the one a single process computes). GPU: Solve with the table equals Solve without it
(kp_overrides.template_table) and the oracle, and the single-rank collective prepare equals kp_solve."""
import os

import numpy as np
import pytest


def test_row_partition():
    from kpamd.sharding import row_range, rows_per_rank
    for n_rows in (0, 1, 5, 63, 64, 257, 1000):
        for n in (1, 2, 3, 4, 8):
            seen = []
            for r in range(n):
                lo, hi = row_range(n_rows, r, n)
                assert 0 <= lo <= hi <= n_rows and hi - lo <= rows_per_rank(n_rows, n)
                seen += list(range(lo, hi))
            assert seen == list(range(n_rows))


def _rows(catalog):
    """(NodePool requirements + pod node selector, requests) rows: config 2's pools x a few of its shapes."""
    from kpamd import synth
    prob = synth.config2(catalog, n_pods=64, seed=2)
    rows = []
    for pool in prob.nodepools:
        for sh in prob.shapes[::37]:
            reqs = list(pool.requirements) + [(k, "In", [v]) for k, v in sorted((sh.node_selector or {}).items())]
            rows.append((reqs, dict(sh.requests)))
    return rows


def _table(catalog, rows, lo, hi):
    from oracle import pyoracle
    out = np.zeros((hi - lo, len(catalog)), dtype=np.uint8)
    for i in range(lo, hi):
        kept, _ = pyoracle.compatible_available_filter(catalog, *rows[i])
        out[i - lo] = kept
    return out


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import kpamd
    from kpamd import catalog as catmod
    from kpamd.sharding import row_range, rows_per_rank
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cat = catmod.build_catalog(kpamd.load_lib())
        rows = _rows(cat)
        n, rpr = len(rows), rows_per_rank(len(rows), world)
        lo, hi = row_range(n, rank, world)
        mine = np.zeros((rpr, len(cat)), dtype=np.uint8)  # padded chunk: every rank sends rpr rows
        mine[: hi - lo] = _table(cat, rows, lo, hi)
        parts = [torch.zeros((rpr, len(cat)), dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(parts, torch.from_numpy(mine))
        full = torch.cat(parts)[:n].numpy()
        q.put((rank, full.tobytes()))
    finally:
        dist.destroy_process_group()


def test_table_allgather_gloo_world2(catalog):
    import multiprocessing as mp
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    rows = _rows(catalog)
    want = _table(catalog, rows, 0, len(rows)).tobytes()
    assert out[0] == out[1] == want
    assert np.frombuffer(want, dtype=np.uint8).any(), "some (pool, shape) row keeps types"


def _canon(res):
    return (res["placement"].tolist(),
            [(nc["nodepool"], tuple(nc["pods"]), tuple(nc["options"])) for nc in res["nodeclaims"]])


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["2", "5"])
def test_solve_with_and_without_table(ctx, catalog, cfg, ov):
    import kpamd
    from kpamd import synth
    from oracle import pyoracle
    prob = synth.config2(catalog, n_pods=3000, seed=2) if cfg == "2" else synth.config5(catalog, n_pods=4000)
    with_table = kpamd.Scheduler(ctx, prob).solve()
    ov(template_table=1)
    without = kpamd.Scheduler(ctx, prob).solve()
    assert _canon(with_table) == _canon(without)
    if cfg == "5":
        assert _canon(with_table) == _canon(pyoracle.solve(prob))


@pytest.mark.gpu
def test_prepare_comm_single_rank(ctx, catalog):
    import kpamd
    from kpamd import synth
    prob = synth.config5(catalog, n_pods=2000)
    comm = kpamd.Comm(ctx, kpamd.comm_unique_id(), 1, 0)
    try:
        plan = kpamd.Scheduler(ctx, prob).prepare(comm)
        try:
            got = plan.run(read=True)
        finally:
            plan.close()
    finally:
        comm.close()
    assert _canon(got) == _canon(kpamd.Scheduler(ctx, prob).solve())
