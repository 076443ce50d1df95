"""Row-range sharding used by the collectives behind the C ABI.

kp_solve_prepare_comm splits the (shape-level x NodePool template) options table by shape-level rows: every rank
gets ceil(rows / ranks) rows (the last ranks may get fewer or none) and contributes a padded chunk of exactly that
many rows to one ncclAllGather, so the gathered buffer is the table in row order (kp_host.cpp, SolvePrepare).
"""


def rows_per_rank(n_rows, n_ranks):
    return (n_rows + n_ranks - 1) // n_ranks if n_ranks > 0 else 0


def row_range(n_rows, rank, n_ranks):
    """[lo, hi) rows computed by `rank` (may be empty)."""
    rpr = rows_per_rank(n_rows, n_ranks)
    return min(n_rows, rank * rpr), min(n_rows, (rank + 1) * rpr)
