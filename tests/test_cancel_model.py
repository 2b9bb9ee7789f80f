"""The cancel plan's formula on the CPU (tools/flow_cancel_model.py, plan_book_q): a DEL of
maker m removes clamp(depth_s - Q, 0, v_m), Q from the segment's records alone.  Replayed per
book over several batches (old makers included) and compared with the C oracle: every cancel's
volume, every level's final depth and side set."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import flow_cancel_model as M  # noqa: E402


@pytest.mark.parametrize("seed,n_sym,aggr", [(1, 6, 0.1), (7, 2, 0.1), (3, 12, 0.02)])
def test_q_formula_exact_vs_oracle(seed, n_sym, aggr):
    M.check(n_sym=n_sym, batch=2500, nbatch=3, seed=seed, aggr=aggr, plan=M.plan_book_q)
