"""HIP engine (MI355X) — the stream layouts real hosts get, exact against the C oracle at bench
size (tests/layout_check.py says what each leg runs).

* the four-queue layout in a fresh process whose HIP runtime really has 4 hardware queues
  (GPU_MAX_HW_QUEUES=4, what a host that does not set the variable gets): started before this
  process touches the GPU (the file name sorts first); since round 6 it plans the hottest book
  early on a fourth stream of its own;
* the same layout chosen by gome_config.hw_queues = 4 in this process (16 real queues: the layout's
  own event dependencies, without the serialisation a shared queue adds);
* no reserved plan CUs (gome_config.plan_cus < 0: the layout of a host beside RCCL);
* the default layout with the early plan and admission ahead switched off by flag.
"""
import json
import os
import subprocess
import sys

import pytest

from gome_amd.abi import GOME_FLAG_NO_ADM_AHEAD, GOME_FLAG_NO_EARLY

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _no_early(res):
    return all(x == 0 for leg in res.values() if isinstance(leg, dict) for x in leg.get("early", []) + leg.get("adm_ahead", []))


def _four_queue(res):
    """The four-queue layout (round 6): the early plan on its own fourth stream, no admission ahead."""
    return (sum(res["config3_device"]["early"]) >= 2 and sum(res["config3_host"]["early"]) >= 1 and
            all(x == 0 for leg in res.values() if isinstance(leg, dict) for x in leg.get("adm_ahead", [])))


def test_four_hw_queues_in_a_fresh_process():
    env = dict(os.environ, GPU_MAX_HW_QUEUES="4", GOME_HW_QUEUES="4", OMP_NUM_THREADS="4")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "layout_check.py")], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["hw_queues"] == 4 and res["GPU_MAX_HW_QUEUES"] == "4", res
    assert _four_queue(res), res
    assert min(res["config4_device"]["flow_cancels"]) > 100000, res


def test_four_queue_layout_by_config():
    from tests.layout_check import check_layout
    res = check_layout(dict(hw_queues=4), "hw_queues=4")
    assert _four_queue(res), res


def test_no_plan_cus_layout():
    from tests.layout_check import check_layout
    res = check_layout(dict(plan_cus=-1), "plan_cus=-1")
    assert sum(res["config3_device"]["early"]) >= 1, res   # (the early plan still runs)
    assert sum(res["config4_device"]["adm_ahead"]) >= 1, res


def test_default_layout_without_early_and_ahead():
    from tests.layout_check import check_layout
    res = check_layout(dict(flags=GOME_FLAG_NO_EARLY | GOME_FLAG_NO_ADM_AHEAD), "no early / ahead")
    assert _no_early(res), res
