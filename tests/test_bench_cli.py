"""bench.py's multi-rank launch on the GPU box (-m gpu): a plain
`python bench.py --gpus 2` starts torchrun as a child and the JSON line reports
the two ranks. The rehearsal uses the gloo backend with both ranks on the one
GPU (the box has one); the RCCL fan-in itself is covered by
test_gpu_frames.py::test_rccl_rank_group_equals_single_dispatch and the
driver's 8-GPU run."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("mode", ["strong", "weak"])
def test_gpus_2_from_a_plain_invocation(mode):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--mode", mode, "--steps", "3", "--warmup", "1", "--no-cpu", "--config", "2"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["ranks_seen"] == 2
    assert out["scaling"] == ("strong" if mode == "strong" else "weak")
    assert out["value"] > 0 and out["roofline"]["frac"] < 1


def test_strong_mode_over_rt_group_one_rank():
    """The N > 1 default's code path (rt_group, ncclCommInitRank, the grouped
    ncclSend/ncclRecv fan-in, unstripe) with one rank: the 1-GPU rehearsal of what the driver's
    8-GPU run measures."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--mode", "strong", "--steps", "5",
                        "--warmup", "2", "--no-cpu"], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    assert len(lines) == 1, lines[:5]  # stdout is the JSON line alone (RCCL's banner goes to stderr)
    out = json.loads(lines[0])
    assert out["mode"] == "strong" and out["scaling"] == "strong" and out["n_gpus"] == 1
    assert out["gather"].startswith("rt_group") and out["frames_in_flight"] >= 2
    assert out["value"] > 0
