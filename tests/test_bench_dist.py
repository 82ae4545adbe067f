"""bench.py's multi-rank path on the GPU box: two ranks launched as the
driver launches N ranks (torch.distributed.run, 127.0.0.1), sharing the one
GPU over gloo (RCCL refuses two ranks on one device).  Checks the contract
line that only rank 0 prints: n_gpus, the summed work over the max-over-ranks
time, both ranks' validation, and the column/row shard layouts."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--config", "2", "--dist-backend", "gloo",
           "--no-cpu-baseline"] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    return lines[0]


def test_two_ranks_default_is_cfg_column_split():
    """The N>1 default is the north star's layout: the config itself (here
    cfg 2) split over the ranks by output columns (strong scaling), plus the
    row split of the same config as `alt_shard`."""
    d = _run([])
    cfg = d["config"]
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert cfg["columns_per_gpu"] == 2048 and cfg["rows_per_gpu"] == 1024 and cfg["N"] == 4096
    assert "column-shard x2 (strong)" in cfg["parallelism"]
    alt = d["alt_shard"]
    assert alt["shard"] == "rows" and alt["rows_per_gpu"] == 512 and alt["columns_per_gpu"] == 4096
    assert alt["value"] > 0
    assert d["validation"]["worst_err_over_bound"] <= 1.0


def test_two_ranks_weak_scaling():
    d = _run(["--scaling", "weak"])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["steps"] == 3
    cfg = d["config"]
    per_rank = 1024 * cfg["nnz_per_gpu"] + 1024 * 4096  # add-ops of rank 0's block per step
    # value = both ranks' add-ops per step (rank 1's W has its own seed) / the slower rank's step time
    total_per_step = d["value"] * 1e9 * d["ms_per_step"] * 1e-3
    assert 1.95 < total_per_step / per_rank < 2.05
    assert d["validation"]["worst_err_over_bound"] <= 1.0


@pytest.mark.parametrize("shard", ["cols", "rows"])
def test_two_ranks_strong_scaling(shard):
    d = _run(["--scaling", "strong", "--shard", shard])
    cfg = d["config"]
    assert d["scaling"] == "strong"
    if shard == "cols":
        assert cfg["columns_per_gpu"] == 2048 and cfg["rows_per_gpu"] == 1024
    else:
        assert cfg["columns_per_gpu"] == 4096 and cfg["rows_per_gpu"] == 512
    assert d["validation"]["worst_err_over_bound"] <= 1.0
