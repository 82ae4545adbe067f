"""Shared fixtures.  `-m "not gpu"` runs on any host (oracle vs golden vectors,
host logic, ABI); `-m gpu` needs a gfx950 device and calls the HIP library
through its C ABI."""
import glob
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "sparse-matrix-multiplication-benchmark_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: full BASELINE-size cases")
    config.addinivalue_line("markers", "config_parity: the BASELINE-config / golden-fixture parity checks; "
                                       "collected first so that a -x stop elsewhere never hides a config")
    config.addinivalue_line("markers", "run_last: long end-to-end runs (the reference's own harness), collected "
                                       "after everything else so a -x stop there hides no parity test")


def pytest_collection_modifyitems(session, config, items):
    """Run every `config_parity` test before everything else and every
    `run_last` test after everything else (stable order inside each group):
    the driver runs `pytest -x`, and the per-row parity verdict must not
    depend on an unrelated test, or on a long end-to-end run, further up."""
    first = [it for it in items if it.get_closest_marker("config_parity")]
    last = [it for it in items if it.get_closest_marker("run_last") and not it.get_closest_marker("config_parity")]
    rest = [it for it in items if not it.get_closest_marker("config_parity") and not it.get_closest_marker("run_last")]
    items[:] = first + rest + last


def load_golden(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    d["meta"] = json.loads(bytes(d["meta"]).decode())
    return d


GOLDEN_NAMES = sorted(
    os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz")) if "sparseformat" not in p
)


BCSR_GOLDEN = os.path.join(GOLDEN, "bcsr")
BCSR_GOLDEN_NAMES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(BCSR_GOLDEN, "*.npz")))


def load_bcsr_golden(name):
    z = np.load(os.path.join(BCSR_GOLDEN, name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    d["meta"] = json.loads(bytes(d["meta"]).decode())
    return d


def bcsr_of(g):
    """The reference's bcsr_from_dense output stored in a BCSR fixture."""
    import pyoracle

    K, N = g["Wd"].shape
    r, c = int(g["r"]), int(g["c"])
    return pyoracle.BCSR(r, c, K // r, N // c, g["rs"], g["ci"], g["vals"])


@pytest.fixture(scope="session")
def oracle():
    import pyoracle

    return pyoracle.load_oracle()


@pytest.fixture(scope="session")
def golden_names():
    return GOLDEN_NAMES


def tcsc_of(g):
    import pyoracle

    K, N = g["Wd"].shape
    return pyoracle.TCSC(K, N, g["csp"], g["csn"], g["rip"], g["rin"])

# paths for spawned worker processes (they re-import without conftest's sys.path edits)
PKG_DIR_FOR_WORKERS = PKG
ORACLE_DIR_FOR_WORKERS = os.path.join(ROOT, "oracle")
