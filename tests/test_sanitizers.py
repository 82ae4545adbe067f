"""Host code of libtcsc_amd.so under AddressSanitizer and ThreadSanitizer
("-fsanitize=address for host code"; GPU sanitizers are not
available).  `make asan tsan` instruments the host-side sources (the format
builders, the host API with its per-device copy pools and fingerprint pool,
the BCSR host API) and builds tests/native/host_selftest.cpp against each
build; the self-test drives the pools from 8 threads at once and checks its
results.  A sanitizer report makes the binary exit non-zero.  No GPU: the
drop-in calls take their no-device error path."""
import os
import subprocess

import pytest

from conftest import PKG


@pytest.fixture(scope="module")
def built():
    subprocess.check_call(["make", "-s", "-C", PKG, "-j8", "asan", "tsan"])


@pytest.mark.parametrize("san", ["asan", "tsan"])
def test_host_selftest_under_sanitizer(built, san):
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=0:exitcode=23"
    env["TSAN_OPTIONS"] = "exitcode=23:halt_on_error=1"
    env["HIP_VISIBLE_DEVICES"] = ""  # the no-device path, also on a GPU host
    r = subprocess.run([os.path.join(PKG, "bin", f"host_selftest_{san}")], capture_output=True, text=True,
                       timeout=300, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "host_selftest: OK" in out
    assert "Sanitizer" not in out, out[-4000:]
