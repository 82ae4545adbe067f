"""The reference's own harness, unmodified, on the GPU (the north star's
"drops in under the existing main.cpp").

oracle/_ref/main_amd is /root/reference/main.cpp compiled in place against
its own headers and linked against libtcsc_amd.so instead of sparse/tcsc.c +
dense/dense.c (oracle/Makefile target `harness`; the g++-mangled names come
from csrc/tcsc_cxx_abi.cpp).  For each of its five cases (main.cpp:258-264)
it validates every tcsc_sgemm_* variant with its own compare() (abs tol 1e-4,
dense.c:42-59) against its own CPU gemm_basic and exit(1)s on a mismatch
(main.cpp:299-368), then times all six functions with its cycle counter.

The test runs it as a child process and requires "[OK] All validation tests
passed!" for all five cases, with no "[ERROR]" line and no early exit.  Case
5's timing leg (main.cpp:376, the naive CPU gemm_basic at 256x1024x4096 under
REP=50) takes minutes, so the child is stopped once case 5 has validated; the
four complete timing tables before it are parsed (harness/out2csv.py) to
check that every legacy line is there.  The output is kept in
gpurun_out/main_amd_out.txt when that directory exists (profiles/ holds a
committed copy per round).
"""
import os
import signal
import subprocess
import sys
import time

import pytest

from conftest import PKG, ROOT

pytestmark = [pytest.mark.gpu, pytest.mark.config_parity]

BIN = os.path.join(ROOT, "oracle", "_ref", "main_amd")
CASES = [(1, 512, 2048), (1, 1024, 4096), (1, 2048, 8192), (256, 512, 2048), (256, 1024, 4096)]
OK = "[OK] All validation tests passed!"


def test_reference_main_cpp_validates_every_case():
    assert os.path.exists(BIN), "oracle/_ref/main_amd missing: build it with `make -C oracle harness`"
    import tcsc_amd  # noqa: F401  (fails loudly without the library)

    sys.path.insert(0, os.path.join(PKG, "harness"))
    import out2csv

    env = dict(os.environ)
    env.pop("TCSC_PATH", None)
    p = subprocess.Popen([BIN], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, bufsize=1,
                         cwd=ROOT, env=env, start_new_session=True)
    lines, oks, errors = [], 0, []
    t0 = time.time()
    try:
        for line in p.stdout:
            lines.append(line.rstrip("\n"))
            if "[ERROR]" in line:
                errors.append(line.strip())
            if OK in line:
                oks += 1
                print(f"main_amd: case {oks} validated at {time.time() - t0:.1f} s", flush=True)
                if oks == len(CASES):
                    break
            if time.time() - t0 > 600:
                break
    finally:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGKILL)
        p.wait()
    out = "\n".join(lines) + "\n"
    if os.path.isdir(os.path.join(ROOT, "gpurun_out")):
        with open(os.path.join(ROOT, "gpurun_out", "main_amd_out.txt"), "w") as f:
            f.write(out)
    assert not errors, errors
    assert oks == len(CASES), f"{oks} of {len(CASES)} cases validated; rc={p.returncode}\n{out[-3000:]}"
    # cases 1-4 ran their timing legs to the end: every legacy line, parseable
    algos, cases = out2csv.parse(lines)
    assert [(c["M"], c["K"], c["N"]) for c in cases] == CASES
    for c in cases[:4]:
        for name in ("GEMM", "TCSC_basic", "TCSC_opt", "TCSC_PReLU_basic", "TCSC_PReLU_sep", "TCSC_PReLU_otg"):
            assert name in c["algo"] and float(c["algo"][name][0]) > 0, (c["M"], c["K"], c["N"], name)
