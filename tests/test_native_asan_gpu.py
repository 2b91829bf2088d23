"""AddressSanitizer run of libmtts's host code: tests/native/asan_driver is the
engine / Local / codec sources compiled with host-side ASan (`make -C tests/native`, done on
the build side like libmtts itself) plus a C driver that walks every C entry point and its error
paths.  Any heap overflow, use-after-free or leak in engine.cpp / local.cpp / codec.cpp fails
the run; leaks inside the ROCm runtime are suppressed (tests/native/lsan.supp)."""
import os
import subprocess
import time

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
EXE = os.path.join(HERE, "native", "asan_driver")


def test_asan_driver_clean():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(EXE):
        pytest.skip("tests/native/asan_driver not built (make -C tests/native)")
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:protect_shadow_gap=0:halt_on_error=1:verify_asan_link_order=0"
    env["LSAN_OPTIONS"] = "suppressions=" + os.path.join(HERE, "native", "lsan.supp")
    # progress log of the driver's phases (flushed per line) where a GPU session keeps it
    # (gpurun_out/ comes back from the box); the driver's own watchdog ends a phase that runs
    # past MTTS_ASAN_PHASE_TIMEOUT s with exit code 3 and names it, and this timeout (below the
    # 180-s silence window of a GPU session) covers the leak check after the last phase
    logdir = os.path.join(os.path.dirname(HERE), "gpurun_out")
    os.makedirs(logdir, exist_ok=True)
    log = os.path.join(logdir, "asan_driver.log")
    with open(log, "w"):
        pass
    env["MTTS_ASAN_LOG"] = log
    env.setdefault("MTTS_ASAN_PHASE_TIMEOUT", "60")
    t0 = time.time()
    try:
        r = subprocess.run([EXE], env=env, capture_output=True, text=True, timeout=150)
    except subprocess.TimeoutExpired as ex:
        tail = open(log).read()[-3000:]
        pytest.fail(f"asan driver still running after {time.time() - t0:.0f} s; its phase log ends:\n{tail}\n"
                    f"stderr tail:\n{(ex.stderr or b'')[-2000:]!r}")
    out = r.stdout + r.stderr
    phases = open(log).read()
    assert r.returncode == 0, phases[-2000:] + "\n" + out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "ERROR: LeakSanitizer" not in out, out[-4000:]
    assert "asan driver: ok (0 failed checks)" in out, out[-4000:]
