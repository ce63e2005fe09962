"""the CPU restatement under AddressSanitizer + UndefinedBehaviorSanitizer.

`make -C oracle san` builds oracle/san_check.c with sl_oracle.c and sl_cpu_step.c
under -fsanitize=address,undefined (host only; GPU sanitizers are not available on
the MI355X pool).  The driver visits 2x2 .. 64x64 boards, both RNG modes, resets,
wide views and every action.  Any report (or leak) fails the run."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(REPO, "oracle")


def test_oracle_c_under_asan_ubsan():
    try:
        subprocess.run(["make", "-s", "-C", ORACLE, "san"], check=True, capture_output=True,
                       timeout=300)
    except (subprocess.CalledProcessError, FileNotFoundError) as e:
        pytest.skip("sanitizer build unavailable: %s" % getattr(e, "stderr", e))
    env = dict(os.environ)
    # another preloaded library may precede the ASan runtime: do not abort on it
    env["ASAN_OPTIONS"] = "detect_leaks=1:verify_asan_link_order=0:halt_on_error=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    r = subprocess.run([os.path.join(ORACLE, "_build", "san_check")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "san_check ok" in r.stdout
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
