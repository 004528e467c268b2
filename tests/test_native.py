"""Native (C++) runtime tests incl. sanitizer builds of the in-process fake
cluster (the reference has no race detection at all)."""
import subprocess

import pytest

from conftest import ROOT, free_port_block


@pytest.mark.parametrize("target", ["native_test", "native_test_asan", "native_test_tsan"])
def test_native_runtime(target):
    subprocess.check_call(["make", "-C", ROOT, "-s", "build/" + target])
    env = {"TSAN_OPTIONS": "halt_on_error=1", "PATH": "/usr/bin:/bin"}
    r = subprocess.run([ROOT + "/build/" + target, str(free_port_block(120))], stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "NATIVE_TESTS_OK" in r.stdout, r.stdout[-4000:]
    assert "WARNING: ThreadSanitizer" not in r.stdout
