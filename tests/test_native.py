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


def test_configure_toggles(tmp_path):
    """./configure writes config.mk; --disable-hip drops every hipcc step from `make all`,
    --disable-trace compiles trace scopes out (parity: configure:22-120)."""
    import shutil

    work = tmp_path / "src"
    shutil.copytree(ROOT, work, ignore=shutil.ignore_patterns(".git", "build", "gpurun_out", "*.so", "bin"))
    r = subprocess.run(["./configure", "--disable-hip", "--disable-trace"], cwd=work, stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True)
    assert r.returncode == 0, r.stdout
    cfg = (work / "config.mk").read_text()
    assert "KUNGFU_ENABLE_HIP := 0" in cfg and "KUNGFU_ENABLE_TRACE := 0" in cfg
    dry = subprocess.run(["make", "-n", "all"], cwd=work, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                         text=True).stdout
    assert "hipcc" not in dry and "-DKUNGFU_DISABLE_TRACE" in dry and "libkungfu_amd.so" in dry
    # the trace-less runtime still compiles
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Icsrc/include", "-DKUNGFU_DISABLE_TRACE",
                        "csrc/runtime/session.cpp"], cwd=work, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True)
    assert r.returncode == 0, r.stdout[-2000:]
    subprocess.run(["./configure"], cwd=work, check=True, stdout=subprocess.PIPE)
    dry = subprocess.run(["make", "-n", "all"], cwd=work, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                         text=True).stdout
    assert "hipcc" in dry and "-DKUNGFU_DISABLE_TRACE" not in dry
