import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (run with -m gpu)")
    config.addinivalue_line("markers", "slow: multi-process / long tests")


def _built():
    return os.path.exists(os.path.join(ROOT, "bin", "kungfu-run")) and any(
        f.startswith("_kungfu") for f in os.listdir(os.path.join(ROOT, "kungfu_amd")))


def pytest_sessionstart(session):
    if not _built():
        subprocess.check_call(["make", "-C", ROOT, "-j8", "runtime", "launcher"])


_port_base = [20000 + (os.getpid() % 200) * 100]


def free_port_block(n: int = 16) -> int:
    """Returns the first port of n consecutive free TCP ports."""
    while True:
        base = _port_base[0]
        _port_base[0] += n + 7
        if _port_base[0] > 60000:
            _port_base[0] = 20000
        ok = True
        for p in range(base, base + n):
            s = socket.socket()
            try:
                s.bind(("0.0.0.0", p))
            except OSError:
                ok = False
            finally:
                s.close()
            if not ok:
                break
        if ok:
            return base


def kungfu_run(np_, script_args, strategy=None, timeout=120, extra=None, env=None, port_base=None, raw=False):
    """Run ``python script_args...`` (or the program ``script_args[0]`` itself when ``raw``)
    under kungfu-run on 127.0.0.1."""
    base = port_base or free_port_block(np_ + 2)
    cmd = [os.path.join(ROOT, "bin", "kungfu-run"), "-q", "-np", str(np_), "-H", "127.0.0.1:%d" % max(np_, 1),
           "-port-range", "%d-%d" % (base + 1, base + 1 + max(np_, 1) + 4), "-port", str(base)]
    if strategy:
        cmd += ["-strategy", strategy]
    if extra:
        cmd += extra
    cmd += ([] if raw else [sys.executable]) + list(script_args)
    e = dict(os.environ)
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    if env:
        e.update(env)
    return subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=timeout, env=e, text=True)


@pytest.fixture
def run():
    return kungfu_run


def worker(name):
    return os.path.join(ROOT, "tests", "workers", name)
