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


def _ephemeral_floor() -> int:
    """Lowest port of the kernel's ephemeral range: fixed ports are picked below it, where no
    socket of a running job (RCCL bootstrap / proxy, torch stores) is handed one by the kernel --
    a block that was free when checked could otherwise be taken before a worker binds it."""
    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
            return int(f.read().split()[0])
    except (OSError, ValueError, IndexError):
        return 32768


_EPHEMERAL_FLOOR = _ephemeral_floor()
_PORT_LO = 10000
_port_base = [_PORT_LO + (os.getpid() % 200) * 100]


def free_port_block(n: int = 16) -> int:
    """Returns the first port of n consecutive free TCP ports."""
    top = _EPHEMERAL_FLOOR if _EPHEMERAL_FLOOR > _PORT_LO + 4 * n else 60000
    while True:
        base = _port_base[0]
        if base + n >= top:
            _port_base[0] = _PORT_LO
            continue
        _port_base[0] += n + 7
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


def run_fake_hosts(script_args, hosts=2, per_host=2, env=None, timeout=240):
    """Start hosts x per_host peers directly with the kungfu-run env contract, host h on
    127.0.0.<h+1> (the runtime groups hosts by IPv4; all of 127/8 reaches this machine), so
    multi-host code paths (cross-host stages, local communicators) run on one box.
    Returns (returncodes, combined output)."""
    base = free_port_block(hosts * per_host + 2)
    peers = ["127.0.0.%d:%d" % (h + 1, base + h * per_host + i) for h in range(hosts) for i in range(per_host)]
    procs = []
    for p in peers:
        e = dict(os.environ, KUNGFU_SELF_SPEC=p, KUNGFU_INIT_PEERS=",".join(peers), KUNGFU_INIT_RUNNERS="",
                 KUNGFU_INIT_CLUSTER_VERSION="0", PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""),
                 OMP_NUM_THREADS="2")
        if env:
            e.update(env)
        procs.append(subprocess.Popen([sys.executable] + list(script_args), env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for pr in procs:
            outs.append(pr.communicate(timeout=timeout)[0])
    finally:
        for pr in procs:
            if pr.poll() is None:
                pr.kill()
                pr.wait()
    return [pr.returncode for pr in procs], "\n".join(outs)
