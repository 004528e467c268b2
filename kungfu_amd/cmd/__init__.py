"""Console entry points (parity: srcs/python/kungfu/cmd/__init__.py:4-6, which
calls the launcher embedded in libkungfu).  The launcher is the native
``bin/kungfu-run``; these wrappers run it as a child process and exit with
its status (no exec, so nothing here ever touches the GPU first)."""
import os
import subprocess
import sys

from .._lib import bin_path


def _run(name: str) -> None:
    exe = bin_path(name)
    if not os.path.exists(exe):
        sys.stderr.write("%s is not built; run `make -C %s launcher`\n" % (exe, os.path.dirname(os.path.dirname(exe))))
        sys.exit(2)
    sys.exit(subprocess.call([exe] + sys.argv[1:]))


def run() -> None:
    _run("kungfu-run")


def config_server() -> None:
    _run("kungfu-config-server")


def rrun() -> None:
    _run("kungfu-rrun")


def distribute() -> None:
    _run("kungfu-distribute")
