"""The KUNGFU_* settings registry (kungfu_amd/knobs.py): every variable the
sources read is registered, unknown / misspelt ones warn with a suggestion, and developer A/B
knobs are ignored unless KUNGFU_DEV_KNOBS=1."""
import os
import re
import subprocess
import sys

import pytest

from conftest import ROOT

from kungfu_amd import knobs


def _source_names():
    names = set()
    pat = re.compile(r"KUNGFU_[A-Z0-9_]+")
    for d in ("kungfu_amd", "csrc", "bench.py", "__graft_entry__.py"):
        p = os.path.join(ROOT, d)
        files = [p] if os.path.isfile(p) else [os.path.join(dp, f) for dp, _, fs in os.walk(p) for f in fs]
        for f in files:
            if not f.endswith((".py", ".cpp", ".hpp", ".hip", ".h")) or f.endswith("knobs.py"):
                continue
            with open(f, errors="replace") as fh:
                names.update(pat.findall(fh.read()))
    return names


def test_every_source_knob_is_registered():
    missing = []
    for n in sorted(_source_names()):
        if n in knobs.KNOBS or n in knobs.MACROS or n in knobs.RETIRED or n.startswith(knobs.PREFIXES):
            continue
        if n.endswith("_") and any(k.startswith(n) for k in knobs.KNOBS):  # a prefix built at run time
            continue
        missing.append(n)
    assert not missing, "register these in kungfu_amd/knobs.py: %s" % missing


def test_unknown_and_dev_knobs_warn():
    env = {"KUNGFU_BUCKET_MBB": "8", "KUNGFU_CONV_TILE_RULES": "1", "KUNGFU_BUCKET_MB": "16", "PATH": "/x",
           "KUNGFU_LINEAR_GEMM": "1"}
    msgs = knobs.check_environ(env)
    assert any("KUNGFU_BUCKET_MBB" in m and "did you mean KUNGFU_BUCKET_MB" in m for m in msgs), msgs
    assert any("KUNGFU_CONV_TILE_RULES" in m and "IGNORED" in m for m in msgs), msgs
    assert any("KUNGFU_LINEAR_GEMM" in m and "retired" in m for m in msgs), msgs
    assert not any("KUNGFU_BUCKET_MB " in m or m.endswith("KUNGFU_BUCKET_MB") for m in msgs), msgs
    env["KUNGFU_DEV_KNOBS"] = "1"
    assert not any("TILE_RULES" in m for m in knobs.check_environ(env))


def test_dev_knob_needs_dev_flag(monkeypatch):
    monkeypatch.setenv("KUNGFU_VGG_FUSED", "0")
    monkeypatch.delenv("KUNGFU_DEV_KNOBS", raising=False)
    assert knobs.get("KUNGFU_VGG_FUSED") == "1"
    monkeypatch.setenv("KUNGFU_DEV_KNOBS", "1")
    assert knobs.get("KUNGFU_VGG_FUSED") == "0"
    with pytest.raises(KeyError):
        knobs.get("KUNGFU_NOT_A_KNOB")


def test_import_warns_on_misspelt_knob():
    e = dict(os.environ, KUNGFU_TAIL_BUCKET_M="2", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", "import kungfu_amd"], env=e, stderr=subprocess.PIPE, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    assert "unknown setting KUNGFU_TAIL_BUCKET_M" in r.stderr and "KUNGFU_TAIL_BUCKET_MB" in r.stderr, r.stderr


def test_knob_table_lists_every_knob():
    t = knobs.table()
    assert all("`%s`" % n in t for n in knobs.KNOBS)
