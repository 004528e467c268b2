"""Checkpoint / resume: rank-0 atomic save, resume with a different peer count."""
import re

import pytest

from conftest import kungfu_run, worker


@pytest.mark.parametrize("kind", ["flat", "torch_sgd", "torch_adam"])
def test_save_then_resume_with_other_cluster_sizes(tmp_path, kind):
    """per-tensor optimizers whose state exists only on rank 0 after the
    load must not desynchronise the state broadcasts (hang / wrong pairing)."""
    r = kungfu_run(2, [worker("ckpt.py"), "--dir", str(tmp_path), "--phase", "save", "--kind", kind], timeout=120)
    assert r.returncode == 0, r.stdout[-3000:]
    saved = set(re.findall(r"SAVED rank=\d h=(\w+)", r.stdout))
    assert len(saved) == 1  # replicas identical at save time
    assert (tmp_path / "ckpt-3.pt").exists() and not list(tmp_path.glob(".*tmp*"))
    for np_ in (1, 3):
        r = kungfu_run(np_, [worker("ckpt.py"), "--dir", str(tmp_path), "--phase", "resume", "--kind", kind],
                       timeout=120)
        assert r.returncode == 0, r.stdout[-3000:]
        resumed = set(re.findall(r"RESUMED rank=\d h=(\w+)", r.stdout))
        assert resumed == saved, (resumed, saved)
        after = re.findall(r"AFTER rank=\d h=(\w+)", r.stdout)
        assert len(after) == np_ and len(set(after)) == 1
