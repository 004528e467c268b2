"""kungfu-run launcher: simple mode, fail-fast, timeout, env contract, and
watch-mode elastic resize with the builtin config server
(parity: scripts/tests/run-tensorflow-resize-test.sh, runner/local/local.go:77-80)."""
import os
import re
import subprocess
import sys
import textwrap

from conftest import ROOT, free_port_block, kungfu_run, worker


def _script(tmp_path, body):
    p = tmp_path / "w.py"
    p.write_text(textwrap.dedent(body))
    return str(p)


def test_env_contract(tmp_path):
    s = _script(tmp_path, """
        import os
        keys = ["KUNGFU_SELF_SPEC", "KUNGFU_INIT_PEERS", "KUNGFU_INIT_RUNNERS", "KUNGFU_PARENT_ID",
                "KUNGFU_INIT_CLUSTER_VERSION", "KUNGFU_ALLREDUCE_STRATEGY", "KUNGFU_JOB_START_TIMESTAMP",
                "KUNGFU_PROC_START_TIMESTAMP", "KUNGFU_HIP_VISIBLE_DEVICES"]
        assert all(k in os.environ for k in keys), [k for k in keys if k not in os.environ]
        assert os.environ["KUNGFU_SELF_SPEC"] in os.environ["KUNGFU_INIT_PEERS"].split(",")
        print("ENV_OK", os.environ["KUNGFU_SELF_SPEC"], os.environ["KUNGFU_ALLREDUCE_STRATEGY"])
    """)
    r = kungfu_run(3, [s], strategy="RING")
    assert r.returncode == 0, r.stdout
    assert r.stdout.count("ENV_OK") == 3 and "RING" in r.stdout


def test_fail_fast(tmp_path):
    s = _script(tmp_path, """
        import os, sys, time
        peers = os.environ["KUNGFU_INIT_PEERS"].split(",")
        if peers.index(os.environ["KUNGFU_SELF_SPEC"]) == 1:
            sys.exit(3)
        time.sleep(60)
    """)
    r = kungfu_run(2, [s], timeout=60)
    assert r.returncode != 0
    assert "exited with error" in r.stdout


def test_timeout(tmp_path):
    s = _script(tmp_path, "import time; time.sleep(60)\n")
    r = kungfu_run(1, [s], extra=["-timeout", "2s"], timeout=60)
    assert r.returncode == 124


def test_logdir_and_prefix(tmp_path):
    s = _script(tmp_path, "print('hello-from-worker')\n")
    logdir = tmp_path / "logs"
    r = kungfu_run(2, [s], extra=["-logdir", str(logdir)])
    assert r.returncode == 0
    assert "::stdout] hello-from-worker" in r.stdout
    files = os.listdir(logdir)
    assert any(f.endswith(".stdout.log") for f in files), files


def test_elastic_resize_watch_mode():
    base = free_port_block(16)
    cfg = base + 15
    r = kungfu_run(1, [worker("elastic.py"), "--schedule", "1:3,2:3,3:3,1:3", "--max-step", "12"], timeout=240,
                   port_base=base,
                   extra=["-w", "-builtin-config-port", str(cfg), "-config-server",
                          "http://127.0.0.1:%d/config" % cfg, "-H", "127.0.0.1:4"])
    assert r.returncode == 0, r.stdout[-5000:]
    done = re.findall(r"ELASTIC_DONE rank=(\d+) np=(\d+) step=(\d+) w=([\d.]+) v=(\d+)", r.stdout)
    assert len(done) == 1, r.stdout[-5000:]
    rank, np_, step, w, v = done[0]
    assert (rank, np_, step) == ("0", "1", "12")
    assert float(w) == 100.0  # rank 0's model survived every resize
    assert int(v) == 3  # three membership changes
    assert r.stdout.count("ELASTIC_DETACHED") == 2  # the two extra workers left at the 3 -> 1 shrink
    assert "resize 1 -> 2" in r.stdout and "resize 2 -> 3" in r.stdout


def test_config_server_rest():
    from kungfu_amd._lib import runtime as K
    import json

    port = free_port_block(1)
    s = K.ConfigServer(port)
    s.start()
    url = "http://127.0.0.1:%d/config" % port
    st, body = K.http_request("GET", url, "")
    assert st == 404
    c = {"Runners": ["127.0.0.1:38080"], "Workers": ["127.0.0.1:10000", "127.0.0.1:10001"]}
    st, _ = K.http_request("PUT", url, json.dumps(c))
    assert st == 200
    st, body = K.http_request("GET", url, "")
    assert st == 200 and json.loads(body)["Workers"] == c["Workers"]
    bad = {"Runners": ["127.0.0.1:38080"], "Workers": ["10.0.0.9:10000"]}
    st, _ = K.http_request("PUT", url, json.dumps(bad))
    assert st == 400
    st, _ = K.http_request("DELETE", url, "")
    assert st == 200
    st, _ = K.http_request("GET", url, "")
    assert st == 404
    s.stop()


def test_config_server_binary(tmp_path):
    port = free_port_block(1)
    p = subprocess.Popen([os.path.join(ROOT, "bin", "kungfu-config-server"), "-port", str(port), "-ttl", "20"])
    try:
        import time
        from kungfu_amd._lib import runtime as K
        for _ in range(50):
            st, _ = K.http_request("GET", "http://127.0.0.1:%d/config" % port, "")
            if st != -1:
                break
            time.sleep(0.1)
        assert st == 404
        K.http_request("GET", "http://127.0.0.1:%d/stop" % port, "")
        assert p.wait(timeout=10) == 0
    finally:
        if p.poll() is None:
            p.kill()


def test_modelarts_platform_discovery(tmp_path):
    """-platform modelarts: runner list from DLS_TASK_* / BATCH_CUSTOM<i>_HOSTS (reference
    srcs/go/platforms/modelarts/modelarts.go); a one-container job runs on 127.0.0.1."""
    s = _script(tmp_path, """
        import os
        print("MA_OK", os.environ["KUNGFU_SELF_SPEC"], os.environ["KUNGFU_INIT_RUNNERS"])
    """)
    env = dict(os.environ, DLS_TASK_INDEX="0", DLS_TASK_NUMBER="1")
    r = subprocess.run([os.path.join(ROOT, "bin", "kungfu-run"), "-platform", "modelarts", "-np", "2",
                        sys.executable, s], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout
    assert r.stdout.count("MA_OK") == 2 and "127.0.0.1:38888" in r.stdout
    env = dict(os.environ, DLS_TASK_INDEX="0", DLS_TASK_NUMBER="2", BATCH_CUSTOM0_HOSTS="127.0.0.1:38888")
    r = subprocess.run([os.path.join(ROOT, "bin", "kungfu-run"), "-platform", "modelarts", "-np", "2",
                        sys.executable, s], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=120)
    assert r.returncode != 0 and "BATCH_CUSTOM1_HOSTS not set" in r.stdout


def test_kill_peer_via_control_message(tmp_path):
    """Fault injection (parity: kungfu-test-util -kill, tests/go/cmd/kungfu-test-util):
    the "exit" control message ends a worker; the launcher then finishes."""
    import subprocess
    import sys
    import time

    from conftest import ROOT, free_port_block

    s = _script(tmp_path, """
        import os, sys, time
        import kungfu_amd as kf
        kf.init()
        print("READY", os.environ["KUNGFU_SELF_SPEC"], flush=True)
        time.sleep(120)
        print("NOT_KILLED", flush=True)
    """)
    base = free_port_block(6)
    cmd = [os.path.join(ROOT, "bin", "kungfu-run"), "-q", "-np", "2", "-H", "127.0.0.1:2",
           "-port-range", "%d-%d" % (base + 1, base + 5), "-port", str(base), sys.executable, s]
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env)
    specs, lines = [], []
    t0 = time.time()
    try:
        while len(specs) < 2 and time.time() - t0 < 60:
            line = p.stdout.readline()
            if not line:
                break
            lines.append(line)
            if "READY" in line:
                specs.append(line.split("READY", 1)[1].split()[0])
        assert len(specs) == 2, "".join(lines)
        k = subprocess.run([os.path.join(ROOT, "bin", "kungfu-test-util"), "-kill"] + specs,
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=30)
        assert k.returncode == 0, k.stdout
        out, _ = p.communicate(timeout=60)
    finally:
        if p.poll() is None:
            p.kill()
    assert p.returncode == 0, out
    assert "NOT_KILLED" not in out
    assert time.time() - t0 < 90


def test_monitoring_http_metrics(tmp_path):
    """Net monitor (parity: tests/go/cmd/kungfu-test-monitor): egress counters exposed over
    HTTP on port + 10000 and as the egress_rates op."""
    s = _script(tmp_path, """
        import os, time, urllib.request
        import torch
        import kungfu_amd as kf
        from kungfu_amd import ops
        kf.init()
        for _ in range(5):
            ops.all_reduce(torch.ones(1 << 16))
        port = int(os.environ["KUNGFU_SELF_SPEC"].split(":")[1]) + 10000
        opener = urllib.request.build_opener(urllib.request.ProxyHandler({}))
        txt = opener.open("http://127.0.0.1:%d/metrics" % port, timeout=10).read().decode()
        assert "egress_total_bytes" in txt, txt
        vals = [float(l.split()[-1]) for l in txt.splitlines() if l.startswith("egress_total_bytes")]
        assert vals and max(vals) > 0, txt
        time.sleep(1.2)
        r = ops.egress_rates()
        assert r.shape == (kf.current_cluster_size(),)
        kf.run_barrier()
        print("MONITOR_OK", flush=True)
    """)
    r = kungfu_run(2, [s], timeout=120, env={"KUNGFU_CONFIG_ENABLE_MONITORING": "true"})
    assert r.returncode == 0, r.stdout[-3000:]
    assert r.stdout.count("MONITOR_OK") == 2, r.stdout[-3000:]


def test_bad_worker_cancels_job():
    """Fault injection (parity: tests/go/cmd/kungfu-bad-worker): rank 0 of the native
    bad worker exits 1 after 3 all-reduce steps; the peers block in the next collective
    and kungfu-run cancels them (any failure cancels all)."""
    from conftest import ROOT

    r = kungfu_run(3, [os.path.join(ROOT, "bin", "kungfu-bad-worker"), "-error-after", "3"], timeout=60, raw=True)
    assert r.returncode != 0, r.stdout[-3000:]
    assert "rank 0 fails at step 3" in r.stdout
    assert r.stdout.count("step 2 ok") == 3  # every worker completed the collectives before the failure
    assert "exited with error" in r.stdout


def test_retry_on_stderr_prefix(tmp_path):
    """The runner restarts a worker whose first stderr line starts with
    KUNGFU_CONFIG_RETRY_STDERR_PREFIX (parity: the ld.so-bug hack,
    srcs/go/utils/runner/local/hack.go:14-35, injected like kungfu-bench-allreduce
    -rand-nccl-failure)."""
    marker = tmp_path / "attempts"
    s = _script(tmp_path, """
        import os, sys
        m = %r
        n = int(open(m).read()) if os.path.exists(m) else 0
        open(m, "w").write(str(n + 1))
        if n < 2:
            sys.stderr.write("Inconsistency detected by ld.so: injected failure\\n")
            sys.stderr.flush()
            sys.exit(1)
        print("RETRY_WORKER_OK attempt=%%d" %% (n + 1), flush=True)
    """ % str(marker))
    r = kungfu_run(1, [s], timeout=60, env={"KUNGFU_CONFIG_RETRY_STDERR_PREFIX": "Inconsistency detected by ld.so"})
    assert r.returncode == 0, r.stdout[-3000:]
    assert "RETRY_WORKER_OK attempt=3" in r.stdout
    assert r.stdout.count("restarting") == 2
    # without the prefix configured the same failure is fatal
    marker.unlink()
    r = kungfu_run(1, [s], timeout=60)
    assert r.returncode != 0
