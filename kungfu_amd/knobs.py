"""One registry of every ``KUNGFU_*`` environment variable the framework reads.

Three kinds:

* ``user``     -- documented configuration (timeouts, bucket sizes, data plane, kill switches
  that route an op back to the library path);
* ``launcher`` -- set by ``kungfu-run`` / the elastic runtime for its workers (the worker env
  contract, parity ``srcs/go/kungfu/env/envs.go``); users do not set these by hand;
* ``test``     -- hooks the test suite uses (colocated ranks, injected pre-flight faults);
* ``dev``      -- A/B switches kept for re-measuring a design decision (most of them select an
  alternative that measured slower, see profiles/README.md).  They are honoured ONLY when
  ``KUNGFU_DEV_KNOBS=1`` is also set -- in Python (:func:`get`) and in the kernels
  (``kfk::dev_knob``, csrc/kernels/common.hpp) -- so a stale shell variable cannot silently
  slow a production run down.  Numerics-changing experiments are not knobs at all (e.g. the
  BN-finalize skip is compiled in only with ``-DKUNGFU_DEV_EXPERIMENTS``).

:func:`check_environ` (called once at ``import kungfu_amd``) warns about every set ``KUNGFU_*``
variable that is not registered (a misspelt knob would otherwise be ignored silently, with a
close-match suggestion) and about dev knobs that are set without ``KUNGFU_DEV_KNOBS=1``.
"""
from __future__ import annotations

import difflib
import os
import warnings
from typing import Dict, NamedTuple, Optional


class Knob(NamedTuple):
    default: Optional[str]
    kind: str  # user | launcher | test | dev
    doc: str


class KnobWarning(UserWarning):
    pass


def _u(default, doc):
    return Knob(default, "user", doc)


def _l(doc):
    return Knob(None, "launcher", doc)


def _t(default, doc):
    return Knob(default, "test", doc)


def _d(default, doc):
    return Knob(default, "dev", doc)


KNOBS: Dict[str, Knob] = {
    # -- runtime / transport (csrc/runtime) ------------------------------------------------
    "KUNGFU_CONFIG_LOG_LEVEL": _u("INFO", "runtime log level (DEBUG/INFO/WARN/ERROR)"),
    "KUNGFU_CONFIG_ENABLE_MONITORING": _u("false", "net monitor + /metrics endpoint"),
    "KUNGFU_CONFIG_MONITORING_PERIOD": _u("1s", "net monitor sampling period"),
    "KUNGFU_CONFIG_ENABLE_STALL_DETECTION": _u("false", "log host collectives that take > 10 s"),
    "KUNGFU_CONFIG_ENABLE_TRACE": _u("false", "print trace-scope reports at exit"),
    "KUNGFU_CONFIG_CHUNK_SIZE_MIB": _u("1", "host all-reduce chunk size (strategies rotate per chunk)"),
    "KUNGFU_CONFIG_STRATEGY_HASH_METHOD": _u("SIMPLE", "chunk -> strategy assignment (SIMPLE | NAME)"),
    "KUNGFU_CONFIG_CONN_RETRY_COUNT": _u("500", "TCP dial retries"),
    "KUNGFU_CONFIG_CONN_RETRY_PERIOD": _u("200ms", "TCP dial retry period"),
    "KUNGFU_CONFIG_USE_UNIX_SOCK": _u("true", "same-host peers over Unix sockets"),
    "KUNGFU_CONFIG_WAIT_RUNNER_TIMEOUT": _u("120s", "elastic: wait for a runner"),
    "KUNGFU_CONFIG_RETRY_STDERR_PREFIX": _u(None, "runner restarts a worker whose stderr starts with this"),
    "KUNGFU_ALLREDUCE_STRATEGY": _u("AUTO", "host all-reduce topology strategy"),
    "KUNGFU_OP_TIMEOUT_S": _u("0", "host collective watchdog: abort (exit 3) after this many seconds; 0 = off"),
    "KUNGFU_MNIST_DIR": _u(None, "MNIST idx files for the examples"),
    "KUNGFU_PLATFORM": _u(None, "launcher platform hint (ModelArts discovery)"),
    # -- device data plane (kungfu_amd/parallel, csrc/kernels/rccl_comm.hip) -------------------
    "KUNGFU_GPU_DATAPLANE": _u("rccl", "rccl | host (stage device collectives through host memory)"),
    "KUNGFU_GPU_ALLREDUCE": _u("rccl", "rccl | graph (bucket all-reduce along the KungFu strategy graphs)"),
    "KUNGFU_BUCKET_MB": _u("32", "S-SGD gradient bucket size (MiB)"),
    "KUNGFU_TAIL_BUCKET_MB": _u("4", "size cap of the buckets holding the first layers (exposed tail)"),
    "KUNGFU_RCCL_TIMEOUT_S": _u("600", "RCCL watchdog stall timeout; setting it explicitly makes a stall fatal"),
    "KUNGFU_RCCL_STALL_ACTION": _u("log", "log | abort: what a stalled RCCL collective does"),
    "KUNGFU_RCCL_INIT_TIMEOUT_S": _u("300", "communicator init / finalize deadline"),
    "KUNGFU_RCCL_BLOCKING": _u("0", "1: blocking communicator init (no deadline, no CTA budget)"),
    "KUNGFU_RCCL_MIN_CTAS": _u("0", "ncclConfig_t.minCTAs (0 = RCCL default); _<SCOPE> suffix per scope"),
    "KUNGFU_RCCL_MAX_CTAS": _u("0", "ncclConfig_t.maxCTAs (0 = RCCL default); _<SCOPE> suffix per scope"),
    "KUNGFU_NATIVE_BACKTRACE": _u("0", "1: print a native backtrace on SIGSEGV/SIGBUS/SIGABRT (debugging)"),
    "KUNGFU_RCCL_COLOCATE": _t("0", "1: several RCCL ranks on one GPU (socket transport; tests)"),
    "KUNGFU_COMM_EMULATE": _u(None, "ranks=R,ctas=C,busbw=GB/s,lat_us=L: model an R-rank all-reduce on one GPU"),
    "KUNGFU_PREFLIGHT_TIMEOUT_S": _u("60", "bench pre-flight: deadline of each device check"),
    "KUNGFU_PREFLIGHT_CORRUPT": _t(None, "test hook: this rank corrupts its pre-flight buffer"),
    "KUNGFU_PREFLIGHT_CORRUPT_WHAT": _t("ipc", "test hook: ipc | allreduce | stall (reports a stall without stalling)"),
    "KUNGFU_FORCE_DEVICE": _t(None, "pin every rank to this HIP device (colocated tests)"),
    "KUNGFU_INIT_CKPT": _u(None, "elastic: initial checkpoint step"),
    # -- kernel routing kill switches (1 = our HIP kernel, 0 = library path) --------------------
    "KUNGFU_CONV3X3": _u("1", "3x3 convolutions on the MFMA kernel"),
    "KUNGFU_CONV_RECT": _u("1", "rectangular-window convolutions on the MFMA kernel"),
    "KUNGFU_WGRAD": _u("1", "weight gradients on the split-K MFMA kernel"),
    "KUNGFU_WGRAD_RECT": _u("1", "rectangular-window weight gradients on the MFMA kernels"),
    "KUNGFU_FUSED_BLOCK": _u("1", "ResNet bottleneck as one fused autograd node"),
    "KUNGFU_STEM": _u("1", "ResNet stem conv on the MFMA stem kernel"),
    "KUNGFU_LINEAR_WGRAD": _u("1", "linear-layer weight gradients on the split-K MFMA kernel"),
    "KUNGFU_DEV_KNOBS": _u("0", "1: honour the dev (A/B) knobs below"),
    # -- launcher / worker env contract (csrc/launcher/job.cpp, csrc/runtime/peer.cpp) ---------
    "KUNGFU_SELF_SPEC": _l("this worker's host:port"),
    "KUNGFU_INIT_PEERS": _l("initial peer list"),
    "KUNGFU_INIT_RUNNERS": _l("initial runner list"),
    "KUNGFU_INIT_CLUSTER_VERSION": _l("initial cluster version"),
    "KUNGFU_PARENT_ID": _l("runner that started this worker"),
    "KUNGFU_CONFIG_SERVER": _l("elastic config server URL"),
    "KUNGFU_JOB_START_TIMESTAMP": _l("job start time"),
    "KUNGFU_PROC_START_TIMESTAMP": _l("worker start time"),
    "KUNGFU_HIP_DEVICE_ORDINAL": _l("the worker's HIP device"),
    "KUNGFU_HIP_VISIBLE_DEVICES": _l("devices assigned to the worker (-isolate-gpus)"),
    "KUNGFU_ALLOW_XGMI": _l("several workers may share a GPU (-allow-xgmi)"),
    "KUNGFU_SELF_IP": _l("this worker's IP (single mode)"),
    # -- dev A/B knobs (need KUNGFU_DEV_KNOBS=1) ----------------------------------------------
    "KUNGFU_CONV_TILE_RULES": _d("2", "1 = the round-2 conv tile defaults"),
    "KUNGFU_WGRAD_PLAN": _d("2", "1: the round-5 weight-gradient plan rules (tile variant, row-image kernel, split counts)"),
    "KUNGFU_CONV_T224": _d("1", "0: no 224x256 conv tiles (one- or two-round grids of 256x256 tiles keep them)"),
    "KUNGFU_CONV_ROWS": _d("1", "0: stride-1 3x3 convs with Cin = Cout = 64 on the tap-wise kernel, not the row-image one"),
    "KUNGFU_VGG_FUSED": _d("1", "VGG-16 conv/ReLU/pool stack as one autograd node (0: the per-layer modules)"),
    "KUNGFU_GRAPH_MULTIRANK": _u("1", "0: GraphedStep keeps multi-rank RCCL steps eager (capture uses the comm stream as origin)"),
}

# Round 5: A/B knobs whose question is settled are gone -- the measured winner
# is the only code path (or a module attribute the tests flip), the negative results are recorded in
# profiles/README.md.  Setting one warns that it no longer does anything.
RETIRED: Dict[str, str] = {
    "KUNGFU_LINEAR_GEMM": "linear layers on gemm.hip measured slower than hipBLASLt (r4_gemm_nt.md)",
    "KUNGFU_LINEAR_WGRAD_ATOMICS": "atomic split-K linear wgrad measured 3 % slower (r4t29)",
    "KUNGFU_GELU_FWD": "the one-exponential GELU forward measured 0.6 % slower (r4t20)",
    "KUNGFU_WGRAD_STREAM": "weight gradients on a side stream measured 1.2 % slower (r3)",
    "KUNGFU_BN_INLAUNCH_FIN": "BN finalize inside the conv launch measured 0.55 ms/step slower (r3)",
    "KUNGFU_CONV_PRIO": "s_setprio in the conv tiles measured neutral (r3)",
    "KUNGFU_STEM_FUSED_BWD": "the one-pass fused stem backward measured slower (r3)",
    "KUNGFU_COMM_STREAM_PRIORITY": "a high-priority comm stream measured 2x slower (r1)",
    "KUNGFU_BN_SKIP_FINALIZE": "timing-only experiment (wrong numerics), retired",
    "KUNGFU_BERT_GEMM": "unused",
    "KUNGFU_CONV_STAGGER": "the measured winner is the only path: on (+0.8 %, r3)",
    "KUNGFU_CONV_PERSIST_BLOCKS": "the measured winner is the only path: 4 persistent blocks per CU",
    "KUNGFU_WGRAD_STAGGER": "the measured winner is the only path: on for 256x256 tiles only (r3)",
    "KUNGFU_WROWS_STAGGER": "the measured winner is the only path: on (r3)",
    "KUNGFU_WGRAD_KB32": "the measured winner is the only path: off (r4t1)",
    "KUNGFU_BN_NT": "the measured winner is the only path: non-temporal loads (r3f)",
    "KUNGFU_BN_MAXGRID": "the measured winner is the only path: the kernel default grid",
    "KUNGFU_ATTN_BWD_WAVES": "the measured winner is the only path: 8 waves (r4t15)",
    "KUNGFU_BN_CONCAT": "the measured winner is the only path: on (module attribute ops.fused_bn.CONCAT_ENABLED)",
    "KUNGFU_BN_BATCH_FIN": "the measured winner is the only path: on (r4t25; module attribute ops.fused_bn._BATCH_FIN)",
    "KUNGFU_LN_BIAS_LINK": "the measured winner is the only path: on (module attribute ops.layernorm._BIAS_LINK)",
    "KUNGFU_GELU_BIAS_LINK": "the measured winner is the only path: on (module attribute ops.linear._GELU_LINK)",
    "KUNGFU_RESIDUAL_LINK": "the measured winner is the only path: on (r4t14; module attribute ops.linear._RES_LINK)",
    "KUNGFU_LINEAR_DIRECT_WGRAD": "the measured winner is the only path: on (module attribute ops.linear._DIRECT_WGRAD)",
    "KUNGFU_FUSED_XENT": "the measured winner is the only path: on (r4t22; module attribute ops.xent._ENABLED)",
    "KUNGFU_PAIR_NATIVE": "the measured winner is the only path: the native prefetch thread (r4t22)",
    "KUNGFU_GRAPH_SEGMENTED": "the whole-graph N-rank layout is gone: N-rank capture is always segmented (r6)",
}

# compile-time switches (-D...), not environment variables; listed so the source lint knows them
MACROS = ("KUNGFU_CONV_BUFLD", "KUNGFU_WGRAD_BUFLD", "KUNGFU_WGRAD_AUX", "KUNGFU_DISABLE_TRACE",
          "KUNGFU_ENABLE_TRACE", "KUNGFU_DEV_EXPERIMENTS", "KUNGFU_AMD_CAPI_H", "KUNGFU_ENABLE_HIP")

# prefixes with a free suffix (per-scope overrides)
PREFIXES = ("KUNGFU_RCCL_MIN_CTAS_", "KUNGFU_RCCL_MAX_CTAS_")


def dev_enabled() -> bool:
    return os.environ.get("KUNGFU_DEV_KNOBS", "0") not in ("", "0")


def get(name: str, default: Optional[str] = None) -> Optional[str]:
    """The value of a registered knob (its registered default when unset; ``default``
    overrides that).  Dev knobs read as their default unless ``KUNGFU_DEV_KNOBS=1``."""
    k = KNOBS.get(name)
    if k is None:
        raise KeyError("unregistered knob %s (add it to kungfu_amd/knobs.py)" % name)
    dflt = default if default is not None else k.default
    if k.kind == "dev" and not dev_enabled():
        return dflt
    return os.environ.get(name, dflt)


def get_int(name: str, default: Optional[int] = None) -> int:
    v = get(name, None if default is None else str(default))
    return int(v) if v not in (None, "") else 0


_checked = [False]


def check_environ(environ=None) -> list:
    """Warn (once per process) about unknown ``KUNGFU_*`` variables and ignored dev knobs.
    Returns the warning messages."""
    env = os.environ if environ is None else environ
    msgs = []
    for name in sorted(env):
        if not name.startswith("KUNGFU_"):
            continue
        if name in KNOBS:
            if KNOBS[name].kind == "dev" and not (env.get("KUNGFU_DEV_KNOBS", "0") not in ("", "0")):
                msgs.append("%s is a developer A/B knob and is IGNORED without KUNGFU_DEV_KNOBS=1" % name)
            continue
        if name.startswith(PREFIXES):
            continue
        if name in RETIRED:
            msgs.append("%s is retired and has no effect: %s" % (name, RETIRED[name]))
            continue
        close = difflib.get_close_matches(name, list(KNOBS), n=1, cutoff=0.75)
        msgs.append("unknown setting %s%s (see kungfu_amd/knobs.py)" % (
            name, " -- did you mean %s?" % close[0] if close else ""))
    for m in msgs:
        warnings.warn("kungfu_amd: " + m, KnobWarning, stacklevel=3)
    return msgs


def check_environ_once() -> None:
    if not _checked[0]:
        _checked[0] = True
        check_environ()


def table() -> str:
    """Markdown tables of every knob, one per kind (docs/KNOBS.md is generated from this), then the
    retired ones."""
    heads = {"user": "Configuration", "dev": "Developer A/B switches (need KUNGFU_DEV_KNOBS=1)",
             "test": "Test hooks", "launcher": "Worker environment set by the launcher (not set by hand)"}
    out = []
    for kind in ("user", "dev", "test", "launcher"):
        rows = ["## %s" % heads[kind], "", "| variable | default | meaning |", "|---|---|---|"]
        for n, k in KNOBS.items():
            if k.kind == kind:
                rows.append("| `%s` | %s | %s |" % (n, "" if k.default is None else "`%s`" % k.default, k.doc))
        out.append("\n".join(rows))
    rows = ["## Retired (setting one only warns)", "", "| variable | why |", "|---|---|"]
    rows += ["| `%s` | %s |" % (n, why) for n, why in RETIRED.items()]
    out.append("\n".join(rows))
    return "\n\n".join(out) + "\n"
