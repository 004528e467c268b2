#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 SynchronousSGD training throughput on MI355X.

Metric (BASELINE.json): images/sec ResNet-50 SynchronousSGD at 1/2/4/8 MI355X.
The reference's comparable number is ~344 img/s/GPU (KungFu S-SGD, 256 images
per GPU, 16 x V100); ``vs_baseline`` = value / (344.2 * n_gpus).

Config: ResNet-50 (v1.5, 25.56 M params, random init), synthetic ImageNet-shaped
data (224x224x3, 1000 classes), 256 images per GPU (weak scaling), bf16 autocast
compute with f32 master weights, channels_last, SGD momentum 0.9 + wd 1e-4 via
``kungfu_amd.optimizers.SynchronousSGDOptimizer`` (bucketed RCCL all-reduce
overlapped with backward, fused HIP SGD step), one process per GPU.

BERT-base (BASELINE.json config 5): ``--model bert_base --optimizer gns`` trains the
110 M-parameter encoder on synthetic 128-token pre-training batches (MLM on 20
masked positions + NSP, AdamW) through S-SGD with the gradient-noise-scale
monitor and reports sequences/s (and tokens/s in ``config``).

Usage:
    python bench.py [--gpus 1] [--steps 20] [--warmup 5]
    python bench.py --model bert_base --optimizer gns
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \\
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_PER_GPU = 5507.0 / 16  # KungFu S-SGD ResNet-50, global batch 4096 on 16 x V100
METRIC = "images/sec/GPU ResNet-50 SynchronousSGD at 1/2/4/8 MI355X; scaling efficiency"
# The reference's other sync-scalability panels (global batch 4096 on 16 x V100):
# (metric, per-GPU baseline img/s) for --model; the headline (default) is ResNet-50.
MODEL_BASELINES = {
    "resnet50": (METRIC, BASELINE_PER_GPU),
    "vgg16": ("images/sec/GPU VGG16 SynchronousSGD at 1/2/4/8 MI355X", 3330.0 / 16),
    "inception_v3": ("images/sec/GPU InceptionV3 SynchronousSGD at 1/2/4/8 MI355X", 7426.0 / 16),
    # BASELINE.json config 5; the reference publishes no BERT number
    "bert_base": ("sequences/sec/GPU BERT-base (seq 128) SynchronousSGD + gradient-noise-scale monitor", None),
}


def _setup_env():
    # MIOpen tuning database shipped in-tree (find results for these shapes),
    # so a fresh box skips the multi-minute exhaustive search.  With several
    # ranks on one node each gets its own copy (no lock contention on the
    # sqlite caches when they compile / look up kernels at the same time).
    tdir = os.path.join(ROOT, "kungfu_amd", "tuning", "miopen")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and "MIOPEN_USER_DB_PATH" not in os.environ:
        import shutil
        import tempfile

        dst = os.path.join(tempfile.gettempdir(), "kungfu_miopen_%s_%s" % (os.getuid(), os.environ.get("LOCAL_RANK", "0")))
        if not os.path.isdir(dst):
            shutil.copytree(tdir, dst)
        tdir = dst
    os.environ.setdefault("MIOPEN_USER_DB_PATH", tdir)
    os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", tdir)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    # failure detection: a stalled RCCL collective or host op ends the run with a
    # message naming the op and rank (exit 3) instead of hanging until an outer timeout
    os.environ.setdefault("KUNGFU_RCCL_TIMEOUT_S", "300")
    os.environ.setdefault("KUNGFU_OP_TIMEOUT_S", "900")
    # RCCL CTA budget of the gradient all-reduces: >= 16 CTAs per collective (the comm emulation,
    # profiles/r4_comm_emulation.md: fewer cost +0.3 .. +3.4 ms/step at N = 8), at most 64 (a quarter
    # of the 256 CUs' wave slots of one SIMD each, leaving the backward its CUs).  RCCL needs the pair
    # (a floor alone is rejected by ncclCommInitRankConfig).  Reported in verify.rccl_ctas.
    os.environ.setdefault("KUNGFU_RCCL_MIN_CTAS", "16")
    os.environ.setdefault("KUNGFU_RCCL_MAX_CTAS", "64")


def _launcher_env() -> bool:
    return "KUNGFU_SELF_SPEC" in os.environ or "WORLD_SIZE" in os.environ


def _self_launch(n: int) -> int:
    """``--gpus N`` (N > 1) without a launcher: start N ranks (one per GPU) with
    ``torch.distributed.run`` as CHILD processes and return their exit status.  The
    parent never touches the GPU (no HIP call before or after), so nothing is
    re-exec'd from a process holding a device context; rank 0's JSON line reaches
    stdout through the inherited file descriptors."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    print("bench.py: launching %d ranks: %s" % (n, " ".join(cmd)), file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def _elastic_launch(schedule: str) -> int:
    """``--elastic`` without a launcher: run this script under ``kungfu-run -w`` (watch mode,
    built-in config server), starting with the schedule's first size; relay the final
    rank 0's JSON line (the launcher prefixes worker output) to stdout."""
    import socket
    import subprocess

    sizes = [int(p.split(":")[0]) for p in schedule.split(",") if p]

    # below the kernel's ephemeral range: the running job's own sockets (RCCL bootstrap / proxy,
    # stores) get ephemeral ports, which could take a port of a block checked free earlier
    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
            floor = int(f.read().split()[0])
    except (OSError, ValueError, IndexError):
        floor = 32768

    def free_block(n):
        for base in list(range(11000 + (os.getpid() % 97) * 97, floor - n, 97)) + list(range(11000, floor - n, 89)):
            ok = True
            for q in range(base, base + n):
                sk = socket.socket()
                try:
                    sk.bind(("0.0.0.0", q))
                except OSError:
                    ok = False
                finally:
                    sk.close()
                if not ok:
                    break
            if ok:
                return base
        raise RuntimeError("no free port block")

    base = free_block(max(sizes) + 8)
    cfg = base + max(sizes) + 6
    cmd = [os.path.join(ROOT, "bin", "kungfu-run"), "-q", "-w", "-np", str(sizes[0]), "-H", "127.0.0.1:%d" % max(sizes),
           "-port", str(base), "-port-range", "%d-%d" % (base + 1, base + 1 + max(sizes) + 4),
           "-builtin-config-port", str(cfg), "-config-server", "http://127.0.0.1:%d/config" % cfg,
           sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    print("bench.py: elastic run %s: %s" % (schedule, " ".join(cmd)), file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1)
    for line in p.stdout:
        i = line.find('{"metric"')
        if i >= 0:
            print(line[i:].rstrip("\n"), flush=True)
        else:
            sys.stderr.write(line)
    return p.wait()


def _elastic_loop(a, model, opt, step, sync, bert):
    """Config 5 as one command: train through the ``--elastic`` schedule with
    ``ElasticTrainer`` (resize via the config server, state re-broadcast, RCCL communicators
    rebuilt for every cluster version); per phase: throughput (each phase's first step --
    communicator setup, learned bucket order -- is not timed), replica checksum agreement,
    the gradient noise scale; plus every resize's latency.  The final rank 0 prints one JSON.

    Parity: srcs/python/kungfu/tensorflow/experimental/hook/elastic.py:68-84 (ElasticHook +
    ResizeProfiler), benchmarks/adaptation/bench-adaptation.sh, srcs/go/kungfu/peer/peer.go:168-276."""
    import torch

    import kungfu_amd as kf
    from kungfu_amd.elastic import ElasticTrainer

    sched = kf.ops.StepBasedSchedule(a.elastic)
    total = sum(int(p.split(":")[1]) for p in a.elastic.split(",") if p)
    tr = ElasticTrainer(model, opt, local_batch_size=a.batch, schedule=a.elastic)
    phases, cur = [], None
    while True:
        tr.before_step()
        if tr.step >= total:
            break
        n, ver = kf.current_cluster_size(), kf.cluster_version()
        if cur is None or cur["version"] != ver:
            cur = {"version": ver, "np": n, "first_step": tr.step, "steps": 0, "times": []}
            phases.append(cur)
        t0 = time.perf_counter()
        loss = step()
        sync()
        cur["times"].append(time.perf_counter() - t0)
        cur["steps"] += 1
        cur["loss"] = float(loss.detach())
        last = tr.step + 1 >= total
        if last or sched(tr.step + 1) != n:  # phase end: are the replicas identical?
            ck = _replica_checksum(opt, model)
            cks = kf.ops.all_gather(ck).view(n, 2)
            cur["replicas_consistent"] = bool((cks == cks[0:1]).all())
            cur["replica_checksum"] = [float(v) for v in cks[0].tolist()]
            cur["gradient_noise_scale"] = getattr(opt, "noise_scale", None)
        if last:
            tr.step += 1
            break
        if tr.after_step():
            break
    if kf.detached() or kf.current_rank() != 0:
        kf.finalize()
        return
    out = []
    for ph in phases:
        ts = ph["times"][1:] or ph["times"]
        thr = a.batch * ph["np"] * len(ts) / sum(ts)
        out.append({"np": ph["np"], "cluster_version": ph["version"], "first_step": ph["first_step"],
                    "steps": ph["steps"], "timed_steps": len(ts), "value": round(thr, 2),
                    "ms_per_step": round(1000 * sum(ts) / len(ts), 3), "final_loss": round(ph["loss"], 4),
                    "replicas_consistent": ph.get("replicas_consistent"),
                    "gradient_noise_scale": ph.get("gradient_noise_scale")})
    resizes = [{"from": o, "to": nn, "seconds": round(d, 3)} for d, o, nn in tr.profiler.records]
    unit = "sequences/sec" if bert else "images/sec"
    res = {
        "metric": "%s/sec %s elastic %s (%s)" % ("sequences" if bert else "images", a.model, a.optimizer, a.elastic),
        "value": out[-1]["value"] if out else None,
        "unit": unit + " (aggregate over the final phase's ranks)",
        "n_gpus": out[-1]["np"] if out else None,
        "steps": total,
        "higher_is_better": True,
        "dtype": "bf16" if a.device == "cuda" else "f32",
        "data": "synthetic",
        "config": {"model": a.model, "per_gpu_batch": a.batch, "seq_len": a.seq_len if bert else None,
                   "optimizer": a.optimizer, "schedule": a.elastic},
        "phases": out,
        "resizes": resizes,
        "all_phases_consistent": all(p["replicas_consistent"] for p in out),
    }
    print(json.dumps(res), flush=True)
    kf.finalize()


def _replica_checksum(opt, model):
    """(sum, weighted sum) in float64 over every trainable parameter -- equal on every
    rank iff the replicas are (bitwise up to f64 summation) identical."""
    import torch

    space = getattr(opt, "space", None)
    ps = [space.flat_param] if space is not None else [p.detach().reshape(-1) for p in model.parameters()]
    tot = torch.zeros(2, dtype=torch.float64, device=ps[0].device)
    for f in ps:
        f64 = f.detach().double()
        w = torch.arange(1, f64.numel() + 1, device=f64.device, dtype=torch.float64).remainder_(977.0).add_(1.0)
        tot[0] += f64.sum()
        tot[1] += (f64 * w).sum()
    return tot.cpu()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs (ranks) on this node; > 1 without a launcher env self-launches N ranks")
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=8)
    p.add_argument("--batch", type=int, default=None, help="images (sequences) per GPU: 256 (BERT: 128)")
    p.add_argument("--model", default="resnet50")
    p.add_argument("--seq-len", type=int, default=128, help="BERT sequence length")
    p.add_argument("--adam", type=int, default=-1, help="1: AdamW inner optimizer (default for BERT), 0: SGD momentum")
    p.add_argument("--optimizer", default="ssgd", choices=["ssgd", "sma", "pair", "ada", "gns", "local"])
    p.add_argument("--force-comm", type=int, default=1,
                   help="1: S-SGD buckets go through the communicator even with one GPU (RCCL 1-rank all-reduce)")
    p.add_argument("--comm-dtype", default="auto", choices=["auto", "f32", "bf16"],
                   help="gradient dtype on the wire (S-SGD / GNS).  auto: bf16 when gradients cross ranks on GPUs "
                        "(N > 1, or the --emulate-comm model of it), f32 otherwise -- emulated 8 ranks: BERT-base "
                        "18.41-18.55 -> 17.26-17.29 ms/step, ResNet-50 21.09-21.20 -> 21.06-21.08 "
                        "(profiles/r6_multirank_defaults.md)")
    p.add_argument("--overlap", type=int, default=1, help="S-SGD: all-reduce buckets during backward")
    p.add_argument("--fused-bn", type=int, default=-1, help="1: HIP fused BN(+add)+ReLU; -1: auto")
    p.add_argument("--bucket-mb", type=float, default=None)
    p.add_argument("--bf16-shadow", type=int, default=1,
                   help="1: bf16 compute weights from one cast of the flat f32 master + direct bucket gradients")
    p.add_argument("--lr", type=float, default=0.01,
                   help="SGD learning rate; 0.01 = the reference benchmark's (benchmarks/system/benchmark_kungfu.py:99)")
    p.add_argument("--graph", type=int, default=-1,
                   help="1: capture the whole training step into a hipGraph after 3 eager steps and replay it "
                        "(kungfu_amd.parallel.graphs.GraphedStep; N > 1: graph segments with eager collectives); "
                        "-1 (default): on for ResNet-50 / Inception-v3 with S-SGD (replay measured bit-identical "
                        "to eager); off for BERT and VGG-16 (measured no gain)")
    p.add_argument("--json-out", default=None)
    p.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                   help="cpu: f32 on CPU peers over the host transport (tests of the launch / verify path only)")
    p.add_argument("--image-size", type=int, default=224)
    p.add_argument("--preflight", type=int, default=1,
                   help="N > 1: check P2P access, a 64 MiB RCCL all-reduce (values + busbw) and a HIP-IPC pull "
                        "from the neighbouring device before warm-up; exit 5 naming the failing rank pair")
    p.add_argument("--emulate-comm", type=int, default=0, metavar="RANKS",
                   help="N = 1 only: replace every bucket all-reduce by comm_emu.hip, the local footprint (CTAs, "
                        "HBM traffic, modelled xGMI time) of a RANKS-rank ring all-reduce -- a MODEL of the N-rank step")
    p.add_argument("--emulate-ctas", type=int, default=16, help="--emulate-comm: workgroups per all-reduce")
    p.add_argument("--emulate-busbw", type=float, default=350.0, help="--emulate-comm: modelled ring busbw, GB/s")
    p.add_argument("--emulate-lat-us", type=float, default=25.0, help="--emulate-comm: modelled per-collective latency")
    p.add_argument("--comm-probe", type=int, default=3, metavar="STEPS",
                   help="after the timed steps: this many extra (untimed, eager) steps with HIP events around every "
                        "bucket collective -> verify.comm_per_bucket_ms / exposed_comm_ms (0 = off)")
    p.add_argument("--elastic", default=None, metavar="SIZE:STEPS,...",
                   help="elastic run (config 5): resize the job along this schedule, e.g. 4:20,8:20 "
                        "(self-launches kungfu-run -w with its built-in config server)")
    a = p.parse_args()
    if a.elastic and not _launcher_env():
        sys.exit(_elastic_launch(a.elastic))
    if a.gpus is not None and a.gpus > 1 and not _launcher_env():
        sys.exit(_self_launch(a.gpus))
    world_env = int(os.environ.get("WORLD_SIZE", "0")) or None
    bert = a.model.startswith("bert")
    if a.batch is None:
        a.batch = 128 if bert else 256
    if a.adam < 0:
        a.adam = 1 if bert else 0
    _setup_env()
    if a.emulate_comm:
        if a.gpus not in (None, 1) or world_env not in (None, 1) or a.device != "cuda":
            print("bench.py: --emulate-comm models an N-rank job on ONE GPU", file=sys.stderr, flush=True)
            sys.exit(2)
        a.force_comm = 1
        os.environ["KUNGFU_COMM_EMULATE"] = "ranks=%d,ctas=%d,busbw=%g,lat_us=%g" % (
            a.emulate_comm, a.emulate_ctas, a.emulate_busbw, a.emulate_lat_us)

    import torch
    import torch.nn.functional as F

    import kungfu_amd as kf
    from kungfu_amd.models import get_model

    kf.init()
    rank, size = kf.current_rank(), kf.current_cluster_size()
    if a.gpus is None or a.elastic:
        a.gpus = size
    if size != a.gpus or (world_env is not None and world_env != size):
        print("bench.py: --gpus %d but the job has %d ranks (WORLD_SIZE=%s); refusing to report a mislabelled "
              "number" % (a.gpus, size, world_env), file=sys.stderr, flush=True)
        sys.exit(2)
    dev_idx = kf.get_hip_index()
    cuda = a.device == "cuda"
    if cuda:
        torch.cuda.set_device(dev_idx)
        dev = torch.device("cuda", dev_idx)
    else:
        dev = torch.device("cpu")
        a.bf16_shadow = 0

    def sync():
        if cuda:
            torch.cuda.synchronize()
    torch.backends.cudnn.benchmark = False  # MIOpen immediate mode + in-tree find-db
    torch.manual_seed(1234)  # same init everywhere (broadcast_parameters makes it exact)

    fused_bn = a.fused_bn
    if fused_bn < 0:
        from kungfu_amd.ops import fused_bn as fb

        fused_bn = 1 if fb.available() else 0
    model = (get_model(a.model, fused_bn=bool(fused_bn)) if a.model.startswith("resnet") or a.model in ("inception_v3", "vgg16")
             else get_model(a.model))
    model = model.to(dev)
    if not bert:
        model = model.to(memory_format=torch.channels_last) if cuda else model
    if a.adam:
        base = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=0.01)
        opt_desc = "AdamW lr=1e-4 wd=0.01"
    else:
        base = torch.optim.SGD(model.parameters(), lr=a.lr, momentum=0.9, weight_decay=1e-4)
        opt_desc = "SGD momentum=0.9 wd=1e-4"
    if a.comm_dtype == "auto":
        # elastic: every rank must pick the same wire dtype whatever the size it started at (a rank
        # that joins at 2 and one that started alone would otherwise reduce bf16 against f32 and hang)
        a.comm_dtype = "bf16" if cuda and (size > 1 or a.emulate_comm or a.elastic) else "f32"
    comm_dtype = torch.bfloat16 if a.comm_dtype == "bf16" else None
    if a.optimizer == "ssgd":
        opt = kf.optimizers.SynchronousSGDOptimizer(base, named_parameters=model.named_parameters(),
                                                    bucket_mb=a.bucket_mb, overlap=bool(a.overlap),
                                                    force_comm=bool(a.force_comm), comm_dtype=comm_dtype)
    elif a.optimizer == "gns":  # S-SGD + gradient-noise-scale monitor (K5 every step)
        opt = kf.optimizers.MonitorGradientNoiseScaleOptimizer(base, device_batch_size=a.batch,
                                                               named_parameters=model.named_parameters(),
                                                               monitor_single=bool(a.force_comm),
                                                               comm_dtype=comm_dtype)
    elif a.optimizer == "local":  # diagnostics only: fused flat SGD, no gradient exchange
        from kungfu_amd.optimizers.core import KungFuOptimizer

        opt = KungFuOptimizer(base, named_parameters=model.named_parameters())
    elif a.optimizer == "sma":
        opt = kf.optimizers.SynchronousAveragingOptimizer(base, named_parameters=model.named_parameters(),
                                                          force_comm=bool(a.force_comm))
    elif a.optimizer == "pair":
        opt = kf.optimizers.PairAveragingOptimizer(base, named_parameters=model.named_parameters(),
                                                   force_comm=bool(a.force_comm) and cuda)
    else:
        opt = kf.optimizers.AdaptiveSGDOptimizer(base, named_parameters=model.named_parameters(), change_step=10)
    if not a.elastic:  # elastic: ElasticTrainer broadcasts at every membership change
        kf.broadcast_parameters(model.state_dict())
    if a.bf16_shadow and getattr(opt, "space", None) is not None:
        from kungfu_amd.parallel.mixed import enable_bf16_shadow

        enable_bf16_shadow(model, opt)

    # every rank draws its own synthetic batch, so identical replicas at the end prove
    # that the gradient exchange (not identical inputs) kept them in step
    torch.manual_seed(1234 + 7919 * rank)
    if bert:
        from kungfu_amd.models.bert import pretraining_loss, synthetic_pretraining_batch

        data = synthetic_pretraining_batch(a.batch, a.seq_len, device=dev)

        def compute_loss():
            return pretraining_loss(model, data)
    else:
        x = torch.randn(a.batch, 3, a.image_size, a.image_size, device=dev)
        x = x.to(memory_format=torch.channels_last) if cuda else x
        y = torch.randint(0, 1000, (a.batch,), device=dev)

        def compute_loss():
            return F.cross_entropy(model(x).float(), y)

    def step():
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=cuda):
            loss = compute_loss()
        loss.backward()
        opt.step()
        return loss

    if a.elastic:
        return _elastic_loop(a, model, opt, step, sync, bert)
    graphed = None
    if a.graph < 0:
        # ResNet-50 / Inception-v3 with S-SGD.  N = 1: one whole-step graph.  N > 1 (and the 1-GPU
        # model of it, --emulate-comm): graph SEGMENTS cut at every bucket launch with the collectives
        # issued eagerly between replays (parallel/graphs.py) for ResNet-50 -- emulated 8-rank
        # 21.15-21.18 vs eager 21.19-21.22 ms/step (r5t6; one graph with the collectives inside:
        # 21.55-21.59) -- but EAGER for Inception-v3, whose segments measured slower (emulated 8-rank
        # 20.45 vs 20.32-20.34 ms, r6t11; r5: 20.92-20.95 vs 20.81-20.83).  BERT: replay measured
        # 2.4 % slower (r4t31); VGG-16: +0.4 % only (r4_host_overhead.md)
        multi = size > 1 or bool(a.emulate_comm)
        a.graph = 0 if (bert or a.model == "vgg16" or a.optimizer not in ("ssgd", "local")
                        or (a.model == "inception_v3" and multi)) else 1
    if a.graph and cuda:
        from kungfu_amd.parallel.graphs import GraphedStep

        graphed = GraphedStep(step, opt, warmup=3)
        step = graphed
        a.warmup = max(a.warmup, 4)  # the capture happens inside warm-up

    preflight = None
    if size > 1 and a.preflight:
        # before warm-up: a broken link / IPC path is named here instead of hanging a step
        from kungfu_amd.parallel import preflight as pf

        try:
            preflight = pf.run(dev)
        except pf.PreflightError as e:
            print("bench.py: rank %d: %s" % (rank, e), file=sys.stderr, flush=True)
            if rank == 0:
                print("bench.py: pre-flight report: %s" % json.dumps(e.report), file=sys.stderr, flush=True)
            kf.finalize()
            sys.exit(5)

    t_w0 = time.time()
    first_loss = None
    warm_losses = []
    for i in range(a.warmup):
        l0 = step().detach()  # no reference to the step's autograd graph outlives the step
        warm_losses.append(float(l0))
        if i == 0:
            first_loss = float(l0)
    sync()
    warm_s = time.time() - t_w0
    # the timed steps' losses: one 4-byte device copy per step (a replayed graph returns the same
    # static tensor every step), read back after the timed region
    loss_buf = torch.zeros(a.steps, dtype=torch.float32, device=dev)

    kf.run_barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = step().detach()
        loss_buf[i].copy_(loss)
    sync()
    kf.run_barrier()
    dt = time.perf_counter() - t0
    # max over ranks (host transport, outside the timed region); per-rank spread
    dt_all = (kf.ops.all_gather(torch.tensor([dt], dtype=torch.float64)).view(-1).tolist() if size > 1 else [dt])
    dt_max = max(dt_all)
    value = a.batch * size * a.steps / dt_max
    reducer = getattr(opt, "reducer", None)
    comm_probe = None
    if a.comm_probe > 0 and cuda and reducer is not None and not reducer.skip:
        # untimed: where an N-rank step's communication goes, per bucket (HIP events, eager steps)
        reducer.probe = []
        for _ in range(a.comm_probe):
            (graphed._eager() if graphed is not None else step()).detach()
        comm_probe = reducer.probe_summary()
        reducer.probe = None
        sync()
    if reducer is not None:
        comm_info = reducer.describe()
    elif getattr(opt, "averager", None) is not None:  # SMA / AdaSGD: model all-reduce per step
        c = opt.averager.comm
        comm_info = {"comm_ranks": c.size if c is not None else size, "comm_plane": c.plane if c is not None else "skip",
                     "comm_bytes_per_step": opt.space.numel * 4 if c is not None else 0, "overlap": True}
    elif getattr(opt, "store", None) is not None:  # pair averaging: device model store pulls
        comm_info = {"comm_ranks": size, "comm_plane": "ipc" if size > 1 else "ipc-self",
                     "pulls": opt.pulls, "dropped": opt.store.dropped, "prefetch": opt.prefetcher is not None,
                     "comm_bytes_per_step": opt.space.numel * 4}
    else:
        comm_info = {"comm_ranks": size}
    # replica consistency: after synchronous training every rank holds the same weights
    ck = _replica_checksum(opt, model)
    cks = kf.ops.all_gather(ck).view(size, 2) if size > 1 else ck.view(1, 2)
    sync_algo = a.optimizer in ("ssgd", "gns")
    consistent = bool((cks == cks[0:1]).all()) if sync_algo else None
    try:
        rccl_ver = kf.show_rccl_version()
    except Exception:
        rccl_ver = None
    from kungfu_amd._lib import hip as _hip_mod

    try:
        # every collective has completed (synchronised above); give the watchdog thread (50 ms
        # poll period) a moment to retire their events before reading its counters
        t_wd = time.time() + 2.0
        wd = dict(_hip_mod().rccl_watchdog_info())
        while wd["pending"] and time.time() < t_wd:
            time.sleep(0.02)
            wd = dict(_hip_mod().rccl_watchdog_info())
    except Exception:
        wd = None
    verify = {
        "launch": kf.launch_mode(),
        "world_size": size,
        "comm_ranks": comm_info.get("comm_ranks", size),
        "comm_plane": comm_info.get("comm_plane"),
        "rccl_version": rccl_ver,
        "per_rank_img_s": {"min": round(a.batch * a.steps / max(dt_all), 2),
                           "max": round(a.batch * a.steps / min(dt_all), 2)},
        "replicas_consistent": consistent,
        "replica_checksum": [float(x) for x in cks[0].tolist()],
        "rccl_watchdog": ({"ops_watched": wd["registered"], "pending": wd["pending"], "timeout_s": wd["timeout_s"],
                           "abort_on_stall": wd.get("abort_on_stall")} if wd else None),
        "rccl_ctas": list(getattr(getattr(reducer, "comm", None), "ctas", (0, 0)) or (0, 0)),
        "comm_per_bucket_ms": comm_probe["comm_per_bucket_ms"] if comm_probe else None,
        "exposed_comm_ms": comm_probe["exposed_comm_ms"] if comm_probe else None,
        "comm_probe": comm_probe,
        "preflight": preflight if preflight is not None else ("skipped (one rank)" if size == 1 else "disabled"),
    }
    if sync_algo and not consistent:
        print("bench.py: REPLICAS DIVERGED: per-rank checksums %s" % cks.tolist(), file=sys.stderr, flush=True)
    losses = [round(v, 4) for v in loss_buf.tolist()]
    if rank == 0 and first_loss is not None and losses and losses[-1] > first_loss:
        print("bench.py: WARNING: the loss rose over the run (%.4f -> %.4f at lr %g): a numerics regression or "
              "a learning rate too high for this synthetic batch" % (first_loss, losses[-1], a.lr),
              file=sys.stderr, flush=True)
    metric, base_per_gpu = MODEL_BASELINES.get(a.model, (METRIC.replace("ResNet-50", a.model), None))
    if a.emulate_comm:  # a model, never the headline: say so in the metric itself
        metric = "MODEL (1 GPU, %d-rank comm emulated): %s" % (a.emulate_comm, metric)
        base_per_gpu = None
        comm_info["emulated"] = reducer.comm.describe() if reducer is not None and reducer.comm is not None else None
    unit = "sequences/sec (aggregate over n_gpus)" if bert else "images/sec (aggregate over n_gpus)"
    res = {
        "metric": metric,
        "value": round(value, 2),
        "unit": unit,
        "n_gpus": size,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(1000 * dt_max / a.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / (base_per_gpu * size), 3) if base_per_gpu else None,
        "dtype": "bf16" if cuda else "f32",
        "data": ("synthetic (random token ids, 20 masked positions per sequence, random MLM/NSP labels; "
                 "random-init weights)" if bert else
                 "synthetic (random %dx%dx3 images, random labels; random-init weights)" % (a.image_size, a.image_size)),
        "config": {
            "model": a.model,
            "global_batch": a.batch * size,
            "per_gpu_batch": a.batch,
            "seq_len": a.seq_len if bert else None,
            "image_size": None if bert else a.image_size,
            "parallelism": "dp%d" % size,
            "optimizer": "%s(%s)" % (a.optimizer, opt_desc),
            "fused_bn_hip": bool(fused_bn),
            "bf16_shadow_weights": bool(a.bf16_shadow),
            "hip_graph": ({"replays": graphed.replays, "captured": graphed.graph is not None, "disabled": graphed.disabled,
                           "segments": len(graphed.segs) if graphed.segs else (1 if graphed.graph is not None else 0)}
                          if graphed is not None else False),
            "per_gpu_img_s": round(value / size, 2),
            "tokens_per_s": round(value * a.seq_len, 1) if bert else None,
            "gradient_noise_scale": (opt.noise_scale if a.optimizer == "gns" else None),
            "baseline_per_gpu_img_s": round(base_per_gpu, 1) if base_per_gpu else None,
            "warmup_s": round(warm_s, 1),
            "initial_loss": round(first_loss, 4) if first_loss is not None else None,
            "final_loss": round(float(loss.detach()), 4),
            "lr": a.lr if not bert else None,
            "warmup_losses": [round(v, 4) for v in warm_losses],
            "losses": losses,
            "comm": comm_info,
        },
        "verify": verify,
    }
    if rank == 0:
        line = json.dumps(res)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    kf.finalize()
    if sync_algo and not consistent:
        sys.exit(4)


if __name__ == "__main__":
    main()
