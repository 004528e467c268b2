"""Multi-GPU pre-flight: prove the data planes work before a job spends its time training.

Run by ``bench.py --gpus N`` (N > 1) before warm-up (and usable by any trainer), so that the
first run on a new node diagnoses itself instead of hanging or reporting a meaningless number.
Every rank checks:

1. **P2P matrix** -- ``hipDeviceCanAccessPeer`` and ``hipExtGetLinkTypeAndHopCount`` from its
   device to the device of every other rank (link type 4 = xGMI; "n/a" when ranks share a
   device, e.g. the colocated one-GPU tests).
2. **RCCL all-reduce** of 64 MiB with a value check (every element is an exact integer sum)
   and the measured bus bandwidth ``2 (n-1)/n * bytes / t`` (rccl-tests' definition).
3. **HIP-IPC pull** of one buffer exported by the NEXT rank (the pair-averaging store's
   transport: ``hipIpcOpenMemHandle`` + a device copy over xGMI), compared bytewise with the
   pattern that rank wrote, plus its bandwidth.

The per-rank results are all-gathered over the HOST transport (independent of RCCL / xGMI), so
every rank learns every failure; on any failure each rank raises :class:`PreflightError` naming
the failing rank pairs (bench.py exits 5).  With CPU tensors only the value check runs (host
plane).  A stalled RCCL check is bounded (``KUNGFU_PREFLIGHT_TIMEOUT_S``, default 60 s).

Bounded on the stall paths: a rank whose all-reduce did not complete says so over the
host transport and EVERY rank then skips the IPC check (its device work would queue behind the
stuck collective); the IPC fill is ordered by an event wait bounded like the others, never a
device-wide synchronise; and a pull that timed out keeps both its mapping and the exporter's
buffer alive (the copy may still be in flight) -- the process is about to fail anyway.

Test hook: ``KUNGFU_PREFLIGHT_CORRUPT=<rank>`` makes that rank corrupt one element of its IPC
buffer after filling it (``ipc``) or of its all-reduce contribution (``KUNGFU_PREFLIGHT_CORRUPT_WHAT
=allreduce``), or report its all-reduce as stalled without stalling it (``stall``), so the failure
paths are exercised.

Parity: the reference checks every NCCL call's result and synchronises
(``srcs/cpp/src/nccl/gpu_collective.cpp:96-152``); it has no pre-flight -- this is the
MI355X-first replacement for discovering a broken link in the middle of training.
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, List, Optional

import torch

from .. import ops
from .._lib import hip, runtime

_ALLREDUCE_BYTES = 64 << 20
_IPC_BYTES = 16 << 20
_PATTERN = 251


class PreflightError(RuntimeError):
    def __init__(self, msg: str, report: dict):
        super().__init__(msg)
        self.report = report


def _corrupt(what: str) -> bool:
    r = os.environ.get("KUNGFU_PREFLIGHT_CORRUPT")
    return (r is not None and r != "" and int(r) == runtime.rank()
            and os.environ.get("KUNGFU_PREFLIGHT_CORRUPT_WHAT", "ipc") == what)


def _pattern(n: int, rank: int, device) -> torch.Tensor:
    """(rank + 1) * (i % 251 + 1): integers, so sums over ranks are exact in f32."""
    i = torch.arange(n, device=device, dtype=torch.int64).remainder_(_PATTERN).add_(1).float()
    return i.mul_(rank + 1)


def _wait(ev: torch.cuda.Event, timeout_s: float, what: str) -> bool:
    t_end = time.time() + timeout_s
    while not ev.query():
        if time.time() > t_end:
            return False
        time.sleep(0.001)
    return True


def _allgather_json(obj: dict, name: str) -> List[dict]:
    """All-gather one JSON document per rank over the host transport (fixed 4 KiB slots)."""
    raw = json.dumps(obj, separators=(",", ":")).encode()
    slot = 4096
    if len(raw) > slot:
        raw = json.dumps({"rank": obj.get("rank"), "ok": obj.get("ok"), "errors": obj.get("errors", [])[:4],
                          "truncated": True}).encode()[:slot]
    buf = torch.zeros(slot, dtype=torch.uint8)
    buf[:len(raw)] = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
    allb = ops.all_gather(buf, name=name).view(-1, slot)
    out = []
    for row in allb:
        b = bytes(row.tolist()).rstrip(b"\0")
        out.append(json.loads(b.decode()))
    return out


def _p2p(dev_index: int, devs: List[int]) -> dict:
    links = {int(p): (int(c), int(t), int(h)) for p, c, t, h in hip().device_links(dev_index)}
    row = {}
    for r, d in enumerate(devs):
        if r == runtime.rank():
            continue
        if d == dev_index:
            row[str(r)] = "n/a (same device)"
        elif d in links:
            c, t, h = links[d]
            row[str(r)] = {"device": d, "can_access_peer": bool(c == 1), "link_type": t,
                           "link": {4: "xgmi", 2: "pcie"}.get(t, str(t)), "hops": h}
        else:
            row[str(r)] = "n/a (device %d not visible)" % d
    return row


def _check_allreduce(comm, device, timeout_s: float) -> dict:
    n = runtime.size()
    elems = _ALLREDUCE_BYTES // 4
    rank = runtime.rank()
    x = _pattern(elems, rank, device)
    if _corrupt("allreduce"):
        x[elems // 3] += 1.0
    want_scale = n * (n + 1) / 2
    if device.type == "cpu":
        t0 = time.perf_counter()
        x = ops.all_reduce(x, op="sum", name="kf:preflight:ar")
        dt = time.perf_counter() - t0
        bad = int((x != _pattern(elems, 0, device).mul_(want_scale)).sum())
        return {"ok": bad == 0, "bad_elements": bad, "bytes": _ALLREDUCE_BYTES, "plane": "host",
                "busbw_gbs": round(2 * (n - 1) / n * _ALLREDUCE_BYTES / dt / 1e9, 2)}
    s = comm.stream
    s.wait_stream(torch.cuda.current_stream(device))
    reps = 5
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    with torch.cuda.stream(s):
        y = torch.empty_like(x)
        comm.all_reduce(x, y, op="sum", stream=s, tag="preflight warm-up")
        ok = _wait_record(s, timeout_s)
        if not ok:
            return {"ok": False, "stalled": True, "plane": comm.plane,
                    "error": "RCCL all-reduce did not complete within %.0f s" % timeout_s}
        bad = int((y != _pattern(elems, 0, device).mul_(want_scale)).sum())
        evs[0].record(s)
        for _ in range(reps):
            comm.all_reduce(x, y, op="sum", stream=s, tag="preflight timing")
        evs[1].record(s)
        if not _wait(evs[1], timeout_s, "timing"):
            return {"ok": False, "stalled": True, "plane": comm.plane,
                    "error": "RCCL all-reduce timing loop did not complete within %.0f s" % timeout_s}
    t = evs[0].elapsed_time(evs[1]) / 1e3 / reps
    return {"ok": bad == 0, "bad_elements": bad, "bytes": _ALLREDUCE_BYTES, "plane": comm.plane,
            "ms": round(t * 1e3, 3), "algbw_gbs": round(_ALLREDUCE_BYTES / t / 1e9, 2),
            "busbw_gbs": round(2 * (n - 1) / n * _ALLREDUCE_BYTES / t / 1e9, 2),
            "ctas": list(getattr(comm, "ctas", (0, 0)))}


def _wait_record(stream, timeout_s: float) -> bool:
    ev = torch.cuda.Event()
    ev.record(stream)
    return _wait(ev, timeout_s, "")


# buffers of a timed-out IPC pull: a copy may still be reading / writing them, so they are never
# freed (the pre-flight is failing; the process exits soon after)
_LEAKED: list = []


def _check_ipc(device, timeout_s: float) -> dict:
    """Export one buffer with this rank's pattern, pull the next rank's over HIP IPC, compare."""
    H = hip()
    n, rank = runtime.size(), runtime.rank()
    elems = _IPC_BYTES // 4
    buf = H.ipc_alloc(elems, device.index)
    buf.copy_(_pattern(elems, rank, device))
    if _corrupt("ipc"):
        buf[elems // 2] = -1.0
    # the fill must be complete before a peer pulls: wait for THIS stream's work, bounded (a
    # device-wide synchronise would also wait for other streams' possibly stuck work)
    filled = _wait_record(torch.cuda.current_stream(device), timeout_s)
    mine = torch.frombuffer(bytearray(H.ipc_handle(buf)), dtype=torch.uint8).clone()
    allh = ops.all_gather(mine, name="kf:preflight:ipc")
    peer = (rank + 1) % n
    hosts = runtime.peers().split(",")
    pending = False
    if not filled:
        res = {"ok": False, "peer": peer, "error": "IPC buffer fill did not complete within %.0f s" % timeout_s}
        pending = True
    elif hosts[peer].split(":")[0] != hosts[rank].split(":")[0]:
        res = {"ok": True, "peer": peer, "skipped": "peer on another host (no IPC)"}
    else:
        try:
            remote = H.ipc_open(bytes(allh[peer].tolist()), elems, device.index)
            local = torch.empty(elems, dtype=torch.float32, device=device)
            local.copy_(remote)  # warm (maps, enables peer access)
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            local.copy_(remote)
            en.record()
            if not _wait(en, timeout_s, "ipc"):
                res = {"ok": False, "peer": peer, "error": "IPC pull did not complete within %.0f s" % timeout_s}
                pending = True
                _LEAKED.extend([remote, local])
            else:
                bad = int((local != _pattern(elems, peer, device)).sum())
                t = st.elapsed_time(en) / 1e3
                res = {"ok": bad == 0, "peer": peer, "bad_elements": bad, "bytes": _IPC_BYTES,
                       "pull_gbs": round(_IPC_BYTES / t / 1e9, 2)}
            del remote
        except Exception as e:  # noqa: BLE001 -- reported, then raised collectively
            res = {"ok": False, "peer": peer, "error": "%s: %s" % (type(e).__name__, e)}
    # every rank is done reading before any owner frees its exported buffer; an owner whose
    # buffer a peer may still be copying (that peer's pull timed out) keeps it
    flags = ops.all_gather(torch.tensor([1 if pending else 0], dtype=torch.int32),
                           name="kf:preflight:ipc_done").view(-1).tolist()
    if any(flags):
        _LEAKED.append(buf)
    del buf
    return res


def run(device: Optional[torch.device] = None, comm=None) -> dict:
    """Run the pre-flight on every rank (collective); returns the job-wide report.
    Raises :class:`PreflightError` on every rank if any check failed anywhere."""
    from .comm import get_device_comm

    n, rank = runtime.size(), runtime.rank()
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    timeout_s = float(os.environ.get("KUNGFU_PREFLIGHT_TIMEOUT_S", "60"))
    t0 = time.time()
    mine: Dict[str, object] = {"rank": rank, "errors": []}
    cuda = device.type == "cuda"
    devs = [int(v) for v in ops.all_gather(torch.tensor([device.index if cuda else -1], dtype=torch.int64),
                                           name="kf:preflight:devs").view(-1).tolist()]
    mine["device"] = devs[rank]
    if cuda:
        try:
            mine["p2p"] = _p2p(device.index, devs)
            for r, v in mine["p2p"].items():
                if isinstance(v, dict) and not v["can_access_peer"]:
                    mine["errors"].append("no peer access %d -> %s (device %d -> %d)" % (rank, r, device.index,
                                                                                           v["device"]))
        except Exception as e:  # noqa: BLE001
            mine["p2p"] = "error: %s" % e
            mine["errors"].append("P2P query failed on rank %d: %s" % (rank, e))
    if comm is None:
        comm = get_device_comm(device=device)
    try:
        ar = _check_allreduce(comm, device, timeout_s)
    except Exception as e:  # noqa: BLE001
        ar = {"ok": False, "error": "%s: %s" % (type(e).__name__, e)}
    if _corrupt("stall"):
        # test hook: the collective ran (the peers are not left waiting in it), this rank then
        # reports it as stalled -- the stall path without a stuck kernel on the box
        ar = {"ok": False, "stalled": True, "plane": ar.get("plane", "?"),
              "error": "all-reduce did not complete within %.0f s (simulated)" % timeout_s}
    mine["allreduce"] = ar
    if not ar["ok"]:
        mine["errors"].append("all-reduce check failed on rank %d: %s" % (
            rank, ar.get("error") or "%d wrong elements" % ar.get("bad_elements", -1)))
    # the IPC check queues device work; behind a stuck collective it would hang -- skip it on
    # every rank (the decision is collective, over the host transport) if any rank stalled
    stalled = [r for r, v in enumerate(ops.all_gather(torch.tensor([1 if ar.get("stalled") else 0],
                                                                   dtype=torch.int32),
                                                      name="kf:preflight:stalled").view(-1).tolist()) if v]
    if cuda and n > 1 and stalled:
        mine["ipc"] = {"ok": True, "peer": (rank + 1) % n,
                       "skipped": "all-reduce stalled on rank(s) %s" % ",".join(map(str, stalled))}
    elif cuda and n > 1:
        ipc = _check_ipc(device, timeout_s)
        mine["ipc"] = ipc
        if not ipc["ok"]:
            mine["errors"].append("IPC pull %d <- %d failed: %s" % (
                rank, ipc["peer"], ipc.get("error") or "%d wrong elements" % ipc.get("bad_elements", -1)))
    mine["ok"] = not mine["errors"]
    rows = _allgather_json(mine, "kf:preflight:report")
    errors = [e for r in rows for e in r.get("errors", [])]
    report = {"ok": not errors, "ranks": n, "seconds": round(time.time() - t0, 2), "devices": devs,
              "allreduce_busbw_gbs": {str(r["rank"]): r.get("allreduce", {}).get("busbw_gbs") for r in rows},
              "ipc_pull_gbs": {str(r["rank"]): (r.get("ipc") or {}).get("pull_gbs") for r in rows},
              "p2p": {str(r["rank"]): r.get("p2p", "n/a") for r in rows},
              "rccl_ctas": (rows[0].get("allreduce") or {}).get("ctas"),
              "ipc_skipped": {str(r["rank"]): (r.get("ipc") or {}).get("skipped") for r in rows
                              if (r.get("ipc") or {}).get("skipped")},
              "errors": errors}
    if errors:
        raise PreflightError("pre-flight failed: " + "; ".join(errors), report)
    return report
