"""PairAveragingOptimizer (AD-PSGD: asynchronous decentralized pair averaging).

Parity: ``srcs/python/kungfu/tensorflow/optimizers/async_sgd.py:13-142``: each
step pick a random peer != self, *pull* its (fused) model from its store,
``v <- (v + v_peer) / 2``, apply local gradients, save the model to the own
store; a save + barrier at step 0; no global synchronisation afterwards.

MI355X design:
* the model store is device resident: three dedicated HIP allocations per peer
  (a ring), exported with HIP IPC at start-up (handles exchanged once through
  the host runtime's all-gather).  A pull is a one-sided device copy from the
  peer's buffer over xGMI -- the owner does not participate -- then one fused
  K4 kernel averages into the flat parameter buffer.
* publication protocol (torn-read free, unlike the reference's unguarded blob,
  SURVEY §5.2): the owner snapshots version k into ring slot k % 3 at the end
  of step k, and ADVERTISES ``(slot, k)`` in its host store at the start of
  step k+1, after host-waiting on that copy's event -- an advertised slot is
  always complete.  Slot k % 3 is next written by snapshot k+3, which is issued
  only after version k+2 has been advertised.  A reader therefore (1) fetches
  the 16-byte record, (2) copies the slot and waits for its own copy, (3)
  fetches the record again: if the advertised version advanced by 2 or more
  the copy may overlap a rewrite and is dropped (``dropped`` counts them), else
  it is an exact snapshot of version k.
* peers on other hosts (no IPC) are pulled through the host P2P store
  (device -> host snapshot on the owner, TCP pull on the reader), which copies
  under the store's lock.
CPU tensors use the host P2P store for everything.
"""
from __future__ import annotations

import random
import struct
from typing import Dict, List, Optional

import torch

from .. import ops
from .._lib import dtype_code, hip, runtime
from ..utils.trace import traced
from .core import KungFuOptimizer

_REC = "kf:pair:rec"


class DeviceModelStore:
    SLOTS = 3

    def __init__(self, numel: int, device: torch.device, name: str):
        H = hip()
        self.numel = numel
        self.name = name
        self.device = device
        self.rank, self.size = runtime.rank(), runtime.size()
        self.bufs = [H.ipc_alloc(numel, device.index) for _ in range(self.SLOTS)]
        hs = b"".join(H.ipc_handle(b) for b in self.bufs)
        mine = torch.frombuffer(bytearray(hs), dtype=torch.uint8).clone()
        allh = ops.all_gather(mine, name="kf:pair:handles:" + name)
        hosts = runtime.peers().split(",")
        my_host = hosts[self.rank].split(":")[0]
        self.local: Dict[int, bool] = {}
        self.peer_bufs: Dict[int, List[torch.Tensor]] = {}
        for r in range(self.size):
            if r == self.rank:
                continue
            same_host = hosts[r].split(":")[0] == my_host
            self.local[r] = same_host
            if same_host:
                raw = bytes(allh[r].tolist())
                self.peer_bufs[r] = [H.ipc_open(raw[i * 64:(i + 1) * 64], numel, device.index)
                                     for i in range(self.SLOTS)]
        self.cross_host = not all(self.local.values()) if self.local else False
        self.version = 0  # last advertised version
        self._next = 0  # version of the next snapshot
        self._pending: Optional[torch.cuda.Event] = None
        self._pending_ver = 0
        self._host_copy = None
        self.dropped = 0
        self.last_pulled = None  # (peer, version) of the last accepted pull

    def publish(self, flat: torch.Tensor):
        """Snapshot ``flat`` into ring slot version % 3 (stream-ordered)."""
        self._next += 1
        ver = self._next
        self.bufs[ver % self.SLOTS].copy_(flat, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._pending, self._pending_ver = ev, ver
        if self.cross_host:
            self._host_copy = flat.detach().to("cpu", non_blocking=False)

    def advertise(self):
        if self._pending is None:
            return
        self._pending.synchronize()  # issued one iteration ago: normally already complete
        self.version = self._pending_ver
        rec = torch.tensor([self.version % self.SLOTS, self.version], dtype=torch.int64)
        runtime.save(_REC + self.name, rec.data_ptr(), 16)
        if self._host_copy is not None:
            runtime.save("kf:pair:model:" + self.name, self._host_copy.data_ptr(), self.numel * 4)
        self._pending = None

    def _record(self, target: int):
        if target == self.rank:  # forced self-pull (one peer): the own advertised record
            return (self.version % self.SLOTS, self.version) if self.version else None
        rec = torch.zeros(2, dtype=torch.int64)
        if not runtime.request(target, "", _REC + self.name, rec.data_ptr(), 16):
            return None
        return int(rec[0]), int(rec[1])

    @traced("pair::pull")
    def pull(self, target: int, out: torch.Tensor, stream=None, after_event=None) -> Optional[torch.cuda.Event]:
        """Copy ``target``'s latest advertised snapshot into ``out``.  Returns the copy's
        completion event (None: nothing valid was pulled).  The copy runs on ``stream``
        (default: current) after ``after_event``; this call host-waits for it (it is meant
        to run on the prefetch thread, off the training loop's critical path)."""
        rec = self._record(target)
        if rec is None:
            return None
        slot, ver = rec
        if target == self.rank or self.local.get(target, False):
            src = self.bufs[slot] if target == self.rank else self.peer_bufs[target][slot]
            s = stream if stream is not None else torch.cuda.current_stream(self.device)
            with torch.cuda.stream(s):
                if after_event is not None:
                    s.wait_event(after_event)
                out.copy_(src, non_blocking=True)
                done = torch.cuda.Event()
                done.record(s)
            done.synchronize()
            after = self._record(target)
            if after is None or after[1] - ver >= self.SLOTS - 1:
                self.dropped += 1  # the owner may have started rewriting this slot
                return None
            self.last_pulled = (target, ver)
            return done
        h = torch.empty(self.numel, dtype=torch.float32)
        if not runtime.request(target, "", "kf:pair:model:" + self.name, h.data_ptr(), self.numel * 4):
            return None
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        with torch.cuda.stream(s):
            if after_event is not None:
                s.wait_event(after_event)
            out.copy_(h, non_blocking=False)
            done = torch.cuda.Event()
            done.record(s)
        done.synchronize()
        self.last_pulled = (target, ver)
        return done


class _Prefetcher:
    """Pulls the NEXT step's peer model on a host thread + a dedicated copy stream while
    the training loop enqueues forward/backward (parity: the reference's
    ``AsyncModelAveraging`` / ``AsyncRequestModel`` prefetch buffer with a callback,
    srcs/cpp/src/tensorflow/ops/cpu/peer_to_peer.cpp:166-238,424-510).  The thread first
    advertises the snapshot published at the end of the step (its host wait on that copy
    happens here, not in the training loop), then pulls; the compute stream only waits on
    the copy's event."""

    def __init__(self, store: DeviceModelStore, out: torch.Tensor):
        import threading

        self.store, self.out = store, out
        self.stream = torch.cuda.Stream(device=store.device)
        self._threading = threading
        self.thread = None
        self.result: Optional[torch.cuda.Event] = None
        self.error: Optional[BaseException] = None

    def start(self, target: int, consumed: Optional[torch.cuda.Event]):
        def run():
            try:
                torch.cuda.set_device(self.store.device)
                self.store.advertise()
                self.result = self.store.pull(target, self.out, stream=self.stream, after_event=consumed)
            except BaseException as e:  # noqa: BLE001 -- re-raised in the training thread
                self.error = e

        self.result, self.error = None, None
        self.thread = self._threading.Thread(target=run, name="kungfu-pair-prefetch", daemon=True)
        self.thread.start()
        if not getattr(self, "_atexit", False):  # never leave a pull in flight at shutdown
            import atexit

            atexit.register(self._drain)
            self._atexit = True

    def _drain(self):
        t = self.thread
        if t is not None:
            t.join(timeout=60)

    def finish(self) -> Optional[torch.cuda.Event]:
        if self.thread is None:
            return None
        self.thread.join()
        self.thread = None
        if self.error is not None:
            raise self.error
        return self.result


class _NativePrefetcher:
    """The same prefetch on a C++ thread (csrc/kernels/pair_prefetch.hip): advertise + pull without
    Python or the GIL off the training thread; ``finish`` makes the compute stream wait on the
    copy natively (returns True), so the training loop only enqueues the averaging kernel."""

    def __init__(self, store: DeviceModelStore, out: torch.Tensor):
        import os

        from .. import _lib

        lib = os.path.join(os.path.dirname(os.path.abspath(_lib.__file__)), "lib", "libkungfu_amd.so")
        self.store, self.out = store, out
        self.p = hip().PairPrefetcher(lib, store.device.index, store.rank, _REC + store.name,
                                      "kf:pair:model:" + store.name, store.numel * 4, store.SLOTS)
        self.stage = (torch.empty(store.numel, dtype=torch.float32, pin_memory=True) if store.cross_host else None)
        self.thread = None  # truthy while a job is in flight (synchronize() checks it)
        self._keep = ()
        self._target = -1

    def start(self, target: int, consumed: Optional[torch.cuda.Event]):
        st = self.store
        pend, host = st._pending, st._host_copy
        own = st.version
        if pend is not None:  # advertised by the native thread: the store's state moves on now
            st.version, st._pending = st._pending_ver, None
        if target == st.rank:
            src = [b.data_ptr() for b in st.bufs]
        elif st.local.get(target, False):
            src = [b.data_ptr() for b in st.peer_bufs[target]]
        else:
            src = []
        self._keep = (pend, host, consumed)  # alive until the native thread is done with them
        self._target = target
        self.p.start(pend.cuda_event if pend is not None else 0, st.version if pend is not None else 0,
                     host.data_ptr() if (pend is not None and host is not None) else 0, target, src, own,
                     self.out.data_ptr(), consumed.cuda_event if consumed is not None else 0,
                     self.stage.data_ptr() if self.stage is not None else 0)
        self.thread = True

    def finish(self):
        if not self.thread:
            return None
        status, ver, _ = self.p.finish(torch.cuda.current_stream(self.store.device).cuda_stream)
        self.thread, self._keep = None, ()
        if status == 2:
            self.store.dropped += 1
            return None
        if status != 1:
            return None
        self.store.last_pulled = (self._target, ver)
        return True  # the current stream already waits on the copy


class _PairAveraging(KungFuOptimizer):
    def __init__(self, optimizer, named_parameters=None, fuse_requests: bool = True,
                 fused_model_name: str = "model", fused: bool = True, seed: Optional[int] = None,
                 peer_selection: str = "random", prefetch: bool = True, force_comm: bool = False):
        super().__init__(optimizer, named_parameters, fused=fused)
        self.force_comm = force_comm
        if peer_selection not in ("random", "roundrobin"):
            raise ValueError("peer_selection must be 'random' or 'roundrobin'")
        self.peer_selection = peer_selection
        self._rr = 0
        self.fused_model_name = fused_model_name
        self.fuse_requests = fuse_requests
        self.rank, self.size = runtime.rank(), runtime.size()
        self.rng = random.Random(self.rank if seed is None else seed + self.rank)
        self.step_count = 0
        self.last_target = -1
        self.store: Optional[DeviceModelStore] = None
        self.prefetcher: Optional[_Prefetcher] = None
        self.pulls = 0
        if self.space is not None and (self.size > 1 or force_comm) and self.space.device.type == "cuda":
            self.store = DeviceModelStore(self.space.numel, self.space.device, fused_model_name)
            self._other = torch.empty_like(self.space.flat_param)
            if prefetch:
                native = hasattr(hip(), "PairPrefetcher")
                self.prefetcher = (_NativePrefetcher if native else _Prefetcher)(self.store, self._other)
        self._consumed: Optional[torch.cuda.Event] = None

    def random_peer(self) -> int:
        if self.size == 1:
            return 0  # force_comm: self-pull
        t = self.rng.randrange(self.size)
        return (t + 1) % self.size if t == self.rank else t

    def next_peer(self) -> int:
        """Peer for this step: uniform random (AD-PSGD) or round-robin over the others
        (the reference's SelectionStrategy, ops/cpu/peer_to_peer.cpp:8-63)."""
        if self.peer_selection == "random":
            return self.random_peer()
        others = [r for r in range(self.size) if r != self.rank] or [self.rank]
        t = others[self._rr % len(others)]
        self._rr += 1
        return t

    # -- CPU / host-store helpers --------------------------------------------
    def _host_vars(self):
        return [p for p in self.params if p.grad is not None]

    def _host_save(self):
        vs = self._host_vars()
        if self.fuse_requests:
            ops.save_variable(ops.fuse([v.detach() for v in vs]), name=self.fused_model_name)
        else:
            for i, v in enumerate(vs):
                ops.save_variable(v, name="%s:%d" % (self.fused_model_name, i))

    def _host_pull_average(self, target):
        vs = self._host_vars()
        with torch.no_grad():
            if self.fuse_requests:
                tmpl = ops.fuse([v.detach() for v in vs])
                other = ops.request_variable(target, self.fused_model_name, tmpl.shape, tmpl.dtype)
                if other is None:
                    return
                others = ops.split_like(other, [v.shape for v in vs])
            else:
                others = [ops.request_variable(target, "%s:%d" % (self.fused_model_name, i), v.shape, v.dtype)
                          for i, v in enumerate(vs)]
            for v, o in zip(vs, others):
                if o is not None:
                    v.add_(o.to(v.device)).mul_(0.5)

    # -- algorithm ----------------------------------------------------------------
    def _average(self, done):
        """``done``: the pull's completion event, True (the native prefetcher already made the
        current stream wait on it) or None (nothing pulled)."""
        if done is None:
            return
        cur = torch.cuda.current_stream(self.space.device)
        if done is not True:
            cur.wait_event(done)  # normally complete already: no stall
        from ..parallel.flat import note_param_write

        note_param_write()
        hip().axpby(self.space.flat_param, self._other, None, 0.5, 0.5)
        self.pulls += 1
        ev = torch.cuda.Event()
        ev.record(cur)  # the next prefetch may overwrite _other only after this kernel
        self._consumed = ev

    def _before_step(self):
        if self.size == 1 and not self.force_comm:
            return
        if self.step_count == 0:
            if self.store is not None:
                self.store.publish(self.space.flat_param)
                self.store.advertise()
            else:
                self._host_save()
            if self.size > 1:
                runtime.barrier()
            if self.prefetcher is not None:  # first step: a synchronous pull
                self.last_target = self.next_peer()
                self._average(self.store.pull(self.last_target, self._other))
                return
        if self.prefetcher is not None:
            self._average(self.prefetcher.finish())
            return
        target = self.next_peer()
        self.last_target = target
        if self.store is not None:
            self.store.advertise()
            self._average(self.store.pull(target, self._other))
        else:
            self._host_pull_average(target)

    def _after_step(self):
        self.step_count += 1
        if self.size == 1 and not self.force_comm:
            return
        if self.store is not None:
            self.store.publish(self.space.flat_param)
            if self.prefetcher is not None:
                # the next step's pull (and this step's advertisement) overlap its forward/backward
                self.last_target = self.next_peer()
                self.prefetcher.start(self.last_target, self._consumed)
        else:
            self._host_save()

    def synchronize(self):
        """Wait for an in-flight prefetch (e.g. before a checkpoint or a resize)."""
        if self.prefetcher is not None and self.prefetcher.thread is not None:
            self._average(self.prefetcher.finish())


def PairAveragingOptimizer(optimizer, named_parameters=None, fuse_requests: bool = True,
                           fused_model_name: str = "model", fused: bool = True, name=None, use_locking=False,
                           with_keras=False, peer_selection: str = "random", prefetch: bool = True,
                           force_comm: bool = False):
    """Wrap ``optimizer`` with AD-PSGD pair averaging (see module doc).

    * ``prefetch=True`` (GPU): the model averaged in at step k+1 is pulled while step k+1's
      forward/backward are enqueued (host thread + copy stream), like the reference's
      ``AsyncModelAveraging``; ``False`` pulls synchronously at the start of each step.
    * ``force_comm=True``: with one peer, pull the own published snapshot through the same
      store/copy path (exercises and profiles the device store at N=1)."""
    return _PairAveraging(optimizer, named_parameters, fuse_requests=fuse_requests,
                          fused_model_name=fused_model_name, fused=fused, peer_selection=peer_selection,
                          prefetch=prefetch, force_comm=force_comm)
