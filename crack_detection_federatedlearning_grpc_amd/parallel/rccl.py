"""FedAvg over RCCL (xGMI) for on-node GPU clients.

The reference aggregates by gathering 8.2 MB pickles over gRPC into the server, averaging in host NumPy and
broadcasting back (fl_server.py:92-105, 158-161; SURVEY §2.3 "collective call sites"). Here every GPU client holds
its model in ONE flat fp32 device buffer (``models/spec.py`` layout: all 112 Keras arrays, BN moving statistics
included - the reference averages those too) and the round's aggregation is

    w <- sum_k (n_k / sum n) * w_k       (pre-scale on the device, then one SUM all-reduce)

issued as a few layer-ordered buckets with ``torch.distributed`` (backend "nccl" = RCCL on ROCm) so the first
buckets' collectives overlap the pre-scaling of later ones; equal n_k reproduces the reference's plain mean.
An 8-way ring all-reduce of 8.2 MB moves 2*7/8*S = 14.4 MB per GPU - tens of microseconds over the 7 xGMI links,
against seconds of local training per round.

``RcclAggregator`` is the FL-client data plane (rendezvous parameters come from the server's READY reply);
``FedAvgAllReduce`` is the same reduction bound to an engine's device buffer (bench / in-process trainers).
On CPU-only hosts the same code runs over gloo (tests).

The RCCL group is built to OWN its collective (``init_rccl_group``):

* the collectives run on c10d's per-device RCCL stream, created HIGH priority (``ProcessGroupNCCL.Options
  .is_high_priority_stream``): under the next round's forward they get their own hardware queue ahead of the
  compute queue instead of sharing its priority;
* the FedAvg pre-scale n_k / sum n is fused into the reduction - ``ncclRedOpCreatePreMulSum`` with a DEVICE scalar
  (``dist._make_nccl_premul_sum``): RCCL multiplies each rank's input by that rank's weight inside the all-reduce
  kernel, so there is no per-bucket scaling kernel on the compute stream (gloo keeps the separate ``mul_``);
* the channel count is capped (``ncclConfig_t.maxCTAs`` via ``Options.config.max_ctas``, and ``NCCL_MAX_NCHANNELS``
  in the rank environment before the communicator exists): each RCCL channel is one resident workgroup, so the
  cap bounds the CUs an in-flight all-reduce takes from the next round's kernels. Default 16
  (``RCCL_MAX_CHANNELS_DEFAULT``; ``CFL_RCCL_MAX_CHANNELS`` / config ``rccl_max_channels``, 0 = RCCL's own choice):
  an 8-GPU MI355X node is fully connected (7 xGMI links per GPU), so 16 rings still drive every link in both
  directions while 240 of the 256 CUs keep computing; the 8.2 MB model moves in ~2 MB buckets, far below the
  message size at which more channels pay.
"""
from __future__ import annotations

import os
import time
from datetime import timedelta
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist


RCCL_MAX_CHANNELS_DEFAULT = 16


def rccl_channel_cap(explicit: Optional[int] = None) -> int:
    """The RCCL channel cap of this process: ``explicit`` (config ``rccl_max_channels``) if given, else
    ``CFL_RCCL_MAX_CHANNELS``, else ``RCCL_MAX_CHANNELS_DEFAULT``; 0 = no cap."""
    if explicit is not None and int(explicit) >= 0:
        return int(explicit)
    v = os.environ.get("CFL_RCCL_MAX_CHANNELS", "")
    return int(v) if v.strip() else RCCL_MAX_CHANNELS_DEFAULT


def rccl_env(env: Dict[str, str], cap: Optional[int] = None) -> Dict[str, str]:
    """A rank's environment for RCCL (launchers set it before the child starts): dmabuf IPC (the host driver has no
    legacy IPC) and the channel cap as ``NCCL_MAX_NCHANNELS`` unless the caller already chose one."""
    env = dict(env)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    c = rccl_channel_cap(cap)
    if c > 0:
        env.setdefault("NCCL_MAX_NCHANNELS", str(c))
    return env


def rccl_pg_options(cap: Optional[int] = None):
    """``ProcessGroupNCCL.Options`` of the FedAvg group: high-priority collective stream + channel cap."""
    opts = dist.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    c = rccl_channel_cap(cap)
    if c > 0:
        opts.config.max_ctas = c
    return opts


def init_rccl_group(device: torch.device, *, init_method: Optional[str] = None, rank: Optional[int] = None,
                    world_size: Optional[int] = None, timeout: Optional[timedelta] = None,
                    cap: Optional[int] = None) -> None:
    """``dist.init_process_group("nccl")`` for one GPU client: eager communicator bound to ``device``, collectives
    on a high-priority stream, channel cap in the options and (for the communicator's own env read) in
    ``NCCL_MAX_NCHANNELS`` before RCCL initialises. ``init_method`` None = the env:// rendezvous (torchrun /
    ``parallel/spawn.py``)."""
    c = rccl_channel_cap(cap)
    if c > 0:
        os.environ.setdefault("NCCL_MAX_NCHANNELS", str(c))
    kw = {}
    if init_method is not None:
        kw.update(init_method=init_method, rank=int(rank), world_size=int(world_size))
    if timeout is not None:
        kw["timeout"] = timeout
    dist.init_process_group("nccl", pg_options=rccl_pg_options(c), device_id=device, **kw)


def group_stream_info(group=None) -> Dict[str, object]:
    """What the RCCL backend of ``group`` was built with (tests / bench JSON): high-priority stream, channel cap."""
    pg = group if group is not None else dist.distributed_c10d._get_default_group()
    be = pg._get_backend(torch.device("cuda"))
    o = be.options
    return {"high_priority_stream": bool(o.is_high_priority_stream), "max_ctas": int(o.config.max_ctas),
            "nccl_max_nchannels": os.environ.get("NCCL_MAX_NCHANNELS")}


def rccl_placement_error(n_ranks: int, device: str = "auto", backend: str = "nccl",
                         rank: Optional[int] = None) -> Optional[str]:
    """Why ``n_ranks`` RCCL clients (or client ``rank`` of them) cannot run here, or None. RCCL refuses two ranks
    of one communicator on one GPU ("duplicate GPU"), but only at its first collective - after a whole round of
    training - so the launchers check up front instead of mapping ``rank % device_count`` onto a shared card.
    gloo (``backend``) and CPU clients are not constrained. ``torch.cuda.device_count()`` does not initialise HIP
    on this image, so a launcher may call this before it starts its GPU children."""
    if backend != "nccl" or device == "cpu":
        return None
    ndev = torch.cuda.device_count()
    if ndev == 0 and device != "cuda":
        return None                                   # auto on a CPU host: the clients fall back to gloo
    need = n_ranks if rank is None else rank + 1
    if need > ndev:
        who = f"{n_ranks} RCCL clients need" if rank is None else f"RCCL client rank {rank} needs"
        return (f"{who} {need} visible GPUs (one per client), found {ndev}: RCCL refuses two ranks on one GPU - "
                f"use --dist-backend gloo to rehearse N clients on fewer GPUs")
    return None


def premul_enabled(group=None) -> bool:
    """Fuse the FedAvg pre-scale into the all-reduce (PreMulSum with a device scalar): RCCL groups only;
    ``CFL_RCCL_PREMUL=0`` restores the separate scaling kernel."""
    return dist.get_backend(group) == "nccl" and os.environ.get("CFL_RCCL_PREMUL", "1") != "0"


def _buckets(n: int, bucket_elems: int, first: int = 0) -> List[slice]:
    """Layer-ordered buckets of ``bucket_elems``; ``first`` > 0: the first bucket ends exactly there (e.g. at the
    encoder's last parameter, so the next round's encoder forward waits for that bucket alone)."""
    out, s = [], 0
    if 0 < first < n:
        out.append(slice(0, first))
        s = first
    out += [slice(a, min(n, a + bucket_elems)) for a in range(s, n, bucket_elems)]
    return out


class FedAvgAllReduce:
    def __init__(self, flat: torch.Tensor, table=None, world: Optional[int] = None, bucket_mb: float = 2.0,
                 group=None, first_bucket: int = 0):
        self.flat = flat
        self.group = group
        self.world = world or dist.get_world_size(group)
        self.buckets = _buckets(flat.numel(), max(1024, int(bucket_mb * (1 << 20)) // 4), first_bucket)
        self._side = None
        self.premul = premul_enabled(group)   # pre-scale fused into the all-reduce (RCCL PreMulSum)
        self.timing = False               # record hipEvents around each call's collectives (bench.py)
        self.timings: List[tuple] = []    # per call: (issue, last all-reduce done, last bucket repacked) events

    def _weight(self, n_local: float, weighted: bool):
        """This client's FedAvg weight n_k / sum n. The sample-count all-reduce runs on EVERY call (each rank
        must issue the same sequence of collectives; a per-rank cache could desynchronise them) and stays on the
        device (no host sync): the weight is a 1-element tensor the bucket scaling broadcasts."""
        if not weighted:
            return 1.0 / float(self.world)
        t = torch.tensor([float(n_local)], dtype=torch.float32, device=self.flat.device)
        tot = t.clone()
        dist.all_reduce(tot, group=self.group)
        return t / tot.clamp_min(1e-12)

    def total_samples(self, n_local: float) -> float:
        t = torch.tensor([float(n_local)], dtype=torch.float64, device=self.flat.device)
        dist.all_reduce(t, group=self.group)
        return float(t.item())

    def _reduce_op(self, w):
        """(op, scale-first) of one FedAvg call: RCCL -> PreMulSum with this rank's weight (a device tensor or a
        float), fused into the all-reduce; otherwise SUM after a separate in-place scale."""
        if self.premul:
            return dist._make_nccl_premul_sum(w), False
        return dist.ReduceOp.SUM, True

    def average(self, n_local: float, weighted: bool = True) -> None:
        w = self._weight(n_local, weighted)
        op, scale = self._reduce_op(w)
        works = []
        for sl in self.buckets:
            b = self.flat[sl]
            if scale:
                b.mul_(w)
            works.append(dist.all_reduce(b, op=op, group=self.group, async_op=True))
        for wk in works:
            wk.wait()

    def average_async(self, n_local: float, weighted: bool = True,
                      on_bucket: Optional[Callable[[slice], None]] = None) -> List[Tuple[slice, object]]:
        """Overlapped FedAvg: the buckets' all-reduces are issued in forward-layer order and each bucket's
        completion is chained onto a side HIP stream, where ``on_bucket`` (e.g. the bf16 repack of the layers in
        that bucket) runs and a per-bucket event is recorded. Returns [(bucket slice, event)] - the consumer waits
        per layer (``UNetEngine.defer_until``) instead of on the whole model, so the next round's setup and early
        layers overlap the late buckets. On CPU / gloo the reduction is synchronous and no events are returned."""
        if self.flat.device.type != "cuda":
            self.average(n_local, weighted)
            if on_bucket is not None:
                for sl in self.buckets:
                    on_bucket(sl)
            return []
        t_issue = None
        if self.timing:
            t_issue = torch.cuda.Event(enable_timing=True)
            t_issue.record(torch.cuda.current_stream(self.flat.device))
        w = self._weight(n_local, weighted)
        if self._side is None:
            # high priority: HIP gives it its own hardware queue (a default-priority stream may be multiplexed onto
            # the compute stream's queue - GPU_MAX_HW_QUEUES=4 - and then cannot overlap it; measured with
            # tools/overlap_summary.py), and the per-bucket repack that gates the next round's layers goes first
            self._side = torch.cuda.Stream(device=self.flat.device, priority=-1)
        out = []
        t_ar = None
        op, scale = self._reduce_op(w)
        for i, sl in enumerate(self.buckets):
            b = self.flat[sl]
            if scale:
                b.mul_(w)
            # RCCL: enqueued on the group's high-priority stream behind the compute stream's work so far; with
            # PreMulSum the kernel scales each rank's input by its weight on the fly (nothing on the compute stream)
            work = dist.all_reduce(b, op=op, group=self.group, async_op=True)
            with torch.cuda.stream(self._side):
                work.wait()                                   # side stream <- this bucket's collective
                if self.timing and i == len(self.buckets) - 1:
                    t_ar = torch.cuda.Event(enable_timing=True)
                    t_ar.record(self._side)
                if on_bucket is not None:
                    on_bucket(sl)
                ev = torch.cuda.Event(enable_timing=self.timing)
                ev.record(self._side)
            out.append((sl, ev))
        if self.timing:
            self.timings.append((t_issue, t_ar, out[-1][1]))
        return out

    def timing_summary(self) -> Dict[str, float]:
        """Mean over the recorded calls (events must be complete, e.g. after a synchronize): ``allreduce_ms`` =
        issue of the first bucket's pre-scale on the compute stream -> last bucket's all-reduce done on the side
        stream (weight all-reduce + bucketed SUM all-reduces); ``allreduce_repack_ms`` = ... -> last bucket's bf16
        repack done."""
        if not self.timings:
            return {}
        ar = [a.elapsed_time(b) for a, b, _ in self.timings]
        rp = [a.elapsed_time(c) for a, _, c in self.timings]
        return {"allreduce_ms": float(np.mean(ar)), "allreduce_repack_ms": float(np.mean(rp)),
                "allreduce_calls": len(ar), "allreduce_buckets": len(self.buckets),
                "allreduce_bytes": int(self.flat.numel() * self.flat.element_size())}


class RcclAggregator:
    """FL-client data plane: weighted all-reduce between the registered clients.

    ``backend``: "nccl" (RCCL over xGMI, the product path) or "gloo" (CPU clients, and the one-GPU rehearsal of
    N clients sharing a card, which RCCL refuses). Collectives stay asynchronous to the host - no
    ``TORCH_NCCL_BLOCKING_WAIT``, which would serialise the bucketed all-reduce bucket by bucket on the host: the
    side stream waits on each bucket's collective, and a dead peer is detected by the ``PendingFedAvg`` watchdog's
    deadline (``timeout_s``), which fires before the process group's own timeout so this process aborts the
    communicator first and the client can fall back to gRPC."""

    def __init__(self, rank: int, world: int, addr: str, port: int, device: Optional[torch.device] = None,
                 timeout_s: float = 300.0, backend: Optional[str] = None, max_channels: Optional[int] = None):
        self.rank, self.world = rank, world
        cuda = device is not None and device.type == "cuda"
        backend = backend or ("nccl" if cuda else "gloo")
        if backend == "nccl" and not cuda:
            backend = "gloo"                                   # CPU clients: RCCL needs a GPU
        self.timeout_s = float(timeout_s)
        if not dist.is_initialized():
            # gloo raises on its own timeout (the host waits in work.wait()); under RCCL the group timeout only
            # arms the watchdog, so it is set past the host-side deadline of wait_complete
            pg_timeout = self.timeout_s if backend == "gloo" else self.timeout_s + 60.0
            if backend == "nccl":
                init_rccl_group(device, init_method=f"tcp://{addr}:{port}", rank=rank, world_size=world,
                                timeout=timedelta(seconds=pg_timeout), cap=max_channels)
            else:
                dist.init_process_group(backend, init_method=f"tcp://{addr}:{port}", rank=rank, world_size=world,
                                        timeout=timedelta(seconds=pg_timeout))
        self.device = device if cuda else torch.device("cpu")
        self._cached = None
        self._backup: Optional[torch.Tensor] = None
        self._avg: Optional[torch.Tensor] = None
        print(f"[rccl] rank {rank}/{world} world_size {world} backend {dist.get_backend()} device "
              f"{self.device if not cuda else torch.cuda.get_device_name(device)} ({self.device})", flush=True)

    @classmethod
    def from_ready_info(cls, info: Dict, cfg=None) -> "RcclAggregator":
        dev = None
        if torch.cuda.is_available() and (cfg is None or cfg.device != "cpu"):
            dev = torch.device("cuda", torch.cuda.current_device())
        return cls(int(info.get("rank", 0)), int(info["world_size"]), str(info.get("dist_addr") or "127.0.0.1"),
                   int(info["dist_port"]), dev, timeout_s=float(getattr(cfg, "rccl_timeout_s", 300.0)),
                   backend=getattr(cfg, "dist_backend", None) or None,
                   max_channels=getattr(cfg, "rccl_max_channels", None))

    def _reducer(self, flat: torch.Tensor, first_bucket: int = 0) -> FedAvgAllReduce:
        key = (flat.data_ptr(), flat.numel(), first_bucket)
        if self._cached is None or self._cached[0] != key:
            self._cached = (key, FedAvgAllReduce(flat, world=self.world, first_bucket=first_bucket))
        return self._cached[1]

    def average(self, arrays: Sequence[np.ndarray], n_local: float) -> List[np.ndarray]:
        """Host-array form (trainers without a device buffer, e.g. the CPU oracle over gloo)."""
        shapes = [np.shape(a) for a in arrays]
        flat = torch.as_tensor(np.concatenate([np.asarray(a, np.float32).reshape(-1) for a in arrays])).to(self.device)
        FedAvgAllReduce(flat, world=self.world).average(float(max(n_local, 1)))
        out, off = [], 0
        host = flat.cpu().numpy()
        for s in shapes:
            n = int(np.prod(s)) if s else 1
            out.append(host[off:off + n].reshape(s).copy())
            off += n
        return out

    def average_device(self, flat: torch.Tensor, n_local: float,
                       on_bucket: Optional[Callable[[slice], None]] = None,
                       first_bucket: int = 0) -> List[Tuple[slice, object]]:
        """Device-resident FedAvg of a trainer's flat fp32 parameter buffer, in place: bucketed weighted
        all-reduce on a side stream (no host staging); returns the per-bucket events for ``defer_until``."""
        return self._reducer(flat, first_bucket).average_async(float(max(n_local, 1)), on_bucket=on_bucket)

    def fedavg_device_async(self, flat: torch.Tensor, n_local: float,
                            on_bucket: Optional[Callable[[slice], None]] = None,
                            first_bucket: int = 0) -> "PendingFedAvg":
        """The product path's FedAvg, off the host's critical path: the local model is copied (``backup``, 8 MB
        device copy on the compute stream), the bucketed weighted all-reduce is issued in place on the side stream
        (``average_device``), and after the last bucket the side stream also copies the average into ``avg`` (the
        round's global model, kept for rank 0's upload and for a restore when the server ends the run while the next
        round trains). Nothing here waits: the returned ``PendingFedAvg`` carries the bucket events for the engine's
        per-layer waits (``defer_until``) and a watchdog thread that polls the last event against the deadline
        (``timeout_s``) - on expiry it aborts the communicator and drains the side stream, and the caller's next
        ``wait()`` reports the failure (the rollback and the gRPC fallback run there). A failure while ISSUING
        (e.g. a dead peer under gloo, whose collectives run on the host) is rolled back here already."""
        if self._backup is None or self._backup.numel() != flat.numel() or self._backup.device != flat.device:
            self._backup = torch.empty_like(flat)
            self._avg = torch.empty_like(flat)
        self._backup.copy_(flat)
        red = self._reducer(flat, first_bucket)
        red.timing = flat.device.type == "cuda"
        n_b, seen = len(red.buckets), [0]
        avg = self._avg

        def hook(sl: slice) -> None:
            if on_bucket is not None:
                on_bucket(sl)
            seen[0] += 1
            if seen[0] == n_b:              # on the side stream, behind every bucket's collective and repack
                avg.copy_(flat)
        try:
            evs = red.average_async(float(max(n_local, 1)), on_bucket=hook)
        except BaseException as e:
            self.abort()
            self._drain_side(flat)
            flat.copy_(self._backup)
            return PendingFedAvg(self, flat, [], None, avg, self._backup, error=e)
        timing = red.timings[-1] if red.timing and red.timings else None
        red.timings = []
        return PendingFedAvg(self, flat, evs, timing, avg, self._backup)

    def fedavg_device(self, flat: torch.Tensor, n_local: float,
                      on_bucket: Optional[Callable[[slice], None]] = None,
                      first_bucket: int = 0) -> List[Tuple[slice, object]]:
        """Blocking form of ``fedavg_device_async`` (the synchronous report of the last round, host-array callers,
        tests): issue, wait for the watchdog's verdict, roll back and re-raise on failure. The buckets are pre-scaled
        (w_k * n_k / sum n) and reduced in place, so a failure part-way would leave ``flat`` a mix of scaled, reduced
        and untouched buckets: the rollback restores the pre-FedAvg copy after the side stream has drained (no queued
        bucket work lands after the restore); the caller then uploads its unchanged local weights over gRPC."""
        pending = self.fedavg_device_async(flat, n_local, on_bucket=on_bucket, first_bucket=first_bucket)
        if not pending.wait():
            raise pending.error
        return pending.events

    def _drain_side(self, flat: torch.Tensor, drain_s: float = 30.0, order: bool = True) -> None:
        """After an abort, work still queued on the aggregation side stream (the in-place all-reduce output of an
        issued bucket, the per-bucket bf16 repacks) could land AFTER the rollback and overwrite the restored
        weights with a partly reduced bucket. Wait (host deadline) for the side stream to drain and (``order``)
        order the current stream behind it; if it never drains the weights cannot be trusted: exit non-zero."""
        side = self.side_stream()
        if side is None or flat.device.type != "cuda":
            return
        ev = torch.cuda.Event()
        ev.record(side)
        end = time.monotonic() + drain_s
        while not ev.query():
            if time.monotonic() > end:
                print(f"[rccl] aggregation side stream did not drain {drain_s:.0f} s after the abort; the local "
                      f"weights may be partly overwritten - exiting", flush=True)
                os._exit(70)
            time.sleep(1e-3)
        if order:
            torch.cuda.current_stream(flat.device).wait_stream(side)

    def side_stream(self):
        red = self._cached[1] if self._cached is not None else None
        return red._side if red is not None else None

    def abort(self) -> None:
        """A peer died or a collective timed out: tear the communicator down without a collective shutdown
        (``ncclCommAbort`` under RCCL), so the surviving clients can carry on over gRPC."""
        if not dist.is_initialized():
            return
        try:
            from torch.distributed.distributed_c10d import _abort_process_group
            _abort_process_group()
        except Exception:
            pass
        try:
            dist.destroy_process_group()
        except Exception:
            pass

    def close(self) -> None:
        if dist.is_initialized():
            dist.destroy_process_group()


class PendingFedAvg:
    """An issued device FedAvg of the FL product path (``RcclAggregator.fedavg_device_async``).

    The reference blocks completely around its aggregation (gather -> NumPy mean -> 20 s poll,
    /root/reference/fl_server.py:92-135, fl_client.py:136-155). Here the collective runs on the side stream while
    the training thread goes on: ``events`` feed the engine's per-layer waits, and a daemon WATCHDOG thread polls
    the last bucket's event (1 ms period, no spin on the training thread) against the aggregator's deadline. On
    expiry it records the failure, aborts the communicator and drains the side stream; ``wait()`` - called where
    the client needs the verdict (the round report, or the join before the next FedAvg) - then orders the caller's
    stream behind the drained side stream and restores the pre-FedAvg local model (``rollback``) unless told not
    to. ``stats()`` gives the hipEvent split of the collective: ``allreduce_ms`` (issue -> last bucket reduced) and
    ``allreduce_exposed_ms`` (how long the next round's first step actually stalled for it, when an engine's
    ``stall_log`` recorded that step's waits)."""

    poll_s = 1e-3

    def __init__(self, agg: "RcclAggregator", flat: torch.Tensor, events, timing, avg: torch.Tensor,
                 backup: torch.Tensor, error: Optional[BaseException] = None):
        import threading
        self.agg, self.flat, self.events, self.timing = agg, flat, list(events), timing
        self.avg, self.backup = avg, backup
        self.error = error
        self.engine = None                  # set by the trainer: its stall_log holds the next step's waits
        self._done = threading.Event()
        self._rolled = error is not None    # an issue-time failure was rolled back by the aggregator already
        if error is not None or not self.events:
            self._done.set()
            self._t = None
        else:
            self._t = threading.Thread(target=self._watch, name="fedavg-watchdog", daemon=True)
            self._t.start()

    def _poll_done(self, ev) -> bool:
        return bool(ev.query())

    def _watch(self) -> None:
        ev = self.events[-1][1]
        end = time.monotonic() + self.agg.timeout_s
        try:
            while not self._poll_done(ev):
                if time.monotonic() > end:
                    raise TimeoutError(f"FedAvg all-reduce not complete after {self.agg.timeout_s:.0f} s "
                                       f"(peer lost?)")
                time.sleep(self.poll_s)
        except BaseException as e:           # a peer died / the collective can never finish
            self.error = e
            self.agg.abort()
            self.agg._drain_side(self.flat, order=False)
        finally:
            self._done.set()

    @property
    def done(self) -> bool:
        return self._done.is_set()

    def wait(self, rollback: bool = True) -> bool:
        """True iff the collective completed. On failure (after the watchdog has aborted the communicator and the
        side stream has drained) the caller's stream is ordered behind the side stream and, with ``rollback``, the
        flat buffer is restored to the pre-FedAvg local model."""
        self._done.wait()
        if self.error is None:
            return True
        side = self.agg.side_stream()
        if side is not None and self.flat.device.type == "cuda":
            torch.cuda.current_stream(self.flat.device).wait_stream(side)
        if rollback and not self._rolled:
            self.flat.copy_(self.backup)
            self._rolled = True
        return False

    def _host(self, t: torch.Tensor) -> np.ndarray:
        """Host copy of a buffer written on the compute or the side stream, taken on a private stream that waits for
        the collective's last event (not on the compute stream, which may already run the next round)."""
        if t.device.type != "cuda":
            return t.detach().numpy().copy()
        s = torch.cuda.Stream(device=t.device)
        if self.events:
            s.wait_event(self.events[-1][1])
        with torch.cuda.stream(s):
            out = t.cpu().numpy().copy()
        return out

    def host_average(self) -> np.ndarray:
        """The round's global model (valid after a successful ``wait``)."""
        return self._host(self.avg)

    def host_backup(self) -> np.ndarray:
        """The pre-FedAvg local model (what a failed round uploads over gRPC)."""
        return self._host(self.backup)

    def stats(self) -> Dict[str, float]:
        """hipEvent timings, read once the events are complete (e.g. after the next round)."""
        out: Dict[str, float] = {}
        if self.timing is None or self.error is not None:
            return out
        t_issue, t_ar, _t_last = self.timing
        out["allreduce_ms"] = float(t_issue.elapsed_time(t_ar))
        st = getattr(self.engine, "stall_log", None) if self.engine is not None else None
        if st and len(st) >= 2:
            # the compute stream's two stall brackets (before / after each wait on the buckets): only the time the
            # next round's first step actually waited, not the work queued between the issue and the first wait
            (b0, a0), (b1, a1) = st[0], st[1]
            out["allreduce_exposed_ms"] = float(b0.elapsed_time(a0) + b1.elapsed_time(a1))
        return out
