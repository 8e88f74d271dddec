"""Process-group helpers: one process per GPU, ``torch.distributed`` for the
control plane, RCCL (backend "nccl" on ROCm) or native RCCL communicators for
the data plane.

This is the MI355X replacement of the reference's coordination layer
(SURVEY §2.7/§5.8): the driver rendezvous of lightgbm/.../NetworkManager.scala
becomes the torchrun/TCPStore rendezvous (rank, world size, master address),
and LightGBM's socket linkers / VW's spanning tree / Horovod become RCCL
collectives over xGMI.
"""
from __future__ import annotations

import os
from typing import Any, List, Optional

import numpy as np


def _dist():
    try:
        import torch.distributed as dist

        return dist if dist.is_available() else None
    except Exception:  # pragma: no cover
        return None


def is_initialized() -> bool:
    d = _dist()
    return bool(d and d.is_initialized())


def rank() -> int:
    d = _dist()
    return d.get_rank() if d and d.is_initialized() else 0


def world_size() -> int:
    d = _dist()
    return d.get_world_size() if d and d.is_initialized() else 1


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def local_device() -> int:
    """this rank's GPU index: LOCAL_RANK over the visible devices (a launcher that gives each rank a single
    visible device maps every rank to its device 0)"""
    import torch

    n = torch.cuda.device_count()
    return local_rank() % n if n > 0 else -1


def backend() -> Optional[str]:
    d = _dist()
    return d.get_backend() if d and d.is_initialized() else None


def init_from_env(backend_name: Optional[str] = None, timeout_s: float = 1200.0) -> bool:
    """Initialise the default process group from torchrun-style env vars."""
    d = _dist()
    if d is None or d.is_initialized():
        return bool(d and d.is_initialized())
    if "RANK" not in os.environ or "WORLD_SIZE" not in os.environ:
        return False
    import datetime

    import torch

    if backend_name is None:
        backend_name = "nccl" if torch.cuda.is_available() else "gloo"
    if backend_name == "nccl":
        torch.cuda.set_device(local_device())
    d.init_process_group(backend=backend_name, timeout=datetime.timedelta(seconds=timeout_s))
    return True


def barrier() -> None:
    if is_initialized():
        d = _dist()
        if backend() == "nccl":
            import torch

            d.barrier(device_ids=[torch.cuda.current_device()])
        else:
            d.barrier()


def broadcast_object(obj: Any, src: int = 0) -> Any:
    if not is_initialized() or world_size() == 1:
        return obj
    d = _dist()
    lst = [obj]
    d.broadcast_object_list(lst, src=src)
    return lst[0]


def all_gather_object(obj: Any) -> List[Any]:
    if not is_initialized() or world_size() == 1:
        return [obj]
    d = _dist()
    out = [None] * world_size()
    d.all_gather_object(out, obj)
    return out


class _ShmReducer:
    """Host allreduce for ranks that share one machine (the local executors, the shared-device rehearsal): the
    ranks meet in one POSIX shared-memory segment instead of gloo's loopback TCP (~0.8 ms per call for a 24 KB
    histogram on this host; ~150 calls per small 5-iteration fit). Rank r writes its array into its slot of the
    call's half (calls alternate halves), then publishes the call number in its flag; every rank waits for all
    flags and sums the slots in rank order - the same bits on every rank, exact for int64. A rank can reuse a
    half only after every rank entered the next call, i.e. finished reading this one. Flags are written after
    the data (x86 stores are not reordered with other stores)."""

    _SLOT = 1 << 20  # bytes per rank per half (larger arrays go in pieces)

    def __init__(self, world: int, rk: int, name: Optional[str]):
        from .executor import attach_shm

        self.world, self.rank = world, rk
        size = 64 * world + 2 * world * self._SLOT
        if name is None:
            from multiprocessing import shared_memory

            self.shm = shared_memory.SharedMemory(create=True, size=size)
            self.owner = True
        else:
            self.shm = attach_shm(name)
            self.owner = False
        self.flags = np.ndarray((world, 8), dtype=np.int64, buffer=self.shm.buf)  # one 64-B line per rank
        self.calls = 0
        if self.owner:
            self.flags[:] = 0

    def publish_pid(self) -> None:
        self.flags[self.rank, 1] = os.getpid()

    def _dead_peer(self, k: int) -> Optional[int]:
        """a rank that has not arrived at call k and whose process is gone (or a zombie)"""
        for r in range(self.world):
            if r == self.rank or int(self.flags[r, 0]) >= k:
                continue
            pid = int(self.flags[r, 1])
            if pid > 0 and not _pid_alive(pid):
                return r
        return None

    def allreduce(self, a: np.ndarray) -> None:
        flat = a.reshape(-1)
        per = self._SLOT // flat.itemsize
        for s in range(0, max(1, flat.size), per):
            self._one(flat[s:s + per])

    def _one(self, x: np.ndarray) -> None:
        import time

        self.calls += 1
        k = self.calls
        half = k & 1
        base = 64 * self.world + half * self.world * self._SLOT
        n = x.size

        def slot(r):
            return np.ndarray(n, dtype=x.dtype, buffer=self.shm.buf, offset=base + r * self._SLOT)

        slot(self.rank)[...] = x
        self.flags[self.rank, 0] = k
        spins, t0, tcheck = 0, None, 0.0
        while int(self.flags[:, 0].min()) < k:
            spins += 1
            if spins > 2000:
                now = time.monotonic()
                if t0 is None:
                    t0 = now
                elif now - t0 > _SHM_TIMEOUT_S:
                    raise TimeoutError(f"shared-memory allreduce: a peer did not arrive within {_SHM_TIMEOUT_S}s")
                if now - tcheck > 0.01:  # a dead peer fails the collective (gloo would see its socket close)
                    tcheck = now
                    dead = self._dead_peer(k)
                    if dead is not None:
                        raise RuntimeError(f"shared-memory allreduce: rank {dead} died")
                time.sleep(20e-6)
        acc = slot(0).copy()
        for r in range(1, self.world):
            acc += slot(r)
        x[...] = acc

    def close(self) -> None:
        try:
            self.shm.close()
            if self.owner:
                self.shm.unlink()
        except Exception:  # noqa: BLE001 - already gone
            pass


def _pid_alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split(")")[-1].split()[0] != "Z"
    except OSError:
        return True


_SHM_TIMEOUT_S = float(os.environ.get("SML_SHM_ALLREDUCE_TIMEOUT_S", "1200"))
_shm_reducer: Optional[_ShmReducer] = None
_shm_key = None


def _same_host_reducer() -> Optional[_ShmReducer]:
    """The shared-memory reducer of the default group when every rank runs on this host (gloo groups only;
    SML_SHM_ALLREDUCE=0 keeps gloo). Built collectively on first use, rebuilt when the group changes."""
    global _shm_reducer, _shm_key
    if os.environ.get("SML_SHM_ALLREDUCE", "1") == "0":
        return None
    d = _dist()
    key = (id(d.group.WORLD), world_size(), rank())
    if _shm_key == key:
        return _shm_reducer
    import socket

    if _shm_reducer is not None:
        _shm_reducer.close()
    hosts = all_gather_object(socket.gethostname())
    red = None
    if len(set(hosts)) == 1:
        if rank() == 0:
            red = _ShmReducer(world_size(), 0, None)
            broadcast_object(red.shm.name)
        else:
            red = _ShmReducer(world_size(), rank(), broadcast_object(None))
        red.publish_pid()
        barrier()  # every rank attached (and its pid published) before any reduces or rank 0 may unlink at exit
        # multiprocessing's exit hook runs in spawned children too (they end in os._exit: atexit does not)
        from multiprocessing import util

        util.Finalize(red, red.close, exitpriority=10)
    _shm_reducer, _shm_key = red, key
    return red


def close_shm_reducer() -> None:
    """Release the shared-memory reducer (a task process calls this before its group goes away)."""
    global _shm_reducer, _shm_key
    if _shm_reducer is not None:
        _shm_reducer.close()
    _shm_reducer, _shm_key = None, None


def allreduce_numpy(a: np.ndarray) -> None:
    """In-place sum of a float64 or int64 host array over the default group (int64: exact)."""
    if not is_initialized() or world_size() == 1:
        return
    import torch

    d = _dist()
    if backend() != "nccl" and a.flags.c_contiguous and a.dtype in (np.float64, np.int64):
        red = _same_host_reducer()
        if red is not None:
            red.allreduce(a)
            return
    if backend() == "nccl":
        t = torch.from_numpy(np.ascontiguousarray(a)).to(f"cuda:{torch.cuda.current_device()}")
        d.all_reduce(t)
        a[...] = t.cpu().numpy()
    else:
        t = torch.from_numpy(a)  # shares memory with `a`
        d.all_reduce(t)


_comm_cache: dict = {}
p2p_status: dict = {}


def _single_node() -> bool:
    """Every rank on one host. Collective on every rank (the hostname gather runs even when
    LOCAL_WORLD_SIZE is set, so ranks with different environments cannot split into different paths)."""
    import socket

    hosts = all_gather_object(socket.gethostname())
    lw = os.environ.get("LOCAL_WORLD_SIZE")
    return len(set(hosts)) == 1 and (lw is None or int(lw) == world_size())


def maybe_p2p(comm, device: int):
    """Wrap a device communicator in the intra-node one-shot P2P allreduce
    (see :func:`gbdt_comm`). The decision is collective: every rank calls
    this and all end up on the same path."""
    from ..ops import native

    single = _single_node()  # collective: every rank runs it, whatever its own P2P setting
    want = os.environ.get("SML_GBDT_P2P", "1") != "0" and world_size() <= 8 and single
    # agree before touching IPC so no rank waits in the self-test alone
    flags = all_gather_object(bool(want))
    if not all(flags):
        p2p_status.update(active=False, reason="disabled or multi-node")
        return comm
    cap = int(os.environ.get("SML_GBDT_P2P_CAP", str(1 << 20)))
    c, ok, why = native.gbdt().p2p_comm(comm, device, cap, float(os.environ.get("SML_GBDT_P2P_TIMEOUT_MS", "60000")))
    p2p_status.update(active=bool(ok), reason=why)
    return c


def _abort_quietly(c) -> None:
    abort = getattr(c, "abort", None)
    if abort is not None:
        try:
            abort()
        except Exception:  # noqa: BLE001 - best effort on a communicator that is being thrown away
            pass


def init_with_retries(make, what: str, retries: int = 3, delay_s: float = 1.0, prepare=None):
    """Collective network initialisation with the reference's retry policy (NetworkManager.scala:195-218,
    3 retries, 1 s doubled).

    Two agreement points per attempt, both over the control plane, so no rank can be left blocked inside a
    collective init its peers never entered:

    1. ``prepare()`` (non-collective: device selection, unique-id creation) runs on every rank and the
       outcomes are all-gathered; the collective ``make(payload)`` is only entered when every rank is ready.
       ``payload`` is rank 0's ``prepare()`` result (e.g. the ncclUniqueId), broadcast with the outcomes.
    2. ``make`` itself must be bounded (the native RCCL init is non-blocking with a deadline and aborts
       itself on timeout); its outcomes are all-gathered, and if any rank failed every rank aborts the
       communicator it built and all retry together with a fresh ``prepare()``.
    """
    import time

    for attempt in range(retries + 1):
        c, err, payload = None, None, None
        if prepare is not None:
            try:
                payload = prepare()
            except Exception as e:  # noqa: BLE001 - shared with the other ranks below
                err = f"rank {rank()} (prepare): {type(e).__name__}: {e}"
            outcomes = all_gather_object((err, payload if rank() == 0 else None))
            errs = [e for e, _ in outcomes if e]
            payload = outcomes[0][1]
        else:
            errs = []
        if not errs:
            try:
                c = make(payload) if prepare is not None else make()
            except Exception as e:  # noqa: BLE001
                err = f"rank {rank()}: {type(e).__name__}: {e}"
            errs = [e for e in all_gather_object(err) if e]
            if not errs:
                return c
        if c is not None:
            _abort_quietly(c)  # a peer failed: this rank's communicator is half of a broken group
        del c
        if attempt == retries:
            raise RuntimeError(f"{what} initialisation failed after {retries} retries: " + "; ".join(errs))
        time.sleep(delay_s)
        delay_s *= 2
    raise AssertionError("unreachable")


def evict_comm(reason: str = "") -> None:
    """Drop cached communicators (called when a fit re-raises a CommError: an aborted communicator must not
    be handed to the next fit of this process)."""
    for c in list(_comm_cache.values()):
        _abort_quietly(c)
    _comm_cache.clear()
    p2p_status.clear()


def gbdt_comm(use_gpu: bool, shared_device: bool = False):
    """Communicator for the native GBDT engine, or None when world == 1.

    GPU runs get a native RCCL communicator whose ncclUniqueId is broadcast
    over the control plane, so histogram allreduces are enqueued on the
    engine's own HIP stream with no Python round trip; CPU runs get a host
    communicator that reduces through the default (gloo) group.

    When every rank is on one node the RCCL communicator is wrapped in the
    one-shot P2P allreduce (``csrc/gbdt/comm_p2p.hip``, K21): per-split
    histograms (~114 KB) go over xGMI in a single kernel instead of a
    latency-bound ring; larger messages still use RCCL.  ``SML_GBDT_P2P=0``
    disables it; if IPC set-up or its start-up self-test fails on any rank,
    all ranks stay on RCCL together.

    ``shared_device``: ranks share GPUs (more ranks than devices, e.g. a
    rehearsal on a one-GPU box). RCCL cannot place two ranks on one device, so
    the P2P allreduce wraps the host (gloo) communicator instead.
    """
    if world_size() <= 1:
        return None
    from ..ops import native

    shared_device = shared_device or os.environ.get("SML_GBDT_SHARED_DEVICE") == "1"
    g = native.gbdt()
    key = ("shared" if use_gpu and shared_device else "rccl" if use_gpu else "host", world_size())
    if key in _comm_cache:
        if not getattr(_comm_cache[key], "aborted", False):
            return _comm_cache[key]
        del _comm_cache[key]  # aborted by a CommError in an earlier fit: rebuild
    if use_gpu and shared_device:
        import torch

        host = g.host_comm(rank(), world_size(), lambda arr: allreduce_numpy(arr))
        c = maybe_p2p(host, torch.cuda.current_device())
    elif use_gpu:
        import torch

        dev = torch.cuda.current_device() if torch.cuda.is_available() else -1

        timeout_ms = float(os.environ.get("SML_RCCL_INIT_TIMEOUT_MS", "120000"))

        def prepare():
            if dev >= 0:
                torch.cuda.set_device(dev)
            return g.rccl_unique_id() if rank() == 0 else None

        def make(uid):
            return g.rccl_comm(uid, rank(), world_size(), dev, timeout_ms)

        c = init_with_retries(make, "RCCL communicator", prepare=prepare)
        c = maybe_p2p(c, dev)
    else:
        c = g.host_comm(rank(), world_size(), lambda arr: allreduce_numpy(arr))
    _comm_cache[key] = c
    return c
