"""Multi-GPU execution: one process per GPU, packets sharded, one RCCL sum-reduce.

The reference parallelises only over packets with OpenMP and sums per-thread detector
copies serially after the loop (``ARTES.f90:534-546``, ``959-975``).  Here each rank
transports the disjoint global packet range ``[k*N/G, (k+1)*N/G)`` on its own GPU (the
RNG is keyed by the global packet id, so the result does not depend on G), and the
detector tensor ``[4][4][ny][nx]`` (plus 8 packet-level moments, counters and error
codes) is summed with ONE ``all_reduce`` per (wavelength, detector direction)
(SURVEY.md §5, §8e).  The payload is ~80 KB at 25x25 pixels: latency-bound, so a
single flat RCCL all-reduce over xGMI is the whole exchange.

``torch.distributed`` with backend ``nccl`` is RCCL on ROCm; ``gloo`` is used for the
CPU tests of this module.
"""

from __future__ import annotations

import os
import sys
from dataclasses import dataclass

import numpy as np

# collectives this process issued, by path (tests/test_gpu_dist_cli.py checks that the RCCL
# branch of allreduce_numpy ran): "host" (gloo, in place) and "device" (nccl, via the GPU)
COLLECTIVES = {"host": 0, "device": 0}


@dataclass
class Rank:
    rank: int = 0
    world: int = 1
    local_rank: int = 0


def env_rank() -> Rank:
    return Rank(int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
                int(os.environ.get("LOCAL_RANK", 0)))


def device_of(r: Rank) -> int:
    """The HIP device of rank ``r``: ``local_rank`` modulo the visible devices.  One rule for
    every entry point (``init``'s RCCL device, ``bench.py``, the drop-in CLI): a launcher that
    shows each rank only its own GPU must not make rank 3 ask for device 3, and ranks sharing
    one card (the gloo rehearsal on a one-GPU box) all use device 0.  Counting devices does
    not initialise the GPU on this image."""
    import torch

    return r.local_rank % max(1, torch.cuda.device_count())


def init(backend: str | None = None) -> Rank:
    """Initialise torch.distributed from the torchrun environment (no-op for one process,
    unless ARTES_DIST_FORCE=1: a one-rank group, to exercise the collective path)."""
    r = env_rank()
    if r.world > 1 or os.environ.get("ARTES_DIST_FORCE") == "1":
        import torch.distributed as dist

        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29511")
            backend = backend or os.environ.get("ARTES_DIST_BACKEND")   # gloo: multi-rank rehearsal on one GPU
            if backend is None:
                import torch

                backend = "nccl" if torch.cuda.is_available() else "gloo"
            kw = {}
            if backend == "nccl":
                import torch

                d = device_of(r)
                torch.cuda.set_device(d)
                kw["device_id"] = torch.device("cuda", d)
            dist.init_process_group(backend=backend, rank=r.rank, world_size=r.world, **kw)
    return r


def shard(n_packets: int, rank: int, world: int) -> tuple[int, int]:
    """Global packet range of ``rank``: ``[k*N//G, (k+1)*N//G)``, as (first, count)."""
    lo = (n_packets * rank) // world
    hi = (n_packets * (rank + 1)) // world
    return lo, hi - lo


def group_active() -> bool:
    """A process group is open (``init`` with several ranks, or one rank under
    ARTES_DIST_FORCE=1).  (No torch import when none was made.)"""
    d = sys.modules.get("torch.distributed")
    return d is not None and d.is_available() and d.is_initialized()


def reduces(world: int) -> bool:
    """Whether a call made for ``world`` ranks sums over the open process group: only when the
    group has exactly that many ranks.  A one-rank group (ARTES_DIST_FORCE=1) exercises the
    collective path at world size 1; a caller's unsharded run (world 1) inside a host
    application's own multi-rank group is not reduced, since every rank of that group then
    transported every packet.  A sharded call (world > 1) without a matching group fails."""
    if not group_active():
        if world > 1:
            raise RuntimeError(f"a {world}-rank call needs an open process group (artes_amd.dist.init)")
        return False
    import torch.distributed as dist

    size = dist.get_world_size()
    if world > 1 and size != world:
        raise RuntimeError(f"a {world}-rank call inside a process group of {size} ranks")
    return size == max(world, 1)


def allreduce_numpy(arrays: list[np.ndarray], world: int) -> list[np.ndarray]:
    """Sum host arrays over ranks: in place under gloo, through the rank's GPU under nccl."""
    if not reduces(world):
        return arrays
    import torch
    import torch.distributed as dist

    # RCCL reduces device memory only: under the nccl backend the host arrays travel
    # through the rank's GPU in ONE flat buffer (one all_reduce per call, as in bench.py)
    on_gpu = dist.get_backend() == "nccl"
    flat = np.concatenate([np.ascontiguousarray(a, dtype=np.float64).ravel() for a in arrays])
    t = torch.from_numpy(flat)
    if on_gpu:
        t = t.to(torch.device("cuda", torch.cuda.current_device()))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    COLLECTIVES["device" if on_gpu else "host"] += 1
    flat = t.cpu().numpy() if on_gpu else t.numpy()
    out, at = [], 0
    for a in arrays:
        v = flat[at:at + a.size].reshape(a.shape)
        at += a.size
        out.append(v.astype(a.dtype) if a.dtype != np.float64 else v.copy())
    return out


def broadcast_int(value: int, r: Rank) -> int:
    """Rank 0's non-negative ``value`` (< 2^64) on every rank: the clock seed of a CLI run
    must be the same on every shard, or the global packet ids would not map to one RNG
    stream set (the result would then depend on the rank start times)."""
    if not reduces(r.world):
        return int(value)
    parts = np.array([value >> 32, value & 0xFFFFFFFF], dtype=np.float64) if r.rank == 0 else np.zeros(2)
    (out,) = allreduce_numpy([parts], r.world)   # exact: each half < 2^32
    return (int(out[0]) << 32) | int(out[1])


def run_sharded(transport, n_packets: int, seed: int, r: Rank):
    """Run ``transport(first, count, seed) -> RunResult`` on this rank's shard and sum
    the results over all ranks (host tensors; the GPU bench uses device tensors + RCCL)."""
    first, count = shard(n_packets, r.rank, r.world)
    res = transport(first, count, seed)
    if reduces(r.world):
        flows = [k for k in ("flow_global", "flow_latitudinal") if getattr(res, k, None) is not None]
        red = allreduce_numpy([res.det, res.totals, res.counters.astype(np.float64), res.err.astype(np.float64)]
                              + [getattr(res, k) for k in flows], r.world)
        res.det, res.totals = red[0], red[1]
        res.counters = np.rint(red[2]).astype(np.uint64)
        res.err = np.rint(red[3]).astype(np.uint64)
        for k, v in zip(flows, red[4:]):
            setattr(res, k, v)
    return res
