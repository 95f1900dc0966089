"""Multi-GPU batch demodulation: one process per GPU, streams sharded, decoded
bytes all-gathered.

Streams are independent, so the batch shards with no data-path exchange:
rank r demodulates the contiguous streams shard_range(B, r, world) on its own
GPU.  The one collective is the gather of the decoded byte buffers, so every
rank (or the caller on rank 0) ends with the whole batch's output, exactly as
a single-GPU call would have produced it.

Wire format of the gather (fixed size per rank, so it is one all-gather):
  payload [world][max_local][cap] uint8   decoded bytes, zero padded
  lengths [world][max_local]      int64   bytes per stream (-1 = no stream)
On the GPU path the payload moves over RCCL (xGMI) through libamr's
amr_allgather; on CPU (gloo) the same packing goes through
torch.distributed.all_gather -- that is how tests/test_multi.py covers the
N > 1 logic without a GPU.
"""
from __future__ import annotations

import numpy as np


def shard_range(n_streams: int, rank: int, world: int):
    """Contiguous, balanced [lo, hi) of the streams owned by `rank`."""
    base, extra = divmod(n_streams, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def max_local(n_streams: int, world: int) -> int:
    return -(-n_streams // world)


def pack(outs, max_streams: int, cap: int):
    """list[bytes] -> (payload [max_streams][cap] uint8, lengths [max_streams] int64)."""
    payload = np.zeros((max_streams, cap), np.uint8)
    lengths = np.full(max_streams, -1, np.int64)
    for i, o in enumerate(outs):
        if len(o) > cap:
            raise ValueError("decoded stream longer than the gather capacity")
        payload[i, :len(o)] = np.frombuffer(o, np.uint8)
        lengths[i] = len(o)
    return payload, lengths


def unpack(payload: np.ndarray, lengths: np.ndarray):
    """Inverse of pack over the gathered [world][max_local] layout, rank-major."""
    out = []
    for p, ln in zip(payload.reshape(-1, payload.shape[-1]), lengths.reshape(-1)):
        if ln >= 0:
            out.append(p[:ln].tobytes())
    return out


def gather_gloo(outs, n_streams: int, cap: int, dist):
    """CPU path: the same packed all-gather over torch.distributed (gloo)."""
    import torch
    world = dist.get_world_size()
    m = max_local(n_streams, world)
    payload, lengths = pack(outs, m, cap)
    pt = torch.from_numpy(payload)
    lt = torch.from_numpy(lengths)
    pts = [torch.empty_like(pt) for _ in range(world)]
    lts = [torch.empty_like(lt) for _ in range(world)]
    dist.all_gather(pts, pt)
    dist.all_gather(lts, lt)
    return unpack(np.stack([t.numpy() for t in pts]), np.stack([t.numpy() for t in lts]))


def demod_sharded(x: np.ndarray, demod_batch, rank: int, world: int, gather):
    """Demodulate this rank's shard of x with demod_batch and gather the result.

    x          : [B, N] the whole batch (each rank may hold only its shard's rows
                 in practice; rows outside the shard are not touched)
    demod_batch: callable([b, N]) -> list[bytes]  (modem.qpsk_demodulate_batch etc.)
    gather     : callable(list[bytes] local) -> list[bytes] global
    """
    lo, hi = shard_range(x.shape[0], rank, world)
    local = demod_batch(x[lo:hi]) if hi > lo else []
    return gather(local)
