"""Row-sharded sampling MPC over several GPUs (one process per GPU).

The reference runs all N rollouts of one MPC problem on one device
(centroidal_nmpc_jax.py:820-842: vmap over `num_parallel_computations`).  Here the rows of
one problem are split over ranks, rows [r*N/W, (r+1)*N/W) on rank r.  The only data exchange
of the step is one all-gather of a fixed-size per-rank record (rank order):

    [m_r, s_r, best row, pad | v_r (P) | K (row, cost) keys | K elite rows (K x P)]

with m_r the rank's minimum cost, s_r = sum exp(-(c - m_r)), v_r = sum exp(-(c - m_r)) * noise
(K = 1 except CEM, K = num_elite).  Every rank then merges the W records identically
(srbd_step_finish), so the new parameters agree bit for bit on all ranks without a broadcast.
Over RCCL the gather is `all_gather_into_tensor` on the stream the library launches on.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib


class RecordExchange:
    """The path's one collective: all-gather of equal-size float32 records in rank order."""

    def __init__(self, record_floats: int, world: int, device, group=None, stream=None):
        import torch

        self.torch = torch
        self.world = world
        self.group = group
        self.stream = stream  # the stream the record producer and the merge run on (CUDA only)
        self.local = torch.zeros(record_floats, dtype=torch.float32, device=device)
        self.gathered = torch.zeros(world * record_floats, dtype=torch.float32, device=device)
        self._parts = list(self.gathered.view(world, record_floats).unbind(0))

    def __call__(self) -> "torch.Tensor":
        import torch.distributed as dist

        if self.local.is_cuda:
            with self.torch.cuda.stream(self.stream):
                dist.all_gather_into_tensor(self.gathered, self.local, group=self.group)
        else:  # gloo: list form, written straight into the views of `gathered`
            dist.all_gather(self._parts, self.local, group=self.group)
        return self.gathered


def shard_rows(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """(first row, row count) of `rank` (matches the library's build_model)."""
    a = rank * n_total // world
    return a, (rank + 1) * n_total // world - a


class ShardedSamplingMPC:
    """One rank of a row-sharded MPC problem on the current process's GPU.

    cfg: an _lib.SrbdConfig with the GLOBAL num_samples; rank / world_size / device_id are set here.
    The library and the RCCL gather share one dedicated (non-default) torch stream, so the gather
    is ordered after the rollout and before the merge without host synchronisation.  (The legacy
    null stream cannot be handed to srbd_set_stream: a NULL handle selects the context's own stream.)
    """

    def __init__(self, cfg: _lib.SrbdConfig, rank: int, world: int, device_index: int, group=None):
        import torch

        cfg.rank, cfg.world_size, cfg.device_id = int(rank), int(world), int(device_index)
        cfg.use_graph = 0
        self.ctx = _lib.Context(cfg)
        self.rank, self.world = rank, world
        self.device = torch.device("cuda", device_index)
        self.stream = torch.cuda.Stream(self.device)
        self.ctx.set_stream(self.stream.cuda_stream)
        with torch.cuda.stream(self.stream):
            self.exchange = RecordExchange(self.ctx.record_floats(), world, self.device, group, self.stream)
        self.P = self.ctx.P
        self.result = _lib.SrbdResult()

    def step(self, state, ref, contact, best, sigma=None, noise_local=None, seed=42, counter=0):
        """One MPC iteration; returns (best, sigma, result) identical on every rank."""
        f = lambda a: None if a is None else _lib.fptr(np.ascontiguousarray(a, np.float32))  # noqa: E731
        state = np.ascontiguousarray(state, np.float32)
        ref = np.ascontiguousarray(ref, np.float32)
        contact = np.ascontiguousarray(contact, np.float32)
        best = np.array(best, np.float32).reshape(self.P).copy()
        sig = None if sigma is None else np.array(np.broadcast_to(sigma, (self.P,)), np.float32)
        noise = None if noise_local is None else np.ascontiguousarray(noise_local, np.float32)
        h = self.ctx.h
        self.ctx.check(_lib.lib.srbd_step_local(h, f(state), f(ref), f(contact), contact.shape[1], f(best), f(sig),
                                                f(noise), C.c_uint64(int(seed)), C.c_uint64(int(counter)),
                                                C.c_void_p(self.exchange.local.data_ptr())), "srbd_step_local")
        g = self.exchange()
        self.ctx.check(_lib.lib.srbd_step_finish(h, C.c_void_p(g.data_ptr()), self.world, _lib.fptr(best), f(sig),
                                                 C.byref(self.result), None), "srbd_step_finish")
        return best, sig, self.result

    def device_step(self):
        """Device-resident step (warm start kept on the device; benchmark chain)."""
        h = self.ctx.h
        self.ctx.check(_lib.lib.srbd_device_step_local(h, C.c_void_p(self.exchange.local.data_ptr())),
                       "srbd_device_step_local")
        g = self.exchange()
        self.ctx.check(_lib.lib.srbd_device_step_finish(h, C.c_void_p(g.data_ptr()), self.world),
                       "srbd_device_step_finish")

    def close(self):
        self.ctx.set_stream(None)
        self.ctx.close()
